#!/bin/bash
# Cluster prep (role of the reference's prep-cluster.sh): passwordless ssh for the hostfile's
# nodes, then the per-node readiness check (GPUs, xGMI topology, RDMA NIC state) on each.
# usage: prep-cluster.sh [hostfile]   (default ~/nodeips.txt; without one: this node only)
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
HOSTFILE=${1:-$HOME/nodeips.txt}
if [ ! -f "$HOSTFILE" ]; then
  bash "$HERE/node-check.sh"
  exit 0
fi
bash "$HERE/setup-pwdless-ssh.sh" "$HOSTFILE"
while read -r h; do
  [ -z "$h" ] && continue
  ssh "$h" "bash -s" < "$HERE/node-check.sh" || echo "node-check failed on $h"
done < "$HOSTFILE"
