#!/bin/bash
# Passwordless ssh between the nodes listed in a hostfile (one host per line). Only needed
# for multi-node runs; a single 8x MI355X node needs none of this.
# usage: setup-pwdless-ssh.sh [hostfile]   (default ~/nodeips.txt)
HOSTFILE=${1:-$HOME/nodeips.txt}
[ -f "$HOSTFILE" ] || { echo "no hostfile $HOSTFILE" >&2; exit 1; }
[ -f "$HOME/.ssh/id_ed25519" ] || ssh-keygen -t ed25519 -N "" -f "$HOME/.ssh/id_ed25519" -q
mkdir -p "$HOME/.ssh"
grep -q "StrictHostKeyChecking" "$HOME/.ssh/config" 2>/dev/null || \
  printf 'Host *\n    StrictHostKeyChecking accept-new\n    ConnectTimeout 5\n' >> "$HOME/.ssh/config"
chmod 600 "$HOME/.ssh/config"
while read -r h; do
  [ -z "$h" ] && continue
  echo "[ssh] authorizing $h"
  ssh-copy-id -i "$HOME/.ssh/id_ed25519.pub" "$h" >/dev/null 2>&1 || echo "  could not reach $h"
done < "$HOSTFILE"
