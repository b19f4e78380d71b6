#!/bin/bash
# Host settings for an 8x MI355X training node (role of the reference's update_config.sh).
# Default: report. With --apply (root): set them.
#   * locked-memory limit unlimited (RCCL / IPC buffers)
#   * automatic NUMA balancing off (page migration stalls the GPU feeders)
#   * open-files limit raised (one process per GPU + RCCL sockets)
APPLY=0
[ "$1" = "--apply" ] && APPLY=1
echo "[update_config] memlock: $(ulimit -l)   nofile: $(ulimit -n)"
nb=/proc/sys/kernel/numa_balancing
[ -r $nb ] && echo "[update_config] numa_balancing: $(cat $nb) (recommended 0)"
if [ "$APPLY" = 1 ]; then
  if [ "$(id -u)" != 0 ]; then echo "--apply needs root" >&2; exit 1; fi
  printf '* soft memlock unlimited\n* hard memlock unlimited\n* soft nofile 1048576\n* hard nofile 1048576\n' \
    > /etc/security/limits.d/90-hcb-mi355x.conf
  [ -w $nb ] && echo 0 > $nb
  echo "[update_config] applied (re-login for limits)"
fi
