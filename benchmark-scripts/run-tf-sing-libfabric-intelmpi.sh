#!/bin/bash
# MI355X-native replacement of the reference runner of the same name
# (/root/reference/benchmark-scripts/run-tf-sing-libfabric-intelmpi.sh): same positional CLI,
# one worker process per MI355X, RCCL over xGMI ("ib") or RCCL sockets ("sock").
#
# usage: ./run-tf-sing-libfabric-intelmpi.sh <NUM_NODES> <WORKERS_PER_SOCKET> <batch_size> <fabric(ib,sock)>
# e.g.   ./run-tf-sing-libfabric-intelmpi.sh 1 4 64 ib        # 8 workers on a 2-socket 8x MI355X node
#        DEVICE=cpu ./run-tf-sing-libfabric-intelmpi.sh 1 1 32 sock   # CPU path (BASELINE config 1)
set -e
if [ "$#" -ne 4 ]; then
  echo "usage: $0 <NUM_NODES> <WORKERS_PER_SOCKET> <batch_size> <fabric(ib,sock)>" >&2
  exit 1
fi
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(dirname "$HERE")"
export PYTHONPATH="$REPO${PYTHONPATH:+:$PYTHONPATH}"
# like the reference IMPI runner (run-tf-sing-libfabric-intelmpi.sh:94-105): fusion threshold
# passed, no HOROVOD_MPI_THREADS_DISABLE, no core pinning, transport debug output on
# (NCCL_DEBUG=INFO is set by the launcher plan as the I_MPI_DEBUG=5 analogue)
export HOROVOD_FUSION_THRESHOLD=${HOROVOD_FUSION_THRESHOLD:-134217728}
export HSA_ENABLE_IPC_MODE_LEGACY=0
python3 -m azure_hc_intel_tf_amd.launch.run_tf_sing --flavor libfabric-intelmpi "$@"
