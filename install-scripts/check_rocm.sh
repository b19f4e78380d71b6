#!/bin/bash
# Verify the ROCm stack the framework needs (replaces the reference's OFED / dev-tools /
# GCC / MPI installers: on MI355X the fabric (xGMI) and collectives (RCCL) ship with ROCm).
ROCM=${ROCM_PATH:-/opt/rocm}
ok=1
need() { if [ -e "$1" ]; then echo "  ok   $1"; else echo "  MISSING $1"; ok=0; fi; }
echo "[check_rocm] ROCm at $ROCM (version $(cat $ROCM/.info/version 2>/dev/null || echo unknown))"
need "$ROCM/bin/hipcc"
need "$ROCM/lib/librccl.so"
need "$ROCM/include/rccl/rccl.h"
need "$ROCM/lib/libamdhip64.so"
if command -v rocm-smi >/dev/null 2>&1; then
  n=$(rocm-smi --showid 2>/dev/null | grep -c "GPU\[" || true)
  echo "  GPUs visible to rocm-smi: $n"
else
  echo "  rocm-smi not on PATH (no driver on this host?)"
fi
python3 - <<'PY' || ok=0
import torch
print(f"  PyTorch {torch.__version__} HIP {torch.version.hip}")
assert torch.version.hip, "PyTorch is not a ROCm build"
PY
[ "$ok" = 1 ] || { echo "[check_rocm] incomplete ROCm stack" >&2; exit 1; }
