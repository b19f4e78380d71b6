#!/bin/bash
# Per-node readiness check for an 8x MI355X node (what the reference's prep-cluster verified
# per node over pssh -- IB port state -- becomes GPU + xGMI + RDMA-NIC state here).
echo "== $(hostname)"
if command -v rocm-smi >/dev/null 2>&1; then
  echo "-- GPUs"
  rocm-smi --showproductname 2>/dev/null | grep -E "GPU\[[0-9]+\].*(Card Series|Card SKU)" | head -16
  echo "-- xGMI link topology (hops / link type between GPU pairs)"
  rocm-smi --showtopotype 2>/dev/null | sed -n '1,20p'
else
  echo "rocm-smi not found"
fi
if command -v ibv_devinfo >/dev/null 2>&1; then
  echo "-- RDMA NIC port state (multi-node only)"
  ibv_devinfo 2>/dev/null | grep -E "hca_id|state" | head -32
fi
echo "-- HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-unset} (0 needed for dmabuf IPC)"
