"""Diagnostic: fp32-output vs plane-output BN backward (bn_bwd_apply_acc) on identical inputs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from azure_hc_intel_tf_amd.ops import functional as Fn, _ext
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype

_ext.load()
set_gpu_compute_dtype(torch.float32)
Fn.set_f32_native(True)
Fn.set_deterministic(True)
DEV = "cuda"
torch.manual_seed(21)
C, N, H, R = 256, 4, 9, 8
M = N * H * H
z = torch.randn(N, H, H, C, device=DEV) * 2 + 0.5
mean = z.view(-1, C).mean(0)
invstd = torch.rsqrt(z.view(-1, C).var(0, unbiased=False) + 1e-5)
gamma = torch.rand(C, device=DEV) + 0.5
beta = torch.randn(C, device=DEV) * 0.1
dy = torch.randn(N, H, H, C, device=DEV)
sv = Fn.BNSaved(mean, invstd)
for mode in (0, 2):
    res = []
    for planes in (False, True, False, True):
        dz = Fn.Planes.empty((N, H, H, C), DEV) if planes else torch.empty_like(z)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        acc_b = torch.zeros(R * 2 * C, device=DEV)
        Fn.bn_backward_acc(dy, None, z, sv, gamma, beta, mode, dg, db, dz, acc_b, R)
        torch.cuda.synchronize()
        res.append((dz.float() if planes else dz, dg.clone(), db.clone(), acc_b.clone()))
    for i in range(1, 4):
        a, b = res[0], res[i]
        print(f"mode {mode} run0 vs run{i}: dz maxdiff {float((a[0]-b[0]).abs().max()):.3e} "
              f"dg {float((a[1]-b[1]).abs().max()):.3e} db {float((a[2]-b[2]).abs().max()):.3e} "
              f"acc {float((a[3]-b[3]).abs().max()):.3e}")
    print("dz ref scale", float(res[0][0].abs().max()))
