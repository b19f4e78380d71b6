#!/usr/bin/env python3
"""Where does the fp32 HIP path (bf16x6 GEMMs) lose precision? Prints
  (1) per-op relative errors of conv fwd / dgrad / wgrad against fp64 for a few shapes,
  (2) the shallow net (stem + one bottleneck + classifier) per-tensor gradient errors of
      (a) the fp32 HIP path and (b) the fp32 PyTorch/MIOpen path, both against the fp32 CPU path,
      and the forward loss difference of each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import azure_hc_intel_tf_amd  # noqa: E402,F401
import torch  # noqa: E402

from azure_hc_intel_tf_amd.models import resnet  # noqa: E402
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype  # noqa: E402
from azure_hc_intel_tf_amd.nn.params import ParamStore  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402
from azure_hc_intel_tf_amd.ops.functional import ConvSpec  # noqa: E402
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item(), ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def conv_ops():
    set_gpu_compute_dtype(torch.float32)
    Fn.set_f32_native(True)
    for cin, cout, k, s, pad, H in [(64, 64, 3, 1, 1, 28), (256, 64, 1, 1, 0, 28), (512, 512, 3, 1, 1, 7),
                                    (2048, 512, 1, 1, 0, 7)]:
        spec = ConvSpec(cin=cin, cin_pad=cin, cout=cout, kh=k, kw=k, sh=s, sw=s, pt=pad, pl=pad, pb=pad, pr=pad)
        ps = ParamStore(seed=5)
        p = ps.add("w", (cout, k, k, cin), True, ps.variance_scaling(k * k * cin))
        pk = ps.add_pack(p, cout, k, k, cin, spec.Kpad, spec.Kpad_t, want_tr=True)
        ps.finalize("cuda", dtype_pack=torch.bfloat16, pack_lo=True)
        ps.repack()
        torch.manual_seed(0)
        N = 8
        x = torch.randn(N, H, H, cin, device="cuda")
        P, Q = spec.out_hw(H, H)
        xd = x.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
        wd = p.data.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
        ref = torch.nn.functional.conv2d(xd, wd, stride=s, padding=pad)
        y = torch.empty(N, P, Q, cout, device="cuda")
        Fn.conv_forward(x, spec, pk.pack, p.data, y)
        dz = torch.randn(N, P, Q, cout, device="cuda")
        ref.backward(dz.double().cpu().permute(0, 3, 1, 2))
        dx = torch.zeros(N, H, H, cin, device="cuda")
        Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False)
        dw = torch.zeros(cout, spec.K, device="cuda")
        Fn.conv_wgrad(dz, x, spec, dw)
        # fp32 CPU conv for scale: what true fp32 rounding gives
        y32 = torch.nn.functional.conv2d(x.cpu().permute(0, 3, 1, 2), p.data.cpu().permute(0, 3, 1, 2), stride=s,
                                         padding=pad)
        print(f"conv {cin}->{cout} k{k}: fwd {rel(y, ref.permute(0, 2, 3, 1))}  (fp32 CPU {rel(y32.permute(0, 2, 3, 1), ref.permute(0, 2, 3, 1))})"
              f"  dgrad {rel(dx, xd.grad.permute(0, 2, 3, 1))}  wgrad {rel(dw.view(cout, k, k, cin), wd.grad.permute(0, 2, 3, 1))}",
              flush=True)
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


def shallow(device, **kw):
    resnet.LAYER_COUNTS.setdefault(1, (1,))
    if str(device).startswith("cuda"):
        kw.setdefault("compute_dtype", "bf16")  # the 16-bit path (create_model defaults to fp32)
    return resnet.ResNet(depth=1, device=device, **kw)


def grads(mg, mc):
    out = []
    for pg, pc in zip(mg.ps.params, mc.ps.params):
        a, b = pg.grad.float().cpu().flatten(), pc.grad.float().flatten()
        if pg.name.startswith("conv0/conv2d"):
            a, b = pg.grad[..., :3].float().cpu().flatten(), pc.grad[..., :3].float().flatten()
        out.append((pg.name, rel(a, b)))
    return out


def shallow_net():
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = (img_c - 127.0) / 60.0
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    for label, native in (("fp32 HIP (bf16x6)", True), ("fp32 PyTorch/MIOpen", False)):
        old = resnet.ResNet.F32_NATIVE_OK
        resnet.ResNet.F32_NATIVE_OK = native
        try:
            mf = shallow("cuda", compute_dtype="fp32", **kw)
        finally:
            resnet.ResNet.F32_NATIVE_OK = old
        assert mf.native == native
        tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tf._forward_backward(img_c.cuda(), lab_c.cuda())
        torch.cuda.synchronize()
        print(f"== {label}: loss {tf.row_loss.mean().item():.7f} vs CPU {tc.row_loss.mean().item():.7f}", flush=True)
        for name, (r, m) in grads(mf, mc):
            print(f"   {name:40s} rel {r:.2e}  max {m:.2e}", flush=True)
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


if __name__ == "__main__":
    conv_ops()
    shallow_net()
