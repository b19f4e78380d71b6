#!/usr/bin/env python3
"""The bf16 gradient-accuracy floor of the shallow ResNet (stem + max pool + one bottleneck block
+ classifier; tests/test_determinism_gpu.py): what a stock PyTorch bf16 pipeline gives on this
net, against which the hand-written bf16 path is judged.

Three GPU runs of the same weights / batch, each against the fp32 CPU step of our framework:
  * torch-fp32  : a plain torch.nn.functional mirror of the net (NCHW channels_last, MIOpen) in
                  fp32 -- pins the mirror itself (must agree to ~1e-5);
  * autocast    : the same mirror under torch.autocast(bfloat16) -- the floor;
  * hip-bf16    : our bf16 path (HIP kernels, fused BN epilogues, space-to-depth stem).
Per parameter tensor: relative-norm error rel = |g - g_ref| / |g_ref| and the ratio
hip / autocast. Prints one line per tensor and a JSON summary line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import azure_hc_intel_tf_amd  # noqa: E402,F401
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from azure_hc_intel_tf_amd.models import resnet  # noqa: E402
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch  # noqa: E402

KW = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
BATCH = 32


def shallow(device, **kw):
    resnet.LAYER_COUNTS.setdefault(1, (1,))  # stem + max pool + ONE bottleneck block + classifier
    if str(device).startswith("cuda"):
        kw.setdefault("compute_dtype", "bf16")  # the 16-bit path (create_model defaults to fp32)
    return resnet.ResNet(depth=1, device=device, **KW, **kw)


def _conv(x, w_krsc, stride, pad):
    return F.conv2d(x, w_krsc.permute(0, 3, 1, 2), stride=stride, padding=pad)


def _bn(x, g, b, relu):
    y = F.batch_norm(x, None, None, g, b, training=True, momentum=0.0, eps=1e-5)
    return F.relu(y) if relu else y


def mirror_grads(params, img_nhwc, lab, device, autocast):
    """torch.nn.functional mirror of the shallow net (tf_cnn_benchmarks padding: 'SAME_RESNET'
    7x7/2 = symmetric pad 3; max pool 3x3/2 'SAME' = pad bottom/right 1 on the even input).
    Returns {param name: grad in our layout (KRSC convs)}."""
    P = {n: t.detach().to(device).clone().requires_grad_(True) for n, t in params.items()}
    x = img_nhwc.to(device).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        h = _bn(_conv(x, P["conv0/conv2d/kernel"], 2, 3), P["conv0/batchnorm/gamma"], P["conv0/batchnorm/beta"], True)
        h = F.max_pool2d(F.pad(h, (0, 1, 0, 1), value=float("-inf")), 3, 2)
        pre = "stage1/block1/"

        def cbn(name, t, stride, pad, relu):
            return _bn(_conv(t, P[pre + name + "/conv2d/kernel"], stride, pad), P[pre + name + "/batchnorm/gamma"],
                       P[pre + name + "/batchnorm/beta"], relu)

        sc = cbn("shortcut", h, 1, 0, False)
        a = cbn("conv1", h, 1, 0, True)
        b = cbn("conv2", a, 1, 1, True)
        y = F.relu(cbn("conv3", b, 1, 0, False) + sc)
        feat = y.float().mean(dim=(2, 3))
        w = P["logits/affine/weights"]
        logits = feat @ w.view(w.shape[0], -1).t() + P["logits/affine/biases"]
        loss = F.cross_entropy(logits.float(), lab.to(device))
    loss.backward()
    return {n: t.grad.detach().float().cpu() for n, t in P.items()}, float(loss.detach())


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def main():
    mc = shallow("cpu")
    img_c, lab_c = synthetic_batch(mc, BATCH, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, BATCH, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    ref = {p.name: p.grad.float().clone() for p in mc.ps.params}
    params = {p.name: p.data.clone() for p in mc.ps.params}
    cpu_loss = tc.row_loss.mean().item()

    mg = shallow("cuda")
    assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
    tg = Trainer(mg, BATCH, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    torch.cuda.synchronize()
    hip = {p.name: p.grad.float().cpu() for p in mg.ps.params}

    f32, loss32 = mirror_grads(params, img_c, lab_c, "cuda", autocast=False)
    ac, lossac = mirror_grads(params, img_c, lab_c, "cuda", autocast=True)
    print(f"loss: cpu {cpu_loss:.6f} torch-fp32 {loss32:.6f} autocast {lossac:.6f} "
          f"hip-bf16 {tg.row_loss.mean().item():.6f}")
    print(f"{'tensor':40s} {'torch-fp32':>11s} {'autocast':>10s} {'hip-bf16':>10s} {'hip/ac':>7s}")
    rows = []
    for name in ref:
        r, sl = ref[name], (lambda t: t)
        if name.startswith("conv0/conv2d"):  # the 3 real input channels
            sl = (lambda t: t[..., :3])
        e32, eac, ehip = (rel(sl(d[name]).flatten(), sl(r).flatten()) for d in (f32, ac, hip))
        rows.append({"tensor": name, "torch_fp32": e32, "autocast": eac, "hip_bf16": ehip, "ratio": ehip / eac})
        print(f"{name:40s} {e32:11.2e} {eac:10.2e} {ehip:10.2e} {ehip / eac:7.2f}", flush=True)
    print(json.dumps({"max_ratio": max(r["ratio"] for r in rows), "max_mirror_err": max(r["torch_fp32"] for r in rows),
                      "rows": rows}))


if __name__ == "__main__":
    main()
