"""Where does the fp32 zoo's GPU-vs-CPU gradient gap come from?

For a BN-free SequentialCNN (AlexNet, LeNet, VGG, ...) at fp32 this records, in one forward +
backward of each path on the same weights and images (dropout off):

* every ReLU mask and max-pool window argmax of the GPU step (hand-written HIP kernels: bf16x6
  plane GEMMs, fp32 pools) and of the fp32 CPU step (PyTorch / oneDNN);
* an fp64 autograd MIRROR of the network whose ReLU masks and max-pool argmaxes are FORCED to the
  GPU's decisions (or to the CPU's).

With the decisions forced, the mirror's gradient is what either path would compute in exact
arithmetic given its own discrete choices, so
  |g_gpu - mirror(gpu decisions)| / |mirror|   is the GPU kernels' pure fp32 rounding error, and
  |g_cpu - mirror(cpu decisions)| / |mirror|   the CPU's;
the remaining GPU-vs-CPU gap is the flips: decisions whose input sits within rounding of the ReLU
threshold / a tie between window elements, counted per layer.

    python tools/zoo_flip_probe.py alexnet 67 4     (GPU box)
"""
from __future__ import annotations

import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

from azure_hc_intel_tf_amd.models import create_model  # noqa: E402
from azure_hc_intel_tf_amd.models import sequential  # noqa: E402
from azure_hc_intel_tf_amd.models.sequential import Flatten  # noqa: E402
from azure_hc_intel_tf_amd.nn.layers import ConvBN, Dropout, Pool, set_gpu_compute_dtype  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch  # noqa: E402


def _record(model):
    """Wrap the model's conv / pool forwards: per layer, the ReLU mask (conv + ReLU) or the pool's
    input (the argmax is recomputed from it for the CPU path; the GPU's own uint8 argmax is kept)."""
    rec = {}
    for l in model.seq:
        if isinstance(l, ConvBN) and l.relu:
            f = l.forward

            def fw(x, *a, _l=l, _f=f, **k):
                y = _f(x, *a, **k)
                rec[_l.name] = ("relu", (Fn.from_planes(y) if Fn.is_planes(y) else y).float().cpu() > 0)
                return y
            l.forward = fw
        elif isinstance(l, Pool) and l.is_max:
            f = l.forward

            def pw(x, *a, _l=l, _f=f, **k):
                y = _f(x, *a, **k)
                xin = (Fn.from_planes(x) if Fn.is_planes(x) else x).float().cpu()
                amax = _l._saved[2].cpu().clone() if (_l._saved is not None and _l._saved[2] is not None) else None
                rec[_l.name] = ("pool", xin, amax)
                return y
            l.forward = pw
    return rec


def _windows(x, l):
    """[N, P, Q, C, kh*kw] window values of an NHWC pool input (VALID / SAME pads with -inf)."""
    pt, pb, pl, pr = l.pads
    kh, kw = l.k
    sh, sw = l.s
    xt = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=-float("inf"))
    u = xt.unfold(2, kh, sh).unfold(3, kw, sw)  # N C P Q kh kw
    N, C, P, Q = u.shape[:4]
    return u.reshape(N, C, P, Q, kh * kw).permute(0, 2, 3, 1, 4)


def _first_max(win):
    m = win.max(-1, keepdim=True).values
    idx = torch.arange(win.shape[-1], dtype=torch.int64)
    return torch.where(win == m, idx, win.shape[-1]).min(-1).values


def mirror_grads(model_cpu, images, labels, decisions):
    """fp64 forward / backward of the SequentialCNN with every ReLU mask and max-pool argmax taken
    from ``decisions`` (layer name -> bool mask / int64 window index). Returns {param name: grad}."""
    P = {p.name: p.data.detach().double().clone().requires_grad_(True) for p in model_cpu.ps.params}
    x = images.double()
    for l in model_cpu.seq:
        if isinstance(l, ConvBN):
            s = l.spec
            w = P[f"{l.name}/conv2d/kernel"].permute(0, 3, 1, 2)
            xt = F.pad(x.permute(0, 3, 1, 2), (s.pl, s.pr, s.pt, s.pb))
            y = F.conv2d(xt, w, bias=P[f"{l.name}/conv2d/bias"], stride=(s.sh, s.sw)).permute(0, 2, 3, 1)
            x = y * decisions[l.name].to(y.dtype) if l.relu else y
        elif isinstance(l, Pool):
            win = _windows(x, l)
            if l.is_max:
                x = win.gather(-1, decisions[l.name].unsqueeze(-1)).squeeze(-1)
            else:
                x = win.mean(-1)
        elif isinstance(l, Flatten):
            x = x.reshape(x.shape[0], 1, 1, -1)
        elif isinstance(l, Dropout):
            assert l.keep >= 1.0
        else:
            raise NotImplementedError(type(l).__name__)
    fc = model_cpu.fc
    logits = x.reshape(x.shape[0], -1) @ P[f"{fc.name}/affine/weights"].reshape(fc.ncls, -1).t() \
        + P[f"{fc.name}/affine/biases"]
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    return {n: t.grad for n, t in P.items()}


def _flat(model, g):
    return torch.cat([g[p.name].reshape(-1) for p in model.ps.params])


def probe(name: str, size: int, batch: int, seed: int = 9, img_seed: int = 4, verbose: bool = True):
    """Returns a dict: per-layer flip counts (GPU vs CPU and vs the fp64 mirror) and the relative
    gradient errors GPU / CPU vs the decision-forced fp64 mirrors."""
    old_keep = sequential.SequentialCNN.dropout_keep
    sequential.SequentialCNN.dropout_keep = 1.0
    kw = dict(image_size=size, seed=seed, image_channels=8)
    try:
        mg = create_model(name, device="cuda", compute_dtype="fp32", **kw)
        mc = create_model(name, device="cpu", **kw)
        img, lab = synthetic_batch(mc, batch, seed=img_seed)
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
        rg, rc = _record(mg), _record(mc)
        tg = Trainer(mg, batch, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img.cuda(), lab.cuda())
        torch.cuda.synchronize()
        gg = torch.cat([p.grad.reshape(-1).double().cpu() for p in mg.ps.params])
        tc = Trainer(mc, batch, constant_lr(0.0), weight_decay=0.0)
        tc._forward_backward(img, lab)
        gc = torch.cat([p.grad.reshape(-1).double() for p in mc.ps.params])
        dec_g, dec_c, flips = {}, {}, []
        for l in mc.seq:
            if l.name not in rg:
                continue
            kind = rg[l.name][0]
            if kind == "relu":
                a, b = rg[l.name][1], rc[l.name][1]
                dec_g[l.name], dec_c[l.name] = a, b
                flips.append((l.name, "relu", int((a != b).sum()), a.numel()))
            else:
                _, xg, amax = rg[l.name]
                _, xc, _ = rc[l.name]
                ag = amax.to(torch.int64) if amax is not None else _first_max(_windows(xg, l))
                ac = _first_max(_windows(xc, l))
                dec_g[l.name], dec_c[l.name] = ag, ac
                flips.append((l.name, "maxpool", int((ag != ac).sum()), ag.numel()))
        mirror_g = _flat(mc, mirror_grads(mc, img, lab, dec_g))
        mirror_c = _flat(mc, mirror_grads(mc, img, lab, dec_c))

        def rel(a, b):
            return float((a - b).norm() / b.norm())
        out = {"flips": flips, "gpu_vs_cpu": rel(gg, gc), "gpu_vs_mirror_gpu": rel(gg, mirror_g),
               "cpu_vs_mirror_cpu": rel(gc, mirror_c), "mirror_gpu_vs_mirror_cpu": rel(mirror_g, mirror_c),
               "cpu_vs_mirror_gpu": rel(gc, mirror_g)}
        if verbose:
            print(f"== {name} {size}px bs={batch} (fp32 GPU step vs fp32 CPU step, dropout off, wd 0)")
            for n, k, f, tot in flips:
                print(f"  {n:14s} {k:8s} GPU/CPU decision flips {f:6d} of {tot}")
            for k, v in out.items():
                if k != "flips":
                    print(f"  {k:26s} {v:.3e}")
        return out
    finally:
        sequential.SequentialCNN.dropout_keep = old_keep
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


if __name__ == "__main__":
    a = sys.argv[1:]
    cases = [(a[0], int(a[1]), int(a[2]))] if a else [("alexnet", 67, 4), ("lenet", 28, 8), ("vgg11", 32, 4),
                                                        ("overfeat", 95, 4)]
    for c in cases:
        probe(*c)
