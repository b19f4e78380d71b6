#!/usr/bin/env python3
"""fp32 shallow-net gradient check (tests/test_determinism_gpu.py's first half) with every
tensor printed, for the Trainer built with and without graphs, after optional pre-steps:
    python tools/diag_fp32_shallow.py [--bf16-first]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch

from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
from test_determinism_gpu import _grad_errors, _shallow


def main():
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    if "--bf16-first" in sys.argv:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    for graph in (False, True, False):
        mf = _shallow("cuda", compute_dtype="fp32", **kw)
        tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=graph)
        tf._forward_backward(img_c.cuda(), lab_c.cuda())
        torch.cuda.synchronize()
        print(f"== use_graph={graph} native={mf.native} f32_native={Fn._F32_NATIVE[0]} det={Fn.deterministic()}")
        for err, rel, cos, name in _grad_errors(mf, mc):
            print(f"   {name:40s} err {err:.2e} rel {rel:.2e} cos {cos}")


if __name__ == "__main__" and "--scan" not in sys.argv and "--stages" not in sys.argv and "--bn" not in sys.argv \
        and "--ref" not in sys.argv and "--both" not in sys.argv \
        and "--saved" not in sys.argv and "--gap" not in sys.argv and "--bncmp" not in sys.argv:
    main()


def scan():
    """which cuda tensors held by the fp32 model's layers are not fp32 (run with no bf16 model first)"""
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    for l in mf.all_layers():
        for k, v in vars(l).items():
            if torch.is_tensor(v) and v.is_cuda and v.dtype not in (torch.float32, torch.int64, torch.uint8, torch.int32):
                print("  non-fp32:", getattr(l, "name", type(l).__name__), k, v.dtype, tuple(v.shape))
    fc = mf.fc
    print("fc lo", Fn.lo_pack(fc.pack.tr) is not None, "pack lo", Fn.lo_pack(fc.pack.pack) is not None,
          "x dtype", None if fc._x is None else fc._x.dtype)
    lo = Fn.lo_pack(fc.pack.tr)
    if lo is not None:
        print("fc tr lo abs max", float(lo.abs().max()), "hi abs max", float(fc.pack.tr.float().abs().max()))


if __name__ == "__main__" and "--scan" in sys.argv:
    scan()


def stages(bf16_first):
    """relative error of the FC data gradient (first backward op) vs an fp64 reference, per run setup"""
    from azure_hc_intel_tf_amd.nn import layers as L
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    cap = {}
    orig = L.Logits.backward

    def fc_bwd(self, dlogits):
        w = self.w.data.view(self.ncls, self.cin).double()
        cap["ref"] = dlogits[:, :self.ncls].double() @ w
        cap["dl"] = dlogits.clone()
        out = orig(self, dlogits)
        cap["out"] = out.double()
        return out

    L.Logits.backward = fc_bwd
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    L.Logits.backward = orig
    r, o = cap["ref"], cap["out"]
    print(f"bf16_first={bf16_first} fc dgrad rel err {float((o - r).norm() / r.norm()):.3e} "
          f"dlogits dtype {cap['dl'].dtype} cfg {Fn.conv_plan(32, mf.fc.cin, mf.fc.ld)}")


if __name__ == "__main__" and "--stages" in sys.argv:
    stages("--bf16-first" in sys.argv)


def bnstage(bf16_first):
    """the block's conv3 BN backward (first BN backward of the step) vs the CPU path on the same inputs"""
    from azure_hc_intel_tf_amd.nn import layers as L
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    orig = L.ConvBN.backward
    done = []

    def bwd(self, dy, dx=None, accumulate=False, want_gres=False, dx_bn=None):
        first = not done and self.bn
        if first:
            x, z, y, saved, had_res = self._saved
            inp = dict(dy=dy.clone(), z=z.clone(), y=None if y is None else y.clone(), mean=saved.mean.clone(),
                       invstd=saved.invstd.clone(), pre=self._pre_reduced, had_res=had_res)
            g0, b0 = self.gamma.grad.clone(), self.beta.grad.clone()
        out = orig(self, dy, dx, accumulate, want_gres, dx_bn)
        if first:
            done.append(1)
            torch.cuda.synchronize()
            C = z.shape[-1]
            mode = (1 if inp["had_res"] else 2) if self.relu else 0
            dzc = torch.empty(inp["z"].shape)
            dgc, dbc = torch.zeros(C), torch.zeros(C)
            Fn.bn_backward(inp["dy"].cpu(), None if inp["y"] is None else inp["y"].cpu(), inp["z"].cpu(),
                           Fn.BNSaved(inp["mean"].cpu(), inp["invstd"].cpu()), self.gamma.data.cpu(),
                           self.beta.data.cpu(), mode, dgc, dbc, dzc, None)
            dg = (self.gamma.grad - g0).cpu()
            db = (self.beta.grad - b0).cpu()
            dzg = out[0] if isinstance(out, tuple) else out
            print(f"bf16_first={bf16_first} layer {self.name} pre_reduced={inp['pre']} mode={mode} "
                  f"dgamma rel {float((dg - dgc).norm() / dgc.norm()):.3e} dbeta rel {float((db - dbc).norm() / dbc.norm()):.3e}",
                  flush=True)
        return out

    L.ConvBN.backward = bwd
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    L.ConvBN.backward = orig


if __name__ == "__main__" and "--bn" in sys.argv:
    bnstage("--bf16-first" in sys.argv)


def refcheck(bf16_first):
    """does anything after the CPU step change the CPU model's gradients?"""
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    g0 = mc.ps.grad.clone()
    l0 = tc.row_loss.clone()
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    print(f"bf16_first={bf16_first}: cpu grads changed by later work: {not torch.equal(g0, mc.ps.grad)} "
          f"(max |diff| {float((g0 - mc.ps.grad).abs().max()):.3e}); gpu vs saved cpu grads rel "
          f"{float((mf.ps.grad.cpu() - g0).norm() / g0.norm()):.3e}; gpu vs current cpu grads rel "
          f"{float((mf.ps.grad.cpu() - mc.ps.grad).norm() / mc.ps.grad.norm()):.3e}; "
          f"loss cpu {float(l0.mean()):.7f} gpu {float(tf.row_loss.mean()):.7f}", flush=True)
    # a second CPU step on a fresh CPU model now
    mc2 = _shallow("cpu", **kw)
    tc2 = Trainer(mc2, 32, constant_lr(0.0), weight_decay=0.0)
    tc2._forward_backward(img_c, lab_c)
    print(f"   fresh CPU model now vs first CPU grads rel {float((mc2.ps.grad - g0).norm() / g0.norm()):.3e}; "
          f"vs gpu {float((mf.ps.grad.cpu() - mc2.ps.grad).norm() / mc2.ps.grad.norm()):.3e}", flush=True)


if __name__ == "__main__" and "--ref" in sys.argv:
    refcheck("--bf16-first" in sys.argv)


def both(bf16_first):
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    fg, fc = mf.ps.grad.cpu(), mc.ps.grad
    print(f"== bf16_first={bf16_first} flat rel {float((fg - fc).norm() / fc.norm()):.3e}")
    for pg, pc in zip(mf.ps.params, mc.ps.params):
        a = fg[pg.offset:pg.offset + pg.numel]
        b = fc[pc.offset:pc.offset + pc.numel]
        va, vb = pg.grad.float().cpu().flatten(), pc.grad.float().flatten()
        print(f"   {pg.name:38s} {pc.name:38s} off {pg.offset}/{pc.offset} slice-rel "
              f"{float((a - b).norm() / (b.norm() + 1e-30)):.2e} view-rel {float((va - vb).norm() / (vb.norm() + 1e-30)):.2e} "
              f"view==slice {torch.equal(va, a)}/{torch.equal(vb, b)}", flush=True)


if __name__ == "__main__" and "--both" in sys.argv:
    both("--bf16-first" in sys.argv)


def saved_stats(bf16_first):
    from azure_hc_intel_tf_amd.nn.layers import ConvBN
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward(img_c, lab_c)
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tf._forward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    print(f"== bf16_first={bf16_first}")
    for lf, lc in zip(mf.all_layers(), mc.all_layers()):
        if isinstance(lf, ConvBN) and lf.bn and lf._saved is not None and lc._saved is not None:
            sf, sc = lf._saved[3], lc._saved[3]
            zf, zc = lf._saved[1], lc._saved[1]
            r = lambda a, b: float((a.cpu().double() - b.double()).norm() / b.double().norm())
            print(f"   {lf.name:28s} z rel {r(zf, zc):.2e} mean rel {r(sf.mean, sc.mean):.2e} invstd rel {r(sf.invstd, sc.invstd):.2e}"
                  f" shift max {float(lf.shift.data.abs().max()) if lf.shift is not None else 0:.3e}", flush=True)


if __name__ == "__main__" and "--saved" in sys.argv:
    saved_stats("--bf16-first" in sys.argv)


def gapcheck(bf16_first):
    from azure_hc_intel_tf_amd.nn import layers as L
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    cap = {}
    og, ob = None, L.ConvBN.backward
    for cls in vars(L).values():
        if isinstance(cls, type) and issubclass(cls, L.Layer) and cls.__name__ in ("GlobalAvgPool", "GAP", "GlobalPool"):
            og = cls
    print("gap class", og)
    orig_g = og.backward

    def gb(self, dy):
        out = orig_g(self, dy)
        cap["dy"], cap["dx"], cap["hw"] = dy.double().clone(), out.double().clone(), self.in_shape[0] * self.in_shape[1]
        print("gap dtypes", dy.dtype, out.dtype, flush=True)
        return out

    og.backward = gb
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    og.backward = orig_g
    ref = (cap["dy"] / cap["hw"]).view(cap["dy"].shape[0], 1, 1, -1).expand_as(cap["dx"])
    print(f"bf16_first={bf16_first} gap bwd rel {float((cap['dx'] - ref).norm() / ref.norm()):.3e}", flush=True)


if __name__ == "__main__" and "--gap" in sys.argv:
    gapcheck("--bf16-first" in sys.argv)


def bncmp(bf16_first):
    """first BN backward of the step: the GPU fp32 run's inputs / outputs against the CPU run's"""
    from azure_hc_intel_tf_amd.nn import layers as L
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    orig = L.ConvBN.backward
    cap = {}

    def bwd(self, dy, dx=None, accumulate=False, want_gres=False, dx_bn=None):
        key = "gpu" if dy.is_cuda else "cpu"
        first = key not in cap and self.bn
        if first:
            x, z, y, saved, had_res = self._saved
            rec = dict(dy=dy.double().cpu().clone(), z=z.double().cpu().clone(),
                       y=None if y is None else y.double().cpu().clone(), name=self.name)
            g0, b0 = self.gamma.grad.clone(), self.beta.grad.clone()
        out = orig(self, dy, dx, accumulate, want_gres, dx_bn)
        if first:
            rec["dg"] = (self.gamma.grad - g0).double().cpu()
            rec["db"] = (self.beta.grad - b0).double().cpu()
            o = out[0] if isinstance(out, tuple) else out
            rec["dz"] = None if o is None else o.double().cpu().clone()
            cap[key] = rec
        return out

    L.ConvBN.backward = bwd
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    if bf16_first:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        cap.pop("gpu", None)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
        cap.pop("gpu", None)
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    L.ConvBN.backward = orig
    c, g = cap["cpu"], cap["gpu"]
    r = lambda a, b: float((a - b).norm() / (b.norm() + 1e-30))
    print(f"bf16_first={bf16_first} layer cpu {c['name']} gpu {g['name']}: dy {r(g['dy'], c['dy']):.2e} z {r(g['z'], c['z']):.2e} "
          f"y {r(g['y'], c['y']) if c['y'] is not None else -1:.2e} -> dgamma {r(g['dg'], c['dg']):.2e} dbeta {r(g['db'], c['db']):.2e} "
          f"dz {r(g['dz'], c['dz']) if c['dz'] is not None and g['dz'] is not None else -1:.2e}", flush=True)
    if c["y"] is not None:
        mc_ = (c["y"] > 0) != (g["y"] > 0)
        print(f"   relu mask flips: {int(mc_.sum())} of {mc_.numel()}; y==0 count cpu {int((c['y'] == 0).sum())} gpu {int((g['y'] == 0).sum())}")


if __name__ == "__main__" and "--bncmp" in sys.argv:
    bncmp("--bf16-first" in sys.argv)
