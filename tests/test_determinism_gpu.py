"""Opt-in deterministic GPU training (HCB_DETERMINISTIC / functional.set_deterministic): two
fresh runs from the same seed give bitwise-equal weights and losses; and a shallow net's
hand-written GPU gradients compared elementwise against the fp32 CPU path."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model, resnet
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def _run(steps=4, size=96, batch=16, lr=0.05):
    torch.manual_seed(0)
    m = create_model("resnet50", image_size=size, device="cuda", seed=21, compute_dtype="bf16")
    img, lab = synthetic_batch(m, batch, seed=3)
    t = Trainer(m, batch, constant_lr(lr), use_graph=True, graph_warmup=1)
    tr = torch.zeros(steps, device="cuda")
    for i in range(steps):
        tr[i:i + 1].copy_(t.step(img, lab))
    torch.cuda.synchronize()
    return m.ps.master.clone(), t.row_loss.clone(), tr


def test_deterministic_mode_is_bitwise_reproducible():
    Fn.set_deterministic(True)
    try:
        w1, l1, tr1 = _run()
        w2, l2, tr2 = _run()
    finally:
        Fn.set_deterministic(False)
    assert torch.isfinite(tr1).all()
    assert torch.equal(l1, l2), "per-row losses differ between identical deterministic runs"
    assert torch.equal(w1, w2), f"{int((w1 != w2).sum())} weights differ between identical deterministic runs"


def test_deterministic_mode_trains_like_default():
    """Deterministic mode changes only the ORDER of fp32 sums (no split-K, one accumulator slot per
    tile), so its trajectory must look like one more default-mode run. The bound is the run-to-run
    spread of the default mode itself, measured here (4 runs: their atomics reorder between runs),
    not an observed constant: this tiny-batch bf16 net amplifies any rounding-order difference
    chaotically (a 1-ulp change of the stem BN's coefficients moved step 3 by ~4%:
    profiles/r5_stem_prologue_determinism.txt), and a fixed 3% band failed correct code."""
    Fn.set_deterministic(True)
    try:
        _, _, trd = _run(steps=6, lr=0.01)
    finally:
        Fn.set_deterministic(False)
    runs = torch.stack([_run(steps=6, lr=0.01)[2] for _ in range(4)]).cpu()
    trd = trd.cpu()
    lo, hi = runs.min(0).values, runs.max(0).values
    band = 2.0 * (hi - lo) + 2e-3 * hi.abs()
    assert bool(((trd >= lo - band) & (trd <= hi + band)).all()), (trd.tolist(), runs.tolist())
    # the first steps, before the chaos has amplified anything, against a tight fixed bound (a
    # regression of the deterministic split-K / statistics path shows up here, whatever the band):
    # step 0 is the forward of identical weights (only the fp32 summation order differs; bf16
    # activations turn a reordered sum into an occasional 1-ulp flip: the default runs spread by up
    # to ~3e-3 at step 0 on this 4-image batch, and the deterministic run -- bitwise the same every
    # time, 7.59103 -- sat 1.2e-3 above a tightly clustered set of default runs once): 3e-3 of their
    # mean, or their own spread if larger
    mean = runs.mean(0)
    tol0 = max(3e-3 * abs(float(mean[0])), float(hi[0] - lo[0]))
    assert abs(float(trd[0] - mean[0])) <= tol0, (trd.tolist(), runs.tolist())
    assert abs(float(trd[1] - mean[1])) <= 3e-2 * abs(float(mean[1])), (trd.tolist(), runs.tolist())
    # (a stable learning rate: at 0.05 this tiny-batch run diverges)
    assert float(trd[-1]) < float(trd[0]) - 2.0 and float(runs[:, -1].max()) < float(runs[:, 0].min()) - 2.0


def _shallow(device, **kw):
    resnet.LAYER_COUNTS.setdefault(1, (1,))  # stem + max pool + ONE bottleneck block + classifier
    if str(device).startswith("cuda"):
        kw.setdefault("compute_dtype", "bf16")  # the 16-bit path (create_model defaults to fp32)
    return resnet.ResNet(depth=1, device=device, **kw)


def _grad_errors(mg, mc):
    out = []
    for pg, pc in zip(mg.ps.params, mc.ps.params):
        a, b = pg.grad.float().cpu().flatten(), pc.grad.float().flatten()
        if pg.name.startswith("conv0/conv2d"):  # compare the 3 real input channels only
            a, b = pg.grad[..., :3].float().cpu().flatten(), pc.grad[..., :3].float().flatten()
        scale = b.abs().max().item()
        if scale == 0:
            assert a.abs().max().item() == 0, pg.name
            continue
        err = (a - b).abs().max().item() / scale
        rel = ((a - b).norm() / b.norm()).item()
        cos = float(a @ b / (a.norm() * b.norm()))
        out.append((round(err, 5), round(rel, 5), round(cos, 6), pg.name))
    return out


def test_shallow_net_gradients_elementwise_vs_fp32_cpu():
    """Stem + one bottleneck block: every parameter gradient of the GPU backward against the
    fp32 CPU path, element by element (max error scaled by each tensor's largest gradient).

    * The fp32 reference-precision GPU path must agree to fp32 rounding: 1e-6-level relative
      errors (measured 1e-7..5e-6 per tensor). It is only bounded at 5e-3 / cosine 0.99999 because
      ReLU is discontinuous: the block output holds ~262k exact zeros, and ONE element whose
      pre-activation lies within fp32 rounding of 0 can land on the other side of the mask than in
      the CPU run (it depends on the fp32 atomic order of the BN statistics); that single flip
      shifts the first BN backward's dgamma by 4e-4 and, through the BN mean subtraction, every
      earlier gradient by ~1.8e-3 (tools/diag_fp32_shallow.py --bncmp: "relu mask flips: 1 of
      524288"). A real fp32 defect (e.g. a two-term bf16 split, 2^-17) shows up as >1e-2.
    * The hand-written bf16 path (bf16 activations, fused BN epilogues, space-to-depth stem):
      measured on MI355X the error grows with backward depth -- classifier 0.3 %, block
      conv3 / BN 1.5 %, conv2 ~10 %, conv1 / stem ~12-15 % of the largest gradient, every tensor
      at cosine >= 0.99 -- the bf16 rounding of activations and of dy amplified by each BN
      backward's mean subtraction (and max-pool argmax ties that bf16 rounding flips)."""
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mg, mc = _shallow("cuda", **kw), _shallow("cpu", **kw)
    mf = _shallow("cuda", compute_dtype="fp32", **kw)
    assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    tc._forward_backward(img_c, lab_c)
    torch.cuda.synchronize()
    assert abs(tg.row_loss.mean().item() - tc.row_loss.mean().item()) < 0.02
    tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0)
    tf._forward_backward(img_c.cuda(), lab_c.cuda())
    torch.cuda.synchronize()
    for err, rel, cos, name in _grad_errors(mf, mc):
        print("fp32 GPU grad check", err, rel, cos, name)
        assert rel < 5e-3 and err < 5e-2 and cos > 0.99999, (name, err, rel, cos)
    for err, rel, cos, name in _grad_errors(mg, mc):
        print("bf16 GPU grad check", err, rel, cos, name)
        assert err < 0.25 and rel < 0.2 and cos > 0.985, (name, err, rel, cos)


def test_bf16_gradients_within_the_autocast_floor():
    """The bf16 gradient-accuracy floor (tools/bf16_floor.py): the shallow net through a plain
    torch.nn.functional mirror under torch.autocast(bfloat16) (MIOpen, channels_last) against
    the fp32 CPU step gives each parameter's bf16-pipeline error; the hand-written bf16 path
    (bf16 activations, fused BN epilogues, space-to-depth stem) must stay within 1.5x of it
    per tensor. The fp32 run of the mirror pins the mirror itself. Measured on MI355X: ratios
    0.67-1.05 (profiles/r3_bf16_grad_floor.txt)."""
    import sys
    import os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import bf16_floor as BF

    mc = BF.shallow("cpu")
    img_c, lab_c = synthetic_batch(mc, BF.BATCH, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, BF.BATCH, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    ref = {p.name: p.grad.float().clone() for p in mc.ps.params}
    params = {p.name: p.data.clone() for p in mc.ps.params}
    mg = BF.shallow("cuda")
    tg = Trainer(mg, BF.BATCH, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    torch.cuda.synchronize()
    hip = {p.name: p.grad.float().cpu() for p in mg.ps.params}
    f32, _ = BF.mirror_grads(params, img_c, lab_c, "cuda", autocast=False)
    ac, _ = BF.mirror_grads(params, img_c, lab_c, "cuda", autocast=True)
    for name, r in ref.items():
        sl = (lambda t: t[..., :3]) if name.startswith("conv0/conv2d") else (lambda t: t)
        e32, eac, ehip = (BF.rel(sl(d[name]).flatten(), sl(r).flatten()) for d in (f32, ac, hip))
        print("bf16 floor", name, e32, eac, ehip, ehip / eac)
        # the fp32 mirror pins the MIRROR (not the HIP kernels): it only has to sit an order of
        # magnitude below the bf16 floor it calibrates. No absolute bound: MIOpen's fp32 algorithm
        # choice varies by box (1.8e-3 on the stem weight gradient on one box, < 1e-4 on others)
        assert e32 < 0.1 * eac, (name, e32, eac)
        assert ehip < 1.5 * eac, (name, ehip, eac)
