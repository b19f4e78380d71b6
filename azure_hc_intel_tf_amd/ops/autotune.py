"""Per-shape kernel configuration autotuning for the implicit-GEMM convolutions (the
``cudnn.benchmark`` / MIOpen find-db role, done for our own kernels).

For every distinct GEMM problem of a model (forward conv, data-grad conv, weight-grad conv)
each candidate block-tile configuration (and split-K factor for weight gradients) is timed
with HIP events on scratch buffers of the real shapes, and the fastest is recorded. The
table is cached in JSON (``tuned/<arch>.json``, shipped in-tree so a multi-GPU run does not
re-tune) and consulted by ``functional.conv_cfg`` / ``functional.wgrad_cfg``.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Tuple

import torch

from . import _ext
from . import functional as Fn

_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned")
# HCB_TUNED_TABLE: another table file (A/B timing of two tunings on one box)
DEFAULT_CACHE = os.environ.get("HCB_TUNED_TABLE") or os.path.join(_DIR, "mi355x.json")
# bump whenever the kernel config set changes: entries of another version are re-tuned
CACHE_VERSION = 5  # 5: keys carry the filter tap count


def _key_str(k) -> str:
    return "|".join(str(v) for v in k)


def _key_parse(s: str):
    parts = s.split("|")
    return (parts[0],) + tuple(int(p) for p in parts[1:])


def load_cache(path: str = DEFAULT_CACHE) -> int:
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        d = json.load(f)
    if d.get("version") != CACHE_VERSION:
        return 0
    table = {}
    for k, v in d.get("entries", {}).items():
        table[_key_parse(k)] = tuple(v) if isinstance(v, list) else v
    Fn.set_tuned(table)
    return len(table)


def save_cache(path: str = DEFAULT_CACHE) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
        if d.get("version") == CACHE_VERSION:
            old = d.get("entries", {})
    for k, v in Fn._tuned.items():
        old[_key_str(k)] = list(v) if isinstance(v, tuple) else v
    with open(path, "w") as f:
        json.dump({"arch": "gfx950", "version": CACHE_VERSION, "entries": old}, f, indent=0, sort_keys=True)


_SCRATCH = {}
# per-launch isolated timing (module switch): each candidate launch timed on its own after a 64 MB
# eviction write, median of the launches. Measured against the default back-to-back timing:
# +0.3% step (within run-to-run noise), equal with the KU=2 configs offered (profiles/r3x_ku2_cache_ab.txt)
TUNE_ISOLATE = os.environ.get("HCB_TUNE_ISOLATE", "0") == "1"


def _time(fn, reps=None) -> float:
    # HCB_TUNE_REPS: timed launches per candidate (default 20; a 20-launch fp32 retune ran the step
    # 1.3% faster than the 5-launch one, interleaved A/B: profiles/r4rt_fp32_retune_reps.txt)
    reps = reps or int(os.environ.get("HCB_TUNE_REPS", "20"))
    fn()
    if TUNE_ISOLATE:
        # step-like timing: each launch timed on its own, after a 64 MB write that evicts the
        # candidate's operands from L2 and ends any overlap with the previous launch (back-to-back
        # launches of one kernel favour configs the training step does not: profiles/r3x_ku2_cache_ab.txt)
        buf = _SCRATCH.get("buf")
        if buf is None:
            buf = _SCRATCH["buf"] = torch.empty(16 << 20, dtype=torch.float32, device="cuda")
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s, e in ev:
            buf.fill_(1.0)
            s.record()
            fn()
            e.record()
        ev[-1][1].synchronize()
        return sorted(s.elapsed_time(e) for s, e in ev)[reps // 2]
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def _act():
    """16-bit activation dtype of the kernel library being tuned (bf16 / IEEE-fp16 build)."""
    from ..nn.layers import act_dtype

    return act_dtype("cuda")


def _bf(shape, dev):
    return torch.randn(shape, device=dev).to(_act())


def tune_conv_layer(layer, batch: int, dev, verbose=False) -> List[Tuple]:
    """Tune fwd / dgrad / wgrad problems of one ConvBN layer (skips already-tuned keys)."""
    hcb = _ext.ops()
    spec = layer.spec
    H, W, Cin = layer.in_shape
    P, Q, Cout = layer.out_shape
    N = batch
    out = []
    M = N * P * Q
    geo = Fn.dgrad_problem(spec, N, H, W, P, Q)
    taps = spec.kh * spec.kw
    keys = [Fn.fwd_key(M, Cout, spec.K, taps), Fn.wgrad_key(Cout, spec.K, M, taps)]
    phases = Fn.dgrad_phases(spec, H, W) if layer.need_dx and Fn.uses_dgrad_phases(spec, H, W) else []
    if layer.need_dx:
        keys.append(Fn.fwd_key(geo[0], Cin, geo[1], taps))
        keys.append(Fn.dgb_key(geo[0], Cin, geo[1], taps))
    for ph in phases:  # the stride-phase GEMMs of a strided k x k data gradient
        pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
        keys += [Fn.fwd_key(pm, Cin, pk, pt), Fn.dgb_key(pm, Cin, pk, pt)]
    if all(k in Fn._tuned for k in keys):
        return out
    x = _bf((N, H, W, Cin), dev)
    dz = _bf((N, P, Q, Cout), dev)
    # forward
    k = Fn.fwd_key(M, Cout, spec.K, taps)
    if k not in Fn._tuned:
        y = torch.empty((N, P, Q, Cout), dtype=_act(), device=dev)
        best = None
        acc = torch.zeros(8 * 2 * Cout, dtype=torch.float32, device=dev)
        for cfg in Fn.fwd_candidates(Cout, Fn.patch_eligible(spec)):
            for sp in Fn.splitk_candidates(cfg, M, Cout, spec.K):
                plan = cfg if sp == 1 else [cfg, sp]
                t = _time(lambda: Fn.conv_forward(x, spec, layer.pack.pack, None, y, stats=acc, cfg=plan,
                                                  stats_R=8))
                if best is None or t < best[0]:
                    best = (t, plan)
        Fn._tuned[k] = best[1]
        out.append((k, best))
    # data gradient
    if layer.need_dx:
        dx = torch.zeros((N, H, W, Cin), dtype=_act(), device=dev)
        dpatch = Fn.patch_eligible(spec, dgrad=True) and not phases
        k = Fn.fwd_key(geo[0], Cin, geo[1], taps)
        if k not in Fn._tuned:
            best = None
            for cfg in Fn.fwd_candidates(Cin, dpatch):
                for sp in Fn.splitk_candidates(cfg, geo[0], Cin, geo[1]):
                    plan = cfg if sp == 1 else [cfg, sp]
                    t = _time(lambda: Fn.conv_dgrad(dz, spec, layer.pack.tr, None, dx, False, cfg=plan))
                    if best is None or t < best[0]:
                        best = (t, plan)
            Fn._tuned[k] = best[1]
            out.append((k, best))
        # the same GEMM with the fused BN-backward epilogue (ReLU mask from y, residual
        # beta-accumulate: the heaviest epilogue), used when a BN layer consumes this dx
        k = Fn.dgb_key(geo[0], Cin, geo[1], taps)
        if k not in Fn._tuned:
            z = _bf((N, H, W, Cin), dev)
            yv = _bf((N, H, W, Cin), dev)
            stats = [torch.rand(Cin, device=dev) + 0.5 for _ in range(4)]
            bacc = torch.zeros(8 * 2 * Cin, dtype=torch.float32, device=dev)
            bnb = Fn.BNBwdFuse(z, yv, Fn.BNSaved(stats[0], stats[1]), stats[2], stats[3], 1, bacc, 8)
            best = None
            for cfg in Fn.fwd_candidates(Cin, dpatch):
                for sp in Fn.splitk_candidates(cfg, geo[0], Cin, geo[1]):
                    plan = cfg if sp == 1 else [cfg, sp]
                    t = _time(lambda: Fn.conv_dgrad(dz, spec, layer.pack.tr, None, dx, True, cfg=plan, bnb=bnb))
                    if best is None or t < best[0]:
                        best = (t, plan)
            Fn._tuned[k] = best[1]
            out.append((k, best))
        for ph in phases:
            pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
            for fused in (False, True):
                k = (Fn.dgb_key if fused else Fn.fwd_key)(pm, Cin, pk, pt)
                if k in Fn._tuned:
                    continue
                bnbp = None
                if fused:
                    z = _bf((N, H, W, Cin), dev)
                    yv = _bf((N, H, W, Cin), dev)
                    st = [torch.rand(Cin, device=dev) + 0.5 for _ in range(4)]
                    bnbp = Fn.BNBwdFuse(z, yv, Fn.BNSaved(st[0], st[1]), st[2], st[3], 1,
                                        torch.zeros(8 * 2 * Cin, dtype=torch.float32, device=dev), 8)
                best = None
                for cfg in Fn.fwd_candidates(Cin):
                    for sp in Fn.splitk_candidates(cfg, pm, Cin, pk):
                        plan = cfg if sp == 1 else [cfg, sp]
                        t = _time(lambda: Fn.dgrad_phase(dz, spec, layer.pack.tr, dx, fused, ph, cfg=plan, bnb=bnbp))
                        if best is None or t < best[0]:
                            best = (t, plan)
                Fn._tuned[k] = best[1]
                out.append((k, best))
    # weight gradient
    k = Fn.wgrad_key(Cout, spec.K, M, taps)
    if k not in Fn._tuned:
        dw = torch.zeros((Cout, spec.K), dtype=torch.float32, device=dev)
        best = None
        for cfg, splits in Fn.wgrad_candidates(Cout, spec.K, M):
            t = _time(lambda: Fn.conv_wgrad(dz, x, spec, dw, cfg=(cfg, splits)))
            if best is None or t < best[0]:
                best = (t, (cfg, splits))
        Fn._tuned[k] = best[1]
        out.append((k, best))
    if verbose:
        for kk, (t, c) in out:
            print(f"  tuned {kk}: cfg={c} {t * 1000:.1f} us")
    return out


def _planes(shape, dev):
    return Fn.Planes(torch.randn((3,) + tuple(shape), device=dev).to(torch.bfloat16))


def _best(cands, run):
    best = None
    for plan in cands:
        t = _time(lambda: run(plan))
        if best is None or t < best[0]:
            best = (t, plan)
    return best


def tune_conv_layer_p3(layer, batch: int, dev, verbose=False) -> List[Tuple]:
    """fp32 path: tune the bf16-plane GEMMs (conv_p3.hip) of one ConvBN layer -- forward, data
    gradient (or its stride phases), weight gradient -- over their own tile / split-K sets."""
    spec = layer.spec
    H, W, Cin = layer.in_shape
    P, Q, Cout = layer.out_shape
    N = batch
    M = N * P * Q
    taps = spec.kh * spec.kw
    geo = Fn.dgrad_problem(spec, N, H, W, P, Q)
    phases = Fn.dgrad_phases(spec, H, W) if layer.need_dx and Fn.uses_dgrad_phases(spec, H, W) else []
    keys = [Fn.fwd3_key(M, Cout, spec.K, taps), Fn.wgrad3_key(Cout, spec.K, M, taps)]
    if layer.need_dx and not phases:
        keys.append(Fn.fwd3_key(geo[0], Cin, geo[1], taps))
    for ph in phases:
        pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
        keys.append(Fn.fwd3_key(pm, Cin, pk, pt))
    out = []
    if all(k in Fn._tuned for k in keys):
        return out
    x = _planes((N, H, W, Cin), dev)
    dz = _planes((N, P, Q, Cout), dev)
    k = keys[0]
    if k not in Fn._tuned:
        y = torch.empty((N, P, Q, Cout), dtype=torch.float32, device=dev)
        acc = torch.zeros(8 * 2 * Cout, dtype=torch.float32, device=dev)
        best = _best(Fn.p3_candidates(M, Cout, spec.K),
                     lambda plan: Fn.conv_forward(x, spec, layer.pack.pack, None, y, stats=acc, cfg=plan, stats_R=8))
        Fn._tuned[k] = list(best[1])
        out.append((k, best))
    if layer.need_dx:
        dx = torch.zeros((N, H, W, Cin), dtype=torch.float32, device=dev)
        if not phases:
            k = Fn.fwd3_key(geo[0], Cin, geo[1], taps)
            if k not in Fn._tuned:
                best = _best(Fn.p3_candidates(geo[0], Cin, geo[1]),
                             lambda plan: Fn.conv_dgrad(dz, spec, layer.pack.tr, None, dx, False, cfg=plan))
                Fn._tuned[k] = list(best[1])
                out.append((k, best))
        for ph in phases:
            pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
            k = Fn.fwd3_key(pm, Cin, pk, pt)
            if k in Fn._tuned:
                continue
            best = _best(Fn.p3_candidates(pm, Cin, pk),
                         lambda plan: Fn.dgrad_phase(dz, spec, layer.pack.tr, dx, True, ph, cfg=plan))
            Fn._tuned[k] = list(best[1])
            out.append((k, best))
    k = Fn.wgrad3_key(Cout, spec.K, M, taps)
    if k not in Fn._tuned:
        dw = torch.zeros((Cout, spec.K), dtype=torch.float32, device=dev)
        best = _best(Fn.wgrad_p3_candidates(Cout, spec.K, M), lambda plan: Fn.conv_wgrad(dz, x, spec, dw, cfg=plan))
        Fn._tuned[k] = list(best[1])
        out.append((k, best))
    if verbose:
        for kk, (t, c) in out:
            print(f"  tuned {kk}: cfg={c} {t * 1000:.1f} us")
    return out


def tune_model(model, batch: int, verbose=False, cache: str = DEFAULT_CACHE, save=True) -> int:
    from ..nn.layers import ConvBN

    dev = model.device
    model.ps.repack()
    n = 0
    p3 = getattr(model, "compute_dtype", None) == "fp32" and model.native
    if hasattr(model, "activate"):
        model.activate()
    for l in model.all_layers():
        if isinstance(l, ConvBN) and l.bn:
            view = l.tune_view() if hasattr(l, "tune_view") else l
            n += len((tune_conv_layer_p3 if p3 else tune_conv_layer)(view, batch, dev, verbose))
    torch.cuda.synchronize()
    if save and n and cache:
        try:
            save_cache(cache)
        except OSError:
            pass
    return n
