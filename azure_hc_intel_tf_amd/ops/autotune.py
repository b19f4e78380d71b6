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
# HCB_TUNED_TABLE: another table file (A/B timing of two tunings on one box); a relative path that
# does not exist from the working directory is taken from the repository root (tools that run the
# bench from another directory, e.g. rocprofv3 under /tmp, would otherwise silently re-tune)


def _table_path(v):
    if not v or os.path.isabs(v) or os.path.exists(v):
        return v
    alt = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), v)
    return alt if os.path.exists(alt) else v


DEFAULT_CACHE = _table_path(os.environ.get("HCB_TUNED_TABLE")) or os.path.join(_DIR, "mi355x.json")
# bump whenever the kernel config set changes: entries of another version are re-tuned
CACHE_VERSION = 6  # 5: keys carry the filter tap count; 6: round-5 pruned cfgs / stream-K plans gone


def _entry_valid(key, val) -> bool:
    """A cached plan whose cfg the current kernel set still has (and splits >= 1): entries of
    removed configs would otherwise fall through to a kernel's default launcher, untuned."""
    tiles = {"fwd": Fn._CONV_TILES, "dgb": Fn._CONV_TILES, "wgrad": Fn._WGRAD_TILES, "fwd3": Fn._P3_TILES,
             "wgrad3": Fn._WP3_TILES}.get(key[0])
    cfg, splits = (val[0], val[1]) if isinstance(val, (tuple, list)) else (val, 1)
    return tiles is not None and int(cfg) in tiles and int(splits) >= 1


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
        key, val = _key_parse(k), tuple(v) if isinstance(v, list) else v
        if _entry_valid(key, val):
            table[key] = val
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


def _plans(cfgs_splits):
    return [c if sp == 1 else [c, sp] for c, sp in cfgs_splits]


def layer_problems(layer, batch: int, dev) -> List[Tuple]:
    """The GEMM problems of one ConvBN layer on the 16-bit kernels: (key, candidate plans, run(plan))
    for the forward, the data gradient (plain and with the fused BN-backward epilogue, or the
    stride-phase GEMMs of a strided k x k data gradient) and the weight gradient. Scratch operands
    of the real shapes are made once per layer, when the first run is called."""
    spec = layer.spec
    H, W, Cin = layer.in_shape
    P, Q, Cout = layer.out_shape
    N = batch
    M = N * P * Q
    geo = Fn.dgrad_problem(spec, N, H, W, P, Q)
    taps = spec.kh * spec.kw
    phases = Fn.dgrad_phases(spec, H, W) if layer.need_dx and Fn.uses_dgrad_phases(spec, H, W) else []
    buf = {}

    def ops():
        if not buf:
            buf["x"] = _bf((N, H, W, Cin), dev)
            buf["dz"] = _bf((N, P, Q, Cout), dev)
            buf["y"] = torch.empty((N, P, Q, Cout), dtype=_act(), device=dev)
            buf["acc"] = torch.zeros(8 * 2 * Cout, dtype=torch.float32, device=dev)
            buf["dx"] = torch.zeros((N, H, W, Cin), dtype=_act(), device=dev)
            buf["dw"] = torch.zeros((Cout, spec.K), dtype=torch.float32, device=dev)
            z, yv = _bf((N, H, W, Cin), dev), _bf((N, H, W, Cin), dev)
            st = [torch.rand(Cin, device=dev) + 0.5 for _ in range(4)]
            buf["bnb"] = Fn.BNBwdFuse(z, yv, Fn.BNSaved(st[0], st[1]), st[2], st[3], 1,
                                      torch.zeros(8 * 2 * Cin, dtype=torch.float32, device=dev), 8)
        return buf

    out = []
    fc = Fn.fwd_candidates(Cout, Fn.patch_eligible(spec))
    out.append((Fn.fwd_key(M, Cout, spec.K, taps),
                _plans((c, sp) for c in fc for sp in Fn.splitk_candidates(c, M, Cout, spec.K)),
                lambda plan: Fn.conv_forward(ops()["x"], spec, layer.pack.pack, None, ops()["y"], stats=ops()["acc"],
                                             cfg=plan, stats_R=8)))
    if layer.need_dx:
        dpatch = Fn.patch_eligible(spec, dgrad=True) and not phases
        dc = _plans((c, sp) for c in Fn.fwd_candidates(Cin, dpatch)
                    for sp in Fn.splitk_candidates(c, geo[0], Cin, geo[1]))
        out.append((Fn.fwd_key(geo[0], Cin, geo[1], taps), dc,
                    lambda plan: Fn.conv_dgrad(ops()["dz"], spec, layer.pack.tr, None, ops()["dx"], False, cfg=plan)))
        # the same GEMM with the fused BN-backward epilogue (ReLU mask from y, residual
        # beta-accumulate: the heaviest epilogue), used when a BN layer consumes this dx
        out.append((Fn.dgb_key(geo[0], Cin, geo[1], taps), dc,
                    lambda plan: Fn.conv_dgrad(ops()["dz"], spec, layer.pack.tr, None, ops()["dx"], True, cfg=plan,
                                               bnb=ops()["bnb"])))
        for ph in phases:
            pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
            pc = _plans((c, sp) for c in Fn.fwd_candidates(Cin) for sp in Fn.splitk_candidates(c, pm, Cin, pk))
            for fused in (False, True):
                out.append(((Fn.dgb_key if fused else Fn.fwd_key)(pm, Cin, pk, pt), pc,
                            lambda plan, ph=ph, fused=fused: Fn.dgrad_phase(
                                ops()["dz"], spec, layer.pack.tr, ops()["dx"], fused, ph, cfg=plan,
                                bnb=ops()["bnb"] if fused else None)))
    out.append((Fn.wgrad_key(Cout, spec.K, M, taps), [(c, s) for c, s in Fn.wgrad_candidates(Cout, spec.K, M)],
                lambda plan: Fn.conv_wgrad(ops()["dz"], ops()["x"], spec, ops()["dw"], cfg=tuple(plan))))
    return out


def _planes(shape, dev):
    return Fn.Planes(torch.randn((3,) + tuple(shape), device=dev).to(torch.bfloat16))


def layer_problems_p3(layer, batch: int, dev) -> List[Tuple]:
    """fp32 path: the bf16-plane GEMMs (conv_p3.hip) of one ConvBN layer -- forward, data gradient
    (or its stride phases, with the fused BN-backward epilogue), weight gradient -- as (key,
    candidate plans, run(plan)) over their own tile / split-K sets."""
    spec = layer.spec
    H, W, Cin = layer.in_shape
    P, Q, Cout = layer.out_shape
    N = batch
    M = N * P * Q
    taps = spec.kh * spec.kw
    geo = Fn.dgrad_problem(spec, N, H, W, P, Q)
    phases = Fn.dgrad_phases(spec, H, W) if layer.need_dx and Fn.uses_dgrad_phases(spec, H, W) else []
    buf = {}

    def ops():
        if not buf:
            buf["x"] = _planes((N, H, W, Cin), dev)
            buf["dz"] = _planes((N, P, Q, Cout), dev)
            buf["y"] = torch.empty((N, P, Q, Cout), dtype=torch.float32, device=dev)
            buf["acc"] = torch.zeros(8 * 2 * Cout, dtype=torch.float32, device=dev)
            buf["dx"] = torch.zeros((N, H, W, Cin), dtype=torch.float32, device=dev)
            buf["dw"] = torch.zeros((Cout, spec.K), dtype=torch.float32, device=dev)
        return buf

    out = [(Fn.fwd3_key(M, Cout, spec.K, taps), [list(c) for c in Fn.p3_candidates(M, Cout, spec.K)],
            lambda plan: Fn.conv_forward(ops()["x"], spec, layer.pack.pack, None, ops()["y"], stats=ops()["acc"],
                                         cfg=plan, stats_R=8))]
    if layer.need_dx:
        if not phases:
            out.append((Fn.fwd3_key(geo[0], Cin, geo[1], taps), [list(c) for c in Fn.p3_candidates(geo[0], Cin, geo[1])],
                        lambda plan: Fn.conv_dgrad(ops()["dz"], spec, layer.pack.tr, None, ops()["dx"], False,
                                                   cfg=plan)))
        for ph in phases:
            pm, pk, pt = Fn.dgrad_phase_problem(spec, N, ph)
            out.append((Fn.fwd3_key(pm, Cin, pk, pt), [list(c) for c in Fn.p3_candidates(pm, Cin, pk)],
                        lambda plan, ph=ph: Fn.dgrad_phase(ops()["dz"], spec, layer.pack.tr, ops()["dx"], True, ph,
                                                           cfg=plan)))
    out.append((Fn.wgrad3_key(Cout, spec.K, M, taps), [list(c) for c in Fn.wgrad_p3_candidates(Cout, spec.K, M)],
                lambda plan: Fn.conv_wgrad(ops()["dz"], ops()["x"], spec, ops()["dw"], cfg=tuple(plan))))
    return out


def _best(cands, run):
    best = None
    for plan in cands:
        t = _time(lambda: run(plan))
        if best is None or t < best[0]:
            best = (t, plan)
    return best


def model_problems(model, batch: int):
    """Every distinct conv GEMM problem of a model: {key: [count, candidates, run]} in layer
    order (count = how many layers of the step launch that problem)."""
    from ..nn.layers import ConvBN

    p3 = getattr(model, "compute_dtype", None) == "fp32" and model.native
    probs = {}
    for l in model.all_layers():
        if isinstance(l, ConvBN) and l.bn:
            view = l.tune_view() if hasattr(l, "tune_view") else l
            for key, cands, run in (layer_problems_p3 if p3 else layer_problems)(view, batch, model.device):
                if key in probs:
                    probs[key][0] += 1
                else:
                    probs[key] = [1, cands, run]
    return probs


def tune_conv_layer(layer, batch: int, dev, verbose=False) -> List[Tuple]:
    """Tune the untuned GEMM problems of one ConvBN layer (isolated launches of each candidate)."""
    out = []
    for key, cands, run in layer_problems(layer, batch, dev):
        if key in Fn._tuned:
            continue
        best = _best(cands, run)
        Fn._tuned[key] = best[1]
        out.append((key, best))
    if verbose:
        for kk, (t, c) in out:
            print(f"  tuned {kk}: cfg={c} {t * 1000:.1f} us")
    return out


def tune_conv_layer_p3(layer, batch: int, dev, verbose=False) -> List[Tuple]:
    """fp32 path: tune the untuned bf16-plane GEMM problems of one ConvBN layer."""
    out = []
    for key, cands, run in layer_problems_p3(layer, batch, dev):
        if key in Fn._tuned:
            continue
        best = _best(cands, run)
        Fn._tuned[key] = list(best[1])
        out.append((key, best))
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
