#!/usr/bin/env python3
"""Wave quantization of the fp32 step's plane GEMMs ("first, measure"), from the
tuned table alone (CPU, no GPU needed):

    python tools/quant_report.py [--model resnet50] [--batch 64] [--table path]

For every conv GEMM launch of one training step (forward, data gradient or its stride phases,
weight gradient) the plan the step uses (cfg, split-K) gives

    tiles   = ceil(M / BM) * ceil(N / BN) * splits     (work items of the launch)
    slots   = 256 CUs x workgroups per CU the cfg is built for
    rounds  = ceil(tiles / slots)
    fill    = tiles / (rounds * slots)                   (1.0 = every slot busy every round)

A persistent cfg walks its tiles with a grid of min(tiles, slots) workgroups: same rounds / fill.
``ideal`` is the fraction of the launch's time an ideally balanced schedule of the same per-tile
cost would save: 1 - fill. The table is sorted by FLOP-weighted idle share.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from azure_hc_intel_tf_amd.models import create_model  # noqa: E402
from azure_hc_intel_tf_amd.nn.layers import ConvBN  # noqa: E402
from azure_hc_intel_tf_amd.ops import autotune  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402
from azure_hc_intel_tf_amd.ops.functional import ConvSpec  # noqa: E402

N_CU = 256


def fwd_geom(cfg):
    bm, bn = Fn._P3_TILES[cfg]
    return bm, bn, Fn._P3_OCC.get(cfg, 1), cfg in Fn._P3_PERSIST


def wgrad_geom(cfg):
    bm, bn = Fn._WP3_TILES[cfg]
    return bm, bn, Fn._WP3_OCC.get(cfg, 1), cfg >= 16


def row(kind, name, M, N, K, plan, geom, flop):
    cfg, splits = plan
    bm, bn, occ, persist = geom(cfg)
    tiles = math.ceil(M / bm) * math.ceil(N / bn) * splits
    slots = N_CU * occ
    rounds = math.ceil(tiles / slots)
    fill = tiles / (rounds * slots)
    return dict(kind=kind, name=name, M=M, N=N, K=K, cfg=cfg, splits=splits, tile=f"{bm}x{bn}", occ=occ,
                persist=persist, tiles=tiles, slots=slots, rounds=rounds, fill=fill, flop=flop)


def problems(model, batch):
    out = []
    for l in model.all_layers():
        if not (isinstance(l, ConvBN) and l.bn):
            continue
        spec = l.spec
        H, W, Cin = l.in_shape
        P, Q, Cout = l.out_shape
        taps = spec.kh * spec.kw
        name = l.name
        if name == "conv0":  # the GPU stem: the S2D fold read as a 4x1 conv over 64-channel row windows
            spec = ConvSpec(cin=64, cin_pad=64, cout=Cout, kh=4, kw=1)
            taps = 4
        M = batch * P * Q
        flop = 2.0 * M * Cout * spec.K
        out.append(row("fwd", name, M, Cout, spec.K, Fn.p3_plan(M, Cout, spec.K, taps), fwd_geom, flop))
        if l.need_dx:
            geo = Fn.dgrad_problem(spec, batch, H, W, P, Q)
            if Fn.uses_dgrad_phases(spec, H, W):
                for ph in Fn.dgrad_phases(spec, H, W):
                    pm, pk, pt = Fn.dgrad_phase_problem(spec, batch, ph)
                    out.append(row("dgrad", name, pm, Cin, pk, Fn.p3_plan(pm, Cin, pk, pt), fwd_geom, 2.0 * pm * Cin * pk))
            else:
                out.append(row("dgrad", name, geo[0], Cin, geo[1], Fn.p3_plan(geo[0], Cin, geo[1], taps), fwd_geom,
                               2.0 * geo[0] * Cin * geo[1]))
        out.append(row("wgrad", name, Cout, spec.K, M, Fn.wgrad_p3_plan(Cout, spec.K, M, taps), wgrad_geom, flop))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--table", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    n = autotune.load_cache(a.table or autotune.DEFAULT_CACHE)
    m = create_model(a.model, device="cpu")
    rows = problems(m, a.batch)
    tot = sum(r["flop"] for r in rows)
    idle = sum(r["flop"] * (1 - r["fill"]) for r in rows)
    print(f"# {a.model} bs={a.batch} fp32 plane GEMMs: {len(rows)} launches per step, {n} tuned entries")
    print(f"# FLOP-weighted fill {1 - idle / tot:.3f}  (idle-slot share of the GEMM work {idle / tot:.3f})")
    for k in ("fwd", "dgrad", "wgrad"):
        rk = [r for r in rows if r["kind"] == k]
        t = sum(r["flop"] for r in rk)
        i = sum(r["flop"] * (1 - r["fill"]) for r in rk)
        print(f"#   {k:6s} {len(rk):3d} launches, FLOP-weighted fill {1 - i / t:.3f}")
    print(f"{'kind':6s} {'layer':26s} {'M':>7s} {'N':>5s} {'K':>7s} cfg spl {'tile':8s} occ P {'tiles':>5s} {'slots':>5s} "
          f"rnd  fill  GFLOP idle-GF")
    rows.sort(key=lambda r: -r["flop"] * (1 - r["fill"]))
    for r in rows[:a.top]:
        print(f"{r['kind']:6s} {r['name']:26s} {r['M']:7d} {r['N']:5d} {r['K']:7d} {r['cfg']:3d} {r['splits']:3d} "
              f"{r['tile']:8s} {r['occ']:3d} {'p' if r['persist'] else '-'} {r['tiles']:5d} {r['slots']:5d} "
              f"{r['rounds']:3d} {r['fill']:5.2f} {r['flop'] / 1e9:6.1f} {r['flop'] * (1 - r['fill']) / 1e9:6.2f}")


if __name__ == "__main__":
    main()
