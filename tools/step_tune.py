#!/usr/bin/env python3
"""Step-level conv autotuner: accept a kernel configuration only if the REPLAYED TRAINING STEP gets
faster (per-layer winners timed as isolated launches repeatedly lost or tied in
the step, where L2 state and the neighbouring kernels differ).

    python tools/step_tune.py [--dtype fp32|bf16] [--model resnet50] [--batch 64] [--top 24]
                              [--cands 3] [--retune] [--out gpurun_out/step_tune.json]

1. Every conv GEMM problem of the model (forward, data gradient, weight gradient) is enumerated
   with its candidate plans (``autotune.model_problems``). With --retune the problems are first
   re-tuned in isolation from scratch (the old per-layer method: the starting point).
2. Every candidate of every problem is timed in isolation once; problems are ranked by
   (isolated time of the current plan) x (launches per step).
3. For the --top problems, the --cands best isolated candidates that differ from the current plan
   are tried IN THE STEP: the step graph is re-captured with the candidate and timed by interleaved
   A/B (current, candidate, current, candidate, ...; median of each) against the current plan. A
   candidate is kept only if it beats the current plan by more than the noise band measured on
   this box at start (spread of repeated measurements of one plan set), and is then re-confirmed.
4. The table is saved (in-tree cache + --out copy) with the accepted changes; the log lists every
   trial. The result is the starting table's step time vs the final one, same process.
"""
import argparse
import json
import os
import shutil
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, resnet_lr_schedule, synthetic_batch


def log(*a):
    print(*a, flush=True)


class StepTimer:
    """Re-captures the trainer's step graph on demand and times replays with HIP events."""

    def __init__(self, trainer, images, labels, reps):
        self.tr, self.images, self.labels, self.reps = trainer, images, labels, reps
        self.captures = 0

    def recapture(self):
        tr = self.tr
        for g in (tr._g_all, tr._g_fb, tr._g_opt):
            if g is not None:
                g.reset()
        tr._g_all = tr._g_fb = tr._g_opt = None
        tr._segs = None
        tr._static = None
        self.tr.step(self.images, self.labels)  # captures (steps_done >= graph_warmup)
        self.captures += 1

    def time(self) -> float:
        """ms per step over self.reps replays of the current graph (after 3 untimed)."""
        for _ in range(3):
            self.tr.step(self.images, self.labels)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(self.reps):
            self.tr.step(self.images, self.labels)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / self.reps

    def measure(self, table_patch=None) -> float:
        saved = {}
        if table_patch:
            for k, v in table_patch.items():
                saved[k] = Fn._tuned.get(k)
                Fn._tuned[k] = v
        try:
            self.recapture()
            return self.time()
        finally:
            for k, v in saved.items():
                if v is None:
                    Fn._tuned.pop(k, None)
                else:
                    Fn._tuned[k] = v


def aa_band(timer, rounds, reps=4):
    """Interleaved A/A: the SAME table in both arms of an A/B with `rounds`
    rounds (each measurement a fresh capture, as in ab()), repeated `reps` times. The band is the
    largest |median(A) - median(A')|: the difference an A/B of two identical tables shows on this box,
    in this process -- the drift of repeated captures included, which the old spread-of-6-captures
    band (0.08%) missed (0.3-0.8% in round 5)."""
    diffs = []
    for _ in range(reps):
        a, b = [], []
        for r in range(rounds):  # ABBA: a drift between consecutive captures cancels
            if r % 2 == 0:
                a.append(timer.measure())
                b.append(timer.measure())
            else:
                b.append(timer.measure())
                a.append(timer.measure())
        diffs.append(abs(statistics.median(a) - statistics.median(b)))
    return max(diffs), diffs


def ab(timer, key, cur, cand, rounds):
    """Interleaved A/B of one problem's plan: medians (ms/step) of the current and the candidate, in
    ABBA order (round 6: with A always first, the second capture of every pair measured ~0.1 ms
    slower -- an identical table included, profiles/r6_step_tune_order.txt -- which biased every
    in-step comparison against the candidate)."""
    a, b = [], []
    for r in range(rounds):
        if r % 2 == 0:
            a.append(timer.measure({key: cur}))
            b.append(timer.measure({key: cand}))
        else:
            b.append(timer.measure({key: cand}))
            a.append(timer.measure({key: cur}))
    return statistics.median(a), statistics.median(b)


# persistent twins (conv_p3.hip launch_p3_persist / launch_wgrad_p3): forward / data-grad tile cfg ->
# persistent cfg (single split), weight-grad cfg -> persistent cfg (same splits)
FWD_TWIN = {15: 18, 14: 19, 16: 20, 17: 21, 7: 22}
WGRAD_TWIN = {12: 16, 13: 17, 15: 18}


def twin_plans(key, cur):
    c, sp = (cur[0], cur[1]) if isinstance(cur, list) else (cur, 1)
    if key[0] == "fwd3" and c in FWD_TWIN:
        return [[FWD_TWIN[c], 1]]
    if key[0] == "wgrad3" and c in WGRAD_TWIN:
        return [[WGRAD_TWIN[c], sp]]
    return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top", type=int, default=24)
    ap.add_argument("--cands", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--retune", action="store_true")
    ap.add_argument("--kinds", default="", help="comma-separated key kinds to step-tune (e.g. wgrad3); default all")
    ap.add_argument("--twins", action="store_true",
                    help="fp32: try only the persistent twin of each problem's current tile (conv_p3_persist.h)")
    ap.add_argument("--budget_s", type=float, default=900.0)
    ap.add_argument("--aa_only", action="store_true", help="measure and print the interleaved A/A band only")
    ap.add_argument("--aa_reps", type=int, default=4)
    ap.add_argument("--try_plan", action="append", default=[],
                    help="interleaved in-step A/B of one plan change instead of tuning: kind,M,N,K,taps=cfg,splits "
                         "(repeatable; each tried alone against the current table)")
    ap.add_argument("--knob_ab", default="",
                    help="interleaved in-step A/B of a kernel switch instead of tuning: p3p_bnb:A:B")
    ap.add_argument("--out", default="gpurun_out/step_tune.json")
    a = ap.parse_args()
    t_start = time.time()
    dev = torch.device("cuda")
    model = create_model(a.model, device=dev, compute_dtype=a.dtype)
    autotune.load_cache()
    model.ps.repack()
    if hasattr(model, "activate"):
        model.activate()
    probs = autotune.model_problems(model, a.batch)
    log(f"[step_tune] {a.model} bs{a.batch} {a.dtype}: {len(probs)} conv GEMM problems")
    if a.retune:
        for k in probs:
            Fn._tuned.pop(k, None)
        autotune.tune_model(model, a.batch, verbose=True, save=False)
        log(f"[step_tune] isolated re-tune done ({time.time() - t_start:.0f} s)")
    else:
        autotune.tune_model(model, a.batch, save=False)  # fills any missing entry
    start_table = {k: Fn._tuned[k] for k in probs}

    # isolated timing of every candidate (ranking and candidate shortlist)
    iso = {}
    for k, (cnt, cands, run) in ([] if a.aa_only or a.knob_ab or a.try_plan else probs.items()):
        iso[k] = {json.dumps(c): autotune._time(lambda: run(c)) for c in cands}
        cur = json.dumps(Fn._tuned[k] if not isinstance(Fn._tuned[k], tuple) else list(Fn._tuned[k]))
        if cur not in iso[k]:
            iso[k][cur] = autotune._time(lambda: run(json.loads(cur)))
        log(f"  iso {k}: {len(cands)} candidates, current {cur} {iso[k][cur] * 1000:.1f} us, "
            f"best {min(iso[k].values()) * 1000:.1f} us")
    torch.cuda.synchronize()
    log(f"[step_tune] isolated candidate timing done ({time.time() - t_start:.0f} s)")

    def cur_s(k):
        v = Fn._tuned[k]
        return json.dumps(list(v) if isinstance(v, tuple) else v)

    kinds = [k for k in a.kinds.split(",") if k]
    order = [] if a.aa_only or a.knob_ab or a.try_plan else sorted((k for k in probs if not kinds or k[0] in kinds),
                                        key=lambda k: -iso[k][cur_s(k)] * probs[k][0])

    images, labels = synthetic_batch(model, a.batch)
    trainer = Trainer(model, a.batch, resnet_lr_schedule(a.batch), use_graph=True)
    for _ in range(3):
        trainer.step(images, labels)
    timer = StepTimer(trainer, images, labels, a.reps)
    base = [timer.measure() for _ in range(6)]
    t0 = statistics.median(base)
    noise, diffs = aa_band(timer, a.rounds, a.aa_reps)
    log(f"[step_tune] start: {t0:.4f} ms/step (6 captures: {' '.join(f'{x:.4f}' for x in base)}; spread "
        f"{max(base) - min(base):.4f} ms); interleaved A/A band {noise:.4f} ms = {100 * noise / t0:.2f}% "
        f"({a.aa_reps} A/As of {a.rounds} rounds: {' '.join(f'{d:.4f}' for d in diffs)})")
    if a.try_plan:
        for spec in a.try_plan:
            ks, vs = spec.split("=")
            kp = ks.split(",")
            key = (kp[0],) + tuple(int(v) for v in kp[1:])
            cand = [int(v) for v in vs.split(",")]
            cur = Fn._tuned.get(key)
            cur = list(cur) if isinstance(cur, (tuple, list)) else cur
            ta, tb = ab(timer, key, cur, cand, a.aa_reps * a.rounds)
            log(f"[step_tune] try {key}: {cur} {ta:.4f} ms/step vs {cand} {tb:.4f} ms/step ({100 * (ta - tb) / ta:+.2f}%; "
                f"A/A band {100 * noise / t0:.2f}%)")
        return
    if a.knob_ab:
        name, va, vb = a.knob_ab.split(":")
        setter = {"p3p_bnb": Fn.set_p3p_bnb}[name]
        ta, tb = [], []
        for r in range(a.aa_reps * a.rounds):  # ABBA
            for v, t in (((va, ta), (vb, tb)) if r % 2 == 0 else ((vb, tb), (va, ta))):
                setter(int(v))
                t.append(timer.measure())
        ma, mb = statistics.median(ta), statistics.median(tb)
        log(f"[step_tune] knob {name}: {va} {ma:.4f} ms/step vs {vb} {mb:.4f} ms/step ({100 * (ma - mb) / ma:+.2f}%; "
            f"A/A band {100 * noise / t0:.2f}%) A: {' '.join(f'{x:.4f}' for x in ta)} B: {' '.join(f'{x:.4f}' for x in tb)}")
        return
    if a.aa_only:
        return

    trials = []
    for k in order[:a.top]:
        if time.time() - t_start > a.budget_s:
            log("[step_tune] time budget reached")
            break
        cur = cur_s(k)
        shortlist = [c for c in sorted(iso[k], key=iso[k].get) if c != cur][:a.cands]
        if a.twins:
            shortlist = [json.dumps(t) for t in twin_plans(k, json.loads(cur))]
        best_c, best_gain, best_i = None, 0.0, -1
        for c in shortlist:
            ta, tb = ab(timer, k, json.loads(cur), json.loads(c), a.rounds)
            gain = ta - tb
            trials.append({"key": list(k), "count": probs[k][0], "cur": cur, "cand": c,
                           "iso_cur_us": iso[k][cur] * 1000, "iso_cand_us": iso[k][c] * 1000,
                           "step_cur_ms": ta, "step_cand_ms": tb})
            log(f"  {k} x{probs[k][0]}: {cur} -> {c}: iso {iso[k][cur] * 1000:.1f} -> {iso[k][c] * 1000:.1f} us; "
                f"step {ta:.4f} -> {tb:.4f} ms")
            if gain > max(noise, 0.0005 * ta) and gain > best_gain:
                best_c, best_gain, best_i = c, gain, len(trials) - 1
        if best_c is not None:
            # re-confirm the winner before keeping it
            ta, tb = ab(timer, k, json.loads(cur), json.loads(best_c), a.rounds + 1)
            if ta - tb > max(noise, 0.0005 * ta):
                Fn._tuned[k] = json.loads(best_c)
                log(f"  ACCEPT {k}: {cur} -> {best_c} ({ta:.4f} -> {tb:.4f} ms)")
                trials[best_i]["accepted"] = True
            else:
                log(f"  reject {k}: {best_c} not confirmed ({ta:.4f} -> {tb:.4f} ms)")

    # final: start table vs tuned table, interleaved
    final_patch = {k: Fn._tuned[k] for k in probs}
    s_t, f_t = [], []
    for r in range(4):  # ABBA
        if r % 2 == 0:
            s_t.append(timer.measure(start_table))
            f_t.append(timer.measure(final_patch))
        else:
            f_t.append(timer.measure(final_patch))
            s_t.append(timer.measure(start_table))
    changed = {str(k): [start_table[k], final_patch[k]] for k in probs if start_table[k] != final_patch[k]}
    res = {"model": a.model, "batch": a.batch, "dtype": a.dtype, "problems": len(probs),
           "start_ms": statistics.median(s_t), "final_ms": statistics.median(f_t), "noise_ms": noise,
           "start_samples": s_t, "final_samples": f_t, "changed": changed, "trials": trials,
           "captures": timer.captures, "seconds": time.time() - t_start}
    log(f"[step_tune] start table {res['start_ms']:.4f} ms/step -> tuned {res['final_ms']:.4f} ms/step "
        f"({len(changed)} problems changed, {timer.captures} captures, {res['seconds']:.0f} s)")
    autotune.save_cache()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1, default=str)
    shutil.copy(autotune.DEFAULT_CACHE, os.path.join(os.path.dirname(os.path.abspath(a.out)), "mi355x.json"))


if __name__ == "__main__":
    main()
