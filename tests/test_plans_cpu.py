"""CPU checks of the GEMM plan tables and helpers the GPU paths rely on: the persistent plane-GEMM
twins (conv_p3_persist.h) in the candidate sets and the step tuner's twin map, the stem's row-window
GEMM geometry and the step-start clear."""
import os
import sys

import torch

from azure_hc_intel_tf_amd.nn.layers import StemS2D
from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import functional as Fn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_persistent_twins_in_candidate_sets():
    fwd = Fn.p3_candidates(200704, 256, 64)
    cfgs = {c for c, _ in fwd}
    assert {18, 19, 20, 21, 22} <= cfgs
    assert all(s == 1 for c, s in fwd if c >= 18), "persistent forward twins run without split-K"
    assert Fn._P3_TILES[18] == Fn._P3_TILES[15] and Fn._P3_TILES[19] == Fn._P3_TILES[14]
    assert Fn._P3_TILES[22] == Fn._P3_TILES[7]
    wg = Fn.wgrad_p3_candidates(256, 2304, 12544)
    assert {16, 17, 18} <= {c for c, _ in wg}
    assert Fn._WP3_TILES[16] == Fn._WP3_TILES[12] and Fn._WP3_TILES[18] == Fn._WP3_TILES[15]


def test_step_tuner_twin_map():
    import step_tune as st

    assert st.twin_plans(("fwd3", 200704, 256, 64, 1), [15, 1]) == [[18, 1]]
    assert st.twin_plans(("fwd3", 12544, 256, 2304, 9), [8, 1]) == []
    assert st.twin_plans(("wgrad3", 256, 2304, 12544, 9), [12, 7]) == [[16, 7]]
    for src, dst in st.FWD_TWIN.items():
        assert Fn._P3_TILES[src] == Fn._P3_TILES[dst]
    for src, dst in st.WGRAD_TWIN.items():
        assert Fn._WP3_TILES[src] == Fn._WP3_TILES[dst]


def test_stem_row_window_geometry():
    """fold_spec reads the 16-channel fold as a 4x1 conv over 64-channel windows: the same K and
    weight layout as the 4x4 form, the same 112x112 output (pr = -3 trims the windows that run past
    a fold row)."""
    ps = ParamStore(seed=1)
    st = StemS2D(ps, "conv0", (224, 224, 8), 64, relu=True, need_dx=False, logical_cin=3)
    fs = st.fold_spec
    assert (fs.cin_pad, fs.kh, fs.kw, fs.K) == (64, 4, 1, 256)
    Hs, Ws, C = st.fold_shape
    assert C == 16 and fs.out_hw(Hs, Ws) == st.out_shape[:2] == (112, 112)


def test_zero_bufs():
    bufs = [torch.randn(37), torch.randn(5, 3)]
    Fn.zero_bufs(bufs)
    assert all(float(b.abs().sum()) == 0.0 for b in bufs)


def test_learning_rate_written_only_when_it_moves():
    """The step writes hyper[0] (the device-side learning rate) only when the schedule changes it:
    a constant schedule adds no fill kernel between graph replays."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.trainer import Trainer, synthetic_batch

    m = create_model("trivial", image_size=16, device="cpu", seed=5)
    t = Trainer(m, 4, lambda s: 0.1 if s < 2 else 0.05)
    img, lab = synthetic_batch(m, 4, seed=1)
    seen = []
    for _ in range(4):
        t.step(img, lab)
        seen.append(round(float(t.hyper[0]), 6))
    assert seen == [0.1, 0.1, 0.05, 0.05]
    assert t._lr_dev == 0.05


def test_streamk_cfgs_share_the_persistent_tiles():
    """cfg 23-27 are the stream-K form of the persistent cfg 18-22: same tiles / occupancy, no
    split-K candidates of their own, and a plan that needs the split-K workspace."""
    for sk, pc in Fn._P3_STREAMK.items():
        assert Fn._P3_TILES[sk] == Fn._P3_TILES[pc] and Fn._P3_OCC.get(sk, 1) == Fn._P3_OCC.get(pc, 1)
        assert Fn._P3_PERSIST[sk] == Fn._P3_PERSIST.get(pc, pc)
    cands = Fn.p3_candidates(12544, 256, 2304)
    assert {27} <= {c for c, _ in cands}
    assert all(s == 1 for c, s in cands if c in Fn._P3_STREAMK)


def test_b_resident_cfgs_only_where_the_weights_fit():
    """cfg 31-36 (a workgroup's weight slice resident in LDS) are candidates only where the K x BN
    planes of one N tile fit beside the A ring: the 1x1 GEMMs with K <= 256, not the 3x3 ones."""
    c = {c for c, _ in Fn.p3_candidates(200704, 256, 64)}
    assert {31, 32, 33, 34} <= c
    c = {c for c, _ in Fn.p3_candidates(200704, 64, 256)}
    assert {33, 34, 35} <= c and 36 not in c
    assert not set(Fn._P3_BRES) & {c for c, _ in Fn.p3_candidates(200704, 64, 576)}
    assert {33, 34, 35} <= {c for c, _ in Fn.p3_candidates(12544, 1024, 256)}
    assert {36} <= {c for c, _ in Fn.p3_candidates(50176, 512, 128)}
    assert not set(Fn._P3_BRES) & {c for c, _ in Fn.p3_candidates(3136, 2048, 512)}
    assert all(s == 1 for c, s in Fn.p3_candidates(200704, 256, 64) if c in Fn._P3_BRES)
