"""Primitive training ops on NHWC activations with explicit forward / backward halves.

Each op has two implementations selected by the device of its tensors:

* GPU (MI355X): the hand-written gfx950 HIP kernels in ``csrc/kernels`` via
  ``torch.ops.hcb`` -- bf16 activations, fp32 accumulation / statistics / masters.
  There is NO PyTorch fallback for GPU tensors: a missing library raises.
* CPU: a PyTorch reference of the same math (fp32), which is the reference's
  ``--device=cpu`` path (/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:75;
  BASELINE config 1) and the oracle the GPU numerics tests compare against.

Activations are ``[N, H, W, C]`` tensors whose channel dim may be a strided slice of a
wider buffer (``t.stride(2) = ld``): Inception's branch outputs are written straight into
their channel window of the concat buffer (no concat kernel).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _ext


def ld(t) -> int:
    """Pixel stride (elements) of an NHWC activation (supports channel-slice views and Planes)."""
    if t.dim() == 4:
        assert t.stride(3) == 1, "activation channels must be contiguous"
        return t.stride(2)
    assert t.dim() == 2 and t.stride(1) == 1
    return t.stride(0)


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# --------------------------------------------------------------------------- conv
_DET = [os.environ.get("HCB_DETERMINISTIC", "0") == "1"]


def set_deterministic(on: bool = True) -> None:
    """Opt-in bitwise-reproducible GPU training (HCB_DETERMINISTIC=1): no split-K (conv and
    weight-gradient tiles have a single writer), BN statistic / backward accumulators with one
    replica per contributing tile or block (every fp32 slot receives exactly one add, summed
    later in a fixed order), single-block bias column sums. Slower; for debugging and the
    determinism test."""
    _DET[0] = bool(on)
    for ns in _ext.loaded_namespaces():
        ns.set_deterministic(bool(on))


def deterministic() -> bool:
    return _DET[0]


def set_p3p_bnb(level: int) -> None:
    """Fused BN-backward data gradients on the persistent plane GEMMs (conv_p3_persist.h BNB): 0
    never (the non-persistent twin runs; the default: level 1 measured 0.38% slower in the fp32 step,
    profiles/r6_persistent_bnb.txt), 1 ReLU modes 0 / 2, 2 every mode. Takes effect at the next
    launch (a captured step graph must be re-captured). Env default: HCB_P3P_BNB."""
    for ns in _ext.loaded_namespaces():
        ns.set_p3p_bnb(int(level))


def det_replicas(M: int) -> int:
    """Accumulator replicas for an M-row BN layer in deterministic mode: one per 64 rows covers
    every GEMM row tile (tiles are >= 64 rows) and every BN-backward row block."""
    return max(1, (M + 63) // 64)


# IEEE-fp16 activations through the fp16 build of the HIP kernels (a module switch: tests set it
# False to run fp16 through the PyTorch / MIOpen path, the round-2 reference-precision form)
F16_NATIVE = True


# fp32 activations through the HIP kernels (--compute_dtype fp32, the reference's precision):
# bf16x6 GEMMs (every fp32 operand split into bf16 hi + mid + lo while staged, the six MFMA
# products down to 2^-16 relative, fp32 accumulation) and fp32 BN / pool / loss kernels. Set by the active model
# (CNNModel.activate) for the models whose whole op set has the fp32 kernels (ResNet v1 / v1.5);
# other models keep the PyTorch path in fp32.
_F32_NATIVE = [False]


def set_f32_native(on: bool) -> None:
    _F32_NATIVE[0] = bool(on)


def register_lo(pack, lo) -> None:
    """Attach (lo = None: detach) the mid / lo packs to the pack tensor ``pack``."""
    pack.hcb_lo = lo


def lo_pack(w):
    """The [2][n] mid / lo bf16 packs of weight pack ``w`` (fp32 path), or None. Held on the pack
    tensor itself (``w.hcb_lo``, set by ParamStore.finalize), so it lives and dies with the pack."""
    if w is None:
        return None
    lo = getattr(w, "hcb_lo", None)
    if lo is None or lo.shape[-1] != w.numel() or lo.device != w.device:
        return None
    return lo


def _f32o(t) -> int:
    return 1 if t.dtype == torch.float32 else 0


class Planes:
    """An fp32 tensor held as three bf16 PLANES, hi / mid / lo (``t``: bf16 ``[3, *shape]``; hi + mid +
    lo == the fp32 value exactly, 8 + 8 + 8 significant bits): the fp32 path's GEMM-operand format.
    The producing kernel (BN apply, BN backward, the split kernel) writes it, so the bf16x6 GEMMs
    (csrc/kernels/conv_p3.hip) stage plain bf16 tiles by LDS-DMA with no per-use split. It stands in
    for an fp32 activation: ``shape`` / ``dtype`` (float32) / ``device`` / ``stride`` / ``view`` are
    those of the logical tensor."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        assert t.dtype == torch.bfloat16 and t.dim() >= 2 and t.shape[0] == 3, "planes are bf16 [3, ...]"
        self.t = t

    @staticmethod
    def empty(shape, device) -> "Planes":
        return Planes(torch.empty((3,) + tuple(shape), dtype=torch.bfloat16, device=device))

    @property
    def shape(self):
        return self.t.shape[1:]

    @property
    def dtype(self):
        return torch.float32

    @property
    def device(self):
        return self.t.device

    @property
    def is_cuda(self) -> bool:
        return self.t.is_cuda

    def dim(self) -> int:
        return self.t.dim() - 1

    def stride(self, i: int) -> int:
        return self.t.stride(i + 1 if i >= 0 else i)

    def numel(self) -> int:
        return self.t[0].numel()

    def is_contiguous(self) -> bool:
        return self.t.is_contiguous()

    def view(self, *shape) -> "Planes":
        if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
            shape = tuple(shape[0])
        return Planes(self.t.view((3,) + tuple(shape)))

    def reshape(self, *shape) -> "Planes":
        return self.view(*shape)

    def __getitem__(self, idx) -> "Planes":
        """A view of the logical tensor (e.g. ``x[..., a:b]``: the channel window of a concat
        buffer an Inception branch writes); the three planes keep their stride."""
        if not isinstance(idx, tuple):
            idx = (idx,)
        return Planes(self.t[(slice(None),) + idx])

    def float(self) -> torch.Tensor:
        """The fp32 value (hi + (mid + lo), exact)."""
        return self.t[0].float() + (self.t[1].float() + self.t[2].float())


def is_planes(t) -> bool:
    return isinstance(t, Planes)


def planes_mode() -> bool:
    """True while an fp32-native model is active: its GEMM operands are stored as Planes."""
    return _F32_NATIVE[0]


def to_planes(x: torch.Tensor) -> Planes:
    """fp32 [..., C] (C % 8 == 0; rows may be strided) -> Planes of the same logical shape (one
    launch on the GPU)."""
    if isinstance(x, Planes):
        return x
    assert x.dtype == torch.float32 and x.shape[-1] % 8 == 0
    out = Planes.empty(tuple(x.shape), x.device)
    C = x.shape[-1]
    rows = x.numel() // C
    if x.is_cuda:
        xv = x if x.dim() >= 2 else x.view(1, -1)
        ldx = xv.stride(-2) if xv.dim() >= 2 and xv.shape[-2] > 1 else C
        if not _rows_uniform(xv, C):
            xv = xv.contiguous()
            ldx = C
        _ext.ops().split_planes(xv, ldx, rows, C, out.t, C)
        return out
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    out.t[0].copy_(h)
    out.t[1].copy_(m)
    out.t[2].copy_((r - m.float()).to(torch.bfloat16))
    return out


def _rows_uniform(x: torch.Tensor, C: int) -> bool:
    """x's rows of C channels are evenly strided (one row stride over every leading dim)."""
    if x.stride(-1) != 1:
        return False
    ld = x.stride(-2) if x.dim() >= 2 else C
    exp = ld
    for d in range(x.dim() - 2, -1, -1):
        if x.shape[d] > 1 and x.stride(d) != exp:
            return False
        exp *= x.shape[d]
    return True


def _pl(t):
    """The tensor a kernel binding receives for t (Planes -> its [3, ...] bf16 storage)."""
    return t.t if isinstance(t, Planes) else t


def native(t) -> bool:
    """True when ``t`` goes through the hand-written HIP kernels: a bf16 (or, with the fp16
    build, IEEE-fp16) activation on the GPU, or an fp32 one while an fp32-native model is
    active. Other tensors take the PyTorch path below (MIOpen / rocBLAS on the GPU), the same
    code as the CPU path."""
    if isinstance(t, Planes):
        return t.is_cuda
    return t.is_cuda and (t.dtype == torch.bfloat16 or (t.dtype == torch.float16 and F16_NATIVE)
                          or (t.dtype == torch.float32 and _F32_NATIVE[0]))


@dataclass
class ConvSpec:
    """Geometry of one convolution (NHWC activations, KRSC weights)."""

    cin: int          # logical input channels (stem: 3)
    cin_pad: int      # channels as stored (multiple of 8; stem 3 -> 8)
    cout: int
    kh: int
    kw: int
    sh: int = 1
    sw: int = 1
    pt: int = 0       # top / left padding (bottom / right implied by the output size)
    pl: int = 0
    pb: int = 0
    pr: int = 0
    dh: int = 1
    dw: int = 1

    @property
    def K(self) -> int:
        return self.kh * self.kw * self.cin_pad

    @property
    def Kpad(self) -> int:
        return _round_up(self.K, 64)

    @property
    def Kt(self) -> int:  # reduction length of the data-gradient GEMM
        return self.kh * self.kw * self.cout

    @property
    def Kpad_t(self) -> int:
        return _round_up(self.Kt, 64)

    def out_hw(self, H: int, W: int):
        P = (H + self.pt + self.pb - self.dh * (self.kh - 1) - 1) // self.sh + 1
        Q = (W + self.pl + self.pr - self.dw * (self.kw - 1) - 1) // self.sw + 1
        return P, Q


def same_pads(size: int, k: int, s: int, d: int = 1):
    """TensorFlow 'SAME' padding (extra padding at the end)."""
    out = (size + s - 1) // s
    eff = d * (k - 1) + 1
    total = max((out - 1) * s + eff - size, 0)
    return total // 2, total - total // 2


# ----------------------------------------------------------------- tile selection
# cfg -> block tile; 0-3 register-staged main loop, 4-7 LDS-DMA ring (same tiles)
_CONV_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 64), 3: (64, 128),
               4: (128, 128), 5: (128, 64), 6: (64, 64), 7: (64, 128),
               8: (128, 128), 9: (128, 128), 10: (128, 64), 11: (64, 128),
               12: (128, 128), 13: (128, 128), 14: (256, 128), 15: (128, 256), 16: (64, 128),
               # 3x3 / stride-1 kernels with the input patch resident in LDS (conv3x3_patch.hip)
               17: (128, 128), 18: (256, 128), 19: (256, 64), 20: (128, 64), 21: (128, 128),
               }
# (cfg 22-37 -- two k-steps per stage, occupancy-sized two-slot rings, the register-pipelined loop --
# and 100-117, the plane kernel on one 16-bit plane, were measured without a step gain and removed in
# round 5: profiles/r5_prune_variants.txt)
PATCH_CFG0 = 17
PATCH_CFGS = (17, 18, 19, 20, 21)
# weight-grad cfg -> (Nout tile, K tile); 0-2 register-staged, 3-14 LDS-DMA rings
_WGRAD_TILES = {0: (128, 128), 1: (64, 128), 2: (64, 64), 3: (128, 128), 4: (128, 128), 5: (256, 128),
                6: (128, 256), 7: (64, 128), 8: (64, 64), 9: (64, 128), 10: (64, 64), 11: (128, 64),
                12: (64, 128), 13: (128, 64), 14: (64, 128)}
N_CU = 256
_tuned: dict = {}


# Tuning keys carry the filter tap count: GEMMs of equal (M, N, K) but different geometry
# (a 1x1 over K channels vs a 4x4 over K/16) have different im2col loaders and best tiles.
def fwd_key(M: int, N: int, K: int, taps: int = 1):
    return ("fwd", M, N, K, taps)


def dgb_key(M: int, N: int, K: int, taps: int = 1):
    """Data-grad GEMM with the fused BN-backward epilogue (its own tuning entry: the epilogue
    reads z / y / the beta source, which moves the best tile away from the plain GEMM's)."""
    return ("dgb", M, N, K, taps)


def wgrad_key(Nout: int, K: int, M: int, taps: int = 1):
    return ("wgrad", Nout, K, M, taps)


def fwd_candidates(N: int, patch: bool = False):
    """Tile configs worth timing for a GEMM with N output columns; ``patch``: the problem is a
    3x3 / stride-1 / pad-1 conv over a multiple of 64 channels (patch_eligible), so the
    LDS-resident-patch kernels are candidates too."""
    if N <= 64:
        return [1, 2, 5, 6, 10] + ([19, 20] if patch else [])
    c = [0, 3, 1, 2, 4, 7, 5, 6, 8, 9, 10, 11, 12, 13, 14, 16]
    c = c + [15] if N > 128 else c
    return c + ([17, 18, 19, 20, 21] if patch else [])


def patch_eligible(spec: "ConvSpec", dgrad: bool = False) -> bool:
    """The forward (or, ``dgrad``, the data-gradient) GEMM of this conv can run on the 3x3
    patch kernels: 3x3, stride 1, pad 1 (same-size output), undilated, and the GEMM's input
    channels (cin, or cout for the data gradient) a multiple of 64."""
    c = spec.cout if dgrad else spec.cin_pad
    return (spec.kh == 3 and spec.kw == 3 and spec.sh == 1 and spec.sw == 1 and spec.pt == 1 and spec.pl == 1
            and spec.pb == 1 and spec.pr == 1 and spec.dh == 1 and spec.dw == 1 and c % 64 == 0)


def wgrad_candidates(Nout: int, K: int, M: int):
    ksteps = math.ceil(M / 64)
    out = []
    for c, (bm, bn) in _WGRAD_TILES.items():
        tiles = math.ceil(Nout / bm) * math.ceil(K / bn)
        for s in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
            if s > 1 and ksteps // s < 2:
                break
            if tiles * s > 8 * N_CU:
                break
            out.append((c, s))
    return out


# split-K scratch (fp32 partial-tile slabs + self-resetting per-tile tickets), one per process
SPLITK_WS_FLOATS = 32 << 20
SPLITK_MAX_TILES = 1 << 16
_splitk = {}


def ensure_splitk_workspace(device) -> None:
    """One workspace per device, registered with each kernel library (bf16 / fp16 build) that
    launches convs; the libraries never run concurrently on one stream."""
    dev = torch.device(device)
    key = _ext._ACT[0]
    if _splitk.get("dev") != dev:
        _splitk.clear()
        _splitk.update(dev=dev, ws=torch.empty(SPLITK_WS_FLOATS, dtype=torch.float32, device=dev),
                       cnt=torch.zeros(SPLITK_MAX_TILES, dtype=torch.int32, device=dev), libs=set())
    if key in _splitk["libs"]:
        return
    _ext.ops().set_splitk_workspace(_splitk["ws"], _splitk["cnt"])
    _splitk["libs"].add(key)


def splitk_candidates(cfg: int, M: int, N: int, K: int):
    """split-K factors worth timing for an LDS-DMA config: only while the grid is below ~2
    workgroups per CU and every split keeps >= 4 k-steps."""
    if cfg < 4:
        return [1]
    bm, bn = _CONV_TILES[cfg]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    ksteps = math.ceil(K / 64)
    out = [1]
    for s in (2, 3, 4, 6, 8):
        if tiles * (s - 1) >= 2 * N_CU or ksteps // s < 4 or tiles * s * bm * bn > SPLITK_WS_FLOATS:
            break
        if cfg in PATCH_CFGS and s > ksteps // 9:  # the patch kernels split over 64-channel slabs
            break
        out.append(s)
    return out


def conv_plan(M: int, N: int, K: int, taps: int = 1):
    """(cfg, splits) for C[M,N] (+K)."""
    c = conv_cfg(M, N, K, taps)
    return (c[0], c[1]) if isinstance(c, (tuple, list)) else (c, 1)


def conv_cfg(M: int, N: int, K: int, taps: int = 1):
    """Block tile for C[M,N] (+K): the autotuned choice if known (an int cfg or a [cfg, splits]
    pair), else the biggest tile that still gives >= 2 workgroups per CU."""
    key = fwd_key(M, N, K, taps)
    if key in _tuned:
        return _tuned[key]
    cands = [c for c in fwd_candidates(N) if c < 4]
    for c in cands:
        bm, bn = _CONV_TILES[c]
        if math.ceil(M / bm) * math.ceil(N / bn) >= 2 * N_CU:
            return c
    return cands[-1]


def wgrad_cfg(Nout: int, K: int, M: int, taps: int = 1):
    """(tile cfg, split-K) for dW[Nout, K] reduced over M pixels."""
    key = wgrad_key(Nout, K, M, taps)
    if key in _tuned:
        return tuple(_tuned[key])
    c = 0 if Nout >= 128 and K >= 128 else (1 if K >= 128 else 2)
    bm, bn = _WGRAD_TILES[c]
    tiles = math.ceil(Nout / bm) * math.ceil(K / bn)
    ksteps = math.ceil(M / 64)
    target = 2 * N_CU
    splits = max(1, min(ksteps // 4 if ksteps >= 4 else 1, math.ceil(target / tiles)))
    return c, splits


def dgrad_problem(spec, N, H, W, P, Q):
    """(M, K) of the data-gradient GEMM of a conv."""
    Cdz = spec.cout if spec.cout % 8 == 0 else _round_up(spec.cout, 8)
    K = spec.kh * spec.kw * Cdz
    if (spec.sh > 1 or spec.sw > 1) and spec.kh == 1 and spec.kw == 1 and spec.pt == 0 and spec.pl == 0:
        return N * P * Q, K
    return N * H * W, K


def set_tuned(table: dict) -> None:
    _tuned.update(table)


# ---- fp32 path (Planes operands, conv_p3.hip): its own tile sets and tuning keys
# cfg -> block tile (conv_p3.hip): 0-6 64-deep two-slot rings, 7-13 32-deep slots (bigger tiles per CU),
# 14-17 32-deep slots sized for two / three workgroups per CU
_P3_TILES = {0: (128, 64), 1: (64, 128), 2: (128, 64), 3: (64, 128), 4: (64, 64), 5: (128, 64), 6: (64, 128),
             7: (128, 128), 8: (128, 128), 9: (128, 128), 10: (256, 128), 11: (128, 256), 12: (64, 128),
             13: (128, 64), 14: (128, 64), 15: (64, 128), 16: (64, 64), 17: (64, 64),
             18: (64, 128), 19: (128, 64), 20: (64, 64), 21: (64, 64), 22: (128, 128),
             23: (64, 128), 24: (128, 64), 25: (64, 64), 26: (64, 64), 27: (128, 128), 28: (128, 128),
             31: (64, 256), 32: (128, 256), 33: (64, 64), 34: (128, 64),
             35: (128, 64), 36: (128, 128)}
# workgroups per CU each plane-GEMM cfg is built for
_P3_OCC = {14: 2, 15: 2, 16: 2, 17: 3, 18: 2, 19: 2, 20: 2, 21: 3, 23: 2, 24: 2, 25: 2, 26: 3}
# persistent short-K twins (conv_p3_persist.h): one workgroup per resident slot walks its tiles with
# the LDS-DMA ring running across tile boundaries and a register epilogue; no split-K (a problem
# with an epilogue they do not serve -- fused BN backward, beta, bias -- runs the twin)
_P3_PERSIST = {18: 15, 19: 14, 20: 16, 21: 17, 22: 7, 23: 15, 24: 14, 25: 16, 26: 17, 27: 7, 28: 8,
               31: 15, 32: 15, 33: 16, 34: 14, 35: 14, 36: 7}
# the persistent kernel with each workgroup's weight slice resident in LDS (conv_p3_persist.h BRES):
# every k-step's planes of one N tile (K x BN x 6 B) beside the A ring; cfg -> ring slots
_P3_BRES = {31: 3, 32: 2, 33: 3, 34: 2, 35: 2, 36: 2}


def p3_bres_fits(cfg: int, N: int, K: int) -> bool:
    """Whether a B-resident cfg serves an (N, K) problem (else its launcher falls back)."""
    bm, bn = _P3_TILES[cfg]
    kpad = -(-K // 64) * 64
    return _P3_BRES[cfg] * 3 * bm * 64 + kpad * 3 * bn * 2 + 4 * N <= 160 * 1024
# their STREAM-K form (conv_p3_persist.h SK): every workgroup a contiguous, equal share of all (tile,
# k-step) iterations -- no wave-quantization tail; split tiles meet through the split-K workspace.
# sk cfg -> the cfg it falls back to (the whole-tile persistent form; 28 -- cfg 8's geometry -- cfg 8)
_P3_STREAMK = {23: 18, 24: 19, 25: 20, 26: 21, 27: 22, 28: 8}  # (29 / 30 retired: profiles/r6_quantization_streamk.txt)
# wgrad cfg -> block tile: 0-5 64-deep slots, 6-11 32-deep slots (128x128 / 256x128 / 128x256 tiles),
# 12-15 32-deep slots, two / three workgroups per CU
_WP3_TILES = {0: (128, 64), 1: (64, 128), 2: (64, 64), 3: (128, 64), 4: (64, 128), 5: (64, 64),
              6: (128, 128), 7: (128, 128), 8: (256, 128), 9: (128, 256), 10: (128, 128), 11: (128, 64),
              12: (128, 64), 13: (64, 128), 14: (64, 64), 15: (64, 64),
              16: (128, 64), 17: (64, 128), 18: (64, 64)}  # 16-18: persistent twins of 12, 13, 15
_WP3_OCC = {12: 2, 13: 2, 14: 2, 15: 3, 16: 2, 17: 2, 18: 3}  # workgroups per CU the weight-grad tile is built for


def fwd3_key(M: int, N: int, K: int, taps: int = 1):
    return ("fwd3", M, N, K, taps)


def wgrad3_key(Nout: int, K: int, M: int, taps: int = 1):
    return ("wgrad3", Nout, K, M, taps)


def p3_candidates(M: int, N: int, K: int):
    """(cfg, splits) worth timing for an fp32 (Planes) forward / data-grad GEMM: every tile, with
    split-K factors that bring the grid close to whole rounds of the 256 CUs (one workgroup fits per
    CU: 144 KB of LDS) -- a 196-tile layer leaves 60 CUs idle, 4 splits run it in 3.06 rounds --
    while every split keeps >= 2 64-deep k-steps. (Stream-K shares were measured 11-30% slower per
    layer and removed: profiles/r4v_streamk_probe.txt, profiles/r5_prune_variants.txt.)"""
    out = []
    ksteps = math.ceil(K / 64)
    for c, (bm, bn) in _P3_TILES.items():
        if (N <= 64 and bn > 64) or (N <= 128 and bn > 128) or (M <= 4096 and bm > 128):
            continue
        if c in _P3_BRES and not p3_bres_fits(c, N, K):
            continue
        tiles = math.ceil(M / bm) * math.ceil(N / bn)
        out.append((c, 1))
        if c in _P3_PERSIST:
            continue
        for s in (2, 3, 4, 5, 6, 8, 12, 16):
            if tiles * s > 6 * N_CU or ksteps // s < 2 or tiles * s * bm * bn > SPLITK_WS_FLOATS:
                break
            out.append((c, s))
    return out


def p3_plan(M: int, N: int, K: int, taps: int = 1):
    """(cfg, splits) of an fp32 (Planes) forward / data-grad GEMM: tuned, else 128x64 (64x128 for
    wide outputs) with split-K up to ~one workgroup per CU."""
    key = fwd3_key(M, N, K, taps)
    if key in _tuned:
        c = _tuned[key]
        return (int(c[0]), int(c[1])) if isinstance(c, (tuple, list)) else (int(c), 1)
    cfg = 7 if N >= 128 else 13
    bm, bn = _P3_TILES[cfg]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    ksteps = math.ceil(K / 64)
    s = 1
    while tiles * (s + 1) <= N_CU and ksteps // (s + 1) >= 3 and s < 8:
        s += 1
    return cfg, s


def wgrad_p3_candidates(Nout: int, K: int, M: int):
    ksteps = math.ceil(M / 64)
    out = []
    for c, (bm, bn) in _WP3_TILES.items():
        if (Nout <= 64 and bm > 64) or (K <= 64 and bn > 64) or (Nout < 256 and bm > 128) \
                or (K < 256 and bn > 128):
            continue
        tiles = math.ceil(Nout / bm) * math.ceil(K / bn)
        # powers of two, plus the split counts that fill whole rounds of the resident workgroups
        # (36 128x128 tiles: 7 splits = 252 workgroups, where 8 = 288 runs a second, 1/8-full round)
        slots = N_CU * _WP3_OCC.get(c, 1)
        fill = {max(1, r * slots // tiles) for r in (1, 2, 3)}
        for s in sorted({1, 2, 4, 8, 16, 32, 64, 128, 256} | fill):
            if s > 1 and ksteps // s < 2:
                break
            if tiles * s > 4 * N_CU:
                break
            out.append((c, s))
    return out


def wgrad_p3_plan(Nout: int, K: int, M: int, taps: int = 1):
    key = wgrad3_key(Nout, K, M, taps)
    if key in _tuned:
        c = _tuned[key]
        return int(c[0]), int(c[1])
    c = 0 if Nout >= 128 else (1 if K >= 128 else 2)
    bm, bn = _WP3_TILES[c]
    tiles = math.ceil(Nout / bm) * math.ceil(K / bn)
    ksteps = math.ceil(M / 64)
    splits = max(1, min(ksteps // 4 if ksteps >= 4 else 1, math.ceil(2 * N_CU / tiles)))
    return c, splits


def _plan3(cfg, M, N, K, device, taps: int = 1):
    if cfg is None:
        cfg, splits = p3_plan(M, N, K, taps)
    elif isinstance(cfg, (tuple, list)):
        cfg, splits = cfg
    else:
        splits = 1
    splits = max(1, min(int(splits), max(K // 64, 1)))
    if _DET[0]:
        splits = 1
    if splits != 1 or int(cfg) in _P3_STREAMK:
        ensure_splitk_workspace(device)
    return int(cfg), int(splits)


# ---------------------------------------------------------------- conv forward
def conv_forward(x, spec: ConvSpec, wpack, w_master, out, stats=None, bias=None, cfg=None, relu=False,
                 stats_R: int = 0, residual=None, stats_shift=None):
    """out[N,P,Q,cout] = conv(x, W) (+bias) [ReLU]. GPU: fp32 acc, bf16 (or fp32) out + fused BN
    statistics: per-tile slab (stats_R=0) or fp32 atomics into stats_R replicas of [2][cout].
    ``stats_shift`` (fp32 [cout]): the statistics are sums of (v - shift) and (v - shift)^2, which
    keeps the single-pass variance exact when |mean| >> std; the BN apply gets the same shift."""
    if is_planes(x) or (native(x) and x.dtype == torch.float32):
        return _conv_forward_p3(x, spec, wpack, out, stats, bias, cfg, relu, stats_R, residual, stats_shift)
    N, H, W, _ = x.shape
    P, Q = spec.out_hw(H, W)
    if native(x):
        M = N * P * Q
        cfg, splits = _plan(cfg, M, spec.cout, spec.K, x.device, spec.kh * spec.kw)
        out_f32 = out.dtype == torch.float32
        geom = [N, H, W, spec.cin_pad, ld(x), P, Q, spec.kh, spec.kw, spec.sh, spec.sw, spec.pt, spec.pl,
                spec.dh, spec.dw, 1, 1, spec.cout, spec.K, spec.Kpad, ld(out), 0, P, Q, 1, 1,
                1 if residual is not None else 0, 1 if out_f32 else 0, 1 if relu else 0, int(stats_R), splits]
        if residual is not None:  # beta-accumulate epilogue: out = conv(x) + residual (same layout)
            assert ld(residual) == ld(out) and residual.shape == out.shape
        _ext.ops().conv_igemm(x, wpack, out, residual, bias, stats, geom, cfg, stats_shift, None)
        return out
    xt = x.permute(0, 3, 1, 2)
    if spec.pt or spec.pb or spec.pl or spec.pr:
        xt = F.pad(xt, (spec.pl, spec.pr, spec.pt, spec.pb))
    wt = w_master.permute(0, 3, 1, 2).to(x.dtype)
    y = F.conv2d(xt, wt, bias=None if bias is None else bias.to(x.dtype), stride=(spec.sh, spec.sw), dilation=(spec.dh, spec.dw))
    if relu:
        y = torch.relu(y)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual
    out.copy_(y)
    return out


def _conv_forward_p3(x, spec: ConvSpec, wpack, out, stats, bias, cfg, relu, stats_R, residual, stats_shift):
    """fp32 forward conv on bf16 planes (bf16x6 MFMA GEMM, conv_p3.hip): x Planes (an fp32 tensor
    is split first), fp32 out with the fused BN statistics / bias / ReLU / residual epilogue."""
    x = to_planes(x)
    N, H, W, _ = x.shape
    P, Q = spec.out_hw(H, W)
    M = N * P * Q
    cfg, splits = _plan3(cfg, M, spec.cout, spec.K, x.device, spec.kh * spec.kw)
    w_lo = lo_pack(wpack)
    assert w_lo is not None and out.dtype == torch.float32, "fp32 conv needs the mid / lo weight packs and an fp32 output"
    if residual is not None:
        assert ld(residual) == ld(out) and residual.shape == out.shape and residual.dtype == torch.float32
    geom = [N, H, W, spec.cin_pad, ld(x), P, Q, spec.kh, spec.kw, spec.sh, spec.sw, spec.pt, spec.pl,
            spec.dh, spec.dw, 1, 1, spec.cout, spec.K, spec.Kpad, ld(out), 0, P, Q, 1, 1,
            1 if residual is not None else 0, 1, 1 if relu else 0, int(stats_R), splits]
    _ext.ops().conv_p3(x.t, wpack, w_lo, out, residual, bias, stats, geom, cfg, stats_shift)
    return out


def _plan(cfg, M, N, K, device, taps: int = 1):
    """Normalise a cfg argument (None = tuned / heuristic, int, or (cfg, splits))."""
    if cfg is None:
        cfg, splits = conv_plan(M, N, K, taps)
    elif isinstance(cfg, (tuple, list)):
        cfg, splits = cfg
    else:
        splits = 1
    if _DET[0]:
        splits = 1
    if splits > 1:
        ensure_splitk_workspace(device)
    return int(cfg), int(splits)


def zero_bufs(ts):
    """Zero fp32 tensors: one HIP launch on the GPU (tensors 16-byte aligned), ``zero_`` elsewhere."""
    if ts and ts[0].is_cuda:
        _ext.ops().zero_bufs(list(ts))
        return
    for t in ts:
        t.zero_()


def relu_backward(dy, y, dz):
    if native(dy):
        _ext.ops().relu_bwd(dy, y, dz)
        return dz
    dz.copy_(dy * (y > 0).to(dy.dtype))
    return dz


def conv_stats_slab(x_shape, spec: ConvSpec, device, cfg=None):
    N, H, W, _ = x_shape
    P, Q = spec.out_hw(H, W)
    M = N * P * Q
    if cfg is None:
        cfg = conv_plan(M, spec.cout, spec.K, spec.kh * spec.kw)[0]
    bm = _CONV_TILES[cfg][0]
    T = math.ceil(M / bm)
    return torch.empty(T * 2 * spec.cout, dtype=torch.float32, device=device), T, cfg


# ---------------------------------------------------------------- conv data grad
class BNBwdFuse:
    """Request to fold a BN layer's backward reduction into the data-grad GEMM that produces
    that layer's dy (ConvParams::bnb_* in csrc/kernels/kernels.h). The GEMM output becomes
    g = dy * relu_mask; on the GPU sum(g) and sum(g * xhat) are added to ``acc`` replicas, so
    the BN backward only runs its apply pass (``bn_backward_acc(..., pre_reduced=True)``)."""

    def __init__(self, z, y, saved: "BNSaved", gamma, beta, mode: int, acc, R: int):
        self.z, self.y, self.saved, self.gamma, self.beta = z, y, saved, gamma, beta
        self.mode, self.acc, self.R = mode, acc, R

    def gate_cpu(self, g):
        """CPU semantics of the fused epilogue's gating (the reductions stay in bn_backward)."""
        if self.mode == 1:
            g.mul_((self.y > 0).to(g.dtype))
        elif self.mode == 2:
            xhat = (self.z - self.saved.mean) * self.saved.invstd
            g.mul_(((xhat * self.gamma + self.beta) > 0).to(g.dtype))
        return g


# strided 1x1 data gradients zero their stride cells' gaps in the GEMM epilogue (False: a separate
# zero-fill of dx first; the A/B switch HCB_REMAP_FILL=0)
REMAP_FILL = os.environ.get("HCB_REMAP_FILL", "1") != "0"

# strided k x k data gradients as sh*sw stride-phase GEMMs (module switch, False: one GEMM over the
# zero-dilated dz, which spends (sh*sw - 1)/(sh*sw) of its MFMA work on the inserted zeros)
DGRAD_PHASES = True
_phase_packs = {}


def dgrad_phases(spec: ConvSpec, H: int, W: int):
    """Stride phases of a strided conv's data gradient: for every output parity (ph, pw) the
    forward taps r = r0 + sh*j that reach rows h = sh*i + ph, as a stride-1 correlation of dz
    with the flipped sub-kernel. Yields (ph, pw, Hph, Wph, (r taps), (s taps), pad_t, pad_l);
    taps in the sub-kernel's order (flipped), None when a phase has no tap."""
    out = []
    for ph in range(spec.sh):
        for pw in range(spec.sw):
            Hph, Wph = -(-(H - ph) // spec.sh), -(-(W - pw) // spec.sw)
            r0, c0 = (ph + spec.pt) % spec.sh, (pw + spec.pl) % spec.sw
            rs = list(range(r0, spec.kh, spec.sh))
            ss = list(range(c0, spec.kw, spec.sw))
            if not rs or not ss or Hph <= 0 or Wph <= 0:
                out.append(None)
                continue
            a, b = (ph + spec.pt - r0) // spec.sh, (pw + spec.pl - c0) // spec.sw
            out.append((ph, pw, Hph, Wph, rs[::-1], ss[::-1], len(rs) - 1 - a, len(ss) - 1 - b))
    return out


def _phase_pack(wtr, spec: ConvSpec, Cdz: int, rs, ss):
    """[cin_pad][Kpad] operand of one phase: the columns of the transposed-flipped data-grad pack
    (column block (kh-1-r)*kw + (kw-1-s) holds forward tap (r, s)) for the phase's taps, in the
    sub-kernel's order; refreshed from the current pack on every call."""
    C = spec.cin_pad
    K = len(rs) * len(ss) * Cdz
    lead = tuple(wtr.shape[:-1])  # () for a pack, (2,) for the fp32 path's mid / lo pair
    # the sub-pack's CONTENT is refreshed below on every call; the key pins what must match for
    # the buffer itself to be reusable (a freed pack's address can come back with another dtype,
    # e.g. the fp16 build's packs followed by bf16 ones)
    Kp = _round_up(K, 64)
    key = (wtr.data_ptr(), wtr.dtype, wtr.device, lead, C, Kp, tuple(rs), tuple(ss))
    ent = _phase_packs.get(key)
    if ent is None:
        taps = [(spec.kh - 1 - r) * spec.kw + (spec.kw - 1 - s) for r in rs for s in ss]
        ent = (torch.zeros(lead + (C, Kp), dtype=wtr.dtype, device=wtr.device),
               torch.tensor(taps, dtype=torch.int64, device=wtr.device))
        _phase_packs[key] = ent
    sub, idx = ent
    trv = wtr.view(*lead, C, -1)[..., :spec.kh * spec.kw * Cdz].view(*lead, C, spec.kh * spec.kw, Cdz)
    sub[..., :K].view(*lead, C, len(rs) * len(ss), Cdz).copy_(trv.index_select(-2, idx))
    return (sub.view(*lead, -1) if lead else sub), K


def dgrad_phase_problem(spec: ConvSpec, N: int, phase):
    """(M, K, taps) of one stride-phase data-grad GEMM (its tuning key)."""
    _, _, Hph, Wph, rs, ss, _, _ = phase
    Cdz = spec.cout if spec.cout % 8 == 0 else _round_up(spec.cout, 8)
    return N * Hph * Wph, len(rs) * len(ss) * Cdz, len(rs) * len(ss)


def dgrad_phase(dz, spec: ConvSpec, wtr, dx, accumulate: bool, phase, cfg=None, bnb: "BNBwdFuse" = None):
    """One stride-phase GEMM of a strided k x k data gradient (see dgrad_phases)."""
    N, P, Q, _ = dz.shape
    _, H, W, _ = dx.shape
    ph, pw, Hph, Wph, rs, ss, pad_t, pad_l = phase
    Cdz = spec.cout if spec.cout % 8 == 0 else _round_up(spec.cout, 8)
    sub, Kph = _phase_pack(wtr, spec, Cdz, rs, ss)
    M, _, taps = dgrad_phase_problem(spec, N, phase)
    if dz.dtype == torch.float32:  # fp32 path: Planes operands
        lo = lo_pack(wtr)
        assert lo is not None, "fp32 data gradient needs the mid / lo weight packs"
        w_lo, _ = _phase_pack(lo, spec, Cdz, rs, ss)
        dz = to_planes(dz)
        cfg, splits = _plan3(cfg, M, spec.cin_pad, Kph, dz.device, taps)
        geom = [N, P, Q, Cdz, ld(dz), Hph, Wph, len(rs), len(ss), 1, 1, pad_t, pad_l, 1, 1, 1, 1,
                spec.cin_pad, Kph, sub.shape[1], ld(dx), 1, H, W, spec.sh, spec.sw, 1 if accumulate else 0, 1,
                0, 0, splits, ph, pw]
        _p3_dgrad_launch(dz, sub, w_lo, dx, accumulate, geom, cfg, bnb)
        return
    geom = [N, P, Q, Cdz, ld(dz), Hph, Wph, len(rs), len(ss), 1, 1, pad_t, pad_l, 1, 1, 1, 1,
            spec.cin_pad, Kph, sub.shape[1], ld(dx), 1, H, W, spec.sh, spec.sw, 1 if accumulate else 0, _f32o(dx)]
    if cfg is None and bnb is not None:
        cfg = _tuned.get(dgb_key(M, spec.cin_pad, Kph, taps))
    cfg, splits = _plan(cfg, M, spec.cin_pad, Kph, dz.device, taps)
    geom = geom + [0, 0, splits, ph, pw]
    if bnb is not None:
        _ext.ops().conv_igemm_bnb(dz, sub, dx, dx if accumulate else None, geom, cfg, bnb.z,
                                  bnb.y if bnb.mode == 1 else None, ld(bnb.z), bnb.saved.mean,
                                  bnb.saved.invstd, bnb.gamma, bnb.beta, bnb.acc, bnb.R, bnb.mode)
    else:
        _ext.ops().conv_igemm(dz, sub, dx, dx if accumulate else None, None, None, geom, cfg, None, None)


def _p3_dgrad_launch(dz: "Planes", w, w_lo, dx, accumulate: bool, geom, cfg: int, bnb: "BNBwdFuse" = None):
    """One fp32 (Planes) data-gradient GEMM, with the consuming BN layer's backward reduction fused
    into its epilogue when ``bnb`` is given (z fp32, the ReLU mask from the hi plane of y)."""
    if bnb is None:
        _ext.ops().conv_p3(dz.t, w, w_lo, dx, dx if accumulate else None, None, None, geom, cfg, None)
        return
    _ext.ops().conv_p3_bnb(dz.t, w, w_lo, dx, dx if accumulate else None, geom, cfg, bnb.z,
                           _pl(bnb.y) if bnb.mode == 1 else None, ld(bnb.z), bnb.saved.mean, bnb.saved.invstd,
                           bnb.gamma, bnb.beta, bnb.acc, bnb.R, bnb.mode)


def uses_dgrad_phases(spec: ConvSpec, H: int, W: int) -> bool:
    return ((spec.sh > 1 or spec.sw > 1) and DGRAD_PHASES and not (spec.kh == 1 and spec.kw == 1)
            and spec.dh == 1 and spec.dw == 1 and all(ph is not None for ph in dgrad_phases(spec, H, W)))


def conv_dgrad(dz, spec: ConvSpec, wtr, w_master, dx, accumulate: bool, cfg=None, bnb: "BNBwdFuse" = None):
    """dx[N,H,W,cin] (+)= conv_transpose(dz, W). A strided 1x1 writes every pixel of dx when not
    accumulating: its GEMM rows (one per dz pixel) also zero the rest of their stride cell (remap
    2, igemm_epilogue.h epi_fill_cell), so dx needs no zero-fill. With ``bnb`` the result is gated
    by the consuming BN layer's ReLU mask and its backward sums are fused."""
    N, P, Q, _ = dz.shape
    _, H, W, _ = dx.shape
    if native(dz):
        Cdz = spec.cout if spec.cout % 8 == 0 else _round_up(spec.cout, 8)
        K = spec.kh * spec.kw * Cdz
        Kpad = spec.Kpad_t
        assert K <= Kpad
        strided = spec.sh > 1 or spec.sw > 1
        if cfg is None and uses_dgrad_phases(spec, H, W):
            # one stride-1 GEMM per output parity over dz, rows scattered to (sh*i + ph, sw*j + pw)
            for phase in dgrad_phases(spec, H, W):
                dgrad_phase(dz, spec, wtr, dx, accumulate, phase, None, bnb)
            return dx
        if strided and spec.kh == 1 and spec.kw == 1 and spec.pt == 0 and spec.pl == 0:
            # 1x1 strided: dense GEMM over dz pixels, scatter rows to (p*sh, q*sw)
            M = N * P * Q
            fill = REMAP_FILL and not accumulate and P * spec.sh >= H and Q * spec.sw >= W
            if not accumulate and not fill:
                dx.zero_()  # cells that do not tile dx: pixels past the last cell stay 0
            geom = [N, P, Q, Cdz, ld(dz), P, Q, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1, spec.cin_pad, K, Kpad,
                    ld(dx), 2 if fill else 1, H, W, spec.sh, spec.sw, 1 if accumulate else 0, _f32o(dx)]
        else:
            M = N * H * W
            pt = spec.dh * (spec.kh - 1) - spec.pt
            pl = spec.dw * (spec.kw - 1) - spec.pl
            geom = [N, P, Q, Cdz, ld(dz), H, W, spec.kh, spec.kw, 1, 1, pt, pl, spec.dh, spec.dw,
                    spec.sh, spec.sw, spec.cin_pad, K, Kpad, ld(dx), 0, H, W, 1, 1,
                    1 if accumulate else 0, _f32o(dx)]
        taps = spec.kh * spec.kw
        if dz.dtype == torch.float32:  # fp32 path: Planes operands (bf16x6 GEMM, conv_p3.hip)
            w_lo = lo_pack(wtr)
            assert w_lo is not None, "fp32 data gradient needs the mid / lo weight packs"
            dz = to_planes(dz)
            geom[4] = ld(dz)
            cfg, splits = _plan3(cfg, M, spec.cin_pad, K, dz.device, taps)
            _p3_dgrad_launch(dz, wtr, w_lo, dx, accumulate, geom + [0, 0, splits], cfg, bnb)
            return dx
        if cfg is None and bnb is not None:
            cfg = _tuned.get(dgb_key(M, spec.cin_pad, K, taps))
        cfg, splits = _plan(cfg, M, spec.cin_pad, K, dz.device, taps)
        geom = geom + [0, 0, splits]
        if bnb is not None:
            _ext.ops().conv_igemm_bnb(dz, wtr, dx, dx if accumulate else None, geom, cfg, bnb.z,
                                      bnb.y if bnb.mode == 1 else None, ld(bnb.z), bnb.saved.mean,
                                      bnb.saved.invstd, bnb.gamma, bnb.beta, bnb.acc, bnb.R, bnb.mode)
        else:
            _ext.ops().conv_igemm(dz, wtr, dx, dx if accumulate else None, None, None, geom, cfg, None, None)
        return dx
    Hp = H + spec.pt + spec.pb
    Wp = W + spec.pl + spec.pr
    wt = w_master.permute(0, 3, 1, 2).to(dz.dtype)
    g = torch.nn.grad.conv2d_input((N, spec.cin_pad, Hp, Wp), wt, dz.permute(0, 3, 1, 2),
                                   stride=(spec.sh, spec.sw), dilation=(spec.dh, spec.dw))
    g = g[:, :, spec.pt:spec.pt + H, spec.pl:spec.pl + W].permute(0, 2, 3, 1)
    if accumulate:
        dx.add_(g)
    else:
        dx.copy_(g)
    if bnb is not None:
        bnb.gate_cpu(dx)
    return dx


# ---------------------------------------------------------------- conv weight grad
def conv_wgrad(dz, x, spec: ConvSpec, dw, cfg=None):
    """dw[cout, kh, kw, cin_pad] (fp32) += sum over pixels of dz (x) im2col(x)."""
    N, H, W, _ = x.shape
    _, P, Q, _ = dz.shape
    if native(dz) and dz.dtype == torch.float32:  # fp32 path: Planes operands (conv_p3.hip)
        dz, x = to_planes(dz), to_planes(x)
        M = N * P * Q
        cfg, splits = cfg if cfg is not None else wgrad_p3_plan(spec.cout, spec.K, M, spec.kh * spec.kw)
        if _DET[0]:
            splits = 1
        geom = [N, H, W, spec.cin_pad, ld(x), P, Q, spec.kh, spec.kw, spec.sh, spec.sw, spec.pt, spec.pl,
                spec.dh, spec.dw, spec.cout, ld(dz)]
        _ext.ops().conv_wgrad_p3(dz.t, x.t, dw, geom, int(cfg), int(splits))
        return dw
    if native(dz):
        M = N * P * Q
        cfg, splits = cfg if cfg is not None else wgrad_cfg(spec.cout, spec.K, M, spec.kh * spec.kw)
        if _DET[0]:
            splits = 1  # sole writer per dW tile: no float atomics
        geom = [N, H, W, spec.cin_pad, ld(x), P, Q, spec.kh, spec.kw, spec.sh, spec.sw, spec.pt, spec.pl,
                spec.dh, spec.dw, spec.cout, ld(dz)]
        _ext.ops().conv_wgrad(dz, x, dw, geom, cfg, splits)
        return dw
    xt = x.permute(0, 3, 1, 2)
    if spec.pt or spec.pb or spec.pl or spec.pr:
        xt = F.pad(xt, (spec.pl, spec.pr, spec.pt, spec.pb))
    g = torch.nn.grad.conv2d_weight(xt, (spec.cout, spec.cin_pad, spec.kh, spec.kw), dz.permute(0, 3, 1, 2),
                                    stride=(spec.sh, spec.sw), dilation=(spec.dh, spec.dw))
    dw.add_(g.permute(0, 2, 3, 1).reshape(dw.shape).to(dw.dtype))
    return dw


# --------------------------------------------------------------------------- BN
class BNSaved:
    __slots__ = ("mean", "invstd")

    def __init__(self, mean, invstd):
        self.mean = mean
        self.invstd = invstd


def bn_inference(z, gamma, beta, running_mean, running_var, eps, out, relu: bool, residual=None):
    """Inference BN (``--forward_only``: tf_cnn_benchmarks builds the model with
    phase_train=False): out = act(gamma*(z-moving_mean)/sqrt(moving_var+eps) + beta [+ res])."""
    N, H, W, C = z.shape
    if native(z) and z.dtype == torch.float32:
        # fp32 path: the fp32 apply kernel of training (bn_apply_acc, z / out / residual fp32) fed
        # moving statistics as one replica of shifted sums -- shift = moving mean, sum 0, sum of
        # squares M * moving var -- so its mean is the moving mean exactly and its variance the moving
        # variance to an ulp; no running-stat pointers (nothing updated), scratch saved stats
        M = N * H * W
        acc = torch.stack([torch.zeros_like(running_var), running_var * float(M)]).unsqueeze(0).contiguous()
        scratch = torch.empty(2, C, dtype=torch.float32, device=z.device)
        if residual is not None:  # the kernel reads a residual in out's format (fp32, or planes)
            if is_planes(out) and not is_planes(residual):
                residual = to_planes(residual)
            elif not is_planes(out) and is_planes(residual):
                residual = from_planes(residual)
        _ext.ops().bn_apply_acc(z, ld(z), _pl(out), ld(out), _pl(residual), ld(residual) if residual is not None else 0,
                                M, C, acc, 1, eps, 1.0, gamma, beta, 1 if relu else 0, scratch[0], scratch[1],
                                None, None, running_mean)
        return out
    invstd = torch.rsqrt(running_var + eps)
    if native(z):
        _ext.ops().bn_apply(z, ld(z), out, ld(out), residual, ld(residual) if residual is not None else 0,
                            N * H * W, C, running_mean, invstd, gamma, beta, 1 if relu else 0)
        return out
    y = (z - running_mean) * (invstd * gamma) + beta
    if residual is not None:
        y = y + residual
    out.copy_(torch.relu(y) if relu else y)
    return out


def bn_forward(z, gamma, beta, running_mean, running_var, momentum, eps, out, relu: bool,
               residual=None, stats=None, stats_T: int = 0):
    """Training BN: batch stats (from a fused conv slab when given), running-stat update,
    out = act(gamma*xhat + beta [+ residual])."""
    N, H, W, C = z.shape
    M = N * H * W
    if native(z):
        hcb = _ext.ops()
        if stats is None:
            stats_T = hcb.bn_partials(M, C)
            stats = torch.empty(stats_T * 2 * C, dtype=torch.float32, device=z.device)
            hcb.bn_stats(z, M, C, ld(z), stats)
        mean = torch.empty(C, dtype=torch.float32, device=z.device)
        invstd = torch.empty_like(mean)
        hcb.bn_finalize(stats, stats_T, C, float(M), eps, momentum, mean, invstd, running_mean, running_var)
        hcb.bn_apply(z, ld(z), out, ld(out), residual, ld(residual) if residual is not None else 0, M, C,
                     mean, invstd, gamma, beta, 1 if relu else 0)
        return BNSaved(mean, invstd)
    zf = z.reshape(M, C) if z.is_contiguous() else z.contiguous().reshape(M, C)
    if zf.dtype == torch.float16:  # fused batch norm keeps its statistics in fp32 (TF semantics)
        zf = zf.float()
    mean = zf.mean(0)
    var = zf.var(0, unbiased=False)
    invstd = torch.rsqrt(var + eps)
    with torch.no_grad():
        if running_mean is not None:
            unb = var * M / max(M - 1, 1)
            running_mean.mul_(momentum).add_((1 - momentum) * mean)
            running_var.mul_(momentum).add_((1 - momentum) * unb)
    y = (z.to(mean.dtype) - mean) * (invstd * gamma) + beta
    if residual is not None:
        y = y + residual
    if relu:
        y = torch.relu(y)
    out.copy_(y)
    return BNSaved(mean, invstd)


def bn_forward_acc(z, gamma, beta, running_mean, running_var, momentum, eps, out, relu: bool, acc, R: int,
                   saved_mean, saved_invstd, residual=None, shift=None, res_bn=None):
    """GPU BN forward whose batch statistics were accumulated by the producing conv's epilogue
    into ``acc`` (R replicas of [2][C]); mean/invstd are derived inside the apply kernel (no
    finalize launch) and written to saved_mean / saved_invstd for the backward. ``shift``:
    the per-channel offset the producing conv subtracted before accumulating (conv_forward).
    ``res_bn`` = (acc, gamma, beta, saved_mean, saved_invstd, running_mean, running_var, shift) of a
    second BN applied to ``residual`` in the same pass (a projection shortcut's raw conv output:
    its normalised tensor is never written); same M, C and replica count R."""
    N, H, W, C = z.shape
    M = N * H * W
    _ext.ops().bn_apply_acc(z, ld(z), _pl(out), ld(out), _pl(residual), ld(residual) if residual is not None else 0,
                            M, C, acc, R, eps, momentum, gamma, beta, 1 if relu else 0, saved_mean, saved_invstd,
                            running_mean, running_var, shift, *(res_bn or ()))
    return BNSaved(saved_mean, saved_invstd)


def bn_relu_maxpool_acc(z, gamma, beta, running_mean, running_var, momentum, eps, acc, R: int, saved_mean,
                        saved_invstd, out, argmax, kh, kw, sh, sw, pads, shift=None):
    """GPU: BN (conv-epilogue statistics in ``acc``) + ReLU + max pool in one kernel; writes the
    pooled ``out`` and the uint8 window ``argmax`` only (the BN+ReLU activation is not stored)."""
    N, H, W, C = z.shape
    _, P, Q, _ = out.shape
    pt, pb, pl, pr = pads
    _ext.ops().bn_relu_maxpool_acc(z, _pl(out), argmax, [N, H, W, C, P, Q, ld(out), kh, kw, sh, sw, pt, pl], acc, R, eps,
                                   momentum, gamma, beta, saved_mean, saved_invstd, running_mean, running_var, shift)
    return BNSaved(saved_mean, saved_invstd)


def bn_stats_acc(x, acc, R: int, shift=None):
    """GPU BN statistics of ``x`` [N, H, W, C] (fp32 or 16-bit, rows of C channels, row stride ld(x))
    accumulated into ``acc`` (R replicas of [2][C], zeroed per step): sums of (v - shift) and
    (v - shift)^2 -- what a producing conv's epilogue leaves for bn_forward_acc, for a BN whose
    input is not a GEMM output (ResNet v2's pre-activation / final BN)."""
    C = x.shape[-1]
    _ext.ops().bn_stats_acc(x, ld(x), x.numel() // C, C, acc, R, shift)


def from_planes(x):
    """Planes -> the fp32 tensor (hi + mid + lo, exact; one launch on the GPU)."""
    if not isinstance(x, Planes):
        return x
    C = x.shape[-1]
    out = torch.empty(tuple(x.shape), dtype=torch.float32, device=x.device)
    if x.is_cuda:
        _ext.ops().merge_planes(x.t, ld(x), x.numel() // C, C, out, C)
        return out
    out.copy_(x.float())
    return out


def bn_backward_acc(dy, y, z, saved: BNSaved, gamma, beta, relu_mode: int, dgamma, dbeta, dz, acc, R: int,
                    gres=None, pre_reduced: bool = False, shift_out=None, pool=None, add=None):
    """GPU BN(+ReLU) backward with the dgamma/dbeta reduction accumulated in ``acc`` replicas
    (zeroed per step) and consumed directly by the apply kernel. ``pre_reduced``: dy is already
    the gated g and ``acc`` already holds its sums (a BNBwdFuse data-grad epilogue produced it),
    so only the apply pass runs. ``shift_out``: receives this step's batch mean, the statistics
    shift of the layer's next forward. ``pool`` = (amax, [H, W, P, Q, k, s, pt, pl]): dy is the
    gradient of the max pool that followed this BN+ReLU (the ResNet stem) and both passes gather
    the full-size dy from it through the pool's argmax (it is never materialised). ``add``: a tensor of
    dz's layout added to dz in the apply pass (dz = BN'(dy) + add; plain dz, not planes)."""
    N, H, W, C = z.shape
    M = N * H * W
    hcb = _ext.ops()
    if pre_reduced:
        assert gres is None, "pre-reduced dy is itself the residual gradient"
        hcb.bn_bwd_apply_acc(dy, ld(dy), None, 0, z, ld(z), _pl(dz), ld(dz), M, C, saved.mean, saved.invstd, gamma,
                             beta, acc, R, dgamma, dbeta, 0, shift_out)
        return dz
    ym = _pl(y) if relu_mode == 1 else None
    pa, pg = pool if pool is not None else (None, None)
    hcb.bn_bwd_reduce_acc(dy, ld(dy), ym, ld(y) if relu_mode == 1 else 0, z, ld(z), M, C, saved.mean, saved.invstd,
                          gamma, beta, relu_mode, acc, R, gres, ld(gres) if gres is not None else 0, pa, pg)
    hcb.bn_bwd_apply_acc(dy, ld(dy), ym, ld(y) if relu_mode == 1 else 0, z, ld(z), _pl(dz), ld(dz), M, C, saved.mean,
                         saved.invstd, gamma, beta, acc, R, dgamma, dbeta, relu_mode, shift_out, pa, pg, add,
                         ld(add) if add is not None else 0)
    return dz


def bn_backward(dy, y, z, saved: BNSaved, gamma, beta, relu_mode: int, dgamma, dbeta, dz, gres=None):
    """BN(+ReLU) backward. relu_mode: 0 none, 1 mask from stored output y (residual blocks),
    2 mask recomputed from z. Writes dgamma/dbeta (fp32, overwrite), dz, and optionally the
    masked upstream gradient gres (the residual branch's gradient)."""
    N, H, W, C = z.shape
    M = N * H * W
    if native(z):
        hcb = _ext.ops()
        T = hcb.bn_partials(M, C)
        slab = torch.empty(T * 2 * C, dtype=torch.float32, device=z.device)
        hcb.bn_bwd_reduce(dy, ld(dy), y if relu_mode == 1 else None, ld(y) if relu_mode == 1 else 0, z, ld(z),
                          M, C, saved.mean, saved.invstd, gamma, beta, relu_mode, slab, gres,
                          ld(gres) if gres is not None else 0)
        hcb.bn_bwd_finalize(slab, T, C, dgamma, dbeta)
        hcb.bn_bwd_apply(dy, ld(dy), y if relu_mode == 1 else None, ld(y) if relu_mode == 1 else 0, z, ld(z),
                         dz, ld(dz), M, C, saved.mean, saved.invstd, gamma, beta, dgamma, dbeta, relu_mode)
        return dz
    if z.dtype == torch.float16:  # backward reductions in fp32 as well
        z, dy = z.float(), dy.float()
        y = y.float() if y is not None else None
    xhat = (z - saved.mean) * saved.invstd
    g = dy
    if relu_mode == 1:
        g = dy * (y > 0).to(dy.dtype)
    elif relu_mode == 2:
        g = dy * ((xhat * gamma + beta) > 0).to(dy.dtype)
    gf = g.reshape(-1, C) if g.is_contiguous() else g.contiguous().reshape(-1, C)
    xf = xhat.reshape(-1, C)
    db = gf.sum(0)
    dg = (gf * xf).sum(0)
    dbeta.copy_(db)
    dgamma.copy_(dg)
    dz.copy_(gamma.to(g.dtype) * saved.invstd * (g - db / M - xhat * dg / M))
    if gres is not None:
        gres.copy_(g)
    return dz


# ----------------------------------------------------------------------- pooling
def pool_geom(x, out, kh, kw, sh, sw, pt, pl, is_max, incl_pad):
    N, H, W, C = x.shape
    _, P, Q, _ = out.shape
    return [N, H, W, C, ld(x), P, Q, ld(out), kh, kw, sh, sw, pt, pl, 1 if is_max else 0, 1 if incl_pad else 0]


def pool_forward(x, out, kh, kw, sh, sw, pads, is_max, incl_pad=False, argmax=None):
    """argmax (GPU, max pool): uint8 [N,P,Q,C] window position of the first maximum, which
    makes the backward a cheap gather."""
    pt, pb, pl, pr = pads
    if is_planes(x):  # fp32 path: planes in, planes out (the consumer is a GEMM or a concat window)
        assert is_planes(out), "a pool of Planes writes Planes"
        _ext.ops().pool_fwd_p3(x.t, out.t, argmax, pool_geom(x, out, kh, kw, sh, sw, pt, pl, is_max, incl_pad))
        return out
    if native(x):
        _ext.ops().pool_fwd(x, out, argmax, pool_geom(x, out, kh, kw, sh, sw, pt, pl, is_max, incl_pad))
        return out
    xt = x.permute(0, 3, 1, 2)
    if is_max:
        xt = F.pad(xt, (pl, pr, pt, pb), value=-float("inf"))
        y = F.max_pool2d(xt, (kh, kw), (sh, sw))
    else:
        if incl_pad:
            y = F.avg_pool2d(F.pad(xt, (pl, pr, pt, pb)), (kh, kw), (sh, sw))
        else:
            ones = torch.ones_like(xt[:, :1])
            s = F.avg_pool2d(F.pad(xt, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
            c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
            y = s / c
    out.copy_(y.permute(0, 2, 3, 1))
    return out


def pool_backward(dy, x, y, dx, kh, kw, sh, sw, pads, is_max, incl_pad=False, accumulate=False, argmax=None):
    pt, pb, pl, pr = pads
    if is_planes(x) or is_planes(y):
        # fp32 path (the ResNet stem pool, Inception's pools): the argmax gather and the 3x3/1
        # average gather read dy (and the argmax) only -- x / y stand in with fp32 tensors of
        # their shapes (dx / dy)
        assert (is_max and argmax is not None) or (not is_max and (kh, kw, sh, sw) == (3, 3, 1, 1))
        y = dy
        if is_planes(x):
            x = dx
    if native(x):
        # the kernel walks x / dx with one pixel stride and y / dy with another: align views
        if ld(y) != ld(dy):
            y = y.contiguous() if ld(dy) == y.shape[3] else y
            dy = dy.contiguous() if ld(y) != ld(dy) else dy
        if ld(dx) != ld(x):
            tmp = dx.contiguous() if accumulate else torch.empty(dx.shape, dtype=dx.dtype, device=dx.device)
            xc = x.contiguous()
            _ext.ops().pool_bwd(dy, xc, y, argmax, tmp, pool_geom(xc, dy, kh, kw, sh, sw, pt, pl, is_max, incl_pad),
                                accumulate)
            dx.copy_(tmp)
            return dx
        _ext.ops().pool_bwd(dy, x, y, argmax, dx, pool_geom(x, dy, kh, kw, sh, sw, pt, pl, is_max, incl_pad),
                            accumulate)
        return dx
    with torch.enable_grad():
        xr = x.detach().clone().requires_grad_(True)
        yy = torch.empty_like(y)
        xt = xr.permute(0, 3, 1, 2)
        if is_max:
            t = F.max_pool2d(F.pad(xt, (pl, pr, pt, pb), value=-float("inf")), (kh, kw), (sh, sw))
        elif incl_pad:
            t = F.avg_pool2d(F.pad(xt, (pl, pr, pt, pb)), (kh, kw), (sh, sw))
        else:
            ones = torch.ones_like(xt[:, :1])
            s = F.avg_pool2d(F.pad(xt, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
            c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
            t = s / c
        del yy
        (g,) = torch.autograd.grad(t, xr, dy.permute(0, 3, 1, 2))
    if accumulate:
        dx.add_(g)
    else:
        dx.copy_(g)
    return dx


def gap_forward(x, out):
    N, H, W, C = x.shape
    if is_planes(x):
        out = out if is_planes(out) else None
        assert out is not None, "gap_forward of Planes writes Planes"
        _ext.ops().gap_fwd_p3(x.t, out.t, N, H * W, C)
        return out
    if native(x):
        assert x.is_contiguous()
        _ext.ops().gap_fwd(x, out, N, H * W, C)
        return out
    out.copy_(x.mean(dim=(1, 2)))
    return out


def gap_backward(dy, dx):
    N, H, W, C = dx.shape
    if native(dy):
        _ext.ops().gap_bwd(dy, dx, N, H * W, C)
        return dx
    dx.copy_((dy / (H * W)).view(N, 1, 1, C).expand(N, H, W, C))
    return dx


# ------------------------------------------------------------------------- loss
def softmax_xent(logits, labels, ncls, row_loss, dlogits, scale, scale_dev=None, dl32=None,
                 label_smoothing: float = 0.0):
    """Per-row cross entropy (into row_loss) and dlogits = (softmax - target) * scale, target =
    onehot, or (1 - ls) * onehot + ls / ncls with ``label_smoothing`` ls (tf_cnn_benchmarks
    --label_smoothing through tf.losses.softmax_cross_entropy)
    (* scale_dev[0], a device-resident loss scale, when given); ``dl32``: with 16-bit dlogits,
    also the unrounded fp32 values (same layout), from which the classifier's bias gradient is
    summed (its batch sum cancels to ~1% of the terms: bf16 rounding of each term would cost
    ~5x the error of the fp32-loss reference, tools/bf16_floor.py)."""
    B = labels.numel()
    if native(dlogits):
        _ext.ops().softmax_xent(logits, ld(logits), labels, ncls, row_loss, dlogits, ld(dlogits), scale, scale_dev,
                                dl32, float(label_smoothing))
        return
    if scale_dev is not None:
        scale = scale * float(scale_dev.reshape(-1)[0])
    lg = logits[:, :ncls].float()
    lse = torch.logsumexp(lg, dim=1)
    ls = float(label_smoothing)
    pos, neg = 1.0 - ls, ls / ncls
    row_loss.copy_(lse - pos * lg.gather(1, labels.view(-1, 1)).view(-1) - (neg * lg.sum(1) if ls else 0.0))
    p = torch.softmax(lg, dim=1)
    if ls:
        p -= neg
    p[torch.arange(B), labels] -= pos
    dlogits.zero_()
    dlogits[:, :ncls].copy_(p * scale)


def add(a, b, out=None):
    """out = a + b on activations (bf16 HIP kernel on the GPU)."""
    out = torch.empty_like(a) if out is None else out
    if native(a):
        a, b = a.contiguous(), b.contiguous()
        _ext.ops().add_bf16(a, b, out)
        return out
    torch.add(a, b, out=out)
    return out


def dropout_forward(x, y, mask, keep: float, seed: int, step):
    """y = x * m / keep with m ~ Bernoulli(keep) (tf.nn.dropout). GPU: the mask is a hash of
    (seed, step[0], index), one bit per element in ``mask`` (uint8, numel/8); ``step`` is a
    device int64 counter so captured-graph replays draw fresh masks. CPU: ``mask`` is a bool
    tensor of x's shape drawn from a generator seeded with (seed, step)."""
    if native(x):
        _ext.ops().dropout_fwd(x, y, mask, float(keep), int(seed), step)
        return y
    g = torch.Generator().manual_seed(int(seed) * 1000003 + int(step[0]))
    m = (torch.rand(x.shape, generator=g) < keep).to(x.device)
    mask.copy_(m)
    y.copy_(x * m.to(x.dtype) / keep)
    return y


def dropout_backward(dy, mask, dx, keep: float):
    if native(dy):
        _ext.ops().dropout_bwd(dy, mask, dx, float(keep))
        return dx
    dx.copy_(dy * mask.to(dy.dtype) / keep)
    return dx


def colsum(g, M, N, out):
    if native(g):
        _ext.ops().colsum(g, ld(g), M, N, out)
        return out
    out.copy_(g[:M, :N].float().sum(0))
    return out


# -------------------------------------------------------------------- optimizer
def nonfinite(g, flag):
    """flag[0] = 1 if g holds an Inf/NaN (flag must be zeroed by the caller)."""
    if g.is_cuda:  # the fp32 flat gradient buffer: same kernel in every compute mode
        _ext.ops().nonfinite(g, flag)
        return
    if not bool(torch.isfinite(g).all()):
        flag.view(-1)[0] = 1.0


def loss_total(row_loss, B: int, l2, half_wd: float, loss):
    """loss[0] = mean(row_loss[:B]) + half_wd * l2[0] (l2 None: the mean alone) -- the step's reported
    loss in one launch (tf_cnn_benchmarks' total_loss = cross entropy + weight decay * l2 term)."""
    if row_loss.is_cuda:
        _ext.ops().loss_total(row_loss, B, l2, half_wd, loss)
        return
    t = row_loss[:B].mean()
    if l2 is not None:
        t = t + half_wd * l2.view(-1)[0]
    loss.view(-1)[0] = t


def loss_scale_update(hyper, world: int, dynamic: bool):
    """hyper = [lr, mu, wd, grad_scale, found_inf, loss_scale, good_steps, interval]: dynamic
    loss-scale step (halve on overflow, double after `interval` clean steps), then
    grad_scale = 1 / (world * loss_scale)."""
    if hyper.is_cuda:
        _ext.ops().loss_scale_update(hyper, float(world), bool(dynamic))
        return
    h = hyper
    S = float(h[5])
    if dynamic:
        if float(h[4]) != 0.0:
            S = max(S * 0.5, 1.0)
            h[6] = 0.0
        else:
            h[6] += 1.0
            if float(h[6]) >= float(h[7]):
                S *= 2.0
                h[6] = 0.0
        h[5] = S
    h[3] = 1.0 / (world * S)


def sgd_momentum(w, mom, g, n_decay, hyper, l2=None, nesterov=False):
    """TF ApplyMomentum on the flat parameter buffer: hyper = [lr, momentum, wd, grad_scale
    (, found_inf, ...)]; a set found_inf skips the update (loss scaling)."""
    if w.is_cuda:
        _ext.ops().sgd_momentum(w, mom, g, n_decay, hyper, l2, nesterov)
        return
    if hyper.numel() > 4 and float(hyper[4]) != 0.0:
        return
    lr, mu, wd, gs = [float(v) for v in hyper[:4].tolist()]
    gg = g * gs
    if n_decay > 0:
        if l2 is not None:
            l2 += (w[:n_decay] * w[:n_decay]).sum()
        gg[:n_decay] += wd * w[:n_decay]
    mom.mul_(mu).add_(gg)
    if nesterov:
        w.sub_(lr * (gg + mu * mom))
    else:
        w.sub_(lr * mom)
