// torch.library registrations (namespace `hcb`; `hcb16` for the IEEE-fp16 build of the same
// sources, -DHCB_F16 -Dhcb=hcb16) for the hand-written gfx950 kernels.
//
// Every op is a thin, allocation-free launcher: Python pre-allocates outputs with the
// caching allocator (so the whole training step can be captured in a HIP graph) and
// passes geometry as an int list; the launcher validates shapes / byte ranges on the
// host BEFORE anything reaches the GPU (an out-of-range gather must never be launched)
// and enqueues on the current HIP stream.
#include <algorithm>
#include <vector>

#include <torch/library.h>
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <c10/hip/HIPStream.h>
#include <c10/util/Exception.h>

#include "kernels/kernels.h"

using at::Tensor;

#ifdef HCB_F16
constexpr at::ScalarType kAct = at::kHalf;  // 16-bit activation / GEMM operand type of this build
#define HCB_ACT_NAME "float16"
#else
constexpr at::ScalarType kAct = at::kBFloat16;
#define HCB_ACT_NAME "bfloat16"
#endif
// library name through one macro level, so -Dhcb=hcb16 also renames the torch.library namespace
#define HCB_TORCH_LIBRARY(ns, m) TORCH_LIBRARY(ns, m)
#define HCB_TORCH_LIBRARY_IMPL(ns, k, m) TORCH_LIBRARY_IMPL(ns, k, m)

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// raw pointers (the Python side owns and keeps the tensors alive; no static Tensor dtor at exit)
float* g_splitk_ws = nullptr;
int64_t g_splitk_ws_bytes = 0;
unsigned* g_splitk_cnt = nullptr;
int64_t g_splitk_cnt_n = 0;

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "hcb: ", name, " must be a GPU tensor");
}
void check_act(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == kAct, "hcb: ", name, " must be " HCB_ACT_NAME " (the activation dtype of this build)");
}
// an activation of this build's 16-bit type, or (bf16 library only) fp32 -- the reference
// precision path (--compute_dtype fp32); returns true for fp32
bool check_act_or_f32(const Tensor& t, const char* name) {
  check_cuda(t, name);
#ifndef HCB_F16
  if (t.scalar_type() == at::kFloat) return true;
#endif
  TORCH_CHECK(t.scalar_type() == kAct, "hcb: ", name, " must be " HCB_ACT_NAME " or float32");
  return false;
}
bool same_act(const Tensor& a, const Tensor& b, const char* name) {
  const bool f = check_act_or_f32(b, name);
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "hcb: ", name, " dtype differs from the other activations");
  return f;
}
void check_f32(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, "hcb: ", name, " must be float32");
}
// bytes addressable from t.data_ptr() to the end of its storage
int64_t avail_bytes(const Tensor& t) {
  return (int64_t)t.storage().nbytes() - t.storage_offset() * (int64_t)t.element_size();
}
void check_range(const Tensor& t, int64_t need_bytes, const char* name) {
  TORCH_CHECK(need_bytes <= avail_bytes(t), "hcb: ", name, " needs ", need_bytes,
              " bytes but only ", avail_bytes(t), " are addressable");
}
void check_align16(const void* p, const char* name) {
  TORCH_CHECK(((uintptr_t)p & 15) == 0, "hcb: ", name, " must be 16-byte aligned");
}

// fp32 path (conv_p3.hip): a plane tensor is bf16 [3, ...] (plane t = select(0, t))
int64_t check_planes(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() >= 2 && t.size(0) == 3,
              "hcb: ", name, " must be bf16 planes [3, ...]");
  TORCH_CHECK(t.stride(-1) == 1, "hcb: ", name, " channels must be contiguous");
  check_align16(t.data_ptr(), name);
  TORCH_CHECK((t.stride(0) * 2) % 16 == 0, "hcb: ", name, " plane stride must keep 16-byte alignment");
  return t.stride(0);  // elements between planes
}

// Bytes of an NHWC conv input that the kernels may address. ldx < C is a ROW WINDOW: pixel w's C
// "channels" are the ldx channels of pixels w, w+1, ... (the space-to-depth stem's 4x4 filter read as
// 4x1 over 64-channel windows of 16-channel pixels: one contiguous 128-byte row per filter row,
// StemS2D.fold_spec); the buffer then ends with the tensor and the windows of the last pixels, which
// no output reads, run out of range (zeros).
static int64_t x_span_bytes(int64_t N, int64_t H, int64_t W, int64_t C, int64_t ldx, int64_t e) {
  return ldx >= C ? ((N * H * W - 1) * ldx + C) * e : N * H * W * ldx * e;
}

// geom = [N,H,W,C,ldx, P,Q,R,S, sh,sw,ph,pw,dh,dw,idh,idw, Nout,K,Kpad,ldy,
//         remap,OH,OW,osh,osw, beta,out_f32]
hcb::ConvParams conv_params(const Tensor& x, const Tensor& w, const Tensor& y, const c10::optional<Tensor>& yres,
                            const c10::optional<Tensor>& bias, const c10::optional<Tensor>& stats,
                            at::IntArrayRef g, int64_t cfg) {
  TORCH_CHECK(g.size() >= 28 && g.size() <= 33,
              "hcb.conv_igemm: geom must have 28 (+relu, +stats_R, +splits, +remap origin h, w) entries");
  const bool f32 = check_act_or_f32(x, "x");  // fp32: bf16x6 path (w = high pack, w_lo set by the caller)
  check_act(w, "w");
  check_cuda(y, "y");
  hcb::ConvParams p{};
  p.N = g[0]; p.H = g[1]; p.W = g[2]; p.C = g[3]; p.ldx = g[4];
  p.P = g[5]; p.Q = g[6]; p.R = g[7]; p.S = g[8];
  p.stride_h = g[9]; p.stride_w = g[10]; p.pad_h = g[11]; p.pad_w = g[12];
  p.dil_h = g[13]; p.dil_w = g[14]; p.idil_h = g[15]; p.idil_w = g[16];
  p.Nout = g[17]; p.K = g[18]; p.Kpad = g[19]; p.ldy = g[20];
  p.remap = g[21]; p.OH = g[22]; p.OW = g[23]; p.osh = g[24]; p.osw = g[25];
  p.beta = g[26]; p.out_f32 = g[27];
  p.relu = g.size() > 28 ? (int)g[28] : 0;
  p.stats_R = g.size() > 29 ? (int)g[29] : 0;
  p.splits = g.size() > 30 ? (int)g[30] : 1;
  p.oh0 = g.size() > 31 ? (int)g[31] : 0;
  p.ow0 = g.size() > 32 ? (int)g[32] : 0;
  p.M = p.N * p.P * p.Q;
  TORCH_CHECK(p.C % 8 == 0 && p.ldx % 8 == 0 && (p.ldx >= p.C || p.C % p.ldx == 0),
              "hcb.conv_igemm: C, ldx must be multiples of 8 (ldx < C: a row window, C a multiple of ldx)");
  TORCH_CHECK(p.Kpad % 64 == 0 && p.Kpad >= p.K && p.K == p.R * p.S * p.C,
              "hcb.conv_igemm: Kpad must be a multiple of 64 >= K = R*S*C");
  TORCH_CHECK(p.ldy % 8 == 0 && p.ldy >= ((p.Nout + 7) / 8) * 8, "hcb.conv_igemm: bad ldy");
  TORCH_CHECK(p.idil_h >= 1 && p.idil_w >= 1 && p.dil_h >= 1 && p.dil_w >= 1, "hcb.conv_igemm: bad dilation");
  TORCH_CHECK(p.M > 0 && p.Nout > 0, "hcb.conv_igemm: empty problem");
  const int64_t xe = f32 ? 4 : 2;
  int64_t xb = x_span_bytes(p.N, p.H, p.W, p.C, p.ldx, xe);
  int64_t wb = (int64_t)p.Nout * p.Kpad * 2;
  TORCH_CHECK(xb < (1ll << 31) && wb < (1ll << 31), "hcb.conv_igemm: operand exceeds 2 GiB buffer range");
  check_range(x, xb, "x");
  check_range(w, wb, "w");
  int64_t rows = p.remap ? (int64_t)p.N * p.OH * p.OW : (int64_t)p.M;
  TORCH_CHECK(p.remap >= 0 && p.remap <= 2, "hcb.conv_igemm: remap is 0, 1 or 2");
  if (p.remap) {
    TORCH_CHECK(p.oh0 >= 0 && p.ow0 >= 0 && (p.P - 1) * p.osh + p.oh0 < p.OH && (p.Q - 1) * p.osw + p.ow0 < p.OW,
                "hcb.conv_igemm: remap out of range");
    // remap 2 zeroes each GEMM pixel's whole stride cell: the cells must cover the output
    TORCH_CHECK(p.remap != 2 || (!p.beta && p.oh0 == 0 && p.ow0 == 0 && p.P * p.osh >= p.OH && p.Q * p.osw >= p.OW),
                "hcb.conv_igemm: remap 2 needs cells covering the output and no beta");
  } else {
    TORCH_CHECK(p.oh0 == 0 && p.ow0 == 0, "hcb.conv_igemm: a remap origin needs remap");
  }
  int64_t esz = p.out_f32 ? 4 : 2;
  TORCH_CHECK(!f32 || p.out_f32, "hcb.conv_igemm: fp32 inputs give an fp32 output (out_f32)");
  TORCH_CHECK(y.scalar_type() == (p.out_f32 ? at::kFloat : kAct), "hcb.conv_igemm: y dtype");
  check_range(y, rows * p.ldy * esz - (p.ldy - ((p.Nout + 7) / 8) * 8) * esz, "y");
  check_align16(x.data_ptr(), "x");
  check_align16(w.data_ptr(), "w");
  check_align16(y.data_ptr(), "y");
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.y = y.data_ptr();
  p.yres = nullptr;
  if (p.beta) {
    TORCH_CHECK(yres.has_value(), "hcb.conv_igemm: beta needs yres");
    check_range(*yres, rows * p.ldy * esz - (p.ldy - ((p.Nout + 7) / 8) * 8) * esz, "yres");
    check_align16(yres->data_ptr(), "yres");
    p.yres = yres->data_ptr();
  }
  p.bias = nullptr;
  if (bias.has_value()) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() >= p.Nout, "hcb.conv_igemm: bias too small");
    p.bias = bias->data_ptr<float>();
  }
  p.stats = nullptr;
  if (stats.has_value()) {
    check_f32(*stats, "stats");
    int tiles_m = (p.M + hcb::conv_tile_m(cfg) - 1) / hcb::conv_tile_m(cfg);
    int64_t rows = p.stats_R > 0 ? p.stats_R : tiles_m;
    TORCH_CHECK(stats->numel() >= rows * 2 * p.Nout, "hcb.conv_igemm: stats buffer too small");
    p.stats = stats->data_ptr<float>();
  }
  p.x_bytes = (uint32_t)xb;
  p.w_bytes = (uint32_t)wb;
  TORCH_CHECK(p.splits >= 1 && p.splits <= p.Kpad / 64, "hcb.conv_igemm: 1 <= splits <= k-steps");
  if (p.splits > 1) {
    TORCH_CHECK(cfg >= 4, "hcb.conv_igemm: split-K needs an LDS-DMA config (cfg >= 4)");
    TORCH_CHECK(g_splitk_ws != nullptr && g_splitk_cnt != nullptr, "hcb.conv_igemm: split-K workspace not set");
    const int bm = hcb::conv_tile_m((int)cfg), bn = hcb::conv_tile_n((int)cfg);
    const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * ((p.Nout + bn - 1) / bn);
    TORCH_CHECK(tiles * p.splits * bm * bn * 4 <= g_splitk_ws_bytes, "hcb.conv_igemm: split-K workspace too small");
    TORCH_CHECK(tiles <= g_splitk_cnt_n, "hcb.conv_igemm: split-K counter array too small");
    p.ws = g_splitk_ws;
    p.cnt = g_splitk_cnt;
  }
  return p;
}

// split-K scratch shared by every conv launch of the process (one compute stream): fp32 slabs
// and zero-initialised per-tile tickets that the kernels leave zeroed
void set_splitk_workspace(const Tensor& ws, const Tensor& cnt) {
  check_f32(ws, "ws");
  check_cuda(cnt, "cnt");
  TORCH_CHECK(cnt.scalar_type() == at::kInt && cnt.is_contiguous() && ws.is_contiguous(), "hcb: bad split-K workspace");
  g_splitk_ws = ws.data_ptr<float>();
  g_splitk_ws_bytes = ws.numel() * 4;
  g_splitk_cnt = reinterpret_cast<unsigned*>(cnt.data_ptr<int>());
  g_splitk_cnt_n = cnt.numel();
}

void set_p3p_bnb(int64_t v) {
  TORCH_CHECK(v >= 0 && v <= 2, "hcb.set_p3p_bnb: 0, 1 or 2");
  hcb::set_p3p_bnb((int)v);
}

const float* opt_f32(const c10::optional<Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value()) return nullptr;
  check_f32(*t, what);
  TORCH_CHECK(t->numel() >= n, "hcb: ", what, " too small");
  return t->data_ptr<float>();
}

void conv_igemm(const Tensor& x, const Tensor& w, const Tensor& y, const c10::optional<Tensor>& yres,
                const c10::optional<Tensor>& bias, const c10::optional<Tensor>& stats,
                at::IntArrayRef g, int64_t cfg, const c10::optional<Tensor>& stats_shift,
                const c10::optional<Tensor>& w_lo) {
  hcb::ConvParams p = conv_params(x, w, y, yres, bias, stats, g, cfg);
  TORCH_CHECK(!stats_shift.has_value() || p.stats != nullptr, "hcb.conv_igemm: stats_shift without stats");
  p.stats_shift = opt_f32(stats_shift, p.Nout, "stats_shift");
  p.w_lo = p.w_lo2 = nullptr;
  TORCH_CHECK(x.scalar_type() != at::kFloat && !w_lo.has_value(),
              "hcb.conv_igemm: 16-bit operands only (fp32 runs on the plane GEMMs: hcb.conv_p3)");
  hcb::launch_conv_igemm(p, (int)cfg, cur_stream());
}

// data-grad conv whose output is the dy of a BN layer: the epilogue gates it with the
// layer's ReLU mask (mode 1: y > 0, 2: recomputed from z, 0: none), stores g and adds
// sum(g), sum(g*xhat) per channel into acc [R][2][Nout] (see ConvParams::bnb_*)
// the fused BN-backward fields of a data-grad GEMM; f32: the fp32 path (z fp32, y the [3, ...] bf16
// planes of the activation -- the epilogue reads the hi plane -- output g fp32)
void set_bnb(hcb::ConvParams& p, const Tensor& z, const c10::optional<Tensor>& yact, int64_t ld, const Tensor& mean,
             const Tensor& invstd, const Tensor& gamma, const Tensor& beta, const Tensor& acc, int64_t R, int64_t mode,
             bool f32) {
  TORCH_CHECK(!p.relu && p.bias == nullptr, "hcb.conv_igemm_bnb: no bias / relu");
  TORCH_CHECK(p.out_f32 == (f32 ? 1 : 0), "hcb.conv_igemm_bnb: 16-bit output (fp32 on the fp32 path)");
  TORCH_CHECK(mode >= 0 && mode <= 2 && R >= 1, "hcb.conv_igemm_bnb: bad mode / R");
  TORCH_CHECK(ld % 8 == 0 && ld >= ((p.Nout + 7) / 8) * 8, "hcb.conv_igemm_bnb: bad ld");
  int64_t rows = p.remap ? (int64_t)p.N * p.OH * p.OW : (int64_t)p.M;
  const int64_t zsz = f32 ? 4 : 2;
  if (f32)
    check_f32(z, "z");
  else
    check_act(z, "z");
  check_range(z, ((rows - 1) * ld + ((p.Nout + 7) / 8) * 8) * zsz, "z");
  check_align16(z.data_ptr(), "z");
  p.bnb_y = nullptr;
  if (mode == 1) {
    TORCH_CHECK(yact.has_value(), "hcb.conv_igemm_bnb: mode 1 needs y");
    if (f32)
      check_planes(*yact, "y");
    else
      check_act(*yact, "y");
    check_range(*yact, ((rows - 1) * ld + ((p.Nout + 7) / 8) * 8) * 2, "y");
    check_align16(yact->data_ptr(), "y");
    p.bnb_y = yact->data_ptr();
  }
  for (const Tensor* t : {&mean, &invstd, &gamma, &beta}) {
    check_f32(*t, "bn param");
    TORCH_CHECK(t->numel() >= p.Nout, "hcb.conv_igemm_bnb: per-channel tensor too small");
  }
  check_f32(acc, "acc");
  TORCH_CHECK(acc.numel() >= R * 2 * p.Nout, "hcb.conv_igemm_bnb: acc too small");
  p.bnb_z = z.data_ptr();
  p.bnb_ld = (int)ld;
  p.bnb_mean = mean.data_ptr<float>();
  p.bnb_invstd = invstd.data_ptr<float>();
  p.bnb_gamma = gamma.data_ptr<float>();
  p.bnb_beta = beta.data_ptr<float>();
  p.bnb_acc = acc.data_ptr<float>();
  p.bnb_mode = (int)mode;
  p.bnb_R = (int)R;
}


// data-grad conv whose output is the dy of a BN layer: the epilogue gates it with the
// layer's ReLU mask (mode 1: y > 0, 2: recomputed from z, 0: none), stores g and adds
// sum(g), sum(g*xhat) per channel into acc [R][2][Nout] (see ConvParams::bnb_*)
void conv_igemm_bnb(const Tensor& x, const Tensor& w, const Tensor& y, const c10::optional<Tensor>& yres,
                    at::IntArrayRef g, int64_t cfg, const Tensor& z, const c10::optional<Tensor>& yact,
                    int64_t ld, const Tensor& mean, const Tensor& invstd, const Tensor& gamma, const Tensor& beta,
                    const Tensor& acc, int64_t R, int64_t mode) {
  hcb::ConvParams p = conv_params(x, w, y, yres, c10::nullopt, c10::nullopt, g, cfg);
  set_bnb(p, z, yact, ld, mean, invstd, gamma, beta, acc, R, mode, false);
  hcb::launch_conv_igemm(p, (int)cfg, cur_stream());
}

int64_t conv_tiles_m(int64_t M, int64_t cfg) {
  int t = hcb::conv_tile_m((int)cfg);
  return (M + t - 1) / t;
}

// geom = [N,H,W,C,ldx, P,Q,R,S, sh,sw,ph,pw,dh,dw, Nout,ldy]
void conv_wgrad(const Tensor& dy, const Tensor& x, const Tensor& dw, at::IntArrayRef g, int64_t cfg,
                int64_t splits) {
  TORCH_CHECK(g.size() == 17, "hcb.conv_wgrad: geom must have 17 entries");
  const bool f32 = same_act(dy, x, "x");
  TORCH_CHECK(!f32, "hcb.conv_wgrad: 16-bit operands only (fp32 runs on the plane GEMMs: hcb.conv_wgrad_p3)");
  check_f32(dw, "dw");
  hcb::WgradParams p{};
  const int64_t e = 2;
  p.N = g[0]; p.H = g[1]; p.W = g[2]; p.C = g[3]; p.ldx = g[4];
  p.P = g[5]; p.Q = g[6]; p.R = g[7]; p.S = g[8];
  p.stride_h = g[9]; p.stride_w = g[10]; p.pad_h = g[11]; p.pad_w = g[12];
  p.dil_h = g[13]; p.dil_w = g[14];
  p.Nout = g[15]; p.ldy = g[16];
  p.K = p.R * p.S * p.C;
  p.M = p.N * p.P * p.Q;
  TORCH_CHECK(p.C % 8 == 0 && p.ldx % 8 == 0, "hcb.conv_wgrad: C, ldx multiples of 8");
  TORCH_CHECK(p.ldy % 8 == 0 && p.ldy >= p.Nout, "hcb.conv_wgrad: bad ldy");
  TORCH_CHECK(splits >= 1, "hcb.conv_wgrad: splits >= 1");
  int64_t xb = x_span_bytes(p.N, p.H, p.W, p.C, p.ldx, e);
  int64_t yb = ((int64_t)p.M - 1) * p.ldy * e + (int64_t)((p.Nout + 7) / 8) * 8 * e;
  TORCH_CHECK(xb < (1ll << 31) && yb < (1ll << 31), "hcb.conv_wgrad: operand exceeds 2 GiB");
  check_range(x, xb, "x");
  check_range(dy, yb, "dy");
  check_range(dw, (int64_t)p.Nout * p.K * 4, "dw");
  check_align16(x.data_ptr(), "x");
  check_align16(dy.data_ptr(), "dy");
  int nkt = (p.M + 63) / 64;
  int per = (nkt + (int)splits - 1) / (int)splits;
  p.ksteps_per_split = per;
  int eff_splits = (nkt + per - 1) / per;
  p.fd_pq = hcb::make_fastdiv((uint32_t)(p.P * p.Q));
  p.fd_q = hcb::make_fastdiv((uint32_t)p.Q);
  p.fd_c = hcb::make_fastdiv((uint32_t)p.C);
  p.fd_s = hcb::make_fastdiv((uint32_t)p.S);
  p.dy = dy.data_ptr();
  p.x = x.data_ptr();
  p.dw = dw.data_ptr<float>();
  p.dy_bytes = (uint32_t)yb;
  p.x_bytes = (uint32_t)xb;
  hcb::launch_conv_wgrad(p, (int)cfg, eff_splits, cur_stream());
}

void bn_stats(const Tensor& x, int64_t M, int64_t C, int64_t ldx, const Tensor& slab) {
  check_act(x, "x");
  check_f32(slab, "slab");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && ldx % 8 == 0, "hcb.bn_stats: C % 8 == 0, C <= 2048");
  check_range(x, ((M - 1) * ldx + C) * 2, "x");
  int T = hcb::bn_num_partials((int)M, (int)C);
  TORCH_CHECK(slab.numel() >= (int64_t)T * 2 * C, "hcb.bn_stats: slab too small");
  hcb::launch_bn_stats(x.data_ptr(), (int)M, (int)C, (int)ldx, slab.data_ptr<float>(), T, cur_stream());
}

int64_t bn_partials(int64_t M, int64_t C) { return hcb::bn_num_partials((int)M, (int)C); }

void bn_finalize(const Tensor& slab, int64_t T, int64_t C, double count, double eps, double momentum,
                 const Tensor& mean, const Tensor& invstd, const c10::optional<Tensor>& rm,
                 const c10::optional<Tensor>& rv) {
  check_f32(slab, "slab");
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  TORCH_CHECK(slab.numel() >= T * 2 * C && mean.numel() >= C && invstd.numel() >= C, "hcb.bn_finalize: sizes");
  float* rmp = nullptr;
  float* rvp = nullptr;
  if (rm.has_value() && rv.has_value()) {
    check_f32(*rm, "running_mean");
    check_f32(*rv, "running_var");
    rmp = rm->data_ptr<float>();
    rvp = rv->data_ptr<float>();
  }
  TORCH_CHECK(C <= 64 * 64, "hcb.bn_finalize: C too large");
  Tensor part = at::empty({(int64_t)hcb::bn_finalize_splits((int)T) * 2 * C},
                          at::TensorOptions().dtype(at::kDouble).device(slab.device()));
  hcb::launch_bn_finalize_split(slab.data_ptr<float>(), (int)T, (int)C, part.data_ptr<double>(), 1, count,
                                (float)eps, (float)momentum, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                rmp, rvp, nullptr, nullptr, cur_stream());
}

void bn_apply(const Tensor& x, int64_t ldx, const Tensor& y, int64_t ldy, const c10::optional<Tensor>& res,
              int64_t ldr, int64_t M, int64_t C, const Tensor& mean, const Tensor& invstd,
              const Tensor& gamma, const Tensor& beta, int64_t relu) {
  check_act(x, "x");
  check_act(y, "y");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && ldx % 8 == 0 && ldy % 8 == 0, "hcb.bn_apply: C/ld");
  check_range(x, ((M - 1) * ldx + C) * 2, "x");
  check_range(y, ((M - 1) * ldy + C) * 2, "y");
  const void* rp = nullptr;
  if (res.has_value()) {
    check_act(*res, "res");
    TORCH_CHECK(ldr % 8 == 0, "hcb.bn_apply: ldr");
    check_range(*res, ((M - 1) * ldr + C) * 2, "res");
    rp = res->data_ptr();
  }
  hcb::launch_bn_apply(x.data_ptr(), (int)ldx, y.data_ptr(), (int)ldy, rp, (int)ldr, (int)M, (int)C,
                       mean.data_ptr<float>(), invstd.data_ptr<float>(), gamma.data_ptr<float>(),
                       beta.data_ptr<float>(), (int)relu, cur_stream());
}

void bn_bwd_reduce(const Tensor& dy, int64_t lddy, const c10::optional<Tensor>& y, int64_t ldyv,
                   const Tensor& x, int64_t ldx, int64_t M, int64_t C, const Tensor& mean,
                   const Tensor& invstd, const Tensor& gamma, const Tensor& beta, int64_t relu,
                   const Tensor& slab, const c10::optional<Tensor>& gout, int64_t ldg) {
  check_act(dy, "dy");
  check_act(x, "x");
  check_f32(slab, "slab");
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "hcb.bn_bwd_reduce: C");
  check_range(dy, ((M - 1) * lddy + C) * 2, "dy");
  check_range(x, ((M - 1) * ldx + C) * 2, "x");
  const void* yp = nullptr;
  if (relu == 1) {
    TORCH_CHECK(y.has_value(), "hcb.bn_bwd_reduce: relu=1 needs y");
    check_range(*y, ((M - 1) * ldyv + C) * 2, "y");
    yp = y->data_ptr();
  }
  void* gp = nullptr;
  if (gout.has_value()) {
    check_act(*gout, "gout");
    check_range(*gout, ((M - 1) * ldg + C) * 2, "gout");
    gp = gout->data_ptr();
  }
  int T = hcb::bn_num_partials((int)M, (int)C);
  TORCH_CHECK(slab.numel() >= (int64_t)T * 2 * C, "hcb.bn_bwd_reduce: slab too small");
  hcb::launch_bn_bwd_reduce2(dy.data_ptr(), (int)lddy, yp, (int)ldyv, x.data_ptr(), (int)ldx, (int)M,
                             (int)C, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                             gamma.data_ptr<float>(), beta.data_ptr<float>(), (int)relu,
                             slab.data_ptr<float>(), T, gp, (int)ldg, cur_stream());
}

void bn_bwd_finalize(const Tensor& slab, int64_t T, int64_t C, const Tensor& dgamma, const Tensor& dbeta) {
  check_f32(slab, "slab");
  check_f32(dgamma, "dgamma");
  check_f32(dbeta, "dbeta");
  TORCH_CHECK(C <= 64 * 64 && slab.numel() >= T * 2 * C, "hcb.bn_bwd_finalize: sizes");
  Tensor part = at::empty({(int64_t)hcb::bn_finalize_splits((int)T) * 2 * C},
                          at::TensorOptions().dtype(at::kDouble).device(slab.device()));
  hcb::launch_bn_finalize_split(slab.data_ptr<float>(), (int)T, (int)C, part.data_ptr<double>(), 0, 0.0, 0.f,
                                0.f, nullptr, nullptr, nullptr, nullptr, dgamma.data_ptr<float>(),
                                dbeta.data_ptr<float>(), cur_stream());
}

void bn_bwd_apply(const Tensor& dy, int64_t lddy, const c10::optional<Tensor>& y, int64_t ldyv,
                  const Tensor& x, int64_t ldx, const Tensor& dx, int64_t lddx, int64_t M, int64_t C,
                  const Tensor& mean, const Tensor& invstd, const Tensor& gamma, const Tensor& beta,
                  const Tensor& dgamma, const Tensor& dbeta, int64_t relu) {
  check_act(dy, "dy");
  check_act(x, "x");
  check_act(dx, "dx");
  check_range(dy, ((M - 1) * lddy + C) * 2, "dy");
  check_range(x, ((M - 1) * ldx + C) * 2, "x");
  check_range(dx, ((M - 1) * lddx + C) * 2, "dx");
  const void* yp = nullptr;
  if (relu == 1) {
    TORCH_CHECK(y.has_value(), "hcb.bn_bwd_apply: relu=1 needs y");
    check_range(*y, ((M - 1) * ldyv + C) * 2, "y");
    yp = y->data_ptr();
  }
  hcb::launch_bn_bwd_apply2(dy.data_ptr(), (int)lddy, yp, (int)ldyv, x.data_ptr(), (int)ldx,
                            dx.data_ptr(), (int)lddx, (int)M, (int)C, mean.data_ptr<float>(),
                            invstd.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                            dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), (int)relu, cur_stream());
}

// geom = [N,H,W,C,P,Q,ldy,kh,kw,sh,sw,ph,pw]; z contiguous [N,H,W,C]
void bn_relu_maxpool_acc(const Tensor& z, const Tensor& y, const Tensor& amax, at::IntArrayRef g, const Tensor& acc,
                         int64_t R, double eps, double momentum, const Tensor& gamma, const Tensor& beta,
                         const Tensor& saved_mean, const Tensor& saved_invstd, const Tensor& run_mean,
                         const Tensor& run_var, const c10::optional<Tensor>& shift) {
  TORCH_CHECK(g.size() == 13, "hcb.bn_relu_maxpool_acc: geom");
  const bool f32 = check_act_or_f32(z, "z");
  // fp32 z with a bf16 y: y is the [3, ...] bf16 planes of the fp32 output (conv_p3 operands)
  const bool yp3 = f32 && y.scalar_type() == at::kBFloat16;
  const int64_t yps = yp3 ? check_planes(y, "y") : 0;
  if (!yp3) same_act(z, y, "y");
  const int64_t e = f32 ? 4 : 2;
  check_cuda(amax, "amax");
  const int64_t N = g[0], H = g[1], W = g[2], C = g[3], P = g[4], Q = g[5], ldy = g[6];
  TORCH_CHECK(z.is_contiguous() && z.numel() == N * H * W * C, "hcb.bn_relu_maxpool_acc: z contiguous [N,H,W,C]");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && ldy % 8 == 0 && ldy >= C, "hcb.bn_relu_maxpool_acc: C / ldy");
  TORCH_CHECK(g[7] * g[8] <= 255, "hcb.bn_relu_maxpool_acc: window too large for the uint8 argmax");
  check_range(y, yp3 ? (2 * yps + (N * P * Q - 1) * ldy + C) * 2 : ((N * P * Q - 1) * ldy + C) * e, "y");
  TORCH_CHECK(amax.scalar_type() == at::kByte && amax.is_contiguous() && amax.numel() >= N * P * Q * C,
              "hcb.bn_relu_maxpool_acc: amax uint8 [N,P,Q,C]");
  TORCH_CHECK(N * P * Q < (1ll << 31) && N * H * W < (1ll << 31), "hcb.bn_relu_maxpool_acc: 32-bit index range");
  for (const Tensor* t : {&acc, &gamma, &beta, &saved_mean, &saved_invstd, &run_mean, &run_var}) check_f32(*t, "bn");
  TORCH_CHECK(acc.numel() >= R * 2 * C && gamma.numel() >= C && beta.numel() >= C && saved_mean.numel() >= C &&
                  saved_invstd.numel() >= C && run_mean.numel() >= C && run_var.numel() >= C,
              "hcb.bn_relu_maxpool_acc: per-channel tensors too small");
  hcb::launch_bn_relu_maxpool_acc(z.data_ptr(), N, H, W, C, y.data_ptr(), P, Q, ldy, amax.data_ptr(), g[7], g[8], g[9],
                                  g[10], g[11], g[12], acc.data_ptr<float>(), R, (float)eps, (float)momentum,
                                  gamma.data_ptr<float>(), beta.data_ptr<float>(), saved_mean.data_ptr<float>(),
                                  saved_invstd.data_ptr<float>(), run_mean.data_ptr<float>(),
                                  run_var.data_ptr<float>(), opt_f32(shift, C, "shift"), cur_stream(), f32, yps);
}

// geom = [N,H,W,C,ldx,P,Q,ldy,kh,kw,sh,sw,ph,pw,is_max,incl_pad]
void pool_fwd(const Tensor& x, const Tensor& y, const c10::optional<Tensor>& idx, at::IntArrayRef g) {
  TORCH_CHECK(g.size() == 16, "hcb.pool_fwd: geom");
  check_act(x, "x");
  check_act(y, "y");
  TORCH_CHECK(g[3] % 8 == 0 && g[4] % 8 == 0 && g[7] % 8 == 0, "hcb.pool_fwd: C/ld % 8");
  TORCH_CHECK(g[0] * g[5] * g[6] * (g[3] / 8) < (1ll << 31), "hcb.pool_fwd: 32-bit index range");
  check_range(x, ((g[0] * g[1] * g[2] - 1) * g[4] + g[3]) * 2, "x");
  check_range(y, ((g[0] * g[5] * g[6] - 1) * g[7] + g[3]) * 2, "y");
  void* ip = nullptr;
  if (idx.has_value()) {
    TORCH_CHECK(idx->scalar_type() == at::kByte && idx->is_contiguous() && idx->numel() >= g[0] * g[5] * g[6] * g[3],
                "hcb.pool_fwd: idx must be contiguous uint8 [N,P,Q,C]");
    ip = idx->data_ptr();
  }
  hcb::launch_pool_fwd(x.data_ptr(), y.data_ptr(), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8],
                       g[9], g[10], g[11], g[12], g[13], g[14], g[15], ip, cur_stream());
}

// fp32 path: the pool on bf16 planes; x / y [3][N][H|P][W|Q][ld] (channel-slice views allowed)
void pool_fwd_p3(const Tensor& x, const Tensor& y, const c10::optional<Tensor>& idx, at::IntArrayRef g) {
  TORCH_CHECK(g.size() == 16, "hcb.pool_fwd_p3: geom");
  const int64_t xps = check_planes(x, "x"), yps = check_planes(y, "y");
  TORCH_CHECK(g[3] % 8 == 0 && g[4] % 8 == 0 && g[7] % 8 == 0, "hcb.pool_fwd_p3: C/ld % 8");
  TORCH_CHECK(g[0] * g[5] * g[6] * (g[3] / 8) < (1ll << 31), "hcb.pool_fwd_p3: 32-bit index range");
  check_range(x, (2 * xps + (g[0] * g[1] * g[2] - 1) * g[4] + g[3]) * 2, "x");
  check_range(y, (2 * yps + (g[0] * g[5] * g[6] - 1) * g[7] + g[3]) * 2, "y");
  void* ip = nullptr;
  if (idx.has_value()) {
    TORCH_CHECK(g[14] && idx->scalar_type() == at::kByte && idx->is_contiguous() &&
                    idx->numel() >= g[0] * g[5] * g[6] * g[3],
                "hcb.pool_fwd_p3: idx (max pool only) must be contiguous uint8 [N,P,Q,C]");
    ip = idx->data_ptr();
  }
  hcb::launch_pool_fwd_p3((const uint16_t*)x.data_ptr(), xps, (uint16_t*)y.data_ptr(), yps, g[0], g[1], g[2], g[3],
                          g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], g[15], ip,
                          cur_stream());
}

void pool_bwd(const Tensor& dy, const Tensor& x, const Tensor& y, const c10::optional<Tensor>& idx,
              const Tensor& dx, at::IntArrayRef g, bool accumulate) {
  TORCH_CHECK(g.size() == 16, "hcb.pool_bwd: geom");
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, x, "x");
  same_act(dy, y, "y");
  same_act(dy, dx, "dx");
  const int64_t e = f32 ? 4 : 2;
  check_range(x, ((g[0] * g[1] * g[2] - 1) * g[4] + g[3]) * e, "x");
  check_range(dx, ((g[0] * g[1] * g[2] - 1) * g[4] + g[3]) * e, "dx");
  check_range(y, ((g[0] * g[5] * g[6] - 1) * g[7] + g[3]) * e, "y");
  check_range(dy, ((g[0] * g[5] * g[6] - 1) * g[7] + g[3]) * e, "dy");
  if (f32)  // the fp32 kernel set: the argmax-gather max-pool backward, the 3x3/1 average pool
    TORCH_CHECK((g[14] && idx.has_value() && g[8] == g[9] && g[10] == g[11] && (g[8] + g[10] - 1) / g[10] <= 3 &&
                 g[0] * g[1] <= 65535 && g[0] * g[1] * g[2] * g[4] < (1ll << 31) &&
                 g[0] * g[5] * g[6] * std::max(g[7], g[3]) < (1ll << 31)) ||
                    (!g[14] && g[8] == 3 && g[9] == 3 && g[10] == 1 && g[11] == 1 &&
                     g[0] * g[5] * g[6] * g[7] * 4 < 0x7fffffffLL),
                "hcb.pool_bwd: fp32 supports the square max pool with its argmax and the 3x3/1 average pool");
  TORCH_CHECK(g[3] % 8 == 0 && g[4] % 8 == 0 && g[7] % 8 == 0, "hcb.pool_bwd: C/ld % 8");
  TORCH_CHECK(g[0] * g[1] * g[2] * (g[3] / 8) < (1ll << 31), "hcb.pool_bwd: 32-bit index range");
  if (idx.has_value())
    TORCH_CHECK(idx->scalar_type() == at::kByte && idx->is_contiguous() && idx->numel() >= g[0] * g[5] * g[6] * g[3],
                "hcb.pool_bwd: idx must be contiguous uint8 [N,P,Q,C]");
  hcb::launch_pool_bwd(dy.data_ptr(), x.data_ptr(), y.data_ptr(), dx.data_ptr(), g[0], g[1], g[2], g[3],
                       g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], g[15],
                       accumulate ? 1 : 0, idx.has_value() ? idx->data_ptr() : nullptr, cur_stream(), f32);
}

void gap_fwd(const Tensor& x, const Tensor& y, int64_t N, int64_t HW, int64_t C) {
  const bool f32 = check_act_or_f32(x, "x");
  same_act(x, y, "y");
  const int64_t e = f32 ? 4 : 2;
  TORCH_CHECK(C % 8 == 0, "hcb.gap_fwd: C % 8");
  check_range(x, N * HW * C * e, "x");
  check_range(y, N * C * e, "y");
  hcb::launch_gap_fwd(x.data_ptr(), y.data_ptr(), (int)N, (int)HW, (int)C, cur_stream(), f32);
}

void gap_bwd(const Tensor& dy, const Tensor& dx, int64_t N, int64_t HW, int64_t C) {
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, dx, "dx");
  const int64_t e = f32 ? 4 : 2;
  check_range(dy, N * C * e, "dy");
  check_range(dx, N * HW * C * e, "dx");
  hcb::launch_gap_bwd(dy.data_ptr(), dx.data_ptr(), (int)N, (int)HW, (int)C, cur_stream(), f32);
}

void softmax_xent(const Tensor& logits, int64_t ld, const Tensor& labels, int64_t ncls,
                  const Tensor& row_loss, const Tensor& dlogits, int64_t lddl, double scale,
                  const c10::optional<Tensor>& scale_dev, const c10::optional<Tensor>& dl32,
                  double label_smoothing) {
  check_f32(logits, "logits");
  TORCH_CHECK(label_smoothing >= 0.0 && label_smoothing <= 1.0, "hcb.softmax_xent: label_smoothing in [0, 1]");
  check_cuda(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kLong, "hcb.softmax_xent: labels int64");
  const bool f32 = check_act_or_f32(dlogits, "dlogits");
  int64_t B = labels.numel();
  check_range(logits, B * ld * 4, "logits");
  check_range(dlogits, B * lddl * (f32 ? 4 : 2), "dlogits");
  TORCH_CHECK(row_loss.numel() >= B, "hcb.softmax_xent: row_loss");
  float* d32 = nullptr;
  if (dl32.has_value()) {  // 16-bit dlogits: also the unrounded fp32 values (the bias gradient's source)
    TORCH_CHECK(!f32, "hcb.softmax_xent: dl32 only with 16-bit dlogits");
    check_f32(*dl32, "dl32");
    check_range(*dl32, B * lddl * 4, "dl32");
    d32 = dl32->data_ptr<float>();
  }
  hcb::launch_softmax_xent(logits.data_ptr<float>(), (int)ld, labels.data_ptr<int64_t>(), (int)B, (int)ncls,
                           row_loss.data_ptr<float>(), dlogits.data_ptr(), (int)lddl, (float)scale,
                           scale_dev.has_value() ? scale_dev->data_ptr<float>() : nullptr, cur_stream(), f32, d32,
                           (float)label_smoothing);
}

void nonfinite(const Tensor& g, const Tensor& flag) {
  check_f32(g, "g");
  check_f32(flag, "flag");
  TORCH_CHECK(g.is_contiguous() && flag.numel() >= 1, "hcb.nonfinite: args");
  check_align16(g.data_ptr(), "g");
  hcb::launch_nonfinite(g.data_ptr<float>(), g.numel(), flag.data_ptr<float>(), cur_stream());
}

void loss_total(const Tensor& row_loss, int64_t B, const c10::optional<Tensor>& l2, double half_wd,
                const Tensor& loss) {
  check_f32(row_loss, "row_loss");
  check_f32(loss, "loss");
  TORCH_CHECK(B >= 1 && row_loss.numel() >= B && loss.numel() >= 1, "hcb.loss_total: args");
  const float* l2p = nullptr;
  if (l2.has_value()) {
    check_f32(*l2, "l2");
    TORCH_CHECK(l2->numel() >= 1 && l2->is_contiguous(), "hcb.loss_total: l2");
    l2p = l2->data_ptr<float>();
  }
  hcb::launch_loss_total(row_loss.data_ptr<float>(), (int)B, l2p, l2p ? (int)l2->numel() : 0, (float)half_wd,
                         loss.data_ptr<float>(), cur_stream());
}

void loss_scale_update(const Tensor& hyper, double world, bool dynamic) {
  check_f32(hyper, "hyper");
  TORCH_CHECK(hyper.numel() >= 8 && hyper.is_contiguous(), "hcb.loss_scale_update: hyper[8]");
  hcb::launch_loss_scale_update(hyper.data_ptr<float>(), (float)world, dynamic ? 1 : 0, cur_stream());
}

// zero up to ZERO_BUFS contiguous fp32 tensors (16-byte aligned) in one launch
void zero_bufs(at::TensorList ts) {
  TORCH_CHECK(ts.size() >= 1 && ts.size() <= (size_t)hcb::ZERO_BUFS, "hcb.zero_bufs: 1..", hcb::ZERO_BUFS, " tensors");
  float* ptrs[hcb::ZERO_BUFS];
  int64_t ns[hcb::ZERO_BUFS];
  for (size_t i = 0; i < ts.size(); ++i) {
    check_f32(ts[i], "zero_bufs");
    TORCH_CHECK(ts[i].is_contiguous(), "hcb.zero_bufs: contiguous tensors only");
    check_align16(ts[i].data_ptr(), "zero_bufs");
    ptrs[i] = ts[i].data_ptr<float>();
    ns[i] = ts[i].numel();
  }
  hcb::launch_zero_bufs(ptrs, ns, (int)ts.size(), cur_stream());
}

void colsum(const Tensor& g, int64_t ld, int64_t M, int64_t N, const Tensor& out) {
  check_cuda(g, "g");
  check_f32(out, "out");
  bool f32 = g.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || g.scalar_type() == kAct, "hcb.colsum: dtype");
  // the kernel reads whole 8-column vectors: rows padded to 8 columns, 16-byte aligned
  TORCH_CHECK(ld % 8 == 0 && ld >= ((N + 7) / 8) * 8, "hcb.colsum: ld must be a multiple of 8 covering N");
  check_range(g, ((M - 1) * ld + ((N + 7) / 8) * 8) * (f32 ? 4 : 2), "g");
  check_align16(g.data_ptr(), "g");
  TORCH_CHECK(out.numel() >= N, "hcb.colsum: out too small");
  hcb::launch_colsum2(g.data_ptr(), (int)ld, (int)M, (int)N, f32 ? 1 : 0, out.data_ptr<float>(), cur_stream());
}

void sgd_momentum(const Tensor& w, const Tensor& mom, const Tensor& g, int64_t n_decay, const Tensor& hyper,
                  const c10::optional<Tensor>& l2, bool nesterov) {
  check_f32(w, "w");
  check_f32(mom, "mom");
  check_f32(g, "g");
  check_f32(hyper, "hyper");
  TORCH_CHECK(w.is_contiguous() && mom.is_contiguous() && g.is_contiguous(), "hcb.sgd_momentum: contiguous");
  TORCH_CHECK(w.numel() == mom.numel() && w.numel() == g.numel(), "hcb.sgd_momentum: sizes");
  check_align16(w.data_ptr(), "w");
  check_align16(mom.data_ptr(), "mom");
  check_align16(g.data_ptr(), "g");
  int slots = 0;
  if (l2.has_value()) {  // 1 slot: atomic sum (caller zeroes); more: per-block partials (loss_total sums)
    check_f32(*l2, "l2");
    slots = (int)l2->numel();
    TORCH_CHECK(l2->is_contiguous() && (slots == 1 || slots >= hcb::sgd_grid(w.numel())),
                "hcb.sgd_momentum: l2 must hold 1 or >= ", hcb::sgd_grid(w.numel()), " floats");
  }
  hcb::launch_sgd_momentum(w.data_ptr<float>(), mom.data_ptr<float>(), g.data_ptr<float>(), w.numel(),
                           n_decay, hyper.data_ptr<float>(), l2.has_value() ? l2->data_ptr<float>() : nullptr,
                           slots, nesterov ? 1 : 0, (int)hyper.numel(), cur_stream());
}

void weight_pack(const Tensor& master, const Tensor& pack, const Tensor& table, int64_t max_work, int64_t lo) {
  check_f32(master, "master");
  int64_t pstride = 0;
  if (lo == 3) {  // all three planes: pack is [3][n] bf16 (plane t at t * stride(0))
    pstride = check_planes(pack, "pack");
    TORCH_CHECK(pack.dim() == 2, "hcb.weight_pack: planes [3][n]");
  } else {
    TORCH_CHECK(lo >= 0 && lo <= 2, "hcb.weight_pack: lo 0..3");
    check_act(pack, "pack");
  }
  check_cuda(table, "table");
  TORCH_CHECK(table.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) == 9, "hcb.weight_pack: table [n][9] int64");
  TORCH_CHECK(table.is_contiguous(), "hcb.weight_pack: table contiguous");
  hcb::launch_weight_pack(master.data_ptr<float>(), (uint16_t*)pack.data_ptr(),
                          reinterpret_cast<const hcb::WPackEntry*>(table.data_ptr<int64_t>()),
                          (int)table.size(0), max_work, cur_stream(), (int)lo, pstride);
}

void cast_f32_bf16(const Tensor& x, const Tensor& y) {
  check_f32(x, "x");
  check_act(y, "y");
  TORCH_CHECK(x.numel() == y.numel() && x.is_contiguous() && y.is_contiguous(), "hcb.cast: shape");
  hcb::launch_cast_f32_bf16(x.data_ptr<float>(), (uint16_t*)y.data_ptr(), x.numel(), cur_stream());
}

void add_bf16(const Tensor& a, const Tensor& b, const Tensor& y) {
  check_act(a, "a");
  check_act(b, "b");
  check_act(y, "y");
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == y.numel() && a.numel() % 8 == 0, "hcb.add_bf16: sizes");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && y.is_contiguous(), "hcb.add_bf16: contiguous");
  hcb::launch_add_bf16(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), cur_stream());
}

// ---- finalize-free BN (statistics in R replicas of [2][C], fp32 atomics)
void bn_apply_acc(const Tensor& x, int64_t ldx, const Tensor& y, int64_t ldy, const c10::optional<Tensor>& res,
                  int64_t ldr, int64_t M, int64_t C, const Tensor& acc, int64_t R, double eps, double momentum,
                  const Tensor& gamma, const Tensor& beta, int64_t relu, const Tensor& saved_mean,
                  const Tensor& saved_invstd, const c10::optional<Tensor>& rm, const c10::optional<Tensor>& rv,
                  const c10::optional<Tensor>& shift, const c10::optional<Tensor>& res_acc, const c10::optional<Tensor>& res_gamma,
                  const c10::optional<Tensor>& res_beta, const c10::optional<Tensor>& res_saved_mean,
                  const c10::optional<Tensor>& res_saved_invstd, const c10::optional<Tensor>& res_rm,
                  const c10::optional<Tensor>& res_rv, const c10::optional<Tensor>& res_shift) {
  const bool f32 = check_act_or_f32(x, "x");
  // fp32 z with a bf16 y: y is written as [3, ...] bf16 planes; a bf16 residual is planes too
  const bool yp3 = f32 && y.scalar_type() == at::kBFloat16;
  const int64_t yps = yp3 ? check_planes(y, "y") : 0;
  if (!yp3) same_act(x, y, "y");
  int64_t rps = 0;
  const int64_t e = f32 ? 4 : 2;
  check_f32(acc, "acc");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && ldx % 8 == 0 && ldy % 8 == 0 && R >= 1, "hcb.bn_apply_acc: C/ld/R");
  TORCH_CHECK(acc.numel() >= R * 2 * C && saved_mean.numel() >= C && saved_invstd.numel() >= C, "hcb.bn_apply_acc: sizes");
  check_range(x, ((M - 1) * ldx + C) * e, "x");
  check_range(y, yp3 ? (2 * yps + (M - 1) * ldy + C) * 2 : ((M - 1) * ldy + C) * e, "y");
  const void* rp = nullptr;
  if (res.has_value()) {
    TORCH_CHECK(ldr % 8 == 0, "hcb.bn_apply_acc: ldr");
    if (yp3 && res->scalar_type() == at::kBFloat16) {
      TORCH_CHECK(!res_acc.has_value(), "hcb.bn_apply_acc: a residual BN reads the fp32 z_sc, not planes");
      rps = check_planes(*res, "res");
      check_range(*res, (2 * rps + (M - 1) * ldr + C) * 2, "res");
    } else {
      same_act(x, *res, "res");
      check_range(*res, ((M - 1) * ldr + C) * e, "res");
      TORCH_CHECK(!yp3 || res_acc.has_value(), "hcb.bn_apply_acc: a plain fp32-path residual must be planes");
    }
    rp = res->data_ptr();
  }
  // residual BN (projection shortcut): the residual is that BN's raw input z_sc
  hcb::ResBN rb{};
  if (res_acc.has_value()) {
    TORCH_CHECK(rp != nullptr && res_gamma && res_beta && res_saved_mean && res_saved_invstd,
                "hcb.bn_apply_acc: a residual BN needs res plus its acc / gamma / beta / saved stats");
    rb.acc = opt_f32(res_acc, R * 2 * C, "res_acc");
    rb.gamma = opt_f32(res_gamma, C, "res_gamma");
    rb.beta = opt_f32(res_beta, C, "res_beta");
    rb.saved_mean = const_cast<float*>(opt_f32(res_saved_mean, C, "res_saved_mean"));
    rb.saved_invstd = const_cast<float*>(opt_f32(res_saved_invstd, C, "res_saved_invstd"));
    rb.run_mean = const_cast<float*>(opt_f32(res_rm, C, "res_running_mean"));
    rb.run_var = const_cast<float*>(opt_f32(res_rv, C, "res_running_var"));
    TORCH_CHECK((rb.run_mean == nullptr) == (rb.run_var == nullptr), "hcb.bn_apply_acc: residual running stats");
    rb.shift = opt_f32(res_shift, C, "res_shift");
  }
  hcb::launch_bn_apply_acc(x.data_ptr(), (int)ldx, y.data_ptr(), (int)ldy, rp, (int)ldr, (int)M, (int)C,
                           acc.data_ptr<float>(), (int)R, (float)eps, (float)momentum, gamma.data_ptr<float>(),
                           beta.data_ptr<float>(), (int)relu, saved_mean.data_ptr<float>(),
                           saved_invstd.data_ptr<float>(), rm.has_value() ? rm->data_ptr<float>() : nullptr,
                           rv.has_value() ? rv->data_ptr<float>() : nullptr, opt_f32(shift, C, "shift"),
                           res_acc.has_value() ? &rb : nullptr, cur_stream(), f32, yps, rps);
}

// pooled-gradient source (pool_amax / pool_geom = [H, W, P, Q, k, s, pt, pl]): dy is the max-pool
// gradient [N][P][Q] (row stride lddy) and amax its window-local argmax [N][P][Q][C]; returns the
// number of dy rows to range-check
int64_t pool_src(hcb::PoolSrc& ps, const Tensor& dy, int64_t lddy, int64_t M, int64_t C,
                 const c10::optional<Tensor>& amax, at::OptionalIntArrayRef geom) {
  TORCH_CHECK(amax.has_value() == geom.has_value(), "hcb.bn_bwd: pool_amax and pool_geom go together");
  if (!amax.has_value()) return M;
  TORCH_CHECK(geom->size() == 8, "hcb.bn_bwd: pool_geom = [H, W, P, Q, k, s, pt, pl]");
  const auto g = *geom;
  ps.H = (int)g[0]; ps.W = (int)g[1]; ps.P = (int)g[2]; ps.Q = (int)g[3];
  ps.k = (int)g[4]; ps.s = (int)g[5]; ps.pt = (int)g[6]; ps.pl = (int)g[7];
  ps.C = (int)C;
  ps.ldp = (int)lddy;
  TORCH_CHECK(ps.H > 0 && ps.W > 0 && M % ((int64_t)ps.H * ps.W) == 0, "hcb.bn_bwd: M vs H x W");
  TORCH_CHECK(ps.s >= 1 && ps.k >= 1 && ps.k <= 2 * ps.s && ps.pt >= 0 && ps.pl >= 0 && ps.pt < ps.k && ps.pl < ps.k,
              "hcb.bn_bwd: pool windows must overlap at most 2 x 2 per pixel");
  const int64_t N = M / ((int64_t)ps.H * ps.W), rows = N * ps.P * ps.Q;
  TORCH_CHECK(amax->scalar_type() == at::kByte && amax->is_cuda() && amax->is_contiguous() &&
                  amax->numel() >= rows * C, "hcb.bn_bwd: pool_amax must be uint8 [N][P][Q][C]");
  TORCH_CHECK(lddy % 8 == 0, "hcb.bn_bwd: pooled dy row stride");
  ps.dyp = dy.data_ptr();
  ps.amax = amax->data_ptr<uint8_t>();
  return rows;
}

void bn_bwd_reduce_acc(const Tensor& dy, int64_t lddy, const c10::optional<Tensor>& y, int64_t ldyv,
                       const Tensor& x, int64_t ldx, int64_t M, int64_t C, const Tensor& mean, const Tensor& invstd,
                       const Tensor& gamma, const Tensor& beta, int64_t relu, const Tensor& acc, int64_t R,
                       const c10::optional<Tensor>& gout, int64_t ldg, const c10::optional<Tensor>& pool_amax,
                       at::OptionalIntArrayRef pool_geom) {
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, x, "x");
  const int64_t e = f32 ? 4 : 2;
  check_f32(acc, "acc");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && R >= 1 && acc.numel() >= R * 2 * C, "hcb.bn_bwd_reduce_acc: C/R");
  hcb::PoolSrc ps{};
  const int64_t dyrows = pool_src(ps, dy, lddy, M, C, pool_amax, pool_geom);
  TORCH_CHECK(!pool_amax.has_value() || (!gout.has_value() && relu != 1), "hcb.bn_bwd_reduce_acc: pooled dy: no gout / y");
  check_range(dy, ((dyrows - 1) * lddy + C) * e, "dy");
  check_range(x, ((M - 1) * ldx + C) * e, "x");
  const void* yp = nullptr;
  bool yh = false;  // fp32 path: y given as its bf16 planes, the mask read from the hi plane
  if (relu == 1) {
    TORCH_CHECK(y.has_value(), "hcb.bn_bwd_reduce_acc: relu=1 needs y");
    yh = f32 && y->scalar_type() == at::kBFloat16;
    if (yh) {
      check_planes(*y, "y");
      check_range(*y, ((M - 1) * ldyv + C) * 2, "y");
    } else {
      same_act(dy, *y, "y");
      check_range(*y, ((M - 1) * ldyv + C) * e, "y");
    }
    yp = y->data_ptr();
  }
  void* gp = nullptr;
  if (gout.has_value()) {
    same_act(dy, *gout, "gout");
    check_range(*gout, ((M - 1) * ldg + C) * e, "gout");
    gp = gout->data_ptr();
  }
  hcb::launch_bn_bwd_reduce_acc(dy.data_ptr(), (int)lddy, yp, (int)ldyv, x.data_ptr(), (int)ldx, (int)M, (int)C,
                                mean.data_ptr<float>(), invstd.data_ptr<float>(), gamma.data_ptr<float>(),
                                beta.data_ptr<float>(), (int)relu, acc.data_ptr<float>(), (int)R, gp, (int)ldg,
                                cur_stream(), f32, yh, pool_amax.has_value() ? &ps : nullptr);
}

void bn_bwd_apply_acc(const Tensor& dy, int64_t lddy, const c10::optional<Tensor>& y, int64_t ldyv,
                      const Tensor& x, int64_t ldx, const Tensor& dx, int64_t lddx, int64_t M, int64_t C,
                      const Tensor& mean, const Tensor& invstd, const Tensor& gamma, const Tensor& beta,
                      const Tensor& acc, int64_t R, const Tensor& dgamma, const Tensor& dbeta, int64_t relu,
                      const c10::optional<Tensor>& shift_out, const c10::optional<Tensor>& pool_amax,
                      at::OptionalIntArrayRef pool_geom, const c10::optional<Tensor>& add, int64_t ldadd) {
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, x, "x");
  // fp32 dy with a bf16 dx: dx is written as [3, ...] bf16 planes (the data / weight-gradient
  // GEMM operand format)
  const bool dp3 = f32 && dx.scalar_type() == at::kBFloat16;
  const int64_t dxps = dp3 ? check_planes(dx, "dx") : 0;
  if (!dp3) same_act(dy, dx, "dx");
  const int64_t e = f32 ? 4 : 2;
  if (add.has_value()) {  // dx = BN'(dy) + add: plain dx (no planes), no pooled dy
    same_act(dy, *add, "add");
    TORCH_CHECK(!dp3 && !pool_amax.has_value() && ldadd % 8 == 0, "hcb.bn_bwd_apply_acc: add needs a plain dx");
    check_range(*add, ((M - 1) * ldadd + C) * e, "add");
  }
  check_f32(acc, "acc");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && R >= 1 && acc.numel() >= R * 2 * C, "hcb.bn_bwd_apply_acc: C/R");
  hcb::PoolSrc ps{};
  const int64_t dyrows = pool_src(ps, dy, lddy, M, C, pool_amax, pool_geom);
  TORCH_CHECK(!pool_amax.has_value() || (relu != 1 && dp3 == f32), "hcb.bn_bwd_apply_acc: pooled dy: no y; fp32 writes planes");
  check_range(dy, ((dyrows - 1) * lddy + C) * e, "dy");
  check_range(x, ((M - 1) * ldx + C) * e, "x");
  check_range(dx, dp3 ? (2 * dxps + (M - 1) * lddx + C) * 2 : ((M - 1) * lddx + C) * e, "dx");
  const void* yp = nullptr;
  bool yh = false;
  if (relu == 1) {
    TORCH_CHECK(y.has_value(), "hcb.bn_bwd_apply_acc: relu=1 needs y");
    yh = f32 && y->scalar_type() == at::kBFloat16;
    if (yh) {
      check_planes(*y, "y");
      check_range(*y, ((M - 1) * ldyv + C) * 2, "y");
    } else {
      same_act(dy, *y, "y");
      check_range(*y, ((M - 1) * ldyv + C) * e, "y");
    }
    yp = y->data_ptr();
  }
  hcb::launch_bn_bwd_apply_acc(dy.data_ptr(), (int)lddy, yp, (int)ldyv, x.data_ptr(), (int)ldx, dx.data_ptr(),
                               (int)lddx, (int)M, (int)C, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                               gamma.data_ptr<float>(), beta.data_ptr<float>(), acc.data_ptr<float>(), (int)R,
                               dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), (int)relu,
                               const_cast<float*>(opt_f32(shift_out, C, "shift_out")), cur_stream(), f32, yh, dxps,
                               pool_amax.has_value() ? &ps : nullptr, add.has_value() ? add->data_ptr() : nullptr,
                               (int)ldadd);
}

void bn_stats_acc(const Tensor& x, int64_t ldx, int64_t M, int64_t C, const Tensor& acc, int64_t R,
                  const c10::optional<Tensor>& shift) {
  const bool f32 = check_act_or_f32(x, "x");
  check_f32(acc, "acc");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && ldx % 8 == 0 && ldx >= C && R >= 1 && M >= 1, "hcb.bn_stats_acc: C/ld/R");
  TORCH_CHECK(acc.numel() >= R * 2 * C, "hcb.bn_stats_acc: acc too small");
  check_range(x, ((M - 1) * ldx + C) * (f32 ? 4 : 2), "x");
  hcb::launch_bn_stats_acc(x.data_ptr(), (int)ldx, (int)M, (int)C, opt_f32(shift, C, "shift"), acc.data_ptr<float>(),
                           (int)R, cur_stream(), f32);
}

void relu_bwd(const Tensor& dy, const Tensor& y, const Tensor& dz) {
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, y, "y");
  same_act(dy, dz, "dz");
  TORCH_CHECK(dy.numel() == y.numel() && dy.numel() == dz.numel() && dy.numel() % 8 == 0, "hcb.relu_bwd: sizes");
  TORCH_CHECK(dy.is_contiguous() && y.is_contiguous() && dz.is_contiguous(), "hcb.relu_bwd: contiguous");
  hcb::launch_relu_bwd(dy.data_ptr(), y.data_ptr(), dz.data_ptr(), dy.numel(), cur_stream(), f32);
}

void dropout_fwd(const Tensor& x, const Tensor& y, const Tensor& mask, double keep, int64_t seed, const Tensor& step) {
  const bool f32 = check_act_or_f32(x, "x");
  same_act(x, y, "y");
  check_cuda(mask, "mask");
  check_cuda(step, "step");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && mask.is_contiguous(), "hcb.dropout_fwd: contiguous");
  TORCH_CHECK(x.numel() == y.numel() && x.numel() % 8 == 0 && mask.scalar_type() == at::kByte &&
                  mask.numel() * 8 >= x.numel(),
              "hcb.dropout_fwd: sizes (mask: one bit per element)");
  TORCH_CHECK(step.scalar_type() == at::kLong && step.numel() >= 1, "hcb.dropout_fwd: step int64");
  TORCH_CHECK(keep > 0.0 && keep <= 1.0, "hcb.dropout_fwd: 0 < keep <= 1");
  hcb::launch_dropout_fwd(x.data_ptr(), y.data_ptr(), mask.data_ptr<uint8_t>(), x.numel(), (float)keep, (uint64_t)seed,
                          step.data_ptr<int64_t>(), cur_stream(), f32);
}

void dropout_bwd(const Tensor& dy, const Tensor& mask, const Tensor& dx, double keep) {
  const bool f32 = check_act_or_f32(dy, "dy");
  same_act(dy, dx, "dx");
  check_cuda(mask, "mask");
  TORCH_CHECK(dy.is_contiguous() && dx.is_contiguous() && mask.is_contiguous(), "hcb.dropout_bwd: contiguous");
  TORCH_CHECK(dy.numel() == dx.numel() && dy.numel() % 8 == 0 && mask.scalar_type() == at::kByte &&
                  mask.numel() * 8 >= dy.numel(),
              "hcb.dropout_bwd: sizes");
  TORCH_CHECK(keep > 0.0 && keep <= 1.0, "hcb.dropout_bwd: 0 < keep <= 1");
  hcb::launch_dropout_bwd(dy.data_ptr(), mask.data_ptr<uint8_t>(), dx.data_ptr(), dy.numel(), (float)keep, cur_stream(),
                          f32);
}

void scale_f32(const Tensor& x, double s) {
  check_f32(x, "x");
  TORCH_CHECK(x.is_contiguous(), "hcb.scale_f32: contiguous");
  hcb::launch_scale_f32(x.data_ptr<float>(), x.numel(), (float)s, cur_stream());
}

void l2norm_sq(const Tensor& x, const Tensor& out) {
  check_f32(x, "x");
  check_f32(out, "out");
  hcb::launch_l2norm_sq(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), cur_stream());
}

void synth_images(const Tensor& out, int64_t C, int64_t Cpad, double mean, double std, int64_t seed) {
  const bool f32 = check_act_or_f32(out, "out");
  TORCH_CHECK(out.numel() % Cpad == 0, "hcb.synth_images: numel % Cpad");
  hcb::launch_synth_images(out.data_ptr(), out.numel() / Cpad, (int)C, (int)Cpad, (float)mean, (float)std,
                           (uint64_t)seed, cur_stream(), f32);
}

void synth_labels(const Tensor& out, int64_t ncls, int64_t seed) {
  check_cuda(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kLong, "hcb.synth_labels: int64");
  hcb::launch_synth_labels(out.data_ptr<int64_t>(), (int)out.numel(), (int)ncls, (uint64_t)seed, cur_stream());
}

// desc_host: the CPU copy of desc, used to check every crop lies inside src before launching
void preprocess_images(const Tensor& src, const Tensor& desc, const Tensor& desc_host, const Tensor& out,
                       at::ArrayRef<double> scale, at::ArrayRef<double> bias) {
  check_cuda(src, "src");
  check_cuda(desc, "desc");
  const bool f32 = check_act_or_f32(out, "out");  // the fp32 path's input is fp32
  TORCH_CHECK(src.scalar_type() == at::kByte && src.is_contiguous(), "hcb.preprocess_images: src uint8 contiguous");
  TORCH_CHECK(desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 4 && desc.is_contiguous(),
              "hcb.preprocess_images: desc int64 [B][4]");
  TORCH_CHECK(!desc_host.is_cuda() && desc_host.scalar_type() == at::kLong && desc_host.is_contiguous() &&
                  desc_host.sizes() == desc.sizes(),
              "hcb.preprocess_images: desc_host must be the CPU copy of desc");
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous() && out.size(1) == out.size(2) && out.size(3) % 8 == 0 &&
                  out.size(3) >= 8,
              "hcb.preprocess_images: out [B][S][S][Cpad] contiguous, Cpad % 8 == 0");
  TORCH_CHECK(scale.size() == 3 && bias.size() == 3, "hcb.preprocess_images: 3 scales / biases");
  const int64_t B = desc.size(0);
  TORCH_CHECK(B <= out.size(0), "hcb.preprocess_images: more crops than output images");
  const int64_t* d = desc_host.data_ptr<int64_t>();
  for (int64_t i = 0; i < B; ++i) {
    TORCH_CHECK(d[4 * i] >= 0 && d[4 * i + 1] > 0 && d[4 * i + 2] > 0 &&
                    d[4 * i] + d[4 * i + 1] * d[4 * i + 2] * 3 <= src.numel(),
                "hcb.preprocess_images: crop ", i, " outside the staging buffer");
  }
  TORCH_CHECK(out.size(1) * out.size(1) < (1ll << 31), "hcb.preprocess_images: image too large");
  const float sc[3] = {(float)scale[0], (float)scale[1], (float)scale[2]};
  const float bi[3] = {(float)bias[0], (float)bias[1], (float)bias[2]};
  if (B == 0) return;
  hcb::launch_preprocess_images(src.data_ptr<uint8_t>(), desc.data_ptr<int64_t>(), (int)B, out.data_ptr(),
                                (int)out.size(1), (int)out.size(3), sc, bi, f32, cur_stream());
}

static int pack_mode(const Tensor& t, const char* what) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "hcb.", what, ": wire dtype must be float32, bfloat16 or float16");
  }
  return 0;
}

void bucket_pack(const Tensor& src, const Tensor& dst, double scale) {
  check_f32(src, "src");
  check_cuda(dst, "dst");
  TORCH_CHECK(dst.is_contiguous() && src.numel() == dst.numel(), "hcb.bucket_pack: sizes");
  hcb::launch_bucket_pack(src.data_ptr<float>(), dst.data_ptr(), src.numel(), (float)scale, pack_mode(dst, "bucket_pack"),
                          cur_stream());
}

void bucket_unpack(const Tensor& src, const Tensor& dst, double scale) {
  check_cuda(src, "src");
  check_f32(dst, "dst");
  TORCH_CHECK(src.is_contiguous() && src.numel() == dst.numel(), "hcb.bucket_unpack: sizes");
  hcb::launch_bucket_unpack(src.data_ptr(), dst.data_ptr<float>(), src.numel(), (float)scale,
                            pack_mode(src, "bucket_unpack"), cur_stream());
}

// ---------------------------------------------------------------- space-to-depth stem
void stem_s2d(const Tensor& x, const Tensor& out, int64_t pad) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  if (x.scalar_type() == at::kFloat) {  // fp32 image -> the folded tensor's three bf16 planes [3][N][Hs][Ws][16]
    const int64_t ops = check_planes(out, "out");
    TORCH_CHECK(x.dim() == 4 && out.dim() == 5 && x.is_contiguous() && out.select(0, 0).is_contiguous() &&
                    x.size(3) >= 4 && x.size(3) % 4 == 0 && out.size(4) == 16 && out.size(1) == x.size(0),
                "hcb.stem_s2d: fp32 x [N][H][W][>=4, multiple of 4] -> planes [3][N][Hs][Ws][16]");
    const int64_t H = x.size(1), W = x.size(2), Hs = out.size(2), Ws = out.size(3);
    TORCH_CHECK(2 * Hs - 1 - pad < H + 8 && 2 * Ws - 1 - pad < W + 8 && x.numel() < (1ll << 31),
                "hcb.stem_s2d: folded extent");
    hcb::launch_stem_s2d_f32(x.data_ptr<float>(), (int)x.size(0), (int)H, (int)W, (int)x.size(3),
                             reinterpret_cast<uint16_t*>(out.data_ptr()), ops, (int)Hs, (int)Ws, (int)pad,
                             cur_stream());
    return;
  }
  TORCH_CHECK(x.dim() == 4 && out.dim() == 4 && x.scalar_type() == kAct && out.scalar_type() == kAct,
              "hcb.stem_s2d: 16-bit NHWC tensors");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.size(3) >= 4 && x.size(3) % 4 == 0 && out.size(3) == 16 &&
                  out.size(0) == x.size(0),
              "hcb.stem_s2d: x [N][H][W][>=4, multiple of 4] -> out [N][Hs][Ws][16]");
  const int64_t H = x.size(1), W = x.size(2), Hs = out.size(1), Ws = out.size(2);
  TORCH_CHECK(2 * Hs - 1 - pad < H + 8 && 2 * Ws - 1 - pad < W + 8 && x.numel() < (1ll << 31),
              "hcb.stem_s2d: folded extent");
  hcb::launch_stem_s2d(reinterpret_cast<const uint16_t*>(x.data_ptr()), (int)x.size(0), (int)H, (int)W,
                       (int)x.size(3), reinterpret_cast<uint16_t*>(out.data_ptr()), (int)Hs, (int)Ws, (int)pad,
                       cur_stream());
}

void stem_wfold(const Tensor& w, const Tensor& wp) {
  check_f32(w, "w");
  check_cuda(wp, "wp");
  TORCH_CHECK(w.dim() == 4 && w.size(1) == 7 && w.size(2) == 7 && w.size(3) >= 3 && w.is_contiguous(),
              "hcb.stem_wfold: w [cout][7][7][>=3] fp32");
  // wp: the bf16 pack [cout][256], or (fp32 path) its hi / mid / lo planes [3][cout][256]
  const bool p3 = wp.dim() == 3 && wp.size(0) == 3 && wp.scalar_type() == at::kBFloat16;
  TORCH_CHECK((p3 || wp.scalar_type() == kAct) && wp.is_contiguous() && wp.numel() == (p3 ? 3 : 1) * w.size(0) * 256,
              "hcb.stem_wfold: wp bf16 [cout][256] or planes [3][cout][256]");
  hcb::launch_stem_wfold(w.data_ptr<float>(), (int)w.size(0), (int)w.size(3),
                         reinterpret_cast<uint16_t*>(wp.data_ptr()), cur_stream(), p3);
}

void stem_wgrad_unfold(const Tensor& dwp, const Tensor& dw) {
  check_f32(dwp, "dwp");
  check_f32(dw, "dw");
  TORCH_CHECK(dw.dim() == 4 && dw.size(1) == 7 && dw.size(2) == 7 && dw.size(3) >= 3 && dw.is_contiguous() &&
                  dwp.is_contiguous() && dwp.numel() == dw.size(0) * 256,
              "hcb.stem_wgrad_unfold: dwp [cout][256] -> dw [cout][7][7][>=3]");
  hcb::launch_stem_wgrad_unfold(dwp.data_ptr<float>(), (int)dw.size(0), (int)dw.size(3), dw.data_ptr<float>(),
                                cur_stream());
}

// ---- fp32 path on bf16 planes (conv_p3.hip)

// geom as conv_igemm; x: planes of the input, w: hi pack, w_lo: [2][n] mid / lo packs; y fp32
hcb::ConvParams p3_params(const Tensor& x, const Tensor& w, const Tensor& w_lo, const Tensor& y,
                          const c10::optional<Tensor>& yres, const c10::optional<Tensor>& bias,
                          const c10::optional<Tensor>& stats, at::IntArrayRef g, int64_t cfg,
                          const c10::optional<Tensor>& stats_shift) {
  const int64_t xps = check_planes(x, "x");
  TORCH_CHECK(cfg >= 0 && cfg < 37, "hcb.conv_p3: cfg 0..36");
  // conv_params validates geometry and byte ranges on plane 0 (a bf16 tensor of this build's type);
  // split-K is validated here against the p3 tiles
  std::vector<int64_t> g1(g.begin(), g.end());
  const int64_t splits = g1.size() > 30 ? g1[30] : 1;
  if (g1.size() > 30) g1[30] = 1;
  hcb::ConvParams p = conv_params(x.select(0, 0), w, y, yres, bias, c10::nullopt, g1, 0);
  const int bm = hcb::p3_tile_m((int)cfg), bn = hcb::p3_tile_n((int)cfg);
  const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * ((p.Nout + bn - 1) / bn);
  p.splits = (int)splits;
  TORCH_CHECK(p.splits >= 1 && p.splits <= p.Kpad / 64, "hcb.conv_p3: 1 <= splits <= k-steps");
  TORCH_CHECK(p.out_f32 && y.scalar_type() == at::kFloat, "hcb.conv_p3: fp32 output");
  check_range(x, 2 * xps * 2 + (int64_t)p.x_bytes, "x planes");
  TORCH_CHECK(2 * xps * 2 < (1ll << 32), "hcb.conv_p3: plane stride exceeds the 32-bit offset range");
  p.x_plane = (uint32_t)(xps * 2);
  TORCH_CHECK(w_lo.dim() == 2 && w_lo.size(0) == 2 && w_lo.stride(1) == 1 && w_lo.scalar_type() == w.scalar_type() &&
                  w_lo.size(1) >= (int64_t)p.Nout * p.Kpad,
              "hcb.conv_p3: w_lo must be [2][>= Nout*Kpad] of the pack's type");
  const Tensor m = w_lo.select(0, 0), l = w_lo.select(0, 1);
  check_align16(m.data_ptr(), "w_lo[0]");
  check_align16(l.data_ptr(), "w_lo[1]");
  p.w_lo = m.data_ptr();
  p.w_lo2 = l.data_ptr();
  p.stats = nullptr;
  if (stats.has_value()) {
    check_f32(*stats, "stats");
    const int tiles_m = (p.M + hcb::p3_tile_m((int)cfg) - 1) / hcb::p3_tile_m((int)cfg);
    const int64_t rows = p.stats_R > 0 ? p.stats_R : tiles_m;
    TORCH_CHECK(stats->numel() >= rows * 2 * p.Nout, "hcb.conv_p3: stats buffer too small");
    p.stats = stats->data_ptr<float>();
  }
  TORCH_CHECK(!stats_shift.has_value() || p.stats != nullptr, "hcb.conv_p3: stats_shift without stats");
  p.stats_shift = opt_f32(stats_shift, p.Nout, "stats_shift");
  if (p.splits > 1) {
    TORCH_CHECK(g_splitk_ws != nullptr && g_splitk_cnt != nullptr, "hcb.conv_p3: split-K workspace not set");
    TORCH_CHECK(tiles * p.splits * bm * bn * 4 <= g_splitk_ws_bytes, "hcb.conv_p3: split-K workspace too small");
    TORCH_CHECK(tiles <= g_splitk_cnt_n, "hcb.conv_p3: split-K counter array too small");
    p.ws = g_splitk_ws;
    p.cnt = g_splitk_cnt;
  }
  if (cfg >= 23 && cfg <= 30) {  // stream-K (conv_p3_persist.h): the launcher sizes its shares against the workspace
    TORCH_CHECK(g_splitk_ws != nullptr && g_splitk_cnt != nullptr, "hcb.conv_p3: stream-K needs the split-K workspace");
    p.ws = g_splitk_ws;
    p.cnt = g_splitk_cnt;
  }
  p.ws_floats = p.ws != nullptr ? g_splitk_ws_bytes / 4 : 0;
  p.cnt_n = p.cnt != nullptr ? (int)g_splitk_cnt_n : 0;
  return p;
}

void conv_p3(const Tensor& x, const Tensor& w, const Tensor& w_lo, const Tensor& y, const c10::optional<Tensor>& yres,
             const c10::optional<Tensor>& bias, const c10::optional<Tensor>& stats, at::IntArrayRef g, int64_t cfg,
             const c10::optional<Tensor>& stats_shift) {
  hcb::ConvParams p = p3_params(x, w, w_lo, y, yres, bias, stats, g, cfg, stats_shift);
  hcb::launch_conv_p3(p, (int)cfg, cur_stream());
}

// fp32 data gradient with the fused BN-backward epilogue (see conv_igemm_bnb): z fp32, yact the
// activation's planes (mode 1), output g fp32
void conv_p3_bnb(const Tensor& x, const Tensor& w, const Tensor& w_lo, const Tensor& y,
                 const c10::optional<Tensor>& yres, at::IntArrayRef g, int64_t cfg, const Tensor& z,
                 const c10::optional<Tensor>& yact, int64_t ld, const Tensor& mean, const Tensor& invstd,
                 const Tensor& gamma, const Tensor& beta, const Tensor& acc, int64_t R, int64_t mode) {
  hcb::ConvParams p = p3_params(x, w, w_lo, y, yres, c10::nullopt, c10::nullopt, g, cfg, c10::nullopt);
  set_bnb(p, z, yact, ld, mean, invstd, gamma, beta, acc, R, mode, true);
  hcb::launch_conv_p3(p, (int)cfg, cur_stream());
}

// geom as conv_wgrad; dy / x planes
void conv_wgrad_p3(const Tensor& dy, const Tensor& x, const Tensor& dw, at::IntArrayRef g, int64_t cfg,
                   int64_t splits) {
  TORCH_CHECK(g.size() == 17, "hcb.conv_wgrad_p3: geom must have 17 entries");
  const int64_t dps = check_planes(dy, "dy"), xps = check_planes(x, "x");
  TORCH_CHECK(cfg >= 0 && cfg < 19, "hcb.conv_wgrad_p3: cfg 0..18");
  check_f32(dw, "dw");
  hcb::WgradParams p{};
  p.N = g[0]; p.H = g[1]; p.W = g[2]; p.C = g[3]; p.ldx = g[4];
  p.P = g[5]; p.Q = g[6]; p.R = g[7]; p.S = g[8];
  p.stride_h = g[9]; p.stride_w = g[10]; p.pad_h = g[11]; p.pad_w = g[12];
  p.dil_h = g[13]; p.dil_w = g[14];
  p.Nout = g[15]; p.ldy = g[16];
  p.K = p.R * p.S * p.C;
  p.M = p.N * p.P * p.Q;
  TORCH_CHECK(p.C % 8 == 0 && p.ldx % 8 == 0, "hcb.conv_wgrad_p3: C, ldx multiples of 8");
  TORCH_CHECK(p.ldy % 8 == 0 && p.ldy >= p.Nout, "hcb.conv_wgrad_p3: bad ldy");
  TORCH_CHECK(splits >= 1, "hcb.conv_wgrad_p3: splits >= 1");
  const int64_t xb = x_span_bytes(p.N, p.H, p.W, p.C, p.ldx, 2);
  const int64_t yb = ((int64_t)p.M - 1) * p.ldy * 2 + (int64_t)((p.Nout + 7) / 8) * 8 * 2;
  TORCH_CHECK(xb < (1ll << 31) && yb < (1ll << 31), "hcb.conv_wgrad_p3: operand exceeds 2 GiB");
  TORCH_CHECK(2 * xps * 2 < (1ll << 32) && 2 * dps * 2 < (1ll << 32), "hcb.conv_wgrad_p3: plane stride range");
  check_range(x, 2 * xps * 2 + xb, "x planes");
  check_range(dy, 2 * dps * 2 + yb, "dy planes");
  check_range(dw, (int64_t)p.Nout * p.K * 4, "dw");
  TORCH_CHECK(cfg < 16 || (int64_t)p.Nout * p.K * 4 < (1ll << 31),
              "hcb.conv_wgrad_p3: the persistent configs address dW through a 32-bit buffer offset");
  const int nkt = (p.M + 63) / 64;
  const int per = (nkt + (int)splits - 1) / (int)splits;
  p.ksteps_per_split = per;
  const int eff_splits = (nkt + per - 1) / per;
  p.fd_pq = hcb::make_fastdiv((uint32_t)(p.P * p.Q));
  p.fd_q = hcb::make_fastdiv((uint32_t)p.Q);
  p.fd_c = hcb::make_fastdiv((uint32_t)p.C);
  p.fd_s = hcb::make_fastdiv((uint32_t)p.S);
  p.dy = dy.data_ptr();
  p.x = x.data_ptr();
  p.dw = dw.data_ptr<float>();
  p.dy_bytes = (uint32_t)yb;
  p.x_bytes = (uint32_t)xb;
  p.dy_plane = (uint32_t)(dps * 2);
  p.x_plane = (uint32_t)(xps * 2);
  hcb::launch_wgrad_p3(p, (int)cfg, eff_splits, cur_stream());
}

// fp32 x [rows][ldx] (first C channels) -> planes out [3][rows][ldo]
void split_planes(const Tensor& x, int64_t ldx, int64_t rows, int64_t C, const Tensor& out, int64_t ldo) {
  check_f32(x, "x");
  const int64_t ps = check_planes(out, "out");
  TORCH_CHECK(C % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && ldx >= C && ldo >= C, "hcb.split_planes: C / ld % 8");
  check_align16(x.data_ptr(), "x");
  check_range(x, ((rows - 1) * ldx + C) * 4, "x");
  check_range(out, (2 * ps + (rows - 1) * ldo + C) * 2, "out");
  TORCH_CHECK(ps >= (rows - 1) * ldo + C, "hcb.split_planes: planes overlap");
  hcb::launch_split_planes(x.data_ptr<float>(), (int)ldx, rows, (int)C, (uint16_t*)out.data_ptr(), (int)ldo, ps,
                           cur_stream());
}

void merge_planes(const Tensor& in, int64_t ldi, int64_t rows, int64_t C, const Tensor& y, int64_t ldy) {
  const int64_t ps = check_planes(in, "in");
  check_f32(y, "y");
  TORCH_CHECK(C % 8 == 0 && ldi % 8 == 0 && ldy % 8 == 0, "hcb.merge_planes: C / ld % 8");
  check_align16(y.data_ptr(), "y");
  check_range(in, (2 * ps + (rows - 1) * ldi + C) * 2, "in");
  check_range(y, ((rows - 1) * ldy + C) * 4, "y");
  hcb::launch_merge_planes((const uint16_t*)in.data_ptr(), (int)ldi, ps, rows, (int)C, y.data_ptr<float>(), (int)ldy,
                           cur_stream());
}

void gap_fwd_p3(const Tensor& x, const Tensor& y, int64_t N, int64_t HW, int64_t C) {
  const int64_t xps = check_planes(x, "x"), yps = check_planes(y, "y");
  TORCH_CHECK(C % 8 == 0, "hcb.gap_fwd_p3: C % 8");
  check_range(x, (2 * xps + N * HW * C) * 2, "x");
  check_range(y, (2 * yps + N * C) * 2, "y");
  hcb::launch_gap_fwd_p3((const uint16_t*)x.data_ptr(), xps, (uint16_t*)y.data_ptr(), yps, (int)N, (int)HW, (int)C,
                         cur_stream());
}

void set_deterministic(bool on) { hcb::set_deterministic(on); }

}  // namespace


HCB_TORCH_LIBRARY(hcb, m) {
  m.def("conv_igemm(Tensor x, Tensor w, Tensor(a!) y, Tensor? yres, Tensor? bias, Tensor(b!)? stats, int[] geom, int cfg, Tensor? stats_shift=None, Tensor? w_lo=None) -> ()");
  m.def("conv_igemm_bnb(Tensor x, Tensor w, Tensor(a!) y, Tensor? yres, int[] geom, int cfg, Tensor z, Tensor? yact, int ld, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, Tensor(b!) acc, int R, int mode) -> ()");
  m.def("conv_tiles_m(int M, int cfg) -> int", conv_tiles_m);
  m.def("set_splitk_workspace(Tensor ws, Tensor cnt) -> ()");
  m.def("set_p3p_bnb(int v) -> ()", set_p3p_bnb);
  m.def("conv_wgrad(Tensor dy, Tensor x, Tensor(a!) dw, int[] geom, int cfg, int splits) -> ()");
  m.def("bn_stats(Tensor x, int M, int C, int ldx, Tensor(a!) slab) -> ()");
  m.def("bn_partials(int M, int C) -> int", bn_partials);
  m.def("bn_finalize(Tensor slab, int T, int C, float count, float eps, float momentum, Tensor(a!) mean, Tensor(b!) invstd, Tensor(c!)? running_mean, Tensor(d!)? running_var) -> ()");
  m.def("bn_apply(Tensor x, int ldx, Tensor(a!) y, int ldy, Tensor? res, int ldr, int M, int C, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, int relu) -> ()");
  m.def("bn_bwd_reduce(Tensor dy, int lddy, Tensor? y, int ldyv, Tensor x, int ldx, int M, int C, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, int relu, Tensor(a!) slab, Tensor(b!)? gout, int ldg) -> ()");
  m.def("bn_bwd_finalize(Tensor slab, int T, int C, Tensor(a!) dgamma, Tensor(b!) dbeta) -> ()");
  m.def("bn_bwd_apply(Tensor dy, int lddy, Tensor? y, int ldyv, Tensor x, int ldx, Tensor(a!) dx, int lddx, int M, int C, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, Tensor dgamma, Tensor dbeta, int relu) -> ()");
  m.def("pool_fwd(Tensor x, Tensor(a!) y, Tensor(b!)? idx, int[] geom) -> ()");
  m.def("pool_bwd(Tensor dy, Tensor x, Tensor y, Tensor? idx, Tensor(a!) dx, int[] geom, bool accumulate) -> ()");
  m.def("pool_fwd_p3(Tensor x, Tensor(a!) y, Tensor(b!)? idx, int[] geom) -> ()");
  m.def("gap_fwd(Tensor x, Tensor(a!) y, int N, int HW, int C) -> ()");
  m.def("gap_bwd(Tensor dy, Tensor(a!) dx, int N, int HW, int C) -> ()");
  m.def("softmax_xent(Tensor logits, int ld, Tensor labels, int ncls, Tensor(a!) row_loss, Tensor(b!) dlogits, int lddl, float scale, Tensor? scale_dev=None, Tensor(c!)? dl32=None, float label_smoothing=0.0) -> ()");
  m.def("nonfinite(Tensor g, Tensor(a!) flag) -> ()");
  m.def("loss_total(Tensor row_loss, int B, Tensor? l2, float half_wd, Tensor(a!) loss) -> ()");
  m.def("loss_scale_update(Tensor(a!) hyper, float world, bool dynamic) -> ()");
  m.def("colsum(Tensor g, int ld, int M, int N, Tensor(a!) out) -> ()");
  m.def("zero_bufs(Tensor(a!)[] ts) -> ()");
  m.def("sgd_momentum(Tensor(a!) w, Tensor(b!) mom, Tensor g, int n_decay, Tensor hyper, Tensor(c!)? l2, bool nesterov) -> ()");
  m.def("weight_pack(Tensor master, Tensor(a!) pack, Tensor table, int max_work, int lo=0) -> ()");
  m.def("cast_f32_bf16(Tensor x, Tensor(a!) y) -> ()");
  m.def("add_bf16(Tensor a, Tensor b, Tensor(a!) y) -> ()");
  m.def("scale_f32(Tensor(a!) x, float s) -> ()");
  m.def("relu_bwd(Tensor dy, Tensor y, Tensor(a!) dz) -> ()");
  m.def("bn_apply_acc(Tensor x, int ldx, Tensor(a!) y, int ldy, Tensor? res, int ldr, int M, int C, Tensor acc, int R, float eps, float momentum, Tensor gamma, Tensor beta, int relu, Tensor(b!) saved_mean, Tensor(c!) saved_invstd, Tensor(d!)? running_mean, Tensor(e!)? running_var, Tensor? shift=None, Tensor? res_acc=None, Tensor? res_gamma=None, Tensor? res_beta=None, Tensor(g!)? res_saved_mean=None, Tensor(h!)? res_saved_invstd=None, Tensor(i!)? res_running_mean=None, Tensor(j!)? res_running_var=None, Tensor? res_shift=None) -> ()");
  m.def("bn_bwd_reduce_acc(Tensor dy, int lddy, Tensor? y, int ldyv, Tensor x, int ldx, int M, int C, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, int relu, Tensor(a!) acc, int R, Tensor(b!)? gout, int ldg, Tensor? pool_amax=None, int[]? pool_geom=None) -> ()");
  m.def("bn_bwd_apply_acc(Tensor dy, int lddy, Tensor? y, int ldyv, Tensor x, int ldx, Tensor(a!) dx, int lddx, int M, int C, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, Tensor acc, int R, Tensor(b!) dgamma, Tensor(c!) dbeta, int relu, Tensor(d!)? shift_out=None, Tensor? pool_amax=None, int[]? pool_geom=None, Tensor? add=None, int ldadd=0) -> ()");
  m.def("bn_stats_acc(Tensor x, int ldx, int M, int C, Tensor(a!) acc, int R, Tensor? shift=None) -> ()");
  m.def("l2norm_sq(Tensor x, Tensor(a!) out) -> ()");
  m.def("preprocess_images(Tensor src, Tensor desc, Tensor desc_host, Tensor(a!) out, float[] scale, float[] bias) -> ()");
  m.def("bn_relu_maxpool_acc(Tensor z, Tensor(a!) y, Tensor(b!) amax, int[] geom, Tensor acc, int R, float eps, "
        "float momentum, Tensor gamma, Tensor beta, Tensor(c!) saved_mean, Tensor(d!) saved_invstd, "
        "Tensor(e!) run_mean, Tensor(f!) run_var, Tensor? shift=None) -> ()");
  m.def("dropout_fwd(Tensor x, Tensor(a!) y, Tensor(b!) mask, float keep, int seed, Tensor step) -> ()");
  m.def("dropout_bwd(Tensor dy, Tensor mask, Tensor(a!) dx, float keep) -> ()");
  m.def("synth_images(Tensor(a!) out, int C, int Cpad, float mean, float std, int seed) -> ()");
  m.def("synth_labels(Tensor(a!) out, int ncls, int seed) -> ()");
  m.def("bucket_pack(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("bucket_unpack(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("stem_s2d(Tensor x, Tensor(a!) out, int pad) -> ()");
  m.def("set_deterministic(bool on) -> ()", set_deterministic);
  m.def("stem_wfold(Tensor w, Tensor(a!) wp) -> ()");
  m.def("stem_wgrad_unfold(Tensor dwp, Tensor(a!) dw) -> ()");
  m.def("conv_p3(Tensor x, Tensor w, Tensor w_lo, Tensor(a!) y, Tensor? yres, Tensor? bias, Tensor(b!)? stats, int[] geom, int cfg, Tensor? stats_shift=None) -> ()");
  m.def("conv_wgrad_p3(Tensor dy, Tensor x, Tensor(a!) dw, int[] geom, int cfg, int splits) -> ()");
  m.def("conv_p3_bnb(Tensor x, Tensor w, Tensor w_lo, Tensor(a!) y, Tensor? yres, int[] geom, int cfg, Tensor z, Tensor? yact, int ld, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta, Tensor(b!) acc, int R, int mode) -> ()");
  m.def("split_planes(Tensor x, int ldx, int rows, int C, Tensor(a!) out, int ldo) -> ()");
  m.def("merge_planes(Tensor x, int ldi, int rows, int C, Tensor(a!) y, int ldy) -> ()");
  m.def("gap_fwd_p3(Tensor x, Tensor(a!) y, int N, int HW, int C) -> ()");
}

HCB_TORCH_LIBRARY_IMPL(hcb, CUDA, m) {
  m.impl("conv_igemm", conv_igemm);
  m.impl("conv_igemm_bnb", conv_igemm_bnb);
  m.impl("nonfinite", nonfinite);
  m.impl("loss_total", loss_total);
  m.impl("loss_scale_update", loss_scale_update);
  m.impl("set_splitk_workspace", set_splitk_workspace);
  m.impl("conv_wgrad", conv_wgrad);
  m.impl("bn_stats", bn_stats);
  m.impl("bn_finalize", bn_finalize);
  m.impl("bn_apply", bn_apply);
  m.impl("bn_bwd_reduce", bn_bwd_reduce);
  m.impl("bn_bwd_finalize", bn_bwd_finalize);
  m.impl("bn_bwd_apply", bn_bwd_apply);
  m.impl("pool_fwd", pool_fwd);
  m.impl("pool_bwd", pool_bwd);
  m.impl("pool_fwd_p3", pool_fwd_p3);
  m.impl("gap_fwd", gap_fwd);
  m.impl("gap_bwd", gap_bwd);
  m.impl("softmax_xent", softmax_xent);
  m.impl("colsum", colsum);
  m.impl("zero_bufs", zero_bufs);
  m.impl("sgd_momentum", sgd_momentum);
  m.impl("weight_pack", weight_pack);
  m.impl("cast_f32_bf16", cast_f32_bf16);
  m.impl("add_bf16", add_bf16);
  m.impl("scale_f32", scale_f32);
  m.impl("relu_bwd", relu_bwd);
  m.impl("bn_apply_acc", bn_apply_acc);
  m.impl("bn_bwd_reduce_acc", bn_bwd_reduce_acc);
  m.impl("bn_bwd_apply_acc", bn_bwd_apply_acc);
  m.impl("bn_stats_acc", bn_stats_acc);
  m.impl("l2norm_sq", l2norm_sq);
  m.impl("synth_images", synth_images);
  m.impl("dropout_fwd", dropout_fwd);
  m.impl("bn_relu_maxpool_acc", bn_relu_maxpool_acc);
  m.impl("dropout_bwd", dropout_bwd);
  m.impl("preprocess_images", preprocess_images);
  m.impl("synth_labels", synth_labels);
  m.impl("bucket_pack", bucket_pack);
  m.impl("bucket_unpack", bucket_unpack);
  m.impl("stem_s2d", stem_s2d);
  m.impl("stem_wfold", stem_wfold);
  m.impl("stem_wgrad_unfold", stem_wgrad_unfold);
  m.impl("conv_p3", conv_p3);
  m.impl("conv_wgrad_p3", conv_wgrad_p3);
  m.impl("conv_p3_bnb", conv_p3_bnb);
  m.impl("split_planes", split_planes);
  m.impl("merge_planes", merge_planes);
  m.impl("gap_fwd_p3", gap_fwd_p3);
}
