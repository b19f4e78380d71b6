// Host-visible launch interface of the HIP kernels (no torch headers here so the
// .hip translation units compile in seconds).
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <hip/hip_runtime_api.h>
#endif
#include <stdint.h>

namespace hcb {

// Unsigned division by a runtime-invariant divisor: q = (umulhi(n, m) + n) >> s,
// exact for n < 2^31 (round-up magic number method).
struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
#if defined(__HIPCC__)
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}
#endif

// ---------------------------------------------------------------- implicit GEMM conv
struct ConvParams {
  const void* x;   // NHWC bf16 input, pixel stride ldx elements
  const void* w;   // [Nout][Kpad] bf16
  void* y;         // output rows, stride ldy (bf16 or fp32)
  const void* yres;  // beta-accumulate source (same layout as y)
  const float* bias;  // [Nout] or null
  float* stats;       // [tiles_m][2][Nout] or null
  // per-column shift K of the BN statistics (null = 0): the epilogue accumulates sum(v - K) and
  // sum((v - K)^2), so var = E[(v-K)^2] - E[v-K]^2 stays well conditioned when |mean| >> std
  // (K = the layer's batch mean of the previous step, written by its BN backward)
  const float* stats_shift;
  int N, H, W, C, ldx;
  int P, Q, R, S;
  int stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, idil_h, idil_w;
  int Nout, K, Kpad, ldy;
  int M;
  int remap, OH, OW, osh, osw;  // remap 2: also zero the rest of each stride cell (igemm_epilogue.h)
  int oh0, ow0;  // remap origin: GEMM pixel (p, q) -> output pixel (p*osh + oh0, q*osw + ow0)
  int beta, out_f32;
  int relu;     // fused ReLU in the epilogue (affine layers without BN)
  int stats_R;  // 0: per-tile slab [tiles][2][Nout]; R>0: atomics into [R][2][Nout] replicas
  uint32_t x_bytes, w_bytes;
  // Fused BN-backward reduction (a data-grad GEMM whose output is the dy of a BN layer):
  // the epilogue gates its output with the layer's ReLU mask (bnb_mode 1: y > 0, 2: recomputed
  // from z, 0: none), stores g instead of dy,
  // and accumulates sum(g), sum(g * xhat) per channel into bnb_acc replicas [bnb_R][2][Nout].
  // z / y rows share the output's row index (after remap) with row stride bnb_ld.
  const void* bnb_z;
  const void* bnb_y;
  const float *bnb_mean, *bnb_invstd, *bnb_gamma, *bnb_beta;
  float* bnb_acc;
  int bnb_mode, bnb_R, bnb_ld;
  // In-launch split-K (LDS-DMA kernels): `splits` blocks per output tile each reduce a
  // contiguous k-step range; all but the last arriver park fp32 partials in ws slabs
  // [tile][split][tile elems], the last one (agent-scope ticket in cnt[tile], self-resetting)
  // sums them and runs the epilogue.
  int splits;
  float* ws;
  unsigned* cnt;
  int64_t ws_floats;  // capacity of ws / cnt (set whenever the workspace is registered)
  int cnt_n;
  // plane GEMMs (conv_p3.hip, the fp32 path): the mid and lo bf16 weight packs beside w (hi)
  const void* w_lo;
  const void* w_lo2;
  // 3x3 / stride-1 patch kernels (conv3x3_patch.hip; set by their launcher): LDS rows reserved
  // per input-patch buffer, and division-free index math (output pixel -> (n, p, q), padded
  // linear index -> (n, h', w'))
  int patch_rows;
  FastDiv fd_hw, fd_w, fd_hw2, fd_w2;
  // bf16-plane operands (conv_p3.hip): x is three bf16 planes x_plane bytes apart, each x_bytes long
  uint32_t x_plane;
};
void launch_conv_igemm(const ConvParams& p, int cfg, hipStream_t st);
// cfg >= CONV_PATCH_CFG0: the 3x3 / stride 1 / pad 1 kernels with the input patch resident in
// LDS. Returns false (nothing launched) when the problem or the LDS budget does not fit them.
constexpr int CONV_PATCH_CFG0 = 17;
bool launch_conv3x3_patch(const ConvParams& p, int cfg, hipStream_t st);
bool conv3x3_patch_eligible(const ConvParams& p);
// deterministic reductions (misc.hip): colsum / BN-backward reduce grids limited so that
// every fp32 accumulator slot receives a single add
void set_deterministic(bool on);
bool deterministic();
int conv_tile_m(int cfg);
int conv_tile_n(int cfg);

// weight-gradient implicit GEMM: dW[Nout][K] += sum_m dY[m][Nout] * im2col(X)[m][K]
struct WgradParams {
  const void* dy;  // [M][ldy] 16-bit (the hi plane on the plane path)
  const void* x;   // NHWC 16-bit (the hi plane on the plane path), pixel stride ldx
  float* dw;       // [Nout][K] fp32 (atomically accumulated)
  int N, H, W, C, ldx;
  int P, Q, R, S;
  int stride_h, stride_w, pad_h, pad_w, dil_h, dil_w;
  int Nout, K, M, ldy;
  int ksteps_per_split;
  FastDiv fd_pq, fd_q, fd_c, fd_s;
  uint32_t dy_bytes, x_bytes;
  // bf16-plane operands (conv_p3.hip): dy / x as three bf16 planes dy_plane / x_plane bytes apart
  uint32_t dy_plane, x_plane;
};
void launch_conv_wgrad(const WgradParams& p, int cfg, int splits, hipStream_t st);
int wgrad_tile_m(int cfg);
int wgrad_tile_n(int cfg);

// fp32 convolutions on bf16 hi / mid / lo planes (conv_p3.hip): forward / data-gradient GEMM (x
// planes, weight packs w / w_lo / w_lo2, fp32 output) and weight gradient (dy and x planes)
void launch_conv_p3(const ConvParams& p, int cfg, hipStream_t st);
// fused BN-backward data gradients on the persistent cfgs 18-27 (conv_p3_persist.h BNB): 0 never
// (the twin runs; default -- 0.38% slower step with 1, profiles/r6_persistent_bnb.txt), 1 ReLU
// modes 0 / 2, 2 every mode; initialised from HCB_P3P_BNB
void set_p3p_bnb(int v);
int p3_tile_m(int cfg);
int p3_tile_n(int cfg);
int p3_slot_k(int cfg);
void launch_wgrad_p3(const WgradParams& p, int cfg, int splits, hipStream_t st);
int wgrad_p3_tile_m(int cfg);
int wgrad_p3_tile_n(int cfg);
// fp32 [rows][ldx] <-> bf16 planes [3][rows][ldo] (plane stride `plane` elements)
void launch_split_planes(const float* x, int ldx, int64_t rows, int C, uint16_t* out, int ldo, int64_t plane,
                         hipStream_t st);
void launch_merge_planes(const uint16_t* in, int ldi, int64_t plane, int64_t rows, int C, float* y, int ldy,
                         hipStream_t st);
// global average pool on planes: x planes [N][HW][C] (plane stride xps) -> y planes [N][C] (yps)
void launch_gap_fwd_p3(const uint16_t* x, int64_t xps, uint16_t* y, int64_t yps, int N, int HW, int C, hipStream_t st);

// ---------------------------------------------------------------- batch norm
// stats slab [T][2][C] -> mean, invstd (fp32) and running stats update
void launch_bn_finalize(const float* slab, int T, int C, double count, float eps, float momentum,
                        float* mean, float* invstd, float* run_mean, float* run_var,
                        hipStream_t st);
// stats directly from an activation tensor [M][C] (when not fused into the producer)
void launch_bn_stats(const void* x, int M, int C, int ldx, float* slab, int T, hipStream_t st);
// y = act(gamma*(x-mean)*invstd + beta [+ res])
void launch_bn_apply(const void* x, int ldx, void* y, int ldy, const void* res, int ldr, int M,
                     int C, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, int relu, hipStream_t st);
int bn_num_partials(int M, int C);
// one-launch finalize (split rows + last-block combine); part: fp64 scratch [32][2][C]
int bn_finalize_splits(int T);
void launch_bn_finalize_split(const float* slab, int T, int C, double* part, int fwd, double count, float eps,
                              float momentum, float* mean, float* invstd, float* run_mean, float* run_var,
                              float* dgamma, float* dbeta, hipStream_t st);
// backward reduce: g = dy*mask (relu: 0 none, 1 mask y>0, 2 mask recomputed from x);
// per-block partial sums of g and g*xhat -> slab; optionally writes g to gout
void launch_bn_bwd_reduce2(const void* dy, int lddy, const void* y, int ldyv, const void* x,
                           int ldx, int M, int C, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, int relu, float* slab, int T,
                           void* gout, int ldg, hipStream_t st);
// dgamma/dbeta from slab
void launch_bn_bwd_finalize(const float* slab, int T, int C, float* dgamma, float* dbeta,
                            hipStream_t st);
// dx = gamma*invstd*(g - dbeta/M - xhat*dgamma/M)
void launch_bn_bwd_apply2(const void* dy, int lddy, const void* y, int ldyv, const void* x,
                          int ldx, void* dx, int lddx, int M, int C, const float* mean,
                          const float* invstd, const float* gamma, const float* beta,
                          const float* dgamma, const float* dbeta, int relu, hipStream_t st);

// finalize-free variants: statistics accumulated in R replicas of [2][C] (fp32 atomics).
// Blocks tile (row split) x (channel group) so each block only reduces its group's replicas.
// A second BatchNorm applied to the residual operand inside the same pass (a projection
// shortcut's conv output z_sc, whose statistics its conv epilogue accumulated): the block output
// is act(BN(x) + BN_sc(res)) and BN_sc's normalised tensor is never written. Same M, C, R.
struct ResBN {
  const float* acc;
  const float* gamma;
  const float* beta;
  float* saved_mean;
  float* saved_invstd;
  float* run_mean;
  float* run_var;
  const float* shift;
};
void launch_bn_apply_acc(const void* x, int ldx, void* y, int ldy, const void* res, int ldr, int M, int C,
                         const float* acc, int R, float eps, float momentum, const float* gamma, const float* beta,
                         int relu, float* saved_mean, float* saved_invstd, float* run_mean, float* run_var,
                         const float* shift, const ResBN* res_bn, hipStream_t st, bool f32 = false, int64_t yps = 0,
                         int64_t rps = 0);
// BN(acc statistics) + ReLU + max pool (NHWC, C contiguous): pooled y [N,P,Q] (row stride ldy) and
// the uint8 window argmax [N,P,Q,C]; the BN+ReLU activation itself is not materialised
void launch_bn_relu_maxpool_acc(const void* z, int N, int H, int W, int C, void* y, int P, int Q, int ldy, void* amax,
                                int kh, int kw, int sh, int sw, int ph, int pw, const float* acc, int R, float eps,
                                float momentum, const float* gamma, const float* beta, float* saved_mean,
                                float* saved_invstd, float* run_mean, float* run_var, const float* shift, hipStream_t st,
                                bool f32 = false, int64_t yps = 0);
// pooled-gradient source of the BN backward kernels (bn.hip pool_gather): dy of pixel m of an
// [N][H][W][C] map gathered from the max-pool gradient dyp [N][P][Q] (row stride ldp) through the
// window-local argmax amax [N][P][Q][C] of a k x k / s pool with top / left padding pt / pl
struct PoolSrc {
  const void* dyp;
  const uint8_t* amax;
  int ldp, H, W, P, Q, k, s, pt, pl, C;
};
void launch_bn_bwd_reduce_acc(const void* dy, int lddy, const void* y, int ldyv, const void* x, int ldx, int M,
                              int C, const float* mean, const float* invstd, const float* gamma, const float* beta,
                              int relu, float* acc, int R, void* gout, int ldg, hipStream_t st, bool f32 = false,
                              bool yh = false, const PoolSrc* pool = nullptr);
void launch_bn_bwd_apply_acc(const void* dy, int lddy, const void* y, int ldyv, const void* x, int ldx, void* dx,
                             int lddx, int M, int C, const float* mean, const float* invstd, const float* gamma,
                             const float* beta, const float* acc, int R, float* dgamma, float* dbeta, int relu, float* shift_out, hipStream_t st,
                             bool f32 = false, bool yh = false, int64_t dxps = 0, const PoolSrc* pool = nullptr,
                             const void* add = nullptr, int ldadd = 0);
// BN statistics of x (no producing GEMM epilogue) into R replicas of [2][C]: sums of (v - K), (v - K)^2
void launch_bn_stats_acc(const void* x, int ldx, int M, int C, const float* shift, float* acc, int R, hipStream_t st,
                         bool f32);
// fp32 path, plane-stored tensors: (yps / rps / dxps > 0) outputs / residuals as bf16 hi / mid / lo
// planes with that plane stride in elements; yh: the ReLU-mask source y is the bf16 hi plane

// ---------------------------------------------------------------- pooling
void launch_pool_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int P, int Q,
                     int ldy, int kh, int kw, int sh, int sw, int ph, int pw, int is_max,
                     int count_include_pad, void* idx, hipStream_t st);
void launch_pool_bwd(const void* dy, const void* x, const void* y, void* dx, int N, int H, int W,
                     int C, int ldx, int P, int Q, int ldy, int kh, int kw, int sh, int sw, int ph,
                     int pw, int is_max, int count_include_pad, int accum, const void* idx,
                     hipStream_t st, bool f32 = false);
// fp32 path: k x k max / average pool on bf16 planes (x / y plane strides xps / yps elements)
void launch_pool_fwd_p3(const uint16_t* x, int64_t xps, uint16_t* y, int64_t yps, int N, int H, int W, int C, int ldx,
                        int P, int Q, int ldy, int kh, int kw, int sh, int sw, int ph, int pw, int is_max,
                        int count_include_pad, void* idx, hipStream_t st);
void launch_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st, bool f32 = false);
void launch_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st, bool f32 = false);

// ---------------------------------------------------------------- loss / fc helpers
void launch_softmax_xent(const float* logits, int ld, const int64_t* labels, int B, int ncls,
                         float* row_loss, void* dlogits, int lddl, float scale, const float* scale_dev,
                         hipStream_t st, bool f32 = false, float* dl32 = nullptr,
                         float label_smoothing = 0.f);
constexpr int ZERO_BUFS = 6;
void launch_zero_bufs(float* const* ptrs, const int64_t* ns, int nb, hipStream_t st);
void launch_colsum2(const void* g, int ld, int M, int N, int is_f32, float* out, hipStream_t st);

// ---------------------------------------------------------------- optimizer / weights
// hyper (device fp32): [lr, momentum, weight_decay, grad_scale(, found_inf, loss_scale,
// good_steps, interval)] so a captured graph picks up a new learning rate every replay; with
// hyper_n > 4 the update is skipped when found_inf != 0 (loss scaling)
// l2_slots > 1: per-block w^2 partials into l2_out[0:l2_slots] (>= sgd_grid(n)), summed by loss_total
int sgd_grid(int64_t n);
void launch_sgd_momentum(float* w, float* mom, const float* g, int64_t n, int64_t n_decay,
                         const float* hyper, float* l2_out, int l2_slots, int nesterov, int hyper_n, hipStream_t st);
void launch_nonfinite(const float* g, int64_t n, float* flag, hipStream_t st);
void launch_loss_total(const float* row_loss, int B, const float* l2, int l2_n, float half_wd, float* loss,
                       hipStream_t st);
void launch_loss_scale_update(float* hyper, float world, int dynamic, hipStream_t st);
struct WPackEntry {  // all int64 so the table is a plain int64 tensor [n][9]
  int64_t src_off;   // fp32 master offset (elements)
  int64_t pack_off;  // bf16 packed [Nout][Kpad] offset (elements), -1 = skip
  int64_t tr_off;    // bf16 transposed-flipped [C][Kpad_t] offset, -1 = skip
  int64_t Nout, R, S, C, Kpad, Kpad_t;
};
// lo: 0 the bf16 pack (the hi plane), 1 / 2 the mid / lo plane alone, 3 all three planes (plane
// stride pstride elements: the fp32 path's pack planes in one pass)
void launch_weight_pack(const float* master, uint16_t* pack, const WPackEntry* entries_dev,
                        int n_entries, int64_t max_work, hipStream_t st, int lo = 0, int64_t pstride = 0);
// dropout on bf16 activations (n % 8 == 0): mask = 1 bit per element packed 8 per byte
void launch_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float keep, uint64_t seed,
                        const int64_t* step, hipStream_t st, bool f32 = false);
void launch_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float keep, hipStream_t st,
                        bool f32 = false);
void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st);
void launch_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st);
void launch_add_bf16(const void* a, const void* b, void* y, int64_t n, hipStream_t st);
void launch_scale_f32(float* x, int64_t n, float s, hipStream_t st);
void launch_relu_bwd(const void* dy, const void* y, void* dz, int64_t n, hipStream_t st, bool f32 = false);
void launch_l2norm_sq(const float* x, int64_t n, float* out, hipStream_t st);

// ---------------------------------------------------------------- data
void launch_synth_images(void* out, int64_t n_pix, int C, int Cpad, float mean, float std,
                         uint64_t seed, hipStream_t st, bool f32 = false);
void launch_synth_labels(int64_t* out, int n, int ncls, uint64_t seed, hipStream_t st);
// real data: batch of RGB uint8 crops (desc [B][4] = byte offset, h, w, flip) -> bilinear resize
// to S x S, optional horizontal flip, x*scale[c]+bias[c], NHWC bf16 with Cpad channels
void launch_preprocess_images(const uint8_t* src, const int64_t* desc, int B, void* out, int S, int Cpad,
                              const float* scale, const float* bias, bool f32, hipStream_t st);

// ---------------------------------------------------------------- space-to-depth stem (stem.hip)
void launch_stem_s2d_f32(const float* x, int N, int H, int W, int ldx, uint16_t* out, int64_t plane, int Hs, int Ws,
                         int pad, hipStream_t st);
void launch_stem_s2d(const uint16_t* x, int N, int H, int W, int ldx, uint16_t* out, int Hs, int Ws, int pad,
                     hipStream_t st);
void launch_stem_wfold(const float* w, int cout, int cs, uint16_t* wp, hipStream_t st, bool p3 = false);
void launch_stem_wgrad_unfold(const float* dwp, int cout, int cs, float* dw, hipStream_t st);

// ---------------------------------------------------------------- gradient buckets
// One-shot xGMI allreduce (xgmi.hip): bases = every rank's IPC-mapped staging region.
int xgmi_max_ranks();
void launch_xgmi_allreduce(const float* const* bases, int R, int rank, const float* in, float* out, int64_t n,
                           int64_t cap, float scale, unsigned* err, unsigned spin, hipStream_t st);
void launch_bucket_pack(const float* src, void* dst, int64_t n, float scale, int mode,
                        hipStream_t st);
void launch_bucket_unpack(const void* src, float* dst, int64_t n, float scale, int mode,
                          hipStream_t st);
// debug: one wave sleeps ~ms milliseconds (bounded, s_memrealtime-timed) on stream st
void launch_debug_sleep(int ms, hipStream_t st);

}  // namespace hcb
