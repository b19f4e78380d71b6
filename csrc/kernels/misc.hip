// Loss, optimizer, weight-preparation, data and gradient-bucket kernels (gfx950).
//
//   * softmax_xent: tf.losses.sparse_softmax_cross_entropy + its gradient in one pass
//     (label_smoothing ls: targets (1-ls)*onehot + ls/ncls, tf.losses.softmax_cross_entropy's form)
//     (one 256-thread block per row, wave64 shuffles + LDS for the row max / sum).
//   * sgd_momentum: TF ApplyMomentum over ALL parameters in ONE launch (flat fp32
//     master/momentum/grad buffers; L2 weight decay folded in as wd*w for the decayed
//     prefix, Horovod averaging / loss-scale folded in as grad_scale, and the L2 term of
//     the reported total_loss reduced on the fly) — SURVEY.md §2.6 "ApplyMomentum",
//     "L2 weight decay"; tf_cnn_benchmarks flags --optimizer=momentum
//     (/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:73).
//   * weight_pack: one multi-tensor launch producing the bf16 GEMM operands of every
//     conv from the fp32 masters: [Cout][Kpad] for fwd and the flipped/transposed
//     [Cin][Kpad_t] for the data gradient.
//   * synth: tf_cnn_benchmarks synthetic ImageNet (truncated normal, mean 127, sd 60,
//     generated once on device) + uniform labels.
//   * bucket pack/unpack: Horovod fusion-buffer memcpy-in/out role with scale and
//     optional bf16 compression.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace hcb {

// ------------------------------------------------------------------ softmax xent
template <typename T = uint16_t>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits, int ld,
                                                           const int64_t* __restrict__ labels,
                                                           int ncls, float* row_loss,
                                                           T* dl, int lddl, float scale,
                                                           const float* scale_dev, float* dl32, float ls) {
  __shared__ float red[12];
  if (scale_dev != nullptr) scale *= *scale_dev;  // device-resident loss scale
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* lr = logits + (size_t)row * ld;
  float mx = -INFINITY;
  for (int c = tid; c < ncls; c += 256) mx = fmaxf(mx, lr[c]);
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f, sl = 0.f;
  for (int c = tid; c < ncls; c += 256) {
    s += __expf(lr[c] - mx);
    sl += lr[c];  // (the smoothed targets' uniform part weighs every logit)
  }
  s = wave_sum(s);
  if (ls != 0.f) sl = wave_sum(sl);
  if (lane == 0) {
    red[4 + wid] = s;
    red[8 + wid] = sl;
  }
  __syncthreads();
  s = red[4] + red[5] + red[6] + red[7];
  const float lse = mx + __logf(s);
  const int lab = (int)labels[row];
  const float pos = 1.f - ls, neg = ls / (float)ncls;  // target = pos * onehot + neg
  if (tid == 0)
    row_loss[row] = ls != 0.f ? lse - pos * lr[lab] - neg * (red[8] + red[9] + red[10] + red[11]) : lse - lr[lab];
  const float inv = 1.f / s;
  for (int c = tid; c < lddl; c += 256) {
    float g = 0.f;
    if (c < ncls) g = (__expf(lr[c] - mx) * inv - ((c == lab ? pos : 0.f) + neg)) * scale;
    if constexpr (sizeof(T) == 4) {
      dl[(size_t)row * lddl + c] = g;
    } else {
      dl[(size_t)row * lddl + c] = f2act(g);
      if (dl32 != nullptr) dl32[(size_t)row * lddl + c] = g;  // unrounded: the bias gradient's source
    }
  }
}

// column sums: out[n] = sum_m g[m][n] (bf16 or fp32 input, fp32 out). A block covers 256 columns
// (32 lanes x 8-column vectors) and 8 row lanes that stride over M; the 8 row partials meet in
// LDS. One block row (gridDim.x == 1, `direct`): the block is the column's only writer and
// stores the sum; otherwise one fp32 atomic per column and block into `out` zeroed by
// zero_f32_kernel just before. (The bias gradient of a conv over a 224x224 map reduces 3.2 M
// rows.) No hipMemsetAsync: inside a captured step graph with the runtime's packet capture on,
// the memset node of the 1001-float fc-bias gradient left non-zero garbage (tools/pc_buffer_bisect.py,
// tools/graph_fork_repro.hip mode 10, profiles/r4_packet_capture_root_cause.txt).
__global__ void zero_f32_kernel(float* out, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = 0.f;
}
// Step-start clears in ONE launch (the flat gradient, the BN statistic accumulators, scratch
// accumulators): up to ZERO_BUFS fp32 buffers, 16-byte stores over each buffer's 4-float body and
// dword stores over its tail. Replaces the per-buffer torch fill kernels of the captured step (and
// never a memset node: see colsum below).
struct ZeroBufs {
  float* p[ZERO_BUFS];
  int64_t n[ZERO_BUFS];
  int nb;
};
__global__ __launch_bounds__(256) void zero_bufs_kernel(ZeroBufs z) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int b = 0; b < z.nb; ++b) {
    float* p = z.p[b];
    const int64_t n = z.n[b], n4 = n >> 2;
    f32x4* p4 = reinterpret_cast<f32x4*>(p);
    for (int64_t i = t0; i < n4; i += stride) p4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t i = (n4 << 2) + t0; i < n; i += stride) p[i] = 0.f;
  }
}
void launch_zero_bufs(float* const* ptrs, const int64_t* ns, int nb, hipStream_t st) {
  ZeroBufs z{};
  int64_t tot = 0;
  for (int b = 0; b < nb; ++b) {
    z.p[b] = ptrs[b];
    z.n[b] = ns[b];
    tot += ns[b];
  }
  z.nb = nb;
  int64_t blocks = (tot / 4 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(zero_bufs_kernel, dim3((unsigned)blocks), dim3(256), 0, st, z);
}

__global__ __launch_bounds__(256) void colsum_kernel(const void* g, int ld, int M, int N, int is_f32,
                                                     float* out, int direct) {
  __shared__ float part[8][257];
  const int lane = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = (blockIdx.y * 32 + lane) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    for (int m = blockIdx.x * 8 + rl; m < M; m += gridDim.x * 8) {
      float f[8];
      if (is_f32) {
        const f32x4* r = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(g) + (size_t)m * ld + c0);
        const f32x4 a = r[0], b = r[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[e] = a[e];
          f[4 + e] = b[e];
        }
      } else {
        unpack8(*reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(g) + (size_t)m * ld + c0), f);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[rl][lane * 8 + e] = acc[e];
  __syncthreads();
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c < N) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) s += part[r][threadIdx.x];
    if (direct)
      out[c] = s;
    else
      atomicAdd(out + c, s);
  }
}

__global__ __launch_bounds__(256) void sgd_momentum_kernel(float* __restrict__ w,
                                                           float* __restrict__ mom,
                                                           const float* __restrict__ g, int64_t n,
                                                           int64_t n_decay,
                                                           const float* __restrict__ hyper,
                                                           float* l2_out, int l2_slots, int nesterov,
                                                           int hyper_n) {
  __shared__ float red[4];
  // l2_slots > 1: this block's sum of w^2 goes to its OWN slot l2_out[blockIdx.x] (plain store, no
  // zeroing launch; block 0 clears the slots past the grid) and loss_total sums the slots in a fixed
  // order -- the reported loss is run-to-run deterministic. l2_slots == 1: one atomic per block
  // into l2_out[0] (zeroed by the caller).
  // loss scaling: hyper[4] = "non-finite gradient seen" -> skip the whole update (TF
  // LossScaleOptimizer semantics); the flag is wave-uniform so every block exits together
  if (hyper_n > 4 && hyper[4] != 0.f) {
    if (l2_out != nullptr && l2_slots > 1) {
      for (int i = threadIdx.x; i < l2_slots; i += blockDim.x)
        if (i % (int)gridDim.x == (int)blockIdx.x) l2_out[i] = 0.f;
    }
    return;
  }
  const float lr = hyper[0], mu = hyper[1], wd = hyper[2], gscale = hyper[3];
  float l2 = 0.f;
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 wv = reinterpret_cast<f32x4*>(w)[i];
    f32x4 mv = reinterpret_cast<f32x4*>(mom)[i];
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int64_t j = i * 4 + e;
      float gg = gv[e] * gscale;
      if (j < n_decay) {
        gg += wd * wv[e];
        l2 += wv[e] * wv[e];
      }
      float m = mu * mv[e] + gg;
      mv[e] = m;
      wv[e] -= nesterov ? lr * (gg + mu * m) : lr * m;
    }
    reinterpret_cast<f32x4*>(w)[i] = wv;
    reinterpret_cast<f32x4*>(mom)[i] = mv;
  }
  // scalar tail
  for (int64_t j = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    float gg = g[j] * gscale;
    if (j < n_decay) {
      gg += wd * w[j];
      l2 += w[j] * w[j];
    }
    float m = mu * mom[j] + gg;
    mom[j] = m;
    w[j] -= nesterov ? lr * (gg + mu * m) : lr * m;
  }
  if (l2_out != nullptr) {
    l2 = wave_sum(l2);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l2;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float t = (red[0] + red[1]) + (red[2] + red[3]);
      if (l2_slots > 1)
        l2_out[blockIdx.x] = t;
      else
        atomicAdd(l2_out, t);
    }
    if (l2_slots > 1 && blockIdx.x == 0)
      for (int i = (int)gridDim.x + threadIdx.x; i < l2_slots; i += blockDim.x) l2_out[i] = 0.f;
  }
}

__global__ __launch_bounds__(256) void l2norm_kernel(const float* __restrict__ x, int64_t n,
                                                     float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += x[i] * x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

// ------------------------------------------------------------------ weights
// Per entry the work is (A) the row-padded copy [Nout][K] -> [Nout][Kpad] in 8-element vectors
// (two 16-byte reads, one 16-byte write per lane; pad columns stay zero from allocation) and
// (B) the flipped/transposed data-grad operand [C][tap*Nout + kk] <- W[kk][R-1-r][S-1-s][c],
// a 64x64 LDS-tiled transpose per (tap, kk-tile, c-tile) so both the fp32 reads (along c) and
// the bf16 writes (along kk) are coalesced. Blocks grid-stride over A chunks then B tiles.
// lo: pack the later terms of the fp32 path's three-way bf16 split w = hi + mid + lo (the bf16x6
// GEMMs' weight operands) instead of w, into a buffer of the same layout: lo = 1 the residual
// r = w - bf16(w) (stored as bf16: mid), lo = 2 what is left, r - bf16(r) (stored as bf16: lo)
__device__ __forceinline__ float wp_val(float v, int lo) {
  if (lo == 0) return v;
  const float r = v - bf2f(f2bf(v));
  return lo == 1 ? r : r - bf2f(f2bf(r));
}
// P3 (the fp32 path): all three bf16 planes hi / mid / lo of every pack in one pass over the
// masters, plane t at pack + t * pstride
template <bool P3>
__global__ __launch_bounds__(256) void weight_pack_kernel(const float* __restrict__ master,
                                                          uint16_t* __restrict__ pack,
                                                          const WPackEntry* __restrict__ ents, int lo,
                                                          int64_t pstride) {
  constexpr int NPL = P3 ? 3 : 1;
  __shared__ float tile[64][65];
  const WPackEntry e = ents[blockIdx.y];
  const int R = (int)e.R, S = (int)e.S, C = (int)e.C, Nout = (int)e.Nout;
  const int Kpad = (int)e.Kpad, Kpad_t = (int)e.Kpad_t;
  const int K = R * S * C, K8 = K / 8;
  const float* src = master + e.src_off;
  const int tid = threadIdx.x;
  const int nA = e.pack_off >= 0 ? (Nout * K8 + 255) / 256 : 0;
  const int tkk = (Nout + 63) / 64, tc = (C + 63) / 64;
  const int nB = e.tr_off >= 0 ? R * S * tkk * tc : 0;
  for (int u = blockIdx.x; u < nA + nB; u += gridDim.x) {
    if (u < nA) {
      const int i = u * 256 + tid;
      if (i < Nout * K8) {
        const int j = i / K8, k8 = i - j * K8;
        const float4* s4 = reinterpret_cast<const float4*>(src + (size_t)j * K + k8 * 8);
        const float4 a = s4[0], b = s4[1];
#pragma unroll
        for (int t = 0; t < NPL; ++t) {
          const int l = P3 ? t : lo;
          u32x4 v;
          v[0] = pack2(wp_val(a.x, l), wp_val(a.y, l));
          v[1] = pack2(wp_val(a.z, l), wp_val(a.w, l));
          v[2] = pack2(wp_val(b.x, l), wp_val(b.y, l));
          v[3] = pack2(wp_val(b.z, l), wp_val(b.w, l));
          *reinterpret_cast<u32x4*>(pack + t * pstride + e.pack_off + (size_t)j * Kpad + k8 * 8) = v;
        }
      }
      continue;
    }
    int t = u - nA;
    const int ci = t % tc;
    t /= tc;
    const int ki = t % tkk;
    const int tap = t / tkk;
    const int rr = tap / S, ss = tap - rr * S;
    const int kk0 = ki * 64, c0 = ci * 64;
    // load W[kk0+row][R-1-rr][S-1-ss][c0 .. c0+63] (fp32, float4 along c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tid >> 4) + 16 * q, c4 = (tid & 15) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kk0 + row < Nout && c0 + c4 < C)
        v = *reinterpret_cast<const float4*>(src + ((size_t)((kk0 + row) * R + (R - 1 - rr)) * S + (S - 1 - ss)) * C +
                                             c0 + c4);
      tile[row][c4] = P3 ? v.x : wp_val(v.x, lo);  // P3: the raw value, split at the pack stage
      tile[row][c4 + 1] = P3 ? v.y : wp_val(v.y, lo);
      tile[row][c4 + 2] = P3 ? v.z : wp_val(v.z, lo);
      tile[row][c4 + 3] = P3 ? v.w : wp_val(v.w, lo);
    }
    __syncthreads();
    {
      const int c = tid >> 2, k16 = (tid & 3) * 16;
      if (c0 + c < C) {
        const size_t o = (size_t)e.tr_off + (size_t)(c0 + c) * Kpad_t + (size_t)tap * Nout + kk0 + k16;
#pragma unroll
        for (int t = 0; t < NPL; ++t) {
          auto tv = [&](int k) { return P3 ? wp_val(tile[k][c], t) : tile[k][c]; };
          uint16_t* pk = pack + t * pstride;
          if (kk0 + k16 + 16 <= Nout && (o & 7) == 0) {
            u32x4 v0, v1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v0[q] = pack2(tv(k16 + 2 * q), tv(k16 + 2 * q + 1));
              v1[q] = pack2(tv(k16 + 8 + 2 * q), tv(k16 + 9 + 2 * q));
            }
            reinterpret_cast<u32x4*>(pk + o)[0] = v0;
            reinterpret_cast<u32x4*>(pk + o)[1] = v1;
          } else {
            for (int q = 0; q < 16 && kk0 + k16 + q < Nout; ++q) pk[o + q] = f2act(tv(k16 + q));
          }
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ dropout
// tf.nn.dropout semantics: keep with probability `keep`, scale kept values by 1/keep. The mask
// bit of element i is a counter-based hash of (seed, step, i) -- no RNG state to carry -- and
// `step` is read from device memory so every replay of a captured graph draws a new mask.
__device__ __forceinline__ uint32_t dropout_mix32(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

// T: the build's 16-bit activation type or fp32 (the zoo models' fp32 path)
template <typename T>
__global__ __launch_bounds__(256) void dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask, int64_t n8, uint32_t thresh,
                                                          float inv_keep, uint64_t seed,
                                                          const int64_t* __restrict__ step) {
  const uint64_t base = seed * 0x9E3779B97F4A7C15ull + (uint64_t)(*step) * 0xD1B54A32D192ED03ull;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    Act8<T> v;
    v.load(x + i * 8);
    v.to_f(f);
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool keep = dropout_mix32(base + (uint64_t)(i * 8 + e)) < thresh;
      f[e] = keep ? f[e] * inv_keep : 0.f;
      bits |= (keep ? 1u : 0u) << e;
    }
    Act8<T>::store(y + i * 8, f);
    mask[i] = (uint8_t)bits;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          T* __restrict__ dx, int64_t n8, float inv_keep) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    Act8<T> v;
    v.load(dy + i * 8);
    v.to_f(f);
    const uint32_t bits = mask[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = ((bits >> e) & 1u) ? f[e] * inv_keep : 0.f;
    Act8<T>::store(dx + i * 8, f);
  }
}

__global__ void cast_f32_bf16_kernel(const float* x, uint16_t* y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2act(x[i]);
}
__global__ void cast_bf16_f32_kernel(const uint16_t* x, float* y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = act2f(x[i]);
}
__global__ void add_bf16_kernel(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float fa[8], fb[8];
    unpack8(reinterpret_cast<const u32x4*>(a)[i], fa);
    unpack8(reinterpret_cast<const u32x4*>(b)[i], fb);
#pragma unroll
    for (int e = 0; e < 8; ++e) fa[e] += fb[e];
    reinterpret_cast<u32x4*>(y)[i] = pack8(fa);
  }
}
// dz = dy * (y > 0), 8 elements per thread (16-bit or fp32)
template <typename T>
__global__ void relu_bwd_kernel(const T* dy, const T* y, T* dz, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float d[8], v[8];
    Act8<T> a, b;
    a.load(dy + i * 8);
    b.load(y + i * 8);
    a.to_f(d);
    b.to_f(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = v[e] > 0.f ? d[e] : 0.f;
    Act8<T>::store(dz + i * 8, d);
  }
}

__global__ void scale_f32_kernel(float* x, int64_t n, float s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= s;
}

// ------------------------------------------------------------------ synthetic data
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float u01(uint64_t key) {
  return ((mix32(key) >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T = uint16_t>
__global__ void synth_images_kernel(T* out, int64_t n_pix, int C, int Cpad, float mean,
                                    float std, uint64_t seed) {
  const int64_t total = n_pix * Cpad;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % Cpad);
    float v = 0.f;
    if (c < C) {
      // truncated normal: resample until |z| <= 2 (tf.truncated_normal)
      float z = 0.f;
      for (uint64_t a = 0; a < 64; ++a) {
        uint64_t key = seed * 0x9E3779B97F4A7C15ULL + (uint64_t)i * 128 + 2 * a;
        float u1 = u01(key), u2 = u01(key + 1);
        z = sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
        if (fabsf(z) <= 2.f) break;
        z = 0.f;
      }
      v = mean + std * z;
    }
    if constexpr (sizeof(T) == 4)
      out[i] = v;
    else
      out[i] = f2act(v);
  }
}

__global__ void synth_labels_kernel(int64_t* out, int n, int ncls, uint64_t seed) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int64_t)(mix32(seed * 0x2545F4914F6CDD1DULL + i) % (uint32_t)ncls);
}

// ------------------------------------------------------------------ gradient buckets
// Horovod Compression for the fused gradient buffer: mode 0 = fp32 (scaled copy), 1 = bf16,
// 2 = IEEE fp16 (Compression.fp16). Four elements per thread, 16-byte fp32 loads; the tail
// (n % 4) is handled by the first threads of the grid.
template <int MODE>
__global__ __launch_bounds__(256) void bucket_pack_kernel(const float* __restrict__ src, void* __restrict__ dst,
                                                          int64_t n, float scale) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t i = t0; i < n4; i += stride) {
    f32x4 v = reinterpret_cast<const f32x4*>(src)[i] * scale;
    if constexpr (MODE == 0) {
      reinterpret_cast<f32x4*>(dst)[i] = v;
    } else if constexpr (MODE == 1) {
      reinterpret_cast<u32x2*>(dst)[i] = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
    } else {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      reinterpret_cast<h4*>(dst)[i] = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
    }
  }
  for (int64_t i = 4 * n4 + t0; i < n; i += stride) {
    const float v = src[i] * scale;
    if constexpr (MODE == 0)
      reinterpret_cast<float*>(dst)[i] = v;
    else if constexpr (MODE == 1)
      reinterpret_cast<uint16_t*>(dst)[i] = f2bf(v);
    else
      reinterpret_cast<_Float16*>(dst)[i] = (_Float16)v;
  }
}
template <int MODE>
__global__ __launch_bounds__(256) void bucket_unpack_kernel(const void* __restrict__ src, float* __restrict__ dst,
                                                            int64_t n, float scale) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t i = t0; i < n4; i += stride) {
    f32x4 v;
    if constexpr (MODE == 0) {
      v = reinterpret_cast<const f32x4*>(src)[i];
    } else if constexpr (MODE == 1) {
      u32x2 u = reinterpret_cast<const u32x2*>(src)[i];
      v = f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
                __uint_as_float(u[1] & 0xffff0000u)};
    } else {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 h = reinterpret_cast<const h4*>(src)[i];
      v = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    }
    reinterpret_cast<f32x4*>(dst)[i] = v * scale;
  }
  for (int64_t i = 4 * n4 + t0; i < n; i += stride) {
    float v;
    if constexpr (MODE == 0)
      v = reinterpret_cast<const float*>(src)[i];
    else if constexpr (MODE == 1)
      v = bf2f(reinterpret_cast<const uint16_t*>(src)[i]);
    else
      v = (float)reinterpret_cast<const _Float16*>(src)[i];
    dst[i] = v * scale;
  }
}

static int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

void launch_softmax_xent(const float* logits, int ld, const int64_t* labels, int B, int ncls,
                         float* row_loss, void* dlogits, int lddl, float scale, const float* scale_dev,
                         hipStream_t st, bool f32, float* dl32, float label_smoothing) {
  if (f32)
    hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(B), dim3(256), 0, st, logits, ld, labels, ncls, row_loss,
                       (float*)dlogits, lddl, scale, scale_dev, (float*)nullptr, label_smoothing);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<uint16_t>, dim3(B), dim3(256), 0, st, logits, ld, labels, ncls, row_loss,
                       (uint16_t*)dlogits, lddl, scale, scale_dev, dl32, label_smoothing);
}

// ------------------------------------------------------------------ loss scaling
// flag[0] = 1 when any gradient element is Inf/NaN (the caller zeroes the flag first)
__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ g, int64_t n, float* flag) {
  int bad = 0;
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
    bad |= !(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]) && isfinite(v[3]));
  }
  for (int64_t j = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(g[j]);
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = 1.f;  // benign race: every writer stores 1
}
// hyper = [lr, mu, wd, grad_scale, found_inf, loss_scale, good_steps, interval]; one thread.
// dynamic: halve on overflow (floor 1), double after `interval` clean steps; then
// grad_scale = 1 / (world * loss_scale) for the next step.
__global__ void loss_scale_update_kernel(float* hyper, float world, int dynamic) {
  float S = hyper[5];
  if (dynamic) {
    if (hyper[4] != 0.f) {
      S = fmaxf(S * 0.5f, 1.f);
      hyper[6] = 0.f;
    } else {
      hyper[6] += 1.f;
      if (hyper[6] >= hyper[7]) {
        S *= 2.f;
        hyper[6] = 0.f;
      }
    }
    hyper[5] = S;
  }
  hyper[3] = 1.f / (world * S);
}
// loss[0] = mean(row_loss[0:B]) + half_wd * sum(l2[0:l2_n]) (l2 may be null; l2_n > 1: the
// optimizer's per-block partials): the step's reported loss in one launch (one workgroup, fixed
// reduction order) instead of mean / mul / add / copy kernels.
__global__ __launch_bounds__(256) void loss_total_kernel(const float* __restrict__ row_loss, int B,
                                                         const float* __restrict__ l2, int l2_n, float half_wd,
                                                         float* __restrict__ loss) {
  __shared__ float part[8];
  float s = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) s += row_loss[i];
  if (l2)
    for (int i = threadIdx.x; i < l2_n; i += 256) q += l2[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  if ((threadIdx.x & 63) == 0) {
    part[threadIdx.x >> 6] = s;
    part[4 + (threadIdx.x >> 6)] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = ((part[0] + part[1]) + (part[2] + part[3])) / (float)B;
    if (l2) t += half_wd * ((part[4] + part[5]) + (part[6] + part[7]));
    loss[0] = t;
  }
}
void launch_loss_total(const float* row_loss, int B, const float* l2, int l2_n, float half_wd, float* loss,
                       hipStream_t st) {
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(256), 0, st, row_loss, B, l2, l2_n, half_wd, loss);
}
void launch_nonfinite(const float* g, int64_t n, float* flag, hipStream_t st) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, g, n, flag);
}
void launch_loss_scale_update(float* hyper, float world, int dynamic, hipStream_t st) {
  hipLaunchKernelGGL(loss_scale_update_kernel, dim3(1), dim3(1), 0, st, hyper, world, dynamic);
}
// Deterministic mode (hcb.set_deterministic): reductions whose float atomics would add in a
// run-dependent order are launched so that every accumulator slot receives exactly one add.
static bool g_deterministic = false;
void set_deterministic(bool on) { g_deterministic = on; }
bool deterministic() { return g_deterministic; }

void launch_colsum2(const void* g, int ld, int M, int N, int is_f32, float* out, hipStream_t st) {
  const int gy = (N + 255) / 256;
  int gx = g_deterministic ? 1 : (M + 63) / 64;  // >= 8 rows per thread
  const int cap = (2048 + gy - 1) / gy;
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  // HCB_COLSUM_MEMSET=1: the round-3 form (memset node + atomics), kept only to reproduce the
  // packet-capture finding (tools/pc_buffer_bisect.py)
  static const bool legacy = [] {
    const char* e = std::getenv("HCB_COLSUM_MEMSET");
    return e != nullptr && e[0] == '1';
  }();
  if (legacy) {
    (void)hipMemsetAsync(out, 0, (size_t)N * sizeof(float), st);
    hipLaunchKernelGGL(colsum_kernel, dim3(gx, gy), dim3(256), 0, st, g, ld, M, N, is_f32, out, 0);
    return;
  }
  if (gx > 1) hipLaunchKernelGGL(zero_f32_kernel, dim3((N + 255) / 256), dim3(256), 0, st, out, N);
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, gy), dim3(256), 0, st, g, ld, M, N, is_f32, out, gx == 1 ? 1 : 0);
}
int sgd_grid(int64_t n) { return grid_for((n + 3) / 4); }
void launch_sgd_momentum(float* w, float* mom, const float* g, int64_t n, int64_t n_decay,
                         const float* hyper, float* l2_out, int l2_slots, int nesterov, int hyper_n, hipStream_t st) {
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(sgd_grid(n)), dim3(256), 0, st, w, mom, g,
                     n, n_decay, hyper, l2_out, l2_slots, nesterov, hyper_n);
}
void launch_l2norm_sq(const float* x, int64_t n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(l2norm_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, out);
}
void launch_weight_pack(const float* master, uint16_t* pack, const WPackEntry* entries_dev,
                        int n_entries, int64_t max_work, hipStream_t st, int lo, int64_t pstride) {
  int64_t units = max_work / 2048 + 2;  // A chunks are 2048 elements, B tiles 4096
  int gx = units > 1024 ? 1024 : (int)units;
  if (lo == 3)  // all three planes, plane stride pstride
    hipLaunchKernelGGL(weight_pack_kernel<true>, dim3(gx, n_entries), dim3(256), 0, st, master, pack, entries_dev, 0,
                       pstride);
  else
    hipLaunchKernelGGL(weight_pack_kernel<false>, dim3(gx, n_entries), dim3(256), 0, st, master, pack, entries_dev,
                       lo, (int64_t)0);
}
void launch_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float keep, uint64_t seed,
                        const int64_t* step, hipStream_t st, bool f32) {
  const uint32_t thresh = keep >= 1.f ? 0xffffffffu : (uint32_t)((double)keep * 4294967296.0);
  if (f32)
    hipLaunchKernelGGL(dropout_fwd_kernel<float>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const float*)x, (float*)y,
                       mask, n / 8, thresh, 1.f / keep, seed, step);
  else
    hipLaunchKernelGGL(dropout_fwd_kernel<uint16_t>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const uint16_t*)x,
                       (uint16_t*)y, mask, n / 8, thresh, 1.f / keep, seed, step);
}
void launch_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float keep, hipStream_t st,
                        bool f32) {
  if (f32)
    hipLaunchKernelGGL(dropout_bwd_kernel<float>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const float*)dy, mask,
                       (float*)dx, n / 8, 1.f / keep);
  else
    hipLaunchKernelGGL(dropout_bwd_kernel<uint16_t>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const uint16_t*)dy,
                       mask, (uint16_t*)dx, n / 8, 1.f / keep);
}
void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n);
}
void launch_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n);
}
void launch_add_bf16(const void* a, const void* b, void* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(add_bf16_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, (const uint16_t*)a,
                     (const uint16_t*)b, (uint16_t*)y, n / 8);
}
void launch_relu_bwd(const void* dy, const void* y, void* dz, int64_t n, hipStream_t st, bool f32) {
  if (f32)
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const float*)dy,
                       (const float*)y, (float*)dz, n / 8);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<uint16_t>, dim3(grid_for(n / 8)), dim3(256), 0, st, (const uint16_t*)dy,
                       (const uint16_t*)y, (uint16_t*)dz, n / 8);
}
void launch_scale_f32(float* x, int64_t n, float s, hipStream_t st) {
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, s);
}
void launch_synth_images(void* out, int64_t n_pix, int C, int Cpad, float mean, float std,
                         uint64_t seed, hipStream_t st, bool f32) {
  if (f32)
    hipLaunchKernelGGL(synth_images_kernel<float>, dim3(grid_for(n_pix * Cpad)), dim3(256), 0, st, (float*)out, n_pix,
                       C, Cpad, mean, std, seed);
  else
    hipLaunchKernelGGL(synth_images_kernel<uint16_t>, dim3(grid_for(n_pix * Cpad)), dim3(256), 0, st,
                       (uint16_t*)out, n_pix, C, Cpad, mean, std, seed);
}
void launch_synth_labels(int64_t* out, int n, int ncls, uint64_t seed, hipStream_t st) {
  hipLaunchKernelGGL(synth_labels_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out, n, ncls,
                     seed);
}
static int pack_grid(int64_t n) {
  int64_t g = ((n >> 2) + 255) / 256;
  if (g > 2048) g = 2048;
  return (int)(g < 1 ? 1 : g);
}
// mode: 0 fp32, 1 bf16, 2 fp16 (anything else is rejected by the callers)
void launch_bucket_pack(const float* src, void* dst, int64_t n, float scale, int mode, hipStream_t st) {
  if (mode == 1)
    hipLaunchKernelGGL(bucket_pack_kernel<1>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
  else if (mode == 2)
    hipLaunchKernelGGL(bucket_pack_kernel<2>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
  else
    hipLaunchKernelGGL(bucket_pack_kernel<0>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
}
void launch_bucket_unpack(const void* src, float* dst, int64_t n, float scale, int mode, hipStream_t st) {
  if (mode == 1)
    hipLaunchKernelGGL(bucket_unpack_kernel<1>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
  else if (mode == 2)
    hipLaunchKernelGGL(bucket_unpack_kernel<2>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
  else
    hipLaunchKernelGGL(bucket_unpack_kernel<0>, dim3(pack_grid(n)), dim3(256), 0, st, src, dst, n, scale);
}

// Debug only (HCB_COMM_DEBUG_SLEEP_MS): a single wave that sleeps for ~ms milliseconds on the
// 100 MHz real-time counter, so a stalled collective can be staged on one GPU. Bounded: the
// loop exits after the requested time (ms is clamped to 10 s on the host).
__global__ __launch_bounds__(64) void debug_sleep_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
void launch_debug_sleep(int ms, hipStream_t st) {
  if (ms <= 0) return;
  if (ms > 10000) ms = 10000;
  hipLaunchKernelGGL(debug_sleep_kernel, dim3(1), dim3(64), 0, st, (uint64_t)ms * 100000ull);
}

}  // namespace hcb
