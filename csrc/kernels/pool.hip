// Pooling kernels, NHWC bf16 (MKL-DNN max/avg pool role):
//   * generic k x k max / average pool with TF-style (possibly asymmetric) padding:
//     ResNet's 3x3/2 'SAME' max pool, Inception's 3x3/1 avg-pool branches and 3x3/2
//     max-pool reductions, 8x8 avg pool heads.
//   * backward as a GATHER over the (at most ceil(k/s)^2) windows covering an input
//     pixel, so no atomics; the max pool recomputes the first-max position of each
//     window (TF semantics: gradient goes to the first maximal element).
//   * global average pool (spatial mean) fwd/bwd.
// Each thread handles one pixel x 8 channels (16-byte vectors).
#include "common.h"
#include "kernels.h"

namespace hcb {

__global__ __launch_bounds__(256) void pool_fwd_kernel(const uint16_t* __restrict__ x,
                                                       uint16_t* __restrict__ y, int N, int H,
                                                       int W, int C, int ldx, int P, int Q,
                                                       int ldy, int kh, int kw, int sh, int sw,
                                                       int ph, int pw, int is_max, int incl_pad,
                                                       uint8_t* __restrict__ amax) {
  // 32-bit index math (the host checks N*P*Q*C/8 < 2^31): 64-bit div/mod is emulated
  const unsigned CV = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int cv = (int)(idx % CV);
    const unsigned pix = idx / CV;
    const int q = (int)(pix % (unsigned)Q);
    const unsigned t = pix / (unsigned)Q;
    const int p = (int)(t % (unsigned)P);
    const int n = (int)(t / (unsigned)P);
    int h0 = p * sh - ph, w0 = q * sw - pw;
    float acc[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] = is_max ? -INFINITY : 0.f;
      arg[e] = 255;
    }
    int cnt = 0;
    for (int r = 0; r < kh; ++r) {
      int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < kw; ++s) {
        int w = w0 + s;
        if (w < 0 || w >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(x + ((size_t)(n * H + h) * W + w) * ldx + cv * 8), f);
        ++cnt;
        if (is_max) {
          const int pos = r * kw + s;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (f[e] > acc[e]) {  // strict: the FIRST maximal element keeps the gradient
              acc[e] = f[e];
              arg[e] = pos;
            }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += f[e];
        }
      }
    }
    if (!is_max) {
      float div = incl_pad ? (float)(kh * kw) : (float)(cnt > 0 ? cnt : 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] /= div;
    }
    *reinterpret_cast<u32x4*>(y + ((size_t)(n * P + p) * Q + q) * ldy + cv * 8) = pack8(acc);
    if (is_max && amax != nullptr) {
      u32x2 a;
      a[0] = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
      a[1] = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
      *reinterpret_cast<u32x2*>(amax + ((size_t)(n * P + p) * Q + q) * C + cv * 8) = a;
    }
  }
}

__global__ __launch_bounds__(256) void pool_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ y, uint16_t* __restrict__ dx, int N, int H, int W, int C, int ldx,
    int P, int Q, int ldy, int kh, int kw, int sh, int sw, int ph, int pw, int is_max,
    int incl_pad, int accum, const uint8_t* __restrict__ amax) {
  const unsigned CV = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * H * W * CV;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int cv = (int)(idx % CV);
    const unsigned pix = idx / CV;
    const int w = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    float xv[8], g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
    if (is_max)
      unpack8(*reinterpret_cast<const u32x4*>(x + ((size_t)(n * H + h) * W + w) * ldx + cv * 8), xv);
    // windows p with p*sh - ph <= h <= p*sh - ph + kh - 1
    int p_lo = (h + ph - kh + sh) / sh;  // ceil((h+ph-kh+1)/sh) for non-negative numerators
    if (h + ph - kh + 1 <= 0) p_lo = 0;
    int p_hi = (h + ph) / sh;
    if (p_hi > P - 1) p_hi = P - 1;
    int q_lo = (w + pw - kw + sw) / sw;
    if (w + pw - kw + 1 <= 0) q_lo = 0;
    int q_hi = (w + pw) / sw;
    if (q_hi > Q - 1) q_hi = Q - 1;
    for (int p = p_lo; p <= p_hi; ++p) {
      for (int q = q_lo; q <= q_hi; ++q) {
        float d[8];
        unpack8(*reinterpret_cast<const u32x4*>(dy + ((size_t)(n * P + p) * Q + q) * ldy + cv * 8), d);
        int h0 = p * sh - ph, w0 = q * sw - pw;
        if (is_max && amax != nullptr) {
          const int mine = (h - h0) * kw + (w - w0);
          u32x2 a = *reinterpret_cast<const u32x2*>(amax + ((size_t)(n * P + p) * Q + q) * C + cv * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if ((int)((a[e >> 2] >> (8 * (e & 3))) & 0xff) == mine) g[e] += d[e];
        } else if (is_max) {
          float yv[8];
          unpack8(*reinterpret_cast<const u32x4*>(y + ((size_t)(n * P + p) * Q + q) * ldy + cv * 8), yv);
          // first position (row-major within the window) holding the max, per channel
          int mine = (h - h0) * kw + (w - w0);
          int first[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) first[e] = 1 << 30;
          for (int r = 0; r < kh; ++r) {
            int hh = h0 + r;
            if (hh < 0 || hh >= H) continue;
            for (int s = 0; s < kw; ++s) {
              int ww = w0 + s;
              if (ww < 0 || ww >= W) continue;
              int pos = r * kw + s;
              if (pos > mine) break;
              float f[8];
              unpack8(*reinterpret_cast<const u32x4*>(x + ((size_t)(n * H + hh) * W + ww) * ldx + cv * 8), f);
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (f[e] == yv[e] && pos < first[e]) first[e] = pos;
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (first[e] == mine) g[e] += d[e];
        } else {
          int cnt;
          if (incl_pad) {
            cnt = kh * kw;
          } else {
            int hs = h0 < 0 ? 0 : h0, he = h0 + kh > H ? H : h0 + kh;
            int ws = w0 < 0 ? 0 : w0, we = w0 + kw > W ? W : w0 + kw;
            cnt = (he - hs) * (we - ws);
          }
          float inv = 1.f / (float)cnt;
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] += d[e] * inv;
        }
      }
    }
    uint16_t* dp = dx + ((size_t)(n * H + h) * W + w) * ldx + cv * 8;
    if (accum) {
      float o[8];
      unpack8(*reinterpret_cast<const u32x4*>(dp), o);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += o[e];
    }
    *reinterpret_cast<u32x4*>(dp) = pack8(g);
  }
}

// 3x3 stride-1 pools (Inception's 3x3/1 'SAME' average-pool branches and the 3x3/1 max pool of
// the last module): all nine window loads are issued before any is used -- raw buffer loads
// whose out-of-range offset returns zero stand in for the halo -- instead of one dependent
// load per loop trip of the generic kernel.
template <bool IS_MAX>
__global__ __launch_bounds__(256) void pool3s1_fwd_kernel(const uint16_t* __restrict__ x, uint32_t x_bytes,
                                                          uint16_t* __restrict__ y, int N, int H, int W, int C,
                                                          int ldx, int P, int Q, int ldy, int ph, int pw,
                                                          int incl_pad, uint8_t* __restrict__ amax) {
  const unsigned CV = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, x_bytes);
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int cv = (int)(idx % CV);
    const unsigned pix = idx / CV;
    const int q = (int)(pix % (unsigned)Q);
    const unsigned t = pix / (unsigned)Q;
    const int p = (int)(t % (unsigned)P);
    const int n = (int)(t / (unsigned)P);
    const int h0 = p - ph, w0 = q - pw;
    u32x4 v[9];
    bool ok[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int h = h0 + r, w = w0 + s2;
        const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        ok[r * 3 + s2] = in;
        v[r * 3 + s2] = buf_load16(xr, in ? (uint32_t)(((n * H + h) * W + w) * ldx + cv * 8) * 2u : HCB_OOB);
      }
    float acc[8];
    if constexpr (IS_MAX) {
      int arg[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[e] = -INFINITY;
        arg[e] = 255;
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (!ok[k]) continue;
        float f[8];
        unpack8(v[k], f);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (f[e] > acc[e]) {  // strict: the FIRST maximal element keeps the gradient
            acc[e] = f[e];
            arg[e] = k;
          }
      }
      if (amax != nullptr) {
        u32x2 a;
        a[0] = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
        a[1] = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
        *reinterpret_cast<u32x2*>(amax + ((size_t)(n * P + p) * Q + q) * C + cv * 8) = a;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {  // out-of-range taps loaded zeros
        float f[8];
        unpack8(v[k], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
      }
      const int vr = ((unsigned)h0 < (unsigned)H) + ((unsigned)(h0 + 1) < (unsigned)H) +
                     ((unsigned)(h0 + 2) < (unsigned)H);
      const int vc = ((unsigned)w0 < (unsigned)W) + ((unsigned)(w0 + 1) < (unsigned)W) + ((unsigned)(w0 + 2) < (unsigned)W);
      const float inv = 1.f / (float)(incl_pad ? 9 : (vr * vc > 0 ? vr * vc : 1));
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= inv;
    }
    *reinterpret_cast<u32x4*>(y + ((size_t)(n * P + p) * Q + q) * ldy + cv * 8) = pack8(acc);
  }
}

// Average-pool 3x3/1 backward as a gather: the (up to) nine windows covering a pixel, each
// scaled by 1 / (its valid-tap count), all loads in flight together. T: the 16-bit activation
// type, or fp32 (the fp32 path's Inception pool branches: dy / dx are fp32 gradients).
template <typename T = uint16_t>
__global__ __launch_bounds__(256) void avgpool3s1_bwd_kernel(const T* __restrict__ dy, uint32_t dy_bytes,
                                                             T* __restrict__ dx, int N, int H, int W, int C,
                                                             int ldx, int P, int Q, int ldy, int ph, int pw,
                                                             int incl_pad, int accum) {
  const unsigned CV = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * H * W * CV;
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(dy, dy_bytes);
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int cv = (int)(idx % CV);
    const unsigned pix = idx / CV;
    const int w = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    Act8<T> d[9];
    float sc[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int p = h + ph - i, q = w + pw - j;  // windows p - ph <= h <= p - ph + 2
        const bool in = (unsigned)p < (unsigned)P && (unsigned)q < (unsigned)Q;
        d[i * 3 + j].load(dr, in ? (uint32_t)(((n * P + p) * Q + q) * ldy + cv * 8) * Act8<T>::ESZ : HCB_OOB);
        const int hs = p - ph, ws = q - pw;
        const int vr = ((unsigned)hs < (unsigned)H) + ((unsigned)(hs + 1) < (unsigned)H) + ((unsigned)(hs + 2) < (unsigned)H);
        const int vc = ((unsigned)ws < (unsigned)W) + ((unsigned)(ws + 1) < (unsigned)W) + ((unsigned)(ws + 2) < (unsigned)W);
        sc[i * 3 + j] = in ? 1.f / (float)(incl_pad ? 9 : (vr * vc > 0 ? vr * vc : 1)) : 0.f;
      }
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float f[8];
      d[k].to_f(f);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += f[e] * sc[k];
    }
    T* dp = dx + ((size_t)(n * H + h) * W + w) * ldx + cv * 8;
    if (accum) {
      float o[8];
      Act8<T> ov;
      ov.load(dp);
      ov.to_f(o);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += o[e];
    }
    Act8<T>::store(dp, g);
  }
}

// fp32 path (--compute_dtype fp32; Inception-v3's 3x3/2 max-pool reductions and 3x3/1 average /
// max pool branches): k x k pool on bf16 PLANES -- x and y are [3][N][H|P][W|Q][ld] with plane
// strides xps / yps (elements), each window value the exact fp32 hi + mid + lo. The maximum is
// split back into planes (the split is canonical: the winning element's own planes, bit for bit);
// the average is summed and divided in fp32, then split. One thread per output pixel x 8 channels,
// the window's 3 plane loads per tap issued together.
__global__ __launch_bounds__(256) void pool_fwd_p3_kernel(const uint16_t* __restrict__ x, int64_t xps,
                                                          uint16_t* __restrict__ y, int64_t yps, int N, int H, int W,
                                                          int C, int ldx, int P, int Q, int ldy, int kh, int kw,
                                                          int sh, int sw, int ph, int pw, int is_max, int incl_pad,
                                                          uint8_t* __restrict__ amax) {
  const unsigned CV = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int cv = (int)(idx % CV);
    const unsigned pix = idx / CV;
    const int q = (int)(pix % (unsigned)Q);
    const unsigned t = pix / (unsigned)Q;
    const int p = (int)(t % (unsigned)P);
    const int n = (int)(t / (unsigned)P);
    const int h0 = p * sh - ph, w0 = q * sw - pw;
    float acc[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] = is_max ? -INFINITY : 0.f;
      arg[e] = 255;
    }
    int cnt = 0;
    for (int r = 0; r < kh; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int s2 = 0; s2 < kw; ++s2) {
        const int w = w0 + s2;
        if (w < 0 || w >= W) continue;
        const uint16_t* src = x + ((size_t)(n * H + h) * W + w) * ldx + cv * 8;
        float f[8];
        merge_p3(*reinterpret_cast<const u32x4*>(src), *reinterpret_cast<const u32x4*>(src + xps),
                 *reinterpret_cast<const u32x4*>(src + 2 * xps), f);
        ++cnt;
        if (is_max) {
          const int pos = r * kw + s2;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (f[e] > acc[e]) {  // strict: the FIRST maximal element keeps the gradient
              acc[e] = f[e];
              arg[e] = pos;
            }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += f[e];
        }
      }
    }
    if (!is_max) {
      const float div = incl_pad ? (float)(kh * kw) : (float)(cnt > 0 ? cnt : 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] /= div;
    }
    store_p3(y + ((size_t)(n * P + p) * Q + q) * ldy + cv * 8, yps, acc);
    if (is_max && amax != nullptr) {
      u32x2 a;
      a[0] = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
      a[1] = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
      *reinterpret_cast<u32x2*>(amax + ((size_t)(n * P + p) * Q + q) * C + cv * 8) = a;
    }
  }
}

// Max-pool backward from the recorded argmax when at most NPW x NPW windows cover a pixel
// (ceil(k/s) <= NPW; ResNet's 3x3/2: 2x2): the candidate windows are unrolled so all their dy /
// argmax loads are in flight together instead of one loop trip at a time. Grid: x over the
// (w, channel vector) pairs of one input row, y = n * H + h, so the row / image indices are
// wave-uniform (no per-thread divisions: the earlier flat index cost four runtime-divisor
// divides per 8-channel item) and offsets are 32-bit.
template <int NPW, typename T = uint16_t>
__global__ __launch_bounds__(256) void maxpool_bwd_amax_kernel(
    const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int ldx, int P, int Q,
    int ldy, int kw, int sh, int sw, int ph, int pw, int accum, const uint8_t* __restrict__ amax, int cv_shift) {
  const int CV = C >> 3;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= W * CV) return;
  const int w = cv_shift >= 0 ? idx >> cv_shift : idx / CV;
  const int cv = idx - w * CV;
  const int t = blockIdx.y;  // n * H + h (uniform)
  const int n = t / H, h = t - n * H;
  // windows p with p*sh - ph <= h, i.e. p <= (h+ph)/sh, and h < p*sh - ph + kh
  const int p_hi = (h + ph) / sh, q_hi = (w + pw) / sw;
  Act8<T> d[NPW][NPW];
  u32x2 a[NPW][NPW];
  bool ok[NPW][NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int p = p_hi - i;
    const bool pok = p >= 0 && p < P && h - (p * sh - ph) < kw;  // uniform
    const uint32_t prow = (uint32_t)(n * P + (pok ? p : 0)) * (uint32_t)Q;
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const int q = q_hi - j;
      ok[i][j] = pok && q >= 0 && q < Q && w - (q * sw - pw) < kw;  // kh == kw
      const uint32_t o = prow + (uint32_t)(ok[i][j] ? q : 0);
      d[i][j].load(dy + o * (uint32_t)ldy + cv * 8);
      a[i][j] = *reinterpret_cast<const u32x2*>(amax + o * (uint32_t)C + cv * 8);
    }
  }
  float g[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
  for (int i = 0; i < NPW; ++i)
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const int p = p_hi - i, q = q_hi - j;
      const int mine = (h - (p * sh - ph)) * kw + (w - (q * sw - pw));
      if (!ok[i][j]) continue;
      float f[8];
      d[i][j].to_f(f);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if ((int)((a[i][j][e >> 2] >> (8 * (e & 3))) & 0xff) == mine) g[e] += f[e];
    }
  T* dp = dx + ((uint32_t)t * (uint32_t)W + (uint32_t)w) * (uint32_t)ldx + cv * 8;
  if (accum) {
    float o[8];
    Act8<T> ov;
    ov.load(dp);
    ov.to_f(o);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] += o[e];
  }
  Act8<T>::store(dp, g);
}

// The ResNet stem pool (3x3, stride 2, top / left pad 0 or 1 -- TF 'SAME' pads 0 before, 1 after --
// even H / W): one thread per 2x2 input block (rows 2a, 2a+1; cols 2b, 2b+1) x 8 channels. The
// block meets exactly the windows p in {a-1+ph, a+ph}, q in {b-1+pw, b+pw}, so 4 window loads
// (dy + argmax) serve 4 pixels -- the per-pixel kernel above loads 4 windows for EVERY pixel,
// ~4x the L2 -> CU traffic for the same result.
template <typename T = uint16_t>
__global__ __launch_bounds__(256) void maxpool_bwd_amax_s2_kernel(
    const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
    int ph, int pw, int accum, const uint8_t* __restrict__ amax, int cv_shift) {
  const int CV = C >> 3, W2 = W >> 1, H2 = H >> 1;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= W2 * CV) return;
  const int b = cv_shift >= 0 ? idx >> cv_shift : idx / CV;
  const int cv = idx - b * CV;
  const int t = blockIdx.y;  // n * H2 + a (uniform)
  const int n = t / H2, a = t - n * H2;
  Act8<T> d[2][2];
  u32x2 am[2][2];
  bool ok[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = a - 1 + ph + i, q = b - 1 + pw + j;
      ok[i][j] = p >= 0 && p < P && q >= 0 && q < Q;
      const uint32_t o = (uint32_t)(n * P + (ok[i][j] ? p : 0)) * (uint32_t)Q + (uint32_t)(ok[i][j] ? q : 0);
      d[i][j].load(dy + o * (uint32_t)ldy + cv * 8);
      am[i][j] = *reinterpret_cast<const u32x2*>(amax + o * (uint32_t)C + cv * 8);
    }
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int h = 2 * a + dh, w = 2 * b + dw;
      float g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = 0.f;
      // higher window first, the per-pixel kernels' summation order (bitwise-equal results)
#pragma unroll
      for (int i = 1; i >= 0; --i)
#pragma unroll
        for (int j = 1; j >= 0; --j) {
          // position in window (p, q), which starts at row 2p - ph, column 2q - pw
          const int rh = h - (2 * (a - 1 + ph + i) - ph), rw = w - (2 * (b - 1 + pw + j) - pw);
          if (!ok[i][j] || rh < 0 || rh > 2 || rw < 0 || rw > 2) continue;
          const int mine = rh * 3 + rw;
          float f[8];
          d[i][j].to_f(f);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if ((int)((am[i][j][e >> 2] >> (8 * (e & 3))) & 0xff) == mine) g[e] += f[e];
        }
      T* dp = dx + ((uint32_t)(n * H + h) * (uint32_t)W + (uint32_t)w) * (uint32_t)ldx + cv * 8;
      if (accum) {
        float o[8];
        Act8<T> ov;
        ov.load(dp);
        ov.to_f(o);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] += o[e];
      }
      Act8<T>::store(dp, g);
    }
}

// global average pool [N][HW][C] -> [N][C]
template <typename T = uint16_t>
__global__ __launch_bounds__(256) void gap_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int HW,
                                                      int C) {
  const int CV = C >> 3;
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * CV) return;
  int n = idx / CV, cv = idx % CV;
  float acc[8] = {0};
  for (int i = 0; i < HW; ++i) {
    float f[8];
    Act8<T> v;
    v.load(x + ((size_t)n * HW + i) * C + cv * 8);
    v.to_f(f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += f[e];
  }
  float inv = 1.f / (float)HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] *= inv;
  Act8<T>::store(y + (size_t)n * C + cv * 8, acc);
}

template <typename T = uint16_t>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW,
                                                      int C) {
  const int CV = C >> 3;
  const long total = (long)N * HW * CV;
  float inv = 1.f / (float)HW;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    int cv = (int)(idx % CV);
    long pix = idx / CV;
    int n = (int)(pix / HW);
    float f[8];
    Act8<T> v;
    v.load(dy + (size_t)n * C + cv * 8);
    v.to_f(f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= inv;
    Act8<T>::store(dx + (size_t)pix * C + cv * 8, f);
  }
}

static int ew_grid(long total) {
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

void launch_pool_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int P, int Q,
                     int ldy, int kh, int kw, int sh, int sw, int ph, int pw, int is_max,
                     int count_include_pad, void* idx, hipStream_t st) {
  long total = (long)N * P * Q * (C / 8);
  const long xbytes = (long)N * H * W * ldx * 2;
  if (kh == 3 && kw == 3 && sh == 1 && sw == 1 && xbytes < 0x7fffffffL) {
    if (is_max)
      hipLaunchKernelGGL(pool3s1_fwd_kernel<true>, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)x,
                         (uint32_t)xbytes, (uint16_t*)y, N, H, W, C, ldx, P, Q, ldy, ph, pw, count_include_pad,
                         (uint8_t*)idx);
    else
      hipLaunchKernelGGL(pool3s1_fwd_kernel<false>, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)x,
                         (uint32_t)xbytes, (uint16_t*)y, N, H, W, C, ldx, P, Q, ldy, ph, pw, count_include_pad,
                         (uint8_t*)idx);
    return;
  }
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)x,
                     (uint16_t*)y, N, H, W, C, ldx, P, Q, ldy, kh, kw, sh, sw, ph, pw, is_max,
                     count_include_pad, (uint8_t*)idx);
}

void launch_pool_bwd(const void* dy, const void* x, const void* y, void* dx, int N, int H, int W,
                     int C, int ldx, int P, int Q, int ldy, int kh, int kw, int sh, int sw, int ph,
                     int pw, int is_max, int count_include_pad, int accum, const void* idx,
                     hipStream_t st, bool f32) {
  long total = (long)N * H * W * (C / 8);
  // argmax gather: 2-D grid (input row, w x channel vector); 32-bit offsets
  const bool amax_ok = is_max && idx != nullptr && kh == kw && sh == sw && (long)N * H <= 65535 &&
                       (long)N * H * W * ldx < (1l << 31) && (long)N * P * Q * (ldy > C ? ldy : C) < (1l << 31);
  const int cvn = C / 8;
  const int cv_shift = (cvn & (cvn - 1)) == 0 ? __builtin_ctz((unsigned)cvn) : -1;
  const dim3 agrid((unsigned)((W * cvn + 255) / 256), (unsigned)(N * H));
  if (amax_ok && kh == 3 && sh == 2 && ph >= 0 && ph <= 1 && pw >= 0 && pw <= 1 && H % 2 == 0 && W % 2 == 0) {
    const dim3 g2((unsigned)((W / 2 * cvn + 255) / 256), (unsigned)(N * H / 2));
    if (f32)
      hipLaunchKernelGGL((maxpool_bwd_amax_s2_kernel<float>), g2, dim3(256), 0, st, (const float*)dy, (float*)dx, N, H,
                         W, C, ldx, P, Q, ldy, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    else
      hipLaunchKernelGGL((maxpool_bwd_amax_s2_kernel<uint16_t>), g2, dim3(256), 0, st, (const uint16_t*)dy,
                         (uint16_t*)dx, N, H, W, C, ldx, P, Q, ldy, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    return;
  }
  if (f32) {  // fp32 path: the argmax-gather max pool, the 3x3/1 average pool
    if (!is_max && kh == 3 && kw == 3 && sh == 1 && sw == 1) {
      const long b32 = (long)N * P * Q * ldy * 4;
      if (b32 >= 0x7fffffffL) return;  // rejected on the host
      hipLaunchKernelGGL(avgpool3s1_bwd_kernel<float>, dim3(ew_grid(total)), dim3(256), 0, st, (const float*)dy,
                         (uint32_t)b32, (float*)dx, N, H, W, C, ldx, P, Q, ldy, ph, pw, count_include_pad, accum);
      return;
    }
    if (!amax_ok || (kh + sh - 1) / sh > 3) return;  // rejected on the host (bindings.cpp)
    if ((kh + sh - 1) / sh <= 2)
      hipLaunchKernelGGL((maxpool_bwd_amax_kernel<2, float>), agrid, dim3(256), 0, st, (const float*)dy, (float*)dx, N,
                         H, W, C, ldx, P, Q, ldy, kw, sh, sw, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    else
      hipLaunchKernelGGL((maxpool_bwd_amax_kernel<3, float>), agrid, dim3(256), 0, st, (const float*)dy, (float*)dx, N,
                         H, W, C, ldx, P, Q, ldy, kw, sh, sw, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    return;
  }
  if (amax_ok && (kh + sh - 1) / sh <= 2) {
    hipLaunchKernelGGL(maxpool_bwd_amax_kernel<2>, agrid, dim3(256), 0, st, (const uint16_t*)dy, (uint16_t*)dx, N, H,
                       W, C, ldx, P, Q, ldy, kw, sh, sw, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    return;
  }
  if (amax_ok && (kh + sh - 1) / sh <= 3) {
    hipLaunchKernelGGL(maxpool_bwd_amax_kernel<3>, agrid, dim3(256), 0, st, (const uint16_t*)dy, (uint16_t*)dx, N, H,
                       W, C, ldx, P, Q, ldy, kw, sh, sw, ph, pw, accum, (const uint8_t*)idx, cv_shift);
    return;
  }
  const long dybytes = (long)N * P * Q * ldy * 2;
  if (!is_max && kh == 3 && kw == 3 && sh == 1 && sw == 1 && dybytes < 0x7fffffffL) {
    hipLaunchKernelGGL(avgpool3s1_bwd_kernel<uint16_t>, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)dy,
                       (uint32_t)dybytes, (uint16_t*)dx, N, H, W, C, ldx, P, Q, ldy, ph, pw, count_include_pad, accum);
    return;
  }
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)dy,
                     (const uint16_t*)x, (const uint16_t*)y, (uint16_t*)dx, N, H, W, C, ldx, P, Q,
                     ldy, kh, kw, sh, sw, ph, pw, is_max, count_include_pad, accum,
                     (const uint8_t*)idx);
}

void launch_pool_fwd_p3(const uint16_t* x, int64_t xps, uint16_t* y, int64_t yps, int N, int H, int W, int C, int ldx,
                        int P, int Q, int ldy, int kh, int kw, int sh, int sw, int ph, int pw, int is_max,
                        int count_include_pad, void* idx, hipStream_t st) {
  const long total = (long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(pool_fwd_p3_kernel, dim3(ew_grid(total)), dim3(256), 0, st, x, xps, y, yps, N, H, W, C, ldx, P,
                     Q, ldy, kh, kw, sh, sw, ph, pw, is_max, count_include_pad, (uint8_t*)idx);
}

void launch_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st, bool f32) {
  int total = N * (C / 8);
  if (f32)
    hipLaunchKernelGGL(gap_fwd_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, st, (const float*)x, (float*)y,
                       N, HW, C);
  else
    hipLaunchKernelGGL(gap_fwd_kernel<uint16_t>, dim3((total + 255) / 256), dim3(256), 0, st, (const uint16_t*)x,
                       (uint16_t*)y, N, HW, C);
}

void launch_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st, bool f32) {
  long total = (long)N * HW * (C / 8);
  if (f32)
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(ew_grid(total)), dim3(256), 0, st, (const float*)dy, (float*)dx, N,
                       HW, C);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<uint16_t>, dim3(ew_grid(total)), dim3(256), 0, st, (const uint16_t*)dy,
                       (uint16_t*)dx, N, HW, C);
}

}  // namespace hcb
