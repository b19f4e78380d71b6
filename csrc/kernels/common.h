// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this framework.
//
// Everything here is written for wave64 CDNA4: 64-lane wave reductions, bf16 vector
// access in 16-byte units (guide: always vectorize bf16), raw buffer loads whose
// out-of-range offsets return zero (used for the implicit-GEMM padding halo).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

#define HCB_LDS __attribute__((address_space(3)))

// Offset used to force a buffer load out of range (returns 0).
#define HCB_OOB 0x80000000u

// 16-bit activation type of this build of the library: bf16 (default) or, with -DHCB_F16, IEEE
// fp16 (the reference's --use_fp16 precision; the same sources are compiled a second time into
// _hcb_kernels_f16.so with the namespace renamed to hcb16). Activations, GEMM operands and
// 16-bit gradients use act2f / f2act / pack8 / unpack8 / mfma16; explicitly-bf16 data (the
// bf16 wire format of the gradient buckets) keeps bf2f / f2bf.
#ifdef HCB_F16
typedef _Float16 act16x8 __attribute__((ext_vector_type(8)));
#else
typedef __bf16 act16x8 __attribute__((ext_vector_type(8)));
#endif

namespace hcb {

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even f32 -> bf16 (NaN stays NaN through the plain cast path).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<uint16_t*>(&b);
}
#ifdef HCB_F16
__device__ __forceinline__ float act2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ uint16_t f2act(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ f32x4 mfma16(const act16x8& a, const act16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
#else
__device__ __forceinline__ float act2f(uint16_t v) { return bf2f(v); }
__device__ __forceinline__ uint16_t f2act(float f) { return f2bf(f); }
__device__ __forceinline__ f32x4 mfma16(const act16x8& a, const act16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
#endif
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2act(lo) | ((uint32_t)f2act(hi) << 16);
}
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#ifdef HCB_F16
    f[2 * i] = act2f((uint16_t)(v[i] & 0xffffu));
    f[2 * i + 1] = act2f((uint16_t)(v[i] >> 16));
#else
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
#endif
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

// fp32 path (--compute_dtype fp32): 8 fp32 values (two 16-byte loads a, b) split into three
// bf16 terms x = hi + mid + lo (8 + 8 + 8 significant bits: the fp32 value to ~2^-24, where a
// two-term split keeps only ~2^-17 -- measured too coarse: that per-element operand error is
// amplified ~30x by the batch sums of BN backward). The GEMMs then issue the six products
// hi*hi + hi*mid + mid*hi + mid*mid + hi*lo + lo*hi (bf16x6, fp32 accumulation); the dropped
// mid*lo, lo*mid, lo*lo are ~2^-24. Always bf16, whatever the 16-bit type of the library build.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split3_8(const u32x4& a, const u32x4& b, u32x4& hi, u32x4& mid, u32x4& lo) {
  float f[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = __uint_as_float(a[i]);
    f[4 + i] = __uint_as_float(b[i]);
  }
  bf16x8 h, m, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = (__bf16)f[i];
    const float r = f[i] - (float)h[i];  // exact (Sterbenz)
    m[i] = (__bf16)r;
    l[i] = (__bf16)(r - (float)m[i]);
  }
  hi = __builtin_bit_cast(u32x4, h);
  mid = __builtin_bit_cast(u32x4, m);
  lo = __builtin_bit_cast(u32x4, l);
}
// 8 bf16 values (always bf16, whatever the build's 16-bit type) -> fp32
__device__ __forceinline__ void unpack_bf16x8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
// 8 fp32 values stored as their bf16 hi / mid / lo PLANES (the fp32 path's GEMM-operand format:
// plane t of an [rows][ld] tensor at t * plane elements; hi + mid + lo == the fp32 value)
__device__ __forceinline__ void store_p3(uint16_t* p, int64_t plane, const float* f) {
  u32x4 a, b, hi, mid, lo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = __float_as_uint(f[i]);
    b[i] = __float_as_uint(f[4 + i]);
  }
  split3_8(a, b, hi, mid, lo);
  *reinterpret_cast<u32x4*>(p) = hi;
  *reinterpret_cast<u32x4*>(p + plane) = mid;
  *reinterpret_cast<u32x4*>(p + 2 * plane) = lo;
}
// the fp32 value of 8 plane-stored elements (16-byte loads of the three planes)
__device__ __forceinline__ void merge_p3(const u32x4& h, const u32x4& m, const u32x4& l, float* f) {
  float a[8], b[8];
  unpack_bf16x8(h, f);
  unpack_bf16x8(m, a);
  unpack_bf16x8(l, b);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] += a[e] + b[e];
}

__device__ __forceinline__ f32x4 mfma_bf16(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

// A vector of 8 consecutive channels of an activation tensor whose element type T is the 16-bit
// type of the build (uint16_t storage) or fp32 (the --compute_dtype fp32 path): one 16-byte
// access, or two. Byte offsets are element offsets * ESZ; an HCB_OOB offset reads zeros.
template <typename T>
struct Act8;
template <>
struct Act8<uint16_t> {
  static constexpr uint32_t ESZ = 2;
  u32x4 v;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t off) { v = buf_load16(r, off); }
  __device__ __forceinline__ void load(const uint16_t* p) { v = *reinterpret_cast<const u32x4*>(p); }
  __device__ __forceinline__ void to_f(float* f) const { unpack8(v, f); }
  __device__ __forceinline__ void set_f(const float* f) { v = pack8(f); }
  __device__ __forceinline__ static void store(uint16_t* p, const float* f) {
    *reinterpret_cast<u32x4*>(p) = pack8(f);
  }
};
template <>
struct Act8<float> {
  static constexpr uint32_t ESZ = 4;
  u32x4 a, b;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    a = buf_load16(r, off);
    b = buf_load16(r, off + 16u);  // HCB_OOB + 16 stays out of range
  }
  __device__ __forceinline__ void load(const float* p) {
    a = reinterpret_cast<const u32x4*>(p)[0];
    b = reinterpret_cast<const u32x4*>(p)[1];
  }
  __device__ __forceinline__ void to_f(float* f) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i] = __uint_as_float(a[i]);
      f[4 + i] = __uint_as_float(b[i]);
    }
  }
  __device__ __forceinline__ void set_f(const float* f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = __float_as_uint(f[i]);
      b[i] = __float_as_uint(f[4 + i]);
    }
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    reinterpret_cast<f32x4*>(p)[0] = f32x4{f[0], f[1], f[2], f[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{f[4], f[5], f[6], f[7]};
  }
};

// LDS-DMA: 16 bytes per lane from the buffer straight into LDS at (wave-uniform) lds + lane*16.
// Kept in a __device__ helper so the host compilation pass never sees the LDS address-space
// cast (a kernel template body containing it loses its host launch stub).
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (HCB_LDS void*)lds, 16, off, 0, 0, 0);
}
__device__ __forceinline__ int wave_id_uniform() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (MI355X: 8 XCDs, blocks dealt
// round-robin). Consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg < nx) return orig;
  int q = nwg / nx, r = nwg % nx;
  int xcd = orig % nx, idx = orig / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace hcb
