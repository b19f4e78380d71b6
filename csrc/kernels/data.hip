// Real-data preprocessing on the GPU: the resize / flip / normalise / layout half of
// tf_cnn_benchmarks' ImageNet training preprocessing (distorted crop -> resize_bilinear ->
// random_flip_left_right -> scale to [-1, 1]; SURVEY.md §2.2 "preprocessing.py"), for the
// `--data_dir` path the reference runs (/root/reference/benchmark-scripts/
// run-tf-sing-ucx-openmpi.sh:19,80-81).
//
// Host side (csrc/data/tfrecord.cpp + Pillow) reads, decodes and crops; the crops of a batch
// are packed back to back as RGB uint8 in one staging buffer, moved with one H2D copy, and this
// kernel writes the model's NHWC input in place -- 16-bit (the build's activation type) or fp32
// (the fp32 path's input, F32) -- with channels 3..Cpad-1 zero, so every conv operand stays a whole
// number of 16-byte vectors. One thread per output pixel, 16-byte stores; bilinear sampling follows TF1 resize_bilinear (align_corners=False, no half-pixel
// offset): src = dst * in / out.
#include "common.h"
#include "kernels.h"

namespace hcb {

template <bool F32>
__global__ __launch_bounds__(256) void preprocess_images_kernel(const uint8_t* __restrict__ src,
                                                                const int64_t* __restrict__ desc,
                                                                void* __restrict__ out, int S, int Cpad,
                                                                float s0, float s1, float s2, float b0, float b1,
                                                                float b2) {
  const int img = blockIdx.y;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= S * S) return;
  const int64_t off = desc[img * 4 + 0];
  const int h = (int)desc[img * 4 + 1], w = (int)desc[img * 4 + 2], flip = (int)desc[img * 4 + 3];
  const int y = pix / S, xo = pix - y * S;
  const int x = flip ? S - 1 - xo : xo;
  const float fy = (float)y * ((float)h / (float)S), fx = (float)x * ((float)w / (float)S);
  const int y0 = min((int)fy, h - 1), x0 = min((int)fx, w - 1);
  const int y1 = min(y0 + 1, h - 1), x1 = min(x0 + 1, w - 1);
  const float ly = fy - (float)y0, lx = fx - (float)x0;
  const uint8_t* p = src + off;
  float v[8];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float a = p[((size_t)y0 * w + x0) * 3 + c], b = p[((size_t)y0 * w + x1) * 3 + c];
    const float cc = p[((size_t)y1 * w + x0) * 3 + c], d = p[((size_t)y1 * w + x1) * 3 + c];
    const float top = a + (b - a) * lx, bot = cc + (d - cc) * lx;
    v[c] = top + (bot - top) * ly;
  }
  v[0] = v[0] * s0 + b0;
  v[1] = v[1] * s1 + b1;
  v[2] = v[2] * s2 + b2;
#pragma unroll
  for (int c = 3; c < 8; ++c) v[c] = 0.f;
  const size_t base = ((size_t)img * S * S + pix) * Cpad;
  if constexpr (F32) {
    float* o = reinterpret_cast<float*>(out) + base;
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], 0.f);
    for (int c = 4; c < Cpad; c += 4) *reinterpret_cast<float4*>(o + c) = make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    uint16_t* o = reinterpret_cast<uint16_t*>(out) + base;
    *reinterpret_cast<u32x4*>(o) = pack8(v);
    for (int c = 8; c < Cpad; c += 8) *reinterpret_cast<u32x4*>(o + c) = u32x4{0u, 0u, 0u, 0u};
  }
}

void launch_preprocess_images(const uint8_t* src, const int64_t* desc, int B, void* out, int S, int Cpad,
                              const float* scale, const float* bias, bool f32, hipStream_t st) {
  dim3 grid((S * S + 255) / 256, B);
  if (f32)
    hipLaunchKernelGGL(preprocess_images_kernel<true>, grid, dim3(256), 0, st, src, desc, out, S, Cpad, scale[0],
                       scale[1], scale[2], bias[0], bias[1], bias[2]);
  else
    hipLaunchKernelGGL(preprocess_images_kernel<false>, grid, dim3(256), 0, st, src, desc, out, S, Cpad, scale[0],
                       scale[1], scale[2], bias[0], bias[1], bias[2]);
}

}  // namespace hcb
