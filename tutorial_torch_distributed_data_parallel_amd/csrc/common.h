// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this package.
//
// Every kernel in csrc/ is written for a 64-lane wavefront and launched on the caller's HIP stream
// (the PyTorch current stream, or the reducer's comm stream); none of them allocate or synchronise,
// so all of them are safe to capture into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdp {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}

// Round-to-nearest-even f32 -> bf16 (NaN-preserving: a NaN input keeps a quiet-NaN payload).
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Division by a runtime-constant divisor as multiply-high + add + shift (no integer divide in
// kernel loops); exact for numerators < 2^31.
struct FastDiv {
  uint32_t d, m, s;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << s) - d)) / d + 1);
  if (d == 1) { f.m = 0; f.s = 0; }
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

}  // namespace tdp
