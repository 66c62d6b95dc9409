// Exact three-way bf16 split of fp32 values (x = hi + mid + lo, 3 x 8 significand bits): the
// representation the planes GEMM (gemm_planes.hip) reads its activation operand in. Producers
// that write an activation for a skinny Linear emit the three planes next to the fp32 tensor.
// Identical instruction sequence to gemm_f32_fast.hip split3_pair (RNE v_cvt_pk_bf16_f32, scalar
// residual subtractions), so planes are bit-identical to the in-kernel split.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdp {

__device__ __forceinline__ void split3_bits(float x0, float x1, unsigned& h, unsigned& m,
                                            unsigned& l) {
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  typedef __bf16 bf2_ __attribute__((ext_vector_type(2)));
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{x0, x1}, bf2_));
  const float r0 = x0 - __uint_as_float(hu << 16), r1 = x1 - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{r0, r1}, bf2_));
  const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{s0, s1}, bf2_));
}

// four adjacent values -> their planes at o, o + ps, o + 2 ps (8-B stores)
__device__ __forceinline__ void store_planes4(uint16_t* o, long ps, float v0, float v1, float v2,
                                              float v3) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  unsigned h0, m0, l0, h1, m1, l1;
  split3_bits(v0, v1, h0, m0, l0);
  split3_bits(v2, v3, h1, m1, l1);
  *reinterpret_cast<u32x2_*>(o) = u32x2_{h0, h1};
  *reinterpret_cast<u32x2_*>(o + ps) = u32x2_{m0, m1};
  *reinterpret_cast<u32x2_*>(o + 2 * ps) = u32x2_{l0, l1};
}

}  // namespace tdp
