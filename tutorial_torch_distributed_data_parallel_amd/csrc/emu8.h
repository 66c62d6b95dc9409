// Host API of the large-tile split-bf16 fp32 GEMM (csrc/gemm_emu8.hip): C = A . op(B) (+ beta C),
// A [M][K] fp32 (row stride lda), B [N][K] (b_kcontig) or [K][N] (row stride ldb), K % 32 == 0,
// 16-B aligned A / B rows. 256 x 256 tiles, 8 waves, one workgroup per CU.
#pragma once
#include <hip/hip_runtime.h>

namespace tdp {

struct GemmEmu8Args {
  const float* A = nullptr;
  const float* B = nullptr;
  float* C = nullptr;
  long lda = 0, ldb = 0, ldc = 0;
  bool b_kcontig = true;
  int M = 0, N = 0, K = 0;
  float beta = 0.f;
  const float* bias = nullptr;  // C = relu?(A.B^T + bias + beta C)
  bool relu = false;
};
// The 256 x 256 kernel fills the chip on this shape: one plain-epilogue GEMM with >= 256 output
// tiles in nearly whole waves (gemm_f32's planner prefers it there; profiles/r9/gemm_emu8_r9.md)
bool gemm_emu8_fits(int M, int N, int K, int num_cus);
bool gemm_emu8_ok(const GemmEmu8Args& a);
void gemm_emu8_run(const GemmEmu8Args& a, hipStream_t s);
// variant: 8 waves (wave tile 128 x 64, default) or 4 (128 x 128, one wave per SIMD)
bool gemm_emu8_set_waves(int waves);

}  // namespace tdp
