// One cross-entropy row by one lane (a classifier head with few classes): shared by the fused
// loss kernels (csrc/loss.hip ce_fwd) and the fused head + loss kernel (csrc/gemm_skinny.hip
// head_ce), so both produce bit-identical per-row values.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdp {

struct RowOut {
  float lse;
  float loss;
  float correct;
  float valid;
};

// One row handled by one lane (small C) -- logits row in registers-free sequential scan.
__device__ inline RowOut row_serial(const float* x, int C, int64_t y, int ignore_index, float eps) {
  float mx = -INFINITY;
  int arg = 0;
  float sumx = 0.f;
  for (int c = 0; c < C; ++c) {
    const float v = x[c];
    if (v > mx) { mx = v; arg = c; }
    sumx += v;
  }
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += __expf(x[c] - mx);
  RowOut o;
  o.lse = mx + __logf(se);
  const bool valid = (y != ignore_index) && y >= 0 && y < C;
  o.valid = valid ? 1.f : 0.f;
  o.loss = valid ? (o.lse - (1.f - eps) * x[y] - (eps / C) * sumx) : 0.f;
  o.correct = (valid && arg == (int)y) ? 1.f : 0.f;
  return o;
}

}  // namespace tdp
