// ReLU backward fused with the bias gradient.
//
// For a Linear(+ReLU) layer the backward needs g = dy * (y > 0) twice (weight and input
// gradients) and db = sum over the batch of g. One pass reads dy and y once, writes g and
// per-row-slice column partial sums; a second tiny kernel folds the partials into db. The GEMMs
// then consume g unmasked, which keeps their LDS-DMA staging free of extra operands.
#include "common.h"
#include "kernels.h"

namespace tdp {
namespace {

// block: 64 column groups (x4 when VEC) x 4 row groups; grid.y slices the rows
template <bool VEC>
__global__ __launch_bounds__(256) void relu_bias_part_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ y,
                                                             int B, int N, long ld,
                                                             float* __restrict__ g,
                                                             float* __restrict__ part,
                                                             int rows_per) {
  constexpr int W = VEC ? 4 : 1;
  __shared__ float red[4][64 * W];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = (blockIdx.x * 64 + lane) * W;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(B, r0 + rows_per);
  float s[W];
#pragma unroll
  for (int e = 0; e < W; ++e) s[e] = 0.f;
  if (col < N) {
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += 4) {
      const long off = (long)r * ld + col;
      if (VEC) {
        f32x4 d = *reinterpret_cast<const f32x4*>(dy + off);
        if (y) {
          const f32x4 m = *reinterpret_cast<const f32x4*>(y + off);
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
          *reinterpret_cast<f32x4*>(g + (long)r * N + col) = d;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += d[e];
      } else {
        float d = dy[off];
        if (y) {
          d = y[off] > 0.f ? d : 0.f;
          g[(long)r * N + col] = d;
        }
        s[0] += d;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < W; ++e) red[rg][lane * W + e] = s[e];
  __syncthreads();
  if (rg == 0 && col < N && part) {
#pragma unroll
    for (int e = 0; e < W; ++e)
      part[(long)blockIdx.y * N + col + e] =
          red[0][lane * W + e] + red[1][lane * W + e] + red[2][lane * W + e] +
          red[3][lane * W + e];
  }
}

__global__ void bias_final_kernel(const float* __restrict__ part, int slices, int N,
                                  float* __restrict__ db, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float t = 0.f;
  for (int z = 0; z < slices; ++z) t += part[(long)z * N + c];
  db[c] = (beta != 0.f ? beta * db[c] : 0.f) + t;
}

}  // namespace

// `part` is carved from `g`'s tail when the caller provides db; see bindings (workspace).
void relu_bias_bwd_ws(const float* dy, const float* y, int B, int N, long ld, float* g,
                      float* db, float beta_db, float* part, int slices, hipStream_t s) {
  const bool vec = (N % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)dy & 15) == 0) &&
                   (y == nullptr || ((uintptr_t)y & 15) == 0) && (((uintptr_t)g & 15) == 0);
  const int rows_per = (B + slices - 1) / slices;
  const int cols = vec ? N / 4 : N;
  dim3 grid((cols + 63) / 64, slices);
  if (vec)
    hipLaunchKernelGGL(relu_bias_part_kernel<true>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per);
  else
    hipLaunchKernelGGL(relu_bias_part_kernel<false>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per);
  if (db)
    hipLaunchKernelGGL(bias_final_kernel, dim3((N + 255) / 256), dim3(256), 0, s, part, slices,
                       N, db, beta_db);
}

int relu_bias_slices(int B, int N, int num_cus) {
  const int col_blocks = ((N % 4 == 0) ? N / 4 : N) / 64 + 1;
  int sl = (2 * num_cus + col_blocks - 1) / col_blocks;
  const int cap = (B + 15) / 16;  // >= 16 rows per slice
  if (sl > cap) sl = cap;
  return sl < 1 ? 1 : sl;
}

}  // namespace tdp
