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

// block: CGB column groups (x4 when VEC) x 256/CGB row groups; grid.y slices the rows. CGB
// follows N (16 groups for a 64-channel conv output) so no lane idles on narrow outputs (a fixed
// 64-group block left 3/4 of the lanes of AlexNet's 64-channel layers idle).
template <bool VEC>
__global__ __launch_bounds__(256) void relu_bias_part_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ y,
                                                             int B, int N, long ld,
                                                             float* __restrict__ g,
                                                             float* __restrict__ part,
                                                             int rows_per, int cgb) {
  constexpr int W = VEC ? 4 : 1;
  __shared__ f32x4 red[256];
  const int rgn = 256 / cgb;
  const int cl = threadIdx.x % cgb, rg = threadIdx.x / cgb;
  const int col = (blockIdx.x * cgb + cl) * W;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(B, r0 + rows_per);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < N && rg < rgn) {
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += rgn) {
      const long off = (long)r * ld + col;
      if (VEC) {
        f32x4 d = *reinterpret_cast<const f32x4*>(dy + off);
        if (y) {
          const f32x4 m = *reinterpret_cast<const f32x4*>(y + off);
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
          *reinterpret_cast<f32x4*>(g + (long)r * N + col) = d;
        }
        s += d;
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
  if (!part) return;
  red[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0 && col < N) {
    f32x4 t = red[cl];
    for (int i = 1; i < rgn; ++i) t += red[i * cgb + cl];
#pragma unroll
    for (int e = 0; e < W; ++e) part[(long)blockIdx.y * N + col + e] = t[e];
  }
}

// column groups per block of relu_bias_part_kernel
int relu_bias_cgb(int N) {
  const int cg = (N % 4 == 0) ? N / 4 : N;
  return cg <= 128 ? (cg < 1 ? 1 : cg) : 64;
}

}  // namespace

// `part` is carved from `g`'s tail when the caller provides db; see bindings (workspace).
void relu_bias_bwd_ws(const float* dy, const float* y, int B, int N, long ld, float* g,
                      float* db, float beta_db, float* part, int slices, hipStream_t s) {
  const bool vec = (N % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)dy & 15) == 0) &&
                   (y == nullptr || ((uintptr_t)y & 15) == 0) && (((uintptr_t)g & 15) == 0);
  const int rows_per = (B + slices - 1) / slices;
  const int cols = vec ? N / 4 : N;
  const int cgb = vec ? relu_bias_cgb(N) : (N <= 128 ? N : 64);
  dim3 grid((cols + cgb - 1) / cgb, slices);
  if (vec)
    hipLaunchKernelGGL(relu_bias_part_kernel<true>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per, cgb);
  else
    hipLaunchKernelGGL(relu_bias_part_kernel<false>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per, cgb);
  // db = beta*db + column sums of the partials: the split-axis-parallel split-K combine
  if (db) splitk_reduce(part, slices, 1, N, db, false, N, nullptr, beta_db, false, s);
}

int relu_bias_slices(int B, int N, int num_cus) {
  const int cg = (N % 4 == 0) ? N / 4 : N;
  const int cgb = (N % 4 == 0) ? relu_bias_cgb(N) : (N <= 128 ? N : 64);
  const int col_blocks = (cg + cgb - 1) / cgb;
  int sl = (8 * num_cus + col_blocks - 1) / col_blocks;  // streaming: ~8 workgroups per CU
  const int cap = (B + 15) / 16;  // >= 16 rows per slice
  if (sl > cap) sl = cap;
  return sl < 1 ? 1 : sl;
}

}  // namespace tdp

// ------------------------------------------------------------------ batch gather
// One launch gathers a batch of samples AND their labels by the sampler's indices (the loader's
// two index_selects were two launches per step): workgroup b copies sample idx[b] (F floats,
// float4 when F % 4 == 0) and lane 0 copies its label. Indices are checked on the host side of
// the epoch (DistributedSampler output) and clamped here, so a bad index cannot fault.
namespace tdp {
namespace {
__global__ __launch_bounds__(256) void gather_batch_kernel(const float* __restrict__ x,
                                                           const int64_t* __restrict__ y,
                                                           const int64_t* __restrict__ idx,
                                                           long n, long F, float* __restrict__ xb,
                                                           int64_t* __restrict__ yb) {
  // grid.y splits a row into slices: B = 128 rows alone would leave half of the 256 CUs idle
  const int b = blockIdx.x;
  long i = idx[b];
  i = i < 0 ? 0 : (i >= n ? n - 1 : i);
  const float* src = x + i * F;
  float* dst = xb + (long)b * F;
  const long step = 256L * gridDim.y, k0 = threadIdx.x + 256L * blockIdx.y;
  if ((F & 3) == 0) {
    const long F4 = F >> 2;
    for (long k = k0; k < F4; k += step)
      reinterpret_cast<f32x4*>(dst)[k] = reinterpret_cast<const f32x4*>(src)[k];
  } else {
    for (long k = k0; k < F; k += step) dst[k] = src[k];
  }
  if (threadIdx.x == 0 && blockIdx.y == 0) yb[b] = y[i];
}
}  // namespace

void gather_batch(const float* x, const int64_t* y, const int64_t* idx, long n, long F, int B,
                  float* xb, int64_t* yb, hipStream_t s) {
  if (B <= 0) return;
  const long units = (F & 3) == 0 ? F / 4 : F;  // float4 (or float) moves per row
  const long want = (units + 255) / 256;
  const int slices = (int)(want < 8 ? (want < 1 ? 1 : want) : 8);
  hipLaunchKernelGGL(gather_batch_kernel, dim3(B, slices), dim3(256), 0, s, x, y, idx, n, F, xb,
                     yb);
}
}  // namespace tdp
