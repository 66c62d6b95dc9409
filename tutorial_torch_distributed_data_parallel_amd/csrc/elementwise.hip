#include <algorithm>
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
                                                             int rows_per, int cgb, float gscale) {
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
          *reinterpret_cast<f32x4*>(g + (long)r * N + col) = d * gscale;
        }
        s += d;
      } else {
        float d = dy[off];
        if (y) {
          d = y[off] > 0.f ? d : 0.f;
          g[(long)r * N + col] = d * gscale;
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
                      float* db, float beta_db, float* part, int slices, hipStream_t s,
                      float gscale) {
  const bool vec = (N % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)dy & 15) == 0) &&
                   (y == nullptr || ((uintptr_t)y & 15) == 0) && (((uintptr_t)g & 15) == 0);
  const int rows_per = (B + slices - 1) / slices;
  const int cols = vec ? N / 4 : N;
  const int cgb = vec ? relu_bias_cgb(N) : (N <= 128 ? N : 64);
  dim3 grid((cols + cgb - 1) / cgb, slices);
  if (vec)
    hipLaunchKernelGGL(relu_bias_part_kernel<true>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per, cgb, gscale);
  else
    hipLaunchKernelGGL(relu_bias_part_kernel<false>, grid, dim3(256), 0, s, dy, y, B, N, ld, g,
                       db ? part : nullptr, rows_per, cgb, gscale);
  // db = beta*db + column sums of the partials: the split-axis-parallel split-K combine
  if (db) splitk_reduce(part, slices, 1, N, db, false, N, nullptr, beta_db, false, s);
}

// y[r][c] = relu?(x[r][c] + b[c]) over [B][N] (N % 4 == 0, 16-B aligned rows): the bias + ReLU
// of an output that no GEMM epilogue produced (the tensor-sharded step's reduce-scattered fc2
// output, parallel/tensor_parallel.py) in one pass
namespace {
__global__ __launch_bounds__(256) void bias_act_rows_kernel(const float* __restrict__ x, long ldx,
                                                            const float* __restrict__ b,
                                                            float* __restrict__ y, long ldy,
                                                            int B, int N4, int relu) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long)B * N4) return;
  const int r = (int)(t / N4), c = (int)(t % N4) * 4;
  f32x4 v = *reinterpret_cast<const f32x4*>(x + (long)r * ldx + c) +
            *reinterpret_cast<const f32x4*>(b + c);
  if (relu) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
  }
  *reinterpret_cast<f32x4*>(y + (long)r * ldy + c) = v;
}
}  // namespace

void bias_act_rows(const float* x, long ldx, const float* b, float* y, long ldy, int B, int N,
                   bool relu, hipStream_t s) {
  const long n = (long)B * (N / 4);
  if (n <= 0) return;
  hipLaunchKernelGGL(bias_act_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x,
                     ldx, b, y, ldy, B, N / 4, relu ? 1 : 0);
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
namespace {
// general form with 32-bit magic-number index math (total < 2^31)
struct Copy4D32 {
  FastDiv d3, d2, d1;
  int sz3, sz2, sz1, ssz[4];
  long ds[4], ss[4];
};

template <bool ACC>
__global__ __launch_bounds__(256) void copy4d32_kernel(const float* __restrict__ src,
                                                       float* __restrict__ dst, Copy4D32 c,
                                                       uint32_t total) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t q3 = fdiv(i, c.d3);
    const int i3 = (int)(i - q3 * (uint32_t)c.sz3);
    const uint32_t q2 = fdiv(q3, c.d2);
    const int i2 = (int)(q3 - q2 * (uint32_t)c.sz2);
    const uint32_t i0 = fdiv(q2, c.d1);
    const int i1 = (int)(q2 - i0 * (uint32_t)c.sz1);
    const bool in = (int)i0 < c.ssz[0] && i1 < c.ssz[1] && i2 < c.ssz[2] && i3 < c.ssz[3];
    const float v = in ? src[i0 * c.ss[0] + i1 * c.ss[1] + i2 * c.ss[2] + i3 * c.ss[3]] : 0.f;
    float* d = dst + i0 * c.ds[0] + i1 * c.ds[1] + i2 * c.ds[2] + i3 * c.ds[3];
    if (ACC) {
      if (in) *d += v;
    } else {
      *d = v;
    }
  }
}

template <bool ACC>
__global__ __launch_bounds__(256) void copy4d_kernel(const float* __restrict__ src,
                                                     float* __restrict__ dst, Copy4D c,
                                                     long total) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    long r = i, idx[4];
#pragma unroll
    for (int d = 3; d >= 0; --d) {
      idx[d] = r % c.dsz[d];
      r /= c.dsz[d];
    }
    long so = 0, doff = 0;
    bool in = true;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      in = in && idx[d] < c.ssz[d];
      so += idx[d] * c.src_stride[d];
      doff += idx[d] * c.dst_stride[d];
    }
    if (ACC) {
      if (in) dst[doff] += src[so];
    } else {
      dst[doff] = in ? src[so] : 0.f;
    }
  }
}
}  // namespace

namespace {
// channels-last fast path of copy4d: dim 1 (channels) has unit stride on both sides, so every
// (n, h, w) row is C contiguous floats -- float4 per lane, 32-bit magic-number index math
struct RowsCopy {
  int C4d, C4s, H, W;
  FastDiv dC4, dW, dH;
  long ds0, ds2, ds3, ss0, ss2, ss3;
};

template <bool ACC>
__global__ __launch_bounds__(256) void copy4d_rows_kernel(const float* __restrict__ src,
                                                          float* __restrict__ dst, RowsCopy c,
                                                          uint32_t total) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t q = fdiv(i, c.dC4);
    const int c4 = (int)(i - q * (uint32_t)c.C4d);
    const uint32_t q2 = fdiv(q, c.dW);
    const int w = (int)(q - q2 * (uint32_t)c.W);
    const uint32_t n = fdiv(q2, c.dH);
    const int h = (int)(q2 - n * (uint32_t)c.H);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (c4 < c.C4s)
      v = *reinterpret_cast<const f32x4*>(src + n * c.ss0 + h * c.ss2 + w * c.ss3 + 4 * c4);
    else if (ACC)
      continue;
    f32x4* d = reinterpret_cast<f32x4*>(dst + n * c.ds0 + h * c.ds2 + w * c.ds3 + 4 * c4);
    if (ACC) v += *d;
    *d = v;
  }
}
}  // namespace

void copy4d(const float* src, float* dst, const Copy4D& c, hipStream_t s) {
  const long total = c.dsz[0] * c.dsz[1] * c.dsz[2] * c.dsz[3];
  if (total <= 0) return;
  if (c.accumulate && c.ssz[0] * c.ssz[1] * c.ssz[2] * c.ssz[3] == 0) return;  // += nothing
  // rows fast path: unit channel stride, 16-B aligned rows, same spatial extent
  const bool empty_src = c.ssz[0] * c.ssz[1] * c.ssz[2] * c.ssz[3] == 0;
  const bool rows = c.dst_stride[1] == 1 && (empty_src || c.src_stride[1] == 1) &&
                    c.dsz[1] % 4 == 0 && (empty_src || c.ssz[1] % 4 == 0) &&
                    (empty_src || (c.ssz[0] >= c.dsz[0] && c.ssz[2] >= c.dsz[2] &&
                                   c.ssz[3] >= c.dsz[3])) &&
                    ((uintptr_t)dst & 15) == 0 && (empty_src || ((uintptr_t)src & 15) == 0) &&
                    c.dst_stride[0] % 4 == 0 && c.dst_stride[2] % 4 == 0 &&
                    c.dst_stride[3] % 4 == 0 &&
                    (empty_src || (c.src_stride[0] % 4 == 0 && c.src_stride[2] % 4 == 0 &&
                                   c.src_stride[3] % 4 == 0)) &&
                    total / 4 < (1L << 31);
  if (rows) {
    RowsCopy r{};
    r.C4d = (int)(c.dsz[1] / 4);
    r.C4s = empty_src ? 0 : (int)(std::min(c.ssz[1], c.dsz[1]) / 4);
    r.H = (int)c.dsz[2];
    r.W = (int)c.dsz[3];
    r.dC4 = make_fastdiv(r.C4d);
    r.dW = make_fastdiv(r.W);
    r.dH = make_fastdiv(r.H);
    r.ds0 = c.dst_stride[0]; r.ds2 = c.dst_stride[2]; r.ds3 = c.dst_stride[3];
    r.ss0 = c.src_stride[0]; r.ss2 = c.src_stride[2]; r.ss3 = c.src_stride[3];
    const uint32_t n4 = (uint32_t)(total / 4);
    long g = ((long)n4 + 255) / 256;
    if (g > 8192) g = 8192;
    if (c.accumulate)
      hipLaunchKernelGGL(copy4d_rows_kernel<true>, dim3((unsigned)g), dim3(256), 0, s, src, dst,
                         r, n4);
    else
      hipLaunchKernelGGL(copy4d_rows_kernel<false>, dim3((unsigned)g), dim3(256), 0, s, src, dst,
                         r, n4);
    return;
  }
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (total < (1L << 31) && c.dsz[1] < (1L << 31) && c.dsz[2] < (1L << 31) &&
      c.dsz[3] < (1L << 31)) {
    Copy4D32 k{};
    k.sz3 = (int)c.dsz[3]; k.sz2 = (int)c.dsz[2]; k.sz1 = (int)c.dsz[1];
    k.d3 = make_fastdiv(k.sz3); k.d2 = make_fastdiv(k.sz2); k.d1 = make_fastdiv(k.sz1);
    for (int d = 0; d < 4; ++d) {
      k.ssz[d] = (int)std::min<long>(c.ssz[d], 1L << 30);
      k.ds[d] = c.dst_stride[d];
      k.ss[d] = c.src_stride[d];
    }
    if (c.accumulate)
      hipLaunchKernelGGL(copy4d32_kernel<true>, dim3((unsigned)g), dim3(256), 0, s, src, dst, k,
                         (uint32_t)total);
    else
      hipLaunchKernelGGL(copy4d32_kernel<false>, dim3((unsigned)g), dim3(256), 0, s, src, dst, k,
                         (uint32_t)total);
    return;
  }
  if (c.accumulate)
    hipLaunchKernelGGL(copy4d_kernel<true>, dim3((unsigned)g), dim3(256), 0, s, src, dst, c,
                       total);
  else
    hipLaunchKernelGGL(copy4d_kernel<false>, dim3((unsigned)g), dim3(256), 0, s, src, dst, c,
                       total);
}

}  // namespace tdp

// ------------------------------------------------------------------ factored gradient staging
// Factored synchronisation of a Linear weight (reducer.h FactorJob): this rank's factors go into
// its slots of the all-gather buffers in one launch -- gdst = alpha * g (alpha = 1/W: the GEMM
// over the gathered factors then yields the AVERAGED gradient) and xdst = x. Both row-contiguous,
// element counts % 4 == 0: float4 grid-stride copies, the first ng/4 units are g's.
namespace tdp {
namespace {
__global__ __launch_bounds__(256) void factor_stage_kernel(const f32x4* __restrict__ g,
                                                           const f32x4* __restrict__ x,
                                                           f32x4* __restrict__ gdst,
                                                           f32x4* __restrict__ xdst, long ng4,
                                                           long nx4, float alpha) {
  const long total = ng4 + nx4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += 256L * gridDim.x) {
    if (i < ng4) gdst[i] = g[i] * alpha;
    else xdst[i - ng4] = x[i - ng4];
  }
}
}  // namespace

void factor_stage(const float* g, const float* x, float* gdst, float* xdst, long ng, long nx,
                  float alpha, hipStream_t s) {
  const long units = (ng + nx) / 4;
  long grid = (units + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(factor_stage_kernel, dim3((unsigned)grid), dim3(256), 0, s,
                     reinterpret_cast<const f32x4*>(g), reinterpret_cast<const f32x4*>(x),
                     reinterpret_cast<f32x4*>(gdst), reinterpret_cast<f32x4*>(xdst), ng / 4,
                     nx / 4, alpha);
}

}  // namespace tdp
