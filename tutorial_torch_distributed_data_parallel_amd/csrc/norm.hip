// Batch-norm kernels for BatchNorm1d/2d and SyncBatchNorm.
//
// The reference only recommends SyncBatchNorm in prose (REF/README.md:79-81); the north-star
// configs need it (BASELINE.json "toy MLP + SyncBatchNorm", ResNet-50). These kernels are the
// MI355X-native counterparts of the ATen ops torch's SyncBatchNorm autograd function chains
// (TORCH/nn/modules/_functions.py:7-209):
//   batch_norm_stats                   -> bn_moments   (Welford per lane, Chan merge)
//   batch_norm_gather_stats_with_counts-> bn_merge     (count-weighted merge + running stats)
//   batch_norm_elemt                   -> bn_elemt     (+ optional fused ReLU)
//   batch_norm_backward_reduce         -> bn_bwd_reduce (+ dw/db written straight to the grad)
//   batch_norm_backward_elemt          -> bn_bwd_elemt
// x is viewed as [N][C][HW]. For HW == 1 (BatchNorm1d on [N, C]) a workgroup owns 64 adjacent
// channels (one per lane, coalesced across the wave) and its 4 waves split the rows; for HW > 1 a
// workgroup owns one channel (coalesced along HW). Either way the N*HW axis can additionally be
// split over blockIdx.y so that a small-C layer still puts >= 1 workgroup on every CU.
#include "common.h"
#include "kernels.h"

namespace tdp {
namespace {

struct Wf {
  float n, mean, m2;
};

__device__ __forceinline__ Wf wf_merge(Wf a, Wf b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  Wf r;
  r.n = n;
  r.mean = fmaf(d, fb, a.mean);
  r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
  return r;
}

__device__ __forceinline__ void wf_push(Wf& w, float x) {
  w.n += 1.f;
  const float d = x - w.mean;
  w.mean = fmaf(d, 1.f / w.n, w.mean);
  w.m2 = fmaf(d, x - w.mean, w.m2);
}

__device__ __forceinline__ Wf wf_wave(Wf w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Wf t;
    t.n = __shfl_xor(w.n, o, 64);
    t.mean = __shfl_xor(w.mean, o, 64);
    t.m2 = __shfl_xor(w.m2, o, 64);
    w = wf_merge(w, t);
  }
  return w;
}

__device__ __forceinline__ void range_of(long total, int splits, int z, long& b, long& e) {
  const long per = (total + splits - 1) / splits;
  b = (long)z * per;
  e = b + per < total ? b + per : total;
}

// -------------------------------------------------------------------------------- moments
__global__ __launch_bounds__(256) void moments_1d(const float* __restrict__ x, int N, int C,
                                                  int splits, float* __restrict__ ws,
                                                  float* __restrict__ mean,
                                                  float* __restrict__ var) {
  __shared__ Wf sh[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  Wf w{0.f, 0.f, 0.f};
  if (c < C)
    for (long n = b + g; n < e; n += 4) wf_push(w, x[n * C + c]);
  sh[g][lane] = w;
  __syncthreads();
  if (g == 0 && c < C) {
    w = wf_merge(wf_merge(sh[0][lane], sh[1][lane]), wf_merge(sh[2][lane], sh[3][lane]));
    if (splits == 1) {
      mean[c] = w.mean;
      var[c] = w.n > 0.f ? w.m2 / w.n : 0.f;
    } else {
      float* o = ws + (long)blockIdx.y * 3 * C;
      o[c] = w.n; o[C + c] = w.mean; o[2 * C + c] = w.m2;
    }
  }
}

__global__ __launch_bounds__(256) void moments_2d(const float* __restrict__ x, int N, int C,
                                                  int HW, int splits, float* __restrict__ ws,
                                                  float* __restrict__ mean,
                                                  float* __restrict__ var) {
  __shared__ Wf sh[4];
  const int c = blockIdx.x;
  long b, e;
  range_of((long)N * HW, splits, blockIdx.y, b, e);
  Wf w{0.f, 0.f, 0.f};
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const long n = i / HW, hw = i - n * HW;
    wf_push(w, x[(n * C + c) * HW + hw]);
  }
  w = wf_wave(w);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    w = wf_merge(wf_merge(sh[0], sh[1]), wf_merge(sh[2], sh[3]));
    if (splits == 1) {
      mean[c] = w.mean;
      var[c] = w.n > 0.f ? w.m2 / w.n : 0.f;
    } else {
      float* o = ws + (long)blockIdx.y * 3 * C;
      o[c] = w.n; o[C + c] = w.mean; o[2 * C + c] = w.m2;
    }
  }
}

__global__ void moments_final(const float* __restrict__ ws, int C, int splits,
                              float* __restrict__ mean, float* __restrict__ var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  Wf w{0.f, 0.f, 0.f};
  for (int z = 0; z < splits; ++z) {
    const float* o = ws + (long)z * 3 * C;
    w = wf_merge(w, Wf{o[c], o[C + c], o[2 * C + c]});
  }
  mean[c] = w.mean;
  var[c] = w.n > 0.f ? w.m2 / w.n : 0.f;
}

// Rows of `g`: [mean(C) | var(C) | count], stride 2C+1. Zero-count ranks drop out, as in
// batch_norm_gather_stats_with_counts (TORCH/nn/modules/_functions.py:96-115).
__global__ void merge_kernel(const float* __restrict__ g, int R, int C, float eps, float momentum,
                             float* __restrict__ mean, float* __restrict__ invstd,
                             float* __restrict__ rmean, float* __restrict__ rvar) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long stride = 2L * C + 1;
  Wf w{0.f, 0.f, 0.f};
  for (int r = 0; r < R; ++r) {
    const float* row = g + r * stride;
    const float n = row[2 * C];
    if (n <= 0.f) continue;
    w = wf_merge(w, Wf{n, row[c], row[C + c] * n});
  }
  const float v = w.n > 0.f ? w.m2 / w.n : 0.f;
  mean[c] = w.mean;
  invstd[c] = rsqrtf(v + eps);
  if (c == 0) invstd[C] = w.n;  // stats layout [mean | invstd | count]
  if (rmean) {
    const float unbiased = w.n > 1.f ? w.m2 / (w.n - 1.f) : v;
    rmean[c] = fmaf(momentum, w.mean - rmean[c], rmean[c]);
    rvar[c] = fmaf(momentum, unbiased - rvar[c], rvar[c]);
  }
}

// -------------------------------------------------------------------------------- elementwise
__device__ __forceinline__ int chan_of(long i, int C, int HW) {
  return HW == 1 ? (int)(i % C) : (int)((i / HW) % C);
}

__global__ __launch_bounds__(256) void elemt_kernel(const float* __restrict__ x,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ invstd,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ b, long total,
                                                    int C, int HW, int relu, int eval, float eps,
                                                    float* __restrict__ y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = chan_of(i, C, HW);
    const float is = eval ? rsqrtf(invstd[c] + eps) : invstd[c];
    const float sc = is * (w ? w[c] : 1.f);
    float v = fmaf(x[i] - mean[c], sc, b ? b[c] : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    y[i] = v;
  }
}

// -------------------------------------------------------------------------------- backward
__device__ __forceinline__ float masked_dy(const float* dy, const float* yr, long off) {
  const float g = dy[off];
  return (yr && !(yr[off] > 0.f)) ? 0.f : g;
}

__global__ __launch_bounds__(256) void bwd_reduce_1d(const float* __restrict__ dy,
                                                     const float* __restrict__ x,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ yr, int N, int C,
                                                     int splits, float* __restrict__ part) {
  __shared__ float s0[4][64], s1[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  float a = 0.f, m = 0.f;
  if (c < C) {
    const float mu = mean[c];
    for (long n = b + g; n < e; n += 4) {
      const long off = n * C + c;
      const float d = masked_dy(dy, yr, off);
      a += d;
      m = fmaf(d, x[off] - mu, m);
    }
  }
  s0[g][lane] = a;
  s1[g][lane] = m;
  __syncthreads();
  if (g == 0 && c < C) {
    float* o = part + (long)blockIdx.y * 2 * C;
    o[c] = s0[0][lane] + s0[1][lane] + s0[2][lane] + s0[3][lane];
    o[C + c] = s1[0][lane] + s1[1][lane] + s1[2][lane] + s1[3][lane];
  }
}

__global__ __launch_bounds__(256) void bwd_reduce_2d(const float* __restrict__ dy,
                                                     const float* __restrict__ x,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ yr, int N, int C,
                                                     int HW, int splits,
                                                     float* __restrict__ part) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  long b, e;
  range_of((long)N * HW, splits, blockIdx.y, b, e);
  const float mu = mean[c];
  float a = 0.f, m = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const long n = i / HW, hw = i - n * HW;
    const long off = (n * C + c) * HW + hw;
    const float d = masked_dy(dy, yr, off);
    a += d;
    m = fmaf(d, x[off] - mu, m);
  }
  a = block_sum<256>(a, red);
  m = block_sum<256>(m, red);
  if (threadIdx.x == 0) {
    float* o = part + (long)blockIdx.y * 2 * C;
    o[c] = a;
    o[C + c] = m;
  }
}

__global__ void bwd_reduce_final(const float* __restrict__ part, int C, int splits,
                                 const float* __restrict__ invstd, float* __restrict__ sums,
                                 float* __restrict__ dw, float* __restrict__ db, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, m = 0.f;
  for (int z = 0; z < splits; ++z) {
    a += part[(long)z * 2 * C + c];
    m += part[(long)z * 2 * C + C + c];
  }
  sums[c] = a;
  sums[C + c] = m;
  if (dw) dw[c] = (beta != 0.f ? beta * dw[c] : 0.f) + m * invstd[c];
  if (db) db[c] = (beta != 0.f ? beta * db[c] : 0.f) + a;
}

__global__ __launch_bounds__(256) void bwd_elemt_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ w,
    const float* __restrict__ sums, const float* __restrict__ yr, const float* __restrict__ cnt,
    long total, int C, int HW, float* __restrict__ dx) {
  const float inv_count = 1.f / cnt[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = chan_of(i, C, HW);
    const float is = invstd[c];
    const float mdy = sums[c] * inv_count;
    const float mdyx = sums[C + c] * inv_count;
    const float d = masked_dy(dy, yr, i);
    const float v = (d - mdy - (x[i] - mean[c]) * is * is * mdyx) * is * (w ? w[c] : 1.f);
    dx[i] = v;
  }
}

inline int ew_grid(long total) {
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

int bn_splits(int N, int C, int HW, int num_cus) {
  if (HW == 1) {
    const int blocks = (C + 63) / 64;
    int s = (num_cus + blocks - 1) / blocks;
    const int cap = (N + 31) / 32;  // keep >= 32 rows per split
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
  }
  int s = (2 * num_cus + C - 1) / C;
  const long cap = ((long)N * HW + 4095) / 4096;  // keep >= 4K elements per split
  if (s > cap) s = (int)cap;
  return s < 1 ? 1 : s;
}

long bn_ws_floats(int C, int splits) { return 3L * C * (splits > 0 ? splits : 1); }

void bn_moments(const float* x, int N, int C, int HW, int splits, float* ws, float* mean,
                float* var, hipStream_t s) {
  if (HW == 1)
    hipLaunchKernelGGL(moments_1d, dim3((C + 63) / 64, splits), dim3(256), 0, s, x, N, C, splits,
                       ws, mean, var);
  else
    hipLaunchKernelGGL(moments_2d, dim3(C, splits), dim3(256), 0, s, x, N, C, HW, splits, ws,
                       mean, var);
  if (splits > 1)
    hipLaunchKernelGGL(moments_final, dim3((C + 255) / 256), dim3(256), 0, s, ws, C, splits, mean,
                       var);
}

void bn_merge(const float* gathered, int R, int C, float eps, float momentum, float* mean,
              float* invstd, float* running_mean, float* running_var, hipStream_t s) {
  hipLaunchKernelGGL(merge_kernel, dim3((C + 255) / 256), dim3(256), 0, s, gathered, R, C, eps,
                     momentum, mean, invstd, running_mean, running_var);
}

void bn_elemt(const float* x, const float* mean, const float* invstd, const float* w,
              const float* b, int N, int C, int HW, bool relu, float* y, hipStream_t s) {
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, mean, invstd, w, b,
                     total, C, HW, relu ? 1 : 0, 0, 0.f, y);
}

void bn_eval(const float* x, const float* rmean, const float* rvar, const float* w,
             const float* b, int N, int C, int HW, float eps, bool relu, float* y, hipStream_t s) {
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, rmean, rvar, w, b,
                     total, C, HW, relu ? 1 : 0, 1, eps, y);
}

void bn_bwd_reduce(const float* dy, const float* x, const float* mean, const float* invstd,
                   const float* y_relu, int N, int C, int HW, int splits, float* ws, float* sums,
                   float* dw, float* db, float grad_beta, hipStream_t s) {
  // partials always go through ws (2*C*splits floats); the final kernel also writes dw/db
  if (HW == 1)
    hipLaunchKernelGGL(bwd_reduce_1d, dim3((C + 63) / 64, splits), dim3(256), 0, s, dy, x, mean,
                       y_relu, N, C, splits, ws);
  else
    hipLaunchKernelGGL(bwd_reduce_2d, dim3(C, splits), dim3(256), 0, s, dy, x, mean, y_relu, N, C,
                       HW, splits, ws);
  hipLaunchKernelGGL(bwd_reduce_final, dim3((C + 255) / 256), dim3(256), 0, s, ws, C, splits,
                     invstd, sums, dw, db, grad_beta);
}

void bn_bwd_elemt(const float* dy, const float* x, const float* mean, const float* invstd,
                  const float* w, const float* sums, const float* y_relu, const float* count,
                  int N, int C, int HW, float* dx, hipStream_t s) {
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(bwd_elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, dy, x, mean, invstd,
                     w, sums, y_relu, count, total, C, HW, dx);
}

}  // namespace tdp
