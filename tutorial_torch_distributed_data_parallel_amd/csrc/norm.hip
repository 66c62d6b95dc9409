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
#include <cstdlib>
#include <initializer_list>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "optim_elem.h"
#include "split_bf16.h"

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
                                                  float* __restrict__ var,
    float* __restrict__ cnt_out, float cnt) {
  if (cnt_out && splits == 1 && blockIdx.x == 0 && threadIdx.x == 0) *cnt_out = cnt;
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
                                                  float* __restrict__ var,
    float* __restrict__ cnt_out, float cnt) {
  if (cnt_out && splits == 1 && blockIdx.x == 0 && threadIdx.x == 0) *cnt_out = cnt;
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

// Split partials -> final: a workgroup owns 16 channels; its 16 lane groups of 16 take every
// 16th split (each partial row is read 16 channels = 64 B at a time) and merge through LDS. (The
// first form -- 64 channels, 4 split groups -- was latency-bound on its 64-step dependent merge
// chains: 37 us per BN layer in the ResNet-50 profile, 2 ms per step.) Also writes the element
// count into the stats (`cnt_out`), so no separate fill is launched.
__global__ __launch_bounds__(256) void moments_final(const float* __restrict__ ws, int C,
                                                     int splits, float* __restrict__ mean,
                                                     float* __restrict__ var,
                                                     float* __restrict__ cnt_out, float cnt) {
  __shared__ Wf sh[16][16];
  const int lane = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lane;
  Wf w{0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int z = g; z < splits; z += 16) {
      const float* o = ws + (long)z * 3 * C;
      w = wf_merge(w, Wf{o[c], o[C + c], o[2 * C + c]});
    }
  }
  sh[g][lane] = w;
  __syncthreads();
  if (threadIdx.x < 16 && c < C) {
    Wf a = wf_merge(wf_merge(sh[0][lane], sh[1][lane]), wf_merge(sh[2][lane], sh[3][lane]));
    Wf b = wf_merge(wf_merge(sh[4][lane], sh[5][lane]), wf_merge(sh[6][lane], sh[7][lane]));
    Wf d = wf_merge(wf_merge(sh[8][lane], sh[9][lane]), wf_merge(sh[10][lane], sh[11][lane]));
    Wf e = wf_merge(wf_merge(sh[12][lane], sh[13][lane]), wf_merge(sh[14][lane], sh[15][lane]));
    w = wf_merge(wf_merge(a, b), wf_merge(d, e));
    mean[c] = w.mean;
    var[c] = w.n > 0.f ? w.m2 / w.n : 0.f;
  }
  if (cnt_out && blockIdx.x == 0 && threadIdx.x == 0) *cnt_out = cnt;
}

// First level of the per-tile partial merge: block (channel group of 16, chunk of kPartChunk
// tiles); 16 lane groups take every 16th tile of the chunk, merged through LDS -> ws
// [chunks][3][C] (moments_final finishes). Parallel over chunks: a 3136-tile layer-1 output is
// 49 chunks of 64 (256-tile chunks left 52 workgroups for a 64-channel layer, each lane on a
// 16-step dependent merge chain: 12.7 us per BN layer in profiles/r9/resnet50_dp1_kernels_r9ai.md)
constexpr int kPartChunk = 64;
__global__ __launch_bounds__(256) void moments_partials_l1(const float* __restrict__ part, int T,
                                                           int C, float* __restrict__ ws) {
  __shared__ Wf sh[16][16];
  const int lane = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lane;
  const int z0 = blockIdx.y * kPartChunk;
  Wf w{0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int z = z0 + g; z < z0 + kPartChunk && z < T; z += 16) {
      const float* o = part + (long)z * 3 * C;
      w = wf_merge(w, Wf{o[c], o[C + c], o[2 * C + c]});
    }
  }
  sh[g][lane] = w;
  __syncthreads();
  if (threadIdx.x < 16 && c < C) {
    Wf a = wf_merge(wf_merge(sh[0][lane], sh[1][lane]), wf_merge(sh[2][lane], sh[3][lane]));
    Wf b = wf_merge(wf_merge(sh[4][lane], sh[5][lane]), wf_merge(sh[6][lane], sh[7][lane]));
    Wf d = wf_merge(wf_merge(sh[8][lane], sh[9][lane]), wf_merge(sh[10][lane], sh[11][lane]));
    Wf e = wf_merge(wf_merge(sh[12][lane], sh[13][lane]), wf_merge(sh[14][lane], sh[15][lane]));
    w = wf_merge(wf_merge(a, b), wf_merge(d, e));
    float* o = ws + (long)blockIdx.y * 3 * C;
    o[c] = w.n; o[C + c] = w.mean; o[2 * C + c] = w.m2;
  }
}

// Rows of `g`: [mean(C) | var(C) | count], stride 2C+1. Zero-count ranks drop out, as in
// batch_norm_gather_stats_with_counts (TORCH/nn/modules/_functions.py:96-115).
__global__ void merge_kernel(const float* __restrict__ g, int R, int C, float eps, float momentum,
                             float* __restrict__ mean, float* __restrict__ invstd,
                             float* __restrict__ rmean, float* __restrict__ rvar,
                             int64_t* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (nbt && c == 0) *nbt += 1;  // BatchNorm's num_batches_tracked (one thread, no ATen add_)
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

__global__ __launch_bounds__(256) void bwd_reduce_final(const float* __restrict__ part, int C,
                                                        int splits,
                                                        const float* __restrict__ invstd,
                                                        float* __restrict__ sums,
                                                        float* __restrict__ dw,
                                                        float* __restrict__ db, float beta) {
  // 16 channels per workgroup x 16 split groups (as moments_final)
  __shared__ float s0[16][16], s1[16][16];
  const int lane = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lane;
  float a = 0.f, m = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int z = g; z < splits; z += 16) {
      a += part[(long)z * 2 * C + c];
      m += part[(long)z * 2 * C + C + c];
    }
  }
  s0[g][lane] = a;
  s1[g][lane] = m;
  __syncthreads();
  if (threadIdx.x >= 16 || c >= C) return;
  a = 0.f;
  m = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    a += s0[k][lane];
    m += s1[k][lane];
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

// ------------------------------------------------------------------ [rows, C] with C % 4 == 0
// BatchNorm1d and channels_last BatchNorm2d (NHWC activations are a [pixels, C] matrix). A
// workgroup owns CB = min(C, 1024) channels; a thread owns 4 adjacent channels (one 16-B load
// per row, rows coalesced across lanes) and walks rows with stride RPW = 256 / (CB / 4); the
// RPW row groups are merged through LDS. One reciprocal per row serves 4 Welford updates.
__device__ __forceinline__ void rows4_layout(int C, int& CB, int& LPR, int& RPW,
                                             int threads = 256) {
  CB = C < 1024 ? C : 1024;
  LPR = CB / 4;
  RPW = threads / LPR;
}

// The two row reductions run 1024-thread workgroups, one per CU: 16 waves keep enough loads in
// flight to stream at HBM rate (256-thread workgroups at one per CU read 3.7-4.4 TB/s; more
// workgroups per CU instead multiply the split partials the final kernels merge serially). The
// RPW row groups of a workgroup are merged by a tree in LDS.
constexpr int kRedT = 1024;

__device__ __forceinline__ int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__global__ __launch_bounds__(kRedT) void moments_rows4(const float* __restrict__ x, int N, int C,
                                                       int splits, float* __restrict__ ws,
                                                       float* __restrict__ mean,
                                                       float* __restrict__ var,
    float* __restrict__ cnt_out, float cnt) {
  if (cnt_out && splits == 1 && blockIdx.x == 0 && threadIdx.x == 0) *cnt_out = cnt;
  __shared__ float sh[3][4096];
  int CB, LPR, RPW;
  rows4_layout(C, CB, LPR, RPW, kRedT);
  const int t = threadIdx.x, cq = t % LPR, rg = t / LPR;
  const int c = blockIdx.x * CB + 4 * cq;
  const bool act = rg < RPW && c < C;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  float n = 0.f, mu[4] = {0.f, 0.f, 0.f, 0.f}, m2[4] = {0.f, 0.f, 0.f, 0.f};
  if (act) {
#pragma unroll 4
    for (long r = b + rg; r < e; r += RPW) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * C + c);
      n += 1.f;
      const float inv = 1.f / n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[j] - mu[j];
        mu[j] = fmaf(d, inv, mu[j]);
        m2[j] = fmaf(d, v[j] - mu[j], m2[j]);
      }
    }
  }
  if (rg < RPW) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = rg * CB + 4 * cq + j;
      sh[0][q] = n;
      sh[1][q] = mu[j];
      sh[2][q] = m2[j];
    }
  }
  // tree merge of the RPW row groups (Chan), log2(RPW) levels
  for (int st = pow2_ceil(RPW) >> 1; st > 0; st >>= 1) {
    __syncthreads();
    for (int i = t; i < st * CB; i += kRedT) {
      const int g = i / CB, k = i - g * CB;
      if (g + st < RPW) {
        const Wf w = wf_merge(Wf{sh[0][i], sh[1][i], sh[2][i]},
                              Wf{sh[0][i + st * CB], sh[1][i + st * CB], sh[2][i + st * CB]});
        sh[0][i] = w.n; sh[1][i] = w.mean; sh[2][i] = w.m2;
      }
      (void)k;
    }
  }
  __syncthreads();
  for (int k = t; k < CB; k += kRedT) {
    const int ch = blockIdx.x * CB + k;
    if (ch >= C) continue;
    const Wf w{sh[0][k], sh[1][k], sh[2][k]};
    if (splits == 1) {
      mean[ch] = w.mean;
      var[ch] = w.n > 0.f ? w.m2 / w.n : 0.f;
    } else {
      float* o = ws + (long)blockIdx.y * 3 * C;
      o[ch] = w.n; o[C + ch] = w.mean; o[2 * C + ch] = w.m2;
    }
  }
}

__global__ __launch_bounds__(kRedT) void bwd_reduce_rows4(const float* __restrict__ dy,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ yr, int N,
                                                          int C, int splits,
                                                          float* __restrict__ part,
                                                          const uint8_t* __restrict__ mk) {
  __shared__ float sh[2][4096];
  int CB, LPR, RPW;
  rows4_layout(C, CB, LPR, RPW, kRedT);
  const int t = threadIdx.x, cq = t % LPR, rg = t / LPR;
  const int c = blockIdx.x * CB + 4 * cq;
  const bool act = rg < RPW && c < C;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  float a[4] = {0.f, 0.f, 0.f, 0.f}, m[4] = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c);
#pragma unroll 4
    for (long r = b + rg; r < e; r += RPW) {
      const long off = r * C + c;
      f32x4 d = *reinterpret_cast<const f32x4*>(dy + off);
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + off);
      if (mk) {
        const uint32_t bits = mk[off >> 2];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = ((bits >> j) & 1u) ? d[j] : 0.f;
      } else if (yr) {
        const f32x4 yv = *reinterpret_cast<const f32x4*>(yr + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += d[j];
        m[j] = fmaf(d[j], xv[j] - mu[j], m[j]);
      }
    }
  }
  if (rg < RPW) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sh[0][rg * CB + 4 * cq + j] = a[j];
      sh[1][rg * CB + 4 * cq + j] = m[j];
    }
  }
  for (int st = pow2_ceil(RPW) >> 1; st > 0; st >>= 1) {
    __syncthreads();
    for (int i = t; i < st * CB; i += kRedT) {
      if (i / CB + st < RPW) {
        sh[0][i] += sh[0][i + st * CB];
        sh[1][i] += sh[1][i + st * CB];
      }
    }
  }
  __syncthreads();
  for (int k = t; k < CB; k += kRedT) {
    const int ch = blockIdx.x * CB + k;
    if (ch >= C) continue;
    float* o = part + (long)blockIdx.y * 2 * C;
    o[ch] = sh[0][k];
    o[C + ch] = sh[1][k];
  }
}

// y = relu?(x * sc + sh) with per-channel sc/sh computed once per thread
// LocalMerge (one rank: no gather): `invstd` holds this rank's biased variance; the kernel
// derives invstd itself, and the workgroups of the first row split write the merged stats
// [mean | invstd | count] and advance the running statistics -- bn_merge's work without its launch
struct LocalMerge {
  float* stats;  // [2C + 1] out; null = off
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float momentum;
};

__global__ __launch_bounds__(256) void elemt_rows4(const float* __restrict__ x,
                                                   const float* __restrict__ mean,
                                                   const float* __restrict__ invstd,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ bb, int N, int C,
                                                   int splits, int relu, int eval, float eps,
                                                   const float* __restrict__ res,
                                                   float* __restrict__ y,
                                                   uint8_t* __restrict__ mk,
                                                   uint16_t* __restrict__ pl, LocalMerge lm) {
  int CB, LPR, RPW;
  rows4_layout(C, CB, LPR, RPW);
  const int t = threadIdx.x, cq = t % LPR, rg = t / LPR;
  const int c = blockIdx.x * CB + 4 * cq;
  if (rg >= RPW || c >= C) return;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  float sc[4], sf[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float is = (eval || lm.stats) ? rsqrtf(invstd[c + j] + eps) : invstd[c + j];
    sc[j] = is * (w ? w[c + j] : 1.f);
    sf[j] = (bb ? bb[c + j] : 0.f) - mean[c + j] * sc[j];
    if (lm.stats && blockIdx.y == 0 && rg == 0) {
      const float n = invstd[C];  // the local count (moments layout [mean | var | count])
      lm.stats[c + j] = mean[c + j];
      lm.stats[C + c + j] = is;
      if (lm.rmean) {
        const float v = invstd[c + j];
        const float unbiased = n > 1.f ? v * n / (n - 1.f) : v;
        lm.rmean[c + j] = fmaf(lm.momentum, mean[c + j] - lm.rmean[c + j], lm.rmean[c + j]);
        lm.rvar[c + j] = fmaf(lm.momentum, unbiased - lm.rvar[c + j], lm.rvar[c + j]);
      }
      if (c + j == 0) {
        lm.stats[2 * C] = n;
        if (lm.nbt) *lm.nbt += 1;
      }
    }
  }
#pragma unroll 4
  for (long r = b + rg; r < e; r += RPW) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * C + c);
    // residual join (ResNet: relu(bn3(conv3) + identity)) fused into the normalisation
    const f32x4 rv = res ? *reinterpret_cast<const f32x4*>(res + r * C + c)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float q = fmaf(v[j], sc[j], sf[j]) + rv[j];
      o[j] = relu ? fmaxf(q, 0.f) : q;
    }
    *reinterpret_cast<f32x4*>(y + r * C + c) = o;
    // bf16 split planes of the output for a consuming skinny Linear (planes GEMM)
    if (pl) store_planes4(pl + r * C + c, (long)N * C, o[0], o[1], o[2], o[3]);
    // ReLU mask for the backward: one byte per 4 channels (64 lanes: 64 consecutive bytes)
    if (mk)
      mk[(r * C + c) >> 2] = (uint8_t)((o[0] > 0.f ? 1 : 0) | (o[1] > 0.f ? 2 : 0) |
                                       (o[2] > 0.f ? 4 : 0) | (o[3] > 0.f ? 8 : 0));
  }
}

// dx = d*k1 + x*k2 + k3 (d = dy masked by y > 0), constants per channel
__global__ __launch_bounds__(256) void bwd_elemt_rows4(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ w,
    const float* __restrict__ sums, const float* __restrict__ yr, const float* __restrict__ cnt,
    int N, int C, int splits, float* __restrict__ dx, float* __restrict__ dres,
    const uint8_t* __restrict__ mk, uint16_t* __restrict__ pl) {
  int CB, LPR, RPW;
  rows4_layout(C, CB, LPR, RPW);
  const int t = threadIdx.x, cq = t % LPR, rg = t / LPR;
  const int c = blockIdx.x * CB + 4 * cq;
  if (rg >= RPW || c >= C) return;
  long b, e;
  range_of(N, splits, blockIdx.y, b, e);
  const float inv_count = 1.f / cnt[0];
  float k1[4], k2[4], k3[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float is = invstd[c + j];
    const float mdy = sums[c + j] * inv_count;
    const float mdyx = sums[C + c + j] * inv_count;
    const float sw = is * (w ? w[c + j] : 1.f);
    const float q = is * is * mdyx;
    k1[j] = sw;
    k2[j] = -q * sw;
    k3[j] = (mean[c + j] * q - mdy) * sw;
  }
#pragma unroll 4
  for (long r = b + rg; r < e; r += RPW) {
    const long off = r * C + c;
    f32x4 d = *reinterpret_cast<const f32x4*>(dy + off);
    const f32x4 xv = *reinterpret_cast<const f32x4*>(x + off);
    if (mk) {
      const uint32_t bits = mk[off >> 2];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = ((bits >> j) & 1u) ? d[j] : 0.f;
    } else if (yr) {
      const f32x4 yv = *reinterpret_cast<const f32x4*>(yr + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
    }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf(d[j], k1[j], fmaf(xv[j], k2[j], k3[j]));
    *reinterpret_cast<f32x4*>(dx + off) = o;
    if (pl) store_planes4(pl + off, (long)N * C, o[0], o[1], o[2], o[3]);
    // gradient of the fused residual input: the ReLU-masked dy itself
    if (dres) *reinterpret_cast<f32x4*>(dres + off) = d;
  }
}

// ------------------------------------------------------- BatchNorm1d, one rank, whole columns
// A workgroup owns 16 channels (4 quads) and every row of a [N <= 512][C] batch: thread t takes
// quad t & 3 and rows t >> 2, t >> 2 + 64, ... (IT = ceil(N / 64) float4 per thread, held in
// registers between the reduction and the element pass), so the column sums need no cross-
// workgroup partials: statistics + normalisation (and sums + input gradient in the backward) are
// one launch each instead of bn_moments + bn_elemt_local (bn_bwd_reduce + its final merge +
// bn_bwd_elemt). The element formulas are elemt_rows4's / bwd_elemt_rows4's.
constexpr int kB1Cols = 16, kB1Lanes = 64;

// per-channel sums of the block's 64 row groups, tree-reduced in a fixed order; every thread
// returns its quad's 4 totals
__device__ __forceinline__ f32x4 b1_reduce(f32x4 v, f32x4 (*sh)[4]) {
  const int q = threadIdx.x & 3, rg = threadIdx.x >> 2;
  sh[rg][q] = v;
#pragma unroll
  for (int st = kB1Lanes / 2; st > 0; st >>= 1) {
    __syncthreads();
    if (rg < st) sh[rg][q] += sh[rg + st][q];
  }
  __syncthreads();
  const f32x4 r = sh[0][q];
  __syncthreads();  // sh is reused by the next reduction
  return r;
}

// MODE kB1Local: this batch's statistics, then the normalisation (one rank).
// MODE kB1Moments (SyncBatchNorm, before the all-gather): only the batch's moments
//   [mean | var | count] -- bn_moments' layout -- into `stats`.
// MODE kB1Gathered (after it): the R ranks' gathered moments `g` [R][2C+1] merged per channel in
//   rank order exactly as merge_kernel does (zero-count ranks dropped), then the normalisation:
//   bn_merge + bn_elemt in one launch.
constexpr int kB1Local = 0, kB1Moments = 1, kB1Gathered = 2;

template <int IT, int MODE>
__global__ __launch_bounds__(256) void bn1d_local_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bb, int N,
    int C, int relu, float eps, float momentum, float* __restrict__ stats,
    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float* __restrict__ y, uint8_t* __restrict__ mk, uint16_t* __restrict__ pl,
    const float* __restrict__ g, int R) {
  __shared__ f32x4 sh[kB1Lanes][4];
  const int q = threadIdx.x & 3, rg = threadIdx.x >> 2;
  const int c = blockIdx.x * kB1Cols + 4 * q;
  f32x4 v[IT];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rg + kB1Lanes * i;
    v[i] = r < N ? *reinterpret_cast<const f32x4*>(x + (long)r * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i];
  }
  f32x4 mean, var;
  float n, m2t[4];
  if constexpr (MODE == kB1Gathered) {
    Wf wf[4] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const long stride = 2L * C + 1;
    for (int rk = 0; rk < R; ++rk) {
      const float* row = g + rk * stride;
      const float nr = row[2 * C];
      if (nr <= 0.f) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = wf_merge(wf[j], Wf{nr, row[c + j], row[C + c + j] * nr});
    }
    n = wf[0].n;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mean[j] = wf[j].mean;
      var[j] = wf[j].n > 0.f ? wf[j].m2 / wf[j].n : 0.f;
      m2t[j] = wf[j].m2;
    }
  } else {
    n = (float)N;
    mean = b1_reduce(s, sh) / n;
    f32x4 m2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (rg + kB1Lanes * i < N) {
        const f32x4 d = v[i] - mean;
        m2 += d * d;
      }
    }
    var = b1_reduce(m2, sh) / n;
#pragma unroll
    for (int j = 0; j < 4; ++j) m2t[j] = var[j] * n;
  }
  if constexpr (MODE == kB1Moments) {
    if (rg == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[c + j] = mean[j];
        stats[C + c + j] = var[j];
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) stats[2 * C] = n;
    return;
  }
  float sc[4], sf[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float is = rsqrtf(var[j] + eps);
    sc[j] = is * (w ? w[c + j] : 1.f);
    sf[j] = (bb ? bb[c + j] : 0.f) - mean[j] * sc[j];
    if (rg == 0) {
      stats[c + j] = mean[j];
      stats[C + c + j] = is;
      if (rmean) {
        const float unbiased = MODE == kB1Gathered
                                   ? (n > 1.f ? m2t[j] / (n - 1.f) : var[j])
                                   : (n > 1.f ? var[j] * n / (n - 1.f) : var[j]);
        rmean[c + j] = fmaf(momentum, mean[j] - rmean[c + j], rmean[c + j]);
        rvar[c + j] = fmaf(momentum, unbiased - rvar[c + j], rvar[c + j]);
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stats[2 * C] = n;
    if (nbt) *nbt += 1;
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rg + kB1Lanes * i;
    if (r >= N) continue;
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = fmaf(v[i][j], sc[j], sf[j]);
      o[j] = relu ? fmaxf(t, 0.f) : t;
    }
    *reinterpret_cast<f32x4*>(y + (long)r * C + c) = o;
    if (pl) store_planes4(pl + (long)r * C + c, (long)N * C, o[0], o[1], o[2], o[3]);
    if (mk)
      mk[((long)r * C + c) >> 2] = (uint8_t)((o[0] > 0.f ? 1 : 0) | (o[1] > 0.f ? 2 : 0) |
                                             (o[2] > 0.f ? 4 : 0) | (o[3] > 0.f ? 8 : 0));
  }
}

// One parameter element's optimizer step, split so that its loads (hyper block, p, state) are
// issued at kernel start and the update itself costs no memory round trip at the end
struct OptElem {
  OptEpilogue o;
  float p, s0, s1;
  __device__ __forceinline__ void load(const OptEpilogue& e, int i) {
    o = e;
    if (o.kind == 1) {
      load_hyper(o.sgd);
      p = o.p[i];
      s0 = (o.sgd.momentum != 0.f && !o.sgd.first_step) ? o.s0[i] : 0.f;
    } else if (o.kind == 2) {
      load_hyper(o.adam);
      p = o.p[i];
      s0 = o.s0[i];
      s1 = o.s1[i];
    }
  }
  __device__ __forceinline__ void step(int i, float g) {
    if (o.kind == 1) {
      sgd_elem(p, g, s0, o.sgd);
      o.p[i] = p;
      if (o.sgd.momentum != 0.f) o.s0[i] = s0;
    } else if (o.kind == 2) {
      adam_elem(p, g, s0, s1, o.s2 ? o.s2 + i : nullptr, o.adam);
      o.p[i] = p;
      o.s0[i] = s0;
      o.s1[i] = s1;
    }
  }
};

// SUMS (SyncBatchNorm, before the all-reduce): only this batch's [sum dy | sum dy (x - mean)]
// into `sums` and the local dw / db -- bn_bwd_reduce in one launch; bn_bwd_elemt follows
template <int IT, bool SUMS>
__global__ __launch_bounds__(256) void bn1d_local_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ stats,
    const float* __restrict__ w, int N, int C, const uint8_t* __restrict__ mk,
    float* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    uint16_t* __restrict__ pl, OptEpilogue wo, OptEpilogue bo, float* __restrict__ sums) {
  __shared__ f32x4 sh[kB1Lanes][4];
  __shared__ float tot[2][kB1Cols];  // this block's sum dy | sum dy (x - mean), per channel
  const int q = threadIdx.x & 3, rg = threadIdx.x >> 2;
  const int c = blockIdx.x * kB1Cols + 4 * q;
  // in-place update (wo / bo): thread t < 32 owns element t & 15 of w (t < 16) or b; its loads go
  // out now, behind the streaming loads below
  const bool upd = (wo.kind || bo.kind) && threadIdx.x < 2 * kB1Cols;
  const int uc = blockIdx.x * kB1Cols + (threadIdx.x & (kB1Cols - 1));
  const bool ub = threadIdx.x >= kB1Cols;
  OptElem ue;
  ue.o.kind = 0;
  if (upd) ue.load(ub ? bo : wo, uc);
  const f32x4 mu = *reinterpret_cast<const f32x4*>(stats + c);
  f32x4 d[IT], xv[IT];
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, m = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rg + kB1Lanes * i;
    if (r < N) {
      const long off = (long)r * C + c;
      d[i] = *reinterpret_cast<const f32x4*>(dy + off);
      xv[i] = *reinterpret_cast<const f32x4*>(x + off);
      if (mk) {
        const uint32_t bits = mk[off >> 2];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = ((bits >> j) & 1u) ? d[i][j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += d[i][j];
        m[j] = fmaf(d[i][j], xv[i][j] - mu[j], m[j]);
      }
    }
  }
  const f32x4 sdy = b1_reduce(a, sh);
  const f32x4 sdyx = b1_reduce(m, sh);
  if constexpr (SUMS) {
    if (rg == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sums[c + j] = sdy[j];
        sums[C + c + j] = sdyx[j];
        if (dw) dw[c + j] = sdyx[j] * stats[C + c + j];
        if (db) db[c + j] = sdy[j];
      }
    }
    return;
  }
  const float inv_count = 1.f / stats[2 * C];
  float k1[4], k2[4], k3[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float is = stats[C + c + j];
    const float mdy = sdy[j] * inv_count, mdyx = sdyx[j] * inv_count;
    const float sw = is * (w ? w[c + j] : 1.f);
    const float qq = is * is * mdyx;
    k1[j] = sw;
    k2[j] = -qq * sw;
    k3[j] = (mu[j] * qq - mdy) * sw;
  }
  // dw / db are complete here. World size 1 + fused optimizer: the affine parameters are
  // updated in place (the optimizer's element update, as the weight-gradient GEMM epilogue does)
  // instead of storing their gradients, once every thread has read w
  if (rg == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gw = sdyx[j] * stats[C + c + j], gb = sdy[j];
      if (!wo.kind && dw) dw[c + j] = gw;
      if (!bo.kind && db) db[c + j] = gb;
      tot[0][4 * q + j] = gb;
      tot[1][4 * q + j] = gw;
    }
  }
  if (wo.kind || bo.kind) {
    __syncthreads();
    if (upd && ue.o.kind) ue.step(uc, tot[ub ? 0 : 1][threadIdx.x & (kB1Cols - 1)]);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rg + kB1Lanes * i;
    if (r >= N) continue;
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf(d[i][j], k1[j], fmaf(xv[i][j], k2[j], k3[j]));
    *reinterpret_cast<f32x4*>(dx + (long)r * C + c) = o;
    if (pl) store_planes4(pl + (long)r * C + c, (long)N * C, o[0], o[1], o[2], o[3]);
  }
}

inline bool rows4_ok(int C, int HW, std::initializer_list<const void*> ptrs) {
  if (HW != 1 || C % 4) return false;
  for (const void* q : ptrs)
    if (q && ((uintptr_t)q & 15)) return false;
  return true;
}

inline int rows4_nblk(int C) { return (C + 1023) / 1024; }

// row splits for the streaming (elementwise) rows4 kernels: ~4 workgroups per CU
inline int rows4_ew_splits(int N, int C) {
  const int CB = C < 1024 ? C : 1024, RPW = 256 / (CB / 4);
  const int nblk = rows4_nblk(C);
  long s = (1024 + nblk - 1) / nblk;
  const long cap = (N + 4L * RPW - 1) / (4L * RPW);  // >= 4 row iterations per thread
  if (s > cap) s = cap;
  return s < 1 ? 1 : (int)s;
}

inline int ew_grid(long total) {
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

int bn_splits(int N, int C, int HW, int num_cus) {
  if (HW == 1 && C % 4 == 0) {
    // rows4 reductions (1024-thread workgroups): one workgroup per CU, >= 8 row iterations per
    // thread
    constexpr int per_cu = 1;
    const int CB = C < 1024 ? C : 1024, RPW = kRedT / (CB / 4);
    const int nblk = rows4_nblk(C);
    long s = ((long)per_cu * num_cus + nblk - 1) / nblk;
    const long cap = (N + 8L * RPW - 1) / (8L * RPW);
    if (s > cap) s = cap;
    return s < 1 ? 1 : (int)s;
  }
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

long bn_partials_ws_floats(int T, int C) { return 3L * C * ((T + kPartChunk - 1) / kPartChunk); }

void bn_moments_partials(const float* part, int T, int C, float* ws, float* mean, float* var,
                         float* count_out, float cnt, hipStream_t s) {
  const int chunks = (T + kPartChunk - 1) / kPartChunk;
  hipLaunchKernelGGL(moments_partials_l1, dim3((C + 15) / 16, chunks), dim3(256), 0, s, part, T,
                     C, ws);
  hipLaunchKernelGGL(moments_final, dim3((C + 15) / 16), dim3(256), 0, s, ws, C, chunks, mean,
                     var, count_out, cnt);
}

void bn_moments(const float* x, int N, int C, int HW, int splits, float* ws, float* mean,
                float* var, float* count_out, hipStream_t s) {
  const float cnt = (float)((double)N * HW);
  if (rows4_ok(C, HW, {x}))
    hipLaunchKernelGGL(moments_rows4, dim3(rows4_nblk(C), splits), dim3(kRedT), 0, s, x, N, C,
                       splits, ws, mean, var, count_out, cnt);
  else if (HW == 1)
    hipLaunchKernelGGL(moments_1d, dim3((C + 63) / 64, splits), dim3(256), 0, s, x, N, C, splits,
                       ws, mean, var, count_out, cnt);
  else
    hipLaunchKernelGGL(moments_2d, dim3(C, splits), dim3(256), 0, s, x, N, C, HW, splits, ws,
                       mean, var, count_out, cnt);
  if (splits > 1)
    hipLaunchKernelGGL(moments_final, dim3((C + 15) / 16), dim3(256), 0, s, ws, C, splits, mean,
                       var, count_out, cnt);
}

void bn_merge(const float* gathered, int R, int C, float eps, float momentum, float* mean,
              float* invstd, float* running_mean, float* running_var, int64_t* num_batches,
              hipStream_t s) {
  hipLaunchKernelGGL(merge_kernel, dim3((C + 255) / 256), dim3(256), 0, s, gathered, R, C, eps,
                     momentum, mean, invstd, running_mean, running_var, num_batches);
}

bool bn_elemt_local(const float* x, const float* moments, const float* w, const float* b, int N,
                    int C, bool relu, float eps, float momentum, float* stats, float* rmean,
                    float* rvar, int64_t* nbt, float* y, uint8_t* mask_out, uint16_t* planes_out,
                    hipStream_t s, const float* residual) {
  if (!rows4_ok(C, 1, {x, y, moments, w, b, stats, residual})) return false;
  const int sp = rows4_ew_splits(N, C);
  hipLaunchKernelGGL(elemt_rows4, dim3(rows4_nblk(C), sp), dim3(256), 0, s, x, moments,
                     moments + C, w, b, N, C, sp, relu ? 1 : 0, 0, eps, residual, y,
                     relu ? mask_out : nullptr, planes_out,
                     LocalMerge{stats, rmean, rvar, nbt, momentum});
  return true;
}

void bn_elemt(const float* x, const float* mean, const float* invstd, const float* w,
              const float* b, int N, int C, int HW, bool relu, float* y, hipStream_t s,
              const float* residual, uint8_t* mask_out, uint16_t* planes_out) {
  if (rows4_ok(C, HW, {x, y, mean, invstd, w, b, residual})) {
    const int sp = rows4_ew_splits(N, C);
    hipLaunchKernelGGL(elemt_rows4, dim3(rows4_nblk(C), sp), dim3(256), 0, s, x, mean, invstd, w,
                       b, N, C, sp, relu ? 1 : 0, 0, 0.f, residual, y, relu ? mask_out : nullptr,
                       planes_out, LocalMerge{});
    return;
  }
  if (residual) throw std::runtime_error("bn_elemt: a fused residual needs the [rows, C%4] form");
  if (mask_out) throw std::runtime_error("bn_elemt: a ReLU mask needs the [rows, C%4] form");
  if (planes_out) throw std::runtime_error("bn_elemt: planes need the [rows, C%4] form");
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, mean, invstd, w, b,
                     total, C, HW, relu ? 1 : 0, 0, 0.f, y);
}

void bn_eval(const float* x, const float* rmean, const float* rvar, const float* w,
             const float* b, int N, int C, int HW, float eps, bool relu, float* y, hipStream_t s) {
  if (rows4_ok(C, HW, {x, y})) {
    const int sp = rows4_ew_splits(N, C);
    hipLaunchKernelGGL(elemt_rows4, dim3(rows4_nblk(C), sp), dim3(256), 0, s, x, rmean, rvar, w,
                       b, N, C, sp, relu ? 1 : 0, 1, eps, (const float*)nullptr, y,
                       (uint8_t*)nullptr, (uint16_t*)nullptr, LocalMerge{});
    return;
  }
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, rmean, rvar, w, b,
                     total, C, HW, relu ? 1 : 0, 1, eps, y);
}

void bn_bwd_reduce(const float* dy, const float* x, const float* mean, const float* invstd,
                   const float* y_relu, int N, int C, int HW, int splits, float* ws, float* sums,
                   float* dw, float* db, float grad_beta, hipStream_t s, const uint8_t* mask) {
  // partials always go through ws (2*C*splits floats); the final kernel also writes dw/db
  if (rows4_ok(C, HW, {dy, x, y_relu, mean}))
    hipLaunchKernelGGL(bwd_reduce_rows4, dim3(rows4_nblk(C), splits), dim3(kRedT), 0, s, dy, x,
                       mean, y_relu, N, C, splits, ws, mask);
  else if (mask)
    throw std::runtime_error("bn_bwd_reduce: a ReLU mask needs the [rows, C%4] form");
  else if (HW == 1)
    hipLaunchKernelGGL(bwd_reduce_1d, dim3((C + 63) / 64, splits), dim3(256), 0, s, dy, x, mean,
                       y_relu, N, C, splits, ws);
  else
    hipLaunchKernelGGL(bwd_reduce_2d, dim3(C, splits), dim3(256), 0, s, dy, x, mean, y_relu, N, C,
                       HW, splits, ws);
  hipLaunchKernelGGL(bwd_reduce_final, dim3((C + 15) / 16), dim3(256), 0, s, ws, C, splits,
                     invstd, sums, dw, db, grad_beta);
}

void bn_bwd_elemt(const float* dy, const float* x, const float* mean, const float* invstd,
                  const float* w, const float* sums, const float* y_relu, const float* count,
                  int N, int C, int HW, float* dx, hipStream_t s, float* dres,
                  const uint8_t* mask, uint16_t* planes_out) {
  if (rows4_ok(C, HW, {dy, x, y_relu, dx, dres})) {
    const int sp = rows4_ew_splits(N, C);
    hipLaunchKernelGGL(bwd_elemt_rows4, dim3(rows4_nblk(C), sp), dim3(256), 0, s, dy, x, mean,
                       invstd, w, sums, y_relu, count, N, C, sp, dx, dres, mask, planes_out);
    return;
  }
  if (planes_out) throw std::runtime_error("bn_bwd_elemt: planes need the [rows, C%4] form");
  if (dres) throw std::runtime_error("bn_bwd_elemt: a fused residual needs the [rows, C%4] form");
  if (mask) throw std::runtime_error("bn_bwd_elemt: a ReLU mask needs the [rows, C%4] form");
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(bwd_elemt_kernel, dim3(ew_grid(total)), dim3(256), 0, s, dy, x, mean, invstd,
                     w, sums, y_relu, count, total, C, HW, dx);
}

bool bn1d_local_fwd(const float* x, const float* w, const float* b, int N, int C, bool relu,
                    float eps, float momentum, float* stats, float* rmean, float* rvar,
                    int64_t* nbt, float* y, uint8_t* mask_out, uint16_t* planes_out,
                    hipStream_t s) {
  if (N < 1 || N > kBn1dMaxRows || C % kB1Cols) return false;
  for (const void* q : {(const void*)x, (const void*)y, (const void*)w, (const void*)b})
    if (q && ((uintptr_t)q & 15)) return false;
  const dim3 g(C / kB1Cols), t(256);
  const int r = relu ? 1 : 0;
  uint8_t* mk = relu ? mask_out : nullptr;
#define B1F(IT) hipLaunchKernelGGL((bn1d_local_fwd_kernel<IT, kB1Local>), g, t, 0, s, x, w, b, N, \
                                   C, r, eps, momentum, stats, rmean, rvar, nbt, y, mk, \
                                   planes_out, (const float*)nullptr, 0)
  if (N <= 64) B1F(1);
  else if (N <= 128) B1F(2);
  else if (N <= 256) B1F(4);
  else B1F(8);
#undef B1F
  return true;
}

bool bn1d_local_bwd(const float* dy, const float* x, const float* stats, const float* w, int N,
                    int C, const uint8_t* mask, float* dx, float* dw, float* db,
                    uint16_t* planes_out, hipStream_t s, const OptEpilogue* wopt,
                    const OptEpilogue* bopt) {
  if (N < 1 || N > kBn1dMaxRows || C % kB1Cols) return false;
  for (const void* q : {(const void*)dy, (const void*)x, (const void*)dx, (const void*)stats})
    if (q && ((uintptr_t)q & 15)) return false;
  const dim3 g(C / kB1Cols), t(256);
  const OptEpilogue wo = wopt ? *wopt : OptEpilogue{}, bo = bopt ? *bopt : OptEpilogue{};
#define B1B(IT) hipLaunchKernelGGL((bn1d_local_bwd_kernel<IT, false>), g, t, 0, s, dy, x, stats, \
                                   w, N, C, mask, dx, dw, db, planes_out, wo, bo, (float*)nullptr)
  if (N <= 64) B1B(1);
  else if (N <= 128) B1B(2);
  else if (N <= 256) B1B(4);
  else B1B(8);
#undef B1B
  return true;
}

bool bn1d_moments(const float* x, int N, int C, float* moments, hipStream_t s) {
  if (N < 1 || N > kBn1dMaxRows || C % kB1Cols || ((uintptr_t)x & 15)) return false;
  const dim3 g(C / kB1Cols), t(256);
#define B1M(IT) hipLaunchKernelGGL((bn1d_local_fwd_kernel<IT, kB1Moments>), g, t, 0, s, x, \
                                   (const float*)nullptr, (const float*)nullptr, N, C, 0, 0.f, \
                                   0.f, moments, (float*)nullptr, (float*)nullptr, \
                                   (int64_t*)nullptr, (float*)nullptr, (uint8_t*)nullptr, \
                                   (uint16_t*)nullptr, (const float*)nullptr, 0)
  if (N <= 64) B1M(1);
  else if (N <= 128) B1M(2);
  else if (N <= 256) B1M(4);
  else B1M(8);
#undef B1M
  return true;
}

bool bn1d_gathered_fwd(const float* x, const float* gathered, int R, const float* w,
                       const float* b, int N, int C, bool relu, float eps, float momentum,
                       float* stats, float* rmean, float* rvar, int64_t* nbt, float* y,
                       uint8_t* mask_out, uint16_t* planes_out, hipStream_t s) {
  if (N < 1 || N > kBn1dMaxRows || C % kB1Cols || R < 1) return false;
  for (const void* q : {(const void*)x, (const void*)y, (const void*)w, (const void*)b})
    if (q && ((uintptr_t)q & 15)) return false;
  const dim3 g(C / kB1Cols), t(256);
  const int r = relu ? 1 : 0;
  uint8_t* mk = relu ? mask_out : nullptr;
#define B1G(IT) hipLaunchKernelGGL((bn1d_local_fwd_kernel<IT, kB1Gathered>), g, t, 0, s, x, w, b, \
                                   N, C, r, eps, momentum, stats, rmean, rvar, nbt, y, mk, \
                                   planes_out, gathered, R)
  if (N <= 64) B1G(1);
  else if (N <= 128) B1G(2);
  else if (N <= 256) B1G(4);
  else B1G(8);
#undef B1G
  return true;
}

bool bn1d_sums(const float* dy, const float* x, const float* stats, int N, int C,
               const uint8_t* mask, float* sums, float* dw, float* db, hipStream_t s) {
  if (N < 1 || N > kBn1dMaxRows || C % kB1Cols) return false;
  for (const void* q : {(const void*)dy, (const void*)x, (const void*)stats})
    if (q && ((uintptr_t)q & 15)) return false;
  const dim3 g(C / kB1Cols), t(256);
#define B1S(IT) hipLaunchKernelGGL((bn1d_local_bwd_kernel<IT, true>), g, t, 0, s, dy, x, stats, \
                                   (const float*)nullptr, N, C, mask, (float*)nullptr, dw, db, \
                                   (uint16_t*)nullptr, OptEpilogue{}, OptEpilogue{}, sums)
  if (N <= 64) B1S(1);
  else if (N <= 128) B1S(2);
  else if (N <= 256) B1S(4);
  else B1S(8);
#undef B1S
  return true;
}

}  // namespace tdp
