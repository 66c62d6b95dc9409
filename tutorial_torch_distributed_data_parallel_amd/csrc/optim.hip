// Fused optimizer steps and small elementwise utilities.
//
// The reference steps torch.optim.Adam (REF/multi-GPU-training-torch.py:249), which on the GPU runs
// _multi_tensor_adam: ~7 _foreach passes over p/g/m/v (TORCH/optim/adam.py:
// 683-800). Here each optimizer is ONE pass: every element of p, g and the state is read once and
// p and the state written once (SGD+momentum 20 B/elem, Adam 28 B/elem), f32x4-vectorised and
// grid-strided. The "flat" form runs over the whole parameter arena of a DDP model (params and
// grads are views into two equally laid out flat buffers, see parallel/arena.py); the "multi"
// form walks a device-side chunk table for arbitrary parameter lists.
//
// `grad_scale` folds the 1/world_size gradient averaging into the update when the reducer used a
// SUM all-reduce, so no separate div_ pass over the gradients is needed (K24).
#include "common.h"
#include "kernels.h"
#include "optim_elem.h"

namespace tdp {
namespace {

template <bool VEC>
__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p,
                                                       const float* __restrict__ g,
                                                       float* __restrict__ buf, long n,
                                                       SgdHyper h) {
  load_hyper(h);
  const long n4 = VEC ? n / 4 : 0;
  const long stride = (long)gridDim.x * blockDim.x;
  const bool mom = h.momentum != 0.f;
  const bool mrd = mom && !h.first_step;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // main body: U float4 per stream in flight per lane (one HBM round trip per U elements), and
  // non-temporal traffic -- every element is touched once per step
  constexpr int U = 4;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 pv[U], gv[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i + u * stride);
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i + u * stride);
      bv[u] = mrd ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(buf) + i + u * stride)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = pv[u][e], be = bv[u][e];
        sgd_elem(pe, gv[u][e], be, h);
        pv[u][e] = pe;
        bv[u][e] = be;
      }
      __builtin_nontemporal_store(pv[u], reinterpret_cast<f32x4*>(p) + i + u * stride);
      if (mom) __builtin_nontemporal_store(bv[u], reinterpret_cast<f32x4*>(buf) + i + u * stride);
    }
  }
  for (; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (mom && !h.first_step) bv = reinterpret_cast<f32x4*>(buf)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], be = bv[e];
      sgd_elem(pe, gv[e], be, h);
      pv[e] = pe;
      bv[e] = be;
    }
    reinterpret_cast<f32x4*>(p)[i] = pv;
    if (mom) reinterpret_cast<f32x4*>(buf)[i] = bv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pe = p[i], be = (mom && !h.first_step) ? buf[i] : 0.f;
    sgd_elem(pe, g[i], be, h);
    p[i] = pe;
    if (mom) buf[i] = be;
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void adam_flat_kernel(float* __restrict__ p,
                                                        const float* __restrict__ g,
                                                        float* __restrict__ m,
                                                        float* __restrict__ v,
                                                        float* __restrict__ vmax, long n,
                                                        AdamHyper h) {
  load_hyper(h);
  const long n4 = VEC ? n / 4 : 0;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // main body (no amsgrad): U float4 per stream in flight per lane, non-temporal traffic
  constexpr int U = 2;
  if (!h.amsgrad) {
    for (; i + (U - 1) * stride < n4; i += U * stride) {
      f32x4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long j = i + u * stride;
        pv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + j);
        gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + j);
        mv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m) + j);
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v) + j);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pe = pv[u][e], me = mv[u][e], ve = vv[u][e];
          adam_elem(pe, gv[u][e], me, ve, nullptr, h);
          pv[u][e] = pe; mv[u][e] = me; vv[u][e] = ve;
        }
        const long j = i + u * stride;
        __builtin_nontemporal_store(pv[u], reinterpret_cast<f32x4*>(p) + j);
        __builtin_nontemporal_store(mv[u], reinterpret_cast<f32x4*>(m) + j);
        __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4*>(v) + j);
      }
    }
  }
  for (; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mv = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    f32x4 xv = {0.f, 0.f, 0.f, 0.f};
    if (h.amsgrad) xv = reinterpret_cast<f32x4*>(vmax)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], me = mv[e], ve = vv[e], xe = xv[e];
      adam_elem(pe, gv[e], me, ve, &xe, h);
      pv[e] = pe; mv[e] = me; vv[e] = ve; xv[e] = xe;
    }
    reinterpret_cast<f32x4*>(p)[i] = pv;
    reinterpret_cast<f32x4*>(m)[i] = mv;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (h.amsgrad) reinterpret_cast<f32x4*>(vmax)[i] = xv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pe = p[i], me = m[i], ve = v[i];
    float xe = h.amsgrad ? vmax[i] : 0.f;
    adam_elem(pe, g[i], me, ve, &xe, h);
    p[i] = pe; m[i] = me; v[i] = ve;
    if (h.amsgrad) vmax[i] = xe;
  }
}

// One workgroup per chunk-table entry (chunks are <= 64K elements, built on the host).
__global__ __launch_bounds__(256) void sgd_multi_kernel(const TensorChunk* __restrict__ table,
                                                        SgdHyper h) {
  load_hyper(h);
  const TensorChunk c = table[blockIdx.x];
  const bool mom = h.momentum != 0.f;
  for (long i = threadIdx.x; i < c.n; i += blockDim.x) {
    float pe = c.p[i], be = (mom && !h.first_step) ? c.s0[i] : 0.f;
    sgd_elem(pe, c.g[i], be, h);
    c.p[i] = pe;
    if (mom) c.s0[i] = be;
  }
}

__global__ __launch_bounds__(256) void adam_multi_kernel(const TensorChunk* __restrict__ table,
                                                         AdamHyper h) {
  load_hyper(h);
  const TensorChunk c = table[blockIdx.x];
  for (long i = threadIdx.x; i < c.n; i += blockDim.x) {
    float pe = c.p[i], me = c.s0[i], ve = c.s1[i];
    float xe = h.amsgrad ? c.s2[i] : 0.f;
    adam_elem(pe, c.g[i], me, ve, &xe, h);
    c.p[i] = pe; c.s0[i] = me; c.s1[i] = ve;
    if (h.amsgrad) c.s2[i] = xe;
  }
}

__global__ void scale_kernel(float* x, long n, float a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    x[i] *= a;
}

__global__ void fill_kernel(float* x, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    x[i] = v;
}

__global__ void f2bf_kernel(const float* __restrict__ x, unsigned short* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = f32_to_bf16(x[i]);
}

__global__ void bf2f_kernel(const unsigned short* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = bf16_to_f32(x[i]);
}

// ---------------------------------------------------------------- device hyper block (kernels.h)
__global__ void opt_step_begin_kernel(float* d, int kind) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int* di = reinterpret_cast<int*>(d);
  const int t = di[kHStep] + 1;
  di[kHStep] = t;
  d[kHFirst] = d[kHFirstNext];
  d[kHFirstNext] = 0.f;
  d[kHScale] = 1.f;
  d[kHSumsq] = 0.f;
  if (kind == 2) {
    // double precision like torch's host-side bias corrections (TORCH/optim/adam.py)
    d[kHBc1] = (float)(1.0 - pow((double)d[kHMom], (double)t));
    d[kHBc2] = (float)sqrt(1.0 - pow((double)d[kHDamp], (double)t));
  }
}

__global__ void clip_coef_kernel(float* d) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float norm = sqrtf(d[kHSumsq]);
  d[kHNorm] = norm;
  const float mx = d[kHMaxNorm];
  // torch.nn.utils.clip_grad_norm_: coef = max_norm / (total_norm + 1e-6), clamped to 1
  d[kHScale] = mx > 0.f ? fminf(1.f, mx / (norm + 1e-6f)) : 1.f;
}

// Deterministic two-pass sum of squares over a RangeSet: every workgroup of a FIXED grid writes
// its partial to d[kHPartials + blockIdx.x]; the finish kernel adds them in index order. The
// result is therefore bit-identical on every rank that holds the same values (the clip
// coefficient must agree across replicas).
__device__ __forceinline__ long range_index_d(const RangeSet& r, long e);

__global__ __launch_bounds__(256) void sumsq_ranges_kernel(const float* __restrict__ x,
                                                           RangeSet r, long total, float* d) {
  __shared__ float red[4];
  float s = 0.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const float v = x[range_index_d(r, e)];
    s = fmaf(v, v, s);
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) d[kHPartials + blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sumsq_finish_kernel(float* d, int parts) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < parts; i += 256) s += d[kHPartials + i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) d[kHSumsq] += s;
}

__global__ __launch_bounds__(256) void scale_ranges_kernel(float* __restrict__ x, RangeSet r,
                                                           long total, const float* d) {
  const float a = d[kHScale];
  if (a == 1.f) return;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x)
    x[range_index_d(r, e)] *= a;
}

__device__ __forceinline__ long range_index_d(const RangeSet& r, long e) {
  for (int i = 0; i < r.n; ++i) {
    if (e < r.len[i]) return r.begin[i] + e;
    e -= r.len[i];
  }
  return -1;
}

inline int grid_for(long work, int cap = 2048) {
  long g = (work + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

void sgd_flat(float* p, const float* g, float* buf, long n, const SgdHyper& h, hipStream_t s) {
  if (n <= 0) return;
  // grid capped at 2048 workgroups (8 per CU) and grid-strided (Guideline 11)
  if (al16(p) && al16(g) && (buf == nullptr || al16(buf)))
    hipLaunchKernelGGL(sgd_flat_kernel<true>, dim3(grid_for(n / 4)), dim3(256), 0, s, p, g, buf,
                       n, h);
  else
    hipLaunchKernelGGL(sgd_flat_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s, p, g, buf, n,
                       h);
}

// ------------------------------------------------------------------ multi-range (one launch)
namespace {
// element e of the concatenated ranges -> arena index (ranges are few: linear scan)
__device__ __forceinline__ long range_index(const RangeSet& r, long e) {
  for (int i = 0; i < r.n; ++i) {
    if (e < r.len[i]) return r.begin[i] + e;
    e -= r.len[i];
  }
  return -1;
}

__global__ __launch_bounds__(256) void sgd_ranges_kernel(float* __restrict__ p,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ buf, RangeSet r,
                                                         long total, SgdHyper h) {
  load_hyper(h);
  const bool mom = h.momentum != 0.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const long i = range_index(r, e);
    float pe = p[i], be = (mom && !h.first_step) ? buf[i] : 0.f;
    sgd_elem(pe, g[i], be, h);
    p[i] = pe;
    if (mom) buf[i] = be;
  }
}

__global__ __launch_bounds__(256) void adam_ranges_kernel(float* __restrict__ p,
                                                          const float* __restrict__ g,
                                                          float* __restrict__ m,
                                                          float* __restrict__ v,
                                                          float* __restrict__ vmax, RangeSet r,
                                                          long total, AdamHyper h) {
  load_hyper(h);
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const long i = range_index(r, e);
    float pe = p[i], me = m[i], ve = v[i];
    adam_elem(pe, g[i], me, ve, vmax ? vmax + i : nullptr, h);
    p[i] = pe;
    m[i] = me;
    v[i] = ve;
  }
}
}  // namespace

static long range_total(const RangeSet& r) {
  long t = 0;
  for (int i = 0; i < r.n; ++i) t += r.len[i];
  return t;
}

void sgd_ranges(float* p, const float* g, float* buf, const RangeSet& r, const SgdHyper& h,
                hipStream_t s) {
  const long total = range_total(r);
  if (total <= 0) return;
  hipLaunchKernelGGL(sgd_ranges_kernel, dim3(grid_for(total)), dim3(256), 0, s, p, g, buf, r,
                     total, h);
}

void adam_ranges(float* p, const float* g, float* m, float* v, float* vmax, const RangeSet& r,
                 const AdamHyper& h, hipStream_t s) {
  const long total = range_total(r);
  if (total <= 0) return;
  hipLaunchKernelGGL(adam_ranges_kernel, dim3(grid_for(total)), dim3(256), 0, s, p, g, m, v,
                     vmax, r, total, h);
}

void adam_flat(float* p, const float* g, float* m, float* v, float* vmax, long n,
               const AdamHyper& h, hipStream_t s) {
  if (n <= 0) return;
  if (al16(p) && al16(g) && al16(m) && al16(v) && (vmax == nullptr || al16(vmax)))
    hipLaunchKernelGGL(adam_flat_kernel<true>, dim3(grid_for(n / 4)), dim3(256), 0, s, p, g, m,
                       v, vmax, n, h);
  else
    hipLaunchKernelGGL(adam_flat_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v,
                       vmax, n, h);
}

void sgd_multi(const TensorChunk* table, int count, const SgdHyper& h, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(sgd_multi_kernel, dim3(count), dim3(256), 0, s, table, h);
}

void adam_multi(const TensorChunk* table, int count, const AdamHyper& h, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(adam_multi_kernel, dim3(count), dim3(256), 0, s, table, h);
}

void scale_inplace(float* x, long n, float a, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, a);
}

void fill_f32(float* x, long n, float v, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, v);
}

void f32_to_bf16_copy(const float* x, uint16_t* y, long n, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(f2bf_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, (unsigned short*)y, n);
}

void bf16_to_f32_copy(const uint16_t* x, float* y, long n, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(bf2f_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const unsigned short*)x,
                       y, n);
}

void opt_step_begin(float* dev, int kind, hipStream_t s) {
  hipLaunchKernelGGL(opt_step_begin_kernel, dim3(1), dim3(64), 0, s, dev, kind);
}

void clip_coef_from_sumsq(float* dev, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, s, dev);
}

void sumsq_ranges(const float* x, const RangeSet& r, float* dev, hipStream_t s) {
  long total = 0;
  for (int i = 0; i < r.n; ++i) total += r.len[i];
  if (total <= 0) return;
  const int parts = grid_for(total, kHPartialsMax);
  hipLaunchKernelGGL(sumsq_ranges_kernel, dim3(parts), dim3(256), 0, s, x, r, total, dev);
  hipLaunchKernelGGL(sumsq_finish_kernel, dim3(1), dim3(256), 0, s, dev, parts);
}

void scale_ranges_by(float* x, const RangeSet& r, const float* dev, hipStream_t s) {
  long total = 0;
  for (int i = 0; i < r.n; ++i) total += r.len[i];
  if (total > 0)
    hipLaunchKernelGGL(scale_ranges_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, r, total,
                       dev);
}

}  // namespace tdp
