// Pooling, dropout and residual elementwise kernels for the CNN models (AlexNet, ResNet-50).
//
// K3/K5/K9 max_pool2d_with_indices (+K20 backward), K10/K21 adaptive_avg_pool2d
// (+ backward; identity fast path handled by the caller), K11/K19 dropout (+ backward), plus the
// residual add+ReLU of ResNet bottlenecks. Max-pool backward is a GATHER over the (at most
// ceil(k/s)^2) windows that contain an input element, checking the saved argmax -- deterministic,
// no atomics. Dropout masks come from a counter-based hash of (seed, element index), so the
// backward regenerates the mask instead of storing it.
#include <initializer_list>

#include "common.h"
#include "kernels.h"
#include "pool.h"

namespace tdp {
namespace {

inline int ew_grid(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int NC, int H, int W, int P,
                                   int Q, int k, int s, int pad, float* __restrict__ y,
                                   int* __restrict__ idx) {
  const long total = (long)NC * P * Q;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % Q);
    const long t = i / Q;
    const int p = (int)(t % P);
    const long nc = t / P;
    const float* xp = x + nc * H * W;
    const int h0 = p * s - pad, w0 = q * s - pad;
    float best = -INFINITY;
    int bi = -1;
    for (int r = 0; r < k; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int c = 0; c < k; ++c) {
        const int w = w0 + c;
        if (w < 0 || w >= W) continue;
        const float v = xp[h * W + w];
        // first maximum wins; a NaN wins and then sticks (torch's max_pool2d propagates NaN)
        if (bi < 0 || (v > best && best == best) || (v != v && best == best)) {
          best = v;
          bi = h * W + w;
        }
      }
    }
    y[i] = best;
    if (idx) idx[i] = bi;
  }
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, const int* __restrict__ idx,
                                   int NC, int H, int W, int P, int Q, int k, int s, int pad,
                                   float* __restrict__ dx) {
  const long total = (long)NC * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const long t = i / W;
    const int h = (int)(t % H);
    const long nc = t / H;
    const int me = h * W + w;
    // windows p with p*s - pad <= h <= p*s - pad + k - 1
    const int plo = max(0, (h + pad - k + s) / s), phi = min(P - 1, (h + pad) / s);
    const int qlo = max(0, (w + pad - k + s) / s), qhi = min(Q - 1, (w + pad) / s);
    float acc = 0.f;
    for (int p = plo; p <= phi; ++p)
      for (int q = qlo; q <= qhi; ++q) {
        const long o = (nc * P + p) * Q + q;
        if (idx[o] == me) acc += dy[o];
      }
    dx[i] = acc;
  }
}

__global__ void avgpool_fwd_kernel(const float* __restrict__ x, int NC, int H, int W, int P,
                                   int Q, float* __restrict__ y) {
  const long total = (long)NC * P * Q;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % Q);
    const long t = i / Q;
    const int p = (int)(t % P);
    const long nc = t / P;
    const int h0 = (p * H) / P, h1 = ((p + 1) * H + P - 1) / P;
    const int w0 = (q * W) / Q, w1 = ((q + 1) * W + Q - 1) / Q;
    const float* xp = x + nc * H * W;
    float acc = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) acc += xp[h * W + w];
    y[i] = acc / (float)((h1 - h0) * (w1 - w0));
  }
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, int NC, int H, int W, int P,
                                   int Q, float* __restrict__ dx) {
  const long total = (long)NC * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const long t = i / W;
    const int h = (int)(t % H);
    const long nc = t / H;
    float acc = 0.f;
    // output cells whose adaptive window contains (h, w)
    for (int p = (h * P) / H; p < P && (p * H) / P <= h; ++p) {
      const int h0 = (p * H) / P, h1 = ((p + 1) * H + P - 1) / P;
      if (h < h0 || h >= h1) continue;
      for (int q = (w * Q) / W; q < Q && (q * W) / Q <= w; ++q) {
        const int w0 = (q * W) / Q, w1 = ((q + 1) * W + Q - 1) / Q;
        if (w < w0 || w >= w1) continue;
        acc += dy[(nc * P + p) * Q + q] / (float)((h1 - h0) * (w1 - w0));
      }
    }
    dx[i] = acc;
  }
}

__device__ __forceinline__ uint32_t hash32(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

__global__ void dropout_kernel(const float* __restrict__ x, long n, float p, uint64_t seed,
                               float* __restrict__ y) {
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  const float scale = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = hash32(seed, i) >= thr ? x[i] * scale : 0.f;
}

// 16-B vectorised elementwise ops (n % 4 == 0 and 16-B aligned operands, checked on the host)
__global__ void add_relu_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                long n, int relu, float* __restrict__ y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float v = a[i] + b[i];
    y[i] = relu ? fmaxf(v, 0.f) : v;
  }
}

__global__ void add_relu4_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                 long n4, int relu, f32x4* __restrict__ y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    f32x4 v = a[i] + b[i];
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    y[i] = v;
  }
}

__global__ void relu_mask_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                 long n, float* __restrict__ g) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    g[i] = y[i] > 0.f ? dy[i] : 0.f;
}

__global__ void relu_mask4_kernel(const f32x4* __restrict__ dy, const f32x4* __restrict__ y,
                                  long n4, f32x4* __restrict__ g) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    const f32x4 d = dy[i], v = y[i];
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] > 0.f ? d[j] : 0.f;
    g[i] = o;
  }
}

inline bool vec4_ok(long n, std::initializer_list<const void*> ptrs) {
  if (n % 4) return false;
  for (const void* q : ptrs)
    if ((uintptr_t)q & 15) return false;
  return true;
}

// ---- NHWC (channels_last) variants: consecutive threads walk the channel dimension, so every
// access is coalesced; index math is 32-bit (host checks numel < 2^31).
__global__ void maxpool_nhwc_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C,
                                        int P, int Q, int k, int s, int pad,
                                        float* __restrict__ y, int* __restrict__ idx) {
  const unsigned total = (unsigned)N * P * Q * C;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C, t = i / C;
    const unsigned q = t % Q, t2 = t / Q;
    const unsigned p = t2 % P, n = t2 / P;
    const int h0 = (int)p * s - pad, w0 = (int)q * s - pad;
    const float* xp = x + (size_t)n * H * W * C + c;
    float best = -INFINITY;
    int bi = -1;
    for (int r = 0; r < k; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int cc = 0; cc < k; ++cc) {
        const int w = w0 + cc;
        if (w < 0 || w >= W) continue;
        const float v = xp[(size_t)(h * W + w) * C];
        if (bi < 0 || (v > best && best == best) || (v != v && best == best)) {
          best = v;
          bi = h * W + w;
        }
      }
    }
    y[i] = best;
    idx[i] = bi;
  }
}

__global__ void maxpool_nhwc_bwd_kernel(const float* __restrict__ dy, const int* __restrict__ idx,
                                        int N, int H, int W, int C, int P, int Q, int k, int s,
                                        int pad, float* __restrict__ dx) {
  const unsigned total = (unsigned)N * H * W * C;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C, t = i / C;
    const int w = (int)(t % W);
    const unsigned t2 = t / W;
    const int h = (int)(t2 % H);
    const unsigned n = t2 / H;
    const int me = h * W + w;
    const int plo = max(0, (h + pad - k + s) / s), phi = min(P - 1, (h + pad) / s);
    const int qlo = max(0, (w + pad - k + s) / s), qhi = min(Q - 1, (w + pad) / s);
    float acc = 0.f;
    for (int p = plo; p <= phi; ++p)
      for (int q = qlo; q <= qhi; ++q) {
        const size_t o = (((size_t)n * P + p) * Q + q) * C + c;
        if (idx[o] == me) acc += dy[o];
      }
    dx[i] = acc;
  }
}

// 4-channel forms (C % 4 == 0): one thread per (pixel, 4 channels) — 16-B loads/stores and a
// quarter of the index divisions. The scalar forms were integer-division bound (AlexNet: 3
// max-pool backward calls = 246 us/step for ~0.4 GB of traffic).
typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void maxpool_nhwc_fwd4_kernel(const f32x4* __restrict__ x, int N, int H, int W, int C4,
                                         int P, int Q, int k, int s, int pad,
                                         f32x4* __restrict__ y, i32x4* __restrict__ idx) {
  const unsigned total = (unsigned)N * P * Q * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C4, t = i / C4;
    const unsigned q = t % Q, t2 = t / Q;
    const unsigned p = t2 % P, n = t2 / P;
    const int h0 = (int)p * s - pad, w0 = (int)q * s - pad;
    const f32x4* xp = x + (size_t)n * H * W * C4 + c;
    f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    i32x4 bi = {-1, -1, -1, -1};
    for (int r = 0; r < k; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int cc = 0; cc < k; ++cc) {
        const int w = w0 + cc;
        if (w < 0 || w >= W) continue;
        const f32x4 v = xp[(size_t)(h * W + w) * C4];
        const int at = h * W + w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float b = best[e];
          if (bi[e] < 0 || (v[e] > b && b == b) || (v[e] != v[e] && b == b)) {
            best[e] = v[e];
            bi[e] = at;
          }
        }
      }
    }
    y[i] = best;
    idx[i] = bi;
  }
}

__global__ void maxpool_nhwc_bwd4_kernel(const f32x4* __restrict__ dy,
                                         const i32x4* __restrict__ idx, int N, int H, int W,
                                         int C4, int P, int Q, int k, int s, int pad,
                                         f32x4* __restrict__ dx) {
  const unsigned total = (unsigned)N * H * W * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C4, t = i / C4;
    const int w = (int)(t % W);
    const unsigned t2 = t / W;
    const int h = (int)(t2 % H);
    const unsigned n = t2 / H;
    const int me = h * W + w;
    const int plo = max(0, (h + pad - k + s) / s), phi = min(P - 1, (h + pad) / s);
    const int qlo = max(0, (w + pad - k + s) / s), qhi = min(Q - 1, (w + pad) / s);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int p = plo; p <= phi; ++p)
      for (int q = qlo; q <= qhi; ++q) {
        const size_t o = (((size_t)n * P + p) * Q + q) * C4 + c;
        const i32x4 id = idx[o];
        const f32x4 g = dy[o];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += id[e] == me ? g[e] : 0.f;
      }
    dx[i] = acc;
  }
}

__global__ void avgpool_nhwc_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C,
                                        int P, int Q, float* __restrict__ y) {
  const unsigned total = (unsigned)N * P * Q * C;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C, t = i / C;
    const int q = (int)(t % Q);
    const unsigned t2 = t / Q;
    const int p = (int)(t2 % P);
    const unsigned n = t2 / P;
    const int h0 = (p * H) / P, h1 = ((p + 1) * H + P - 1) / P;
    const int w0 = (q * W) / Q, w1 = ((q + 1) * W + Q - 1) / Q;
    const float* xp = x + (size_t)n * H * W * C + c;
    float acc = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) acc += xp[(size_t)(h * W + w) * C];
    y[i] = acc / (float)((h1 - h0) * (w1 - w0));
  }
}

__global__ void avgpool_nhwc_bwd_kernel(const float* __restrict__ dy, int N, int H, int W, int C,
                                        int P, int Q, float* __restrict__ dx) {
  const unsigned total = (unsigned)N * H * W * C;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const unsigned c = i % C, t = i / C;
    const int w = (int)(t % W);
    const unsigned t2 = t / W;
    const int h = (int)(t2 % H);
    const unsigned n = t2 / H;
    float acc = 0.f;
    for (int p = (h * P) / H; p < P && (p * H) / P <= h; ++p) {
      const int h0 = (p * H) / P, h1 = ((p + 1) * H + P - 1) / P;
      if (h < h0 || h >= h1) continue;
      for (int q = (w * Q) / W; q < Q && (q * W) / Q <= w; ++q) {
        const int w0 = (q * W) / Q, w1 = ((q + 1) * W + Q - 1) / Q;
        if (w < w0 || w >= w1) continue;
        acc += dy[(((size_t)n * P + p) * Q + q) * C + c] / (float)((h1 - h0) * (w1 - w0));
      }
    }
    dx[i] = acc;
  }
}

}  // namespace

void maxpool2d_fwd(const float* x, int NC, int H, int W, int P, int Q, int k, int s, int pad,
                   float* y, int* idx, hipStream_t st) {
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(ew_grid((long)NC * P * Q)), dim3(256), 0, st, x, NC,
                     H, W, P, Q, k, s, pad, y, idx);
}

void maxpool2d_bwd(const float* dy, const int* idx, int NC, int H, int W, int P, int Q, int k,
                   int s, int pad, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(ew_grid((long)NC * H * W)), dim3(256), 0, st, dy,
                     idx, NC, H, W, P, Q, k, s, pad, dx);
}

void avgpool2d_adaptive_fwd(const float* x, int NC, int H, int W, int P, int Q, float* y,
                            hipStream_t st) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(ew_grid((long)NC * P * Q)), dim3(256), 0, st, x, NC,
                     H, W, P, Q, y);
}

void avgpool2d_adaptive_bwd(const float* dy, int NC, int H, int W, int P, int Q, float* dx,
                            hipStream_t st) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(ew_grid((long)NC * H * W)), dim3(256), 0, st, dy,
                     NC, H, W, P, Q, dx);
}

void dropout_apply(const float* x, long n, float p, uint64_t seed, float* y, hipStream_t st) {
  hipLaunchKernelGGL(dropout_kernel, dim3(ew_grid(n)), dim3(256), 0, st, x, n, p, seed, y);
}

void add_relu(const float* a, const float* b, long n, bool relu, float* y, hipStream_t st) {
  if (vec4_ok(n, {a, b, y})) {
    hipLaunchKernelGGL(add_relu4_kernel, dim3(ew_grid(n / 4)), dim3(256), 0, st,
                       (const f32x4*)a, (const f32x4*)b, n / 4, relu ? 1 : 0, (f32x4*)y);
    return;
  }
  hipLaunchKernelGGL(add_relu_kernel, dim3(ew_grid(n)), dim3(256), 0, st, a, b, n, relu ? 1 : 0,
                     y);
}

void maxpool2d_nhwc_fwd(const float* x, int N, int H, int W, int C, int P, int Q, int k, int s,
                        int pad, float* y, int* idx, hipStream_t st) {
  if (vec4_ok((long)C, {x, y, idx})) {
    hipLaunchKernelGGL(maxpool_nhwc_fwd4_kernel, dim3(ew_grid((long)N * P * Q * C / 4)),
                       dim3(256), 0, st, (const f32x4*)x, N, H, W, C / 4, P, Q, k, s, pad,
                       (f32x4*)y, (i32x4*)idx);
    return;
  }
  hipLaunchKernelGGL(maxpool_nhwc_fwd_kernel, dim3(ew_grid((long)N * P * Q * C)), dim3(256), 0,
                     st, x, N, H, W, C, P, Q, k, s, pad, y, idx);
}

void maxpool2d_nhwc_bwd(const float* dy, const int* idx, int N, int H, int W, int C, int P, int Q,
                        int k, int s, int pad, float* dx, hipStream_t st) {
  if (vec4_ok((long)C, {dy, idx, dx})) {
    hipLaunchKernelGGL(maxpool_nhwc_bwd4_kernel, dim3(ew_grid((long)N * H * W * C / 4)),
                       dim3(256), 0, st, (const f32x4*)dy, (const i32x4*)idx, N, H, W, C / 4, P,
                       Q, k, s, pad, (f32x4*)dx);
    return;
  }
  hipLaunchKernelGGL(maxpool_nhwc_bwd_kernel, dim3(ew_grid((long)N * H * W * C)), dim3(256), 0,
                     st, dy, idx, N, H, W, C, P, Q, k, s, pad, dx);
}

void avgpool2d_nhwc_fwd(const float* x, int N, int H, int W, int C, int P, int Q, float* y,
                        hipStream_t st) {
  hipLaunchKernelGGL(avgpool_nhwc_fwd_kernel, dim3(ew_grid((long)N * P * Q * C)), dim3(256), 0,
                     st, x, N, H, W, C, P, Q, y);
}

void avgpool2d_nhwc_bwd(const float* dy, int N, int H, int W, int C, int P, int Q, float* dx,
                        hipStream_t st) {
  hipLaunchKernelGGL(avgpool_nhwc_bwd_kernel, dim3(ew_grid((long)N * H * W * C)), dim3(256), 0,
                     st, dy, N, H, W, C, P, Q, dx);
}

void relu_mask(const float* dy, const float* y, long n, float* g, hipStream_t st) {
  if (vec4_ok(n, {dy, y, g})) {
    hipLaunchKernelGGL(relu_mask4_kernel, dim3(ew_grid(n / 4)), dim3(256), 0, st,
                       (const f32x4*)dy, (const f32x4*)y, n / 4, (f32x4*)g);
    return;
  }
  hipLaunchKernelGGL(relu_mask_kernel, dim3(ew_grid(n)), dim3(256), 0, st, dy, y, n, g);
}

}  // namespace tdp
