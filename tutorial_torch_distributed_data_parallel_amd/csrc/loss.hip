// Fused cross-entropy (log_softmax + nll_loss) forward/backward and the eval accuracy count.
//
// Replaces the reference's nn.CrossEntropyLoss (REF/multi-GPU-training-torch.py:248, SURVEY.md
// §2.5 K15/K16) and the `torch.max(outputs.data, 1)` + `(predicted == labels).sum().item()`
// accuracy bookkeeping of evaluate() (REF/multi-GPU-training-torch.py:149-151, K27). Per-step
// metrics are accumulated on the device (acc[0] loss sum, acc[1] correct, acc[2] rows) instead of
// the reference's `loss.item()` host sync every iteration (K28).
//
// Semantics follow torch.nn.functional.cross_entropy with class-index targets: ignore_index rows
// contribute nothing and are excluded from the mean's denominator; label_smoothing eps mixes
// (1-eps)*nll with eps*mean_c(-log p_c).
#include "ce_row.h"
#include "common.h"
#include "kernels.h"

namespace tdp {
namespace {

// One row handled by a whole wave (large C).
__device__ RowOut row_wave(const float* x, int C, int64_t y, int ignore_index, float eps) {
  const int lane = threadIdx.x & 63;
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  float sumx = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = x[c];
    if (v > mx) { mx = v; arg = c; }
    sumx += v;
  }
  // argmax with lowest index on ties (torch.max semantics on the first maximal element)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  sumx = wave_sum(sumx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(x[c] - mx);
  se = wave_sum(se);
  RowOut o;
  o.lse = mx + __logf(se);
  const bool valid = (y != ignore_index) && y >= 0 && y < C;
  o.valid = valid ? 1.f : 0.f;
  o.loss = valid ? (o.lse - (1.f - eps) * x[y] - (eps / C) * sumx) : 0.f;
  o.correct = (valid && arg == (int)y) ? 1.f : 0.f;
  return o;
}

// Single-workgroup fused forward: deterministic reduction, one launch.
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ labels, int B,
                                                     int C, long ld, int ignore_index, float eps,
                                                     int mean, float* out_loss, float* lse,
                                                     float* acc, int count_only,
                                                     float* __restrict__ dpre) {
  __shared__ float red[4];
  float ls = 0.f, cr = 0.f, vd = 0.f;
  if (C <= 32 && B <= 256) {
    // one row per lane (a classifier head at batch <= 256): the three sums in ONE cross-wave
    // reduction, the logits gradient written from the lane's own lse (no re-read of lse[],
    // no second pass over the batch) -- ~half the latency of the general path
    __shared__ float red3[4][3];
    const int r = threadIdx.x;
    RowOut o{0.f, 0.f, 0.f, 0.f};
    int64_t y = ignore_index;
    if (r < B) {
      y = labels[r];
      o = row_serial(logits + (long)r * ld, C, y, ignore_index, eps);
      if (lse) lse[r] = o.lse;
    }
    ls = wave_sum(o.loss);
    cr = wave_sum(o.correct);
    vd = wave_sum(o.valid);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
      red3[wid][0] = ls;
      red3[wid][1] = cr;
      red3[wid][2] = vd;
    }
    __syncthreads();
    ls = red3[0][0] + red3[1][0] + red3[2][0] + red3[3][0];
    cr = red3[0][1] + red3[1][1] + red3[2][1] + red3[3][1];
    vd = red3[0][2] + red3[1][2] + red3[2][2] + red3[3][2];
    if (dpre && r < B) {
      const float g = mean ? 1.f / vd : 1.f;
      const bool valid = o.valid != 0.f;
      const float* x = logits + (long)r * ld;
      for (int c = 0; c < C; ++c) {
        float v = 0.f;
        if (valid) {
          const float pr = __expf(x[c] - o.lse);
          v = g * (pr - (c == (int)y ? (1.f - eps) : 0.f) - eps / C);
        }
        dpre[r * C + c] = v;
      }
    }
    if (threadIdx.x == 0) {
      if (!count_only) {
        if (out_loss) out_loss[0] = mean ? (vd > 0.f ? ls / vd : NAN) : ls;
        if (lse) lse[B] = vd;
        if (acc) acc[0] += ls;
      }
      if (acc) { acc[1] += cr; acc[2] += vd; }
    }
    return;
  }
  if (C <= 32) {
    for (int r = threadIdx.x; r < B; r += 256) {
      const RowOut o = row_serial(logits + (long)r * ld, C, labels[r], ignore_index, eps);
      if (lse) lse[r] = o.lse;
      ls += o.loss; cr += o.correct; vd += o.valid;
    }
  } else {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int r = wid; r < B; r += 4) {
      const RowOut o = row_wave(logits + (long)r * ld, C, labels[r], ignore_index, eps);
      if (lane == 0) {
        if (lse) lse[r] = o.lse;
        ls += o.loss; cr += o.correct; vd += o.valid;
      }
    }
  }
  ls = block_sum<256>(ls, red);
  cr = block_sum<256>(cr, red);
  vd = block_sum<256>(vd, red);
  if (dpre) {
    // the logits gradient for an upstream gradient of exactly 1 (the loss.backward() seed):
    // the backward then needs no kernel (ops/loss.py). lse[r] was written by this workgroup
    // before block_sum's barriers.
    const float g = mean ? 1.f / vd : 1.f;
    for (int i = threadIdx.x; i < B * C; i += 256) {
      const int r = i / C, c = i % C;
      const int64_t y = labels[r];
      const bool valid = (y != ignore_index) && y >= 0 && y < C;
      float v = 0.f;
      if (valid) {
        const float p = __expf(logits[(long)r * ld + c] - lse[r]);
        v = g * (p - (c == (int)y ? (1.f - eps) : 0.f) - eps / C);
      }
      dpre[i] = v;
    }
  }
  if (threadIdx.x == 0) {
    if (!count_only) {
      if (out_loss) out_loss[0] = mean ? (vd > 0.f ? ls / vd : NAN) : ls;
      if (lse) lse[B] = vd;  // denominator for the backward
      if (acc) acc[0] += ls;
    }
    if (acc) { acc[1] += cr; acc[2] += vd; }
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ gout, int B, int C,
                                                     long ld, int ignore_index, float eps,
                                                     int mean, float* __restrict__ d) {
  const long total = (long)B * C;
  const float g = gout[0] * (mean ? 1.f / lse[B] : 1.f);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i % C);
    const int64_t y = labels[r];
    const bool valid = (y != ignore_index) && y >= 0 && y < C;
    float v = 0.f;
    if (valid) {
      const float p = __expf(logits[(long)r * ld + c] - lse[r]);
      v = g * (p - (c == (int)y ? (1.f - eps) : 0.f) - eps / C);
    }
    d[(long)r * C + c] = v;
  }
}

}  // namespace

void cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, long ld,
                       int ignore_index, float label_smoothing, bool mean, float* out_loss,
                       float* lse_out, float* acc, hipStream_t s, float* dpre) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, s, logits, labels, B, C, ld,
                     ignore_index, label_smoothing, mean ? 1 : 0, out_loss, lse_out, acc, 0,
                     dpre);
}

void cross_entropy_bwd(const float* logits, const int64_t* labels, const float* lse,
                       const float* gout, int B, int C, long ld, int ignore_index,
                       float label_smoothing, bool mean, float* dlogits, hipStream_t s) {
  const long total = (long)B * C;
  int grid = (int)((total + 255) / 256);
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(grid), dim3(256), 0, s, logits, labels, lse, gout, B, C,
                     ld, ignore_index, label_smoothing, mean ? 1 : 0, dlogits);
}

void count_correct(const float* logits, const int64_t* labels, int B, int C, long ld, float* acc,
                   hipStream_t s) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, s, logits, labels, B, C, ld, -100,
                     0.f, 0, (float*)nullptr, (float*)nullptr, acc, 1, (float*)nullptr);
}

}  // namespace tdp
