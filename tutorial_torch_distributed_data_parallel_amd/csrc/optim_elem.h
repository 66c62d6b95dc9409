// Per-element optimizer updates shared by the flat / multi-tensor optimizer kernels (optim.hip)
// and the weight-gradient GEMM epilogue that applies the update in place of storing the gradient
// (gemm_f32_fast.hip, OptEpilogue). Semantics are torch's: TORCH/optim/sgd.py (momentum buffer
// initialised to the first gradient, dampening, nesterov, maximize, L2 weight decay) and
// TORCH/optim/adam.py (bias-corrected, L2 vs decoupled weight decay, amsgrad).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace tdp {

// Take the per-step scalars from the device hyper block when there is one (kernels.h HyperSlot).
// Uniform loads at kernel start; the structural flags stay as launched.
__device__ __forceinline__ void load_hyper(SgdHyper& h) {
  const float* d = h.dev;
  if (d == nullptr) return;
  h.lr = d[kHLr];
  if (h.momentum != 0.f) h.momentum = d[kHMom];  // zero momentum is structural (no buffer)
  h.dampening = d[kHDamp];
  h.weight_decay = d[kHWd];
  h.first_step = d[kHFirst] != 0.f;
  h.grad_scale *= d[kHScale];
}

__device__ __forceinline__ void load_hyper(AdamHyper& h) {
  const float* d = h.dev;
  if (d == nullptr) return;
  h.lr = d[kHLr];
  h.beta1 = d[kHMom];
  h.beta2 = d[kHDamp];
  h.weight_decay = d[kHWd];
  h.eps = d[kHEps];
  h.bc1 = d[kHBc1];
  h.bc2_sqrt = d[kHBc2];
  h.grad_scale *= d[kHScale];
}

__device__ __forceinline__ void sgd_elem(float& p, float g, float& b, const SgdHyper& h) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
  if (h.momentum != 0.f) {
    b = h.first_step ? g : fmaf(b, h.momentum, (1.f - h.dampening) * g);
    g = h.nesterov ? fmaf(h.momentum, b, g) : b;
  }
  p = fmaf(-h.lr, g, p);
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float* vmax,
                                          const AdamHyper& h) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if (h.weight_decay != 0.f) {
    if (h.decoupled) p *= (1.f - h.lr * h.weight_decay);
    else g = fmaf(h.weight_decay, p, g);
  }
  m = fmaf(1.f - h.beta1, g - m, m);  // lerp(m, g, 1-beta1)
  v = fmaf(v, h.beta2, (1.f - h.beta2) * g * g);
  float vv = v;
  if (h.amsgrad) {
    vv = fmaxf(*vmax, v);
    *vmax = vv;
  }
  const float denom = sqrtf(vv) / h.bc2_sqrt + h.eps;
  p = fmaf(-(h.lr / h.bc1), m / denom, p);
}

}  // namespace tdp
