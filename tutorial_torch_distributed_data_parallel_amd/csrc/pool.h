// Pooling / dropout / residual elementwise API (see pool.hip). NC = N*C planes of HxW -> PxQ.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdp {
void maxpool2d_fwd(const float* x, int NC, int H, int W, int P, int Q, int k, int s, int pad,
                   float* y, int* idx, hipStream_t st);
void maxpool2d_bwd(const float* dy, const int* idx, int NC, int H, int W, int P, int Q, int k,
                   int s, int pad, float* dx, hipStream_t st);
void avgpool2d_adaptive_fwd(const float* x, int NC, int H, int W, int P, int Q, float* y,
                            hipStream_t st);
void avgpool2d_adaptive_bwd(const float* dy, int NC, int H, int W, int P, int Q, float* dx,
                            hipStream_t st);
// y = x * keep / (1-p), keep = hash(seed, i) >= p * 2^32   (the backward re-applies the same mask)
void dropout_apply(const float* x, long n, float p, uint64_t seed, float* y, hipStream_t st);
void add_relu(const float* a, const float* b, long n, bool relu, float* y, hipStream_t st);
void relu_mask(const float* dy, const float* y, long n, float* g, hipStream_t st);
// NHWC (channels_last) pooling; idx holds h*W+w of the window maximum
void maxpool2d_nhwc_fwd(const float* x, int N, int H, int W, int C, int P, int Q, int k, int s,
                        int pad, float* y, int* idx, hipStream_t st);
void maxpool2d_nhwc_bwd(const float* dy, const int* idx, int N, int H, int W, int C, int P, int Q,
                        int k, int s, int pad, float* dx, hipStream_t st);
void avgpool2d_nhwc_fwd(const float* x, int N, int H, int W, int C, int P, int Q, float* y,
                        hipStream_t st);
void avgpool2d_nhwc_bwd(const float* dy, int N, int H, int W, int C, int P, int Q, float* dx,
                        hipStream_t st);
}  // namespace tdp
