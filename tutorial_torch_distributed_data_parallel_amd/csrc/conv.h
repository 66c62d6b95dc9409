// Implicit-GEMM convolution API (see conv.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tdp {

constexpr int kConvFwd = 0, kConvDgrad = 1, kConvWgrad = 2;

// x: [N][C][H][W], w: [Cout][C][R][S], y: [N][Cout][P][Q]
struct ConvGeom {
  int N, C, H, W, Cout, R, S, P, Q, sh, sw, ph, pw;
};

struct ConvPlan {
  int mode = 0;
  int M = 0, N = 0, K = 0;
  int fm = 2, fn = 2;
  int bm = 128;  // NHWC fast path: block rows (128, or 256 = FM 4 for K-contiguous A)
  int splits = 1, k_per_split = 0;
  long ws_floats = 0;
};

ConvPlan conv_plan(int mode, const ConvGeom& g, int num_cus);
// FWD: A = w, B = x, C = y (bias/relu epilogue); DGRAD: A = w, B = dy, C = dx;
// WGRAD: A = dy, B = x, C = dw (C += beta * old when beta != 0).
void conv_run(const ConvPlan& pl, const ConvGeom& g, const float* A, const float* B, float* C,
              const float* bias, bool relu, float beta, float* ws, hipStream_t s);

// NHWC implicit GEMM on the LDS-DMA MFMA pipeline (gemm_f32_fast.hip). Requires C % 4 == 0,
// Cout % 4 == 0 and (for DGRAD) power-of-two strides; plan.fm holds the pipeline depth.
bool conv_nhwc_ok(int mode, const ConvGeom& g);
// weight gradient computed as dW^T [R*S*C][Cout] (small Cout: keeps the 128-row tiles full)
bool conv_wgrad_transposed(const ConvGeom& g);
void conv_set_wgrad_transposed(int mode);  // -1 auto, 0 / 1 force
void conv_set_wgrad_target(int per_cu);     // split-K workgroups per CU (<= 0: auto)
// measured (FN, split-K) per exact geometry + pass (gemm_f32_fast.hip "plan table")
void conv_plan_db_put(int mode, const ConvGeom& g, int fn, int splits);
void conv_plan_db_clear();
long conv_plan_db_size();
ConvPlan conv_nhwc_plan(int mode, const ConvGeom& g, int num_cus);
// Input gradient with B read from the weight's own [Cout][R][S][C] storage (no transposed copy):
// the (phase) taps of the full R x S filter, (r, s) = (r0 + rp*sh, s0 + sp*sw); see WTap.
struct WeightTaps {
  int R, S, r0, s0, sh, sw;
};
// stats (optional, forward only): [tiles_m][3][N] per-tile column (count, mean, M2) of the
// output, written when the plan is unsplit with the row-vector epilogue and no bias / ReLU /
// beta; returns whether it was written
bool conv_nhwc_run(const ConvPlan& pl, const ConvGeom& g, const float* A, const float* B,
                   float* C, const float* bias, bool relu, float beta, float* ws,
                   hipStream_t s, const WeightTaps* wtap = nullptr, float* stats = nullptr);

// NCHW ReLU backward + per-channel bias gradient: g = dy*(y>0) (if y), db = sum over n,hw.
int chan_splits(int N, int C, int HW, int num_cus);
void chan_relu_bias_bwd(const float* dy, const float* y, int N, int C, int HW, float* g,
                        float* db, float beta, float* part, int splits, hipStream_t s);

}  // namespace tdp
