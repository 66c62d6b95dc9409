// Host API of the bf16-split-planes kernels (csrc/gemm_planes.hip): the skinny GEMM that reads
// its activation operand as exact bf16 hi / mid / lo planes, and the producers of such planes.
#pragma once
#include "kernels.h"

namespace tdp {

// Skinny-M fp32 GEMM from pre-split bf16 planes of A (csrc/gemm_planes.hip):
//   C[M,N] = A[M,K] . op(B)[K,N] (+bias)(ReLU)(* (gate > 0)), A given as its exact bf16 split
//   planes Ap [3][M][K] (x = hi + mid + lo, plane stride ps, row stride lda; split_planes or a
//   producer's epilogue makes them), B fp32 [N][K] (b_kcontig) or [K][N]. K % 32 == 0.
//   out_planes (optional): the planes of the finished C ([3][M][N], plane stride out_ps) for the
//   next skinny GEMM that reads C as its A.
struct GemmPlanesArgs {
  const uint16_t* Ap = nullptr;
  long ps = 0, lda = 0;
  const float* B = nullptr;
  long ldb = 0;
  bool b_kcontig = true;
  float* C = nullptr;
  long ldc = 0;
  const float* bias = nullptr;
  bool relu = false;
  const float* gate = nullptr;
  long ldgate = 0;
  uint16_t* out_planes = nullptr;
  long out_ps = 0;
  int M = 0, N = 0, K = 0;
};
bool gemm_planes_ok(const GemmPlanesArgs& a);
GemmPlan gemm_planes_plan(const GemmPlanesArgs& a, int num_cus);
// measurements: pipeline stages (2 | 3), B prefetch distance (2 stages only), split-K override
// (0 = planned); returns false (and changes nothing) for an invalid combination
bool gemm_planes_set_cfg(int stages, int pf, int splits);
void gemm_planes_run(const GemmPlanesArgs& a, const GemmPlan& plan, float* ws, hipStream_t s);
// x [rows][cols] (row stride ldx, cols % 4 == 0) -> planes [3][rows][cols] (plane stride ps)
void split_planes(const float* x, long ldx, int rows, int cols, uint16_t* planes, long ps,
                  hipStream_t s);

// gather_batch (kernels.h) that also writes the planes of the gathered rows: planes [3][B][F]
// (plane stride B*F), F % 4 == 0. cursor (optional, int64 [2] = {position, 0}): the batch is
// idx[cursor[0] .. + B) and the kernel advances cursor[0] by B (a captured step reads the next
// batch of the epoch's order at every replay). row_counters: the cursor is int64 [2 + B] (zeros
// after the first two), per-row arrival counters that let several workgroups share a row
void gather_batch_planes(const float* x, const int64_t* y, const int64_t* idx, long n, long F,
                         int B, float* xb, int64_t* yb, uint16_t* planes, hipStream_t s,
                         int64_t* cursor = nullptr, long nidx = 0, bool row_counters = false);

// Backward of a head Linear(I -> O <= 16) in one launch (csrc/gemm_skinny.hip): dx = g . W
// (gated by gate > 0 when given, planes of dx when dxp != null), dW = g^T . x, db = sum_b g
// (when db != null). g [B][O], x [B][I], W [O][I]; I % 4 == 0, 16-B aligned W / dx / gate rows.
// dx == null: no input gradient (head_ce computed it in the forward).
// wopt / bopt (kind != 0): apply that optimizer update to W / b instead of storing dW / db.
// false = shape not supported (nothing launched).
bool head_bwd(const float* g, long ldg, const float* x, long ldx, const float* w, long ldw,
              float* dx, long lddx, const float* gate, long ldgate, uint16_t* dxp, long dxps,
              float* dw, long lddw, float* db, int B, int O, int I, hipStream_t s,
              const OptEpilogue* wopt = nullptr, const OptEpilogue* bopt = nullptr);

// Forward of a head Linear(I -> O <= 16) + cross-entropy in one launch (csrc/gemm_skinny.hip
// head_ce_kernel, B <= 256 rows): logits [B][O], lse [B + 1] (lse[B] = valid rows), loss, the
// metric accumulator acc [3] (optional); with dpre (training): the logits gradient for a unit
// upstream gradient and, with dx, the input gradient dlogits . W (gated by gate > 0, planes into
// dxp when given). rowbuf [B][4] scratch; ticket: 9 zeroed unsigned words, zero again afterwards.
// false = shape not supported (nothing launched).
bool head_ce(const float* x, long ldx, const float* w, long ldw, const float* bias,
             const int64_t* labels, int B, int O, int I, int ignore_index, float smoothing,
             bool mean, float* logits, float* lse, float* rowbuf, unsigned* ticket, float* loss,
             float* acc, float* dpre, float* dx, long lddx, const float* gate, long ldgate,
             uint16_t* dxp, long dxps, hipStream_t s);

}  // namespace tdp
