// Host-side launch API of the hand-written gfx950 kernels.
//
// These functions take raw device pointers plus the HIP stream to launch on; they never allocate,
// copy or synchronise (workspaces are passed in), so bindings.cpp can wrap them for PyTorch
// tensors and every launch stays hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace tdp {

// ------------------------------------------------------------------------------------------------
// Optimizer hyper-parameters (fused single-pass updates, csrc/optim.hip + optim_elem.h)
// ------------------------------------------------------------------------------------------------
//
// Device-resident hyper-parameter block ("hyper block": kHSlots floats in device memory, one per
// optimizer parameter group). A kernel whose SgdHyper / AdamHyper has `dev != nullptr` takes the
// per-step scalars from the block instead of its by-value fields, so a step captured into a
// hipGraph replays with the CURRENT learning rate, Adam step count and bias corrections: the host
// rewrites the block with a stream-ordered copy when a hyper-parameter changes, opt_step_begin()
// advances the step counter / bias corrections / SGD first-step flag on the device, and the
// gradient-clipping kernels leave their coefficient in kHScale. The structural flags (nesterov,
// maximize, amsgrad, decoupled, momentum == 0) stay by-value: changing them needs a re-capture.
enum HyperSlot : int {
  kHLr = 0,
  kHMom = 1,        // SGD momentum | Adam beta1
  kHDamp = 2,       // SGD dampening | Adam beta2
  kHWd = 3,         // weight decay
  kHEps = 4,        // Adam eps
  kHBc1 = 5,        // Adam 1 - beta1^t          (written by opt_step_begin)
  kHBc2 = 6,        // Adam sqrt(1 - beta2^t)    (written by opt_step_begin)
  kHFirst = 7,      // SGD: momentum buffers are initialised by this step (1/0)
  kHFirstNext = 8,  // host request: the next step initialises the momentum buffers
  kHScale = 9,      // gradient multiplier of this step (clip coefficient; 1 = none)
  kHSumsq = 10,     // squared-gradient-norm accumulator of this step
  kHMaxNorm = 11,   // clip threshold (<= 0: no clipping)
  kHStep = 12,      // int32: optimizer step count t (advanced by opt_step_begin)
  kHNorm = 13,      // total gradient norm of the last clipped step (for the caller)
  kHPartials = 16,  // workspace: per-workgroup partial sums of the deterministic norm reduction
  kHPartialsMax = 1024,
  kHSlots = kHPartials + kHPartialsMax
};

struct SgdHyper {
  float lr, momentum, dampening, weight_decay;
  bool nesterov, maximize, first_step;
  float grad_scale;  // grads are multiplied by this first (1/world for sum-reduced grads)
  const float* dev = nullptr;  // hyper block (kHLr.. kHScale override the fields above)
};

struct AdamHyper {
  float lr, beta1, beta2, eps, weight_decay;
  bool amsgrad, maximize, decoupled;  // decoupled = AdamW
  float bc1, bc2_sqrt;                // 1-beta1^t, sqrt(1-beta2^t)
  float grad_scale;
  const float* dev = nullptr;  // hyper block (see HyperSlot)
};

// Advance a hyper block by one optimizer step (one thread): step += 1, Adam bias corrections for
// the new step (kind 2), first-step flag from the host request, clip accumulators reset.
void opt_step_begin(float* dev, int kind, hipStream_t s);
// one-lane empty kernel on s (a graph node; see reducer.cpp pick_stream)
// Global-norm clipping on the device: kHNorm = sqrt(kHSumsq) and
// kHScale = min(1, kHMaxNorm / (kHNorm + 1e-6)) (torch.nn.utils.clip_grad_norm_ semantics).
void clip_coef_from_sumsq(float* dev, hipStream_t s);
// kHSumsq += sum of squares of x[begin[i] : begin[i] + len[i]) for every range (one launch)
struct RangeSet;
void sumsq_ranges(const float* x, const RangeSet& r, float* dev, hipStream_t s);
// x[ranges] *= dev[kHScale] (per-rank clip before aggregation)
void scale_ranges_by(float* x, const RangeSet& r, const float* dev, hipStream_t s);

// Optimizer update applied by a GEMM epilogue in place of storing the result: when C is a weight
// gradient, the epilogue reads p / state at C's element index (same layout and leading dimension
// as C), updates them and never writes C. Used for the weight-gradient GEMMs when the gradient
// needs no cross-rank reduction (world size 1): it removes the gradient's HBM write + re-read and
// overlaps the update's memory traffic with the GEMM's MFMA work.
struct OptEpilogue {
  int kind = 0;  // 0 none, 1 SGD, 2 Adam
  float* p = nullptr;
  float* s0 = nullptr;  // momentum buffer / exp_avg
  float* s1 = nullptr;  // exp_avg_sq
  float* s2 = nullptr;  // max_exp_avg_sq
  SgdHyper sgd{};
  AdamHyper adam{};
};

// ------------------------------------------------------------------------------------------------
// fp32 GEMM on v_mfma_f32_32x32x2_f32 (exact f32, the dtype of the reference's nn.Linear).
//   C[M,N] = op(A)[M,K] . op(B)[K,N]  (+ bias[N]) (+ beta*C) (ReLU)
//   a_kcontig: A stored [M][K] (else [K][M]);  b_kcontig: B stored [N][K] (else [K][N]).
//   mask (optional, A's layout, leading dim ldmask): A is replaced by 0 where mask <= 0 -- the
//   ReLU backward of the layer that produced `mask`, fused into the operand load.
//   rowsum (optional, [M]): rowsum = rowsum_beta*rowsum + sum_k A[m,k] (bias gradient).
// ------------------------------------------------------------------------------------------------
struct GemmF32Args {
  const float* A = nullptr;
  const float* B = nullptr;
  float* C = nullptr;
  const float* mask = nullptr;
  const float* bias = nullptr;
  float* rowsum = nullptr;
  long lda = 0, ldb = 0, ldc = 0, ldmask = 0;
  int M = 0, N = 0, K = 0;
  bool a_kcontig = true, b_kcontig = true;
  float beta = 0.f, rowsum_beta = 0.f;
  bool relu = false;
  OptEpilogue opt;  // kind != 0: apply the optimizer instead of storing C (needs splits == 1)
  // with opt and rowsum (rowsum_beta == 0): also apply the optimizer to the bias elements at
  // bias_opt's pointers with the row sums as their gradient, instead of storing rowsum (the
  // layer's bias update rides on the weight-gradient GEMM; hyper-parameters are opt's)
  OptEpilogue bias_opt;
  // optional C-shaped gate, applied last: C = epilogue(C) * (gate > 0). The input gradient of a
  // Linear whose input is a ReLU output leaves already masked, so the producer's backward
  // needs no separate mask pass (ops/linear.py)
  const float* gate = nullptr;
  long ldgate = 0;
};

struct GemmPlan {
  bool fast = false;    // LDS-DMA pipelined kernel (gemm_f32_fast.hip) vs generic
  bool lockstep = false;  // optimizer epilogue by wgrad_lockstep_kernel (gemm_f32_fast.hip)
  int tile = 0;         // generic: tile-table index; fast: FN (block tile 128 x 64*FN)
  int bm = 128, bn = 64;
  int stages = 2;       // fast kernel pipeline depth
  int splits = 1;
  int k_per_split = 0;
  long ws_floats = 0;   // split-K workspace needed (0 when splits == 1)
  int skinny = 0;       // > 0: one of the skinny kernels (gemm_skinny.hip) runs instead
  int grid = 0;         // fast kernel: > 0 = persistent launch of this many workgroups
  bool emu8 = false;    // the 256 x 256 split-bf16 kernel (gemm_emu8.hip) runs instead
};

GemmPlan gemm_f32_plan(const GemmF32Args& a, int num_cus);
// C[M][N] = 0 where !(gate > 0) (the generic GEMM path's gate epilogue)
void gate_inplace(float* C, long ldc, const float* gate, long ldg, int M, int N, hipStream_t s);
void gemm_f32_run(const GemmF32Args& a, const GemmPlan& plan, float* ws, hipStream_t s);
bool gemm_f32_fast_ok(const GemmF32Args& a);
// skinny GEMM kind for a dimension <= 16 (1: N, 2: K, 3: M; 0: not applicable), and its launch
int gemm_skinny_kind(const GemmF32Args& a);
void gemm_skinny_run(int kind, const GemmF32Args& a, hipStream_t s);
// C (contiguous, ldc == N) holds a finished gradient: apply a.opt as a flat update over it
void gemm_opt_fallback(const GemmF32Args& a, hipStream_t s);
void gemm_f32_fast_plan(const GemmF32Args& a, int num_cus, GemmPlan& plan);
void gemm_f32_fast_run(const GemmF32Args& a, const GemmPlan& plan, float* ws, hipStream_t s);
// two weight-gradient + optimizer GEMMs (both with a.opt) in one persistent launch, when their
// plans allow it (gemm_f32_fast_pair_ok: the default epilogue variants, persistent 128 x 128)
bool gemm_f32_fast_pair_ok(const GemmF32Args& a1, const GemmPlan& p1, const GemmF32Args& a2,
                           const GemmPlan& p2);
void gemm_f32_fast_run_pair(const GemmF32Args& a1, const GemmPlan& p1, const GemmF32Args& a2,
                            const GemmPlan& p2, hipStream_t s);
void gemm_f32_set_lockstep(bool on);  // A/B: false = the persistent epilogue kernel
bool gemm_f32_lockstep();
// set by tests/benchmarks: 0 = auto, 1 = force generic kernel, 2 = force fast kernel
void gemm_f32_set_mode(int mode);
// benchmarking knob: force the fast kernel's tile width / split-K / stages (0 = planner's choice)
void gemm_f32_set_override(int fn, int splits, int stages);
// row-vector (LDS-staged, 16-B) output stores of the fast GEMM on / off (measurements, tests)
void gemm_f32_set_cvec(bool on);
// fast GEMM products: split-bf16 emulation on the bf16 matrix core (default) or native f32 MFMA
void gemm_f32_set_emu(bool on);
bool gemm_f32_emu();
// fast-GEMM block rows: 0 auto, 128 or 256 forced (measurements, tests)
void gemm_f32_set_bm(int bm);
// optimizer-epilogue variant (SGD flags, Adam flags, persistent grid on/off, workgroups per CU);
// negative = keep. Returns the active {sgd, adam, persist, wgs}.
std::vector<int> gemm_f32_set_opt_variant(int sgd, int adam, int persist, int wgs);

// bf16-operand GEMM (AMP path): same contract, A/B bf16 (uint16 storage), C fp32 or bf16.
struct GemmBF16Args {
  const uint16_t* A = nullptr;
  const uint16_t* B = nullptr;
  void* C = nullptr;
  bool c_bf16 = false;
  const uint16_t* mask = nullptr;
  const float* bias = nullptr;
  float* rowsum = nullptr;
  long lda = 0, ldb = 0, ldc = 0, ldmask = 0;
  int M = 0, N = 0, K = 0;
  bool a_kcontig = true, b_kcontig = true;
  float beta = 0.f, rowsum_beta = 0.f;
  bool relu = false;
};
GemmPlan gemm_bf16_plan(const GemmBF16Args& a, int num_cus);
void gemm_bf16_run(const GemmBF16Args& a, const GemmPlan& plan, float* ws, hipStream_t s);

// split-K combine + epilogue: C = epi(sum_z ws[z]) ; C fp32 or bf16
void splitk_reduce(const float* ws, int splits, int M, int N, void* C, bool c_bf16, long ldc,
                   const float* bias, float beta, bool relu, hipStream_t s,
                   const float* gate = nullptr, long ldgate = 0);

// ------------------------------------------------------------------------------------------------
// Loss / metrics
// ------------------------------------------------------------------------------------------------
// Fused cross-entropy forward over logits[B,C] (fp32), int64 labels.
//   out_loss[0] = mean (or sum) loss over non-ignored rows; also optional device accumulators:
//   acc[0] += sum loss, acc[1] += #correct (argmax == label), acc[2] += #counted rows.
//   lse_out[B] (optional) saves log-sum-exp per row for the backward.
void cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, long ld,
                       int ignore_index, float label_smoothing, bool mean, float* out_loss,
                       float* lse_out, float* acc, hipStream_t s, float* dpre = nullptr);
// dlogits = gout[0] * d(loss)/d(logits)
void cross_entropy_bwd(const float* logits, const int64_t* labels, const float* lse,
                       const float* gout, int B, int C, long ld, int ignore_index,
                       float label_smoothing, bool mean, float* dlogits, hipStream_t s);
// argmax/correct counting only (eval): acc[1] += correct, acc[2] += rows
void count_correct(const float* logits, const int64_t* labels, int B, int C, long ld, float* acc,
                   hipStream_t s);

// ------------------------------------------------------------------------------------------------
// Optimizers: fused single-pass updates over a flat arena or a multi-tensor chunk table.
// ------------------------------------------------------------------------------------------------
void sgd_flat(float* p, const float* g, float* buf, long n, const SgdHyper& h, hipStream_t s);
// Up to kMaxRanges disjoint element ranges [begin, begin + len) of equally laid out flat buffers
// (parameter / gradient / state arenas), updated by ONE launch (the world-size-1 reducer collects
// every range the weight-gradient epilogues did not already update).
constexpr int kMaxRanges = 16;
struct RangeSet {
  int n = 0;
  long begin[kMaxRanges];
  long len[kMaxRanges];
};
void sgd_ranges(float* p, const float* g, float* buf, const RangeSet& r, const SgdHyper& h,
                hipStream_t s);
void adam_ranges(float* p, const float* g, float* m, float* v, float* vmax, const RangeSet& r,
                 const AdamHyper& h, hipStream_t s);

void adam_flat(float* p, const float* g, float* m, float* v, float* vmax, long n,
               const AdamHyper& h, hipStream_t s);

// Multi-tensor form: `table` is a device array of TensorChunk records.
struct TensorChunk {
  float* p;
  const float* g;
  float* s0;  // momentum buf / exp_avg
  float* s1;  // exp_avg_sq
  float* s2;  // max_exp_avg_sq
  long n;
};
void sgd_multi(const TensorChunk* table, int count, const SgdHyper& h, hipStream_t s);
void adam_multi(const TensorChunk* table, int count, const AdamHyper& h, hipStream_t s);

// elementwise helpers
void scale_inplace(float* x, long n, float a, hipStream_t s);
// ReLU backward + bias gradient in one pass over dy[B][N] (row stride ld):
//   g[B][N] = dy * (y > 0) (written only when y != null), db = beta_db*db + sum_rows(g).
//   `part` holds slices*N floats of column partial sums (slices from relu_bias_slices).
int relu_bias_slices(int B, int N, int num_cus);
// y = relu?(x + b) row-wise over [B][N] (N % 4 == 0, 16-B aligned rows and bias)
void bias_act_rows(const float* x, long ldx, const float* b, float* y, long ldy, int B, int N,
                   bool relu, hipStream_t s);
void relu_bias_bwd_ws(const float* dy, const float* y, int B, int N, long ld, float* g,
                      float* db, float beta_db, float* part, int slices, hipStream_t s,
                      float gscale = 1.f);  // g = gscale * dy * (y > 0) (db unscaled)
void fill_f32(float* x, long n, float v, hipStream_t s);
// 4-D strided copy over dst's logical shape; elements outside src's shape are written as 0
// (accumulate: dst += src, and elements outside src's shape are left alone)
struct Copy4D {
  long dsz[4], dst_stride[4], ssz[4], src_stride[4];
  bool accumulate;
};
void copy4d(const float* src, float* dst, const Copy4D& c, hipStream_t s);
// xb[b] = x[idx[b]] (rows of F floats), yb[b] = y[idx[b]]: a loader batch in one launch
void gather_batch(const float* x, const int64_t* y, const int64_t* idx, long n, long F, int B,
                  float* xb, int64_t* yb, hipStream_t s);
void f32_to_bf16_copy(const float* x, uint16_t* y, long n, hipStream_t s);
// gdst[0:ng) = alpha * g, xdst[0:nx) = x (ng, nx % 4 == 0, 16-B aligned): one launch
void factor_stage(const float* g, const float* x, float* gdst, float* xdst, long ng, long nx,
                  float alpha, hipStream_t s);
// uint8 [B][Hs][Ws][C] -> bilinear resize to Ho x Wo (align_corners=False), optional per-sample
// horizontal flip (flip[b] != 0), optional PIL-style rounding, /255, (v - mean) / std; output
// channels_last [B][Ho][Wo][C] or NCHW. C in {1, 3, 4}.
struct ImageNorm {
  float mean[4];
  float inv_std[4];
};
void image_transform(const uint8_t* x, const uint8_t* flip, float* out, int B, int Hs, int Ws,
                     int C, int Ho, int Wo, const ImageNorm& nrm, bool round_u8,
                     bool channels_last, hipStream_t s);
void bf16_to_f32_copy(const uint16_t* x, float* y, long n, hipStream_t s);

// ------------------------------------------------------------------------------------------------
// Batch norm (BatchNorm1d/2d and SyncBatchNorm). x is viewed as [N][C][HW] (HW = 1 for 1d).
// Reductions that need more parallelism than C workgroups split the N*HW axis into `splits`
// parts whose partials go to `ws` (bn_ws_floats tells how many floats it needs).
// ------------------------------------------------------------------------------------------------
int bn_splits(int N, int C, int HW, int num_cus);
long bn_ws_floats(int C, int splits);  // >= max(3C, 2C) * splits
// per-channel mean and biased variance (Welford per lane, Chan merges across lanes/blocks)
// (count_out, optional: the element count N*HW is written there -- the stats' third field)
void bn_moments(const float* x, int N, int C, int HW, int splits, float* ws, float* mean,
                float* var, float* count_out, hipStream_t s);
// merge R ranks' rows [mean(C) | var(C) | count(1)] (row stride 2C+1) -> mean, invstd, with the
// total count written at invstd[C] (callers pass invstd = mean + C of one [2C+1] stats buffer);
// running stats (optional) updated with momentum and the unbiased variance.
// num_batches (optional): BatchNorm's num_batches_tracked, incremented by the kernel
void bn_merge(const float* gathered, int R, int C, float eps, float momentum, float* mean,
              float* invstd, float* running_mean, float* running_var, int64_t* num_batches,
              hipStream_t s);
// y = (x - mean) * invstd * w + b (optional ReLU). w/b may be null (affine=False).
// residual (optional, [rows, C] form only): y = relu?(bn(x) + residual), the ResNet join
// mask_out (optional, [rows, C] form with relu): the ReLU mask as one byte per 4 channels (bit j =
// channel 4q+j > 0) -- what the backward reads instead of y (1/16 of the bytes)
// planes_out (optional, [rows, C] form): the output's bf16 split planes [3][rows][C] too
void bn_elemt(const float* x, const float* mean, const float* invstd, const float* w,
              const float* b, int N, int C, int HW, bool relu, float* y, hipStream_t s,
              const float* residual = nullptr, uint8_t* mask_out = nullptr,
              uint16_t* planes_out = nullptr);
// One rank (no gather): normalise [N][C] from this rank's moments [mean | var | count] and do
// bn_merge's work in the same launch (stats [mean | invstd | count] out, running stats, the
// batch counter). false = not the [rows, C % 4] form (nothing launched).
bool bn_elemt_local(const float* x, const float* moments, const float* w, const float* b, int N,
                    int C, bool relu, float eps, float momentum, float* stats, float* rmean,
                    float* rvar, int64_t* nbt, float* y, uint8_t* mask_out, uint16_t* planes_out,
                    hipStream_t s, const float* residual = nullptr);
// part [T][3][C] per-row-tile (count, mean, M2) -> mean, var (biased), count (= cnt): the
// moments of a convolution output whose forward GEMM epilogue produced them
void bn_moments_partials(const float* part, int T, int C, float* ws, float* mean, float* var,
                         float* count_out, float cnt, hipStream_t s);
long bn_partials_ws_floats(int T, int C);
// eval: y = (x - rmean) * rsqrt(rvar + eps) * w + b (optional ReLU)
void bn_eval(const float* x, const float* rmean, const float* rvar, const float* w,
             const float* b, int N, int C, int HW, float eps, bool relu, float* y, hipStream_t s);
// sums[0:C] = sum dy, sums[C:2C] = sum dy*(x-mean), with dy masked by (y > 0) when y != null
// (fused ReLU). dw/db (optional, accumulate when beta != 0): dw = sum_dy_xmu*invstd, db = sum_dy.
void bn_bwd_reduce(const float* dy, const float* x, const float* mean, const float* invstd,
                   const float* y_relu, int N, int C, int HW, int splits, float* ws, float* sums,
                   float* dw, float* db, float grad_beta, hipStream_t s,
                   const uint8_t* mask = nullptr);
// dx = w*invstd*(dy - sum_dy/cnt - (x-mean)*invstd^2*sum_dy_xmu/cnt), sums possibly all-reduced.
// dres (optional, [rows, C] form only): also write the masked dy -- the gradient of a fused
// residual input
void bn_bwd_elemt(const float* dy, const float* x, const float* mean, const float* invstd,
                  const float* w, const float* sums, const float* y_relu, const float* count,
                  int N, int C, int HW, float* dx, hipStream_t s, float* dres = nullptr,
                  const uint8_t* mask = nullptr, uint16_t* planes_out = nullptr);
// One rank, a batch of rows (BatchNorm1d on [N][C], N <= kBn1dMaxRows, C % 16 == 0): the
// statistics and the normalisation in ONE launch -- a workgroup owns 16 channels and ALL N rows,
// so it needs nobody else's partial sums (bn_moments + bn_elemt_local otherwise). Writes y, the
// stats [mean | invstd | count], the running statistics, the batch counter, and optionally the
// ReLU mask / bf16 planes exactly as bn_elemt_local does. false = shape not taken (nothing ran).
constexpr int kBn1dMaxRows = 512;
bool bn1d_local_fwd(const float* x, const float* w, const float* b, int N, int C, bool relu,
                    float eps, float momentum, float* stats, float* rmean, float* rvar,
                    int64_t* nbt, float* y, uint8_t* mask_out, uint16_t* planes_out,
                    hipStream_t s);
// The matching backward, one launch: sums (bn_bwd_reduce), dw / db (overwritten, when given) and
// dx (+ planes) from the same registers (bn_bwd_elemt). mask: the forward's ReLU mask or null.
// wopt / bopt (world size 1, fused optimizer): update w / b in place instead of writing dw / db.
// SyncBatchNorm halves of the same whole-column kernels (N <= kBn1dMaxRows, C % 16 == 0):
// bn1d_moments = bn_moments ([mean | var | count]); bn1d_gathered_fwd = bn_merge + bn_elemt over
// the all-gathered [R][2C+1] moments; bn1d_sums = bn_bwd_reduce (local sums + dw / db).
bool bn1d_moments(const float* x, int N, int C, float* moments, hipStream_t s);
bool bn1d_gathered_fwd(const float* x, const float* gathered, int R, const float* w,
                       const float* b, int N, int C, bool relu, float eps, float momentum,
                       float* stats, float* rmean, float* rvar, int64_t* nbt, float* y,
                       uint8_t* mask_out, uint16_t* planes_out, hipStream_t s);
bool bn1d_sums(const float* dy, const float* x, const float* stats, int N, int C,
               const uint8_t* mask, float* sums, float* dw, float* db, hipStream_t s);
bool bn1d_local_bwd(const float* dy, const float* x, const float* stats, const float* w, int N,
                    int C, const uint8_t* mask, float* dx, float* dw, float* db,
                    uint16_t* planes_out, hipStream_t s, const OptEpilogue* wopt = nullptr,
                    const OptEpilogue* bopt = nullptr);

}  // namespace tdp
