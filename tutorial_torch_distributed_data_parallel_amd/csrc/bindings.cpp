// pybind11 bindings: PyTorch tensors -> raw pointers + the current HIP stream for every native
// launcher in kernels.h, plus the RCCL communicator and the gradient reducer.
//
// Every op checks device/dtype/layout and raises on misuse: there is no silent fallback to ATen
// inside the extension (CPU execution is handled, explicitly, by the Python ops layer).
#include <c10/hip/HIPStream.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <cmath>
#include <map>
#include <mutex>

#include "comm.h"
#include "conv.h"
#include "emu8.h"
#include "kernels.h"
#include "planes.h"
#include "loader.h"
#include "peer.h"
#include "pool.h"
#include "reducer.h"

namespace py = pybind11;
using at::Tensor;
using namespace tdp;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// CUs the compute kernels plan for (comm.h compute_cus: physical minus TDP_COMM_CUS)
int num_cus(int device) { return compute_cus(device); }

#define CHECK_GPU(x) TORCH_CHECK((x).is_cuda(), #x " must be on the GPU")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be float32")
#define CHECK_ROWMAJOR(x) \
  TORCH_CHECK((x).dim() == 2 && (x).stride(1) == 1, #x " must be 2-D with unit inner stride")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

float* fptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

// --------------------------------------------------------------------------------------- GEMM
// A: [M,K] if a_kcontig else [K,M];  B: [N,K] if b_kcontig else [K,N];  C: [M,N]
void gemm_f32_op(const Tensor& A, const Tensor& B, Tensor& C, bool a_kcontig, bool b_kcontig,
                 const c10::optional<Tensor>& mask, const c10::optional<Tensor>& bias,
                 const c10::optional<Tensor>& rowsum, double beta, double rowsum_beta,
                 bool relu, const c10::optional<Tensor>& gate) {
  CHECK_GPU(A); CHECK_GPU(B); CHECK_GPU(C);
  CHECK_F32(A); CHECK_F32(B); CHECK_F32(C);
  CHECK_ROWMAJOR(A); CHECK_ROWMAJOR(B); CHECK_ROWMAJOR(C);
  const int M = (int)C.size(0), N = (int)C.size(1);
  const int K = (int)(a_kcontig ? A.size(1) : A.size(0));
  TORCH_CHECK((a_kcontig ? A.size(0) : A.size(1)) == M, "gemm: A rows != C rows");
  TORCH_CHECK((b_kcontig ? B.size(0) : B.size(1)) == N, "gemm: B cols != C cols");
  TORCH_CHECK((b_kcontig ? B.size(1) : B.size(0)) == K, "gemm: inner dims differ");
  GemmF32Args a;
  a.A = A.data_ptr<float>(); a.B = B.data_ptr<float>(); a.C = C.data_ptr<float>();
  a.lda = A.stride(0); a.ldb = B.stride(0); a.ldc = C.stride(0);
  a.M = M; a.N = N; a.K = K;
  a.a_kcontig = a_kcontig; a.b_kcontig = b_kcontig;
  if (mask.has_value() && mask->defined()) {
    CHECK_GPU(*mask); CHECK_F32(*mask); CHECK_ROWMAJOR(*mask);
    TORCH_CHECK(mask->sizes() == A.sizes(), "gemm: mask must have A's shape");
    a.mask = mask->data_ptr<float>();
    a.ldmask = mask->stride(0);
  }
  if (bias.has_value() && bias->defined()) {
    CHECK_GPU(*bias); CHECK_F32(*bias); CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() == N, "gemm: bias must have N elements");
    a.bias = bias->data_ptr<float>();
  }
  if (rowsum.has_value() && rowsum->defined()) {
    CHECK_GPU(*rowsum); CHECK_F32(*rowsum); CHECK_CONTIG(*rowsum);
    TORCH_CHECK(rowsum->numel() == M, "gemm: rowsum must have M elements");
    a.rowsum = rowsum->data_ptr<float>();
  }
  a.beta = (float)beta;
  a.rowsum_beta = (float)rowsum_beta;
  a.relu = relu;
  bool gate_after = false;
  if (gate.has_value() && gate->defined()) {
    CHECK_GPU(*gate); CHECK_F32(*gate); CHECK_ROWMAJOR(*gate);
    TORCH_CHECK(gate->size(0) == M && gate->size(1) == N, "gemm: gate must have C's shape");
    a.gate = gate->data_ptr<float>();
    a.ldgate = gate->stride(0);
    // the fast kernel's row-vector epilogue reads the gate as 16-B rows
    gate_after = (((uintptr_t)a.gate & 15) != 0 || a.ldgate % 4 != 0);
  }
  GemmPlan plan = gemm_f32_plan(a, num_cus(C.get_device()));
  const float* g = a.gate;
  if (gate_after && plan.fast) a.gate = nullptr;
  else gate_after = false;
  Tensor ws;
  if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, C.options());
  gemm_f32_run(a, plan, plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  if (gate_after) gate_inplace(a.C, a.ldc, g, gate->stride(0), M, N, cur_stream());
}

// Returns whether the epilogue ran. Weight-gradient GEMM whose epilogue applies the DDP's fused optimizer to arena elements
// [offset, offset + M*N) instead of storing the gradient into C (world size 1, see
// RcclBackend::epilogue_opt). C must be that contiguous arena slice (its contents are left as
// they were: the gradient is never materialised).
// The weight-gradient + optimizer GEMM behind SyncBackend::held_epilogue (gemm_f32_opt
// hold=True): its arguments, plan and tensors until the next held call pairs with it
// (gemm_f32_fast_run_pair) or the backend runs it alone at the end of backward.
struct HeldGemm {
  GemmF32Args a;
  GemmPlan plan;
  // A and B, which the launch reads. Not C or the row sums: the epilogue writes neither, and an
  // extra reference to a gradient slot would make autograd clone it instead of taking it
  std::vector<Tensor> keep;
  hipStream_t stream = nullptr;
};
static std::shared_ptr<HeldGemm> g_held;
static const SyncBackend* g_held_backend = nullptr;

bool gemm_f32_opt_op(const Tensor& A, const Tensor& B, Tensor& C, bool a_kcontig, bool b_kcontig,
                     SyncBackend& backend, int64_t offset, const c10::optional<Tensor>& rowsum,
                     double rowsum_beta, int64_t bias_offset, int64_t bias_span, bool hold) {
  CHECK_GPU(A); CHECK_GPU(B); CHECK_GPU(C);
  CHECK_F32(A); CHECK_F32(B); CHECK_F32(C);
  CHECK_ROWMAJOR(A); CHECK_ROWMAJOR(B); CHECK_CONTIG(C);
  const int M = (int)C.size(0), N = (int)C.size(1);
  const int K = (int)(a_kcontig ? A.size(1) : A.size(0));
  TORCH_CHECK((a_kcontig ? A.size(0) : A.size(1)) == M, "gemm: A rows != C rows");
  TORCH_CHECK((b_kcontig ? B.size(0) : B.size(1)) == N, "gemm: B cols != C cols");
  TORCH_CHECK((b_kcontig ? B.size(1) : B.size(0)) == K, "gemm: inner dims differ");
  TORCH_CHECK(backend.epilogue_allowed(), "optimizer epilogue: no fused optimizer at world 1");
  auto ops = std::dynamic_pointer_cast<RcclOps>(backend.ops());
  TORCH_CHECK(ops != nullptr, "optimizer epilogue needs the device (RCCL) backend");
  GemmF32Args a;
  a.A = A.data_ptr<float>(); a.B = B.data_ptr<float>(); a.C = C.data_ptr<float>();
  a.lda = A.stride(0); a.ldb = B.stride(0); a.ldc = N;
  a.M = M; a.N = N; a.K = K;
  a.a_kcontig = a_kcontig; a.b_kcontig = b_kcontig;
  if (rowsum.has_value() && rowsum->defined()) {
    CHECK_GPU(*rowsum); CHECK_F32(*rowsum); CHECK_CONTIG(*rowsum);
    TORCH_CHECK(rowsum->numel() == M, "gemm: rowsum must have M elements");
    a.rowsum = rowsum->data_ptr<float>();
    a.rowsum_beta = (float)rowsum_beta;
  }
  TORCH_CHECK((int64_t)M * N < (int64_t)1 << 31, "optimizer epilogue: parameter too large");
  // the epilogue exists on the fast kernel's weight-gradient layout without split-K; any other
  // plan stores the gradient and leaves the update to the reducer's end-of-backward launch
  GemmF32Args probe = a;
  probe.opt.kind = 1;
  const GemmPlan pp = gemm_f32_plan(probe, num_cus(C.get_device()));
  const bool epi = pp.fast && !pp.skinny && pp.splits == 1 && !a_kcontig && !b_kcontig;
  if (epi) {
    const FusedOptimizer& f = ops->fused;
    backend.note_epilogue(offset, (int64_t)M * N);
    a.opt.kind = f.kind;
    a.opt.p = f.p + offset;
    a.opt.s0 = f.s0 ? f.s0 + offset : nullptr;
    a.opt.s1 = f.s1 ? f.s1 + offset : nullptr;
    a.opt.s2 = f.s2 ? f.s2 + offset : nullptr;
    a.opt.sgd = f.sgd;    // scalars: from the device hyper block (f.sgd.dev)
    a.opt.adam = f.adam;
    if (bias_offset >= 0 && a.rowsum != nullptr && a.rowsum_beta == 0.f) {
      // the layer's bias [bias_offset, + M) is updated from the row sums by the same kernel;
      // its arena span (alignment padding included) is marked done for the reducer
      TORCH_CHECK(bias_span >= M, "optimizer epilogue: bias span shorter than the bias");
      backend.note_epilogue(bias_offset, bias_span);
      a.bias_opt.kind = f.kind;
      a.bias_opt.p = f.p + bias_offset;
      a.bias_opt.s0 = f.s0 ? f.s0 + bias_offset : nullptr;
      a.bias_opt.s1 = f.s1 ? f.s1 + bias_offset : nullptr;
      a.bias_opt.s2 = f.s2 ? f.s2 + bias_offset : nullptr;
    }
  }
  const GemmPlan plan = gemm_f32_plan(a, num_cus(C.get_device()));
  const hipStream_t s = cur_stream();
  if (epi && hold) {
    // world size 1, consecutive layers: the first weight-gradient GEMM waits for the second and
    // both run as one persistent launch (nothing reads the updated weights before the next
    // forward; the end of backward runs a GEMM still held)
    if (backend.held_epilogue && g_held && g_held_backend == &backend && g_held->stream == s &&
        gemm_f32_fast_pair_ok(g_held->a, g_held->plan, a, plan)) {
      backend.held_epilogue = nullptr;
      gemm_f32_fast_run_pair(g_held->a, g_held->plan, a, plan, s);
      g_held.reset();
      return epi;
    }
    backend.run_held_epilogue(s);  // a held GEMM this one cannot pair with runs alone first
    if (plan.ws_floats == 0 && (a.rowsum == nullptr || a.bias_opt.kind != 0) &&
        gemm_f32_fast_pair_ok(a, plan, a, plan)) {
      auto h = std::make_shared<HeldGemm>();
      h->a = a;
      h->plan = plan;
      h->keep = {A, B};
      h->stream = s;
      g_held = h;
      g_held_backend = &backend;
      backend.held_epilogue = [h](hipStream_t st) {
        gemm_f32_run(h->a, h->plan, nullptr, st);
        h->keep.clear();  // stream-ordered: later users of the memory run after this launch
      };
      return epi;
    }
  }
  Tensor ws;
  if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, C.options());
  gemm_f32_run(a, plan, plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, s);
  return epi;
}

// Skinny GEMM from the bf16 split planes of A (csrc/gemm_planes.hip):
//   Ap [3][M][K] bf16 (contiguous), B [N][K] (b_kcontig) or [K][N] fp32, C [M][N] fp32;
//   out_planes (optional) [3][M][N] bf16 receives the planes of the finished C.
void gemm_planes_op(const Tensor& Ap, const Tensor& B, Tensor& C, bool b_kcontig,
                    const c10::optional<Tensor>& bias, bool relu,
                    const c10::optional<Tensor>& gate, const c10::optional<Tensor>& out_planes) {
  CHECK_GPU(Ap); CHECK_GPU(B); CHECK_GPU(C);
  TORCH_CHECK(Ap.scalar_type() == at::kBFloat16 && Ap.dim() == 3 && Ap.size(0) == 3 &&
                  Ap.is_contiguous(), "gemm_planes: Ap must be a contiguous [3, M, K] bf16 tensor");
  CHECK_F32(B); CHECK_F32(C); CHECK_ROWMAJOR(B); CHECK_ROWMAJOR(C);
  const int M = (int)C.size(0), N = (int)C.size(1), K = (int)Ap.size(2);
  TORCH_CHECK(Ap.size(1) == M, "gemm_planes: A rows != C rows");
  TORCH_CHECK((b_kcontig ? B.size(0) : B.size(1)) == N, "gemm_planes: B cols != C cols");
  TORCH_CHECK((b_kcontig ? B.size(1) : B.size(0)) == K, "gemm_planes: inner dims differ");
  GemmPlanesArgs a;
  a.Ap = reinterpret_cast<const uint16_t*>(Ap.data_ptr());
  a.ps = Ap.stride(0); a.lda = Ap.stride(1);
  a.B = B.data_ptr<float>(); a.ldb = B.stride(0); a.b_kcontig = b_kcontig;
  a.C = C.data_ptr<float>(); a.ldc = C.stride(0);
  a.M = M; a.N = N; a.K = K;
  a.relu = relu;
  if (bias.has_value() && bias->defined()) {
    CHECK_GPU(*bias); CHECK_F32(*bias); CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() == N, "gemm_planes: bias must have N elements");
    a.bias = bias->data_ptr<float>();
  }
  if (gate.has_value() && gate->defined()) {
    CHECK_GPU(*gate); CHECK_F32(*gate); CHECK_ROWMAJOR(*gate);
    TORCH_CHECK(gate->size(0) == M && gate->size(1) == N, "gemm_planes: gate must have C's shape");
    a.gate = gate->data_ptr<float>();
    a.ldgate = gate->stride(0);
  }
  if (out_planes.has_value() && out_planes->defined()) {
    const Tensor& o = *out_planes;
    CHECK_GPU(o);
    TORCH_CHECK(o.scalar_type() == at::kBFloat16 && o.is_contiguous() && o.dim() == 3 &&
                    o.size(0) == 3 && o.size(1) == M && o.size(2) == N,
                "gemm_planes: out_planes must be a contiguous [3, M, N] bf16 tensor");
    a.out_planes = reinterpret_cast<uint16_t*>(o.data_ptr());
    a.out_ps = o.stride(0);
  }
  TORCH_CHECK(gemm_planes_ok(a), "gemm_planes: unsupported shape / alignment (K % 32, N % 4, "
              "16-B aligned rows)");
  const GemmPlan plan = gemm_planes_plan(a, num_cus(C.get_device()));
  Tensor ws;
  if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, C.options());
  gemm_planes_run(a, plan, plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
}

// x [rows, cols] fp32 (unit inner stride) -> its exact bf16 split planes [3, rows, cols]
// large-tile split-bf16 GEMM (csrc/gemm_emu8.hip): A [M,K]; B [N,K] if b_kcontig else [K,N]
void gemm_emu8_op(const Tensor& A, const Tensor& B, Tensor& C, bool b_kcontig, double beta) {
  CHECK_GPU(A); CHECK_GPU(B); CHECK_GPU(C);
  CHECK_F32(A); CHECK_F32(B); CHECK_F32(C);
  CHECK_ROWMAJOR(A); CHECK_ROWMAJOR(B); CHECK_ROWMAJOR(C);
  GemmEmu8Args a;
  a.M = (int)C.size(0);
  a.N = (int)C.size(1);
  a.K = (int)A.size(1);
  TORCH_CHECK(A.size(0) == a.M, "gemm_emu8: A rows != C rows");
  TORCH_CHECK((b_kcontig ? B.size(0) : B.size(1)) == a.N, "gemm_emu8: B cols != C cols");
  TORCH_CHECK((b_kcontig ? B.size(1) : B.size(0)) == a.K, "gemm_emu8: inner dims differ");
  a.A = A.data_ptr<float>();
  a.B = B.data_ptr<float>();
  a.C = C.data_ptr<float>();
  a.lda = A.stride(0);
  a.ldb = B.stride(0);
  a.ldc = C.stride(0);
  a.b_kcontig = b_kcontig;
  a.beta = (float)beta;
  TORCH_CHECK(gemm_emu8_ok(a), "gemm_emu8: K % 32 == 0 and 16-B aligned rows required");
  gemm_emu8_run(a, cur_stream());
}

Tensor split_planes_op(const Tensor& x) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_ROWMAJOR(x);
  const int rows = (int)x.size(0), cols = (int)x.size(1);
  TORCH_CHECK(cols % 4 == 0 && x.stride(0) % 4 == 0 && ((uintptr_t)x.data_ptr() & 15) == 0,
              "split_planes: cols % 4 == 0 and 16-B aligned rows required");
  Tensor p = at::empty({3, rows, cols}, x.options().dtype(at::kBFloat16));
  split_planes(x.data_ptr<float>(), x.stride(0), rows, cols,
               reinterpret_cast<uint16_t*>(p.data_ptr()), p.stride(0), cur_stream());
  return p;
}

// Head Linear backward in one launch (planes.h head_bwd): fills dx, dw, db (optional); returns
// (launched, planes of dx or None). g [B, O] (O <= 16), x [B, I], w [O, I], dx [B, I], dw [O, I].
py::tuple head_bwd_op(const Tensor& g, const Tensor& x, const Tensor& w,
                      const c10::optional<Tensor>& dx_opt, Tensor& dw,
                      const c10::optional<Tensor>& db, const c10::optional<Tensor>& gate,
                      bool planes, SyncBackend* backend, int64_t w_offset, int64_t b_offset,
                      int64_t b_span) {
  CHECK_GPU(g); CHECK_GPU(x); CHECK_GPU(w); CHECK_GPU(dw);
  CHECK_F32(g); CHECK_F32(x); CHECK_F32(w); CHECK_F32(dw);
  CHECK_ROWMAJOR(g); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(w);
  CHECK_ROWMAJOR(dw);
  const int B = (int)g.size(0), O = (int)g.size(1), I = (int)x.size(1);
  TORCH_CHECK(x.size(0) == B && w.size(0) == O && w.size(1) == I && dw.size(0) == O &&
                  dw.size(1) == I,
              "head_bwd: shape mismatch");
  // dx None: only dW / db (the input gradient came out of head_ce's forward)
  const bool has_dx = dx_opt.has_value() && dx_opt->defined();
  Tensor dx;
  if (has_dx) {
    dx = *dx_opt;
    CHECK_GPU(dx); CHECK_F32(dx); CHECK_ROWMAJOR(dx);
    TORCH_CHECK(dx.size(0) == B && dx.size(1) == I, "head_bwd: dx shape mismatch");
  }
  planes = planes && has_dx;
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    CHECK_GPU(*db); CHECK_F32(*db); CHECK_CONTIG(*db);
    TORCH_CHECK(db->numel() == O, "head_bwd: db must have O elements");
    dbp = db->data_ptr<float>();
  }
  const float* gp = nullptr;
  long ldgate = 0;
  if (gate.has_value() && gate->defined()) {
    CHECK_GPU(*gate); CHECK_F32(*gate); CHECK_ROWMAJOR(*gate);
    TORCH_CHECK(gate->size(0) == B && gate->size(1) == I, "head_bwd: gate must have dx's shape");
    gp = gate->data_ptr<float>();
    ldgate = gate->stride(0);
  }
  Tensor pl;
  if (planes) pl = at::empty({3, (long)B, (long)I}, dx.options().dtype(at::kBFloat16));
  // world size 1 + fused optimizer (backend given): W and b are updated by the kernel instead of
  // storing their gradients; their arena ranges are marked done for the reducer
  OptEpilogue wo, bo;
  if (backend != nullptr && w_offset >= 0) {
    TORCH_CHECK(backend->epilogue_allowed(), "head_bwd: optimizer epilogue not allowed");
    auto ops = std::dynamic_pointer_cast<RcclOps>(backend->ops());
    TORCH_CHECK(ops != nullptr, "head_bwd: optimizer epilogue needs the device backend");
    TORCH_CHECK(dw.is_contiguous(), "head_bwd: dw must be the contiguous arena slot");
    const FusedOptimizer& f = ops->fused;
    auto at_off = [&](int64_t off) {
      OptEpilogue o;
      o.kind = f.kind;
      o.p = f.p + off;
      o.s0 = f.s0 ? f.s0 + off : nullptr;
      o.s1 = f.s1 ? f.s1 + off : nullptr;
      o.s2 = f.s2 ? f.s2 + off : nullptr;
      o.sgd = f.sgd;
      o.adam = f.adam;
      return o;
    };
    wo = at_off(w_offset);
    if (dbp != nullptr && b_offset >= 0) {
      TORCH_CHECK(b_span >= O, "head_bwd: bias span shorter than the bias");
      bo = at_off(b_offset);
    }
  }
  const bool ok = head_bwd(g.data_ptr<float>(), g.stride(0), x.data_ptr<float>(), x.stride(0),
                           w.data_ptr<float>(), w.stride(0),
                           has_dx ? dx.data_ptr<float>() : nullptr, has_dx ? dx.stride(0) : 0,
                           gp, ldgate,
                           planes ? reinterpret_cast<uint16_t*>(pl.data_ptr()) : nullptr,
                           planes ? pl.stride(0) : 0, dw.data_ptr<float>(), dw.stride(0), dbp, B,
                           O, I, cur_stream(), wo.kind ? &wo : nullptr, bo.kind ? &bo : nullptr);
  if (ok && wo.kind) backend->note_epilogue(w_offset, (int64_t)O * I);
  if (ok && bo.kind) backend->note_epilogue(b_offset, b_span);
  if (ok && planes) return py::make_tuple(true, pl);
  return py::make_tuple(ok, py::none());
}

// Head Linear + cross-entropy forward in one launch (planes.h head_ce). x [B, I] (B <= 256),
// w [O, I] (O <= 16), labels [B] int64, ticket: 9 zeroed int32 scratch words (zero again after
// the launch). Returns [loss, lse [B + 1], logits [B, O]] + with_grad: [dlogits (unit seed),
// dx [B, I], planes of dx or an empty tensor]; an empty list when the shape is not supported.
std::vector<Tensor> head_ce_op(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                               const Tensor& labels, int64_t ignore_index, double smoothing,
                               bool mean, const c10::optional<Tensor>& acc, bool with_grad,
                               const c10::optional<Tensor>& gate, bool planes,
                               Tensor& ticket) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_ROWMAJOR(x);
  CHECK_GPU(w); CHECK_F32(w); CHECK_ROWMAJOR(w);
  CHECK_GPU(labels); CHECK_CONTIG(labels); CHECK_GPU(ticket); CHECK_CONTIG(ticket);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  TORCH_CHECK(ticket.scalar_type() == at::kInt && ticket.numel() >= 9, "ticket: 9 int32 words");
  const int B = (int)x.size(0), I = (int)x.size(1), O = (int)w.size(0);
  TORCH_CHECK(w.size(1) == I && labels.numel() == B, "head_ce: shape mismatch");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_GPU(*bias); CHECK_F32(*bias); CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() == O, "head_ce: bias must have O elements");
    bp = bias->data_ptr<float>();
  }
  float* accp = nullptr;
  if (acc.has_value() && acc->defined()) {
    CHECK_GPU(*acc); CHECK_F32(*acc);
    TORCH_CHECK(acc->numel() >= 3, "acc needs 3 floats");
    accp = acc->data_ptr<float>();
  }
  const float* gp = nullptr;
  long ldgate = 0;
  if (gate.has_value() && gate->defined()) {
    CHECK_GPU(*gate); CHECK_F32(*gate); CHECK_ROWMAJOR(*gate);
    TORCH_CHECK(gate->size(0) == B && gate->size(1) == I, "head_ce: gate must have x's shape");
    gp = gate->data_ptr<float>();
    ldgate = gate->stride(0);
  }
  auto o = x.options();
  Tensor loss = at::empty({}, o), lse = at::empty({B + 1}, o), logits = at::empty({B, O}, o);
  Tensor rowbuf = at::empty({B, 4}, o);
  Tensor d, dx, pl;
  if (with_grad) {
    d = at::empty({B, O}, o);
    dx = at::empty({B, I}, o);
    if (planes) pl = at::empty({3, (long)B, (long)I}, o.dtype(at::kBFloat16));
  }
  const bool ok = head_ce(
      x.data_ptr<float>(), x.stride(0), w.data_ptr<float>(), w.stride(0), bp,
      labels.data_ptr<int64_t>(), B, O, I, (int)ignore_index, (float)smoothing, mean,
      logits.data_ptr<float>(), lse.data_ptr<float>(), rowbuf.data_ptr<float>(),
      reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), loss.data_ptr<float>(), accp,
      with_grad ? d.data_ptr<float>() : nullptr, with_grad ? dx.data_ptr<float>() : nullptr,
      with_grad ? dx.stride(0) : 0, gp, ldgate,
      (with_grad && planes) ? reinterpret_cast<uint16_t*>(pl.data_ptr()) : nullptr,
      (with_grad && planes) ? pl.stride(0) : 0, cur_stream());
  if (!ok) return {};
  if (!with_grad) return {loss, lse, logits};
  return {loss, lse, logits, d, dx, planes ? pl : at::empty({0}, o)};
}

std::vector<int64_t> gemm_planes_plan_op(int M, int N, int K, int cus) {
  GemmPlanesArgs a;
  a.M = M; a.N = N; a.K = K;
  const GemmPlan p = gemm_planes_plan(a, cus);
  return {p.splits, p.k_per_split, p.ws_floats};
}

std::vector<int64_t> gemm_f32_plan_op(int M, int N, int K, bool rowsum, int cus) {
  GemmF32Args a;
  a.M = M; a.N = N; a.K = K;
  a.rowsum = rowsum ? reinterpret_cast<float*>(16) : nullptr;
  a.a_kcontig = true; a.b_kcontig = true;
  a.A = reinterpret_cast<const float*>(256); a.B = reinterpret_cast<const float*>(256);
  a.lda = K; a.ldb = K;
  const GemmPlan p = gemm_f32_plan(a, cus);
  return {p.fast ? 1 : 0, p.tile, p.bm, p.bn, p.stages, p.splits, p.k_per_split, p.ws_floats};
}

// ----------------------------------------------------------------------------------------- loss
std::vector<Tensor> ce_fwd_op(const Tensor& logits, const Tensor& labels, int64_t ignore_index,
                              double smoothing, bool mean, const c10::optional<Tensor>& acc,
                              bool with_grad) {
  CHECK_GPU(logits); CHECK_F32(logits); CHECK_ROWMAJOR(logits);
  CHECK_GPU(labels); CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  TORCH_CHECK(labels.numel() == B, "labels must have one entry per row");
  auto loss = at::empty({}, logits.options());
  auto lse = at::empty({B + 1}, logits.options());
  float* accp = nullptr;
  if (acc.has_value() && acc->defined()) {
    CHECK_GPU(*acc); CHECK_F32(*acc);
    TORCH_CHECK(acc->numel() >= 3, "acc needs 3 floats");
    accp = acc->data_ptr<float>();
  }
  // with_grad: also the logits gradient for an upstream gradient of 1 (one launch for the
  // training step's loss forward + backward; single workgroup, so bounded to small B*C)
  Tensor d;
  if (with_grad) {
    TORCH_CHECK((int64_t)B * C <= (1 << 16), "ce_fwd with_grad: B*C too large");
    d = at::empty({B, C}, logits.options());
  }
  cross_entropy_fwd(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), B, C, logits.stride(0),
                    (int)ignore_index, (float)smoothing, mean, loss.data_ptr<float>(),
                    lse.data_ptr<float>(), accp, cur_stream(),
                    with_grad ? d.data_ptr<float>() : nullptr);
  if (with_grad) return {loss, lse, d};
  return {loss, lse};
}

Tensor ce_bwd_op(const Tensor& logits, const Tensor& labels, const Tensor& lse,
                 const Tensor& gout, int64_t ignore_index, double smoothing, bool mean) {
  CHECK_GPU(logits); CHECK_F32(logits); CHECK_ROWMAJOR(logits);
  CHECK_GPU(gout); CHECK_F32(gout);
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  auto d = at::empty({B, C}, logits.options());
  auto g = gout.contiguous();
  cross_entropy_bwd(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                    g.data_ptr<float>(), B, C, logits.stride(0), (int)ignore_index,
                    (float)smoothing, mean, d.data_ptr<float>(), cur_stream());
  return d;
}

void count_correct_op(const Tensor& logits, const Tensor& labels, Tensor& acc) {
  CHECK_GPU(logits); CHECK_F32(logits); CHECK_ROWMAJOR(logits);
  CHECK_GPU(acc); CHECK_F32(acc);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  count_correct(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), (int)logits.size(0),
                (int)logits.size(1), logits.stride(0), acc.data_ptr<float>(), cur_stream());
}

// ---------------------------------------------------------------------------------- optimizers
const float* hyper_ptr(const c10::optional<Tensor>& blk) {
  if (!blk.has_value() || !blk->defined()) return nullptr;
  CHECK_GPU(*blk); CHECK_F32(*blk); CHECK_CONTIG(*blk);
  TORCH_CHECK(blk->numel() >= kHSlots, "hyper block needs ", kHSlots, " floats");
  return blk->data_ptr<float>();
}

// `hyper` (optional device hyper block, kernels.h HyperSlot): the kernel reads lr / momentum /
// betas / bias corrections / first-step flag / clip coefficient from it (graph-replay safe);
// the by-value arguments then only carry the structural flags.
void sgd_flat_op(Tensor& p, const Tensor& g, const c10::optional<Tensor>& buf, double lr,
                 double momentum, double dampening, double wd, bool nesterov, bool maximize,
                 bool first_step, double grad_scale, const c10::optional<Tensor>& hyper) {
  CHECK_GPU(p); CHECK_F32(p); CHECK_CONTIG(p); CHECK_GPU(g); CHECK_F32(g); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "sgd: p/g size mismatch");
  if (momentum != 0.0)
    TORCH_CHECK(buf.has_value() && buf->numel() == p.numel(), "sgd: momentum buffer required");
  SgdHyper h{(float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, maximize,
             first_step, (float)grad_scale, hyper_ptr(hyper)};
  sgd_flat(p.data_ptr<float>(), g.data_ptr<float>(), fptr(buf), p.numel(), h, cur_stream());
}

void adam_flat_op(Tensor& p, const Tensor& g, Tensor& m, Tensor& v,
                  const c10::optional<Tensor>& vmax, double lr, double b1, double b2, double eps,
                  double wd, bool amsgrad, bool maximize, bool decoupled, int64_t step,
                  double grad_scale, const c10::optional<Tensor>& hyper) {
  CHECK_GPU(p); CHECK_F32(p); CHECK_CONTIG(p);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(),
              "adam: size mismatch");
  if (amsgrad) TORCH_CHECK(vmax.has_value() && vmax->numel() == p.numel(), "adam: need vmax");
  AdamHyper h{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, amsgrad, maximize,
              decoupled, (float)(1.0 - std::pow(b1, (double)step)),
              (float)std::sqrt(1.0 - std::pow(b2, (double)step)), (float)grad_scale,
              hyper_ptr(hyper)};
  adam_flat(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
            fptr(vmax), p.numel(), h, cur_stream());
}

void opt_step_begin_op(Tensor& hyper, int64_t kind) {
  opt_step_begin(const_cast<float*>(hyper_ptr(hyper)), (int)kind, cur_stream());
}

// torch.nn.utils.clip_grad_norm_ over a list of gradients, entirely on the device: one
// deterministic sum-of-squares pass per <= 16 tensors into the block, the coefficient, one
// scaling pass. Returns nothing; the total norm is left at hyper[kHNorm].
void clip_grad_norm_op(const std::vector<Tensor>& grads, Tensor& hyper, double max_norm) {
  float* blk = const_cast<float*>(hyper_ptr(hyper));
  hipStream_t s = cur_stream();
  // reset the accumulator and set the threshold without a host round trip
  fill_f32(blk + kHSumsq, 1, 0.f, s);
  fill_f32(blk + kHMaxNorm, 1, (float)max_norm, s);
  RangeSet one;
  one.n = 1;
  one.begin[0] = 0;
  for (const auto& g : grads) {
    CHECK_GPU(g); CHECK_F32(g); CHECK_CONTIG(g);
    one.len[0] = (long)g.numel();
    sumsq_ranges(g.data_ptr<float>(), one, blk, s);
  }
  clip_coef_from_sumsq(blk, s);
  for (const auto& g : grads) {
    one.len[0] = (long)g.numel();
    scale_ranges_by(g.data_ptr<float>(), one, blk, s);
  }
}

// Build the chunk table (<= 64K elements per workgroup) on the host, ship it with the launch.
Tensor chunk_table(const std::vector<Tensor>& ps, const std::vector<Tensor>& gs,
                   const std::vector<Tensor>& s0, const std::vector<Tensor>& s1,
                   const std::vector<Tensor>& s2, int* count) {
  constexpr long CH = 65536;
  std::vector<TensorChunk> tab;
  for (size_t i = 0; i < ps.size(); ++i) {
    const long n = ps[i].numel();
    TORCH_CHECK(gs[i].numel() == n, "multi-tensor: grad size mismatch");
    for (long o = 0; o < n; o += CH) {
      TensorChunk c;
      c.p = ps[i].data_ptr<float>() + o;
      c.g = gs[i].data_ptr<float>() + o;
      c.s0 = s0.empty() ? nullptr : s0[i].data_ptr<float>() + o;
      c.s1 = s1.empty() ? nullptr : s1[i].data_ptr<float>() + o;
      c.s2 = s2.empty() ? nullptr : s2[i].data_ptr<float>() + o;
      c.n = std::min(CH, n - o);
      tab.push_back(c);
    }
  }
  *count = (int)tab.size();
  auto host = at::empty({(int64_t)(tab.size() * sizeof(TensorChunk))},
                        at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  std::memcpy(host.data_ptr(), tab.data(), tab.size() * sizeof(TensorChunk));
  return host.to(ps[0].device(), /*non_blocking=*/true);
}

void sgd_multi_op(const std::vector<Tensor>& ps, const std::vector<Tensor>& gs,
                  const std::vector<Tensor>& bufs, double lr, double momentum, double dampening,
                  double wd, bool nesterov, bool maximize, bool first_step, double grad_scale,
                  const c10::optional<Tensor>& hyper) {
  if (ps.empty()) return;
  for (auto& t : ps) { CHECK_GPU(t); CHECK_F32(t); CHECK_CONTIG(t); }
  for (auto& t : gs) { CHECK_F32(t); CHECK_CONTIG(t); }
  int count = 0;
  auto tab = chunk_table(ps, gs, bufs, {}, {}, &count);
  SgdHyper h{(float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, maximize,
             first_step, (float)grad_scale, hyper_ptr(hyper)};
  sgd_multi(reinterpret_cast<const TensorChunk*>(tab.data_ptr()), count, h, cur_stream());
}

void adam_multi_op(const std::vector<Tensor>& ps, const std::vector<Tensor>& gs,
                   const std::vector<Tensor>& ms, const std::vector<Tensor>& vs,
                   const std::vector<Tensor>& vmaxs, double lr, double b1, double b2, double eps,
                   double wd, bool amsgrad, bool maximize, bool decoupled, int64_t step,
                   double grad_scale, const c10::optional<Tensor>& hyper) {
  if (ps.empty()) return;
  for (auto& t : ps) { CHECK_GPU(t); CHECK_F32(t); CHECK_CONTIG(t); }
  int count = 0;
  auto tab = chunk_table(ps, gs, ms, vs, amsgrad ? vmaxs : std::vector<Tensor>{}, &count);
  AdamHyper h{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, amsgrad, maximize,
              decoupled, (float)(1.0 - std::pow(b1, (double)step)),
              (float)std::sqrt(1.0 - std::pow(b2, (double)step)), (float)grad_scale,
              hyper_ptr(hyper)};
  adam_multi(reinterpret_cast<const TensorChunk*>(tab.data_ptr()), count, h, cur_stream());
}

// g = dy*(y>0) (new tensor; dy itself when y is None), db (optional) = sum over rows of g
Tensor relu_bias_bwd_op(const Tensor& dy, const c10::optional<Tensor>& y,
                        const c10::optional<Tensor>& db, double beta_db, double gscale) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_ROWMAJOR(dy);
  const int B = (int)dy.size(0), N = (int)dy.size(1);
  const bool has_y = y.has_value() && y->defined();
  TORCH_CHECK(gscale == 1.0 || has_y, "relu_bias_bwd: gscale needs the ReLU output y");
  Tensor g = dy;
  if (has_y) {
    CHECK_ROWMAJOR(*y);
    TORCH_CHECK(y->sizes() == dy.sizes() && y->stride(0) == dy.stride(0), "relu mask layout");
    g = at::empty({B, N}, dy.options());
  }
  float* dbp = fptr(db);
  if (!has_y && dbp == nullptr) return g;
  const int slices = relu_bias_slices(B, N, num_cus(dy.get_device()));
  Tensor part;
  if (dbp) part = at::empty({(int64_t)slices * N}, dy.options());
  relu_bias_bwd_ws(dy.data_ptr<float>(), has_y ? y->data_ptr<float>() : nullptr, B, N,
                   dy.stride(0), g.data_ptr<float>(), dbp, (float)beta_db,
                   dbp ? part.data_ptr<float>() : nullptr, slices, cur_stream(), (float)gscale);
  return g;
}

// y = relu?(x + b) row-wise (x [B, N] row-major, N % 4 == 0, 16-B aligned)
Tensor bias_act_op(const Tensor& x, const Tensor& b, bool relu) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_ROWMAJOR(x); CHECK_GPU(b); CHECK_F32(b); CHECK_CONTIG(b);
  const int B = (int)x.size(0), N = (int)x.size(1);
  TORCH_CHECK(b.numel() == N && N % 4 == 0 && x.stride(0) % 4 == 0 &&
                  x.data_ptr<float>() != nullptr && ((uintptr_t)x.data_ptr() & 15) == 0 &&
                  ((uintptr_t)b.data_ptr() & 15) == 0,
              "bias_act: N % 4 == 0 and 16-B aligned rows / bias required");
  Tensor y = at::empty({B, N}, x.options());
  bias_act_rows(x.data_ptr<float>(), x.stride(0), b.data_ptr<float>(), y.data_ptr<float>(), N,
                B, N, relu, cur_stream());
  return y;
}

// ------------------------------------------------------------------------------------ misc ops
void scale_op(Tensor& x, double a) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  scale_inplace(x.data_ptr<float>(), x.numel(), (float)a, cur_stream());
}

void cast_f32_bf16_op(const Tensor& x, Tensor& y) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_CONTIG(y);
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.numel() == x.numel(), "cast: bad output");
  f32_to_bf16_copy(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(y.data_ptr()), x.numel(),
                   cur_stream());
}

// ------------------------------------------------------------------------------------ batchnorm
// x viewed as [N, C, HW]
void bn_dims(const Tensor& x, int& N, int& C, int& HW) {
  TORCH_CHECK(x.dim() >= 2, "batchnorm input must be at least 2-D");
  N = (int)x.size(0);
  C = (int)x.size(1);
  HW = (int)(x.numel() / ((int64_t)N * C));
}

std::vector<Tensor> bn_moments_op(const Tensor& x) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  int N, C, HW;
  bn_dims(x, N, C, HW);
  const int splits = bn_splits(N, C, HW, num_cus(x.get_device()));
  auto out = at::empty({2 * C + 1}, x.options());  // [mean | var | count]
  Tensor ws = at::empty({bn_ws_floats(C, splits)}, x.options());
  bn_moments(x.data_ptr<float>(), N, C, HW, splits, ws.data_ptr<float>(), out.data_ptr<float>(),
             out.data_ptr<float>() + C, out.data_ptr<float>() + 2 * C, cur_stream());
  return {out};
}

// gathered: R rows of [mean | var | count] -> stats [mean | invstd | total count]
Tensor bn_merge_op(const Tensor& gathered, int64_t C, double eps, double momentum,
                   const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar,
                   const c10::optional<Tensor>& num_batches) {
  CHECK_GPU(gathered); CHECK_F32(gathered); CHECK_CONTIG(gathered);
  const int R = (int)(gathered.numel() / (2 * C + 1));
  TORCH_CHECK((int64_t)R * (2 * C + 1) == gathered.numel(), "bn_merge: bad gathered size");
  auto stats = at::empty({2 * C + 1}, gathered.options());
  float* sp = stats.data_ptr<float>();
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    CHECK_GPU(*num_batches);
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
                "bn_merge: num_batches_tracked must be one int64");
    nb = num_batches->data_ptr<int64_t>();
  }
  bn_merge(gathered.data_ptr<float>(), R, (int)C, (float)eps, (float)momentum, sp, sp + C,
           fptr(rmean), fptr(rvar), nb, cur_stream());
  return stats;
}

// the ReLU mask of the [rows, C % 4 == 0] form: uint8, one byte per 4 channels
static const uint8_t* mask_ptr(const c10::optional<Tensor>& m, const Tensor& x) {
  if (!m.has_value() || !m->defined()) return nullptr;
  CHECK_GPU(*m); CHECK_CONTIG(*m);
  TORCH_CHECK(m->scalar_type() == at::kByte, "bn ReLU mask must be uint8");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 4 == 0 && m->numel() == x.numel() / 4,
              "bn ReLU mask: [rows, C/4] bytes for a [rows, C % 4 == 0] input");
  return m->data_ptr<uint8_t>();
}

static uint16_t* planes_ptr(const c10::optional<Tensor>& p, const Tensor& x) {
  if (!p.has_value() || !p->defined()) return nullptr;
  CHECK_GPU(*p);
  TORCH_CHECK(p->scalar_type() == at::kBFloat16 && p->is_contiguous() && x.dim() == 2 &&
                  p->numel() == 3 * x.numel() && x.size(1) % 4 == 0,
              "planes_out: a contiguous [3, rows, C % 4 == 0] bf16 tensor");
  return reinterpret_cast<uint16_t*>(p->data_ptr());
}

Tensor bn_elemt_op(const Tensor& x, const Tensor& stats, const c10::optional<Tensor>& w,
                   const c10::optional<Tensor>& b, bool relu,
                   const c10::optional<Tensor>& residual,
                   const c10::optional<Tensor>& mask_out,
                   const c10::optional<Tensor>& planes_out) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  int N, C, HW;
  bn_dims(x, N, C, HW);
  TORCH_CHECK(stats.numel() == 2 * C + 1, "bn_elemt: stats must be [2C+1]");
  if (residual.has_value() && residual->defined()) {
    CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->sizes() == x.sizes(), "bn_elemt: residual must have x's shape");
  }
  auto y = at::empty_like(x);
  const float* sp = stats.data_ptr<float>();
  bn_elemt(x.data_ptr<float>(), sp, sp + C, fptr(w), fptr(b), N, C, HW, relu,
           y.data_ptr<float>(), cur_stream(), fptr(residual),
           const_cast<uint8_t*>(mask_ptr(mask_out, x)), planes_ptr(planes_out, x));
  return y;
}

// one rank: (y, stats) from this rank's moments [mean | var | count] -- bn_merge fused in
std::vector<Tensor> bn_elemt_local_op(const Tensor& x, const Tensor& moments,
                                      const c10::optional<Tensor>& w,
                                      const c10::optional<Tensor>& b, bool relu, double eps,
                                      double momentum, const c10::optional<Tensor>& rmean,
                                      const c10::optional<Tensor>& rvar,
                                      const c10::optional<Tensor>& num_batches,
                                      const c10::optional<Tensor>& mask_out,
                                      const c10::optional<Tensor>& planes_out,
                                      const c10::optional<Tensor>& residual) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2, "bn_elemt_local: [rows, C] input");
  if (residual.has_value() && residual->defined()) {
    CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->sizes() == x.sizes(), "bn_elemt_local: residual must have x's shape");
  }
  const int N = (int)x.size(0), C = (int)x.size(1);
  TORCH_CHECK(moments.numel() == 2 * C + 1, "bn_elemt_local: moments must be [2C+1]");
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
                "bn_elemt_local: num_batches_tracked must be one int64");
    nb = num_batches->data_ptr<int64_t>();
  }
  auto y = at::empty_like(x);
  auto stats = at::empty({2 * C + 1}, x.options());
  const bool ok = bn_elemt_local(x.data_ptr<float>(), moments.data_ptr<float>(), fptr(w),
                                 fptr(b), N, C, relu, (float)eps, (float)momentum,
                                 stats.data_ptr<float>(), fptr(rmean), fptr(rvar), nb,
                                 y.data_ptr<float>(), const_cast<uint8_t*>(mask_ptr(mask_out, x)),
                                 planes_ptr(planes_out, x), cur_stream(), fptr(residual));
  if (!ok) return {};
  return {y, stats};
}

// one rank, a batch of rows: (y, stats) with the statistics computed in the same launch
// (bn1d_local_fwd); [] when the shape is not taken (the caller runs bn_moments + bn_elemt_local)
std::vector<Tensor> bn1d_local_fwd_op(const Tensor& x, const c10::optional<Tensor>& w,
                                      const c10::optional<Tensor>& b, bool relu, double eps,
                                      double momentum, const c10::optional<Tensor>& rmean,
                                      const c10::optional<Tensor>& rvar,
                                      const c10::optional<Tensor>& num_batches,
                                      const c10::optional<Tensor>& mask_out,
                                      const c10::optional<Tensor>& planes_out) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2, "bn1d_local_fwd: [rows, C] input");
  const int N = (int)x.size(0), C = (int)x.size(1);
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
                "bn1d_local_fwd: num_batches_tracked must be one int64");
    nb = num_batches->data_ptr<int64_t>();
  }
  for (const auto* t : {&w, &b, &rmean, &rvar})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->numel() == C && (*t)->is_contiguous(), "bn1d_local_fwd: [C] parameters");
  auto y = at::empty_like(x);
  auto stats = at::empty({2 * C + 1}, x.options());
  const bool ok = bn1d_local_fwd(x.data_ptr<float>(), fptr(w), fptr(b), N, C, relu, (float)eps,
                                 (float)momentum, stats.data_ptr<float>(), fptr(rmean),
                                 fptr(rvar), nb, y.data_ptr<float>(),
                                 const_cast<uint8_t*>(mask_ptr(mask_out, x)),
                                 planes_ptr(planes_out, x), cur_stream());
  if (!ok) return {};
  return {y, stats};
}

// SyncBatchNorm halves (csrc/norm.hip whole-column kernels); undefined / [] when not taken
Tensor bn1d_moments_op(const Tensor& x) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2, "bn1d_moments: [rows, C] input");
  const int N = (int)x.size(0), C = (int)x.size(1);
  auto m = at::empty({2 * C + 1}, x.options());
  if (!bn1d_moments(x.data_ptr<float>(), N, C, m.data_ptr<float>(), cur_stream())) return Tensor();
  return m;
}

std::vector<Tensor> bn1d_gathered_fwd_op(const Tensor& x, const Tensor& gathered,
                                         const c10::optional<Tensor>& w,
                                         const c10::optional<Tensor>& b, bool relu, double eps,
                                         double momentum, const c10::optional<Tensor>& rmean,
                                         const c10::optional<Tensor>& rvar,
                                         const c10::optional<Tensor>& num_batches,
                                         const c10::optional<Tensor>& mask_out,
                                         const c10::optional<Tensor>& planes_out) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_GPU(gathered); CHECK_CONTIG(gathered);
  TORCH_CHECK(x.dim() == 2, "bn1d_gathered_fwd: [rows, C] input");
  const int N = (int)x.size(0), C = (int)x.size(1);
  TORCH_CHECK(gathered.scalar_type() == at::kFloat && gathered.numel() % (2 * C + 1) == 0,
              "bn1d_gathered_fwd: gathered must be [R][2C+1] fp32 moments");
  const int R = (int)(gathered.numel() / (2 * C + 1));
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
                "bn1d_gathered_fwd: num_batches_tracked must be one int64");
    nb = num_batches->data_ptr<int64_t>();
  }
  for (const auto* t : {&w, &b, &rmean, &rvar})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->numel() == C && (*t)->is_contiguous(),
                  "bn1d_gathered_fwd: [C] parameters");
  auto y = at::empty_like(x);
  auto stats = at::empty({2 * C + 1}, x.options());
  const bool ok = bn1d_gathered_fwd(x.data_ptr<float>(), gathered.data_ptr<float>(), R, fptr(w),
                                    fptr(b), N, C, relu, (float)eps, (float)momentum,
                                    stats.data_ptr<float>(), fptr(rmean), fptr(rvar), nb,
                                    y.data_ptr<float>(),
                                    const_cast<uint8_t*>(mask_ptr(mask_out, x)),
                                    planes_ptr(planes_out, x), cur_stream());
  if (!ok) return {};
  return {y, stats};
}

Tensor bn1d_sums_op(const Tensor& dy, const Tensor& x, const Tensor& stats,
                    const c10::optional<Tensor>& mask, const c10::optional<Tensor>& dw,
                    const c10::optional<Tensor>& db) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes(), "bn1d_sums: [rows, C] dy and x");
  const int N = (int)x.size(0), C = (int)x.size(1);
  TORCH_CHECK(stats.numel() == 2 * C + 1, "bn1d_sums: stats must be [2C+1]");
  for (const auto* t : {&dw, &db})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->numel() == C && (*t)->is_contiguous(), "bn1d_sums: [C] gradients");
  auto sums = at::empty({2 * C}, x.options());
  if (!bn1d_sums(dy.data_ptr<float>(), x.data_ptr<float>(), stats.data_ptr<float>(), N, C,
                 mask_ptr(mask, x), sums.data_ptr<float>(), fptr(dw), fptr(db), cur_stream()))
    return Tensor();
  return sums;
}

// its backward: dx (dw / db overwritten when given); undefined when the shape is not taken
Tensor bn1d_local_bwd_op(const Tensor& dy, const Tensor& x, const Tensor& stats,
                         const c10::optional<Tensor>& w, const c10::optional<Tensor>& mask,
                         const c10::optional<Tensor>& dw, const c10::optional<Tensor>& db,
                         const c10::optional<Tensor>& planes_out, SyncBackend* backend,
                         int64_t w_offset, int64_t w_span, int64_t b_offset, int64_t b_span) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes(), "bn1d_local_bwd: [rows, C] dy and x");
  const int N = (int)x.size(0), C = (int)x.size(1);
  TORCH_CHECK(stats.numel() == 2 * C + 1, "bn1d_local_bwd: stats must be [2C+1]");
  for (const auto* t : {&dw, &db})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->numel() == C && (*t)->is_contiguous(), "bn1d_local_bwd: [C] gradients");
  // world size 1 + fused optimizer (backend given): w / b updated in place by the kernel, their
  // arena ranges marked done for the reducer (as head_bwd does)
  OptEpilogue wo, bo;
  if (backend != nullptr && (w_offset >= 0 || b_offset >= 0)) {
    TORCH_CHECK(backend->epilogue_allowed(), "bn1d_local_bwd: optimizer epilogue not allowed");
    auto ops = std::dynamic_pointer_cast<RcclOps>(backend->ops());
    TORCH_CHECK(ops != nullptr, "bn1d_local_bwd: optimizer epilogue needs the device backend");
    const FusedOptimizer& f = ops->fused;
    auto at_off = [&](int64_t off) {
      OptEpilogue o;
      o.kind = f.kind;
      o.p = f.p + off;
      o.s0 = f.s0 ? f.s0 + off : nullptr;
      o.s1 = f.s1 ? f.s1 + off : nullptr;
      o.s2 = f.s2 ? f.s2 + off : nullptr;
      o.sgd = f.sgd;
      o.adam = f.adam;
      return o;
    };
    if (w_offset >= 0) {
      TORCH_CHECK(w_span >= C && w.has_value() && w->defined() &&
                      w->data_ptr<float>() == f.p + w_offset,
                  "bn1d_local_bwd: w must be the arena parameter at w_offset");
      wo = at_off(w_offset);
    }
    if (b_offset >= 0) {
      TORCH_CHECK(b_span >= C, "bn1d_local_bwd: bias span shorter than the bias");
      bo = at_off(b_offset);
    }
  }
  auto dx = at::empty_like(x);
  const bool ok = bn1d_local_bwd(dy.data_ptr<float>(), x.data_ptr<float>(),
                                 stats.data_ptr<float>(), fptr(w), N, C, mask_ptr(mask, x),
                                 dx.data_ptr<float>(), fptr(dw), fptr(db),
                                 planes_ptr(planes_out, x), cur_stream(), wo.kind ? &wo : nullptr,
                                 bo.kind ? &bo : nullptr);
  if (!ok) return Tensor();
  if (wo.kind) backend->note_epilogue(w_offset, w_span);
  if (bo.kind) backend->note_epilogue(b_offset, b_span);
  return dx;
}

Tensor bn_eval_op(const Tensor& x, const Tensor& rmean, const Tensor& rvar,
                  const c10::optional<Tensor>& w, const c10::optional<Tensor>& b, double eps,
                  bool relu) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  int N, C, HW;
  bn_dims(x, N, C, HW);
  auto y = at::empty_like(x);
  bn_eval(x.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(), fptr(w), fptr(b),
          N, C, HW, (float)eps, relu, y.data_ptr<float>(), cur_stream());
  return y;
}

// returns sums [sum_dy(C) | sum_dy_xmu(C)] ; writes dw/db when given (grad_beta: accumulate)
Tensor bn_bwd_reduce_op(const Tensor& dy, const Tensor& x, const Tensor& stats,
                        const c10::optional<Tensor>& y_relu, const c10::optional<Tensor>& dw,
                        const c10::optional<Tensor>& db, double grad_beta,
                        const c10::optional<Tensor>& mask) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  int N, C, HW;
  bn_dims(x, N, C, HW);
  const int splits = bn_splits(N, C, HW, num_cus(x.get_device()));
  auto sums = at::empty({2 * C}, x.options());
  Tensor ws = at::empty({2L * C * splits}, x.options());
  const float* sp = stats.data_ptr<float>();
  bn_bwd_reduce(dy.data_ptr<float>(), x.data_ptr<float>(), sp, sp + C, fptr(y_relu), N, C, HW,
                splits, ws.data_ptr<float>(), sums.data_ptr<float>(), fptr(dw), fptr(db),
                (float)grad_beta, cur_stream(), mask_ptr(mask, x));
  return sums;
}

// returns dx, or [dx, dresidual] when residual_grad (the fused residual input's gradient)
std::vector<Tensor> bn_bwd_elemt_op(const Tensor& dy, const Tensor& x, const Tensor& stats,
                                    const c10::optional<Tensor>& w, const Tensor& sums,
                                    const c10::optional<Tensor>& y_relu, bool residual_grad,
                                    const c10::optional<Tensor>& mask,
                                    const c10::optional<Tensor>& planes_out) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  int N, C, HW;
  bn_dims(x, N, C, HW);
  auto dx = at::empty_like(x);
  Tensor dres;
  if (residual_grad) dres = at::empty_like(x);
  const float* sp = stats.data_ptr<float>();
  bn_bwd_elemt(dy.data_ptr<float>(), x.data_ptr<float>(), sp, sp + C, fptr(w),
               sums.data_ptr<float>(), fptr(y_relu), sp + 2 * C, N, C, HW, dx.data_ptr<float>(),
               cur_stream(), residual_grad ? dres.data_ptr<float>() : nullptr,
               mask_ptr(mask, x), planes_ptr(planes_out, x));
  if (residual_grad) return {dx, dres};
  return {dx};
}

// ---------------------------------------------------------------------------------- conv / pool
ConvGeom conv_geom(const std::vector<int64_t>& xs, const std::vector<int64_t>& ws,
                   int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  TORCH_CHECK(xs.size() == 4 && ws.size() == 4, "conv2d: 4-D input and weight expected");
  TORCH_CHECK(xs[1] == ws[1], "conv2d: input channels ", xs[1], " != weight channels ", ws[1],
              " (groups are not supported)");
  ConvGeom g;
  g.N = (int)xs[0]; g.C = (int)xs[1]; g.H = (int)xs[2]; g.W = (int)xs[3];
  g.Cout = (int)ws[0]; g.R = (int)ws[2]; g.S = (int)ws[3];
  g.sh = (int)sh; g.sw = (int)sw; g.ph = (int)ph; g.pw = (int)pw;
  g.P = (g.H + 2 * g.ph - g.R) / g.sh + 1;
  g.Q = (g.W + 2 * g.pw - g.S) / g.sw + 1;
  TORCH_CHECK(g.P > 0 && g.Q > 0, "conv2d: empty output");
  TORCH_CHECK((long)g.N * g.C * g.H * g.W < (1L << 31) && (long)g.N * g.Cout * g.P * g.Q < (1L << 31),
              "conv2d: tensors must have < 2^31 elements");
  return g;
}

Tensor conv_exec(int mode, const ConvGeom& g, const Tensor& A, const Tensor& B, Tensor C,
                 const c10::optional<Tensor>& bias, bool relu, double beta) {
  const ConvPlan pl = conv_plan(mode, g, num_cus(C.get_device()));
  Tensor ws;
  if (pl.ws_floats > 0) ws = at::empty({pl.ws_floats}, C.options());
  conv_run(pl, g, A.data_ptr<float>(), B.data_ptr<float>(), C.data_ptr<float>(), fptr(bias),
           relu, (float)beta, pl.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  return C;
}

Tensor conv2d_fwd_op(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                     int64_t sh, int64_t sw, int64_t ph, int64_t pw, bool relu) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_GPU(w); CHECK_F32(w); CHECK_CONTIG(w);
  const ConvGeom g = conv_geom(x.sizes().vec(), w.sizes().vec(), sh, sw, ph, pw);
  auto y = at::empty({g.N, g.Cout, g.P, g.Q}, x.options());
  return conv_exec(kConvFwd, g, w, x, y, bias, relu, 0.0);
}

Tensor conv2d_dgrad_op(const Tensor& dy, const Tensor& w, std::vector<int64_t> x_shape,
                       int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(w);
  const ConvGeom g = conv_geom(x_shape, w.sizes().vec(), sh, sw, ph, pw);
  TORCH_CHECK(dy.size(2) == g.P && dy.size(3) == g.Q, "conv2d dgrad: dy shape mismatch");
  auto dx = at::empty(x_shape, dy.options());
  return conv_exec(kConvDgrad, g, w, dy, dx, c10::nullopt, false, 0.0);
}

void conv2d_wgrad_op(const Tensor& dy, const Tensor& x, Tensor& dw, int64_t sh, int64_t sw,
                     int64_t ph, int64_t pw, double beta) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_CONTIG(dw);
  const ConvGeom g = conv_geom(x.sizes().vec(), dw.sizes().vec(), sh, sw, ph, pw);
  conv_exec(kConvWgrad, g, dy, x, dw, c10::nullopt, false, beta);
}

// ------------------------------------------------------------- NHWC (channels_last) conv path
#define CHECK_CL(x)                                                                      \
  TORCH_CHECK((x).dim() == 4 && (x).is_contiguous(at::MemoryFormat::ChannelsLast),       \
              #x " must be a channels_last 4-D tensor")

ConvGeom nhwc_geom(const std::vector<int64_t>& xs, int64_t cout, int64_t R, int64_t S,
                   int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  return conv_geom(xs, {cout, xs[1], R, S}, sh, sw, ph, pw);
}

Tensor conv_nhwc_exec(int mode, const ConvGeom& g, const Tensor& A, const Tensor& B, Tensor C,
                      const c10::optional<Tensor>& bias, bool relu, double beta,
                      const WeightTaps* wtap = nullptr, Tensor* stats = nullptr) {
  TORCH_CHECK(conv_nhwc_ok(mode, g), "conv (NHWC): channels must be multiples of 4 and "
              "input-gradient strides powers of two");
  const ConvPlan pl = conv_nhwc_plan(mode, g, num_cus(C.get_device()));
  Tensor ws;
  if (pl.ws_floats > 0) ws = at::empty({pl.ws_floats}, C.options());
  Tensor st;
  if (stats != nullptr && pl.splits == 1)
    st = at::empty({(pl.M + pl.bm - 1) / pl.bm, 3, (int64_t)pl.N}, C.options());
  const bool wrote = conv_nhwc_run(pl, g, A.data_ptr<float>(), B.data_ptr<float>(),
                                   C.data_ptr<float>(), fptr(bias), relu, (float)beta,
                                   pl.ws_floats > 0 ? ws.data_ptr<float>() : nullptr,
                                   cur_stream(), wtap, st.defined() ? st.data_ptr<float>() : nullptr);
  if (stats != nullptr) *stats = wrote ? st : Tensor();
  return C;
}

// the weight parameter [Cout, C, R, S] in channels_last memory = a contiguous [Cout][R][S][C]
void check_weight_cl(const Tensor& w) {
  CHECK_GPU(w); CHECK_F32(w);
  TORCH_CHECK(w.dim() == 4 && w.permute({0, 2, 3, 1}).is_contiguous(),
              "conv weight must be channels_last ([Cout][R][S][C] memory)");
}

// Input gradient straight from the channels_last weight parameter (stride 1); with `out`,
// written there as out = dgrad + beta * out (a residual block's shared input gradient)
Tensor conv_nhwc_dgrad_w_op(const Tensor& dy, const Tensor& w, std::vector<int64_t> x_shape,
                            int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                            const c10::optional<Tensor>& out, double beta) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CL(dy);
  check_weight_cl(w);
  const int64_t R = w.size(2), S = w.size(3);
  TORCH_CHECK(sh == 1 && sw == 1, "dgrad_w: stride 1 (strided gradients go by phases)");
  const ConvGeom g = nhwc_geom(x_shape, dy.size(1), R, S, sh, sw, ph, pw);
  TORCH_CHECK(w.size(0) == g.Cout && w.size(1) == g.C, "dgrad_w: weight shape");
  TORCH_CHECK(dy.size(2) == g.P && dy.size(3) == g.Q && dy.size(0) == g.N, "dgrad_w: dy shape");
  Tensor dx;
  if (out.has_value()) {
    dx = *out;
    CHECK_GPU(dx); CHECK_F32(dx); CHECK_CL(dx);
    TORCH_CHECK(dx.sizes().vec() == x_shape, "dgrad_w: out shape");
  } else {
    TORCH_CHECK(beta == 0.0, "dgrad_w: beta needs out");
    dx = at::empty(x_shape, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  const WeightTaps t{(int)R, (int)S, 0, 0, 1, 1};
  return conv_nhwc_exec(kConvDgrad, g, dy, w, dx, c10::nullopt, false, beta, &t);
}

// One stride phase of a strided input gradient with the phase's taps read from the weight
Tensor conv_nhwc_dgrad_phase_w_op(const Tensor& dy, const Tensor& w, int64_t Hp, int64_t Wp,
                                  int64_t Rp, int64_t Sp, int64_t da, int64_t db, int64_t r0,
                                  int64_t s0, int64_t sh, int64_t sw) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CL(dy);
  check_weight_cl(w);
  ConvGeom g;
  g.N = (int)dy.size(0); g.Cout = (int)dy.size(1); g.P = (int)dy.size(2); g.Q = (int)dy.size(3);
  g.C = (int)w.size(1); g.H = (int)Hp; g.W = (int)Wp; g.R = (int)Rp; g.S = (int)Sp;
  g.sh = 1; g.sw = 1; g.ph = (int)da; g.pw = (int)db;
  TORCH_CHECK(w.size(0) == g.Cout, "dgrad phase: weight / dy channels differ");
  TORCH_CHECK(Rp > 0 && Sp > 0 && Hp > 0 && Wp > 0, "dgrad phase: empty phase");
  TORCH_CHECK(r0 + (Rp - 1) * sh < w.size(2) && s0 + (Sp - 1) * sw < w.size(3),
              "dgrad phase: taps outside the filter");
  TORCH_CHECK((long)g.N * g.C * Hp * Wp < (1L << 31), "dgrad phase: < 2^31 elements");
  auto out = at::empty({g.N, (int64_t)g.C, Hp, Wp},
                       dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const WeightTaps t{(int)w.size(2), (int)w.size(3), (int)r0, (int)s0, (int)sh, (int)sw};
  return conv_nhwc_exec(kConvDgrad, g, dy, w, out, c10::nullopt, false, 0.0, &t);
}

// dst = src over dst's logical shape (any strides); where an index is outside src's shape the
// element is 0 (channel padding / un-padding, layout changes, strided phase scatters).
// accumulate: dst += src where src has the index, dst unchanged elsewhere
void copy4d_op(Tensor& dst, const Tensor& src, bool accumulate) {
  CHECK_GPU(dst); CHECK_GPU(src); CHECK_F32(dst); CHECK_F32(src);
  TORCH_CHECK(dst.dim() == 4 && src.dim() == 4, "copy4d: 4-D tensors");
  Copy4D c{};
  for (int i = 0; i < 4; ++i) {
    c.dsz[i] = dst.size(i); c.dst_stride[i] = dst.stride(i);
    c.ssz[i] = src.size(i); c.src_stride[i] = src.stride(i);
  }
  c.accumulate = accumulate;
  copy4d(src.data_ptr<float>(), dst.data_ptr<float>(), c, cur_stream());
}

// x channels_last [N,C,H,W]; wt [Cout, R*S*C] (k = (r, s, c)) -> y channels_last
Tensor conv_nhwc_fwd_op(const Tensor& x, const Tensor& wt, const c10::optional<Tensor>& bias,
                        int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                        bool relu) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CL(x); CHECK_GPU(wt); CHECK_CONTIG(wt);
  const ConvGeom g = nhwc_geom(x.sizes().vec(), wt.size(0), R, S, sh, sw, ph, pw);
  TORCH_CHECK(wt.numel() == (int64_t)g.Cout * R * S * g.C, "conv (NHWC): weight size mismatch");
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == g.Cout, "bias size");
  auto y = at::empty({g.N, g.Cout, g.P, g.Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  return conv_nhwc_exec(kConvFwd, g, x, wt, y, bias, relu, 0.0);
}

// Forward that also returns the output's per-tile column (count, mean, M2) for a following
// BatchNorm (bn_moments_partials), or an undefined tensor when the plan cannot produce them
std::vector<Tensor> conv_nhwc_fwd_stats_op(const Tensor& x, const Tensor& wt, int64_t R,
                                           int64_t S, int64_t sh, int64_t sw, int64_t ph,
                                           int64_t pw) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CL(x); CHECK_GPU(wt); CHECK_CONTIG(wt);
  const ConvGeom g = nhwc_geom(x.sizes().vec(), wt.size(0), R, S, sh, sw, ph, pw);
  TORCH_CHECK(wt.numel() == (int64_t)g.Cout * R * S * g.C, "conv (NHWC): weight size mismatch");
  auto y = at::empty({g.N, g.Cout, g.P, g.Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor st;
  conv_nhwc_exec(kConvFwd, g, x, wt, y, c10::nullopt, false, 0.0, nullptr, &st);
  return {y, st};
}

// part [T, 3, C] per-tile (count, mean, M2) -> [mean(C) | var(C) | count], bn_moments' layout
Tensor bn_moments_partials_op(const Tensor& part, double count) {
  CHECK_GPU(part); CHECK_F32(part); CHECK_CONTIG(part);
  TORCH_CHECK(part.dim() == 3 && part.size(1) == 3, "bn_moments_partials: part [T, 3, C]");
  const int T = (int)part.size(0), C = (int)part.size(2);
  auto st = at::empty({2 * C + 1}, part.options());
  auto ws = at::empty({bn_partials_ws_floats(T, C)}, part.options());
  float* sp = st.data_ptr<float>();
  bn_moments_partials(part.data_ptr<float>(), T, C, ws.data_ptr<float>(), sp, sp + C,
                      sp + 2 * C, (float)count, cur_stream());
  return st;
}

// dy channels_last [N,Cout,P,Q]; w2 [R*S*Cout, C] -> dx channels_last x_shape
Tensor conv_nhwc_dgrad_op(const Tensor& dy, const Tensor& w2, std::vector<int64_t> x_shape,
                          int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CL(dy); CHECK_CONTIG(w2);
  const ConvGeom g = nhwc_geom(x_shape, dy.size(1), R, S, sh, sw, ph, pw);
  TORCH_CHECK(dy.size(2) == g.P && dy.size(3) == g.Q && dy.size(0) == g.N, "dgrad: dy shape");
  TORCH_CHECK(w2.numel() == (int64_t)g.Cout * R * S * g.C, "dgrad: weight size mismatch");
  auto dx = at::empty(x_shape, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  return conv_nhwc_exec(kConvDgrad, g, dy, w2, dx, c10::nullopt, false, 0.0);
}

// One stride phase of a strided input gradient, computed as a stride-1 implicit GEMM over the
// phase's sub-grid: out[n][i][j][c] = sum_(t,u,co) dy[n][i+da-t][j+db-u][co] * w2p[t][u][co][c]
// (w2p = the phase's taps of W2). Returns a channels_last [N, C, Hp, Wp] tensor.
Tensor conv_nhwc_dgrad_phase_op(const Tensor& dy, const Tensor& w2p, int64_t C, int64_t Hp,
                                int64_t Wp, int64_t Rp, int64_t Sp, int64_t da, int64_t db) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CL(dy); CHECK_CONTIG(w2p);
  ConvGeom g;
  g.N = (int)dy.size(0); g.Cout = (int)dy.size(1); g.P = (int)dy.size(2); g.Q = (int)dy.size(3);
  g.C = (int)C; g.H = (int)Hp; g.W = (int)Wp; g.R = (int)Rp; g.S = (int)Sp;
  g.sh = 1; g.sw = 1; g.ph = (int)da; g.pw = (int)db;
  TORCH_CHECK(Rp > 0 && Sp > 0 && Hp > 0 && Wp > 0, "dgrad phase: empty phase");
  TORCH_CHECK(w2p.numel() == Rp * Sp * g.Cout * C, "dgrad phase: weight size mismatch");
  TORCH_CHECK((long)g.N * C * Hp * Wp < (1L << 31), "dgrad phase: < 2^31 elements");
  auto out = at::empty({g.N, (int64_t)C, Hp, Wp},
                       dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  return conv_nhwc_exec(kConvDgrad, g, dy, w2p, out, c10::nullopt, false, 0.0);
}

// dy channels_last, x channels_last -> dwt [Cout, R*S*C] (dwt = beta*dwt + grad)
void conv_nhwc_wgrad_op(const Tensor& dy, const Tensor& x, Tensor& dwt, int64_t R, int64_t S,
                        int64_t sh, int64_t sw, int64_t ph, int64_t pw, double beta) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CL(dy); CHECK_CL(x); CHECK_CONTIG(dwt);
  const ConvGeom g = nhwc_geom(x.sizes().vec(), dy.size(1), R, S, sh, sw, ph, pw);
  TORCH_CHECK(dy.size(2) == g.P && dy.size(3) == g.Q, "wgrad: dy shape");
  TORCH_CHECK(dwt.numel() == (int64_t)g.Cout * R * S * g.C, "wgrad: dw size mismatch");
  conv_nhwc_exec(kConvWgrad, g, dy, x, dwt, c10::nullopt, false, beta);
}

// NHWC pooling: x channels_last -> y channels_last
std::vector<Tensor> maxpool_nhwc_fwd_op(const Tensor& x, int64_t k, int64_t s, int64_t pad) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CL(x);
  TORCH_CHECK(x.numel() < (1L << 31), "max_pool2d: < 2^31 elements");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int P = (H + 2 * (int)pad - (int)k) / (int)s + 1, Q = (W + 2 * (int)pad - (int)k) / (int)s + 1;
  auto y = at::empty({N, C, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, C, P, Q},
                       x.options().dtype(at::kInt).memory_format(at::MemoryFormat::ChannelsLast));
  maxpool2d_nhwc_fwd(x.data_ptr<float>(), N, H, W, C, P, Q, (int)k, (int)s, (int)pad,
                     y.data_ptr<float>(), idx.data_ptr<int>(), cur_stream());
  return {y, idx};
}

Tensor maxpool_nhwc_bwd_op(const Tensor& dy, const Tensor& idx, std::vector<int64_t> x_shape,
                           int64_t k, int64_t s, int64_t pad) {
  CHECK_GPU(dy); CHECK_CL(dy); CHECK_CL(idx);
  auto dx = at::empty(x_shape, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  maxpool2d_nhwc_bwd(dy.data_ptr<float>(), idx.data_ptr<int>(), (int)x_shape[0],
                     (int)x_shape[2], (int)x_shape[3], (int)x_shape[1], (int)dy.size(2),
                     (int)dy.size(3), (int)k, (int)s, (int)pad, dx.data_ptr<float>(),
                     cur_stream());
  return dx;
}

Tensor avgpool_nhwc_fwd_op(const Tensor& x, int64_t P, int64_t Q) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CL(x);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  auto y = at::empty({N, C, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  avgpool2d_nhwc_fwd(x.data_ptr<float>(), N, H, W, C, (int)P, (int)Q, y.data_ptr<float>(),
                     cur_stream());
  return y;
}

Tensor avgpool_nhwc_bwd_op(const Tensor& dy, std::vector<int64_t> x_shape) {
  CHECK_GPU(dy); CHECK_F32(dy);
  auto d = dy.contiguous(at::MemoryFormat::ChannelsLast);
  auto dx = at::empty(x_shape, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  avgpool2d_nhwc_bwd(d.data_ptr<float>(), (int)x_shape[0], (int)x_shape[2], (int)x_shape[3],
                     (int)x_shape[1], (int)dy.size(2), (int)dy.size(3), dx.data_ptr<float>(),
                     cur_stream());
  return dx;
}

// NCHW: g = dy*(y>0) (new tensor, or dy itself when y is None); db (optional) = per-channel sum
Tensor chan_relu_bias_bwd_op(const Tensor& dy, const c10::optional<Tensor>& y,
                             const c10::optional<Tensor>& db, double beta) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_CONTIG(dy);
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  const int HW = (int)(dy.numel() / ((int64_t)N * C));
  const bool has_y = y.has_value() && y->defined();
  Tensor g = has_y ? at::empty_like(dy) : dy;
  float* dbp = fptr(db);
  if (!has_y && !dbp) return g;
  const int sp = chan_splits(N, C, HW, num_cus(dy.get_device()));
  Tensor part = at::empty({(int64_t)sp * C}, dy.options());
  chan_relu_bias_bwd(dy.data_ptr<float>(), has_y ? y->data_ptr<float>() : nullptr, N, C, HW,
                     g.data_ptr<float>(), dbp, (float)beta, part.data_ptr<float>(), sp,
                     cur_stream());
  return g;
}

std::vector<Tensor> maxpool2d_fwd_op(const Tensor& x, int64_t k, int64_t s, int64_t pad) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4, "max_pool2d: 4-D input expected");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int P = (H + 2 * (int)pad - (int)k) / (int)s + 1, Q = (W + 2 * (int)pad - (int)k) / (int)s + 1;
  auto y = at::empty({N, C, P, Q}, x.options());
  auto idx = at::empty({N, C, P, Q}, x.options().dtype(at::kInt));
  maxpool2d_fwd(x.data_ptr<float>(), N * C, H, W, P, Q, (int)k, (int)s, (int)pad,
                y.data_ptr<float>(), idx.data_ptr<int>(), cur_stream());
  return {y, idx};
}

Tensor maxpool2d_bwd_op(const Tensor& dy, const Tensor& idx, std::vector<int64_t> x_shape,
                        int64_t k, int64_t s, int64_t pad) {
  CHECK_GPU(dy); CHECK_CONTIG(dy); CHECK_CONTIG(idx);
  auto dx = at::empty(x_shape, dy.options());
  maxpool2d_bwd(dy.contiguous().data_ptr<float>(), idx.data_ptr<int>(),
                (int)(x_shape[0] * x_shape[1]), (int)x_shape[2], (int)x_shape[3],
                (int)dy.size(2), (int)dy.size(3), (int)k, (int)s, (int)pad, dx.data_ptr<float>(),
                cur_stream());
  return dx;
}

Tensor avgpool_fwd_op(const Tensor& x, int64_t P, int64_t Q) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  auto y = at::empty({N, C, P, Q}, x.options());
  avgpool2d_adaptive_fwd(x.data_ptr<float>(), N * C, H, W, (int)P, (int)Q, y.data_ptr<float>(),
                         cur_stream());
  return y;
}

Tensor avgpool_bwd_op(const Tensor& dy, std::vector<int64_t> x_shape) {
  CHECK_GPU(dy); CHECK_F32(dy);
  auto d = dy.contiguous();
  auto dx = at::empty(x_shape, dy.options());
  avgpool2d_adaptive_bwd(d.data_ptr<float>(), (int)(x_shape[0] * x_shape[1]), (int)x_shape[2],
                         (int)x_shape[3], (int)dy.size(2), (int)dy.size(3), dx.data_ptr<float>(),
                         cur_stream());
  return dx;
}

Tensor dropout_op(const Tensor& x, double p, int64_t seed) {
  CHECK_GPU(x); CHECK_F32(x);
  TORCH_CHECK(x.is_non_overlapping_and_dense(), "dropout: dense input expected");
  auto y = at::empty_like(x);
  dropout_apply(x.data_ptr<float>(), x.numel(), (float)p, (uint64_t)seed, y.data_ptr<float>(),
                cur_stream());
  return y;
}

// elementwise ops work on any dense layout; operands must share it (callers make them match)
#define CHECK_SAME_DENSE(a, b)                                                             \
  TORCH_CHECK((a).is_non_overlapping_and_dense() && (a).sizes() == (b).sizes() &&          \
                  (a).strides() == (b).strides(),                                          \
              #a " and " #b " must be dense tensors of the same shape and layout")

Tensor add_relu_op(const Tensor& a, const Tensor& b, bool relu) {
  CHECK_GPU(a); CHECK_F32(a); CHECK_F32(b); CHECK_SAME_DENSE(a, b);
  auto y = at::empty_like(a);
  add_relu(a.data_ptr<float>(), b.data_ptr<float>(), a.numel(), relu, y.data_ptr<float>(),
           cur_stream());
  return y;
}

Tensor relu_mask_op(const Tensor& dy, const Tensor& y) {
  CHECK_GPU(dy); CHECK_F32(dy); CHECK_SAME_DENSE(dy, y);
  auto g = at::empty_like(dy);
  relu_mask(dy.data_ptr<float>(), y.data_ptr<float>(), dy.numel(), g.data_ptr<float>(),
            cur_stream());
  return g;
}

// x [n, ...] fp32 contiguous, y [n] int64, idx [B] int64 (all on the GPU) -> (x[idx], y[idx])
std::vector<Tensor> gather_batch_op(const Tensor& x, const Tensor& y, const Tensor& idx,
                                    bool planes, const c10::optional<Tensor>& cursor,
                                    int64_t batch) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_GPU(y); CHECK_CONTIG(y); CHECK_GPU(idx);
  CHECK_CONTIG(idx);
  TORCH_CHECK(y.scalar_type() == at::kLong && idx.scalar_type() == at::kLong && idx.dim() == 1,
              "gather_batch: int64 labels and a 1-d int64 index");
  TORCH_CHECK(x.dim() >= 1 && y.dim() == 1 && y.size(0) == x.size(0) && x.size(0) > 0,
              "gather_batch: x [n, ...] and y [n]");
  const long n = x.size(0), F = x.numel() / n;
  int B = (int)idx.numel();
  int64_t* cur = nullptr;
  if (cursor.has_value() && cursor->defined()) {
    // cursor form: idx is the epoch's whole order, the batch is `batch` entries from cursor[0]
    CHECK_GPU(*cursor); CHECK_CONTIG(*cursor);
    TORCH_CHECK(cursor->scalar_type() == at::kLong &&
                    (cursor->numel() == 2 || cursor->numel() == 2 + batch),
                "gather_batch: cursor must be an int64 [2] or [2 + batch] device tensor "
                "{position, 0, per-row arrivals (zero)}");
    TORCH_CHECK(batch > 0 && batch <= idx.numel(), "gather_batch: bad batch for the cursor");
    TORCH_CHECK(planes && F % 4 == 0 && ((uintptr_t)x.data_ptr() & 15) == 0,
                "gather_batch: the cursor form is the planes gather (F % 4 == 0)");
    cur = cursor->data_ptr<int64_t>();
    B = (int)batch;
  }
  auto xs = x.sizes().vec();
  xs[0] = B;
  auto xb = at::empty(xs, x.options());
  auto yb = at::empty({B}, y.options());
  if (planes && F % 4 == 0 && ((uintptr_t)x.data_ptr() & 15) == 0) {
    // also the bf16 split planes of the batch rows [3][B][F] (the planes GEMM's A operand)
    auto p = at::empty({3, (long)B, F}, x.options().dtype(at::kBFloat16));
    gather_batch_planes(x.data_ptr<float>(), y.data_ptr<int64_t>(), idx.data_ptr<int64_t>(), n, F,
                        B, xb.data_ptr<float>(), yb.data_ptr<int64_t>(),
                        reinterpret_cast<uint16_t*>(p.data_ptr()), cur_stream(), cur,
                        (long)idx.numel(), cur != nullptr && cursor->numel() == 2 + batch);
    return {xb, yb, p};
  }
  gather_batch(x.data_ptr<float>(), y.data_ptr<int64_t>(), idx.data_ptr<int64_t>(), n, F, B,
               xb.data_ptr<float>(), yb.data_ptr<int64_t>(), cur_stream());
  return {xb, yb};
}

// ---------------------------------------------------------------------------------------- comm
ncclDataType_t nccl_dt(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL");
  }
  return ncclFloat32;
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "unknown reduce op ", op);
  return ncclSum;
}

py::bytes unique_id_op() {
  auto v = Communicator::unique_id();
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

std::shared_ptr<Communicator> make_comm(py::bytes uid, int rank, int world, int device) {
  std::string s = uid;
  std::vector<uint8_t> v(s.begin(), s.end());
  py::gil_scoped_release nogil;  // ncclCommInitRank blocks until every rank joined
  return std::make_shared<Communicator>(v, rank, world, device);
}

// Host-relay communicator: the Communicator interface with every collective carried by a Python
// object (parallel/relay.py: device -> host copy, torch.distributed/gloo, host -> device copy).
// RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so this is how W processes that
// share ONE MI355X run the production device path -- RcclOps, the sharded / factored / replicated
// updates, SyncBatchNorm, the DDP constructor broadcast -- with real rank != 0 slots, row shards
// and cross-rank bit-identity checks (tests/test_relay_gpu.py). Each call drains the stream the
// collective was ordered on, hands the relay tensors aliasing the device buffers, and returns
// after the relay has written the result back and synchronised the device, so the work enqueued
// on that stream afterwards sees it. Eager only: a collective issued while the stream is being
// captured raises (hipGraph capture then falls back to eager on every rank, train/graph.py).
at::ScalarType at_dtype(ncclDataType_t dt) {
  switch (dt) {
    case ncclFloat32: return at::kFloat;
    case ncclFloat64: return at::kDouble;
    case ncclFloat16: return at::kHalf;
    case ncclBfloat16: return at::kBFloat16;
    case ncclInt32: return at::kInt;
    case ncclInt64: return at::kLong;
    case ncclUint8: return at::kByte;
    case ncclInt8: return at::kChar;
    default: TORCH_CHECK(false, "relay: unsupported RCCL dtype");
  }
  return at::kFloat;
}

const char* op_name(ncclRedOp_t op) {
  switch (op) {
    case ncclSum: return "sum";
    case ncclAvg: return "avg";
    case ncclMax: return "max";
    case ncclMin: return "min";
    case ncclProd: return "prod";
    default: TORCH_CHECK(false, "relay: unsupported reduce op");
  }
  return "sum";
}

class RelayCommunicator : public Communicator {
 public:
  RelayCommunicator(int rank, int world, int device, py::object relay)
      : Communicator(rank, world, device), relay_(std::move(relay)) {}
  ~RelayCommunicator() override {
    py::gil_scoped_acquire g;
    relay_ = py::object();
  }
  bool native_rccl() const override { return false; }

  void all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                  hipStream_t s) override {
    drain(s, "all_reduce");
    py::gil_scoped_acquire g;
    relay_.attr("all_reduce")(view(send, count, dt), view(recv, count, dt), op_name(op));
  }
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) override {
    drain(s, "broadcast");
    py::gil_scoped_acquire g;
    relay_.attr("broadcast")(view(buf, count, dt), root);
  }
  void all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                  hipStream_t s) override {
    drain(s, "all_gather");
    py::gil_scoped_acquire g;
    relay_.attr("all_gather")(view(send, send_count, dt),
                              view(recv, send_count * (size_t)world(), dt));
  }
  void reduce_scatter(const void* send, void* recv, size_t recv_count, ncclDataType_t dt,
                      ncclRedOp_t op, hipStream_t s) override {
    drain(s, "reduce_scatter");
    py::gil_scoped_acquire g;
    relay_.attr("reduce_scatter")(view(send, recv_count * (size_t)world(), dt),
                                  view(recv, recv_count, dt), op_name(op));
  }
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) override {
    drain(s, "send");
    py::gil_scoped_acquire g;
    relay_.attr("send")(view(buf, count, dt), peer);
  }
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) override {
    drain(s, "recv");
    py::gil_scoped_acquire g;
    relay_.attr("recv")(view(buf, count, dt), peer);
  }
  void group_start() override {}
  void group_end() override {}
  void abort() override {}

 private:
  void drain(hipStream_t s, const char* what) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    check_hip(hipStreamIsCapturing(s, &cap), "hipStreamIsCapturing");
    if (cap != hipStreamCaptureStatusNone)
      throw std::runtime_error(std::string("host-relay communicator: ") + what +
                               " cannot be captured into a hipGraph (eager only)");
    py::gil_scoped_release nogil;
    check_hip(hipStreamSynchronize(s), "hipStreamSynchronize(relay)");
  }
  Tensor view(const void* p, size_t n, ncclDataType_t dt) const {
    auto opts = at::TensorOptions().dtype(at_dtype(dt)).device(at::kCUDA, device());
    return at::from_blob(const_cast<void*>(p), {(int64_t)n}, opts);
  }
  py::object relay_;
};

std::shared_ptr<PeerCommunicator> make_peer_comm(int rank, int world, int device,
                                                 int64_t slot_bytes) {
  return std::make_shared<PeerCommunicator>(rank, world, device, slot_bytes);
}

std::shared_ptr<RelayCommunicator> make_relay_comm(int rank, int world, int device,
                                                   py::object relay) {
  return std::make_shared<RelayCommunicator>(rank, world, device, std::move(relay));
}

// SyncOps over Python callables: torch.distributed (gloo) collectives and torch math on CPU arenas
// (parallel/ddp.py _cpu_sync_ops). The C++ SyncBackend algorithm -- bucket order, sharding, tails,
// clipping, deferred updates -- runs unchanged on top, so the multi-rank logic is exercised by
// the gloo tests at any world size.
struct PyOps : SyncOps {
  int rank_, world_;
  py::object fns;  // object with one method per operation
  PyOps(int rank, int world, py::object f) : rank_(rank), world_(world), fns(std::move(f)) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool on_device() const override { return false; }
  static py::list pylist(const Ranges& r) {
    py::list l;
    for (const auto& x : r) l.append(py::make_tuple(x.first, x.second));
    return l;
  }
  void all_reduce_avg(int64_t off, int64_t n, hipStream_t) override {
    fns.attr("all_reduce_avg")(off, n);
  }
  void reduce_scatter_avg(int64_t off, int64_t cnt, hipStream_t) override {
    fns.attr("reduce_scatter_avg")(off, cnt);
  }
  void all_gather_params(int64_t off, int64_t cnt, hipStream_t) override {
    fns.attr("all_gather_params")(off, cnt);
  }
  void zero_grads(int64_t off, int64_t n, hipStream_t) override { fns.attr("zero_grads")(off, n); }
  void opt_begin(hipStream_t) override { fns.attr("opt_begin")(); }
  void opt_update(const Ranges& r, hipStream_t) override { fns.attr("opt_update")(pylist(r)); }
  void clip_begin(int b, hipStream_t) override { fns.attr("clip_begin")(b); }
  void grad_sumsq(int b, const Ranges& r, hipStream_t) override {
    fns.attr("grad_sumsq")(b, pylist(r));
  }
  void sumsq_all_reduce(int b, hipStream_t) override { fns.attr("sumsq_all_reduce")(b); }
  void clip_coef(int b, hipStream_t) override { fns.attr("clip_coef")(b); }
  void scale_grads(int b, const Ranges& r, hipStream_t) override {
    fns.attr("scale_grads")(b, pylist(r));
  }
  void factor_sync(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j, hipStream_t,
                   hipStream_t) override {
    fns.attr("factor_sync")(begin, own, cnt, j.B, j.out, j.in, j.bias_off, j.replicate,
                            reinterpret_cast<intptr_t>(j.g_all),
                            reinterpret_cast<intptr_t>(j.x_all));
  }
};

// ------------------------------------------------------------------------------ input pipeline
// uint8 NHWC batch (device) -> normalised float [B, C, Ho, Wo], channels_last or NCHW memory
Tensor image_transform_op(const Tensor& x, const c10::optional<Tensor>& flip, int64_t Ho,
                          int64_t Wo, std::vector<double> mean, std::vector<double> stdv,
                          bool round_u8, bool channels_last) {
  CHECK_GPU(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4, "image_transform: uint8 [B,H,W,C]");
  const int B = (int)x.size(0), Hs = (int)x.size(1), Ws = (int)x.size(2), C = (int)x.size(3);
  TORCH_CHECK(C == 1 || C == 3 || C == 4, "image_transform: 1, 3 or 4 channels");
  TORCH_CHECK((int)mean.size() == C && (int)stdv.size() == C, "image_transform: mean/std size");
  const uint8_t* fl = nullptr;
  if (flip.has_value() && flip->defined()) {
    CHECK_GPU(*flip); CHECK_CONTIG(*flip);
    TORCH_CHECK(flip->scalar_type() == at::kByte && flip->numel() == B, "flip: uint8 [B]");
    fl = flip->data_ptr<uint8_t>();
  }
  ImageNorm nrm{};
  for (int c = 0; c < C; ++c) {
    nrm.mean[c] = (float)mean[c];
    nrm.inv_std[c] = (float)(1.0 / stdv[c]);
  }
  auto opts = x.options().dtype(at::kFloat);
  Tensor out = channels_last
                   ? at::empty({B, C, Ho, Wo}, opts.memory_format(at::MemoryFormat::ChannelsLast))
                   : at::empty({B, C, Ho, Wo}, opts);
  image_transform(x.data_ptr<uint8_t>(), fl, out.data_ptr<float>(), B, Hs, Ws, C, (int)Ho,
                  (int)Wo, nrm, round_u8, channels_last, cur_stream());
  return out;
}

// the native prefetcher plus the tensors whose memory it reads
struct PyHostLoader {
  Tensor data, labels;
  std::vector<int64_t> sample_shape;
  int64_t row_bytes = 0;
  bool pinned = true;
  std::unique_ptr<HostBatchLoader> L;
};

std::shared_ptr<PyHostLoader> make_host_loader(Tensor data, Tensor labels, int batch, int depth,
                                               int threads, bool pinned) {
  TORCH_CHECK(!data.is_cuda() && !labels.is_cuda(), "host loader: CPU tensors");
  TORCH_CHECK(data.scalar_type() == at::kByte, "host loader: uint8 samples");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.dim() == 1, "host loader: int64 labels");
  TORCH_CHECK(data.dim() >= 2 && data.size(0) == labels.size(0), "host loader: [n, ...] samples");
  auto h = std::make_shared<PyHostLoader>();
  h->data = data.contiguous();
  h->labels = labels.contiguous();
  h->sample_shape.assign(data.sizes().begin() + 1, data.sizes().end());
  h->row_bytes = h->data.numel() / h->data.size(0);
  h->pinned = pinned;
  h->L = std::make_unique<HostBatchLoader>(h->data.data_ptr<uint8_t>(),
                                           h->labels.data_ptr<int64_t>(), h->data.size(0),
                                           h->row_bytes, batch, depth, threads, pinned);
  return h;
}

// next batch: (x uint8 [rows, ...], y int64 [rows], flip uint8 [rows]) on `device` (async
// copies on the current stream from pinned staging), or None at the end of the epoch
py::object host_loader_next(PyHostLoader& h, const std::string& device) {
  const uint8_t *x = nullptr, *fl = nullptr;
  const int64_t* y = nullptr;
  int rows = 0, slot = -1;
  {
    py::gil_scoped_release nogil;  // workers may still be gathering this batch
    slot = h.L->next(&x, &y, &fl, &rows);
  }
  if (slot < 0) return py::none();
  std::vector<int64_t> xs{rows};
  xs.insert(xs.end(), h.sample_shape.begin(), h.sample_shape.end());
  const at::Device dev(device);
  auto u8 = at::TensorOptions().dtype(at::kByte).device(dev);
  Tensor dx = at::empty(xs, u8), dfl = at::empty({rows}, u8);
  Tensor dy = at::empty({rows}, at::TensorOptions().dtype(at::kLong).device(dev));
  if (dev.is_cuda()) {
    hipStream_t s = cur_stream();
    check_hip(hipMemcpyAsync(dx.data_ptr(), x, (size_t)rows * h.row_bytes,
                             hipMemcpyHostToDevice, s), "loader H2D x");
    check_hip(hipMemcpyAsync(dy.data_ptr(), y, (size_t)rows * sizeof(int64_t),
                             hipMemcpyHostToDevice, s), "loader H2D y");
    check_hip(hipMemcpyAsync(dfl.data_ptr(), fl, (size_t)rows, hipMemcpyHostToDevice, s),
              "loader H2D flip");
    h.L->release(slot, s);
  } else {
    std::memcpy(dx.data_ptr(), x, (size_t)rows * h.row_bytes);
    std::memcpy(dy.data_ptr(), y, (size_t)rows * sizeof(int64_t));
    std::memcpy(dfl.data_ptr(), fl, (size_t)rows);
    h.L->release(slot, nullptr);
  }
  return py::make_tuple(dx, dy, dfl);
}

float* block_ptr(const c10::optional<Tensor>& blk) {
  return const_cast<float*>(hyper_ptr(blk));
}

// Weight-gradient GEMM whose epilogue applies SGD to explicit tensors (the tensor-sharded
// wrapper's shards: their gradient is complete on this rank, no reduction precedes the update):
// p / buf are C-shaped contiguous slices of the parameter and momentum arenas, the scalars come
// from the optimizer's device hyper block. With rowsum and bias_p the bias is updated from the
// row sums by the same kernel. Returns whether the epilogue ran; if not, C (and rowsum) hold the
// gradient as from gemm_f32 and the caller updates them another way.
bool gemm_f32_sgd_op(const Tensor& A, const Tensor& B, Tensor& C, bool a_kcontig, bool b_kcontig,
                     const Tensor& p, const c10::optional<Tensor>& buf, const Tensor& hyper,
                     bool nesterov, bool maximize, const c10::optional<Tensor>& rowsum,
                     const c10::optional<Tensor>& bias_p, const c10::optional<Tensor>& bias_buf) {
  CHECK_GPU(A); CHECK_GPU(B); CHECK_GPU(C); CHECK_GPU(p); CHECK_GPU(hyper);
  CHECK_F32(A); CHECK_F32(B); CHECK_F32(C); CHECK_F32(p);
  CHECK_ROWMAJOR(A); CHECK_ROWMAJOR(B); CHECK_CONTIG(C); CHECK_CONTIG(p);
  const int M = (int)C.size(0), N = (int)C.size(1);
  const int K = (int)(a_kcontig ? A.size(1) : A.size(0));
  TORCH_CHECK((a_kcontig ? A.size(0) : A.size(1)) == M, "gemm: A rows != C rows");
  TORCH_CHECK((b_kcontig ? B.size(0) : B.size(1)) == N, "gemm: B cols != C cols");
  TORCH_CHECK((b_kcontig ? B.size(1) : B.size(0)) == K, "gemm: inner dims differ");
  TORCH_CHECK(p.numel() == (int64_t)M * N, "gemm_f32_sgd: p must have C's elements");
  const bool mom = buf.has_value() && buf->defined();
  if (mom) {
    CHECK_GPU(*buf); CHECK_F32(*buf); CHECK_CONTIG(*buf);
    TORCH_CHECK(buf->numel() == p.numel(), "gemm_f32_sgd: momentum buffer size");
  }
  TORCH_CHECK((int64_t)M * N < (int64_t)1 << 31, "gemm_f32_sgd: parameter too large");
  GemmF32Args a;
  a.A = A.data_ptr<float>(); a.B = B.data_ptr<float>(); a.C = C.data_ptr<float>();
  a.lda = A.stride(0); a.ldb = B.stride(0); a.ldc = N;
  a.M = M; a.N = N; a.K = K;
  a.a_kcontig = a_kcontig; a.b_kcontig = b_kcontig;
  if (rowsum.has_value() && rowsum->defined()) {
    CHECK_GPU(*rowsum); CHECK_F32(*rowsum); CHECK_CONTIG(*rowsum);
    TORCH_CHECK(rowsum->numel() == M, "gemm: rowsum must have M elements");
    a.rowsum = rowsum->data_ptr<float>();
  }
  GemmF32Args probe = a;
  probe.opt.kind = 1;
  const GemmPlan pp = gemm_f32_plan(probe, num_cus(C.get_device()));
  const bool epi = pp.fast && !pp.skinny && pp.splits == 1 && !a_kcontig && !b_kcontig;
  if (epi) {
    const SgdHyper h{0.f, mom ? 1.f : 0.f, 0.f, 0.f, nesterov, maximize, false, 1.f,
                     block_ptr(hyper)};
    a.opt.kind = 1;
    a.opt.p = p.data_ptr<float>();
    a.opt.s0 = mom ? buf->data_ptr<float>() : nullptr;
    a.opt.sgd = h;
    if (a.rowsum != nullptr && bias_p.has_value() && bias_p->defined()) {
      CHECK_GPU(*bias_p); CHECK_F32(*bias_p); CHECK_CONTIG(*bias_p);
      TORCH_CHECK(bias_p->numel() == M, "gemm_f32_sgd: the bias must have M elements");
      TORCH_CHECK(!mom || (bias_buf.has_value() && bias_buf->defined() &&
                           bias_buf->numel() == M), "gemm_f32_sgd: bias momentum buffer");
      a.bias_opt.kind = 1;
      a.bias_opt.p = bias_p->data_ptr<float>();
      a.bias_opt.s0 = mom ? bias_buf->data_ptr<float>() : nullptr;
    }
  }
  const GemmPlan plan = gemm_f32_plan(a, num_cus(C.get_device()));
  Tensor ws;
  if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, C.options());
  gemm_f32_run(a, plan, plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  return epi;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950-native kernels, RCCL communicator and gradient reducer";
  m.def("num_cus", &num_cus);
  m.def("reserved_cus", &reserved_cus);
  // a failed stream capture leaves its error as the thread's last HIP error; the next checked
  // launch would report it although the eager fallback is fine: read (and so clear) it
  m.def("take_last_hip_error", []() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? std::string() : std::string(hipGetErrorString(e));
  });
  m.def("set_reserved_cus", &set_reserved_cus);
  m.def("gemm_f32", &gemm_f32_op, py::arg("A"), py::arg("B"), py::arg("C"),
        py::arg("a_kcontig"), py::arg("b_kcontig"), py::arg("mask") = py::none(),
        py::arg("bias") = py::none(), py::arg("rowsum") = py::none(), py::arg("beta") = 0.0,
        py::arg("rowsum_beta") = 0.0, py::arg("relu") = false, py::arg("gate") = py::none());
  m.def("gemm_f32_opt", &gemm_f32_opt_op, py::arg("A"), py::arg("B"), py::arg("C"),
        py::arg("a_kcontig"), py::arg("b_kcontig"), py::arg("backend"), py::arg("offset"),
        py::arg("rowsum") = py::none(), py::arg("rowsum_beta") = 0.0,
        py::arg("bias_offset") = -1, py::arg("bias_span") = 0, py::arg("hold") = false);
  m.def("gemm_f32_sgd", &gemm_f32_sgd_op, py::arg("A"), py::arg("B"), py::arg("C"),
        py::arg("a_kcontig"), py::arg("b_kcontig"), py::arg("p"), py::arg("buf"),
        py::arg("hyper"), py::arg("nesterov") = false, py::arg("maximize") = false,
        py::arg("rowsum") = py::none(), py::arg("bias_p") = py::none(),
        py::arg("bias_buf") = py::none());
  m.def("gemm_f32_plan", &gemm_f32_plan_op);
  m.def("gemm_planes", &gemm_planes_op, py::arg("Ap"), py::arg("B"), py::arg("C"),
        py::arg("b_kcontig"), py::arg("bias") = py::none(), py::arg("relu") = false,
        py::arg("gate") = py::none(), py::arg("out_planes") = py::none());
  m.def("split_planes", &split_planes_op);
  m.def("gemm_emu8", &gemm_emu8_op, py::arg("A"), py::arg("B"), py::arg("C"),
        py::arg("b_kcontig") = true, py::arg("beta") = 0.0);
  m.def("gemm_emu8_set_waves", &gemm_emu8_set_waves);
  m.def("head_bwd", &head_bwd_op, py::arg("g"), py::arg("x"), py::arg("w"), py::arg("dx"),
        py::arg("dw"), py::arg("db") = py::none(), py::arg("gate") = py::none(),
        py::arg("planes") = false, py::arg("backend") = nullptr, py::arg("w_offset") = -1,
        py::arg("b_offset") = -1, py::arg("b_span") = 0);
  m.def("head_ce", &head_ce_op, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("labels"),
        py::arg("ignore_index"), py::arg("smoothing"), py::arg("mean"), py::arg("acc"),
        py::arg("with_grad"), py::arg("gate"), py::arg("planes"), py::arg("ticket"));
  m.def("gemm_planes_plan", &gemm_planes_plan_op);
  m.def("gemm_planes_set_cfg", &gemm_planes_set_cfg,
        "planes GEMM variant: stages 2 / 3 (one wave group), 4 = default (3 stages, two wave "
        "groups); pf = B prefetch (2 stages only); splits > 0 = split-K override",
        py::arg("stages") = 4, py::arg("pf") = 0,
        py::arg("splits") = 0);
  m.def("gemm_f32_set_mode", &gemm_f32_set_mode);
  m.def("gemm_f32_set_override", &gemm_f32_set_override);
  m.def("gemm_f32_set_cvec", &gemm_f32_set_cvec);
  m.def("gemm_f32_set_bm", &gemm_f32_set_bm);
  m.def("gemm_f32_set_emu", &gemm_f32_set_emu);
  m.def("gemm_f32_emu", &gemm_f32_emu);
  m.def("gemm_f32_set_lockstep", &gemm_f32_set_lockstep,
        "A/B: the lockstep weight-gradient + optimizer kernel (default off)");
  m.def("gemm_f32_lockstep", &gemm_f32_lockstep);
  m.def("relu_bias_bwd", &relu_bias_bwd_op, py::arg("dy"), py::arg("y") = py::none(),
        py::arg("db") = py::none(), py::arg("beta_db") = 0.0, py::arg("gscale") = 1.0);
  m.def("bias_act", &bias_act_op, py::arg("x"), py::arg("b"), py::arg("relu") = false);
  m.def("ce_fwd", &ce_fwd_op, py::arg("logits"), py::arg("labels"), py::arg("ignore_index"),
        py::arg("smoothing"), py::arg("mean"), py::arg("acc"), py::arg("with_grad") = false);
  m.def("ce_bwd", &ce_bwd_op);
  m.def("count_correct", &count_correct_op);
  m.def("sgd_flat", &sgd_flat_op, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"),
        py::arg("maximize"), py::arg("first_step"), py::arg("grad_scale") = 1.0,
        py::arg("hyper") = py::none());
  m.def("opt_step_begin", &opt_step_begin_op, py::arg("hyper"), py::arg("kind"));
  m.def("clip_grad_norm", &clip_grad_norm_op, py::arg("grads"), py::arg("hyper"),
        py::arg("max_norm"));
  m.def("hyper_slots", []() {
    return py::dict(py::arg("lr") = (int)kHLr, py::arg("mom") = (int)kHMom,
                    py::arg("damp") = (int)kHDamp, py::arg("wd") = (int)kHWd,
                    py::arg("eps") = (int)kHEps, py::arg("bc1") = (int)kHBc1,
                    py::arg("bc2") = (int)kHBc2, py::arg("first") = (int)kHFirst,
                    py::arg("first_next") = (int)kHFirstNext, py::arg("scale") = (int)kHScale,
                    py::arg("sumsq") = (int)kHSumsq, py::arg("max_norm") = (int)kHMaxNorm,
                    py::arg("step") = (int)kHStep, py::arg("norm") = (int)kHNorm,
                    py::arg("size") = (int)kHSlots);
  });
  m.def("gemm_f32_set_opt_variant", &gemm_f32_set_opt_variant, py::arg("sgd") = -1,
        py::arg("adam") = -1, py::arg("persist") = -1, py::arg("wgs") = -1);
  m.def("adam_flat", &adam_flat_op, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"),
        py::arg("vmax"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("weight_decay"), py::arg("amsgrad"), py::arg("maximize"), py::arg("decoupled"),
        py::arg("step"), py::arg("grad_scale") = 1.0, py::arg("hyper") = py::none());
  m.def("sgd_multi", &sgd_multi_op, py::arg("ps"), py::arg("gs"), py::arg("bufs"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"),
        py::arg("maximize"), py::arg("first_step"), py::arg("grad_scale") = 1.0,
        py::arg("hyper") = py::none());
  m.def("adam_multi", &adam_multi_op, py::arg("ps"), py::arg("gs"), py::arg("ms"), py::arg("vs"),
        py::arg("vmaxs"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("weight_decay"), py::arg("amsgrad"), py::arg("maximize"), py::arg("decoupled"),
        py::arg("step"), py::arg("grad_scale") = 1.0, py::arg("hyper") = py::none());
  m.def("scale_", &scale_op);
  m.def("cast_f32_bf16", &cast_f32_bf16_op);
  m.def("conv2d_fwd", &conv2d_fwd_op);
  m.def("conv_nhwc_fwd", &conv_nhwc_fwd_op);
  m.def("conv_nhwc_dgrad", &conv_nhwc_dgrad_op);
  m.def("conv_nhwc_wgrad", &conv_nhwc_wgrad_op);
  m.def("conv_nhwc_dgrad_phase", &conv_nhwc_dgrad_phase_op);
  m.def("conv_nhwc_fwd_stats", &conv_nhwc_fwd_stats_op);
  m.def("bn_moments_partials", &bn_moments_partials_op, py::arg("part"), py::arg("count"));
  m.def("conv_nhwc_dgrad_w", &conv_nhwc_dgrad_w_op, py::arg("dy"), py::arg("w"),
        py::arg("x_shape"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("out") = py::none(), py::arg("beta") = 0.0);
  m.def("conv_nhwc_dgrad_phase_w", &conv_nhwc_dgrad_phase_w_op);
  m.def("copy4d", &copy4d_op, py::arg("dst"), py::arg("src"), py::arg("accumulate") = false);
  m.def("conv_wgrad_transposed", [](int64_t cout, int64_t R, int64_t S, int64_t C) {
    ConvGeom g{};
    g.Cout = (int)cout; g.R = (int)R; g.S = (int)S; g.C = (int)C;
    return conv_wgrad_transposed(g);
  }, py::arg("cout"), py::arg("R") = 0, py::arg("S") = 0, py::arg("C") = 0);
  m.def("conv_set_wgrad_transposed", &conv_set_wgrad_transposed);
  m.def("conv_set_wgrad_target", &conv_set_wgrad_target);
  // geom = [N, C, H, W, Cout, R, S, P, Q, sh, sw, ph, pw] of the NHWC GEMM call (mode 0 fwd,
  // 1 input gradient, 2 weight gradient; an input-gradient stride phase is its own geometry)
  m.def("conv_plan_db_put", [](int64_t mode, std::vector<int64_t> v, int64_t fn, int64_t splits) {
    TORCH_CHECK(v.size() == 13, "conv_plan_db_put: geometry of 13 ints");
    ConvGeom g{(int)v[0], (int)v[1], (int)v[2], (int)v[3], (int)v[4], (int)v[5], (int)v[6],
               (int)v[7], (int)v[8], (int)v[9], (int)v[10], (int)v[11], (int)v[12]};
    conv_plan_db_put((int)mode, g, (int)fn, (int)splits);
  });
  m.def("conv_plan_db_clear", &conv_plan_db_clear);
  m.def("conv_plan_db_size", &conv_plan_db_size);
  m.def("conv2d_dgrad", &conv2d_dgrad_op);
  m.def("conv2d_wgrad", &conv2d_wgrad_op);
  m.def("chan_relu_bias_bwd", &chan_relu_bias_bwd_op, py::arg("dy"), py::arg("y") = py::none(),
        py::arg("db") = py::none(), py::arg("beta") = 0.0);
  m.def("maxpool2d_fwd", &maxpool2d_fwd_op);
  m.def("maxpool_nhwc_fwd", &maxpool_nhwc_fwd_op);
  m.def("maxpool_nhwc_bwd", &maxpool_nhwc_bwd_op);
  m.def("avgpool_nhwc_fwd", &avgpool_nhwc_fwd_op);
  m.def("avgpool_nhwc_bwd", &avgpool_nhwc_bwd_op);
  m.def("maxpool2d_bwd", &maxpool2d_bwd_op);
  m.def("avgpool_fwd", &avgpool_fwd_op);
  m.def("avgpool_bwd", &avgpool_bwd_op);
  m.def("dropout", &dropout_op);
  m.def("add_relu", &add_relu_op);
  m.def("relu_mask", &relu_mask_op);
  // this rank's factors of a factored Linear weight into slot `rank` of the all-gather buffers:
  // g [B][out] * alpha and x [B][in]; each slot holds `slot_rows` >= B rows (the batch size the
  // ranks agreed on) and rows B.. are zeroed, so a smaller (ragged last) batch on some rank
  // still issues the same collectives and contributes exactly its own rows to g_all^T x_all
  m.def("factor_stage", [](const Tensor& g, const c10::optional<Tensor>& xo, Tensor& g_all,
                          Tensor& x_all, int64_t rank, double alpha, int64_t slot_rows) {
    // x = None: x was staged (and gathered) at forward time; only g goes into its slot
    CHECK_GPU(g); CHECK_F32(g); CHECK_CONTIG(g);
    CHECK_GPU(g_all); CHECK_F32(g_all); CHECK_CONTIG(g_all);
    CHECK_GPU(x_all); CHECK_F32(x_all); CHECK_CONTIG(x_all);
    const bool has_x = xo.has_value();
    const Tensor x = has_x ? *xo : g;
    if (has_x) { CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x); }
    TORCH_CHECK(g.dim() == 2 && x.dim() == 2 && g.size(0) == x.size(0), "factor_stage: [B][*]");
    const int64_t B = g.size(0), out = g.size(1), in = has_x ? x.size(1) : 0;
    const int64_t rows = slot_rows < 0 ? B : slot_rows;
    TORCH_CHECK(B <= rows, "factor_stage: batch larger than the agreed slot");
    const int64_t ng = B * out, nx = B * in, sg = rows * out, sx = rows * in;
    TORCH_CHECK(ng % 4 == 0 && nx % 4 == 0 && sg % 4 == 0 && sx % 4 == 0,
                "factor_stage: sizes must be multiples of 4");
    TORCH_CHECK((rank + 1) * sg <= g_all.numel() && (rank + 1) * sx <= x_all.numel(),
                "factor_stage: slot out of range");
    float* gd = g_all.data_ptr<float>() + rank * sg;
    float* xd = x_all.data_ptr<float>() + rank * sx;
    hipStream_t s = cur_stream();
    if (B > 0)
      factor_stage(g.data_ptr<float>(), has_x ? x.data_ptr<float>() : nullptr, gd,
                   has_x ? xd : nullptr, ng, nx, (float)alpha, s);
    if (rows > B) {
      check_hip(hipMemsetAsync(gd + ng, 0, sizeof(float) * (size_t)(sg - ng), s), "memset(pad)");
      if (has_x)
        check_hip(hipMemsetAsync(xd + nx, 0, sizeof(float) * (size_t)(sx - nx), s), "memset(pad)");
    }
  }, py::arg("g"), py::arg("x"), py::arg("g_all"), py::arg("x_all"), py::arg("rank"),
     py::arg("alpha"), py::arg("slot_rows") = -1);
  m.def("gather_batch", &gather_batch_op, py::arg("x"), py::arg("y"), py::arg("idx"),
        py::arg("planes") = false, py::arg("cursor") = py::none(), py::arg("batch") = 0);
  m.def("image_transform", &image_transform_op, py::arg("x"), py::arg("flip"), py::arg("Ho"),
        py::arg("Wo"), py::arg("mean"), py::arg("std"), py::arg("round_u8") = true,
        py::arg("channels_last") = true);
  py::class_<PyHostLoader, std::shared_ptr<PyHostLoader>>(m, "HostBatchLoader")
      .def(py::init(&make_host_loader), py::arg("data"), py::arg("labels"), py::arg("batch"),
           py::arg("depth") = 4, py::arg("threads") = 2, py::arg("pinned") = true)
      .def("start_epoch",
           [](PyHostLoader& h, std::vector<int64_t> idx, bool drop_last, uint64_t seed,
              double p) { h.L->start_epoch(idx, drop_last, seed, (float)p); },
           py::arg("indices"), py::arg("drop_last") = false, py::arg("flip_seed") = 0,
           py::arg("flip_p") = 0.0)
      .def("num_batches", [](PyHostLoader& h) { return h.L->num_batches(); })
      .def("next", &host_loader_next, py::arg("device"));
  m.def("bn_moments", &bn_moments_op);
  m.def("bn_merge", &bn_merge_op, py::arg("gathered"), py::arg("C"), py::arg("eps"),
        py::arg("momentum"), py::arg("rmean"), py::arg("rvar"),
        py::arg("num_batches") = py::none());
  m.def("bn_elemt", &bn_elemt_op, py::arg("x"), py::arg("stats"), py::arg("w"), py::arg("b"),
        py::arg("relu"), py::arg("residual") = py::none(), py::arg("mask_out") = py::none(),
        py::arg("planes_out") = py::none());
  m.def("bn_elemt_local", &bn_elemt_local_op, py::arg("x"), py::arg("moments"), py::arg("w"),
        py::arg("b"), py::arg("relu"), py::arg("eps"), py::arg("momentum"),
        py::arg("rmean") = py::none(), py::arg("rvar") = py::none(),
        py::arg("num_batches") = py::none(), py::arg("mask_out") = py::none(),
        py::arg("planes_out") = py::none(), py::arg("residual") = py::none());
  m.def("bn1d_local_fwd", &bn1d_local_fwd_op, py::arg("x"), py::arg("w"), py::arg("b"),
        py::arg("relu"), py::arg("eps"), py::arg("momentum"), py::arg("rmean") = py::none(),
        py::arg("rvar") = py::none(), py::arg("num_batches") = py::none(),
        py::arg("mask_out") = py::none(), py::arg("planes_out") = py::none());
  m.def("bn1d_local_bwd", &bn1d_local_bwd_op, py::arg("dy"), py::arg("x"), py::arg("stats"),
        py::arg("w"), py::arg("mask") = py::none(), py::arg("dw") = py::none(),
        py::arg("db") = py::none(), py::arg("planes_out") = py::none(),
        py::arg("backend") = nullptr, py::arg("w_offset") = -1, py::arg("w_span") = 0,
        py::arg("b_offset") = -1, py::arg("b_span") = 0);
  m.def("bn1d_moments", &bn1d_moments_op, py::arg("x"));
  m.def("bn1d_gathered_fwd", &bn1d_gathered_fwd_op, py::arg("x"), py::arg("gathered"),
        py::arg("w"), py::arg("b"), py::arg("relu"), py::arg("eps"), py::arg("momentum"),
        py::arg("rmean") = py::none(), py::arg("rvar") = py::none(),
        py::arg("num_batches") = py::none(), py::arg("mask_out") = py::none(),
        py::arg("planes_out") = py::none());
  m.def("bn1d_sums", &bn1d_sums_op, py::arg("dy"), py::arg("x"), py::arg("stats"),
        py::arg("mask") = py::none(), py::arg("dw") = py::none(), py::arg("db") = py::none());
  m.def("bn_eval", &bn_eval_op);
  m.def("bn_bwd_reduce", &bn_bwd_reduce_op, py::arg("dy"), py::arg("x"), py::arg("stats"),
        py::arg("y_relu"), py::arg("dw"), py::arg("db"), py::arg("grad_beta"),
        py::arg("mask") = py::none());
  m.def("bn_bwd_elemt", &bn_bwd_elemt_op, py::arg("dy"), py::arg("x"), py::arg("stats"),
        py::arg("w"), py::arg("sums"), py::arg("y_relu"), py::arg("residual_grad") = false,
        py::arg("mask") = py::none(), py::arg("planes_out") = py::none());

  m.def("rccl_unique_id", &unique_id_op);
  m.def("debug_spin_ms", [](int ms) { debug_spin_ms(ms, cur_stream()); });
  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def(py::init(&make_comm))
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def_property_readonly("device", &Communicator::device)
      .def_property_readonly("native_rccl", &Communicator::native_rccl)
      .def_property_readonly("nranks", &Communicator::nranks)
      // collectives enqueued on the CURRENT stream (ordered with surrounding PyTorch work)
      .def("all_reduce",
           [](Communicator& c, Tensor& t, const std::string& op) {
             CHECK_GPU(t); CHECK_CONTIG(t);
             c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dt(t), nccl_op(op),
                          cur_stream());
           })
      .def("broadcast",
           [](Communicator& c, Tensor& t, int root) {
             CHECK_GPU(t); CHECK_CONTIG(t);
             c.broadcast(t.data_ptr(), t.numel(), nccl_dt(t), root, cur_stream());
           })
      .def("all_gather",
           [](Communicator& c, Tensor& out, const Tensor& in) {
             CHECK_GPU(in); CHECK_CONTIG(in); CHECK_CONTIG(out);
             TORCH_CHECK(out.numel() == in.numel() * c.world(), "all_gather: bad output size");
             c.all_gather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dt(in), cur_stream());
           })
      .def("reduce_scatter",
           [](Communicator& c, Tensor& out, const Tensor& in, const std::string& op) {
             CHECK_GPU(in); CHECK_CONTIG(in); CHECK_CONTIG(out);
             TORCH_CHECK(in.numel() == out.numel() * c.world(), "reduce_scatter: bad sizes");
             c.reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dt(in),
                              nccl_op(op), cur_stream());
           })
      .def("send",
           [](Communicator& c, const Tensor& t, int peer) {
             c.send(t.data_ptr(), t.numel(), nccl_dt(t), peer, cur_stream());
           })
      .def("recv",
           [](Communicator& c, Tensor& t, int peer) {
             c.recv(t.data_ptr(), t.numel(), nccl_dt(t), peer, cur_stream());
           })
      .def("group_start", &Communicator::group_start)
      .def("group_end", &Communicator::group_end)
      .def("abort", &Communicator::abort)
      // collective watchdog (comm.h): the work on the current stream must finish in time
      .def("watch_current",
           [](Communicator& c, const std::string& what) { c.watch(cur_stream(), what.c_str()); })
      .def_property("timeout", &Communicator::timeout, &Communicator::set_timeout)
      .def("set_watch_single_rank", &Communicator::set_watch_single_rank)
      .def("pending_watches", &Communicator::pending_watches)
      // block the host until everything enqueued on the current stream (incl. comms) finished
      .def("synchronize_current", [](Communicator&) {
        py::gil_scoped_release nogil;
        check_hip(hipStreamSynchronize(cur_stream()), "hipStreamSynchronize");
      });

  py::class_<RelayCommunicator, Communicator, std::shared_ptr<RelayCommunicator>>(
      m, "RelayCommunicator")
      .def(py::init(&make_relay_comm), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("relay"));

  py::class_<PeerCommunicator, Communicator, std::shared_ptr<PeerCommunicator>>(
      m, "PeerCommunicator")
      .def(py::init(&make_peer_comm), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("slot_bytes") = (int64_t)64 << 20)
      .def("local_handle", [](const PeerCommunicator& c) {
        auto v = c.local_handle();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("connect", [](PeerCommunicator& c, const std::vector<py::bytes>& hs) {
        std::vector<std::vector<uint8_t>> v;
        for (const auto& h : hs) {
          std::string s = h;
          v.emplace_back(s.begin(), s.end());
        }
        c.connect(v);
      })
      .def_property_readonly("slot_bytes", &PeerCommunicator::slot_bytes)
      .def("inject_stall_ms", &PeerCommunicator::inject_stall_ms)
      .def("device_error", [](PeerCommunicator& c) {
        std::string w;
        return c.device_error(&w) ? py::object(py::str(w)) : py::object(py::none());
      });

  py::class_<ReducerBackend, std::shared_ptr<ReducerBackend>>(m, "ReducerBackend")
      .def("last_comm_ms", &ReducerBackend::last_comm_ms);
  py::class_<SyncOps, std::shared_ptr<SyncOps>>(m, "SyncOps")
      .def_property_readonly("rank", &SyncOps::rank)
      .def_property_readonly("world", &SyncOps::world);
  py::class_<RcclOps, SyncOps, std::shared_ptr<RcclOps>>(m, "RcclOps")
      .def(py::init([](std::shared_ptr<Communicator> comm, Tensor grad, Tensor param,
                       int compression) {
             CHECK_GPU(grad); CHECK_CONTIG(grad); CHECK_F32(grad);
             CHECK_GPU(param); CHECK_CONTIG(param); CHECK_F32(param);
             TORCH_CHECK(grad.numel() == param.numel(), "grad/param arenas differ in size");
             return std::make_shared<RcclOps>(comm, grad.data_ptr<float>(), param.data_ptr<float>(),
                                              grad.numel(), static_cast<Compression>(compression));
           }),
           py::arg("comm"), py::arg("grad"), py::arg("param"), py::arg("compression") = 0)
      // fused optimizer over the arenas; scalars come from the device hyper block
      .def("set_fused_sgd",
           [](RcclOps& o, Tensor p, c10::optional<Tensor> buf, bool momentum, bool nesterov,
              bool maximize, Tensor hyper) {
             CHECK_GPU(p); CHECK_F32(p); CHECK_CONTIG(p);
             TORCH_CHECK(!momentum || (buf.has_value() && buf->numel() == p.numel()),
                         "fused SGD: momentum buffer required");
             o.fused.kind = 1;
             o.fused.p = p.data_ptr<float>();
             o.fused.s0 = momentum ? fptr(buf) : nullptr;
             o.fused.s1 = o.fused.s2 = nullptr;
             o.fused.hyper = block_ptr(hyper);
             o.fused.sgd = SgdHyper{0.f, momentum ? 1.f : 0.f, 0.f, 0.f, nesterov, maximize, false,
                                    1.f, o.fused.hyper};
           })
      .def("set_fused_adam",
           [](RcclOps& o, Tensor p, Tensor m, Tensor v, c10::optional<Tensor> vmax, bool amsgrad,
              bool maximize, bool decoupled, Tensor hyper) {
             CHECK_GPU(p); CHECK_F32(p); CHECK_CONTIG(p);
             TORCH_CHECK(m.numel() == p.numel() && v.numel() == p.numel(), "fused Adam: state size");
             TORCH_CHECK(!amsgrad || (vmax.has_value() && vmax->numel() == p.numel()),
                         "fused Adam: amsgrad needs max_exp_avg_sq");
             o.fused.kind = 2;
             o.fused.p = p.data_ptr<float>();
             o.fused.s0 = m.data_ptr<float>();
             o.fused.s1 = v.data_ptr<float>();
             o.fused.s2 = amsgrad ? fptr(vmax) : nullptr;
             o.fused.hyper = block_ptr(hyper);
             o.fused.adam = AdamHyper{0.f, 0.f, 0.f, 0.f, 0.f, amsgrad, maximize, decoupled,
                                      1.f, 1.f, 1.f, o.fused.hyper};
           })
      .def_readwrite("skip_collectives", &RcclOps::skip_collectives)
      .def("clear_fused", [](RcclOps& o) { o.fused = FusedOptimizer{}; })
      .def("set_clip_block", [](RcclOps& o, c10::optional<Tensor> blk) {
        o.clip_block = block_ptr(blk);
      });
  py::class_<PyOps, SyncOps, std::shared_ptr<PyOps>>(m, "PyOps")
      .def(py::init<int, int, py::object>(), py::arg("rank"), py::arg("world"), py::arg("fns"));
  py::class_<SyncBackend, ReducerBackend, std::shared_ptr<SyncBackend>>(m, "SyncBackend")
      .def(py::init<std::shared_ptr<SyncOps>, int64_t, int, bool, bool>(), py::arg("ops"),
           py::arg("numel"), py::arg("num_buckets"), py::arg("timing") = false,
           py::arg("skip_single_rank") = true)
      .def_readwrite("fused_kind", &SyncBackend::fused_kind)
      .def_readwrite("shard", &SyncBackend::shard)
      .def_readwrite("compressed", &SyncBackend::compressed)
      .def_readwrite("skip_opt_begin", &SyncBackend::skip_opt_begin)
      .def_property("clip", [](SyncBackend& b) { return (int)b.clip; },
                    [](SyncBackend& b, int v) {
                      TORCH_CHECK(v >= 0 && v <= 2, "clip mode 0 none | 1 global | 2 local");
                      b.clip = static_cast<ClipMode>(v);
                    })
      .def_property_readonly("epilogue_allowed", &SyncBackend::epilogue_allowed)
      .def_property_readonly("collective", &SyncBackend::collective)
      .def("owned_shard", &SyncBackend::owned_shard)
      .def("arm_factor",
           [](SyncBackend& b, int bucket, Tensor& g_all, Tensor& x_all, int B, int out, int in,
              int64_t bias_off, int bias_bucket, bool replicate, bool x_ready, int rep_rows,
              const c10::optional<Tensor>& g_src, double g_scale, bool g_ready) {
             // device buffers for RcclOps; host buffers for PyOps (the CPU twin looks them up by
             // address in parallel/ddp.py _CpuSyncOps.factor_sync)
             TORCH_CHECK(g_all.is_cuda() == b.ops()->on_device() &&
                         x_all.is_cuda() == b.ops()->on_device(),
                         "arm_factor: buffers must live where the sync ops run");
             CHECK_F32(g_all); CHECK_CONTIG(g_all);
             CHECK_F32(x_all); CHECK_CONTIG(x_all);
             const int64_t W = b.ops()->world();
             TORCH_CHECK(g_all.numel() == W * B * out && x_all.numel() == W * B * in,
                         "arm_factor: buffers must hold W*B rows of out / in floats");
             FactorJob j;
             j.g_all = g_all.data_ptr<float>();
             j.x_all = x_all.data_ptr<float>();
             j.B = B; j.out = out; j.in = in;
             j.bias_off = bias_off;
             j.replicate = replicate;
             j.x_ready = x_ready;
             j.g_ready = g_ready;
             j.rep_rows = replicate ? out : rep_rows;
             // g_scale: the factor of the update applied to the gathered g (1/W when the slots
             // hold unscaled g). Every rank must gather the same convention whichever way its own
             // slot was filled (out of place at a full batch, staged at a ragged one).
             j.g_scale = (float)g_scale;
             if (g_src.has_value()) {  // out-of-place g gather straight from the layer's buffer
               CHECK_GPU(*g_src); CHECK_F32(*g_src); CHECK_CONTIG(*g_src);
               TORCH_CHECK(g_src->numel() == (int64_t)B * out, "arm_factor: g must be [B][out]");
               j.g_src = g_src->data_ptr<float>();
             }
             b.arm_factor(bucket, j, bias_bucket);
           },
           py::arg("bucket"), py::arg("g_all"), py::arg("x_all"), py::arg("B"), py::arg("out"),
           py::arg("in"), py::arg("bias_off"), py::arg("bias_bucket"),
           py::arg("replicate") = false, py::arg("x_ready") = false, py::arg("rep_rows") = 0,
           py::arg("g_src") = py::none(), py::arg("g_scale") = 1.0, py::arg("g_ready") = false)
      .def("prefetch_factor_x",
           [](SyncBackend& b, int bucket, Tensor& x_all, int B, int in,
              const c10::optional<Tensor>& x) {
             CHECK_GPU(x_all); CHECK_F32(x_all); CHECK_CONTIG(x_all);
             TORCH_CHECK(x_all.numel() == (int64_t)b.ops()->world() * B * in,
                         "prefetch_factor_x: x_all must hold W*B rows of in floats");
             const float* src = nullptr;
             if (x.has_value()) {  // out of place: this rank's rows straight from the input
               CHECK_GPU(*x); CHECK_F32(*x); CHECK_CONTIG(*x);
               TORCH_CHECK(x->numel() == (int64_t)B * in, "prefetch_factor_x: x must be [B][in]");
               src = x->data_ptr<float>();
             }
             b.prefetch_factor_x(bucket, x_all.data_ptr<float>(), src, B, in, cur_stream());
           }, py::arg("bucket"), py::arg("x_all"), py::arg("B"), py::arg("in"),
           py::arg("x") = py::none())
      .def("flush", [](SyncBackend& b) { b.flush(cur_stream()); })
      .def("reserve_factor",
           [](SyncBackend& b, int64_t begin, int64_t end, Tensor& g_all, Tensor& x_all, int B,
              int out, int in, int64_t bias_off, bool replicate, int rep_rows) {
             FactorJob j;
             j.rep_rows = replicate ? out : rep_rows;
             j.g_all = g_all.data_ptr<float>();
             j.x_all = x_all.data_ptr<float>();
             j.B = B; j.out = out; j.in = in;
             j.bias_off = bias_off;
             j.replicate = replicate;
             b.reserve_factor(begin, end, j);
           })
      .def("begin_iteration", [](SyncBackend& b, bool gpu) {
        b.begin_iteration(gpu ? cur_stream() : nullptr);
      });

  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init<std::vector<int64_t>, std::vector<int64_t>, std::vector<int64_t>,
                    std::shared_ptr<ReducerBackend>>())
      .def_static("compute_bucket_bounds", &Reducer::compute_bucket_bounds)
      .def("prepare_for_backward",
           [](Reducer& r, bool gpu) { r.prepare_for_backward(gpu ? cur_stream() : nullptr); },
           py::arg("gpu") = false)
      .def_property_readonly("head_of_line_waits", &Reducer::head_of_line_waits)
      .def("mark_ready",
           [](Reducer& r, int p, bool gpu) { r.mark_ready(p, gpu ? cur_stream() : nullptr); })
      .def("finalize", [](Reducer& r, bool gpu,
                          bool allow_unused) { r.finalize(gpu ? cur_stream() : nullptr,
                                                          allow_unused); })
      .def_property_readonly("expecting", &Reducer::expecting)
      .def_property_readonly("iteration", &Reducer::iteration)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def("bucket_bounds", &Reducer::bucket_bounds)
      .def("ready_order", &Reducer::ready_order)
      .def("unready_params", &Reducer::unready_params)
      .def("last_comm_ms", &Reducer::last_comm_ms);
}
