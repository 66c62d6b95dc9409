#include "reducer.h"

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace tdp {

// ------------------------------------------------------------------------------------------------
// RcclOps: the MI355X side effects
// ------------------------------------------------------------------------------------------------
RcclOps::RcclOps(std::shared_ptr<Communicator> comm, float* grad, float* param, int64_t numel,
                 Compression compression)
    : comm_(std::move(comm)), grad_(grad), param_(param), numel_(numel),
      compression_(compression) {
  if (compression_ == Compression::BF16)
    check_hip(hipMalloc(&wire_, sizeof(uint16_t) * (size_t)numel_), "hipMalloc(wire)");
}

RcclOps::~RcclOps() {
  for (auto e : fac_ev_)
    if (e) (void)hipEventDestroy(e);
  if (wire_) (void)hipFree(wire_);
  if (factor_ws_) (void)hipFree(factor_ws_);
  if (factor_part_) (void)hipFree(factor_part_);
}

void RcclOps::all_reduce_avg(int64_t off, int64_t n, hipStream_t s) {
  if (n <= 0 || skip_collectives) return;
  float* g = grad_ + off;
  if (compression_ == Compression::BF16) {
    uint16_t* w = wire_ + off;
    f32_to_bf16_copy(g, w, n, s);
    comm_->all_reduce(w, w, (size_t)n, ncclBfloat16, ncclAvg, s);
    bf16_to_f32_copy(w, g, n, s);
  } else {
    comm_->all_reduce(g, g, (size_t)n, ncclFloat32, ncclAvg, s);
  }
}

void RcclOps::reduce_scatter_avg(int64_t off, int64_t cnt, hipStream_t s) {
  if (cnt <= 0 || skip_collectives) return;
  float* g = grad_ + off;
  // in place: RCCL's recvbuff == sendbuff + rank * recvcount
  comm_->reduce_scatter(g, g + (int64_t)comm_->rank() * cnt, (size_t)cnt, ncclFloat32, ncclAvg, s);
}

void RcclOps::all_gather_params(int64_t off, int64_t cnt, hipStream_t s) {
  if (cnt <= 0 || skip_collectives) return;
  float* p = param_ + off;
  comm_->all_gather(p + (int64_t)comm_->rank() * cnt, p, (size_t)cnt, ncclFloat32, s);
}

void RcclOps::zero_grads(int64_t off, int64_t n, hipStream_t s) {
  if (n > 0)
    check_hip(hipMemsetAsync(grad_ + off, 0, (size_t)n * sizeof(float), s), "hipMemsetAsync");
}

void RcclOps::opt_begin(hipStream_t s) {
  if (fused.kind != 0 && fused.hyper) opt_step_begin(fused.hyper, fused.kind, s);
}

// Ranges of at least kFlat elements get the vectorised flat kernel (several float4 per stream in
// flight); the small rest (biases, shard tails) goes out in multi-range launches.
static constexpr int64_t kFlat = 1 << 16;

template <class F>
static void for_range_sets(const Ranges& r, F&& f) {
  RangeSet rs;
  for (const auto& x : r) {
    if (x.second <= x.first) continue;
    rs.begin[rs.n] = x.first;
    rs.len[rs.n] = x.second - x.first;
    if (++rs.n == kMaxRanges) {
      f(rs);
      rs.n = 0;
    }
  }
  if (rs.n > 0) f(rs);
}

void RcclOps::opt_update(const Ranges& r, hipStream_t s) { opt_update_scaled(r, 1.f, s); }

void RcclOps::opt_update_scaled(const Ranges& r, float scale, hipStream_t s) {
  if (fused.kind == 0) return;
  SgdHyper sgd = fused.sgd;
  AdamHyper adam = fused.adam;
  sgd.grad_scale *= scale;
  adam.grad_scale *= scale;
  Ranges small;
  for (const auto& x : r) {
    const int64_t n = x.second - x.first, o = x.first;
    if (n <= 0) continue;
    if (n < kFlat) {
      small.push_back(x);
      continue;
    }
    if (fused.kind == 1)
      sgd_flat(fused.p + o, grad_ + o, fused.s0 ? fused.s0 + o : nullptr, n, sgd, s);
    else
      adam_flat(fused.p + o, grad_ + o, fused.s0 + o, fused.s1 + o,
                fused.s2 ? fused.s2 + o : nullptr, n, adam, s);
  }
  for_range_sets(small, [&](const RangeSet& rs) {
    if (fused.kind == 1) sgd_ranges(fused.p, grad_, fused.s0, rs, sgd, s);
    else adam_ranges(fused.p, grad_, fused.s0, fused.s1, fused.s2, rs, adam, s);
  });
}

void RcclOps::clip_begin(int b, hipStream_t s) {
  if (b == 1 && clip_block) opt_step_begin(clip_block, 0, s);
}

void RcclOps::grad_sumsq(int b, const Ranges& r, hipStream_t s) {
  float* blk = block(b);
  if (!blk) throw std::runtime_error("gradient clipping without a hyper block");
  for_range_sets(r, [&](const RangeSet& rs) { sumsq_ranges(grad_, rs, blk, s); });
}

void RcclOps::sumsq_all_reduce(int b, hipStream_t s) {
  float* blk = block(b);
  if (comm_->world() > 1 && !skip_collectives)
    comm_->all_reduce(blk + kHSumsq, blk + kHSumsq, 1, ncclFloat32, ncclSum, s);
}

void RcclOps::clip_coef(int b, hipStream_t s) { clip_coef_from_sumsq(block(b), s); }

void RcclOps::scale_grads(int b, const Ranges& r, hipStream_t s) {
  const float* blk = block(b);
  for_range_sets(r, [&](const RangeSet& rs) { scale_ranges_by(grad_, rs, blk, s); });
}

void SyncOps::factor_sync(int64_t, int64_t, int64_t, const FactorJob&, hipStream_t,
                          hipStream_t) {
  throw std::runtime_error("factored gradient synchronisation needs the device backend");
}

void SyncOps::factor_reserve(int64_t, int64_t, int64_t, const FactorJob&) {}

void SyncOps::factor_gather_x(float*, const float*, int, int, hipStream_t) {
  throw std::runtime_error("forward-time factor gathers need the device backend");
}

void RcclOps::factor_gather_x(float* x_all, const float* x_src, int B, int in, hipStream_t s) {
  if (skip_collectives) return;
  const int r = comm_->rank();
  comm_->all_gather(x_src ? x_src : x_all + (int64_t)r * B * in, x_all, (size_t)B * in,
                    ncclFloat32, s);
}

// The shard GEMM of a factored job, planned once for factor_sync and factor_reserve: this
// rank's rows of the averaged gradient, dW[m0:m0+rows][:] = g_all[:, m0:m0+rows]^T x_all.
struct RcclOps::FactorPlan {
  GemmF32Args a;
  GemmPlan plan;
  bool epi = false, bias_in_gemm = false;
  int bias_slices = 0;  // > 0: the bias column sums run as their own launch with this workspace
};

RcclOps::FactorPlan RcclOps::plan_factor(int64_t begin, int64_t own, int64_t cnt,
                                         const FactorJob& j) const {
  const int W = comm_->world();
  if (cnt <= 0 || cnt % j.in != 0) throw std::runtime_error("factor_sync: shard is not whole rows");
  int dev = 0;
  check_hip(hipGetDevice(&dev), "hipGetDevice");
  const int cus = compute_cus(dev);
  FactorPlan f;
  const int64_t m0 = (own - begin) / j.in;
  GemmF32Args& a = f.a;
  a.A = j.g_all + m0;  // stored [K = W*B][out]: MN-contiguous A, column offset m0
  a.lda = j.out;
  a.a_kcontig = false;
  a.B = j.x_all;       // stored [K][in]
  a.ldb = j.in;
  a.b_kcontig = false;
  a.C = grad_ + own;
  a.ldc = j.in;
  a.M = (int)(cnt / j.in);
  a.N = j.in;
  a.K = W * j.B;
  GemmF32Args probe = a;
  probe.opt.kind = 1;
  const GemmPlan pp = gemm_f32_plan(probe, cus);
  f.epi = fused.kind != 0 && pp.fast && !pp.skinny && pp.splits == 1;
  // replicated job: this rank owns every row, so the GEMM's row sums of the gathered g ARE the
  // whole averaged bias gradient -- the epilogue updates the bias from them (no separate column
  // reduction + update launches); a sharded job would only see its own rows' bias entries
  f.bias_in_gemm = f.epi && j.bias_off >= 0 && j.replicate && a.M == j.out;
  if (j.bias_off >= 0 && !f.bias_in_gemm) f.bias_slices = relu_bias_slices(W * j.B, j.out, cus);
  if (f.epi) {
    // the epilogue updates p / state at C's element index: the arena offset `own`
    a.opt.kind = fused.kind;
    a.opt.p = fused.p + own;
    a.opt.s0 = fused.s0 ? fused.s0 + own : nullptr;
    a.opt.s1 = fused.s1 ? fused.s1 + own : nullptr;
    a.opt.s2 = fused.s2 ? fused.s2 + own : nullptr;
    a.opt.sgd = fused.sgd;
    a.opt.adam = fused.adam;
    a.opt.sgd.grad_scale *= j.g_scale;  // unscaled gathered g: the 1/W of the average here
    a.opt.adam.grad_scale *= j.g_scale;
    if (f.bias_in_gemm) {
      a.rowsum = grad_ + j.bias_off;  // selects the row-sum tiles; never written (bias_opt)
      a.rowsum_beta = 0.f;
      a.bias_opt.kind = fused.kind;
      a.bias_opt.p = fused.p + j.bias_off;
      a.bias_opt.s0 = fused.s0 ? fused.s0 + j.bias_off : nullptr;
      a.bias_opt.s1 = fused.s1 ? fused.s1 + j.bias_off : nullptr;
      a.bias_opt.s2 = fused.s2 ? fused.s2 + j.bias_off : nullptr;
    }
  }
  f.plan = gemm_f32_plan(a, cus);
  return f;
}

void RcclOps::grow_factor_ws(const FactorPlan& f, int out, hipStream_t s) {
  auto grow = [&](float*& buf, int64_t& have, int64_t want, const char* what) {
    if (want <= have) return;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (s) check_hip(hipStreamIsCapturing(s, &cap), "hipStreamIsCapturing");
    if (cap != hipStreamCaptureStatusNone)
      throw std::runtime_error(std::string("factor_sync: ") + what +
                               " must be sized before capture (DDP.settle reserves it)");
    if (buf) check_hip(hipFree(buf), "hipFree");
    check_hip(hipMalloc(&buf, sizeof(float) * (size_t)want), "hipMalloc(factor)");
    have = want;
  };
  if (f.bias_slices > 0)
    grow(factor_part_, factor_part_floats_, (int64_t)f.bias_slices * out, "bias workspace");
  grow(factor_ws_, factor_ws_floats_, f.plan.ws_floats, "split-K workspace");
}

void RcclOps::factor_reserve(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j) {
  // eager, outside any capture: size the job's workspaces for the current bucket layout (a
  // rebuild between the first factored step and a capture changes the plans)
  grow_factor_ws(plan_factor(begin, own, cnt, j), j.out, nullptr);
}

void RcclOps::factor_sync(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j,
                          hipStream_t s, hipStream_t compute) {
  const int W = comm_->world(), r = comm_->rank();
  if (cnt <= 0 || cnt % j.in != 0) throw std::runtime_error("factor_sync: shard is not whole rows");
  if (!skip_collectives && !(j.g_ready && j.x_ready)) {
    // this rank's factor rows: out of place from the layer's buffer (g_src), or already at
    // slot r (staged on the compute stream); one RCCL group, so g and x share one launch and
    // the links carry both back to back -- each only when it was not gathered earlier
    // (x at forward time, g before the layer's input-gradient GEMM: prefetch_factor_x)
    comm_->group_start();
    if (!j.g_ready)
      comm_->all_gather(j.g_src ? j.g_src : j.g_all + (int64_t)r * j.B * j.out, j.g_all,
                        (size_t)j.B * j.out, ncclFloat32, s);
    if (!j.x_ready)
      comm_->all_gather(j.x_all + (int64_t)r * j.B * j.in, j.x_all, (size_t)j.B * j.in,
                        ncclFloat32, s);
    comm_->group_end();
  }
  // The job's arithmetic (bias column sums, shard GEMM with the update in its epilogue) runs on
  // the COMPUTE stream when the collectives ride a side stream: the comm stream then carries
  // only collectives, so the next job's gathers and this job's parameter all-gather are not
  // queued behind GEMMs (toy MLP at W > 1: fc1's g gather overlaps fc2's GEMM, fc2's parameter
  // all-gather overlaps fc1's GEMM; profiles/r8). Cross-stream edges are events (graph edges
  // under capture).
  hipStream_t gs = s;
  if (compute && compute != s) {
    for (auto& e : fac_ev_)
      if (!e) check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    if (j.gathered) {
      check_hip(hipStreamWaitEvent(compute, j.gathered, 0), "hipStreamWaitEvent(gathered)");
    } else {
      check_hip(hipEventRecord(fac_ev_[0], s), "hipEventRecord(factor)");
      check_hip(hipStreamWaitEvent(compute, fac_ev_[0], 0), "hipStreamWaitEvent(factor)");
    }
    gs = compute;
  }
  const FactorPlan f = plan_factor(begin, own, cnt, j);
  grow_factor_ws(f, j.out, gs);
  const bool split = !j.replicate && j.rep_rows > 0;
  const int64_t rep = split ? (int64_t)j.rep_rows * j.in : 0;  // replicated [begin, begin + rep)
  FactorPlan fr;
  if (split) {
    fr = plan_factor(begin, begin, rep, j);
    grow_factor_ws(fr, j.out, gs);
  }
  if (f.bias_slices > 0) {
    // the whole averaged bias gradient (column sums of the gathered g / W) and its update, on
    // every rank: identical inputs, identical results, no collective
    relu_bias_bwd_ws(j.g_all, nullptr, W * j.B, j.out, j.out, nullptr, grad_ + j.bias_off, 0.f,
                     factor_part_, f.bias_slices, gs);
    opt_update_scaled({{j.bias_off, j.bias_off + j.out}}, j.g_scale, gs);
  }
  gemm_f32_run(f.a, f.plan, factor_ws_, gs);
  if (!f.epi) opt_update_scaled({{own, own + cnt}}, j.g_scale, gs);
  if (!j.replicate) {
    if (gs != s) {
      check_hip(hipEventRecord(fac_ev_[1], gs), "hipEventRecord(factor)");
      check_hip(hipStreamWaitEvent(s, fac_ev_[1], 0), "hipStreamWaitEvent(factor)");
    }
    all_gather_params(begin + rep, cnt, s);  // the sharded rows only
  }
  if (split) {
    // the replicated rows, computed by every rank while the sharded rows travel
    gemm_f32_run(fr.a, fr.plan, factor_ws_, gs);
    if (!fr.epi) opt_update_scaled({{begin, begin + rep}}, j.g_scale, gs);
  }
}

// ------------------------------------------------------------------------------------------------
// SyncBackend: the bucket algorithm
// ------------------------------------------------------------------------------------------------
SyncBackend::SyncBackend(std::shared_ptr<SyncOps> ops, int64_t numel, int num_buckets,
                         bool timing, bool skip_single_rank)
    : ops_(std::move(ops)), numel_(numel), timing_(timing), skip_single_rank_(skip_single_rank) {
  factor_.resize(num_buckets);
  factor_skip_.assign(num_buckets, 0);
  gdone_set_.assign(num_buckets, 0);
  if (ops_->on_device()) {
    ready_.resize(num_buckets);
    for (auto& e : ready_) check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    gdone_.resize(num_buckets);
    for (auto& e : gdone_) check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    check_hip(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "event");
    if (timing_) {
      check_hip(hipEventCreate(&t0_), "event");
      check_hip(hipEventCreate(&t1_), "event");
    }
  } else {
    timing_ = false;
  }
}

SyncBackend::~SyncBackend() {
  for (auto& e : ready_) (void)hipEventDestroy(e);
  for (auto& e : gdone_) (void)hipEventDestroy(e);
  if (done_) (void)hipEventDestroy(done_);
  if (t0_) (void)hipEventDestroy(t0_);
  if (t1_) (void)hipEventDestroy(t1_);
}

bool SyncBackend::epilogue_allowed() const {
  return fused_kind != 0 && ops_->world() == 1 && skip_single_rank_ && !compressed &&
         clip == ClipMode::NONE && ops_->on_device();
}

void SyncBackend::note_epilogue(int64_t off, int64_t n) {
  if (!epilogue_allowed()) throw std::runtime_error("optimizer epilogue needs world size 1");
  if (off < 0 || n <= 0 || off + n > numel_) throw std::runtime_error("epilogue range");
  const Range r{off, off + n};
  for (const auto& e : epi_done_)
    if (e.first < r.second && r.first < e.second)
      throw std::runtime_error("optimizer epilogue: a parameter range was updated twice");
  epi_done_.insert(std::lower_bound(epi_done_.begin(), epi_done_.end(), r), r);
}

Range SyncBackend::owned_shard(int64_t begin, int64_t end) const {
  const int W = ops_->world(), r = ops_->rank();
  // shards are multiples of 64 elements so every rank's slice stays 256-B aligned for the
  // vectorised update kernels; the remainder (< 64 W elements) is all-reduced and replicated
  const int64_t cnt = (end - begin) / W / 64 * 64;
  return {begin + (int64_t)r * cnt, begin + (int64_t)(r + 1) * cnt};
}

void SyncBackend::arm_factor(int bucket, const FactorJob& j, int bias_bucket) {
  const int nb = (int)factor_.size();
  if (bucket < 0 || bucket >= nb || bias_bucket >= nb) throw std::runtime_error("arm_factor: bucket");
  if (j.B <= 0 || !j.g_all || !j.x_all) throw std::runtime_error("arm_factor: empty job");
  if ((j.bias_off >= 0) != (bias_bucket >= 0)) throw std::runtime_error("arm_factor: bias");
  factor_[bucket] = j;
  if (bias_bucket >= 0) factor_skip_[bias_bucket] = 1;
}

Range SyncBackend::factor_own(int64_t begin, int64_t end, const FactorJob& j) const {
  // replicated: every row; sharded / split: this rank's share of the rows past the replicated
  if (j.replicate) return {begin, end};
  return owned_shard(begin + (int64_t)j.rep_rows * j.in, end);
}

void SyncBackend::reserve_factor(int64_t begin, int64_t end, const FactorJob& j) {
  if (!ops_->on_device()) return;
  const Range own = factor_own(begin, end, j);
  if (own.second > own.first) ops_->factor_reserve(begin, own.first, own.second - own.first, j);
  if (!j.replicate && j.rep_rows > 0)
    ops_->factor_reserve(begin, begin, (int64_t)j.rep_rows * j.in, j);
}

void SyncBackend::prefetch_factor_x(int bucket, float* x_all, const float* x_src, int B, int in,
                                    hipStream_t compute) {
  if (!collective() || !ops_->on_device()) return;
  if (bucket < 0 || bucket >= (int)factor_.size()) throw std::runtime_error("prefetch: bucket");
  issue(bucket, compute, [this, bucket, x_all, x_src, B, in, compute](hipStream_t cs) {
    ops_->factor_gather_x(x_all, x_src, B, in, cs);
    if (cs != compute) {  // a side-stream gather: mark its end for the bucket's job
      check_hip(hipEventRecord(gdone_[bucket], cs), "hipEventRecord(gathered)");
      gdone_set_[bucket] = 1;
    }
  });
}

void SyncBackend::begin_iteration(hipStream_t compute) {
  // an iteration that never reached wait_all (an exception, an aborted capture) must not leak
  // its stream choice into this one
  launched_side_ = launched_any_ = false;
  forks_.clear();
  held_epilogue = nullptr;
  for (auto& f : factor_) f.B = 0;
  std::fill(factor_skip_.begin(), factor_skip_.end(), 0);
  std::fill(gdone_set_.begin(), gdone_set_.end(), 0);
  epi_done_.clear();
  pending_.clear();
  deferred_.clear();
  if (fused_kind != 0 && !(skip_opt_begin && fused_kind == 1 && clip == ClipMode::NONE))
    ops_->opt_begin(compute);
  if (clip == ClipMode::LOCAL) ops_->clip_begin(1, compute);
}

static std::vector<hipGraphNode_t> capture_frontier(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  check_hip(hipStreamGetCaptureInfo_v2(s, &st, nullptr, nullptr, &deps, &n),
            "hipStreamGetCaptureInfo_v2");
  return std::vector<hipGraphNode_t>(deps, deps + n);
}

hipStream_t SyncBackend::pick_stream(int bucket, hipStream_t compute, bool* deferred) {
  *deferred = false;
  if (!ops_->on_device()) return nullptr;
  // Stream choice (measured on MI355X, profiles/side_stream_eager.md): in EAGER execution a
  // side stream costs 1.5-3x step time -- a hipStreamWaitEvent left pending on one hardware
  // queue while the host runs ahead slows every launch on the other queue. Inside a hipGraph the
  // same dependency is a graph edge and the collectives overlap backward. So: side stream while
  // capturing, the compute stream itself otherwise.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  check_hip(hipStreamIsCapturing(compute, &cap), "hipStreamIsCapturing");
  const bool capturing = cap == hipStreamCaptureStatusActive;
  bool side = capturing;
  if (!side && launched_side_) side = true;  // never switch streams within one iteration
  hipStream_t cs = side ? ops_->comm_stream() : compute;
  if (side) {
    launched_side_ = true;
    check_hip(hipEventRecord(ready_[bucket], compute), "hipEventRecord");
    // Captured fork: when the collective is captured before the compute chain's next node,
    // HIP's replay puts the chain on a different stream at every fork and, after a few buckets,
    // on the collectives' hardware queue -- backward serialised behind an all-reduce (measured:
    // profiles/graph_fork_order_r3.md; consistent with the first child edge of a node inheriting
    // its stream). So the side branch is deferred until the compute chain has its next node
    // (issue / flush_forks). The round-3 form captured an empty marker kernel first instead
    // (15 us per fork on the replay, profiles/r7/mlp_rehearsal_kernels_r7a.md; A/B against the
    // deferred fork: profiles/r8/fork_form_ab_r8a.md).
    if (capturing) {
      if (forks_.empty()) fork_deps_ = capture_frontier(compute);
      *deferred = true;
      return cs;
    }
    enter_side(bucket, cs);
    return cs;
  }
  if (!launched_any_ && timing_) check_hip(hipEventRecord(t0_, cs), "hipEventRecord");
  launched_any_ = true;
  return cs;
}

void SyncBackend::enter_side(int bucket, hipStream_t cs) {
  check_hip(hipStreamWaitEvent(cs, ready_[bucket], 0), "hipStreamWaitEvent");
  if (!launched_any_ && timing_) check_hip(hipEventRecord(t0_, cs), "hipEventRecord");
  launched_any_ = true;
}

void SyncBackend::issue(int bucket, hipStream_t compute, std::function<void(hipStream_t)> fn) {
  bool deferred = false;
  hipStream_t cs = pick_stream(bucket, compute, &deferred);
  if (deferred) {
    launched_any_ = true;
    forks_.push_back({bucket, std::move(fn)});
    return;
  }
  fn(cs);
}

void SyncBackend::flush_forks(hipStream_t compute, bool force) {
  if (forks_.empty()) return;
  // the compute stream captured a node since the first deferred fork: its chain owns the
  // producer's first child edge now, so the side branches can be captured
  if (!force && capture_frontier(compute) == fork_deps_) return;
  auto forks = std::move(forks_);
  forks_.clear();
  hipStream_t cs = ops_->comm_stream();
  for (auto& f : forks) {
    enter_side(f.bucket, cs);
    f.fn(cs);
  }
}

static bool is_sharded(const SyncBackend& b, int W) {
  return b.fused_kind != 0 && b.shard && W > 1 && !b.compressed;
}

void SyncBackend::reduce_bucket(int64_t begin, int64_t end, hipStream_t cs) {
  const int64_t n = end - begin;
  if (n <= 0) return;
  if (is_sharded(*this, ops_->world())) {
    // Sharded update (ZeRO-1 inside DDP): reduce-scatter the averaged gradient so this rank owns
    // 1/W of the bucket, update only that shard, all-gather the updated parameters. Same bytes
    // on the wire as the all-reduce, 1/W of the optimizer's HBM traffic; the parameters end up
    // identical on every rank, exactly as after all-reduce + replicated update.
    const Range own = owned_shard(begin, end);
    const int64_t cnt = own.second - own.first;
    const int64_t body = cnt * ops_->world();
    if (cnt > 0) ops_->reduce_scatter_avg(begin, cnt, cs);
    if (n > body) ops_->all_reduce_avg(begin + body, n - body, cs);
  } else {
    ops_->all_reduce_avg(begin, n, cs);
  }
}

Ranges SyncBackend::minus_epilogue(const Ranges& in) const {
  Ranges out;
  for (const auto& d : in) {
    int64_t cur = d.first;
    for (const auto& r : epi_done_) {  // sorted, disjoint
      if (r.second <= cur || r.first >= d.second) continue;
      if (r.first > cur) out.push_back({cur, r.first});
      cur = std::max(cur, r.second);
    }
    if (cur < d.second) out.push_back({cur, d.second});
  }
  return out;
}

Ranges SyncBackend::update_ranges(int64_t begin, int64_t end) const {
  if (!is_sharded(*this, ops_->world())) return minus_epilogue({{begin, end}});
  const Range own = owned_shard(begin, end);
  const int64_t body = (own.second - own.first) * ops_->world();
  Ranges r;
  if (own.second > own.first) r.push_back(own);
  if (begin + body < end) r.push_back({begin + body, end});
  return minus_epilogue(r);
}

void SyncBackend::finish_bucket(int64_t begin, int64_t end, hipStream_t cs) {
  if (fused_kind == 0 || end <= begin) return;
  ops_->opt_update(update_ranges(begin, end), cs);
  if (is_sharded(*this, ops_->world())) {
    const Range own = owned_shard(begin, end);
    const int64_t cnt = own.second - own.first;
    if (cnt > 0) ops_->all_gather_params(begin, cnt, cs);
  }
}

void SyncBackend::launch(int bucket, int64_t begin, int64_t end, hipStream_t compute) {
  if (end <= begin) return;
  flush_forks(compute, false);
  if (clip == ClipMode::LOCAL) {
    // the local norm needs the whole local gradient: nothing goes on the wire before backward ends
    pending_.push_back({begin, end});
    launched_any_ = true;
    return;
  }
  if (!collective()) {
    // one rank: the average over ranks is the local gradient -- no collective, no stream hop;
    // the bucket updates the GEMM epilogues did not do are applied by one launch at the end
    if (fused_kind != 0) {
      deferred_.push_back({begin, end});
      launched_any_ = true;
    }
    return;
  }
  if (bucket < (int)factor_skip_.size() && factor_skip_[bucket]) {
    factor_skip_[bucket] = 0;  // a factored bias: its weight's job averages and updates it
    return;
  }
  if (bucket < (int)factor_.size() && factor_[bucket].B > 0) {
    const FactorJob j = factor_[bucket];
    factor_[bucket].B = 0;
    // replicated jobs own the whole weight; sharded ones this rank's 1/W of its rows; split
    // ones this rank's 1/W of the rows past the replicated ones
    const Range own = factor_own(begin, end, j);
    const int64_t cnt = own.second - own.first;
    const int64_t shared = end - begin - (j.replicate ? 0 : (int64_t)j.rep_rows * j.in);
    if (fused_kind == 0 || clip != ClipMode::NONE || compressed ||
        (!j.replicate && (j.rep_rows < 0 || j.rep_rows >= j.out ||
                          cnt * ops_->world() != shared || cnt % j.in != 0)) ||
        (int64_t)j.out * j.in != end - begin)
      throw std::runtime_error("factored bucket: needs the fused optimizer, no clipping / "
                               "compression, and one whole-row-sharded weight per bucket");
    const int64_t own0 = own.first;
    issue(bucket, compute, [this, bucket, begin, own0, cnt, j, compute](hipStream_t cs) {
      FactorJob jj = j;
      // runs after the bucket's gather forks (forks run in issue order): both factors gathered
      // on the side stream -> the job waits for exactly those gathers
      if (j.g_ready && j.x_ready && cs != compute && gdone_set_[bucket]) jj.gathered = gdone_[bucket];
      gdone_set_[bucket] = 0;
      ops_->factor_sync(begin, own0, cnt, jj, cs, compute);
    });
    return;
  }
  if (clip == ClipMode::GLOBAL && fused_kind != 0)
    pending_.push_back({begin, end});  // the update needs the norm of every bucket
  const bool finish = fused_kind != 0 && clip != ClipMode::GLOBAL;
  issue(bucket, compute, [this, begin, end, finish](hipStream_t cs) {
    reduce_bucket(begin, end, cs);
    if (finish) finish_bucket(begin, end, cs);
  });
}

void SyncBackend::run_clip_local(hipStream_t s) {
  Ranges all;
  for (const auto& p : pending_) all.push_back({p.begin, p.end});
  ops_->grad_sumsq(1, all, s);  // this rank's own gradient: no collective
  ops_->clip_coef(1, s);
  ops_->scale_grads(1, all, s);
  const auto buckets = pending_;
  pending_.clear();
  for (const auto& p : buckets) {
    if (collective()) {
      reduce_bucket(p.begin, p.end, s);
      finish_bucket(p.begin, p.end, s);
    } else if (fused_kind != 0) {
      deferred_.push_back({p.begin, p.end});
    }
  }
}

void SyncBackend::run_clip_global(hipStream_t s) {
  // norm of the averaged gradient: with sharding each rank holds its shards (+ the replicated
  // tails, counted once by rank 0) and one 1-element all-reduce sums the parts; otherwise every
  // rank holds the whole averaged gradient and computes the same norm locally (deterministic
  // reduction: bit-identical on every rank)
  const bool sh = is_sharded(*this, ops_->world());
  Ranges norm_r;
  for (const auto& p : pending_) {
    if (!sh) {
      norm_r.push_back({p.begin, p.end});
      continue;
    }
    const Range own = owned_shard(p.begin, p.end);
    const int64_t body = (own.second - own.first) * ops_->world();
    if (own.second > own.first) norm_r.push_back(own);
    if (ops_->rank() == 0 && p.begin + body < p.end) norm_r.push_back({p.begin + body, p.end});
  }
  ops_->grad_sumsq(0, norm_r, s);
  if (sh) ops_->sumsq_all_reduce(0, s);
  ops_->clip_coef(0, s);  // the update kernels multiply their gradient by it
  const auto buckets = pending_;
  pending_.clear();
  for (const auto& p : buckets) finish_bucket(p.begin, p.end, s);
}

void SyncBackend::wait_all(hipStream_t compute) {
  run_held_epilogue(compute);
  flush_forks(compute, true);  // end of backward: nothing left for the compute chain to own
  // 1. join the comm stream: the compute stream waits for every bucket launched on it
  if (launched_side_) {
    launched_side_ = false;
    hipStream_t cs = ops_->comm_stream();
    if (timing_) {
      check_hip(hipEventRecord(t1_, cs), "hipEventRecord");
      timed_pending_ = true;
    }
    check_hip(hipEventRecord(done_, cs), "hipEventRecord");
    check_hip(hipStreamWaitEvent(compute, done_, 0), "hipStreamWaitEvent");
  }
  launched_any_ = false;
  // 2. work that needed the whole backward, on the compute stream
  if (clip == ClipMode::LOCAL && !pending_.empty()) run_clip_local(compute);
  if (clip == ClipMode::GLOBAL && fused_kind != 0) {
    if (!deferred_.empty()) {  // world size 1: the deferred buckets ARE the gradient
      for (const auto& d : deferred_) pending_.push_back({d.first, d.second});
      deferred_.clear();
    }
    if (!pending_.empty()) run_clip_global(compute);
  }
  // 3. world size 1: the bucket updates not done by GEMM epilogues, merged, in few launches
  if (!deferred_.empty()) {
    std::sort(deferred_.begin(), deferred_.end());
    Ranges merged;
    for (const auto& t : minus_epilogue(deferred_)) {
      if (!merged.empty() && merged.back().second == t.first) merged.back().second = t.second;
      else merged.push_back(t);
    }
    deferred_.clear();
    ops_->opt_update(merged, compute);
  }
  if (collective()) ops_->watch(compute, "DDP gradient synchronisation");
}

void SyncBackend::zero(int64_t begin, int64_t end, hipStream_t compute) {
  ops_->zero_grads(begin, end - begin, compute);
}

double SyncBackend::last_comm_ms() {
  if (!timing_ || !timed_pending_) return -1.0;
  if (hipEventQuery(t1_) != hipSuccess) return -1.0;  // not finished yet: never block here
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, t0_, t1_) != hipSuccess) return -1.0;
  return ms;
}

// ------------------------------------------------------------------------------------------------
// Reducer
// ------------------------------------------------------------------------------------------------
std::vector<int64_t> Reducer::compute_bucket_bounds(const std::vector<int64_t>& offsets,
                                                    const std::vector<int64_t>& numels,
                                                    int64_t arena_numel, int elem_size,
                                                    int64_t first_cap_bytes, int64_t cap_bytes,
                                                    int64_t split_bytes) {
  std::vector<int64_t> b{0};
  int64_t cur_bytes = 0;
  const int64_t split = split_bytes > 0 ? std::max<int64_t>(split_bytes / elem_size, 1) : 0;
  for (size_t i = 0; i < offsets.size(); ++i) {
    const int64_t cap = (b.size() == 1 ? first_cap_bytes : cap_bytes);
    const int64_t bytes = numels[i] * elem_size;
    // A partial bucket smaller than the first-bucket cap in front of a parameter that alone
    // overflows the cap rides along with it instead of going out as its own collective: such a
    // tiny collective costs a full RCCL latency (tens of us on xGMI) for no overlap gained --
    // the big parameter's gradient lands right after it (toy MLP: fc3 + fc2.bias join fc2.weight).
    const bool merge_small = bytes > cap && cur_bytes > 0 && cur_bytes < first_cap_bytes;
    if (cur_bytes > 0 && cur_bytes + bytes > cap && !merge_small) {
      b.push_back(offsets[i]);
      cur_bytes = 0;
    }
    if (split > 0 && numels[i] > split) {
      // a large parameter gets its own buckets, cut every `split` elements
      if (!merge_small && b.back() != offsets[i]) b.push_back(offsets[i]);
      for (int64_t s = split; s < numels[i]; s += split) b.push_back(offsets[i] + s);
      const int64_t tail = offsets[i] + numels[i];
      if (i + 1 < offsets.size()) b.push_back(tail);
      cur_bytes = 0;
      continue;
    }
    cur_bytes += bytes;
  }
  if (b.back() != arena_numel) b.push_back(arena_numel);
  // drop empty ranges (can appear with zero-sized params or padding)
  std::vector<int64_t> out{b[0]};
  for (size_t i = 1; i < b.size(); ++i)
    if (b[i] > out.back()) out.push_back(b[i]);
  if (out.size() == 1) out.push_back(std::max<int64_t>(arena_numel, 0));
  return out;
}

Reducer::Reducer(std::vector<int64_t> offsets, std::vector<int64_t> numels,
                 std::vector<int64_t> bucket_bounds, std::shared_ptr<ReducerBackend> backend)
    : offsets_(std::move(offsets)),
      numels_(std::move(numels)),
      bounds_(std::move(bucket_bounds)),
      backend_(std::move(backend)) {
  if (offsets_.size() != numels_.size()) throw std::runtime_error("offsets/numels mismatch");
  if (bounds_.size() < 2) throw std::runtime_error("need at least one bucket");
  const int nb = num_buckets();
  param_buckets_.resize(offsets_.size());
  bucket_nparams_.assign(nb, 0);
  for (size_t p = 0; p < offsets_.size(); ++p) {
    const int64_t a = offsets_[p], e = offsets_[p] + numels_[p];
    if (numels_[p] == 0) continue;
    // first bucket whose end is > a
    int b = (int)(std::upper_bound(bounds_.begin(), bounds_.end(), a) - bounds_.begin()) - 1;
    for (; b < nb && bounds_[b] < e; ++b) {
      param_buckets_[p].push_back(b);
      bucket_nparams_[b]++;
    }
  }
  pending_ = bucket_nparams_;
  param_ready_.assign(offsets_.size(), 0);
  bucket_ready_.assign(nb, 0);
}

void Reducer::prepare_for_backward(hipStream_t compute) {
  backend_->begin_iteration(compute);
  pending_ = bucket_nparams_;
  std::fill(param_ready_.begin(), param_ready_.end(), 0);
  for (int b = 0; b < num_buckets(); ++b) bucket_ready_[b] = (bucket_nparams_[b] == 0);
  hol_seen_.assign(num_buckets(), 0);
  next_bucket_ = 0;
  expecting_ = true;
}

void Reducer::mark_ready(int p, hipStream_t compute) {
  if (!expecting_) return;
  if (p < 0 || p >= (int)offsets_.size()) throw std::runtime_error("bad parameter index");
  if (param_ready_[p])
    throw std::runtime_error(
        "Expected to mark a variable ready only once (parameter " + std::to_string(p) +
        " produced a gradient twice in one backward; reentrant backward or a parameter used in "
        "two autograd graphs is not supported)");
  param_ready_[p] = 1;
  if (iteration_ == 0) first_ready_order_.push_back(p);
  for (int b : param_buckets_[p])
    if (--pending_[b] == 0) bucket_ready_[b] = 1;
  launch_ready(compute);
}

void Reducer::launch_ready(hipStream_t compute) {
  const int nb = num_buckets();
  // head-of-line accounting: a complete bucket stuck behind an incomplete lower-index one
  if (next_bucket_ < nb && !bucket_ready_[next_bucket_])
    for (int b = next_bucket_ + 1; b < nb; ++b)
      if (bucket_ready_[b] && !hol_seen_[b]) {
        hol_seen_[b] = 1;
        ++hol_waits_;
      }
  while (next_bucket_ < nb && bucket_ready_[next_bucket_]) {
    backend_->launch(next_bucket_, bounds_[next_bucket_], bounds_[next_bucket_ + 1], compute);
    ++next_bucket_;
  }
}

std::vector<int> Reducer::unready_params() const {
  std::vector<int> out;
  for (size_t p = 0; p < param_ready_.size(); ++p)
    if (!param_ready_[p] && numels_[p] > 0) out.push_back((int)p);
  return out;
}

void Reducer::finalize(hipStream_t compute, bool allow_unused) {
  if (!expecting_) return;
  const auto unready = unready_params();
  if (!unready.empty()) {
    if (!allow_unused) {
      std::string idx;
      for (size_t i = 0; i < unready.size() && i < 16; ++i)
        idx += (i ? ", " : "") + std::to_string(unready[i]);
      throw std::runtime_error(
          "Expected to have finished reduction in the prior iteration before starting a new "
          "one: parameters [" + idx + "] received no gradient. Pass find_unused_parameters=True "
          "if some parameters do not take part in the loss.");
    }
    for (int p : unready) {
      // an unused parameter contributes a zero gradient (the slot may hold last step's values)
      backend_->zero(offsets_[p], offsets_[p] + numels_[p], compute);
      param_ready_[p] = 1;
      if (iteration_ == 0) first_ready_order_.push_back(p);
      for (int b : param_buckets_[p])
        if (--pending_[b] == 0) bucket_ready_[b] = 1;
    }
    launch_ready(compute);
  }
  if (next_bucket_ != num_buckets())
    throw std::runtime_error("reducer: not every bucket became ready");
  backend_->wait_all(compute);
  expecting_ = false;
  ++iteration_;
}

}  // namespace tdp
