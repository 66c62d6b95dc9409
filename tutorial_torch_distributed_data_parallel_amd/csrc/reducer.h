// Gradient reducer: DDP's C++ Reducer re-designed around a flat gradient arena.
//
// torch DDP (TORCH/nn/parallel/distributed.py:1163-1275) copies every
// gradient into a bucket, divides by world size, all-reduces, and copies back (K24: 2 x 217 MiB of
// copies per AlexNet step), starts from one all-parameter bucket and rebuilds buckets after
// iteration 0. Here:
//   * every parameter's .grad IS a view of one flat arena, so a bucket is a contiguous
//     [begin, end) element range: no copy-in, no copy-out; the arena is laid out in backward
//     order (re-laid out once from the observed ready order, parallel/ddp.py _rebuild_buckets);
//   * a bucket boundary may fall inside a large parameter (fc1's 144 MiB weight is split);
//   * averaging is ncclAvg inside the collective (no div_ pass);
//   * buckets launch strictly in index order as soon as every parameter overlapping them is
//     ready (identical collective order on every rank). While a hipGraph is being captured they
//     go to the communicator's high-priority stream after an event recorded on the compute
//     stream (overlapping backward) and finalize() makes the compute stream wait on the last
//     bucket; in eager execution they are issued on the compute stream itself, because a
//     cross-queue wait left pending while the host runs ahead was measured to slow every kernel
//     on MI355X (profiles/side_stream_eager.md). Either way no host sync is needed.
//
// The bucket / shard / clip ALGORITHM (SyncBackend) is separated from its side effects (SyncOps):
// RcclOps runs it on MI355X (RCCL collectives over xGMI + gfx950 optimizer kernels); PyOps
// (bindings.cpp) runs the very same C++ logic over torch.distributed/gloo with torch math on CPU
// arenas, which is how the multi-rank paths (sharded update, tails, clipping) are tested without
// a multi-GPU node.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "comm.h"
#include "kernels.h"

namespace tdp {

using Range = std::pair<int64_t, int64_t>;  // [first, second) arena elements
using Ranges = std::vector<Range>;

struct ReducerBackend {
  virtual ~ReducerBackend() = default;
  // start of an iteration's backward (forward of a step that will sync gradients)
  virtual void begin_iteration(hipStream_t compute) { (void)compute; }
  // average arena elements [begin, end) across ranks, ordered after work already on `compute`
  virtual void launch(int bucket, int64_t begin, int64_t end, hipStream_t compute) = 0;
  // make `compute` wait for every bucket launched so far in this iteration
  virtual void wait_all(hipStream_t compute) = 0;
  // zero arena elements [begin, end) (gradients of parameters unused in this iteration)
  virtual void zero(int64_t begin, int64_t end, hipStream_t compute) = 0;
  // device-side comm time of the last finished iteration in ms (-1 when unknown)
  virtual double last_comm_ms() { return -1.0; }
};

// Gradient compression for the wire: NONE sends the arena dtype (fp32), BF16 casts each bucket to
// bf16 on the comm stream, all-reduces that and casts back (torch's bf16_compress_hook).
enum class Compression : int { NONE = 0, BF16 = 1 };

// Gradient clipping done inside the reduction.
//   GLOBAL: torch.nn.utils.clip_grad_norm_ of the AVERAGED gradient, before the fused optimizer
//           update (the norm of the whole model needs every bucket: updates wait for the last one).
//   LOCAL:  the README pitfall "clip gradients before they are aggregated"
//           (REF/README.md:92-95): every rank clips its OWN gradient to max_norm before any byte
//           goes on the wire, so one rank's exploding gradient cannot dominate the average.
enum class ClipMode : int { NONE = 0, GLOBAL = 1, LOCAL = 2 };

// Factored synchronisation of one Linear weight W[out][in] (its own bucket, sharded by rows):
// the averaged gradient (1/W) sum_r g_r^T x_r has rank <= W*B, so instead of reduce-scattering the
// out*in gradient every rank all-gathers the factors -- g_r [B][out] (already scaled by 1/W) and
// x_r [B][in], which the compute stream wrote into this rank's slots of g_all / x_all -- and
// computes ITS row shard of the averaged gradient with one GEMM of depth W*B, whose epilogue
// applies the fused optimizer; the updated rows are then all-gathered as in the sharded update.
struct FactorJob {
  float* g_all = nullptr;  // [W*B][out], rank r's rows at r*B
  float* x_all = nullptr;  // [W*B][in]
  int B = 0, out = 0, in = 0;
  // arena offset of the layer's bias (-1: none): its averaged gradient is the column sum of
  // g_all, which every rank holds after the all-gather, so every rank updates the whole bias
  // itself -- the bias bucket issues no collective at all
  int64_t bias_off = -1;
  // replicated: every rank computes ALL rows of the averaged gradient (GEMM depth W*B over the
  // whole weight) and updates them itself -- identical inputs and kernel, identical parameters --
  // so no parameter all-gather follows. Chosen when W*B is small enough that the extra GEMM rows
  // cost less than the out*in*(W-1)/W all-gather on xGMI (parallel/ddp.py factor_replicate).
  bool replicate = false;
  // split job (0 < rep_rows < out, replicate false): rows [0, rep_rows) replicated -- every rank
  // computes and updates them, overlapped with the all-gather of the rest -- and rows
  // [rep_rows, out) sharded over the ranks as in a sharded job (parallel/commmodel.py
  // "factored-split": at W = 8 it hides most of the parameter all-gather of the last bucket)
  int rep_rows = 0;
  // x_all was already all-gathered at forward time (SyncBackend::prefetch_factor_x): the job
  // gathers only g
  bool x_ready = false;
  // g_all was already all-gathered at the start of the layer's backward, before its input-
  // gradient GEMM (DDP.factor_prefetch_g -> SyncBackend::prefetch_factor_x with g): the gather
  // overlaps that GEMM and the job gathers nothing
  bool g_ready = false;
  // out-of-place g gather: this rank's g [B][out] straight from the layer's gradient buffer
  // (no staging copy into slot r)
  const float* g_src = nullptr;
  // factor applied to the gathered g by the update (1/W on the device path, where every rank's
  // slot holds unscaled g whether it was read in place or staged; 1 on the CPU twin)
  float g_scale = 1.f;
  // both factors were gathered by earlier side-stream forks and this event was recorded right
  // after the last of them: the job's compute-stream arithmetic waits on it alone, not on
  // everything queued on the side stream since (e.g. the previous job's parameter all-gather,
  // when fc1's g gather was issued from fc2's backward: DDP.factor_prefetch_g)
  hipEvent_t gathered = nullptr;
};

// Side effects of the sync algorithm. Offsets are arena elements; streams are ignored off-device.
struct SyncOps {
  virtual ~SyncOps() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual bool on_device() const = 0;
  virtual hipStream_t comm_stream() { return nullptr; }
  // gradient arena collectives, in place, averaged over ranks
  virtual void all_reduce_avg(int64_t off, int64_t n, hipStream_t s) = 0;
  // [off, off + W*cnt): rank r ends up with the average of its slice [off + r*cnt, +cnt)
  virtual void reduce_scatter_avg(int64_t off, int64_t cnt, hipStream_t s) = 0;
  // parameter arena: every rank's slice [off + r*cnt, +cnt) -> everyone, in place
  virtual void all_gather_params(int64_t off, int64_t cnt, hipStream_t s) = 0;
  virtual void zero_grads(int64_t off, int64_t n, hipStream_t s) = 0;
  // fused optimizer (ranges of p / grad / state, one launch per call)
  virtual void opt_begin(hipStream_t s) = 0;
  virtual void opt_update(const Ranges& r, hipStream_t s) = 0;
  // clipping: `block` 0 = the optimizer's hyper block (GLOBAL), 1 = the DDP clip block (LOCAL)
  virtual void clip_begin(int block, hipStream_t s) = 0;
  virtual void grad_sumsq(int block, const Ranges& r, hipStream_t s) = 0;  // += ||g[r]||^2
  virtual void sumsq_all_reduce(int block, hipStream_t s) = 0;             // sum over ranks
  virtual void clip_coef(int block, hipStream_t s) = 0;                    // from sumsq
  virtual void scale_grads(int block, const Ranges& r, hipStream_t s) = 0; // g[r] *= coef
  // collective watchdog: the work enqueued on `s` so far must finish within the timeout
  virtual void watch(hipStream_t s, const char* what) { (void)s; (void)what; }
  // factored weight bucket [begin, begin + W*cnt): this rank owns [own, own + cnt) (FactorJob)
  // `s` carries the collectives; `compute` (when a different stream) runs the job's GEMM and
  // updates, so the comm stream stays free for the next job's gathers (see RcclOps)
  virtual void factor_sync(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j,
                           hipStream_t s, hipStream_t compute);
  // forward-time all-gather of a factored weight's x_all ([W*B][in]): from this rank's rows at
  // slot r (x_src null) or straight from the layer's input x_src [B][in] (out of place)
  virtual void factor_gather_x(float* x_all, const float* x_src, int B, int in, hipStream_t s);
  // size the workspaces factor_sync(begin, own, cnt, j) will need (eagerly, before a capture)
  virtual void factor_reserve(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j);
};

// Device implementation: RCCL communicator + gfx950 kernels over the device arenas.
struct FusedOptimizer {
  int kind = 0;  // 0 none, 1 SGD, 2 Adam
  float* p = nullptr;
  float* s0 = nullptr;  // momentum buffer / exp_avg
  float* s1 = nullptr;  // exp_avg_sq
  float* s2 = nullptr;  // max_exp_avg_sq
  SgdHyper sgd{};       // structural flags; per-step scalars come from `hyper`
  AdamHyper adam{};
  float* hyper = nullptr;  // device hyper block of the optimizer (kernels.h HyperSlot)
};

class RcclOps : public SyncOps {
 public:
  RcclOps(std::shared_ptr<Communicator> comm, float* grad, float* param, int64_t numel,
          Compression compression);
  ~RcclOps() override;
  int rank() const override { return comm_->rank(); }
  int world() const override { return comm_->world(); }
  bool on_device() const override { return true; }
  hipStream_t comm_stream() override { return comm_->comm_stream(); }
  void all_reduce_avg(int64_t off, int64_t n, hipStream_t s) override;
  void reduce_scatter_avg(int64_t off, int64_t cnt, hipStream_t s) override;
  void all_gather_params(int64_t off, int64_t cnt, hipStream_t s) override;
  void zero_grads(int64_t off, int64_t n, hipStream_t s) override;
  void opt_begin(hipStream_t s) override;
  void opt_update(const Ranges& r, hipStream_t s) override;
  void clip_begin(int block, hipStream_t s) override;
  void grad_sumsq(int block, const Ranges& r, hipStream_t s) override;
  void sumsq_all_reduce(int block, hipStream_t s) override;
  void clip_coef(int block, hipStream_t s) override;
  void scale_grads(int block, const Ranges& r, hipStream_t s) override;
  void watch(hipStream_t s, const char* what) override { comm_->watch(s, what); }
  void factor_sync(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j,
                   hipStream_t s, hipStream_t compute) override;
  void factor_gather_x(float* x_all, const float* x_src, int B, int in, hipStream_t s) override;
  // opt_update with the gradient multiplied by `scale` first (factored jobs over unscaled g)
  void opt_update_scaled(const Ranges& r, float scale, hipStream_t s);
  void factor_reserve(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j) override;

  FusedOptimizer fused;
  float* clip_block = nullptr;  // DDP-owned hyper block for LOCAL clipping
  Compression compression() const { return compression_; }
  // measurement only (bench.py compute-only rehearsal): collectives become no-ops
  bool skip_collectives = false;
  std::shared_ptr<Communicator> comm() const { return comm_; }

 private:
  struct FactorPlan;
  FactorPlan plan_factor(int64_t begin, int64_t own, int64_t cnt, const FactorJob& j) const;
  void grow_factor_ws(const FactorPlan& f, int out, hipStream_t s);
  float* block(int b) const { return b == 0 ? fused.hyper : clip_block; }
  std::shared_ptr<Communicator> comm_;
  float* grad_;
  float* param_;
  int64_t numel_;
  Compression compression_;
  uint16_t* wire_ = nullptr;  // bf16 staging buffer for compressed buckets
  float* factor_ws_ = nullptr;  // split-K workspace of factored shard GEMMs (grown eagerly)
  int64_t factor_ws_floats_ = 0;
  float* factor_part_ = nullptr;  // column-sum partials of the factored biases
  int64_t factor_part_floats_ = 0;
  hipEvent_t fac_ev_[2] = {nullptr, nullptr};  // comm <-> compute edges of a factored job
};

// The bucket algorithm (one instance per DDP model).
class SyncBackend : public ReducerBackend {
 public:
  SyncBackend(std::shared_ptr<SyncOps> ops, int64_t numel, int num_buckets, bool timing,
              bool skip_single_rank);
  ~SyncBackend() override;
  void begin_iteration(hipStream_t compute) override;
  void launch(int bucket, int64_t begin, int64_t end, hipStream_t compute) override;
  void wait_all(hipStream_t compute) override;
  void zero(int64_t begin, int64_t end, hipStream_t compute) override;
  double last_comm_ms() override;

  // configuration (set by parallel/ddp.py)
  int fused_kind = 0;     // 0 none, 1 SGD, 2 Adam (ops apply it)
  bool shard = false;     // world > 1: reduce-scatter / update own 1/W / all-gather
  ClipMode clip = ClipMode::NONE;
  bool compressed = false;  // wire compression active (sharding needs the plain fp32 path)
  // SGD in steady state (first-step flags consumed, no clipping): the per-iteration hyper-block
  // advance changes nothing the update reads, so its launch is skipped (set by parallel/ddp.py)
  bool skip_opt_begin = false;

  // Optimizer-in-GEMM-epilogue (world size 1 only: the local gradient IS the averaged one): the
  // weight-gradient GEMM of arena elements [off, off + n) applies the fused optimizer instead of
  // storing the gradient; the range is recorded so the bucket update skips it.
  bool epilogue_allowed() const;
  void note_epilogue(int64_t off, int64_t n);
  // A weight-gradient + optimizer GEMM held back so the next layer's can share its launch
  // (bindings.cpp gemm_f32_opt hold=True, gemm_f32_fast_run_pair): run by that call, or alone
  // at the start of wait_all (end of backward); dropped with the iteration's other state by
  // begin_iteration. The held GEMM's tensors live in the closure until it runs.
  std::function<void(hipStream_t)> held_epilogue;
  void run_held_epilogue(hipStream_t s) {
    if (!held_epilogue) return;
    auto f = std::move(held_epilogue);
    held_epilogue = nullptr;
    f(s);
  }

  // the shard of bucket [begin, end) this rank owns under the sharded update (tail excluded)
  Range owned_shard(int64_t begin, int64_t end) const;
  // Arm bucket `bucket` (exactly one Linear weight) for factored synchronisation in this
  // iteration: its launch runs ops.factor_sync instead of reduce-scatter / update / all-gather.
  // `bias_bucket` (>= 0): the bucket holding exactly the layer's bias, updated by the job.
  void arm_factor(int bucket, const FactorJob& j, int bias_bucket);
  // Forward-time gather of a factored weight's input factor: x exists as
  // soon as the layer's forward runs, so its all-gather is issued then -- on the comm stream,
  // as a deferred fork while capturing -- and overlaps the rest of forward and backward; the
  // bucket's job at backward time then gathers only g (FactorJob::x_ready).
  void prefetch_factor_x(int bucket, float* x_all, const float* x_src, int B, int in,
                         hipStream_t compute);
  // eagerly size the workspaces of the factored job of bucket [begin, end) (DDP.settle, before
  // a capture: the first factored step may have run under another bucket layout)
  void reserve_factor(int64_t begin, int64_t end, const FactorJob& j);
  // the rows of bucket [begin, end) this rank computes under job j (elements)
  Range factor_own(int64_t begin, int64_t end, const FactorJob& j) const;
  // capture the deferred side branches once the compute stream has a node behind them (a
  // caller that just launched compute work: ops/linear.py after a factored layer's forward GEMM)
  void flush(hipStream_t compute) { flush_forks(compute, false); }
  std::shared_ptr<SyncOps> ops() const { return ops_; }
  bool collective() const { return !(skip_single_rank_ && ops_->world() == 1); }

 private:
  struct Pending {
    int64_t begin, end;
  };
  void reduce_bucket(int64_t begin, int64_t end, hipStream_t cs);   // collectives only
  void finish_bucket(int64_t begin, int64_t end, hipStream_t cs);   // update + all-gather
  Ranges update_ranges(int64_t begin, int64_t end) const;           // own ranges minus epilogue
  Ranges minus_epilogue(const Ranges& in) const;
  // Run `fn` (a bucket's collectives + update) on the stream pick_stream chooses. While a graph
  // is captured with the comm stream as a side branch, the fork is DEFERRED: the ready event is
  // recorded now, but the side-stream wait and `fn` are captured only once the compute stream
  // has captured its next node (flush_forks), so the compute chain is the producer's first child
  // -- what keeps the two branches on separate hardware queues at replay
  // (profiles/graph_fork_order_r3.md: "compute_first") without an empty marker kernel.
  void issue(int bucket, hipStream_t compute, std::function<void(hipStream_t)> fn);
  void flush_forks(hipStream_t compute, bool force);
  hipStream_t pick_stream(int bucket, hipStream_t compute, bool* deferred);
  void enter_side(int bucket, hipStream_t cs);
  void run_clip_local(hipStream_t cs);
  void run_clip_global(hipStream_t cs);

  std::shared_ptr<SyncOps> ops_;
  int64_t numel_;
  bool timing_, skip_single_rank_;
  Ranges epi_done_;              // ranges updated by GEMM epilogues this iteration (sorted)
  std::vector<Pending> pending_; // buckets reduced but not yet updated (clipping) / not reduced
  Ranges deferred_;              // world size 1: bucket updates deferred to the end of backward
  std::vector<FactorJob> factor_;  // per bucket, armed for this iteration when B > 0
  std::vector<char> factor_skip_;  // per bucket: a factored bias, handled by its weight's job
  struct Fork {
    int bucket;
    std::function<void(hipStream_t)> fn;
  };
  std::vector<Fork> forks_;               // deferred side-stream launches (capture only)
  std::vector<hipGraphNode_t> fork_deps_; // compute stream's capture frontier at the first one
  std::vector<hipEvent_t> ready_;
  std::vector<hipEvent_t> gdone_;  // per bucket: recorded after its last factor gather fork
  std::vector<char> gdone_set_;    // ... in this iteration, on the side stream
  hipEvent_t done_ = nullptr, t0_ = nullptr, t1_ = nullptr;
  bool launched_any_ = false, timed_pending_ = false, launched_side_ = false;
};

class Reducer {
 public:
  Reducer(std::vector<int64_t> offsets, std::vector<int64_t> numels,
          std::vector<int64_t> bucket_bounds, std::shared_ptr<ReducerBackend> backend);

  // Boundaries (element offsets, first 0, last = arena numel) for parameters laid out at
  // `offsets` (ascending). Small parameters are grouped up to cap_bytes (first_cap_bytes for the
  // first bucket); a parameter larger than split_bytes (> 0) is cut into split_bytes pieces; a
  // partial bucket under first_cap_bytes is merged into a following parameter that alone
  // overflows the cap.
  static std::vector<int64_t> compute_bucket_bounds(const std::vector<int64_t>& offsets,
                                                    const std::vector<int64_t>& numels,
                                                    int64_t arena_numel, int elem_size,
                                                    int64_t first_cap_bytes, int64_t cap_bytes,
                                                    int64_t split_bytes);

  void prepare_for_backward(hipStream_t compute);
  void mark_ready(int param, hipStream_t compute);
  // launch whatever is left, zero never-ready params when allowed, make `compute` wait
  void finalize(hipStream_t compute, bool allow_unused);

  bool expecting() const { return expecting_; }
  int64_t iteration() const { return iteration_; }
  std::vector<int64_t> bucket_bounds() const { return bounds_; }
  std::vector<int> ready_order() const { return first_ready_order_; }
  // buckets (summed over iterations) that were complete while a lower-indexed bucket was not:
  // each one waited only because buckets launch in index order
  int64_t head_of_line_waits() const { return hol_waits_; }
  std::vector<int> unready_params() const;
  int num_buckets() const { return (int)bounds_.size() - 1; }
  double last_comm_ms() { return backend_->last_comm_ms(); }

 private:
  void launch_ready(hipStream_t compute);

  std::vector<int64_t> offsets_, numels_, bounds_;
  std::vector<std::vector<int>> param_buckets_;
  std::vector<int> bucket_nparams_, pending_;
  std::vector<char> param_ready_, bucket_ready_;
  std::vector<int> first_ready_order_;
  std::shared_ptr<ReducerBackend> backend_;
  int next_bucket_ = 0;
  bool expecting_ = false;
  int64_t iteration_ = 0;
  int64_t hol_waits_ = 0;
  std::vector<char> hol_seen_;
};

}  // namespace tdp
