// Gradient reducer: DDP's C++ Reducer re-designed around a flat gradient arena.
//
// torch DDP (TORCH/nn/parallel/distributed.py:1163-1275) copies every
// gradient into a bucket, divides by world size, all-reduces, and copies back (K24: 2 x 217 MiB of
// copies per AlexNet step), starts from one all-parameter bucket and rebuilds buckets after
// iteration 0. Here:
//   * every parameter's .grad IS a view of one flat arena laid out in backward order, so a bucket
//     is just a contiguous [begin, end) element range: no copy-in, no copy-out;
//   * a bucket boundary may fall inside a large parameter (fc1's 144 MiB weight can be split);
//   * averaging is ncclAvg inside the all-reduce (no div_ pass);
//   * buckets launch strictly in index order as soon as every parameter overlapping them is
//     ready (identical collective order on every rank). While a hipGraph is being captured they
//     go to the communicator's high-priority stream after an event recorded on the compute
//     stream (overlapping backward) and finalize() makes the compute stream wait on the last
//     bucket; in eager execution they are issued on the compute stream itself, because a
//     cross-queue wait left pending while the host runs ahead was measured to slow every kernel
//     on MI355X (see RcclBackend::launch). Either way no host sync is needed.
// The backend is abstract so that the same bucketing/readiness logic runs over RCCL on MI355X
// and over torch.distributed (gloo) in the CPU tests.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "comm.h"
#include "kernels.h"

namespace tdp {

struct ReducerBackend {
  virtual ~ReducerBackend() = default;
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

// Optimizer update fused into the reduction (torch's DDP._register_fused_optim idea): as soon as a
// bucket's averaged gradient exists, its slice of the parameter arena is updated on the comm
// stream, overlapping the update of early buckets with the backward compute / all-reduce of
// later ones. Parameters, gradients and optimizer state share the arena layout, so a bucket's
// update is the flat kernel on [begin, end) of every buffer.
struct FusedOptimizer {
  int kind = 0;  // 0 none, 1 SGD, 2 Adam
  float* p = nullptr;
  float* s0 = nullptr;  // momentum buffer / exp_avg
  float* s1 = nullptr;  // exp_avg_sq
  float* s2 = nullptr;  // max_exp_avg_sq
  SgdHyper sgd{};
  AdamHyper adam{};
  float adam_beta1 = 0.9f, adam_beta2 = 0.999f;
  int64_t adam_step = 0;       // incremented when the first bucket of an iteration updates
  std::vector<char> fresh;     // per bucket: SGD momentum not yet initialised
  bool shard = false;          // reduce-scatter / update 1/W / all-gather (world > 1)
};

class RcclBackend : public ReducerBackend {
 public:
  RcclBackend(std::shared_ptr<Communicator> comm, void* arena, int64_t numel, int elem_size,
              int num_buckets, Compression compression, bool timing, bool skip_single_rank);
  ~RcclBackend() override;
  void launch(int bucket, int64_t begin, int64_t end, hipStream_t compute) override;
  void wait_all(hipStream_t compute) override;
  void zero(int64_t begin, int64_t end, hipStream_t compute) override;
  double last_comm_ms() override;
  // called after a bucket's all-reduce is enqueued, with the comm stream (fused optimizer hook)
  std::function<void(int, int64_t, int64_t, hipStream_t)> post_bucket;
  FusedOptimizer fused;

  // Optimizer-in-GEMM-epilogue (world size 1 only: the local gradient IS the averaged one): the
  // weight-gradient GEMM of arena elements [off, off + n) applies the fused optimizer instead of
  // storing the gradient. Returns the epilogue arguments (pointers offset to `off`, this
  // iteration's hyper-parameters) and records the range so the bucket update skips it.
  OptEpilogue epilogue_opt(int64_t off, int64_t n);
  bool epilogue_allowed() const;
  void set_epilogue_fresh(bool v) { epi_fresh_ = v; }

 private:
  void apply_fused(int64_t off, int64_t cnt, bool first, hipStream_t cs);
  void apply_fused_range(int64_t off, int64_t cnt, bool first, hipStream_t cs);
  void flush_deferred(hipStream_t compute);
  std::vector<std::pair<int64_t, int64_t>> epi_done_;  // ranges updated by GEMM epilogues
  // world size 1: bucket updates deferred to the end of backward, applied by one launch
  std::vector<std::pair<int64_t, int64_t>> deferred_;
  bool deferred_first_ = false;
  bool epi_fresh_ = false;        // SGD momentum of epilogue-updated ranges not yet initialised
  bool bucket0_launched_ = false;  // this iteration's Adam step counter already advanced
  std::shared_ptr<Communicator> comm_;
  char* arena_;
  int64_t numel_;
  int elem_size_;
  Compression compression_;
  bool timing_, skip_single_rank_;
  std::vector<hipEvent_t> ready_;
  hipEvent_t done_ = nullptr, t0_ = nullptr, t1_ = nullptr;
  bool launched_any_ = false, timed_pending_ = false;
  // where bucket collectives run: auto = side stream only while capturing a hipGraph
  // hostjoin: side stream, but the end-of-backward join is a host wait on the comm stream's
  // event instead of a device-side hipStreamWaitEvent on the compute stream; nojoin: no join
  // at all (measurement only: the next forward may race the last buckets)
  enum {
    kStreamAuto = 0, kStreamSide = 1, kStreamCompute = 2, kStreamHostSync = 3,
    kStreamHostJoin = 4, kStreamNoJoin = 5
  };
  int stream_mode_ = kStreamAuto;
  bool launched_side_ = false;
  uint16_t* wire_ = nullptr;  // bf16 staging buffer for compressed buckets
};

class Reducer {
 public:
  Reducer(std::vector<int64_t> offsets, std::vector<int64_t> numels,
          std::vector<int64_t> bucket_bounds, std::shared_ptr<ReducerBackend> backend);

  // Boundaries (element offsets, first 0, last = arena numel) for parameters laid out at
  // `offsets` (ascending). Small parameters are grouped up to cap_bytes (first_cap_bytes for the
  // first bucket); a parameter larger than split_bytes (> 0) is cut into split_bytes pieces.
  static std::vector<int64_t> compute_bucket_bounds(const std::vector<int64_t>& offsets,
                                                    const std::vector<int64_t>& numels,
                                                    int64_t arena_numel, int elem_size,
                                                    int64_t first_cap_bytes, int64_t cap_bytes,
                                                    int64_t split_bytes);

  void prepare_for_backward();
  void mark_ready(int param, hipStream_t compute);
  // launch whatever is left, zero never-ready params when allowed, make `compute` wait
  void finalize(hipStream_t compute, bool allow_unused);

  bool expecting() const { return expecting_; }
  int64_t iteration() const { return iteration_; }
  std::vector<int64_t> bucket_bounds() const { return bounds_; }
  std::vector<int> ready_order() const { return first_ready_order_; }
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
};

}  // namespace tdp
