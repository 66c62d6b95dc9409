#include "reducer.h"

#include <algorithm>
#include <cstdlib>
#include <string>
#include <cmath>
#include <stdexcept>

#include "kernels.h"

namespace tdp {

// ------------------------------------------------------------------------------------------------
// RcclBackend
// ------------------------------------------------------------------------------------------------
RcclBackend::RcclBackend(std::shared_ptr<Communicator> comm, void* arena, int64_t numel,
                         int elem_size, int num_buckets, Compression compression, bool timing,
                         bool skip_single_rank)
    : comm_(std::move(comm)),
      arena_(static_cast<char*>(arena)),
      numel_(numel),
      elem_size_(elem_size),
      compression_(compression),
      timing_(timing),
      skip_single_rank_(skip_single_rank) {
  if (compression_ == Compression::BF16 && elem_size_ != 4)
    throw std::runtime_error("bf16 gradient compression needs an fp32 arena");
  ready_.resize(num_buckets);
  for (auto& e : ready_) check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
  check_hip(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "event");
  if (timing_) {
    check_hip(hipEventCreate(&t0_), "event");
    check_hip(hipEventCreate(&t1_), "event");
  }
  if (compression_ == Compression::BF16)
    check_hip(hipMalloc(&wire_, sizeof(uint16_t) * (size_t)numel_), "hipMalloc(wire)");
  const char* mode = std::getenv("TDP_COMM_STREAM");
  const std::string m = mode ? mode : "auto";
  stream_mode_ = m == "side" ? kStreamSide
                 : m == "compute" ? kStreamCompute
                 : m == "hostsync" ? kStreamHostSync
                 : m == "hostjoin" ? kStreamHostJoin
                 : m == "nojoin" ? kStreamNoJoin
                                   : kStreamAuto;
}

RcclBackend::~RcclBackend() {
  for (auto& e : ready_) (void)hipEventDestroy(e);
  if (done_) (void)hipEventDestroy(done_);
  if (t0_) (void)hipEventDestroy(t0_);
  if (t1_) (void)hipEventDestroy(t1_);
  if (wire_) (void)hipFree(wire_);
}

static ncclDataType_t nccl_dtype(int elem_size) {
  switch (elem_size) {
    case 4: return ncclFloat32;
    case 2: return ncclBfloat16;
    case 8: return ncclFloat64;
    default: throw std::runtime_error("unsupported arena element size");
  }
}

void RcclBackend::launch(int bucket, int64_t begin, int64_t end, hipStream_t compute) {
  const bool collective = !(skip_single_rank_ && comm_->world() == 1);
  if (!collective) {
    // one rank: the average over ranks is the local gradient -- no collective, no stream hop.
    // With a fused optimizer the remaining (non-epilogue) updates of every bucket are applied
    // by one launch when backward ends (flush_deferred).
    if (fused.kind != 0 && end > begin) {
      if (fused.kind == 1 && !fused.fresh.empty()) {
        deferred_first_ = deferred_first_ || (bool)fused.fresh[bucket];
        fused.fresh[bucket] = 0;
      }
      if (fused.kind == 2 && bucket == 0 && !bucket0_launched_) {
        ++fused.adam_step;
        bucket0_launched_ = true;
      }
      deferred_.push_back({begin, end});
      launched_any_ = true;
    }
    if (post_bucket) post_bucket(bucket, begin, end, compute);
    return;
  }
  // Stream choice (measured on MI355X, profiles/bench/mode*.json): in EAGER execution a side
  // stream costs 1.5-3x step time -- a hipStreamWaitEvent barrier left pending on one hardware
  // queue while the host runs ahead slows every kernel dispatched on the other queue (ResNet-50:
  // 95 ms vs 65 ms). Inside a hipGraph the same dependency is free and the all-reduce overlaps
  // backward. So: side stream while capturing, the compute stream itself otherwise
  // (TDP_COMM_STREAM=side|compute|hostsync overrides for measurements).
  bool side = true;
  if (stream_mode_ == kStreamAuto) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    check_hip(hipStreamIsCapturing(compute, &cap), "hipStreamIsCapturing");
    side = cap == hipStreamCaptureStatusActive;
  } else {
    side = stream_mode_ != kStreamCompute;
  }
  if (!side && launched_side_) side = true;  // never switch streams within one iteration
  hipStream_t cs = side ? comm_->comm_stream() : compute;
  if (side) {
    launched_side_ = true;
    check_hip(hipEventRecord(ready_[bucket], compute), "hipEventRecord");
    if (stream_mode_ == kStreamHostSync)
      check_hip(hipEventSynchronize(ready_[bucket]), "hipEventSynchronize");
    else
      check_hip(hipStreamWaitEvent(cs, ready_[bucket], 0), "hipStreamWaitEvent");
  }
  if (!launched_any_ && timing_) check_hip(hipEventRecord(t0_, cs), "hipEventRecord");
  launched_any_ = true;
  const int64_t n = end - begin;
  const int W = comm_->world();
  bool first = false;
  if (n > 0 && fused.kind == 1 && !fused.fresh.empty()) {
    first = (bool)fused.fresh[bucket];
    fused.fresh[bucket] = 0;
  }
  if (n > 0 && fused.kind == 2 && bucket == 0 && !bucket0_launched_) {
    ++fused.adam_step;
    bucket0_launched_ = true;
  }
  float* g = reinterpret_cast<float*>(arena_) + begin;
  if (n > 0 && collective && fused.kind != 0 && fused.shard && W > 1 &&
      compression_ == Compression::NONE && elem_size_ == 4) {
    // Sharded update (ZeRO-1 inside DDP): reduce-scatter the averaged gradient so this rank owns
    // 1/W of the bucket, update only that shard, all-gather the updated parameters. Same bytes
    // on the wire as the all-reduce, 1/W of the optimizer's HBM traffic; the parameters end up
    // identical on every rank, exactly as after all-reduce + replicated update. The < W-element
    // tail that does not divide evenly is all-reduced and updated everywhere.
    const int r = comm_->rank();
    const int64_t cnt = n / W, body = cnt * W, tail = n - body;
    if (cnt > 0) {
      comm_->reduce_scatter(g, g + (int64_t)r * cnt, (size_t)cnt, ncclFloat32, ncclAvg, cs);
      apply_fused(begin + (int64_t)r * cnt, cnt, first, cs);
      comm_->all_gather(fused.p + begin + (int64_t)r * cnt, fused.p + begin, (size_t)cnt,
                        ncclFloat32, cs);
    }
    if (tail > 0) {
      comm_->all_reduce(g + body, g + body, (size_t)tail, ncclFloat32, ncclAvg, cs);
      apply_fused(begin + body, tail, first, cs);
    }
  } else {
    if (n > 0 && collective) {
      char* ptr = arena_ + begin * elem_size_;
      if (compression_ == Compression::BF16) {
        uint16_t* w = wire_ + begin;
        f32_to_bf16_copy(reinterpret_cast<float*>(ptr), w, n, cs);
        comm_->all_reduce(w, w, (size_t)n, ncclBfloat16, ncclAvg, cs);
        bf16_to_f32_copy(w, reinterpret_cast<float*>(ptr), n, cs);
      } else {
        comm_->all_reduce(ptr, ptr, (size_t)n, nccl_dtype(elem_size_), ncclAvg, cs);
      }
    }
    if (n > 0) apply_fused(begin, n, first, cs);
  }
  if (post_bucket) post_bucket(bucket, begin, end, cs);
}

// optimizer update of arena elements [off, off + cnt) minus the ranges a GEMM epilogue already
// updated this iteration (no-op without a fused optimizer)
void RcclBackend::apply_fused(int64_t off, int64_t cnt, bool first, hipStream_t cs) {
  if (cnt <= 0 || fused.kind == 0) return;
  int64_t cur = off;
  const int64_t end = off + cnt;
  for (const auto& r : epi_done_) {  // sorted, disjoint
    if (r.second <= cur || r.first >= end) continue;
    if (r.first > cur) apply_fused_range(cur, r.first - cur, first, cs);
    cur = std::max(cur, r.second);
  }
  if (cur < end) apply_fused_range(cur, end - cur, first, cs);
}

bool RcclBackend::epilogue_allowed() const {
  return fused.kind != 0 && comm_->world() == 1 && skip_single_rank_ &&
         compression_ == Compression::NONE && elem_size_ == 4;
}

OptEpilogue RcclBackend::epilogue_opt(int64_t off, int64_t n) {
  if (!epilogue_allowed()) throw std::runtime_error("optimizer epilogue needs world size 1");
  if (off < 0 || n <= 0 || off + n > numel_) throw std::runtime_error("epilogue range");
  OptEpilogue o;
  o.kind = fused.kind;
  o.p = fused.p + off;
  o.s0 = fused.s0 ? fused.s0 + off : nullptr;
  o.s1 = fused.s1 ? fused.s1 + off : nullptr;
  o.s2 = fused.s2 ? fused.s2 + off : nullptr;
  if (fused.kind == 1) {
    o.sgd = fused.sgd;
    o.sgd.first_step = epi_fresh_;
  } else {
    // the step counter advances with this iteration's first bucket; an epilogue can run before it
    const double t = (double)(fused.adam_step + (bucket0_launched_ ? 0 : 1));
    o.adam = fused.adam;
    o.adam.bc1 = (float)(1.0 - std::pow((double)fused.adam_beta1, t));
    o.adam.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)fused.adam_beta2, t));
  }
  auto it = std::lower_bound(epi_done_.begin(), epi_done_.end(), std::make_pair(off, off + n));
  epi_done_.insert(it, {off, off + n});
  return o;
}

void RcclBackend::apply_fused_range(int64_t off, int64_t cnt, bool first, hipStream_t cs) {
  if (cnt <= 0) return;
  float* g = reinterpret_cast<float*>(arena_) + off;
  if (fused.kind == 1) {
    SgdHyper h = fused.sgd;
    h.first_step = first;
    sgd_flat(fused.p + off, g, fused.s0 ? fused.s0 + off : nullptr, cnt, h, cs);
  } else if (fused.kind == 2) {
    AdamHyper h = fused.adam;
    const double t = (double)(fused.adam_step > 0 ? fused.adam_step : 1);
    h.bc1 = (float)(1.0 - std::pow((double)fused.adam_beta1, t));
    h.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)fused.adam_beta2, t));
    adam_flat(fused.p + off, g, fused.s0 + off, fused.s1 + off,
              fused.s2 ? fused.s2 + off : nullptr, cnt, h, cs);
  }
}

// Apply the deferred world-size-1 bucket updates minus the epilogue-updated ranges, in launches
// of up to kMaxRanges ranges (one launch for the models here: biases + small weights).
void RcclBackend::flush_deferred(hipStream_t compute) {
  if (deferred_.empty()) return;
  std::sort(deferred_.begin(), deferred_.end());
  std::vector<std::pair<int64_t, int64_t>> todo;
  for (const auto& d : deferred_) {
    int64_t cur = d.first;
    for (const auto& r : epi_done_) {
      if (r.second <= cur || r.first >= d.second) continue;
      if (r.first > cur) todo.push_back({cur, r.first});
      cur = std::max(cur, r.second);
    }
    if (cur < d.second) todo.push_back({cur, d.second});
  }
  // merge touching ranges
  std::vector<std::pair<int64_t, int64_t>> merged;
  for (const auto& t : todo) {
    if (!merged.empty() && merged.back().second == t.first) merged.back().second = t.second;
    else merged.push_back(t);
  }
  const bool first = deferred_first_;
  deferred_.clear();
  deferred_first_ = false;
  float* g = reinterpret_cast<float*>(arena_);
  for (size_t i0 = 0; i0 < merged.size(); i0 += kMaxRanges) {
    RangeSet rs;
    for (size_t i = i0; i < merged.size() && rs.n < kMaxRanges; ++i) {
      rs.begin[rs.n] = merged[i].first;
      rs.len[rs.n] = merged[i].second - merged[i].first;
      ++rs.n;
    }
    if (fused.kind == 1) {
      SgdHyper h = fused.sgd;
      h.first_step = first;
      sgd_ranges(fused.p, g, fused.s0, rs, h, compute);
    } else if (fused.kind == 2) {
      AdamHyper h = fused.adam;
      const double t = (double)(fused.adam_step > 0 ? fused.adam_step : 1);
      h.bc1 = (float)(1.0 - std::pow((double)fused.adam_beta1, t));
      h.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)fused.adam_beta2, t));
      adam_ranges(fused.p, g, fused.s0, fused.s1, fused.s2, rs, h, compute);
    }
  }
}

void RcclBackend::wait_all(hipStream_t compute) {
  flush_deferred(compute);
  // iteration boundary: epilogue bookkeeping restarts
  epi_done_.clear();
  if (fused.kind != 0) epi_fresh_ = false;
  bucket0_launched_ = false;
  if (!launched_any_) return;
  if (!launched_side_) {  // everything ran on the compute stream: already ordered
    launched_any_ = false;
    return;
  }
  launched_side_ = false;
  hipStream_t cs = comm_->comm_stream();
  if (timing_) {
    check_hip(hipEventRecord(t1_, cs), "hipEventRecord");
    timed_pending_ = true;
  }
  launched_any_ = false;
  if (stream_mode_ == kStreamNoJoin) return;
  check_hip(hipEventRecord(done_, cs), "hipEventRecord");
  if (stream_mode_ == kStreamHostJoin) {
    check_hip(hipEventSynchronize(done_), "hipEventSynchronize");
    return;
  }
  check_hip(hipStreamWaitEvent(compute, done_, 0), "hipStreamWaitEvent");
}

void RcclBackend::zero(int64_t begin, int64_t end, hipStream_t compute) {
  if (end > begin)
    check_hip(hipMemsetAsync(arena_ + begin * elem_size_, 0, (size_t)(end - begin) * elem_size_,
                             compute),
              "hipMemsetAsync");
}

double RcclBackend::last_comm_ms() {
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
    if (cur_bytes > 0 && cur_bytes + bytes > cap) {
      b.push_back(offsets[i]);
      cur_bytes = 0;
    }
    if (split > 0 && numels[i] > split) {
      // a large parameter gets its own buckets, cut every `split` elements
      if (b.back() != offsets[i]) b.push_back(offsets[i]);
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

void Reducer::prepare_for_backward() {
  pending_ = bucket_nparams_;
  std::fill(param_ready_.begin(), param_ready_.end(), 0);
  for (int b = 0; b < num_buckets(); ++b) bucket_ready_[b] = (bucket_nparams_[b] == 0);
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
