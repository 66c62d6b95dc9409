#include "loader.h"

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

#include "comm.h"  // check_hip

namespace tdp {

HostBatchLoader::HostBatchLoader(const uint8_t* data, const int64_t* labels, int64_t n,
                                 int64_t row_bytes, int batch, int depth, int threads,
                                 bool pinned)
    : data_(data), labels_(labels), n_(n), row_bytes_(row_bytes), batch_(batch),
      pinned_(pinned) {
  if (n <= 0 || row_bytes <= 0 || batch <= 0) throw std::runtime_error("loader: bad geometry");
  depth = depth < 2 ? 2 : depth;
  threads = threads < 1 ? 1 : threads;
  slots_.resize(depth);
  auto alloc = [&](size_t bytes, const char* what) -> void* {
    void* p = nullptr;
    if (pinned_) check_hip(hipHostMalloc(&p, bytes, hipHostMallocDefault), what);
    else p = ::operator new(bytes);
    return p;
  };
  for (auto& s : slots_) {
    s.x = static_cast<uint8_t*>(alloc((size_t)batch * row_bytes, "hipHostMalloc(loader x)"));
    s.y = static_cast<int64_t*>(alloc((size_t)batch * sizeof(int64_t), "hipHostMalloc(loader y)"));
    s.flip = static_cast<uint8_t*>(alloc((size_t)batch, "hipHostMalloc(loader flip)"));
    if (pinned_)
      check_hip(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate(loader)");
  }
  for (int t = 0; t < threads; ++t) threads_.emplace_back([this] { worker(); });
}

HostBatchLoader::~HostBatchLoader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
  for (auto& s : slots_) {
    if (pinned_) {
      if (s.state == IN_FLIGHT) (void)hipEventSynchronize(s.done);
      (void)hipEventDestroy(s.done);
      (void)hipHostFree(s.x);
      (void)hipHostFree(s.y);
      (void)hipHostFree(s.flip);
    } else {
      ::operator delete(s.x);
      ::operator delete(s.y);
      ::operator delete(s.flip);
    }
  }
}

void HostBatchLoader::start_epoch(const std::vector<int64_t>& idx, bool drop_last,
                                  uint64_t flip_seed, float flip_p) {
  for (int64_t i : idx)
    if (i < 0 || i >= n_) throw std::runtime_error("loader: sample index out of range");
  std::lock_guard<std::mutex> lk(mu_);
  ++epoch_gen_;
  idx_ = idx;
  const int64_t full = (int64_t)idx_.size() / batch_;
  nbatches_ = (drop_last || (int64_t)idx_.size() % batch_ == 0) ? full : full + 1;
  next_gather_ = next_consume_ = 0;
  flip_seed_ = flip_seed;
  flip_p_ = flip_p;
  // gathered batches of the previous epoch are dropped; slots still being gathered are freed
  // by their worker (generation mismatch), slots the consumer holds by release()
  for (auto& s : slots_)
    if (s.state == READY) s.state = FREE;
  cv_.notify_all();
}

static inline uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void HostBatchLoader::worker() {
  // event queries from this thread must not invalidate a step the main thread is capturing
  hipStreamCaptureMode relaxed = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&relaxed);
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<int64_t> rows;
  while (!stop_) {
    // recycle slots whose H2D copy has completed
    bool inflight = false;
    for (auto& s : slots_)
      if (s.state == IN_FLIGHT) {
        if (!pinned_ || hipEventQuery(s.done) == hipSuccess) s.state = FREE;
        else inflight = true;
      }
    Slot* slot = nullptr;
    if (next_gather_ < nbatches_)
      for (auto& s : slots_)
        if (s.state == FREE) {
          slot = &s;
          break;
        }
    if (slot == nullptr) {
      if (inflight) cv_.wait_for(lk, std::chrono::microseconds(200));
      else cv_.wait(lk);
      continue;
    }
    const int64_t b = next_gather_++;
    const uint64_t gen = epoch_gen_, seed = flip_seed_;
    const float p = flip_p_;
    const int64_t lo = b * batch_;
    const int64_t hi = std::min<int64_t>(lo + batch_, (int64_t)idx_.size());
    rows.assign(idx_.begin() + lo, idx_.begin() + hi);
    slot->state = CLAIMED;
    lk.unlock();
    // the host work: gather the sampled rows into pinned memory, labels, flip bits
    for (size_t i = 0; i < rows.size(); ++i) {
      std::memcpy(slot->x + i * row_bytes_, data_ + rows[i] * row_bytes_, (size_t)row_bytes_);
      slot->y[i] = labels_[rows[i]];
      const double u = (double)(mix64(seed ^ mix64((uint64_t)(lo + (int64_t)i))) >> 11) *
                       (1.0 / 9007199254740992.0);
      slot->flip[i] = u < (double)p ? 1 : 0;
    }
    lk.lock();
    if (gen == epoch_gen_) {
      slot->batch_id = b;
      slot->rows = (int)rows.size();
      slot->state = READY;
    } else {
      slot->state = FREE;  // the epoch was restarted meanwhile
    }
    cv_.notify_all();
  }
}

int HostBatchLoader::next(const uint8_t** x, const int64_t** y, const uint8_t** flip,
                          int* rows) {
  std::unique_lock<std::mutex> lk(mu_);
  if (next_consume_ >= nbatches_) return -1;
  const int64_t want = next_consume_;
  const uint64_t gen = epoch_gen_;
  for (;;) {
    for (size_t i = 0; i < slots_.size(); ++i) {
      Slot& s = slots_[i];
      if (s.state == READY && s.batch_id == want) {
        s.state = HELD;  // the consumer's until release() records its event
        s.batch_id = -1;
        ++next_consume_;
        *x = s.x;
        *y = s.y;
        *flip = s.flip;
        *rows = s.rows;
        cv_.notify_all();
        return (int)i;
      }
    }
    if (stop_ || gen != epoch_gen_) return -1;
    cv_.wait(lk);
  }
}

void HostBatchLoader::release(int slot, hipStream_t stream) {
  if (slot < 0 || slot >= (int)slots_.size()) throw std::runtime_error("loader: bad slot");
  std::lock_guard<std::mutex> lk(mu_);
  Slot& s = slots_[slot];
  if (s.state != HELD) throw std::runtime_error("loader: release of a slot not held");
  // the event marks the end of the copies that read the slot's pinned memory (without pinned
  // staging the consumer copied synchronously: the slot is free right away)
  if (pinned_) check_hip(hipEventRecord(s.done, stream), "hipEventRecord(loader)");
  s.state = IN_FLIGHT;
  cv_.notify_all();
}

}  // namespace tdp
