// Host-dataset input pipeline: the MI355X-native replacement of the reference's DataLoader with
// 2 worker processes, pin_memory=True and a CPU Resize(224) / RandomHorizontalFlip / Normalize
// chain (REF/multi-GPU-training-torch.py:86-99, REF/data_and_toy_model.py:8-38; SURVEY.md §2.3
// N9, B10).
//
// The CPU side only does what must happen on the host: gathering the sampled rows of a uint8
// HWC dataset (host RAM or a memory map) into PINNED staging slots, plus the per-sample flip
// bits, on a pool of C++ worker threads that run ahead of the training loop by `depth` batches.
// The consumer copies a ready slot to the device with one async copy (tiny: 128 x 32x32x3 bytes
// = 393 KB per CIFAR batch) and the resize / flip / normalise runs on the GPU
// (image.hip: image_transform), so the 224x224 float batch never crosses PCIe.
//
// Slot life cycle: FREE -> CLAIMED (worker gathers) -> READY -> HELD (consumer: H2D copy enqueued, event
// recorded) -> IN_FLIGHT -> (a worker sees the event complete) -> FREE (HELD while the consumer
// holds the slot between next() and release()). A slot's pinned memory
// is therefore never rewritten while its copy may still be reading it.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace tdp {

class HostBatchLoader {
 public:
  // data: n rows of row_bytes (uint8), labels: n int64; both must outlive the loader.
  // pinned=false: plain host staging and no events (CPU-only runs and tests)
  HostBatchLoader(const uint8_t* data, const int64_t* labels, int64_t n, int64_t row_bytes,
                  int batch, int depth, int threads, bool pinned = true);
  ~HostBatchLoader();
  HostBatchLoader(const HostBatchLoader&) = delete;
  HostBatchLoader& operator=(const HostBatchLoader&) = delete;

  // Begin an epoch over `idx` (sample order, e.g. DistributedSampler's); batches of `batch`
  // consecutive indices (the last one short unless drop_last). Flip bits come from a
  // counter-based hash of (flip_seed, sample position), so they are reproducible.
  void start_epoch(const std::vector<int64_t>& idx, bool drop_last, uint64_t flip_seed,
                   float flip_p);
  int64_t num_batches() const { return nbatches_; }

  // Next batch in order: blocks until its slot is gathered. Fills the pinned host pointers
  // (x rows, labels, flip bytes) and the batch size; returns the slot id, or -1 at epoch end.
  int next(const uint8_t** x, const int64_t** y, const uint8_t** flip, int* rows);
  // The consumer enqueued the slot's H2D copies on `stream`; the slot is recycled once the
  // work on `stream` up to now has completed.
  void release(int slot, hipStream_t stream);

 private:
  enum State { FREE, CLAIMED, READY, HELD, IN_FLIGHT };  // CLAIMED: a worker gathers it
  struct Slot {
    uint8_t* x = nullptr;     // pinned [batch][row_bytes]
    int64_t* y = nullptr;     // pinned [batch]
    uint8_t* flip = nullptr;  // pinned [batch]
    hipEvent_t done = nullptr;
    int64_t batch_id = -1;
    int rows = 0;
    State state = FREE;
  };
  void worker();

  const uint8_t* data_;
  const int64_t* labels_;
  int64_t n_, row_bytes_;
  int batch_;
  bool pinned_;
  std::vector<Slot> slots_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  // epoch state
  std::vector<int64_t> idx_;
  int64_t nbatches_ = 0, next_gather_ = 0, next_consume_ = 0;
  uint64_t epoch_gen_ = 0, flip_seed_ = 0;
  float flip_p_ = 0.f;
};

}  // namespace tdp
