#include "comm.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace tdp {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

static std::atomic<int> g_reserved_cus{-1};

int reserved_cus() {
  int v = g_reserved_cus.load();
  if (v < 0) {
    const char* e = std::getenv("TDP_COMM_CUS");
    v = e ? std::max(0, std::atoi(e)) : 0;
    g_reserved_cus.store(v);
  }
  return v;
}

void set_reserved_cus(int n) { g_reserved_cus.store(std::max(0, n)); }

int compute_cus(int device) {
  static std::mutex mu;
  static std::vector<int> cache;
  int phys = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    if ((int)cache.size() <= device) cache.resize(device + 1, 0);
    if (cache[device] == 0)
      check_hip(hipDeviceGetAttribute(&cache[device], hipDeviceAttributeMultiprocessorCount,
                                      device),
                "hipDeviceGetAttribute");
    phys = cache[device];
  }
  return std::max(1, phys - reserved_cus());
}

std::vector<uint8_t> Communicator::unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::vector<uint8_t> out(sizeof(id.internal));
  std::memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

Communicator::Communicator(const std::vector<uint8_t>& uid, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  ncclUniqueId id;
  if (uid.size() != sizeof(id.internal))
    throw std::runtime_error("RCCL unique id must be " + std::to_string(sizeof(id.internal)) +
                             " bytes");
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  make_stream();
  check_nccl(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
}

Communicator::Communicator(int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  make_stream();
}

void Communicator::make_stream() {
  check_hip(hipSetDevice(device_), "hipSetDevice");
  // Highest priority for the comm stream: bucket all-reduces should not queue behind backward
  // GEMMs on the hardware queues (GPU_MAX_HW_QUEUES=4 per process on this pool).
  int lo = 0, hi = 0;
  check_hip(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  check_hip(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi),
            "hipStreamCreateWithPriority");
  // TDP_TIMEOUT_S (seconds) or TDP_TIMEOUT_MIN (minutes); torch's NCCL default is 10 minutes
  if (const char* t = std::getenv("TDP_TIMEOUT_S")) timeout_s_ = std::atof(t);
  else if (const char* m = std::getenv("TDP_TIMEOUT_MIN")) timeout_s_ = 60.0 * std::atof(m);
}

void Communicator::stop_watchdog() {
  if (thread_.joinable()) {
    stop_ = true;
    cv_.notify_all();
    thread_.join();
  }
}

Communicator::~Communicator() {
  stop_watchdog();
  for (auto& w : watches_) (void)hipEventDestroy(w.ev);
  for (auto e : free_events_) (void)hipEventDestroy(e);
  if (comm_) ncclCommDestroy(comm_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void Communicator::start_watchdog() {
  std::unique_lock<std::mutex> lk(mu_);
  if (!thread_.joinable()) thread_ = std::thread([this] { watchdog_loop(); });
}

void Communicator::watch(hipStream_t s, const char* what) {
  if (timeout_s_ <= 0.0 || (world_ <= 1 && !watch_single_)) return;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return;
  std::unique_lock<std::mutex> lk(mu_);
  if (!thread_.joinable()) thread_ = std::thread([this] { watchdog_loop(); });
  hipEvent_t ev;
  if (!free_events_.empty()) {
    ev = free_events_.back();
    free_events_.pop_back();
  } else {
    check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(watch)");
  }
  check_hip(hipEventRecord(ev, s), "hipEventRecord(watch)");
  watches_.push_back({ev, now_s() + timeout_s_, what});
  cv_.notify_all();
}

int Communicator::pending_watches() {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)watches_.size();
}

void Communicator::watchdog_loop() {
  check_hip(hipSetDevice(device_), "hipSetDevice(watchdog)");
  // this thread polls events (hipEventQuery) while the main thread may be recording a hipGraph
  // in global capture mode: relaxed, its queries no longer invalidate that capture (seen as a
  // one-rank capture failure right after replays left watches pending)
  hipStreamCaptureMode relaxed = hipStreamCaptureModeRelaxed;
  check_hip(hipThreadExchangeStreamCaptureMode(&relaxed), "hipThreadExchangeStreamCaptureMode");
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    // retire finished work in order; the oldest unfinished watch decides
    while (!watches_.empty() && hipEventQuery(watches_.front().ev) == hipSuccess) {
      free_events_.push_back(watches_.front().ev);
      watches_.pop_front();
    }
    std::string err;
    if (device_error(&err)) {
      std::fprintf(stderr, "[tdp] %s; aborting the communicator and exiting\n", err.c_str());
      std::fflush(stderr);
      if (comm_) ncclCommAbort(comm_);
      std::_Exit(86);
    }
    if (!watches_.empty() && now_s() > watches_.front().deadline) {
      const Watch w = watches_.front();
      std::fprintf(stderr,
                   "[tdp] RCCL watchdog: rank %d: '%s' did not finish within %.1f s (a peer "
                   "rank is gone or stalled); aborting the communicator and exiting\n",
                   rank_, w.what.c_str(), timeout_s_);
      std::fflush(stderr);
      if (comm_) ncclCommAbort(comm_);
      std::_Exit(86);
    }
    cv_.wait_for(lk, std::chrono::milliseconds(100));
  }
}

int Communicator::nranks() const {
  if (!comm_) return world_;
  int n = 0;
  check_nccl(ncclCommCount(comm_, &n), "ncclCommCount");
  return n;
}

void Communicator::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void Communicator::all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                              ncclRedOp_t op, hipStream_t s) {
  check_nccl(ncclAllReduce(send, recv, count, dt, op, comm_, s), "ncclAllReduce");
}

void Communicator::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  check_nccl(ncclBroadcast(buf, buf, count, dt, root, comm_, s), "ncclBroadcast");
}

void Communicator::all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                              hipStream_t s) {
  check_nccl(ncclAllGather(send, recv, send_count, dt, comm_, s), "ncclAllGather");
}

void Communicator::reduce_scatter(const void* send, void* recv, size_t recv_count,
                                  ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  check_nccl(ncclReduceScatter(send, recv, recv_count, dt, op, comm_, s), "ncclReduceScatter");
}

void Communicator::send(const void* buf, size_t count, ncclDataType_t dt, int peer,
                        hipStream_t s) {
  check_nccl(ncclSend(buf, count, dt, peer, comm_, s), "ncclSend");
}

void Communicator::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) {
  check_nccl(ncclRecv(buf, count, dt, peer, comm_, s), "ncclRecv");
}

void Communicator::group_start() { check_nccl(ncclGroupStart(), "ncclGroupStart"); }
void Communicator::group_end() { check_nccl(ncclGroupEnd(), "ncclGroupEnd"); }

}  // namespace tdp
