// RCCL communicator: one ncclComm_t per rank (one process per MI355X), collectives over xGMI.
//
// MI355X-native counterpart of c10d's ProcessGroupNCCL as the reference uses it (SURVEY.md §2.3
// N1/N3, §2.6): the unique id is exchanged through the rendezvous store by the Python runtime,
// every collective is enqueued on a caller-chosen HIP stream (the reducer passes its dedicated
// high-priority comm stream; synchronous helpers pass the PyTorch current stream), and nothing
// here blocks the host except init/destroy.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tdp {

void check_hip(hipError_t e, const char* what);
void check_nccl(ncclResult_t r, const char* what);

// CUs left to the collectives: kernels that size their grid to the chip (persistent GEMMs,
// split-K / stream planners) plan for (physical CUs - reserved) so concurrently running RCCL
// kernels on the comm stream do not stretch their last wave (TDP_COMM_CUS, default 0).
int reserved_cus();
void set_reserved_cus(int n);
// physical CU count of `device` minus reserved_cus(), at least 1
int compute_cus(int device);

class Communicator {
 public:
  // 128-byte ncclUniqueId as bytes (rank 0 creates it, the store distributes it)
  static std::vector<uint8_t> unique_id();
  Communicator(const std::vector<uint8_t>& uid, int rank, int world, int device);
  virtual ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  hipStream_t comm_stream() const { return stream_; }
  ncclComm_t handle() const { return comm_; }

  virtual void all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                          ncclRedOp_t op, hipStream_t s);
  virtual void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s);
  virtual void all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                          hipStream_t s);
  virtual void reduce_scatter(const void* send, void* recv, size_t recv_count,
                              ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  virtual void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  virtual void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  virtual void group_start();
  virtual void group_end();
  virtual void abort();

  // Collective watchdog (torch's ProcessGroupNCCL watchdog, TORCH/distributed/constants.py:21
  // default 10 min): watch(s, what) records an event on `s` behind the work
  // enqueued so far; a host thread polls the oldest unfinished events and, once one is older
  // than the timeout, reports it, aborts the communicator (which releases RCCL kernels blocked
  // on a dead peer) and ends the process with exit code 86, so a launcher sees the failure
  // instead of a hang. A no-op while `s` is being captured into a hipGraph (the replay is
  // watched by the caller) or when the timeout is 0.
  void watch(hipStream_t s, const char* what);
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  // watch at world size 1 too (tests: the watchdog path on a one-GPU box)
  void set_watch_single_rank(bool on) { watch_single_ = on; }
  double timeout() const { return timeout_s_; }
  int pending_watches();
  // true when collectives really run on RCCL (false: the host relay of bindings.cpp, the peer
  // vehicle of peer.hip)
  virtual bool native_rccl() const { return true; }
  // ranks the transport itself reports (ncclCommCount for RCCL): the bench's self-check that a
  // world-size-N job really built an N-rank communicator
  virtual int nranks() const;
  // an error the transport detected on the device (the peer vehicle's bounded spins); polled by
  // the watchdog thread, which then reports it and exits 86 like a watchdog timeout
  virtual bool device_error(std::string* what) { (void)what; return false; }

 protected:
  // for subclasses that move the bytes themselves: creates the comm stream, no RCCL communicator
  Communicator(int rank, int world, int device);
  void make_stream();
  void start_watchdog();
  // a subclass whose device_error() the watchdog calls stops the thread in ITS destructor
  void stop_watchdog();

 private:
  struct Watch {
    hipEvent_t ev;
    double deadline;
    std::string what;
  };
  void watchdog_loop();
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
  double timeout_s_ = 600.0;
  bool watch_single_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Watch> watches_;
  std::vector<hipEvent_t> free_events_;
  std::thread thread_;
  std::atomic<bool> stop_{false};
};

}  // namespace tdp
