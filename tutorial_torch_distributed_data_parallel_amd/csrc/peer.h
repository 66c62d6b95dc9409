// Peer-memory communicator: W rank processes exchange data through each other's device memory
// (HIP IPC handles), with every collective ONE kernel synchronised by device-side counters.
//
// Why it exists ("a capture-capable multi-rank vehicle on one GPU"): RCCL refuses
// two ranks on one device, and the host relay (parallel/relay.py) cannot be captured into a
// hipGraph. This transport is kernels only -- a collective is a launch on the caller's stream
// whose arguments never change between calls of the same shape, and whose epoch lives in device
// memory -- so the whole multi-rank training step (side-stream bucket collectives, factored
// gathers, fork / join edges) can be captured and replayed with REAL peers on one MI355X. The
// same kernels read peer windows through any mapping HIP IPC gives them, so on a node they are
// also the seed of an xGMI peer-memory all-gather.
//
// Window of rank r (one hipMalloc, exported with hipIpcGetMemHandle, zeroed before export):
//   control lines (64 B apart): epoch, arrive, done, abort, readack[p] for every peer p
//   data slot of `slot_bytes`: rank r's contribution to the current collective
// Protocol of one collective at epoch e (G workgroups per launch, G identical on all ranks):
//   0. a rank that writes its slot first waits until every peer acknowledged reading epoch e-1
//      (readack_r[p] >= G*(e-1));
//   1. each workgroup copies its part of the contribution into the slot, drains its stores,
//      releases (agent scope) and adds 1 to arrive_r;
//   2. each workgroup polls arrive_p >= G*e of the peers it reads, acquires, reads / reduces
//      (peers in rank order: bit-identical results on every rank), then adds 1 to readack_p[r];
//   3. the last workgroup to finish (done counter) advances epoch_r.
// Every spin is bounded (wall clock, TDP_PEER_TIMEOUT_S, default 30 s): on expiry the workgroup
// raises the window's abort word and a host-mapped error word and leaves; later collectives of
// an aborted communicator return at once, and the watchdog thread reports and exits 86.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "comm.h"

namespace tdp {

constexpr int kPeerMaxWorld = 16;

// test hook: one workgroup that waits `ms` of wall-clock time on `s`, then exits (a bounded stall
// in front of a watched collective: the watchdog tests)
void debug_spin_ms(int ms, hipStream_t s);

class PeerCommunicator : public Communicator {
 public:
  PeerCommunicator(int rank, int world, int device, int64_t slot_bytes);
  ~PeerCommunicator() override;
  bool native_rccl() const override { return false; }
  int nranks() const override { return world(); }

  // hipIpcMemHandle of this rank's window (64 bytes); connect() opens every peer's
  std::vector<uint8_t> local_handle() const;
  void connect(const std::vector<std::vector<uint8_t>>& handles);
  int64_t slot_bytes() const { return slot_bytes_; }

  void all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                  hipStream_t s) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                  hipStream_t s) override;
  void reduce_scatter(const void* send, void* recv, size_t recv_count, ncclDataType_t dt,
                      ncclRedOp_t op, hipStream_t s) override;
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) override;
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) override;
  void group_start() override {}
  void group_end() override {}
  void abort() override;
  bool device_error(std::string* what) override;

  // test hook: the next collective's workgroups of this rank stall `ms` before arriving
  // (bounded), so a peer's spin expires (tests/test_peer_gpu.py)
  void inject_stall_ms(int ms) { stall_ms_ = ms; }

 private:
  void launch(int kind, const void* send, void* recv, int64_t n_elems, int64_t seg_stride,
              int esize, ncclDataType_t dt, ncclRedOp_t op, int root, hipStream_t s);
  void check_connected() const;
  // Collectives of one communicator must run one at a time, in issue order, on every rank: the
  // epoch counters (and the slots) are per communicator. A collective issued on another stream
  // than the previous one first waits for it (an event; a graph edge while capturing), as RCCL
  // orders a communicator's operations across streams.
  void order_after_previous(hipStream_t s);
  void note_issued(hipStream_t s);
  hipEvent_t last_ev_ = nullptr;
  hipStream_t last_stream_ = nullptr;
  unsigned long long last_capture_ = 0;  // capture id of the last issue (0 = eager)
  bool have_last_ = false;
  char* win_ = nullptr;                      // own window (control + slot)
  std::vector<char*> peers_;                 // every rank's window as mapped here
  std::vector<bool> opened_;                 // peers_[p] came from hipIpcOpenMemHandle
  int64_t slot_bytes_ = 0;
  uint32_t* err_host_ = nullptr;             // host-mapped error word
  uint32_t* err_dev_ = nullptr;
  uint64_t timeout_ticks_ = 0;
  int clock_khz_ = 100000;
  int stall_ms_ = 0;
};

}  // namespace tdp
