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

#include <cstdint>
#include <string>
#include <vector>

namespace tdp {

void check_hip(hipError_t e, const char* what);
void check_nccl(ncclResult_t r, const char* what);

class Communicator {
 public:
  // 128-byte ncclUniqueId as bytes (rank 0 creates it, the store distributes it)
  static std::vector<uint8_t> unique_id();
  Communicator(const std::vector<uint8_t>& uid, int rank, int world, int device);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  hipStream_t comm_stream() const { return stream_; }
  ncclComm_t handle() const { return comm_; }

  void all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                  hipStream_t s);
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s);
  void all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                  hipStream_t s);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, ncclDataType_t dt,
                      ncclRedOp_t op, hipStream_t s);
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  void group_start();
  void group_end();
  void abort();

 private:
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
};

}  // namespace tdp
