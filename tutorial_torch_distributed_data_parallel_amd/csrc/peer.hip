// Peer-memory communicator (peer.h): one kernel per collective, device-side counters, bounded
// spins. The memory-ordering forms follow the CDNA4 guide's valid cross-XCD hand-off recipes
// (MI355X_MICROARCH.md "inter-workgroup visibility"): producer = plain stores, every storing
// wave drains (vmcnt 0), workgroup barrier, ONE lane releases at agent scope, drains again, and
// adds to a counter with an agent-scope atomic; consumer = ONE lane polls with relaxed
// agent-scope loads, acquires at agent scope, drains, workgroup barrier, then plain loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "peer.h"

namespace tdp {
namespace {

constexpr int kLineBytes = 64;
enum Line { kEpoch = 0, kArrive = 1, kDone = 2, kAbort = 3, kAck0 = 4 };
constexpr int64_t kCtrlBytes = 4096;
static_assert(kLineBytes * (kAck0 + kPeerMaxWorld) <= kCtrlBytes, "control region");
constexpr int kG = 64;    // workgroups per collective launch: identical on every rank
constexpr int kT = 256;   // threads per workgroup

enum Kind { kAllGather = 0, kAllReduce = 1, kReduceScatter = 2, kBroadcast = 3 };
enum Red { kSum = 0, kAvg = 1, kMax = 2, kMin = 3, kProd = 4 };

struct PeerArgs {
  char* win[kPeerMaxWorld];
  const char* send;
  char* recv;
  int64_t n;       // elements of this chunk per rank segment
  int64_t stride;  // elements between rank segments (all-gather: in recv; reduce-scatter: in send)
  int esize;
  int rank, world, kind, root, red;
  uint32_t* err;
  uint64_t timeout;
  uint64_t stall;
};

__device__ inline uint32_t* line(char* w, int l) {
  return reinterpret_cast<uint32_t*>(w + (int64_t)l * kLineBytes);
}
__device__ inline uint32_t poll(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t add(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline bool reached(uint32_t v, uint32_t target) { return (int32_t)(v - target) >= 0; }
__device__ inline void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// lane 0 only: spin until *p >= target; false on timeout or abort (then the error is raised)
__device__ bool wait_ge(uint32_t* p, uint32_t target, char* peer_win, const PeerArgs& a,
                        uint32_t code) {
  uint32_t* abort_own = line(a.win[a.rank], kAbort);
  const long long t0 = wall_clock64();
  for (;;) {
    if (reached(poll(p), target)) return true;
    if (poll(abort_own) != 0 || poll(line(peer_win, kAbort)) != 0) {
      __hip_atomic_store(abort_own, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if ((uint64_t)(wall_clock64() - t0) > a.timeout) {
      __hip_atomic_store(abort_own, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// grid-wide byte copy (all workgroups of the launch share the range)
__device__ void copy_bytes(char* dst, const char* src, int64_t bytes) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const uintptr_t al = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
  if ((al & 15) == 0) {
    const int64_t n16 = bytes >> 4;
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (int64_t i = tid; i < n16; i += nth) d[i] = s[i];
    for (int64_t i = (n16 << 4) + tid; i < bytes; i += nth) dst[i] = src[i];
  } else if ((al & 3) == 0) {
    const int64_t n4 = bytes >> 2;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = tid; i < n4; i += nth) d[i] = s[i];
    for (int64_t i = (n4 << 2) + tid; i < bytes; i += nth) dst[i] = src[i];
  } else {
    for (int64_t i = tid; i < bytes; i += nth) dst[i] = src[i];
  }
}

struct Bf16 {
  uint16_t v;
};

template <class T>
struct Acc {
  using type = T;
  __device__ static T load(const char* p, int64_t i) { return reinterpret_cast<const T*>(p)[i]; }
  __device__ static void store(char* p, int64_t i, T x) { reinterpret_cast<T*>(p)[i] = x; }
};
template <>
struct Acc<Bf16> {
  using type = float;
  __device__ static float load(const char* p, int64_t i) {
    return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[i] << 16);
  }
  __device__ static void store(char* p, int64_t i, float x) {
    uint32_t u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) u |= 0x00400000u;  // NaN stays a quiet NaN
    else u += 0x7fffu + ((u >> 16) & 1u);                    // round to nearest even
    reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)(u >> 16);
  }
};

template <class V>
__device__ inline V combine(V a, V b, int red) {
  switch (red) {
    case kMax: return a > b ? a : b;
    case kMin: return a < b ? a : b;
    case kProd: return a * b;
    default: return a + b;
  }
}

// recv[i] = red over p (rank order) of slot_p[off + i], i < n
template <class T>
__device__ void reduce_slots(const PeerArgs& a, int64_t off) {
  using V = typename Acc<T>::type;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const char* s0 = a.win[0] + kCtrlBytes;
  for (int64_t i = tid; i < a.n; i += nth) {
    V acc = Acc<T>::load(s0, off + i);
    for (int p = 1; p < a.world; ++p)
      acc = combine<V>(acc, Acc<T>::load(a.win[p] + kCtrlBytes, off + i), a.red);
    if (a.red == kAvg) acc = acc / (V)a.world;
    Acc<T>::store(a.recv, i, acc);
  }
}

template <class T>
__global__ __launch_bounds__(kT) void peer_collective_kernel(PeerArgs a) {
  __shared__ uint32_t s_epoch;
  __shared__ int s_ok;
  char* own = a.win[a.rank];
  const uint32_t G = gridDim.x;
  if (threadIdx.x == 0) {
    s_ok = poll(line(own, kAbort)) == 0;
    s_epoch = add(line(own, kEpoch), 0u) + 1u;  // a returning atomic: the coherent value
  }
  __syncthreads();
  if (!s_ok) return;  // an aborted communicator: every later collective returns at once
  const uint32_t e = s_epoch;
  const int W = a.world, r = a.rank;
  const bool writes = a.kind != kBroadcast || r == a.root;
  const int64_t seg = a.n * a.esize;
  char* slot = own + kCtrlBytes;
  // 0. the slot is free once every peer read epoch e-1 from it
  if (writes && e > 1u) {
    if (threadIdx.x == 0)
      for (int p = 0; p < W && s_ok; ++p)
        if (p != r && !wait_ge(line(own, kAck0 + p), G * (e - 1u), a.win[p], a, 1u)) s_ok = 0;
    __syncthreads();
    if (!s_ok) return;
  }
  // 1. this rank's contribution into its slot
  if (writes) {
    if (a.kind == kReduceScatter) {
      for (int q = 0; q < W; ++q)
        copy_bytes(slot + q * seg, a.send + (int64_t)q * a.stride * a.esize, seg);
    } else {
      copy_bytes(slot, a.send, seg);
    }
  }
  if (a.stall && threadIdx.x == 0) {  // test hook (inject_stall_ms): bounded by itself
    const long long t0 = wall_clock64();
    while ((uint64_t)(wall_clock64() - t0) < a.stall) __builtin_amdgcn_s_sleep(127);
  }
  drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain();
    add(line(own, kArrive), 1u);
  }
  // 2. wait for the slots this rank reads, then read them
  if (threadIdx.x == 0) {
    for (int p = 0; p < W && s_ok; ++p) {
      const bool needed = a.kind == kBroadcast ? (p == a.root && r != a.root) : true;
      if (needed && !wait_ge(line(a.win[p], kArrive), G * e, a.win[p], a, 2u)) s_ok = 0;
    }
    if (s_ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain();
  }
  __syncthreads();
  if (!s_ok) return;
  switch (a.kind) {
    case kAllGather:
      for (int p = 0; p < W; ++p)
        copy_bytes(a.recv + (int64_t)p * a.stride * a.esize, a.win[p] + kCtrlBytes, seg);
      break;
    case kAllReduce:
      reduce_slots<T>(a, 0);
      break;
    case kReduceScatter:
      reduce_slots<T>(a, (int64_t)r * a.n);
      break;
    default:  // broadcast
      if (r != a.root) copy_bytes(a.recv, a.win[a.root] + kCtrlBytes, seg);
  }
  // 3. acknowledge the reads (the loads have returned), count this workgroup done
  drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int p = 0; p < W; ++p)
      if (p != r) add(line(a.win[p], kAck0 + r), 1u);
    if (add(line(own, kDone), 1u) + 1u == G * e)
      __hip_atomic_store(line(own, kEpoch), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int dt_size(ncclDataType_t dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: throw std::runtime_error("peer communicator: unsupported dtype");
  }
}

int red_code(ncclRedOp_t op) {
  switch (op) {
    case ncclSum: return kSum;
    case ncclAvg: return kAvg;
    case ncclMax: return kMax;
    case ncclMin: return kMin;
    case ncclProd: return kProd;
    default: throw std::runtime_error("peer communicator: unsupported reduce op");
  }
}

void* kernel_for(ncclDataType_t dt, bool reduces) {
  if (!reduces) return reinterpret_cast<void*>(&peer_collective_kernel<uint8_t>);
  switch (dt) {
    case ncclFloat32: return reinterpret_cast<void*>(&peer_collective_kernel<float>);
    case ncclFloat64: return reinterpret_cast<void*>(&peer_collective_kernel<double>);
    case ncclInt32: return reinterpret_cast<void*>(&peer_collective_kernel<int32_t>);
    case ncclInt64: return reinterpret_cast<void*>(&peer_collective_kernel<int64_t>);
    case ncclBfloat16: return reinterpret_cast<void*>(&peer_collective_kernel<Bf16>);
    default: throw std::runtime_error("peer communicator: no reduction for this dtype");
  }
}

__global__ void debug_spin_kernel(uint64_t ticks) {
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    while ((uint64_t)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(127);
  }
}

}  // namespace

void debug_spin_ms(int ms, hipStream_t s) {
  int dev = 0, khz = 0;
  check_hip(hipGetDevice(&dev), "hipGetDevice");
  check_hip(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev),
            "hipDeviceGetAttribute(wall clock)");
  const uint64_t ticks = (uint64_t)std::max(0, ms) * (uint64_t)(khz > 0 ? khz : 100000);
  hipLaunchKernelGGL(debug_spin_kernel, dim3(1), dim3(64), 0, s, ticks);
  check_hip(hipGetLastError(), "debug_spin_kernel");
}

PeerCommunicator::PeerCommunicator(int rank, int world, int device, int64_t slot_bytes)
    : Communicator(rank, world, device), slot_bytes_(slot_bytes) {
  if (world < 1 || world > kPeerMaxWorld)
    throw std::runtime_error("peer communicator: world size must be in [1, 16]");
  if (slot_bytes_ < 4096 || slot_bytes_ % 256)
    throw std::runtime_error("peer communicator: slot must be >= 4 KiB, a multiple of 256 B");
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipMalloc(&win_, kCtrlBytes + slot_bytes_), "hipMalloc(peer window)");
  check_hip(hipMemset(win_, 0, kCtrlBytes), "hipMemset(peer window)");
  check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 64, hipHostMallocMapped),
            "hipHostMalloc(peer error word)");
  *err_host_ = 0;
  check_hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0),
            "hipHostGetDevicePointer");
  int khz = 0;
  check_hip(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device),
            "hipDeviceGetAttribute(wall clock)");
  double secs = 30.0;
  if (const char* t = std::getenv("TDP_PEER_TIMEOUT_S")) secs = std::atof(t);
  clock_khz_ = khz > 0 ? khz : 100000;
  timeout_ticks_ = (uint64_t)(secs * 1000.0 * clock_khz_);
  peers_.assign(world, nullptr);
  opened_.assign(world, false);
  peers_[rank] = win_;
  check_hip(hipEventCreateWithFlags(&last_ev_, hipEventDisableTiming), "hipEventCreate");
}

static unsigned long long capture_id(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  check_hip(hipStreamGetCaptureInfo(s, &st, &id), "hipStreamGetCaptureInfo");
  return st == hipStreamCaptureStatusActive ? id : 0ull;
}

void PeerCommunicator::order_after_previous(hipStream_t s) {
  // an eager issue cannot wait on a node of a finished capture, nor a capture on eager work
  // (that work is complete before any replay: the callers synchronise around captures)
  if (have_last_ && last_stream_ != s && last_capture_ == capture_id(s))
    check_hip(hipStreamWaitEvent(s, last_ev_, 0), "hipStreamWaitEvent(peer order)");
}

void PeerCommunicator::note_issued(hipStream_t s) {
  check_hip(hipEventRecord(last_ev_, s), "hipEventRecord(peer order)");
  last_stream_ = s;
  last_capture_ = capture_id(s);
  have_last_ = true;
}

PeerCommunicator::~PeerCommunicator() {
  stop_watchdog();  // it calls device_error() of this object
  (void)hipSetDevice(device());
  (void)hipDeviceSynchronize();
  for (int p = 0; p < (int)peers_.size(); ++p)
    if (opened_[p]) (void)hipIpcCloseMemHandle(peers_[p]);
  if (win_) (void)hipFree(win_);
  if (last_ev_) (void)hipEventDestroy(last_ev_);
  if (err_host_) (void)hipHostFree(err_host_);
}

std::vector<uint8_t> PeerCommunicator::local_handle() const {
  hipIpcMemHandle_t h;
  check_hip(hipIpcGetMemHandle(&h, win_), "hipIpcGetMemHandle(peer window)");
  std::vector<uint8_t> out(sizeof(h));
  std::memcpy(out.data(), &h, sizeof(h));
  return out;
}

void PeerCommunicator::connect(const std::vector<std::vector<uint8_t>>& handles) {
  if ((int)handles.size() != world()) throw std::runtime_error("peer connect: one handle per rank");
  check_hip(hipSetDevice(device()), "hipSetDevice");
  for (int p = 0; p < world(); ++p) {
    if (p == rank() || opened_[p]) continue;
    hipIpcMemHandle_t h;
    if (handles[p].size() != sizeof(h)) throw std::runtime_error("peer connect: bad handle size");
    std::memcpy(&h, handles[p].data(), sizeof(h));
    void* ptr = nullptr;
    check_hip(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess),
              "hipIpcOpenMemHandle(peer window)");
    peers_[p] = static_cast<char*>(ptr);
    opened_[p] = true;
  }
  if (world() > 1) start_watchdog();  // reports device-side timeouts even without a watch()
}

void PeerCommunicator::check_connected() const {
  for (auto* p : peers_)
    if (!p) throw std::runtime_error("peer communicator used before connect()");
}

bool PeerCommunicator::device_error(std::string* what) {
  const uint32_t e = __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
  if (e == 0) return false;
  if (what)
    *what = std::string("peer communicator: rank ") + std::to_string(rank()) + ": a bounded " +
            (e == 1 ? "wait for a peer to release its slot" : "wait for a peer's data") +
            " expired (TDP_PEER_TIMEOUT_S; a peer rank is gone or stalled)";
  return true;
}

void PeerCommunicator::abort() {
  // raise the window's abort word: every later collective (here and, through its polls, at the
  // peers) returns at once instead of waiting
  const uint32_t one = 1;
  (void)hipMemcpy(win_ + (int64_t)kAbort * kLineBytes, &one, 4, hipMemcpyHostToDevice);
}

void PeerCommunicator::launch(int kind, const void* send, void* recv, int64_t n_elems,
                              int64_t stride, int esize, ncclDataType_t dt, ncclRedOp_t op,
                              int root, hipStream_t s) {
  PeerArgs a{};
  for (int p = 0; p < world(); ++p) a.win[p] = peers_[p];
  a.send = static_cast<const char*>(send);
  a.recv = static_cast<char*>(recv);
  a.n = n_elems;
  a.stride = stride;
  a.esize = esize;
  a.rank = rank();
  a.world = world();
  a.kind = kind;
  a.root = root;
  const bool reduces = kind == kAllReduce || kind == kReduceScatter;
  a.red = reduces ? red_code(op) : kSum;
  a.err = err_dev_;
  a.timeout = timeout_ticks_;
  a.stall = 0;
  if (stall_ms_ > 0) {
    a.stall = (uint64_t)stall_ms_ * (uint64_t)clock_khz_;  // wall-clock ticks per ms = kHz
    stall_ms_ = 0;
  }
  void* args[] = {&a};
  order_after_previous(s);
  check_hip(hipLaunchKernel(kernel_for(dt, reduces), dim3(kG), dim3(kT), args, 0, s),
            "hipLaunchKernel(peer collective)");
  note_issued(s);
}

void PeerCommunicator::all_gather(const void* send, void* recv, size_t send_count,
                                  ncclDataType_t dt, hipStream_t s) {
  check_connected();
  const int es = dt_size(dt);
  const int64_t n = (int64_t)send_count, cap = slot_bytes_ / es;
  for (int64_t off = 0; off < n; off += cap) {
    const int64_t c = std::min(cap, n - off);
    launch(kAllGather, static_cast<const char*>(send) + off * es,
           static_cast<char*>(recv) + off * es, c, n, es, dt, ncclSum, 0, s);
  }
}

void PeerCommunicator::all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                                  ncclRedOp_t op, hipStream_t s) {
  check_connected();
  const int es = dt_size(dt);
  const int64_t n = (int64_t)count, cap = slot_bytes_ / es;
  for (int64_t off = 0; off < n; off += cap) {
    const int64_t c = std::min(cap, n - off);
    launch(kAllReduce, static_cast<const char*>(send) + off * es,
           static_cast<char*>(recv) + off * es, c, 0, es, dt, op, 0, s);
  }
}

void PeerCommunicator::reduce_scatter(const void* send, void* recv, size_t recv_count,
                                      ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  check_connected();
  const int es = dt_size(dt);
  const int64_t n = (int64_t)recv_count, cap = slot_bytes_ / es / world();
  for (int64_t off = 0; off < n; off += cap) {
    const int64_t c = std::min(cap, n - off);
    launch(kReduceScatter, static_cast<const char*>(send) + off * es,
           static_cast<char*>(recv) + off * es, c, n, es, dt, op, 0, s);
  }
}

void PeerCommunicator::broadcast(void* buf, size_t count, ncclDataType_t dt, int root,
                                 hipStream_t s) {
  check_connected();
  const int es = dt_size(dt);
  const int64_t n = (int64_t)count, cap = slot_bytes_ / es;
  for (int64_t off = 0; off < n; off += cap) {
    const int64_t c = std::min(cap, n - off);
    char* p = static_cast<char*>(buf) + off * es;
    launch(kBroadcast, p, p, c, 0, es, dt, ncclSum, root, s);
  }
}

void PeerCommunicator::send(const void*, size_t, ncclDataType_t, int, hipStream_t) {
  throw std::runtime_error("peer communicator: point-to-point send is not implemented");
}
void PeerCommunicator::recv(void*, size_t, ncclDataType_t, int, hipStream_t) {
  throw std::runtime_error("peer communicator: point-to-point recv is not implemented");
}

}  // namespace tdp
