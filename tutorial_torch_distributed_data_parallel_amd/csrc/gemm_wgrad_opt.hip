// Weight gradient + optimizer update in one launch, warp-specialised (gfx950).
//
// What it computes: for a Linear weight W[M][N] with output gradient g [K][M] (K = batch) and
// input x [K][N], dW = g^T x is never stored -- each 128 x 128 tile of dW goes straight into the
// optimizer update of W's tile and its state (SGD momentum / Adam moments), as the optimizer
// epilogue of gemm_f32_fast.hip does (OptEpilogue, kernels.h). The tile GEMM is short (K = 128
// for the toy MLP), the update streams 16 (SGD) / 24 (Adam) bytes per element through HBM: the
// kernel is HBM-bound, and what it must get right is keeping HBM busy all the time.
//
// Why a second kernel (profiles/r9/*): the persistent epilogue kernel alternates, inside every
// workgroup, an MFMA phase (no HBM traffic) with an update phase (HBM traffic, no MFMA); two
// workgroups per CU overlap the phases only by chance, and the toy MLP's fc1 / fc2 updates ran
// at 4.7 TB/s where a tile-shaped non-temporal stream of the same bytes reaches 5.3-5.5 TB/s
// (dev/micro/stream_sgd.hip). Here ONE 512-thread workgroup per CU splits the roles:
//   * waves 0-3 (math): tile t's gradient -- operands straight from L2 into registers (8-B
//     buffer loads in the MFMA layout: two 32 x 32 tiles per wave interleave their rows /
//     columns so one float2 feeds both; the next 16-deep k-step's loads in flight behind this
//     one's MFMAs), native fp32 products on v_mfma_f32_32x32x2_f32 (no VALU at all: the math
//     only has to stay under the stream's time per tile), then the finished 128 x 128 fp32 tile
//     into one of two LDS buffers G (tile t -> t & 1);
//   * waves 4-7 (stream): p / state loads of the NEXT batch are always in flight (they do not
//     depend on the gradient, so the next tile's first batch is issued before this tile's last
//     update), each batch's gradient chunks are read from G beside its update, and every 16-B p /
//     state chunk is stored non-temporally.
// The roles hand the G buffers over through LDS counters (full / empty per buffer, one increment
// per wave), so the math waves compute tile t+1 while the stream waves update tile t; no barrier is
// shared between the roles. Spins are intra-workgroup only (every wave of a workgroup is resident
// by construction) with s_sleep.
// Bias: the math waves of the first column tile also sum their A values over K (the bias
// gradient) and update the bias (or store the sums) -- GemmF32Args::rowsum / bias_opt semantics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "optim_elem.h"

namespace tdp {
namespace {

constexpr int kWT = 512;  // 8 waves: 4 math + 4 stream
constexpr int kTM = 128, kTN = 128;
constexpr int kGFloats = kTM * kTN;

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct WsParams {
  const float* A;  // [K][M] (lda)
  const float* B;  // [K][N] (ldb)
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  OptEpilogue opt;   // the weight's update (kind 1 SGD, 2 Adam)
  OptEpilogue bopt;  // kind != 0: update the bias (these pointers, opt's hyper) from the row sums
  float* rowsum;     // else, when set: rowsum = rowsum_beta * rowsum + sum_k A
  float rowsum_beta;
  int exp;           // timing experiments only (TDP_WS_EXP): 1 math skips its K loop, 2 stream
                     // skips its HBM traffic (both keep the hand-over), 4 math loads nothing
};

__device__ __forceinline__ int lds_load(const int* c) {
  return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// every LDS operation this wave issued has completed, then one lane counts the wave in
__device__ __forceinline__ void lds_signal(int* c) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void lds_wait(const int* c, int target) {
  while (lds_load(c) < target) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}

template <int KIND>
__global__ __launch_bounds__(kWT) __attribute__((amdgpu_waves_per_eu(2, 2))) void wgrad_opt_kernel(
    WsParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* G = reinterpret_cast<float*>(smem);
  // per G buffer: full[b] / empty[b] count the waves that published / released its uses. Per
  // buffer, not per kernel: waves of one role are not in lockstep, and with one shared counter a
  // wave already on tile t+1 would make tile t look complete. Per buffer, a wave can add to use
  // u+1 only after every wave of the other role has finished use u (see the two waits), so a
  // count of 4 (u + 1) means exactly "use u is complete".
  int* full = reinterpret_cast<int*>(smem + 2 * kGFloats * 4);  // after the two G buffers
  int* empty = full + 2;
  if (threadIdx.x < 4) full[threadIdx.x] = 0;  // full[0..1], empty[0..1]
  __syncthreads();  // the last barrier both roles share

  // XCD-aware persistent tile ranges (gemm_f32_fast.hip's persistent form): blocks b and b + 8
  // share an XCD; each XCD walks a contiguous range of tiles, its workgroups interleaved over
  // it. Tile order: row blocks fastest (tile = tn * tiles_m + tm), so the ~32 tiles an XCD runs
  // at once share ONE column block of x (read from the MALL once per XCD) and walk the rows of
  // g, which stays L2-resident (toy MLP: 2 MB): the math waves' operand loads hit L2. (Column
  // blocks fastest streamed x through L2 once per row panel and exposed MALL latency on every
  // k-step.)
  const int T = p.tiles_m * p.tiles_n;
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int per = q8 + (xcd < r8 ? 1 : 0);
  const int before = xcd * q8 + (xcd < r8 ? xcd : r8);
  const int t0 = (int)((long)T * before / nwg), t1 = (int)((long)T * (before + per) / nwg);
  const int j0 = b / 8;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  constexpr bool SGD = KIND == 1;

  if (wave < 4) {
    // ------------------------------------------------------------------ math waves
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l31 = lane & 31;
    const int nks = (p.exp & 1) ? 0 : (p.K + 15) / 16;
    // operand descriptors from kernel arguments only (wave-uniform: no waterfall loops)
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.A), 0, 0x7fffffff,
                                                      0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, 0x7fffffff,
                                                      0x00020000);
    int i = 0;
    for (int lid = t0 + j0; lid < t1; lid += per, ++i) {
      const int tn = lid / p.tiles_m, tm = lid - tn * p.tiles_m;
      const int m0 = tm * kTM, n0 = tn * kTN;
      // this lane's two rows (tile f = 0, 1) and two columns (tile g = 0, 1); clamped in range
      // (out-of-range rows / columns only feed outputs nobody stores)
      const int am = min(m0 + wm * 64 + 2 * l31, p.M - 2);
      const int bc = min(n0 + wn * 64 + 2 * l31, p.N - 2);
      // k slots: bf16 element e of lane half h is k = k0 + 4h + e (e < 4) or k0 + 4h + e + 4
      // (e >= 4) -- gemm_f32_fast.hip's order (its fp32 fragment reads give lane half h the
      // k = 8q + 4h + s of two consecutive q), so every MFMA sees the same operands in the same
      // slots and the gradient is bit-identical to the persistent epilogue kernel's
      auto kslot = [&](int e) { return 4 * h + e + (e >= 4 ? 4 : 0); };
      // buffer loads: one per-lane byte offset (row pair / column pair of this lane half) and a
      // uniform byte offset per k slot in an SGPR -- no per-slot address registers live
      const unsigned lda = (unsigned)p.lda, ldb = (unsigned)p.ldb;
      const int va = (int)((4u * h * lda + (unsigned)am) * 4u);
      const int vb = (int)((4u * h * ldb + (unsigned)bc) * 4u);
      auto load = [&](int ks, f32x2 (&a)[8], f32x2 (&bv)[8]) {
        const int k0 = ks * 16;
        if (p.exp & 4) {  // timing experiment: no operand loads
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            a[e] = f32x2{1e-3f * e, 2e-3f};
            bv[e] = f32x2{3e-3f, 1e-3f * e};
          }
          return;
        }
        if (k0 + 16 <= p.K) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int ke = k0 + e + (e >= 4 ? 4 : 0);  // + 4h in the lane offset
            a[e] = __builtin_bit_cast(
                f32x2, __builtin_amdgcn_raw_buffer_load_b64(ra, va, (int)(ke * lda * 4u), 0));
            bv[e] = __builtin_bit_cast(
                f32x2, __builtin_amdgcn_raw_buffer_load_b64(rb, vb, (int)(ke * ldb * 4u), 0));
          }
        } else {  // K tail: slots past K read row K - 1 and are zeroed
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int k = k0 + kslot(e);
            const unsigned kc = (unsigned)min(k, p.K - 1);
            const f32x2 xa = *reinterpret_cast<const f32x2*>(p.A + (kc * lda + (unsigned)am));
            const f32x2 xb = *reinterpret_cast<const f32x2*>(p.B + (kc * ldb + (unsigned)bc));
            a[e] = k < p.K ? xa : f32x2{0.f, 0.f};
            bv[e] = k < p.K ? xb : f32x2{0.f, 0.f};
          }
        }
      };
      f32x16 acc[2][2];
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[f][g][r] = 0.f;
      const bool do_rs = tn == 0 && wn == 0 && (p.bopt.kind != 0 || p.rowsum != nullptr);
      // Native fp32 products: v_mfma_f32_32x32x2_f32 (exact f32, an fmaf chain per output) at
      // the f32 rate -- 256 MFMAs x 64 cycles per wave and tile, ~7 us at 2.4 GHz, under the
      // ~12 us the stream waves need for the tile's 256 KB of p / momentum at their HBM share:
      // the math stays off the critical path without any VALU split (the split-bf16 emulation
      // needs ~1200 VALU per wave and tile and 100 more VGPRs, and lost to its own latency here).
      // MFMA e of a 16-deep k-step takes k = k0 + 8 (e >> 2) + 4h + (e & 3) in lane half h:
      // gemm_f32_fast.hip's native-f32 order, so the result is bit-identical to it.
      auto step = [&](const f32x2 (&a)[8], const f32x2 (&bv)[8]) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e][0], bv[e][0], acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e][0], bv[e][1], acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e][1], bv[e][0], acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e][1], bv[e][1], acc[1][1], 0, 0, 0);
        }
      };
      // two k-steps of operands in registers: the next one in flight behind this one's MFMAs
      // (32 MFMAs x 64 cycles of cover for the L2 latency); one loop exit, so the accumulators
      // keep one register assignment
      f32x2 ax[8], bx[8], ay[8], by[8];
      if (nks > 0) load(0, ax, bx);
      if (nks > 1) load(1, ay, by);
      int ks = 0;
      for (; ks + 2 <= nks; ks += 2) {
        step(ax, bx);
        if (ks + 2 < nks) load(ks + 2, ax, bx);
        step(ay, by);
        if (ks + 3 < nks) load(ks + 3, ay, by);
      }
      if (ks < nks) step(ax, bx);

      if (do_rs) {
        // bias gradient: lane l of the two wn == 0 waves sums row m0 + wm * 64 + l over k in
        // order, from L2 (the persistent kernel's sequential order: bit-identical sums); only
        // the first column tile's workgroups do it, and the math waves have slack
        const int m = m0 + wm * 64 + lane;
        const unsigned mc = (unsigned)min(m, p.M - 1);
        float rs = 0.f;
        int k = 0;
        for (; k + 8 <= p.K; k += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = p.A[(unsigned)(k + u) * lda + mc];
#pragma unroll
          for (int u = 0; u < 8; ++u) rs += v[u];
        }
        for (; k < p.K; ++k) rs += p.A[(unsigned)k * lda + mc];
        if (m < p.M) {
          if (p.bopt.kind != 0) {
            // the bias's pointers, the weight's hyper-parameters (GemmF32Args::bias_opt)
            OptEpilogue o = p.opt;
            const OptEpilogue& bo = p.bopt;
            if constexpr (SGD) {
              load_hyper(o.sgd);
              float pe = bo.p[m];
              float bb = (o.sgd.momentum != 0.f && !o.sgd.first_step) ? bo.s0[m] : 0.f;
              sgd_elem(pe, rs, bb, o.sgd);
              bo.p[m] = pe;
              if (o.sgd.momentum != 0.f) bo.s0[m] = bb;
            } else {
              load_hyper(o.adam);
              float pe = bo.p[m], mm = bo.s0[m], vv = bo.s1[m];
              adam_elem(pe, rs, mm, vv, nullptr, o.adam);
              bo.p[m] = pe;
              bo.s0[m] = mm;
              bo.s1[m] = vv;
            }
          } else {
            float* d = p.rowsum + m;
            *d = (p.rowsum_beta != 0.f ? p.rowsum_beta * *d : 0.f) + rs;
          }
        }
      }

      // buffer i & 1 free again: the stream waves have released its previous use (tile i - 2)
      const int bf = i & 1, use = i >> 1;
      lds_wait(empty + bf, 4 * use);
      float* Gb = G + bf * kGFloats;
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int lr = wm * 64 + 2 * rl + f;
          *reinterpret_cast<f32x2*>(Gb + lr * kTN + wn * 64 + 2 * l31) =
              f32x2{acc[f][0][r], acc[f][1][r]};
        }
      lds_signal(full + bf);
    }
    return;
  }

  // -------------------------------------------------------------------- stream waves
  const int ts = threadIdx.x - 256;  // 0..255
  constexpr int IT = kTM * (kTN / 4) / 256;  // 16-B chunks per thread per tile (16)
  constexpr int BI = SGD ? 8 : 4;            // chunks per batch (one set of loads in flight)
  constexpr int NB = IT / BI;                // batches per tile
  static_assert(NB % 2 == 0, "batches alternate between two register sets");
  OptEpilogue o = p.opt;
  if constexpr (SGD) load_hyper(o.sgd);
  else load_hyper(o.adam);
  const bool mom_rd = SGD && o.sgd.momentum != 0.f && !o.sgd.first_step;
  const bool mom_wr = SGD && o.sgd.momentum != 0.f;
  constexpr int NS = SGD ? 2 : 3;  // state arrays streamed with p (SGD: p, momentum)

  // this thread's chunks of a tile: row (ts >> 5) + 8 * it, columns (ts & 31) * 4 .. + 3
  struct Tile {
    long base;  // element index of chunk 0
    int rows;   // chunks it < rows are inside the matrix (rows are whole: N % 4 == 0)
    bool col_ok;
  };
  auto tile_of = [&](int lid) -> Tile {
    const int tn = lid / p.tiles_m, tm = lid - tn * p.tiles_m;
    const int row = tm * kTM + (ts >> 5), col = tn * kTN + (ts & 31) * 4;
    Tile t;
    t.col_ok = col < p.N;
    t.rows = row < p.M ? min(IT, (p.M - row + 7) / 8) : 0;
    t.base = (long)min(row, p.M - 1) * p.ldc + min(col, p.N - 4);
    return t;
  };
  const long step8 = 8 * p.ldc;  // one chunk row further
  struct Set {
    f32x4 v[NS][BI];
  };
  auto issue = [&](const Tile& t, int bt, Set& s) {
#pragma unroll
    for (int u = 0; u < BI; ++u) {
      const int it = bt * BI + u;
      // out-of-range chunks re-read chunk 0 (discarded)
      const long q = t.base + (it < t.rows ? it * step8 : 0);
      s.v[0][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.p + q));
      if constexpr (SGD) {
        if (mom_rd) s.v[1][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s0 + q));
      } else {
        s.v[1][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s0 + q));
        s.v[2][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s1 + q));
      }
    }
  };
  auto update = [&](const Tile& t, int bt, Set& s, const float* Gb) {
    f32x4 gv[BI];
#pragma unroll
    for (int u = 0; u < BI; ++u) {
      const int e = (bt * BI + u) * 256 + ts;
      gv[u] = *reinterpret_cast<const f32x4*>(Gb + (e >> 5) * kTN + (e & 31) * 4);
    }
#pragma unroll
    for (int u = 0; u < BI; ++u) {
      const int it = bt * BI + u;
      if (!t.col_ok || it >= t.rows) continue;
      const long q = t.base + it * step8;
      const f32x4 g4 = gv[u];
      f32x4 pe = s.v[0][u];
      if constexpr (SGD) {
        f32x4 be = mom_rd ? s.v[1][u] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float pc = pe[c], bc = be[c];
          sgd_elem(pc, g4[c], bc, o.sgd);
          pe[c] = pc;
          be[c] = bc;
        }
        __builtin_nontemporal_store(pe, reinterpret_cast<f32x4*>(o.p + q));
        if (mom_wr) __builtin_nontemporal_store(be, reinterpret_cast<f32x4*>(o.s0 + q));
      } else {
        f32x4 me = s.v[1][u], ve = s.v[2][u];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float pc = pe[c], mc = me[c], vc = ve[c];
          adam_elem(pc, g4[c], mc, vc, nullptr, o.adam);
          pe[c] = pc;
          me[c] = mc;
          ve[c] = vc;
        }
        __builtin_nontemporal_store(pe, reinterpret_cast<f32x4*>(o.p + q));
        __builtin_nontemporal_store(me, reinterpret_cast<f32x4*>(o.s0 + q));
        __builtin_nontemporal_store(ve, reinterpret_cast<f32x4*>(o.s1 + q));
      }
    }
  };

  Set s0, s1;
  int i = 0;
  int lid = t0 + j0;
  const bool hbm = (p.exp & 2) == 0;
  Tile cur = tile_of(lid < t1 ? lid : t0);
  if (lid < t1 && hbm) issue(cur, 0, s0);
  for (; lid < t1; lid += per, ++i) {
    const int nxt = lid + per;
    const Tile tn = tile_of(nxt < t1 ? nxt : lid);
    if (hbm) issue(cur, 1, s1);
    // the math waves published tile i into buffer i & 1 (its use i >> 1)
    const int bf = i & 1;
    lds_wait(full + bf, 4 * ((i >> 1) + 1));
    const float* Gb = G + bf * kGFloats;
    if (!hbm) {
      lds_signal(empty + bf);
      cur = tn;
      continue;
    }
#pragma unroll
    for (int bt = 0; bt < NB; bt += 2) {
      update(cur, bt, s0, Gb);
      if (bt + 2 < NB) issue(cur, bt + 2, s0);
      else if (nxt < t1) issue(tn, 0, s0);  // the next tile's first batch: HBM stays busy
      update(cur, bt + 1, s1, Gb);
      if (bt + 3 < NB) issue(cur, bt + 3, s1);
    }
    lds_signal(empty + bf);  // buffer i & 1 read out (the math waves reuse it for tile i + 2)
    cur = tn;
  }
}

// off by default until it beats the persistent epilogue kernel in the whole step
// (profiles/r9/ws_kernel_r9*.md); TDP_WGRAD_WS=1 / wgrad_opt_set_enabled(True) turn it on
bool& ws_enabled() {
  static bool on = [] {
    const char* e = std::getenv("TDP_WGRAD_WS");
    return e && e[0] == '1';
  }();
  return on;
}

}  // namespace

void wgrad_opt_set_enabled(bool on) { ws_enabled() = on; }
bool wgrad_opt_enabled() { return ws_enabled(); }

bool wgrad_opt_ok(const GemmF32Args& a) {
  auto al = [](const void* q, int n) { return ((uintptr_t)q % n) == 0; };
  if (!ws_enabled()) return false;
  if (a.opt.kind != 1 && a.opt.kind != 2) return false;
  if (a.a_kcontig || a.b_kcontig || a.mask || a.gate || a.bias || a.relu || a.beta != 0.f)
    return false;
  if (a.opt.kind == 2 && (a.opt.adam.amsgrad || a.opt.s2)) return false;
  if (a.M < 4 || a.N < 4 || a.K < 1 || a.M % 4 || a.N % 4 || a.lda % 2 || a.ldb % 2 ||
      a.ldc % 4)
    return false;
  // buffer-load byte offsets are 32-bit
  if ((long)a.K * a.lda * 4 >= (1L << 31) || (long)a.K * a.ldb * 4 >= (1L << 31)) return false;
  if (!al(a.A, 8) || !al(a.B, 8) || !al(a.opt.p, 16) || (a.opt.s0 && !al(a.opt.s0, 16)) ||
      (a.opt.s1 && !al(a.opt.s1, 16)))
    return false;
  return true;
}

void wgrad_opt_run(const GemmF32Args& a, int num_cus, hipStream_t s) {
  if (!wgrad_opt_ok(a)) throw std::runtime_error("wgrad_opt: unsupported operands");
  WsParams p{};
  p.A = a.A; p.B = a.B;
  p.lda = a.lda; p.ldb = a.ldb; p.ldc = a.ldc;
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.tiles_m = ceil_div(a.M, kTM);
  p.tiles_n = ceil_div(a.N, kTN);
  p.opt = a.opt;
  const bool bias_upd = a.rowsum != nullptr && a.rowsum_beta == 0.f && a.bias_opt.kind != 0;
  p.bopt = bias_upd ? a.bias_opt : OptEpilogue{};
  p.rowsum = bias_upd ? nullptr : a.rowsum;
  p.rowsum_beta = a.rowsum_beta;
  static const int exp = [] {
    const char* e = std::getenv("TDP_WS_EXP");
    return e ? std::atoi(e) : 0;
  }();
  p.exp = exp;
  const int T = p.tiles_m * p.tiles_n;
  const int grid = std::max(1, std::min(num_cus, T));
  const size_t lds = (size_t)2 * kGFloats * 4 + 16;  // two G buffers + four counters
  if (a.opt.kind == 1) {
    static bool cfg = false;
    if (!cfg) {
      (void)hipFuncSetAttribute((const void*)wgrad_opt_kernel<1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      cfg = true;
    }
    hipLaunchKernelGGL(wgrad_opt_kernel<1>, dim3(grid), dim3(kWT), lds, s, p);
  } else {
    static bool cfg = false;
    if (!cfg) {
      (void)hipFuncSetAttribute((const void*)wgrad_opt_kernel<2>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      cfg = true;
    }
    hipLaunchKernelGGL(wgrad_opt_kernel<2>, dim3(grid), dim3(kWT), lds, s, p);
  }
}

}  // namespace tdp
