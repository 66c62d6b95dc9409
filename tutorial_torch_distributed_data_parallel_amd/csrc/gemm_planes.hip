// Skinny-M fp32 GEMM whose A operand arrives pre-split into three bf16 planes (gfx950).
//
// Why (profiles/micro/gemm_split_cost_exp_r5d.jsonl, gemm_emu_pmc_r4.md): the split-bf16 fast GEMM
// (gemm_f32_fast.hip) splits every fp32 fragment on the VALU inside the K loop, once per wave that
// reads it. For the toy-MLP's skinny GEMMs (M = batch = 128 rows against 4096-9216 columns and
// K = 4096-9216) the small operand A is re-read by every column tile -- 32 tiles x 2 column waves
// = 64 redundant splits of each activation -- while the weight B is streamed from HBM once. Here
// A is split ONCE (by its producer: the gather / split-K reduce / loss head, or split_planes) into
// exact bf16 hi / mid / lo planes x = x0 + x1 + x2 (csrc/gemm_f32_fast.hip split3_pair: the same
// RNE conversions, so the planes are bit-identical to the in-kernel split), and the kernel is
// laid out so that each weight fragment is split by exactly ONE wave:
//   * block tile 128 (all batch rows) x 128 columns, 4 waves side by side (1 x 4): wave w owns
//     columns 32w..32w+31 and all four 32-row MFMA tiles, so its one B fragment per 16-deep K step
//     feeds 4 x 6 v_mfma_f32_32x32x16_bf16 (the six kept split products, smallest first) and its
//     split (~36 VALU) hides under 24 MFMAs (the fast kernel's 2 x 2 waves split 4 fragments per
//     24 MFMAs);
//   * both operands go global -> LDS by global_load_lds_dwordx4 (no VGPR staging), 2 stages of
//     40 KiB (A planes 3 x 8 KiB + B 16 KiB), two workgroups per CU (80 KiB each, 160 KiB LDS);
//     one `s_waitcnt vmcnt(0)` + raw barrier per 32-deep K tile, the next tile's DMA in flight
//     behind the current tile's MFMAs;
//   * A plane rows are 64 B ([128 rows][32 k] bf16): 16-B chunk c of row r sits in slot
//     c ^ ((r >> 2) & 3), so the 16 lanes of a ds_read_b128 phase (rows r..r+15) hit all 64 banks;
//     K-contiguous B rows are 128 B with the fast kernel's (r ^ r >> 3) & 7 swizzle;
//     MN-contiguous B ([32 k][128 cols], the input gradient's W [out][in]) is read per column;
//   * split-K fills the chip (tiles x splits ~ 2 per CU); partial tiles go to a workspace combined
//     by planes_reduce_kernel, whose epilogue (bias, ReLU, C-shaped gate) can also emit the bf16
//     planes of the finished output for the NEXT skinny GEMM (fc1 forward -> fc2 forward).
// Numerics equal the fast kernel's split path (same six products of the same exact terms; only
// the fp32 summation order differs): tests/test_gemm_planes_gpu.py checks both against fp64.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "planes.h"

namespace tdp {
namespace {

constexpr int kT = 256;
constexpr int kBK = 32;
constexpr int kBM = 128, kBN = 128;
constexpr int kAPlane = kBM * kBK * 2;  // 8 KiB: [128 rows][32 k] bf16
constexpr int kABytes = 3 * kAPlane;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef char lds_char;

struct PParams {
  const uint16_t* Ap;
  long ps, lda;
  const float* B;
  long ldb;
  float* C;
  long ldc;
  float* ws;
  const float* bias;
  const float* gate;
  long ldg;
  uint16_t* op;  // optional planes of the finished C: [3][M][N], plane stride ops
  long ops;
  int relu;
  int M, N, K, kps, splits, tiles_n, tiles_mn;
  int prio;
};

// exact 3-way bf16 split of a pair (identical instruction sequence to gemm_f32_fast.hip
// split3_pair: RNE v_cvt_pk_bf16_f32, scalar f32 residuals)
__device__ __forceinline__ void split_pair(float x0, float x1, unsigned& h, unsigned& m,
                                           unsigned& l) {
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x0, x1}, bf2));
  const float r0 = x0 - __uint_as_float(hu << 16), r1 = x1 - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf2));
  const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{s0, s1}, bf2));
}

__device__ __forceinline__ void split_x8(const float (&x)[8], bf8& h, bf8& m, bf8& l) {
  unsigned hs[4], ms[4], ls[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split_pair(x[2 * i], x[2 * i + 1], hs[i], ms[i], ls[i]);
  h = __builtin_bit_cast(bf8, u32x4{hs[0], hs[1], hs[2], hs[3]});
  m = __builtin_bit_cast(bf8, u32x4{ms[0], ms[1], ms[2], ms[3]});
  l = __builtin_bit_cast(bf8, u32x4{ls[0], ls[1], ls[2], ls[3]});
}

// acc += a*b over the six kept split terms (smallest first; a1b2 + a2b1 + a2b2 dropped)
__device__ __forceinline__ f32x16 mfma6(const bf8& ah, const bf8& am, const bf8& al, const bf8& bh,
                                        const bf8& bm, const bf8& bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void glds16(const void* src, lds_char* dst) {
  __builtin_amdgcn_global_load_lds(
      src, (void __attribute__((address_space(3)))*)(
               (__attribute__((address_space(3))) char*)dst), 16, 0, 0);
}

__device__ __forceinline__ int aswz(int row) { return (row >> 2) & 3; }
__device__ __forceinline__ int bswz(int row) { return (row ^ (row >> 3)) & 7; }

// bias, ReLU, gate of four adjacent finished outputs, then C (16-B store) and, when requested,
// the three bf16 planes of the result (8-B stores); returns the stored value
__device__ __forceinline__ f32x4 finish4(const PParams& p, int row, int col, f32x4 v) {
  if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + col);
  if (p.relu) {
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
  }
  if (p.gate) {
    const f32x4 g = *reinterpret_cast<const f32x4*>(p.gate + (long)row * p.ldg + col);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = g[c] > 0.f ? v[c] : 0.f;
  }
  *reinterpret_cast<f32x4*>(p.C + (long)row * p.ldc + col) = v;
  if (p.op) {
    unsigned h0, m0, l0, h1, m1, l1;
    split_pair(v[0], v[1], h0, m0, l0);
    split_pair(v[2], v[3], h1, m1, l1);
    uint16_t* o = p.op + (long)row * p.N + col;
    *reinterpret_cast<u32x2*>(o) = u32x2{h0, h1};
    *reinterpret_cast<u32x2*>(o + p.ops) = u32x2{m0, m1};
    *reinterpret_cast<u32x2*>(o + 2 * p.ops) = u32x2{l0, l1};
  }
  return v;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// S pipeline stages; WN 32-column MFMA tiles per wave (block tile 128 x 128*WN: WN = 2 halves
// the A (L2) traffic per MFMA at 112 KiB of LDS, one workgroup per CU)
template <bool BKC, int S, int WN, int PF>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(S == 2 ? 2 : 1))) void gemm_planes_kernel(
    PParams p) {
  constexpr int BN = kBN * WN;
  constexpr int BBYTES = BN * kBK * 4;
  constexpr int STG = kABytes + BBYTES;
  constexpr int GB = BBYTES / 1024 / 4;  // B chunks per wave per tile
  constexpr int G = 6 + GB;              // LDS-DMA loads per wave per tile
  static_assert(PF == 0 || S == 2, "the B prefetch's counted waits assume two stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, l31 = lane & 31;
  // two workgroups share each SIMD running the same read / split / MFMA sequence; a static
  // priority for every other hardware slot keeps them out of lockstep
  if (p.prio && ((blockIdx.x >> 3) & 1)) __builtin_amdgcn_s_setprio(1);
  // XCD-aware order (bijective): hardware ids b and b + 8 share an XCD; each XCD takes a
  // contiguous range of logical tiles, split-major, so an XCD's workgroups share A's K slices
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  const int z = lid / p.tiles_mn, t = lid % p.tiles_mn;
  const int m0 = (t / p.tiles_n) * kBM, n0 = (t % p.tiles_n) * BN;
  const int kb = z * p.kps;
  const int ke = min(p.K, kb + p.kps);
  const int nk = (ke - kb) / kBK;  // K and kps are multiples of 32 (host-checked)

  // per-lane DMA sources: A = 24 1-KiB chunks (3 planes x 8 row blocks of 16 rows), 6 per wave;
  // B = BN/8 chunks, GB per wave. Out-of-range rows / columns are clamped (discarded outputs).
  const uint16_t* abase[6];
  int adst[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int j = w * 6 + i, plane = j >> 3, rb = j & 7;
    const int row = rb * 16 + (lane >> 2);
    const int gr = min(m0 + row, p.M - 1);
    const int c = (lane & 3) ^ aswz(row);
    abase[i] = p.Ap + plane * p.ps + (long)gr * p.lda + c * 8;
    adst[i] = plane * kAPlane + rb * 1024;
  }
  const float* bbase[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int j = w * GB + i;
    if (BKC) {  // [BN rows][32 k] fp32, 128-B rows, 8 rows per chunk
      const int row = j * 8 + (lane >> 3);
      const int gr = min(n0 + row, p.N - 1);
      bbase[i] = p.B + (long)gr * p.ldb + ((lane & 7) ^ bswz(row)) * 4;
    } else {    // [32 k][BN cols] fp32, BN*4-B rows, 1024 / (BN*4) rows per chunk
      constexpr int LPR = BN / 4, RPC = 1024 / (BN * 4);
      const int krow = RPC * j + lane / LPR;
      const int gc = min(n0 + (lane % LPR) * 4, p.N - 4);
      bbase[i] = p.B + (long)krow * p.ldb + gc;
    }
  }
  // tiles past the end are re-issued at the last tile (same addresses, a stage nobody reads):
  // every iteration then has the same loads in flight, so one counted vmcnt fits all
  auto issue = [&](int kt) {
    lds_char* st = smem + (kt % S) * STG;
    const int k0 = kb + min(kt, nk - 1) * kBK;
#pragma unroll
    for (int i = 0; i < 6; ++i) glds16(abase[i] + k0, st + adst[i]);
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const float* src = BKC ? bbase[i] + k0 : bbase[i] + (long)k0 * p.ldb;
      glds16(src, st + kABytes + (w * GB + i) * 1024);
    }
  };

  f32x16 acc[4][WN];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int g = 0; g < WN; ++g)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][g][r] = 0.f;

  // B prefetch into L2 (PF > 0, two stages only): one dword per 128-B line of the B tile PF
  // tiles beyond the one being DMA'd, so the HBM latency of B is paid PF tiles early and the
  // LDS-DMA hits L2. The load lands in a dummy VGPR that must stay allocated until the load has
  // completed: the counted wait two iterations later covers it (in-order vmcnt), so two dummies
  // alternate (d0 even iterations, d1 odd) and each is consumed (kept live) until then.
  auto prefetch = [&](int kt, float& d) {
    const int k0 = kb + min(kt, nk - 1) * kBK;
    const int line = w * 32 + l31;  // 128 lines of 128 B per B tile (lanes 32-63 duplicate)
    const float* src;
    if (BKC) src = p.B + (long)min(n0 + line, p.N - 1) * p.ldb + k0;
    else src = p.B + (long)(k0 + (line >> 2)) * p.ldb + min(n0 + (line & 3) * 32, p.N - 4);
    asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(src) : "memory");
  };
  // One 32-deep tile = two 16-deep MFMA steps. Software-pipelined by hand (the compiler's own
  // schedule re-used one register set and waited for every 3-fragment LDS read before each
  // group of 6 MFMAs): both steps' B fragments and step 0's A fragments are read up front, step
  // 1's A fragments are in flight while step 0's 24 MFMAs issue, and step 1's B split runs on
  // the VALU between them (1 MFMA : 2 VALU groups).
  auto read_b = [&](const lds_char* st, int s, float (&bv)[8]) {
    const int bcol = w * 32 + l31;
    if (BKC) {
      const int c0 = 4 * s + 2 * h;
      const f32x4 v0 =
          *reinterpret_cast<const f32x4*>(st + kABytes + bcol * 128 + ((c0 ^ bswz(bcol)) * 16));
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(st + kABytes + bcol * 128 +
                                                       (((c0 + 1) ^ bswz(bcol)) * 16));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bv[j] = v0[j];
        bv[4 + j] = v1[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bv[j] = *reinterpret_cast<const float*>(st + kABytes +
                                                ((16 * s + 8 * h + j) * BN + bcol) * 4);
    }
  };
  auto read_a = [&](const lds_char* st, int s, bf8 (&a)[4][3]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int row = f * 32 + l31;
      const int off = row * 64 + (((2 * s + h) ^ aswz(row)) * 16);
#pragma unroll
      for (int q = 0; q < 3; ++q) a[f][q] = *reinterpret_cast<const bf8*>(st + q * kAPlane + off);
    }
  };
  auto compute = [&](int kt) {
    static_assert(WN == 1, "the hand-pipelined step is written for 32 columns per wave");
    const lds_char* st = smem + (kt % S) * STG;
    float b0[8], b1[8];
    bf8 a0[4][3], a1[4][3];
    bf8 x0[3];
    unsigned h1[4], m1[4], l1[4];
    // B of both steps and half of step 0's A, then step 0's B split (a counted lgkmcnt: at most
    // 15 reads may be outstanding), then the rest of step 0's A
    read_b(st, 0, b0);
    read_b(st, 1, b1);
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int row = f * 32 + l31;
        a0[f][q] = *reinterpret_cast<const bf8*>(st + q * kAPlane + row * 64 +
                                                 ((h ^ aswz(row)) * 16));
      }
    __builtin_amdgcn_sched_barrier(0);
    split_x8(b0, x0[0], x0[1], x0[2]);
#pragma unroll
    for (int f = 2; f < 4; ++f)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int row = f * 32 + l31;
        a0[f][q] = *reinterpret_cast<const bf8*>(st + q * kAPlane + row * 64 +
                                                 ((h ^ aswz(row)) * 16));
      }
    __builtin_amdgcn_sched_barrier(0);
    // step 0: row tile f's six MFMAs, then step 1's A reads of tile f and a quarter of step 1's
    // B split (in-order LDS returns keep every wait a counted lgkmcnt <= 9)
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      acc[f][0] = mfma6(a0[f][0], a0[f][1], a0[f][2], x0[0], x0[1], x0[2], acc[f][0]);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int row = f * 32 + l31;
        a1[f][q] = *reinterpret_cast<const bf8*>(st + q * kAPlane + row * 64 +
                                                 (((2 + h) ^ aswz(row)) * 16));
      }
      split_pair(b1[2 * f], b1[2 * f + 1], h1[f], m1[f], l1[f]);
      __builtin_amdgcn_sched_barrier(0);
    }
    const bf8 y0 = __builtin_bit_cast(bf8, u32x4{h1[0], h1[1], h1[2], h1[3]});
    const bf8 y1 = __builtin_bit_cast(bf8, u32x4{m1[0], m1[1], m1[2], m1[3]});
    const bf8 y2 = __builtin_bit_cast(bf8, u32x4{l1[0], l1[1], l1[2], l1[3]});
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f][0] = mfma6(a1[f][0], a1[f][1], a1[f][2], y0, y1, y2, acc[f][0]);
  };
  if constexpr (S == 3) {
    // Cross-tile pipeline (three stages, one workgroup = one wave per SIMD): a tile's B fragments
    // and step-0 A fragments are read -- and its step-0 B split done -- while the PREVIOUS tile's
    // step-1 MFMAs issue, so the matrix pipe never waits for a tile's first LDS reads or split.
    // The wait + barrier sits between a tile's two MFMA steps: tile kt+1 has landed there (its
    // DMA was issued two half-iterations earlier) and tile kt's stage is free for tile kt+3.
    float b0[8], b1[8];
    bf8 a0[4][3], a1[4][3], x0[3];
    auto read_a = [&](const lds_char* st, int s, int f, bf8 (&a)[4][3]) {
      const int row = f * 32 + l31;
      const int off = row * 64 + (((2 * s + h) ^ aswz(row)) * 16);
#pragma unroll
      for (int q = 0; q < 3; ++q) a[f][q] = *reinterpret_cast<const bf8*>(st + q * kAPlane + off);
    };
    if (nk > 0) {
      issue(0);
      issue(1);
      issue(2);
      wait_vmcnt<2 * G>();
      __builtin_amdgcn_s_barrier();
      read_b(smem, 0, b0);
      read_b(smem, 1, b1);
      read_a(smem, 0, 0, a0);
      read_a(smem, 0, 1, a0);
      __builtin_amdgcn_sched_barrier(0);
      split_x8(b0, x0[0], x0[1], x0[2]);
      read_a(smem, 0, 2, a0);
      read_a(smem, 0, 3, a0);
    }
    // One tile, its stage index a compile-time constant (the loop is unrolled by the 3 stages:
    // LDS offsets become immediates and no kt % 3 is computed). Each half-tile is ONE scheduling
    // region whose MFMAs are interleaved with its LDS reads and split VALU by explicit
    // sched_group_barrier patterns (left alone, the compiler issued the 36-VALU splits as blocks
    // between MFMA runs, where no MFMA was in flight).
    // every earlier LDS read into these registers has returned (they were issued a half-tile of
    // MFMAs ago): one wait here instead of the compiler's lgkmcnt(0) in the middle of the region
    auto settle = [&]() {
#pragma unroll
      for (int f = 0; f < 4; ++f)
        asm volatile("" ::"v"(a0[f][0]), "v"(a0[f][1]), "v"(a0[f][2]));
      asm volatile("" ::"v"(x0[0]), "v"(x0[1]), "v"(x0[2]));
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(b1[j]));
    };
    auto tile = [&](int kt, auto stage_tag) {
      constexpr int SG = decltype(stage_tag)::value;
      const lds_char* st = smem + SG * STG;
      const lds_char* sn = smem + ((SG + 1) % 3) * STG;
      unsigned h1[4], m1[4], l1[4];
      settle();
      __builtin_amdgcn_sched_barrier(0);
      // step 0 of tile kt (24 MFMAs); step-1 A reads (12) and the step-1 B split (~36 VALU)
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        acc[f][0] = mfma6(a0[f][0], a0[f][1], a0[f][2], x0[0], x0[1], x0[2], acc[f][0]);
        read_a(st, 1, f, a1);
        split_pair(b1[2 * f], b1[2 * f + 1], h1[f], m1[f], l1[f]);
      }
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
      __builtin_amdgcn_sched_barrier(0);
      const bf8 y0 = __builtin_bit_cast(bf8, u32x4{h1[0], h1[1], h1[2], h1[3]});
      const bf8 y1 = __builtin_bit_cast(bf8, u32x4{m1[0], m1[1], m1[2], m1[3]});
      const bf8 y2 = __builtin_bit_cast(bf8, u32x4{l1[0], l1[1], l1[2], l1[3]});
      // tile kt+1 landed (tile kt+2 may still be in flight); every wave's reads of tile kt done
      wait_vmcnt<G>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int f = 0; f < 4; ++f)  // drained above: keeps the compiler's own wait off the MFMAs
        asm volatile("" ::"v"(a1[f][0]), "v"(a1[f][1]), "v"(a1[f][2]));
      __builtin_amdgcn_sched_barrier(0);
      // step 1 of tile kt (24 MFMAs) with: tile kt+1's B reads (4) first, the DMA of tile kt+3
      // into stage SG (10, every wave has finished reading tile kt), tile kt+1's step-0 A reads
      // (12), then its step-0 B split (~36 VALU) once the B reads have returned
      read_b(sn, 0, b0);
      read_b(sn, 1, b1);
      acc[0][0] = mfma6(a1[0][0], a1[0][1], a1[0][2], y0, y1, y2, acc[0][0]);
      read_a(sn, 0, 0, a0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      __builtin_amdgcn_sched_barrier(0);
      issue(kt + 3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 1; f < 4; ++f) {
        acc[f][0] = mfma6(a1[f][0], a1[f][1], a1[f][2], y0, y1, y2, acc[f][0]);
        read_a(sn, 0, f, a0);
      }
      split_x8(b0, x0[0], x0[1], x0[2]);
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    for (int kt = 0; kt < nk; kt += 3) {
      tile(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nk) tile(kt + 1, std::integral_constant<int, 1>{});
      if (kt + 2 < nk) tile(kt + 2, std::integral_constant<int, 2>{});
    }
  } else {
  float d0 = 0.f, d1 = 0.f;
  auto step = [&](int kt, float& d) {
    // tile kt has landed when at most the S - 2 younger tiles' loads (and the newest prefetch)
    // are still in flight
    if constexpr (PF > 0) {
      wait_vmcnt<1>();
      asm volatile("" ::"v"(d));  // the prefetch of two iterations ago has completed
    } else {
      wait_vmcnt<(S - 2) * G>();
    }
    // every LDS read of the stage the next DMA overwrites has returned (the scheduler may sink
    // the MFMAs that consume the last reads below the barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(kt + S - 1);
    if constexpr (PF > 0) prefetch(kt + S - 1 + PF, d);
    compute(kt);
  };
  if (nk > 0) {
#pragma unroll
    for (int t = 0; t < S - 1; ++t) issue(t);
    if constexpr (PF > 0) prefetch(S - 1 + PF - 1, d1);
  }
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, d0);
    step(kt + 1, d1);
  }
  if (kt < nk) step(kt, d0);
  asm volatile("" ::"v"(d0), "v"(d1));
  }

  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup
  // Epilogue through LDS (the stages are free once every wave has left the K loop): the MFMA
  // layout gives a lane one column of 16 rows -- dword stores, and the store tail of 512
  // workgroups writing 64 KiB each was issue-bound (18 us of a 57-us fc1 forward with the K loop
  // emptied, TDP_PLANES_EXP=7). Staged, every thread stores 16-B row segments: a partial tile to
  // the workspace, or the finished tile (bias / ReLU / gate / planes).
  static_assert(WN == 1 && kBM * (BN + 4) * 4 <= S * STG, "the C tile must fit in the stages");
  constexpr int TS = BN + 4;  // padded LDS row (floats)
  float* T = reinterpret_cast<float*>(smem);
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      T[(f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * TS + w * 32 + l31] = acc[f][0][r];
  __syncthreads();
  constexpr int C4 = BN / 4;             // float4 per tile row
  constexpr int IT = kBM * C4 / kT;      // float4 per thread
  float* ws = p.ws + (long)z * p.M * p.N;
#pragma unroll 4
  for (int i = 0; i < IT; ++i) {
    const int e = i * kT + threadIdx.x;
    const int lr = e / C4, lc = (e % C4) * 4;
    const int row = m0 + lr, col = n0 + lc;
    if (row >= p.M || col >= p.N) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + lr * TS + lc);
    if (p.splits > 1) *reinterpret_cast<f32x4*>(ws + (long)row * p.N + col) = v;
    else finish4(p, row, col, v);
  }
}

// Two waves per SIMD (gemm_planes_set_cfg stages = 4): the same tile, LDS image and three stages
// as the S = 3 kernel, but 512 threads -- wave group q = wave >> 2 computes MFMA step q (k 16q ..
// 16q + 15) of every 32-deep K tile into its own accumulators; the groups are summed through LDS
// at the end. The single-group kernel keeps one wave per SIMD behind its own LDS reads, split and
// MFMA issue (52 % of wave cycles waiting on dependencies, MFMA busy 37 %:
// profiles/r8/mlp_dp1_pmc_r8m.md); here each SIMD has a second wave to issue from while one
// waits (profiles/r9/planes_dual_r9.md). Registers: the S = 3 kernel's 234 fit two waves' 256.
template <bool BKC>
__global__ __launch_bounds__(2 * kT) __attribute__((amdgpu_waves_per_eu(2, 2))) void
gemm_planes_dual_kernel(PParams p) {
  constexpr int S = 3;
  constexpr int BN = kBN;
  constexpr int BBYTES = BN * kBK * 4;
  constexpr int STG = kABytes + BBYTES;
  constexpr int NCH = kABytes / 1024 + BBYTES / 1024;  // 1-KiB DMA chunks per stage (40)
  constexpr int GW = NCH / 8;                          // per wave (5)
  static_assert(NCH % 8 == 0, "chunks split evenly over the 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = wave >> 2, w = wave & 3;  // MFMA step, column slice
  const int h = lane >> 5, l31 = lane & 31;
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  const int z = lid / p.tiles_mn, t = lid % p.tiles_mn;
  const int m0 = (t / p.tiles_n) * kBM, n0 = (t % p.tiles_n) * BN;
  const int kb = z * p.kps;
  const int ke = min(p.K, kb + p.kps);
  const int nk = (ke - kb) / kBK;

  // per-lane DMA sources: chunk j = wave * GW + i; chunks 0-23 are A (plane j >> 3, row block
  // j & 7), 24-39 are B (8 rows of 128 B, K-contiguous; or 1 KiB of [32 k][BN] rows)
  const char* src[GW];
  int dst[GW];
  long kbytes[GW];  // source bytes per unit of k
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int j = wave * GW + i;
    if (j < 24) {
      const int plane = j >> 3, rb = j & 7;
      const int row = rb * 16 + (lane >> 2);
      const int gr = min(m0 + row, p.M - 1);
      const int c = (lane & 3) ^ aswz(row);
      src[i] = reinterpret_cast<const char*>(p.Ap + plane * p.ps + (long)gr * p.lda + c * 8);
      dst[i] = plane * kAPlane + rb * 1024;
      kbytes[i] = 2;
    } else {
      const int jb = j - 24;
      if (BKC) {
        const int row = jb * 8 + (lane >> 3);
        const int gr = min(n0 + row, p.N - 1);
        src[i] = reinterpret_cast<const char*>(p.B + (long)gr * p.ldb +
                                               ((lane & 7) ^ bswz(row)) * 4);
        kbytes[i] = 4;
      } else {
        constexpr int LPR = BN / 4, RPC = 1024 / (BN * 4);
        const int krow = RPC * jb + lane / LPR;
        const int gc = min(n0 + (lane % LPR) * 4, p.N - 4);
        src[i] = reinterpret_cast<const char*>(p.B + (long)krow * p.ldb + gc);
        kbytes[i] = 4 * p.ldb;
      }
      dst[i] = kABytes + jb * 1024;
    }
  }
  auto issue = [&](int kt) {
    lds_char* st = smem + (kt % S) * STG;
    const long k0 = kb + min(kt, nk - 1) * kBK;
#pragma unroll
    for (int i = 0; i < GW; ++i) glds16(src[i] + k0 * kbytes[i], st + dst[i]);
  };

  f32x16 acc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[f][r] = 0.f;

  auto compute = [&](int kt) {
    const lds_char* st = smem + (kt % S) * STG;
    float bv[8];
    const int bcol = w * 32 + l31;
    if (BKC) {
      const int c0 = 4 * q + 2 * h;
      const f32x4 v0 =
          *reinterpret_cast<const f32x4*>(st + kABytes + bcol * 128 + ((c0 ^ bswz(bcol)) * 16));
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(st + kABytes + bcol * 128 +
                                                       (((c0 + 1) ^ bswz(bcol)) * 16));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bv[j] = v0[j];
        bv[4 + j] = v1[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bv[j] = *reinterpret_cast<const float*>(st + kABytes +
                                                ((16 * q + 8 * h + j) * BN + bcol) * 4);
    }
    bf8 a[4][3];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int row = f * 32 + l31;
      const int off = row * 64 + (((2 * q + h) ^ aswz(row)) * 16);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[f][pl] = *reinterpret_cast<const bf8*>(st + pl * kAPlane + off);
    }
    bf8 x0, x1, x2;
    split_x8(bv, x0, x1, x2);
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] = mfma6(a[f][0], a[f][1], a[f][2], x0, x1, x2, acc[f]);
  };

  if (nk > 0) {
#pragma unroll
    for (int t0 = 0; t0 < S - 1; ++t0) issue(t0);
  }
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt<(S - 2) * GW>();  // tile kt landed (tile kt + 1 may still be in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the stage refilled below
    __builtin_amdgcn_s_barrier();
    issue(kt + S - 1);
    compute(kt);
  }
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  // sum the two groups' accumulators, then the S = 3 kernel's LDS-staged epilogue (512 threads)
  constexpr int TS = BN + 4;
  static_assert(kBM * TS * 4 <= S * STG, "the C tile must fit in the stages");
  float* T = reinterpret_cast<float*>(smem);
  __syncthreads();
  if (q == 1) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        T[(f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * TS + w * 32 + l31] = acc[f][r];
  }
  __syncthreads();
  if (q == 0) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* e = T + (f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * TS + w * 32 + l31;
        *e = acc[f][r] + *e;
      }
  }
  __syncthreads();
  constexpr int C4 = BN / 4;
  constexpr int IT = kBM * C4 / (2 * kT);
  float* ws = p.ws + (long)z * p.M * p.N;
#pragma unroll 4
  for (int i = 0; i < IT; ++i) {
    const int e = i * 2 * kT + threadIdx.x;
    const int lr = e / C4, lc = (e % C4) * 4;
    const int row = m0 + lr, col = n0 + lc;
    if (row >= p.M || col >= p.N) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + lr * TS + lc);
    if (p.splits > 1) *reinterpret_cast<f32x4*>(ws + (long)row * p.N + col) = v;
    else finish4(p, row, col, v);
  }
}

// C = epilogue(sum_z ws[z]) over [M][N] (N % 4 == 0), four adjacent outputs per thread
__global__ __launch_bounds__(kT) void planes_reduce_kernel(PParams p) {
  const long ng = (long)p.M * p.N / 4;
  const long idx = (long)blockIdx.x * kT + threadIdx.x;
  if (idx >= ng) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(p.ws) + idx;
  f32x4 a = src[0];
#pragma unroll 4
  for (int z = 1; z < p.splits; ++z) a += src[z * ng];
  const long e0 = idx * 4;
  const int row = (int)(e0 / p.N), col = (int)(e0 - (long)row * p.N);
  finish4(p, row, col, a);
}


// x [rows][cols] (row stride ldx) -> planes [3][rows][cols] (plane stride ps), cols % 4 == 0
__global__ __launch_bounds__(kT) void split_planes_kernel(const float* __restrict__ x, long ldx,
                                                          int rows, int cols, uint16_t* planes,
                                                          long ps) {
  const long ng = (long)rows * cols / 4;
  for (long idx = (long)blockIdx.x * kT + threadIdx.x; idx < ng; idx += (long)gridDim.x * kT) {
    const long e0 = idx * 4;
    const int row = (int)(e0 / cols), col = (int)(e0 - (long)row * cols);
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + (long)row * ldx + col);
    unsigned h0, m0, l0, h1, m1, l1;
    split_pair(v[0], v[1], h0, m0, l0);
    split_pair(v[2], v[3], h1, m1, l1);
    uint16_t* o = planes + (long)row * cols + col;
    *reinterpret_cast<u32x2*>(o) = u32x2{h0, h1};
    *reinterpret_cast<u32x2*>(o + ps) = u32x2{m0, m1};
    *reinterpret_cast<u32x2*>(o + 2 * ps) = u32x2{l0, l1};
  }
}

// gather_batch_kernel (elementwise.hip) + the planes of every gathered float4: the toy-MLP's
// first Linear reads its input batch as planes without a separate split pass
__global__ __launch_bounds__(kT) void gather_planes_kernel(const float* __restrict__ x,
                                                           const int64_t* __restrict__ y,
                                                           const int64_t* __restrict__ idx, long n,
                                                           long F, float* __restrict__ xb,
                                                           int64_t* __restrict__ yb,
                                                           uint16_t* __restrict__ planes,
                                                           long ps, int64_t* cursor,
                                                           long nidx) {
  const int b = blockIdx.x;
  // cursor form (a captured step): the batch is idx[cursor[0] + b] and the workgroup that
  // finishes last advances cursor[0] by B (cursor[1] counts arrivals), so every replay of the
  // same graph reads the next batch of the epoch's order with no per-step index copy
  const int64_t base = cursor ? cursor[0] : 0;
  long k = base + b;
  k = k < 0 ? 0 : (k >= nidx ? nidx - 1 : k);  // a cursor past the order reads its last entry
  long i = idx[k];
  i = i < 0 ? 0 : (i >= n ? n - 1 : i);  // indices checked on the host; clamped so none faults
  const f32x4* src = reinterpret_cast<const f32x4*>(x + i * F);
  f32x4* dst = reinterpret_cast<f32x4*>(xb + (long)b * F);
  uint16_t* o = planes + (long)b * F;
  const long F4 = F >> 2, step = (long)kT * gridDim.y;
  for (long k = threadIdx.x + (long)kT * blockIdx.y; k < F4; k += step) {
    const f32x4 v = src[k];
    dst[k] = v;
    unsigned h0, m0, l0, h1, m1, l1;
    split_pair(v[0], v[1], h0, m0, l0);
    split_pair(v[2], v[3], h1, m1, l1);
    *reinterpret_cast<u32x2*>(o + 4 * k) = u32x2{h0, h1};
    *reinterpret_cast<u32x2*>(o + ps + 4 * k) = u32x2{m0, m1};
    *reinterpret_cast<u32x2*>(o + 2 * ps + 4 * k) = u32x2{l0, l1};
  }
  if (threadIdx.x == 0 && blockIdx.y == 0) yb[b] = y[i];
  if (cursor) {
    __syncthreads();  // every lane of this workgroup has read cursor[0]
    if (threadIdx.x == 0) {
      unsigned long long* c = reinterpret_cast<unsigned long long*>(cursor);
      // two-level arrivals: a row's slices count on the row's own counter (distinct addresses),
      // the row's last slice on the shared one -- B same-address atomics per launch, not B x
      // slices (serialised: 17.6 vs 7.3 us for 8 x 128 arrivals on one counter)
      bool row_done = true;
      if (gridDim.y > 1) {
        row_done = atomicAdd(c + 2 + b, 1ull) == (unsigned long long)gridDim.y - 1;
        if (row_done) atomicExch(c + 2 + b, 0ull);
      }
      // last arrival: every workgroup of the launch has read the position
      if (row_done && atomicAdd(c + 1, 1ull) == (unsigned long long)gridDim.x - 1) {
        atomicAdd(c, (unsigned long long)gridDim.x);
        atomicExch(c + 1, 0ull);
      }
    }
  }
}

inline bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

// variant: pipeline depth (2 stages: 80 KiB, two workgroups per CU; 3: 120 KiB, one; 4: the
// 3-stage image computed by two wave groups, gemm_planes_dual_kernel) and the B prefetch distance
// in tiles (0 = off; two stages only), set by gemm_planes_set_cfg (measurements; with a split-K
// override). One workgroup per CU halves the split-K count (8 for the toy MLP), hence the
// partial-sum traffic of the reduce; the captured toy-MLP step measured 0.371-0.374 ms with 3,0
// vs 0.383-0.386 with 2,0 (profiles/r6/bench_modes_r6j.txt). Default 4,0: 0.3624-0.3637 ms vs
// 0.3657-0.3677 with 3,0, interleaved on one box (profiles/r9/planes_dual_r9k.md). The B
// prefetch measured nothing (the K loop is not HBM-latency bound: TDP_PLANES_EXP experiments,
// profiles/r6/planes_gemm_experiments.md)
struct PlanesCfg {
  int stages, pf, splits;  // splits > 0: split-K override
};
PlanesCfg& planes_cfg() {
  static PlanesCfg c{4, 0, 0};
  return c;
}
}  // namespace

bool gemm_planes_set_cfg(int stages, int pf, int splits) {
  // stages 4 = the two-waves-per-SIMD kernel (gemm_planes_dual_kernel: 3 stages, 512 threads)
  if (!((stages >= 2 && stages <= 4) && pf >= 0 && pf <= 4 && (stages == 2 || pf == 0) &&
        splits >= 0))
    return false;
  planes_cfg() = {stages, pf, splits};
  return true;
}

namespace {

template <bool BKC, int S, int PF>
void launch_planes(const PParams& p, int nblocks, hipStream_t s) {
  const size_t lds = (size_t)S * (kABytes + kBN * kBK * 4);
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)gemm_planes_kernel<BKC, S, 1, PF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL((gemm_planes_kernel<BKC, S, 1, PF>), dim3(nblocks), dim3(kT), lds, s, p);
}

template <bool BKC>
void launch_dual(const PParams& p, int nblocks, hipStream_t s) {
  const size_t lds = (size_t)3 * (kABytes + kBN * kBK * 4);
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)gemm_planes_dual_kernel<BKC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL((gemm_planes_dual_kernel<BKC>), dim3(nblocks), dim3(2 * kT), lds, s, p);
}

template <bool BKC>
void launch_cfg(const PParams& p, const PlanesCfg& c, int nblocks, hipStream_t s) {
  if (c.stages == 4) launch_dual<BKC>(p, nblocks, s);
  else if (c.stages == 3) launch_planes<BKC, 3, 0>(p, nblocks, s);
  else if (c.pf == 1) launch_planes<BKC, 2, 1>(p, nblocks, s);
  else if (c.pf == 2) launch_planes<BKC, 2, 2>(p, nblocks, s);
  else if (c.pf >= 3) launch_planes<BKC, 2, 3>(p, nblocks, s);
  else launch_planes<BKC, 2, 0>(p, nblocks, s);
}

}  // namespace

void gather_batch_planes(const float* x, const int64_t* y, const int64_t* idx, long n, long F,
                         int B, float* xb, int64_t* yb, uint16_t* planes, hipStream_t s,
                         int64_t* cursor, long nidx, bool row_counters) {
  if (F % 4 || !al16(x) || !al16(xb) || ((uintptr_t)planes & 7))
    throw std::runtime_error("gather_batch_planes: F % 4 == 0 and aligned buffers required");
  if (B <= 0) return;
  // row slices: B = 128 rows alone would leave half of the 256 CUs idle
  const long F4 = F / 4;
  // cursor form: several slices per row only with per-row arrival counters (see the kernel)
  const int slices = (cursor && !row_counters)
                         ? 1
                         : (int)std::max<long>(1, std::min<long>(8, (F4 + kT - 1) / kT));
  hipLaunchKernelGGL(gather_planes_kernel, dim3(B, slices), dim3(kT), 0, s, x, y, idx, n, F, xb,
                     yb, planes, (long)B * F, cursor, cursor ? nidx : (long)B);
}

bool gemm_planes_ok(const GemmPlanesArgs& a) {
  if (a.M <= 0 || a.N < 4 || a.K < kBK || a.K % kBK) return false;
  if (!al16(a.Ap) || a.lda % 8 || a.ps % 8 || !al16(a.B) || a.ldb % 4) return false;
  if (a.N % 4 || a.ldc % 4 || !al16(a.C)) return false;
  if (a.bias && !al16(a.bias)) return false;
  if (a.gate && (!al16(a.gate) || a.ldgate % 4)) return false;
  if (a.out_planes && (((uintptr_t)a.out_planes & 7) || a.out_ps % 4)) return false;
  return true;
}

GemmPlan gemm_planes_plan(const GemmPlanesArgs& a, int num_cus) {
  GemmPlan plan;
  plan.fast = true;
  plan.bm = kBM;
  const PlanesCfg cfg = planes_cfg();
  plan.bn = kBN;
  plan.stages = cfg.stages;
  const long tiles = (long)ceil_div(a.M, kBM) * ceil_div(a.N, plan.bn);
  // two workgroups per CU when both fit (2 stages), else one
  const long target = (cfg.stages == 2 ? 2L : 1L) * num_cus;
  int splits = 1;
  if (cfg.splits > 0) {
    splits = cfg.splits;
  } else if (tiles < target) {
    const int want = (int)((target + tiles - 1) / tiles);
    const int kmax = a.K / (kBK * 4);  // >= 4 K tiles per split
    splits = want < kmax ? want : kmax;
    if (splits < 1) splits = 1;
  }
  const int kps = ceil_div(ceil_div(a.K, splits), kBK) * kBK;
  plan.k_per_split = kps;
  plan.splits = ceil_div(a.K, kps);
  plan.ws_floats = plan.splits > 1 ? (long)plan.splits * a.M * a.N : 0;
  return plan;
}

void gemm_planes_run(const GemmPlanesArgs& a, const GemmPlan& plan, float* ws, hipStream_t s) {
  if (!gemm_planes_ok(a)) throw std::runtime_error("gemm_planes: unsupported operands");
  PParams p{};
  p.Ap = a.Ap; p.ps = a.ps; p.lda = a.lda;
  p.B = a.B; p.ldb = a.ldb;
  p.C = a.C; p.ldc = a.ldc;
  p.ws = ws;
  p.bias = a.bias; p.gate = a.gate; p.ldg = a.ldgate;
  p.op = a.out_planes; p.ops = a.out_ps;
  p.relu = a.relu ? 1 : 0;
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.prio = 1;
  p.kps = plan.k_per_split;
  p.splits = plan.splits;
  p.tiles_n = ceil_div(a.N, plan.bn);
  p.tiles_mn = ceil_div(a.M, kBM) * p.tiles_n;
  if (plan.splits > 1 && ws == nullptr) throw std::runtime_error("gemm_planes: workspace missing");
  const int nblocks = p.tiles_mn * plan.splits;
  if (a.b_kcontig) launch_cfg<true>(p, planes_cfg(), nblocks, s);
  else launch_cfg<false>(p, planes_cfg(), nblocks, s);
  if (plan.splits > 1) {
    const long ng = (long)a.M * a.N / 4;
    hipLaunchKernelGGL(planes_reduce_kernel, dim3((unsigned)((ng + kT - 1) / kT)), dim3(kT), 0, s,
                       p);
  }
}

void split_planes(const float* x, long ldx, int rows, int cols, uint16_t* planes, long ps,
                  hipStream_t s) {
  if (cols % 4 || ldx % 4 || !al16(x) || ((uintptr_t)planes & 7) || ps % 4)
    throw std::runtime_error("split_planes: needs cols % 4 == 0 and aligned rows");
  const long ng = (long)rows * cols / 4;
  if (ng <= 0) return;
  const unsigned grid = (unsigned)std::min<long>((ng + kT - 1) / kT, 8192);
  hipLaunchKernelGGL(split_planes_kernel, dim3(grid), dim3(kT), 0, s, x, ldx, rows, cols, planes,
                     ps);
}

}  // namespace tdp
