// Large-tile split-bf16 fp32 GEMM for gfx950: 256 x 256 output tile, 8 waves, one workgroup per CU.
//
// Why (profiles/micro/gemm_emu_pmc_r4.md): the fast kernel (gemm_f32_fast.hip,
// 128 x 128 tile, 4 waves of 64 x 64, two workgroups per CU) splits every fp32 fragment on the
// VALU once per wave that reads it: per 16-deep K step a wave splits 64 + 64 rows x 16 k for
// 4 x 6 MFMAs (1.33 split elements per MFMA; 8.2 VALU per MFMA measured, MFMA busy 49 %).
// Here a wave owns 128 x 64 outputs (4 x 2 MFMA tiles): 128 + 64 rows per 8 x 6 MFMAs (1.0 per
// MFMA), and the workgroup re-reads each operand half as often from L2 (256-wide panels):
//   * C = A . op(B): A [M][K] fp32 K-contiguous, B [N][K] (K-contiguous) or [K][N];
//   * 512 threads = 8 waves in 2 (rows) x 4 (cols); two waves per SIMD (<= 256 VGPR + AGPR);
//   * global -> LDS by global_load_lds_dwordx4 (4 + 4 x 1-KiB pieces per wave per K tile), two
//     64-KiB stages (128 KiB: one workgroup per CU), one `s_waitcnt vmcnt(0)` + raw barrier per
//     32-deep K tile -- the next tile's DMA lands behind the current tile's 2 x 8 x 6 MFMAs per
//     wave (6k cycles per SIMD, far above the DMA latency);
//   * K-contiguous images [256 rows][32 k] with the fast kernel's source-address swizzle
//     (chunk c of row r in slot c ^ ((r ^ r >> 3) & 7): conflict-free ds_read_b128);
//     MN-contiguous B [32 k][256 cols] read as float2 pairs (column tile g of a wave takes the
//     interleaved columns 2i + g);
//   * fragments use the fast kernel's k permutation (lane half h holds k = 16j + 4h + s and
//     16j + 8 + 4h + s of K16 step j, the same for A and B) and its exact three-term split with
//     the six kept products (split3 / mfma6 below: the same instruction sequence).
// Measured against the fast kernel: profiles/r9/gemm_emu8_r9.md.
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "emu8.h"

namespace tdp {
namespace {

constexpr int kBK8 = 32;
constexpr int kTile = 256;
constexpr int kImg = kTile * kBK8 * 4;  // 32 KiB per operand per stage
constexpr int kStage = 2 * kImg;
constexpr int kStages = 2;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef char lds_char;

struct E8Params {
  const float* A;
  const float* B;
  float* C;
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_n, tiles;
  float beta;
  const float* bias;  // optional [N]
  int relu;
};

__device__ __forceinline__ void split_pair8(float x0, float x1, unsigned& h, unsigned& m,
                                            unsigned& l) {
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x0, x1}, bf2));
  const float r0 = x0 - __uint_as_float(hu << 16), r1 = x1 - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf2));
  const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{s0, s1}, bf2));
}

struct Planes {
  bf8 h, m, l;
};

__device__ __forceinline__ Planes split8(const f32x4& x0, const f32x4& x1) {
  unsigned hs[4], ms[4], ls[4];
  split_pair8(x0[0], x0[1], hs[0], ms[0], ls[0]);
  split_pair8(x0[2], x0[3], hs[1], ms[1], ls[1]);
  split_pair8(x1[0], x1[1], hs[2], ms[2], ls[2]);
  split_pair8(x1[2], x1[3], hs[3], ms[3], ls[3]);
  Planes p;
  p.h = __builtin_bit_cast(bf8, u32x4{hs[0], hs[1], hs[2], hs[3]});
  p.m = __builtin_bit_cast(bf8, u32x4{ms[0], ms[1], ms[2], ms[3]});
  p.l = __builtin_bit_cast(bf8, u32x4{ls[0], ls[1], ls[2], ls[3]});
  return p;
}

__device__ __forceinline__ f32x16 mfma6x(const Planes& a, const Planes& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void glds(const float* src, lds_char* dst) {
  __builtin_amdgcn_global_load_lds(
      (const void*)src, (void __attribute__((address_space(3)))*)(
                            (__attribute__((address_space(3))) char*)dst), 16, 0, 0);
}

__device__ __forceinline__ int swz8(int row) { return (row ^ (row >> 3)) & 7; }

// NW = 8: waves 2 x 4, wave tile 128 x 64 (two waves per SIMD); NW = 4: waves 2 x 2, wave tile
// 128 x 128 (one wave per SIMD, 256 accumulator registers: 0.67 split elements per MFMA)
template <bool BKC, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void
gemm_emu8_kernel(E8Params p) {
  constexpr int WNC = kTile / (NW / 2);  // columns per wave
  constexpr int FN = WNC / 32;
  constexpr int NPW = 32 / NW;           // 1-KiB DMA pieces per wave per operand per K tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / (NW / 2), wn = wid % (NW / 2);
  const int h = lane >> 5, l31 = lane & 31;
  // XCD-aware bijective remap: consecutive logical tiles share an XCD (and its L2)
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  const int m0 = (lid / p.tiles_n) * kTile, n0 = (lid % p.tiles_n) * kTile;
  const int nk = p.K / kBK8;

  // DMA sources: piece j = NPW * wid + i of each operand's 32 1-KiB pieces per K tile
  const float* asrc[NPW];
  const float* bsrc[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int j = NPW * wid + i;
    const int row = j * 8 + (lane >> 3);
    const int gr = min(m0 + row, p.M - 1);
    asrc[i] = p.A + (long)gr * p.lda + ((lane & 7) ^ swz8(row)) * 4;
    if (BKC) {
      const int gc = min(n0 + row, p.N - 1);
      bsrc[i] = p.B + (long)gc * p.ldb + ((lane & 7) ^ swz8(row)) * 4;
    } else {
      const int gc = min(n0 + lane * 4, p.N - 4);
      bsrc[i] = p.B + (long)j * p.ldb + gc;  // k row j of the tile
    }
  }
  const long bstep = BKC ? kBK8 : (long)kBK8 * p.ldb;
  auto issue = [&](int kt) {
    lds_char* st = smem + (kt & 1) * kStage;
#pragma unroll
    for (int i = 0; i < NPW; ++i) glds(asrc[i] + (long)kt * kBK8, st + (NPW * wid + i) * 1024);
#pragma unroll
    for (int i = 0; i < NPW; ++i)
      glds(bsrc[i] + (long)kt * bstep, st + kImg + (NPW * wid + i) * 1024);
  };

  f32x16 acc[4][FN];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][g][r] = 0.f;

  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nk) issue(kt + 1);
    const lds_char* st = smem + (kt & 1) * kStage;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      Planes bp[FN];
      if (BKC) {
#pragma unroll
        for (int g = 0; g < FN; ++g) {
          const int row = wn * WNC + g * 32 + l31;
          const lds_char* rb = st + kImg + row * 128;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(rb + (((4 * j + h) ^ swz8(row)) * 16));
          const f32x4 v1 =
              *reinterpret_cast<const f32x4*>(rb + (((4 * j + 2 + h) ^ swz8(row)) * 16));
          bp[g] = split8(v0, v1);
        }
      } else {
        // column tile g takes the interleaved columns 2 i + (g & 1) of the wave's 64-column
        // group g >> 1: one float2 read feeds two tiles
#pragma unroll
        for (int pp = 0; pp < FN / 2; ++pp) {
          f32x4 x[2][2];
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int k = 16 * j + 8 * u + 4 * h + s;
              const f32x2 v = *reinterpret_cast<const f32x2*>(
                  st + kImg + k * 1024 + (wn * WNC + pp * 64 + 2 * l31) * 4);
              x[0][u][s] = v[0];
              x[1][u][s] = v[1];
            }
          bp[2 * pp] = split8(x[0][0], x[0][1]);
          bp[2 * pp + 1] = split8(x[1][0], x[1][1]);
        }
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int row = wm * 128 + f * 32 + l31;
        const lds_char* ra = st + row * 128;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ra + (((4 * j + h) ^ swz8(row)) * 16));
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ra + (((4 * j + 2 + h) ^ swz8(row)) * 16));
        const Planes ap = split8(v0, v1);
#pragma unroll
        for (int g = 0; g < FN; ++g) acc[f][g] = mfma6x(ap, bp[g], acc[f][g]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup

  // epilogue: lane (h, l31) of tile (f, g) holds rows (r & 3) + 8 (r >> 2) + 4 h, column l31
  // (MN-contiguous B: column 2 l31 + (g & 1) of the 64-column group g >> 1)
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g) {
      const int col =
          n0 + wn * WNC + (BKC ? g * 32 + l31 : (g >> 1) * 64 + 2 * l31 + (g & 1));
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < p.M) {
          float* c = p.C + (long)row * p.ldc + col;
          float v = acc[f][g][r] + (p.bias ? p.bias[col] : 0.f);
          if (p.beta != 0.f) v += p.beta * *c;
          *c = p.relu ? fmaxf(v, 0.f) : v;
        }
      }
    }
}

template <bool BKC, int NW>
void launch_e8(const E8Params& p, hipStream_t s) {
  const size_t lds = (size_t)kStages * kStage;
  static bool cfg = false;
  if (!cfg) {
    (void)hipFuncSetAttribute((const void*)gemm_emu8_kernel<BKC, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    cfg = true;
  }
  hipLaunchKernelGGL((gemm_emu8_kernel<BKC, NW>), dim3(p.tiles), dim3(NW * 64), lds, s, p);
}

int& e8_waves() {
  static int w = 8;
  return w;
}

}  // namespace

bool gemm_emu8_set_waves(int w) {
  if (w != 4 && w != 8) return false;
  e8_waves() = w;
  return true;
}

bool gemm_emu8_fits(int M, int N, int K, int num_cus) {
  if (K < 1024 || K % kBK8 || M < 2048 || N < 2048) return false;
  const long tiles = (long)ceil_div(M, kTile) * ceil_div(N, kTile);
  const long waves = (tiles + num_cus - 1) / num_cus;
  return tiles >= num_cus && tiles * 10 >= waves * num_cus * 9;  // >= 90 % of the last wave
}

bool gemm_emu8_ok(const GemmEmu8Args& a) {
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (a.M <= 0 || a.N < 4 || a.K < kBK8 || a.K % kBK8) return false;
  if (!al16(a.A) || !al16(a.B) || a.lda % 4 || a.ldb % 4) return false;
  if (!a.b_kcontig && a.N % 4) return false;
  return true;
}

void gemm_emu8_run(const GemmEmu8Args& a, hipStream_t s) {
  if (!gemm_emu8_ok(a)) throw std::runtime_error("gemm_emu8: unsupported shape / alignment");
  E8Params p;
  p.A = a.A;
  p.B = a.B;
  p.C = a.C;
  p.lda = a.lda;
  p.ldb = a.ldb;
  p.ldc = a.ldc;
  p.M = a.M;
  p.N = a.N;
  p.K = a.K;
  p.tiles_n = ceil_div(a.N, kTile);
  p.tiles = ceil_div(a.M, kTile) * p.tiles_n;
  p.beta = a.beta;
  p.bias = a.bias;
  p.relu = a.relu ? 1 : 0;
  const bool w4 = e8_waves() == 4;
  if (a.b_kcontig) w4 ? launch_e8<true, 4>(p, s) : launch_e8<true, 8>(p, s);
  else w4 ? launch_e8<false, 4>(p, s) : launch_e8<false, 8>(p, s);
}

}  // namespace tdp
