// fp32 GEMM from pre-split bf16 planes (gfx950): C[M][N] = A[M][K] . B[N][K]^T.
//
// gemm_f32_fast.hip splits every fp32 fragment into three bf16 terms on the VALU inside the K
// loop (x = x0 + x1 + x2 exactly, RNE; six of the nine products kept: fp32 accuracy). Where an
// operand is re-read by many output tiles -- square and large GEMMs, the factored weight
// gradient of W ranks (depth W*B) -- that split is repeated by every tile that reads it: the
// fast kernel measured VALU-bound at ~49 % MFMA busy (profiles/micro/gemm_emu_pmc_r4.md), and
// even with the split removed its fp32 LDS pipeline reaches only ~224 TF/s at 4096^3
// (profiles/micro/gemm_split_cost_exp_r5d.jsonl). Here each operand is split ONCE, by
// split_planes (one streaming pass: 4 B read, 6 B written per element), into three bf16 planes
// laid out K-contiguous and zero-padded to a multiple of 32 in K; the GEMM then runs no VALU on
// its operands at all:
//   * 256 threads = 4 waves (2 x 2), block tile 256 x 128, a wave owns 128 x 64 = 4 x 2 32x32
//     tiles, K step 16 (32-B plane rows); per step a wave reads 18 ds_read_b128 operands (one per
//     plane per tile, MFMA-ready: no conversion) and issues 48 v_mfma_f32_32x32x16_bf16.
//   * Global -> LDS by global_load_lds_dwordx4 into four stages of 36 KiB (A 24 + B 12): one
//     workgroup per CU, three stages in flight behind a counted vmcnt (never 0 inside the loop:
//     a vmcnt(0) at every barrier exposed the DMA latency -- the first, two-stage version of this
//     kernel ran at ~170 TF/s, profiles/micro/gemm_planes_r5h.jsonl).
//   * Rows are XOR-swizzled through the DMA SOURCE address (slot = chunk ^ ((row >> 3) & 1)):
//     every 16-lane group of a fragment read covers all 64 banks once (conflict-free).
//   * XCD-aware bijective block order (consecutive tiles of one XCD share the A row panel).
// Products per 32x32x16 step: a2b0, a0b2, a1b1, a1b0, a0b1, a0b0 (smallest first), as the fast
// kernel's mfma_emu6; accuracy is tested against fp64 next to the native f32 MFMA path
// (tests/test_gemm_planes_gpu.py).
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace tdp {
namespace {

typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef char lds_char;

constexpr int kT = 256;
constexpr int kBM = 256, kBN = 128, kBK = 16;  // tile; K step (one 32x32x16 MFMA depth)
constexpr int kRow = kBK * 2;                  // 32 B per plane row per stage
constexpr int kAB = 3 * kBM * kRow;            // 24 KiB: three A planes
constexpr int kBB = 3 * kBN * kRow;            // 12 KiB: three B planes
constexpr int kStg = kAB + kBB;
constexpr int kS = 4;                          // 144 KiB: three stages in flight
constexpr int kUA = kAB / 1024 / 4, kUB = kBB / 1024 / 4;  // 1-KiB DMA units per wave per stage
constexpr int kG = kUA + kUB;                  // DMA instructions per wave per stage
constexpr int kPad = 32;                       // planes are padded in K to a multiple of this

struct PlanesParams {
  const uint16_t* A;  // planes [3][a_rows][ldp] (plane stride a_plane elements)
  const uint16_t* B;
  long a_plane, b_plane, lda, ldb;
  float* C;
  long ldc;
  const float* bias;
  float beta;
  int relu;
  int M, N, K;  // K: padded depth (multiple of 32); pad columns hold zeros
  int tiles_m, tiles_n;
};

// 32-B rows hold two 16-B chunks; rows r and r + 8 share a 32-B bank group, so the chunk slot is
// flipped by row bit 3: a fragment read's 16-lane groups then cover all 64 banks once
__device__ __forceinline__ int swz(int row) { return (row >> 3) & 1; }

__device__ __forceinline__ void glds16(const void* src, lds_char* dst) {
  __builtin_amdgcn_global_load_lds(src, (void __attribute__((address_space(3)))*)(
                                            (__attribute__((address_space(3))) char*)dst),
                                   16, 0, 0);
}

__device__ __forceinline__ f32x16 emu6(const bf8 (&a)[3], const bf8 (&b)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// Per-lane DMA sources of one operand's share of a stage: unit j of this wave covers plane
// j / (R/32), rows (j % (R/32)) * 32 + lane / 2, 16-B slot lane % 2 (chunk = slot ^ swz(row)).
template <int R, int U>
struct PlaneSrc {
  const uint16_t* src[U];
  __device__ __forceinline__ void init(const uint16_t* base, long plane, long ld, int r0,
                                       int rlim, int wid, int lane) {
    constexpr int UPP = R / 32;  // units per plane
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int j = wid * U + i;
      const int pl = j / UPP;
      const int row = (j % UPP) * 32 + (lane >> 1);
      int gr = r0 + row;
      gr = gr < rlim ? gr : rlim - 1;
      const int chunk = (lane & 1) ^ swz(row);
      src[i] = base + pl * plane + (long)gr * ld + chunk * 8;
    }
  }
  __device__ __forceinline__ void issue(int k0, lds_char* dst, int wid) const {
#pragma unroll
    for (int i = 0; i < U; ++i) glds16(src[i] + k0, dst + (wid * U + i) * 1024);
  }
};

__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm_planes_kernel(PlanesParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int h = lane >> 5, l31 = lane & 31;
  // XCD-aware bijective order: hardware ids b, b+8, ... share an XCD and get consecutive tiles
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  const int tm = lid / p.tiles_n, tn = lid % p.tiles_n;
  const int m0 = tm * kBM, n0 = tn * kBN;

  PlaneSrc<kBM, kUA> sa;
  PlaneSrc<kBN, kUB> sb;
  sa.init(p.A, p.a_plane, p.lda, m0, p.M, wid, lane);
  sb.init(p.B, p.b_plane, p.ldb, n0, p.N, wid, lane);
  const int nk = p.K / kBK;

  f32x16 acc[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][g][r] = 0.f;

  // fragment LDS offsets within a stage (plane 0; planes follow at kBM*kRow / kBN*kRow)
  int a_row[4], b_row[2];
#pragma unroll
  for (int f = 0; f < 4; ++f) a_row[f] = wm * 128 + f * 32 + l31;
#pragma unroll
  for (int g = 0; g < 2; ++g) b_row[g] = wn * 64 + g * 32 + l31;

  auto read = [&](const lds_char* st, bf8 (&fa)[4][3], bf8 (&fb)[2][3]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int row = a_row[f];
      const int off = row * kRow + ((h ^ swz(row)) * 16);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        fa[f][pl] = *reinterpret_cast<const bf8*>(st + pl * (kBM * kRow) + off);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int row = b_row[g];
      const int off = kAB + row * kRow + ((h ^ swz(row)) * 16);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        fb[g][pl] = *reinterpret_cast<const bf8*>(st + pl * (kBN * kRow) + off);
    }
  };
  auto issue = [&](int t) {
    lds_char* st = smem + (t % kS) * kStg;
    sa.issue(t * kBK, st, wid);
    sb.issue(t * kBK, st + kAB, wid);
  };

  // S-1 stages in flight ahead of the one being consumed; a counted vmcnt (never 0 inside the
  // loop) keeps the newer stages' DMA outstanding across the barrier
#pragma unroll
  for (int t = 0; t < kS - 1; ++t)
    if (t < nk) issue(t);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;  // stages issued after kt that may still be in flight
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kG) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kG) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // stage kt landed for every wave; every wave left stage kt - 1 (the buffer refilled next)
    __builtin_amdgcn_s_barrier();
    if (kt + kS - 1 < nk) issue(kt + kS - 1);
    const lds_char* st = smem + (kt % kS) * kStg;
    bf8 fa[4][3], fb[2][3];
    read(st, fa, fb);
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int g = 0; g < 2; ++g) acc[f][g] = emu6(fa[f], fb[g], acc[f][g]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup

  // epilogue: lane owns column l31 of each 32x32 tile, rows (r&3) + 8*(r>>2) + 4*h
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int col = n0 + wn * 64 + g * 32 + l31;
      if (col >= p.N) continue;
      const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        float* c = p.C + (long)row * p.ldc + col;
        float v = acc[f][g][r] + bv;
        if (p.beta != 0.f) v += p.beta * *c;
        if (p.relu) v = fmaxf(v, 0.f);
        *c = v;
      }
    }
}

// ---- the split pass ----------------------------------------------------------------------
__device__ __forceinline__ void split8(const float (&x)[8], u32x4& h, u32x4& m, u32x4& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf2));
    const float r0 = a - __uint_as_float(hu << 16), r1 = b - __uint_as_float(hu & 0xffff0000u);
    const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf2));
    const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
    h[i] = hu;
    m[i] = mu;
    l[i] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{s0, s1}, bf2));
  }
}

// K-contiguous source [R][K] (row stride ld) -> planes [3][R][Kp]; one thread per 8 k
__global__ __launch_bounds__(256) void split_planes_k_kernel(const float* __restrict__ src,
                                                             long ld, int R, int K, int Kp,
                                                             uint16_t* __restrict__ dst,
                                                             long plane) {
  const long per_row = Kp / 8;
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= per_row * R) return;
  const int r = (int)(t / per_row), k0 = (int)(t % per_row) * 8;
  const float* s = src + (long)r * ld + k0;
  float x[8];
  if (k0 + 8 <= K && (((uintptr_t)s) & 15) == 0) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(s);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(s + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = v0[e];
      x[4 + e] = v1[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = k0 + e < K ? s[e] : 0.f;
  }
  u32x4 hv, mv, lv;
  split8(x, hv, mv, lv);
  uint16_t* d = dst + (long)r * Kp + k0;
  *reinterpret_cast<u32x4*>(d) = hv;
  *reinterpret_cast<u32x4*>(d + plane) = mv;
  *reinterpret_cast<u32x4*>(d + 2 * plane) = lv;
}

// MN-contiguous source [K][R] (row stride ld) -> planes [3][R][Kp] (transposed through LDS):
// a 64 (k) x 64 (r) tile per workgroup, read along r, written along k
__global__ __launch_bounds__(256) void split_planes_t_kernel(const float* __restrict__ src,
                                                             long ld, int R, int K, int Kp,
                                                             uint16_t* __restrict__ dst,
                                                             long plane) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = k0 + tr + 4 * i, r = r0 + tc;
    tile[tr + 4 * i][tc] = (k < K && r < R) ? src[(long)k * ld + r] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int item = threadIdx.x + 256 * i;  // 64 rows x 8 chunks of 8 k
    const int rr = item >> 3, ch = item & 7;
    const int r = r0 + rr, k = k0 + ch * 8;
    if (r >= R || k >= Kp) continue;
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = tile[ch * 8 + e][rr];
    u32x4 hv, mv, lv;
    split8(x, hv, mv, lv);
    uint16_t* d = dst + (long)r * Kp + k;
    *reinterpret_cast<u32x4*>(d) = hv;
    *reinterpret_cast<u32x4*>(d + plane) = mv;
    *reinterpret_cast<u32x4*>(d + 2 * plane) = lv;
  }
}

}  // namespace

long planes_depth(int K) { return (long)ceil_div(K, kPad) * kPad; }

void split_planes(const float* src, long ld, bool kcontig, int R, int K, uint16_t* dst,
                  hipStream_t s) {
  const long Kp = planes_depth(K);
  const long plane = (long)R * Kp;
  if (R <= 0 || K <= 0) return;
  if (kcontig) {
    const long work = (long)R * (Kp / 8);
    hipLaunchKernelGGL(split_planes_k_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                       s, src, ld, R, K, (int)Kp, dst, plane);
  } else {
    const dim3 grid((unsigned)ceil_div(R, 64), (unsigned)ceil_div(Kp, 64));
    hipLaunchKernelGGL(split_planes_t_kernel, grid, dim3(256), 0, s, src, ld, R, K, (int)Kp, dst,
                       plane);
  }
}

void gemm_planes_run(const uint16_t* A, const uint16_t* B, int M, int N, int K, float* C,
                     long ldc, const float* bias, float beta, bool relu, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const long Kp = planes_depth(K);
  PlanesParams p{};
  p.A = A;
  p.B = B;
  p.a_plane = (long)M * Kp;
  p.b_plane = (long)N * Kp;
  p.lda = Kp;
  p.ldb = Kp;
  p.C = C;
  p.ldc = ldc;
  p.bias = bias;
  p.beta = beta;
  p.relu = relu ? 1 : 0;
  p.M = M;
  p.N = N;
  p.K = (int)Kp;
  p.tiles_m = ceil_div(M, kBM);
  p.tiles_n = ceil_div(N, kBN);
  const size_t lds = (size_t)kS * kStg;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)gemm_planes_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL(gemm_planes_kernel, dim3((unsigned)(p.tiles_m * p.tiles_n)), dim3(kT), lds, s,
                     p);
}

}  // namespace tdp
