// fp32 GEMM for gfx950 on the f32-input matrix core (v_mfma_f32_32x32x2_f32).
//
// Replaces the hipBLASLt addmm/mm calls that torch's nn.Linear makes for the reference's
// classifier layers (REF/data_and_toy_model.py:41-45), with the
// rest of the layer fused in:
//   forward  Y  = X . W^T + b, ReLU          (A=X [M][K],  B=W [N][K])
//   dgrad    dX = (dY*[Y>0]) . W              (A=dY [M][K], B=W [K][N])
//   wgrad    dW = (dY*[Y>0])^T . X, db = sum  (A=dY^T [K][M], B=X [K][N])
// The ReLU backward is applied while staging the A operand (mask), the bias gradient is a row sum
// of the staged A tile, and split-K partials go to a workspace combined by splitk_reduce.
//
// Design (CDNA4): 256-thread workgroups = 4 waves (2x2), each wave owns (BM/2)x(BN/2) of the
// block tile as 32x32 MFMA tiles; K advances in BK=32 steps through two LDS buffers with
// register staging (next tile's global loads issued before the current tile's MFMAs, written to
// the other LDS buffer after them: one barrier per K step). Operands are read from LDS as f32x4
// along K: lane half h of MFMA k-step (q,s) consumes k = 8q + 4h + s, for A and B alike, so a
// single ds_read_b128 feeds four MFMAs. K-contiguous LDS rows are padded by 16 B (row stride
// 36 dwords) which makes those reads bank-conflict-free. f32-in MFMA is exact f32 (a k-ordered
// fmaf chain), so results match torch's fp32 Linear to rounding of the summation order.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "emu8.h"

namespace tdp {
namespace {

constexpr int kThreads = 256;
constexpr int kBK = 32;

struct Params {
  const float* A;
  const float* B;
  float* C;
  const float* mask;
  const float* bias;
  float* rowsum;
  float* ws;
  long lda, ldb, ldc, ldmask;
  int M, N, K;
  int k_per_split;
  float beta, rowsum_beta;
  int relu;
  int splits;
};

// Per-thread share of a ROWS x COLS tile whose COLS are contiguous in global memory.
template <int ROWS, int COLS, bool VEC>
struct Stage {
  static constexpr int TPR = COLS / 4;        // threads per row (one f32x4 each)
  static constexpr int RPP = kThreads / TPR;  // rows per pass
  static constexpr int NV = ROWS / RPP;       // f32x4 per thread
  static_assert(ROWS % RPP == 0, "tile rows must be a multiple of rows-per-pass");
  f32x4 v[NV];

  __device__ __forceinline__ void load(const float* __restrict__ g, long ld, int r0, int c0,
                                       int rlim, int clim, const float* __restrict__ mk,
                                       long ldm) {
    const int cc = (threadIdx.x % TPR) * 4;
    const int rr = threadIdx.x / TPR;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int r = r0 + rr + i * RPP;
      const int c = c0 + cc;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (r < rlim) {
        const float* src = g + (long)r * ld + c;
        if (VEC && c + 3 < clim) {
          x = *reinterpret_cast<const f32x4*>(src);
          if (mk) {
            const f32x4 m = *reinterpret_cast<const f32x4*>(mk + (long)r * ldm + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = m[e] > 0.f ? x[e] : 0.f;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (c + e < clim) {
              float val = src[e];
              if (mk) val = mk[(long)r * ldm + c + e] > 0.f ? val : 0.f;
              x[e] = val;
            }
          }
        }
      }
      v[i] = x;
    }
  }

  __device__ __forceinline__ void store(float* lds, int ld_lds) const {
    const int cc = (threadIdx.x % TPR) * 4;
    const int rr = threadIdx.x / TPR;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      *reinterpret_cast<f32x4*>(lds + (rr + i * RPP) * ld_lds + cc) = v[i];
  }
};

template <int BM, int BN, bool AK, bool BKC, bool VEC>
__global__ __launch_bounds__(kThreads) void gemm_f32_kernel(Params p) {
  constexpr int BK = kBK;
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int A_ROWS = AK ? BM : BK, A_COLS = AK ? BK : BM, A_LD = A_COLS + (AK ? 4 : 0);
  constexpr int B_ROWS = BKC ? BN : BK, B_COLS = BKC ? BK : BN, B_LD = B_COLS + (BKC ? 4 : 0);
  constexpr int A_SZ = A_ROWS * A_LD, B_SZ = B_ROWS * B_LD, STG = A_SZ + B_SZ;
  __shared__ __attribute__((aligned(16))) float smem[2 * STG];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, z = blockIdx.z;
  const int kb = z * p.k_per_split;
  const int ke = min(p.K, kb + p.k_per_split);
  const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  Stage<A_ROWS, A_COLS, VEC> sa;
  Stage<B_ROWS, B_COLS, VEC> sb;
  auto gload = [&](int k0) {
    if (AK) sa.load(p.A, p.lda, m0, k0, p.M, ke, p.mask, p.ldmask);
    else    sa.load(p.A, p.lda, k0, m0, ke, p.M, p.mask, p.ldmask);
    if (BKC) sb.load(p.B, p.ldb, n0, k0, p.N, ke, nullptr, 0);
    else     sb.load(p.B, p.ldb, k0, n0, ke, p.N, nullptr, 0);
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const bool do_rs = (p.rowsum != nullptr) && blockIdx.x == 0;
  float rs = 0.f;

  if (nk > 0) {
    gload(kb);
    sa.store(smem, A_LD);
    sb.store(smem + A_SZ, B_LD);
    __syncthreads();
  }
  const int h4 = (lane >> 5) * 4;
  for (int kt = 0; kt < nk; ++kt) {
    const float* As = smem + (kt & 1) * STG;
    const float* Bs = As + A_SZ;
    if (kt + 1 < nk) gload(kb + (kt + 1) * BK);  // issue early; lands under the MFMAs below
    if (do_rs && threadIdx.x < BM) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k)
        rs += AK ? As[threadIdx.x * A_LD + k] : As[k * A_LD + threadIdx.x];
    }
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      const int kk = q * 8 + h4;
      f32x4 a[FM], b[FN];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int i = wm * TM + fm * 32 + (lane & 31);
        if (AK) {
          a[fm] = *reinterpret_cast<const f32x4*>(As + i * A_LD + kk);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) a[fm][s] = As[(kk + s) * A_LD + i];
        }
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = wn * TN + fn * 32 + (lane & 31);
        if (BKC) {
          b[fn] = *reinterpret_cast<const f32x4*>(Bs + j * B_LD + kk);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) b[fn][s] = Bs[(kk + s) * B_LD + j];
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(a[fm][s], b[fn][s], acc[fm][fn], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      float* nA = smem + ((kt + 1) & 1) * STG;
      sa.store(nA, A_LD);
      sb.store(nA + A_SZ, B_LD);
    }
    __syncthreads();
  }

  if (do_rs && threadIdx.x < BM && m0 + (int)threadIdx.x < p.M) {
    float* dst = p.rowsum + m0 + threadIdx.x;
    *dst = (p.rowsum_beta != 0.f ? p.rowsum_beta * *dst : 0.f) + rs;
  }

  // C/D map of 32x32 MFMA tiles: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  const bool split = p.splits > 1;
  float* wsz = split ? p.ws + (long)z * p.M * p.N : nullptr;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = n0 + wn * TN + fn * 32 + (lane & 31);
      if (col >= p.N) continue;
      const float bcol = (!split && p.bias) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * TM + fm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= p.M) continue;
        float v = acc[fm][fn][r];
        if (split) {
          wsz[(long)row * p.N + col] = v;
        } else {
          float* dst = p.C + (long)row * p.ldc + col;
          v += bcol;
          if (p.beta != 0.f) v += p.beta * *dst;
          if (p.relu) v = fmaxf(v, 0.f);
          *dst = v;
        }
      }
    }
}

// Split-K combine over the flattened [M][N] plane (N % 4 == 0 for VEC: a float4 group never
// straddles a row). A 256-thread block covers G = 256 / ZT consecutive groups x ZT split lanes:
// the split axis is itself spread over threads (tree-reduced in LDS), because a weight gradient
// has few outputs and many splits (ResNet-50 layer1 1x1 wgrad: 4096 outputs x 512 splits — one
// thread per output serialised 512 loads per thread on 4 workgroups).
template <bool VEC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws,
                                                            int splits, int M, int N, void* Cv,
                                                            int c_bf16, long ldc,
                                                            const float* __restrict__ bias,
                                                            float beta, int relu, int zt_log2,
                                                            const float* __restrict__ gate,
                                                            long ldgate) {
  constexpr int W = VEC ? 4 : 1;
  const int ZT = 1 << zt_log2, G = 256 >> zt_log2;
  const int g = threadIdx.x % G, zt = threadIdx.x / G;
  const long plane = (long)M * N;
  const long ng = plane / W;
  const long idx = (long)blockIdx.x * G + g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (idx < ng) {
    if (VEC) {
      const f32x4* src = reinterpret_cast<const f32x4*>(ws) + idx;
      const long step = ng;
#pragma unroll 4
      for (int z = zt; z < splits; z += ZT) acc += src[z * step];
    } else {
      float t = 0.f;
#pragma unroll 4
      for (int z = zt; z < splits; z += ZT) t += ws[z * plane + idx];
      acc[0] = t;
    }
  }
  __shared__ f32x4 red[256];
  if (ZT > 1) {
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int h = ZT >> 1; h > 0; h >>= 1) {
      if (zt < h) red[threadIdx.x] += red[threadIdx.x + h * G];
      __syncthreads();
    }
    acc = red[threadIdx.x];
  }
  if (zt != 0 || idx >= ng) return;
  const long e0 = idx * W;
  const int row = (int)(e0 / N), col = (int)(e0 - (long)row * N);
#pragma unroll
  for (int e = 0; e < W; ++e) {
    float x = acc[e];
    if (bias) x += bias[col + e];
    if (c_bf16) {
      unsigned short* C = reinterpret_cast<unsigned short*>(Cv) + (long)row * ldc + col + e;
      if (beta != 0.f) x += beta * bf16_to_f32(*C);
      if (relu) x = fmaxf(x, 0.f);
      *C = f32_to_bf16(x);
    } else {
      float* C = reinterpret_cast<float*>(Cv) + (long)row * ldc + col + e;
      if (beta != 0.f) x += beta * *C;
      if (relu) x = fmaxf(x, 0.f);
      if (gate && !(gate[(long)row * ldgate + col + e] > 0.f)) x = 0.f;
      *C = x;
    }
  }
}

struct TileCfg {
  int bm, bn;
};
constexpr TileCfg kTiles[] = {{128, 128}, {128, 64}, {64, 64}};

template <int BM, int BN, bool VEC>
void launch_layout(const Params& p, dim3 grid, bool ak, bool bk, hipStream_t s) {
  dim3 block(kThreads);
  if (ak && bk)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, true, true, VEC>), grid, block, 0, s, p);
  else if (ak && !bk)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, true, false, VEC>), grid, block, 0, s, p);
  else if (!ak && !bk)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, false, VEC>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, true, VEC>), grid, block, 0, s, p);
}

template <bool VEC>
void launch_tile(int tile, const Params& p, dim3 grid, bool ak, bool bk, hipStream_t s) {
  switch (tile) {
    case 0: launch_layout<128, 128, VEC>(p, grid, ak, bk, s); break;
    case 1: launch_layout<128, 64, VEC>(p, grid, ak, bk, s); break;
    default: launch_layout<64, 64, VEC>(p, grid, ak, bk, s); break;
  }
}

inline bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

__global__ __launch_bounds__(256) void gate_kernel(float* __restrict__ C, long ldc,
                                                   const float* __restrict__ gate, long ldg, int M,
                                                   int N) {
  const long n = (long)M * N;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int row = (int)(e / N), col = (int)(e % N);
    if (!(gate[row * ldg + col] > 0.f)) C[row * ldc + col] = 0.f;
  }
}

}  // namespace

void gate_inplace(float* C, long ldc, const float* gate, long ldg, int M, int N, hipStream_t s) {
  const long n = (long)M * N;
  if (n <= 0) return;
  const unsigned grid = (unsigned)std::min<long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(gate_kernel, dim3(grid), dim3(256), 0, s, C, ldc, gate, ldg, M, N);
}

static int g_mode = 0;  // 0 auto, 1 generic, 2 fast, 3 auto (skinny allowed; = 0)
void gemm_f32_set_mode(int mode) { g_mode = mode; }

GemmPlan gemm_f32_plan(const GemmF32Args& a, int num_cus) {
  GemmPlan plan;
  if (g_mode == 0 || g_mode == 3) {
    plan.skinny = gemm_skinny_kind(a);
    if (plan.skinny) return plan;
  }
  if (g_mode != 1 && gemm_f32_fast_ok(a)) {
    // a large plain GEMM that fills the chip with 256 x 256 tiles: the one-workgroup-per-CU
    // kernel, bitwise equal and 15-20 % faster (profiles/r9/gemm_emu8_r9.md)
    if ((g_mode == 0 || g_mode == 3) && gemm_f32_emu() && a.a_kcontig && !a.mask && !a.rowsum &&
        !a.gate &&
        a.opt.kind == 0 && gemm_emu8_fits(a.M, a.N, a.K, num_cus)) {
      GemmEmu8Args e;
      e.A = a.A; e.B = a.B; e.C = a.C; e.lda = a.lda; e.ldb = a.ldb; e.ldc = a.ldc;
      e.b_kcontig = a.b_kcontig; e.M = a.M; e.N = a.N; e.K = a.K; e.beta = a.beta;
      if (gemm_emu8_ok(e)) {
        plan.emu8 = true;
        plan.fast = true;
        plan.bm = plan.bn = 256;
        return plan;
      }
    }
    gemm_f32_fast_plan(a, num_cus, plan);
    return plan;
  }
  if (a.M >= 512 && a.N >= 512) plan.tile = 0;
  else if (a.M <= 64) plan.tile = 2;
  else plan.tile = 1;
  plan.bm = kTiles[plan.tile].bm;
  plan.bn = kTiles[plan.tile].bn;
  const long tiles = (long)ceil_div(a.M, plan.bm) * ceil_div(a.N, plan.bn);
  int splits = 1;
  if (a.rowsum == nullptr && tiles < num_cus) {
    // fill the chip: ~1 workgroup per CU, each split keeping >= 8 K-steps of MFMA work
    const int want = (int)((num_cus + tiles - 1) / tiles);
    const int kmax = a.K / (kBK * 8);
    splits = want < kmax ? want : kmax;
    if (splits < 1) splits = 1;
  }
  int kps = ceil_div(a.K, splits);
  kps = ceil_div(kps, kBK) * kBK;
  if (kps <= 0) kps = kBK;
  plan.splits = ceil_div(a.K > 0 ? a.K : 1, kps);
  plan.k_per_split = kps;
  plan.ws_floats = plan.splits > 1 ? (long)plan.splits * a.M * a.N : 0;
  return plan;
}

void gemm_f32_run(const GemmF32Args& a, const GemmPlan& plan, float* ws, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  if (plan.skinny) {
    gemm_skinny_run(plan.skinny, a, s);
    if (a.opt.kind != 0) gemm_opt_fallback(a, s);
    return;
  }
  if (plan.emu8) {
    GemmEmu8Args e;
    e.A = a.A; e.B = a.B; e.C = a.C; e.lda = a.lda; e.ldb = a.ldb; e.ldc = a.ldc;
    e.b_kcontig = a.b_kcontig; e.M = a.M; e.N = a.N; e.K = a.K; e.beta = a.beta;
    e.bias = a.bias; e.relu = a.relu;
    gemm_emu8_run(e, s);
    return;
  }
  if (plan.fast) {
    gemm_f32_fast_run(a, plan, ws, s);
    return;
  }
  Params p;
  p.A = a.A; p.B = a.B; p.C = a.C; p.mask = a.mask; p.bias = a.bias; p.rowsum = a.rowsum;
  p.ws = ws; p.lda = a.lda; p.ldb = a.ldb; p.ldc = a.ldc; p.ldmask = a.ldmask;
  p.M = a.M; p.N = a.N; p.K = a.K; p.k_per_split = plan.k_per_split;
  p.beta = a.beta; p.rowsum_beta = a.rowsum_beta; p.relu = a.relu ? 1 : 0;
  p.splits = plan.splits;
  const bool vec = aligned16(a.A) && aligned16(a.B) && (a.lda % 4 == 0) && (a.ldb % 4 == 0) &&
                   (a.mask == nullptr || (aligned16(a.mask) && a.ldmask % 4 == 0));
  dim3 grid(ceil_div(a.N, plan.bn), ceil_div(a.M, plan.bm), plan.splits);
  if (vec) launch_tile<true>(plan.tile, p, grid, a.a_kcontig, a.b_kcontig, s);
  else launch_tile<false>(plan.tile, p, grid, a.a_kcontig, a.b_kcontig, s);
  if (plan.splits > 1)
    splitk_reduce(ws, plan.splits, a.M, a.N, a.C, false, a.ldc, a.bias, a.beta, a.relu, s,
                  a.gate, a.ldgate);
  else if (a.gate)  // the generic tile kernel has no gate epilogue: one masking pass
    gate_inplace(a.C, a.ldc, a.gate, a.ldgate, a.M, a.N, s);
  if (a.opt.kind != 0) gemm_opt_fallback(a, s);
}

// The generic kernel has no optimizer epilogue: C now holds the gradient, apply the flat update.
void gemm_opt_fallback(const GemmF32Args& a, hipStream_t s) {
  const OptEpilogue& o = a.opt;
  const long n = (long)a.M * a.N;
  if (o.kind == 1) sgd_flat(o.p, a.C, o.s0, n, o.sgd, s);
  else if (o.kind == 2) adam_flat(o.p, a.C, o.s0, o.s1, o.s2, n, o.adam, s);
}

void splitk_reduce(const float* ws, int splits, int M, int N, void* C, bool c_bf16, long ldc,
                   const float* bias, float beta, bool relu, hipStream_t s, const float* gate,
                   long ldgate) {
  const bool vec = (N % 4 == 0) && (ldc % 4 == 0) && aligned16(C) &&
                   (bias == nullptr || aligned16(bias));
  const long groups = vec ? (long)M * N / 4 : (long)M * N;
  // split lanes per output group: enough threads in flight (~1024 per CU) without starving the
  // column axis; at most 64 lanes and never more than the splits
  int zl = 0;
  while (zl < 6 && (2 << zl) <= splits && groups * (2 << zl) <= 256L * 1024) ++zl;
  const int G = 256 >> zl;
  const dim3 grid((unsigned)((groups + G - 1) / G));
  if (vec)
    hipLaunchKernelGGL(splitk_reduce_kernel<true>, grid, dim3(256), 0, s, ws, splits, M, N, C,
                       c_bf16 ? 1 : 0, ldc, bias, beta, relu ? 1 : 0, zl, gate, ldgate);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<false>, grid, dim3(256), 0, s, ws, splits, M, N, C,
                       c_bf16 ? 1 : 0, ldc, bias, beta, relu ? 1 : 0, zl, gate, ldgate);
}

}  // namespace tdp
