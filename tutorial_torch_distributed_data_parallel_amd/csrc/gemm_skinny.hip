// Skinny fp32 GEMMs: one dimension <= 16 (a classifier head with few classes, its gradients).
//
// The toy MLP / AlexNet head Linear(4096, 10) produces three GEMMs with a dimension of 10: the
// forward [B x 10] = X[B x 4096] . W^T (N = 10), the input gradient [B x 4096] = dY[B x 10] . W
// (K = 10) and the weight gradient [10 x 4096] = dY^T . X (M = 10). On the MFMA tile kernels
// they cost a split-K launch + a combine, or a 64-wide tile that is 85 % padding (9-15 us each,
// profiles/mlp_dp1_eager_kernel_stats_v3.md); here each is one small bandwidth-shaped launch:
//   * skinny_n : one workgroup per output row, K spread over its 256 lanes as f32x4 chunks, the
//                N <= 16 dot products kept in registers, reduced across waves at the end;
//   * skinny_k : every lane produces 4 adjacent outputs of a row from the K <= 16 row of A
//                (wave-uniform scalar loads) and K f32x4 rows of B;
//   * skinny_m : A staged in LDS, 64 columns x 4 K-quarters per workgroup, M <= 16
//                accumulators per lane, the quarters combined through LDS; the bias gradient
//                (row sums of A) comes from workgroup 0.
// All three apply the usual epilogue (bias, beta * C, ReLU) and need 16-B aligned rows.
#include <algorithm>
#include <type_traits>

#include "ce_row.h"
#include "common.h"
#include "kernels.h"
#include "optim_elem.h"
#include "planes.h"

namespace tdp {
namespace {

constexpr int kSkinnyMax = 16;

struct SkinnyParams {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  float* rowsum;
  long lda, ldb, ldc;
  int M, N, K;
  float beta, rowsum_beta;
  int relu;
  const float* gate;  // optional C-shaped gate (GemmF32Args::gate)
  long ldg;
};

__device__ __forceinline__ float epi(float v, const SkinnyParams& p, const float* crow, int col,
                                     int row) {
  if (p.bias) v += p.bias[col];
  if (p.beta != 0.f) v += p.beta * crow[col];
  if (p.relu) v = fmaxf(v, 0.f);
  if (p.gate && !(p.gate[(long)row * p.ldg + col] > 0.f)) v = 0.f;
  return v;
}

// C[M, N<=16] = A[M, K] . B[N, K]^T  (A and B K-contiguous, K % 4 == 0). One 256-thread
// workgroup per row: the K axis is spread over all 256 lanes as f32x4 chunks (4 chunks per lane
// for K = 4096, unrolled so every load of the row is in flight at once), then the N partial dot
// products are reduced across the wave (shuffles) and the 4 waves (LDS).
template <int NMAX>
__global__ __launch_bounds__(256) void skinny_n_kernel(SkinnyParams p) {
  __shared__ float red[4][NMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x;
  const float* a = p.A + (long)row * p.lda;
  float acc[NMAX];
#pragma unroll
  for (int n = 0; n < NMAX; ++n) acc[n] = 0.f;
  // B rows past N are clamped to row N-1 (valid, L2-resident) instead of branched over: a
  // per-row branch splits the unrolled body into blocks the loads cannot be hoisted across, one
  // L2 round trip per B row (17 us for 128x4096x10); branch-free, every load of a chunk is in flight
  // together. The extra rows' sums are discarded.
  const float* brow[NMAX];
#pragma unroll
  for (int n = 0; n < NMAX; ++n) brow[n] = p.B + (long)(n < p.N ? n : p.N - 1) * p.ldb;
#pragma unroll 4
  for (int k = threadIdx.x * 4; k < p.K; k += 1024) {
    const f32x4 av = *reinterpret_cast<const f32x4*>(a + k);
    f32x4 bv[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) bv[n] = *reinterpret_cast<const f32x4*>(brow[n] + k);
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
      acc[n] = fmaf(av[0], bv[n][0], fmaf(av[1], bv[n][1], fmaf(av[2], bv[n][2],
                                                                fmaf(av[3], bv[n][3], acc[n]))));
  }
#pragma unroll
  for (int n = 0; n < NMAX; ++n) {
    const float v = wave_sum(acc[n]);
    if (lane == 0) red[w][n] = v;
  }
  __syncthreads();
  if (threadIdx.x < p.N) {
    const int n = threadIdx.x;
    const float v = red[0][n] + red[1][n] + red[2][n] + red[3][n];
    float* crow = p.C + (long)row * p.ldc;
    crow[n] = epi(v, p, crow, n, row);
  }
}

// C[M, N] = A[M, K<=16] . B[K, N]  (A K-contiguous, B [K][N] row-major, N % 4 == 0)
__global__ __launch_bounds__(256) void skinny_k_kernel(SkinnyParams p) {
  const long per_row = p.N / 4;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t >= per_row * p.M) return;
  const int row = (int)(t / per_row);
  const int col = (int)(t % per_row) * 4;
  const float* a = p.A + (long)row * p.lda;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < p.K; ++k) {
    const float av = a[k];
    const f32x4 bv = *reinterpret_cast<const f32x4*>(p.B + (long)k * p.ldb + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = fmaf(av, bv[e], acc[e]);
  }
  float* crow = p.C + (long)row * p.ldc;
  f32x4 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) out[e] = epi(acc[e], p, crow, col + e, row);
  *reinterpret_cast<f32x4*>(crow + col) = out;
}

// C[M<=16, N] = A^T . B with A stored [K][M], B stored [K][N]; rowsum[m] = sum_k A[k][m].
// A (K x M, a few KiB) is staged in LDS once per workgroup; each workgroup owns 64 columns and
// splits K over its 4 waves (unrolled by 8 so the B loads overlap), partials combined in LDS.
template <int MMAX>
__global__ __launch_bounds__(256) void skinny_m_kernel(SkinnyParams p) {
  extern __shared__ float smem[];  // [K][MMAX] copy of A, then reused for the 4 x MMAX x 64 sums
  const int cl = threadIdx.x & 63;
  const int q = threadIdx.x >> 6;  // K quarter
  const int col = blockIdx.x * 64 + cl;
  for (int i = threadIdx.x; i < p.K * MMAX; i += 256) {
    const int k = i / MMAX, m = i % MMAX;
    smem[i] = m < p.M ? p.A[(long)k * p.lda + m] : 0.f;
  }
  __syncthreads();
  const int kq = (p.K + 3) / 4;
  const int k0 = q * kq, k1 = min(p.K, k0 + kq);
  float acc[MMAX];
#pragma unroll
  for (int m = 0; m < MMAX; ++m) acc[m] = 0.f;
  const int cc = col < p.N ? col : p.N - 1;
#pragma unroll 8
  for (int k = k0; k < k1; ++k) {
    const float bv = p.B[(long)k * p.ldb + cc];
    const float* arow = smem + k * MMAX;
#pragma unroll
    for (int m = 0; m < MMAX; ++m) acc[m] = fmaf(arow[m], bv, acc[m]);
  }
  float rs = 0.f;  // bias gradient: block 0 sums A's column m = threadIdx.x over K (from LDS)
  if (p.rowsum && blockIdx.x == 0 && threadIdx.x < p.M)
    for (int k = 0; k < p.K; ++k) rs += smem[k * MMAX + threadIdx.x];
  __syncthreads();  // A no longer needed: reuse LDS for the cross-wave partial sums
  float* red = smem;  // [4][MMAX][64]
#pragma unroll
  for (int m = 0; m < MMAX; ++m) red[(q * MMAX + m) * 64 + cl] = acc[m];
  __syncthreads();
  for (int o = threadIdx.x; o < MMAX * 64; o += 256) {
    const int m = o / 64, c = o % 64;
    const int gc = blockIdx.x * 64 + c;
    if (m < p.M && gc < p.N) {
      const float v = red[(0 * MMAX + m) * 64 + c] + red[(1 * MMAX + m) * 64 + c] +
                      red[(2 * MMAX + m) * 64 + c] + red[(3 * MMAX + m) * 64 + c];
      float* crow = p.C + (long)m * p.ldc;
      crow[gc] = epi(v, p, crow, gc, m);
    }
  }
  if (p.rowsum && blockIdx.x == 0 && threadIdx.x < p.M) {
    const int m = threadIdx.x;
    p.rowsum[m] = (p.rowsum_beta != 0.f ? p.rowsum_beta * p.rowsum[m] : 0.f) + rs;
  }
}

// Backward of a classifier head Linear(I -> O <= 16) in ONE launch (the toy-MLP fc3): the input
// gradient dx[B][I] = g . W (gated by the previous ReLU's output, optionally emitted as bf16 split
// planes for the next skinny GEMM) from the first nb_dx workgroups, the weight gradient
// dW[O][I] = g^T . x and the bias gradient db = sum_b g from the rest -- skinny_k + skinny_m
// (+ a split pass) fused, so the head's backward is one node instead of three.
struct HeadBwdParams {
  const float* g;  // [B][O]
  const float* x;  // [B][I]
  const float* w;  // [O][I]
  float* dx;       // [B][I], row stride lddx
  const float* gate;
  uint16_t* dxp;   // optional planes of dx [3][B][I] (row stride I, plane stride dxps)
  float* dw;       // [O][I], row stride lddw
  float* db;       // optional [O]
  long ldg, ldx, ldw, lddx, ldgate, dxps, lddw;
  int B, O, I, nb_dx;
  // world size 1 + fused optimizer: update W / b in place of storing dW / db (kind != 0;
  // p / state pointers at the parameters' arena offsets, rows of I elements for W)
  OptEpilogue wopt, bopt;
};

__device__ __forceinline__ void opt_apply(const OptEpilogue& o, long i, float g) {
  OptEpilogue h = o;
  if (o.kind == 1) {
    load_hyper(h.sgd);
    float pe = o.p[i];
    float b = (h.sgd.momentum != 0.f && !h.sgd.first_step) ? o.s0[i] : 0.f;
    sgd_elem(pe, g, b, h.sgd);
    o.p[i] = pe;
    if (h.sgd.momentum != 0.f) o.s0[i] = b;
  } else {
    load_hyper(h.adam);
    float pe = o.p[i], m = o.s0[i], v = o.s1[i];
    adam_elem(pe, g, m, v, o.s2 ? o.s2 + i : nullptr, h.adam);
    o.p[i] = pe;
    o.s0[i] = m;
    o.s1[i] = v;
  }
}

__device__ __forceinline__ void split4_pair(float x0, float x1, unsigned& h, unsigned& m,
                                            unsigned& l) {
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  typedef __bf16 bf2_ __attribute__((ext_vector_type(2)));
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{x0, x1}, bf2_));
  const float r0 = x0 - __uint_as_float(hu << 16), r1 = x1 - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{r0, r1}, bf2_));
  const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_{s0, s1}, bf2_));
}

// weight-gradient columns per head_bwd workgroup: 32 when separate workgroups compute dx; 16
// with the in-place update, where each weight workgroup also computes dx for its own columns
// (twice the workgroups for the same work)
constexpr int kHeadCols = 32, kHeadColsOpt = 16;

template <int MMAX, int CW>
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadBwdParams p) {
  extern __shared__ float smem[];
  if ((int)blockIdx.x < p.nb_dx) {
    // input gradient: 4 adjacent outputs of a row per thread, the O <= 16 gradients of the row
    // broadcast from wave-uniform loads
    const long per_row = p.I / 4;
    const long t = blockIdx.x * 256L + threadIdx.x;
    if (t >= per_row * p.B) return;
    const int row = (int)(t / per_row);
    const int col = (int)(t % per_row) * 4;
    const float* gr = p.g + (long)row * p.ldg;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < p.O; ++k) {
      const float gv = gr[k];
      const f32x4 wv = *reinterpret_cast<const f32x4*>(p.w + (long)k * p.ldw + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(gv, wv[e], acc[e]);
    }
    if (p.gate) {
      const f32x4 gv = *reinterpret_cast<const f32x4*>(p.gate + (long)row * p.ldgate + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = gv[e] > 0.f ? acc[e] : 0.f;
    }
    *reinterpret_cast<f32x4*>(p.dx + (long)row * p.lddx + col) = acc;
    if (p.dxp) {
      typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
      unsigned h0, m0, l0, h1, m1, l1;
      split4_pair(acc[0], acc[1], h0, m0, l0);
      split4_pair(acc[2], acc[3], h1, m1, l1);
      uint16_t* o = p.dxp + (long)row * p.I + col;
      *reinterpret_cast<u32x2_*>(o) = u32x2_{h0, h1};
      *reinterpret_cast<u32x2_*>(o + p.dxps) = u32x2_{m0, m1};
      *reinterpret_cast<u32x2_*>(o + 2 * p.dxps) = u32x2_{l0, l1};
    }
    return;
  }
  // weight / bias gradient: g staged in LDS, kHeadCols columns and 256 / kHeadCols batch slices
  // per workgroup, slices combined through LDS; workgroup 0 sums g for the bias. 32 columns x 8
  // slices (not skinny_m's 64 x 4): twice the workgroups and half of each thread's dependent
  // chain of x loads -- this part was the launch's long pole (64 workgroups for I = 4096)
  constexpr int NQ = 256 / CW;
  const int bid = blockIdx.x - p.nb_dx;
  const int cl = threadIdx.x % CW;
  const int q = threadIdx.x / CW;
  const int col = bid * CW + cl;
  for (int i = threadIdx.x; i < p.B * MMAX; i += 256) {
    const int k = i / MMAX, m = i % MMAX;
    smem[i] = m < p.O ? p.g[(long)k * p.ldg + m] : 0.f;
  }
  __syncthreads();
  const int kq = (p.B + NQ - 1) / NQ;
  const int k0 = q * kq, k1 = min(p.B, k0 + kq);
  float acc[MMAX];
#pragma unroll
  for (int m = 0; m < MMAX; ++m) acc[m] = 0.f;
  const int cc = col < p.I ? col : p.I - 1;
#pragma unroll 8
  for (int k = k0; k < k1; ++k) {
    const float bv = p.x[(long)k * p.ldx + cc];
    const float* arow = smem + k * MMAX;
#pragma unroll
    for (int m = 0; m < MMAX; ++m) acc[m] = fmaf(arow[m], bv, acc[m]);
  }
  float rs = 0.f;
  if (p.db && bid == 0 && threadIdx.x < p.O)
    for (int k = 0; k < p.B; ++k) rs += smem[k * MMAX + threadIdx.x];
  if (p.wopt.kind && p.dx) {
    // The update below overwrites W[:, cols] in place, and the input gradient needs the OLD W:
    // dx[:, c] depends on column c of W only, so this workgroup computes dx for its own columns
    // before updating them (no separate dx workgroups: they would read W while other
    // workgroups write it -- a race). 8 column quads x 32 row groups per workgroup.
    constexpr int CQ = CW / 4, RG = 256 / CQ;
    const int c0 = bid * CW + (threadIdx.x % CQ) * 4;
    if (c0 < p.I) {  // I % 4 == 0 (host-checked)
      f32x4 wv[MMAX];
#pragma unroll
      for (int k = 0; k < MMAX; ++k)
        wv[k] = k < p.O ? *reinterpret_cast<const f32x4*>(p.w + (long)k * p.ldw + c0)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
      for (int row = threadIdx.x / CQ; row < p.B; row += RG) {
        const float* grow = smem + row * MMAX;
        f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < MMAX; ++k) {
          const float gv = grow[k];  // zero past O
#pragma unroll
          for (int e = 0; e < 4; ++e) a4[e] = fmaf(gv, wv[k][e], a4[e]);
        }
        if (p.gate) {
          const f32x4 gt = *reinterpret_cast<const f32x4*>(p.gate + (long)row * p.ldgate + c0);
#pragma unroll
          for (int e = 0; e < 4; ++e) a4[e] = gt[e] > 0.f ? a4[e] : 0.f;
        }
        *reinterpret_cast<f32x4*>(p.dx + (long)row * p.lddx + c0) = a4;
        if (p.dxp) {
          typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
          unsigned h0, m0, l0, h1, m1, l1;
          split4_pair(a4[0], a4[1], h0, m0, l0);
          split4_pair(a4[2], a4[3], h1, m1, l1);
          uint16_t* o = p.dxp + (long)row * p.I + c0;
          *reinterpret_cast<u32x2_*>(o) = u32x2_{h0, h1};
          *reinterpret_cast<u32x2_*>(o + p.dxps) = u32x2_{m0, m1};
          *reinterpret_cast<u32x2_*>(o + 2 * p.dxps) = u32x2_{l0, l1};
        }
      }
    }
  }
  __syncthreads();  // also: every W[:, cols] read of this workgroup precedes its update
  float* red = smem;  // [NQ][MMAX][CW]
#pragma unroll
  for (int m = 0; m < MMAX; ++m) red[(q * MMAX + m) * CW + cl] = acc[m];
  __syncthreads();
  for (int o = threadIdx.x; o < MMAX * CW; o += 256) {
    const int m = o / CW, c = o % CW;
    const int gc = bid * CW + c;
    if (m < p.O && gc < p.I) {
      float v = red[m * CW + c];
#pragma unroll
      for (int qq = 1; qq < NQ; ++qq) v += red[(qq * MMAX + m) * CW + c];
      if (p.wopt.kind) opt_apply(p.wopt, (long)m * p.I + gc, v);
      else p.dw[(long)m * p.lddw + gc] = v;
    }
  }
  if (p.db && bid == 0 && threadIdx.x < p.O) {
    if (p.bopt.kind) opt_apply(p.bopt, threadIdx.x, rs);
    else p.db[threadIdx.x] = rs;
  }
}


// Forward of a classifier head Linear(I -> O <= 16) + its cross-entropy loss in ONE launch (the
// toy MLP / AlexNet fc3 + nn.CrossEntropyLoss: REF/multi-GPU-training-torch.py:121-122), one
// 256-thread workgroup per batch row:
//   * the row's O logits exactly as skinny_n_kernel computes them (same K split, same reduction
//     order), + bias;
//   * the row's cross-entropy terms exactly as ce_fwd_kernel's one-row-per-lane path (ce_row.h)
//     and -- training -- the row's logits gradient for a unit upstream gradient; the mean's
//     denominator (valid labels of the batch) is counted by every workgroup from the labels;
//   * training: the row's input gradient dx = dlogits . W, gated by the previous ReLU's output,
//     and its bf16 split planes, exactly as head_bwd_kernel's dx workgroups compute them (the
//     backward then only reduces dW / db: head_bwd with dx == null);
//   * the batch sums (loss, correct, valid -> loss scalar, lse[B], the device metric
//     accumulator) by the LAST workgroup to arrive, over per-row values handed off through
//     write-through (sc1) stores and an agent-scope ticket (no fences; MI355X_MICROARCH.md
//     inter-workgroup visibility), in ce_fwd_kernel's summation order: bit-identical loss.
// The ticket counters (9 words) are zero between launches (each shard's / the global last
// arriver resets its own).
struct HeadCeParams {
  const float* x;
  const float* w;
  const float* bias;
  const int64_t* labels;
  float* logits;   // [B][O]
  float* lse;      // [B + 1]
  float* rowbuf;   // [B][4] per-row loss / correct / valid
  unsigned* ticket;
  float* loss;
  float* acc;      // optional [3]: += loss sum, correct, rows
  float* dpre;     // optional [B][O]: training (dlogits for a unit seed)
  float* dx;       // optional [B][I] (with dpre)
  const float* gate;
  uint16_t* dxp;   // optional planes of dx [3][B][I]
  long ldx, ldw, lddx, ldgate, dxps;
  int B, O, I, ignore_index, mean;
  float eps;
};

template <int NMAX>
__global__ __launch_bounds__(256) void head_ce_kernel(HeadCeParams p) {
  __shared__ float red[4][NMAX + 4];  // partial dot products; [w][NMAX..] batch sums
  __shared__ float lg[NMAX];          // this row's logits, then its logits gradient
  __shared__ int last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x;
  // ---- logits (skinny_n_kernel's body)
  const float* a = p.x + (long)row * p.ldx;
  float acc[NMAX];
#pragma unroll
  for (int n = 0; n < NMAX; ++n) acc[n] = 0.f;
  const float* brow[NMAX];
#pragma unroll
  for (int n = 0; n < NMAX; ++n) brow[n] = p.w + (long)(n < p.O ? n : p.O - 1) * p.ldw;
#pragma unroll 4
  for (int k = threadIdx.x * 4; k < p.I; k += 1024) {
    const f32x4 av = *reinterpret_cast<const f32x4*>(a + k);
    f32x4 bv[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) bv[n] = *reinterpret_cast<const f32x4*>(brow[n] + k);
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
      acc[n] = fmaf(av[0], bv[n][0], fmaf(av[1], bv[n][1], fmaf(av[2], bv[n][2],
                                                                fmaf(av[3], bv[n][3], acc[n]))));
  }
#pragma unroll
  for (int n = 0; n < NMAX; ++n) {
    const float v = wave_sum(acc[n]);
    if (lane == 0) red[w][n] = v;
  }
  // the mean's denominator: valid labels of the whole batch (B <= 256: one per thread)
  float valid = 0.f;
  if ((int)threadIdx.x < p.B) {
    const int64_t y = p.labels[threadIdx.x];
    valid = (y != p.ignore_index && y >= 0 && y < p.O) ? 1.f : 0.f;
  }
  valid = wave_sum(valid);
  if (lane == 0) red[w][NMAX] = valid;
  // the input gradient's W rows (training), loaded now: their L2 round trip overlaps the
  // logits / loss math below instead of following it
  constexpr int kDxChunks = 2;  // column chunks of 4 per thread (I <= 2048 per workgroup)
  const bool do_dx = p.dpre && p.dx;
  const int span = (p.I / 4 + gridDim.y - 1) / gridDim.y * 4;
  const int c0 = blockIdx.y * span, c1 = min(p.I, c0 + span);
  f32x4 wv[kDxChunks][NMAX];
  if (do_dx) {
#pragma unroll
    for (int j = 0; j < kDxChunks; ++j) {
      const int col = min(c0 + (int)threadIdx.x * 4 + 1024 * j, p.I - 4);
#pragma unroll
      for (int k = 0; k < NMAX; ++k) wv[j][k] = *reinterpret_cast<const f32x4*>(brow[k] + col);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < p.O) {
    const int n = threadIdx.x;
    float v = red[0][n] + red[1][n] + red[2][n] + red[3][n];
    if (p.bias) v += p.bias[n];
    lg[n] = v;
    if (blockIdx.y == 0) p.logits[(long)row * p.O + n] = v;
  }
  __syncthreads();
  const float vd = red[0][NMAX] + red[1][NMAX] + red[2][NMAX] + red[3][NMAX];
  // ---- the row's loss terms and logits gradient (ce_fwd_kernel, one row per lane)
  if (threadIdx.x == 0) {
    const int64_t y = p.labels[row];
    const RowOut o = row_serial(lg, p.O, y, p.ignore_index, p.eps);
    if (blockIdx.y == 0) p.lse[row] = o.lse;
    if (p.dpre) {
      const float g = p.mean ? 1.f / vd : 1.f;
      const bool ok = o.valid != 0.f;
      float d[NMAX];
#pragma unroll
      for (int c = 0; c < NMAX; ++c) {
        float v = 0.f;
        if (c < p.O && ok) {
          const float pr = __expf(lg[c] - o.lse);
          v = g * (pr - (c == (int)y ? (1.f - p.eps) : 0.f) - p.eps / p.O);
        }
        d[c] = v;
      }
#pragma unroll
      for (int c = 0; c < NMAX; ++c) {
        if (c < p.O) {
          lg[c] = d[c];
          if (blockIdx.y == 0) p.dpre[(long)row * p.O + c] = d[c];
        }
      }
    }
    // per-row sums, handed to the last workgroup write-through (sc1)
    if (blockIdx.y == 0) {
      float* rb = p.rowbuf + 4L * row;
      __hip_atomic_store(rb + 0, o.loss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rb + 1, o.correct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rb + 2, o.valid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  // ---- the row's input gradient (head_bwd_kernel's dx workgroups: 4 adjacent columns per
  // thread, the O gradients of the row broadcast; same fmaf order), columns split over the
  // gridDim.y workgroups of the row. Every W row of a chunk is loaded up front (rows past O
  // clamped, their terms skipped): the chunk costs one L2 round trip, not O dependent ones.
  if (do_dx) {
#pragma unroll
    for (int j = 0; j < kDxChunks; ++j) {
      const int col = c0 + (int)threadIdx.x * 4 + 1024 * j;
      if (col >= c1) break;
      f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NMAX; ++k) {
        if (k < p.O) {
          const float gv = lg[k];
#pragma unroll
          for (int e = 0; e < 4; ++e) s4[e] = fmaf(gv, wv[j][k][e], s4[e]);
        }
      }
      if (p.gate) {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(p.gate + (long)row * p.ldgate + col);
#pragma unroll
        for (int e = 0; e < 4; ++e) s4[e] = gv[e] > 0.f ? s4[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(p.dx + (long)row * p.lddx + col) = s4;
      if (p.dxp) {
        typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
        unsigned h0, m0, l0, h1, m1, l1;
        split4_pair(s4[0], s4[1], h0, m0, l0);
        split4_pair(s4[2], s4[3], h1, m1, l1);
        uint16_t* o = p.dxp + (long)row * p.I + col;
        *reinterpret_cast<u32x2_*>(o) = u32x2_{h0, h1};
        *reinterpret_cast<u32x2_*>(o + p.dxps) = u32x2_{m0, m1};
        *reinterpret_cast<u32x2_*>(o + 2 * p.dxps) = u32x2_{l0, l1};
      }
    }
  }
  // ---- tickets: the row workgroups (blockIdx.y == 0, the ones that stored row values) arrive
  // on 8 shard counters (row % 8); each shard's last arrival adds to the global counter, whose
  // last arrival reduces the per-row values (one 255 -> 1 fan-in on one address costs ~3 us:
  // MI355X_MICROARCH.md "fanin")
  if (blockIdx.y != 0) return;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sc1 row stores have landed
    const int sh = row & 7;
    const unsigned n_sh = (unsigned)(p.B / 8 + (sh < p.B % 8 ? 1 : 0));
    const unsigned n_glob = (unsigned)(p.B < 8 ? p.B : 8);
    unsigned* tk = p.ticket + 1 + sh;
    int l = 0;
    if (__hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_sh - 1) {
      __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      l = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          n_glob - 1;
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  float ls = 0.f, cr = 0.f, vv = 0.f;
  if ((int)threadIdx.x < p.B) {
    const float* rb = p.rowbuf + 4L * threadIdx.x;
    ls = __hip_atomic_load(rb + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cr = __hip_atomic_load(rb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    vv = __hip_atomic_load(rb + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ls = wave_sum(ls);
  cr = wave_sum(cr);
  vv = wave_sum(vv);
  __syncthreads();  // every wave has read lg / red above: reuse red for the batch sums
  if (lane == 0) {
    red[w][0] = ls;
    red[w][1] = cr;
    red[w][2] = vv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ls = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    cr = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    vv = red[0][2] + red[1][2] + red[2][2] + red[3][2];
    if (p.loss) p.loss[0] = p.mean ? (vv > 0.f ? ls / vv : NAN) : ls;
    p.lse[p.B] = vv;
    if (p.acc) {
      p.acc[0] += ls;
      p.acc[1] += cr;
      p.acc[2] += vv;
    }
    __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

SkinnyParams params_of(const GemmF32Args& a) {
  SkinnyParams p;
  p.A = a.A; p.B = a.B; p.C = a.C; p.bias = a.bias; p.rowsum = a.rowsum;
  p.lda = a.lda; p.ldb = a.ldb; p.ldc = a.ldc;
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.beta = a.beta; p.rowsum_beta = a.rowsum_beta; p.relu = a.relu ? 1 : 0;
  p.gate = a.gate; p.ldg = a.ldgate;
  return p;
}

}  // namespace

int gemm_skinny_kind(const GemmF32Args& a) {
  if (a.mask || a.opt.kind != 0 || a.M <= 0 || a.N <= 0 || a.K <= 0) return 0;
  if (a.a_kcontig && a.b_kcontig && a.N <= kSkinnyMax && a.rowsum == nullptr &&
      a.K % 4 == 0 && al16(a.A) && al16(a.B) && a.lda % 4 == 0 && a.ldb % 4 == 0)
    return 1;
  if (a.a_kcontig && !a.b_kcontig && a.K <= kSkinnyMax && a.rowsum == nullptr &&
      a.N % 4 == 0 && al16(a.B) && al16(a.C) && a.ldb % 4 == 0 && a.ldc % 4 == 0 &&
      (a.bias == nullptr || al16(a.bias)))
    return 2;
  // skinny_m stages A (K x 8 or K x 16 floats) in LDS: keep it within the default 64 KiB
  if (!a.a_kcontig && !a.b_kcontig && a.M <= kSkinnyMax &&
      (long)a.K * (a.M <= 8 ? 8 : kSkinnyMax) * 4 <= 65536)
    return 3;
  return 0;
}

bool head_bwd(const float* g, long ldg, const float* x, long ldx, const float* w, long ldw,
              float* dx, long lddx, const float* gate, long ldgate, uint16_t* dxp, long dxps,
              float* dw, long lddw, float* db, int B, int O, int I, hipStream_t s,
              const OptEpilogue* wopt, const OptEpilogue* bopt) {
  if (O < 1 || O > kSkinnyMax || I % 4 || B < 1 || !al16(w) || (dx && !al16(dx)) || ldw % 4 ||
      lddx % 4 || (gate && (!al16(gate) || ldgate % 4)) || ((uintptr_t)dxp & 7) ||
      (long)B * (O <= 8 ? 8 : kSkinnyMax) * 4 > 65536)
    return false;
  HeadBwdParams p{g, x, w, dx, gate, dxp, dw, db, ldg, ldx, ldw, lddx, ldgate, dxps, lddw,
                  B, O, I, 0, OptEpilogue{}, OptEpilogue{}};
  if (wopt) p.wopt = *wopt;
  if (bopt && db) p.bopt = *bopt;
  const long threads = (long)B * (I / 4);
  // with the in-place update the weight workgroups compute dx themselves (kernel comment)
  // (dx == null: the input gradient exists already -- head_ce computed it in the forward)
  p.nb_dx = (p.wopt.kind || dx == nullptr) ? 0 : (int)((threads + 255) / 256);
  const int cw = p.wopt.kind ? kHeadColsOpt : kHeadCols;
  const int nb_dw = (I + cw - 1) / cw;
  // the 10-class heads get their own width (no FMAs on 6 padding classes)
  const int mm = O <= 8 ? 8 : O <= 10 ? 10 : kSkinnyMax;
  const size_t lds = sizeof(float) * (size_t)std::max(B * mm, mm * 256);
  const dim3 grid(p.nb_dx + nb_dw);
  auto launch = [&](auto cw_tag) {
    constexpr int CW = decltype(cw_tag)::value;
    if (mm == 8) hipLaunchKernelGGL((head_bwd_kernel<8, CW>), grid, dim3(256), lds, s, p);
    else if (mm == 10) hipLaunchKernelGGL((head_bwd_kernel<10, CW>), grid, dim3(256), lds, s, p);
    else hipLaunchKernelGGL((head_bwd_kernel<kSkinnyMax, CW>), grid, dim3(256), lds, s, p);
  };
  if (p.wopt.kind) launch(std::integral_constant<int, kHeadColsOpt>{});
  else launch(std::integral_constant<int, kHeadCols>{});
  return true;
}

bool head_ce(const float* x, long ldx, const float* w, long ldw, const float* bias,
             const int64_t* labels, int B, int O, int I, int ignore_index, float smoothing,
             bool mean, float* logits, float* lse, float* rowbuf, unsigned* ticket, float* loss,
             float* acc, float* dpre, float* dx, long lddx, const float* gate, long ldgate,
             uint16_t* dxp, long dxps, hipStream_t s) {
  if (O < 1 || O > kSkinnyMax || B < 1 || B > 256 || I % 4 || I < 4 || !al16(x) || !al16(w) ||
      ldx % 4 || ldw % 4 || (dx && (!al16(dx) || lddx % 4 || !dpre)) ||
      (gate && (!al16(gate) || ldgate % 4)) || ((uintptr_t)dxp & 7) || (dxp && !dx))
    return false;
  HeadCeParams p{x, w, bias, labels, logits, lse, rowbuf, ticket, loss, acc, dpre, dx, gate, dxp,
                 ldx, ldw, lddx, ldgate, dxps, B, O, I, ignore_index, mean ? 1 : 0, smoothing};
  // training: the row's input-gradient columns split over ys workgroups (each recomputes the
  // row's logits, a few us of L2 reads): B = 128 rows alone would leave half the CUs idle and
  // give every thread 4 dependent column chunks at I = 4096
  // (at most 2 chunks of 4 columns per thread: kDxChunks)
  const int ys = dx ? (int)((I + 2047) / 2048) : 1;
  const dim3 grid(B, ys);
  if (O <= 8) hipLaunchKernelGGL(head_ce_kernel<8>, grid, dim3(256), 0, s, p);
  else if (O <= 10) hipLaunchKernelGGL(head_ce_kernel<10>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(head_ce_kernel<kSkinnyMax>, grid, dim3(256), 0, s, p);
  return true;
}

void gemm_skinny_run(int kind, const GemmF32Args& a, hipStream_t s) {
  const SkinnyParams p = params_of(a);
  if (kind == 1) {
    if (a.N <= 8)
      hipLaunchKernelGGL(skinny_n_kernel<8>, dim3(a.M), dim3(256), 0, s, p);
    else if (a.N <= 10)  // the 10-class heads
      hipLaunchKernelGGL(skinny_n_kernel<10>, dim3(a.M), dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL(skinny_n_kernel<kSkinnyMax>, dim3(a.M), dim3(256), 0, s, p);
  } else if (kind == 2) {
    const long threads = (long)a.M * (a.N / 4);
    hipLaunchKernelGGL(skinny_k_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       p);
  } else {
    const int grid = (a.N + 63) / 64;
    const int mm = a.M <= 8 ? 8 : kSkinnyMax;
    const size_t lds = sizeof(float) * (size_t)std::max(a.K * mm, 4 * mm * 64);
    if (mm == 8)
      hipLaunchKernelGGL(skinny_m_kernel<8>, dim3(grid), dim3(256), lds, s, p);
    else
      hipLaunchKernelGGL(skinny_m_kernel<kSkinnyMax>, dim3(grid), dim3(256), lds, s, p);
  }
}

}  // namespace tdp
