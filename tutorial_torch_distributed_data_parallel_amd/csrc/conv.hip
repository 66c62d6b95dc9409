// Implicit-GEMM 2-D convolution (NCHW, fp32) on v_mfma_f32_32x32x2_f32: forward, input gradient
// and weight gradient, plus the NCHW bias/ReLU backward and pooling helpers.
//
// Replaces what the reference's AlexNet gets from MIOpen (SURVEY.md §2.3 N4, §2.5 K1/K4/K6-K8,
// K22; conv1-conv5 of torchvision AlexNet, REF/data_and_toy_model.py:41-45) and ResNet-50's convs.
// No im2col buffer is ever materialised: each GEMM operand element is gathered straight from the
// activation tensor while staging a K tile into LDS.
//   FWD   : C[co][(n,pq)]  = sum_(c,r,s)    W[co][c,r,s]   * x[n][c][p*sh-ph+r][q*sw-pw+s]
//   DGRAD : C[c][(n,hw)]   = sum_(co,r,s)   W[co][c][r][s] * dy[n][co][(h+ph-r)/sh][(w+pw-s)/sw]
//   WGRAD : C[co][(c,r,s)] = sum_(n,pq)     dy[n][co][pq]  * x[n][c][p*sh-ph+r][q*sw-pw+s]
// Every gathered B element is kpart(k) + npart(n), valid when the spatial coordinate
// (kh+nh, kw+nw) falls inside the source tensor; the (k, n) decompositions use multiply-shift
// division by precomputed magic numbers (no integer divide instructions in the loop).
// Structure: 256-thread workgroups, 4 waves (2x2), wave tile (32*FM)x(32*FN) as 32x32 MFMA
// tiles, BK = 32, register-staged double buffer (next tile's gathers issued before the current
// tile's MFMAs, one barrier per K step), A in LDS as [m][k] (+16 B pad; ds_read_b128 feeds four
// MFMAs with the permuted k = 8q+4h+s), B as [k][n] (ds_read_b32, conflict-free).
#include "common.h"
#include "conv.h"
#include "kernels.h"

namespace tdp {
namespace {

constexpr int kCT = 256;
constexpr int kCBK = 32;

struct ConvParams {
  const float* A;    // FWD/DGRAD: weights; WGRAD: dy (gradient of the conv output)
  const float* B;    // FWD/WGRAD: x; DGRAD: dy
  float* C;          // FWD: y; DGRAD: dx; WGRAD: dw (or split-K workspace)
  const float* bias;
  int M, N, K;       // GEMM view
  int Nimg, Cin, H, W, Cout, R, S, P, Q, sh, sw, ph, pw;
  FastDiv dRS, dS, dPQ, dQ, dHW, dW;
  int k_per_split, splits;
  int relu;
  float beta;
};

// ---- per-mode decompositions -------------------------------------------------------------
// A element address (always in range for m < M, k < K)
template <int MODE>
__device__ __forceinline__ long a_kpart(const ConvParams& p, int k) {
  if (MODE == kConvFwd) return k;                                   // W[co][k]
  if (MODE == kConvDgrad) {                                         // W[co][c][rs], k=(co,rs)
    const uint32_t co = fdiv(k, p.dRS);
    return (long)co * p.Cin * p.R * p.S + (k - co * p.dRS.d);
  }
  const uint32_t img = fdiv(k, p.dPQ);                              // dy[img][co][pq], k=(img,pq)
  return (long)img * p.Cout * p.P * p.Q + (k - img * p.dPQ.d);
}

template <int MODE>
__device__ __forceinline__ long a_mstride(const ConvParams& p) {
  if (MODE == kConvFwd) return p.K;
  if (MODE == kConvDgrad) return p.R * p.S;
  return (long)p.P * p.Q;
}

// B element: kpart + npart, valid if 0 <= kh+nh < HB and 0 <= kw+nw < WB
struct BPart {
  long off;
  int h, w;
};

template <int MODE>
__device__ __forceinline__ BPart b_kpart(const ConvParams& p, int k) {
  BPart b;
  if (MODE == kConvFwd) {  // k = (c, r, s)
    const uint32_t c = fdiv(k, p.dRS);
    const uint32_t rs = k - c * p.dRS.d;
    const uint32_t r = fdiv(rs, p.dS);
    const uint32_t s = rs - r * p.dS.d;
    b.h = r; b.w = s;
    b.off = (long)c * p.H * p.W + r * p.W + s;
  } else if (MODE == kConvDgrad) {  // k = (co, r, s); source dy[n][co][p][q]
    const uint32_t co = fdiv(k, p.dRS);
    const uint32_t rs = k - co * p.dRS.d;
    const uint32_t r = fdiv(rs, p.dS);
    const uint32_t s = rs - r * p.dS.d;
    b.h = -(int)r; b.w = -(int)s;
    b.off = (long)co * p.P * p.Q;  // the (p, q) part is added after the stride division
  } else {  // WGRAD: k = (img, p, q); source x
    const uint32_t img = fdiv(k, p.dPQ);
    const uint32_t pq = k - img * p.dPQ.d;
    const uint32_t pp = fdiv(pq, p.dQ);
    const uint32_t qq = pq - pp * p.dQ.d;
    b.h = (int)pp * p.sh - p.ph;
    b.w = (int)qq * p.sw - p.pw;
    b.off = (long)img * p.Cin * p.H * p.W + (long)b.h * p.W + b.w;
  }
  return b;
}

template <int MODE>
__device__ __forceinline__ BPart b_npart(const ConvParams& p, int n) {
  BPart b;
  if (MODE == kConvFwd) {  // n = (img, p, q)
    const uint32_t img = fdiv(n, p.dPQ);
    const uint32_t pq = n - img * p.dPQ.d;
    const uint32_t pp = fdiv(pq, p.dQ);
    const uint32_t qq = pq - pp * p.dQ.d;
    b.h = (int)pp * p.sh - p.ph;
    b.w = (int)qq * p.sw - p.pw;
    b.off = (long)img * p.Cin * p.H * p.W + (long)b.h * p.W + b.w;
  } else if (MODE == kConvDgrad) {  // n = (img, h, w) of dx
    const uint32_t img = fdiv(n, p.dHW);
    const uint32_t hw = n - img * p.dHW.d;
    const uint32_t hh = fdiv(hw, p.dW);
    const uint32_t ww = hw - hh * p.dW.d;
    b.h = (int)hh + p.ph;
    b.w = (int)ww + p.pw;
    b.off = (long)img * p.Cout * p.P * p.Q;
  } else {  // WGRAD: n = (c, r, s)
    const uint32_t c = fdiv(n, p.dRS);
    const uint32_t rs = n - c * p.dRS.d;
    const uint32_t r = fdiv(rs, p.dS);
    const uint32_t s = rs - r * p.dS.d;
    b.h = r; b.w = s;
    b.off = (long)c * p.H * p.W + r * p.W + s;
  }
  return b;
}

template <int MODE>
__device__ __forceinline__ float b_load(const ConvParams& p, const BPart& kp, const BPart& np) {
  int hh = kp.h + np.h, ww = kp.w + np.w;
  if (MODE == kConvDgrad) {
    // hh = h + ph - r must be a multiple of the stride; output row p = hh / sh
    if (p.sh > 1) {
      if (hh < 0 || (hh % p.sh) != 0) return 0.f;
      hh /= p.sh;
    }
    if (p.sw > 1) {
      if (ww < 0 || (ww % p.sw) != 0) return 0.f;
      ww /= p.sw;
    }
    if ((unsigned)hh >= (unsigned)p.P || (unsigned)ww >= (unsigned)p.Q) return 0.f;
    return p.B[kp.off + np.off + (long)hh * p.Q + ww];
  }
  if ((unsigned)hh >= (unsigned)p.H || (unsigned)ww >= (unsigned)p.W) return 0.f;
  return p.B[kp.off + np.off];
}

// epilogue address of output element (m, n)
template <int MODE>
__device__ __forceinline__ long c_colpart(const ConvParams& p, int n) {
  if (MODE == kConvWgrad) return n;
  if (MODE == kConvFwd) {
    const uint32_t img = fdiv(n, p.dPQ);
    return (long)img * p.Cout * p.P * p.Q + (n - img * p.dPQ.d);
  }
  const uint32_t img = fdiv(n, p.dHW);
  return (long)img * p.Cin * p.H * p.W + (n - img * p.dHW.d);
}

template <int MODE>
__device__ __forceinline__ long c_rowstride(const ConvParams& p) {
  if (MODE == kConvWgrad) return p.N;
  if (MODE == kConvFwd) return (long)p.P * p.Q;
  return (long)p.H * p.W;
}

template <int MODE, int FM, int FN>
__global__ __launch_bounds__(kCT) void conv_igemm_kernel(ConvParams p) {
  constexpr int BK = kCBK;
  constexpr int BM = 64 * FM, BN = 64 * FN;
  constexpr int A_LD = BK + 4;
  constexpr int A_SZ = BM * A_LD, B_SZ = BK * BN, STG = A_SZ + B_SZ;
  constexpr int AV = BM / 8;          // A elements per thread per tile (k fixed per thread)
  constexpr int BV = BK * BN / kCT;   // B elements per thread per tile (n fixed per thread)
  constexpr int B_KSTEP = kCT / BN;   // k rows covered per pass
  __shared__ __attribute__((aligned(16))) float smem[2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, z = blockIdx.z;
  const int kb = z * p.k_per_split;
  const int ke = min(p.K, kb + p.k_per_split);
  const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  // A staging: thread -> (k_local fixed, BM/8 rows)
  const int a_k = tid % 32, a_m0 = tid / 32;
  const long a_ms = a_mstride<MODE>(p);
  // B staging: thread -> (n_local fixed, BV k rows)
  const int b_n = tid % BN, b_k0 = tid / BN;
  const int gn = n0 + b_n;
  const bool n_ok = gn < p.N;
  const BPart np = b_npart<MODE>(p, n_ok ? gn : 0);

  float ra[AV], rb[BV];
  auto gload = [&](int k0) {
    const int ka = k0 + a_k;
    const bool ka_ok = ka < ke;
    const long ak = a_kpart<MODE>(p, ka_ok ? ka : kb);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int m = m0 + a_m0 + 8 * i;
      ra[i] = (ka_ok && m < p.M) ? p.A[ak + (long)m * a_ms] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int k = k0 + b_k0 + B_KSTEP * i;
      float v = 0.f;
      if (n_ok && k < ke) v = b_load<MODE>(p, b_kpart<MODE>(p, k), np);
      rb[i] = v;
    }
  };
  auto lstore = [&](float* st) {
#pragma unroll
    for (int i = 0; i < AV; ++i) st[(a_m0 + 8 * i) * A_LD + a_k] = ra[i];
    float* bs = st + A_SZ;
#pragma unroll
    for (int i = 0; i < BV; ++i) bs[(b_k0 + B_KSTEP * i) * BN + b_n] = rb[i];
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    gload(kb);
    lstore(smem);
    __syncthreads();
  }
  const int h = lane >> 5, l31 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const float* As = smem + (kt & 1) * STG;
    const float* Bs = As + A_SZ;
    if (kt + 1 < nk) gload(kb + (kt + 1) * BK);
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      const int kk = q * 8 + 4 * h;
      f32x4 a[FM];
      float b[FN][4];
#pragma unroll
      for (int f = 0; f < FM; ++f)
        a[f] = *reinterpret_cast<const f32x4*>(As + (wm * 32 * FM + f * 32 + l31) * A_LD + kk);
#pragma unroll
      for (int g = 0; g < FN; ++g)
#pragma unroll
        for (int s = 0; s < 4; ++s) b[g][s] = Bs[(kk + s) * BN + wn * 32 * FN + g * 32 + l31];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[f][s], b[g][s], acc[f][g], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(smem + ((kt + 1) & 1) * STG);
    __syncthreads();
  }

  const bool split = p.splits > 1;
  const long rstride = split ? p.N : c_rowstride<MODE>(p);
  float* out = split ? p.C + (long)z * p.M * p.N : p.C;
#pragma unroll
  for (int g = 0; g < FN; ++g) {
    const int col = n0 + wn * 32 * FN + g * 32 + l31;
    if (col >= p.N) continue;
    const long cp = split ? col : c_colpart<MODE>(p, col);
#pragma unroll
    for (int f = 0; f < FM; ++f) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 * FM + f * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        float v = acc[f][g][r];
        float* dst = out + cp + (long)row * rstride;
        if (!split) {
          if (p.bias) v += p.bias[row];
          if (p.beta != 0.f) v += p.beta * *dst;
          if (p.relu) v = fmaxf(v, 0.f);
        }
        *dst = v;
      }
    }
  }
}

template <int MODE>
void launch_mode(const ConvParams& p, int fm, int fn, dim3 grid, hipStream_t s) {
  if (fm == 1 && fn == 1) hipLaunchKernelGGL((conv_igemm_kernel<MODE, 1, 1>), grid, dim3(kCT), 0, s, p);
  else if (fm == 1) hipLaunchKernelGGL((conv_igemm_kernel<MODE, 1, 2>), grid, dim3(kCT), 0, s, p);
  else if (fn == 1) hipLaunchKernelGGL((conv_igemm_kernel<MODE, 2, 1>), grid, dim3(kCT), 0, s, p);
  else hipLaunchKernelGGL((conv_igemm_kernel<MODE, 2, 2>), grid, dim3(kCT), 0, s, p);
}

// ------------------------------------------------------------------------- NCHW helpers
// g = dy * (y > 0) (if y), db[c] = beta*db[c] + sum_{n,hw} g   (grid: C x splits)
__global__ __launch_bounds__(256) void chan_relu_bias_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ y,
                                                             int N, int C, int HW,
                                                             float* __restrict__ g,
                                                             float* __restrict__ part,
                                                             int splits) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  const long total = (long)N * HW;
  const long per = (total + splits - 1) / splits;
  const long b = (long)blockIdx.y * per, e = min(total, b + per);
  float s = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const long n = i / HW, hw = i - n * HW;
    const long off = (n * C + c) * HW + hw;
    float d = dy[off];
    if (y) {
      d = y[off] > 0.f ? d : 0.f;
      g[off] = d;
    }
    s += d;
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0 && part) part[(long)blockIdx.y * C + c] = s;
}

__global__ void chan_final_kernel(const float* __restrict__ part, int splits, int C,
                                  float* __restrict__ db, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float t = 0.f;
  for (int z = 0; z < splits; ++z) t += part[(long)z * C + c];
  db[c] = (beta != 0.f ? beta * db[c] : 0.f) + t;
}

}  // namespace

ConvPlan conv_plan(int mode, const ConvGeom& g, int num_cus) {
  ConvPlan pl;
  pl.mode = mode;
  if (mode == kConvFwd) { pl.M = g.Cout; pl.N = g.N * g.P * g.Q; pl.K = g.C * g.R * g.S; }
  else if (mode == kConvDgrad) { pl.M = g.C; pl.N = g.N * g.H * g.W; pl.K = g.Cout * g.R * g.S; }
  else { pl.M = g.Cout; pl.N = g.C * g.R * g.S; pl.K = g.N * g.P * g.Q; }
  pl.fm = pl.M <= 64 ? 1 : 2;
  pl.fn = pl.N <= 64 ? 1 : 2;
  const long tiles = (long)ceil_div(pl.M, 64 * pl.fm) * ceil_div(pl.N, 64 * pl.fn);
  int splits = 1;
  // only the weight gradient (output [Cout][C*R*S], reduction over every output pixel) splits K:
  // forward / input-gradient outputs are NCHW and their pixel dimension already fills the chip
  if (mode == kConvWgrad && tiles < 2L * num_cus) {
    const int want = (int)((2L * num_cus + tiles - 1) / tiles);
    const int kmax = pl.K / (kCBK * 8);
    splits = want < kmax ? want : kmax;
    if (splits < 1) splits = 1;
  }
  int kps = ceil_div(ceil_div(pl.K, splits), kCBK) * kCBK;
  pl.k_per_split = kps;
  pl.splits = ceil_div(pl.K, kps);
  pl.ws_floats = pl.splits > 1 ? (long)pl.splits * pl.M * pl.N : 0;
  return pl;
}

void conv_run(const ConvPlan& pl, const ConvGeom& g, const float* A, const float* B, float* C,
              const float* bias, bool relu, float beta, float* ws, hipStream_t s) {
  ConvParams p;
  p.A = A; p.B = B; p.C = pl.splits > 1 ? ws : C; p.bias = bias;
  p.M = pl.M; p.N = pl.N; p.K = pl.K;
  p.Nimg = g.N; p.Cin = g.C; p.H = g.H; p.W = g.W; p.Cout = g.Cout; p.R = g.R; p.S = g.S;
  p.P = g.P; p.Q = g.Q; p.sh = g.sh; p.sw = g.sw; p.ph = g.ph; p.pw = g.pw;
  p.dRS = make_fastdiv(g.R * g.S); p.dS = make_fastdiv(g.S);
  p.dPQ = make_fastdiv(g.P * g.Q); p.dQ = make_fastdiv(g.Q);
  p.dHW = make_fastdiv(g.H * g.W); p.dW = make_fastdiv(g.W);
  p.k_per_split = pl.k_per_split;
  p.splits = pl.splits;
  p.relu = relu ? 1 : 0;
  p.beta = beta;
  dim3 grid(ceil_div(pl.N, 64 * pl.fn), ceil_div(pl.M, 64 * pl.fm), pl.splits);
  if (pl.mode == kConvFwd) launch_mode<kConvFwd>(p, pl.fm, pl.fn, grid, s);
  else if (pl.mode == kConvDgrad) launch_mode<kConvDgrad>(p, pl.fm, pl.fn, grid, s);
  else launch_mode<kConvWgrad>(p, pl.fm, pl.fn, grid, s);
  if (pl.splits > 1) {
    // combine partials; for FWD/DGRAD the output is NCHW, not [M][N]: only WGRAD splits
    splitk_reduce(ws, pl.splits, pl.M, pl.N, C, false, pl.N, nullptr, beta, false, s);
  }
}

int chan_splits(int N, int C, int HW, int num_cus) {
  int sp = (2 * num_cus + C - 1) / C;
  const long cap = ((long)N * HW + 4095) / 4096;
  if (sp > cap) sp = (int)cap;
  return sp < 1 ? 1 : sp;
}

void chan_relu_bias_bwd(const float* dy, const float* y, int N, int C, int HW, float* g,
                        float* db, float beta, float* part, int splits, hipStream_t s) {
  hipLaunchKernelGGL(chan_relu_bias_kernel, dim3(C, splits), dim3(256), 0, s, dy, y, N, C, HW,
                     g, db ? part : nullptr, splits);
  if (db)
    hipLaunchKernelGGL(chan_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, splits,
                       C, db, beta);
}

}  // namespace tdp
