// Fast fp32 GEMM for gfx950: v_mfma_f32_32x32x2_f32 fed by a multi-stage LDS-DMA pipeline.
//
// Used for every aligned shape (contiguous dims % 4 == 0, 16-B aligned operands); gemm_f32.hip
// keeps a register-staged generic kernel for the rest. Structure (MI355X-specific choices):
//   * 256 threads = 4 waves (2x2); a wave owns 64 x 32*FN outputs as FM=2 x FN 32x32 MFMA tiles;
//     block tile 128 x 64*FN, K step BK = 32.
//   * Global -> LDS by global_load_lds_dwordx4 (no VGPR staging, no ds_write): S stages in flight,
//     one counted `s_waitcnt vmcnt` + one raw s_barrier per K step (guide §5 "Pipelining across
//     barriers"; __syncthreads would drain the DMA queue). All LDS lives in one dynamic array.
//   * K-contiguous tiles ([rows][32 floats], 128-B rows) are XOR-swizzled through the SOURCE
//     address (chunk c of row r lands in slot c ^ (r & 7)) since the DMA image is lane-linear;
//     fragments are read with ds_read_b128: lane half h of k-step (q, s) consumes k = 8q+4h+s,
//     so one b128 read feeds 4 MFMAs.
//   * MN-contiguous tiles ([32 k][cols], 512-B rows, conflict-free as is) are read with
//     ds_read_b64 covering two 32x32 tiles at once: tile f takes the interleaved rows/cols
//     2*i + f, so a lane's two operands are adjacent in memory. The epilogue undoes the
//     interleave (and stores float2 when the output columns are interleaved).
//   * Fragments for q+1 are read while the 16 MFMAs of q issue (register double-buffer), so one
//     wave per SIMD keeps the matrix pipe busy.
//   * Out-of-range rows/cols are clamped to valid addresses (they only feed discarded outputs);
//     the K tail is zeroed on the fragment read of the last tile.
//   * Block ids are remapped so the workgroups of one XCD share one split-K slice / row panel of
//     the operand every tile re-reads (L2 locality, guide §5.5 T1; bijective form).
//   * Implicit-GEMM convolution (NHWC activations) runs through the SAME pipeline: only the
//     per-lane DMA source addresses change. An "implicit" operand computes, per 16-B chunk, the
//     activation pixel + channel that GEMM element (row, k) reads (im2col for the forward pass,
//     its transpose-stride form for the input gradient, shifted pixels for the weight gradient);
//     taps that fall into the zero padding read a 16-B zero page. With C % 32 == 0 a K tile
//     never straddles a filter tap, so the tap decomposition is one scalar computation per tile.
#include <cstdlib>
#include <type_traits>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "conv.h"
#include "kernels.h"
#include "optim_elem.h"

namespace tdp {
namespace {

constexpr int kT = 256;
constexpr int kBK = 32;

// Geometry of an implicit (convolution) operand; the "row grid" is the pixel grid GEMM rows
// (FWD/DGRAD A) or GEMM k (WGRAD B) walk over, the source is the NHWC tensor being gathered.
struct ConvInfo {
  const float* zero;        // >= 16 B of zeros (padding taps)
  int Hs, Ws, Cs;           // source tensor dims
  int S, sh, sw, ph, pw;
  int shl, swl;             // log2 of the strides (DGRAD)
  int grid_pq, grid_q;      // row-grid pixels per image / per row
  int uniform;              // Cs % 32 == 0: one filter tap per K tile
  FastDiv dC, dS, dPQ, dQ;
};

// Input-gradient B read straight from the conv weight's [Cout][Rf][Sf][C] storage (the
// parameter's channels_last memory) -- no per-step transposed weight copy. GEMM row k =
// (tap t, co) with co fastest (the dy gather's k order); t = (rp, sp) walks the stride phase's
// Rp x Sp sub-grid of filter taps (r, s) = (r0 + rp*sh, s0 + sp*sw) (stride 1: the whole filter).
struct WTap {
  int Cout, Sp, r0, s0, sh, sw, Sf, C;
  long rs;      // weight row stride Rf*Sf*C
  int uniform;  // Cout % 32 == 0: a 32-deep K tile is one tap (decomposed once, wave-uniform)
  FastDiv dCout, dSp;
};

struct FastParams {
  ConvInfo cv;
  WTap wt;
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  float* rowsum;  // optional [M]: sum over K of A (bias gradient), only with an MN-contig A
  float* ws;
  long lda, ldb, ldc;
  int M, N, K;
  int k_per_split, splits;
  int tiles_n, tiles_m;
  float beta, rowsum_beta;
  int relu;
  int cvec;  // C (or the split-K workspace) takes 16-B row stores: N % 4 == 0, aligned rows
  float* stats;  // optional [tiles_m][3][N]: per-tile column (count, mean, M2) of the stored C
  OptEpilogue opt;  // kind != 0 (splits == 1 only): update p/state instead of storing C
  OptEpilogue bopt;  // kind != 0 (with opt and rowsum): update the bias from the row sums
  int prio;         // EMU: static wave priority for every other hardware slot (A/B knob)
  const float* gate;  // optional C-shaped gate (GemmF32Args::gate), non-split epilogues
  long ldg;
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef char lds_char;  // generic pointer into the dynamic LDS array (reads infer ds_read)
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---- fp32 GEMM on the bf16 matrix core (EMU kernels) ----------------------------------------
// gfx950 runs v_mfma_f32_32x32x2_f32 at 1/16 of the bf16 rate (64 vs 1024 FLOP/clk/SIMD). An
// fp32 operand splits EXACTLY into three bf16 terms x = x0 + x1 + x2 (x0 = RNE_bf16(x),
// x1 = RNE_bf16(x - x0), x2 = x - x0 - x1: 24 significand bits = 3 x 8, every subtraction exact),
// so a*b = sum_ij a_i b_j with the six terms of weight >= 2^-16 kept and a1b2 + a2b1 + a2b2
// (<= ~2^-24 |a||b|, the size of one fp32 rounding of the product) dropped. Each bf16 x bf16
// product is exact in the fp32 accumulator, so the result carries fp32 accuracy (error bound
// tested against fp64 next to the native f32 MFMA path: tests/test_gemm_emu_gpu.py) at 6 x 32
// instead of 8 x 64 cycles per 32x32x16 step: a 2.67x higher matrix-core ceiling. The split
// runs on the VALU from the SAME fp32 LDS fragments the f32 path reads (v_cvt_pk_bf16_f32 does
// the RNE pair conversion), and overlaps the previous step's MFMAs.
// K order: the bf16 MFMA gives lane half h the k-slots 8h..8h+7; the f32 fragment reads give
// lane half h the k = 8q + 4h + s (s < 4) of two consecutive q -- the same permutation for A and
// B, so the dot products are unchanged.
__device__ __forceinline__ void split3_pair(float x0, float x1, unsigned& h, unsigned& m,
                                            unsigned& l) {
  // scalar f32 subtractions (built with -fno-slp-vectorize: no v_pk_add_f32)
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x0, x1}, bf2));
  const float r0 = x0 - __uint_as_float(hu << 16), r1 = x1 - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf2));
  const float s0 = r0 - __uint_as_float(mu << 16), s1 = r1 - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{s0, s1}, bf2));
}
// 8 fp32 (two f32 k-steps of 4) -> three bf16x8 MFMA operands
__device__ __forceinline__ void split3_x8(const float (&x0)[4], const float (&x1)[4], bf8& h,
                                          bf8& m, bf8& l) {
  unsigned hs[4], ms[4], ls[4];
  split3_pair(x0[0], x0[1], hs[0], ms[0], ls[0]);
  split3_pair(x0[2], x0[3], hs[1], ms[1], ls[1]);
  split3_pair(x1[0], x1[1], hs[2], ms[2], ls[2]);
  split3_pair(x1[2], x1[3], hs[3], ms[3], ls[3]);
  const u32x4 hv = {hs[0], hs[1], hs[2], hs[3]};
  const u32x4 mv = {ms[0], ms[1], ms[2], ms[3]};
  const u32x4 lv = {ls[0], ls[1], ls[2], ls[3]};
  h = __builtin_bit_cast(bf8, hv);
  m = __builtin_bit_cast(bf8, mv);
  l = __builtin_bit_cast(bf8, lv);
}
// acc += a*b over the six kept split terms (smallest first)
__device__ __forceinline__ f32x16 mfma_emu6(const bf8& ah, const bf8& am, const bf8& al,
                                            const bf8& bh, const bf8& bm, const bf8& bl,
                                            f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  return acc;
}

// optimizer-epilogue variant flags, or-ed into the OPTK template argument next to the kind
constexpr int kOptWide = 4;  // wider HBM batches: register SGD both row tiles, LDS paths 2x loads
constexpr int kOptNT = 8;    // non-temporal p / state loads and stores
constexpr int kOptLds = 16;  // 128-wide paired tiles: gradient tile staged through LDS,
                             // float4 p / optimizer-state traffic (SGD and Adam)
constexpr int kOptG = 32;    // the lockstep kernel's math waves: the finished gradient tile goes
                             // to the LDS buffer after the stages (wgrad_lockstep_kernel), no update
constexpr int kOptPT = 64;   // with kOptNT | kOptLds (SGD, Adam): the updated parameters are stored with
                             // the default policy (momentum stays non-temporal), so the next
                             // forward's weight read can hit the 256 MiB Infinity Cache

template <bool NT>
__device__ __forceinline__ f32x2 ld_epi(const float* q) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(q));
  else return *reinterpret_cast<const f32x2*>(q);
}
template <bool NT>
__device__ __forceinline__ void st_epi(float* q, f32x2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(q));
  else *reinterpret_cast<f32x2*>(q) = v;
}

__device__ __forceinline__ void glds16(const float* src, lds_char* dst) {
  __builtin_amdgcn_global_load_lds(
      (const void*)src, (void __attribute__((address_space(3)))*)(
          (__attribute__((address_space(3))) char*)dst), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Row swizzle of K-contiguous tiles: slot(row, chunk) = chunk ^ swz(row). XOR-ing in row bits 3-5
// makes every 16-lane group of a ds_read_b128 (rows r..r+31 of one fragment) hit 16 distinct
// (row parity, slot) pairs = all 64 banks: conflict-free (plain `row & 7` left a 2-way conflict,
// SQ_LDS_BANK_CONFLICT = 4 cycles per read in the first profile).
__device__ __forceinline__ int swz(int row) { return (row ^ (row >> 3)) & 7; }

// Per-lane source pointers of one operand's share of a K tile, computed once per workgroup:
// only the k offset changes from tile to tile (clamped on the K tail).
template <int R, bool KC>
struct TileSrc {
  // K-contiguous [R][32] tile: CH = R/8 1-KiB chunks, CH/4 per wave
  // MN-contiguous [32][R] tile: CH = 32*R*4/1024 chunks, CH/4 per wave
  static constexpr int CH = KC ? R / 8 : (32 * R * 4) / 1024;
  static constexpr int NPW = CH / 4;
  const float* base[NPW];
  int koff[NPW];  // K-contig: k offset of the lane's 16-B chunk; MN: row (k) within the tile
  long ld;

  __device__ __forceinline__ void init(const float* g, long ld_, int r0, int rlim, int wid,
                                       int lane) {
    ld = ld_;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      if (KC) {
        const int row = j * 8 + (lane >> 3);
        int gr = r0 + row;
        gr = gr < rlim ? gr : rlim - 1;
        base[i] = g + (long)gr * ld;
        koff[i] = ((lane & 7) ^ swz(row)) * 4;
      } else {
        constexpr int LPR = R / 4;                 // lanes per 512-B row
        constexpr int RPC = 1024 / (R * 4);        // rows per chunk
        const int row = j * RPC + lane / LPR;
        int gc = r0 + (lane % LPR) * 4;
        gc = gc < rlim ? gc : rlim - 4;
        base[i] = g + gc;
        koff[i] = row;
      }
    }
  }

  __device__ __forceinline__ void issue(int k0, int klim, char* dst, int wid) const {
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      if (KC) {
        int gk = k0 + koff[i];
        gk = gk < klim ? gk : klim - 4;
        glds16(base[i] + gk, dst + j * 1024);
      } else {
        int gk = k0 + koff[i];
        gk = gk < klim ? gk : klim - 1;
        glds16(base[i] + (long)gk * ld, dst + j * 1024);
      }
    }
  }
};

// Operand source kinds
// (kImWgradT: the same shifted-pixel operand as kImWgrad, used as A of the transposed weight
// gradient dW^T[(r,s,c)][co] = x_shifted^T . dy when Cout is too small for a 128-row tile)
constexpr int kDenseK = 0, kDenseMN = 1, kImFwd = 2, kImDgrad = 3, kImWgrad = 4,
              kImWgradT = 5, kWTap = 6;

// Implicit K-contiguous A (rows = pixels of the row grid, k = (r, s, c) with c fastest):
//   FWD   : source x,  pixel (n, p, q), tap reads x[n][p*sh-ph+r][q*sw-pw+s][c]
//   DGRAD : source dy, pixel (n, h, w) of dx, tap reads dy[n][(h+ph-r)/sh][(w+pw-s)/sw][c]
//           (only when both divisions are exact; strides are powers of two)
template <int R, int MODE>
struct ImSrcA {
  static constexpr int NPW = R / 8 / 4;
  const float* img[NPW];
  int hb[NPW], wb[NPW], koff[NPW];

  __device__ __forceinline__ void init(const FastParams& p, int r0, int rlim, int wid,
                                       int lane) {
    const ConvInfo& cv = p.cv;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      const int row = j * 8 + (lane >> 3);
      int gr = r0 + row;
      gr = gr < rlim ? gr : rlim - 1;
      const uint32_t n = fdiv(gr, cv.dPQ);
      const uint32_t pq = gr - n * cv.grid_pq;
      const uint32_t y = fdiv(pq, cv.dQ);
      const uint32_t x = pq - y * cv.grid_q;
      img[i] = p.A + (long)n * cv.Hs * cv.Ws * cv.Cs;
      if (MODE == kImFwd) {
        hb[i] = (int)y * cv.sh - cv.ph;
        wb[i] = (int)x * cv.sw - cv.pw;
      } else {
        hb[i] = (int)y + cv.ph;
        wb[i] = (int)x + cv.pw;
      }
      koff[i] = ((lane & 7) ^ swz(row)) * 4;
    }
  }

  __device__ __forceinline__ void issue(const FastParams& p, int k0, int klim, char* dst,
                                        int wid) const {
    const ConvInfo& cv = p.cv;
    int ur = 0, us = 0, uc = 0;
    if (cv.uniform) {  // k0 is wave-uniform: scalar decomposition, one tap for the whole tile
      const uint32_t rs = fdiv(k0, cv.dC);
      uc = k0 - rs * cv.Cs;
      ur = fdiv(rs, cv.dS);
      us = rs - ur * cv.S;
    }
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      const int k = k0 + koff[i];
      int r, s, c;
      if (cv.uniform) {
        r = ur; s = us; c = uc + koff[i];
      } else {
        const uint32_t rs = fdiv(k, cv.dC);
        c = k - rs * cv.Cs;
        r = fdiv(rs, cv.dS);
        s = rs - r * cv.S;
      }
      bool ok = k < klim;
      int h, w;
      if (MODE == kImFwd) {
        h = hb[i] + r;
        w = wb[i] + s;
      } else {
        const int hh = hb[i] - r, ww = wb[i] - s;
        ok = ok && hh >= 0 && ww >= 0 && !(hh & ((1 << cv.shl) - 1)) &&
             !(ww & ((1 << cv.swl) - 1));
        h = hh >> cv.shl;
        w = ww >> cv.swl;
      }
      ok = ok && (unsigned)h < (unsigned)cv.Hs && (unsigned)w < (unsigned)cv.Ws;
      const float* src = ok ? img[i] + ((long)h * cv.Ws + w) * cv.Cs + c : cv.zero;
      glds16(src, dst + j * 1024);
    }
  }
};

// Implicit MN-contiguous B of the weight gradient: k = dy pixel (n, p, q), columns
// (r, s, c) with c fastest; element = x[n][p*sh-ph+r][q*sw-pw+s][c]. A lane's 4 columns share
// one tap (Cs % 4 == 0), fixed for the whole kernel; only the pixel changes per tile.
template <int R, bool IS_A = false>
struct ImSrcB {
  static constexpr int CH = (32 * R * 4) / 1024, NPW = CH / 4;
  static constexpr int LPR = R / 4, RPC = 1024 / (R * 4);
  int th, tw, coff;
  int koff[NPW];

  __device__ __forceinline__ void init(const FastParams& p, int r0, int rlim, int wid,
                                       int lane) {
    const ConvInfo& cv = p.cv;
    int gc = r0 + (lane % LPR) * 4;
    gc = gc < rlim ? gc : rlim - 4;
    const uint32_t rs = fdiv(gc, cv.dC);
    coff = gc - rs * cv.Cs;
    const int r = fdiv(rs, cv.dS);
    const int s = rs - r * cv.S;
    th = r - cv.ph;
    tw = s - cv.pw;
#pragma unroll
    for (int i = 0; i < NPW; ++i) koff[i] = (wid * NPW + i) * RPC + lane / LPR;
  }

  __device__ __forceinline__ void issue(const FastParams& p, int k0, int klim, char* dst,
                                        int wid) const {
    const ConvInfo& cv = p.cv;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      int gk = k0 + koff[i];
      gk = gk < klim ? gk : klim - 1;
      const uint32_t n = fdiv(gk, cv.dPQ);
      const uint32_t pq = gk - n * cv.grid_pq;
      const uint32_t y = fdiv(pq, cv.dQ);
      const uint32_t x = pq - y * cv.grid_q;
      const int h = (int)y * cv.sh + th, w = (int)x * cv.sw + tw;
      const bool ok = (unsigned)h < (unsigned)cv.Hs && (unsigned)w < (unsigned)cv.Ws;
      const float* src =
          ok ? (IS_A ? p.A : p.B) + (((long)n * cv.Hs + h) * cv.Ws + w) * cv.Cs + coff : cv.zero;
      glds16(src, dst + j * 1024);
    }
  }
};

// MN-contiguous B of the input gradient gathered from the weight storage (see WTap)
template <int R>
struct WTapSrc {
  static constexpr int CH = (32 * R * 4) / 1024, NPW = CH / 4;
  static constexpr int LPR = R / 4, RPC = 1024 / (R * 4);
  const float* base;
  int koff[NPW];

  __device__ __forceinline__ void init(const FastParams& p, int r0, int rlim, int wid,
                                       int lane) {
    int gc = r0 + (lane % LPR) * 4;
    gc = gc < rlim ? gc : rlim - 4;
    base = p.B + gc;
#pragma unroll
    for (int i = 0; i < NPW; ++i) koff[i] = (wid * NPW + i) * RPC + lane / LPR;
  }

  __device__ __forceinline__ void issue(const FastParams& p, int k0, int klim, char* dst,
                                        int wid) const {
    const WTap& w = p.wt;
    if (w.uniform) {
      // one tap for the whole tile (k0 is a multiple of 32, Cout of 32, K of 32): the tap and
      // the tile's first output channel are scalar; a lane only adds its row offset
      const uint32_t q = fdiv(k0, w.dCout);
      const int co0 = k0 - (int)q * w.Cout;
      const uint32_t rp = fdiv(q, w.dSp);
      const int sp = (int)q - (int)rp * w.Sp;
      const int tap = (w.r0 + (int)rp * w.sh) * w.Sf + w.s0 + sp * w.sw;
      const float* tb = base + (long)co0 * w.rs + (long)tap * w.C;
#pragma unroll
      for (int i = 0; i < NPW; ++i)
        glds16(tb + (long)koff[i] * w.rs, dst + (wid * NPW + i) * 1024);
      return;
    }
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int j = wid * NPW + i;
      int gk = k0 + koff[i];
      gk = gk < klim ? gk : klim - 1;
      const uint32_t q = fdiv(gk, w.dCout);
      const int co = gk - (int)q * w.Cout;
      const uint32_t rp = fdiv(q, w.dSp);
      const int sp = (int)q - (int)rp * w.Sp;
      const int tap = (w.r0 + (int)rp * w.sh) * w.Sf + w.s0 + sp * w.sw;
      glds16(base + (long)co * w.rs + (long)tap * w.C, dst + j * 1024);
    }
  }
};

template <int R, int KIND, bool IS_A>
struct SrcOf;
template <int R, bool IS_A>
struct SrcOf<R, kDenseK, IS_A> {
  TileSrc<R, true> t;
  __device__ __forceinline__ void init(const FastParams& p, int r0, int rlim, int wid, int lane) {
    t.init(IS_A ? p.A : p.B, IS_A ? p.lda : p.ldb, r0, rlim, wid, lane);
  }
  __device__ __forceinline__ void issue(const FastParams&, int k0, int klim, char* dst,
                                        int wid) const {
    t.issue(k0, klim, dst, wid);
  }
};
template <int R, bool IS_A>
struct SrcOf<R, kDenseMN, IS_A> {
  TileSrc<R, false> t;
  __device__ __forceinline__ void init(const FastParams& p, int r0, int rlim, int wid, int lane) {
    t.init(IS_A ? p.A : p.B, IS_A ? p.lda : p.ldb, r0, rlim, wid, lane);
  }
  __device__ __forceinline__ void issue(const FastParams&, int k0, int klim, char* dst,
                                        int wid) const {
    t.issue(k0, klim, dst, wid);
  }
};
template <int R>
struct SrcOf<R, kImFwd, true> : ImSrcA<R, kImFwd> {};
template <int R>
struct SrcOf<R, kImDgrad, true> : ImSrcA<R, kImDgrad> {};
template <int R>
struct SrcOf<R, kImWgrad, false> : ImSrcB<R, false> {};
template <int R>
struct SrcOf<R, kImWgradT, true> : ImSrcB<R, true> {};
template <int R>
struct SrcOf<R, kWTap, false> : WTapSrc<R> {};

// One output tile (logical id `lid`): the workgroup body of gemm_f32_fast_kernel.
// FM = 32-row MFMA tiles per wave (block rows BM = 64 * FM): 2, or 4 for a K-contiguous A (twice
// the MFMAs per barrier and per B fragment read, for the long-M convolution GEMMs).
template <int FN, int AKIND, int BKIND, int S, int OPTK, int FM, bool EMU>
__device__ __forceinline__ void gemm_tile(const FastParams& p, const int lid, lds_char* smem) {
  constexpr bool AK = AKIND != kDenseMN && AKIND != kImWgradT;
  constexpr bool BKC = BKIND == kDenseK;
  static_assert(FM == 2 || (FM == 4 && AK && OPTK == 0), "FM 4: K-contiguous A, plain epilogue");
  constexpr int BM = 64 * FM, BN = 64 * FN;
  constexpr int WR = 32 * FM;  // rows per wave
  constexpr int A_BYTES = BM * kBK * 4, B_BYTES = BN * kBK * 4;
  constexpr int STG = A_BYTES + B_BYTES;
  constexpr int GA = A_BYTES / 1024 / 4, GB = B_BYTES / 1024 / 4;  // glds per wave per tile
  constexpr int G = GA + GB;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_mn = p.tiles_n * p.tiles_m;
  const int z = lid / tiles_mn;
  const int t_mn = lid % tiles_mn;
  const int tm = t_mn / p.tiles_n, tn = t_mn % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kb = z * p.k_per_split;
  const int ke = min(p.K, kb + p.k_per_split);
  const int nk = (ke - kb + kBK - 1) / kBK;

  SrcOf<BM, AKIND, true> srcA;
  SrcOf<BN, BKIND, false> srcB;
  srcA.init(p, m0, p.M, wid, lane);
  srcB.init(p, n0, p.N, wid, lane);
  auto issue = [&](int t) {
    lds_char* st = smem + (t % S) * STG;
    const int k0 = kb + t * kBK;
    srcA.issue(p, k0, ke, st, wid);
    srcB.issue(p, k0, ke, st + A_BYTES, wid);
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t);

  const int h = lane >> 5, l31 = lane & 31;
  // per-lane LDS byte offsets of the fragment reads (within a stage)
  int a_off[FM], b_off[FN];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int row = wm * WR + f * 32 + l31;
    a_off[f] = AK ? row * 128 : (wm * 64 + 2 * l31) * 4;
  }
#pragma unroll
  for (int g = 0; g < FN; ++g) {
    const int row = wn * (32 * FN) + g * 32 + l31;
    // MN-contiguous B: FN == 2 interleaves the two tiles' columns (ds_read_b64), FN == 1 reads
    // the wave's 32 columns directly (ds_read_b32)
    b_off[g] = BKC ? A_BYTES + row * 128
                   : A_BYTES + (FN == 2 ? (wn * 64 + 2 * l31) * 4 : (wn * 32 + l31) * 4);
  }

  // fragment registers: value of tile f at k-step s of one q
  float av[2][FM][4], bv[2][FN][4];
  auto read_frag = [&](const lds_char* st, int q, float (&a)[FM][4], float (&bb)[FN][4]) {
    if (AK) {
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int row = wm * WR + f * 32 + l31;
        const int slot = (2 * q + h) ^ swz(row);
        const f32x4 v = *reinterpret_cast<const f32x4*>(st + a_off[f] + slot * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s) a[f][s] = v[s];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 8 * q + 4 * h + s;
        const f32x2 v = *reinterpret_cast<const f32x2*>(st + k * (BM * 4) + a_off[0]);
        a[0][s] = v[0];
        a[1][s] = v[1];
      }
    }
    if (BKC) {
#pragma unroll
      for (int g = 0; g < FN; ++g) {
        const int row = wn * (32 * FN) + g * 32 + l31;
        const int slot = (2 * q + h) ^ swz(row);
        const f32x4 v = *reinterpret_cast<const f32x4*>(st + b_off[g] + slot * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s) bb[g][s] = v[s];
      }
    } else if (FN == 2) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 8 * q + 4 * h + s;
        const f32x2 v = *reinterpret_cast<const f32x2*>(st + k * (BN * 4) + b_off[0]);
        bb[0][s] = v[0];
        bb[FN - 1][s] = v[1];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 8 * q + 4 * h + s;
        bb[0][s] = *reinterpret_cast<const float*>(st + k * (BN * 4) + b_off[0]);
      }
    }
  };

  // bias gradient: the workgroups of the first column tile also sum their A tiles over K
  const bool do_rs = !AK && p.rowsum != nullptr && tn == 0;
  float rs = 0.f;
  // K loop with the tail tile peeled: only the last tile can be partial, so every other
  // iteration is one branch-free basic block (no per-lane tail zeroing, no merge copies)
  auto ktile = [&](const int kt, auto tail_tag) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    wait_vmcnt<(S - 2) * G>();
    __builtin_amdgcn_s_barrier();
    issue(kt + S - 1);  // refill the stage every wave finished reading (kt - 1)
    const lds_char* st = smem + (kt % S) * STG;
    const int kvalid = ke - (kb + kt * kBK);  // < 32 only on the K tail
    if (do_rs && threadIdx.x < BM) {
      const int kmax = kvalid < kBK ? kvalid : kBK;
      for (int k = 0; k < kmax; ++k)
        rs += *reinterpret_cast<const float*>(st + k * (BM * 4) + threadIdx.x * 4);
    }
    if constexpr (EMU) {
      if (!TAIL || kvalid >= kBK) {
        // Full K tile, one basic block: split step 0 (exposed), then step 0's MFMAs with step 1's
        // split VALU requested in between (sched_group_barrier, 1 MFMA : ~6 VALU -- an in-order
        // wave's VALU only co-executes with MFMAs it issues in between them), then step 1's MFMAs
        // (the co-resident wave's split runs beside them). The scheduler honours the hint only in
        // part (ISA: most of the split still runs as blocks between MFMA runs); the measured
        // levers were the scalar subtractions, the peeled tail and the static priority
        // (profiles/micro/gemm_emu_pmc_r4.md, gemm_emu_prio_ab_r4l.txt).
        constexpr int NF = FM + FN, NB = FM * FN;
        // register budget (two waves per SIMD: <= 256 VGPR + AGPR): step 1's fp32 fragments are
        // read only after step 0's are split (dead)
        float a4[4][FM][4], b4[4][FN][4];
        bf8 xh[2][NF], xm[2][NF], xl[2][NF];  // fragment i: A tile i (< FM) or B tile i - FM
        auto split_frag = [&](int j, int i) {
          if (i < FM) split3_x8(a4[2 * j][i], a4[2 * j + 1][i], xh[j][i], xm[j][i], xl[j][i]);
          else split3_x8(b4[2 * j][i - FM], b4[2 * j + 1][i - FM], xh[j][i], xm[j][i], xl[j][i]);
        };
        read_frag(st, 0, a4[0], b4[0]);
        read_frag(st, 1, a4[1], b4[1]);
#pragma unroll
        for (int i = 0; i < NF; ++i) split_frag(0, i);
        __builtin_amdgcn_sched_barrier(0);
        read_frag(st, 2, a4[2], b4[2]);
        read_frag(st, 3, a4[3], b4[3]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < NB; ++c) {
          const int f = c / FN, g = c % FN;
          acc[f][g] = mfma_emu6(xh[0][f], xm[0][f], xl[0][f], xh[0][FM + g], xm[0][FM + g],
                                xl[0][FM + g], acc[f][g]);
#pragma unroll
          for (int i = c; i < NF; i += NB) split_frag(1, i);
          // 36 VALU per split fragment (4 pairs x 9), spread over the chunk's 6 MFMAs; chunk 0
          // carries two fragments when NF > NB
          if (c == 0 && NF > NB) {
#pragma unroll
            for (int u = 0; u < 6; ++u) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);
            }
          } else {
#pragma unroll
            for (int u = 0; u < 6; ++u) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = mfma_emu6(xh[1][f], xm[1][f], xl[1][f], xh[1][FM + g], xm[1][FM + g],
                                  xl[1][FM + g], acc[f][g]);
        return;
      }
      // K tail: two bf16 K16 steps, q pair (2j, 2j+1) feeds one 32x32x16 step
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        read_frag(st, 2 * j, av[0], bv[0]);
        read_frag(st, 2 * j + 1, av[1], bv[1]);
        if (TAIL && kvalid < kBK) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              if (8 * (2 * j + u) + 4 * h + s >= kvalid) {
#pragma unroll
                for (int f = 0; f < FM; ++f) av[u][f][s] = 0.f;
#pragma unroll
                for (int g = 0; g < FN; ++g) bv[u][g][s] = 0.f;
              }
            }
        }
        bf8 ah[FM], am[FM], al[FM], bh[FN], bm[FN], bl[FN];
#pragma unroll
        for (int f = 0; f < FM; ++f) split3_x8(av[0][f], av[1][f], ah[f], am[f], al[f]);
#pragma unroll
        for (int g = 0; g < FN; ++g) split3_x8(bv[0][g], bv[1][g], bh[g], bm[g], bl[g]);
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = mfma_emu6(ah[f], am[f], al[f], bh[g], bm[g], bl[g], acc[f][g]);
      }
      return;
    }
    read_frag(st, 0, av[0], bv[0]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < 3) read_frag(st, q + 1, av[(q + 1) & 1], bv[(q + 1) & 1]);
      float (&a)[FM][4] = av[q & 1];
      float (&bb)[FN][4] = bv[q & 1];
      if (TAIL && kvalid < kBK) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if (8 * q + 4 * h + s >= kvalid) {
#pragma unroll
            for (int f = 0; f < FM; ++f) a[f][s] = 0.f;
#pragma unroll
            for (int g = 0; g < FN; ++g) bb[g][s] = 0.f;
          }
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[f][s], bb[g][s], acc[f][g], 0, 0,
                                                             0);
    }
  };
  for (int kt = 0; kt < nk - 1; ++kt) ktile(kt, std::false_type{});
  if (nk > 0) ktile(nk - 1, std::true_type{});
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup
  if (do_rs && threadIdx.x < BM && m0 + (int)threadIdx.x < p.M) {
    const int m = m0 + threadIdx.x;
    if (OPTK != 0 && p.bopt.kind != 0) {
      // the bias gradient is complete here (K = the whole batch): update the bias in place
      // (same optimizer and hyper block as the weight) instead of storing the gradient
      OptEpilogue o = p.opt;
      if constexpr ((OPTK & 3) == 1) {
        load_hyper(o.sgd);
        float pe = p.bopt.p[m];
        float b = (o.sgd.momentum != 0.f && !o.sgd.first_step) ? p.bopt.s0[m] : 0.f;
        sgd_elem(pe, rs, b, o.sgd);
        p.bopt.p[m] = pe;
        if (o.sgd.momentum != 0.f) p.bopt.s0[m] = b;
      } else if constexpr ((OPTK & 3) == 2) {
        load_hyper(o.adam);
        float pe = p.bopt.p[m], mm = p.bopt.s0[m], vv = p.bopt.s1[m];
        adam_elem(pe, rs, mm, vv, p.bopt.s2 ? p.bopt.s2 + m : nullptr, o.adam);
        p.bopt.p[m] = pe;
        p.bopt.s0[m] = mm;
        p.bopt.s1[m] = vv;
      }
    } else {
      float* d = p.rowsum + m;
      *d = (p.rowsum_beta != 0.f ? p.rowsum_beta * *d : 0.f) + rs;
    }
  }

  // epilogue
  const bool split = p.splits > 1;
  if (OPTK != 0) {
    // optimizer epilogue (no split-K by construction): C is a weight gradient; update the
    // parameter and its optimizer state at C's index instead of storing C. The epilogue is
    // latency-bound (each element is read, updated, written back), so every p / state load of a
    // batch is issued before the first update: one HBM round trip per batch. A batch is the whole
    // FM x 16 x FN accumulator set for FN == 1, one row tile (16 adjacent column pairs) for
    // FN == 2. With interleaved MN-contiguous B (FN == 2) a lane owns two ADJACENT columns, read
    // and written as float2 (two half-sector stores per line would force partial write-backs).
    // Offsets are 32-bit (a parameter has < 2^31 elements; checked on the host).
    // OPTK = kind (1 SGD, 2 Adam) | kOptWide (PAIR SGD: both row tiles in one batch, one HBM
    // round trip per tile) | kOptNT (non-temporal p / state traffic: touched once per step, so it
    // should not evict the L2-resident dY / X operand tiles)
    if constexpr ((OPTK & kOptG) != 0) {
      // lockstep kernel: the stream waves read the previous tile's gradient from G until the
      // first barrier here; the second publishes this tile's. Two barriers, always (the stream
      // waves count them).
      static_assert(FN == 2 && FM == 2 && !AK && !BKC, "kOptG: the 128 x 128 MN x MN tile");
      float* G = reinterpret_cast<float*>(smem + S * STG);
      __syncthreads();
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int lr = wm * 64 + 2 * rl + f;
          *reinterpret_cast<f32x2*>(G + lr * BN + wn * 64 + 2 * l31) =
              f32x2{acc[f][0][r], acc[f][FN - 1][r]};
        }
      __syncthreads();
      return;
    }
    constexpr bool SGD = (OPTK & 3) == 1;
    constexpr bool NT = (OPTK & kOptNT) != 0;
    // per-step scalars from the device hyper block (graph-replay safe, kernels.h HyperSlot)
    OptEpilogue o = p.opt;
    if constexpr (SGD) load_hyper(o.sgd);
    else load_hyper(o.adam);
    const bool mom_rd = SGD && o.sgd.momentum != 0.f && !o.sgd.first_step;
    const bool mom_wr = SGD && o.sgd.momentum != 0.f;
    constexpr bool PAIR = !BKC && FN == 2;
    constexpr int NG = PAIR ? 1 : FN;       // column groups per accumulator row
    constexpr int NE = PAIR ? 2 : 1;        // elements per group
    if constexpr (SGD && PAIR && !AK && (OPTK & kOptLds) != 0) {
      // kOptLds: stage the 128 x 128 gradient tile through LDS (the pipeline stages are free
      // once every wave has left the K loop) so each p / momentum access is a 16-B-per-lane,
      // 512-B-per-row coalesced float4 (the MFMA layout alone gives lanes column PAIRS).
      static_assert(BM * BN * 4 <= S * STG, "gradient tile must fit in the LDS stages");
      float* T = reinterpret_cast<float*>(smem);
      __syncthreads();  // every wave is done reading the last K stage
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int lr = wm * 64 + 2 * rl + f;
          *reinterpret_cast<f32x2*>(T + lr * BN + wn * 64 + 2 * l31) =
              f32x2{acc[f][0][r], acc[f][FN - 1][r]};
        }
      __syncthreads();
      constexpr int C4 = BN / 4;                  // float4 per tile row
      constexpr int IT = BM * C4 / kT;            // float4 per thread (16)
      // float4 per batch (one HBM round trip); kOptWide: the whole tile's p / momentum loads in
      // flight at once (128 VGPRs: the K loop's fragments are dead here)
      constexpr int HB = (OPTK & kOptWide) != 0 ? IT : 8;
#pragma unroll
      for (int i0 = 0; i0 < IT; i0 += HB) {
        int gi[HB];
        f32x4 pv4[HB], mv4[HB];
#pragma unroll
        for (int i = 0; i < HB; ++i) {
          const int e = (i0 + i) * kT + threadIdx.x;
          const int row = m0 + e / C4, col = n0 + (e % C4) * 4;
          gi[i] = (row < p.M && col < p.N) ? row * (int)p.ldc + col : -1;
          const int q = gi[i] < 0 ? 0 : gi[i];
          if constexpr (NT) {
            pv4[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.p + q));
            if (mom_rd) mv4[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s0 + q));
          } else {
            pv4[i] = *reinterpret_cast<const f32x4*>(o.p + q);
            if (mom_rd) mv4[i] = *reinterpret_cast<const f32x4*>(o.s0 + q);
          }
        }
#pragma unroll
        for (int i = 0; i < HB; ++i) {
          if (gi[i] < 0) continue;
          const int e = (i0 + i) * kT + threadIdx.x;
          const f32x4 g4 = *reinterpret_cast<const f32x4*>(T + (e / C4) * BN + (e % C4) * 4);
          f32x4 pe = pv4[i], be = mom_rd ? mv4[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float pc = pe[c], bc = be[c];
            sgd_elem(pc, g4[c], bc, o.sgd);
            pe[c] = pc;
            be[c] = bc;
          }
          if constexpr (NT) {
            if constexpr ((OPTK & kOptPT) != 0) *reinterpret_cast<f32x4*>(o.p + gi[i]) = pe;
            else __builtin_nontemporal_store(pe, reinterpret_cast<f32x4*>(o.p + gi[i]));
            if (mom_wr) __builtin_nontemporal_store(be, reinterpret_cast<f32x4*>(o.s0 + gi[i]));
          } else {
            *reinterpret_cast<f32x4*>(o.p + gi[i]) = pe;
            if (mom_wr) *reinterpret_cast<f32x4*>(o.s0 + gi[i]) = be;
          }
        }
      }
      return;  // the persistent loop's barrier protects T before the next tile's DMA
    }
    if constexpr (!SGD && PAIR && !AK && (OPTK & kOptLds) != 0) {
      // the same LDS staging for Adam: p, exp_avg, exp_avg_sq as float4 rows (4 per batch)
      static_assert(BM * BN * 4 <= S * STG, "gradient tile must fit in the LDS stages");
      float* T = reinterpret_cast<float*>(smem);
      __syncthreads();
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int lr = wm * 64 + 2 * rl + f;
          *reinterpret_cast<f32x2*>(T + lr * BN + wn * 64 + 2 * l31) =
              f32x2{acc[f][0][r], acc[f][FN - 1][r]};
        }
      __syncthreads();
      constexpr int C4 = BN / 4;
      constexpr int IT = BM * C4 / kT;
      constexpr int HB = (OPTK & kOptWide) != 0 ? 8 : 4;  // kOptWide: twice the loads in flight
#pragma unroll
      for (int i0 = 0; i0 < IT; i0 += HB) {
        int gi[HB];
        f32x4 pv4[HB], mv4[HB], vv4[HB];
#pragma unroll
        for (int i = 0; i < HB; ++i) {
          const int e = (i0 + i) * kT + threadIdx.x;
          const int row = m0 + e / C4, col = n0 + (e % C4) * 4;
          gi[i] = (row < p.M && col < p.N) ? row * (int)p.ldc + col : -1;
          const int q = gi[i] < 0 ? 0 : gi[i];
          if constexpr (NT) {
            pv4[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.p + q));
            mv4[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s0 + q));
            vv4[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(o.s1 + q));
          } else {
            pv4[i] = *reinterpret_cast<const f32x4*>(o.p + q);
            mv4[i] = *reinterpret_cast<const f32x4*>(o.s0 + q);
            vv4[i] = *reinterpret_cast<const f32x4*>(o.s1 + q);
          }
        }
#pragma unroll
        for (int i = 0; i < HB; ++i) {
          if (gi[i] < 0) continue;
          const int e = (i0 + i) * kT + threadIdx.x;
          const f32x4 g4 = *reinterpret_cast<const f32x4*>(T + (e / C4) * BN + (e % C4) * 4);
          f32x4 pe = pv4[i], me = mv4[i], ve = vv4[i];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float pc = pe[c], mc = me[c], vc = ve[c];
            adam_elem(pc, g4[c], mc, vc, o.s2 ? o.s2 + gi[i] + c : nullptr, o.adam);
            pe[c] = pc;
            me[c] = mc;
            ve[c] = vc;
          }
          if constexpr (NT) {
            if constexpr ((OPTK & kOptPT) != 0) *reinterpret_cast<f32x4*>(o.p + gi[i]) = pe;
            else __builtin_nontemporal_store(pe, reinterpret_cast<f32x4*>(o.p + gi[i]));
            __builtin_nontemporal_store(me, reinterpret_cast<f32x4*>(o.s0 + gi[i]));
            __builtin_nontemporal_store(ve, reinterpret_cast<f32x4*>(o.s1 + gi[i]));
          } else {
            *reinterpret_cast<f32x4*>(o.p + gi[i]) = pe;
            *reinterpret_cast<f32x4*>(o.s0 + gi[i]) = me;
            *reinterpret_cast<f32x4*>(o.s1 + gi[i]) = ve;
          }
        }
      }
      return;
    }
    constexpr bool WIDE = SGD && (OPTK & kOptWide) != 0;
    constexpr int FB = PAIR ? (WIDE ? FM : 1) : (SGD ? FM : 1);  // row tiles per batch
    constexpr int RB = (PAIR && !SGD) ? 8 : 16;    // accumulator rows per batch (Adam: 3 arrays)
    constexpr int NB = FB * RB * NG;        // groups per batch
#pragma unroll
    for (int f0 = 0; f0 < FM; f0 += FB) {
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += RB) {
      int idx[NB];
      float pv[NB * NE], s0v[NB * NE], s1v[SGD ? 1 : NB * NE];
#pragma unroll
      for (int fb = 0; fb < FB; ++fb) {
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
          const int f = f0 + fb, r = r0 + rr;
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int row = m0 + wm * WR + (AK ? f * 32 + rl : 2 * rl + f);
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            const int col = PAIR ? n0 + wn * 64 + 2 * l31 : n0 + wn * (32 * FN) + g * 32 + l31;
            const int j = (fb * RB + rr) * NG + g;
            // PAIR: N % 4 == 0 (fast-path precondition), so col + 1 < N whenever col < N;
            // out-of-range lanes are marked by idx = -1 (and read element 0)
            const bool ok = row < p.M && col < p.N;
            idx[j] = ok ? row * (int)p.ldc + col : -1;
            const int i = ok ? idx[j] : 0;
            if (PAIR) {
              const f32x2 v = ld_epi<NT>(o.p + i);
              pv[2 * j] = v[0]; pv[2 * j + 1] = v[1];
              if (!SGD || mom_rd) {
                const f32x2 w = ld_epi<NT>(o.s0 + i);
                s0v[2 * j] = w[0]; s0v[2 * j + 1] = w[1];
              }
              if (!SGD) {
                const f32x2 u = ld_epi<NT>(o.s1 + i);
                s1v[2 * j] = u[0]; s1v[2 * j + 1] = u[1];
              }
            } else {
              pv[j] = o.p[i];
              if (!SGD || mom_rd) s0v[j] = o.s0[i];
              if (!SGD) s1v[j] = o.s1[i];
            }
          }
        }
      }
#pragma unroll
      for (int fb = 0; fb < FB; ++fb) {
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            const int j = (fb * RB + rr) * NG + g;
            const int i = idx[j];
            if (i < 0) continue;
#pragma unroll
            for (int e = 0; e < NE; ++e) {
              const float gr = acc[f0 + fb][PAIR ? e : g][r0 + rr];
              float pe = pv[j * NE + e];
              float b0 = (!SGD || mom_rd) ? s0v[j * NE + e] : 0.f;
              if (SGD) {
                sgd_elem(pe, gr, b0, o.sgd);
              } else {
                float b1 = s1v[j * NE + e];
                adam_elem(pe, gr, b0, b1, o.s2 ? o.s2 + i + e : nullptr, o.adam);
                s1v[j * NE + e] = b1;
              }
              pv[j * NE + e] = pe;
              s0v[j * NE + e] = b0;
            }
            if (PAIR) {
              st_epi<NT>(o.p + i, f32x2{pv[2 * j], pv[2 * j + 1]});
              if (!SGD || mom_wr) st_epi<NT>(o.s0 + i, f32x2{s0v[2 * j], s0v[2 * j + 1]});
              if (!SGD) st_epi<NT>(o.s1 + i, f32x2{s1v[2 * j], s1v[2 * j + 1]});
            } else {
              o.p[i] = pv[j];
              if (!SGD || mom_wr) o.s0[i] = s0v[j];
              if (!SGD) o.s1[i] = s1v[j];
            }
          }
        }
      }
      }
    }
    return;
  }
  float* out = split ? p.ws + (long)z * p.M * p.N : p.C;
  const long ldo = split ? p.N : p.ldc;
  if (BM * BN * 4 <= S * STG && p.cvec) {
    // Row-vector store: the tile goes through LDS (the pipeline stages are free once every wave
    // has left the K loop) and leaves as 16-B-per-lane row segments. The accumulator layout
    // alone gives each lane one column (or a column pair) of 16 rows: dword stores, 4x the
    // store instructions, and the store tail is issue-bound (an output-heavy GEMM such as a 1x1
    // convolution with K = 64 spent most of its time there).
    constexpr int PAD = (BM * (BN + 8) * 4 <= S * STG) ? 8 : 0;  // 4-row offset = 32 banks
    constexpr int TS = BN + PAD;
    float* T = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is done reading the last K stage
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int lr = wm * WR + (AK ? f * 32 + rl : 2 * rl + f);
        if (BKC || FN == 1) {
#pragma unroll
          for (int g = 0; g < FN; ++g) T[lr * TS + wn * (32 * FN) + g * 32 + l31] = acc[f][g][r];
        } else {
          *reinterpret_cast<f32x2*>(T + lr * TS + wn * 64 + 2 * l31) =
              f32x2{acc[f][0][r], acc[f][FN - 1][r]};
        }
      }
    __syncthreads();
    constexpr int C4 = BN / 4;          // float4 per tile row
    constexpr int IT = BM * C4 / kT;    // float4 per thread (8 or 16)
    constexpr int HB = 8;               // C loads in flight per batch (beta != 0)
    const bool rmw = !split && p.beta != 0.f;
#pragma unroll
    for (int i0 = 0; i0 < IT; i0 += HB) {
      f32x4 cold[HB];
      if (rmw) {
#pragma unroll
        for (int i = 0; i < HB; ++i) {
          const int e = (i0 + i) * kT + threadIdx.x;
          const int row = m0 + e / C4, col = n0 + (e % C4) * 4;
          const bool ok = row < p.M && col < p.N;
          cold[i] = *reinterpret_cast<const f32x4*>(out + (ok ? row * ldo + col : 0));
        }
      }
#pragma unroll
      for (int i = 0; i < HB; ++i) {
        const int e = (i0 + i) * kT + threadIdx.x;
        const int lr = e / C4, lc = (e % C4) * 4;
        const int row = m0 + lr, col = n0 + lc;
        if (row >= p.M || col >= p.N) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(T + lr * TS + lc);
        if (!split) {
          if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + col);
          if (rmw) v += p.beta * cold[i];
          if (p.relu) {
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
          }
          if (p.gate) {
            const f32x4 gv = *reinterpret_cast<const f32x4*>(p.gate + row * p.ldg + col);
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = gv[c] > 0.f ? v[c] : 0.f;
          }
        }
        *reinterpret_cast<f32x4*>(out + row * ldo + col) = v;
      }
    }
    if (p.stats != nullptr && !split) {
      // Batch-norm statistics of this tile's columns, from the tile still in LDS (a convolution
      // whose output feeds a BatchNorm: the moments pass over the whole output is skipped).
      // Shifted sums about the tile's first row keep the one-pass variance exact in practice
      // (the deviations are O(std)); tiles merge with Chan's formula (bn_moments_partials).
      const int lc = (threadIdx.x % C4) * 4;
      const f32x4 k4 = *reinterpret_cast<const f32x4*>(T + lc);
      f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int lr = (i * kT + threadIdx.x) / C4;
        if (m0 + lr < p.M) {
          const f32x4 d = *reinterpret_cast<const f32x4*>(T + lr * TS + lc) - k4;
          s1 += d;
          s2 += d * d;
        }
      }
      __syncthreads();  // every T read is done: the LDS becomes the cross-thread scratch
      float* R = T;
      *reinterpret_cast<f32x4*>(R + threadIdx.x * 12) = s1;
      *reinterpret_cast<f32x4*>(R + threadIdx.x * 12 + 4) = s2;
      *reinterpret_cast<f32x4*>(R + threadIdx.x * 12 + 8) = k4;
      __syncthreads();
      constexpr int GRP = kT / C4;  // threads sharing a column quad
      const float n = (float)min(BM, p.M - m0);
      for (int c = threadIdx.x; c < BN; c += kT) {
        const int q = c >> 2, j = c & 3, col = n0 + c;
        if (col >= p.N) continue;
        float a = 0.f, b = 0.f;
#pragma unroll 4
        for (int g = 0; g < GRP; ++g) {
          a += R[(g * C4 + q) * 12 + j];
          b += R[(g * C4 + q) * 12 + 4 + j];
        }
        const float mean_d = a / n;
        float* o = p.stats + (long)(m0 / BM) * 3 * p.N;
        o[col] = n;
        o[p.N + col] = R[q * 12 + 8 + j] + mean_d;
        o[2 * p.N + col] = fmaxf(b - a * mean_d, 0.f);
      }
    }
    return;  // a persistent loop's barrier protects T before the next tile's DMA
  }
  // beta != 0 reads C: all 16 rows of an f-slab are loaded before any store, so the loads are
  // in flight together (interleaved with the stores to `out` they would serialise on the
  // possible aliasing: one memory round trip per row)
  const bool rmw = !split && p.beta != 0.f;
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    float cold[16][2];
    if (rmw) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int row = m0 + wm * WR + (AK ? f * 32 + rl : 2 * rl + f);
        const float* orow = out + (long)(row < p.M ? row : 0) * ldo;
        if (BKC || FN == 1) {
#pragma unroll
          for (int g = 0; g < FN; ++g) {
            const int col = n0 + wn * (32 * FN) + g * 32 + l31;
            cold[r][g] = (row < p.M && col < p.N) ? orow[col] : 0.f;
          }
        } else {
          const int col = n0 + wn * 64 + 2 * l31;
          if (row < p.M && col + 1 < p.N) {
            const f32x2 o = *reinterpret_cast<const f32x2*>(orow + col);
            cold[r][0] = o[0];
            cold[r][1] = o[1];
          } else {
            cold[r][0] = (row < p.M && col < p.N) ? orow[col] : 0.f;
            cold[r][1] = 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int row = m0 + wm * WR + (AK ? f * 32 + rl : 2 * rl + f);
      if (row >= p.M) continue;
      float* orow = out + (long)row * ldo;
      if (BKC || FN == 1) {
#pragma unroll
        for (int g = 0; g < FN; ++g) {
          const int col = n0 + wn * (32 * FN) + g * 32 + l31;
          if (col >= p.N) continue;
          float v = acc[f][g][r];
          if (!split) {
            if (p.bias) v += p.bias[col];
            if (rmw) v += p.beta * cold[r][g];
            if (p.relu) v = fmaxf(v, 0.f);
            if (p.gate && !(p.gate[(long)row * p.ldg + col] > 0.f)) v = 0.f;
          }
          orow[col] = v;
        }
      } else {
        const int col = n0 + wn * 64 + 2 * l31;  // (g=0, g=1) are adjacent columns
        f32x2 v = {acc[f][0][r], acc[f][FN - 1][r]};
        if (col + 1 < p.N) {
          if (!split) {
            if (p.bias) { v[0] += p.bias[col]; v[1] += p.bias[col + 1]; }
            if (rmw) {
              v[0] += p.beta * cold[r][0];
              v[1] += p.beta * cold[r][1];
            }
            if (p.relu) { v[0] = fmaxf(v[0], 0.f); v[1] = fmaxf(v[1], 0.f); }
            if (p.gate) {
              const float* gr = p.gate + (long)row * p.ldg + col;
              if (!(gr[0] > 0.f)) v[0] = 0.f;
              if (!(gr[1] > 0.f)) v[1] = 0.f;
            }
          }
          *reinterpret_cast<f32x2*>(orow + col) = v;
        } else if (col < p.N) {
          float x = v[0];
          if (!split) {
            if (p.bias) x += p.bias[col];
            if (rmw) x += p.beta * cold[r][0];
            if (p.relu) x = fmaxf(x, 0.f);
            if (p.gate && !(p.gate[(long)row * p.ldg + col] > 0.f)) x = 0.f;
          }
          orow[col] = x;
        }
      }
    }
  }
}

template <int FN, int AKIND, int BKIND, int S, int OPTK, int FM, bool EMU>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(2))) void gemm_f32_fast_kernel(FastParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = smem_raw;
  if constexpr (EMU) {
    // two workgroups share each SIMD and run the same VALU-split / MFMA sequence; equal priority
    // keeps them in lockstep (both split, then both wait on the matrix pipe). A static priority
    // for every other hardware slot lets one wave's split run beside the other's MFMAs.
    if (p.prio && ((blockIdx.x >> 3) & 1)) __builtin_amdgcn_s_setprio(1);
  }
  // XCD-aware tile order (bijective): hardware ids b and b+8 share an XCD; each XCD gets a
  // contiguous range of logical tiles, ordered split-major so an XCD shares one K slice.
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  if constexpr (OPTK != 0) {
    // Persistent form of the optimizer-epilogue kernel (grid = 2 workgroups per CU when the
    // planner asks for it): each workgroup walks tiles of its XCD's range. A tile alternates an
    // MFMA phase with an HBM-bound epilogue (read p + state, write them back); with one tile
    // per workgroup the two workgroups of a CU run both phases in lockstep (fc1 wgrad+SGD
    // measured = GEMM time + epilogue time). Persistence plus a start offset for the second
    // workgroup of each CU lets one workgroup's epilogue stream while the other computes.
    const int T = p.tiles_m * p.tiles_n;
    const int q8 = nwg / 8, r8 = nwg % 8;
    const int per = q8 + (xcd < r8 ? 1 : 0);            // workgroups on this XCD
    const int before = xcd * q8 + (xcd < r8 ? xcd : r8);  // workgroups on lower XCDs
    const int j = b / 8;
    // tiles split in proportion to the workgroups of each XCD (an XCD may have none)
    const int t0 = (int)((long)T * before / nwg), t1 = (int)((long)T * (before + per) / nwg);
    if (t1 - t0 > per && j >= per / 2) {
      __builtin_amdgcn_s_sleep(127);
      __builtin_amdgcn_s_sleep(127);
    }
    for (int lid = t0 + j; lid < t1; lid += per) {
      gemm_tile<FN, AKIND, BKIND, S, OPTK, FM, EMU>(p, lid, smem);
      __builtin_amdgcn_s_barrier();  // every wave is done with this tile's LDS stages
    }
  } else {
    const int q8 = nwg / 8, r8 = nwg % 8;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    gemm_tile<FN, AKIND, BKIND, S, OPTK, FM, EMU>(p, lid, smem);
  }
}

// Two weight-gradient + optimizer GEMMs of one backward in ONE persistent launch (world size 1,
// consecutive Linear layers: ops/linear.py holds the first back until the second arrives,
// SyncBackend::held_epilogue). Each persistent kernel ends on a partial round of tiles (toy MLP
// fc2: 1024 tiles, fc1: 2304, on 512 workgroups) and restarts its MFMA-only first tiles with
// no epilogue traffic to overlap; one launch over both tile sets pays that once. Tiles
// [0, T_p) are p's, the rest q's; same XCD-contiguous split as the single kernel.
template <int OPTK>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(2))) void
gemm_f32_pair_kernel(FastParams p, FastParams q) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = smem_raw;
  if (p.prio && ((blockIdx.x >> 3) & 1)) __builtin_amdgcn_s_setprio(1);
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int Tp = p.tiles_m * p.tiles_n, T = Tp + q.tiles_m * q.tiles_n;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int per = q8 + (xcd < r8 ? 1 : 0);
  const int before = xcd * q8 + (xcd < r8 ? xcd : r8);
  const int j = b / 8;
  const int t0 = (int)((long)T * before / nwg), t1 = (int)((long)T * (before + per) / nwg);
  if (t1 - t0 > per && j >= per / 2) {
    __builtin_amdgcn_s_sleep(127);
    __builtin_amdgcn_s_sleep(127);
  }
  for (int lid = t0 + j; lid < t1; lid += per) {
    if (lid < Tp) gemm_tile<2, kDenseMN, kDenseMN, 2, OPTK, 2, true>(p, lid, smem);
    else gemm_tile<2, kDenseMN, kDenseMN, 2, OPTK, 2, true>(q, lid - Tp, smem);
    __builtin_amdgcn_s_barrier();
  }
}

// Weight gradient + optimizer update with the roles split inside ONE 512-thread workgroup per
// CU, in lockstep (profiles/r9/wgrad_lockstep_r9*.md). The persistent epilogue kernel above
// alternates, in every workgroup, a K loop (no HBM traffic) with an HBM-bound update; the two
// workgroups of a CU overlap those phases only by chance. Here waves 0-3 run exactly that K
// loop (gemm_tile, kOptG: the 2-stage LDS-DMA pipeline, split-bf16 MFMAs -- bit-identical
// gradients) for tile j while waves 4-7 stream the update of tile j - 1 (p / state loads of the
// next chunk group always in flight, non-temporal), reading its gradient from an LDS buffer G.
// Both roles execute the same barriers: the K loop's one per 32-deep K tile, two around the G
// hand-over and one per tile -- the stream waves place their four chunk groups on the K loop's
// barrier intervals, and a last step with no K work drains the final tile. No spin-waits, no
// counters: the hardware barrier is the hand-over. (A version with independent roles handing
// the tile over through LDS counters lost to the math waves' operand latency and their VALU /
// MFMA interference with the stream: profiles/r9/wgrad_split_roles_r9.md.)
template <int KIND>
__global__ __launch_bounds__(2 * kT) __attribute__((amdgpu_waves_per_eu(2, 2))) void
wgrad_lockstep_kernel(FastParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = smem_raw;
  constexpr int S = 2, FN = 2, FM = 2;
  constexpr int STG = 64 * FM * kBK * 4 + 64 * FN * kBK * 4;
  constexpr int OPTK = KIND | kOptG;
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b % 8;
  const int T = p.tiles_m * p.tiles_n;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int per = q8 + (xcd < r8 ? 1 : 0);
  const int before = xcd * q8 + (xcd < r8 ? xcd : r8);
  const int t0 = (int)((long)T * before / nwg), t1 = (int)((long)T * (before + per) / nwg);
  const int j0 = b / 8;
  const int ntiles = t1 - t0 > j0 ? (t1 - t0 - j0 + per - 1) / per : 0;
  const int nk = (p.K + kBK - 1) / kBK;  // the K loop's barriers per tile (K % 128 == 0: 4n)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < 4) {
    for (int j = 0; j < ntiles; ++j) {
      gemm_tile<FN, kDenseMN, kDenseMN, S, OPTK, FM, true>(p, t0 + j0 + j * per, smem);
      __builtin_amdgcn_s_barrier();  // every wave is done with this tile's LDS stages
    }
    // the drain step: the stream waves update the last tile; match their barriers
    if (ntiles > 0) {
      for (int q = 0; q < nk + 3; ++q) __builtin_amdgcn_s_barrier();
    }
    return;
  }
  // ---------------------------------------------------------------- stream waves (4-7)
  constexpr bool SGD = KIND == 1;
  constexpr int BN = 64 * FN;
  constexpr int IT = 128 * (BN / 4) / kT;  // 16-B chunks per thread per tile (16)
  constexpr int GI = IT / 4;               // chunks per group (4 groups per tile)
  constexpr int NS = SGD ? 2 : 3;
  const float* G = reinterpret_cast<const float*>(smem + S * STG);
  const int ts = threadIdx.x - kT;
  OptEpilogue o = p.opt;
  if constexpr (SGD) load_hyper(o.sgd);
  else load_hyper(o.adam);
  const bool mom_rd = SGD && o.sgd.momentum != 0.f && !o.sgd.first_step;
  const bool mom_wr = SGD && o.sgd.momentum != 0.f;
  const long step8 = 8 * p.ldc;
  struct Tile {
    long base;
    int rows;
    bool col_ok;
  };
  auto tile_of = [&](int j) -> Tile {
    const int lid = t0 + j0 + j * per;
    const int tm = lid / p.tiles_n, tn = lid - tm * p.tiles_n;  // gemm_tile's order
    const int row = tm * 128 + (ts >> 5), col = tn * BN + (ts & 31) * 4;
    Tile t;
    t.col_ok = col < p.N;
    t.rows = row < p.M ? min(IT, (p.M - row + 7) / 8) : 0;
    t.base = (long)min(row, p.M - 1) * p.ldc + min(col, p.N - 4);
    return t;
  };
  struct Set {
    f32x4 v[NS][GI];
  };
  auto issue = [&](const Tile& t, int g, Set& s) {
#pragma unroll
    for (int u = 0; u < GI; ++u) {
      const int it = g * GI + u;
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
  auto update = [&](const Tile& t, int g, Set& s) {
    f32x4 gv[GI];
#pragma unroll
    for (int u = 0; u < GI; ++u) {
      const int e = (g * GI + u) * kT + ts;
      gv[u] = *reinterpret_cast<const f32x4*>(G + (e >> 5) * BN + (e & 31) * 4);
    }
#pragma unroll
    for (int u = 0; u < GI; ++u) {
      const int it = g * GI + u;
      if (!t.col_ok || it >= t.rows) continue;
      const long q = t.base + it * step8;
      f32x4 pe = s.v[0][u];
      if constexpr (SGD) {
        f32x4 be = mom_rd ? s.v[1][u] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float pc = pe[c], bc = be[c];
          sgd_elem(pc, gv[u][c], bc, o.sgd);
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
          adam_elem(pc, gv[u][c], mc, vc, nullptr, o.adam);
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
  if (ntiles == 0) return;
  const int ng = nk / 4;  // barrier intervals per chunk group
  // one register set per chunk group: the loads of the next TWO groups are in flight while a
  // group is updated (HBM latency under load spans more than one barrier interval: one group
  // ahead measured 223 us for the two toy-MLP kernels, two 194, three 204); group g of every
  // tile lives in set g, so the issue two ahead wraps into the next tile's groups 0 / 1
  Set st[4];
  Tile cur = tile_of(0);
  issue(cur, 0, st[0]);  // tile 0's first groups: in flight while the math waves compute tile 0
  issue(cur, 1, st[1]);
  // step 0: no gradient yet -- the K loop's barriers and the three around G / the tile
  for (int q = 0; q < nk + 3; ++q) __builtin_amdgcn_s_barrier();
  for (int j = 1; j <= ntiles; ++j) {
    // step j: update tile j - 1 (its gradient in G) while the math waves compute tile j
    const Tile nt = tile_of(j < ntiles ? j : j - 1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g < 2) issue(cur, g + 2, st[g + 2]);
      else if (j < ntiles) issue(nt, g - 2, st[g - 2]);  // the next tile's groups 0 and 1
      update(cur, g, st[g]);
      for (int q = 0; q < ng; ++q) __builtin_amdgcn_s_barrier();
    }
    for (int q = 0; q < 3; ++q) __builtin_amdgcn_s_barrier();  // G hand-over (2) + tile end
    cur = nt;
  }
}

template <int FN, int AKIND, int BKIND, int S, int OPT, int FM, bool EMU>
void launch_fast(const FastParams& p, int nblocks, hipStream_t s) {
  constexpr int STG = 64 * FM * kBK * 4 + 64 * FN * kBK * 4;
  const size_t lds = (size_t)S * STG;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)gemm_f32_fast_kernel<FN, AKIND, BKIND, S, OPT, FM, EMU>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL((gemm_f32_fast_kernel<FN, AKIND, BKIND, S, OPT, FM, EMU>), dim3(nblocks),
                     dim3(kT), lds, s, p);
}

// fp32 products on the bf16 matrix core (split3 emulation, see split3_pair) unless
// TDP_GEMM_EMU=0 (or gemm_f32_set_emu(false)) selects the native v_mfma_f32_32x32x2_f32 path
// same-box A/B (profiles/micro/gemm_emu_prio_ab_r4l.txt): toy MLP 0.4069 -> 0.3975 ms/step,
// ResNet-50 35.57 -> 35.43; the isolated GEMMs do not move.
static constexpr int o_emu_prio = 1;
bool o_emu = [] {
  const char* e = std::getenv("TDP_GEMM_EMU");
  return !(e && e[0] == '0');
}();

// bm = 256: the FM 4 kernel (64-wide tile, 2 stages = 80 KiB of LDS, two workgroups per CU);
// instantiated for K-contiguous A operands only
template <int AKIND, int BKIND, int OPT, bool EMU>
void launch_kinds_t(const FastParams& p, int fn, int stages, int nblocks, hipStream_t s, int bm) {
  constexpr bool AK = AKIND != kDenseMN && AKIND != kImWgradT;
  if constexpr (AK && OPT == 0) {
    if (bm == 256) {
      launch_fast<1, AKIND, BKIND, 2, 0, 4, EMU>(p, nblocks, s);
      return;
    }
  }
  if (fn == 1) {
    if (stages == 3) launch_fast<1, AKIND, BKIND, 3, OPT, 2, EMU>(p, nblocks, s);
    else launch_fast<1, AKIND, BKIND, 2, OPT, 2, EMU>(p, nblocks, s);
  } else {
    if (stages == 3) launch_fast<2, AKIND, BKIND, 3, OPT, 2, EMU>(p, nblocks, s);
    else launch_fast<2, AKIND, BKIND, 2, OPT, 2, EMU>(p, nblocks, s);
  }
}
template <int AKIND, int BKIND, int OPT = 0>
void launch_kinds(const FastParams& p, int fn, int stages, int nblocks, hipStream_t s,
                  int bm = 128) {
  if (o_emu) launch_kinds_t<AKIND, BKIND, OPT, true>(p, fn, stages, nblocks, s, bm);
  else launch_kinds_t<AKIND, BKIND, OPT, false>(p, fn, stages, nblocks, s, bm);
}

}  // namespace

bool gemm_f32_fast_ok(const GemmF32Args& a) {
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (a.mask) return false;
  if (a.rowsum && a.a_kcontig) return false;  // row sums are taken from the [k][m] A tile
  if (!al(a.A) || !al(a.B) || a.lda % 4 || a.ldb % 4) return false;
  if (a.K < 4 || a.K % 4) return false;
  if (!a.a_kcontig && a.M % 4) return false;
  if (!a.b_kcontig && a.N % 4) return false;
  if (a.a_kcontig && !a.b_kcontig) return true;
  return true;
}

// Plan: tile width (FN), split-K and pipeline depth so that every CU runs TWO workgroups (two
// waves per SIMD: one wave's barrier / LDS latency hides behind the other's MFMAs -- the first
// PMC profile showed 53 % MFMA-busy at one workgroup per CU) while keeping >= 8 K steps per split.
// LDS per workgroup must stay <= 80 KiB for two per CU: FN=1 (24 KiB/stage) allows 3 stages,
// FN=2 (32 KiB/stage) 2 stages.
static int o_fn = 0, o_splits = 0, o_stages = 0;

// Optimizer-epilogue variant (defaults: LDS-staged non-temporal epilogue on a persistent grid of
// two workgroups per CU, profiles/opt_epilogue_variants.md), overridable at run time
// (gemm_f32_set_opt_variant) so one test process can cover every variant.
struct OptVariant {
  int sgd, adam, wgs;
  bool persist;
};
static OptVariant& opt_variant() {
  static OptVariant v{kOptLds | kOptNT, kOptLds | kOptNT | kOptPT, 2, true};
  return v;
}

std::vector<int> gemm_f32_set_opt_variant(int sgd, int adam, int persist, int wgs) {
  OptVariant& v = opt_variant();
  if (sgd >= 0) v.sgd = sgd & (kOptWide | kOptNT | kOptLds | kOptPT);
  if (adam >= 0) v.adam = adam & (kOptWide | kOptNT | kOptLds | kOptPT);
  if (persist >= 0) v.persist = persist != 0;
  if (wgs > 0) v.wgs = wgs;
  return {v.sgd, v.adam, v.persist ? 1 : 0, v.wgs};
}
void gemm_f32_set_override(int fn, int splits, int stages) {
  o_fn = fn; o_splits = splits; o_stages = stages;
}
// Row-vector (LDS-staged) output stores: 16-B aligned rows of C, bias and the workspace
static bool o_no_cvec = false;  // gemm_f32_set_cvec(false): A/B measurements
static int o_bm = 0;            // 0 auto, 128 / 256 forced (gemm_f32_set_bm: sweeps)
void gemm_f32_set_emu(bool on) { o_emu = on; }
bool gemm_f32_emu() { return o_emu; }
void gemm_f32_set_bm(int bm) { o_bm = (bm == 128 || bm == 256) ? bm : 0; }
void gemm_f32_set_cvec(bool on) { o_no_cvec = !on; }
static bool c_vec_ok(int N, long ldc, const float* C, const float* bias, int splits) {
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (N % 4) return false;
  if (splits > 1) return true;  // the workspace: N-float rows of an aligned allocation
  return ldc % 4 == 0 && al(C) && (bias == nullptr || al(bias));
}

// The lockstep weight-gradient + optimizer kernel (wgrad_lockstep_kernel): the optimizer
// epilogue's layout (A = dY^T, B = X, both MN-contiguous), the split-bf16 products, K a
// multiple of 128 (four chunk groups on the K loop's barrier intervals), SGD / Adam without
// amsgrad. Opt-in: TDP_WGRAD_LOCKSTEP=1 / gemm_f32_set_lockstep(true).
static bool o_lockstep = [] {  // opt-in: measured at parity with the persistent kernel, not
  const char* e = std::getenv("TDP_WGRAD_LOCKSTEP");  // better (profiles/r9/wgrad_split_roles_r9.md)
  return e && e[0] == '1';
}();
void gemm_f32_set_lockstep(bool on) { o_lockstep = on; }
bool gemm_f32_lockstep() { return o_lockstep; }
static bool lockstep_ok(const GemmF32Args& a) {
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!o_lockstep || !o_emu || a.a_kcontig || a.b_kcontig || a.mask || a.gate) return false;
  if (a.opt.kind != 1 && a.opt.kind != 2) return false;
  if (a.opt.kind == 2 && (a.opt.adam.amsgrad || a.opt.s2)) return false;
  if (a.K < 128 || a.K % 128 || a.M % 4 || a.N % 4 || a.ldc % 4) return false;
  if (!al(a.opt.p) || (a.opt.s0 && !al(a.opt.s0)) || (a.opt.s1 && !al(a.opt.s1))) return false;
  return true;
}

void gemm_f32_fast_plan(const GemmF32Args& a, int num_cus, GemmPlan& plan) {
  // 128-wide tiles split the fewest fragments per MFMA; with split-bf16 products (VALU-heavy
  // per fragment) they win on the skinny-M GEMMs too (toy-MLP fc1 forward 84.5 -> 68.4 us,
  // fc2 forward 40.7 -> 38.4, fc2 input gradient 45.0 -> 39.6: profiles/micro/gemm_plan_sweep_emu_r4f.log)
  int fn = (a.N >= 512 && (a.M >= 512 || o_emu)) ? 2 : 1;
  if (o_fn == 1 || o_fn == 2) fn = o_fn;
  const int bn = 64 * fn;
  const long tiles = (long)ceil_div(a.M, 128) * ceil_div(a.N, bn);
  const long target = 2L * num_cus;
  int splits = 1;
  if (tiles < target && a.rowsum == nullptr) {
    const int want = (int)((target + tiles - 1) / tiles);
    const int kmax = a.K / (kBK * 8);
    splits = want < kmax ? want : kmax;
    if (splits < 1) splits = 1;
  }
  if (o_splits > 0 && a.rowsum == nullptr) splits = o_splits;
  if (a.opt.kind != 0) splits = 1;  // the optimizer epilogue needs the complete K sum
  plan.grid = 0;
  plan.lockstep = false;
  if (a.opt.kind != 0 && lockstep_ok(a)) {
    plan.lockstep = true;  // one 512-thread workgroup per CU, roles in lockstep
    plan.grid = num_cus;
  } else if (a.opt.kind != 0) {
    // persistent: 2 workgroups per CU (gemm_f32_set_opt_variant overrides, for measurements:
    // 3 fit with FN=1)
    const OptVariant& v = opt_variant();
    if (v.persist) plan.grid = (v.wgs >= 1 && v.wgs <= 4 ? v.wgs : 2) * num_cus;
  }
  int kps = ceil_div(ceil_div(a.K, splits), kBK) * kBK;
  plan.fast = true;
  plan.bm = (o_bm == 256 && fn == 1 && splits == 1 && a.a_kcontig && a.opt.kind == 0) ? 256 : 128;
  plan.bn = bn;
  plan.tile = fn;
  plan.k_per_split = kps;
  plan.splits = ceil_div(a.K, kps);
  plan.ws_floats = plan.splits > 1 ? (long)plan.splits * a.M * a.N : 0;
  const int nk = ceil_div(kps, kBK);
  plan.stages = (fn == 1 && nk > 4) ? 3 : 2;
  if (o_stages == 2 || o_stages == 3) plan.stages = o_stages;
}

static FastParams fast_params(const GemmF32Args& a, const GemmPlan& plan, float* ws) {
  FastParams p{};  // zero: every optional pointer (stats, wt, ...) unset unless assigned below
  p.prio = o_emu_prio;
  p.A = a.A; p.B = a.B; p.C = a.C; p.bias = a.bias; p.ws = ws;
  p.gate = a.gate; p.ldg = a.ldgate;
  p.rowsum = a.rowsum; p.rowsum_beta = a.rowsum_beta;
  p.lda = a.lda; p.ldb = a.ldb; p.ldc = a.ldc;
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.k_per_split = plan.k_per_split;
  p.splits = plan.splits;
  p.tiles_m = ceil_div(a.M, plan.bm);
  p.tiles_n = ceil_div(a.N, plan.bn);
  p.beta = plan.splits > 1 ? 0.f : a.beta;
  p.relu = (plan.splits > 1 ? false : a.relu) ? 1 : 0;
  p.cvec = c_vec_ok(a.N, a.ldc, a.C, a.bias, plan.splits) && !o_no_cvec;
  p.opt = a.opt;
  p.bopt = (a.opt.kind != 0 && a.rowsum != nullptr && a.rowsum_beta == 0.f) ? a.bias_opt
                                                                             : OptEpilogue{};
  return p;
}

// The pair launch exists for the default epilogue variants on the persistent 128 x 128 plan.
static int pair_variant(const GemmF32Args& a, const GemmPlan& plan) {
  if (!o_emu || plan.lockstep || !plan.fast || plan.skinny || plan.emu8 || plan.grid <= 0 ||
      plan.splits != 1 || plan.tile != 2 || plan.stages != 2 || plan.bm != 128 ||
      a.a_kcontig || a.b_kcontig || a.mask || a.gate)
    return -1;
  const int v = a.opt.kind == 1 ? opt_variant().sgd : a.opt.kind == 2 ? opt_variant().adam : -1;
  if (v != (kOptLds | kOptNT) && v != (kOptLds | kOptNT | kOptPT)) return -1;
  return a.opt.kind | v;
}

bool gemm_f32_fast_pair_ok(const GemmF32Args& a1, const GemmPlan& p1, const GemmF32Args& a2,
                           const GemmPlan& p2) {
  const int v = pair_variant(a1, p1);
  return v >= 0 && v == pair_variant(a2, p2) && p1.grid == p2.grid;
}

template <int OPTK>
static void launch_pair(const FastParams& p, const FastParams& q, int nb, hipStream_t s) {
  constexpr int STG = 64 * 2 * kBK * 4 + 64 * 2 * kBK * 4;
  const size_t lds = (size_t)2 * STG;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)gemm_f32_pair_kernel<OPTK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL(gemm_f32_pair_kernel<OPTK>, dim3(nb), dim3(kT), lds, s, p, q);
}

void gemm_f32_fast_run_pair(const GemmF32Args& a1, const GemmPlan& p1, const GemmF32Args& a2,
                            const GemmPlan& p2, hipStream_t s) {
  if (!gemm_f32_fast_pair_ok(a1, p1, a2, p2))
    throw std::runtime_error("gemm_f32_fast_run_pair: the two GEMMs do not share a pair plan");
  const FastParams p = fast_params(a1, p1, nullptr), q = fast_params(a2, p2, nullptr);
  const int nb = std::max(1, std::min(p1.grid, p.tiles_m * p.tiles_n + q.tiles_m * q.tiles_n));
  switch (pair_variant(a1, p1)) {
    case 1 | kOptLds | kOptNT: launch_pair<1 | kOptLds | kOptNT>(p, q, nb, s); break;
    case 1 | kOptLds | kOptNT | kOptPT: launch_pair<1 | kOptLds | kOptNT | kOptPT>(p, q, nb, s); break;
    case 2 | kOptLds | kOptNT: launch_pair<2 | kOptLds | kOptNT>(p, q, nb, s); break;
    default: launch_pair<2 | kOptLds | kOptNT | kOptPT>(p, q, nb, s); break;
  }
}

void gemm_f32_fast_run(const GemmF32Args& a, const GemmPlan& plan, float* ws, hipStream_t s) {
  FastParams p = fast_params(a, plan, ws);
  const int nblocks = p.tiles_m * p.tiles_n * plan.splits;
  const bool ak = a.a_kcontig, bk = a.b_kcontig;
  const int fn = plan.tile, st = plan.stages;
  // the optimizer epilogue is instantiated for the weight-gradient layout only (A = dY^T and
  // B = X both MN-contiguous); any other use stores C and applies the flat update afterwards
  const bool opt = a.opt.kind != 0 && plan.splits == 1 && !ak && !bk;
  if (opt && plan.lockstep) {
    const int nb = std::max(1, std::min(plan.grid, nblocks));
    constexpr int STG = 64 * 2 * kBK * 4 + 64 * 2 * kBK * 4;
    const size_t lds = (size_t)2 * STG + 128 * 128 * 4;  // 2 stages + the gradient buffer G
    if (a.opt.kind == 1) {
      static bool cfg = false;
      if (!cfg) {
        (void)hipFuncSetAttribute((const void*)wgrad_lockstep_kernel<1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        cfg = true;
      }
      hipLaunchKernelGGL(wgrad_lockstep_kernel<1>, dim3(nb), dim3(2 * kT), lds, s, p);
    } else {
      static bool cfg = false;
      if (!cfg) {
        (void)hipFuncSetAttribute((const void*)wgrad_lockstep_kernel<2>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        cfg = true;
      }
      hipLaunchKernelGGL(wgrad_lockstep_kernel<2>, dim3(nb), dim3(2 * kT), lds, s, p);
    }
    return;
  }
  if (opt) {
    const int nb = plan.grid > 0 && plan.grid < nblocks ? plan.grid : nblocks;
    // SGD epilogue variant flags (kOptWide | kOptNT | kOptLds | kOptPT,
    // gemm_f32_set_opt_variant). kOptLds | kOptNT: toy MLP 0.457-0.460 ms/step (one run of four
    // 0.498), kOptLds alone 0.468, kOptNT 0.487, plain 0.507, kOptWide 0.56 (register pressure;
    // profiles/opt_epilogue_variants.md). With kOptLds, kOptWide = one batch per tile. + kOptPT
    // was -0.6 %, +0.8 % and +-0 % on three boxes: the default stays without it
    // (profiles/r10/param_store_policy_r10m.md).
    // Non-128-wide tiles ignore kOptLds.
    const int variant = opt_variant().sgd;
    // Adam epilogue flags (kOptLds | kOptNT): toy MLP + Adam 0.555 ms/step vs 0.566 LDS only,
    // 0.594 register epilogue (profiles/opt_epilogue_variants.md); default + kOptPT: -1.2 % and
    // -0.8 % on two boxes (profiles/r10/param_store_policy_r10m.md)
    const int adam_variant = opt_variant().adam;
    if (a.opt.kind == 1) {
      switch (variant) {
        case kOptLds: launch_kinds<kDenseMN, kDenseMN, 1 | kOptLds>(p, fn, st, nb, s); break;
        case kOptLds | kOptNT:
          launch_kinds<kDenseMN, kDenseMN, 1 | kOptLds | kOptNT>(p, fn, st, nb, s);
          break;
        case kOptLds | kOptNT | kOptWide:
          launch_kinds<kDenseMN, kDenseMN, 1 | kOptLds | kOptNT | kOptWide>(p, fn, st, nb, s);
          break;
        case kOptLds | kOptNT | kOptPT:
          launch_kinds<kDenseMN, kDenseMN, 1 | kOptLds | kOptNT | kOptPT>(p, fn, st, nb, s);
          break;
        case kOptWide: launch_kinds<kDenseMN, kDenseMN, 1 | kOptWide>(p, fn, st, nb, s); break;
        case kOptNT: launch_kinds<kDenseMN, kDenseMN, 1 | kOptNT>(p, fn, st, nb, s); break;
        case kOptWide | kOptNT:
          launch_kinds<kDenseMN, kDenseMN, 1 | kOptWide | kOptNT>(p, fn, st, nb, s);
          break;
        default: launch_kinds<kDenseMN, kDenseMN, 1>(p, fn, st, nb, s);
      }
    } else if (adam_variant == (kOptLds | kOptNT)) {
      launch_kinds<kDenseMN, kDenseMN, 2 | kOptLds | kOptNT>(p, fn, st, nb, s);
    } else if (adam_variant == (kOptLds | kOptNT | kOptPT)) {
      launch_kinds<kDenseMN, kDenseMN, 2 | kOptLds | kOptNT | kOptPT>(p, fn, st, nb, s);
    } else if (adam_variant == (kOptLds | kOptNT | kOptWide)) {
      launch_kinds<kDenseMN, kDenseMN, 2 | kOptLds | kOptNT | kOptWide>(p, fn, st, nb, s);
    } else if (adam_variant == kOptLds) {
      launch_kinds<kDenseMN, kDenseMN, 2 | kOptLds>(p, fn, st, nb, s);
    } else {
      launch_kinds<kDenseMN, kDenseMN, 2>(p, fn, st, nb, s);
    }
    return;
  }
  p.opt.kind = 0;
  if (ak && bk) launch_kinds<kDenseK, kDenseK>(p, fn, st, nblocks, s, plan.bm);
  else if (ak && !bk) launch_kinds<kDenseK, kDenseMN>(p, fn, st, nblocks, s, plan.bm);
  else if (!ak && !bk) launch_kinds<kDenseMN, kDenseMN>(p, fn, st, nblocks, s);
  else launch_kinds<kDenseMN, kDenseK>(p, fn, st, nblocks, s);
  if (plan.splits > 1)
    splitk_reduce(ws, plan.splits, a.M, a.N, a.C, false, a.ldc, a.bias, a.beta, a.relu, s,
                  a.gate, a.ldgate);
  if (a.opt.kind != 0) gemm_opt_fallback(a, s);
}

// ------------------------------------------------------------------ implicit-GEMM convolution
static const float* zero_page() {
  static float* z = nullptr;
  if (!z) {
    (void)hipMalloc(&z, 256);
    (void)hipMemset(z, 0, 256);
  }
  return z;
}

static int ilog2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

// Weight-gradient orientation: dWt [Cout][R*S*C] (M = Cout) or dWt^T [R*S*C][Cout] (M = R*S*C).
// Pick the one whose 128 x (64*fn) tiles waste the fewest padded MACs (Cout = 192 wastes a
// quarter of its second 128-row tile as M, nothing as N = 3 x 64); ties keep M = Cout.
static int o_wgrad_t = -1;  // -1 auto, 0 / 1 force (per-layer sweeps)
void conv_set_wgrad_transposed(int mode) { o_wgrad_t = mode; }
// Weight-gradient tile width: the 128-wide tile (FN = 2, twice the MACs per LDS byte) whenever it
// pads N no more than the 64-wide one (measured: AlexNet features.8 / ResNet-50 3x3 wgrads run
// 1.3-1.7x faster with FN = 2 at equal workgroup counts).
static int wgrad_fn(int M, int N) {
  return (M >= 128 && N >= 128 && 2 * ceil_div(N, 128) == ceil_div(N, 64)) ? 2 : 1;
}
static long padded_macs(int M, int N) {
  const int bn = 64 * wgrad_fn(M, N);
  return (long)ceil_div(M, 128) * 128 * ((long)ceil_div(N, bn) * bn);
}
// Workgroups the weight-gradient split-K aims for, in units of CUs. K = N*P*Q is long and the
// tile count small, so the split count sets the grid. Measured per layer (scripts/sweep_wgrad.py,
// profiles/wgrad_split_target.md): 1x1 filters are bound by the partial-sum traffic and want
// the fewest splits that fill the chip (2 per CU); R*S > 1 filters re-read each pixel R*S times
// from L2 and gain from 8 per CU (AlexNet features.3: 898 us at 2, 710 us at 8).
static int o_wgrad_target = 0;  // > 0: override (sweeps)
void conv_set_wgrad_target(int per_cu) { o_wgrad_target = per_cu > 0 ? per_cu : 0; }
static bool wgrad_transposed(const ConvGeom& g) {
  if (o_wgrad_t == 0 || o_wgrad_t == 1) return o_wgrad_t == 1;
  const int rsc = g.R * g.S * g.C;
  if (rsc <= 0) return g.Cout < 128;
  const long t = padded_macs(rsc, g.Cout), n = padded_macs(g.Cout, rsc);
  return t != n ? t < n : g.Cout < 128;
}
bool conv_wgrad_transposed(const ConvGeom& g) { return wgrad_transposed(g); }

// Measured plan table (tile width, split-K) per exact convolution geometry and pass -- the
// MIOpen perf-db idea: the heuristic planner above cannot see wave quantisation (a grid of T
// workgroups on 3 (FN 1) or 2 (FN 2) slots per CU runs ceil(T / slots) rounds; ResNet-50's
// layer3/4 3x3 convolutions lose up to 20 % to a near-empty last round). Entries come from
// scripts/tune_conv_plans.py sweeps (pkg/perfdb/*.json, registered at import by ops/conv.py);
// geometries not in the table use the heuristic. Overrides (gemm_f32_set_override) win.
struct PlanKey {
  int v[14];
  bool operator==(const PlanKey& o) const {
    for (int i = 0; i < 14; ++i)
      if (v[i] != o.v[i]) return false;
    return true;
  }
};
struct PlanKeyHash {
  size_t operator()(const PlanKey& k) const {
    size_t h = 1469598103934665603ull;
    for (int i = 0; i < 14; ++i) h = (h ^ (size_t)(unsigned)k.v[i]) * 1099511628211ull;
    return h;
  }
};
static std::unordered_map<PlanKey, std::pair<int, int>, PlanKeyHash>& plan_db() {
  static std::unordered_map<PlanKey, std::pair<int, int>, PlanKeyHash> db;
  return db;
}
static PlanKey plan_key(int mode, const ConvGeom& g) {
  return PlanKey{{mode, g.N, g.C, g.H, g.W, g.Cout, g.R, g.S, g.P, g.Q, g.sh, g.sw, g.ph, g.pw}};
}
void conv_plan_db_put(int mode, const ConvGeom& g, int fn, int splits) {
  if ((fn != 1 && fn != 2) || splits < 1) throw std::runtime_error("conv plan db: bad plan");
  plan_db()[plan_key(mode, g)] = {fn, splits};
}
void conv_plan_db_clear() { plan_db().clear(); }
long conv_plan_db_size() { return (long)plan_db().size(); }

bool conv_nhwc_ok(int mode, const ConvGeom& g) {
  if (g.C % 4 || g.Cout % 4) return false;
  if (mode == kConvDgrad && (ilog2_exact(g.sh) < 0 || ilog2_exact(g.sw) < 0)) return false;
  return true;
}

ConvPlan conv_nhwc_plan(int mode, const ConvGeom& g, int num_cus) {
  ConvPlan pl;
  pl.mode = mode;
  if (mode == kConvFwd) { pl.M = g.N * g.P * g.Q; pl.N = g.Cout; pl.K = g.R * g.S * g.C; }
  else if (mode == kConvDgrad) { pl.M = g.N * g.H * g.W; pl.N = g.C; pl.K = g.R * g.S * g.Cout; }
  else if (!wgrad_transposed(g)) { pl.M = g.Cout; pl.N = g.R * g.S * g.C; pl.K = g.N * g.P * g.Q; }
  else { pl.M = g.R * g.S * g.C; pl.N = g.Cout; pl.K = g.N * g.P * g.Q; }
  GemmF32Args a{};
  a.M = pl.M; a.N = pl.N; a.K = pl.K;
  GemmPlan gp;
  gemm_f32_fast_plan(a, num_cus, gp);
  const bool free_plan = o_fn == 0 && o_splits == 0 && o_stages == 0 && o_bm == 0;
  const auto hit = free_plan ? plan_db().find(plan_key(mode, g)) : plan_db().end();
  if (hit != plan_db().end()) {
    const int fn = hit->second.first;
    const int kps = ceil_div(ceil_div(pl.K, hit->second.second), kBK) * kBK;
    gp.tile = fn;
    gp.k_per_split = kps;
    gp.splits = ceil_div(pl.K, kps);
    gp.ws_floats = gp.splits > 1 ? (long)gp.splits * pl.M * pl.N : 0;
    gp.stages = 2;
  } else if (mode == kConvWgrad && o_fn == 0 && o_splits == 0) {
    const int fn = wgrad_fn(pl.M, pl.N);
    const long tiles = (long)ceil_div(pl.M, 128) * ceil_div(pl.N, 64 * fn);
    const int per_cu = o_wgrad_target > 0 ? o_wgrad_target : (g.R * g.S == 1 ? 2 : 8);
    const long target = (long)per_cu * num_cus;
    const int kmax = pl.K / (kBK * 8);
    int splits = (int)((target + tiles - 1) / tiles);
    splits = splits < kmax ? splits : kmax;
    if (splits < 1) splits = 1;
    const int kps = ceil_div(ceil_div(pl.K, splits), kBK) * kBK;
    gp.tile = fn;
    gp.k_per_split = kps;
    gp.splits = ceil_div(pl.K, kps);
    gp.ws_floats = gp.splits > 1 ? (long)gp.splits * pl.M * pl.N : 0;
    gp.stages = 2;
    if (o_stages == 2 || o_stages == 3) gp.stages = o_stages;
  } else if (mode != kConvWgrad && o_fn == 0 && g.R * g.S > 1 && pl.N % 128 == 0 &&
             pl.N >= 256) {
    // R*S > 1 forward / input gradient with N (Cout / C) a multiple of 128: the 128-wide tile
    // (AlexNet features.8 input gradient 377 -> 351 us, ResNet-50 layer3 3x3 346 -> 331 us)
    const long tiles = (long)ceil_div(pl.M, 128) * (pl.N / 128);
    if (tiles >= 2L * num_cus) {
      gp.tile = 2;
      gp.splits = 1;
      gp.k_per_split = ceil_div(pl.K, kBK) * kBK;
      gp.ws_floats = 0;
    }
  }
  // Convolutions: the 64-wide tile keeps 2 LDS stages (48 KiB, 3 workgroups per CU instead of
  // 2 with 3 stages); measured faster on 86 of 112 (layer, plan) pairs of AlexNet / ResNet-50
  // and on every forward / input-gradient shape (scripts/sweep_conv_fd.py).
  if (gp.tile == 1 && o_stages == 0) gp.stages = 2;
  // 256-row tiles (FM 4: half the B traffic and barriers per MFMA) only on request
  // (gemm_f32_set_bm): measured 3-34 % SLOWER than 128 rows on every ResNet-50 / AlexNet forward
  // and input-gradient shape with the 64-wide tile (profiles/micro/gemm_bm256_ab.jsonl) -- two
  // workgroups per CU instead of three hide less of the operand-load latency
  pl.bm = 128;
  if (mode != kConvWgrad && gp.tile == 1 && gp.splits == 1 && o_bm == 256) pl.bm = 256;
  if (pl.bm == 256) gp.stages = 2;
  pl.fn = gp.tile;
  pl.fm = gp.stages;  // pipeline depth (the NHWC path always uses BM = 128)
  pl.splits = gp.splits;
  pl.k_per_split = gp.k_per_split;
  pl.ws_floats = gp.ws_floats;
  return pl;
}

// FWD  : A = x (NHWC), B = Wt [Cout][R*S*C],  C = y  [N*P*Q][Cout] (+bias, relu)
// DGRAD: A = dy (NHWC), B = W2 [R*S*Cout][C], C = dx [N*H*W][C]
// WGRAD: A = dy [N*P*Q][Cout], B = x (NHWC),  C = dWt [Cout][R*S*C] (beta: accumulate);
//        when conv_wgrad_transposed(g): C = dWt^T [R*S*C][Cout] (A/B arguments unchanged)
bool conv_nhwc_run(const ConvPlan& pl, const ConvGeom& g, const float* A, const float* B,
                   float* C, const float* bias, bool relu, float beta, float* ws,
                   hipStream_t s, const WeightTaps* wtap, float* stats) {
  FastParams p{};
  p.prio = o_emu_prio;
  if (wtap) {
    if (pl.mode != kConvDgrad) throw std::runtime_error("weight taps are for the input gradient");
    p.wt.Cout = g.Cout; p.wt.Sp = g.S;
    p.wt.r0 = wtap->r0; p.wt.s0 = wtap->s0; p.wt.sh = wtap->sh; p.wt.sw = wtap->sw;
    p.wt.Sf = wtap->S; p.wt.C = g.C;
    p.wt.rs = (long)wtap->R * wtap->S * g.C;
    p.wt.uniform = g.Cout % 32 == 0 ? 1 : 0;
    p.wt.dCout = make_fastdiv(g.Cout);
    p.wt.dSp = make_fastdiv(g.S);
  }
  ConvInfo& cv = p.cv;
  cv.zero = zero_page();
  cv.S = g.S; cv.sh = g.sh; cv.sw = g.sw; cv.ph = g.ph; cv.pw = g.pw;
  cv.shl = ilog2_exact(g.sh) < 0 ? 0 : ilog2_exact(g.sh);
  cv.swl = ilog2_exact(g.sw) < 0 ? 0 : ilog2_exact(g.sw);
  if (pl.mode == kConvDgrad) {
    cv.Hs = g.P; cv.Ws = g.Q; cv.Cs = g.Cout;
    cv.grid_pq = g.H * g.W; cv.grid_q = g.W;
  } else {
    cv.Hs = g.H; cv.Ws = g.W; cv.Cs = g.C;
    cv.grid_pq = g.P * g.Q; cv.grid_q = g.Q;
  }
  cv.uniform = (cv.Cs % 32 == 0) ? 1 : 0;
  cv.dC = make_fastdiv(cv.Cs);
  cv.dS = make_fastdiv(g.S);
  cv.dPQ = make_fastdiv(cv.grid_pq);
  cv.dQ = make_fastdiv(cv.grid_q);
  p.A = A; p.B = B; p.C = C; p.bias = bias; p.ws = ws;
  p.rowsum = nullptr; p.rowsum_beta = 0.f;
  p.M = pl.M; p.N = pl.N; p.K = pl.K;
  const bool wt = pl.mode == kConvWgrad && wgrad_transposed(g);
  if (wt) {  // A = implicit x^T, B = dy [K][Cout]
    p.A = B; p.B = A;
  }
  if (pl.mode == kConvFwd) { p.lda = 0; p.ldb = pl.K; p.ldc = pl.N; }
  else if (pl.mode == kConvDgrad) { p.lda = 0; p.ldb = pl.N; p.ldc = pl.N; }
  else if (!wt) { p.lda = pl.M; p.ldb = 0; p.ldc = pl.N; }
  else { p.lda = 0; p.ldb = pl.N; p.ldc = pl.N; }
  p.k_per_split = pl.k_per_split;
  p.splits = pl.splits;
  p.tiles_m = ceil_div(pl.M, pl.bm);
  p.tiles_n = ceil_div(pl.N, 64 * pl.fn);
  p.beta = pl.splits > 1 ? 0.f : beta;
  p.relu = (pl.splits > 1 ? false : relu) ? 1 : 0;
  p.cvec = c_vec_ok(pl.N, p.ldc, C, bias, pl.splits) && !o_no_cvec;
  // column statistics ride on the row-vector epilogue of an unsplit, plain forward GEMM
  const bool stats_ok = stats != nullptr && pl.mode == kConvFwd && pl.splits == 1 && p.cvec &&
                        bias == nullptr && !relu && beta == 0.f;
  p.stats = stats_ok ? stats : nullptr;
  const int nblocks = p.tiles_m * p.tiles_n * pl.splits;
  const int fn = pl.fn, st = pl.fm;
  if (pl.mode == kConvFwd) launch_kinds<kImFwd, kDenseK>(p, fn, st, nblocks, s, pl.bm);
  else if (pl.mode == kConvDgrad && wtap)
    launch_kinds<kImDgrad, kWTap>(p, fn, st, nblocks, s, pl.bm);
  else if (pl.mode == kConvDgrad) launch_kinds<kImDgrad, kDenseMN>(p, fn, st, nblocks, s, pl.bm);
  else if (!wt) launch_kinds<kDenseMN, kImWgrad>(p, fn, st, nblocks, s);
  else launch_kinds<kImWgradT, kDenseMN>(p, fn, st, nblocks, s);
  if (pl.splits > 1)
    splitk_reduce(ws, pl.splits, pl.M, pl.N, C, false, pl.N, bias, beta, relu, s);
  return p.stats != nullptr;
}

}  // namespace tdp
