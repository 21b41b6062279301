// gemm_fw_k: the dense per-pixel GEMM kernel template (see gemm.hip for the
// host side).  Included by the per-tile-size translation units gemm_w8.hip,
// gemm_w4.hip and gemm_w2.hip, which instantiate every epilogue variant of one
// tile size in parallel compile jobs (one TU with all ~70 variants took 13
// minutes to build).
#pragma once
// Dense per-pixel GEMM on the gfx950 matrix cores: the 1x1 layers of the
// X-UNet (FiLM projections `xunet.py:74-87`, attention in/out projections
// `xunet.py:154-177`, NIN skips `xunet.py:128-129`) and their input gradients,
//
//     O[n][m] = epi(sum_k A[m][k] * B[n][k])
//
// with A the bf16 weight ([M][lda], K contiguous), B the NHWC activations
// ([N][ldb], K contiguous) and O / R NHWC bf16 rows (strides ldo / ldr).
// Epilogue (compile-time flags F): (alpha * acc + bias[m] + R[n][m]) * scale
// with an fp32 (F_B32) or bf16 (F_B16) bias, a residual (F_RES) and the
// GroupNorm partial statistics of O (F_GN); or F_DSILU: alpha * acc *
// dsilu(R[n][m]) -- the FiLM input gradient through the SiLU of the
// conditioning embedding.
//
// Schedule ("fat waves"): a 256-thread block = 2 x 2 waves, one per SIMD, each
// owning WI x WJ MFMA 16x16x32 tiles (8 x 8 = 128 x 128 outputs and 256 fp32
// accumulators for the big layers, 4 x 4 / 2 x 2 for small problems):
//   * LDS stages of K = 64 (two MFMA K-steps), two of them: 128-byte rows
//     (whole cache lines per DMA row) with the chunk swizzle c ^ (row & 7):
//     conflict-free ds_read_b128;
//   * K-step s: WI*WJ slots, each one MFMA plus at most one other
//     instruction -- a fragment read of step s + 1 (into the other register
//     set) or, in odd steps, an LDS-DMA piece of the stage after next and the
//     loader's cursor update.  Odd steps open with the wait for the next
//     stage and the ONLY barrier of the stage;
//   * the MFMAs are inline asm with "a"-constrained accumulators (the
//     compiler's own lowering splits 256 accumulators between the register
//     files and shuffles them every K-tile); the epilogue reads them out one
//     fragment pair at a time (a bulk read ahead of it spilled);
//   * persistent: each block walks tiles rb, rb + G, ... as ONE stream of
//     stages, so the next tile's DMA is in flight during the epilogue; the
//     bias rides on a DMA into one of 4 LDS slots; the next tile's first
//     fragments are read after the epilogue (not held across it);
//   * epilogue specialised at compile time (flags F): fragment pairs become
//     16-byte rows by v_permlane16_swap and leave as exactly WI*WJ/2 buffer
//     stores per wave (masked lanes get an out-of-range offset), so the next
//     tile's counted waits step over them; explicit fmas, so every variant
//     rounds alike;
//   * per-tile buffer descriptors (rows m0 / n0 based): 32-bit offsets for
//     any operand size, rows past M / N read as zeros; one VGPR per operand
//     for the DMA offsets (piece rows added by an opaque v_add at the DMA);
//   * bijective XCD remap + grouped tile order: the tiles an XCD runs at once
//     share their activation panels.
#include "common.h"
#include "mfma_gemm.h"

#include <algorithm>
#include <cstdlib>
#include <utility>

namespace {
constexpr int G_BK = 32;         // K per MFMA step
constexpr int G_PK = 64;         // K per LDS stage (two steps): 128-byte rows, whole cache lines per DMA row

// 16-byte chunk c (0..7) of row r of a stage: XOR swizzle by r & 7 (the
// ds_read_b128 lane groups read 16 rows at one chunk: conflict-free)
__device__ __forceinline__ int g_swz(int row, int chunk) { return row * G_PK + ((chunk ^ (row & 7)) << 3); }

template <int WI, int WJ, int NST = 2, int NW = 4>
struct GCfg {
  // NW waves as 2 (M) x NW/2 (N), each 16*WI x 16*WJ outputs
  static constexpr int WGN = NW / 2;
  static constexpr int BM = 32 * WI, BN = 16 * WJ * WGN;
  static constexpr int STAGE = (BM + BN) * G_PK;         // bf16 per stage (two K-steps)
  static constexpr int BIAS = NST * STAGE;               // 4 slots of 256 fp32
  static constexpr int LDS = BIAS + 4 * 512;
  static constexpr int RA = BM / NW, RB = BN / NW;       // operand rows each wave DMAs per stage
  static constexpr int DA = RA / 8, DB = RB / 8;         // DMA pieces (8 rows x 128 B) per wave and stage
  static constexpr int ND = DA + DB;
  static constexpr int NM = WI * WJ;                     // MFMAs per wave and K-tile
  static constexpr int NR = WI + WJ;                     // fragment reads
  static constexpr int NS = WI * WJ / 2;                 // epilogue stores per wave
};

// F_CAT: B is the virtual channel concat [B | B2] of two [N][ldb] tensors
// split at K1 = ldb = K / 2 (the decoder's NIN skip over [h | skip]): one
// GEMM over both halves instead of a GEMM plus a residual-accumulating one
// F_MF: M is a multiple of the tile height (no channel masks; packed epilogue)
enum : int { F_B32 = 1, F_B16 = 2, F_RES = 4, F_GN = 8, F_DSILU = 16, F_CAT = 32, F_MF = 64 };

// Epilogue parameters of one tile (32-bit offsets from the tile's row base).
struct GEpi {
  const bf16* R;                 // residual / pre-activation rows n0.. of this tile
  bf16* obase;                   // output rows n0.. (buffer descriptor base / size: descriptors stay out of
  int orec, rrec;                // structs and lambda signatures, which the host pass also type-checks)
  int M, ldo, ldr;
  float as, bs, rs;              // acc, bias and residual factors
  int m0;
  int wm, wn, lane;
};
}  // namespace

// Residual / pre-activation rows of fragment pair (ii, 2jp), (ii, 2jp + 1):
// 8-byte reads through a range-checked descriptor (rows past the tile end and
// channels past M read as zero without a branch).  Issued a whole fragment
// row ahead of their use (g_epi_rows): each read-then-use pair waited for
// every older vector-memory op -- the next tile's stage DMAs and the previous
// pair's store -- once per pair, 32 serial round trips per 256 x 256 tile.
typedef unsigned g_u2l __attribute__((ext_vector_type(2)));
template <int WI, int WJ, int II, int JP>
__device__ __forceinline__ void g_epi_rload(const GEpi& e, g_u2l& rx, g_u2l& ry) {
  const int fr = e.lane & 15, fq = e.lane >> 4;
  const int cl = e.m0 + e.wm * 16 * WI + II * 16 + fq * 4;
  const int px = e.wn * 16 * WJ + 2 * JP * 16 + fr;
  const bool cok = cl < e.M;
  rx = g_load8(e.R, e.rrec, cok ? (px * e.ldr + cl) * 2 : (int)0x80000000);
  ry = g_load8(e.R, e.rrec, cok ? ((px + 16) * e.ldr + cl) * 2 : (int)0x80000000);
}

// Fragment pair (ii, 2jp), (ii, 2jp + 1) -> one 16-byte store per lane.  Before
// the swap lane (fq, fr) holds channels fq*4..+3 of pixels P(2jp, fr) /
// P(2jp+1, fr); v_permlane16_swap (odd rows of X <-> even rows of Y) leaves it
// 8 consecutive channels ((fq >> 1) * 8..) of pixel P(2jp + (fq & 1), fr).
// cb: this lane's 4 bias values (already times scale).
template <int F, int WI, int WJ, int II, int JP>
__device__ __forceinline__ void g_epi_pair(const f32x4 (&acc)[WI][WJ], const GEpi& e, const f32x4& cb,
                                           float (&gs)[WI][2], float (&gq)[WI][2], const g_u2l& rx2,
                                           const g_u2l& ry2) {
#pragma clang fp contract(off)      // explicit fmas: every instantiation rounds alike
  const int fr = e.lane & 15, fq = e.lane >> 4;
  // accumulators leave the AGPRs here, one pair at a time (plain reads were
  // hoisted as one 256-register block ahead of the epilogue, spilling)
  f32x4 x, y;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(x[k]) : "a"(acc[II][2 * JP][k]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(y[k]) : "a"(acc[II][2 * JP + 1][k]));
  }
  const int cl = e.m0 + e.wm * 16 * WI + II * 16 + fq * 4;        // channel (pre-swap)
  const int px = e.wn * 16 * WJ + 2 * JP * 16 + fr;               // tile-local pixel (pre-swap)
  float vx[4], vy[4];
  (void)cl;
  (void)px;
  if constexpr ((F & F_RES) || (F & F_DSILU)) {
    const bf16x4 rx = __builtin_bit_cast(bf16x4, rx2), ry = __builtin_bit_cast(bf16x4, ry2);
    if constexpr (F & F_DSILU) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        vx[k] = x[k] * e.as * dsiluf_((float)rx[k]);
        vy[k] = y[k] * e.as * dsiluf_((float)ry[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        vx[k] = __builtin_fmaf((float)rx[k], e.rs, __builtin_fmaf(x[k], e.as, cb[k]));
        vy[k] = __builtin_fmaf((float)ry[k], e.rs, __builtin_fmaf(y[k], e.as, cb[k]));
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      vx[k] = __builtin_fmaf(x[k], e.as, cb[k]);
      vy[k] = __builtin_fmaf(y[k], e.as, cb[k]);
    }
  }
  bf16x4 ox, oy;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ox[k] = (bf16)vx[k];
    oy[k] = (bf16)vy[k];
  }
  if constexpr (F & F_GN) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float fx = (float)ox[k], fy = (float)oy[k];
      gs[II][(2 * JP * 16) / 64] += fx + fy;
      gq[II][(2 * JP * 16) / 64] += fx * fx + fy * fy;
    }
  }
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  const u2 ux = __builtin_bit_cast(u2, ox), uy = __builtin_bit_cast(u2, oy);
  const auto s0 = __builtin_amdgcn_permlane16_swap(ux[0], uy[0], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(ux[1], uy[1], false, false);
  const g_u4 v = {s0[0], s1[0], s0[1], s1[1]};
  const int pl = e.wn * 16 * WJ + (2 * JP + (fq & 1)) * 16 + fr;    // tile-local pixel (post-swap)
  const int cs = e.m0 + e.wm * 16 * WI + II * 16 + (fq >> 1) * 8;
  g_store16(e.obase, e.orec, v, cs < e.M ? (pl * e.ldo + cs) * 2 : (int)0x80000000);
  __builtin_amdgcn_sched_barrier(0);       // one pair at a time: bounded live registers
}

// ---- F_MF epilogue: M a multiple of the tile (every FiLM / projection width).
// No channel masks: each lane's store / residual offsets are one per-tile base
// plus compile-time steps (fragment row ii: +32 bytes, an immediate; pair jp:
// +64 pixel rows), and the arithmetic is packed -- per fragment pair 8
// accumulator reads, 4 v_pk_fma (bias / scale), 4 v_cvt_pk_bf16_f32, 2 swaps
// and one store.  The generic epilogue above spent ~36 instructions per pair
// on per-element fmas, single-value converts re-packed by v_perm / v_alignbit
// and masked-lane address math (1161 per 256 x 256 tile and wave, ~12 % of a
// K = 1024 tile's time with the matrix pipe idle).
typedef float g_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned g_cvt_pk(g_f2 v) {
  unsigned r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(v[0]), "v"(v[1]));
  return r;
}
__device__ __forceinline__ g_f2 g_bf2f(unsigned u) {      // two packed bf16 -> fp32 (exact)
  return g_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
template <int F, int WI, int WJ, int II, int JP>
__device__ __forceinline__ void g_epi_pair_mf(const f32x4 (&acc)[WI][WJ], bf16* ob, int orec, int so, g_f2 as2,
                                              g_f2 rs2, g_f2 c01, g_f2 c23, float as, const g_u2l& rx2,
                                              const g_u2l& ry2) {
#pragma clang fp contract(off)
  f32x4 x, y;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(x[k]) : "a"(acc[II][2 * JP][k]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(y[k]) : "a"(acc[II][2 * JP + 1][k]));
  }
  g_f2 x0 = {x[0], x[1]}, x1 = {x[2], x[3]}, y0 = {y[0], y[1]}, y1 = {y[2], y[3]};
  if constexpr (F & F_DSILU) {
    const bf16x4 rx = __builtin_bit_cast(bf16x4, rx2), ry = __builtin_bit_cast(bf16x4, ry2);
    x0 = g_f2{x[0] * as * dsiluf_((float)rx[0]), x[1] * as * dsiluf_((float)rx[1])};
    x1 = g_f2{x[2] * as * dsiluf_((float)rx[2]), x[3] * as * dsiluf_((float)rx[3])};
    y0 = g_f2{y[0] * as * dsiluf_((float)ry[0]), y[1] * as * dsiluf_((float)ry[1])};
    y1 = g_f2{y[2] * as * dsiluf_((float)ry[2]), y[3] * as * dsiluf_((float)ry[3])};
  } else {
    x0 = __builtin_elementwise_fma(x0, as2, c01);
    x1 = __builtin_elementwise_fma(x1, as2, c23);
    y0 = __builtin_elementwise_fma(y0, as2, c01);
    y1 = __builtin_elementwise_fma(y1, as2, c23);
    if constexpr (F & F_RES) {
      x0 = __builtin_elementwise_fma(g_bf2f(rx2[0]), rs2, x0);
      x1 = __builtin_elementwise_fma(g_bf2f(rx2[1]), rs2, x1);
      y0 = __builtin_elementwise_fma(g_bf2f(ry2[0]), rs2, y0);
      y1 = __builtin_elementwise_fma(g_bf2f(ry2[1]), rs2, y1);
    }
  }
  const auto s0 = __builtin_amdgcn_permlane16_swap(g_cvt_pk(x0), g_cvt_pk(y0), false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(g_cvt_pk(x1), g_cvt_pk(y1), false, false);
  const g_u4 v = {s0[0], s1[0], s0[1], s1[1]};
  g_store16(ob, orec, v, so + II * 32);
  __builtin_amdgcn_sched_barrier(0);
}

// NST: LDS stages in the ring (NST - 1 DMAs in flight).  The small problems
// (one or two tiles per CU, K <= 1024: attention / NIN projections and their
// input gradients at 8x8 .. 32x32) are latency-bound with two stages -- each
// stage waits a whole HBM round trip for 8 MFMAs -- so they take 4.
template <int WI, int WJ, int F, int NST = 2, int NW = 4>
__global__ void __launch_bounds__(64 * NW, 1)
gemm_fw_k(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ O, const float* __restrict__ bias,
          const bf16* __restrict__ R, int M, int N, int K, int lda, int ldb, int ldo, int ldr, float alpha,
          float scale, int mt, int nt, int gm, float* __restrict__ gnp, int gn_groups, int gn_hw,
          const bf16* __restrict__ B2, int K1) {
  constexpr bool BIAS = (F & (F_B32 | F_B16)) != 0, BBF = (F & F_B16) != 0;
  using C = GCfg<WI, WJ, NST, NW>;
  // 4 bias slots: the loader may run at most 3 tiles ahead -- NST 4 needs K >= 128 (host)
  static_assert(NST == 2 || NST == 4, "stage ring of 2 or 4");
  __shared__ __attribute__((aligned(16))) bf16 smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const int G = gridDim.x;
  int rb = blockIdx.x;
  {
    const int q = G / 8, r = G % 8, xcd = rb % 8;
    rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + rb / 8;
  }
  const int ntiles = mt * nt;
  if (rb >= ntiles) return;
  const int nk = K / G_BK;                   // K-steps: even (K % 64 == 0), >= 4

  // tile id -> (m tile, n tile): m fastest inside groups of gm m tiles
  auto tile_mn = [&](int tl, int& mb_, int& nb_) {
    const int full = mt / gm, span = gm * nt;
    if (tl < full * span) {
      const int g = tl / span, r = tl - g * span;
      mb_ = g * gm + r % gm;
      nb_ = r / gm;
    } else {
      const int rem = mt - full * gm, r = tl - full * span;
      mb_ = full * gm + r % rem;
      nb_ = r / rem;
    }
  };

  // loader: per operand DA / DB pieces of 8 rows (128-byte rows, 8 lanes a
  // row), lane -> (row lane >> 3, LDS slot lane & 7 holding chunk slot ^ (row & 7))
  // One VGPR per operand: piece q adds q * 8 rows, an opaque (never hoisted)
  // v_add at the DMA -- sixteen live offsets spilled the 8x8 variants.
  int aoff, boff;
  {
    const int chunk = (lane & 7) ^ (lane >> 3);
    aoff = ((wave * C::RA + (lane >> 3)) * lda + chunk * 8) * 2;
    boff = ((wave * C::RB + (lane >> 3)) * ldb + chunk * 8) * 2;
  }
  const int astep = 8 * lda * 2, bstep = 8 * ldb * 2;
  auto piece_off = [](int base, int step) { return g_vadd(base, step); };
  const int fr = lane & 15, fq = lane >> 4;
  // fragment read offsets (bf16 elements within a stage) of the stage's
  // first K-step; the second K-step is chunk + 4 (offset fh); fragment i is
  // 16 rows further (16 * G_PK elements: the swizzle depends on row & 7 only)
  const int fa0 = g_swz(wm * 16 * WI + fr, fq), fb0 = g_swz(C::BM + wn * 16 * WJ + fr, fq);
  const int fa1 = g_swz(wm * 16 * WI + fr, fq + 4), fb1 = g_swz(C::BM + wn * 16 * WJ + fr, fq + 4);

  // loader cursor: tile ltile (descriptors lA / lB), byte offset lkb of its
  // next K-tile; the following tile's descriptors are prepared when the
  // cursor enters a tile
  int ltile = rb, lkb = 0;
  struct Ops {                               // one tile's operand panels: descriptor bases / sizes
    const bf16* a;
    const bf16* b;
    const bf16* b2;                          // F_CAT: second half, based K1 elements early (K offsets run on)
    int ra, rb, rb2;
    long m0;
  };
  Ops lo, no;
  auto ops_of = [&](int tl) -> Ops {
    const bool v = tl < ntiles;
    int mb_ = 0, nb_ = 0;
    if (v) tile_mn(tl, mb_, nb_);
    const long m0 = (long)mb_ * C::BM, n0 = (long)nb_ * C::BN;
    const long arows = M - m0 < C::BM ? M - m0 : C::BM, brows = N - n0 < C::BN ? N - n0 : C::BN;
    Ops o;
    o.a = A + m0 * lda;
#if defined(D3D_GEMM_X_L2B)            // timing-only build (wrong results): every tile reads B rows 0.. (L2-resident)
    o.b = B;
#else
    o.b = B + n0 * ldb;
#endif
    o.ra = v ? (int)((arows - 1) * lda + K) * 2 : 0;
    o.rb = v ? (int)((brows - 1) * ldb + K) * 2 : 0;
    if constexpr ((F & F_CAT) != 0) {
      // each half ends exactly at its last valid row: rows past N read zeros
      // (ldb = K1 < K, so the plain range would reach into the next rows)
      o.b2 = B2 + n0 * ldb - K1;
      o.rb = v ? (int)(brows * ldb) * 2 : 0;
      o.rb2 = v ? (int)(brows * ldb + K1) * 2 : 0;
    } else {
      o.b2 = nullptr;
      o.rb2 = 0;
    }
    o.m0 = v ? m0 : -1;
    return o;
  };
  lo = ops_of(ltile);
  no = ops_of(ltile + G);
  int lbslot = 0;                            // bias slot of the loader's tile (tile count & 3)
  // bias of the loader's tile: wave 0 DMAs it (one instruction) with the tile's first K-tile
  auto bias_dma = [&]() {
    if (BIAS && wave == 0 && lo.m0 >= 0) {
      const long m0 = lo.m0;
      g_dma(BBF ? (const void*)(reinterpret_cast<const bf16*>(bias) + m0) : (const void*)(bias + m0),
            (int)((M - m0 < C::BM ? M - m0 : C::BM) * (BBF ? 2 : 4)), smem + C::BIAS + lbslot * 512, lane * 16, 0);
    }
  };
  auto advance = [&]() {                     // after the pieces of one stage (two K-steps)
    lkb += G_PK * 2;
    if (lkb == K * 2) {
      lkb = 0;
      lo = no;
      lbslot = (lbslot + 1) & 3;
      ltile += G;
      no = ops_of(ltile + G);
    }
  };
  auto dma = [&](int st, int d) {            // piece d (< DA: A, else B) into stage st
    if (d < C::DA)
      g_dma(lo.a, lo.ra, smem + st * C::STAGE + (wave * C::RA + d * 8) * G_PK,
            d ? piece_off(aoff, d * astep) : aoff, lkb);
    else if constexpr ((F & F_CAT) != 0) {
      const bool hi = lkb >= 2 * K1;         // K-stages never straddle the split (K1 % 64 == 0)
      g_dma(hi ? lo.b2 : lo.b, hi ? lo.rb2 : lo.rb,
            smem + st * C::STAGE + (C::BM + wave * C::RB + (d - C::DA) * 8) * G_PK,
            d > C::DA ? piece_off(boff, (d - C::DA) * bstep) : boff, lkb);
    } else {
#if defined(D3D_GEMM_X_SKIPB)        // timing-only builds (wrong results): B's DMA not issued / ...
      return;
#endif
#if defined(D3D_GEMM_X_ZEROB)        // ... issued against an empty descriptor (no traffic)
      g_dma(lo.b, 0, smem + st * C::STAGE + (C::BM + wave * C::RB + (d - C::DA) * 8) * G_PK,
            d > C::DA ? piece_off(boff, (d - C::DA) * bstep) : boff, lkb);
#else
#ifndef D3D_GEMM_B_CPOL
#define D3D_GEMM_B_CPOL 0          // cache policy of the activation (B) stream: A/B build knob
#endif
      g_dma_cp<D3D_GEMM_B_CPOL>(lo.b, lo.rb, smem + st * C::STAGE + (C::BM + wave * C::RB + (d - C::DA) * 8) * G_PK,
                                d > C::DA ? piece_off(boff, (d - C::DA) * bstep) : boff, lkb);
#endif
    }
  };

  bf16x8 a0[WI], b0[WJ], a1[WI], b1[WJ];
  f32x4 acc[WI][WJ];
  int tile = rb, ti = 0, mb, nb;
  tile_mn(tile, mb, nb);
  bias_dma();
#pragma unroll
  for (int k = 0; k < NST; ++k) {            // stages 0 .. NST-1 (may run into the next tiles)
#pragma unroll
    for (int d = 0; d < C::ND; ++d) dma(k, d);
    advance();
    // the cursor entered the next tile: its bias (K = 128 crosses inside the
    // prologue; without this the second tile of a block read a stale slot)
    if (lkb == 0) bias_dma();
  }
  // stage 0 landed (a bias DMA between stages only makes the count stricter)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 1) * C::ND) : "memory");
  G_BAR();
#pragma unroll
  for (int j = 0; j < WJ; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + fb0 + j * 16 * G_PK);
#pragma unroll
  for (int i = 0; i < WI; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + fa0 + i * 16 * G_PK);

  // K-step s = 2p + h uses stage p & 1.  Body s: NM slots, each one MFMA of
  // K-step s plus at most one other instruction -- the fragment reads of
  // s + 1 (B fragments first: the next step's first row needs all of them)
  // and, in odd bodies, the DMA of stage p + 2 into stage p & 1 (free: its
  // last fragments were read in body 2p) and the cursor update.  Odd bodies
  // open with the wait for stage p + 1 (issued one stage earlier; after an
  // epilogue its NS stores may stay in flight) and the only barrier of the
  // stage: it publishes stage p + 1 and frees stage p & 1.
  int s = 0;
  auto body = [&](auto first, auto odd, auto last, bf16x8(&ca)[WI], bf16x8(&cb)[WJ], bf16x8(&na)[WI],
                  bf16x8(&nbf)[WJ], bool after_epi) {
    constexpr bool ODD = decltype(odd)::value, LAST = decltype(last)::value;
    if constexpr (ODD) {
      // lgkmcnt(0): this wave's fragment reads of the stage the DMAs below
      // refill (issued in the previous body) must have completed before the
      // barrier frees that stage.  Without it another wave's DMA could land
      // on top of a read still queued in the LDS pipeline -- which happened
      // whenever an LDS-heavy kernel shared the CU (the per-pixel weight
      // gradients on the side stream): wrong GEMM outputs under co-residency
      // (tools/stress_concurrent.py, profiles/race_graph_wgrad_flush_r3.txt).
      // stage p + 1 landed; stages p + 2 .. p + NST - 1 (and the epilogue's
      // stores) may stay in flight
      if (after_epi) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * C::ND + C::NS) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * C::ND) : "memory");
      G_BAR();
    }
    // next K-step's fragments: second half of this stage, or first half of the next
    const bf16* sn = smem + (ODD ? (((s >> 1) + 1) & (NST - 1)) : ((s >> 1) & (NST - 1))) * C::STAGE;
    const int ra = ODD ? fa0 : fa1, rbo = ODD ? fb0 : fb1;
    const int ls = (s >> 1) & (NST - 1);        // stage p's slot: refilled with stage p + NST
    g_for(std::make_integer_sequence<int, C::NM>{}, [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (decltype(first)::value) g_mma0(acc[k / WJ][k % WJ], ca[k / WJ], cb[k % WJ]);
      else g_mma(acc[k / WJ][k % WJ], ca[k / WJ], cb[k % WJ]);
      g_for(std::make_integer_sequence<int, C::NR>{}, [&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if constexpr (!LAST && r * C::NM / C::NR == k) {
          if constexpr (r < WJ) nbf[r] = *reinterpret_cast<const bf16x8*>(sn + rbo + r * 16 * G_PK);
          else na[r - WJ] = *reinterpret_cast<const bf16x8*>(sn + ra + (r - WJ) * 16 * G_PK);
        }
      });
      if constexpr (ODD) {
        // DMA pieces at slots (2d + 1) * NM / (2 ND); the cursor moves after the last
        g_for(std::make_integer_sequence<int, C::ND>{}, [&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if constexpr ((2 * d + 1) * C::NM / (2 * C::ND) == k) {
            dma(ls, d);
            if constexpr (d == C::ND - 1) {
              advance();
              if (lkb == 0) bias_dma();
            }
          }
        });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    ++s;
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;

  // (the tile's last K-step reads no fragments: the next tile's first ones
  // are read after the epilogue, so they do not occupy registers across it)
  while (true) {
    body(T_{}, F_{}, F_{}, a0, b0, a1, b1, false);
    body(F_{}, T_{}, F_{}, a1, b1, a0, b0, ti > 0);
    for (int t = 2; t < nk - 2; t += 2) {
      body(F_{}, F_{}, F_{}, a0, b0, a1, b1, false);
      body(F_{}, T_{}, F_{}, a1, b1, a0, b0, false);
    }
    body(F_{}, F_{}, F_{}, a0, b0, a1, b1, false);
    body(F_{}, T_{}, T_{}, a1, b1, a0, b0, false);
    // ---- epilogue of tile (mb, nb)
    if constexpr ((F & F_MF) != 0) {
      static_assert((F & F_GN) == 0, "F_MF: no GroupNorm partials");
      constexpr bool RR = (F & (F_RES | F_DSILU)) != 0;
      const long m0 = (long)mb * C::BM, n0 = (long)nb * C::BN;
      const long rows = N - n0 < C::BN ? N - n0 : C::BN;
      bf16* ob = O + n0 * ldo;
      const int orec = (int)(rows * ldo * 2);
      const bf16* rbs = RR ? R + n0 * ldr : nullptr;
      const int rrec = RR ? (int)(rows * ldr * 2) : 0;
      int ln = lane;                       // opaque: per-lane offsets stay inside the tile loop
      asm volatile("" : "+v"(ln));
      const int fr = ln & 15, fq = ln >> 4;
      const int cw = (int)m0 + wm * 16 * WI;
      // store: pixel wn*16WJ + (2jp + (fq&1))*16 + fr, channel cw + ii*16 + (fq>>1)*8
      const int so0 = ((wn * 16 * WJ + (fq & 1) * 16 + fr) * ldo + cw + (fq >> 1) * 8) * 2;
      // residual (pre-swap): pixel wn*16WJ + 2jp*16 + fr (+16 for the pair's second), channel cw + ii*16 + fq*4
      const int ro0 = RR ? ((wn * 16 * WJ + fr) * ldr + cw + fq * 4) * 2 : 0;
      const float as = (F & F_DSILU) ? alpha : alpha * scale;
      const g_f2 as2 = {as, as}, rs2 = {scale, scale};
      const bf16* sb = smem + C::BIAS + (ti & 3) * 512;
      g_u2l rbuf[2][WJ / 2][2];
      auto rload = [&](auto ic, int slot) {
        constexpr int ii = decltype(ic)::value;
        g_for(std::make_integer_sequence<int, WJ / 2>{}, [&](auto jc) {
          constexpr int jp = decltype(jc)::value;
          rbuf[slot][jp][0] = g_load8(rbs, rrec, ro0 + jp * 64 * ldr + ii * 32);
          rbuf[slot][jp][1] = g_load8(rbs, rrec, ro0 + (jp * 64 + 32) * ldr + ii * 32);
        });
      };
      if constexpr (RR) rload(std::integral_constant<int, 0>{}, 0);
      g_for(std::make_integer_sequence<int, WI>{}, [&](auto ic) {
        constexpr int ii = decltype(ic)::value;
        if constexpr (RR && ii + 1 < WI) rload(std::integral_constant<int, ii + 1>{}, (ii + 1) & 1);
        g_f2 c01 = {0.f, 0.f}, c23 = {0.f, 0.f};
        const int cl = wm * 16 * WI + ii * 16 + fq * 4;
        if constexpr (F & F_B32) {
          const f32x4 c4 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(sb) + cl);
          c01 = g_f2{c4[0], c4[1]} * rs2;
          c23 = g_f2{c4[2], c4[3]} * rs2;
        } else if constexpr (F & F_B16) {
          const bf16x4 c4 = *reinterpret_cast<const bf16x4*>(sb + cl);
          c01 = g_f2{(float)c4[0], (float)c4[1]} * rs2;
          c23 = g_f2{(float)c4[2], (float)c4[3]} * rs2;
        }
        g_for(std::make_integer_sequence<int, WJ / 2>{}, [&](auto jc) {
          constexpr int jp = decltype(jc)::value;
          g_epi_pair_mf<F, WI, WJ, ii, jp>(acc, ob, orec, so0 + jp * 64 * ldo, as2, rs2, c01, c23, as,
                                           rbuf[ii & 1][jp][0], rbuf[ii & 1][jp][1]);
        });
      });
    } else {
      GEpi e;
      const long m0 = (long)mb * C::BM, n0 = (long)nb * C::BN;
      const long rows = N - n0 < C::BN ? N - n0 : C::BN;
      e.obase = O + n0 * ldo;
      e.orec = (int)(rows * ldo * 2);
      e.R = (F & (F_RES | F_DSILU)) ? R + n0 * ldr : nullptr;
      e.rrec = (F & (F_RES | F_DSILU)) ? (int)(rows * ldr * 2) : 0;
      e.M = M;
      e.ldo = ldo;
      e.ldr = ldr;
      e.as = (F & F_DSILU) ? alpha : alpha * scale;
      e.bs = scale;
      e.rs = scale;
      e.m0 = (int)m0;
      e.wm = wm;
      e.wn = wn;
      // an opaque copy of the lane id: the per-lane addressing below cannot be
      // hoisted out of the tile loop (where it would occupy registers across
      // the K loop)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      e.lane = ln;
      float gs[WI][2], gq[WI][2];
#pragma unroll
      for (int i = 0; i < WI; ++i) gs[i][0] = gq[i][0] = gs[i][1] = gq[i][1] = 0.f;
      const bf16* sb = smem + C::BIAS + (ti & 3) * 512;
      // residual rows: fragment row ii + PD's reads are issued before row
      // ii's pairs (PD + 1 row buffers, compile-time indexed): each row's
      // reads get PD rows of epilogue work to land in
#ifdef D3D_GEMM_EPI_SERIAL
      constexpr bool RD = false;                 // A/B build: each pair reads its rows right before use
      constexpr bool RS = (F & (F_RES | F_DSILU)) != 0;
#else
      constexpr bool RD = (F & (F_RES | F_DSILU)) != 0;
      constexpr bool RS = false;
#endif
#ifndef D3D_GEMM_EPI_PD
#define D3D_GEMM_EPI_PD 1        // 3 rows ahead measured -0.4 % bs128 (profiles/r5/epi_pd/)
#endif
      constexpr int PD = D3D_GEMM_EPI_PD < WI - 1 ? D3D_GEMM_EPI_PD : (WI > 1 ? WI - 1 : 1);
      constexpr int NB = PD + 1;
      g_u2l rbuf[NB][WJ / 2][2];
      if constexpr (RD) {
        g_for(std::make_integer_sequence<int, PD>{}, [&](auto rc) {
          constexpr int r0 = decltype(rc)::value;
          g_for(std::make_integer_sequence<int, WJ / 2>{}, [&](auto jc) {
            g_epi_rload<WI, WJ, r0, decltype(jc)::value>(e, rbuf[r0 % NB][decltype(jc)::value][0],
                                                          rbuf[r0 % NB][decltype(jc)::value][1]);
          });
        });
      }
      g_for(std::make_integer_sequence<int, WI>{}, [&](auto ic) {
        constexpr int ii = decltype(ic)::value;
        if constexpr (RD && ii + PD < WI) {
          g_for(std::make_integer_sequence<int, WJ / 2>{}, [&](auto jc) {
            g_epi_rload<WI, WJ, ii + PD, decltype(jc)::value>(e, rbuf[(ii + PD) % NB][decltype(jc)::value][0],
                                                               rbuf[(ii + PD) % NB][decltype(jc)::value][1]);
          });
        }
        f32x4 cb = {0.f, 0.f, 0.f, 0.f};
        const int cl = wm * 16 * WI + ii * 16 + (ln >> 4) * 4;       // tile-local channel of the lane
        if constexpr (F & F_B32) {
          cb = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(sb) + cl);
        } else if constexpr (F & F_B16) {
          const bf16x4 c4 = *reinterpret_cast<const bf16x4*>(sb + cl);
#pragma unroll
          for (int k = 0; k < 4; ++k) cb[k] = (float)c4[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) cb[k] *= scale;
        g_for(std::make_integer_sequence<int, WJ / 2>{}, [&](auto jc) {
          constexpr int jp = decltype(jc)::value;
          if constexpr (RS) g_epi_rload<WI, WJ, ii, jp>(e, rbuf[ii % NB][jp][0], rbuf[ii % NB][jp][1]);
          g_epi_pair<F, WI, WJ, ii, jp>(acc, e, cb, gs, gq, rbuf[ii % NB][jp][0], rbuf[ii % NB][jp][1]);
        });
      });
      if constexpr ((F & F_GN) && WJ >= 4) {
        float s2[WI][WJ / 4], q2[WI][WJ / 4];
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int h = 0; h < WJ / 4; ++h) {
            s2[i][h] = gs[i][h];
            q2[i][h] = gq[i][h];
          }
        gn_part_store<WI, WJ / 4>(s2, q2, ln, (int)(m0 + wm * 16 * WI), n0 + wn * 16 * WJ, M, gn_groups, gn_hw, N,
                                  gnp);
      }
    }
    tile += G;
    if (tile >= ntiles) break;
    ++ti;
    tile_mn(tile, mb, nb);
    {   // first fragments of the next tile: stage s / 2, published by the last body's barrier
      const bf16* sn = smem + ((s >> 1) & (NST - 1)) * C::STAGE;
#pragma unroll
      for (int j = 0; j < WJ; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(sn + fb0 + j * 16 * G_PK);
#pragma unroll
      for (int i = 0; i < WI; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(sn + fa0 + i * 16 * G_PK);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the block ends
}


// Launch arguments shared by the host dispatcher (gemm.hip) and the per-tile
// instantiation units.
struct GArgs {
  int G_;
  hipStream_t st;
  const void *A, *B;
  void* O;
  const void *bias, *R;
  int M, N, K, lda, ldb, ldo, ldr;
  float alpha, scale;
  int mt, nt, gm;
  float* gnp;
  int G, hw;
  const void* B2;
  int K1;
};

// W: 8 / 4 / 2 = 4 waves of W x W fragments (tile 32W x 32W); 9 = 8 waves of
// 8 x 4 fragments (256 x 256 tile, two waves per SIMD)
template <int W, int F, int NST>
static int g_run(const GArgs& a) {
  constexpr int WI = W == 9 ? 8 : W, WJ = W == 9 ? 4 : W, NW = W == 9 ? 8 : 4;
  hipLaunchKernelGGL((gemm_fw_k<WI, WJ, F, NST, NW>), dim3(a.G_), dim3(64 * NW), 0, a.st, (const bf16*)a.A,
                     (const bf16*)a.B, (bf16*)a.O, (const float*)a.bias, (const bf16*)a.R, a.M, a.N, a.K, a.lda, a.ldb,
                     a.ldo, a.ldr, a.alpha, a.scale, a.mt, a.nt, a.gm, a.gnp, a.G, a.hw, (const bf16*)a.B2, a.K1);
  return (int)hipGetLastError();
}

// Epilogue variants instantiated per tile size (F flags, gemm_fw_k), in
// lists small enough to compile in parallel units.
template <int... Fs>
struct GFlags {};
using GFlagsPlain = GFlags<0, F_B32, F_B16, F_RES, F_B32 | F_RES, F_B16 | F_RES, F_DSILU, F_CAT, F_B32 | F_CAT>;
using GFlagsMF = GFlags<F_MF, F_B32 | F_MF, F_B16 | F_MF, F_RES | F_MF, F_B32 | F_RES | F_MF, F_B16 | F_RES | F_MF,
                        F_DSILU | F_MF, F_CAT | F_MF, F_B32 | F_CAT | F_MF>;
using GFlagsGN = GFlags<F_GN, F_B32 | F_GN, F_RES | F_GN, F_B32 | F_RES | F_GN>;

// deep: the 4-stage ring (tiles smaller than 256 x 256 only)
template <int W, int... Fs>
static int g_dispatch(int F, bool deep, const GArgs& a, GFlags<Fs...>) {
  int rc = -2;
  (void)((F == Fs ? (rc = (W < 8 && deep) ? g_run<W, Fs, (W < 8 ? 4 : 2)>(a) : g_run<W, Fs, 2>(a), true)
                  : false) || ...);
  return rc;
}

// Instantiation units (gemm_w*.hip): tile size W (8 / 4 / 2; 9 = the 8-wave 256 x 256 tile), flag list L
// (0 plain + concat, 1 F_MF, 2 GroupNorm partials); -2 when F is not in L.
int gemm_dispatch_w8_0(int F, bool deep, const GArgs& a);
int gemm_dispatch_w8_1(int F, bool deep, const GArgs& a);
int gemm_dispatch_w8_2(int F, bool deep, const GArgs& a);
int gemm_dispatch_w4_0(int F, bool deep, const GArgs& a);
int gemm_dispatch_w4_1(int F, bool deep, const GArgs& a);
int gemm_dispatch_w4_2(int F, bool deep, const GArgs& a);
int gemm_dispatch_w9_0(int F, bool deep, const GArgs& a);
int gemm_dispatch_w9_1(int F, bool deep, const GArgs& a);
int gemm_dispatch_w9_2(int F, bool deep, const GArgs& a);
int gemm_dispatch_w2_0(int F, bool deep, const GArgs& a);
int gemm_dispatch_w2_1(int F, bool deep, const GArgs& a);

static int gemm_dispatch(int W, int F, bool deep, const GArgs& a) {
  int rc = -2;
  if (W == 8) {
    if ((rc = gemm_dispatch_w8_0(F, deep, a)) == -2 && (rc = gemm_dispatch_w8_1(F, deep, a)) == -2)
      rc = gemm_dispatch_w8_2(F, deep, a);
  } else if (W == 9) {
    if ((rc = gemm_dispatch_w9_0(F, deep, a)) == -2 && (rc = gemm_dispatch_w9_1(F, deep, a)) == -2)
      rc = gemm_dispatch_w9_2(F, deep, a);
  } else if (W == 4) {
    if ((rc = gemm_dispatch_w4_0(F, deep, a)) == -2 && (rc = gemm_dispatch_w4_1(F, deep, a)) == -2)
      rc = gemm_dispatch_w4_2(F, deep, a);
  } else if (W == 2) {
    if ((rc = gemm_dispatch_w2_0(F, deep, a)) == -2) rc = gemm_dispatch_w2_1(F, deep, a);
  }
  return rc == -2 ? -1 : rc;
}
