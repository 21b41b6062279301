// Dense per-pixel GEMM on the gfx950 matrix cores: the 1x1 layers of the
// X-UNet (FiLM projections `xunet.py:74-87`, attention in/out projections
// `xunet.py:154-177`, NIN skips `xunet.py:128-129`) as
//
//     O[n][m] = (alpha * sum_k A[m][k] * B[n][k] + bias[m] + R[n][m]) * scale
//
// with A the bf16 weight ([M][lda], K contiguous), B the NHWC activations
// ([N][ldb], K contiguous), O / R NHWC bf16 rows of stride ldo / ldr.
//
// Schedule ("ping-pong", one 256 x 256 output tile per 512-thread block):
//   * 8 waves as 2 (M) x 4 (N), 128 x 64 outputs each (8 x 4 MFMA 16x16x32
//     tiles, 128 fp32 accumulators), two waves per SIMD -- one of each M half;
//   * the M-half-1 waves run one barrier behind the M-half-0 waves, so on every
//     SIMD one wave issues its 16 MFMAs while its partner issues the next
//     phase's ds_reads and LDS-DMA: the matrix core never waits for a
//     fragment read or a DMA issue;
//   * a 64-deep K-tile is four phases (quadrants of the wave tile: 64 x 32 x 64
//     = 16 MFMAs), and its LDS image is four 16-KiB pieces (A rows of M-quarter
//     0 / 2, B rows of N-eighth 0 / 2 of each wave, ...) restaged one piece per
//     phase into the other of two stages -- each piece is read 1-3 phases
//     after the wave's counted `vmcnt(4)` retires it (never `vmcnt(0)` in the
//     loop), and rewritten >= 4 phases after its last read;
//   * LDS-DMA (`buffer_load ... lds`, 16 B per lane) with the XOR chunk swizzle
//     applied to the source address, conflict-free `ds_read_b128` fragments;
//   * per-block buffer descriptors (row base m0 / n0), so 32-bit offsets cover
//     operands of any size and rows past M / N read as zeros;
//   * bijective XCD remap: the blocks of one N tile (sharing the activation
//     panel) run on one XCD.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace {
constexpr int PP_BK = 64;
constexpr int PP_PIECE = 128 * PP_BK;       // bf16 elements per LDS piece (16 KiB)
constexpr int PP_STAGE = 4 * PP_PIECE;      // one K-tile (64 KiB)
// behind the two stages: two 1-KiB bias slots (tile parity) and a 1-KiB sink
// for the aux DMA of K-tiles that carry no bias (see pp_issue)
constexpr int PP_BIAS = 2 * PP_STAGE;       // bf16 offset of the bias slots
constexpr int PP_SINK = PP_BIAS + 1024;
constexpr int PP_LDS = PP_SINK + 512;

__device__ __forceinline__ int pp_swz(int row, int chunk) { return row * PP_BK + ((chunk ^ (row & 7)) << 3); }

// Issue piece `p` (0: A mi0, 1: B ni0, 2: B ni1, 3: A mi1 -> LDS slots 0, 1, 3, 2)
// of K-tile `t` into stage `s & 1`: two 1-KiB DMA instructions per wave.
// Piece 0 carries a third, "aux" instruction in EVERY K-tile, so the counted
// waits stay uniform: on the first K-tile of a tile wave 0 DMAs the tile's 256
// fp32 biases into the bias slot (the epilogue then reads them from LDS -- no
// global load, hence no vmcnt drain of the in-flight pieces, in the epilogue);
// otherwise it is an out-of-range (no memory access) DMA into the sink.
__device__ __forceinline__ void pp_issue(bf16* smem, const bf16* A, const bf16* B, int a_rec, int b_rec, int t, int p,
                                         int wave, const int (&aoff)[2][2], const int (&boff)[2][2], int s,
                                         const float* aux = nullptr, int aux_rec = 0, int aux_dst = PP_SINK) {
  typedef __attribute__((address_space(3))) void lds_void;
  const int slot = p == 0 ? 0 : p == 1 ? 1 : p == 2 ? 3 : 2;
  bf16* dst = smem + (s & 1) * PP_STAGE + slot * PP_PIECE + wave * 16 * PP_BK;
  const int kb = t * PP_BK * 2;
  if (p == 0 || p == 3) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_rec, 0x00020000);
    const int h = p == 3;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, aoff[h][0], kb, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(dst + 8 * PP_BK), 16, aoff[h][1], kb, 0, 0);
    if (p == 0) {
      const __amdgpu_buffer_rsrc_t ra =
          __builtin_amdgcn_make_buffer_rsrc((void*)(aux ? (const void*)aux : (const void*)A), (short)0, aux_rec,
                                            0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(smem + aux_dst), 16,
                                               (int)(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))) * 16,
                                               0, 0, 0);
    }
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_rec, 0x00020000);
    const int h = p == 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, boff[h][0], kb, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(dst + 8 * PP_BK), 16, boff[h][1], kb, 0, 0);
  }
}

#define PP_BAR()                          \
  do {                                    \
    __builtin_amdgcn_sched_barrier(0);    \
    __builtin_amdgcn_s_barrier();         \
    __builtin_amdgcn_sched_barrier(0);    \
  } while (0)
}  // namespace

// Tile id -> (m tile, n tile): m fastest inside groups of `gm` m tiles, so the
// 32 consecutive ids an XCD runs at once share ~gm A panels and ~32/gm B panels.
__device__ __forceinline__ void pp_tile(int tile, int mt, int nt, int gm, int& mb, int& nb) {
  const int full = mt / gm, span = gm * nt;
  if (tile < full * span) {
    const int g = tile / span, r = tile - g * span;
    mb = g * gm + r % gm;
    nb = r / gm;
  } else {
    const int rem = mt - full * gm, r = tile - full * span;
    mb = full * gm + r % rem;
    nb = r / rem;
  }
}

struct PPTile {
  const bf16* A;
  const bf16* B;
  int a_rec, b_rec;
  long m0;
};

__device__ __forceinline__ PPTile pp_tile_ops(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb,
                                              int mb, int nb) {
  const long m0 = (long)mb * 256, n0 = (long)nb * 256;
  const long arows = M - m0 < 256 ? M - m0 : 256, brows = N - n0 < 256 ? N - n0 : 256;
  PPTile o;
  o.A = A + m0 * lda;
  o.B = B + n0 * ldb;
  o.a_rec = (int)((arows - 1) * lda + K) * 2;      // descriptor range: this tile's rows only
  o.b_rec = (int)((brows - 1) * ldb + K) * 2;
  o.m0 = m0;
  return o;
}

// Epilogue of one 256 x 256 tile: acc[ii][jj] holds rows m0 + wr*128 + ii*16 +
// fq*4 + e of pixel n0 + wn*64 + jj*16 + fr; the tile's biases are in LDS.
__device__ __forceinline__ void pp_epi(const f32x4 (&acc)[8][4], const float* __restrict__ sbias, bf16* __restrict__ O,
                                       const bf16* __restrict__ R, int M, int N, int ldo, int ldr, float alpha,
                                       float scale, long m0, long n0, int wr, int wn, int lane,
                                       float* __restrict__ gnp, int gn_groups, int gn_hw) {
  const int fr = lane & 15, fq = lane >> 4;
  const bool vec = (ldo & 3) == 0 && (!R || (ldr & 3) == 0);
  // fused GroupNorm partials of the output (host guarantees vec, M % 4 == 0,
  // gn_hw % 64 == 0): this wave's 64 pixels are one 64-pixel part
  float gs[8][1], gq[8][1];
#pragma unroll
  for (int ii = 0; ii < 8; ++ii) gs[ii][0] = gq[ii][0] = 0.f;
#pragma unroll
  for (int ii = 0; ii < 8; ++ii) {
    const long co = m0 + wr * 128 + ii * 16 + fq * 4;
    if (co >= M) continue;
    const f32x4 cb = sbias ? *reinterpret_cast<const f32x4*>(sbias + wr * 128 + ii * 16 + fq * 4)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const long pix = n0 + wn * 64 + jj * 16 + fr;
      if (pix >= N) continue;
      bf16* dst = O + pix * ldo + co;
      if (vec && co + 3 < M) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[ii][jj][e] * alpha + cb[e];
        if (R) {
          const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(R + pix * ldr + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o4[e] = (bf16)(v[e] * scale);
          const float yv = (float)o4[e];
          gs[ii][0] += yv;
          gq[ii][0] += yv * yv;
        }
        *reinterpret_cast<bf16x4*>(dst) = o4;
      } else {
        for (int e = 0; e < 4 && co + e < M; ++e) {
          float v = acc[ii][jj][e] * alpha + cb[e];
          if (R) v += (float)R[pix * ldr + co + e];
          dst[e] = (bf16)(v * scale);
        }
      }
    }
  }
  if (gnp) gn_part_store<8, 1>(gs, gq, lane, (int)(m0 + wr * 128), n0 + wn * 64, M, gn_groups, gn_hw, N, gnp);
}

// Persistent: each block walks tiles rb, rb + G, ... (rb = XCD-contiguous
// rank of the block, G = grid) as ONE stream of K-tiles -- the next tile's
// first pieces are in flight while this tile's last phases and its epilogue
// run, so neither the prologue latency nor the epilogue stores idle the CU.
__global__ void __launch_bounds__(512, 1)
gemm_pp_k(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ O, const float* __restrict__ bias,
          const bf16* __restrict__ R, int M, int N, int K, int lda, int ldb, int ldo, int ldr, float alpha,
          float scale, int mt, int nt, int gm, float* __restrict__ gnp, int gn_groups, int gn_hw) {
  __shared__ __attribute__((aligned(16))) bf16 smem[PP_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  int rb = blockIdx.x;
  {
    const int q = G / 8, r = G % 8, xcd = rb % 8;
    rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + rb / 8;
  }
  const int ntiles = mt * nt;
  if (rb >= ntiles) return;

  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  int aoff[2][2], boff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int prow = wave * 16 + q * 8 + lrow;                         // row of the 128-row piece
      const int ar = (prow >> 6) * 128 + h * 64 + (prow & 63);
      const int br = (prow >> 5) * 64 + h * 32 + (prow & 31);
      aoff[h][q] = (ar * lda + lchunk * 8) * 2;
      boff[h][q] = (br * ldb + lchunk * 8) * 2;
    }

  f32x4 acc[8][4];
  bf16x8 af[4][2], bq[2][2][2];
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = K / PP_BK;

  auto readA = [&](int st, int h) {
    const bf16* base = smem + st * PP_STAGE + (h ? 2 : 0) * PP_PIECE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][kk] = *reinterpret_cast<const bf16x8*>(base + pp_swz(wr * 64 + i * 16 + fr, kk * 4 + fq));
  };
  auto readB = [&](int st, int h) {
    const bf16* base = smem + st * PP_STAGE + (h ? 3 : 1) * PP_PIECE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bq[h][j][kk] = *reinterpret_cast<const bf16x8*>(base + pp_swz(wn * 32 + j * 16 + fr, kk * 4 + fq));
  };
  auto quad = [&](int mi, int ni) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mi * 4 + i][ni * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bq[ni][j][kk], acc[mi * 4 + i][ni * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  int tile = rb, mb, nb;
  pp_tile(tile, mt, nt, gm, mb, nb);
  PPTile cur = pp_tile_ops(A, B, M, N, K, lda, ldb, mb, nb);
  // aux DMA of a tile's first K-tile: its bias (wave 0), else the sink
  auto aux_of = [&](const PPTile& o, int parity, const float*& src, int& rec, int& dst) {
    src = nullptr;
    rec = 0;
    dst = PP_SINK;
    if (bias && wave == 0) {
      src = bias + o.m0;
      rec = (int)((M - o.m0 < 256 ? M - o.m0 : 256) * 4);
      dst = PP_BIAS + parity * 512;
    }
  };
  {
    const float* as;
    int ar, ad;
    aux_of(cur, 0, as, ar, ad);
    pp_issue(smem, cur.A, cur.B, cur.a_rec, cur.b_rec, 0, 0, wave, aoff, boff, 0, as, ar, ad);
  }
#pragma unroll
  for (int p = 1; p < 4; ++p) pp_issue(smem, cur.A, cur.B, cur.a_rec, cur.b_rec, 0, p, wave, aoff, boff, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  PP_BAR();
  if (wr == 1) PP_BAR();                 // the M-half-1 waves trail by one barrier

  int s = 0;                             // K-tile stream position (LDS stage = s & 1)
  int ti = 0;                            // tiles done by this block (bias slot = ti & 1)
  while (true) {
    const int ntile = tile + G;
    const bool more = ntile < ntiles;
    int nmb = 0, nnb = 0;
    if (more) pp_tile(ntile, mt, nt, gm, nmb, nnb);
    const PPTile nxtop = more ? pp_tile_ops(A, B, M, N, K, lda, ldb, nmb, nnb) : cur;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < nk; ++t, ++s) {
      const int st = s & 1;
      const bool in_tile = t + 1 < nk;
      const bool nxt = in_tile || more;
      // the K-tile after this one in the stream: (this tile, t + 1) or (next tile, 0)
      const PPTile& lo = in_tile ? cur : nxtop;
      const int lt = in_tile ? t + 1 : 0;
      const int ls = s + 1;
      // phase 0: quadrant (0, 0)
      readA(st, 0);
      readB(st, 0);
      if (nxt) {
        const float* as = nullptr;
        int ar = 0, ad = PP_SINK;
        if (!in_tile) aux_of(lo, (ti + 1) & 1, as, ar, ad);
        pp_issue(smem, lo.A, lo.B, lo.a_rec, lo.b_rec, lt, 0, wave, aoff, boff, ls, as, ar, ad);
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      PP_BAR();
      quad(0, 0);
      PP_BAR();
      // phase 1: quadrant (0, 1)
      readB(st, 1);
      if (nxt) {
        pp_issue(smem, lo.A, lo.B, lo.a_rec, lo.b_rec, lt, 1, wave, aoff, boff, ls);
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      PP_BAR();
      quad(0, 1);
      PP_BAR();
      // phase 2: quadrant (1, 1)
      readA(st, 1);
      if (nxt) pp_issue(smem, lo.A, lo.B, lo.a_rec, lo.b_rec, lt, 2, wave, aoff, boff, ls);
      PP_BAR();
      quad(1, 1);
      PP_BAR();
      // phase 3: quadrant (1, 0) from registers
      if (nxt) {
        pp_issue(smem, lo.A, lo.B, lo.a_rec, lo.b_rec, lt, 3, wave, aoff, boff, ls);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      PP_BAR();
      quad(1, 0);
      PP_BAR();
    }

    pp_epi(acc, bias ? reinterpret_cast<const float*>(smem + PP_BIAS) + (ti & 1) * 256 : nullptr, O, R, M, N, ldo, ldr,
           alpha, scale, (long)mb * 256, (long)nb * 256, wr, wn, lane, gnp, gn_groups, gn_hw);
    if (!more) break;
    ++ti;
    tile = ntile;
    mb = nmb;
    nb = nnb;
    cur = nxtop;
  }
  if (wr == 0) PP_BAR();                 // balance the trailing group's extra barrier
}

// ---------------------------------------------------------------- v2 ----
// BK = 32, FOUR LDS stages (32 KiB each: A then B, 256 rows x 64 B), ONE
// ping-pong phase per K-tile: 32 MFMAs per wave between the barriers (512
// cycles of matrix-core work per SIMD and wave, twice the v1 phase, so the
// barrier hand-over costs half as much), the stage of K-tile s + 3 issued in
// phase s (3 K-tiles ~ 3000 cycles of DMA latency budget), a uniform
// `vmcnt(10)` (5 DMA instructions per wave per K-tile: 2 A, 2 B, 1 aux; past
// the end of the stream they are out-of-range no-ops into the sink) and
// `lgkmcnt(0)` before each barrier, so the stage rewritten in phase s (last
// read in phase s - 1) has no reader left.
// 64-byte rows: chunk c of row r sits at 16-byte slot c ^ (((r >> 3) & 1) * 3),
// which makes every ds_read_b128 lane group hit 16 distinct bank slots.
namespace {
constexpr int Q_BK = 32;
constexpr int Q_STAGE = 2 * 256 * Q_BK;     // bf16 elements per stage (A rows 0..255, then B rows)
constexpr int Q_NST = 4;
constexpr int Q_BIAS = Q_NST * Q_STAGE;     // 4 bias slots (tile & 3) of 256 fp32
constexpr int Q_SINK = Q_BIAS + 4 * 512;
constexpr int Q_LDS = Q_SINK + 512;

__device__ __forceinline__ int q_swz(int row, int chunk) {
  return row * Q_BK + ((chunk ^ (((row >> 3) & 1) * 3)) << 3);
}

__device__ __forceinline__ void q_issue(bf16* smem, const PPTile& o, bool valid, int t, int s, const int (&aoff)[2],
                                        const int (&boff)[2], int wave, const float* aux, int aux_rec, int aux_dst) {
  typedef __attribute__((address_space(3))) void lds_void;
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc((void*)o.A, (short)0, valid ? o.a_rec : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc((void*)o.B, (short)0, valid ? o.b_rec : 0, 0x00020000);
  bf16* st = smem + (s & (Q_NST - 1)) * Q_STAGE;
  bf16* dA = valid ? st + wave * 32 * Q_BK : smem + Q_SINK;
  bf16* dB = valid ? st + (256 + wave * 32) * Q_BK : smem + Q_SINK;
  const int step = valid ? 16 * Q_BK : 0;
  const int kb = t * Q_BK * 2;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)dA, 16, aoff[0], kb, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(dA + step), 16, aoff[1], kb, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)dB, 16, boff[0], kb, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dB + step), 16, boff[1], kb, 0, 0);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(aux ? (const void*)aux : (const void*)o.A), (short)0, aux_rec,
                                        0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(smem + aux_dst), 16, lane * 16, 0, 0, 0);
}
}  // namespace

__global__ void __launch_bounds__(512, 1)
gemm_pp2_k(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ O, const float* __restrict__ bias,
           const bf16* __restrict__ R, int M, int N, int K, int lda, int ldb, int ldo, int ldr, float alpha,
           float scale, int mt, int nt, int gm, float* __restrict__ gnp, int gn_groups, int gn_hw) {
  __shared__ __attribute__((aligned(16))) bf16 smem[Q_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  int rb = blockIdx.x;
  {
    const int q = G / 8, r = G % 8, xcd = rb % 8;
    rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + rb / 8;
  }
  const int ntiles = mt * nt;
  if (rb >= ntiles) return;
  const int nk = K / Q_BK;

  // loader: 16-row DMA pieces, lane -> (row lane >> 2, slot lane & 3) holding chunk slot ^ f(row)
  int aoff[2], boff[2];
  {
    const int chunk = (lane & 3) ^ (((lane >> 5) & 1) * 3);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int row = wave * 32 + q * 16 + (lane >> 2);
      aoff[q] = (row * lda + chunk * 8) * 2;
      boff[q] = (row * ldb + chunk * 8) * 2;
    }
  }
  // loader cursor (runs 3 K-tiles ahead of the compute cursor)
  int ltile = rb, lt = 0, lti = 0;
  PPTile lops;
  {
    int mb, nb;
    pp_tile(ltile, mt, nt, gm, mb, nb);
    lops = pp_tile_ops(A, B, M, N, K, lda, ldb, mb, nb);
  }
  auto load_next = [&](int s) {
    const bool valid = ltile < ntiles;
    const float* as = nullptr;
    int ar = 0, ad = Q_SINK;
    if (valid && lt == 0 && bias && wave == 0) {
      as = bias + lops.m0;
      ar = (int)((M - lops.m0 < 256 ? M - lops.m0 : 256) * 4);
      ad = Q_BIAS + (lti & 3) * 512;
    }
    q_issue(smem, lops, valid, lt, s, aoff, boff, wave, as, ar, ad);
    if (valid && ++lt == nk) {
      lt = 0;
      ++lti;
      ltile += G;
      if (ltile < ntiles) {
        int mb, nb;
        pp_tile(ltile, mt, nt, gm, mb, nb);
        lops = pp_tile_ops(A, B, M, N, K, lda, ldb, mb, nb);
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;

  load_next(0);
  load_next(1);
  load_next(2);
  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  PP_BAR();
  if (wr == 1) PP_BAR();                 // the M-half-1 waves trail by one barrier

  int tile = rb, t = 0, ti = 0, mb, nb;
  pp_tile(tile, mt, nt, gm, mb, nb);
  for (int s = 0;; ++s) {
    const bf16* st = smem + (s & (Q_NST - 1)) * Q_STAGE;
    bf16x8 af[8], bq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bq[j] = *reinterpret_cast<const bf16x8*>(st + q_swz(256 + wn * 64 + j * 16 + fr, fq));
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8*>(st + q_swz(wr * 128 + i * 16 + fr, fq));
    load_next(s + 3);
    asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    PP_BAR();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    PP_BAR();
    if (++t == nk) {
      pp_epi(acc, bias ? reinterpret_cast<const float*>(smem + Q_BIAS + (ti & 3) * 512) : nullptr, O, R, M, N, ldo,
             ldr, alpha, scale, (long)mb * 256, (long)nb * 256, wr, wn, lane, gnp, gn_groups, gn_hw);
      tile += G;
      if (tile >= ntiles) break;
      ++ti;
      t = 0;
      pp_tile(tile, mt, nt, gm, mb, nb);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (wr == 0) PP_BAR();                 // balance the trailing group's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the block ends
}

static int g_pp_ver = getenv("D3D_GEMM_V") ? atoi(getenv("D3D_GEMM_V")) : 1;
static int g_pp_grid = getenv("D3D_GEMM_GRID") ? atoi(getenv("D3D_GEMM_GRID")) : 0;   // 0: one block per CU
static int g_pp_gm = getenv("D3D_GEMM_GM") ? atoi(getenv("D3D_GEMM_GM")) : 4;
static int pp_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// Tuning switches for in-process A/B (kernel version, tile-group width, grid);
// a value <= 0 leaves the setting unchanged.
D3D_API void d3d_gemm_tune(int ver, int gm, int grid) {
  if (ver > 0) g_pp_ver = ver;
  if (gm > 0) g_pp_gm = gm;
  if (grid > 0) g_pp_grid = grid;
}

// Shapes the kernel takes: K a multiple of 64, 16-byte aligned operand rows,
// one block's operand rows addressable by 32-bit offsets.
D3D_API int d3d_gemm_nt_ok(int M, int N, int K, int lda, int ldb) {
  if (M <= 0 || N <= 0 || K <= 0 || K % PP_BK) return 0;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K) return 0;
  if (256L * lda * 2 >= (1L << 31) || 256L * ldb * 2 >= (1L << 31)) return 0;
  return 1;
}

// gnp: optional fused GroupNorm partials of the output ([N / gn_hw][G][gn_hw /
// 64] x (sum, sumsq), gn_part_store layout); needs M % 4 == 0, ldo % 4 == 0,
// gn_hw % 64 == 0 and M / G in {4, 8, 16, 32}.
D3D_API int d3d_gemm_nt_gn(const void* A, const void* B, void* O, const float* bias, const void* R, int M, int N,
                           int K, int lda, int ldb, int ldo, int ldr, float alpha, float scale, float* gnp, int G,
                           int hw, hipStream_t st) {
  if (!d3d_gemm_nt_ok(M, N, K, lda, ldb)) return -1;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return -1;
  if (gnp) {
    const int cg = G > 0 ? M / G : 0;
    if (G <= 0 || M % G || M % 4 || ldo % 4 || (R && ldr % 4) || hw <= 0 || hw % 64 || N % hw ||
        !(cg == 4 || cg == 8 || cg == 16 || cg == 32))
      return -1;
  }
  const int mt = cdiv(M, 256), nt = cdiv(N, 256);
  const long tiles = (long)mt * nt;
  if (tiles >= (1L << 31)) return -1;
  const int G_ = (int)std::min<long>(tiles, g_pp_grid > 0 ? g_pp_grid : pp_cus());
  const int gm = std::max(1, std::min(mt, g_pp_gm));
  if (g_pp_ver == 2)
    hipLaunchKernelGGL(gemm_pp2_k, dim3(G_), dim3(512), 0, st, (const bf16*)A, (const bf16*)B, (bf16*)O, bias,
                       (const bf16*)R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, mt, nt, gm, gnp, G, hw);
  else
    hipLaunchKernelGGL(gemm_pp_k, dim3(G_), dim3(512), 0, st, (const bf16*)A, (const bf16*)B, (bf16*)O, bias,
                       (const bf16*)R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, mt, nt, gm, gnp, G, hw);
  return (int)hipGetLastError();
}

D3D_API int d3d_gemm_nt(const void* A, const void* B, void* O, const float* bias, const void* R, int M, int N, int K,
                        int lda, int ldb, int ldo, int ldr, float alpha, float scale, hipStream_t st) {
  return d3d_gemm_nt_gn(A, B, O, bias, R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, nullptr, 0, 0, st);
}
