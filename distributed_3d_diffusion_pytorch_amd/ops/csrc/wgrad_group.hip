// Grouped weight gradients: every deferred weight-gradient job of one flush
// (ops/gradsink.py: the 3x3 ResnetBlock convs `xunet.py:114-126`, the 1x1 NIN
// skips `:129`, the attention projections and 1x1 `:175,190`) in ONE launch,
// plus ONE launch that reduces the split-K slabs of the jobs that need them.
//
// Per job:  dW[co][ci][tap] = scale * sum_p dY[p][co] * X[p + shift(tap)][ci]
//           db[co]          = scale * sum_p dY[p][co]
// (X may be a virtual channel concat [X | X2] split at C1: the decoder's
// skip concat `xunet.py:525`.)
//
// Why grouped: at 16 examples per GPU (the 8-GPU share of the headline batch)
// most weight gradients are far too small to fill 256 CUs alone -- a 1x1
// projection of the 8x8 level is 1 GFLOP -- so each job used to be split-K'd
// over ~1024 blocks, writing up to 100 fp32 slabs of the whole OC x 9 IC
// weight that a per-job reduce kernel then summed (≈390 launches, a quarter
// of the kernel time in slab reductions).  Here the jobs of a flush share one
// grid: a job's blocks are sized by ONE pixel count per block across the
// batch (the planner below), so the small-pixel jobs (8x8 / 16x16 levels)
// run unsplit and write the OIHW gradient straight from their epilogue; only
// the long-reduction jobs (64x64 level) are split, into a few slabs summed by
// the grouped reduce in a fixed order (bitwise reproducible).
//
// Tile engine: the pixel-major LDS-DMA + transposed-read (ds_read_b64_tr_b16)
// weight-gradient tile of conv.hip's conv_wgrad_bufl_k (FAST addressing:
// stride 1, power-of-two images, so a tap's input rows are the output rows
// shifted by a wave-uniform pixel offset; 1x1 jobs are the degenerate
// 1-tap case), with the tap count, shapes and pointers read per block from a
// job table passed by value (no device-side table, graph-capture safe).
#include "common.h"

#include <algorithm>

namespace {

typedef __attribute__((ext_vector_type(4))) short gs16x4;
typedef __attribute__((ext_vector_type(8))) short gs16x8;
typedef __attribute__((address_space(3))) gs16x4 glds_s16x4;

__device__ __forceinline__ gs16x4 gw_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((glds_s16x4*)(p));
}

// The same transposed read as inline asm: the compiler's wait-count pass
// cannot tell an LDS read from the LDS-DMA writes still in flight to the
// OTHER ring slots, and put "s_waitcnt vmcnt(0)" in front of the first read
// of every stage -- every stage waited for the stages issued after it, so no
// DMA ever overlapped compute (the 59 % wait-parked cycles of the 2-stage
// weight-gradient kernel).  Hidden from the pass, the reads are retired by an
// explicit lgkmcnt wait (gw_tr_wait) that also pins the fragment registers.
__device__ __forceinline__ gs16x4 gw_tr_asm(const bf16* p) {
  gs16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int TM, int TN>
__device__ __forceinline__ void gw_tr_wait(bf16x8 (&a)[TM], bf16x8 (&b)[TN]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(b[j]));
}
__device__ __forceinline__ float gw_dot2(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a), __builtin_bit_cast(bf16x2, b), c, false);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t gw_rsrc(const void* p, long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes > 0 ? (bytes < 0x7fffffffL ? bytes : 0x7fffffffL) : 0));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, n, 0x00020000);
}

constexpr int GW_MAX = 16;        // jobs per launch (the sink flushes 8)
constexpr int GW_BM = 128, GW_BN = 128;

struct GwJob {
  const bf16* dy;                 // [P][OC]
  const bf16* x;                  // [P][C1 or IC]
  const bf16* x2;                 // [P][IC - C1] or null
  float* dw;                      // [OC][IC][taps] (OIHW)
  float* db;                      // [OC] or null
  float* slab;                    // splits > 1: [splits][OC][taps * IC]
  float* bslab;                   // splits > 1 and db: [2 splits][OC]
  long P;
  int OC, IC, C1, taps, H, W, lw, lh, ncb, nmb, splits, pps, blk0, acc;
  float scale;
  int pad_;
};
struct GwTable {
  int n, pad_;
  GwJob j[GW_MAX];
};

struct GrJob {
  const float* slab;
  const float* bslab;
  float* dw;
  float* db;
  int OC, IC, taps, splits, blk0, nblk_w, acc;
  float scale;
  int flat, pad_;                 // flat: slabs already in OIHW order (halo tiles): a plain sum over splits
};
struct GrTable {
  int n, pad_;
  GrJob j[GW_MAX];
};

template <int PK>
__device__ __forceinline__ void gw_issue(bf16* sA, bf16* sB, const bf16* __restrict__ dY, const bf16* __restrict__ I,
                                         long in_elems, long p0, long p_end, int OC, int IC, int OH, int OW, int kh,
                                         int kw, int dpix, int lw, int wave, const int* trow, const unsigned* aoff,
                                         const unsigned* boff, const bool* bok, bool on = true) {
  typedef __attribute__((address_space(3))) void lds_void;
  constexpr int PPW = PK / 16;
  // on = false: a pipeline-tail dummy -- zero-record descriptors, so the same
  // number of DMAs is in flight at every wait (the data land in a slot no one
  // reads)
  const __amdgpu_buffer_rsrc_t rA = gw_rsrc(dY + p0 * OC, on ? (p_end - p0) * OC * 2 : 0);
#pragma unroll
  for (int i = 0; i < PPW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sA + (wave * PPW + i) * 4 * GW_BM), 16, aoff[i], 0, 0,
                                             0);
  // the base may lie before the tensor (only masked top-padding rows see it)
  // or past its end on the last stages: the record count clamps at 0
  const long pb = p0 + dpix;
  const __amdgpu_buffer_rsrc_t rB = gw_rsrc(I + pb * IC, on ? (in_elems - pb * IC) * 2 : 0);
  // padding rows of the (wave-uniform) tap: compare against the uniform edge
  // coordinate, branch-free per lane
  const int wedge = kw == 0 ? 0 : OW - 1, hedge = kh == 0 ? 0 : OH - 1;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int pp = (int)p0 + trow[i];
    bool bad = !bok[i];
    if (kw != 1) bad |= (pp & (OW - 1)) == wedge;
    if (kh != 1) bad |= ((pp >> lw) & (OH - 1)) == hedge;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(sB + (wave * PPW + i) * 4 * GW_BN), 16,
                                             bad ? 0x80000000u : boff[i], 0, 0, 0);
  }
}

}  // namespace

// One 128 (output channels) x 128 (input channels of one tap) tile of one
// split of one job per block; 4 waves of 64 x 64 (4 x 4 MFMA 16x16x32 tiles);
// PK pixel rows per LDS stage, two stages, one barrier per stage.
// NS-stage LDS ring, NS - 1 stages in flight: with two stages (one landing
// while the other is read) the waves sat 59 % of their cycles in s_waitcnt /
// s_barrier (profiles/pmc_wgrad): a 32-pixel stage is 16 MFMAs per wave,
// far shorter than a DMA round trip.
template <int PK, int NS>
__global__ void __launch_bounds__(256, 2) wgrad_grp_k(GwTable tab) {
  constexpr int BM = GW_BM, BN = GW_BN;
  constexpr int PER = 2 * (PK / 16);              // DMA instructions per wave per stage
  constexpr int WM = 64, WN = 64, TM = 4, TN = 4;
  constexpr int STAGE = PK * (BM + BN);
  constexpr int PPW = PK / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware remap of the flat block index: consecutive logical blocks (the
  // taps / channel tiles of one split, which read the same dY rows) on one XCD
  int R;
  {
    const int T = gridDim.x, L = blockIdx.x;
    const int q = T / 8, r = T % 8, xcd = L % 8;
    R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
  }
  int k = 0;
  while (k + 1 < tab.n && R >= tab.j[k + 1].blk0) ++k;
  const GwJob& J = tab.j[k];
  const bf16* dY = J.dy;
  const int OC = J.OC, ICt = J.IC, C1 = J.C1, taps = J.taps, OH = J.H, OW = J.W, lw = J.lw;
  const int ncb = J.ncb, nmb = J.nmb, splits = J.splits;
  const long P = J.P;
  const int nt = taps * ncb;
  const int b = R - J.blk0;
  const int bx = b % nt, by = (b / nt) % nmb, split = b / (nt * nmb);
  const int tap = bx / ncb;
  const int ci0g = (bx % ncb) * BN;               // channel tile in the (possibly concatenated) input
  const int m0 = by * BM;
  const int kh = taps == 9 ? tap / 3 : 1, kw = taps == 9 ? tap % 3 : 1;
  const long p_begin = (long)split * J.pps;
  const long p_end = p_begin + J.pps < P ? p_begin + J.pps : P;
  const int dpix = (kh - 1) * OW + (kw - 1);
  const bool second = J.x2 != nullptr && ci0g >= C1;
  const bf16* I = second ? J.x2 : J.x;
  const int IC = J.x2 == nullptr ? ICt : (second ? ICt - C1 : C1);
  const int ci0 = second ? ci0g - C1 : ci0g;
  const long in_elems = P * IC;

  const int lrow = lane >> 4, pch = lane & 15;
  int trow[PPW];
  unsigned aoff[PPW], boff[PPW];
  bool bok[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    trow[i] = (wave * PPW + i) * 4 + lrow;
    const int lc = pch ^ (2 * (trow[i] & 7));
    const int co = m0 + lc * 8;
    aoff[i] = co < OC ? (unsigned)((trow[i] * OC + co) * 2) : 0x80000000u;
    const int ci = ci0 + lc * 8;
    boff[i] = (unsigned)((trow[i] * IC + ci) * 2);
    bok[i] = ci < IC;
  }
  // transpose-read lane offsets (elements): row (4g+q) + swizzled column chunk
  const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
  const int x7 = 2 * ((4 * g + q) & 7);
  int la[TM], lb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) la[i] = (4 * g + q) * 128 + ((((wm * 8 + 2 * i + (pc >> 1)) ^ x7)) << 3) + (pc & 1) * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j) lb[j] = (4 * g + q) * 128 + ((((wn * 8 + 2 * j + (pc >> 1)) ^ x7)) << 3) + (pc & 1) * 4;

  auto issue = [&](long p0, int stage, bool on) {
    bf16* sA = smem + stage * STAGE;
    gw_issue<PK>(sA, sA + PK * BM, dY, I, in_elems, p0, p_end, OC, IC, OH, OW, kh, kw, dpix, lw, wave, trow, aoff,
                 boff, bok, on);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long nsteps = (p_end - p_begin + PK - 1) / PK;
  // bias (column sums of dY): from the A fragments the MFMAs read anyway --
  // lane l of fragment i holds 8 pixels of channel wm*64 + 16i + l%16, so a
  // dot product with (1, 1) per bf16 pair sums them (the wn = 1 waves read the
  // same fragments and skip it)
  const bool do_bias = J.db != nullptr && bx == 0;
  const bool bias_wave = do_bias && wn == 0;
  float bsum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bsum[i] = 0.f;
  const unsigned ones = 0x3F803F80u;              // bf16 (1, 1)
  auto compute = [&](const bf16* a) {
    const bf16* bb = a + PK * BM;
#pragma unroll
    for (int kk = 0; kk < PK / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        gs16x4 lo = gw_tr_asm(bb + lb[j] + kk * 32 * 128);
        gs16x4 hi = gw_tr_asm(bb + lb[j] + kk * 32 * 128 + 16 * 128);
        gs16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        gs16x4 lo = gw_tr_asm(a + la[i] + kk * 32 * 128);
        gs16x4 hi = gw_tr_asm(a + la[i] + kk * 32 * 128 + 16 * 128);
        gs16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
      gw_tr_wait<TM, TN>(af, bfr);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (bias_wave) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const auto u = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, af[i]);
#pragma unroll
          for (int w = 0; w < 4; ++w) bsum[i] = gw_dot2(u[w], ones, bsum[i]);
        }
      }
    }
  };
  // one barrier per stage: wait for this stage's DMA (NS - 2 newer stages may
  // stay in flight), barrier (every wave's DMA landed AND every wave done
  // reading the slot refilled next), issue stage s + NS - 1 into that slot,
  // compute.  Past the last stage the issues are zero-record dummies, so the
  // wait counts stay uniform.
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue(p_begin + t * PK, t, t < nsteps);
  for (long s = 0; s < nsteps; ++s) {
    const int st = (int)(s % NS);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * PER) : "memory");
    __builtin_amdgcn_s_barrier();
    const long nx = s + NS - 1;
    issue(p_begin + (nx < nsteps ? nx : s) * PK, (int)(nx % NS), nx < nsteps);
    __builtin_amdgcn_s_setprio(1);
    compute(smem + st * STAGE);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail dummies drained before exit

  const int fr = lane & 15, fq = lane >> 4;
  const long KW = (long)taps * ICt;
  if (bias_wave) {                                // the four 8-pixel lane groups -> lanes 0..15
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      bsum[i] += __shfl_xor(bsum[i], 16);
      bsum[i] += __shfl_xor(bsum[i], 32);
    }
  }
  if (splits == 1) {
    // unsplit: the OIHW gradient straight from the accumulators (this block
    // is the only writer of its (co, ci, tap) elements)
    const float sc = J.scale;
    float* dw = J.dw;
    const int acc_in = J.acc;
    if (bias_wave && fq == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = m0 + wm * WM + i * 16 + fr;
        if (co < OC) {
          float* d = J.db + co;
          const float v = bsum[i] * sc;
          *d = acc_in ? *d + v : v;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = ci0 + wn * WN + j * 16 + fr;
      if (cl >= IC) continue;
      const int ci = ci0g - ci0 + cl;               // channel within the concatenation
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (co + e < OC) {
            float* d = dw + ((long)(co + e) * ICt + ci) * taps + tap;
            const float v = acc[i][j][e] * sc;
            *d = acc_in ? *d + v : v;
          }
      }
    }
    return;
  }
  if (bias_wave && fq == 0) {                      // bias partial rows (2 split, 2 split + 1) = (sum, 0)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = m0 + wm * WM + i * 16 + fr;
      if (co < OC) {
        J.bslab[((long)split * 2) * OC + co] = bsum[i];
        J.bslab[((long)split * 2 + 1) * OC + co] = 0.f;
      }
    }
  }
  float* slab = J.slab + (long)split * OC * KW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = ci0 + wn * WN + j * 16 + fr;
    if (cl >= IC) continue;
    const int ci = ci0g - ci0 + cl;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < OC) slab[(long)(co + e) * KW + tap * ICt + ci] = acc[i][j][e];
    }
  }
}

// ---------------------------------------------------------- halo tiles ----
// 3x3 stride-1 jobs (power-of-two images, W >= 16): one block = 128 output channels x 64 input
// channels x ALL NINE taps of one pixel split.  Eight waves (two per SIMD);
// wave (wm, wn) owns output channels 64wm.. +63 x input channels 16wn.. +15 x
// the nine taps (4 x 9 = 36 MFMA 16x16x32 tiles, 144 accumulator registers).
// A 32-pixel K-step (half / one row at W >= 32, 2 / 4 rows at W = 16 / 8)
// stages the dY rows [32][128 co] and the input WINDOW [RR + 2 rows][Wm + 2
// px][64 ci] (Wm = min(W, 32), RR = 32 / Wm image rows per step) -- the step's
// pixels with the one-pixel border around them, zero-filled outside the image
// -- so the B fragment of tap (kh, kw) at step pixel k is window row
// f(k) + kh*(Wm + 2) + kw, f(k) = (k / Wm)(Wm + 2) + k % Wm: one window feeds
// the nine taps, and the step's dY fragments are read once for all nine.  Per MFMA
// that is 0.72 transposed LDS reads and 0.07 KB of DMA, against 1.0 and 0.25 KB
// for the per-tap 128 x 128 tile above (which re-reads dY and X once per tap).
constexpr int GH_BM = 128, GH_BN = 64, GH_PK = 32, GH_WR = 34;
// K-step of PK pixels (32 or 64): window rows padded to whole 8-row DMAs
// (<= 3 x 34 = 102 -> 128 at PK = 32, <= 3 x 66 = 198 -> 256 at PK = 64)
template <int PK> struct GhGeom {
  static constexpr int BROWS = PK == 64 ? 256 : 128;
  static constexpr int STAGE = PK * GH_BM + BROWS * GH_BN;    // bf16 elements: 24 KB (PK 32) / 48 KB (PK 64)
  static constexpr int PER_A = PK / 32, PER_B = BROWS / 64;   // DMA instructions per wave per stage
};

// 16-byte chunk swizzle of the 128-byte window rows: the 8 consecutive rows a
// transposed read's 32-lane group touches (any tap offset) land on 64 distinct
// banks
__device__ __forceinline__ int gh_swz(int row) { return 2 * ((row >> 1) & 3); }

template <int PK>
__device__ __forceinline__ void gh_issue(bf16* sA, bf16* sB, const bf16* __restrict__ dY, const bf16* __restrict__ I,
                                         long in_elems, long p0, long p_end, int OC, int IC, int OH, int OW, int lw,
                                         int Wm, int RR, int wave, const unsigned* aoff, const unsigned* boff,
                                         const unsigned* bfl, bool on) {
  typedef __attribute__((address_space(3))) void lds_void;
  typedef GhGeom<PK> Gg;
  const __amdgpu_buffer_rsrc_t rA = gw_rsrc(dY + p0 * OC, on ? (p_end - p0) * OC * 2 : 0);
#pragma unroll
  for (int i = 0; i < Gg::PER_A; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sA + (wave * Gg::PER_A + i) * 4 * GH_BM), 16, aoff[i], 0,
                                             0, 0);
  // window origin: pixel (y - 1, x0 - 1); it may lie before the tensor, and
  // only masked lanes (top row, left column) ever address below the tensor
  const long pb = p0 - OW - 1;
  const __amdgpu_buffer_rsrc_t rB = gw_rsrc(I + pb * IC, on ? (in_elems - pb * IC) * 2 : 0);
  const int x0 = (int)(p0 & (OW - 1)), y = (int)((p0 >> lw) & (OH - 1));
  const unsigned bad = 1u | (y == 0 ? 2u : 0u) | (y + RR == OH ? 4u : 0u) | (x0 == 0 ? 8u : 0u) |
                       (x0 + Wm == OW ? 16u : 0u);
#pragma unroll
  for (int j = 0; j < Gg::PER_B; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(sB + (wave * Gg::PER_B + j) * 8 * GH_BN), 16,
                                             (bfl[j] & bad) ? 0x80000000u : boff[j], 0, 0, 0);
}

template <int NS, int PK>
__global__ void __launch_bounds__(512, 1) wgrad_halo_k(GwTable tab) {
  typedef GhGeom<PK> Gg;
  constexpr int PER = Gg::PER_A + Gg::PER_B;     // DMA instructions per wave per stage
  constexpr int KK = PK / 32;                    // MFMA K slices per step
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * Gg::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int R;
  {
    const int T = gridDim.x, L = blockIdx.x;
    const int q = T / 8, r = T % 8, xcd = L % 8;
    R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
  }
  int k = 0;
  while (k + 1 < tab.n && R >= tab.j[k + 1].blk0) ++k;
  const GwJob& J = tab.j[k];
  const bf16* dY = J.dy;
  const int OC = J.OC, ICt = J.IC, C1 = J.C1, OH = J.H, OW = J.W, lw = J.lw;
  const int ncb = J.ncb, nmb = J.nmb, splits = J.splits;
  const long P = J.P;
  const int b = R - J.blk0;
  const int bx = b % ncb, by = (b / ncb) % nmb, split = b / (ncb * nmb);
  const int m0 = by * GH_BM, ci0g = bx * GH_BN;
  const bool second = J.x2 != nullptr && ci0g >= C1;
  const bf16* I = second ? J.x2 : J.x;
  const int IC = J.x2 == nullptr ? ICt : (second ? ICt - C1 : C1);
  const int ci0 = second ? ci0g - C1 : ci0g;
  const long in_elems = P * IC;
  const long p_begin = (long)split * J.pps;
  const long p_end = p_begin + J.pps < P ? p_begin + J.pps : P;
  const int Wm = OW < PK ? OW : PK, RR = PK / Wm, WR = Wm + 2, NR = RR + 2;

  unsigned aoff[Gg::PER_A], boff[Gg::PER_B], bfl[Gg::PER_B];
  {
    const int lrow = lane >> 4, pch = lane & 15;
#pragma unroll
    for (int i = 0; i < Gg::PER_A; ++i) {
      const int trow = (wave * Gg::PER_A + i) * 4 + lrow;
      const int lc = pch ^ (2 * (trow & 7));
      aoff[i] = (unsigned)((trow * OC + m0 + lc * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < Gg::PER_B; ++j) {
      const int wr = (wave * Gg::PER_B + j) * 8 + (lane >> 3);
      const int kh = wr / WR, px = wr - kh * WR;
      const int chunk = (lane & 7) ^ gh_swz(wr);
      const bool valid = wr < NR * WR;
      boff[j] = valid ? (unsigned)(((kh * OW + px) * IC + ci0 + chunk * 8) * 2) : 0u;
      bfl[j] = (valid ? 0u : 1u) | (kh == 0 ? 2u : 0u) | (kh == NR - 1 ? 4u : 0u) | (px == 0 ? 8u : 0u) |
               (px == WR - 1 ? 16u : 0u);
    }
  }
  // transposed-read offsets (elements in a stage): lane (g, q, pc) reads K row
  // 4g + q (and + 16), 8-element chunk pc >> 1 of its 16 columns, half pc & 1
  // (PK = 64 only on images W >= 64: a step is one row segment, so K slice
  // kk is the slice-0 rows + 32 kk -- the swizzle's period divides 32 -- and
  // the offsets of slice 0 serve every slice through the immediate)
  int la[4], lb[9], lbh[9];
  {
    const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
    const int kr = 4 * g + q, x7 = 2 * (kr & 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) la[i] = kr * GH_BM + (((wm * 8 + 2 * i + (pc >> 1)) ^ x7) << 3) + (pc & 1) * 4;
    const int f0 = (kr / Wm) * WR + kr % Wm, f1 = ((kr + 16) / Wm) * WR + (kr + 16) % Wm;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int r0 = f0 + (t / 3) * WR + (t % 3), r1 = f1 + (t / 3) * WR + (t % 3);
      lb[t] = PK * GH_BM + r0 * GH_BN + (((2 * wn + (pc >> 1)) ^ gh_swz(r0)) << 3) + (pc & 1) * 4;
      lbh[t] = PK * GH_BM + r1 * GH_BN + (((2 * wn + (pc >> 1)) ^ gh_swz(r1)) << 3) + (pc & 1) * 4;
    }
  }
  auto issue = [&](long p0, int stage, bool on) {
    bf16* sA = smem + stage * Gg::STAGE;
    gh_issue<PK>(sA, sA + PK * GH_BM, dY, I, in_elems, p0, p_end, OC, IC, OH, OW, lw, Wm, RR, wave, aoff, boff, bfl,
                 on);
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long nsteps = (p_end - p_begin) / PK;             // (the planner keeps splits on 64-pixel bounds)
  const bool bias_wave = J.db != nullptr && bx == 0 && wn == 0;
  float bsum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bsum[i] = 0.f;
  const unsigned ones = 0x3F803F80u;
  // the dY fragments once per step; the window fragment of tap t + 1 is read
  // while tap t's eight MFMAs run (register budget: 288 accumulators)
  auto rd_b = [&](const bf16* s, int kk, int t) {
    gs16x4 lo = gw_tr_asm(s + lb[t] + kk * 32 * GH_BN);
    gs16x4 hi = gw_tr_asm(s + lbh[t] + kk * 32 * GH_BN);
    gs16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  auto compute = [&](const bf16* s) {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[4], bq[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gs16x4 lo = gw_tr_asm(s + la[i] + kk * 32 * GH_BM);
        gs16x4 hi = gw_tr_asm(s + la[i] + kk * 32 * GH_BM + 16 * GH_BM);
        gs16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#ifdef D3D_WGRAD_HALO_AHEAD1
      bq[0] = rd_b(s, kk, 0);
      gw_tr_wait<4, 1>(af, *reinterpret_cast<bf16x8(*)[1]>(&bq[0]));
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t < 8) bq[(t + 1) % 3] = rd_b(s, kk, t + 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[t % 3], acc[i][t], 0, 0, 0);
        if (t < 8) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          asm volatile("" : "+v"(bq[(t + 1) % 3]));
        }
      }
#else
      // the window fragments of taps t + 1 AND t + 2 are in flight while tap
      // t's MFMAs run (three rotating registers; LDS reads complete in order,
      // so lgkmcnt(2) = everything but the newest fragment's two reads; no
      // scalar loads are in flight inside this loop)
      bq[0] = rd_b(s, kk, 0);
      bq[1] = rd_b(s, kk, 1);
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(af[i]));
      asm volatile("" : "+v"(bq[0]));
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t + 2 < 9) bq[(t + 2) % 3] = rd_b(s, kk, t + 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[t % 3], acc[i][t], 0, 0, 0);
        if (t + 1 < 9) {
          if (t + 2 < 9) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          asm volatile("" : "+v"(bq[(t + 1) % 3]));
        }
      }
#endif
      if (bias_wave) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto u = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, af[i]);
#pragma unroll
          for (int w = 0; w < 4; ++w) bsum[i] = gw_dot2(u[w], ones, bsum[i]);
        }
      }
    }
  };
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue(p_begin + t * PK, t, t < nsteps);
  for (long s = 0; s < nsteps; ++s) {
    const int st = (int)(s % NS);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * PER) : "memory");
    __builtin_amdgcn_s_barrier();
    const long nx = s + NS - 1;
    issue(p_begin + (nx < nsteps ? nx : s) * PK, (int)(nx % NS), nx < nsteps);
    __builtin_amdgcn_s_setprio(1);
    compute(smem + st * Gg::STAGE);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int fr = lane & 15, fq = lane >> 4;
  const int cig = ci0g + 16 * wn + fr;             // input channel within the (concatenated) input
  const int cw = m0 + 64 * wm;                      // this wave's first output channel
  if (bias_wave) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bsum[i] += __shfl_xor(bsum[i], 16);
      bsum[i] += __shfl_xor(bsum[i], 32);
    }
  }
  if (splits == 1) {
    const float sc = J.scale;
    const int acc_in = J.acc;
    if (bias_wave && fq == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* d = J.db + cw + i * 16 + fr;
        const float v = bsum[i] * sc;
        *d = acc_in ? *d + v : v;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float* d = J.dw + ((long)(cw + i * 16 + fq * 4 + e) * ICt + cig) * 9;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float v = acc[i][t][e] * sc;
          d[t] = acc_in ? d[t] + v : v;
        }
      }
    return;
  }
  if (bias_wave && fq == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      J.bslab[((long)split * 2) * OC + cw + i * 16 + fr] = bsum[i];
      J.bslab[((long)split * 2 + 1) * OC + cw + i * 16 + fr] = 0.f;
    }
  }
  // slab in OIHW order ([split][co][ci][tap]): each lane's nine taps are
  // contiguous, and the reduce is a plain coalesced sum over the splits
  float* slab = J.slab + (long)split * OC * 9L * ICt;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* d = slab + ((long)(cw + i * 16 + fq * 4 + e) * ICt + cig) * 9;
#pragma unroll
      for (int t = 0; t < 9; ++t) d[t] = acc[i][t][e];
    }
}

// Grouped split-K reduce: block = (job, co, 64 input channels) summing every
// tap of its channels over the job's slabs, 4 split lanes merged in a fixed
// order through LDS, written as 64 x taps CONTIGUOUS floats of OIHW; blocks
// past a job's nblk_w sum its bias partials.
__global__ void __launch_bounds__(256) wgrad_grp_reduce_k(GrTable tab) {
  __shared__ float red[4][9][64];
  __shared__ float tile[64 * 9];
  const int tid = threadIdx.x;
  const int R = blockIdx.x;
  int k = 0;
  while (k + 1 < tab.n && R >= tab.j[k + 1].blk0) ++k;
  const GrJob& J = tab.j[k];
  const int b = R - J.blk0;
  const int OC = J.OC, IC = J.IC, taps = J.taps, splits = J.splits;
  const int ln = tid >> 6, c = tid & 63;
  if (b >= J.nblk_w) {
    const int co = (b - J.nblk_w) * 64 + c;
    float a0 = 0.f, a1 = 0.f;
    if (co < OC) {
      int r = ln;
      for (; r + 4 < 2 * splits; r += 8) {
        a0 += J.bslab[(long)r * OC + co];
        a1 += J.bslab[(long)(r + 4) * OC + co];
      }
      if (r < 2 * splits) a0 += J.bslab[(long)r * OC + co];
    }
    red[ln][0][c] = a0 + a1;
    __syncthreads();
    if (ln == 0 && co < OC) {
      const float v = (((red[0][0][c] + red[1][0][c]) + red[2][0][c]) + red[3][0][c]) * J.scale;
      J.db[co] = J.acc ? J.db[co] + v : v;
    }
    return;
  }
  if (J.flat) {                                    // OIHW slabs: 1024 consecutive floats per block
    const long total = (long)OC * IC * taps;
    const long e0 = (long)b * 1024 + tid * 4;
    if (e0 >= total) return;
    f32x4 a = *reinterpret_cast<const f32x4*>(J.slab + e0);
    for (int sp = 1; sp < splits; ++sp) a += *reinterpret_cast<const f32x4*>(J.slab + (long)sp * total + e0);
    a *= J.scale;
    f32x4* d = reinterpret_cast<f32x4*>(J.dw + e0);
    *d = J.acc ? *d + a : a;
    return;
  }
  const int ncg = (IC + 63) / 64;
  const int co = b / ncg, ci0 = (b % ncg) * 64;
  const int nci = min(64, IC - ci0);
  const long total = (long)OC * taps * IC;
  float a[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) a[t] = 0.f;
  if (c < nci) {
    const float* src = J.slab + (long)co * taps * IC + ci0 + c;
    for (int sp = ln; sp < splits; sp += 4) {
      const float* s = src + (long)sp * total;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        if (t < taps) a[t] += s[(long)t * IC];
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if (t < taps) red[ln][t][c] = a[t];
  __syncthreads();
  for (int m = tid; m < taps * 64; m += 256) {
    const int t = m >> 6, cc = m & 63;
    tile[cc * taps + t] = (((red[0][t][cc] + red[1][t][cc]) + red[2][t][cc]) + red[3][t][cc]) * J.scale;
  }
  __syncthreads();
  float* dst = J.dw + ((long)co * IC + ci0) * taps;
  for (int m = tid; m < nci * taps; m += 256) dst[m] = J.acc ? dst[m] + tile[m] : tile[m];
}

// ------------------------------------------------------------------ host ----
// Job description of the C ABI (mirrored by ops/hip_impl.py _WgJob).
struct WgJobDesc {
  const void* dy;
  const void* x;
  const void* x2;
  float* dw;
  float* db;
  int N, H, W, OC, IC, C1, taps, acc;
  float scale;
  int pad_;
};
static_assert(sizeof(WgJobDesc) == 80, "WgJobDesc must match hip_impl._WgJob");

static int g_gw_blocks = 512;      // target blocks per grouped launch (2 per CU)
static int g_gw_pk = 32;           // pixel rows per LDS stage (32 or 64)
static int g_gw_minpix = 512;      // lower bound of the pixels per block
// LDS ring stages of wgrad_grp_k (2, 3 or 4): 2 (32 KB, up to four blocks per
// CU) beat the deeper rings (64 KB, two blocks) once the fragment reads stopped
// waiting on the ring's DMAs (profiles/r4/kb_ns*.jsonl, b16_ns_blocks_ab.txt)
static int g_gw_ns = 2;
// 3x3 jobs -> wgrad_halo_k: 0 never; 1 at W >= 32, and at W = 16 with >= 32768
// pixels (the per-tap tile won on the small 16x16 / 8x8 jobs: fewer pixels per
// all-taps block, profiles/r4/halo_wgrad/README.txt)
static int g_gh_on = 1;
// target blocks per halo launch: one block per CU runs at a time, so the
// planner fits the batch into at most this many blocks rounded DOWN to whole
// rounds of the CU count -- 522 blocks on 256 CUs ran as three rounds, the last
// one 2 % full (the mixed decoder batch at 622 instead of ~990 TF/s,
// profiles/r4/halo_wgrad/)
static int g_gh_blocks = 256;
// ... and for flushes of >= 2^g_gh_big_lg2 (tile x pixel) work -- the
// bs128 steps, several 1M-pixel jobs per flush -- half that: twice the
// pixels per block halves the split slabs (written by the blocks, re-read by
// the reduce); the chip is busy with the input-gradient convs there anyway.
// bs128 +2.0 %, bs16 (256 kept by the rule) unchanged, profiles/r5/ab_wgrad_halo_blocks.txt
static int g_gh_blocks_big = 128;
static int g_gh_big_lg2 = 21;
static int g_gh_ns = 2;            // LDS ring stages of wgrad_halo_k (2 or 3)
// pixels per K-step of wgrad_halo_k on W >= 64 jobs (64: half the barriers per MFMA; L0 flush
// 945 -> 1051 TF/s at bs128, profiles/r4/halo_pk64/); 32 elsewhere
static int g_gh_pk = 64;

D3D_API int d3d_wgrad_group_cfg(int blocks, int pk, int minpix) {
  if (blocks > 0) g_gw_blocks = blocks;
  if (pk == 32 || pk == 64) g_gw_pk = pk;
  if (minpix > 0) g_gw_minpix = minpix;
  return 0;
}
D3D_API int d3d_wgrad_group_stages(int ns) {
  if (ns >= 2 && ns <= 4) g_gw_ns = ns;
  return 0;
}
// halo (all-taps) tiles for 3x3 jobs: on (0/1), target blocks, ring stages (2/3); < 0 keeps a value
D3D_API int d3d_wgrad_group_halo(int on, int blocks, int ns) {
  if (on >= 0) g_gh_on = on ? 1 : 0;
  if (blocks > 0) g_gh_blocks = blocks;
  if (ns == 2 || ns == 3) g_gh_ns = ns;
  return 0;
}
// big-flush target blocks and the work threshold (log2 of tile x pixel work); <= 0 keeps a value
D3D_API int d3d_wgrad_group_halo_big(int blocks, int lg2) {
  if (blocks > 0) g_gh_blocks_big = blocks;
  if (lg2 > 0) g_gh_big_lg2 = lg2;
  return 0;
}
D3D_API int d3d_wgrad_group_halo_pk(int pk) {
  if (pk == 32 || pk == 64) g_gh_pk = pk;
  return 0;
}

static int gw_lg2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

// 0 when the grouped kernel takes the job, else the reason (> 0).
D3D_API int d3d_wgrad_group_ok(const WgJobDesc* d) {
  if (d->taps != 1 && d->taps != 9) return 1;
  if (d->OC <= 0 || d->IC <= 0 || d->OC % 8 || d->IC % 8) return 2;
  if (d->taps == 9 && (gw_lg2(d->H) < 0 || gw_lg2(d->W) < 0)) return 3;
  if (d->x2 && (d->C1 <= 0 || d->C1 % GW_BN || d->C1 >= d->IC)) return 4;
  if (((uintptr_t)d->dy | (uintptr_t)d->x | (uintptr_t)d->x2) & 15) return 5;
  if (!d->dw) return 6;
  const long P = (long)d->N * d->H * d->W;
  if (P <= 0 || P >= (1L << 31) - 1) return 7;
  return 0;
}

struct GwPlan {
  int splits[GW_MAX], pps[GW_MAX], tiles[GW_MAX];
  long slab_off[GW_MAX], bslab_off[GW_MAX];
  long ws_floats;
  long blocks;
};

// the all-taps halo tile takes the job (block-shape and alignment conditions)
static bool gh_takes(const WgJobDesc& d) {
  const int Wm = d.W < GH_PK ? d.W : GH_PK;
  const long P = (long)d.N * d.H * d.W;
  if (d.W < 32 && !(d.W == 16 && P >= 32768)) return false;
  return g_gh_on && d.taps == 9 && gw_lg2(d.W) >= 0 && ((uintptr_t)d.dw & 15) == 0 && gw_lg2(d.H) >= 0 && d.H >= GH_PK / Wm &&
         d.OC % GH_BM == 0 && d.IC % GH_BN == 0 && (!d.x2 || d.C1 % GH_BN == 0) &&
         (long)(GH_PK / Wm + 2) * d.W * d.IC * 2 < (1L << 30);
}

// halo: every job of d is a halo job (tiles = 128 x 64 x 9 taps)
static void gw_plan(const WgJobDesc* d, int n, GwPlan& pl, bool halo = false) {
  double work = 0;
  for (int i = 0; i < n; ++i) {
    const long P = (long)d[i].N * d[i].H * d[i].W;
    if (halo) {
      pl.tiles[i] = (d[i].OC / GH_BM) * (d[i].IC / GH_BN);
    } else {
      const int nch = d[i].taps * cdiv(d[i].IC, GW_BN);
      pl.tiles[i] = nch * cdiv(d[i].OC, GW_BM);
    }
    work += (double)pl.tiles[i] * P;
  }
  // one pixel count per block across the batch: ~g_gw_blocks equal blocks
  const int gh_target = work >= (double)(1L << g_gh_big_lg2) ? g_gh_blocks_big : g_gh_blocks;
  long Q = (long)(work / (halo ? gh_target : g_gw_blocks));
  Q = std::max<long>(Q, g_gw_minpix);
  Q = (Q + 63) / 64 * 64;
  if (halo) {
    // whole rounds: the smallest Q whose block count fits the round-down target
    const int cus = device_cus();
    const long T = std::max<long>(cus, (long)g_gh_blocks / cus * cus);
    auto nblk = [&](long q) {
      long t = 0;
      for (int i = 0; i < n; ++i) {
        const long P = (long)d[i].N * d[i].H * d[i].W;
        long s = std::min<long>(std::max<long>((P + q - 1) / q, 1), 64);
        const long pps = ((P + s - 1) / s + 63) / 64 * 64;
        t += (long)pl.tiles[i] * ((P + pps - 1) / pps);
      }
      return t;
    };
    long Pmax = 0;
    for (int i = 0; i < n; ++i) Pmax = std::max<long>(Pmax, (long)d[i].N * d[i].H * d[i].W);
    while (Q < Pmax && nblk(Q) > T) Q += std::max<long>(64, Q / 256 / 64 * 64);   // (unsplit jobs: stop)
  }
  long off = 0, blocks = 0;
  for (int i = 0; i < n; ++i) {
    const long P = (long)d[i].N * d[i].H * d[i].W;
    long s = (P + Q - 1) / Q;
    s = std::min<long>(std::max<long>(s, 1), 64);
    long pps = (P + s - 1) / s;
    pps = (pps + 63) / 64 * 64;
    s = (P + pps - 1) / pps;
    // the dY descriptor spans one split: 31-bit byte count
    while ((long)pps * d[i].OC * 2 >= (1L << 31) - (1L << 20)) {
      ++s;
      pps = ((P + s - 1) / s + 63) / 64 * 64;
      s = (P + pps - 1) / pps;
    }
    pl.splits[i] = (int)s;
    pl.pps[i] = (int)pps;
    pl.slab_off[i] = pl.bslab_off[i] = -1;
    if (s > 1) {
      pl.slab_off[i] = off;
      off += (s * d[i].OC * d[i].taps * (long)d[i].IC + 63) / 64 * 64;
      if (d[i].db) {
        pl.bslab_off[i] = off;
        off += (2 * s * d[i].OC + 63) / 64 * 64;
      }
    }
    blocks += pl.tiles[i] * s;
  }
  pl.ws_floats = off;
  pl.blocks = blocks;
}

// Jobs split by tile engine: the all-taps halo tile (3x3 on W % 32 == 0) and
// the per-tap 128 x 128 tile (everything else); one launch each, planned
// separately (each fills the GPU on its own), one reduce for both.
struct GwSplit {
  WgJobDesc hd[GW_MAX], qd[GW_MAX], od[GW_MAX];
  int hidx[GW_MAX], qidx[GW_MAX], oidx[GW_MAX];
  int hn = 0, qn = 0, on = 0;
  GwPlan hp, qp, op;          // halo 32-pixel steps, halo 64-pixel steps (W >= 64), per-tap tile
  long ws_floats;
};

static void gw_split_plan(const WgJobDesc* d, int n, GwSplit& S) {
  for (int i = 0; i < n; ++i) {
    if (gh_takes(d[i]) && g_gh_pk == 64 && d[i].W >= 64) {
      S.qidx[S.qn] = i;
      S.qd[S.qn++] = d[i];
    } else if (gh_takes(d[i])) {
      S.hidx[S.hn] = i;
      S.hd[S.hn++] = d[i];
    } else {
      S.oidx[S.on] = i;
      S.od[S.on++] = d[i];
    }
  }
  S.hp.ws_floats = S.qp.ws_floats = S.op.ws_floats = 0;
  S.hp.blocks = S.qp.blocks = S.op.blocks = 0;
  if (S.hn) gw_plan(S.hd, S.hn, S.hp, true);
  if (S.qn) gw_plan(S.qd, S.qn, S.qp, true);
  if (S.on) gw_plan(S.od, S.on, S.op, false);
  S.ws_floats = S.hp.ws_floats + S.qp.ws_floats + S.op.ws_floats;
}

// fills tab (and appends the split jobs to rt) for the jobs of one engine
static long gw_tables(const WgJobDesc* d, int n, const GwPlan& pl, float* ws, bool halo, GwTable& tab, GrTable& rt,
                      long& rblk) {
  tab = GwTable{};
  tab.n = n;
  long blk = 0;
  for (int i = 0; i < n; ++i) {
    GwJob& J = tab.j[i];
    const WgJobDesc& D = d[i];
    J.dy = (const bf16*)D.dy;
    J.x = (const bf16*)D.x;
    J.x2 = (const bf16*)D.x2;
    J.dw = D.dw;
    J.db = D.db;
    J.P = (long)D.N * D.H * D.W;
    J.OC = D.OC;
    J.IC = D.IC;
    J.C1 = D.x2 ? D.C1 : D.IC;
    J.taps = D.taps;
    if (D.taps == 1) {             // per-pixel GEMM: rows only, no padding tests
      J.H = J.W = 1;
      J.lw = J.lh = 0;
    } else {
      J.H = D.H;
      J.W = D.W;
      J.lw = gw_lg2(D.W);
      J.lh = gw_lg2(D.H);
    }
    J.ncb = halo ? D.IC / GH_BN : cdiv(D.IC, GW_BN);
    J.nmb = halo ? D.OC / GH_BM : cdiv(D.OC, GW_BM);
    J.splits = pl.splits[i];
    J.pps = pl.pps[i];
    J.blk0 = (int)blk;
    J.acc = D.acc;
    J.scale = D.scale;
    J.slab = pl.splits[i] > 1 ? ws + pl.slab_off[i] : nullptr;
    J.bslab = pl.splits[i] > 1 && D.db ? ws + pl.bslab_off[i] : nullptr;
    blk += (long)pl.tiles[i] * pl.splits[i];
    if (pl.splits[i] > 1) {
      GrJob& Rj = rt.j[rt.n++];
      Rj.slab = J.slab;
      Rj.bslab = J.bslab;
      Rj.dw = D.dw;
      Rj.db = D.db;
      Rj.OC = D.OC;
      Rj.IC = D.IC;
      Rj.taps = D.taps;
      Rj.splits = pl.splits[i];
      Rj.blk0 = (int)rblk;
      // flat: the halo tiles' OIHW slabs, and every 1x1 job's ([co][ci] is OIHW)
      Rj.flat = (halo || D.taps == 1) && ((long)D.OC * D.IC * D.taps) % 4 == 0 && ((uintptr_t)D.dw & 15) == 0;
      Rj.nblk_w = Rj.flat ? (int)cdiv((long)D.OC * D.IC * D.taps, 1024L) : D.OC * cdiv(D.IC, 64);
      Rj.acc = D.acc;
      Rj.scale = D.scale;
      rblk += Rj.nblk_w + (D.db ? cdiv(D.OC, 64) : 0);
    }
  }
  return blk;
}

// Weight gradients of n jobs (n <= 16, each d3d_wgrad_group_ok, no two jobs
// writing the same dw / db) in one grouped launch per tile engine + one
// grouped reduce.  ws == nullptr: returns the workspace size in floats
// (nothing launched).  Otherwise returns 0, or < 0 on error (nothing launched).
D3D_API long d3d_wgrad_group(const WgJobDesc* d, int n, float* ws, long ws_floats, hipStream_t st) {
  if (n < 1 || n > GW_MAX) return -1;
  for (int i = 0; i < n; ++i)
    if (d3d_wgrad_group_ok(d + i)) return -2;
  GwSplit S;
  gw_split_plan(d, n, S);
  if (!ws) return S.ws_floats;
  if (ws_floats < S.ws_floats || S.hp.blocks >= (1L << 31) || S.qp.blocks >= (1L << 31) ||
      S.op.blocks >= (1L << 31))
    return -3;
  GrTable rt{};
  long rblk = 0;
  if (S.qn) {
    GwTable tab;
    const long blk = gw_tables(S.qd, S.qn, S.qp, ws + S.hp.ws_floats, true, tab, rt, rblk);
    hipLaunchKernelGGL((wgrad_halo_k<2, 64>), dim3((unsigned)blk), dim3(512), 0, st, tab);
  }
  if (S.hn) {
    GwTable tab;
    const long blk = gw_tables(S.hd, S.hn, S.hp, ws, true, tab, rt, rblk);
    if (g_gh_ns == 3)
      hipLaunchKernelGGL((wgrad_halo_k<3, 32>), dim3((unsigned)blk), dim3(512), 0, st, tab);
    else
      hipLaunchKernelGGL((wgrad_halo_k<2, 32>), dim3((unsigned)blk), dim3(512), 0, st, tab);
  }
  if (S.on) {
    GwTable tab;
    const long blk = gw_tables(S.od, S.on, S.op, ws + S.hp.ws_floats + S.qp.ws_floats, false, tab, rt, rblk);
    if (g_gw_pk == 64) {
      hipLaunchKernelGGL((wgrad_grp_k<64, 2>), dim3((unsigned)blk), dim3(256), 0, st, tab);
    } else if (g_gw_ns == 4) {
      hipLaunchKernelGGL((wgrad_grp_k<32, 4>), dim3((unsigned)blk), dim3(256), 0, st, tab);
    } else if (g_gw_ns == 3) {
      hipLaunchKernelGGL((wgrad_grp_k<32, 3>), dim3((unsigned)blk), dim3(256), 0, st, tab);
    } else {
      hipLaunchKernelGGL((wgrad_grp_k<32, 2>), dim3((unsigned)blk), dim3(256), 0, st, tab);
    }
  }
  if (rt.n > 0) hipLaunchKernelGGL(wgrad_grp_reduce_k, dim3((unsigned)rblk), dim3(256), 0, st, rt);
  const int e = (int)hipGetLastError();
  return e ? -1000 - e : 0;
}

// Plan introspection for tests / tools: splits and pixels per split of job i.
// (blocks: both launches' blocks; engine[i], when given: 1 = halo tile)
D3D_API int d3d_wgrad_group_plan(const WgJobDesc* d, int n, int* splits, int* pps, long* blocks) {
  if (n < 1 || n > GW_MAX) return -1;
  GwSplit S;
  gw_split_plan(d, n, S);
  for (int i = 0; i < S.hn; ++i) {
    splits[S.hidx[i]] = S.hp.splits[i];
    pps[S.hidx[i]] = S.hp.pps[i];
  }
  for (int i = 0; i < S.qn; ++i) {
    splits[S.qidx[i]] = S.qp.splits[i];
    pps[S.qidx[i]] = S.qp.pps[i];
  }
  for (int i = 0; i < S.on; ++i) {
    splits[S.oidx[i]] = S.op.splits[i];
    pps[S.oidx[i]] = S.op.pps[i];
  }
  if (blocks) *blocks = S.hp.blocks + S.qp.blocks + S.op.blocks;
  return 0;
}
D3D_API int d3d_wgrad_group_engine(const WgJobDesc* d) { return gh_takes(*d) ? 1 : 0; }
