// Small-grid implicit-GEMM 3x3 conv (and 1x1 / per-pixel dense) for the low
// resolution levels at small per-GPU batch: the 8x8 / 16x16 levels at 16-32
// examples per GPU, i.e. the per-GPU share of the global-batch-128 step on 4-8
// GPUs (reference convs: xunet.py:114-126, ResnetBlock conv1/conv2).
//
// Why a separate kernel.  At 16 examples per GPU the 8x8 level is 2,048
// output pixels x 512 channels: 64 blocks of the 128 x 128 tiles (conv_bufl_k),
// so that kernel splits K = 9 x IC eight ways and a second launch sums eight
// fp32 partial slabs (33 MB of partial traffic for a 2 MB output) -- ~36 us per
// conv for 9.7 GFLOP.  Here a block owns a 64 x 64 output tile over the WHOLE
// K: 256 blocks fill the chip with no split, no partial slabs and no epilogue
// launch; the epilogue (bias / per-image bias / residual / scale / GroupNorm
// partial statistics) is fused as in the other conv kernels.
//
//   * 4 waves as 2 (channels) x 2 (pixels), 32 x 32 each: 2 x 2
//     v_mfma_f32_16x16x32_bf16 per 32-deep slice, 8 per 64-deep k-step;
//   * operands land in LDS by buffer-descriptor DMA (buffer_load ... lds,
//     range-checked zero fill for padding taps / tile overhang, XOR chunk
//     swizzle: conflict-free 16-row fragment reads), in a 4-stage ring with
//     one barrier per k-step and counted vmcnt waits, so three k-steps of
//     loads are in flight behind the MFMAs (a 64 x 64 tile is L2-bound: 16 KiB
//     per k-step for 8 MFMA per wave -- the deep ring keeps the L2 pipe full);
//   * XCD-aware block order (consecutive tiles of one channel slab on one XCD
//     share its L2 copy of the weight rows);
//   * GroupNorm partials: the two pixel-half waves of a 64-pixel slot combine
//     through LDS, so the slot layout is the one the GN kernels consume
//     (gn_part_store: [N][G][HW/64] x (sum, sum of squares)).
#include "common.h"

namespace {

// LDS fragment read by inline asm: the compiler's wait-count pass treats every
// LDS load as possibly aliasing any in-flight LDS-DMA write and would put a
// full "s_waitcnt vmcnt(0)" in front of it -- serialising the whole DMA ring
// against the MFMAs.  Ordering here is explicit instead: the counted vmcnt
// wait + barrier before a stage is read, and lds_wait() (which also ties the
// fragment registers, so no MFMA can be scheduled above it) before use.
__device__ __forceinline__ bf16x8 lds_rd128(const bf16* p) {
  bf16x8 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void lds_wait(bf16x8 (&a)[2], bf16x8 (&b)[2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]) :: "memory");
}

constexpr int S64_BM = 64, S64_BN = 64, S64_BK = 64;

// G wave groups (4 waves each) split the K-steps of one 64 x 64 tile
// round-robin (group g takes k-steps g, g + G, ...), each through its own
// NS-stage LDS ring; at the end groups 1.. hand their accumulators to group 0
// through LDS and group 0 sums them in a fixed order (deterministic) and runs
// the epilogue.  G > 1 puts 2-4x the waves on a CU for the small grids (the
// 8x8 / 16x16 levels at batch 16 give only 256-512 tiles): more loads and
// MFMAs in flight per CU where one 4-wave block per tile was latency-bound.
template <int TAPS, bool TRANS, int G = 1, int NS = 4>
__global__ void __launch_bounds__(256 * G, G == 1 ? 2 : 1)
conv_s64_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
           const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O, int in_bytes,
           int w_bytes, int Nimg, int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo, int stride,
           float scale, int res_nmod, float* __restrict__ gnp, int gn_groups, bf16* __restrict__ O2) {
  constexpr int BM = S64_BM, BN = S64_BN, BK = S64_BK;
  constexpr int STAGE = (BM + BN) * BK;                 // elements
  static_assert(G * NS * STAGE * 2 <= 160 * 1024 - 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem_all[G * NS * STAGE];
  __shared__ float gn_x[2][2][2][4];                    // [wm][i][s|q][fq] pixel-half-1 partials
  typedef __attribute__((address_space(3))) void lds_void;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave_g >> 2, wave = wave_g & 3;        // wave group, wave within the group
  bf16* const smem = smem_all + grp * NS * STAGE;
  const int wm = wave >> 1, wn = wave & 1;
  const long Mpix = (long)Nimg * OH * OW;
  // XCD-aware order over the (pixel tile, channel tile) grid, pixel-major
  // within a channel slab
  const int nbx = gridDim.x, nby = gridDim.y;
  int bid = blockIdx.x + nbx * blockIdx.y;
  {
    const int T = nbx * nby, q = T / 8, r = T % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const long n0 = (long)(bid % nbx) * BN;
  const int m0 = (bid / nbx) * BM;
  const int Kp = TAPS * ICp;

  // loader: one 1-KiB DMA piece = 8 rows x 64 k (8 x 16-B chunks); each wave
  // issues 2 pieces of A (weights) and 2 of B (im2col rows) per stage
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, w_bytes, 0x00020000);
  int boff[2], aoff[2];
  unsigned vmask[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int prow = (wave * 2 + i) * 8 + lrow;
    const long p = n0 + prow;
    const bool pv = p < Mpix;
    const unsigned pp = pv ? (unsigned)p : 0u;      // Mpix < 2^31 (host checks operand sizes)
    const int pw = (int)(pp % (unsigned)OW);
    const unsigned t = pp / (unsigned)OW;
    const int poh = (int)(t % (unsigned)OH);
    const int pn = (int)(t / (unsigned)OH);
    const int oh0 = TRANS ? poh : poh * stride, ow0 = TRANS ? pw : pw * stride;
    boff[i] = (((pn * IH + oh0) * IW + ow0) * IC + lchunk * 8) * 2;
    unsigned m = 0;
#pragma unroll
    for (int tp = 0; tp < TAPS; ++tp) {
      const int kh = TAPS == 9 ? tp / 3 : 1, kw = TAPS == 9 ? tp % 3 : 1;
      const int ih = TRANS ? oh0 + 1 - kh : oh0 + kh - 1, iw = TRANS ? ow0 + 1 - kw : ow0 + kw - 1;
      if (pv && ih >= 0 && ih < IH && iw >= 0 && iw < IW) m |= 1u << tp;
    }
    vmask[i] = m;
    // weight rows past the packed tensor (OC overhang) read as zeros
    aoff[i] = ((m0 + prow) * Kp + lchunk * 8) * 2;
  }
  const int lane_cmax = IC - lchunk * 8;

  auto issue = [&](int kstep, int stage) {
    // k-step order: channel chunk major over the nine taps (as conv_bufl_k korder 1)
    const int tap = TAPS == 9 ? kstep % 9 : 0;
    const int c0 = (TAPS == 9 ? kstep / 9 : kstep) * BK;
    const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
    const int tapoff = (TRANS ? ((1 - kh) * IW + (1 - kw)) : ((kh - 1) * IW + (kw - 1))) * IC;
    const int ubyte = (tapoff + c0) * 2;
    const int soffA = (tap * ICp + c0) * 2;
    bf16* sA = smem + stage * STAGE;
    bf16* sB = sA + BM * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sA + (wave * 2 + i) * 8 * BK), 16, aoff[i], soffA, 0, 0);
    const bool cok = c0 < lane_cmax;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned okb = (unsigned)cok & (vmask[i] >> tap) & 1u;   // failed test -> bit 31: zero fill
      const unsigned vo = (unsigned)(boff[i] + ubyte) | ((okb - 1u) & 0x80000000u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rI, (lds_void*)(sB + (wave * 2 + i) * 8 * BK), 16, vo, 0, 0, 0);
    }
  };
  auto swz = [](int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = Kp / BK;
  // this group's k-steps: grp, grp + G, ...; every group runs J iterations
  // (one barrier each) so the block-wide barriers stay matched
  const int nkg = nk > grp ? (nk - grp + G - 1) / G : 0;
  const int J = (nk + G - 1) / G;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkg) issue(grp + s * G, s);
  for (int j = 0; j < J; ++j) {
    // stages j .. j + NS - 2 of this group are in flight (4 DMA pieces each): retire j
    const int after = nkg - 1 - j < NS - 2 ? nkg - 1 - j : NS - 2;
    if (after >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // stage j landed for every wave, and every wave is done reading the
    // buffer the next issue overwrites (it held stage j - 1)
    __builtin_amdgcn_s_barrier();
    if (j + NS - 1 < nkg) issue(grp + (j + NS - 1) * G, (j + NS - 1) % NS);
    if (j >= nkg) continue;
    const bf16* a = smem + (j % NS) * STAGE;
    const bf16* b = a + BM * BK;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lds_rd128(a + swz(wm * 32 + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = lds_rd128(b + swz(wn * 32 + j * 16 + fr, kk * 4 + fq));
      lds_wait(af, bfr);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  if constexpr (G > 1) {
    // groups 1.. hand their accumulators to group 0 through the (drained) ring
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem_all);      // [G - 1][4 waves][2][2][64 lanes]
    if (grp > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) red[((((grp - 1) * 4 + wave) * 2 + i) * 2 + jj) * 64 + lane] = acc[i][jj];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int g = 1; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) acc[i][jj] += red[((((g - 1) * 4 + wave) * 2 + i) * 2 + jj) * 64 + lane];
    }
  }
  const bool lead = grp == 0;                            // group 0 runs the epilogue
  // ---- epilogue: bias / per-image bias / residual / scale, GN partials
  const int OHW = OH * OW;
  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 2 && lead; ++j) {
    const long pix = n0 + wn * 32 + j * 16 + fr;
    if (pix >= Mpix) continue;
    const int img = (int)(pix / OHW);
    const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = m0 + wm * 32 + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cc = co + e < OC ? co + e : OC - 1;
        float t = acc[i][j][e] + (bias ? bias[cc] : 0.f);
        if (row_bias) t += row_bias[(long)img * OC + cc];
        v[e] = t;
      }
      bf16* dst = O + pix * ldo + co;
      if (co + 3 < OC && (ldo & 3) == 0) {
        if (res) {
          const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o4[e] = (bf16)(v[e] * scale);
          const float y = (float)o4[e];
          gs[i] += y;
          gq[i] += y * y;
        }
        *reinterpret_cast<bf16x4*>(dst) = o4;
        if (O2) silu_store4(O2, dst - O, o4);
      } else {
        for (int e = 0; e < 4 && co + e < OC; ++e) {
          float t = v[e];
          if (res) t += (float)res[rpix * ldo + co + e];
          dst[e] = (bf16)(t * scale);
          if (O2) O2[(dst - O) + e] = (bf16)siluf_((float)dst[e]);
          const float y = (float)dst[e];
          gs[i] += y;
          gq[i] += y * y;
        }
      }
    }
  }
  if (!gnp) return;
  // (sum, sum of squares) of the 64-pixel slot per channel group.  Per lane:
  // its 2 pixel columns x 4 channels (already summed).  Reduce the 16 pixels
  // of a fragment column (lanes fr), then the 4-channel lane groups (fq) up to
  // the group width; pixel half wn = 1 hands its sums to wn = 0 through LDS.
  const int Cg = OC / gn_groups;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      gs[i] += __shfl_xor(gs[i], m, 64);
      gq[i] += __shfl_xor(gq[i], m, 64);
    }
    if (Cg >= 8) {
      gs[i] += __shfl_xor(gs[i], 16, 64);
      gq[i] += __shfl_xor(gq[i], 16, 64);
    }
    if (Cg >= 16) {
      gs[i] += __shfl_xor(gs[i], 32, 64);
      gq[i] += __shfl_xor(gq[i], 32, 64);
    }
  }
  if (lead && wn == 1 && fr == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      gn_x[wm][i][0][fq] = gs[i];
      gn_x[wm][i][1][fq] = gq[i];
    }
  }
  __syncthreads();
  if (!lead || wn != 0 || fr != 0) return;
  const long p = n0;                                   // the slot: pixels n0 .. n0 + 63 (64 | OHW)
  if (p >= Mpix) return;
  const long n = p / OHW;
  const int t = (int)(p - n * OHW) / 64;
  const int nparts = OHW / 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int co = m0 + wm * 32 + i * 16 + fq * 4;
    float a = gs[i] + gn_x[wm][i][0][fq], b = gq[i] + gn_x[wm][i][1][fq];
    if (Cg >= 32) {                                    // 32-channel groups: both row tiles of the wave
      if (i != 0 || fq != 0) continue;
      a += gs[1] + gn_x[wm][1][0][0];
      b += gq[1] + gn_x[wm][1][1][0];
    } else if (fq % (Cg / 4) != 0) {
      continue;
    }
    if (co >= OC) continue;
    float* d = gnp + ((n * gn_groups + co / Cg) * nparts + t) * 2;
    d[0] = a;
    d[1] = b;
  }
}


// ------------------------------------------------- small-image halo conv ----
// Stride-1 3x3 conv (and its input gradient, TRANS) of 8- and 16-wide images
// at small grids (the 8x8 / 16x16 levels at 16-32 examples per GPU), with the
// halo staging of conv.hip's conv_halo_k at a 64-channel x 64/128-pixel tile.
// Why: conv_s64_k above streams an im2col row per tap, 16 KiB per 64-deep
// k-step for a 64 x 64 tile (32 FLOP/B), and LDS-DMA fills sustain only
// ~26 B/clk per CU when every CU streams (rocprofv3: TCP->TCC latency ~300-370
// cycles, 2.6k cycles per k-step, 12-16 % MFMA; profiles/r5/s64_diag.txt).
// Here a block owns TR whole rows of one image (TR x OW = 64 or 128 pixels) x
// 64 output channels over the whole K:
//   * per 32-channel chunk the (TR + 2) x (OW + 2) halo (rows padded to a
//     multiple of 8 pixels) is LDS-DMA'd ONCE and feeds the nine taps by
//     address shift, so the input crosses L2 1.6-2.2x instead of 9x: 51-92
//     FLOP per staged byte instead of 32;
//   * the weights of one (tap, chunk) step (64 x 32, 4 KiB, one 1-KiB piece per
//     wave) stream through a 4-slot LDS ring, the halo through two buffers
//     filled one chunk ahead, one barrier per step with counted vmcnt waits
//     (the wait/issue schedule of conv_halo_k);
//   * 4 waves as 2 (channels) x 2 (pixels): 32 x (BN/2) each;
//   * fragment swizzle as conv_halo_k (quarter ^ ((row >> 1) & 2)): the halo
//     row pitch is a multiple of 8 pixels, so every tap shift stays
//     conflict-free;
//   * epilogue: bias, per-image bias, residual (res_nmod broadcast), scale.
//     No GroupNorm partials (the GroupNorms of these levels are whole-image
//     kernels that make their own statistics) and no SiLU companion output:
//     the launcher declines those calls.
constexpr int HSM_CH = 32;

template <int OWT, int TR>
struct HsmGeom {
  static constexpr int BN = TR * OWT;                  // pixels per tile
  static constexpr int HW2 = (OWT + 2 + 7) / 8 * 8;    // halo row pitch (pixels)
  static constexpr int HP = (TR + 2) * HW2;            // halo pixels
  static constexpr int HPW = ((HP + 15) / 16 + 3) / 4; // 1-KiB pieces (16 pixels) per wave
  static constexpr int HBUF = HPW * 4 * 16 * HSM_CH;   // elements per halo buffer
  static constexpr int ABUF = 64 * HSM_CH;             // elements per weight slot
};

// one step's weight piece / one chunk's halo pieces (__device__ functions: a
// buffer resource captured by a kernel lambda can suppress the host stub)
__device__ __forceinline__ void hsm_issue_a(bf16* dst, const bf16* Wp, int w_bytes, int aoff, int soff) {
  typedef __attribute__((address_space(3))) void lds_void;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, w_bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)dst, 16, aoff, soff, 0, 0);
}
template <int HPW>
__device__ __forceinline__ void hsm_issue_b(bf16* hb, const bf16* I, int in_bytes, const unsigned* hoff, int cbyte,
                                            int wave) {
  typedef __attribute__((address_space(3))) void lds_void;
  const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, in_bytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < HPW; ++k)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rI, (lds_void*)(hb + (wave + 4 * k) * 16 * HSM_CH), 16,
                                             hoff[k] + (unsigned)cbyte, 0, 0, 0);
}

// G wave groups (4 waves each) split the channel chunks round-robin (group g
// takes chunks g, g + G, ...), each through its own halo buffers and weight
// ring; groups 1.. hand their accumulators to group 0 through LDS, which sums
// them in a fixed order and runs the epilogue.  With one 4-wave block per CU
// (the grids here are 128-512 blocks) every SIMD held a single wave that
// serialised DMA issue, barrier, fragment reads and MFMAs (~800 cycles per
// 128-cycle MFMA step); G waves per SIMD overlap them.
template <int OWT, int TR, bool TRANS, int G>
__global__ void __launch_bounds__(256 * G, G == 1 ? 2 : 1)
conv_hsm_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
           const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O, int in_bytes,
           int w_bytes, int OH, int IC, int ICp, int OC, float scale, int res_nmod) {
  typedef HsmGeom<OWT, TR> Gm;
  constexpr int BN = Gm::BN, WN = BN / 2, TM = 2, TN = WN / 16;
  constexpr int GLDS = 2 * Gm::HBUF + 4 * Gm::ABUF;     // elements per group
  static_assert(G * GLDS * 2 <= 160 * 1024, "LDS");
  static_assert(G == 1 || (G - 1) * 4 * TM * TN * 64 * 16 <= GLDS * 2 * (G - 1), "reduction area");
  __shared__ __attribute__((aligned(16))) bf16 smem_all[G * GLDS];

  const int lane = threadIdx.x & 63;
  const int wave_g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave_g >> 2, wave = wave_g & 3;
  bf16* const sH = smem_all + grp * GLDS;
  bf16* const sA = sH + 2 * Gm::HBUF;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware order: consecutive tiles of one channel slab on one XCD (its L2
  // keeps the slab's weight rows)
  const int nbx = gridDim.x, nby = gridDim.y;
  int bid = blockIdx.x + nbx * blockIdx.y;
  {
    const int T = nbx * nby, q = T / 8, r = T % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int tile = bid % nbx, m0 = (bid / nbx) * 64;
  const int tpi = OH / TR;
  const int img = tile / tpi, r0 = (tile - img * tpi) * TR;
  const long n0 = ((long)img * OH + r0) * OWT;
  const int Kp = 9 * ICp;

  // weights: row = wave * 16 + (lane >> 2), source quarter = slot ^ ((row >> 1) & 2)
  const int arow = wave * 16 + (lane >> 2);
  const int aoff = ((m0 + arow) * Kp + (((lane & 3) ^ ((arow >> 1) & 2)) << 3)) * 2;
  // halo pieces: flat halo pixel fi = (wave + 4k) * 16 + (lane >> 2)
  unsigned hoff[Gm::HPW];
#pragma unroll
  for (int k = 0; k < Gm::HPW; ++k) {
    const int fi = (wave + 4 * k) * 16 + (lane >> 2);
    const int hr = fi / Gm::HW2, hc = fi - hr * Gm::HW2;
    const int ih = r0 - 1 + hr, iw = hc - 1;
    const bool ok = fi < Gm::HP && ih >= 0 && ih < OH && iw >= 0 && iw < OWT;
    const int q = (lane & 3) ^ ((fi >> 1) & 2);
    const unsigned o = (unsigned)((((img * OH + (ok ? ih : 0)) * OWT + (ok ? iw : 0)) * IC + q * 8) * 2);
    hoff[k] = ok ? o : 0x80000000u;             // past every operand: the range check returns zeros
  }
  const int NCH = IC / HSM_CH;
  const int J = (NCH + G - 1) / G;               // chunk iterations of every group (barriers stay matched)
  // this group's k-th chunk (clamped: loads past the group's last chunk re-read valid data)
  auto gchunk = [&](int k) {
    const int c = grp + k * G;
    return c < NCH ? c : NCH - 1;
  };
  auto issue_a = [&](int s) {                   // group-local step s = 9 k + t
    const int k = s / 9, t = s - k * 9;
    hsm_issue_a(sA + (s & 3) * Gm::ABUF + wave * 16 * HSM_CH, Wp, w_bytes, aoff,
                (t * ICp + gchunk(k) * HSM_CH) * 2);
  };
  auto issue_b = [&](int k) {
    hsm_issue_b<Gm::HPW>(sH + (k & 1) * Gm::HBUF, I, in_bytes, hoff, gchunk(k) * HSM_CH * 2, wave);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  int bo[3][TN], ao[TM];                        // B offsets per kw (a kh shift adds whole pitches), A offsets
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int p = wn * WN + j * 16 + fr;
    const int hp0 = (p / OWT) * Gm::HW2 + (p % OWT);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int hp = hp0 + kw;
      bo[kw][j] = hp * HSM_CH + ((fq ^ ((hp >> 1) & 2)) << 3);
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * 32 + i * 16 + fr;
    ao[i] = row * HSM_CH + ((fq ^ ((row >> 1) & 2)) << 3);
  }

  issue_b(0);
  issue_a(0);
  issue_a(1);
  issue_a(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int k = 0; k < J; ++k) {
    const bf16* hb = sH + (k & 1) * Gm::HBUF;
    const bool live = grp + k * G < NCH;         // wave-uniform
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = k * 9 + t;
      // this step's weights landed (and at t == 0 this chunk's halo); newer loads stay in flight
      if (t >= 1 && t <= 3) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + Gm::HPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      issue_a(s + 3);
      if (t == 0) issue_b(k + 1);
      if (!live) continue;
      const bf16* a = sA + (s & 3) * Gm::ABUF;
      const int kh = TRANS ? 2 - t / 3 : t / 3, kw = TRANS ? 2 - t % 3 : t % 3;
      __builtin_amdgcn_s_setprio(1);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(hb + kh * Gm::HW2 * HSM_CH + bo[kw][j]);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + ao[i]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // tail re-loads drained before exit / reuse

  if constexpr (G > 1) {
    // groups 1.. hand their accumulators to group 0 (area: the drained buffers of groups 1..)
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem_all + GLDS);     // [G - 1][4 waves][TM][TN][64 lanes]
    if (grp > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) red[((((grp - 1) * 4 + wave) * TM + i) * TN + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int g = 1; g < G; ++g)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] += red[((((g - 1) * 4 + wave) * TM + i) * TN + j) * 64 + lane];
  }

  const int OHW = OH * OWT;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = m0 + wm * 32 + i * 16 + fq * 4;
    float cb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[e] = (bias ? bias[co + e] : 0.f) + (row_bias ? row_bias[(long)img * OC + co + e] : 0.f);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long pix = n0 + wn * WN + j * 16 + fr;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + cb[e];
      if (res) {
        const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
        const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * OC + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
      }
      bf16x4 o4;
#pragma unroll
      for (int e = 0; e < 4; ++e) o4[e] = (bf16)(v[e] * scale);
      *reinterpret_cast<bf16x4*>(O + pix * OC + co) = o4;
    }
  }
}

}  // namespace

// 0: wave groups by grid size; 1: one group (the 4-wave form); 2 / 4: 2 / 4
// groups with 2-stage rings; 3: 2 groups with 4-stage rings (A/B, kbench)
static int g_s64_cfg = 0;
D3D_API void d3d_conv_s64_cfg(int cfg) { g_s64_cfg = cfg; }

// Launch the small-tile kernel when it applies; returns 1 if launched (and
// *gn_done = 1 when the GroupNorm partials were written), 0 if not applicable.
extern "C" int d3d_conv_s64_try(const void* I, const void* Wp, const float* bias, const float* row_bias,
                                const void* res, void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW,
                                int OC, int ldo, int stride, int trans, float scale, int res_nmod, int taps,
                                float* gnp, int gn_groups, int* gn_done, hipStream_t st, void* O2) {
  const long Mpix = (long)N * OH * OW;
  const long in_bytes = (long)N * IH * IW * IC * 2;
  const long w_bytes = (long)((OC + 127) / 128 * 128) * taps * ICp * 2;
  if ((trans && stride != 1) || in_bytes >= (1L << 31) || w_bytes >= (1L << 31) || OC % 64 || (taps * ICp) % 64)
    return 0;
  if (gnp) {
    const int Cg = gn_groups > 0 && OC % gn_groups == 0 ? OC / gn_groups : 0;
    if (!((Cg == 4 || Cg == 8 || Cg == 16 || Cg == 32) && (OH * OW) % 64 == 0 && ldo == OC)) gnp = nullptr;
  }
  dim3 grid((unsigned)((Mpix + 63) / 64), (unsigned)(OC / 64), 1);
  const long blocks = (long)grid.x * grid.y;
  const int nk = taps * ICp / 64;
  // wave groups per tile: the grid alone gives ~one 4-wave block per CU
  // (256 tiles) or two (512): split each tile's K over 4 / 2 groups
  int cfg = g_s64_cfg;
  if (cfg == 0) cfg = nk < 8 ? 1 : blocks <= 320 ? 4 : blocks <= 640 ? 2 : 1;
#define S64(TP, TR, GV, NSV)                                                                                    \
  hipLaunchKernelGGL((conv_s64_k<TP, TR, GV, NSV>), grid, dim3(256 * GV), 0, st, (const bf16*)I, (const bf16*)Wp, \
                     bias, row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, N, IH, IW, IC, ICp, OH, \
                     OW, OC, ldo, stride, scale, res_nmod, gnp, gn_groups, (bf16*)O2)
#define S64G(TP, TR)                                                                                            \
  do {                                                                                                          \
    if (cfg == 4) S64(TP, TR, 4, 2);                                                                            \
    else if (cfg == 2) S64(TP, TR, 2, 2);                                                                       \
    else if (cfg == 3) S64(TP, TR, 2, 4);                                                                       \
    else S64(TP, TR, 1, 4);                                                                                     \
  } while (0)
  if (taps == 9) {
    if (trans) S64G(9, true); else S64G(9, false);
  } else {
    if (trans) S64G(1, true); else S64G(1, false);
  }
#undef S64G
#undef S64
  if (gn_done) *gn_done = gnp ? 1 : 0;
  const int e = (int)hipGetLastError();
  return e ? -e : 1;
}

// Small-image halo conv (conv_hsm_k) when it applies: stride 1, 3x3, 8- or
// 16-wide images with 8 | OH, IC % 32 == 0, OC % 64 == 0, contiguous output,
// no GroupNorm partials / SiLU companion requested, and a grid of at least
// 128 blocks.  Returns 1 if launched, 0 if not applicable, < 0 on a launch error.
// 0: off; 1: on, wave groups by image width (default); 2 / 3 / 4: 1 / 2 / 4 (8-wide) or 3 (16-wide)
// groups (A/B knob D3D_CONV_HSM)
static int g_hsm = 1;
D3D_API void d3d_conv_hsm_cfg(int v) { g_hsm = v; }
extern "C" int d3d_conv_hsm_try(const void* I, const void* Wp, const float* bias, const float* row_bias,
                                const void* res, void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW,
                                int OC, int ldo, int stride, int trans, float scale, int res_nmod, int taps,
                                const float* gnp, const void* O2, hipStream_t st) {
  if (!g_hsm || taps != 9 || stride != 1 || IH != OH || IW != OW || ldo != OC || gnp || O2) return 0;
  if ((OW != 8 && OW != 16) || OH % 8 || OC % 64 || IC % HSM_CH || ICp < IC || ICp % HSM_CH) return 0;
  const long in_bytes = (long)N * IH * IW * IC * 2;
  const long w_bytes = (long)((OC + 127) / 128 * 128) * 9 * ICp * 2;
  if (in_bytes >= (1L << 31) || w_bytes >= (1L << 31)) return 0;
  const long tiles = (long)N * (OH / 8);
  if (tiles * (OC / 64) < 128 || tiles >= (1L << 24)) return 0;
  dim3 grid((unsigned)tiles, (unsigned)(OC / 64), 1);
  // auto: 4 (8-wide) / 3 (16-wide) groups on grids of one block per CU, else 2
  // (tools/kbench_s64.py --hsm 2,3,4: 8x8x512 at 32 frames 26.4 -> 24.1 us with
  // 4 groups, at 64 frames 30.2 -> 33.3 us)
  const int gmax = OW == 8 ? 4 : 3;
  int g = g_hsm == 2 ? 1 : g_hsm == 3 ? 2 : g_hsm == 4 ? gmax : (tiles * (OC / 64) <= 320 ? gmax : 2);
#define HSM(OWv, TRv, Gv)                                                                                        \
  hipLaunchKernelGGL((conv_hsm_k<OWv, 8, TRv, Gv>), grid, dim3(256 * Gv), 0, st, (const bf16*)I, (const bf16*)Wp, \
                     bias, row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, OH, IC, ICp, OC,     \
                     scale, res_nmod)
#define HSMG(OWv, TRv, G3)                                                                                       \
  do {                                                                                                          \
    if (g == 1) HSM(OWv, TRv, 1);                                                                               \
    else if (g == 2) HSM(OWv, TRv, 2);                                                                          \
    else HSM(OWv, TRv, G3);                                                                                     \
  } while (0)
  if (OW == 8) {
    if (trans) HSMG(8, true, 4); else HSMG(8, false, 4);
  } else {
    if (trans) HSMG(16, true, 3); else HSMG(16, false, 3);
  }
#undef HSMG
#undef HSM
  const int e = (int)hipGetLastError();
  return e ? -e : 1;
}
