// 3x3 convolution (padding 1, stride s) as implicit GEMM on gfx950 MFMA.
//
// Replaces the 76 Conv2d(3x3) of the X-UNet (xunet.py:114-126,294-297,385,
// 473): 54 % of the model FLOPs (+12 % for the strided conditioning convs).
//
// Forward / dgrad kernel (conv_igemm_k):
//   D[co][pix] = sum_k Wp[co][k] * im2col(I)[k][pix],   k = (tap, ci)
//   * A operand = packed weights [OC_pad][9][IC_pad] bf16 (K-contiguous rows),
//     B operand = im2col gathered on the fly from NHWC input (each pixel's
//     channels are contiguous, so an MFMA B fragment is one 16-byte load);
//   * orientation puts PIXELS on the MFMA column (lane) and 4 consecutive
//     output channels in each lane's accumulators, so the NHWC epilogue stores
//     8 contiguous bytes per lane;
//   * 128x128 block tile, BK=64 (one tap x 64 channels), 4 waves (2x2), each
//     wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles, fp32 accumulate;
//   * register-staged double-buffered LDS (global loads for step t+1 in
//     flight while step t's MFMAs run), XOR-swizzled 128-byte LDS rows so the
//     ds_read_b128 fragment reads are conflict-free;
//   * zero-fill for padding / out-of-range taps / channel tails in the loader;
//   * fused epilogue: + bias[co] + row_bias[image][co] (+ residual) * scale;
//   * TRANS=true computes the input gradient of a strided conv
//     (src = (o + 1 - k) / s when divisible) with weights packed [ci][tap][co].
//
// Weight gradient kernel (conv_wgrad_k):
//   dW[co][(tap,ci)] = sum_pix dY[pix][co] * I[src(pix,tap)][ci]
//   both operands have the reduction (pixel) axis as their SLOW memory axis,
//   so tiles are stored pixel-major in LDS and MFMA fragments are read with
//   the gfx950 transpose read ds_read_b64_tr_b16; rows are padded by 32 B and
//   the pixel order inside a 32-pixel step is permuted identically for both
//   operands so that every transpose read is bank-conflict free.  Split-K over
//   pixels with fp32 partial slabs + a deterministic reduce kernel that also
//   writes the OIHW layout of the parameter gradient.
#include "common.h"
#include <stdlib.h>

#include <algorithm>

D3D_API int d3d_colsum(const float* in, long R, int Cc, float* part, float* out, float* out_odd, int accumulate,
                       hipStream_t st);

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

constexpr int BK = 64;

template <int BM, int BN, bool TRANS, int TAPS>
__global__ void __launch_bounds__(256, 2)
conv_igemm_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
             const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O, int Nimg,
             int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo, int stride, float scale,
             int res_nmod) {
  constexpr int WM = BM / 2, WN = BN / 2;       // 2x2 waves
  constexpr int TM = WM / 16, TN = WN / 16;     // MFMA tiles per wave
  constexpr int A_LD = BM * BK / 8 / 256;       // 16B loads per thread
  constexpr int B_LD = BN * BK / 8 / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * BK];
  bf16* As = smem;
  bf16* Bs = smem + 2 * BM * BK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long Mpix = (long)Nimg * OH * OW;
  // XCD-aware remap: neighbouring pixel tiles (which share input rows and
  // the whole weight panel) land on the same XCD's L2.
  const int nbx = gridDim.x;
  int bid = blockIdx.x;
  {
    int q = nbx / 8, r = nbx % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const long n0 = (long)bid * BN;               // pixel tile start
  const int m0 = blockIdx.y * BM;               // output-channel tile start
  const int Kp = TAPS * ICp;

  // per-thread B rows (pixels): fixed over the K loop
  const int cb = tid & 7;                        // 16B chunk within the BK row
  int pn[B_LD], poh[B_LD], pow_[B_LD];
  bool pvalid[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    long p = n0 + (tid >> 3) + i * 32;
    pvalid[i] = p < Mpix;
    long pp = pvalid[i] ? p : 0;
    pow_[i] = (int)(pp % OW);
    long t = pp / OW;
    poh[i] = (int)(t % OH);
    pn[i] = (int)(t / OH);
  }

  bf16x8 ra[A_LD], rb[B_LD];
  const bf16x8 zero8 = {};
  auto gload = [&](int kstep) {
    const int tap = TAPS == 9 ? kstep / (ICp / BK) : 0;
    const int c0 = (TAPS == 9 ? kstep % (ICp / BK) : kstep) * BK;
    const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;   // 1x1 == centre tap
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      int r = (tid >> 3) + i * 32;
      ra[i] = *reinterpret_cast<const bf16x8*>(Wp + (long)(m0 + r) * Kp + tap * ICp + c0 + cb * 8);
    }
    const int c = c0 + cb * 8;
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      int ih, iw;
      bool ok = pvalid[i] && c < IC;
      if (!TRANS) {
        ih = poh[i] * stride + kh - 1;
        iw = pow_[i] * stride + kw - 1;
      } else if (stride == 1) {      // wave-uniform: no integer division in the common case
        ih = poh[i] + 1 - kh;
        iw = pow_[i] + 1 - kw;
      } else {
        int th = poh[i] + 1 - kh, tw = pow_[i] + 1 - kw;
        ok = ok && th >= 0 && tw >= 0 && (th % stride) == 0 && (tw % stride) == 0;
        ih = th / stride;
        iw = tw / stride;
      }
      ok = ok && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
      rb[i] = ok ? *reinterpret_cast<const bf16x8*>(I + (((long)pn[i] * IH + ih) * IW + iw) * IC + c) : zero8;
    }
  };
  auto swz = [](int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); };
  auto swrite = [&](int buf) {
    bf16* a = As + buf * BM * BK;
    bf16* b = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) *reinterpret_cast<bf16x8*>(a + swz((tid >> 3) + i * 32, cb)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_LD; ++i) *reinterpret_cast<bf16x8*>(b + swz((tid >> 3) + i * 32, cb)) = rb[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = Kp / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload(ks + 1);
    const bf16* a = As + buf * BM * BK;
    const bf16* b = Bs + buf * BN * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int row = wm * WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(a + swz(row, kk * 4 + fq));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int row = wn * WN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(b + swz(row, kk * 4 + fq));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nk) swrite(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: D[co][pix] -> O[pix][co] (NHWC) ----
  const int OHW = OH * OW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    long pix = n0 + wn * WN + j * 16 + fr;
    if (pix >= Mpix) continue;
    int img = (int)(pix / OHW);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int c = co + e < OC ? co + e : OC - 1;
        float t = acc[i][j][e] + (bias ? bias[c] : 0.f);
        if (row_bias) t += row_bias[(long)img * OC + c];
        v[e] = t;
      }
      bf16* dst = O + pix * ldo + co;
      // residual row: same pixel, or (image % res_nmod) for a residual that is
      // broadcast over the batch (per-frame conditioning term)
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
      if (co + 3 < OC && (ldo & 3) == 0) {
        if (res) {
          bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = (bf16)(v[e] * scale);
        *reinterpret_cast<bf16x4*>(dst) = o4;
      } else {
        for (int e = 0; e < 4 && co + e < OC; ++e) {
          float t = v[e];
          if (res) t += (float)res[rpix * ldo + co + e];
          dst[e] = (bf16)(t * scale);
        }
      }
    }
  }
}

// ---------------------------------------------------- glds pipeline ------
// Same GEMM as conv_igemm_k, but operand tiles go global -> LDS directly
// (global_load_lds_dwordx4: no VGPR staging, no ds_write), double-buffered
// with a COUNTED vmcnt so the next tile's DMA stays in flight across the raw
// s_barrier while the current tile's MFMAs run.  LDS images are lane-linear
// per wave instruction (8 rows x 128 B = 1 KiB); the XOR swizzle lives in the
// per-lane SOURCE address (lane L of an instruction loads logical chunk
// (L%8)^(L/8) of its row), read back with the same swizzle -> conflict-free
// ds_read_b128.  Padding / out-of-range taps read from a 16-byte zero page.
template <int TAPS, bool TRANS>
__global__ void __launch_bounds__(256, 2)
conv_glds_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
            const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O,
            const bf16* __restrict__ zero16, int Nimg, int IH, int IW, int IC, int ICp, int OH, int OW, int OC,
            int ldo, int stride, float scale, int res_nmod, float* __restrict__ part, int korder) {
  constexpr int BM = 128, BN = 128, BKk = 64;
  constexpr int WM = 64, WN = 64, TM = 4, TN = 4;
  constexpr int STAGE = (BM + BN) * BKk;           // elements per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE];
  typedef __attribute__((address_space(3))) void lds_void;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long Mpix = (long)Nimg * OH * OW;
  const int nbx = gridDim.x;
  int bid = blockIdx.x;
  {
    int q = nbx / 8, r = nbx % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const long n0 = (long)bid * BN;
  const int m0 = blockIdx.y * BM;
  const int Kp = TAPS * ICp;

  // glds lane mapping: wave w issues instructions i=0..3 covering rows
  // (w*4+i)*8 .. +7 of each tile; lane L -> row +L/8, logical chunk (L%8)^(L/8)
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  int prow[4];
  int pn[4], poh[4], pw[4];
  bool pval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    prow[i] = (wave * 4 + i) * 8 + lrow;
    long p = n0 + prow[i];
    pval[i] = p < Mpix;
    long pp = pval[i] ? p : 0;
    pw[i] = (int)(pp % OW);
    long t = pp / OW;
    poh[i] = (int)(t % OH);
    pn[i] = (int)(t / OH);
  }
  const bf16* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wrow[i] = Wp + (long)(m0 + prow[i]) * Kp + lchunk * 8;

  auto issue = [&](int kstep, int stage) {
    // korder 1 (channel-chunk major): the 9 taps of one 64-channel chunk are
    // consecutive k-steps, so a block's shifted input rows are re-read while
    // they are still in L2/L1 (tap-major order re-reads them ICp/64 steps
    // apart and thrashes the XCD's 4 MB L2 at 64 resident blocks)
    int tap, c0;
    if (TAPS == 9 && korder) {
      tap = kstep % 9;
      c0 = (kstep / 9) * BKk;
    } else {
      tap = TAPS == 9 ? kstep / (ICp / BKk) : 0;
      c0 = (TAPS == 9 ? kstep % (ICp / BKk) : kstep) * BKk;
    }
    const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
    bf16* sA = smem + stage * STAGE;
    bf16* sB = sA + BM * BKk;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(wrow[i] + tap * ICp + c0),
                                       (lds_void*)(sA + (wave * 4 + i) * 8 * BKk), 16, 0, 0);
    const int c = c0 + lchunk * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int ih, iw;
      bool ok = pval[i] && c < IC;
      if (!TRANS) {
        ih = poh[i] * stride + kh - 1;
        iw = pw[i] * stride + kw - 1;
      } else if (stride == 1) {
        ih = poh[i] + 1 - kh;
        iw = pw[i] + 1 - kw;
      } else {
        int th = poh[i] + 1 - kh, tw = pw[i] + 1 - kw;
        ok = ok && th >= 0 && tw >= 0 && (th % stride) == 0 && (tw % stride) == 0;
        ih = th / stride;
        iw = tw / stride;
      }
      ok = ok && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
      const bf16* src = ok ? I + (((long)pn[i] * IH + ih) * IW + iw) * IC + c : zero16;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sB + (wave * 4 + i) * 8 * BKk), 16, 0, 0);
    }
  };
  auto swz = [](int row, int chunk) { return row * BKk + ((chunk ^ (row & 7)) << 3); };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (small grids): blockIdx.z owns k-steps [k0, k1) and writes an
  // fp32 partial slab; conv_splitk_epi_k sums the slabs and applies the epilogue
  const int nk_all = Kp / BKk;
  const int k0 = (int)((long)blockIdx.z * nk_all / gridDim.z);
  const int k1 = (int)((long)(blockIdx.z + 1) * nk_all / gridDim.z);
  const int nk = k1 - k0;
  const int fr = lane & 15, fq = lane >> 4;
  issue(k0, 0);
  for (int ks = 0; ks < nk; ++ks) {
    const int st = ks & 1;
    if (ks + 1 < nk) {
      issue(k0 + ks + 1, st ^ 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // retire stage st, keep st^1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const bf16* a = smem + st * STAGE;
    const bf16* b = a + BM * BKk;
#pragma unroll
    for (int kk = 0; kk < BKk / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + swz(wm * WM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + swz(wn * WN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                             // stage st free for reuse
  }

  const int OHW = OH * OW;
  if (part) {
    float* slab = part + (long)blockIdx.z * Mpix * OC;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      long pix = n0 + wn * WN + j * 16 + fr;
      if (pix >= Mpix) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int co = m0 + wm * WM + i * 16 + fq * 4;
        if (co >= OC) continue;
        *reinterpret_cast<f32x4*>(slab + pix * OC + co) = acc[i][j];
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    long pix = n0 + wn * WN + j * 16 + fr;
    if (pix >= Mpix) continue;
    int img = (int)(pix / OHW);
    const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int cc = co + e < OC ? co + e : OC - 1;
        float t = acc[i][j][e] + (bias ? bias[cc] : 0.f);
        if (row_bias) t += row_bias[(long)img * OC + cc];
        v[e] = t;
      }
      bf16* dst = O + pix * ldo + co;
      if (co + 3 < OC && (ldo & 3) == 0) {
        if (res) {
          bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = (bf16)(v[e] * scale);
        *reinterpret_cast<bf16x4*>(dst) = o4;
      } else {
        for (int e = 0; e < 4 && co + e < OC; ++e) {
          float t = v[e];
          if (res) t += (float)res[rpix * ldo + co + e];
          dst[e] = (bf16)(t * scale);
        }
      }
    }
  }
}

// fused GroupNorm statistics: gn_part_store (common.h)

template <int TAPS, bool TRANS, bool ONEBAR>
__global__ void __launch_bounds__(256, 2)
conv_bufl_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
            const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O,
            int in_bytes, int w_bytes, int Nimg, int IH, int IW, int IC, int ICp, int OH, int OW, int OC,
            int ldo, int stride, float scale, int res_nmod, float* __restrict__ part, int korder,
            float* __restrict__ gnp, int gn_groups, bf16* __restrict__ O2) {
  constexpr int BM = 128, BN = 128, BKk = 64;
  constexpr int WM = 64, WN = 64, TM = 4, TN = 4;
  constexpr int STAGE = (BM + BN) * BKk;           // elements per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE];
  typedef __attribute__((address_space(3))) void lds_void;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long Mpix = (long)Nimg * OH * OW;
  const int nbx = gridDim.x;
  int bid = blockIdx.x;
  {
    int q = nbx / 8, r = nbx % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const long n0 = (long)bid * BN;
  const int m0 = blockIdx.y * BM;
  const int Kp = TAPS * ICp;

  // LDS-DMA through buffer descriptors (buffer_load_dwordx4 ... lds): a
  // 32-bit per-lane byte offset instead of a 64-bit address, and padding /
  // out-of-range taps come back as zeros from the descriptor's range check
  // (offset 0x80000000 is past every operand), so the per-k-step loader work
  // is one add + one mask test per row -- the 64-bit im2col address math of
  // conv_glds_k cost ~12 VALU per MFMA and made that kernel issue-bound.
  // Same lane mapping / XOR swizzle as conv_glds_k.
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, w_bytes, 0x00020000);
  int boff[4], aoff[4];
  unsigned vmask[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int prow = (wave * 4 + i) * 8 + lrow;
    const long p = n0 + prow;
    const bool pv = p < Mpix;
    const long pp = pv ? p : 0;
    const int pw = (int)(pp % OW);
    const long t = pp / OW;
    const int poh = (int)(t % OH);
    const int pn = (int)(t / OH);
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
    aoff[i] = ((m0 + prow) * Kp + lchunk * 8) * 2;
  }
  const int lane_cmax = IC - lchunk * 8;          // chunk valid iff c0 < lane_cmax

  auto issue = [&](int kstep, int stage) {
    int tap, c0;
    if (TAPS == 9 && korder) {
      tap = kstep % 9;
      c0 = (kstep / 9) * BKk;
    } else {
      tap = TAPS == 9 ? kstep / (ICp / BKk) : 0;
      c0 = (TAPS == 9 ? kstep % (ICp / BKk) : kstep) * BKk;
    }
    const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
    const int tapoff = (TRANS ? ((1 - kh) * IW + (1 - kw)) : ((kh - 1) * IW + (kw - 1))) * IC;
    const int ubyte = (tapoff + c0) * 2;            // wave-uniform
    const int soffA = (tap * ICp + c0) * 2;
    bf16* sA = smem + stage * STAGE;
    bf16* sB = sA + BM * BKk;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sA + (wave * 4 + i) * 8 * BKk), 16, aoff[i], soffA, 0,
                                               0);
    const bool cok = c0 < lane_cmax;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // branch-free: a failed test sets bit 31 (past every operand's range)
      const unsigned okb = (unsigned)cok & (vmask[i] >> tap) & 1u;
      const unsigned vo = (unsigned)(boff[i] + ubyte) | ((okb - 1u) & 0x80000000u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rI, (lds_void*)(sB + (wave * 4 + i) * 8 * BKk), 16, vo, 0, 0, 0);
    }
  };
  auto swz = [](int row, int chunk) { return row * BKk + ((chunk ^ (row & 7)) << 3); };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (small grids): blockIdx.z owns k-steps [k0, k1) and writes an
  // fp32 partial slab; conv_splitk_epi_k sums the slabs and applies the epilogue
  const int nk_all = Kp / BKk;
  const int k0 = (int)((long)blockIdx.z * nk_all / gridDim.z);
  const int k1 = (int)((long)(blockIdx.z + 1) * nk_all / gridDim.z);
  const int nk = k1 - k0;
  const int fr = lane & 15, fq = lane >> 4;
  const int OHW = OH * OW;
  // residual prefetch (see conv_halo_k); not on split-K partial launches
  bf16x4 rres[TM][TN];
  const bool pre_res = res != nullptr && part == nullptr && (ldo & 3) == 0;
  if (pre_res) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long pix = n0 + wn * WN + j * 16 + fr;
      const long pc = pix < Mpix ? pix : 0;
      const int img = (int)(pc / OHW);
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pc - (long)img * OHW) : pc;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = m0 + wm * WM + i * 16 + fq * 4;
        rres[i][j] = (pix < Mpix && co + 3 < OC) ? *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co)
                                                 : bf16x4{};
      }
    }
  }
  issue(k0, 0);
  if (ONEBAR) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pre_res) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(__builtin_bit_cast(unsigned long long, rres[i][j])));
    }
    __builtin_amdgcn_s_barrier();
  }
  for (int ks = 0; ks < nk; ++ks) {
    const int st = ks & 1;
    if (ONEBAR) {
      // one barrier per k-step (cdna guide T3/T4 "minimum 2-phase"): stage
      // the next tile first (its buffer was last read before the previous
      // barrier), compute this one at raised priority, then wait + barrier
      if (ks + 1 < nk) issue(k0 + ks + 1, st ^ 1);
    } else {
      if (ks + 1 < nk) {
        issue(k0 + ks + 1, st ^ 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // retire stage st, keep st^1 in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
    }
    const bf16* a = smem + st * STAGE;
    const bf16* b = a + BM * BKk;
    if (ONEBAR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BKk / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + swz(wm * WM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + swz(wn * WN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (ONEBAR) {
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                           // next stage landed everywhere; this one free
      continue;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                             // stage st free for reuse
  }

  if (part) {
    float* slab = part + (long)blockIdx.z * Mpix * OC;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      long pix = n0 + wn * WN + j * 16 + fr;
      if (pix >= Mpix) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int co = m0 + wm * WM + i * 16 + fq * 4;
        if (co >= OC) continue;
        *reinterpret_cast<f32x4*>(slab + pix * OC + co) = acc[i][j];
      }
    }
    return;
  }
  float gs[TM][1], gq[TM][1];                     // fused GroupNorm partials (gn_part_store)
#pragma unroll
  for (int i = 0; i < TM; ++i) gs[i][0] = gq[i][0] = 0.f;
  float cb[TM][4];                                // bias, once per row tile
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[i][e] = (bias && co + e < OC) ? bias[co + e] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    long pix = n0 + wn * WN + j * 16 + fr;
    if (pix >= Mpix) continue;
    int img = (int)(pix / OHW);
    const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int cc = co + e < OC ? co + e : OC - 1;
        float t = acc[i][j][e] + cb[i][e];
        if (row_bias) t += row_bias[(long)img * OC + cc];
        v[e] = t;
      }
      bf16* dst = O + pix * ldo + co;
      if (co + 3 < OC && (ldo & 3) == 0) {
        if (res) {
          if (pre_res) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)rres[i][j][e];
          } else {
            const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
          }
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o4[e] = (bf16)(v[e] * scale);
          const float y = (float)o4[e];
          gs[i][0] += y;
          gq[i][0] += y * y;
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
          gs[i][0] += y;
          gq[i][0] += y * y;
        }
      }
    }
  }
  if (gnp) gn_part_store<TM, 1>(gs, gq, lane, m0 + wm * WM, n0 + wn * WN, OC, gn_groups, OHW, Mpix, gnp);
}

// ------------------------------------------------ 8-wave large tile ------
// conv_bufl_k's loader and LDS image at one 512-thread block per CU with a
// BM x 256 tile (BM = 256 or 128 output channels x 256 pixels).  Why: at two
// 128x128 blocks per CU a BK=64 k-step moves 64 KiB through L2 for 4.2 MFLOP,
// i.e. ~64 B/clk/CU at the MFMA rate -- above the ~56 B/clk/CU the L2 can
// deliver per CU (34.5 TB/s / 256 CUs / 2.4 GHz).  A 256x256 tile halves the
// bytes per FLOP (32 B/clk at the MFMA rate), and its k-step (64 MFMA per wave,
// 2 waves per SIMD, ~2k cycles) is several times the ~250-400 cycle LDS-DMA
// landing latency, so two LDS stages with one barrier per k-step keep the
// next tile in flight behind the whole MFMA phase.  Waves are 2 (channels) x
// 4 (pixels); each owns a (BM/2) x 64 output tile = TM x 4 16x16 MFMA tiles.
// One k-step's LDS-DMA issue for conv_w8_k (a __device__ function: a buffer
// resource captured by a kernel lambda can suppress the kernel's host stub).
template <int TAPS, bool TRANS, int BM, int APW, int BPW>
__device__ __forceinline__ void w8_issue(bf16* sA, const bf16* I, const bf16* Wp, int in_bytes, int w_bytes, int kstep,
                                         int korder, int ICp, int IC, int IW, int wave, const int* aoff,
                                         const int* boff, const unsigned* vmask, int lane_cmax) {
  typedef __attribute__((address_space(3))) void lds_void;
  constexpr int BKk = 64;
  const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, w_bytes, 0x00020000);
  int tap, c0;
  if (TAPS == 9 && korder) {
    tap = kstep % 9;
    c0 = (kstep / 9) * BKk;
  } else {
    tap = TAPS == 9 ? kstep / (ICp / BKk) : 0;
    c0 = (TAPS == 9 ? kstep % (ICp / BKk) : kstep) * BKk;
  }
  const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
  const int tapoff = (TRANS ? ((1 - kh) * IW + (1 - kw)) : ((kh - 1) * IW + (kw - 1))) * IC;
  const int ubyte = (tapoff + c0) * 2;
  const int soffA = (tap * ICp + c0) * 2;
  bf16* sB = sA + BM * BKk;
#pragma unroll
  for (int i = 0; i < APW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sA + (wave * APW + i) * 8 * BKk), 16, aoff[i] + soffA, 0,
                                             0, 0);
  const bool cok = c0 < lane_cmax;
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const unsigned okb = (unsigned)cok & (vmask[i] >> tap) & 1u;     // branch-free select
    const unsigned vo = (unsigned)(boff[i] + ubyte) | ((okb - 1u) & 0x80000000u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rI, (lds_void*)(sB + (wave * BPW + i) * 8 * BKk), 16, vo, 0, 0, 0);
  }
}

// RES = false: no residual operand (res must be null) -- the prefetch
// registers (TM x TN x 2 VGPRs) are not reserved, which the 256-VGPR budget of
// the 8-wave tile needs for its fragment reads (the dgrad and the first conv of
// a ResnetBlock carry no residual).
template <int TAPS, bool TRANS, int BM, int BN, bool RES = true>
__global__ void __launch_bounds__(512, 1)
conv_w8_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
          const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O,
          int in_bytes, int w_bytes, int Nimg, int IH, int IW, int IC, int ICp, int OH, int OW, int OC,
          int ldo, int stride, float scale, int res_nmod, int korder, float* __restrict__ gnp, int gn_groups,
          bf16* __restrict__ O2) {
  constexpr int BKk = 64;
  // 8 waves as 2 x 4 (M x N) over >= 256-pixel tiles; 4 x 2 over the
  // 128-pixel tile (256 x 128: the 32x32 level at 16 examples per GPU, one
  // block per CU) so every wave still owns a whole 64-pixel GN slot
  constexpr int WGN = BN >= 256 ? 4 : 2, WGM = 8 / WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int APW = BM / 64, BPW = BN / 64;      // 1-KiB DMA pieces per wave per operand
  constexpr int STAGE = (BM + BN) * BKk;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE];
  typedef __attribute__((address_space(3))) void lds_void;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // SGPR: LDS-DMA bases stay scalar
  const int wm = wave / WGN, wn = wave % WGN;
  const long Mpix = (long)Nimg * OH * OW;
  const int nbx = gridDim.x;
  int bid = blockIdx.x;
  {
    int q = nbx / 8, r = nbx % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const long n0 = (long)bid * BN;
  const int m0 = blockIdx.y * BM;
  const int Kp = TAPS * ICp;

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  int boff[BPW], aoff[APW];
  unsigned vmask[BPW];
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int prow = (wave * BPW + i) * 8 + lrow;
    const long p = n0 + prow;
    const bool pv = p < Mpix;
    const unsigned pp = pv ? (unsigned)p : 0u;       // 32-bit: Mpix < 2^31 (host checks operand sizes)
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
  }
  // weight rows past the packed tensor (OC tile overhang) fall outside the
  // descriptor's range and read as zeros
#pragma unroll
  for (int i = 0; i < APW; ++i) aoff[i] = ((m0 + (wave * APW + i) * 8 + lrow) * Kp + lchunk * 8) * 2;
  const int lane_cmax = IC - lchunk * 8;

  auto issue = [&](int kstep, int stage) {
    w8_issue<TAPS, TRANS, BM, APW, BPW>(smem + stage * STAGE, I, Wp, in_bytes, w_bytes, kstep, korder, ICp, IC, IW,
                                        wave, aoff, boff, vmask, lane_cmax);
  };
  auto swz = [](int row, int chunk) { return row * BKk + ((chunk ^ (row & 7)) << 3); };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = Kp / BKk;
  const int fr = lane & 15, fq = lane >> 4;
  const int OHW = OH * OW;
  // residual prefetch (see conv_halo_k): issued ahead of the first stage,
  // drained with it, held in registers through the K loop
  bf16x4 rres[RES ? TM : 1][RES ? TN : 1];
  const bool vec_out = (ldo & 3) == 0;
  if (RES && res && vec_out) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long pix = n0 + wn * WN + j * 16 + fr;
      const long pc = pix < Mpix ? pix : 0;
      const int img = (int)(pc / OHW);
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pc - (long)img * OHW) : pc;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = m0 + wm * WM + i * 16 + fq * 4;
        rres[i][j] = (pix < Mpix && co + 3 < OC) ? *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co)
                                                 : bf16x4{};
      }
    }
  }
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (RES) {
    if (res && vec_out) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(__builtin_bit_cast(unsigned long long, rres[i][j])));
    }
  }
  __builtin_amdgcn_s_barrier();
  for (int ks = 0; ks < nk; ++ks) {
    const int st = ks & 1;
    // buffer st^1 was last read before the previous barrier: restage it now,
    // it lands while this k-step's MFMAs run
    if (ks + 1 < nk) issue(ks + 1, st ^ 1);
    const bf16* a = smem + st * STAGE;
    const bf16* b = a + BM * BKk;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BKk / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + swz(wn * WN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + swz(wm * WM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  constexpr int NH = WN / 64;                     // 64-pixel GroupNorm partial slots per wave slice
  float gs[TM][NH], gq[TM][NH];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int h = 0; h < NH; ++h) gs[i][h] = gq[i][h] = 0.f;
  float cb[TM][4];                                // bias, once per row tile
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[i][e] = (bias && co + e < OC) ? bias[co + e] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long pix = n0 + wn * WN + j * 16 + fr;
    if (pix >= Mpix) continue;
    const int img = (int)(pix / OHW);
    const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = m0 + wm * WM + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cc = co + e < OC ? co + e : OC - 1;
        float t = acc[i][j][e] + cb[i][e];
        if (row_bias) t += row_bias[(long)img * OC + cc];
        v[e] = t;
      }
      bf16* dst = O + pix * ldo + co;
      if (co + 3 < OC && vec_out) {
        if constexpr (RES) {
          if (res) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)rres[i][j][e];
          }
        }
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o4[e] = (bf16)(v[e] * scale);
          const float y = (float)o4[e];
          gs[i][j / 4] += y;
          gq[i][j / 4] += y * y;
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
          gs[i][j / 4] += y;
          gq[i][j / 4] += y * y;
        }
      }
    }
  }
  if (gnp) gn_part_store<TM, NH>(gs, gq, lane, m0 + wm * WM, n0 + wn * WN, OC, gn_groups, OHW, Mpix, gnp);
}

// ------------------------------------------------- halo (direct) 3x3 conv ----
// Stride-1 3x3 conv (and its input gradient, TRANS) that stages each input
// pixel in LDS ONCE per 32-channel chunk and feeds all nine taps from it.
// The implicit-GEMM kernels above re-fetch the im2col row of every tap from
// L2: at 128 output channels the 128 x 512 tile moves 80 KiB per 64-deep
// k-step (~39 B/clk/CU at the MFMA rate, against ~56 B/clk of L2->CU
// bandwidth), so the 64x64-level convs ran L2-bound at ~600 TF/s.  Here a
// block owns TR full image rows x OW (= 512 pixels) x 128 output channels:
//   * the (TR+2) x (OW+2) halo of a 32-channel chunk (64-byte pixel rows, 42
//     KiB at OW=64) is LDS-DMA'd once and read by the nine taps by pure
//     address shift -- the MFMA B fragment of tap (kh, kw) is the halo row
//     (r+kh) * (OW+2) + c + kw -- so the input crosses L2 ~1.3x instead of 9x;
//   * the weights of one (tap, chunk) step (128 x 32, 8 KiB, one 1-KiB DMA
//     piece per wave) stream through a 4-deep LDS ring, the halo through two
//     buffers filled one whole chunk (nine steps) ahead; total L2 traffic is
//     ~12 B/clk/CU at the MFMA rate;
//   * XOR swizzle of the 16-byte channel quarter by ((row >> 1) & 2) keeps
//     every 16-row fragment read conflict-free for any tap shift under the
//     ds_read_b128 lane groups ({0-3,12-15,20-27}, ...: lanes fr and fr+4 of
//     neighbouring quarters share a group).  The earlier ((row >> 2) & 3)
//     swizzle was conflict-free only for contiguous 16-lane groups and ran
//     2-way conflicted: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 47 %
//     (profiles/r3/pmc_step/);
//   * one barrier per step; the counted vmcnt waits only for the step's own
//     weights (issue order: weights then halo, so in-order completion lets the
//     halo land up to four steps later).
// Waves are 2 (channels) x 4 (pixels), 64 x 128 each (TM=4, TN=8), as in
// conv_w8_k, and the epilogue (bias / per-image bias / residual / scale,
// fused GroupNorm partials) is the same.
constexpr int HALO_CH = 32;

template <int OWT, int BNT = 512>
struct HaloGeom {
  static constexpr int TR = BNT / OWT;                        // image rows per tile
  // halo row length, padded to a multiple of 8 pixels: the fragment swizzle
  // depends on pixel bits 1-2 only, so a kh shift of whole halo rows keeps it
  // (the tap's B offsets are a constant per kh; the pad pixels are never loaded)
  static constexpr int HW2 = (OWT + 2 + 7) / 8 * 8;
  static constexpr int HP = (TR + 2) * HW2;                    // halo pixels
  static constexpr int HPW = (HP + 127) / 128;                 // 1-KiB pieces per wave (16 pixels each)
  static constexpr int HBUF = HPW * 8 * 16 * HALO_CH;          // bf16 elements per halo buffer
  static constexpr int ABUF = 128 * HALO_CH;                   // bf16 elements per weight ring slot
};

__device__ __forceinline__ void halo_issue_a(bf16* sA, const bf16* Wp, int w_bytes, int aoff, int soff, int wave) {
  typedef __attribute__((address_space(3))) void lds_void;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, w_bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sA + wave * 16 * HALO_CH), 16, aoff, soff, 0, 0);
}

template <int HPW>
__device__ __forceinline__ void halo_issue_b(bf16* sH, const bf16* I, int in_bytes, const unsigned* hoff, int cbyte,
                                             int wave) {
  typedef __attribute__((address_space(3))) void lds_void;
  const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, in_bytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < HPW; ++k)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rI, (lds_void*)(sH + (wave + 8 * k) * 16 * HALO_CH), 16,
                                             hoff[k] + (unsigned)cbyte, 0, 0, 0);
}

// AU: the nine taps unrolled with every B-fragment LDS offset precomputed
// (9 x TN registers): the swizzled address of a tap-shifted halo pixel is not
// linear in the shift, and computing it per step cost ~48 VALU per 32 MFMAs
// on the critical path between the barrier and the first MFMA.  (Without the
// residual prefetch only: with it the register file overflows.)
// P2 (with AU): one barrier per PAIR of taps over an 8-slot weight ring (the
// LDS budget of the 64-wide tile: 2 x 48 KB halo + 64 KB ring = all 160 KB);
// halves the per-MFMA barrier / wait cost.  Needs an even chunk count.
// GNA (with AU, forward, single taps per barrier): the input is the
// PRE-GroupNorm tensor x and the conv runs on silu(x * A + B) -- the
// ResnetBlock's GN0 + SiLU folded into the halo staging (gab [Nimg][IC][2] =
// (A, B) per image and channel, norm.hip gn_ab_k; the image's rows of it sit
// in LDS).  Each lane transforms the 16-byte pieces it DMA'd itself (its 8
// channels are fixed per lane: quarter (lane & 3) ^ ((lane >> 3) & 2)), once
// per chunk, at the step after the chunk's wait, before the barrier that
// publishes it; pads stay zero.  (Not on the tap-pair schedule: its 160 KB of
// LDS leave no room for the table, and the 16 (A, B) registers it would hold
// instead spill it.)
template <int OWT, bool TRANS, int BNT = 512, bool PF = false, bool RES = true, bool AU = false, bool P2 = false,
          bool GNA = false>
__global__ void __launch_bounds__(512, 1)
conv_halo_k(const bf16* __restrict__ I, const bf16* __restrict__ Wp, const float* __restrict__ bias,
            const float* __restrict__ row_bias, const bf16* __restrict__ res, bf16* __restrict__ O, int in_bytes,
            int w_bytes, int Nimg, int OH, int IC, int ICp, int OC, float scale, int res_nmod,
            float* __restrict__ gnp, int gn_groups, bf16* __restrict__ O2, const float* __restrict__ gab) {
  static_assert(!GNA || (AU && !P2 && !TRANS && !PF), "GroupNorm staging: forward, unrolled single-tap schedule");
  __shared__ __attribute__((aligned(16))) float sG[GNA ? 2 * 512 : 4];
  typedef HaloGeom<OWT, BNT> Gm;
  constexpr int BM = 128, BN = BNT, WM = 64, WN = BN / 4, TM = 4, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * Gm::HBUF + (P2 ? 8 : 4) * Gm::ABUF];
  bf16* const sH = smem;                       // [2][HBUF]
  bf16* const sAr = smem + 2 * Gm::HBUF;       // [4 or 8][ABUF]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int OW = OWT, IH = OH, IW = OW;
  const int tiles = Nimg * (OH / Gm::TR);
  int bid = blockIdx.x;
  {
    // XCD-aware: consecutive row tiles (which share halo rows) on one XCD
    int q = tiles / 8, r = tiles % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int img = bid / (OH / Gm::TR);
  const int r0 = (bid - img * (OH / Gm::TR)) * Gm::TR;
  const long n0 = ((long)img * OH + r0) * OW;    // first output pixel of the tile
  const long Mpix = (long)Nimg * OH * OW;
  const int m0 = blockIdx.y * BM;
  const int Kp = 9 * ICp;

  // weights: row = wave*16 + (lane>>2), source quarter = slot ^ ((row>>2)&3)
  const int arow = wave * 16 + (lane >> 2);
  const int aoff = ((m0 + arow) * Kp + (((lane & 3) ^ ((arow >> 1) & 2)) << 3)) * 2;
  // halo pieces: flat halo pixel fi = (wave + 8k)*16 + (lane>>2)
  unsigned hoff[Gm::HPW];
#pragma unroll
  for (int k = 0; k < Gm::HPW; ++k) {
    const int fi = (wave + 8 * k) * 16 + (lane >> 2);
    const int hr = fi / Gm::HW2, hc = fi - hr * Gm::HW2;
    const int ih = r0 - 1 + hr, iw = hc - 1;
    const bool ok = fi < Gm::HP && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
    const int q = (lane & 3) ^ ((fi >> 1) & 2);
    const unsigned o = (unsigned)((((img * IH + (ok ? ih : 0)) * IW + (ok ? iw : 0)) * IC + q * 8) * 2);
    hoff[k] = ok ? o : 0x80000000u;            // past every operand: the range check returns zeros
  }
  // GNA: the in-LDS transform of this lane's own landed pieces of chunk c
  const int gnq = (lane & 3) ^ ((lane >> 3) & 2);
  auto gn_apply = [&](bf16* hb, int c) {
    if constexpr (GNA) {
      // 4 channels at a time, (A, B) re-read from LDS per half piece: few live
      // registers beside the 128 accumulators (holding all 16 spilled)
      // (opaque lane offsets: per-piece addresses hoisted out of the K loop
      // held ~24 registers through it and spilled)
      int lo = lane * 8 + wave * 16 * HALO_CH, to = (c * HALO_CH + gnq * 8) * 2;
      asm volatile("" : "+v"(lo), "+v"(to));
      const f32x4* t = reinterpret_cast<const f32x4*>(sG + to);
#pragma unroll
      for (int k = 0; k < Gm::HPW; ++k) {
        // image border / past the halo: stays zero (a select, not a branch:
        // a divergent region here made the allocator spill the K loop)
        const bool ok = hoff[k] != 0x80000000u;
        bf16x2* q = reinterpret_cast<bf16x2*>(hb + lo + 8 * k * 16 * HALO_CH);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const f32x4 a = t[h];                             // (A, B) of channels 2h, 2h + 1
          const bf16x2 v = q[h];
          bf16x2 o;
          o[0] = (bf16)siluf_(__builtin_fmaf((float)v[0], a[0], a[1]));
          o[1] = (bf16)siluf_(__builtin_fmaf((float)v[1], a[2], a[3]));
          q[h] = ok ? o : v;
          __builtin_amdgcn_sched_barrier(0);              // one channel pair at a time: few live registers
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // written before the publishing barrier
    }
  };

  const int NCH = IC / HALO_CH, S = 9 * NCH;
  auto a_soff = [&](int s) {
    const int ss = s < S ? s : S - 1;          // tail re-loads keep the wait counts uniform
    const int c = ss / 9, t = ss - c * 9;
    return (t * ICp + c * HALO_CH) * 2;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // halo row of each B fragment's pixel at tap (0, 0)
  int hp0[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int p = wn * WN + j * 16 + fr;
    hp0[j] = (p / OWT) * Gm::HW2 + (p % OWT);
  }
  const int OHW = OH * OW;
  // Residual prefetch: issued ahead of the first operand DMA and drained by
  // its full wait, then held in registers through the K loop.  In the
  // epilogue the 8-byte residual reads (16 pixels x 32 B per instruction)
  // were fully exposed -- one block per CU, nothing left to overlap them --
  // and cost +30 % on the level-0 conv (tools/kbench_conv_epi.py).
  // AU: the residual goes straight into the accumulators instead (the
  // epilogue computes (acc + bias + res) * scale either way), which frees
  // the 64 prefetch registers the unrolled-tap offsets need
  constexpr bool RPF = RES && !AU;
  bf16x4 rres[RPF ? TM : 1][RPF ? TN : 1];
  if (RES && res) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long pix = n0 + wn * WN + j * 16 + fr;
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = m0 + wm * WM + i * 16 + fq * 4;
        const bf16x4 r4 = co < OC ? *reinterpret_cast<const bf16x4*>(res + rpix * OC + co) : bf16x4{};
        if constexpr (RPF) {
          rres[i][j] = r4;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = (float)r4[e];
        }
      }
    }
  }

  auto frags = [&](bf16x8 (&af)[TM], bf16x8 (&bfr)[TN], const bf16* a, const bf16* hb, int t) {
    const int kh = TRANS ? 2 - t / 3 : t / 3, kw = TRANS ? 2 - t % 3 : t % 3;
    const int dsh = kh * Gm::HW2 + kw;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int hp = hp0[j] + dsh;
      bfr[j] = *reinterpret_cast<const bf16x8*>(hb + hp * HALO_CH + ((fq ^ ((hp >> 1) & 2)) << 3));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + fr;
      af[i] = *reinterpret_cast<const bf16x8*>(a + row * HALO_CH + ((fq ^ ((row >> 1) & 2)) << 3));
    }
  };
  if constexpr (PF) {
    // fragment double-buffering: step s+1's weights are waited for at step
    // s's barrier (ring issue distance 4), so its LDS fragment reads go out
    // while step s's MFMAs run instead of in front of them
    halo_issue_b<Gm::HPW>(sH, I, in_bytes, hoff, 0, wave);
#pragma unroll
    for (int k = 0; k < 4; ++k) halo_issue_a(sAr + k * Gm::ABUF, Wp, w_bytes, aoff, a_soff(k), wave);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    bf16x8 af[TM], bfr[TN];
    frags(af, bfr, sAr, sH, 0);
    int s = 0;
    for (int c = 0; c < NCH; ++c) {
#pragma unroll 1
      for (int t = 0; t < 9; ++t, ++s) {
        // (lgkmcnt(0): the prefetched fragments of this slot must be read
        // before the barrier frees it for the DMA below)
        if (t >= 1 && t <= 3) {
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 + Gm::HPW) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        halo_issue_a(sAr + ((s + 4) & 3) * Gm::ABUF, Wp, w_bytes, aoff, a_soff(s + 4), wave);
        if (t == 0) {
          const int cn = c + 1 < NCH ? c + 1 : NCH - 1;
          halo_issue_b<Gm::HPW>(sH + ((c + 1) & 1) * Gm::HBUF, I, in_bytes, hoff, cn * HALO_CH * 2, wave);
        }
        bf16x8 an[TM], bn[TN];
        if (s + 1 < S) {
          const int cn = t == 8 ? c + 1 : c, tn = t == 8 ? 0 : t + 1;
          frags(an, bn, sAr + ((s + 1) & 3) * Gm::ABUF, sH + (cn & 1) * Gm::HBUF, tn);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = an[i];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = bn[j];
      }
    }
  } else if constexpr (AU && P2) {
  // prologue: halo of chunk 0, weights of steps 0..3
  halo_issue_b<Gm::HPW>(sH, I, in_bytes, hoff, 0, wave);
#pragma unroll
  for (int k = 0; k < 4; ++k) halo_issue_a(sAr + k * Gm::ABUF, Wp, w_bytes, aoff, a_soff(k), wave);
  int bo[3][TN], ao[TM];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int hp = hp0[j] + kw;
      bo[kw][j] = hp * HALO_CH + ((fq ^ ((hp >> 1) & 2)) << 3);
    }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * WM + i * 16 + fr;
    ao[i] = row * HALO_CH + ((fq ^ ((row >> 1) & 2)) << 3);
  }
  auto step = [&](int s, int t, const bf16* hb) {
    const bf16* a = sAr + (s & 7) * Gm::ABUF;
    const int kh = TRANS ? 2 - t / 3 : t / 3, kw = TRANS ? 2 - t % 3 : t % 3;
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(hb + kh * Gm::HW2 * HALO_CH + bo[kw][j]);
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + ao[i]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };
  // chunks in pairs (18 steps = 9 tap pairs per iteration); step s: chunk s / 9,
  // tap s % 9, weights in ring slot s & 7, issued 4 steps ahead.  Halo of the
  // next chunk issued at the first pair after the previous chunk's last step
  // (pairs 0 and 5 of an iteration); waits allow the newer halo pieces in
  // flight at the two pairs after its issue.
  for (int c2 = 0; c2 < NCH; c2 += 2) {
    const int S0 = c2 * 9;
#pragma unroll
    for (int pp = 0; pp < 9; ++pp) {
      if (pp == 1 || pp == 2 || pp == 6 || pp == 7) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + Gm::HPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      const int s0 = S0 + 2 * pp;
      halo_issue_a(sAr + ((s0 + 4) & 7) * Gm::ABUF, Wp, w_bytes, aoff, a_soff(s0 + 4), wave);
      halo_issue_a(sAr + ((s0 + 5) & 7) * Gm::ABUF, Wp, w_bytes, aoff, a_soff(s0 + 5), wave);
      if (pp == 0 || pp == 5) {
        const int cn0 = c2 + (pp == 0 ? 1 : 2), cn = cn0 < NCH ? cn0 : NCH - 1;
        halo_issue_b<Gm::HPW>(sH + (cn0 & 1) * Gm::HBUF, I, in_bytes, hoff, cn * HALO_CH * 2, wave);
      }
      __builtin_amdgcn_s_setprio(1);
      const int sr0 = 2 * pp, sr1 = 2 * pp + 1;            // steps within the chunk pair
      step(S0 + sr0, sr0 % 9, sH + (sr0 / 9) * Gm::HBUF);
      step(S0 + sr1, sr1 % 9, sH + (sr1 / 9) * Gm::HBUF);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  } else if constexpr (AU) {
  float gt[GNA ? 2 : 1];
  if constexpr (GNA) {                         // this image's (A, B) rows: into LDS behind the prologue DMAs
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = tid + 512 * i;
      gt[i] = j < 2 * IC ? gab[(long)img * IC * 2 + j] : 0.f;
    }
  }
  halo_issue_b<Gm::HPW>(sH, I, in_bytes, hoff, 0, wave);
  halo_issue_a(sAr, Wp, w_bytes, aoff, a_soff(0), wave);
  halo_issue_a(sAr + Gm::ABUF, Wp, w_bytes, aoff, a_soff(1), wave);
  halo_issue_a(sAr + 2 * Gm::ABUF, Wp, w_bytes, aoff, a_soff(2), wave);
  if constexpr (GNA) {
#pragma unroll
    for (int i = 0; i < 2; ++i) sG[tid + 512 * i] = gt[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (GNA) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();              // the table is complete
    gn_apply(sH, 0);
  }
  int bo[3][TN], ao[TM];                       // per kw; the kh shift is a constant (HW2 % 8 == 0)
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int hp = hp0[j] + kw;
      bo[kw][j] = hp * HALO_CH + ((fq ^ ((hp >> 1) & 2)) << 3);
    }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * WM + i * 16 + fr;
    ao[i] = row * HALO_CH + ((fq ^ ((row >> 1) & 2)) << 3);
  }
  for (int c = 0; c < NCH; ++c) {
    const bf16* hb = sH + (c & 1) * Gm::HBUF;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = c * 9 + t;
      if (t >= 1 && t <= 3) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + Gm::HPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      halo_issue_a(sAr + ((s + 3) & 3) * Gm::ABUF, Wp, w_bytes, aoff, a_soff(s + 3), wave);
      if (t == 0) {
        const int cn = c + 1 < NCH ? c + 1 : NCH - 1;
        halo_issue_b<Gm::HPW>(sH + ((c + 1) & 1) * Gm::HBUF, I, in_bytes, hoff, cn * HALO_CH * 2, wave);
      }
      // chunk c + 1 landed at step 4's wait: this lane's pieces, before step 5's barrier
      if (t == 4) gn_apply(sH + ((c + 1) & 1) * Gm::HBUF, c + 1 < NCH ? c + 1 : NCH - 1);
      const bf16* a = sAr + (s & 3) * Gm::ABUF;
      __builtin_amdgcn_s_setprio(1);
      bf16x8 af[TM], bfr[TN];
      const int kh = TRANS ? 2 - t / 3 : t / 3, kw = TRANS ? 2 - t % 3 : t % 3;
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(hb + kh * Gm::HW2 * HALO_CH + bo[kw][j]);
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
  } else {
  halo_issue_b<Gm::HPW>(sH, I, in_bytes, hoff, 0, wave);
  halo_issue_a(sAr, Wp, w_bytes, aoff, a_soff(0), wave);
  halo_issue_a(sAr + Gm::ABUF, Wp, w_bytes, aoff, a_soff(1), wave);
  halo_issue_a(sAr + 2 * Gm::ABUF, Wp, w_bytes, aoff, a_soff(2), wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (RES) {
    if (res) {
      // pin the prefetched values here (keeps the loads ahead of the K loop)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(__builtin_bit_cast(unsigned long long, rres[i][j])));
    }
  }

  for (int c = 0; c < NCH; ++c) {
    const bf16* hb = sH + (c & 1) * Gm::HBUF;
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int s = c * 9 + t;
      // this step's weights landed; newer loads may stay in flight
      if (t >= 1 && t <= 3) {                     // (wave-uniform branch)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + Gm::HPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      halo_issue_a(sAr + ((s + 3) & 3) * Gm::ABUF, Wp, w_bytes, aoff, a_soff(s + 3), wave);
      if (t == 0) {
        const int cn = c + 1 < NCH ? c + 1 : NCH - 1;
        halo_issue_b<Gm::HPW>(sH + ((c + 1) & 1) * Gm::HBUF, I, in_bytes, hoff, cn * HALO_CH * 2, wave);
      }
      const bf16* a = sAr + (s & 3) * Gm::ABUF;
      const int kh = TRANS ? 2 - t / 3 : t / 3, kw = TRANS ? 2 - t % 3 : t % 3;
      const int dsh = kh * Gm::HW2 + kw;
      __builtin_amdgcn_s_setprio(1);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int hp = hp0[j] + dsh;
        bfr[j] = *reinterpret_cast<const bf16x8*>(hb + hp * HALO_CH + ((fq ^ ((hp >> 1) & 2)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(a + row * HALO_CH + ((fq ^ ((row >> 1) & 2)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tail re-loads drained before exit

  constexpr int NH = WN / 64;
  float gs[TM][NH], gq[TM][NH];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int h = 0; h < NH; ++h) gs[i][h] = gq[i][h] = 0.f;
  // per-channel additive terms, once per row tile (not per element)
  float cb[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
      if (co + e < OC) {
        if (bias) t += bias[co + e];
        if (row_bias) t += row_bias[(long)img * OC + co + e];
      }
      cb[i][e] = t;
    }
  }
  // The output tile leaves through LDS (free after the K loop; the tile,
  // BN x 128 bf16 = at most 128 KiB, fits): each lane parks its bf16x4
  // fragments in a [pixel][128 ch] image (16-byte chunks XOR-swizzled by
  // pixel & 15), then the block streams it out as whole 256-byte pixel rows,
  // 16 bytes per lane.  The direct form stored 8 bytes per lane into 16
  // different pixel rows per instruction (32-byte pieces), twice with the
  // SiLU output: store-issue-bound at ~3 B/clk/CU -- the level-0
  // conditioning conv (K = 576, 1024 + 1024 output channels per pixel) ran
  // at 20 % MFMA, ~1.5 TB/s of writes.  D3D_HALO_EPI_DIRECT: the old form
  // (A/B build).
#ifdef D3D_HALO_EPI_DIRECT
  constexpr bool LEPI = false;
#else
  constexpr bool LEPI = true;
#endif
  static_assert(2 * Gm::HBUF + (P2 ? 8 : 4) * Gm::ABUF >= BN * 128, "output tile must fit the LDS");
  const bool lepi = LEPI && (OC % 8) == 0;
  bf16* const sT = smem;                       // [BN][128] bf16, swizzled
  if (lepi) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();              // every wave is done reading the K loop's LDS
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long pix = n0 + wn * WN + j * 16 + fr;
    const int pl = wn * WN + j * 16 + fr;      // tile-local pixel
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = m0 + wm * WM + i * 16 + fq * 4;
      if (co >= OC) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + cb[i][e];
      if constexpr (RPF) {
        if (res) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)rres[i][j][e];
        }
      }
      bf16x4 o4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o4[e] = (bf16)(v[e] * scale);
        const float y = (float)o4[e];
        gs[i][j / 4] += y;
        gq[i][j / 4] += y * y;
      }
      if (lepi) {
        const int cl = wm * WM + i * 16 + fq * 4;          // tile-local channel (0..127)
        *reinterpret_cast<bf16x4*>(sT + pl * 128 + (((cl >> 3) ^ (pl & 15)) << 3) + (cl & 4)) = o4;
      } else {
        *reinterpret_cast<bf16x4*>(O + pix * OC + co) = o4;
        if (O2) silu_store4(O2, pix * OC + co, o4);
      }
    }
  }
  if (gnp) gn_part_store<TM, NH>(gs, gq, lane, m0 + wm * WM, n0 + wn * WN, OC, gn_groups, OHW, Mpix, gnp);
  if (lepi) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // 16 lanes per 256-byte pixel row (channel chunks past OC skipped)
#pragma unroll 4
    for (int idx = tid; idx < BN * 16; idx += 512) {
      const int pl = idx >> 4, c = idx & 15;
      const int co = m0 + c * 8;
      if (co >= OC) continue;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(sT + pl * 128 + ((c ^ (pl & 15)) << 3));
      const long off = (n0 + pl) * OC + co;
      *reinterpret_cast<bf16x8*>(O + off) = v;
      if (O2) {
        bf16x8 s8;
#pragma unroll
        for (int e = 0; e < 8; ++e) s8[e] = (bf16)siluf_((float)v[e]);
        *reinterpret_cast<bf16x8*>(O2 + off) = s8;
      }
    }
  }
}

// split-K epilogue: O[pix][co] = (sum_s part[s][pix][co] + bias + row_bias
// (+ residual)) * scale, 4 channels per thread (OC % 4 == 0).
__global__ void conv_splitk_epi_k(const float* __restrict__ part, int nsplit, long Mpix, int OC, int OHW,
                                  const float* __restrict__ bias, const float* __restrict__ row_bias,
                                  const bf16* __restrict__ res, int res_nmod, bf16* __restrict__ O, int ldo,
                                  float scale, bf16* __restrict__ O2) {
  const long nv = Mpix * (OC / 4);
  const long slab = Mpix * OC;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < nv; v += (long)gridDim.x * blockDim.x) {
    long pix = v / (OC / 4);
    int co = (int)(v % (OC / 4)) * 4;
    f32x4 a = *reinterpret_cast<const f32x4*>(part + pix * OC + co);
    for (int sp = 1; sp < nsplit; ++sp) a += *reinterpret_cast<const f32x4*>(part + sp * slab + pix * OC + co);
    int img = (int)(pix / OHW);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = a[e] + (bias ? bias[co + e] : 0.f);
      if (row_bias) t += row_bias[(long)img * OC + co + e];
      a[e] = t;
    }
    if (res) {
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
      bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * ldo + co);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += (float)r4[e];
    }
    bf16x4 o4;
#pragma unroll
    for (int e = 0; e < 4; ++e) o4[e] = (bf16)(a[e] * scale);
    *reinterpret_cast<bf16x4*>(O + pix * ldo + co) = o4;
    if (O2) silu_store4(O2, pix * ldo + co, o4);
  }
}

// split-K epilogue that also emits the GroupNorm partial statistics of its
// output (gn_part_store layout): one block per (64-pixel part, 64-channel
// slab) -- whole groups (Cg <= 32) of one image, so every (image, group,
// part) slot is written by exactly one block, no atomics.  Statistics are
// taken on the stored bf16 values, like the statistics pass.
__global__ void __launch_bounds__(256) conv_splitk_epi_gn_k(const float* __restrict__ part, int nsplit, long Mpix,
                                                            int OC, int OHW, const float* __restrict__ bias,
                                                            const float* __restrict__ row_bias,
                                                            const bf16* __restrict__ res, int res_nmod,
                                                            bf16* __restrict__ O, float scale,
                                                            float* __restrict__ gnp, int G, bf16* __restrict__ O2) {
  constexpr int CB = 64, TPC = CB / 4, PPI = 256 / TPC;   // 16 threads per pixel, 16 pixels per pass
  __shared__ float s_s[PPI][CB / 4], s_q[PPI][CB / 4];
  const int tid = threadIdx.x, r = tid / TPC, cq = tid % TPC;
  const long pix0 = (long)blockIdx.x * 64;
  const int co = blockIdx.y * CB + cq * 4;
  const long slab = Mpix * OC;
  const int Cg = OC / G;
  float sum = 0.f, sq = 0.f;
  constexpr int KP = 64 / PPI;
  f32x4 acc[KP];                                   // all pixels' slab loads in flight together
#pragma unroll
  for (int k = 0; k < KP; ++k) acc[k] = *reinterpret_cast<const f32x4*>(part + (pix0 + k * PPI + r) * OC + co);
  for (int sp = 1; sp < nsplit; ++sp)
#pragma unroll
    for (int k = 0; k < KP; ++k)
      acc[k] += *reinterpret_cast<const f32x4*>(part + sp * slab + (pix0 + k * PPI + r) * OC + co);
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const long pix = pix0 + k * PPI + r;
    f32x4 a = acc[k];
    const int img = (int)(pix / OHW);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = a[e] + (bias ? bias[co + e] : 0.f);
      if (row_bias) t += row_bias[(long)img * OC + co + e];
      a[e] = t;
    }
    if (res) {
      const long rpix = res_nmod > 0 ? (long)(img % res_nmod) * OHW + (pix - (long)img * OHW) : pix;
      bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + rpix * OC + co);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += (float)r4[e];
    }
    bf16x4 o4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o4[e] = (bf16)(a[e] * scale);
      const float y = (float)o4[e];
      sum += y;
      sq += y * y;
    }
    *reinterpret_cast<bf16x4*>(O + pix * OC + co) = o4;
    if (O2) silu_store4(O2, pix * OC + co, o4);
  }
  s_s[r][cq] = sum;
  s_q[r][cq] = sq;
  __syncthreads();
  const int ng = CB / Cg;                          // groups in this slab
  if (tid < ng) {
    const int q4 = Cg / 4;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < PPI; ++rr)
      for (int j = 0; j < q4; ++j) {
        a += s_s[rr][tid * q4 + j];
        b += s_q[rr][tid * q4 + j];
      }
    const long n = pix0 / OHW;
    const int t = (int)(pix0 - n * OHW) / 64;
    const int g = (blockIdx.y * CB) / Cg + tid;
    float* d = gnp + ((n * G + g) * (OHW / 64) + t) * 2;
    d[0] = a;
    d[1] = b;
  }
}

// ------------------------------------------------------------ wgrad ------
constexpr int WBK = 32;           // pixels per k-step
constexpr int WPAD = 16;          // bf16 elements of row padding (32 B)

__device__ __forceinline__ s16x4 ds_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// The same transposed LDS read as inline asm.  The compiler's wait-count
// pass cannot tell an LDS load from the LDS-DMA writes still in flight to
// the OTHER pipeline stage, so in front of the first ds_read_tr of every
// stage it inserted "s_waitcnt vmcnt(0)" -- i.e. each stage waited for the
// NEXT stage's loads to land before computing, serialising DMA and MFMA.
// With the read in asm the only waits are the kernels' own (counted vmcnt +
// barrier before a stage is read; ds_tr_wait before the fragments are used,
// which ties their registers so no MFMA is scheduled above it).
__device__ __forceinline__ s16x4 ds_tr_asm(const bf16* p) {
  s16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int TM, int TN>
__device__ __forceinline__ void ds_tr_wait(bf16x8 (&a)[TM], bf16x8 (&b)[TN]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(b[j]));
}

template <int BM, int BN, int TAPS>
__global__ void __launch_bounds__(256, 2)
conv_wgrad_k(const bf16* __restrict__ dY, const bf16* __restrict__ I, float* __restrict__ ws, int Nimg, int IH,
             int IW, int IC, int OH, int OW, int OC, int stride, int pix_per_split, int ncb,
             float* __restrict__ bws, int lw, int lh) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ALD = WBK * BM / 8 / 256, BLD = WBK * BN / 8 / 256;
  constexpr int AS = BM + WPAD, BSt = BN + WPAD;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * WBK * (AS + BSt)];
  bf16* As = smem;
  bf16* Bs = smem + 2 * WBK * AS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware remap of the linear block id: the hardware deals consecutive
  // ids round-robin over the 8 XCDs; remapped, all (tap, ci-block) columns of
  // one (co-tile, split) run on ONE XCD, so its dY slab and the shifted input
  // rows are fetched into that XCD's L2 once instead of by every XCD.
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long T = (long)gx * gy * gridDim.z;
    const long L = blockIdx.x + (long)gx * (blockIdx.y + (long)gy * blockIdx.z);
    const long q = T / 8, r = T % 8, xcd = L % 8;
    const long R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    bx = (int)(R % gx);
    by = (int)((R / gx) % gy);
    bz = (int)(R / ((long)gx * gy));
  }
  const int tap = bx / ncb;                         // 0 when TAPS == 1
  const int ci0 = (bx % ncb) * BN;
  const int m0 = by * BM;
  const int split = bz;
  const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
  const long P = (long)Nimg * OH * OW;
  const long p_begin = (long)split * pix_per_split;
  const long p_end = p_begin + pix_per_split < P ? p_begin + pix_per_split : P;
  const int OHW = OH * OW;
  const bf16x8 zero8 = {};
  constexpr int ACH = BM / 8, BCH = BN / 8;   // 16B chunks per row

  bf16x8 ra[ALD], rb[BLD];
  auto gload = [&](long p0) {
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      int idx = tid + i * 256;
      int r = idx / ACH, c = (idx % ACH) * 8;
      long p = p0 + r;
      bool ok = p < p_end && m0 + c < OC;
      ra[i] = ok ? *reinterpret_cast<const bf16x8*>(dY + p * OC + m0 + c) : zero8;
    }
#pragma unroll
    for (int i = 0; i < BLD; ++i) {
      int idx = tid + i * 256;
      int r = idx / BCH, c = (idx % BCH) * 8;
      long p = p0 + r;
      bool ok = p < p_end && ci0 + c < IC;
      int img = 0, oh = 0, ow = 0;
      if (ok) {
        if (lw >= 0) {                 // power-of-two spatial dims: shifts, no division
          ow = (int)(p & (OW - 1));
          long t = p >> lw;
          oh = (int)(t & (OH - 1));
          img = (int)(t >> lh);
        } else {
          img = (int)(p / OHW);
          int rem = (int)(p % OHW);
          oh = rem / OW;
          ow = rem % OW;
        }
      }
      int ih = oh * stride + kh - 1, iw = ow * stride + kw - 1;
      ok = ok && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
      rb[i] = ok ? *reinterpret_cast<const bf16x8*>(I + (((long)img * IH + ih) * IW + iw) * IC + ci0 + c) : zero8;
    }
  };
  auto swrite = [&](int buf) {
    bf16* a = As + buf * WBK * AS;
    bf16* b = Bs + buf * WBK * BSt;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      int idx = tid + i * 256;
      *reinterpret_cast<bf16x8*>(a + (idx / ACH) * AS + (idx % ACH) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BLD; ++i) {
      int idx = tid + i * 256;
      *reinterpret_cast<bf16x8*>(b + (idx / BCH) * BSt + (idx % BCH) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment addressing for ds_read_b64_tr_b16 (see header): group g = lane>>4,
  // in-group lane i = 4q+p -> rows {4g+q, 16+4g+q}, columns 4p..4p+3.
  const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
  const int r1 = 4 * g + q, r2 = 16 + 4 * g + q;
  const long nsteps = (p_end - p_begin + WBK - 1) / WBK;
  if (nsteps > 0) {
    gload(p_begin);
    swrite(0);
  }
  __syncthreads();
  // fused bias gradient: the first (tap, ci) block column of every split also
  // sums its dY tile over pixels (thread -> column tid%BM, rows half tid/BM)
  const bool do_bias = bws != nullptr && bx == 0;
  float bacc = 0.f;
  for (long s = 0; s < nsteps; ++s) {
    const int buf = (int)(s & 1);
    if (s + 1 < nsteps) gload(p_begin + (s + 1) * WBK);
    const bf16* a = As + buf * WBK * AS;
    const bf16* b = Bs + buf * WBK * BSt;
    if (do_bias) {
      const int col = tid % BM, r0 = (tid / BM) * (WBK * BM / 256);
#pragma unroll
      for (int r = 0; r < WBK * BM / 256; ++r) bacc += (float)a[(r0 + r) * AS + col];
    }
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int col = wm * WM + i * 16 + 4 * pc;
      s16x4 lo = ds_tr(a + r1 * AS + col);
      s16x4 hi = ds_tr(a + r2 * AS + col);
      s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = wn * WN + j * 16 + 4 * pc;
      s16x4 lo = ds_tr(b + r1 * BSt + col);
      s16x4 hi = ds_tr(b + r2 * BSt + col);
      s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bfr[j] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (s + 1 < nsteps) swrite(buf ^ 1);
    __syncthreads();
  }
  if (do_bias) {
    const int col = tid % BM, half = tid / BM;
    if (m0 + col < OC) bws[((long)split * (256 / BM) + half) * OC + m0 + col] = bacc;
  }
  // partial slab: ws[split][co][tap*IC + ci]
  const int fr = lane & 15, fq = lane >> 4;
  const long KW = (long)TAPS * IC;
  float* slab = ws + (long)split * OC * KW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int ci = ci0 + wn * WN + j * 16 + fr;
    if (ci >= IC) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < OC) slab[(long)(co + e) * KW + tap * IC + ci] = acc[i][j][e];
    }
  }
}

// glds weight-gradient kernel: same GEMM and split-K as conv_wgrad_k, but
// both operand tiles arrive global -> LDS by DMA (global_load_lds_dwordx4,
// no VGPR staging, no ds_write pass), 64 pixels per stage, 2 stages behind a
// counted vmcnt + raw s_barrier.  The LDS image is unpadded ([pixel][128 ch],
// 256-B rows, lane-linear per 1-KiB DMA piece); bank conflicts of the
// transpose reads are removed by an XOR swizzle instead of padding: logical
// 16-B chunk c of row r lives at physical chunk c ^ 2*(r & 7) (the swizzle is
// applied to the per-lane SOURCE address, rows 8 apart cover all 64 banks).
template <int TAPS, int PK, int NS>
__global__ void __launch_bounds__(256, 2)
conv_wgrad_glds_k(const bf16* __restrict__ dY, const bf16* __restrict__ I, float* __restrict__ ws,
                  const bf16* __restrict__ zero16, int Nimg, int IH, int IW, int IC, int OH, int OW, int OC,
                  int stride, int pix_per_split, int ncb, float* __restrict__ bws, int lw, int lh) {
  constexpr int BM = 128, BN = 128;
  constexpr int WM = 64, WN = 64, TM = 4, TN = 4;
  constexpr int STAGE = PK * (BM + BN);
  constexpr int PPW = PK / 16;                  // 1-KiB DMA pieces per wave per operand per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * STAGE];
  typedef __attribute__((address_space(3))) void lds_void;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long T = (long)gx * gy * gridDim.z;
    const long L = blockIdx.x + (long)gx * (blockIdx.y + (long)gy * blockIdx.z);
    const long q = T / 8, r = T % 8, xcd = L % 8;
    const long R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    bx = (int)(R % gx);
    by = (int)((R / gx) % gy);
    bz = (int)(R / ((long)gx * gy));
  }
  const int tap = bx / ncb;
  const int ci0 = (bx % ncb) * BN;
  const int m0 = by * BM;
  const int split = bz;
  const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
  const long P = (long)Nimg * OH * OW;
  const long p_begin = (long)split * pix_per_split;
  const long p_end = p_begin + pix_per_split < P ? p_begin + pix_per_split : P;
  const int OHW = OH * OW;

  // DMA lane mapping: wave w, piece i covers tile rows (w*PPW+i)*4 .. +3;
  // lane L -> row +L/16, physical chunk L%16, logical chunk (L%16)^(2*(row&7))
  const int lrow = lane >> 4, pch = lane & 15;
  int trow[PPW], lch[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    trow[i] = (wave * PPW + i) * 4 + lrow;
    lch[i] = pch ^ (2 * (trow[i] & 7));
  }
  auto issue = [&](long p0, int stage) {
    bf16* sA = smem + stage * STAGE;
    bf16* sB = sA + PK * BM;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const long p = p0 + trow[i];
      const int co = m0 + lch[i] * 8;
      const bf16* src = (p < p_end && co < OC) ? dY + p * OC + co : zero16;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sA + (wave * PPW + i) * 4 * BM), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const long p = p0 + trow[i];
      const int ci = ci0 + lch[i] * 8;
      bool ok = p < p_end && ci < IC;
      int img = 0, oh = 0, ow = 0;
      if (lw >= 0) {
        ow = (int)(p & (OW - 1));
        long t = p >> lw;
        oh = (int)(t & (OH - 1));
        img = (int)(t >> lh);
      } else {
        img = (int)(p / OHW);
        int rem = (int)(p - (long)img * OHW);
        oh = rem / OW;
        ow = rem - oh * OW;
      }
      const int ih = oh * stride + kh - 1, iw = ow * stride + kw - 1;
      ok = ok && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
      const bf16* src = ok ? I + (((long)img * IH + ih) * IW + iw) * IC + ci : zero16;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sB + (wave * PPW + i) * 4 * BN), 16, 0, 0);
    }
  };
  auto sw = [](int row, int col) { return row * 128 + ((((col >> 3) ^ (2 * (row & 7)))) << 3) + (col & 7); };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
  const long nsteps = (p_end - p_begin + PK - 1) / PK;
  const bool do_bias = bws != nullptr && bx == 0;
  float bacc = 0.f;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (k < nsteps) issue(p_begin + k * PK, k);
  for (long s = 0; s < nsteps; ++s) {
    const int st = (int)(s % NS);
    // retire stage s; the (up to NS-2) stages issued after it stay in flight
    if (NS == 3 && s + 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // stage s visible; stage s-1 fully read by every wave
    if (s + NS - 1 < nsteps) issue(p_begin + (s + NS - 1) * PK, (int)((s + NS - 1) % NS));
    const bf16* a = smem + st * STAGE;
    const bf16* b = a + PK * BM;
    if (do_bias) {
      const int col = tid & 127, r0 = (tid >> 7) * (PK / 2);
#pragma unroll 8
      for (int r = 0; r < PK / 2; ++r) bacc += (float)a[sw(r0 + r, col)];
    }
#pragma unroll
    for (int kk = 0; kk < PK / 32; ++kk) {
      const int r1 = kk * 32 + 4 * g + q, r2 = r1 + 16;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * WM + i * 16 + 4 * pc;
        s16x4 lo = ds_tr(a + sw(r1, col));
        s16x4 hi = ds_tr(a + sw(r2, col));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 16 + 4 * pc;
        s16x4 lo = ds_tr(b + sw(r1, col));
        s16x4 hi = ds_tr(b + sw(r2, col));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads retired before the next top barrier
  }
  if (do_bias) {
    const int col = tid & 127, half = tid >> 7;
    if (m0 + col < OC) bws[((long)split * 2 + half) * OC + m0 + col] = bacc;
  }
  const int fr = lane & 15, fq = lane >> 4;
  const long KW = (long)TAPS * IC;
  float* slab = ws + (long)split * OC * KW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int ci = ci0 + wn * WN + j * 16 + fr;
    if (ci >= IC) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < OC) slab[(long)(co + e) * KW + tap * IC + ci] = acc[i][j][e];
    }
  }
}

// Buffer descriptor whose inputs are forced wave-uniform (readfirstlane):
// hipcc cannot always prove uniformity of values derived through loops and
// would otherwise wrap every buffer op in a waterfall loop (guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes > 0 ? (bytes < 0x7fffffffL ? bytes : 0x7fffffffL) : 0));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, n, 0x00020000);
}

// LDS-DMA issue of one wgrad stage (a __device__ function rather than a
// lambda: buffer-resource values must not appear in host-visible code).
template <int PK, int PPW, bool FAST, bool PAIR>
__device__ __forceinline__ void wgrad_bufl_issue(bf16* sA, bf16* sB, const bf16* __restrict__ dY,
                                                 const bf16* __restrict__ I, long in_elems, long p0, long p_end,
                                                 int OC, int IC, int IH, int IW, int OH, int OW, int OHW, int stride,
                                                 int kh, int kw, int dpix, int lw, int lh, int wave,
                                                 const int* trow, const unsigned* aoff, const unsigned* boff,
                                                 const bool* bok, const int* khl, const int* kwl) {
  typedef __attribute__((address_space(3))) void lds_void;
  constexpr int BM = 128, BN = 128;
  const __amdgpu_buffer_rsrc_t rA = uniform_rsrc(dY + p0 * OC, (p_end - p0) * OC * 2);
#pragma unroll
  for (int i = 0; i < PPW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sA + (wave * PPW + i) * 4 * BM), 16, aoff[i], 0, 0, 0);
  if (FAST) {
    // base may lie before the tensor (pb < 0: only masked top-padding rows
    // see it) or, on the last stages, past its end: the record count is
    // clamped at 0 so nothing beyond the tensor is ever read.  Base halves
    // go through readfirstlane so the descriptor is provably wave-uniform
    // (otherwise hipcc wraps every load in a waterfall loop).
    const long pb = p0 + dpix;
    const __amdgpu_buffer_rsrc_t rB = uniform_rsrc(I + pb * IC, (in_elems - pb * IC) * 2);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      bool ok = bok[i];
      const int pp = (int)p0 + trow[i];            // kh / kw are wave-uniform: at most two tests
      if (kw != 1) {
        const int ow = pp & (OW - 1);
        ok = ok && (kw == 0 ? ow != 0 : ow != OW - 1);
      }
      if (kh != 1) {
        const int oh = (pp >> lw) & (OH - 1);
        ok = ok && (kh == 0 ? oh != 0 : oh != OH - 1);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(sB + (wave * PPW + i) * 4 * BN), 16,
                                               ok ? boff[i] : 0x80000000u, 0, 0, 0);
    }
  } else {
    const __amdgpu_buffer_rsrc_t rB = uniform_rsrc(I, in_elems * 2);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const long p = p0 + trow[i];
      int img, oh, ow;
      if (lw >= 0) {
        ow = (int)(p & (OW - 1));
        const long t = p >> lw;
        oh = (int)(t & (OH - 1));
        img = (int)(t >> lh);
      } else {
        img = (int)(p / OHW);
        const int rr = (int)(p - (long)img * OHW);
        oh = rr / OW;
        ow = rr - oh * OW;
      }
      const int ih = oh * stride + (PAIR ? khl[i] : kh) - 1, iw = ow * stride + (PAIR ? kwl[i] : kw) - 1;
      const bool ok = bok[i] && ih >= 0 && ih < IH && iw >= 0 && iw < IW;
      const unsigned vo = (unsigned)((((img * IH + ih) * IW + iw) * IC) * 2) + (boff[i] - (unsigned)(trow[i] * IC * 2));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(sB + (wave * PPW + i) * 4 * BN), 16,
                                               ok ? vo : 0x80000000u, 0, 0, 0);
    }
  }
}

// Buffer-descriptor LDS-DMA weight-gradient kernel.  Same GEMM, split-K,
// swizzled unpadded LDS image and transpose reads as conv_wgrad_glds_k, with
// the VALU-issue bottleneck of the flat-address loaders removed:
//  * operand descriptors are re-based per stage with scalar math (the pixel
//    window advances by PK), so per-lane offsets are loop-invariant;
//  * the dY descriptor's record count ends at this split's last pixel and
//    the input descriptor's at the tensor end: rows past the range read as
//    zero from the hardware range check (no compare / select);
//  * FAST (stride 1, power-of-two H and W): the input row is the output row
//    shifted by a wave-uniform pixel offset, so the only per-stage lane work
//    is the padding test of the (uniform) tap: at most two mask compares;
//  * transpose-read lane offsets are precomputed and the two LDS stages are
//    unrolled so stage bases fold into instruction immediates.
// PAIR (64-channel inputs, the 51 -> 64 ray-direction half of the
// conditioning convs): the 128-channel B tile holds TWO taps x 64 channels
// instead of one tap with half the tile zero; slab columns tap * 64 + c of
// consecutive taps are contiguous, so the pair writes columns tap0 * 64 + [0,128).
template <int TAPS, int PK, bool FAST, bool PAIR = false>
__global__ void __launch_bounds__(256, 2)
conv_wgrad_bufl_k(const bf16* __restrict__ dY, const bf16* __restrict__ I0, float* __restrict__ ws, long in_pix,
                  int Nimg, int IH, int IW, int ICt, int OH, int OW, int OC, int stride, int pix_per_split, int ncb,
                  float* __restrict__ bws, int lw, int lh, const bf16* __restrict__ I2, int C1) {
  constexpr int BM = 128, BN = 128, NS = 2;
  constexpr int WM = 64, WN = 64, TM = 4, TN = 4;
  constexpr int STAGE = PK * (BM + BN);
  constexpr int PPW = PK / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * STAGE];
  typedef __attribute__((address_space(3))) void lds_void;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long T = (long)gx * gy * gridDim.z;
    const long L = blockIdx.x + (long)gx * (blockIdx.y + (long)gy * blockIdx.z);
    const long q = T / 8, r = T % 8, xcd = L % 8;
    const long R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    bx = (int)(R % gx);
    by = (int)((R / gx) % gy);
    bz = (int)(R / ((long)gx * gy));
  }
  const int tap = PAIR ? 2 * bx : bx / ncb;        // PAIR: first tap of the pair
  const int ci0g = PAIR ? 0 : (bx % ncb) * BN;     // channel tile in the (possibly concatenated) input
  const int m0 = by * BM;
  const int split = bz;
  const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
  const long P = (long)Nimg * OH * OW;
  const long p_begin = (long)split * pix_per_split;
  const long p_end = p_begin + pix_per_split < P ? p_begin + pix_per_split : P;
  const int OHW = OH * OW;
  const int dpix = (kh - 1) * IW + (kw - 1);       // FAST: input pixel = output pixel + dpix
  // virtual channel concat [I0 | I2] (decoder skip concat): a 128-channel
  // tile lies in one source (C1 % 128 == 0), chosen per block
  const bool second = I2 != nullptr && ci0g >= C1;
  const bf16* I = second ? I2 : I0;
  const int IC = I2 == nullptr ? ICt : (second ? ICt - C1 : C1);
  const int ci0 = second ? ci0g - C1 : ci0g;
  const long in_elems = in_pix * IC;

  const int lrow = lane >> 4, pch = lane & 15;
  int trow[PPW], khl[PPW], kwl[PPW];
  unsigned aoff[PPW], boff[PPW];
  bool bok[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    trow[i] = (wave * PPW + i) * 4 + lrow;
    const int lc = pch ^ (2 * (trow[i] & 7));
    const int co = m0 + lc * 8;
    aoff[i] = co < OC ? (unsigned)((trow[i] * OC + co) * 2) : 0x80000000u;
    if (PAIR) {                                    // chunks 0-7: tap, 8-15: tap + 1
      const int tl = tap + (lc >> 3), ci = (lc & 7) * 8;
      boff[i] = (unsigned)((trow[i] * IC + ci) * 2);
      bok[i] = tl < TAPS;
      khl[i] = tl / 3;
      kwl[i] = tl % 3;
    } else {
      const int ci = ci0 + lc * 8;
      boff[i] = (unsigned)((trow[i] * IC + ci) * 2);
      bok[i] = ci < IC;
      khl[i] = kwl[i] = 0;
    }
  }
  // transpose-read lane offsets (elements): row (4g+q) + swizzled column chunk
  const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
  const int x7 = 2 * ((4 * g + q) & 7);
  int la[TM], lb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) la[i] = (4 * g + q) * 128 + ((((wm * 8 + 2 * i + (pc >> 1)) ^ x7)) << 3) + (pc & 1) * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j) lb[j] = (4 * g + q) * 128 + ((((wn * 8 + 2 * j + (pc >> 1)) ^ x7)) << 3) + (pc & 1) * 4;

  auto issue = [&](long p0, int stage) {
    bf16* sA = smem + stage * STAGE;
    wgrad_bufl_issue<PK, PPW, FAST, PAIR>(sA, sA + PK * BM, dY, I, in_elems, p0, p_end, OC, IC, IH, IW, OH, OW, OHW,
                                          stride, kh, kw, dpix, lw, lh, wave, trow, aoff, boff, bok, khl, kwl);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long nsteps = (p_end - p_begin + PK - 1) / PK;
  const bool do_bias = bws != nullptr && bx == 0;
  float bacc = 0.f;
  // bias: thread -> column tid&127, rows half*(PK/2) .. +PK/2 (swizzled reads)
  const int bcol = tid & 127, bhalf = tid >> 7;
  // FAST (stride-1, power-of-two images: every large layer): the issue-then-
  // compute order below, in which the compiler waits for the next stage's DMA
  // before reading this one -- the two co-resident blocks per CU cover each
  // other's waits, and in-graph A/B (profiles/ab_wgrad_order_r2.txt) had it
  // 1.3-1.6x faster than reads-first ordering on these shapes.  Strided /
  // generic addressing: reads-first (-10..15 % on the conditioning convs).
  if constexpr (FAST) {
    auto compute = [&](const bf16* a) {
      const bf16* b = a + PK * BM;
      if (do_bias) {
  #pragma unroll
        for (int r = 0; r < PK / 2; ++r) {
          const int row = bhalf * (PK / 2) + r;
          bacc += (float)a[row * 128 + ((((bcol >> 3) ^ (2 * (row & 7)))) << 3) + (bcol & 7)];
        }
      }
  #pragma unroll
      for (int kk = 0; kk < PK / 32; ++kk) {
        bf16x8 af[TM], bfr[TN];
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          s16x4 lo = ds_tr(a + la[i] + kk * 32 * 128);
          s16x4 hi = ds_tr(a + la[i] + kk * 32 * 128 + 16 * 128);
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, v);
        }
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          s16x4 lo = ds_tr(b + lb[j] + kk * 32 * 128);
          s16x4 hi = ds_tr(b + lb[j] + kk * 32 * 128 + 16 * 128);
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, v);
        }
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    // one barrier per step: wait for this step's DMA, barrier (every wave's
    // DMA landed AND every wave done reading the other slot), issue the next
    // step into the other slot, compute.
    if (nsteps > 0) issue(p_begin, 0);
    for (long s = 0; s < nsteps; ++s) {
      const int st = (int)(s & 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (s + 1 < nsteps) issue(p_begin + (s + 1) * PK, st ^ 1);
      compute(smem + st * STAGE);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else {
    // Per stage: read EVERY fragment of the stage, THEN issue the next stage's
    // LDS-DMA, then run the MFMAs.  With the DMA issued after the reads, the
    // compiler's wait-count pass sees no LDS-DMA in flight at any LDS read (the
    // stage's own DMA is retired by the s_waitcnt builtin below, which the pass
    // accounts for, unlike inline asm), so it inserts no "vmcnt(0)" that would
    // wait for the NEXT stage; the DMA of stage s+1 overlaps stage s's MFMAs
    // while the compiler keeps its fine-grained read / MFMA interleave.
    constexpr int KK = PK / 32;
    auto frags = [&](const bf16* a, bf16x8 (&af)[KK][TM], bf16x8 (&bfr)[KK][TN]) {
      const bf16* b = a + PK * BM;
      if (do_bias) {
  #pragma unroll
        for (int r = 0; r < PK / 2; ++r) {
          const int row = bhalf * (PK / 2) + r;
          bacc += (float)a[row * 128 + ((((bcol >> 3) ^ (2 * (row & 7)))) << 3) + (bcol & 7)];
        }
      }
  #pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          s16x4 lo = ds_tr(a + la[i] + kk * 32 * 128);
          s16x4 hi = ds_tr(a + la[i] + kk * 32 * 128 + 16 * 128);
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[kk][i] = __builtin_bit_cast(bf16x8, v);
        }
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          s16x4 lo = ds_tr(b + lb[j] + kk * 32 * 128);
          s16x4 hi = ds_tr(b + lb[j] + kk * 32 * 128 + 16 * 128);
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[kk][j] = __builtin_bit_cast(bf16x8, v);
        }
      }
    };
    if (nsteps > 0) issue(p_begin, 0);
    for (long s = 0; s < nsteps; ++s) {
      const int st = (int)(s & 1);
      __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0): this stage landed
      __builtin_amdgcn_s_barrier();                    // ... everywhere; the other slot is free
      bf16x8 af[KK][TM], bfr[KK][TN];
      frags(smem + st * STAGE, af, bfr);
      if (s + 1 < nsteps) issue(p_begin + (s + 1) * PK, st ^ 1);
  #pragma unroll
      for (int kk = 0; kk < KK; ++kk)
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    }
  }
  if (do_bias) {
    if (m0 + bcol < OC) bws[((long)split * 2 + bhalf) * OC + m0 + bcol] = bacc;
  }
  const int fr = lane & 15, fq = lane >> 4;
  const long KW = (long)TAPS * ICt;
  float* slab = ws + (long)split * OC * KW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = ci0 + wn * WN + j * 16 + fr;   // channel within the source (PAIR: within the tap pair)
    if (PAIR ? tap * IC + cl >= TAPS * IC : cl >= IC) continue;
    const int ci = ci0g - ci0 + cl;                 // channel within the concatenation
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < OC) slab[(long)(co + e) * KW + tap * ICt + ci] = acc[i][j][e];
    }
  }
}

// ------------------------------------------------ 8-wave weight gradient --
// conv_wgrad_bufl_k at one 512-thread block per CU with a BM (output
// channels) x BN (input channels of one tap) tile and 64-pixel stages.  The
// 128x128 / 32-pixel kernel measured 52-59 % of wave cycles parked on
// vmcnt / barrier (profiles/pmc_wgrad): a stage is only 16 MFMA per wave, far
// shorter than an LDS-DMA round trip.  Here a stage is 64 (BM=256: 128x64
// wave tiles) or 32 MFMA per wave at 2 waves per SIMD, so one stage in flight
// behind the barrier covers the landing latency.  FAST addressing only
// (stride 1, power-of-two H = W, same in/out size): the input rows of a tap
// are the output rows shifted by a wave-uniform pixel offset.
//
// LDS image per stage: [64 pixels][BM] dY and [64 pixels][BN] input, rows of
// W bf16 (W = BM or BN, 256 or 128).  16-B chunk c of row r lives at
// physical chunk (c & ~15) | ((c & 15) ^ 2 * (r & 7)): the 128-wide kernel's
// conflict-free swizzle applied inside each 256-B half of a row (banks repeat
// every 256 B).  The swizzle is in the per-lane DMA source address.
template <int W>
__device__ __forceinline__ int w8w_phys(int c, int r) { return (c & ~15) | ((c & 15) ^ (2 * (r & 7))); }

template <int BM, int BN>
__device__ __forceinline__ void wgrad_w8_issue(bf16* sA, bf16* sB, const bf16* __restrict__ dY,
                                               const bf16* __restrict__ I, long in_elems, long p0, long p_end,
                                               int OC, int IC, int IH, int OH, int OW, int kh, int kw, int dpix,
                                               int lw, int wave, const int* arow, const unsigned* aoff,
                                               const int* brow, const unsigned* boff) {
  typedef __attribute__((address_space(3))) void lds_void;
  constexpr int PK = 64;
  constexpr int APW = PK * BM * 2 / 1024 / 8, BPW = PK * BN * 2 / 1024 / 8;   // 1-KiB pieces per wave
  const __amdgpu_buffer_rsrc_t rA = uniform_rsrc(dY + p0 * OC, (p_end - p0) * OC * 2);
#pragma unroll
  for (int i = 0; i < APW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sA + (wave * APW + i) * 512), 16, aoff[i], 0, 0, 0);
  const long pb = p0 + dpix;
  const __amdgpu_buffer_rsrc_t rB = uniform_rsrc(I + pb * IC, (in_elems - pb * IC) * 2);
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int pp = (int)p0 + brow[i];
    unsigned bad = 0u;                               // tap padding: at most two wave-uniform tests
    if (kw != 1) {
      const int ow = pp & (OW - 1);
      bad |= (unsigned)(kw == 0 ? ow == 0 : ow == OW - 1);
    }
    if (kh != 1) {
      const int oh = (pp >> lw) & (OH - 1);
      bad |= (unsigned)(kh == 0 ? oh == 0 : oh == OH - 1);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(sB + (wave * BPW + i) * 512), 16,
                                             boff[i] | (bad << 31), 0, 0, 0);
  }
}

// TAPS = 1: per-pixel dense weight gradient dY^T X over P rows (the level-
// batched FiLM projections, attention projections, NIN skips); no padding
// tests, any row count.
template <int BM, int BN, int TAPS = 9>
__global__ void __launch_bounds__(512, 1)
conv_wgrad_w8_k(const bf16* __restrict__ dY, const bf16* __restrict__ I, float* __restrict__ ws, long in_pix,
                int Nimg, int IH, int IW, int IC, int OH, int OW, int OC, int pix_per_split, int ncb,
                float* __restrict__ bws, int lw, int lh) {
  constexpr int PK = 64, NS = 2;
  constexpr int WM = BM / 2, WN = BN / 4, TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = PK * (BM + BN);
  constexpr int APW = PK * BM * 2 / 1024 / 8, BPW = PK * BN * 2 / 1024 / 8;
  constexpr int ARP = 1024 / (BM * 2), BRP = 1024 / (BN * 2);          // rows per 1-KiB piece
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long T = (long)gx * gy * gridDim.z;
    const long L = blockIdx.x + (long)gx * (blockIdx.y + (long)gy * blockIdx.z);
    const long q = T / 8, r = T % 8, xcd = L % 8;
    const long R = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    bx = (int)(R % gx);
    by = (int)((R / gx) % gy);
    bz = (int)(R / ((long)gx * gy));
  }
  const int tap = TAPS == 9 ? bx / ncb : 0;
  const int ci0 = (bx % ncb) * BN;
  const int m0 = by * BM;
  const int split = bz;
  const int kh = TAPS == 9 ? tap / 3 : 1, kw = TAPS == 9 ? tap % 3 : 1;
  const long P = (long)Nimg * OH * OW;
  const long p_begin = (long)split * pix_per_split;
  const long p_end = p_begin + pix_per_split < P ? p_begin + pix_per_split : P;
  const int dpix = (kh - 1) * IW + (kw - 1);
  const long in_elems = in_pix * IC;

  // DMA lane mapping: lane L -> row L / (W/8) of its piece, physical chunk
  // L % (W/8), logical chunk w8w_phys(physical, row) (the XOR is an involution)
  int arow[APW], brow[BPW];
  unsigned aoff[APW], boff[BPW];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    arow[i] = (wave * APW + i) * ARP + lane / (BM / 8);
    const int lc = w8w_phys<BM>(lane % (BM / 8), arow[i]);
    const int co = m0 + lc * 8;
    aoff[i] = co < OC ? (unsigned)((arow[i] * OC + co) * 2) : 0x80000000u;
  }
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    brow[i] = (wave * BPW + i) * BRP + lane / (BN / 8);
    const int lc = w8w_phys<BN>(lane % (BN / 8), brow[i]);
    const int ci = ci0 + lc * 8;
    boff[i] = ci < IC ? (unsigned)((brow[i] * IC + ci) * 2) : 0x80000000u;
  }
  // transpose-read lane offsets (elements) for rows 4g+q (+16, +32, +48)
  const int g = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3;
  const int rr = 4 * g + q;
  int la[TM], lb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) la[i] = rr * BM + (w8w_phys<BM>((wm * WM + i * 16) / 8 + (pc >> 1), rr) << 3) + (pc & 1) * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j) lb[j] = rr * BN + (w8w_phys<BN>((wn * WN + j * 16) / 8 + (pc >> 1), rr) << 3) + (pc & 1) * 4;

  auto issue = [&](long p0, int stage) {
    bf16* sA = smem + stage * STAGE;
    wgrad_w8_issue<BM, BN>(sA, sA + PK * BM, dY, I, in_elems, p0, p_end, OC, IC, IH, OH, OW, kh, kw, dpix, lw, wave,
                           arow, aoff, brow, boff);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long nsteps = (p_end - p_begin + PK - 1) / PK;
  // fused bias: the first (tap, ci) column block of every split sums its dY
  // tile; thread -> column tid % BM, half (tid / BM) & 1 of the stage's rows
  const bool do_bias = bws != nullptr && bx == 0 && tid < 2 * BM;
  float bacc = 0.f;
  const int bcol = tid % BM, bhalf = (tid / BM) & 1;
  auto compute = [&](const bf16* a) {
    const bf16* b = a + PK * BM;
    if (do_bias) {
#pragma unroll 8
      for (int r = 0; r < PK / 2; ++r) {
        const int row = bhalf * (PK / 2) + r;
        bacc += (float)a[row * BM + (w8w_phys<BM>(bcol >> 3, row) << 3) + (bcol & 7)];
      }
    }
#pragma unroll
    for (int kk = 0; kk < PK / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        s16x4 lo = ds_tr_asm(b + lb[j] + kk * 32 * BN);
        s16x4 hi = ds_tr_asm(b + lb[j] + kk * 32 * BN + 16 * BN);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        s16x4 lo = ds_tr_asm(a + la[i] + kk * 32 * BM);
        s16x4 hi = ds_tr_asm(a + la[i] + kk * 32 * BM + 16 * BM);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
      ds_tr_wait<TM, TN>(af, bfr);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // one barrier per stage: wait for this stage's DMA, barrier (landed
  // everywhere AND every wave done reading the other buffer), issue the next
  // stage into it, compute at raised MFMA priority
  if (nsteps > 0) issue(p_begin, 0);
  for (long s = 0; s < nsteps; ++s) {
    const int st = (int)(s & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nsteps) issue(p_begin + (s + 1) * PK, st ^ 1);
    __builtin_amdgcn_s_setprio(1);
    compute(smem + st * STAGE);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (do_bias && m0 + bcol < OC) bws[((long)split * 2 + bhalf) * OC + m0 + bcol] = bacc;
  const int fr = lane & 15, fq = lane >> 4;
  const long KW = (long)TAPS * IC;
  float* slab = ws + (long)split * OC * KW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int ci = ci0 + wn * WN + j * 16 + fr;
    if (ci >= IC) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = m0 + wm * WM + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < OC) slab[(long)(co + e) * KW + tap * IC + ci] = acc[i][j][e];
    }
  }
}

// 3x3 split-K reduce with the [co][tap][ci] -> OIHW ([co][ci][tap])
// transposition staged in LDS: a block owns (co, 64 input channels), reads
// the 9 tap rows of every split coalesced (64 consecutive ci each) and writes
// (or accumulates into) 576 CONTIGUOUS floats of dW.  The element-wise
// reduce wrote OIHW 36 B apart (one read-modify-write per 4-B element): ~86
// us for a 2-split 512x512 weight, now bandwidth-bound.  Blocks past
// nblk_w sum the bias partials (brows rows) into db.
template <int TG>
__global__ void __launch_bounds__(256) wgrad_reduce9_k(const float* __restrict__ ws, int OC, int IC, int splits,
                                                       int accumulate, const float* __restrict__ bws, int brows,
                                                       float* __restrict__ dW, float* __restrict__ db, int nblk_w,
                                                       float scale) {
  // block = (co, 64 input channels, TG taps); 256 threads = 64 channels x 4
  // split lanes, each lane folding every 4th split of all TG taps at once
  // (TG x 2 independent loads in flight), lanes merged in fixed order
  // through LDS.  TG < 9 spreads the taps over more blocks when the grid
  // would otherwise be small (many splits over few weights: the 64x64-level
  // wgrad at 16 examples per GPU reduces 108 slabs).
  __shared__ float red[4][TG][64];
  __shared__ float tile[64 * TG];
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= nblk_w) {
    // bias: 64 channels x 4 row lanes x 8 independent accumulators (a single
    // dependent chain over the ~200 partial rows cost ~60 us per launch)
    const int c = ((int)blockIdx.x - nblk_w) * 64 + (tid & 63), ln = tid >> 6;
    float a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = 0.f;
    if (c < OC && db) {
      int k = ln;
      for (; k + 28 < brows; k += 32)
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] += bws[(long)(k + 4 * q) * OC + c];
      for (; k < brows; k += 4) a[0] += bws[(long)k * OC + c];
    }
    red[ln][0][tid & 63] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (ln == 0 && c < OC && db) {
      const float sv = (((red[0][0][tid] + red[1][0][tid]) + red[2][0][tid]) + red[3][0][tid]) * scale;
      db[c] = accumulate ? db[c] + sv : sv;
    }
    return;
  }
  constexpr int NTG = 9 / TG;
  const int ncg = (IC + 63) / 64;
  const int co = blockIdx.x / (ncg * NTG);
  const int rem = blockIdx.x % (ncg * NTG);
  const int ci0 = (rem / NTG) * 64, tap0 = (rem % NTG) * TG;
  const int nci = min(64, IC - ci0);
  const long total = (long)OC * 9 * IC;
  const int ci = tid & 63, ln = tid >> 6;
  constexpr int NC = TG == 1 ? 8 : (TG == 3 ? 4 : 2);     // independent chains per tap
  float a[TG][NC];
#pragma unroll
  for (int t = 0; t < TG; ++t)
#pragma unroll
    for (int c = 0; c < NC; ++c) a[t][c] = 0.f;
  if (ci < nci) {
    const float* src = ws + (long)co * 9 * IC + (long)tap0 * IC + ci0 + ci;
    int sp = ln;
    for (; sp + 4 * (NC - 1) < splits; sp += 4 * NC) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int c = 0; c < NC; ++c) a[t][c] += src[(long)(sp + 4 * c) * total + (long)t * IC];
    }
    for (int c = 0; sp < splits; sp += 4, ++c) {
#pragma unroll
      for (int t = 0; t < TG; ++t) a[t][0] += src[(long)sp * total + (long)t * IC];
    }
  }
#pragma unroll
  for (int t = 0; t < TG; ++t) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) v += a[t][c];
    red[ln][t][ci] = v;
  }
  __syncthreads();
  for (int k = tid; k < TG * 64; k += 256) {
    const int t = k >> 6, c = k & 63;
    tile[c * TG + t] = (((red[0][t][c] + red[1][t][c]) + red[2][t][c]) + red[3][t][c]) * scale;
  }
  __syncthreads();
  if (TG == 9) {                                 // 576 contiguous floats of OIHW
    float* dst = dW + ((long)co * IC + ci0) * 9;
    for (int m = tid; m < nci * 9; m += 256) dst[m] = accumulate ? dst[m] + tile[m] : tile[m];
  } else {
    for (int m = tid; m < nci * TG; m += 256) {
      const int c = m / TG, t = m - c * TG;
      float* d = dW + ((long)co * IC + ci0 + c) * 9 + tap0 + t;
      *d = accumulate ? *d + tile[m] : tile[m];
    }
  }
}

// sum the split slabs and write dW in OIHW fp32 layout (optionally accumulate)
__global__ void wgrad_reduce_k(const float* __restrict__ ws, float* __restrict__ dW, int OC, int IC, int splits,
                               int accumulate, int taps, const float* __restrict__ bws, float* __restrict__ db,
                               int brows) {
  long total = (long)OC * IC * taps;
  if (db) {
    for (long c = blockIdx.x * (long)blockDim.x + threadIdx.x; c < OC; c += (long)gridDim.x * blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < brows; ++k) s += bws[(long)k * OC + c];
      db[c] = accumulate ? db[c] + s : s;
    }
  }
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    // t indexes the slab layout [co][tap][ci] (coalesced reads)
    int ci = (int)(t % IC);
    long r = t / IC;
    int tap = (int)(r % taps);
    int co = (int)(r / taps);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int k = 0;
    for (; k + 4 <= splits; k += 4) {      // 4 independent loads in flight
      s0 += ws[(long)k * total + t];
      s1 += ws[(long)(k + 1) * total + t];
      s2 += ws[(long)(k + 2) * total + t];
      s3 += ws[(long)(k + 3) * total + t];
    }
    for (; k < splits; ++k) s0 += ws[(long)k * total + t];
    float s = (s0 + s1) + (s2 + s3);
    long o = ((long)co * IC + ci) * taps + tap;
    dW[o] = accumulate ? dW[o] + s : s;
  }
}

// Segmented variant: the OC rows of one GEMM belong to several parameters
// (a level-batched FiLM projection: OC = sum of 2C_i).  Row co of segment s
// lands in w[s] + (co - row0[s]) * IC * taps (+ bias in b[s]); the segment table
// travels as a kernel argument, so one launch scatters into every parameter's
// gradient view (no temporary dW, no per-parameter copies).
constexpr int kMaxSegs = 16;
struct WSegs {
  int n;
  int row0[kMaxSegs + 1];
  float* w[kMaxSegs];
  float* b[kMaxSegs];
};

__device__ __forceinline__ int seg_of(const WSegs& sg, int co) {
  int s = 0;
  while (s + 1 < sg.n && co >= sg.row0[s + 1]) ++s;
  return s;
}

__global__ void wgrad_reduce_seg_k(const float* __restrict__ ws, int OC, int IC, int splits, int accumulate,
                                   int taps, const float* __restrict__ bws, int brows, WSegs sg) {
  long total = (long)OC * IC * taps;
  if (bws) {
    for (long c = blockIdx.x * (long)blockDim.x + threadIdx.x; c < OC; c += (long)gridDim.x * blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < brows; ++k) s += bws[(long)k * OC + c];
      int g = seg_of(sg, (int)c);
      float* d = sg.b[g];
      if (d) {
        d += c - sg.row0[g];
        *d = accumulate ? *d + s : s;
      }
    }
  }
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    int ci = (int)(t % IC);
    long r = t / IC;
    int tap = (int)(r % taps);
    int co = (int)(r / taps);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int k = 0;
    for (; k + 4 <= splits; k += 4) {
      s0 += ws[(long)k * total + t];
      s1 += ws[(long)(k + 1) * total + t];
      s2 += ws[(long)(k + 2) * total + t];
      s3 += ws[(long)(k + 3) * total + t];
    }
    for (; k < splits; ++k) s0 += ws[(long)k * total + t];
    float s = (s0 + s1) + (s2 + s3);
    int g = seg_of(sg, co);
    float* d = sg.w[g] + (((long)(co - sg.row0[g]) * IC + ci) * taps + tap);
    *d = accumulate ? *d + s : s;
  }
}

// Split-K slab reduction, parallel over splits as well as outputs: a block
// owns 64 consecutive slab entries (16 float4 columns) and its 16 split lanes
// each sum every 16th split with coalesced 16-B loads; an LDS tree finishes
// the sum in a fixed order (deterministic).  Blocks past the dW range reduce
// the bias partials the same way.  Destination: dW/db (OIHW) or, when
// sg.n > 0, the per-parameter segments of a batched projection.
template <int SL>
__global__ void __launch_bounds__(256) wgrad_reduce2_k(const float* __restrict__ ws, int OC, int IC, int taps,
                                                       int splits, int accumulate, const float* __restrict__ bws,
                                                       int brows, float* __restrict__ dW, float* __restrict__ db,
                                                       WSegs sg, int nblk_w, float scale) {
  // 256 threads = COLS float4 columns x SL split lanes (SL = the split count
  // rounded up to a power of two, <= 16: few splits -> wide blocks)
  constexpr int COLS = 256 / SL;
  __shared__ f32x4 red[SL][COLS];
  const int col = threadIdx.x % COLS, sl = threadIdx.x / COLS;
  const bool is_bias = blockIdx.x >= nblk_w;
  const long total = is_bias ? (long)OC : (long)OC * IC * taps;
  const float* src = is_bias ? bws : ws;
  const int nrows = is_bias ? brows : splits;
  const long base = (long)(is_bias ? blockIdx.x - nblk_w : blockIdx.x) * (COLS * 4) + col * 4;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (base < total) {
    if (base + 3 < total) {
      f32x4 b2 = {0.f, 0.f, 0.f, 0.f};          // two chains: up to ~30 rows per lane for bias partials
      int k = sl;
      for (; k + SL < nrows; k += 2 * SL) {
        a += *reinterpret_cast<const f32x4*>(src + (long)k * total + base);
        b2 += *reinterpret_cast<const f32x4*>(src + (long)(k + SL) * total + base);
      }
      if (k < nrows) a += *reinterpret_cast<const f32x4*>(src + (long)k * total + base);
      a += b2;
    } else {
      for (int k = sl; k < nrows; k += SL)
        for (int e = 0; e < 4 && base + e < total; ++e) a[e] += src[(long)k * total + base + e];
    }
  }
  red[sl][col] = a;
  __syncthreads();
  if (sl == 0) {
    f32x4 t = red[0][col];
#pragma unroll
    for (int k = 1; k < SL; ++k) t += red[k][col];
    t *= scale;                                   // d(scale * dY) = scale * d(dY): no scaled dY copy
    for (int e = 0; e < 4; ++e) {
      const long o = base + e;
      if (o >= total) break;
      float* d;
      if (is_bias) {
        const int c = (int)o;
        if (sg.n > 0) {
          const int g = seg_of(sg, c);
          d = sg.b[g] ? sg.b[g] + (c - sg.row0[g]) : nullptr;
        } else {
          d = db ? db + c : nullptr;
        }
      } else {
        const int ci = (int)(o % IC);
        const long r = o / IC;
        const int tap = (int)(r % taps);
        const int co = (int)(r / taps);
        if (sg.n > 0) {
          const int g = seg_of(sg, co);
          d = sg.w[g] + (((long)(co - sg.row0[g]) * IC + ci) * taps + tap);
        } else {
          d = dW + (((long)co * IC + ci) * taps + tap);
        }
      }
      if (d) *d = accumulate ? *d + t[e] : t[e];
    }
  }
}

// per-image channel sums: block = 256 threads = 32 channel-vectors x 8 row lanes
__global__ void chansum_k(const bf16* __restrict__ dy, float* __restrict__ part, int P, int C, int nchunks) {
  const int img = blockIdx.y, chunk = blockIdx.z;
  const int cv = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rl = threadIdx.x >> 5;      // 0..7
  __shared__ float red[8][32][8];
  f32x8 s = {};
  const int CV = C / 8;
  if (cv < CV) {
    int rows = (P + nchunks - 1) / nchunks;
    int r0 = chunk * rows, r1 = min(P, r0 + rows);
    const bf16* src = dy + (long)img * P * C + cv * 8;
    f32x8 s1 = {}, s2 = {}, s3 = {};              // four independent chains of row loads
    int r = r0 + rl;
    for (; r + 24 < r1; r += 32) {
      s += ld8(src + (long)r * C);
      s1 += ld8(src + (long)(r + 8) * C);
      s2 += ld8(src + (long)(r + 16) * C);
      s3 += ld8(src + (long)(r + 24) * C);
    }
    for (; r < r1; r += 8) s += ld8(src + (long)r * C);
    s = (s + s1) + (s2 + s3);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][threadIdx.x & 31][e] = s[e];
  __syncthreads();
  if (rl == 0 && cv < CV) {
    for (int k = 1; k < 8; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += red[k][threadIdx.x & 31][e];
    float* o = part + ((long)chunk * gridDim.y + img) * C + cv * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = s[e];
  }
}

__global__ void chansum_img_k(const float* __restrict__ part, float* __restrict__ per_img, int Nimg, int C,
                              int nchunks) {
  long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t >= (long)Nimg * C) return;
  int n = (int)(t / C), c = (int)(t % C);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 3 < nchunks; k += 4) {
    s0 += part[((long)k * Nimg + n) * C + c];
    s1 += part[((long)(k + 1) * Nimg + n) * C + c];
    s2 += part[((long)(k + 2) * Nimg + n) * C + c];
    s3 += part[((long)(k + 3) * Nimg + n) * C + c];
  }
  for (; k < nchunks; ++k) s0 += part[((long)k * Nimg + n) * C + c];
  per_img[t] = (s0 + s1) + (s2 + s3);
}

// weight packing: OIHW fp32 -> [OCp][9][ICp] bf16 (forward) or
//                              [ICp][9][OCp] bf16 (transposed, for dgrad)
__global__ void pack_w_k(const float* __restrict__ w, bf16* __restrict__ out, int OC, int IC, int OCp, int ICp,
                         int trans, int taps) {
  long total = trans ? (long)ICp * taps * OCp : (long)OCp * taps * ICp;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    int co, ci, tap;
    if (!trans) {
      ci = (int)(t % ICp);
      long r = t / ICp;
      tap = (int)(r % taps);
      co = (int)(r / taps);
    } else {
      co = (int)(t % OCp);
      long r = t / OCp;
      tap = (int)(r % taps);
      ci = (int)(r / taps);
    }
    float v = (co < OC && ci < IC) ? w[((long)co * IC + ci) * taps + tap] : 0.f;
    out[t] = (bf16)v;
  }
}

// Batched weight refresh: one launch re-derives every cached bf16 operand
// (packed conv/linear weights and plain casts) from the fp32 masters after the
// optimizer step.  blockIdx.y selects the descriptor.
struct PackDesc {
  const float* src;
  bf16* dst;
  int OC, IC, OCp, ICp, taps, mode;     // mode 0: pack, 1: transposed pack, 2: cast (OC elements)
  int blk0;                             // first block of this descriptor in the flattened grid
  int ICs;                              // source IC stride (0: IC) -- channel slices of a weight
  int ldd;                              // mode 1: destination row stride (0: OCp) -- column block of a
                                        // concatenated transposed operand
  int pad_;                             // (host table rows are packed: keep the size a multiple of 8)
};
static_assert(sizeof(PackDesc) == 56, "PackDesc must match hip_impl._desc_tensors");

// One launch repacks every cached bf16 operand.  The grid is flattened over
// descriptors (host-built block -> descriptor map, sizes in hip_impl
// _pack_blocks).  The fp32 masters are OIHW ([OC][IC][taps]) while the
// operands put taps outside the channel axes, so each block stages a tile in
// LDS and reads AND writes it coalesced (element-wise index math here read
// the source 36 B apart and ran at ~1.4 TB/s):
//   mode 0 (fwd [OCp][taps][ICp]): one output row co x 256 input channels;
//   mode 1 (transposed [ICp][taps][OCp]): 32 output x 16 input channels;
//   mode 2 (plain cast): 2048 contiguous elements.
__global__ void __launch_bounds__(256) pack_all_k(const PackDesc* __restrict__ descs,
                                                  const int* __restrict__ blk_desc) {
  __shared__ float tile[32 * 16 * 9];          // 18 KiB: covers both tilings (8 blocks per CU)
  const PackDesc d = descs[blk_desc[blockIdx.x]];
  const int local = blockIdx.x - d.blk0, tid = threadIdx.x;
  const int ics = d.ICs ? d.ICs : d.IC;
  const int T = d.taps;
  if (d.mode == 2) {
    const int t0 = local * 2048 + tid * 8;
    if (t0 >= d.OC) return;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)(t0 + e < d.OC ? d.src[t0 + e] : 0.f);
    if (t0 + 7 < d.OC && ((reinterpret_cast<uintptr_t>(d.dst + t0) & 15) == 0))
      *reinterpret_cast<bf16x8*>(d.dst + t0) = o;
    else
      for (int e = 0; e < 8 && t0 + e < d.OC; ++e) d.dst[t0 + e] = o[e];
    return;
  }
  if (d.mode == 0) {
    const int ncg = (d.ICp + 255) / 256;
    const int co = local / ncg, ci0 = (local % ncg) * 256;
    const int nci = min(256, d.ICp - ci0);
    // src[co][ci0 .. ci0+255][0..T) is one contiguous run of 256*T floats
    for (int k = tid; k < 256 * T; k += 256) {
      const int ci = ci0 + k / T;
      tile[k] = (co < d.OC && ci < d.IC) ? d.src[((long)co * ics + ci) * T + k % T] : 0.f;
    }
    __syncthreads();
    for (int k = tid; k < T * (nci / 8); k += 256) {
      const int tap = k / (nci / 8), c8 = (k % (nci / 8)) * 8;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)tile[(c8 + e) * T + tap];
      *reinterpret_cast<bf16x8*>(d.dst + ((long)co * T + tap) * d.ICp + ci0 + c8) = o;
    }
    return;
  }
  // mode 1: 32 (co) x 16 (ci) x T tile; LDS [co][ci*T + tap]
  const int nct = (d.OCp + 31) / 32;
  const int co0 = (local % nct) * 32, ci0 = (local / nct) * 16;
  for (int k = tid; k < 32 * 16 * T; k += 256) {
    const int r = k / (16 * T), q = k % (16 * T);
    const int co = co0 + r, ci = ci0 + q / T;
    tile[k] = (co < d.OC && ci < d.IC) ? d.src[((long)co * ics + ci) * T + q % T] : 0.f;
  }
  __syncthreads();
  // dst[ci][tap][co0 .. co0+31]: 4 x 16-B stores per (ci, tap)
  for (int k = tid; k < 16 * T * 4; k += 256) {
    const int c8 = (k & 3) * 8, rt = k >> 2;
    const int ci = rt / T, tap = rt % T;
    if (ci0 + ci >= d.ICp || co0 + c8 >= d.OCp) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)tile[(c8 + e) * 16 * T + ci * T + tap];
    *reinterpret_cast<bf16x8*>(d.dst + ((long)(ci0 + ci) * T + tap) * (d.ldd ? d.ldd : d.OCp) + co0 + c8) = o;
  }
}

}  // namespace

// descs: n PackDesc; blk_desc: [total_blocks] descriptor index of every block
D3D_API int d3d_pack_all(const void* descs, const int* blk_desc, int total_blocks, hipStream_t st) {
  if (total_blocks <= 0) return 0;
  hipLaunchKernelGGL(pack_all_k, dim3(total_blocks), dim3(256), 0, st, (const PackDesc*)descs, blk_desc);
  return (int)hipGetLastError();
}

// ============================================================== C ABI =====
// I: [N, IH, IW, IC] bf16 (IC % 8 == 0), Wp: packed [OCp][taps][ICp] bf16 with
// OCp % 128 == 0 and ICp % 64 == 0.  O: [N, OH, OW, ldo] bf16.  taps = 9 (3x3)
// or 1 (1x1 / per-pixel linear).
// Halo variants measured and dropped: 32-wide images (2-7 % slower than
// conv_w8_k, profiles/kbench_conv_halo.jsonl), 256-pixel tiles (10-15 %
// slower than the 4-wave 128x128 kernel, kbench_conv_halo256.jsonl),
// fragment double-buffering (4-15 % slower, ab_halo_prefetch.txt).
// 64 x 64 no-split tiles (conv_small.hip) where the 128 x 128 kernels would
// split K over a small grid (the low-resolution levels at small per-GPU batch)
static int g_s64 = 1;
extern "C" int d3d_conv_s64_try(const void* I, const void* Wp, const float* bias, const float* row_bias,
                                const void* res, void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW,
                                int OC, int ldo, int stride, int trans, float scale, int res_nmod, int taps,
                                float* gnp, int gn_groups, int* gn_done, hipStream_t st, void* O2);
extern "C" int d3d_conv_hsm_try(const void* I, const void* Wp, const float* bias, const float* row_bias,
                                const void* res, void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW,
                                int OC, int ldo, int stride, int trans, float scale, int res_nmod, int taps,
                                const float* gnp, const void* O2, hipStream_t st);
// 64x64 no-split tiles (conv_small.hip) on grids of at most g_s64_maxb
// 128x128 blocks (default 160): the 16x16 / 8x8 levels at 16 examples per GPU
// and the 8x8 level at 32 (in-graph A/B: +1.1 % at bs16; the 16x16 level at
// bs32, 256 such blocks, stays on split-K bufl, which is faster there)
static const long g_s64_maxb = 160;
static bool s64_wanted(long Mpix, int OC, int ICp, int taps) {
  const long blocks128 = ((Mpix + 127) / 128) * ((OC + 127) / 128);
  const long blocks64 = ((Mpix + 63) / 64) * (OC / 64);
  return g_s64 && OC % 64 == 0 && (taps * ICp) % 64 == 0 && blocks128 <= g_s64_maxb && blocks64 >= 128;
}
// 1: the residual-free convs (dgrad, conv1) still run the residual-capable
// kernel variants (round-3 behaviour; A/B switch for the RES template)
static int g_conv_res_always = 0;
// conv_halo_k AU (unrolled taps, precomputed B offsets, residual preloaded into the accumulators); 0 off
static int g_halo_au = 1;
// 32-wide images on the halo kernel (16-row tiles) when the grid fills the chip:
// the 32x32 level at bs128 903 -> 1020 TF/s fwd, 892 -> 979 dgrad against
// conv_w8_k (profiles/r4/halo_w32/)
static int g_halo_w32 = 1;
// 16-wide images (one image per 256-pixel tile) when the grid fills the chip
// (bs128: 16x16x256 dgrad 155 -> 106 us), and 32-wide images in 8-row tiles
// where 16-row ones would not fill it (bs16: 32x32x256 dgrad 139 -> 71 us);
// bench +0.6 % bs128, +1.5 % bs16 (profiles/r4/halo_small/)
static int g_halo_w16 = 1;
static int g_halo_w32s = 1;
static int g_halo_p2 = 1;          // tap pairs per barrier (8-slot weight ring) on the 512-pixel tiles
// knob: bits 0-1 AU (0 off / 1 on), bit 2 the 32-wide halo, bit 3 the 16-wide halo, bit 4 the 8-row
// 32-wide tiles, bit 5 tap pairs per barrier (D3D_HALO_AU=61: all, the default; 29: all but
// the tap pairs -- profiles/r4/halo_p2: fwd -2..4 % on the N=256 levels, bs128 +0.7 %, bs16 +0.3 %)
D3D_API int d3d_conv_halo_cfg(int au) {
  g_halo_au = au & 3;
  g_halo_w32 = (au >> 2) & 1;
  g_halo_w16 = (au >> 3) & 1;
  g_halo_w32s = (au >> 4) & 1;
  g_halo_p2 = (au >> 5) & 1;
  return 0;
}
D3D_API int d3d_conv_res_cfg(int always) {
  g_conv_res_always = always;
  return 0;
}
static int g_conv_impl = -1;      // 0: register-staged, 1: glds pipeline, 2: buffer-descriptor LDS-DMA
static int g_conv_korder = 1;     // glds k-step order: 1 channel-chunk major, 0 tap major
static int g_wgrad_impl = 5;      // 0: register-staged; 1-4: glds (PK,NS) = (64,2) (32,2) (32,3) (64,3); 5: bufl
static const bf16* g_zero16 = nullptr;

D3D_API int d3d_set_wgrad_impl(int impl) {
  g_wgrad_impl = impl;
  return 0;
}

D3D_API int d3d_set_conv_korder(int korder) {
  g_conv_korder = korder;
  return 0;
}

D3D_API int d3d_set_conv_impl(int impl, const void* zero16) {
  g_conv_impl = impl;
  if (zero16) g_zero16 = (const bf16*)zero16;
  return 0;
}

// Split-K factor for the forward / dgrad GEMM: grids far below the 2 blocks
// per CU the kernel runs at (the 8x8 / 16x16 levels at small per-GPU batch:
// 64-128 blocks on 256 CUs) split their K = taps x IC reduction so the chip
// fills; >= 6 k-steps per split keeps the pipeline prologue amortised.
D3D_API int d3d_conv_plan(int N, int OH, int OW, int OC, int ICp, int taps) {
  constexpr int BM = 128, BN = 128;
  long Mpix = (long)N * OH * OW;
  long blocks = ((Mpix + BN - 1) / BN) * ((OC + BM - 1) / BM);
  int nk = taps * ICp / 64;
  static const int target = 512;
  if (blocks >= 384 || (OC & 3) || g_conv_impl < 1) return 1;
  if (g_conv_impl >= 2 && s64_wanted(Mpix, OC, ICp, taps)) return 1;     // no-split small tiles instead
  long want = target / blocks;      // rounded down: no nearly empty extra round of blocks
  long maxs = nk / 6;
  if (want > maxs) want = maxs;
  if (want > 16) want = 16;
  return want < 2 ? 1 : (int)want;
}

// gnp != nullptr: also produce the GroupNorm partial statistics of the
// output (gn_part_store layout, gn_groups groups) when the chosen kernel can;
// *gn_done reports whether it did (the caller runs the statistics pass
// otherwise).
// O2 != nullptr: also write silu(output) to O2 (same layout) when the chosen
// kernel can; *silu_done reports whether it did (the caller runs the SiLU
// pass otherwise).
D3D_API int d3d_conv3(const void* I, const void* Wp, const float* bias, const float* row_bias, const void* res,
                      void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo, int stride,
                      int trans, float scale, int res_nmod, int taps, float* ws, int nsplit, float* gnp,
                      int gn_groups, int* gn_done, void* O2, int* silu_done, hipStream_t st) {
  long Mpix = (long)N * OH * OW;
  if (gn_done) *gn_done = 0;
  if (silu_done) *silu_done = 0;
  if (!silu_done) O2 = nullptr;
  // Operands beyond the kernels' 32-bit buffer offsets (2 GiB: e.g. the
  // 256-channel decoder concat of 128x128 images at one micro-batch of 128):
  // run the conv over image chunks that fit, each at full speed, instead of
  // dropping to the register-staged fallback.  Chunk boundaries are multiples
  // of res_nmod (the broadcast residual's period); per-image operands
  // (output, per-image bias rows, GroupNorm partial slots) are offset, the
  // split-K workspace is reused chunk after chunk on the stream.
  {
    const long img_in = (long)IH * IW * IC * 2, img_out = (long)OH * OW * ldo * 2;
    const long lim = (1L << 31) - (1L << 20);
    if (N > 1 && ((long)N * img_in >= lim || (long)N * img_out >= lim)) {
      long per = lim / std::max(img_in, img_out);
      const int q = res_nmod > 0 ? res_nmod : 1;
      per = per / q * q;
      if (per >= 1) {
        const int parts_per_img = (OH * OW) % 64 == 0 ? OH * OW / 64 : 0;
        int all_gn = 1, all_silu = 1;
        for (int n0 = 0; n0 < N; n0 += (int)per) {
          const int nc = (int)std::min<long>(per, N - n0);
          int d = 0, ds = 0;
          const int rc = d3d_conv3((const char*)I + n0 * img_in, Wp, bias,
                                   row_bias ? row_bias + (long)n0 * OC : nullptr,
                                   res ? (res_nmod > 0 ? res : (const char*)res + n0 * img_out) : nullptr,
                                   (char*)O + n0 * img_out, nc, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans, scale,
                                   res_nmod, taps, ws, nsplit,
                                   gnp ? gnp + (long)n0 * gn_groups * parts_per_img * 2 : nullptr, gn_groups,
                                   gn_done ? &d : nullptr, O2 ? (char*)O2 + n0 * img_out : nullptr,
                                   O2 ? &ds : nullptr, st);
          if (rc) return rc;
          all_gn &= d;
          all_silu &= ds;
        }
        if (gn_done) *gn_done = gnp ? all_gn : 0;
        if (silu_done) *silu_done = O2 ? all_silu : 0;
        return 0;
      }
    }
  }
  if (gnp) {
    const int Cg = gn_groups > 0 && OC % gn_groups == 0 ? OC / gn_groups : 0;
    const bool ok = (Cg == 4 || Cg == 8 || Cg == 16 || Cg == 32) && (OH * OW) % 64 == 0 && Mpix % 64 == 0 &&
                    ldo == OC;
    if (!ok) gnp = nullptr;
  }
  constexpr int BM = 128, BN = 128;
  if (nsplit < 1 || !ws || g_conv_impl < 1) nsplit = 1;
  if (g_conv_impl >= 2 && nsplit == 1 && s64_wanted(Mpix, OC, ICp, taps)) {
    const int rh = d3d_conv_hsm_try(I, Wp, bias, row_bias, res, O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans,
                                    scale, res_nmod, taps, gnp, O2, st);
    if (rh != 0) return rh < 0 ? -rh : 0;
    const int r = d3d_conv_s64_try(I, Wp, bias, row_bias, res, O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans,
                                   scale, res_nmod, taps, gnp, gn_groups, gn_done, st, O2);
    if (r > 0 && silu_done) *silu_done = O2 ? 1 : 0;
    if (r != 0) return r < 0 ? -r : 0;
  }
  dim3 grid((unsigned)((Mpix + BN - 1) / BN), (unsigned)((OC + BM - 1) / BM), (unsigned)nsplit);
  const long in_bytes = (long)N * IH * IW * IC * 2, w_bytes = (long)((OC + 127) / 128 * 128) * taps * ICp * 2;
  if (g_conv_impl == 8 && taps == 9 && stride == 1 && IW == OW && IH == OH && ldo == OC && IC % HALO_CH == 0 &&
      OC % 128 == 0 && (OW == 16 || OW == 32 || OW == 64 || OW == 128) && in_bytes < (1L << 31) &&
      w_bytes < (1L << 31)) {
    // 512-pixel tiles where they fill the chip (64/128-wide images)
    auto nblk = [&](int bn) { return OH % (bn / OW) ? 0L : (long)N * (OH / (bn / OW)) * (OC / 128); };
    if ((OW != 32 || g_halo_w32) && nblk(512) >= 256) {
      dim3 gh((unsigned)(N * (OH / (512 / OW))), (unsigned)(OC / 128), 1);
#define HALO3(OWv, TR, RS, AUv, P2v)                                                                              \
  hipLaunchKernelGGL((conv_halo_k<OWv, TR, 512, false, RS, AUv, (P2v && OWv != 128)>), gh, dim3(512), 0, st, (const bf16*)I,     \
                     (const bf16*)Wp, bias, row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, N, OH, \
                     IC, ICp, OC, scale, res_nmod, gnp, gn_groups, (bf16*)O2, (const float*)nullptr)
#define HALO2(OWv, TR, RS, AUv) HALO3(OWv, TR, RS, AUv, false)
#define HALO(OWv, TR, RS)                                                                                          \
  do {                                                                                                            \
    if (g_halo_au && g_halo_p2 && OWv != 128 && (IC / HALO_CH) % 2 == 0) HALO3(OWv, TR, RS, true, true);          \
    else if (g_halo_au) HALO2(OWv, TR, RS, true);                                                                   \
    else HALO2(OWv, TR, RS, false);                                                                                 \
  } while (0)
      if (OW == 64) {
        if (trans) { if (res || g_conv_res_always) HALO(64, true, true); else HALO(64, true, false); }
        else if (res || g_conv_res_always) HALO(64, false, true); else HALO(64, false, false);
      } else if (OW == 32) {
        if (trans) { if (res || g_conv_res_always) HALO(32, true, true); else HALO(32, true, false); }
        else if (res || g_conv_res_always) HALO(32, false, true); else HALO(32, false, false);
      } else {
        if (trans) { if (res || g_conv_res_always) HALO(128, true, true); else HALO(128, true, false); }
        else if (res || g_conv_res_always) HALO(128, false, true); else HALO(128, false, false);
      }
#undef HALO
#undef HALO2
#undef HALO3
      if (gn_done && gnp) *gn_done = 1;
      if (silu_done && O2) *silu_done = 1;
      return (int)hipGetLastError();
    }
    if (((OW == 16 && g_halo_w16) || (OW == 32 && g_halo_w32s)) && nblk(256) >= 256) {
      // 256-pixel tiles (waves of 64 x 64): a whole 16-wide image, or 8 rows of a
      // 32-wide one where the 16-row tiles would not fill the chip (bs16)
      dim3 gh((unsigned)(N * (OH / (256 / OW))), (unsigned)(OC / 128), 1);
#define HALOS(OWv, TR, RS)                                                                                         \
  hipLaunchKernelGGL((conv_halo_k<OWv, TR, 256, false, RS, true>), gh, dim3(512), 0, st, (const bf16*)I,           \
                     (const bf16*)Wp, bias, row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, N, OH, \
                     IC, ICp, OC, scale, res_nmod, gnp, gn_groups, (bf16*)O2, (const float*)nullptr)
      if (OW == 16) {
        if (trans) { if (res || g_conv_res_always) HALOS(16, true, true); else HALOS(16, true, false); }
        else if (res || g_conv_res_always) HALOS(16, false, true); else HALOS(16, false, false);
      } else {
        if (trans) { if (res || g_conv_res_always) HALOS(32, true, true); else HALOS(32, true, false); }
        else if (res || g_conv_res_always) HALOS(32, false, true); else HALOS(32, false, false);
      }
#undef HALOS
      if (gn_done && gnp) *gn_done = 1;
      if (silu_done && O2) *silu_done = 1;
      return (int)hipGetLastError();
    }
  }
  if (g_conv_impl >= 4 && (!trans || stride == 1) && in_bytes < (1L << 31) && w_bytes < (1L << 31) && OC >= 64) {
    // large-tile 8-wave kernel when its grid still covers every CU
    const int bm = (OC % 256 == 0 || OC > 384) ? 256 : 128;
    // 128 / 384-channel layers only as 128x512 tiles on request (impl 6):
    // 128x256 tiles measured slower than two 128x128 blocks per CU (bufl1)
    const bool wide = bm == 128 && g_conv_impl >= 6;         // w8w, w8n, halo
    int bn = wide ? 512 : 256;
    long ptiles = (Mpix + bn - 1) / bn;
    long blocks = ptiles * ((OC + bm - 1) / bm);
    // impl 7: 256 x 128 tiles when 256 x 256 ones would leave CUs idle but
    // the narrower tile still gives every CU a block
    if (g_conv_impl == 7 && bm == 256 && blocks < 256 && ((Mpix + 127) / 128) * ((OC + 255) / 256) >= 256) {
      bn = 128;
      ptiles = (Mpix + bn - 1) / bn;
      blocks = ptiles * ((OC + bm - 1) / bm);
    }
    if ((bm == 256 || wide) && blocks >= 256) {
      dim3 g8((unsigned)ptiles, (unsigned)((OC + bm - 1) / bm), 1);
#define W8R(TP, TR, BMv, BNv, RS)                                                                                \
  hipLaunchKernelGGL((conv_w8_k<TP, TR, BMv, BNv, RS>), g8, dim3(512), 0, st, (const bf16*)I, (const bf16*)Wp, bias, \
                     row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, N, IH, IW, IC, ICp, OH, OW, \
                     OC, ldo, stride, scale, res_nmod, g_conv_korder, gnp, gn_groups, (bf16*)O2)
#define W8(TP, TR, BMv, BNv)                                                                                     \
  do {                                                                                                          \
    if (res || g_conv_res_always) W8R(TP, TR, BMv, BNv, true); else W8R(TP, TR, BMv, BNv, false);               \
  } while (0)
      if (bn == 128) {
        if (taps == 9) {
          if (trans) W8(9, true, 256, 128); else W8(9, false, 256, 128);
        } else {
          if (trans) W8(1, true, 256, 128); else W8(1, false, 256, 128);
        }
      } else if (bm == 256) {
        if (taps == 9) {
          if (trans) W8(9, true, 256, 256); else W8(9, false, 256, 256);
        } else {
          if (trans) W8(1, true, 256, 256); else W8(1, false, 256, 256);
        }
      } else {
        if (taps == 9) {
          if (trans) W8(9, true, 128, 512); else W8(9, false, 128, 512);
        } else {
          if (trans) W8(1, true, 128, 512); else W8(1, false, 128, 512);
        }
      }
#undef W8
#undef W8R
      if (gn_done && gnp) *gn_done = 1;
      if (silu_done && O2) *silu_done = 1;
      return (int)hipGetLastError();
    }
  }
  if (g_conv_impl >= 2 && (!trans || stride == 1) && in_bytes < (1L << 31) && w_bytes < (1L << 31)) {
    float* part = nsplit > 1 ? ws : nullptr;
#define BUFL(TP, TR, OB)                                                                                         \
  hipLaunchKernelGGL((conv_bufl_k<TP, TR, OB>), grid, dim3(256), 0, st, (const bf16*)I, (const bf16*)Wp, bias,    \
                     row_bias, (const bf16*)res, (bf16*)O, (int)in_bytes, (int)w_bytes, N, IH, IW, IC, ICp, OH, OW, \
                     OC, ldo, stride, scale, res_nmod, part, g_conv_korder, part ? nullptr : gnp, gn_groups,       \
                     part ? nullptr : (bf16*)O2)
    if (g_conv_impl >= 3) {
      if (taps == 9) {
        if (trans) BUFL(9, true, true); else BUFL(9, false, true);
      } else {
        if (trans) BUFL(1, true, true); else BUFL(1, false, true);
      }
    } else {
      if (taps == 9) {
        if (trans) BUFL(9, true, false); else BUFL(9, false, false);
      } else {
        if (trans) BUFL(1, true, false); else BUFL(1, false, false);
      }
    }
#undef BUFL
    if (part && gnp && OC % 64 == 0) {
      // gnp non-null implies ldo == OC, 64 | H*W and Cg <= 32
      hipLaunchKernelGGL(conv_splitk_epi_gn_k, dim3((unsigned)(Mpix / 64), (unsigned)(OC / 64)), dim3(256), 0, st,
                         part, nsplit, Mpix, OC, OH * OW, bias, row_bias, (const bf16*)res, res_nmod, (bf16*)O,
                         scale, gnp, gn_groups, (bf16*)O2);
      if (gn_done) *gn_done = 1;
    } else if (part) {
      long nv = Mpix * (OC / 4);
      long g = (nv + 255) / 256;
      if (g > 4096) g = 4096;
      hipLaunchKernelGGL(conv_splitk_epi_k, dim3((unsigned)g), dim3(256), 0, st, part, nsplit, Mpix, OC, OH * OW,
                         bias, row_bias, (const bf16*)res, res_nmod, (bf16*)O, ldo, scale, (bf16*)O2);
    } else if (gn_done && gnp) {
      *gn_done = 1;
    }
    if (silu_done && O2) *silu_done = 1;
    return (int)hipGetLastError();
  }
  if (g_conv_impl >= 1 && g_zero16) {
    float* part = nsplit > 1 ? ws : nullptr;
#define GLDS(TP, TR)                                                                                             \
  hipLaunchKernelGGL((conv_glds_k<TP, TR>), grid, dim3(256), 0, st, (const bf16*)I, (const bf16*)Wp, bias,        \
                     row_bias, (const bf16*)res, (bf16*)O, g_zero16, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, \
                     scale, res_nmod, part, g_conv_korder)
    if (taps == 9) {
      if (trans) GLDS(9, true); else GLDS(9, false);
    } else {
      if (trans) GLDS(1, true); else GLDS(1, false);
    }
#undef GLDS
    if (part) {
      long nv = Mpix * (OC / 4);
      long g = (nv + 255) / 256;
      if (g > 4096) g = 4096;
      hipLaunchKernelGGL(conv_splitk_epi_k, dim3((unsigned)g), dim3(256), 0, st, part, nsplit, Mpix, OC, OH * OW,
                         bias, row_bias, (const bf16*)res, res_nmod, (bf16*)O, ldo, scale, (bf16*)nullptr);
    }
    return (int)hipGetLastError();
  }
#define LAUNCH(TR, TP)                                                                                             \
  hipLaunchKernelGGL((conv_igemm_k<BM, BN, TR, TP>), grid, dim3(256), 0, st, (const bf16*)I, (const bf16*)Wp, bias, \
                     row_bias, (const bf16*)res, (bf16*)O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, scale,      \
                     res_nmod)
  if (taps == 9) {
    if (trans) LAUNCH(true, 9); else LAUNCH(false, 9);
  } else {
    if (trans) LAUNCH(true, 1); else LAUNCH(false, 1);
  }
#undef LAUNCH
  return (int)hipGetLastError();
}

// ResnetBlock conv1 with GN0 + SiLU folded into the halo staging (conv_halo_k
// GNA): I is the PRE-GroupNorm input x, gab [N][IC][2] the per-(image,
// channel) affine (norm.hip d3d_gn_ab).  Only the halo tiles' forward
// schedules take it; returns -2 (nothing launched) when this shape would run
// another kernel, so the caller keeps the separate GroupNorm pass.
static int conv3_gn_shape(int N, int H, int W, int IC, int OC, int* tile) {
  const long in_bytes = (long)N * H * W * IC * 2, w_bytes = (long)((OC + 127) / 128 * 128) * 9 * ((IC + 63) / 64 * 64) * 2;
  if (g_conv_impl != 8 || !g_halo_au || IC % HALO_CH || OC % 128 || (W != 32 && W != 64) || in_bytes >= (1L << 31) ||
      w_bytes >= (1L << 31) || IC > 512)
    return 0;
  auto nblk = [&](int bn) { return H % (bn / W) ? 0L : (long)N * (H / (bn / W)) * (OC / 128); };
  // (the 512-pixel tiles run the conv without the staging: with it their
  // unrolled-tap schedules need ~20 registers more than the 256 a wave has
  // at two waves per SIMD, and the spill reloads -- counted by vmcnt -- would
  // serialise the DMA pipeline)
  if ((W != 32 || g_halo_w32) && nblk(512) >= 256) return 0;
  if (W == 32 && g_halo_w32s && nblk(256) >= 256) {
    *tile = 256;
    return 1;
  }
  return 0;
}

D3D_API int d3d_conv3_gn_ok(int N, int H, int W, int IC, int OC) {
  int t = 0;
  return conv3_gn_shape(N, H, W, IC, OC, &t);
}

D3D_API int d3d_conv3_gn(const void* I, const void* Wp, const float* bias, void* O, int N, int H, int W, int IC,
                         int ICp, int OC, float* gnp, int gn_groups, int* gn_done, const float* gab, hipStream_t st) {
  int tile = 0;
  if (gn_done) *gn_done = 0;
  if (!conv3_gn_shape(N, H, W, IC, OC, &tile) || ICp != (IC + 63) / 64 * 64) return -2;
  if (gnp) {
    const int Cg = gn_groups > 0 && OC % gn_groups == 0 ? OC / gn_groups : 0;
    if (!((Cg == 4 || Cg == 8 || Cg == 16 || Cg == 32) && (H * W) % 64 == 0)) gnp = nullptr;
  }
  const long in_bytes = (long)N * H * W * IC * 2, w_bytes = (long)((OC + 127) / 128 * 128) * 9 * ICp * 2;
  dim3 gh((unsigned)(N * (H / (tile / W))), (unsigned)(OC / 128), 1);
#define GNL(OWv, BNv, P2v)                                                                                          \
  hipLaunchKernelGGL((conv_halo_k<OWv, false, BNv, false, false, true, P2v, true>), gh, dim3(512), 0, st,            \
                     (const bf16*)I, (const bf16*)Wp, bias, (const float*)nullptr, (const bf16*)nullptr, (bf16*)O,    \
                     (int)in_bytes, (int)w_bytes, N, H, IC, ICp, OC, 1.f, 0, gnp, gn_groups, (bf16*)nullptr, gab)
  GNL(32, 256, false);
  (void)tile;
#undef GNL
  if (gn_done && gnp) *gn_done = 1;
  return (int)hipGetLastError();
}

D3D_API int d3d_conv2(const void* I, const void* Wp, const float* bias, const float* row_bias, const void* res,
                      void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo, int stride,
                      int trans, float scale, int res_nmod, int taps, float* ws, int nsplit, float* gnp,
                      int gn_groups, int* gn_done, hipStream_t st) {
  return d3d_conv3(I, Wp, bias, row_bias, res, O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans, scale,
                   res_nmod, taps, ws, nsplit, gnp, gn_groups, gn_done, nullptr, nullptr, st);
}

D3D_API int d3d_conv(const void* I, const void* Wp, const float* bias, const float* row_bias, const void* res,
                     void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo, int stride,
                     int trans, float scale, int res_nmod, int taps, float* ws, int nsplit, hipStream_t st) {
  return d3d_conv2(I, Wp, bias, row_bias, res, O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans, scale,
                   res_nmod, taps, ws, nsplit, nullptr, 0, nullptr, st);
}

D3D_API int d3d_conv3x3(const void* I, const void* Wp, const float* bias, const float* row_bias, const void* res,
                        void* O, int N, int IH, int IW, int IC, int ICp, int OH, int OW, int OC, int ldo,
                        int stride, int trans, float scale, int res_nmod, hipStream_t st) {
  return d3d_conv(I, Wp, bias, row_bias, res, O, N, IH, IW, IC, ICp, OH, OW, OC, ldo, stride, trans, scale,
                  res_nmod, 9, nullptr, 1, st);
}

// launches wgrad_reduce2_k<SL> with SL = splits rounded up to a power of two
// (<= 16); bias rows (brows = 2 * splits) use the same lanes
static void launch_reduce2(const float* ws, int OC, int IC, int taps, int splits, int accumulate, const float* bws,
                           int brows, float* dW, float* db, WSegs sg, bool want_bias, hipStream_t st,
                           float scale = 1.f) {
  if (taps == 9 && sg.n == 0) {
    // split the taps over more blocks while the grid is below ~1024 blocks
    const long base = (long)OC * ((IC + 63) / 64);
    const int tg = base >= 1024 ? 9 : (base * 3 >= 1024 ? 3 : 1);
    const int nblk_w = (int)(base * (9 / tg));
    const int nblk_b = want_bias ? (OC + 63) / 64 : 0;
#define R9(TGv) hipLaunchKernelGGL(wgrad_reduce9_k<TGv>, dim3(nblk_w + nblk_b), dim3(256), 0, st, ws, OC, IC, splits, \
                                  accumulate, bws, brows, dW, db, nblk_w, scale)
    if (tg == 9) R9(9); else if (tg == 3) R9(3); else R9(1);
#undef R9
    return;
  }
  int SL = 1;
  while (SL < splits && SL < 16) SL <<= 1;
  const long total = (long)OC * IC * taps;
  const int per = 4 * (256 / SL);
  const int nblk_w = (int)((total + per - 1) / per);
  const int nblk_b = want_bias ? (OC + per - 1) / per : 0;
  dim3 grid(nblk_w + nblk_b);
#define RL(S) hipLaunchKernelGGL(wgrad_reduce2_k<S>, grid, dim3(256), 0, st, ws, OC, IC, taps, splits, accumulate, \
                                 bws, brows, dW, db, sg, nblk_w, scale)
  switch (SL) {
    case 1: RL(1); break;
    case 2: RL(2); break;
    case 4: RL(4); break;
    case 8: RL(8); break;
    default: RL(16); break;
  }
#undef RL
}

static void launch_wgrad(const void* dY, const void* I, float* ws, int N, int IH, int IW, int IC, int OH, int OW,
                         int OC, int stride, int pps, int ncb, float* bws, int lw, int lh, int taps, dim3 grid,
                         hipStream_t st, const void* I2 = nullptr, int C1 = 0) {
  constexpr int BM = 128, BN = 128;
  const long in_elems = (long)N * IH * IW * IC;
  // measured exception (profiles/kbench_lin_wgrad.jsonl): very wide per-pixel
  // GEMMs with very long per-split reductions (level-1 batched FiLM,
  // 1024 -> 4608 over 65536-pixel splits) run 1.6x faster register-staged
  const bool wide_long = taps == 1 && (long)OC * IC >= (4L << 20) && pps > 16384;
  // the dY descriptor is re-based per stage (its records span one split), so
  // only the input tensor's size is limited by the 32-bit offsets
  // (the FAST path measured slower on the 144-channel conditioning conv:
  // keep it to full 128-channel tiles).  FAST re-bases the input descriptor
  // per stage, so only the general path is bounded by 32-bit input offsets.
  const bool fast = stride == 1 && lw >= 0 && IH == OH && IW == OW && IC % 128 == 0;
  if (g_wgrad_impl >= 5 && !wide_long && (fast || in_elems * 2 < (1L << 31) - (1L << 20)) &&
      (long)pps * OC * 2 < (1L << 31)) {
    constexpr int PK = 32;
#define WB(TP, F)                                                                                                \
  hipLaunchKernelGGL((conv_wgrad_bufl_k<TP, PK, F>), grid, dim3(256), 0, st, (const bf16*)dY, (const bf16*)I, ws,   \
                     (long)N * IH * IW, N, IH, IW, IC, OH, OW, OC, stride, pps, ncb, bws, lw, lh, (const bf16*)I2, C1)
    if (taps == 9 && IC == 64 && !fast && I2 == nullptr) {
      // tap pairs: the grid's x dimension covers ceil(9 / 2) pairs
      dim3 gp(5, grid.y, grid.z);
      hipLaunchKernelGGL((conv_wgrad_bufl_k<9, PK, false, true>), gp, dim3(256), 0, st, (const bf16*)dY,
                         (const bf16*)I, ws, (long)N * IH * IW, N, IH, IW, IC, OH, OW, OC, stride, pps, 1, bws, lw, lh,
                         (const bf16*)nullptr, 0);
    } else if (taps == 9) {
      if (fast) WB(9, true); else WB(9, false);
    } else {
      if (fast) WB(1, true); else WB(1, false);
    }
#undef WB
    return;
  }
  if (g_wgrad_impl >= 1 && g_wgrad_impl <= 4 && g_zero16) {
#define WG(TP, PKv, NSv)                                                                                         \
  hipLaunchKernelGGL((conv_wgrad_glds_k<TP, PKv, NSv>), grid, dim3(256), 0, st, (const bf16*)dY, (const bf16*)I, ws, \
                     g_zero16, N, IH, IW, IC, OH, OW, OC, stride, pps, ncb, bws, lw, lh)
#define WGT(PKv, NSv) do { if (taps == 9) WG(9, PKv, NSv); else WG(1, PKv, NSv); } while (0)
    switch (g_wgrad_impl) {
      case 2: WGT(32, 2); break;
      case 3: WGT(32, 3); break;
      case 4: WGT(64, 3); break;
      default: WGT(64, 2); break;
    }
#undef WGT
#undef WG
    return;
  }
  if (taps == 9)
    hipLaunchKernelGGL((conv_wgrad_k<BM, BN, 9>), grid, dim3(256), 0, st, (const bf16*)dY, (const bf16*)I, ws, N, IH,
                       IW, IC, OH, OW, OC, stride, pps, ncb, bws, lw, lh);
  else
    hipLaunchKernelGGL((conv_wgrad_k<BM, BN, 1>), grid, dim3(256), 0, st, (const bf16*)dY, (const bf16*)I, ws, N, IH,
                       IW, IC, OH, OW, OC, stride, pps, ncb, bws, lw, lh);
}

D3D_API int d3d_conv_wgrad_plan2(int N, int OH, int OW, int OC, int IC, int taps, int* splits, int* pix_per_split) {
  constexpr int BM = 128, BN = 128;
  long P = (long)N * OH * OW;
  int tiles = (taps == 9 && IC == 64 ? 5 : taps * ((IC + BN - 1) / BN)) * ((OC + BM - 1) / BM);
  // block target: the kernel runs ~4 blocks per CU (32 KiB LDS, 64 VGPRs),
  // so ~1024 blocks fill the chip in one round; rounded down (no straggler
  // round).  Sweep on the X-UNet shapes (profiles/kbench_wgrad_plan.txt):
  // 1024 beats 512 by 10-35 %.  Every extra split costs a full fp32 OCxK slab
  // of write + reduce traffic.
  static const long target = 1024;
  static const bool ceil_ = false;
  long want = ceil_ ? (target + tiles - 1) / tiles : target / tiles;
  long maxs = (P + 255) / 256;       // small reductions (8x8 level at small batch): fill the chip first
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  long pps = (P + want - 1) / want;
  pps = (pps + 63) / 64 * 64;           // multiple of both kernels' pixel step
  *pix_per_split = (int)pps;
  *splits = (int)((P + pps - 1) / pps);
  return 0;
}

// conv_wgrad_w8_k takes a 3x3 stride-1 same-size power-of-two shape when
// at least one of its channel counts fills a 256-wide tile side (the 128x128
// level-0 convs stay on the 4-wave kernel); impl 6 enables it.
// taps == 1 (per-pixel GEMMs): any geometry,
// long reductions (the FiLM projections over every pixel of a level) are
// where the 4-wave kernel's 16-MFMA stages stall most.
static bool wgrad_w8_1x1() {
  static const int v = 1;
  return v != 0;
}

static bool wgrad_w8_ok(int taps, int IH, int IW, int OH, int OW, int IC, int OC, int stride, long in_elems, int* bm,
                        int* bn) {
  auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  // (the input descriptor is re-based per stage: no bound on the input size)
  if (g_wgrad_impl != 6 || IC % 128 || OC % 8) return false;
  if (taps == 1) {
    if (!wgrad_w8_1x1() || stride != 1 || IH != OH || IW != OW) return false;
  } else if (taps != 9 || stride != 1 || IH != OH || IW != OW || !pow2(OH) || !pow2(OW)) {
    return false;
  }
  // 256 output channels per tile: the 128-row form (384 -> 128) measured
  // 1.5x slower than the 4-wave kernel at its 1024-block plan
  *bm = 256;
  *bn = IC >= 256 ? 256 : 128;
  if (OC < 256) return false;
  // short reductions (16x16 / 8x8 levels at small per-GPU batch) cannot give
  // ~one block per CU >= 16 stages each: the 4-wave kernel is faster there
  // (kbench batch 16: 268 vs 196 TF/s at 16x16, 256 channels)
  const long P = in_elems / IC;
  const int tiles = taps * ((IC + *bn - 1) / *bn) * ((OC + *bm - 1) / *bm);
  long splits = 256 / tiles;
  if (splits > P / 1024) splits = P / 1024;
  if (splits < 1) splits = 1;
  // the dY descriptor spans one split: its byte count must fit 31 bits
  if ((P + splits - 1) / splits * OC * 2 >= (1L << 31) - (1L << 20)) return false;
  return tiles * splits >= 128;
}

// Split plan that knows the input geometry (and therefore which kernel runs):
// the 8-wave kernel wants ~one block per CU (256), the 4-wave one ~two.
D3D_API int d3d_conv_wgrad_plan3(int N, int IH, int IW, int OH, int OW, int OC, int IC, int taps, int stride,
                                 int* splits, int* pix_per_split) {
  int bm, bn;
  if (!wgrad_w8_ok(taps, IH, IW, OH, OW, IC, OC, stride, (long)N * IH * IW * IC, &bm, &bn))
    return d3d_conv_wgrad_plan2(N, OH, OW, OC, IC, taps, splits, pix_per_split);
  const long P = (long)N * OH * OW;
  const int tiles = taps * ((IC + bn - 1) / bn) * ((OC + bm - 1) / bm);
  // at one block per CU a grid just past 256 blocks runs a second, nearly
  // empty round: round the split count DOWN to fit one wave of blocks
  long want = 256 / tiles;
  long maxs = (P + 1023) / 1024;        // >= 16 stages of 64 pixels per split
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  long pps = (P + want - 1) / want;
  pps = (pps + 63) / 64 * 64;
  *pix_per_split = (int)pps;
  *splits = (int)((P + pps - 1) / pps);
  return 0;
}

static void launch_wgrad_w8(const void* dY, const void* I, float* ws, int N, int IH, int IW, int IC, int OH, int OW,
                            int OC, int pps, int splits, float* bws, int lw, int lh, int taps, int bn,
                            hipStream_t st) {
  const int ncb = (IC + bn - 1) / bn;
  dim3 g8(taps * ncb, (OC + 255) / 256, splits);
#define WW(BNv, TP)                                                                                              \
  hipLaunchKernelGGL((conv_wgrad_w8_k<256, BNv, TP>), g8, dim3(512), 0, st, (const bf16*)dY, (const bf16*)I, ws,  \
                     (long)N * IH * IW, N, IH, IW, IC, OH, OW, OC, pps, ncb, bws, lw, lh)
  if (taps == 9) {
    if (bn == 256) WW(256, 9); else WW(128, 9);
  } else {
    if (bn == 256) WW(256, 1); else WW(128, 1);
  }
#undef WW
}

D3D_API int d3d_conv_wgrad_plan(int N, int OH, int OW, int OC, int IC, int* splits, int* pix_per_split) {
  return d3d_conv_wgrad_plan2(N, OH, OW, OC, IC, 9, splits, pix_per_split);
}

// dY: [N, OH, OW, OC] bf16 (OC % 8 == 0); I: [N, IH, IW, IC] bf16.
// ws: [splits][OC][taps*IC] fp32 workspace.  dW: [OC][IC][taps] fp32 (OIHW).
// ws: [splits][OC][taps*IC] + (db ? 2*splits*OC : 0) fp32 workspace.
// dW (and db when non-null) are written (accumulate=0) or added to
// (accumulate=1) -- the latter lets kernels deposit straight into the flat
// gradient buffer across micro-batches.
D3D_API int d3d_conv_wgrad3(const void* dY, const void* I, float* ws, float* dW, float* db, int N, int IH, int IW,
                            int IC, int OH, int OW, int OC, int stride, int splits, int pix_per_split, int accumulate,
                            int taps, float scale, hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  long total = (long)OC * IC * taps;
  float* bws = db ? ws + (long)splits * total : nullptr;
  auto lg2 = [](int v) { int l = 0; while ((1 << l) < v) ++l; return (1 << l) == v ? l : -1; };
  int lw = lg2(OW), lh = lg2(OH);
  if (lw < 0 || lh < 0) lw = lh = -1;
  int bm, bn;
  if (wgrad_w8_ok(taps, IH, IW, OH, OW, IC, OC, stride, (long)N * IH * IW * IC, &bm, &bn)) {
    launch_wgrad_w8(dY, I, ws, N, IH, IW, IC, OH, OW, OC, pix_per_split, splits, bws, lw, lh, taps, bn, st);
  } else {
    int ncb = (IC + BN - 1) / BN;
    dim3 grid(taps * ncb, (OC + BM - 1) / BM, splits);
    launch_wgrad(dY, I, ws, N, IH, IW, IC, OH, OW, OC, stride, pix_per_split, ncb, bws, lw, lh, taps, grid, st);
  }
  {
    WSegs none{};
    launch_reduce2(ws, OC, IC, taps, splits, accumulate, bws, splits * (256 / BM), dW, db, none, db != nullptr, st,
                   scale);
  }
  return (int)hipGetLastError();
}

// dW (+ db) of the conv whose output gradient is scale * dY (scale folded
// into the split reduction)
D3D_API int d3d_conv_wgrad2(const void* dY, const void* I, float* ws, float* dW, float* db, int N, int IH, int IW,
                            int IC, int OH, int OW, int OC, int stride, int splits, int pix_per_split, int accumulate,
                            int taps, hipStream_t st) {
  return d3d_conv_wgrad3(dY, I, ws, dW, db, N, IH, IW, IC, OH, OW, OC, stride, splits, pix_per_split, accumulate,
                         taps, 1.f, st);
}

// Per-pixel dense weight gradient over a virtual channel concat [I | I2]
// (I: [rows, C1], I2: [rows, IC - C1], C1 % 128 == 0): dW [OC][IC].  Returns
// -1 (nothing launched) when the buffer kernel cannot take the shape; the
// caller then runs one GEMM per source.
D3D_API int d3d_conv_wgrad_cat(const void* dY, const void* I, const void* I2, int C1, float* ws, float* dW, float* db,
                               int rows, int IC, int OC, int splits, int pix_per_split, int accumulate,
                               hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  if (g_wgrad_impl < 5 || C1 % BN || (long)rows * IC * 2 >= (1L << 30) ||
      (long)pix_per_split * OC * 2 >= (1L << 31))
    return -1;
  const bool wide_long = (long)OC * IC >= (4L << 20) && pix_per_split > 16384;
  if (wide_long) return -1;
  int ncb = (IC + BN - 1) / BN;
  dim3 grid(ncb, (OC + BM - 1) / BM, splits);
  long total = (long)OC * IC;
  float* bws = db ? ws + (long)splits * total : nullptr;
  launch_wgrad(dY, I, ws, rows, 1, 1, IC, 1, 1, OC, 1, pix_per_split, ncb, bws, 0, 0, 1, grid, st, I2, C1);
  WSegs none{};
  launch_reduce2(ws, OC, IC, 1, splits, accumulate, bws, splits * (256 / BM), dW, db, none, db != nullptr, st);
  return (int)hipGetLastError();
}

// Weight gradient of a GEMM whose output rows are split over nseg parameters
// (row0[s] = first row of segment s, ascending; wdst[s] / bdst[s] = that
// parameter's dW / db, bdst entries may be null).  ws as for d3d_conv_wgrad2
// plus 2*splits*OC floats when any bdst is non-null.
D3D_API int d3d_conv_wgrad_seg(const void* dY, const void* I, float* ws, int N, int IH, int IW, int IC, int OH,
                               int OW, int OC, int stride, int splits, int pix_per_split, int accumulate, int taps,
                               int nseg, const int* row0, float* const* wdst, float* const* bdst, hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  if (nseg < 1 || nseg > kMaxSegs) return (int)hipErrorInvalidValue;
  WSegs sg{};
  sg.n = nseg;
  bool any_b = false;
  for (int i = 0; i < nseg; ++i) {
    sg.row0[i] = row0[i];
    sg.w[i] = wdst[i];
    sg.b[i] = bdst ? bdst[i] : nullptr;
    any_b = any_b || sg.b[i];
  }
  sg.row0[nseg] = OC;
  int ncb = (IC + BN - 1) / BN;
  dim3 grid(taps * ncb, (OC + BM - 1) / BM, splits);
  long total = (long)OC * IC * taps;
  float* bws = any_b ? ws + (long)splits * total : nullptr;
  auto lg2 = [](int v) { int l = 0; while ((1 << l) < v) ++l; return (1 << l) == v ? l : -1; };
  int lw = lg2(OW), lh = lg2(OH);
  if (lw < 0 || lh < 0) lw = lh = -1;
  int bm, bn;
  if (wgrad_w8_ok(taps, IH, IW, OH, OW, IC, OC, stride, (long)N * IH * IW * IC, &bm, &bn))
    launch_wgrad_w8(dY, I, ws, N, IH, IW, IC, OH, OW, OC, pix_per_split, splits, bws, lw, lh, taps, bn, st);
  else
    launch_wgrad(dY, I, ws, N, IH, IW, IC, OH, OW, OC, stride, pix_per_split, ncb, bws, lw, lh, taps, grid, st);
  launch_reduce2(ws, OC, IC, taps, splits, accumulate, bws, splits * (256 / BM), (float*)nullptr, (float*)nullptr, sg,
                 bws != nullptr, st);
  return (int)hipGetLastError();
}

// Scatter (accumulate) an already reduced [OC][IC] fp32 weight gradient --
// e.g. a hipBLASLt dY^T X product -- and optional [brows][OC] bias partials
// into the per-parameter segments of a batched projection (same segment
// description as d3d_conv_wgrad_seg).
D3D_API int d3d_wgrad_scatter(const float* ws, int OC, int IC, int splits, int accumulate, const float* bws,
                              int brows, int nseg, const int* row0, float* const* wdst, float* const* bdst,
                              hipStream_t st) {
  if (nseg < 1 || nseg > kMaxSegs) return (int)hipErrorInvalidValue;
  WSegs sg{};
  sg.n = nseg;
  for (int i = 0; i < nseg; ++i) {
    sg.row0[i] = row0[i];
    sg.w[i] = wdst[i];
    sg.b[i] = bdst ? bdst[i] : nullptr;
  }
  sg.row0[nseg] = OC;
  launch_reduce2(ws, OC, IC, 1, splits, accumulate, bws, brows, (float*)nullptr, (float*)nullptr, sg,
                 bws != nullptr, st);
  return (int)hipGetLastError();
}

D3D_API int d3d_conv_wgrad(const void* dY, const void* I, float* ws, float* dW, int N, int IH, int IW, int IC, int OH,
                           int OW, int OC, int stride, int splits, int pix_per_split, int accumulate, int taps,
                           hipStream_t st) {
  return d3d_conv_wgrad2(dY, I, ws, dW, nullptr, N, IH, IW, IC, OH, OW, OC, stride, splits, pix_per_split,
                         accumulate, taps, st);
}

D3D_API int d3d_conv3x3_wgrad(const void* dY, const void* I, float* ws, float* dW, int N, int IH, int IW, int IC,
                              int OH, int OW, int OC, int stride, int splits, int pix_per_split, int accumulate,
                              hipStream_t st) {
  return d3d_conv_wgrad(dY, I, ws, dW, N, IH, IW, IC, OH, OW, OC, stride, splits, pix_per_split, accumulate, 9, st);
}

// per-image (optional) and total channel sums of dY [N, P, C] (C % 8 == 0).
// part: workspace [(nchunks + 1) * N * C + 64 * C] fp32.
D3D_API int d3d_chansum(const void* dY, float* part, float* per_img, float* tot, int N, int P, int C, int nchunks,
                        hipStream_t st) {
  dim3 grid((C / 8 + 31) / 32, N, nchunks);
  hipLaunchKernelGGL(chansum_k, grid, dim3(256), 0, st, (const bf16*)dY, part, P, C, nchunks);
  // per-image sums (written into per_img, or into the part tail when the
  // caller only wants totals), then a parallel column sum over images
  float* pi = per_img ? per_img : part + (long)nchunks * N * C;
  hipLaunchKernelGGL(chansum_img_k, dim3(cdiv((long)N * C, 256)), dim3(256), 0, st, part, pi, N, C, nchunks);
  if (tot) d3d_colsum(pi, N, C, part + (long)(nchunks + 1) * N * C, tot, nullptr, 0, st);
  return (int)hipGetLastError();
}

D3D_API int d3d_pack_weight(const float* w, void* out, int OC, int IC, int OCp, int ICp, int trans, int taps,
                            hipStream_t st) {
  long total = (long)OCp * taps * ICp;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pack_w_k, dim3((int)g), dim3(256), 0, st, w, (bf16*)out, OC, IC, OCp, ICp, trans, taps);
  return (int)hipGetLastError();
}

D3D_API int d3d_pack_conv_weight(const float* w, void* out, int OC, int IC, int OCp, int ICp, int trans,
                                 hipStream_t st) {
  return d3d_pack_weight(w, out, OC, IC, OCp, ICp, trans, 9, st);
}
