// Weight gradients of the per-pixel dense layers on the matrix cores (the
// FiLM projections `xunet.py:74-87` batched per level, and any other wide
// 1x1 layer): a "TN" GEMM that reduces over pixel ROWS,
//
//     Ws[split][m][n] = sum_{p in split} Y[p][m] * X[p][n]     (fp32 slabs)
//     Bs[split][m]    = sum_{p in split} Y[p][m]                (bias partials)
//
// Y: the layer's output gradient [P][ldy] bf16, X: its input [P][ldx] bf16.
// The slabs are summed (and scattered into the parameters' gradients) by the
// split-K reduction of conv.hip (d3d_wgrad_scatter).
//
// Both operands are pixel-major, so an MFMA operand (8 consecutive pixels of
// one channel per lane) is a COLUMN of the loaded tile: the tiles land in LDS
// row-major through LDS-DMA (512-byte rows: whole cache lines) and the
// fragments come out with the gfx950 transposed read ds_read_b64_tr_b16
// (two reads = 8 pixels of one column).  Chunk swizzle c ^ ((row & 3) << 1 |
// ((row >> 3) & 1) << 3): a half-wave's 2 x 4 rows x 2 chunks land on 16
// distinct 16-byte bank slots -- conflict-free transposed reads.
//
// Schedule (as gemm.hip): 2 x 2 waves of 8 x 8 MFMA 16x16x32 tiles (a 256 x
// 256 output tile, 256 fp32 accumulators per lane in AGPRs); 64 pixel rows per
// LDS stage, two stages; every K-step is 64 slots of one MFMA plus at most a
// transposed read of the next K-step's fragments, an LDS-DMA piece of the
// stage after next (odd steps) or a bias dot product; one barrier per stage.
// The bias partial is a v_dot2_f32_bf16 of each Y fragment with (1, 1): 32
// VALU per K-step hidden under 64 MFMAs.  One tile per block, split-K over
// pixels: #tiles x #splits ~ a whole number of waves of blocks over the CUs.
#include "common.h"
#include "mfma_gemm.h"

#include <algorithm>

namespace {
constexpr int T_T = 256;                  // output tile: 256 m (Y columns) x 256 n (X columns)
constexpr int T_RK = 64;                  // pixel rows per LDS stage (two K-steps of 32)
constexpr int T_IMG = T_RK * T_T * 2;     // bytes of one operand image of one stage (32 KB)
// LDS (bytes): Y stage 0 | Y stage 1 | X stage 0 | X stage 1 -- stage and
// K-step offsets of a fragment read (<= 32768 + 16384 + 2048) fit the DS
// instruction's 16-bit immediate, so one address register per fragment
constexpr int T_LDS = 4 * T_IMG;
constexpr int T_X = 2 * T_IMG;

__device__ __forceinline__ int t_swz(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

// one pair of transposed reads -> an 8-pixel MFMA operand
__device__ __forceinline__ void t_frag(g_u4& f, const char* p) {
  const g_u2 lo = g_trd(p), hi = g_trd(p + 4 * 512);
  f = g_u4{lo[0], lo[1], hi[0], hi[1]};
}

__device__ __forceinline__ float t_dot2(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a), __builtin_bit_cast(bf16x2, b), c, false);
}

__device__ __forceinline__ void t_mma(f32x4& c, const g_u4& a, const g_u4& b) {
  g_mma(c, __builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b));
}
__device__ __forceinline__ void t_mma0(f32x4& c, const g_u4& a, const g_u4& b) {
  g_mma0(c, __builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b));
}
}  // namespace

template <int V>
__global__ void __launch_bounds__(256, 1)
wgrad_tn_k(const bf16* __restrict__ Y, const bf16* __restrict__ X, float* __restrict__ ws, float* __restrict__ bws,
           int M, int N, int P, int ldy, int ldx, int rps, int mt, int nt) {
  constexpr int WI = 8, WJ = 8, NM = WI * WJ, ND = 16;
  __shared__ __attribute__((aligned(16))) char smem[T_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;          // n half (X columns: MFMA rows), m half (Y columns)
  int rb = blockIdx.x;
  {   // XCD remap: consecutive logical blocks (the tiles of one split) share an XCD's L2
    const int G = gridDim.x, q = G / 8, r = G % 8, xcd = rb % 8;
    rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + rb / 8;
  }
  const int tiles = mt * nt;
  const int split = rb / tiles, t = rb - split * tiles;
  const int tm = t / nt, tn = t - tm * nt;
  const long p0 = (long)split * rps;
  const int rows = (int)std::min<long>(rps, P - p0);   // a multiple of 128 (host)
  const int nst = rows / T_RK;                         // stages: even, >= 2
  const int m0 = tm * T_T, n0 = tn * T_T;

  // operand descriptors: the split's rows from column m0 / n0 on; records end
  // at the tensor's last element, so columns past M / N of the last row read 0
  const bf16* yb = Y + p0 * ldy + m0;
  const bf16* xb = X + p0 * ldx + n0;
  const int yrec = (int)std::min<long>(((long)(P - 1 - p0) * ldy + M - m0) * 2, 0x7fffffffL);
  const int xrec = (int)std::min<long>(((long)(P - 1 - p0) * ldx + N - n0) * 2, 0x7fffffffL);

  // LDS-DMA pieces: wave w, piece d (0..7) of an operand = rows 16w + 2d, +1
  // (1 KB); lane -> (row h = lane >> 5, physical chunk lane & 31) loads
  // logical chunk (lane & 31) ^ swz(row); swz depends on (d & 1, d >> 2, h):
  // four per-lane base offsets per operand, the row offset added at the DMA
  int yo[4], xo[4];
  {
    const int h = lane >> 5, pc = lane & 31;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int sw = t_swz(2 * (c & 1) + h + 8 * (c >> 1));
      yo[c] = (wave * 16 + h) * ldy * 2 + ((pc ^ sw) << 4);
      xo[c] = (wave * 16 + h) * ldx * 2 + ((pc ^ sw) << 4);
    }
  }
  const int ystep = 2 * ldy * 2, xstep = 2 * ldx * 2;      // bytes per piece (2 rows)
  const int ystage = T_RK * ldy * 2, xstage = T_RK * ldx * 2;
  const g_i4 ydesc = g_desc(yb, yrec), xdesc = g_desc(xb, xrec);
  g_i4 ydesc0 = ydesc, xdesc0 = xdesc;                     // zero records: the DMAs past the last stage
  ydesc0[2] = 0;
  xdesc0[2] = 0;
  const unsigned lds0 = g_lds_u32(smem);
  auto dma = [&](int stage, int buf, int d, bool on) {     // piece d (< 8: Y, else X) of stage into buffer buf
    if (d < 8) {
      g_dma_asm(on ? ydesc : ydesc0, lds0 + buf * T_IMG + (wave * 16 + 2 * d) * 512,
                g_vadd(yo[(d & 1) | ((d >> 2) << 1)], d * ystep + stage * ystage));
    } else {
      const int e = d - 8;
      g_dma_asm(on ? xdesc : xdesc0, lds0 + T_X + buf * T_IMG + (wave * 16 + 2 * e) * 512,
                g_vadd(xo[(e & 1) | ((e >> 2) << 1)], e * xstep + stage * xstage));
    }
  };

  // fragment read addresses (stage 0, K-step half 0): lane (g, q, p) reads
  // row 8g + q, columns 4p.. of the fragment's 16; fragment f sits at chunk
  // 2 (f ^ s') + (p >> 1) of the wave's half (s' = swz >> 1)
  const char* ra[WI];
  const char* rbp[WJ];
  {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int sp = q | ((g & 1) << 2);
    const int rowb = (8 * g + q) * 512 + (p & 1) * 8 + (p >> 1) * 16;
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      ra[f] = smem + T_X + rowb + (wi * 16 + 2 * (f ^ sp)) * 16;
      rbp[f] = smem + rowb + (wj * 16 + 2 * (f ^ sp)) * 16;
    }
  }

  g_u4 a0[WI], b0[WJ], a1[WI], b1[WJ];
  f32x4 acc[WI][WJ];
  float bsum[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) bsum[j] = 0.f;
  const unsigned ones = 0x3F803F80u;                      // bf16 (1, 1)

  // prologue: stages 0 and 1 in flight, stage 0 published, first fragments read
#pragma unroll
  for (int d = 0; d < ND; ++d) dma(0, 0, d, true);
#pragma unroll
  for (int d = 0; d < ND; ++d) dma(1, 1, d, true);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ND) : "memory");
  G_BAR();
#pragma unroll
  for (int j = 0; j < WJ; ++j) t_frag(b0[j], rbp[j]);
#pragma unroll
  for (int i = 0; i < WI; ++i) t_frag(a0[i], ra[i]);

  // K-step s (stage s / 2, buffer (s / 2) & 1, half s & 1): bodies are
  // compile-time in (s mod 4) so every LDS offset is an immediate
  int stage = 0;                                            // stage of the current K-step
  // bias sums: one K-step in 2 * nt per wave -- (tile column tn, wave row wi)
  // take residue 2 tn + wi, so the block's 2 x nt wave pairs cover every step
  // once, at 1 / (2 nt) of the VALU cost (interleaved with every step's MFMAs
  // the dot products cost ~18 %: profiles/kbench_wgrad_tn_r3.jsonl); a small
  // branch around the dot products only (a branch around whole steps makes
  // the 256 accumulators phi nodes and spills them)
  const int bper = 2 * nt, bmine = (V & 1) || !bws ? -1 : 2 * tn + wi;
  int bc = 0;
  auto body = [&](auto first, auto sm4, auto last, g_u4(&ca)[WI], g_u4(&cb)[WJ], g_u4(&na)[WI], g_u4(&nb)[WJ]) {
    constexpr int S4 = decltype(sm4)::value;
    const bool bon = bc == bmine;
    if (++bc == bper) bc = 0;
    constexpr bool ODD = S4 & 1, LAST = decltype(last)::value;
    // this step's fragments (read during the previous step) have landed; before
    // an odd step's barrier this also retires every read of the stage whose
    // buffer the DMA below overwrites
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (ODD) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // stage + 1 landed (this wave's pieces)
      G_BAR();                                              // ... everyone's: published; stage's buffer free
    }
    // next K-step: (S4 + 1) & 3 -> buffer ((S4 + 1) >> 1) & 1, half (S4 + 1) & 1
    constexpr int NOFF = ((((S4 + 1) >> 1) & 1) * T_IMG) + (((S4 + 1) & 1) * 32 * 512);
    constexpr int BUF = (S4 >> 1) & 1;                      // buffer of the current stage (DMA target)
    const bool on = stage + 2 < nst;
    g_for(std::make_integer_sequence<int, NM>{}, [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (decltype(first)::value) t_mma0(acc[k / WJ][k % WJ], ca[k / WJ], cb[k % WJ]);
      else t_mma(acc[k / WJ][k % WJ], ca[k / WJ], cb[k % WJ]);
      if constexpr (!LAST && k % 3 == 0 && k / 3 < 16) {    // 16 operand reads (2 transposed each), B first,
        constexpr int r = k / 3;                            // done by slot 45: landed before the next step
        if constexpr (r < WJ) t_frag(nb[r], rbp[r] + NOFF);
        else t_frag(na[r - WJ], ra[r - WJ] + NOFF);
      }
      if constexpr (k == 48) {                              // bias: every Y fragment (reads all issued)
        if (bon) {
#pragma unroll
          for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int j = 0; j < WJ; ++j) bsum[j] = t_dot2(cb[j][w], ones, bsum[j]);
        }
      }
      if constexpr (V & 2) {
        if constexpr (ODD && k < ND) dma(stage + 2, BUF, k, on);
      } else {
        if constexpr (ODD && (k & 3) == 2) dma(stage + 2, BUF, k / 4, on);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (ODD) ++stage;
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  const int nit = nst / 2;                                  // 4 K-steps per iteration
  if (nit == 1) {
    body(T_{}, I0{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I1{}, F_{}, a1, b1, a0, b0);
    body(F_{}, I2{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I3{}, T_{}, a1, b1, a0, b0);
  } else {
    body(T_{}, I0{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I1{}, F_{}, a1, b1, a0, b0);
    body(F_{}, I2{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I3{}, F_{}, a1, b1, a0, b0);
    for (int it = 1; it < nit - 1; ++it) {
      body(F_{}, I0{}, F_{}, a0, b0, a1, b1);
      body(F_{}, I1{}, F_{}, a1, b1, a0, b0);
      body(F_{}, I2{}, F_{}, a0, b0, a1, b1);
      body(F_{}, I3{}, F_{}, a1, b1, a0, b0);
    }
    body(F_{}, I0{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I1{}, F_{}, a1, b1, a0, b0);
    body(F_{}, I2{}, F_{}, a0, b0, a1, b1);
    body(F_{}, I3{}, T_{}, a1, b1, a0, b0);
  }

  // ---- epilogue: lane (g = lane >> 4, c = lane & 15) of tile (i, j) holds
  // W[m = j-col c][n = 4g..4g+3 of i] -> one 16-byte store
  {
    float* wb = ws + (long)split * M * N;
    const int wrec = M * N * 4;
    const int c = lane & 15, g = lane >> 4;
    g_for(std::make_integer_sequence<int, NM>{}, [&](auto kc) {
      constexpr int k = decltype(kc)::value, i = k / WJ, j = k % WJ;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[e]) : "a"(acc[i][j][e]));
      const int m = m0 + wj * 128 + j * 16 + c, n = n0 + wi * 128 + i * 16 + 4 * g;
      g_store16(wb, wrec, __builtin_bit_cast(g_u4, v), (m < M && n < N) ? (m * N + n) * 4 : (int)0x80000000);
      __builtin_amdgcn_sched_barrier(0);
    });
    if (bws) {                                              // partial row (split, tn, wi)
      // the four K-groups' partial sums of each column -> lanes 0..15
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        float s = bsum[j];
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        const int m = m0 + wj * 128 + j * 16 + c;
        if (g == 0 && m < M) bws[((long)(split * nt + tn) * 2 + wi) * M + m] = s;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ host ----
static int t_var = 0;
D3D_API void d3d_wgrad_tn_tune(int v) { t_var = v; }

static int t_cus() { return device_cus(); }

// Pixel rows per split for `splits` splits: whole 128-row units.
static long t_rps(long P, int splits) { return ((P / 128 + splits - 1) / splits) * 128; }

// Shapes the kernel takes, and the split count: #tiles x #splits blocks in
// whole waves over the CUs (the smallest count within 3 % of the best), each
// split >= 512 pixel rows.  0: not supported.
D3D_API int d3d_wgrad_tn_plan(int M, int N, long P, int ldy, int ldx) {
  if (M <= 0 || N <= 0 || M % 8 || N % 8 || ldy % 8 || ldx % 8 || ldy < M || ldx < N) return 0;
  if (P < 128 || P % 128) return 0;
  if ((long)M * N * 4 >= (1L << 31)) return 0;
  const long tiles = (long)cdiv(M, T_T) * cdiv(N, T_T);
  const long cus = t_cus();
  double best = 1e30;
  int bs = 0;
  double cost[65] = {0};
  for (int s = 1; s <= 64; ++s) {
    const long rps = t_rps(P, s);
    const long used = (P + rps - 1) / rps;
    if (s > 1 && (rps < 512 || used < s)) break;
    if ((rps + 2) * std::max(ldy, ldx) * 2L >= (1L << 31)) { cost[s] = 1e30; continue; }
    const long blocks = tiles * used;
    cost[s] = (double)((blocks + cus - 1) / cus) * rps;       // waves of blocks x rows per block
    if (cost[s] < best) best = cost[s];
    bs = s;
  }
  if (!bs || best >= 1e30) return 0;
  for (int s = 1; s <= bs; ++s)
    if (cost[s] <= best * 1.03) return s;
  return bs;
}

// Y [P][ldy], X [P][ldx] bf16; ws: splits x M x N fp32 slabs; bws: splits x
// 2 cdiv(N, 256) x M fp32 bias partials (nullptr: none).  Returns the number of slabs written
// (<= splits) or < 0.
D3D_API int d3d_wgrad_tn(const void* Y, const void* X, float* ws, float* bws, int M, int N, long P, int ldy, int ldx,
                         int splits, hipStream_t st) {
  if (splits < 1 || d3d_wgrad_tn_plan(M, N, P, ldy, ldx) == 0) return -1;
  if (((uintptr_t)Y | (uintptr_t)X | (uintptr_t)ws) & 15) return -1;
  const long rps = t_rps(P, splits);
  if ((rps + 2) * std::max(ldy, ldx) * 2L >= (1L << 31)) return -1;
  const int used = (int)((P + rps - 1) / rps);
  const int mt = cdiv(M, T_T), nt = cdiv(N, T_T);
  const long blocks = (long)mt * nt * used;
  if (blocks >= (1L << 31)) return -1;
#define T_L(V_)                                                                                                  \
  hipLaunchKernelGGL(wgrad_tn_k<V_>, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16*)Y, (const bf16*)X, ws, bws, \
                     M, N, (int)P, ldy, ldx, (int)rps, mt, nt)
  switch (t_var) {
    case 1: T_L(1); break;
    case 2: T_L(2); break;
    case 3: T_L(3); break;
    default: T_L(0); break;
  }
#undef T_L
  const int e = (int)hipGetLastError();
  return e ? -e : used;
}
