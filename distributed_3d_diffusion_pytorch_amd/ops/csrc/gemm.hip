// Host side of the dense per-pixel GEMM (kernel: gemm_kernel.h, instantiated
// per tile size in gemm_w8.hip / gemm_w4.hip / gemm_w2.hip): tile-size rule,
// shape checks, launch geometry and the epilogue flag set.
#include "gemm_kernel.h"

#include <algorithm>

// ------------------------------------------------------------------ host ----
static int g_cfg_force = 0;     // 0: by problem size; 8 / 4 / 2: force the WI = WJ tile
static int g_gm = 8;
static int g_grid = 0;          // 0: resident blocks on every CU
static int g_deep = 1;          // 4-stage ring for the 64 / 128 tiles of small problems
static int g_cus() { return device_cus(); }

// Tuning switches for in-process A/B (forced tile config, tile-group width,
// grid); 0 leaves a setting unchanged (cfg 1 restores the size rule, cfg -1 / -2
// turn the deep stage ring on / off, grid -1 restores the resident grid).
D3D_API void d3d_gemm_tune(int cfg, int gm, int grid) {
  if (cfg == -1 || cfg == -2) g_deep = cfg == -1;       // -1 / -2: deep stage ring on / off
  else if (cfg == 1) g_cfg_force = 0;
  else if (cfg > 0) g_cfg_force = cfg;
  if (gm > 0) g_gm = gm;
  if (grid > 0) g_grid = grid;
  else if (grid < 0) g_grid = 0;                        // back to resident blocks on every CU
}

// Tile configuration for a problem: the 256 x 256 tile when it gives the chip
// most of a wave of tiles, smaller tiles (more blocks per CU) otherwise.
// Short-K projections (K <= 512, 256-768 output channels: the attention /
// NIN / 1x1 maps and their residual forms) are bandwidth-bound with one
// 256 x 256 block per CU -- its epilogue (residual read, output write) runs
// with nothing else in flight; two 128 x 128 blocks per CU overlap one's
// epilogue with the other's loads (tools/kbench_gemm.py: residual 256->256
// over 262144 pixels 55.9 -> 51.3 us, 512->256 NIN 42.2 -> 40.2 us).
static int g_small_k_w4 = 1;
// packed, mask-free epilogue when M is a multiple of the tile (F_MF); 0: the generic epilogue (A/B)
static int g_mf = 1;
D3D_API void d3d_gemm_mf(int on) { g_mf = on; }
D3D_API void d3d_gemm_small_k(int on) { g_small_k_w4 = on; }
// the 256 x 256 tile on 8 waves (two per SIMD: one wave's LDS-DMA issue and
// waits overlap the other's MFMAs) instead of 4 waves of 128 x 128
static int g_w8_waves = 4;           // 8 measured 3-8 % slower on the FiLM shapes (profiles/r6/gemm_waves.txt)
D3D_API void d3d_gemm_w8_waves(int nw) { g_w8_waves = nw == 4 ? 4 : 8; }
static int g_cfg8(int M, int N, int K);
static int g_cfg(int M, int N, int K) {
  const int w = g_cfg8(M, N, K);
  return w == 8 && g_w8_waves == 8 ? 9 : w;
}
static int g_cfg8(int M, int N, int K) {
  if (g_cfg_force) return g_cfg_force;
  const long cus = g_cus();
  if (g_small_k_w4 && K <= 512 && M >= 256 && M <= 768 && (long)cdiv(M, 128) * cdiv(N, 128) >= cus) return 4;
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  if (t256 >= cus * 3 / 4) return 8;
  const long t128 = (long)cdiv(M, 128) * cdiv(N, 128);
  if (t128 >= cus) return 4;
  return 2;
}

// Shapes the kernel takes: K a multiple of 64 and >= 128, M a multiple of 8,
// 16-byte aligned operand rows, one tile's operand rows addressable by
// 32-bit offsets.
D3D_API int d3d_gemm_nt_ok(int M, int N, int K, int lda, int ldb) {
  if (M <= 0 || N <= 0 || K < 128 || K % 64 || M % 8) return 0;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K) return 0;
  if (256L * lda * 2 >= (1L << 31) || 256L * ldb * 2 >= (1L << 31)) return 0;
  return 1;
}

// epi 0: O = (alpha * A.B^T + bias + R) * scale (+ GroupNorm partials gnp:
// [N / hw][G][hw / 64] x (sum, sumsq), gn_part_store layout; needs hw % 64 ==
// 0 and M / G in {4, 8, 16, 32}); epi 1: O = alpha * A.B^T * dsilu(R).
// bias_bf16: the bias vector is bf16 (else fp32).
D3D_API int d3d_gemm(const void* A, const void* B, void* O, const void* bias_, int bias_bf16, const void* R, int M,
                     int N, int K, int lda, int ldb, int ldo, int ldr, float alpha, float scale, float* gnp, int G,
                     int hw, int epi, hipStream_t st) {
  if (!d3d_gemm_nt_ok(M, N, K, lda, ldb)) return -1;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)O) & 15) return -1;
  if (ldo % 8 || ldo < M || (R && (ldr % 4 || ldr < M || ((uintptr_t)R & 7)))) return -1;
  if (epi == 1 && (!R || bias_ || gnp)) return -1;
  if (gnp && bias_ && bias_bf16) return -1;
  int W = g_cfg(M, N, K);
  if (gnp) {
    const int cg = G > 0 ? M / G : 0;
    if (G <= 0 || M % G || hw <= 0 || hw % 64 || N % hw || !(cg == 4 || cg == 8 || cg == 16 || cg == 32)) return -1;
    if (W == 2) W = 4;                         // the partials need whole 64-pixel parts per wave
  }
  const int BT = W == 9 ? 256 : 32 * W;
  if (256L * ldo * 2 >= (1L << 31) || (R && 256L * ldr * 2 >= (1L << 31)) || (long)M * 2 >= (1L << 31)) return -1;
  const int mt = cdiv(M, BT), nt = cdiv(N, BT);
  const long tiles = (long)mt * nt;
  if (tiles >= (1L << 31)) return -1;
  // deep ring (68 KB / 130 KB of LDS: 2 / 1 blocks per CU) when those
  // resident blocks hold every tile -- the latency-bound small problems
  const bool deep = g_deep && W < 8 && tiles <= (long)g_cus() * (W == 4 ? 1 : 2);
  // (an 8-stage ring for one 64-tile block per CU measured no gain, profiles/r4/gemm_deep8/: removed)
  const int per_cu = W >= 8 ? 1 : W == 4 ? 2 : 4;
  const int G_ = (int)std::min<long>(tiles, g_grid > 0 ? g_grid : (long)g_cus() * per_cu);
  const int gm = std::max(1, std::min(mt, g_gm));
  const int F = (epi == 1 ? F_DSILU
                           : (bias_ ? (bias_bf16 ? F_B16 : F_B32) : 0) | (R ? F_RES : 0) | (gnp ? F_GN : 0)) |
                (g_mf && !gnp && M % BT == 0 ? F_MF : 0);
  const GArgs ga{G_, st, A, B, O, bias_, R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, mt, nt, gm, gnp, G, hw,
                 nullptr, 0};
  return gemm_dispatch(W, F, deep, ga);
}

D3D_API int d3d_gemm_nt_gn(const void* A, const void* B, void* O, const float* bias, const void* R, int M, int N,
                           int K, int lda, int ldb, int ldo, int ldr, float alpha, float scale, float* gnp, int G,
                           int hw, hipStream_t st) {
  return d3d_gemm(A, B, O, bias, 0, R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, gnp, G, hw, 0, st);
}

D3D_API int d3d_gemm_nt(const void* A, const void* B, void* O, const float* bias, const void* R, int M, int N, int K,
                        int lda, int ldb, int ldo, int ldr, float alpha, float scale, hipStream_t st) {
  return d3d_gemm(A, B, O, bias, 0, R, M, N, K, lda, ldb, ldo, ldr, alpha, scale, nullptr, 0, 0, 0, st);
}

// Decoder NIN skip over the virtual concat [B | B2] (two [N][K1] tensors,
// K = 2 K1): O = (alpha * A.[B|B2]^T + bias) * scale as ONE GEMM (fp32 bias or
// none).  Returns -1 for shapes it does not take (the caller runs two GEMMs).
D3D_API int d3d_gemm_cat(const void* A, const void* B, const void* B2, int K1, void* O, const float* bias, int M,
                         int N, int K, int lda, int ldo, float alpha, float scale, hipStream_t st) {
  const int ldb = K1;
  if (M <= 0 || N <= 0 || K1 < 64 || K1 % 64 || K != 2 * K1 || M % 8 || lda % 8 || lda < K) return -1;
  if (256L * lda * 2 >= (1L << 31) || 256L * ldb * 2 + 4L * K1 >= (1L << 31)) return -1;   // per-tile offsets
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)B2 | (uintptr_t)O) & 15) return -1;
  if (ldo % 8 || ldo < M || 256L * ldo * 2 >= (1L << 31)) return -1;
  const int W = g_cfg(M, N, K);
  const int BT = W == 9 ? 256 : 32 * W;
  const int mt = cdiv(M, BT), nt = cdiv(N, BT);
  const long tiles = (long)mt * nt;
  if (tiles >= (1L << 31)) return -1;
  const bool deep = g_deep && W < 8 && tiles <= (long)g_cus() * (W == 4 ? 1 : 2);
  const int per_cu = W >= 8 ? 1 : W == 4 ? 2 : 4;
  const int G_ = (int)std::min<long>(tiles, g_grid > 0 ? g_grid : (long)g_cus() * per_cu);
  const int gm = std::max(1, std::min(mt, g_gm));
  const int F = (bias ? F_B32 | F_CAT : F_CAT) | (g_mf && M % BT == 0 ? F_MF : 0);
  const GArgs ga{G_, st, A, B, O, bias, nullptr, M, N, K, lda, ldb, ldo, ldo, alpha, scale, mt, nt, gm, nullptr, 0, 0,
                 B2, K1};
  return gemm_dispatch(W, F, deep, ga);
}
