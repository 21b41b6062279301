// GroupNorm family for NHWC bf16 activations on gfx950.
//
// Reference ops replaced: nn.GroupNorm(32, C) over the frame-folded batch
// (xunet.py:61-71) x101, the SiLU after GN0/lastgn (xunet.py:140,535), the FiLM
// modulation h*(1+scale)+shift (xunet.py:87) and Dropout(p=0.1)
// (xunet.py:120).  Kernels:
//   gn_stats   : per-(image, chunk) partial moments -> merged (Chan) -> mean/rstd
//   gn_apply   : y = [silu](xhat*gamma+beta)
//   gn_film    : y = dropout((xhat*gamma+beta)*(1+s)+t)          (one pass)
//   gn_bwd_*   : fused backward; the FiLM variant also emits d[scale|shift]
// Memory-bound: every pass moves 16-byte vectors (8 channels per lane); the
// reductions never re-read the input in a second pass (partials in LDS,
// tiny cross-chunk merge kernels).
#include "common.h"
#include <stdlib.h>


namespace {

constexpr int NT = 256;        // threads per block for the chunked kernels

struct Plan {
  int tpr;      // threads per row (C/8)
  int rpi;      // rows per iteration (NT / tpr)
  int nchunks;  // chunks per image
  int rows;     // rows per chunk (multiple of rpi)
};

// blocks per GroupNorm launch: 1024 beat 2048 and 512 by 0.5-1 % on both
// headline configs (the per-block merge / LDS epilogue amortises over more
// rows; profiles/ab_gn_target.txt)
static int g_gn_blocks = 1024;
static int g_gn_red_u = 1, g_gn_app_u = 2;    // rows in flight per thread: backward reduce / apply
// ... except for batches of at most g_gn_small_n images, where 512 measured
// +0.6 % of the bs16 step (32 images) in round 6 and 1024 stays ahead from 64
// images (profiles/r6/knob_sweep_b128.txt; d3d_gn_cfg_small, 0 off)
static int g_gn_small_n = 32, g_gn_small_blocks = 512;
static int gn_target_blocks(int N) { return N <= g_gn_small_n ? g_gn_small_blocks : g_gn_blocks; }

Plan make_plan(int N, int P, int C) {
  Plan p;
  p.tpr = C / 8;
  p.rpi = NT / p.tpr;
  if (p.rpi < 1) p.rpi = 1;
  int target_blocks = gn_target_blocks(N);
  int nch = (target_blocks + N - 1) / N;
  int maxch = (P + p.rpi - 1) / p.rpi;
  if (nch > maxch) nch = maxch;
  // keep >= 4 rows per thread so the per-thread partials amortise the merge
  int min_rows = 4 * p.rpi;
  int maxch2 = (P + min_rows - 1) / min_rows;
  if (nch > maxch2) nch = maxch2;
  if (nch < 1) nch = 1;
  int rows = (P + nch - 1) / nch;
  rows = (rows + p.rpi - 1) / p.rpi * p.rpi;
  p.rows = rows;
  p.nchunks = (P + rows - 1) / rows;
  return p;
}

// Virtual channel concat [x | x2] (decoder skip concatenation, xunet.py:521-531):
// channels [0, C1) live in x ([.., C1]), [C1, C) in x2 ([.., C - C1]); the
// concatenated tensor is never materialised.  x2 == nullptr: plain x [.., C].
struct Cat {
  const bf16* x2;
  bf16* dx2;
  int C1;
};

__device__ __forceinline__ const bf16* xsrc(const bf16* x, const Cat& k, long pix, int c0, int C) {
  if (k.x2 == nullptr) return x + pix * C + c0;
  return c0 < k.C1 ? x + pix * k.C1 + c0 : k.x2 + pix * (C - k.C1) + (c0 - k.C1);
}

__device__ __forceinline__ bf16* dxdst(bf16* dx, const Cat& k, long pix, int c0, int C) {
  if (k.x2 == nullptr) return dx + pix * C + c0;
  return c0 < k.C1 ? dx + pix * k.C1 + c0 : k.dx2 + pix * (C - k.C1) + (c0 - k.C1);
}

// Channel-fixed row walk of the chunked kernels: thread t owns the 8
// channels c0 = (t % cv) * 8 of rows t / cv, t / cv + rpi, ... (rpi = NT / cv
// rows per pass; the NT % cv leftover threads idle), so every per-channel
// constant (affine, group statistics) is loaded once into registers and the
// loop carries no index division.  Rows are processed UNR at a time with all
// loads issued first (memory-level parallelism for a bandwidth-bound pass).
constexpr int UNR = 4;

struct RowSrc {          // one thread's source row pointer / stride (virtual concat aware)
  const bf16* p;
  long ld;
};
__device__ __forceinline__ RowSrc row_src(const bf16* x, const Cat& k, int c0, int C) {
  if (k.x2 == nullptr) return {x + c0, (long)C};
  if (c0 < k.C1) return {x + c0, (long)k.C1};
  return {k.x2 + (c0 - k.C1), (long)(C - k.C1)};
}

// ---------------------------------------------------------------- stats ----
__global__ void __launch_bounds__(NT) gn_stats_partial_k(const bf16* __restrict__ x, int P, int C, int G,
                                                         int rows, int nchunks, float* __restrict__ part, Cat cat) {
  constexpr int U = 2;      // rows in flight per thread
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][rpi][C] + [rpi]
  const int chunk = blockIdx.x, n = blockIdx.y;
  const int tpr = C / 8, rpi = NT / tpr;
  const int tid = threadIdx.x;
  const int roff = tid / tpr, v = tid % tpr, c0 = v * 8;
  const bool active = roff < rpi;
  const int r0 = chunk * rows, r1 = min(P, r0 + rows);
  float sh[8], s[8], q[8];
  float cnt = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { sh[j] = 0.f; s[j] = 0.f; q[j] = 0.f; }
  if (active) {
    const long pix0 = (long)n * P;
    int r = r0 + roff;
    if (r < r1) {
      f32x8 a = ld8(xsrc(x, cat, pix0 + r, c0, C));
#pragma unroll
      for (int j = 0; j < 8; ++j) sh[j] = a[j];
      cnt = 1.f;
      r += rpi;
    }
    const RowSrc src = row_src(x, cat, c0, C);
    for (; r < r1; r += U * rpi) {
      f32x8 a[U];                         // U rows in flight
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (r + u * rpi < r1) a[u] = ld8(src.p + (pix0 + r + u * rpi) * src.ld);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * rpi >= r1) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = a[u][j] - sh[j];
          s[j] += d;
          q[j] += d * d;
        }
        cnt += 1.f;
      }
    }
  }
  // structure of arrays: mean [rpi][C] | m2 [rpi][C] | count [rpi] (one per
  // row lane), each thread's 8 channels two 16-byte stores (the interleaved
  // [rpi][C][3] layout was 84-86 % LDS bank-conflict cycles,
  // profiles/r3/pmc_step/table_bs128.txt)
  const int SL = rpi * C;
  if (active) {
    float mn[8], m2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float m = cnt > 0.f ? s[j] / cnt : 0.f;
      mn[j] = sh[j] + m;
      m2[j] = fmaxf(q[j] - s[j] * m, 0.f);
    }
    float* o = lds + roff * C + c0;
    *reinterpret_cast<f32x4*>(o) = f32x4{mn[0], mn[1], mn[2], mn[3]};
    *reinterpret_cast<f32x4*>(o + 4) = f32x4{mn[4], mn[5], mn[6], mn[7]};
    *reinterpret_cast<f32x4*>(o + SL) = f32x4{m2[0], m2[1], m2[2], m2[3]};
    *reinterpret_cast<f32x4*>(o + SL + 4) = f32x4{m2[4], m2[5], m2[6], m2[7]};
    if (v == 0) lds[2 * SL + roff] = cnt;
  }
  __syncthreads();
  // per group: TPG consecutive lanes (a power of two <= 64: a group never
  // straddles a wave) each merge a strided share of the rpi x Cg entries, then
  // a fixed-order butterfly of Chan merges (deterministic)
  const int Cg = C / G;
  int TPG = 1;
  while (TPG < 64 && TPG * 2 * G <= NT) TPG <<= 1;
  const int E = rpi * Cg;
  for (int g0 = 0; g0 < G; g0 += NT / TPG) {
    const int g = g0 + tid / TPG, sub = tid % TPG;
    Moments acc = {0.f, 0.f, 0.f};
    if (g < G)
      for (int e = sub; e < E; e += TPG) {
        const int rr = e / Cg, cc = e - rr * Cg;
        const Moments b = {lds[2 * SL + rr], lds[rr * C + g * Cg + cc], lds[SL + rr * C + g * Cg + cc]};
        if (b.n > 0.f) acc = merge_moments(acc, b);
      }
    for (int w = 1; w < TPG; w <<= 1) {
      const Moments b = {__shfl_xor(acc.n, w), __shfl_xor(acc.mean, w), __shfl_xor(acc.m2, w)};
      acc = merge_moments(acc, b);
    }
    if (g < G && sub == 0) {
      float* dst = part + (((long)n * nchunks + chunk) * G + g) * 2;
      dst[0] = acc.mean;
      dst[1] = acc.m2;
    }
  }
}

__global__ void gn_stats_final_k(const float* __restrict__ part, int N, int P, int G, int Cg, int rows,
                                 int nchunks, float eps, float* __restrict__ stats) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * G) return;
  int n = t / G, g = t % G;
  Moments acc = {0.f, 0.f, 0.f};
  for (int c = 0; c < nchunks; ++c) {
    int r0 = c * rows, r1 = min(P, r0 + rows);
    const float* p = part + (((long)n * nchunks + c) * G + g) * 2;
    Moments b = {(float)((r1 - r0) * Cg), p[0], p[1]};
    acc = merge_moments(acc, b);
  }
  float var = acc.m2 / acc.n;
  stats[t * 2 + 0] = acc.mean;
  stats[t * 2 + 1] = rsqrtf(fmaxf(var, 0.f) + eps);
}

// ---------------------------------------------------------------- apply ----
template <bool SILU>
__global__ void gn_apply_k(const bf16* __restrict__ x, const float* __restrict__ stats,
                           const float* __restrict__ gamma, const float* __restrict__ beta, bf16* __restrict__ y,
                           long nvec, int C, int Cg, int G, long PC) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    long e = i * 8;
    int c0 = (int)(e % C);
    int n = (int)(e / PC);
    f32x8 a = ld8(x + e);
    f32x8 gm = ld8f(gamma + c0), bt = ld8f(beta + c0);
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int g = (c0 + j) / Cg;
      float mean = stats[(n * G + g) * 2], rstd = stats[(n * G + g) * 2 + 1];
      float h = (a[j] - mean) * rstd * gm[j] + bt[j];
      o[j] = SILU ? siluf_(h) : h;
    }
    st8(y + e, o);
  }
}

__global__ void gn_film_k(const bf16* __restrict__ x, const float* __restrict__ stats,
                          const float* __restrict__ gamma, const float* __restrict__ beta,
                          const bf16* __restrict__ ss, bf16* __restrict__ y, long nvec, int C, int Cg, int G,
                          long PC, float p_drop, uint64_t seed, int ssld, const uint64_t* __restrict__ seed_dev) {
  if (seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;   // graph replays: per-step seed lives on the device
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    long e = i * 8;
    int c0 = (int)(e % C);
    long pix = e / C;
    int n = (int)(e / PC);
    f32x8 a = ld8(x + e);
    f32x8 sc = ld8(ss + pix * ssld + c0);
    f32x8 sf = ld8(ss + pix * ssld + C + c0);
    f32x8 gm = ld8f(gamma + c0), bt = ld8f(beta + c0);
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int g = (c0 + j) / Cg;
      float mean = stats[(n * G + g) * 2], rstd = stats[(n * G + g) * 2 + 1];
      float h = (a[j] - mean) * rstd * gm[j] + bt[j];
      float z = h * (1.f + sc[j]) + sf[j];
      if (p_drop > 0.f) z = drop_elem(dkey, (uint64_t)(e + j), dthr) ? 0.f : z * keep_scale;
      o[j] = z;
    }
    st8(y + e, o);
  }
}

// ----------------------------------------------- chunked apply (fused) ----
// Same chunking as the statistics pass (grid = chunks x images): each block
// merges its image's chunk partials into LDS (the separate finalize launch is
// gone -- at small batch every GroupNorm paid ~10 us for it), block 0 of the
// image also publishes mean / rstd for the backward pass.
// conv_parts > 0: part holds the producing conv's fused epilogue partials
// ([N][G][conv_parts] x (sum, sum of squares) over 64 pixels x Cg channels,
// conv.hip gn_part_store) instead of the statistics pass's chunk moments.
__device__ __forceinline__ void merge_image_stats(const float* __restrict__ part, int n, int nchunks, int G, int P,
                                                  int rows, int Cg, float eps, float* s_st,
                                                  float* __restrict__ stats_out, bool publish, int conv_parts) {
  // NT / G threads per group each fold a strided subset of the parts -- 8
  // loads issued back to back per round, so a 64-part image costs one L2
  // round trip instead of a chain of dependent ones -- then the group's
  // thread merges the subsets in fixed order (deterministic).
  constexpr int B = 8;
  if (G <= NT) {
    __shared__ float s_sub[3 * NT];
    const int subs = NT / G;
    const int g = threadIdx.x % G, sub = threadIdx.x / G;
    const int nparts = conv_parts > 0 ? conv_parts : nchunks;
    Moments m = {0.f, 0.f, 0.f};
    if (sub < subs) {
      for (int t0 = sub; t0 < nparts; t0 += B * subs) {
        float u[B], v[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
          const int t = t0 + k * subs;
          const float* pp = conv_parts > 0 ? part + (((long)n * G + g) * conv_parts + t) * 2
                                           : part + (((long)n * nchunks + t) * G + g) * 2;
          u[k] = t < nparts ? pp[0] : 0.f;
          v[k] = t < nparts ? pp[1] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
          const int t = t0 + k * subs;
          if (t >= nparts) break;
          Moments bm;
          if (conv_parts > 0) {          // (sum, sum of squares) over 64 pixels x Cg channels
            const float cnt = 64.f * Cg, mean = u[k] / cnt;
            bm = {cnt, mean, fmaxf(v[k] - u[k] * mean, 0.f)};
          } else {                        // statistics pass: (mean, M2) over the chunk's rows
            const int q0 = t * rows, q1 = min(P, q0 + rows);
            bm = {(float)((q1 - q0) * Cg), u[k], v[k]};
          }
          m = merge_moments(m, bm);
        }
      }
    }
    s_sub[threadIdx.x * 3 + 0] = m.n;
    s_sub[threadIdx.x * 3 + 1] = m.mean;
    s_sub[threadIdx.x * 3 + 2] = m.m2;
    __syncthreads();
    if (threadIdx.x < G) {
      Moments acc = {0.f, 0.f, 0.f};
      for (int k = 0; k < subs; ++k) {
        const int i = (k * G + g) * 3;
        Moments bm = {s_sub[i], s_sub[i + 1], s_sub[i + 2]};
        if (bm.n > 0.f) acc = merge_moments(acc, bm);
      }
      const float mean = acc.mean, rstd = rsqrtf(fmaxf(acc.m2 / acc.n, 0.f) + eps);
      s_st[g * 2 + 0] = mean;
      s_st[g * 2 + 1] = rstd;
      if (publish) {
        stats_out[(n * G + g) * 2 + 0] = mean;
        stats_out[(n * G + g) * 2 + 1] = rstd;
      }
    }
    __syncthreads();
    return;
  }
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    Moments m = {0.f, 0.f, 0.f};
    if (conv_parts > 0) {            // (G > NT)
      const float cnt = 64.f * Cg;
      const float* pp = part + ((long)n * G + g) * conv_parts * 2;
      for (int t = 0; t < conv_parts; ++t) {
        const float sm = pp[2 * t], q = pp[2 * t + 1];
        const float mean = sm / cnt;
        Moments bm = {cnt, mean, fmaxf(q - sm * mean, 0.f)};
        m = merge_moments(m, bm);
      }
    }
    for (int c = 0; c < (conv_parts > 0 ? 0 : nchunks); ++c) {
      const int q0 = c * rows, q1 = min(P, q0 + rows);
      const float* pp = part + (((long)n * nchunks + c) * G + g) * 2;
      Moments bm = {(float)((q1 - q0) * Cg), pp[0], pp[1]};
      m = merge_moments(m, bm);
    }
    const float mean = m.mean, rstd = rsqrtf(fmaxf(m.m2 / m.n, 0.f) + eps);
    s_st[g * 2 + 0] = mean;
    s_st[g * 2 + 1] = rstd;
    if (publish) {
      stats_out[(n * G + g) * 2 + 0] = mean;
      stats_out[(n * G + g) * 2 + 1] = rstd;
    }
  }
  __syncthreads();
}

// GN0 folded into the next conv's halo staging (conv.hip conv_halo_k GNA):
// per image the statistics, merged exactly as gn_apply2_k merges them (and
// published for the backward), and the apply's per-channel affine
// ab[n][c] = (A, B), A = rstd * gamma, B = beta - mean * A.
__global__ void __launch_bounds__(NT) gn_ab_k(const float* __restrict__ part, float* __restrict__ stats_out,
                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                              float* __restrict__ ab, int P, int C, int G, int rows, int nchunks,
                                              float eps, int conv_parts) {
  __shared__ float s_st[2 * 1024];
  const int n = blockIdx.x, Cg = C / G;
  merge_image_stats(part, n, nchunks, G, P, rows, Cg, eps, s_st, stats_out, true, conv_parts);
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g = c / Cg;
    const float A = s_st[g * 2 + 1] * gamma[c];
    const float B = beta[c] - s_st[g * 2] * A;
    ab[((long)n * C + c) * 2 + 0] = A;
    ab[((long)n * C + c) * 2 + 1] = B;
  }
}

// h = silu(x * A + B) from that table -- the conv's weight-gradient operand,
// rematerialised in the backward with the staging's exact arithmetic
__global__ void gn_ab_silu_k(const bf16* __restrict__ x, const float* __restrict__ ab, bf16* __restrict__ y,
                             long nvec, int C, long PC) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 8;
    const int c0 = (int)(e % C);
    const long n = e / PC;
    const f32x8 xv = ld8(x + e);
    const float* p = ab + (n * C + c0) * 2;
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)(bf16)siluf_(__builtin_fmaf(xv[j], p[2 * j], p[2 * j + 1]));
    st8(y + e, o);
  }
}

// Sum the backward's per-chunk group partials of image n (grp_part
// [N][nchunks][G] x 2) with every thread of the block (batched loads, fixed
// merge order): out[g] = (sum a, sum b).
__device__ __forceinline__ void sum_group_parts(const float* __restrict__ grp_part, int n, int nchunks, int G,
                                                float* s_out) {
  constexpr int B = 8;
  if (G <= NT) {
    __shared__ float s_sub[2 * NT];
    const int subs = NT / G;
    const int g = threadIdx.x % G, sub = threadIdx.x / G;
    float a = 0.f, b = 0.f;
    if (sub < subs) {
      for (int c0 = sub; c0 < nchunks; c0 += B * subs) {
        float u[B], v[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
          const int c = c0 + k * subs;
          const float* pp = grp_part + (((long)n * nchunks + c) * G + g) * 2;
          u[k] = c < nchunks ? pp[0] : 0.f;
          v[k] = c < nchunks ? pp[1] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
          a += u[k];
          b += v[k];
        }
      }
    }
    s_sub[threadIdx.x * 2 + 0] = a;
    s_sub[threadIdx.x * 2 + 1] = b;
    __syncthreads();
    if (threadIdx.x < G) {
      float x = 0.f, y = 0.f;
      for (int k = 0; k < subs; ++k) {
        x += s_sub[(k * G + g) * 2];
        y += s_sub[(k * G + g) * 2 + 1];
      }
      s_out[g * 2 + 0] = x;
      s_out[g * 2 + 1] = y;
    }
    __syncthreads();
    return;
  }
  for (int g = threadIdx.x; g < G; g += NT) {
    float a = 0.f, b = 0.f;
    for (int c = 0; c < nchunks; ++c) {
      const float* pp = grp_part + (((long)n * nchunks + c) * G + g) * 2;
      a += pp[0];
      b += pp[1];
    }
    s_out[g * 2 + 0] = a;
    s_out[g * 2 + 1] = b;
  }
  __syncthreads();
}

// MODE 0: GN, 1: GN+SiLU, 2: GN+FiLM(+dropout)
template <int MODE>
__global__ void __launch_bounds__(NT) gn_apply2_k(const bf16* __restrict__ x, const float* __restrict__ part,
                                                  float* __restrict__ stats_out, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, const bf16* __restrict__ ss,
                                                  bf16* __restrict__ y, int P, int C, int G, int rows, int nchunks,
                                                  float eps, float p_drop, uint64_t seed, int ssld,
                                                  const uint64_t* __restrict__ seed_dev, Cat cat, int conv_parts,
                                                  const int* __restrict__ ss_map) {
  constexpr int U = MODE == 2 ? 2 : UNR;      // rows in flight per thread
  __shared__ float s_st[2 * 1024];
  const int chunk = blockIdx.x, n = blockIdx.y;
  const int Cg = C / G;
  merge_image_stats(part, n, nchunks, G, P, rows, Cg, eps, s_st, stats_out, chunk == 0, conv_parts);
  if (MODE == 2 && seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  const int cv = C / 8, rpi = NT / cv;
  const int tid = threadIdx.x, roff = tid / cv;
  if (roff >= rpi) return;
  const int c0 = (tid % cv) * 8;
  // y = x * A + B with A = rstd * gamma, B = beta - mean * rstd * gamma
  float A[8], Bc[8];
  {
    const f32x8 gm = ld8f(gamma + c0), bt = ld8f(beta + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int g = (c0 + j) / Cg;
      A[j] = s_st[g * 2 + 1] * gm[j];
      Bc[j] = bt[j] - s_st[g * 2] * A[j];
    }
  }
  const RowSrc src = row_src(x, cat, c0, C);
  const long pix0 = (long)n * P;
  // shared conditioning (sampling): image n reads the modulation of
  // conditioning class ss_map[n] (engine/sampler.py)
  const long spix0 = (MODE == 2 && ss_map) ? (long)ss_map[n] * P : pix0;
  const int r1 = min(P, chunk * rows + rows);
  for (int r = chunk * rows + roff; r < r1; r += U * rpi) {
    f32x8 a[U], sc[U], sf[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rpi;
      if (rr < r1) {
        const long pix = pix0 + rr;
        a[u] = ld8(src.p + pix * src.ld);
        if (MODE == 2) {
          sc[u] = ld8(ss + (spix0 + rr) * ssld + c0);
          sf[u] = ld8(ss + (spix0 + rr) * ssld + C + c0);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rpi;
      if (rr >= r1) break;
      const long pix = pix0 + rr;
      const uint64_t e = (uint64_t)pix * C + c0;
      f32x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float h = a[u][j] * A[j] + Bc[j];
        if (MODE == 1) h = siluf_(h);
        if (MODE == 2) {
          h = h * (1.f + sc[u][j]) + sf[u][j];
          if (p_drop > 0.f) h = drop_elem(dkey, e + j, dthr) ? 0.f : h * keep_scale;
        }
        o[j] = h;
      }
      st8(y + pix * C + c0, o);
    }
  }
}

// ------------------------------------------------------------- backward ----
// MODE 0: plain GN, 1: GN+SiLU, 2: GN+FiLM(+dropout)
template <int MODE>
__device__ __forceinline__ void bwd_elem(float xv, float dyv, float mean, float rstd, float gm, float bt, float sc,
                                         float& xhat, float& dA, float& dscale, float& dshift, float keepmul) {
  xhat = (xv - mean) * rstd;
  float h = xhat * gm + bt;
  if (MODE == 0) {
    dA = dyv;
  } else if (MODE == 1) {
    dA = dyv * dsiluf_(h);
  } else {
    float dz = dyv * keepmul;
    dscale = dz * h;
    dshift = dz;
    dA = dz * (1.f + sc);
  }
}

template <int MODE, int U>
__global__ void __launch_bounds__(NT) gn_bwd_reduce_k(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                      const bf16* __restrict__ ss, const float* __restrict__ stats,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      int P, int C, int G, int rows, int nchunks, float p_drop,
                                                      uint64_t seed, bf16* __restrict__ dss,
                                                      float* __restrict__ chan_part, float* __restrict__ grp_part,
                                                      int ssld, const uint64_t* __restrict__ seed_dev, Cat cat) {
  if (seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][rpi][C]
  const int chunk = blockIdx.x, n = blockIdx.y;
  const int tpr = C / 8, rpi = NT / tpr;
  const int tid = threadIdx.x;
  const int roff = tid / tpr, v = tid % tpr, c0 = v * 8;
  const bool active = roff < rpi;
  const int r0 = chunk * rows, r1 = min(P, r0 + rows);
  const int Cg = C / G;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  float dg[8], db[8], gs[8], gs2[8], mean[8], rstd[8];
  f32x8 gm = {}, bt = {};
#pragma unroll
  for (int j = 0; j < 8; ++j) { dg[j] = db[j] = gs[j] = gs2[j] = 0.f; }
  if (active) {
    gm = ld8f(gamma + c0);
    bt = ld8f(beta + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int g = (c0 + j) / Cg;
      mean[j] = stats[(n * G + g) * 2];
      rstd[j] = stats[(n * G + g) * 2 + 1];
    }
    const RowSrc src = row_src(x, cat, c0, C);
    for (int r = r0 + roff; r < r1; r += U * rpi) {
      f32x8 xv[U], dv[U], sc[U];     // loads of U rows first (memory-level parallelism)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * rpi;
        if (rr < r1) {
          const long pix = (long)n * P + rr;
          xv[u] = ld8(src.p + pix * src.ld);
          dv[u] = ld8(dy + pix * C + c0);
          if (MODE == 2) sc[u] = ld8(ss + pix * ssld + c0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * rpi;
        if (rr >= r1) break;
        const long pix = (long)n * P + rr;
        const uint64_t e = (uint64_t)pix * C + c0;
        f32x8 o_s, o_t;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float keepmul = 1.f;
          if (MODE == 2 && p_drop > 0.f) keepmul = drop_elem(dkey, e + j, dthr) ? 0.f : keep_scale;
          float xhat, dA, dsc = 0.f, dsh = 0.f;
          bwd_elem<MODE>(xv[u][j], dv[u][j], mean[j], rstd[j], gm[j], bt[j], MODE == 2 ? sc[u][j] : 0.f, xhat, dA,
                         dsc, dsh, keepmul);
          o_s[j] = dsc;
          o_t[j] = dsh;
          dg[j] += dA * xhat;
          db[j] += dA;
          const float dxh = dA * gm[j];
          gs[j] += dxh;
          gs2[j] += dxh * xhat;
        }
        if (MODE == 2) {
          st8(dss + pix * ssld + c0, o_s);
          st8(dss + pix * ssld + C + c0, o_t);
        }
      }
    }
    // structure-of-arrays [4][rpi][C]: each thread's 8 channels are two
    // 16-byte stores.  (The interleaved [rpi][C][4] layout put every lane of
    // a wave on one bank: 86 % of the kernel's LDS cycles were conflicts,
    // profiles/r3/pmc_step/table_bs16.txt, a fixed cost per block that
    // dominated the small-batch calls.)
    const int SL = rpi * C;
    float* o = lds + roff * C + c0;
    *reinterpret_cast<f32x4*>(o) = f32x4{dg[0], dg[1], dg[2], dg[3]};
    *reinterpret_cast<f32x4*>(o + 4) = f32x4{dg[4], dg[5], dg[6], dg[7]};
    *reinterpret_cast<f32x4*>(o + SL) = f32x4{db[0], db[1], db[2], db[3]};
    *reinterpret_cast<f32x4*>(o + SL + 4) = f32x4{db[4], db[5], db[6], db[7]};
    *reinterpret_cast<f32x4*>(o + 2 * SL) = f32x4{gs[0], gs[1], gs[2], gs[3]};
    *reinterpret_cast<f32x4*>(o + 2 * SL + 4) = f32x4{gs[4], gs[5], gs[6], gs[7]};
    *reinterpret_cast<f32x4*>(o + 3 * SL) = f32x4{gs2[0], gs2[1], gs2[2], gs2[3]};
    *reinterpret_cast<f32x4*>(o + 3 * SL + 4) = f32x4{gs2[4], gs2[5], gs2[6], gs2[7]};
  }
  __syncthreads();
  const int SL = rpi * C;
  const long prow = (long)n * nchunks + chunk, R = (long)gridDim.y * nchunks;
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < rpi; ++rr) {
      a += lds[rr * C + c];
      b += lds[SL + rr * C + c];
    }
    chan_part[(2L * c) * R + prow] = a;         // [2C][R]: one contiguous row per dgamma / dbeta entry
    chan_part[(2L * c + 1) * R + prow] = b;
  }
  // group sums: TPG consecutive lanes per group (a power of two <= 64, so a
  // group never straddles a wave), each summing a strided share of the
  // group's rpi x Cg entries, then a fixed-order butterfly (deterministic)
  int TPG = 1;
  while (TPG < 64 && TPG * 2 * G <= NT) TPG <<= 1;
  const int E = rpi * Cg;
  for (int g0 = 0; g0 < G; g0 += NT / TPG) {
    const int g = g0 + tid / TPG, sub = tid % TPG;
    float a = 0.f, b = 0.f;
    if (g < G)
      for (int e = sub; e < E; e += TPG) {
        const int rr = e / Cg, cc = e - rr * Cg;
        a += lds[2 * SL + rr * C + g * Cg + cc];
        b += lds[3 * SL + rr * C + g * Cg + cc];
      }
    for (int w = 1; w < TPG; w <<= 1) {
      a += __shfl_xor(a, w);
      b += __shfl_xor(b, w);
    }
    if (g < G && sub == 0) {
      grp_part[(prow * G + g) * 2 + 0] = a;
      grp_part[(prow * G + g) * 2 + 1] = b;
    }
  }
}

__global__ void gn_bwd_coef_k(const float* __restrict__ grp_part, int N, int P, int C, int G, int nchunks,
                              float* __restrict__ coef) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * G) return;
  int n = t / G, g = t % G;
  float a = 0.f, b = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const float* p = grp_part + (((long)n * nchunks + c) * G + g) * 2;
    a += p[0];
    b += p[1];
  }
  float inv = 1.f / (float)((long)P * (C / G));
  coef[t * 2 + 0] = a * inv;
  coef[t * 2 + 1] = b * inv;
}

template <int MODE>
__global__ void gn_bwd_apply_k(const bf16* __restrict__ x, const bf16* __restrict__ dy, const bf16* __restrict__ ss,
                               const float* __restrict__ stats, const float* __restrict__ coef,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               bf16* __restrict__ dx, long nvec, int C, int Cg, int G, long PC, float p_drop,
                               uint64_t seed, int ssld, const uint64_t* __restrict__ seed_dev) {
  if (seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    long e = i * 8;
    int c0 = (int)(e % C);
    long pix = e / C;
    int n = (int)(e / PC);
    f32x8 xv = ld8(x + e), dv = ld8(dy + e);
    f32x8 sc = {};
    if (MODE == 2) sc = ld8(ss + pix * ssld + c0);
    f32x8 gm = ld8f(gamma + c0), bt = ld8f(beta + c0);
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int g = (c0 + j) / Cg;
      float mean = stats[(n * G + g) * 2], rstd = stats[(n * G + g) * 2 + 1];
      float c1 = coef[(n * G + g) * 2], c2 = coef[(n * G + g) * 2 + 1];
      float keepmul = 1.f;
      if (MODE == 2 && p_drop > 0.f) keepmul = drop_elem(dkey, (uint64_t)(e + j), dthr) ? 0.f : keep_scale;
      float xhat, dA, dsc, dsh;
      bwd_elem<MODE>(xv[j], dv[j], mean, rstd, gm[j], bt[j], sc[j], xhat, dA, dsc, dsh, keepmul);
      float dxh = dA * gm[j];
      o[j] = rstd * (dxh - c1 - xhat * c2);
    }
    st8(dx + e, o);
  }
}

// Chunked backward apply with the per-image group coefficients merged in
// LDS from the reduce pass's partials (replaces gn_bwd_coef_k + gn_bwd_apply_k).
// dgamma / dbeta of the backward: chan_part is [2C][R] (R = images x
// chunks; row 2c -> dgamma[c], row 2c+1 -> dbeta[c]); one wave sums one
// contiguous row in a fixed order (8 accumulators per lane, butterfly).  Run
// by the leading rows of gn_bwd_apply2_k's grid (dispatched first, they
// overlap the apply work): replaces two colsum launches per backward.
__device__ __forceinline__ void dgb_rowsum(const float* __restrict__ part, long R, int nrows, int row,
                                           float* __restrict__ dgamma, float* __restrict__ dbeta, int acc) {
  if (row >= nrows) return;
  const int lane = threadIdx.x & 63;
  const float* src = part + (long)row * R;
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 0.f;
  long i = lane;
  for (; i + 7 * 64 < R; i += 8 * 64)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += src[i + k * 64];
  for (int k = 0; i < R; i += 64, ++k) a[k & 7] += src[i];
  float t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, 64);
  if (lane == 0) {
    float* o = (row & 1) ? dbeta + (row >> 1) : dgamma + (row >> 1);
    *o = acc ? *o + t : t;
  }
}

template <int MODE, int U>
__global__ void __launch_bounds__(NT) gn_bwd_apply2_k(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                      const bf16* __restrict__ ss, const float* __restrict__ stats,
                                                      const float* __restrict__ grp_part,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      bf16* __restrict__ dx, int P, int C, int G, int rows,
                                                      int nchunks, float p_drop, uint64_t seed, int ssld,
                                                      const uint64_t* __restrict__ seed_dev, Cat cat,
                                                      const float* __restrict__ chan_part,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      int accumulate, int trows, const bf16* __restrict__ dres,
                                                      float dres_scale, long chan_R, const bf16* __restrict__ dres2,
                                                      float dres2_scale) {
  // chan_R: rows of chan_part (the reduce pass's per-block dgamma / dbeta partials)
  if ((int)blockIdx.y < trows) {        // leading grid rows: dgamma / dbeta, 4 rows (waves) per block
    const int blk = blockIdx.y * nchunks + blockIdx.x;
    dgb_rowsum(chan_part, chan_R, 2 * C, blk * (NT / 64) + (threadIdx.x >> 6), dgamma, dbeta, accumulate);
    return;
  }
  __shared__ __attribute__((aligned(16))) float s_c[4 * 1024];      // per group: mean, rstd, c1, c2
  const int chunk = blockIdx.x, n = blockIdx.y - trows;
  const int Cg = C / G;
  const float inv = 1.f / (float)((long)P * Cg);
  __shared__ float s_ab[2 * 1024];
  sum_group_parts(grp_part, n, nchunks, G, s_ab);
  for (int g = threadIdx.x; g < G; g += NT) {
    s_c[g * 4 + 0] = stats[(n * G + g) * 2];
    s_c[g * 4 + 1] = stats[(n * G + g) * 2 + 1];
    s_c[g * 4 + 2] = s_ab[g * 2] * inv;
    s_c[g * 4 + 3] = s_ab[g * 2 + 1] * inv;
  }
  __syncthreads();
  if (MODE == 2 && seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  const int cv = C / 8, rpi = NT / cv;
  const int tid = threadIdx.x, roff = tid / cv;
  if (roff >= rpi) return;
  const int c0 = (tid % cv) * 8;
  float mean[8], rstd[8], c1[8], c2[8], gm[8], bt[8];
  {
    const f32x8 g8 = ld8f(gamma + c0), b8 = ld8f(beta + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int g = (c0 + j) / Cg;
      mean[j] = s_c[g * 4];
      rstd[j] = s_c[g * 4 + 1];
      c1[j] = s_c[g * 4 + 2];
      c2[j] = s_c[g * 4 + 3];
      gm[j] = g8[j];
      bt[j] = b8[j];
    }
  }
  const RowSrc src = row_src(x, cat, c0, C);
  bf16* dst;
  long dld;
  if (cat.x2 == nullptr) { dst = dx + c0; dld = C; }
  else if (c0 < cat.C1) { dst = dx + c0; dld = cat.C1; }
  else { dst = cat.dx2 + (c0 - cat.C1); dld = C - cat.C1; }
  const long pix0 = (long)n * P;
  const int r1 = min(P, chunk * rows + rows);
  for (int r = chunk * rows + roff; r < r1; r += U * rpi) {
    f32x8 xv[U], dv[U], sc[U], rv[U], rv2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rpi;
      if (rr < r1) {
        const long pix = pix0 + rr;
        xv[u] = ld8(src.p + pix * src.ld);
        dv[u] = ld8(dy + pix * C + c0);
        if (MODE == 2) sc[u] = ld8(ss + pix * ssld + c0);
        if (dres) rv[u] = ld8(dres + pix * C + c0);
        if (dres2) rv2[u] = ld8(dres2 + pix * C + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rpi;
      if (rr >= r1) break;
      const long pix = pix0 + rr;
      const uint64_t e = (uint64_t)pix * C + c0;
      f32x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float keepmul = 1.f;
        if (MODE == 2 && p_drop > 0.f) keepmul = drop_elem(dkey, e + j, dthr) ? 0.f : keep_scale;
        float xhat, dA, dsc, dsh;
        bwd_elem<MODE>(xv[u][j], dv[u][j], mean[j], rstd[j], gm[j], bt[j], MODE == 2 ? sc[u][j] : 0.f, xhat, dA,
                       dsc, dsh, keepmul);
        const float dxh = dA * gm[j];
        o[j] = rstd[j] * (dxh - c1[j] - xhat * c2[j]);
      }
      if (dres) o += rv[u] * dres_scale;    // the residual branch's gradient of the same input
      if (dres2) o += rv2[u] * dres2_scale;  // ... and a second consumer's (a decoder skip, models/xunet.py)
      st8(dst + pix * dld, o);
    }
  }
}

// ------------------------------------------------ whole-image kernels ----
// The 16x16 / 8x8 levels (and 32x32 on request): a block owns ONE image x a
// slab of CS channels (whole groups; CS / 8 threads per pixel row, rpi rows
// per pass, U rows per thread) and holds the slab in registers, so every
// statistic the pass needs is reduced inside the block and the pass is ONE
// launch that reads its inputs once, all loads issued up front:
//   forward : statistics (two-pass mean / M2 over the registers) + apply
//             [+ SiLU | + FiLM + dropout] -- no statistics pass, no partials
//             merge, and mean / rstd published for the backward;
//   backward: the group reductions (sum dA*gamma, sum dA*gamma*xhat) AND the
//             apply -- one launch instead of the reduce + apply pair -- plus
//             per-image dgamma / dbeta rows that a column sum (off the
//             critical path, on the weight-gradient stream) folds over images.
// At 32 images of 16x16x256 the chunked pair ran at 0.4-1.2 TB/s, latency
// bound: 128 blocks with a few rows each, three dependent round trips
// (partials -> statistics -> data) per pass.  Reductions are fixed-order
// (column sums over the row lanes, then the group's columns): deterministic.
struct ImgGeom {
  int cv, rpi, tid, roff, v, c0, lg, gs;   // lanes per row, rows per pass, thread, row lane, column, channel, group
  bool act;
};

__device__ __forceinline__ ImgGeom img_geom(int NTI, int CS, int Cg) {
  ImgGeom g;
  g.cv = CS / 8;
  g.rpi = NTI / g.cv;
  g.tid = threadIdx.x;
  g.roff = g.tid / g.cv;
  g.v = g.tid - g.roff * g.cv;
  g.act = g.roff < g.rpi;
  g.c0 = blockIdx.x * CS + g.v * 8;
  g.lg = g.v * 8 / Cg;                     // group within the slab (Cg % 8 == 0: one per thread)
  g.gs = CS / Cg;
  return g;
}

// K values per thread -> per-group block sums (every thread gets its group's
// K totals).  red: LDS [K][NTI] + [K][cv]; fixed order.
template <int K>
__device__ __forceinline__ void img_group_sum(float (&val)[K], float* red, const ImgGeom& g, int NTI, int Cg) {
#pragma unroll
  for (int k = 0; k < K; ++k) red[k * NTI + g.tid] = g.act ? val[k] : 0.f;
  __syncthreads();
  float* col = red + K * NTI;
  if (g.tid < K * g.cv) {                  // column sums over the row lanes
    const int k = g.tid / g.cv, c = g.tid - k * g.cv;
    float a = 0.f;
    for (int r = 0; r < g.rpi; ++r) a += red[k * NTI + r * g.cv + c];
    col[k * g.cv + c] = a;
  }
  __syncthreads();
  const int c8 = Cg / 8;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float a = 0.f;
    for (int j = 0; j < c8; ++j) a += col[k * g.cv + g.lg * c8 + j];
    val[k] = a;
  }
  __syncthreads();                         // red / col may be reused right after
}

template <int NTI, int U, int MODE>
__global__ void __launch_bounds__(NTI) gn_img_fwd_k(const bf16* __restrict__ x, float* __restrict__ stats_out,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    const bf16* __restrict__ ss, bf16* __restrict__ y, int P, int C,
                                                    int G, int CS, float eps, float p_drop, uint64_t seed, int ssld,
                                                    const uint64_t* __restrict__ seed_dev, Cat cat,
                                                    const int* __restrict__ ss_map) {
  __shared__ float red[2 * NTI + 2 * 64];
  const int Cg = C / G, n = blockIdx.y;
  const ImgGeom g = img_geom(NTI, CS, Cg);
  const RowSrc src = row_src(x, cat, g.act ? g.c0 : 0, C);
  const long pix0 = (long)n * P;
  const long spix0 = (MODE == 2 && ss_map) ? (long)ss_map[n] * P : pix0;
  bf16x8 a[U], sc[U], sf[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {            // every load of the slab issued up front
    const int r = g.roff + u * g.rpi;
    if (g.act && r < P) {
      a[u] = *reinterpret_cast<const bf16x8*>(src.p + (pix0 + r) * src.ld);
      if (MODE == 2) {
        sc[u] = *reinterpret_cast<const bf16x8*>(ss + (spix0 + r) * ssld + g.c0);
        sf[u] = *reinterpret_cast<const bf16x8*>(ss + (spix0 + r) * ssld + C + g.c0);
      }
    }
  }
  const float inv = 1.f / (float)((long)P * Cg);
  float m[1] = {0.f};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (g.act && g.roff + u * g.rpi < P)
#pragma unroll
      for (int j = 0; j < 8; ++j) m[0] += (float)a[u][j];
  img_group_sum<1>(m, red, g, NTI, Cg);
  const float mean = m[0] * inv;
  float q[1] = {0.f};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (g.act && g.roff + u * g.rpi < P)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)a[u][j] - mean;
        q[0] += d * d;
      }
  img_group_sum<1>(q, red, g, NTI, Cg);
  const float rstd = rsqrtf(fmaxf(q[0] * inv, 0.f) + eps);
  if (!g.act) return;
  if (g.roff == 0 && (g.v * 8) % Cg == 0) {   // one thread per group publishes mean / rstd
    const int gg = g.c0 / Cg;
    stats_out[((long)n * G + gg) * 2 + 0] = mean;
    stats_out[((long)n * G + gg) * 2 + 1] = rstd;
  }
  if (MODE == 2 && seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  float A[8], Bc[8];
  {
    const f32x8 gm = ld8f(gamma + g.c0), bt = ld8f(beta + g.c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      A[j] = rstd * gm[j];
      Bc[j] = bt[j] - mean * A[j];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = g.roff + u * g.rpi;
    if (r >= P) break;
    const long pix = pix0 + r;
    const uint64_t e = (uint64_t)pix * C + g.c0;
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float h = (float)a[u][j] * A[j] + Bc[j];
      if (MODE == 1) h = siluf_(h);
      if (MODE == 2) {
        h = h * (1.f + (float)sc[u][j]) + (float)sf[u][j];
        if (p_drop > 0.f) h = drop_elem(dkey, e + j, dthr) ? 0.f : h * keep_scale;
      }
      o[j] = h;
    }
    st8(y + pix * C + g.c0, o);
  }
}

template <int NTI, int U, int MODE>
__global__ void __launch_bounds__(NTI) gn_img_bwd_k(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                    const bf16* __restrict__ ss, const float* __restrict__ stats,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    bf16* __restrict__ dx, bf16* __restrict__ dss,
                                                    float* __restrict__ chan_out, int P, int C, int G, int CS,
                                                    float p_drop, uint64_t seed, int ssld,
                                                    const uint64_t* __restrict__ seed_dev, Cat cat,
                                                    const bf16* __restrict__ dres, float dres_scale,
                                                    const bf16* __restrict__ dres2, float dres2_scale) {
  // red: [2][NTI] group partials + columns; later [2][rpi][CS] channel partials (<= 2 * NTI * 8)
  __shared__ __attribute__((aligned(16))) float red[16 * NTI];
  const int Cg = C / G, n = blockIdx.y;
  const ImgGeom g = img_geom(NTI, CS, Cg);
  const int c0 = g.act ? g.c0 : 0;
  const RowSrc src = row_src(x, cat, c0, C);
  const long pix0 = (long)n * P;
  bf16x8 xv[U], dv[U], sc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = g.roff + u * g.rpi;
    if (g.act && r < P) {
      xv[u] = *reinterpret_cast<const bf16x8*>(src.p + (pix0 + r) * src.ld);
      dv[u] = *reinterpret_cast<const bf16x8*>(dy + (pix0 + r) * C + c0);
      if (MODE == 2) sc[u] = *reinterpret_cast<const bf16x8*>(ss + (pix0 + r) * ssld + c0);
    }
  }
  const int gg = c0 / Cg;
  const float mean = stats[((long)n * G + gg) * 2], rstd = stats[((long)n * G + gg) * 2 + 1];
  if (MODE == 2 && seed_dev) seed += *seed_dev * 0x9E3779B97F4A7C15ull;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = drop_key(seed), dthr = drop_threshold(p_drop);
  const f32x8 gm = ld8f(gamma + c0), bt = ld8f(beta + c0);
  float dg[8], db[8], gsum[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) dg[j] = db[j] = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = g.roff + u * g.rpi;
    if (!g.act || r >= P) break;
    const long pix = pix0 + r;
    const uint64_t e = (uint64_t)pix * C + c0;
    f32x8 o_s, o_t;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float keepmul = 1.f;
      if (MODE == 2 && p_drop > 0.f) keepmul = drop_elem(dkey, e + j, dthr) ? 0.f : keep_scale;
      float xhat, dA, dsc = 0.f, dsh = 0.f;
      bwd_elem<MODE>((float)xv[u][j], (float)dv[u][j], mean, rstd, gm[j], bt[j], MODE == 2 ? (float)sc[u][j] : 0.f,
                     xhat, dA, dsc, dsh, keepmul);
      o_s[j] = dsc;
      o_t[j] = dsh;
      dg[j] += dA * xhat;
      db[j] += dA;
      const float dxh = dA * gm[j];
      gsum[0] += dxh;
      gsum[1] += dxh * xhat;
    }
    if (MODE == 2) {
      st8(dss + pix * ssld + c0, o_s);
      st8(dss + pix * ssld + C + c0, o_t);
    }
  }
  img_group_sum<2>(gsum, red, g, NTI, Cg);
  const float inv = 1.f / (float)((long)P * Cg);
  const float c1 = gsum[0] * inv, c2 = gsum[1] * inv;
  // per-image dgamma / dbeta of the slab's channels: [rpi][CS] x 2 in LDS,
  // column sums over the row lanes -> chan_out row n ([N][C] pairs (dg, db))
  {
    const int SL = g.rpi * CS;
    if (g.act) {
      float* o = red + g.roff * CS + g.v * 8;
      *reinterpret_cast<f32x4*>(o) = f32x4{dg[0], dg[1], dg[2], dg[3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{dg[4], dg[5], dg[6], dg[7]};
      *reinterpret_cast<f32x4*>(o + SL) = f32x4{db[0], db[1], db[2], db[3]};
      *reinterpret_cast<f32x4*>(o + SL + 4) = f32x4{db[4], db[5], db[6], db[7]};
    }
    __syncthreads();
    for (int t = g.tid; t < 2 * CS; t += NTI) {
      const int k = t / CS, c = t - k * CS;
      float a = 0.f;
      for (int r = 0; r < g.rpi; ++r) a += red[k * SL + r * CS + c];
      chan_out[((long)n * C + blockIdx.x * CS + c) * 2 + k] = a;
    }
  }
  if (!g.act) return;
  bf16* dst;
  long dld;
  if (cat.x2 == nullptr) { dst = dx + c0; dld = C; }
  else if (c0 < cat.C1) { dst = dx + c0; dld = cat.C1; }
  else { dst = cat.dx2 + (c0 - cat.C1); dld = C - cat.C1; }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = g.roff + u * g.rpi;
    if (r >= P) break;
    const long pix = pix0 + r;
    const uint64_t e = (uint64_t)pix * C + c0;
    f32x8 rv = {}, rv2 = {};
    if (dres) rv = ld8(dres + pix * C + c0);
    if (dres2) rv2 = ld8(dres2 + pix * C + c0);
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float keepmul = 1.f;
      if (MODE == 2 && p_drop > 0.f) keepmul = drop_elem(dkey, e + j, dthr) ? 0.f : keep_scale;
      float xhat, dA, dsc, dsh;
      bwd_elem<MODE>((float)xv[u][j], (float)dv[u][j], mean, rstd, gm[j], bt[j], MODE == 2 ? (float)sc[u][j] : 0.f,
                     xhat, dA, dsc, dsh, keepmul);
      o[j] = rstd * (dA * gm[j] - c1 - xhat * c2);
    }
    if (dres) o += rv * dres_scale;
    if (dres2) o += rv2 * dres2_scale;
    st8(dst + pix * dld, o);
  }
}

// Launch geometry of the whole-image kernels, or ok = 0 when the shape is
// outside them: groups of whole 8-channel vectors, the slab's rows in <= 8
// registers per thread of a 256 / 512-thread block, images up to max_p pixels.
struct ImgPlan {
  int ok, CS, NTI, U;
};
static int g_gn_img_maxp = 256;            // 0: whole-image kernels off (A/B knob, d3d_gn_img_cfg)
// Batches of g_gn_img_wide_lo..hi images also take the 512-thread form at the
// 32x32 level: measured +0.5..1.2 % of the step at 64 / 128 images, but
// -2.0 % at 32 (too few blocks) and -0.9 % at 256 (the chunked kernels
// stream better) -- profiles/r6/knob_sweep_b128.txt.  d3d_gn_img_wide_cfg.
static int g_gn_img_wide_lo = 64, g_gn_img_wide_hi = 128;

ImgPlan img_plan(int P, int C, int G, int N = 0) {
  ImgPlan p{0, 0, 0, 0};
  int maxp = g_gn_img_maxp;
  if (maxp > 0 && maxp < 1024 && N >= g_gn_img_wide_lo && N <= g_gn_img_wide_hi) maxp = 1024;
  if (G <= 0 || C % G || C > 4096 || P < 1 || P > maxp) return p;
  const int Cg = C / G;
  if (Cg % 8) return p;
  int CS = C;
  for (int k = Cg; k < C; k += Cg)
    if (C % k == 0 && k >= 32) { CS = k; break; }
  const int cv = CS / 8;
  for (int nt = 256; nt <= 512; nt *= 2) {
    if (cv > nt) continue;
    const int rpi = nt / cv;
    const int u = (P + rpi - 1) / rpi;
    if (u > 8) continue;
    p.U = u <= 1 ? 1 : u <= 2 ? 2 : u <= 4 ? 4 : 8;
    p.NTI = nt;
    p.CS = CS;
    p.ok = 1;
    return p;
  }
  return p;
}

inline int ew_grid(long nvec) {
  long g = (nvec + 255) / 256;
  if (g > 256L * 16) g = 256L * 16;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// =============================================================== C ABI ====
// Launch-shape knobs (kbench sweeps): blocks per launch, rows in flight per
// thread of the backward reduce (1, 2) and apply (1, 2, 4).  0 keeps a value.
D3D_API int d3d_gn_cfg(int blocks, int red_u, int app_u) {
  if (blocks > 0) g_gn_blocks = blocks;
  if (red_u > 0) g_gn_red_u = red_u;
  if (app_u > 0) g_gn_app_u = app_u;
  return 0;
}

D3D_API int d3d_gn_cfg_small(int max_n, int blocks) {
  if (max_n >= 0) { g_gn_small_n = max_n; g_gn_small_blocks = blocks; }
  return g_gn_small_n;
}

D3D_API int d3d_gn_plan(int N, int P, int C, int* nchunks, int* rows) {
  Plan p = make_plan(N, P, C);
  *nchunks = p.nchunks;
  *rows = p.rows;
  return 0;
}

// stats: [N*G*2] fp32 (mean, rstd); part: workspace [N*nchunks*G*2]
D3D_API int d3d_gn_stats(const void* x, int N, int P, int C, int G, float eps, float* part, float* stats,
                         const void* x2, int C1, hipStream_t st) {
  Plan p = make_plan(N, P, C);
  size_t lds = (size_t)p.rpi * C * 3 * sizeof(float);
  Cat cat{(const bf16*)x2, nullptr, C1};
  hipLaunchKernelGGL(gn_stats_partial_k, dim3(p.nchunks, N), dim3(NT), lds, st, (const bf16*)x, P, C, G, p.rows,
                     p.nchunks, part, cat);
  if (stats)     // legacy form: finalize separately (the fused apply path passes stats = nullptr)
    hipLaunchKernelGGL(gn_stats_final_k, dim3(cdiv((long)N * G, 256)), dim3(256), 0, st, part, N, P, G, C / G,
                       p.rows, p.nchunks, eps, stats);
  return (int)hipGetLastError();
}

// Fused finalize + apply over the statistics pass's partials (part from
// d3d_gn_stats with stats = nullptr).  mode 0 GN, 1 GN+SiLU, 2 GN+FiLM(+dropout;
// ss [N,P,ssld]).  stats_out receives mean / rstd for the backward pass.
D3D_API int d3d_gn_apply2(int mode, const void* x, const float* part, float* stats_out, const float* gamma,
                          const float* beta, const void* ss, void* y, int N, int P, int C, int G, float eps,
                          float p_drop, unsigned long long seed, int ssld, const void* seed_dev, const void* x2,
                          int C1, int conv_parts, const int* ss_map, hipStream_t st) {
  if (G > 1024) return (int)hipErrorInvalidValue;
  Cat cat{(const bf16*)x2, nullptr, C1};
  Plan p = make_plan(N, P, C);
  if (ssld == 0) ssld = 2 * C;
#define AP(M)                                                                                                   \
  hipLaunchKernelGGL(gn_apply2_k<M>, dim3(p.nchunks, N), dim3(NT), 0, st, (const bf16*)x, part, stats_out, gamma, \
                     beta, (const bf16*)ss, (bf16*)y, P, C, G, p.rows, p.nchunks, eps, p_drop, (uint64_t)seed, ssld, \
                     (const uint64_t*)seed_dev, cat, conv_parts, ss_map)
  if (mode == 0) AP(0);
  else if (mode == 1) AP(1);
  else AP(2);
#undef AP
  return (int)hipGetLastError();
}

// GN0 statistics + per-(image, channel) affine for conv_halo_k's GroupNorm
// staging (part / conv_parts as d3d_gn_apply2's); stats_out for the backward.
D3D_API int d3d_gn_ab(const float* part, float* stats_out, const float* gamma, const float* beta, float* ab, int N,
                      int P, int C, int G, float eps, int conv_parts, hipStream_t st) {
  if (G > 1024) return (int)hipErrorInvalidValue;
  Plan p = make_plan(N, P, C);
  hipLaunchKernelGGL(gn_ab_k, dim3(N), dim3(NT), 0, st, part, stats_out, gamma, beta, ab, P, C, G, p.rows, p.nchunks,
                     eps, conv_parts);
  return (int)hipGetLastError();
}

D3D_API int d3d_gn_ab_silu(const void* x, const float* ab, void* y, int N, int P, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long nvec = (long)N * P * C / 8;
  hipLaunchKernelGGL(gn_ab_silu_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, ab, (bf16*)y, nvec, C,
                     (long)P * C);
  return (int)hipGetLastError();
}

D3D_API int d3d_gn_apply(const void* x, const float* stats, const float* gamma, const float* beta, void* y, int N,
                         int P, int C, int G, int silu, hipStream_t st) {
  long nvec = (long)N * P * C / 8;
  if (silu)
    hipLaunchKernelGGL(gn_apply_k<true>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, stats, gamma, beta,
                       (bf16*)y, nvec, C, C / G, G, (long)P * C);
  else
    hipLaunchKernelGGL(gn_apply_k<false>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, stats, gamma, beta,
                       (bf16*)y, nvec, C, C / G, G, (long)P * C);
  return (int)hipGetLastError();
}

// ss: [N, P, ssld] bf16 with scale at channel c and shift at C + c (ssld >= 2C;
// ssld > 2C when ss is a column slice of a level-batched FiLM projection).
D3D_API int d3d_gn_film(const void* x, const float* stats, const float* gamma, const float* beta, const void* ss,
                        void* y, int N, int P, int C, int G, float p_drop, unsigned long long seed, int ssld,
                        const void* seed_dev, hipStream_t st) {
  long nvec = (long)N * P * C / 8;
  hipLaunchKernelGGL(gn_film_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, stats, gamma, beta,
                     (const bf16*)ss, (bf16*)y, nvec, C, C / G, G, (long)P * C, p_drop, (uint64_t)seed,
                     ssld ? ssld : 2 * C, (const uint64_t*)seed_dev);
  return (int)hipGetLastError();
}

// mode: 0 plain, 1 silu, 2 film.  Workspaces: chan_part [2C][N*nchunks],
// grp_part [N*nchunks*G*2 + 64*2*C] (tail = column-sum partials), coef [N*G*2].  Outputs dx (bf16), dgamma/dbeta
// (fp32 [C]) and, for mode 2, dss (bf16 [N,P,2C]).
D3D_API int d3d_gn_bwd2(int mode, const void* x, const void* dy, const void* ss, const float* stats,
                        const float* gamma, const float* beta, int N, int P, int C, int G, float p_drop,
                        unsigned long long seed, void* dx, void* dss, float* dgamma, float* dbeta, float* chan_part,
                        float* grp_part, float* coef, int accumulate, int ssld, const void* seed_dev,
                        const void* x2, void* dx2, int C1, const void* dres, float dres_scale, const void* dres2,
                        float dres2_scale, hipStream_t st) {
  Plan p = make_plan(N, P, C);
  Cat cat{(const bf16*)x2, (bf16*)dx2, C1};
  if (ssld == 0) ssld = 2 * C;
  if (x2) dres = dres2 = nullptr;          // (the caller never combines the two)
  size_t lds = (size_t)p.rpi * C * 4 * sizeof(float);
  dim3 g(p.nchunks, N);
#define RED1(M, U)                                                                                                \
  hipLaunchKernelGGL((gn_bwd_reduce_k<M, U>), g, dim3(NT), lds, st, (const bf16*)x, (const bf16*)dy, (const bf16*)ss, \
                     stats, gamma, beta, P, C, G, p.rows, p.nchunks, p_drop, (uint64_t)seed, (bf16*)dss,          \
                     chan_part, grp_part, ssld, (const uint64_t*)seed_dev, cat)
#define RED(M) if (g_gn_red_u == 2) RED1(M, 2); else RED1(M, 1)
  if (mode == 0) RED(0);
  else if (mode == 1) RED(1);
  else RED(2);
#undef RED
#undef RED1
  // dgamma/dbeta: chan_part is [2C][N*nchunks] -> 2C row sums, 4 per block,
  // by `trows` leading rows of the apply grid
  if (G > 1024) return (int)hipErrorInvalidValue;
  const int tblocks = (2 * C + NT / 64 - 1) / (NT / 64);
  const int trows = (tblocks + p.nchunks - 1) / p.nchunks;
#define APP1(M, U)                                                                                                \
  hipLaunchKernelGGL((gn_bwd_apply2_k<M, U>), dim3(p.nchunks, N + trows), dim3(NT), 0, st, (const bf16*)x,             \
                     (const bf16*)dy, (const bf16*)ss, stats, grp_part, gamma, beta, (bf16*)dx, P, C, G, p.rows,    \
                     p.nchunks, p_drop, (uint64_t)seed, ssld, (const uint64_t*)seed_dev, cat, chan_part, dgamma,    \
                     dbeta, accumulate, trows, (const bf16*)dres, dres_scale, (long)N * p.nchunks,                  \
                     (const bf16*)dres2, dres2_scale)
#define APP(M) if (g_gn_app_u == 4) APP1(M, 4); else if (g_gn_app_u == 1) APP1(M, 1); else APP1(M, 2)
  if (mode == 0) APP(0);
  else if (mode == 1) APP(1);
  else APP(2);
#undef APP
#undef APP1
  return (int)hipGetLastError();
}

D3D_API int d3d_gn_bwd(int mode, const void* x, const void* dy, const void* ss, const float* stats,
                       const float* gamma, const float* beta, int N, int P, int C, int G, float p_drop,
                       unsigned long long seed, void* dx, void* dss, float* dgamma, float* dbeta, float* chan_part,
                       float* grp_part, float* coef, hipStream_t st) {
  return d3d_gn_bwd2(mode, x, dy, ss, stats, gamma, beta, N, P, C, G, p_drop, seed, dx, dss, dgamma, dbeta,
                     chan_part, grp_part, coef, 0, 0, nullptr, nullptr, nullptr, 0, nullptr, 1.f, nullptr, 1.f, st);
}

// ------------------------------------------------ whole-image C ABI ----
D3D_API int d3d_gn_img_cfg(int max_p) {
  if (max_p >= 0) g_gn_img_maxp = max_p;
  return g_gn_img_maxp;
}

D3D_API int d3d_gn_img_wide_cfg(int lo, int hi) {
  if (lo >= 0) { g_gn_img_wide_lo = lo; g_gn_img_wide_hi = hi; }
  return g_gn_img_wide_lo;
}

D3D_API int d3d_gn_img_ok(int P, int C, int G) { return img_plan(P, C, G).ok; }
D3D_API int d3d_gn_img_ok_n(int N, int P, int C, int G) { return img_plan(P, C, G, N).ok; }

// Forward in one launch (statistics from the registers + apply); stats_out
// [N][G] (mean, rstd).  mode 0 GN, 1 GN+SiLU, 2 GN+FiLM(+dropout).
D3D_API int d3d_gn_img_fwd(int mode, const void* x, float* stats_out, const float* gamma, const float* beta,
                           const void* ss, void* y, int N, int P, int C, int G, float eps, float p_drop,
                           unsigned long long seed, int ssld, const void* seed_dev, const void* x2, int C1,
                           const int* ss_map, hipStream_t st) {
  const ImgPlan p = img_plan(P, C, G, N);
  if (!p.ok) return (int)hipErrorInvalidValue;
  Cat cat{(const bf16*)x2, nullptr, C1};
  if (ssld == 0) ssld = 2 * C;
  const dim3 grid(C / p.CS, N);
#define IF1(NT_, U_, M_)                                                                                            \
  hipLaunchKernelGGL((gn_img_fwd_k<NT_, U_, M_>), grid, dim3(NT_), 0, st, (const bf16*)x, stats_out, gamma, beta,  \
                     (const bf16*)ss, (bf16*)y, P, C, G, p.CS, eps, p_drop, (uint64_t)seed, ssld,                 \
                     (const uint64_t*)seed_dev, cat, ss_map)
#define IFU(NT_, M_)                                                                                                \
  if (p.U == 1) IF1(NT_, 1, M_); else if (p.U == 2) IF1(NT_, 2, M_); else if (p.U == 4) IF1(NT_, 4, M_);        \
  else IF1(NT_, 8, M_)
#define IFM(M_) if (p.NTI == 256) { IFU(256, M_); } else { IFU(512, M_); }
  if (mode == 0) { IFM(0); }
  else if (mode == 1) { IFM(1); }
  else { IFM(2); }
#undef IFM
#undef IFU
#undef IF1
  return (int)hipGetLastError();
}

// Backward in one launch: dx (+ dss for mode 2) and per-image dgamma / dbeta
// rows chan_out [N][C][2] (fold them over images with d3d_colsum(chan_out, N,
// 2C, ...) -> dgamma, dbeta).
D3D_API int d3d_gn_img_bwd(int mode, const void* x, const void* dy, const void* ss, const float* stats,
                           const float* gamma, const float* beta, int N, int P, int C, int G, float p_drop,
                           unsigned long long seed, void* dx, void* dss, float* chan_out, int ssld,
                           const void* seed_dev, const void* x2, void* dx2, int C1, const void* dres,
                           float dres_scale, const void* dres2, float dres2_scale, hipStream_t st) {
  const ImgPlan p = img_plan(P, C, G, N);
  if (!p.ok) return (int)hipErrorInvalidValue;
  Cat cat{(const bf16*)x2, (bf16*)dx2, C1};
  if (ssld == 0) ssld = 2 * C;
  if (x2) dres = dres2 = nullptr;
  const dim3 grid(C / p.CS, N);
#define IB1(NT_, U_, M_)                                                                                            \
  hipLaunchKernelGGL((gn_img_bwd_k<NT_, U_, M_>), grid, dim3(NT_), 0, st, (const bf16*)x, (const bf16*)dy,         \
                     (const bf16*)ss, stats, gamma, beta, (bf16*)dx, (bf16*)dss, chan_out, P, C, G, p.CS, p_drop,  \
                     (uint64_t)seed, ssld, (const uint64_t*)seed_dev, cat, (const bf16*)dres, dres_scale,          \
                     (const bf16*)dres2, dres2_scale)
#define IBU(NT_, M_)                                                                                                \
  if (p.U == 1) IB1(NT_, 1, M_); else if (p.U == 2) IB1(NT_, 2, M_); else if (p.U == 4) IB1(NT_, 4, M_);        \
  else IB1(NT_, 8, M_)
#define IBM(M_) if (p.NTI == 256) { IBU(256, M_); } else { IBU(512, M_); }
  if (mode == 0) { IBM(0); }
  else if (mode == 1) { IBM(1); }
  else { IBM(2); }
#undef IBM
#undef IBU
#undef IB1
  return (int)hipGetLastError();
}
