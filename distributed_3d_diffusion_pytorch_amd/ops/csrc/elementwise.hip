// Memory-bound NHWC bf16 elementwise kernels (16-byte vectors, grid-stride).
//
//   silu / dsilu                  : the per-level FiLM input activation
//                                   (xunet.py:84, computed once per level here)
//   avgpool2 / its backward       : ResBlock(resample='down') (xunet.py:23-28)
//   upsample2 / its backward      : ResBlock(resample='up')   (xunet.py:17-20)
//   add_scale                     : (a + b) * s residual epilogue (xunet.py:152,220)
//   sampler_step                  : CFG combine + x0 clamp + posterior + noise
//                                   (train.py:140-166 / sampling.py:85-127, on device)
//   diffusion_fwd2                : the whole training-input draw of one step in one launch:
//                                   t ~ U[0,1), lambda(t), eps, z_t = q_sample, CFG drop
//                                   (train.py:50-60,80-100) -> the stem's NHWC bf16 input
//   diff_loss / diff_loss_bwd     : l2 / l1 / huber epsilon loss read straight from the padded
//                                   NHWC head output (train.py:102-112)
#include "common.h"

namespace {
inline int ew_grid(long nvec) {
  long g = (nvec + 255) / 256;
  if (g > 256L * 16) g = 256L * 16;
  if (g < 1) g = 1;
  return (int)g;
}

#define GRID_LOOP(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

__global__ void silu_k(const bf16* __restrict__ x, bf16* __restrict__ y, long nvec) {
  GRID_LOOP(i, nvec) {
    f32x8 a = ld8(x + i * 8), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = siluf_(a[j]);
    st8(y + i * 8, o);
  }
}

__global__ void dsilu_k(const bf16* __restrict__ x, const bf16* __restrict__ dy, bf16* __restrict__ dx, long nvec) {
  GRID_LOOP(i, nvec) {
    f32x8 a = ld8(x + i * 8), d = ld8(dy + i * 8), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = d[j] * dsiluf_(a[j]);
    st8(dx + i * 8, o);
  }
}

// x [N,H,W,C] -> y [N,H/2,W/2,C]; one thread per output 8-channel vector
__global__ void avgpool2_k(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CV = C / 8;
  long nvec = (long)N * Ho * Wo * CV;
  GRID_LOOP(i, nvec) {
    int cv = (int)(i % CV);
    long pix = i / CV;
    int wo = (int)(pix % Wo);
    long t = pix / Wo;
    int ho = (int)(t % Ho);
    int n = (int)(t / Ho);
    const bf16* b = x + (((long)n * H + 2 * ho) * W + 2 * wo) * C + cv * 8;
    f32x8 a0 = ld8(b), a1 = ld8(b + C), a2 = ld8(b + (long)W * C), a3 = ld8(b + (long)W * C + C);
    st8(y + i * 8, (a0 + a1 + a2 + a3) * 0.25f);
  }
}

__global__ void avgpool2_bwd_k(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CV = C / 8;
  long nvec = (long)N * Ho * Wo * CV;
  GRID_LOOP(i, nvec) {
    int cv = (int)(i % CV);
    long pix = i / CV;
    int wo = (int)(pix % Wo);
    long t = pix / Wo;
    int ho = (int)(t % Ho);
    int n = (int)(t / Ho);
    f32x8 d = ld8(dy + i * 8) * 0.25f;
    bf16* b = dx + (((long)n * H + 2 * ho) * W + 2 * wo) * C + cv * 8;
    st8(b, d);
    st8(b + C, d);
    st8(b + (long)W * C, d);
    st8(b + (long)W * C + C, d);
  }
}

// nearest x2: x [N,H,W,C] -> y [N,2H,2W,C]; one thread per input vector
__global__ void upsample2_k(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C) {
  const int CV = C / 8;
  long nvec = (long)N * H * W * CV;
  GRID_LOOP(i, nvec) {
    int cv = (int)(i % CV);
    long pix = i / CV;
    int w = (int)(pix % W);
    long t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    bf16* b = y + (((long)n * 2 * H + 2 * h) * 2 * W + 2 * w) * C + cv * 8;
    *reinterpret_cast<bf16x8*>(b) = v;
    *reinterpret_cast<bf16x8*>(b + C) = v;
    *reinterpret_cast<bf16x8*>(b + 2L * W * C) = v;
    *reinterpret_cast<bf16x8*>(b + 2L * W * C + C) = v;
  }
}

__global__ void upsample2_bwd_k(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N, int H, int W, int C) {
  const int CV = C / 8;
  long nvec = (long)N * H * W * CV;
  GRID_LOOP(i, nvec) {
    int cv = (int)(i % CV);
    long pix = i / CV;
    int w = (int)(pix % W);
    long t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    const bf16* b = dy + (((long)n * 2 * H + 2 * h) * 2 * W + 2 * w) * C + cv * 8;
    f32x8 s = ld8(b) + ld8(b + C) + ld8(b + 2L * W * C) + ld8(b + 2L * W * C + C);
    st8(dx + i * 8, s);
  }
}

// y = (a + b) * s   (b may be null)
__global__ void add_scale_k(const bf16* __restrict__ a, const bf16* __restrict__ b, bf16* __restrict__ y, float s,
                            long nvec) {
  GRID_LOOP(i, nvec) {
    f32x8 v = ld8(a + i * 8);
    if (b) v = v + ld8(b + i * 8);
    st8(y + i * 8, v * s);
  }
}

// y = (a + b) * s fused with the partial statistics of the GroupNorm that
// consumes y (the attention block output feeding the next block's
// GroupNorm: xunet.py:220 then :140) -- the layout of conv.hip
// gn_part_store, [N][G][P/64] x (sum, sum of squares) over the STORED bf16
// values, so that GroupNorm skips its statistics pass exactly as after a conv.
// One block per (64-pixel part, 64-channel slab): 16 threads per pixel x 4
// channels, 16 pixels per pass; a slab holds whole groups (Cg <= 32) of one
// image, so every (image, group, part) slot is written by exactly one block.
// In place (y == a) is allowed: each element is read and written by one thread.
__global__ void __launch_bounds__(256) add_scale_gn_k(const bf16* a, const bf16* __restrict__ b, bf16* y, float s,
                                                      int C, int P, int G, float* __restrict__ gnp) {
  constexpr int CB = 64, TPC = CB / 4, PPI = 256 / TPC, KP = 64 / PPI;
  __shared__ float s_s[PPI][TPC], s_q[PPI][TPC];
  const int tid = threadIdx.x, r = tid / TPC, cq = tid % TPC;
  const long pix0 = (long)blockIdx.x * 64;
  const int co = blockIdx.y * CB + cq * 4;
  bf16x4 av[KP], bv[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {                 // every load of the block in flight together
    const long off = (pix0 + k * PPI + r) * C + co;
    av[k] = *reinterpret_cast<const bf16x4*>(a + off);
    if (b) bv[k] = *reinterpret_cast<const bf16x4*>(b + off);
  }
  float sum = 0.f, sq = 0.f;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    bf16x4 o4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = (float)av[k][e];
      if (b) v += (float)bv[k][e];
      o4[e] = (bf16)(v * s);
      const float q = (float)o4[e];
      sum += q;
      sq += q * q;
    }
    *reinterpret_cast<bf16x4*>(y + (pix0 + k * PPI + r) * C + co) = o4;
  }
  s_s[r][cq] = sum;
  s_q[r][cq] = sq;
  __syncthreads();
  const int Cg = C / G, ng = CB / Cg;
  if (tid < ng) {
    const int q4 = Cg / 4;
    float u = 0.f, w = 0.f;
    for (int rr = 0; rr < PPI; ++rr)
      for (int j = 0; j < q4; ++j) {
        u += s_s[rr][tid * q4 + j];
        w += s_q[rr][tid * q4 + j];
      }
    const long n = pix0 / P;
    const int t = (int)(pix0 - n * P) / 64;
    const int g = (blockIdx.y * CB) / Cg + tid;
    float* d = gnp + ((n * G + g) * (P / 64) + t) * 2;
    d[0] = u;
    d[1] = w;
  }
}

// CFG ancestral step for fp32 z [b, D]:
//   eps = (1+w) ec - w eu;  x0 = clamp((z - sigma eps)/alpha, -1, 1)
//   mean = alpha_n (z (1-c)/alpha + c x0);  z' = mean + sqrt(var) * N(0,1) * add_noise
__global__ void sampler_step_k(const float* __restrict__ z, const float* __restrict__ ec,
                               const float* __restrict__ eu, const float* __restrict__ w, float* __restrict__ out,
                               int D, long total, float alpha, float sigma, float alpha_n, float c, float var_sqrt,
                               int add_noise, uint64_t seed) {
  GRID_LOOP(i, total) {
    int b = (int)(i / D);
    float wb = w[b];
    float e = (1.f + wb) * ec[i] - wb * eu[i];
    float zi = z[i];
    float x0 = fminf(fmaxf((zi - sigma * e) / alpha, -1.f), 1.f);
    float m = alpha_n * (zi * (1.f - c) / alpha + c * x0);
    if (add_noise) m += var_sqrt * normal01(seed, (uint64_t)i);
    out[i] = m;
  }
}

// ---- graph-replayed sampler (engine/sampler.py GraphedSampler) ----------
// Per-step scalars live in a device block (a replay cannot see new host
// values): prm = [lambda, alpha, sigma, alpha_next, c, sqrt(var), add_noise,
// lambda0]; the step's RNG word is sd[0] (s = seed + sd[0] * golden).
// Noise is counter-based in the GLOBAL chain index (c0 + chain), so a chain
// draws the same numbers whatever the rank sharding.
#define K_XU 0xA0761D6478BD642Full
#define K_NZ 0xE7037ED1A0B428DBull
// CFG batch of one step: xz [4b,H,W,8] bf16 = per example j in [0,2b): frame 0
// = x_cond (j < b) or N(0,1) (j >= b: the unconditional pass), frame 1 = z;
// logsnr [2b,2] = (lambda0, lambda).
__global__ void sampler_inputs_k(const float* __restrict__ xc, const float* __restrict__ z, int b, int HW,
                                 const float* __restrict__ prm, const uint64_t* __restrict__ sd, uint64_t seed,
                                 long c0, bf16* __restrict__ xz, float* __restrict__ logsnr) {
  const uint64_t s = seed + (sd ? sd[0] : 0ull) * 0x9E3779B97F4A7C15ull;
  GRID_LOOP(i, (long)2 * b * HW) {
    const int j = (int)(i / HW);
    const int p = (int)(i - (long)j * HW);
    const int jb = j < b ? j : j - b;
    bf16x8 ox, oz;
#pragma unroll
    for (int c = 0; c < 8; ++c) { ox[c] = (bf16)0.f; oz[c] = (bf16)0.f; }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t e = (size_t)jb * 3 * HW + (size_t)c * HW + p;
      oz[c] = (bf16)z[e];
      ox[c] = (bf16)(j < b ? xc[e] : normal01(s ^ K_XU, (uint64_t)(c0 + jb) * 3 * HW + (uint64_t)c * HW + p));
    }
    *reinterpret_cast<bf16x8*>(xz + ((size_t)2 * j * HW + p) * 8) = ox;
    *reinterpret_cast<bf16x8*>(xz + ((size_t)(2 * j + 1) * HW + p) * 8) = oz;
    if (p == 0) {
      logsnr[2 * j] = prm[7];
      logsnr[2 * j + 1] = prm[0];
    }
  }
}

// Ancestral CFG step reading eps straight from the padded NHWC head output
// y [2b,H,W,8] bf16 (rows [0,b) conditional, [b,2b) unconditional); z fp32
// [b,3,H,W] updated in place.
__global__ void sampler_step2_k(float* __restrict__ z, const bf16* __restrict__ y, const float* __restrict__ w,
                                int b, int HW, const float* __restrict__ prm, const uint64_t* __restrict__ sd,
                                uint64_t seed, long c0) {
  const uint64_t s = seed + (sd ? sd[0] : 0ull) * 0x9E3779B97F4A7C15ull;
  const float alpha = prm[1], sigma = prm[2], alpha_n = prm[3], c = prm[4], var_sqrt = prm[5];
  const bool noise = prm[6] != 0.f;
  GRID_LOOP(i, (long)b * 3 * HW) {
    const int j = (int)(i / (3 * HW));
    const int r = (int)(i - (long)j * 3 * HW);
    const int ch = r / HW, p = r - ch * HW;
    const float ec = (float)y[((size_t)j * HW + p) * 8 + ch];
    const float eu = (float)y[((size_t)(j + b) * HW + p) * 8 + ch];
    const float wb = w[j];
    const float e = (1.f + wb) * ec - wb * eu;
    const float zi = z[i];
    const float x0 = fminf(fmaxf((zi - sigma * e) / alpha, -1.f), 1.f);
    float m = alpha_n * (zi * (1.f - c) / alpha + c * x0);
    if (noise) m += var_sqrt * normal01(s ^ K_NZ, (uint64_t)(c0 + j) * 3 * HW + r);
    z[i] = m;
  }
}

// Counter-based N(0,1) fill: out[i] = N(seed ^ key, off + i)
__global__ void randn_hash_k(float* __restrict__ out, long n, uint64_t seed, long off) {
  GRID_LOOP(i, n) out[i] = normal01(seed, (uint64_t)(off + i));
}

// Training-input draw (train.py:80-100), counter-based so that it is
// reproducible per (step seed, global example index) -- micro-batches,
// graph replays and the torch reference (ops/torch_impl.py
// diffusion_inputs) all draw the same numbers:
//   t_g    = u01(s, 4g)                 lambda = -2 log tan(a t + b)
//   keep_g = u01(s, 4g + 1) > cond_prob
//   eps    = N(s ^ K_EPS, g*3HW + c*HW + p)   x_noise = N(s ^ K_XN, same index)
// Outputs: eps [B,3,H,W] fp32 (loss target), logsnr [B,2] (frame 0 = lambda(0)),
// keep [B] u8, and the stem input xz [2B,H,W,8] bf16 (frame 0 = keep ? x :
// x_noise, frame 1 = alpha z + sigma eps, channels 3..7 zero).
// Graph replays pass seed_dev = the step's device seed block [dropout word,
// draw word, example offset]: s = seed + sd[1] * golden, e0 += sd[2].
#define K_EPS 0x5851F42D4C957F2Dull
#define K_XN 0x14057B7EF767814Full
__global__ void diffusion_fwd2_k(const float* __restrict__ img, int B, int HW, uint64_t seed,
                                 const uint64_t* __restrict__ seed_dev, long e0, float cond_prob, float a, float b0,
                                 float* __restrict__ eps_out, float* __restrict__ logsnr_out,
                                 uint8_t* __restrict__ keep_out, bf16* __restrict__ xz) {
  uint64_t s = seed;
  if (seed_dev) {
    s += seed_dev[1] * 0x9E3779B97F4A7C15ull;
    e0 += (long)seed_dev[2];
  }
  const float lam0 = -2.f * logf(tanf(b0));
  GRID_LOOP(i, (long)B * HW) {
    const int bb = (int)(i / HW);
    const int p = (int)(i - (long)bb * HW);
    const uint64_t g = (uint64_t)(e0 + bb);
    const float t = (hash_u32(s, 4 * g) >> 8) * (1.0f / 16777216.0f);
    const float lam = -2.f * logf(tanf(a * t + b0));
    const bool keep = (hash_u32(s, 4 * g + 1) >> 8) * (1.0f / 16777216.0f) > cond_prob;
    const float alpha = sqrtf(1.f / (1.f + expf(-lam))), sigma = sqrtf(1.f / (1.f + expf(lam)));
    const float* x = img + (size_t)bb * 6 * HW;
    const float* z = x + 3 * (size_t)HW;
    bf16x8 ox, oz;
#pragma unroll
    for (int c = 0; c < 8; ++c) { ox[c] = (bf16)0.f; oz[c] = (bf16)0.f; }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint64_t idx = g * 3 * (uint64_t)HW + (uint64_t)c * HW + p;
      const float e = normal01(s ^ K_EPS, idx);
      eps_out[(size_t)bb * 3 * HW + (size_t)c * HW + p] = e;
      ox[c] = (bf16)(keep ? x[(size_t)c * HW + p] : normal01(s ^ K_XN, idx));
      oz[c] = (bf16)(alpha * z[(size_t)c * HW + p] + sigma * e);
    }
    *reinterpret_cast<bf16x8*>(xz + ((size_t)2 * bb * HW + p) * 8) = ox;
    *reinterpret_cast<bf16x8*>(xz + ((size_t)(2 * bb + 1) * HW + p) * 8) = oz;
    if (p == 0) {
      logsnr_out[2 * bb] = lam0;
      logsnr_out[2 * bb + 1] = lam;
      keep_out[bb] = keep ? 1 : 0;
    }
  }
}

// Epsilon loss over the padded NHWC head output y [B,H,W,CP] bf16 (first 3
// channels valid) against eps [B,3,H,W] fp32: per-block partial sums over a
// fixed grid (deterministic), then one block sums the partials in order.
// mode 0: mean (y - eps)^2, 1: mean |y - eps|.
#define LOSS_BLOCKS 256
__global__ void __launch_bounds__(256) diff_loss_part_k(const bf16* __restrict__ y, const float* __restrict__ eps,
                                                        int B, int HW, int CP, int mode, float* __restrict__ part) {
  float acc = 0.f;
  const long n = (long)B * HW;
  GRID_LOOP(i, n) {
    const int bb = (int)(i / HW);
    const int p = (int)(i - (long)bb * HW);
    const bf16* yp = y + (size_t)i * CP;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float d = (float)yp[c] - eps[(size_t)bb * 3 * HW + (size_t)c * HW + p];
      // 0: l2, 1: l1, 2: huber = smooth_l1 with beta 1 (F.smooth_l1_loss, train.py:108-109)
      const float ad = fabsf(d);
      acc += mode == 0 ? d * d : (mode == 1 ? ad : (ad < 1.f ? 0.5f * d * d : ad - 0.5f));
    }
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) diff_loss_final_k(const float* __restrict__ part, int nparts, float inv_n,
                                                         float* __restrict__ out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += part[i];
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((red[0] + red[1]) + (red[2] + red[3])) * inv_n;
}

// dy [B,H,W,CP] bf16 = dL * d/dy loss (channels >= 3 zero); dL read from the
// device (the upstream gradient of the scalar loss, e.g. a micro-batch weight).
__global__ void diff_loss_bwd_k(const bf16* __restrict__ y, const float* __restrict__ eps,
                                const float* __restrict__ dloss, int B, int HW, int CP, int mode, float inv_n,
                                bf16* __restrict__ dy) {
  const float g = dloss[0] * inv_n;
  GRID_LOOP(i, (long)B * HW) {
    const int bb = (int)(i / HW);
    const int p = (int)(i - (long)bb * HW);
    const bf16* yp = y + (size_t)i * CP;
    bf16x8 o;
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = (bf16)0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float d = (float)yp[c] - eps[(size_t)bb * 3 * HW + (size_t)c * HW + p];
      const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      o[c] = (bf16)(mode == 0 ? 2.f * g * d : (mode == 1 ? g * sgn : g * (fabsf(d) < 1.f ? d : sgn)));
    }
    *reinterpret_cast<bf16x8*>(dy + (size_t)i * CP) = o;
  }
}
}  // namespace

// Gradient of a batch-broadcast residual (the conditioning convs' learned
// per-frame embedding, added to every example with period 2, models/xunet.py
// levels()): out[q] = sum_r in[r][q] over R repeats of a QM-element block,
// bf16 in / out, fp32 accumulation in a fixed order.  One 16-byte vector per
// lane, four repeats in flight (replaces a torch reduction + cast).
namespace {
__global__ void __launch_bounds__(256) period_sum_k(const bf16* __restrict__ in, bf16* __restrict__ out, int R,
                                                    long nvec) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= nvec) return;
  const long stride = nvec * 8;
  const bf16* p = in + i * 8;
  f32x8 a = {};
  int r = 0;
  for (; r + 4 <= R; r += 4) {
    const f32x8 v0 = ld8(p + r * stride), v1 = ld8(p + (r + 1) * stride), v2 = ld8(p + (r + 2) * stride),
                v3 = ld8(p + (r + 3) * stride);
    a += v0;
    a += v1;
    a += v2;
    a += v3;
  }
  for (; r < R; ++r) a += ld8(p + r * stride);
  st8(out + i * 8, a);
}
}  // namespace

D3D_API int d3d_period_sum(const void* in, void* out, int R, long QM, hipStream_t st) {
  if (R < 1 || QM % 8) return (int)hipErrorInvalidValue;
  const long nvec = QM / 8;
  hipLaunchKernelGGL(period_sum_k, dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, st, (const bf16*)in,
                     (bf16*)out, R, nvec);
  return (int)hipGetLastError();
}

D3D_API int d3d_silu(const void* x, void* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(silu_k, dim3(ew_grid(n / 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n / 8);
  return (int)hipGetLastError();
}
D3D_API int d3d_dsilu(const void* x, const void* dy, void* dx, long n, hipStream_t st) {
  hipLaunchKernelGGL(dsilu_k, dim3(ew_grid(n / 8)), dim3(256), 0, st, (const bf16*)x, (const bf16*)dy, (bf16*)dx,
                     n / 8);
  return (int)hipGetLastError();
}
D3D_API int d3d_avgpool2(const void* x, void* y, int N, int H, int W, int C, int backward, hipStream_t st) {
  long nvec = (long)N * (H / 2) * (W / 2) * (C / 8);
  if (backward)
    hipLaunchKernelGGL(avgpool2_bwd_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C);
  else
    hipLaunchKernelGGL(avgpool2_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C);
  return (int)hipGetLastError();
}
// H, W are the LOW-resolution dims in both directions
D3D_API int d3d_upsample2(const void* x, void* y, int N, int H, int W, int C, int backward, hipStream_t st) {
  long nvec = (long)N * H * W * (C / 8);
  if (backward)
    hipLaunchKernelGGL(upsample2_bwd_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C);
  else
    hipLaunchKernelGGL(upsample2_k, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C);
  return (int)hipGetLastError();
}
// y = (a + b) * s over [rows, C] with the GroupNorm partials of y (images of
// P rows, G groups) in gnp [rows/P][G][P/64][2].  Returns -1 (nothing
// launched) when the shape is not covered (the caller then uses
// d3d_add_scale and the statistics pass runs as usual).
D3D_API int d3d_add_scale_gn(const void* a, const void* b, void* y, float s, long rows, int C, int P, int G,
                             float* gnp, hipStream_t st) {
  const int Cg = G > 0 && C % G == 0 ? C / G : 0;
  if (!(Cg == 4 || Cg == 8 || Cg == 16 || Cg == 32) || C % 64 || P % 64 || rows % P) return -1;
  hipLaunchKernelGGL(add_scale_gn_k, dim3((unsigned)(rows / 64), (unsigned)(C / 64)), dim3(256), 0, st,
                     (const bf16*)a, (const bf16*)b, (bf16*)y, s, C, P, G, gnp);
  return (int)hipGetLastError();
}

D3D_API int d3d_add_scale(const void* a, const void* b, void* y, float s, long n, hipStream_t st) {
  hipLaunchKernelGGL(add_scale_k, dim3(ew_grid(n / 8)), dim3(256), 0, st, (const bf16*)a, (const bf16*)b, (bf16*)y,
                     s, n / 8);
  return (int)hipGetLastError();
}
D3D_API int d3d_sampler_step(const float* z, const float* ec, const float* eu, const float* w, float* out, int b,
                             int D, float alpha, float sigma, float alpha_n, float c, float var_sqrt, int add_noise,
                             unsigned long long seed, hipStream_t st) {
  long total = (long)b * D;
  hipLaunchKernelGGL(sampler_step_k, dim3(ew_grid(total / 8 + 1)), dim3(256), 0, st, z, ec, eu, w, out, D, total,
                     alpha, sigma, alpha_n, c, var_sqrt, add_noise, (uint64_t)seed);
  return (int)hipGetLastError();
}
D3D_API int d3d_sampler_inputs(const float* xc, const float* z, int b, int HW, const float* prm, const void* sd,
                               unsigned long long seed, long c0, void* xz, float* logsnr, hipStream_t st) {
  long total = (long)2 * b * HW;
  hipLaunchKernelGGL(sampler_inputs_k, dim3(ew_grid(total)), dim3(256), 0, st, xc, z, b, HW, prm,
                     (const uint64_t*)sd, (uint64_t)seed, c0, (bf16*)xz, logsnr);
  return (int)hipGetLastError();
}
D3D_API int d3d_sampler_step2(float* z, const void* y, const float* w, int b, int HW, const float* prm,
                              const void* sd, unsigned long long seed, long c0, hipStream_t st) {
  long total = (long)b * 3 * HW;
  hipLaunchKernelGGL(sampler_step2_k, dim3(ew_grid(total)), dim3(256), 0, st, z, (const bf16*)y, w, b, HW, prm,
                     (const uint64_t*)sd, (uint64_t)seed, c0);
  return (int)hipGetLastError();
}
D3D_API int d3d_randn_hash(float* out, long n, unsigned long long seed, long off, hipStream_t st) {
  hipLaunchKernelGGL(randn_hash_k, dim3(ew_grid(n)), dim3(256), 0, st, out, n, (uint64_t)seed, off);
  return (int)hipGetLastError();
}
D3D_API int d3d_diffusion_fwd2(const float* img, int B, int HW, unsigned long long seed, const void* seed_dev,
                               long e0, float cond_prob, float a, float b0, float* eps, float* logsnr,
                               unsigned char* keep, void* xz, hipStream_t st) {
  long total = (long)B * HW;
  hipLaunchKernelGGL(diffusion_fwd2_k, dim3(ew_grid(total)), dim3(256), 0, st, img, B, HW, (uint64_t)seed,
                     (const uint64_t*)seed_dev, e0, cond_prob, a, b0, eps, logsnr, keep, (bf16*)xz);
  return (int)hipGetLastError();
}
D3D_API int d3d_diff_loss(const void* y, const float* eps, int B, int HW, int CP, int mode, float* part, float* out,
                          hipStream_t st) {
  if (CP != 8) return -1;
  hipLaunchKernelGGL(diff_loss_part_k, dim3(LOSS_BLOCKS), dim3(256), 0, st, (const bf16*)y, eps, B, HW, CP, mode,
                     part);
  hipLaunchKernelGGL(diff_loss_final_k, dim3(1), dim3(256), 0, st, part, LOSS_BLOCKS, 1.f / (3.f * B * HW), out);
  return (int)hipGetLastError();
}
D3D_API int d3d_diff_loss_bwd(const void* y, const float* eps, const float* dloss, int B, int HW, int CP, int mode,
                              void* dy, hipStream_t st) {
  if (CP != 8) return -1;
  long total = (long)B * HW;
  hipLaunchKernelGGL(diff_loss_bwd_k, dim3(ew_grid(total)), dim3(256), 0, st, (const bf16*)y, eps, dloss, B, HW, CP,
                     mode, 1.f / (3.f * B * HW), (bf16*)dy);
  return (int)hipGetLastError();
}

// ---------------------------------------------------- device words ----
// Per-step scalars (the Adam hyper-parameter block, ...) written by a kernel
// whose arguments carry the values: no host-to-device copy, so the host never
// waits for the stream to drain (a pageable 32-byte H2D copy did, idling the
// GPU for the host's latency once per step).
struct Words8 {
  float v[8];
};

__global__ void set_words_k(float* __restrict__ dst, int n, Words8 w) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = w.v[threadIdx.x];
}

D3D_API int d3d_set_words(float* dst, int n, float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                          float a7, hipStream_t st) {
  if (n < 0 || n > 8) return (int)hipErrorInvalidValue;
  Words8 w{{a0, a1, a2, a3, a4, a5, a6, a7}};
  hipLaunchKernelGGL(set_words_k, dim3(1), dim3(64), 0, st, dst, n, w);
  return (int)hipGetLastError();
}

// The per-step seed block of the graph-replayed step (int64 [dropout word,
// input-draw word, example offset]) in one launch instead of three fills.
struct Words3L {
  long long v[3];
};

__global__ void set_words64_k(long long* __restrict__ dst, int n, Words3L w) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = w.v[threadIdx.x];
}

D3D_API int d3d_set_words64(long long* dst, int n, long long a0, long long a1, long long a2, hipStream_t st) {
  if (n < 0 || n > 3) return (int)hipErrorInvalidValue;
  Words3L w{{a0, a1, a2}};
  hipLaunchKernelGGL(set_words64_k, dim3(1), dim3(64), 0, st, dst, n, w);
  return (int)hipGetLastError();
}
