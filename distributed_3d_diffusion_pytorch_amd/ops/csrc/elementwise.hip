// Memory-bound NHWC bf16 elementwise kernels (16-byte vectors, grid-stride).
//
//   silu / dsilu                  : the per-level FiLM input activation
//                                   (xunet.py:84, computed once per level here)
//   avgpool2 / its backward       : ResBlock(resample='down') (xunet.py:23-28)
//   upsample2 / its backward      : ResBlock(resample='up')   (xunet.py:17-20)
//   add_scale                     : (a + b) * s residual epilogue (xunet.py:152,220)
//   sampler_step                  : CFG combine + x0 clamp + posterior + noise
//                                   (train.py:140-166 / sampling.py:85-127, on device)
//   diffusion_fwd                 : q_sample + CFG-drop input noise (train.py:50-60,95-96)
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

// q_sample + CFG drop on fp32 [B, D] images:
//   z_t = alpha_b z + sigma_b eps ;  x' = mask_b ? x : N(0,1)
__global__ void diffusion_fwd_k(const float* __restrict__ x, const float* __restrict__ z,
                                const float* __restrict__ eps, const float* __restrict__ logsnr,
                                const uint8_t* __restrict__ mask, float* __restrict__ zt, float* __restrict__ xc,
                                int D, long total, uint64_t seed) {
  GRID_LOOP(i, total) {
    int b = (int)(i / D);
    float l = logsnr[b];
    float alpha = sqrtf(sigmoidf_(l)), sigma = sqrtf(sigmoidf_(-l));
    zt[i] = alpha * z[i] + sigma * eps[i];
    xc[i] = mask[b] ? x[i] : normal01(seed, (uint64_t)i);
  }
}
}  // namespace

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
D3D_API int d3d_diffusion_fwd(const float* x, const float* z, const float* eps, const float* logsnr,
                              const unsigned char* mask, float* zt, float* xc, int B, int D, unsigned long long seed,
                              hipStream_t st) {
  long total = (long)B * D;
  hipLaunchKernelGGL(diffusion_fwd_k, dim3(ew_grid(total / 8 + 1)), dim3(256), 0, st, x, z, eps, logsnr, mask, zt,
                     xc, D, total, (uint64_t)seed);
  return (int)hipGetLastError();
}
