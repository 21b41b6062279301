// Fused Adam over the flat fp32 parameter buffer (one launch per step).
//
// Reference: torch.optim.Adam(lr=1e-4, betas=(0.9,0.99)) over 647 tensors
// (train.py:235).  Same arithmetic order as torch's implementation:
//   g  = grad * grad_scale (+ wd * p)           (grad_scale folds DP averaging)
//   m  = lerp(m, g, 1-b1);  v = v*b2 + (1-b2) g^2
//   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)
//   ema = lerp(ema, p, 1-ema_decay)              (optional)
// 16-byte vector loads/stores, grid-stride; HBM-bound (5 fp32 streams).
#include "common.h"

namespace {
__global__ void adam_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, float* __restrict__ ema, long n4, float b1, float b2, float eps,
                       float wd, float step_size, float bc2_sqrt, float grad_scale, float ema_w) {
  const float inv_bc2 = 1.0f / bc2_sqrt;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * grad_scale;
      if (wd != 0.f) gj += wd * pp[j];
      mm[j] = mm[j] + (1.f - b1) * (gj - mm[j]);
      vv[j] = vv[j] * b2 + (1.f - b2) * gj * gj;
      float denom = sqrtf(vv[j]) * inv_bc2 + eps;
      pp[j] = pp[j] - step_size * (mm[j] / denom);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (ema) {
      f32x4 ee = reinterpret_cast<f32x4*>(ema)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) ee[j] = ee[j] + ema_w * (pp[j] - ee[j]);
      reinterpret_cast<f32x4*>(ema)[i] = ee;
    }
  }
}
// Graph-replay form: hyper-parameters read from a device block
// hp = [b1, b2, eps, wd, step_size, bc2_sqrt, grad_scale, ema_w] that the host
// refreshes before each replay (lr warmup / bias correction change per step).
__global__ void adam_dev_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                           float* __restrict__ v, float* __restrict__ ema, long n4, const float* __restrict__ hp) {
  const float b1 = hp[0], b2 = hp[1], eps = hp[2], wd = hp[3], step_size = hp[4], inv_bc2 = 1.0f / hp[5],
              grad_scale = hp[6], ema_w = hp[7];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * grad_scale;
      if (wd != 0.f) gj += wd * pp[j];
      mm[j] = mm[j] + (1.f - b1) * (gj - mm[j]);
      vv[j] = vv[j] * b2 + (1.f - b2) * gj * gj;
      float denom = sqrtf(vv[j]) * inv_bc2 + eps;
      pp[j] = pp[j] - step_size * (mm[j] / denom);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (ema) {
      f32x4 ee = reinterpret_cast<f32x4*>(ema)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) ee[j] = ee[j] + ema_w * (pp[j] - ee[j]);
      reinterpret_cast<f32x4*>(ema)[i] = ee;
    }
  }
}
}  // namespace

D3D_API int d3d_adam_dev(float* p, const float* g, float* m, float* v, float* ema, long n, const float* hp,
                         hipStream_t st) {
  long n4 = n / 4;
  long grid = (n4 + 255) / 256;
  if (grid > 256 * 8) grid = 256 * 8;
  hipLaunchKernelGGL(adam_dev_k, dim3((int)grid), dim3(256), 0, st, p, g, m, v, ema, n4, hp);
  return (int)hipGetLastError();
}

// n must be a multiple of 4 (the flat buffer is padded to 64 elements).
D3D_API int d3d_adam(float* p, const float* g, float* m, float* v, float* ema, long n, float b1, float b2,
                     float eps, float wd, float step_size, float bc2_sqrt, float grad_scale, float ema_decay,
                     hipStream_t st) {
  long n4 = n / 4;
  long grid = (n4 + 255) / 256;
  if (grid > 256 * 8) grid = 256 * 8;
  hipLaunchKernelGGL(adam_k, dim3((int)grid), dim3(256), 0, st, p, g, m, v, ema, n4, b1, b2, eps, wd, step_size,
                     bc2_sqrt, grad_scale, 1.0f - ema_decay);
  return (int)hipGetLastError();
}
