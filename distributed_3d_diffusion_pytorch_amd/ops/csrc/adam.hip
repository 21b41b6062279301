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

__device__ __forceinline__ float adam_elem(float pp, float gg, float& mm, float& vv, float b1, float b2, float eps,
                                           float wd, float step_size, float inv_bc2, float grad_scale) {
  float gj = gg * grad_scale;
  if (wd != 0.f) gj += wd * pp;
  mm = mm + (1.f - b1) * (gj - mm);
  vv = vv * b2 + (1.f - b2) * gj * gj;
  const float denom = sqrtf(vv) * inv_bc2 + eps;
  return pp - step_size * (mm / denom);
}

// ---- fused update + bf16 repack (graph step and eager step) ----------------
// Adam over a table of flat ranges (the parameters that have no packed MFMA
// operand): block -> (range, 4096-element chunk) through a host-built map.
struct AdamRange {
  long start, len;
  int blk0, pad;
};

// zero_g: the gradient is cleared as it is consumed (the graph step's
// gradient zeroing folded into the update: one pass over the buffer fewer)
__global__ void __launch_bounds__(256) adam_ranges_k(float* __restrict__ p, float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     float* __restrict__ ema, const float* __restrict__ hp,
                                                     const AdamRange* __restrict__ ranges,
                                                     const int* __restrict__ blk_range, int zero_g) {
  const AdamRange r = ranges[blk_range[blockIdx.x]];
  const long base = r.start + (long)(blockIdx.x - r.blk0) * 4096;
  const long end = r.start + r.len;
  const float b1 = hp[0], b2 = hp[1], eps = hp[2], wd = hp[3], step_size = hp[4], inv_bc2 = 1.0f / hp[5],
              grad_scale = hp[6], ema_w = hp[7];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = base + ((long)k * 256 + threadIdx.x) * 4;     // ranges are 64-element aligned
    if (i >= end) break;
    f32x4 pp = *reinterpret_cast<f32x4*>(p + i);
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + i);
    if (zero_g) *reinterpret_cast<f32x4*>(g + i) = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 mm = *reinterpret_cast<f32x4*>(m + i);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mj = mm[j], vj = vv[j];
      pp[j] = adam_elem(pp[j], gg[j], mj, vj, b1, b2, eps, wd, step_size, inv_bc2, grad_scale);
      mm[j] = mj;
      vv[j] = vj;
    }
    *reinterpret_cast<f32x4*>(p + i) = pp;
    *reinterpret_cast<f32x4*>(m + i) = mm;
    *reinterpret_cast<f32x4*>(v + i) = vv;
    if (ema) {
      f32x4 ee = *reinterpret_cast<f32x4*>(ema + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) ee[j] = ee[j] + ema_w * (pp[j] - ee[j]);
      *reinterpret_cast<f32x4*>(ema + i) = ee;
    }
  }
}

// Adam of one (32 output x 16 input channel x taps) tile of an OIHW weight
// fused with its bf16 MFMA operands: the updated tile is staged in LDS and
// written as the forward pack [OCp][taps][ICp] and / or the transposed pack
// [ICp][taps][OCp] (the layouts of conv.hip pack_all_k; padding lanes are
// left untouched -- they hold the zeros written when the operand was built).
// Saves the repack's second read of the fp32 masters.
struct AdamTile {
  long off;                    // flat index of the weight
  bf16* dst0;                  // forward pack (or null)
  bf16* dst1;                  // transposed pack (or null)
  int OC, IC, taps, ICp0, OCp1, blk0;
};

__global__ void __launch_bounds__(256) adam_pack_tiles_k(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         float* __restrict__ ema, const float* __restrict__ hp,
                                                         const AdamTile* __restrict__ tiles,
                                                         const int* __restrict__ blk_tile, int zero_g) {
  // rows padded by one float: the transposed reads below step through rows
  // (stride 16 * 9 = 144 floats = 16 mod 32 banks put every row of a lane
  // group on two banks -- 51 % LDS conflict cycles at bs16); 145 spreads them
  __shared__ float tile[32 * (16 * 9 + 1)];
  const AdamTile d = tiles[blk_tile[blockIdx.x]];
  const int local = blockIdx.x - d.blk0, tid = threadIdx.x, T = d.taps;
  const int nct = (d.OC + 31) / 32;
  const int co0 = (local % nct) * 32, ci0 = (local / nct) * 16;
  const int nci = min(16, d.IC - ci0), nco = min(32, d.OC - co0);
  const float b1 = hp[0], b2 = hp[1], eps = hp[2], wd = hp[3], step_size = hp[4], inv_bc2 = 1.0f / hp[5],
              grad_scale = hp[6], ema_w = hp[7];
  // tile element k -> (row r, q = ci * T + tap); each row's 16 * T elements
  // are contiguous in the OIHW master (16 * 9 floats = 576 B)
  const int RW = 16 * T, RP = RW + 1;
  const long rowlen = (long)d.IC * T;
  if (nci == 16 && ((d.off | rowlen) & 3) == 0) {
    // full channel tile: every row is 16 * T contiguous, 16-byte aligned
    // floats -- 16-byte loads / stores of p, g, m, v (and the EMA)
    const int RW4 = RW / 4;
    for (int k = tid; k < 32 * RW4; k += 256) {
      const int r = k / RW4, q = (k - r * RW4) * 4;
      if (r >= nco) continue;
      const long i = d.off + ((long)(co0 + r) * d.IC + ci0) * T + q;
      f32x4 pp = *reinterpret_cast<const f32x4*>(p + i), gg = *reinterpret_cast<const f32x4*>(g + i);
      if (zero_g) *reinterpret_cast<f32x4*>(g + i) = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 mm = *reinterpret_cast<const f32x4*>(m + i), vv = *reinterpret_cast<const f32x4*>(v + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float mj = mm[j], vj = vv[j];
        pp[j] = adam_elem(pp[j], gg[j], mj, vj, b1, b2, eps, wd, step_size, inv_bc2, grad_scale);
        mm[j] = mj;
        vv[j] = vj;
        tile[r * RP + q + j] = pp[j];
      }
      *reinterpret_cast<f32x4*>(p + i) = pp;
      *reinterpret_cast<f32x4*>(m + i) = mm;
      *reinterpret_cast<f32x4*>(v + i) = vv;
      if (ema) {
        f32x4 ee = *reinterpret_cast<const f32x4*>(ema + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) ee[j] = ee[j] + ema_w * (pp[j] - ee[j]);
        *reinterpret_cast<f32x4*>(ema + i) = ee;
      }
    }
  } else {
    for (int k = tid; k < 32 * RW; k += 256) {
      const int r = k / RW, q = k - r * RW;
      const int ci = q / T;
      if (r >= nco || ci >= nci) continue;
      const long i = d.off + ((long)(co0 + r) * d.IC + ci0) * T + q;
      float mm = m[i], vv = v[i];
      const float pn = adam_elem(p[i], g[i], mm, vv, b1, b2, eps, wd, step_size, inv_bc2, grad_scale);
      if (zero_g) g[i] = 0.f;
      p[i] = pn;
      m[i] = mm;
      v[i] = vv;
      if (ema) ema[i] = ema[i] + ema_w * (pn - ema[i]);
      tile[r * RP + q] = pn;
    }
  }
  __syncthreads();
  if (d.dst1) {
    // dst1[ci][tap][co0 .. co0+31]: 8 consecutive output channels per store
    for (int k = tid; k < 16 * T * 4; k += 256) {
      const int c8 = (k & 3) * 8, rt = k >> 2;
      const int ci = rt / T, tap = rt % T;
      if (ci >= nci || c8 >= nco) continue;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)(c8 + e < nco ? tile[(c8 + e) * RP + ci * T + tap] : 0.f);
      *reinterpret_cast<bf16x8*>(d.dst1 + ((long)(ci0 + ci) * T + tap) * d.OCp1 + co0 + c8) = o;
    }
  }
  if (d.dst0) {
    // dst0[co][tap][ci0 .. ci0+15]: two 8-channel stores per (co, tap)
    for (int k = tid; k < 32 * T * 2; k += 256) {
      const int h = k & 1, rt = k >> 1;
      const int r = rt / T, tap = rt % T;
      if (r >= nco || h * 8 >= nci) continue;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ci = h * 8 + e;
        o[e] = (bf16)(ci < nci ? tile[r * RP + ci * T + tap] : 0.f);
      }
      *reinterpret_cast<bf16x8*>(d.dst0 + ((long)(co0 + r) * T + tap) * d.ICp0 + ci0 + h * 8) = o;
    }
  }
}
}  // namespace

// One optimizer step over the flat buffers, repacking the MFMA operands of
// the tile-table weights on the way (the repack of every other cached
// operand -- plain casts, channel slices -- follows as d3d_pack_all).
D3D_API int d3d_adam_fused(float* p, float* g, float* m, float* v, float* ema, const float* hp,
                           const void* ranges, const int* blk_range, int range_blocks, const void* tiles,
                           const int* blk_tile, int tile_blocks, int zero_g, hipStream_t st) {
  if (range_blocks > 0)
    hipLaunchKernelGGL(adam_ranges_k, dim3(range_blocks), dim3(256), 0, st, p, g, m, v, ema, hp,
                       (const AdamRange*)ranges, blk_range, zero_g);
  if (tile_blocks > 0)
    hipLaunchKernelGGL(adam_pack_tiles_k, dim3(tile_blocks), dim3(256), 0, st, p, g, m, v, ema, hp,
                       (const AdamTile*)tiles, blk_tile, zero_g);
  return (int)hipGetLastError();
}

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
