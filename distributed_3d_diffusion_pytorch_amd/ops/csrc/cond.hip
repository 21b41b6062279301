// Conditioning-conv support kernels for the origin / direction split.
//
// Reference: ConditioningProcessor (xunet.py:292-352) convolves the 144-channel
// ray encoding [posenc(origin) 93 ch | posenc(direction) 51 ch] with a 3x3
// conv at stride 2^i.  For a pinhole camera the ray ORIGIN is the camera
// centre -- the same for every pixel -- so its 93 channels form a constant
// image c_n and, with zero padding,
//     conv(c_n)[p] = sum_{taps t valid at p} W_t c_n  =  S_n - sum_{t invalid at p} U_{n,t},
// U_{n,t} = W_t c_n (a [N, 9, OC] table from one tiny GEMM), S_n = sum_t U_{n,t}.
// So the MFMA conv only needs the 51 direction channels (K = 9 x 64 instead
// of 9 x 192: 3x fewer FLOPs), S_n joins the per-image bias of the epilogue,
// and these kernels handle the image border:
//   border_fix  : y[n,p] -= sum_{t invalid at p} U[n,t]   (border pixels only)
//   border_sums : per image, dy summed over the first/last row/column and the
//                 four corners -> the weight gradient of the origin half
//                 (sum over the pixels where each tap is valid, by inclusion-
//                 exclusion from the image total).
#include "common.h"

namespace {

__device__ __forceinline__ bool border_pixel(int b, int OH, int OW, int& oh, int& ow) {
  // strips: top row, bottom row, left column (inner rows), right column (inner rows)
  if (b < OW) { oh = 0; ow = b; return true; }
  b -= OW;
  if (OH > 1) {
    if (b < OW) { oh = OH - 1; ow = b; return true; }
    b -= OW;
  }
  const int inner = OH > 2 ? OH - 2 : 0;
  if (b < inner) { oh = 1 + b; ow = 0; return true; }
  b -= inner;
  if (OW > 1 && b < inner) { oh = 1 + b; ow = OW - 1; return true; }
  return false;
}

// y2 != nullptr: y's SiLU companion (written by the conv epilogue from the
// uncorrected border values) is rewritten at the corrected pixels.
__global__ void border_fix_k(bf16* __restrict__ y, const float* __restrict__ U, int IH, int IW, int OH, int OW,
                             int OC, int stride, bf16* __restrict__ y2) {
  const int n = blockIdx.y;
  int oh, ow;
  if (!border_pixel(blockIdx.x, OH, OW, oh, ow)) return;
  unsigned inv = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ih = oh * stride + t / 3 - 1, iw = ow * stride + t % 3 - 1;
    if (ih < 0 || ih >= IH || iw < 0 || iw >= IW) inv |= 1u << t;
  }
  if (!inv) return;
  bf16* row = y + (((long)n * OH + oh) * OW + ow) * OC;
  const float* Un = U + (long)n * 9 * OC;
  for (int c = threadIdx.x * 8; c < OC; c += blockDim.x * 8) {
    f32x8 v = ld8(row + c);
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (inv & (1u << t)) {
        f32x8 u = ld8f(Un + t * OC + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] -= u[j];
      }
    st8(row + c, v);
    if (y2) {
      const f32x8 r = ld8(row + c);         // the stored (bf16-rounded) values, as the SiLU pass reads them
      f32x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = siluf_(r[j]);
      st8(y2 + (row - y) + c, o);
    }
  }
}

// S[n][k][c], k: 0 first row, 1 last row, 2 first col, 3 last col,
// 4..7 corners (0,0) (0,W-1) (H-1,0) (H-1,W-1).  grid (N, 4 strips).
__global__ void border_sums_k(const bf16* __restrict__ dy, float* __restrict__ S, int OH, int OW, int OC) {
  const int n = blockIdx.x, k = blockIdx.y;
  const bf16* base = dy + (long)n * OH * OW * OC;
  const int len = k < 2 ? OW : OH;
  for (int c = threadIdx.x * 8; c < OC; c += blockDim.x * 8) {
    f32x8 acc = {};
    f32x8 first = {}, last = {};
    for (int i = 0; i < len; ++i) {
      const int oh = k == 0 ? 0 : k == 1 ? OH - 1 : i;
      const int ow = k == 2 ? 0 : k == 3 ? OW - 1 : i;
      f32x8 v = ld8(base + ((long)oh * OW + ow) * OC + c);
      acc += v;
      if (i == 0) first = v;
      if (i == len - 1) last = v;
    }
    float* out = S + ((long)n * 8 + k) * OC + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = acc[j];
    if (k < 2) {       // corners from the row strips
      float* c0 = S + ((long)n * 8 + 4 + 2 * k) * OC + c;
      float* c1 = c0 + OC;
#pragma unroll
      for (int j = 0; j < 8; ++j) { c0[j] = first[j]; c1[j] = last[j]; }
    }
  }
}

}  // namespace

D3D_API int d3d_border_fix(void* y, const float* U, int N, int IH, int IW, int OH, int OW, int OC, int stride,
                           void* y2, hipStream_t st) {
  if (OC % 8) return (int)hipErrorInvalidValue;
  const int nb = OW + (OH > 1 ? OW : 0) + 2 * (OH > 2 ? OH - 2 : 0);
  hipLaunchKernelGGL(border_fix_k, dim3(nb, N), dim3(128), 0, st, (bf16*)y, U, IH, IW, OH, OW, OC, stride, (bf16*)y2);
  return (int)hipGetLastError();
}

D3D_API int d3d_border_sums(const void* dy, float* S, int N, int OH, int OW, int OC, hipStream_t st) {
  if (OC % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(border_sums_k, dim3(N, 4), dim3(128), 0, st, (const bf16*)dy, S, OH, OW, OC);
  return (int)hipGetLastError();
}
