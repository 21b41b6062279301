// Small strided batched fp32 GEMM for the conditioning conv's origin-channel
// algebra (ops/hip_impl.py _CondConv, `xunet.py:292-299`): the per-image tap
// biases U[n, t, o] = sum_k pe[n, k] W[o, k, t], their gradient through the
// border inclusion-exclusion matrix, and the origin half of the weight
// gradient dW[o, k, t] += sum_n dU[n, t, o] pe[n, k].  A few MFLOP each, in
// fp32 (exact parity with the fp32 einsums they replace, no library GEMM
// launch):
//
//     C_b[m][n] = alpha * sum_k A_b[m][k] * B_b[k][n] + beta * C_b[m][n]
//
// with arbitrary element strides (batch, row, column) for every operand, so
// the permuted views above need no copies.  64 x 64 output tile per 256-thread
// block (4 x 4 per thread), K in chunks of 16 through LDS.
#include "common.h"

namespace {
constexpr int SG_T = 64, SG_K = 16;
}

__global__ void __launch_bounds__(256) sgemm_strided_k(const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ C, int M, int N, int K, long sab, long sam,
                                                       long sak, long sbb, long sbk, long sbn, long scb, long scm,
                                                       long scn, float alpha, float beta) {
  __shared__ float As[SG_K][SG_T + 1];
  __shared__ float Bs[SG_K][SG_T + 1];
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * SG_T, n0 = blockIdx.x * SG_T;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const float* a = A + (long)b * sab;
  const float* bb = B + (long)b * sbb;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += SG_K) {
    for (int e = threadIdx.x; e < SG_K * SG_T; e += 256) {
      const int kk = e / SG_T, mm = e % SG_T;
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? a[gm * sam + gk * sak] : 0.f;
      const int gn = n0 + mm;
      Bs[kk][mm] = (gn < N && gk < K) ? bb[gk * sbk + gn * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < SG_K; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* c = C + (long)b * scb;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + ty + 16 * i;
    if (gm >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gn = n0 + tx + 16 * j;
      if (gn >= N) continue;
      float* d = c + gm * scm + gn * scn;
      *d = beta == 0.f ? alpha * acc[i][j] : alpha * acc[i][j] + beta * *d;
    }
  }
}

D3D_API int d3d_sgemm_strided(const float* A, const float* B, float* C, int M, int N, int K, int batch, long sab,
                              long sam, long sak, long sbb, long sbk, long sbn, long scb, long scm, long scn,
                              float alpha, float beta, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return -1;
  dim3 grid(cdiv(N, SG_T), cdiv(M, SG_T), batch);
  if (grid.y > 65535) return -1;
  hipLaunchKernelGGL(sgemm_strided_k, grid, dim3(256), 0, st, A, B, C, M, N, K, sab, sam, sak, sbb, sbk, sbn, scb,
                     scm, scn, alpha, beta);
  return (int)hipGetLastError();
}
