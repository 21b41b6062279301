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

// ----------------------------------------------------- job-table form ----
// Many tiny fp32 products in ONE launch from a device-resident job table:
// the attention block's merged output map W = W_lin . W_out, b = W_lin .
// b_out + b_lin (forward operand, refreshed after each optimizer step) and
// the split of its weight gradient back onto W_lin / W_out (ops/hip_impl.py
// _AttnOut):
//
//     acc = sum_k A[m][k] B[k][n]                (A null: acc = 0)
//     C[m][n] = alpha * acc + beta * C[m][n] + u[m] * (v ? v[n] : 1)   (u optional)
//
// written as fp32 C, and / or bf16 Cb[m][n], and / or bf16 CbT[n][m]
// (row strides ldb / ldbt).  Element strides for every operand, so
// transposed views cost nothing.  64 x 64 tiles; block b runs tile b -
// tile0 of the job whose tile range holds it.
struct SgJob {
  const float* A;
  const float* B;
  float* C;
  bf16* Cb;
  bf16* CbT;
  const float* u;
  const float* v;
  long sam, sak, sbk, sbn, scm, scn;
  int M, N, K, ldb, ldbt, tile0;
  float alpha, beta;
};
static_assert(sizeof(SgJob) == 136, "SgJob must match hip_impl._SgJob");

constexpr int SJ_K = 32;          // K per LDS stage of the job-table form

__global__ void __launch_bounds__(256) sgemm_jobs_k(const SgJob* __restrict__ jobs, int njobs) {
  __shared__ float As[SJ_K][SG_T + 1];
  __shared__ float Bs[SJ_K][SG_T + 1];
  int j = 0;
  while (j + 1 < njobs && (int)blockIdx.x >= jobs[j + 1].tile0) ++j;
  const SgJob& J = jobs[j];
  const int t = blockIdx.x - J.tile0;
  const int ntn = (J.N + SG_T - 1) / SG_T;
  const int m0 = (t / ntn) * SG_T, n0 = (t % ntn) * SG_T;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  // loads walk the operand's contiguous axis across consecutive lanes
  // (k-major when the k stride is 1, else m / n-major): coalesced either way
  const bool a_k = J.sak == 1, b_k = J.sbk == 1;
  if (J.A) {
    for (int k0 = 0; k0 < J.K; k0 += SJ_K) {
      for (int e = threadIdx.x; e < SJ_K * SG_T; e += 256) {
        int kk = e / SG_T, mm = e % SG_T;
        if (a_k) { kk = e % SJ_K; mm = e / SJ_K; }
        const int gm = m0 + mm, gk = k0 + kk;
        As[kk][mm] = (gm < J.M && gk < J.K) ? J.A[gm * J.sam + gk * J.sak] : 0.f;
        int kb = e / SG_T, nn = e % SG_T;
        if (b_k) { kb = e % SJ_K; nn = e / SJ_K; }
        const int gn = n0 + nn, gkb = k0 + kb;
        Bs[kb][nn] = (gn < J.N && gkb < J.K) ? J.B[gkb * J.sbk + gn * J.sbn] : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int kk = 0; kk < SJ_K; ++kk) {
        float av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = As[kk][ty + 16 * i];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = Bs[kk][tx + 16 * q];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[i][q] = __builtin_fmaf(av[i], bv[q], acc[i][q]);
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + ty + 16 * i;
    if (gm >= J.M) continue;
    const float um = J.u ? J.u[gm] : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int gn = n0 + tx + 16 * q;
      if (gn >= J.N) continue;
      float r = J.alpha * acc[i][q];
      if (J.C && J.beta != 0.f) r += J.beta * J.C[gm * J.scm + gn * J.scn];
      if (J.u) r += um * (J.v ? J.v[gn] : 1.f);
      if (J.C) J.C[gm * J.scm + gn * J.scn] = r;
      if (J.Cb) J.Cb[(long)gm * J.ldb + gn] = (bf16)r;
      if (J.CbT) J.CbT[(long)gn * J.ldbt + gm] = (bf16)r;
    }
  }
}

// jobs: device table of njobs SgJob (tile0 ascending, tiles laid out back to
// back); tiles: total blocks.
D3D_API int d3d_sgemm_jobs(const void* jobs, int njobs, int tiles, hipStream_t st) {
  if (njobs <= 0 || tiles <= 0) return -1;
  hipLaunchKernelGGL(sgemm_jobs_k, dim3((unsigned)tiles), dim3(256), 0, st, (const SgJob*)jobs, njobs);
  return (int)hipGetLastError();
}
