// logSNR embedding MLP of the ConditioningProcessor (SURVEY K10;
// reference `xunet.py:32-46` posenc_ddpm, `:273-277` Linear-SiLU-Linear,
// `:305-308` call site):
//
//     pe  = posenc_ddpm(clamp(logsnr, -20, 20))           [R, E]   (R = 2B rows)
//     a1  = pe @ W1^T + b1                                [R, E]
//     out = silu(a1) @ W2^T + b2                          [R, E]
//
// in fp32 (the reference runs this MLP on fp32 activations; it is ~0.1 % of
// the step's FLOPs).  The problem is tiny and row-poor (R = 32..256 against
// E = 1024), so a plain tile per block would occupy a handful of CUs: the
// GEMMs split K over grid.z into fp32 partial slabs that a second launch sums
// in fixed order (deterministic, no atomics) and finishes with the bias /
// activation epilogue.  silu(a1) is never stored -- both the second GEMM and
// the W2 weight gradient apply it while staging a1.
//
// Launches: forward pe, mm, fin, mm, fin; backward mm (dout @ W2), fin
// (x dsilu(a1)), wgrad (W2, b2), wgrad (W1, b1).
#include "common.h"

namespace {
constexpr int MT = 64;     // rows (R) per block tile
constexpr int NTL = 64;    // output columns per block tile
constexpr int KC = 16;     // K staged per LDS step

// pe[r][k]: k < E/2 -> sin(t_r * f_k), else cos(t_r * f_{k - E/2}),
// f_k = exp(-k ln(1e4) / (E/2 - 1)), t_r = clamp(logsnr_r) * 1000 / max_time
__global__ void mlp_pe_k(const float* __restrict__ logsnr, int R, int E, float tscale, float* __restrict__ pe) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)R * E) return;
  const int r = (int)(i / E), k = (int)(i % E), half = E / 2;
  const float l = fminf(fmaxf(logsnr[r], -20.f), 20.f) * tscale;
  const int kk = k < half ? k : k - half;
  const float f = expf((float)kk * (-logf(10000.f) / (float)(half - 1)));
  const float a = l * f;
  pe[i] = k < half ? sinf(a) : cosf(a);
}

// part[z][r][c] = sum_{j in split z} A'(r, j) * B(c, j)
//   A'(r, j) = A[r][j] (ASILU = 0) or silu(A[r][j]) (ASILU = 1)
//   B(c, j)  = W[c][j] (BNN = 0, weight as stored [N][K]) or W[j][c] (BNN = 1, [K][N])
// 256 threads, 4 x 4 outputs each (rows ty*4.., columns tx*4..).
template <int ASILU, int BNN>
__global__ void __launch_bounds__(256) mlp_mm_k(const float* __restrict__ A, const float* __restrict__ W, int R, int N,
                                                int K, int ksplit, float* __restrict__ part) {
  __shared__ float As[KC][MT + 4];
  __shared__ float Bs[KC][NTL + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int c0 = blockIdx.x * NTL, r0 = blockIdx.y * MT;
  const int k0 = blockIdx.z * ksplit, k1 = min(K, k0 + ksplit);
  float acc[4][4] = {};
  for (int kb = k0; kb < k1; kb += KC) {
    {   // A tile: 64 rows x 16 k, one float4 per thread
      const int row = tid >> 2, kq = (tid & 3) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (r0 + row < R) v = *reinterpret_cast<const f32x4*>(A + (long)(r0 + row) * K + kb + kq);
#pragma unroll
      for (int e = 0; e < 4; ++e) As[kq + e][row] = ASILU ? siluf_(v[e]) : v[e];
    }
    if (BNN) {  // W[j][c]: 16 rows j x 64 columns c
      const int j = tid >> 4, cq = (tid & 15) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(W + (long)(kb + j) * N + c0 + cq);
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[j][cq + e] = v[e];
    } else {    // W[c][j]: 64 rows c x 16 k
      const int c = tid >> 2, kq = (tid & 3) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(W + (long)(c0 + c) * K + kb + kq);
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[kq + e][c] = v[e];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&As[k][ty * 4]);
      const f32x4 b = *reinterpret_cast<const f32x4*>(&Bs[k][tx * 4]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* out = part + (long)blockIdx.z * R * N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty * 4 + i;
    if (r < R)
      *reinterpret_cast<f32x4*>(out + (long)r * N + c0 + tx * 4) = f32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
  }
}

// out[r][c] = sum_z part[z][r][c] (fixed order), then
//   EPI 0: + bias[c]            EPI 1: * dsilu(aux[r][c])
template <int EPI>
__global__ void mlp_fin_k(const float* __restrict__ part, int S, int R, int N, const float* __restrict__ bias,
                          const float* __restrict__ aux, float* __restrict__ out) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long RN = (long)R * N;
  if (i * 4 >= RN) return;
  f32x4 s = *reinterpret_cast<const f32x4*>(part + i * 4);
  for (int z = 1; z < S; ++z) s += *reinterpret_cast<const f32x4*>(part + z * RN + i * 4);
  if (EPI == 0) {
    if (bias) s += *reinterpret_cast<const f32x4*>(bias + (i * 4) % N);
  } else {
    const f32x4 a = *reinterpret_cast<const f32x4*>(aux + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] *= dsiluf_(a[e]);
  }
  *reinterpret_cast<f32x4*>(out + i * 4) = s;
}

// dW[c][j] (+)= sum_r G[r][c] * X'(r, j), X' = X or silu(X); db[c] (+)= sum_r G[r][c]
// (computed by the j-tile-0 blocks).  Block tile 64 c x 64 j, R staged 16 rows
// at a time; fixed summation order.
template <int XSILU>
__global__ void __launch_bounds__(256) mlp_wgrad_k(const float* __restrict__ G, const float* __restrict__ X, int R,
                                                   int N, int K, float* __restrict__ dW, float* __restrict__ db,
                                                   int accumulate) {
  __shared__ float Gs[KC][NTL + 4];
  __shared__ float Xs[KC][NTL + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int j0 = blockIdx.x * NTL, c0 = blockIdx.y * NTL;
  float acc[4][4] = {};
  float bsum = 0.f;
  for (int rb = 0; rb < R; rb += KC) {
    {
      const int rr = tid >> 4, q = (tid & 15) * 4;
      f32x4 g = {0.f, 0.f, 0.f, 0.f}, x = {0.f, 0.f, 0.f, 0.f};
      if (rb + rr < R) {
        g = *reinterpret_cast<const f32x4*>(G + (long)(rb + rr) * N + c0 + q);
        x = *reinterpret_cast<const f32x4*>(X + (long)(rb + rr) * K + j0 + q);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Gs[rr][q + e] = g[e];
        Xs[rr][q + e] = XSILU ? siluf_(x[e]) : x[e];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(&Gs[k][ty * 4]);
      const f32x4 x = *reinterpret_cast<const f32x4*>(&Xs[k][tx * 4]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(g[i], x[j], acc[i][j]);
    }
    if (db && blockIdx.x == 0 && tid < NTL)
      for (int k = 0; k < KC; ++k) bsum += Gs[k][tid];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4* o = reinterpret_cast<f32x4*>(dW + (long)(c0 + ty * 4 + i) * K + j0 + tx * 4);
    f32x4 v = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
    if (accumulate) v += *o;
    *o = v;
  }
  if (db && blockIdx.x == 0 && tid < NTL) db[c0 + tid] = accumulate ? db[c0 + tid] + bsum : bsum;
}

int mlp_splits(int R, int N, int K) {
  // enough blocks for ~2 per CU, K chunks of >= 64
  const int tiles = (N / NTL) * ((R + MT - 1) / MT);
  int s = 1;
  while (s < 16 && tiles * s < 512 && K / (s * 2) >= 64 && (K / (s * 2)) % KC == 0) s *= 2;
  return s;
}

bool mlp_ok(int R, int N, int K) { return R > 0 && N % NTL == 0 && K % NTL == 0 && K >= 2 * KC; }
}  // namespace

// Workspace size (floats) for d3d_mlp_mm.
D3D_API long d3d_mlp_ws(int R, int N, int K) { return (long)mlp_splits(R, N, K) * R * N; }

D3D_API int d3d_mlp_pe(const float* logsnr, int R, int E, float tscale, float* pe, hipStream_t st) {
  if (R <= 0 || E < 4 || E % 2) return (int)hipErrorInvalidValue;
  const long n = (long)R * E;
  hipLaunchKernelGGL(mlp_pe_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, logsnr, R, E, tscale, pe);
  return (int)hipGetLastError();
}

// out = epi(A' @ B^T): asilu: A' = silu(A); bnn: W stored [K][N] (else [N][K]);
// epi 0: + bias (may be null), epi 1: * dsilu(aux).  ws: d3d_mlp_ws floats.
D3D_API int d3d_mlp_mm(const float* A, const float* W, int R, int N, int K, int asilu, int bnn, int epi,
                       const float* bias, const float* aux, float* ws, float* out, hipStream_t st) {
  if (!mlp_ok(R, N, K) || (epi == 1 && !aux)) return (int)hipErrorInvalidValue;
  const int S = mlp_splits(R, N, K), ks = K / S;
  dim3 g(N / NTL, (R + MT - 1) / MT, S);
#define MM(AS, BN) hipLaunchKernelGGL((mlp_mm_k<AS, BN>), g, dim3(256), 0, st, A, W, R, N, K, ks, ws)
  if (asilu && bnn) MM(1, 1);
  else if (asilu) MM(1, 0);
  else if (bnn) MM(0, 1);
  else MM(0, 0);
#undef MM
  const long nv = (long)R * N / 4;
  if (epi == 0)
    hipLaunchKernelGGL(mlp_fin_k<0>, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, ws, S, R, N, bias, aux,
                       out);
  else
    hipLaunchKernelGGL(mlp_fin_k<1>, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, ws, S, R, N, bias, aux,
                       out);
  return (int)hipGetLastError();
}

// dW [N][K] (+)= G^T @ X' ; db [N] (+)= colsum(G); xsilu: X' = silu(X)
D3D_API int d3d_mlp_wgrad(const float* G, const float* X, int R, int N, int K, int xsilu, float* dW, float* db,
                          int accumulate, hipStream_t st) {
  if (!mlp_ok(R, N, K)) return (int)hipErrorInvalidValue;
  dim3 g(K / NTL, N / NTL);
  if (xsilu)
    hipLaunchKernelGGL(mlp_wgrad_k<1>, g, dim3(256), 0, st, G, X, R, N, K, dW, db, accumulate);
  else
    hipLaunchKernelGGL(mlp_wgrad_k<0>, g, dim3(256), 0, st, G, X, R, N, K, dW, db, accumulate);
  return (int)hipGetLastError();
}
