// Parallel column reductions used by the backward passes (GroupNorm
// dgamma/dbeta, conv bias / per-image bias gradients).  Replaces serial
// per-column loops: the row axis is split across blocks (stage A) and the
// <= 64 partials are folded per column (stage B).  Deterministic.
#include "common.h"

__global__ void __launch_bounds__(256) colsum_part_k(const float* __restrict__ in, long R, int Cc, int rows_per,
                                                     float* __restrict__ part) {
  __shared__ float red[8][33];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rl = threadIdx.x >> 5;
  const long r0 = (long)blockIdx.y * rows_per;
  long r1 = r0 + rows_per;
  if (r1 > R) r1 = R;
  float s = 0.f;
  if (c < Cc)
    for (long r = r0 + rl; r < r1; r += 8) s += in[r * Cc + c];
  red[rl][threadIdx.x & 31] = s;
  __syncthreads();
  if (rl == 0 && c < Cc) {
#pragma unroll
    for (int k = 1; k < 8; ++k) s += red[k][threadIdx.x & 31];
    part[(long)blockIdx.y * Cc + c] = s;
  }
}

namespace {
// out[c] = sum_k part[k][c] (optionally de-interleaving pairs into two outputs)
__global__ void colsum_final_k(const float* __restrict__ part, int RS, int Cc, float* __restrict__ out,
                               float* __restrict__ out_odd, int accumulate) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Cc) return;
  float s = 0.f;
  for (int k = 0; k < RS; ++k) s += part[(long)k * Cc + c];
  float* dst = out;
  int idx = c;
  if (out_odd) {
    dst = (c & 1) ? out_odd : out;
    idx = c >> 1;
  }
  dst[idx] = accumulate ? dst[idx] + s : s;
}
}  // namespace

// in: [R][Cc] fp32; part: workspace >= 64*Cc floats.  If out_odd != null,
// even columns go to out[c/2] and odd columns to out_odd[c/2].
D3D_API int d3d_colsum(const float* in, long R, int Cc, float* part, float* out, float* out_odd, int accumulate,
                       hipStream_t st) {
  int RS = (int)((R + 63) / 64);
  if (RS > 64) RS = 64;
  if (RS < 1) RS = 1;
  int rows_per = (int)((R + RS - 1) / RS);
  hipLaunchKernelGGL(colsum_part_k, dim3((Cc + 31) / 32, RS), dim3(256), 0, st, in, R, Cc, rows_per, part);
  hipLaunchKernelGGL(colsum_final_k, dim3((Cc + 255) / 256), dim3(256), 0, st, part, RS, Cc, out, out_odd,
                     accumulate);
  return (int)hipGetLastError();
}

// Batched column sums: up to 16 independent [R][Cc] reductions (the
// whole-image GroupNorm's per-image dgamma/dbeta rows of one weight-gradient
// flush) in ONE launch, a block per 256 columns of a job, each column summed
// over its rows in order (deterministic).  Interleaved pairs go to out0 (even
// columns) and out1 (odd columns), accumulated or stored.  Replaces the two
// launches per GroupNorm of d3d_colsum on the weight-gradient stream.
struct ColJob {
  const float* in;
  float* out0;
  float* out1;
  int R, Cc, acc, blk0;
};
constexpr int kMaxColJobs = 16;
struct ColJobs {
  ColJob j[kMaxColJobs];
  int n;
};

namespace {
__global__ void __launch_bounds__(256) colsum_jobs_k(ColJobs t) {
  int k = 0;
#pragma unroll 1
  while (k + 1 < t.n && (int)blockIdx.x >= t.j[k + 1].blk0) ++k;
  const ColJob& J = t.j[k];
  const int c = ((int)blockIdx.x - J.blk0) * 256 + (int)threadIdx.x;
  if (c >= J.Cc) return;
  const float* p = J.in + c;
  const long ld = J.Cc;
  float s = 0.f;
  int r = 0;
  for (; r + 8 <= J.R; r += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(long)(r + u) * ld];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; r < J.R; ++r) s += p[(long)r * ld];
  float* dst = (c & 1) ? J.out1 : J.out0;
  const int idx = c >> 1;
  dst[idx] = J.acc ? dst[idx] + s : s;
}
}  // namespace

D3D_API int d3d_colsum_jobs(const ColJob* jobs, int njobs, hipStream_t st) {
  if (njobs < 1 || njobs > kMaxColJobs) return (int)hipErrorInvalidValue;
  ColJobs t{};
  t.n = njobs;
  int blk = 0;
  for (int i = 0; i < njobs; ++i) {
    t.j[i] = jobs[i];
    if (t.j[i].Cc % 2 || t.j[i].R < 1 || !t.j[i].in || !t.j[i].out0 || !t.j[i].out1) return (int)hipErrorInvalidValue;
    t.j[i].blk0 = blk;
    blk += (t.j[i].Cc + 255) / 256;
  }
  hipLaunchKernelGGL(colsum_jobs_k, dim3(blk), dim3(256), 0, st, t);
  return (int)hipGetLastError();
}
