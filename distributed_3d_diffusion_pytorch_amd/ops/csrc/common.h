// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of d3d_hip.
//
// Conventions:
//   * activations are NHWC bf16 ([N, H, W, C], N = 2*B frame-interleaved);
//   * parameters are fp32 masters, read directly by the kernels (or through a
//     packed bf16 copy for the MFMA operands);
//   * every launcher is `extern "C" int d3d_<op>(..., hipStream_t)` returning
//     the hipError_t of the launch, so Python drives it via ctypes with the
//     current torch stream (graph-capture safe: no allocation, no sync).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define D3D_API extern "C" __attribute__((visibility("default")))
#define WAVE 64

__device__ __forceinline__ f32x8 ld8(const bf16* p) {
  return __builtin_convertvector(*reinterpret_cast<const bf16x8*>(p), f32x8);
}
__device__ __forceinline__ void st8(bf16* p, f32x8 v) {
  *reinterpret_cast<bf16x8*>(p) = __builtin_convertvector(v, bf16x8);
}
__device__ __forceinline__ f32x8 ld8f(const float* p) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// sigmoid through the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the
// IEEE division sequence (~10 VALU: scale, rcp, Newton steps, fixup): every
// SiLU / dSiLU user -- the GroupNorm passes, the FiLM dgrad epilogue, the conv
// SiLU epilogues -- is VALU-heavy.  exp(-x) = inf gives rcp(inf) = 0.
// (D3D_SIGMOID_IEEE: the division form, for the same-box A/B build only.)
#ifdef D3D_SIGMOID_IEEE
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
#else
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
#endif
__device__ __forceinline__ float siluf_(float x) { return x * sigmoidf_(x); }
// d/dx silu(x) = s * (1 + x * (1 - s))
__device__ __forceinline__ float dsiluf_(float x) {
  float s = sigmoidf_(x);
  return s * (1.0f + x * (1.0f - s));
}

// Counter-based RNG for dropout masks: splitmix64 finalizer over
// (seed, element index).  Stateless, so backward regenerates the mask.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (uint32_t)(z >> 32);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  return (hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
}

// Dropout mask: a 32-bit counter hash ("lowbias32": two multiplies) of the
// element index xor a per-call key, compared with p * 2^32.  A quarter of the
// VALU cost of splitmix64 -- the GN-FiLM-dropout passes are VALU-bound on the
// 64-bit mixer.  Forward and backward regenerate the same mask.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(uint64_t seed) {
  return lowbias32((uint32_t)seed ^ lowbias32((uint32_t)(seed >> 32) + 0x9e3779b9U));
}
__device__ __forceinline__ uint32_t drop_threshold(float p) { return (uint32_t)((double)p * 4294967296.0); }
__device__ __forceinline__ bool drop_elem(uint32_t key, uint64_t idx, uint32_t thr) {
  return lowbias32((uint32_t)idx ^ key) < thr;
}

// Box-Muller normal from two counter-based uniforms.
__device__ __forceinline__ float normal01(uint64_t seed, uint64_t idx) {
  float u1 = ((hash_u32(seed, 2 * idx) >> 8) + 1) * (1.0f / 16777217.0f);
  float u2 = (hash_u32(seed, 2 * idx + 1) >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Chan et al. parallel merge of (count, mean, M2) partial moments.
struct Moments {
  float n, mean, m2;
};
__device__ __forceinline__ Moments merge_moments(Moments a, Moments b) {
  float n = a.n + b.n;
  if (n <= 0.f) return a;
  float d = b.mean - a.mean;
  float fb = b.n / n;
  Moments r;
  r.n = n;
  r.mean = a.mean + d * fb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
  return r;
}

// Optional second conv output: silu of the stored (bf16-rounded) output
// values, written next to them by the conv epilogue (the conditioning convs,
// whose output feeds the FiLM projections through a SiLU, xunet.py:84).
__device__ __forceinline__ void silu_store4(bf16* __restrict__ O2, long off, bf16x4 o4) {
  bf16x4 s4;
#pragma unroll
  for (int e = 0; e < 4; ++e) s4[e] = (bf16)siluf_((float)o4[e]);
  *reinterpret_cast<bf16x4*>(O2 + off) = s4;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Compute units of the CURRENT device (launch planners size grids in whole
// waves of blocks per CU), cached per device ordinal: a process that drives
// several GPUs -- or one whose current device is not 0 -- gets each device's
// own count.  (Every MI355X has 256; the cache only avoids the query per launch.)
static inline int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev];
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return n;
}

// ----------------------------------------- fused GroupNorm statistics -----
// GroupNorm partial statistics of a conv output, produced by the conv's
// epilogue so the GroupNorm that consumes the output skips its statistics
// pass (one full read of the activation).  Granularity: one group x 64
// pixels of one image (HW % 64 == 0): gnp[((n * G + g) * nparts + t) * 2] =
// (sum, sum of squares) of the bf16-rounded outputs, t = (pixel % HW) / 64,
// nparts = HW / 64.  Every slot is written by exactly one wave: no atomics,
// deterministic.  s/q: per (16-channel MFMA row tile i, 64-pixel half h)
// lane sums over its 4 channels and its pixels.
template <int TM, int NH>
__device__ __forceinline__ void gn_part_store(float (&s)[TM][NH], float (&q)[TM][NH], int lane, int co_base,
                                              long pix0, int OC, int G, int HW, long Mpix, float* __restrict__ gnp) {
  const int fr = lane & 15, fq = lane >> 4;
  const int Cg = OC / G;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float a = s[i][h], b = q[i][h];
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {         // the 16 pixels of a fragment column
        a += __shfl_xor(a, m, 64);
        b += __shfl_xor(b, m, 64);
      }
      if (Cg >= 8) {                              // 4-channel lane groups -> 8 / 16 / 32-channel groups
        a += __shfl_xor(a, 16, 64);
        b += __shfl_xor(b, 16, 64);
      }
      if (Cg >= 16) {
        a += __shfl_xor(a, 32, 64);
        b += __shfl_xor(b, 32, 64);
      }
      s[i][h] = a;
      q[i][h] = b;
    }
  if (fr != 0) return;
  const int nparts = HW / 64;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int co = co_base + i * 16 + fq * 4;
    if (Cg >= 32) {                               // 32-channel groups span two row tiles
      if ((i & 1) || fq != 0) continue;
    } else if (fq % (Cg / 4) != 0) {
      continue;
    }
    if (co >= OC) continue;
    const int g = co / Cg;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const long p = pix0 + h * 64;
      if (p >= Mpix) continue;
      float a = s[i][h], b = q[i][h];
      if (Cg >= 32 && i + 1 < TM) {
        a += s[i + 1][h];
        b += q[i + 1][h];
      }
      const long n = p / HW;
      const int t = (int)(p - n * HW) / 64;
      float* d = gnp + ((n * G + g) * nparts + t) * 2;
      d[0] = a;
      d[1] = b;
    }
  }
}
