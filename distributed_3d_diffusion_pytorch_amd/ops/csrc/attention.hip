// Fused multi-head self / cross-view attention on gfx950 MFMA.
//
// Reference: AttnLayer / AttnBlock (xunet.py:154-220) -> nn.MultiheadAttention
// with 4 heads, dispatched as bmm -> softmax -> bmm that MATERIALISES the
// [B*4, L, L] probabilities (and head-averaged weights) for both frames and for
// self and cross attention separately.
//
// Here one launch handles every (image, head, 64-query block) of a layer; the
// key/value frame is n (self) or n^1 (cross: the two views of an example are
// adjacent rows of the frame-folded batch).  Input is the packed in_proj
// output qkv [N, L, 3C] (q | k | v, head h at columns h*D..h*D+D-1), output is
// [N, L, C].  Nothing of size L x L ever leaves registers.
//
// Forward (flash, online softmax):  S^T = K Q^T is formed with keys on the
// MFMA rows so that P^T lands in registers already laid out as the B operand
// of O^T = V^T P^T (no LDS round trip for P); V^T fragments come from the
// transpose read ds_read_b64_tr_b16 on a padded [key][D] LDS tile.  The key
// order inside each 32-key MFMA step is permuted identically for both
// operands (sum order is irrelevant), which is what makes the register reuse
// and the conflict-free transpose reads line up.
//
// Backward (flash v2 recompute, one workgroup per 64-key block):
// S = Q K^T and dP = dO V^T with KEYS on the lane, so P and dS are already the
// A operands of dV = P^T dO and dK = dS^T Q; dQ = dS K goes through LDS once
// into a per-key-block fp32 slab, and the slabs are summed in fixed order
// (deterministic, no atomics).  The softmax-backward row term
// D = rowsum(dO * O) is formed in the kernel while the query tile loads (no
// preprocessing launch), and a sequence one workgroup covers (L = 64 with
// 64-key workgroups; 64 < L <= 256 with the 8-wave 256-key workgroup that is
// the default at head dim 64) writes bf16 dQ directly (no slab, no
// conversion launch).  The forward likewise has a one-workgroup-per-(image,
// head) form for 64 < L <= 256 with all of K / V resident in LDS.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ s16x4 ds_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8 tr8(const bf16* base, int stride, int r1, int r2, int col) {
  s16x4 lo = ds_tr(base + r1 * stride + col);
  s16x4 hi = ds_tr(base + r2 * stride + col);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ bf16x8 pack8(f32x4 a, f32x4 b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}
// swizzled [row][D] tile of 16-byte chunks for ds_read_b128 row reads
template <int D>
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * D + ((chunk ^ (row & 7)) << 3);
}

// ------------------------------------------------------------ forward ----
// KALL: one workgroup per (image, head) for L <= 256 -- 16 waves, one per 16
// queries, with the whole K / V of the sequence staged in LDS once (one
// barrier); the 64-query workgroups each re-load every K / V block and wait
// on it (prefetched one block ahead, still one round trip per block).
template <int D, bool KALL = false>
__global__ void __launch_bounds__(KALL ? 1024 : 256) attn_fwd_k(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                               float* __restrict__ lse, int L, int C, int heads,
                                                               int cross, float scale) {
  constexpr int VS = D + 16;                 // padded V row (tr reads)
  constexpr int KC = D / 32;                 // 32-wide k chunks over head dim
  constexpr int DT = D / 16;                 // 16-wide dv tiles
  constexpr int KR = KALL ? 256 : 64, NT = KALL ? 1024 : 256;     // staged key rows, threads
  __shared__ __attribute__((aligned(16))) bf16 Ks[KR * D];
  __shared__ __attribute__((aligned(16))) bf16 Vs[KR * VS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int qblk = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int nkv = cross ? (n ^ 1) : n;
  const int g = lane >> 4, fr = lane & 15;
  const long C3 = 3L * C;
  const int q = qblk * (NT / 4) + w * 16 + fr;
  const bool qok = q < L;                    // ragged last query block (L % 64 != 0)
  const bf16* qrow = qkv + ((long)n * L + (qok ? q : 0)) * C3 + h * D;
  bf16x8 qf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
    qf[kc] = qok ? *reinterpret_cast<const bf16x8*>(qrow + 32 * kc + 8 * g) : bf16x8{};

  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float sl2 = scale * LOG2E;
  const int qq = (lane & 15) >> 2, pc = lane & 3;

  // cooperative K/V block loads, one block ahead: block kb + 64 is in flight
  // in registers while block kb computes (was one HBM round trip per block)
  constexpr int CH = D / 8;                  // chunks per row
  constexpr int NKV = KR * CH / NT;          // chunks per thread of each of K / V
  bf16x8 kr[NKV], vr[NKV];
  auto fetch = [&](int kb) {
#pragma unroll
    for (int i = 0; i < NKV; ++i) {
      int idx = tid + i * NT;
      int r = idx / CH, c = idx % CH;
      const bool kok = kb + r < L;
      const bf16* src = qkv + ((long)nkv * L + (kok ? kb + r : 0)) * C3 + h * D + c * 8;
      kr[i] = kok ? *reinterpret_cast<const bf16x8*>(src + C) : bf16x8{};
      vr[i] = kok ? *reinterpret_cast<const bf16x8*>(src + 2 * C) : bf16x8{};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < NKV; ++i) {
      int idx = tid + i * NT;
      int r = idx / CH, c = idx % CH;
      *reinterpret_cast<bf16x8*>(Ks + swz<D>(r, c)) = kr[i];
      *reinterpret_cast<bf16x8*>(Vs + r * VS + c * 8) = vr[i];
    }
  };
  fetch(0);
  if constexpr (KALL) {                      // every key of the sequence (rows past L zero), one barrier
    stage();
    __syncthreads();
    if (w * 16 >= L) return;                 // no queries for this wave (no barrier follows)
  }
  for (int kb = 0; kb < L; kb += 64) {
    if constexpr (!KALL) {
      stage();
      if (kb + 64 < L) fetch(kb + 64);
      __syncthreads();
    }
    // this key block's rows (the swizzle depends on row & 7 only)
    const bf16* Kb = Ks + (KALL ? kb * D : 0);
    const bf16* Vb = Vs + (KALL ? kb * VS : 0);
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(Kb + swz<D>(16 * kt + fr, 4 * kc + g));
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[kc], s[kt], 0, 0, 0);
      }
    }
    // online softmax over this block's 64 keys for query column q
    float mb = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[kt][i] = kb + 16 * kt + 4 * g + i < L ? s[kt][i] * sl2 : -INFINITY;   // keys past L
        mb = fmaxf(mb, s[kt][i]);
      }
    mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    float mn = fmaxf(m, mb);
    float alpha = exp2f(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[kt][i] = exp2f(s[kt][i] - mn);
        ls += s[kt][i];
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
    // O^T += V^T P^T, two 32-key steps
#pragma unroll
    for (int kc2 = 0; kc2 < 2; ++kc2) {
      bf16x8 pb = pack8(s[2 * kc2], s[2 * kc2 + 1]);
      int r1 = 32 * kc2 + 4 * g + qq, r2 = 32 * kc2 + 16 + 4 * g + qq;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        bf16x8 va = tr8(Vb, VS, r1, r2, 16 * t + 4 * pc);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[t], 0, 0, 0);
      }
    }
    if constexpr (!KALL) __syncthreads();
  }
  if (!qok) return;
  const float inv = 1.f / l;
  bf16* orow = out + ((long)n * L + q) * C + h * D;
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    bf16x4 v4;
#pragma unroll
    for (int i = 0; i < 4; ++i) v4[i] = (bf16)(o[t][i] * inv);
    *reinterpret_cast<bf16x4*>(orow + 16 * t + 4 * g) = v4;
  }
  if (g == 0) lse[((long)n * heads + h) * L + q] = (m + log2f(l)) / LOG2E;
}

// --------------------------------------------------------------- backward --
// KW keys per workgroup (KW / 16 waves of 16 keys).  KW = 64: four 64-key
// blocks per (image, head) at L = 256, each writing its own fp32 dQ slab
// (summed by dq_convert_k).  KW = 256: ONE workgroup owns every key of an
// L <= 256 sequence (8 waves of 2 x 16 keys), so dQ = dS K is complete inside
// it and leaves as bf16 directly: no slabs (4 x N x L x C fp32 written and
// re-read at the 16x16 level: ~270 MB per call at 256 frames), no conversion
// launch, and each query / dO tile is read once instead of once per key block.
template <int D, int KW = 64>
__global__ void __launch_bounds__(KW == 256 ? 512 : 256) attn_bwd_k(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                     const float* __restrict__ lse, const bf16* __restrict__ out,
                                                     float* __restrict__ dq_acc, bf16* __restrict__ dqkv, int L, int C,
                                                     int heads, int cross, float scale) {
  constexpr int KC = D / 32, DT = D / 16;
  // waves (4, or 8 for KW = 256: 2 x 16-key groups per wave -- at 16 waves
  // the 128-register budget spilled), threads, key groups per wave
  constexpr int NWV = KW == 256 ? 8 : 4, NT = 64 * NWV, KG = KW / (16 * NWV);
  constexpr int TS = D + 16;      // padded rows: row reads + tr reads
  constexpr int SS = KW + 8;      // dS tile row stride (bf16)
  __shared__ __attribute__((aligned(16))) bf16 Qs[32 * TS];
  __shared__ __attribute__((aligned(16))) bf16 dOs[32 * TS];
  __shared__ __attribute__((aligned(16))) bf16 Kt[KW * TS];
  __shared__ __attribute__((aligned(16))) bf16 dSs[32 * SS];
  __shared__ float lse_s[32], D_s[32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kblk = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int nkv = cross ? (n ^ 1) : n;
  const int g = lane >> 4, fr = lane & 15, qq = (lane & 15) >> 2, pc = lane & 3;
  const long C3 = 3L * C;
  const int k0 = kblk * KW;
  const float sl2 = scale * LOG2E;
  constexpr int CH = D / 8;

  // K tile of the block (for dQ) and this wave's K / V fragments (B operands)
#pragma unroll
  for (int i = 0; i < KW * CH / NT; ++i) {
    int idx = tid + i * NT;
    int r = idx / CH, c = idx % CH;
    *reinterpret_cast<bf16x8*>(Kt + r * TS + c * 8) =
        k0 + r < L ? *reinterpret_cast<const bf16x8*>(qkv + ((long)nkv * L + k0 + r) * C3 + C + h * D + c * 8)
                   : bf16x8{};
  }
  // key group kg of this wave: keys k0 + 16 (w + NWV kg) + 0..15
  bool kok[KG];
  bf16x8 kf[KG][KC], vf[KG][KC];
  f32x4 dk[KG][DT], dv[KG][DT];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    const int key = k0 + 16 * (w + NWV * kg) + fr;
    kok[kg] = key < L;                            // ragged last key block (L % 64 != 0)
    const bf16* krow = qkv + ((long)nkv * L + (kok[kg] ? key : 0)) * C3 + h * D;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      kf[kg][kc] = kok[kg] ? *reinterpret_cast<const bf16x8*>(krow + C + 32 * kc + 8 * g) : bf16x8{};
      vf[kg][kc] = kok[kg] ? *reinterpret_cast<const bf16x8*>(krow + 2 * C + 32 * kc + 8 * g) : bf16x8{};
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      dk[kg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[kg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float* lse_nh = lse + ((long)n * heads + h) * L;
  const bool direct_dq = L <= KW;                 // one key block: dQ is complete here

  // the query tile (Q, dO rows) and the D-term operands (O, dO row parts) of
  // tile q0 + 32 are loaded into registers while tile q0 computes: the loop
  // was one HBM round trip per 32-query step with nothing to overlap it
  // (7 % MFMA in the bs128 step counters)
  constexpr int NQ = (32 * CH + NT - 1) / NT;     // 16-byte chunks per thread of each of Q / dO
  constexpr int PER = D / 8;                      // D-term elements per lane (8 or 16)
  bf16x8 qr[NQ], dr[NQ], orr[PER / 8], drr[PER / 8];
  float lse_r = 0.f;
  bool lse_ok = false;
  auto fetch = [&](int qb) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      int idx = tid + i * NT;
      int r = idx / CH, c = idx % CH;
      const bool ok = idx < 32 * CH && qb + r < L;
      long row = (long)n * L + (ok ? qb + r : 0);
      qr[i] = ok ? *reinterpret_cast<const bf16x8*>(qkv + row * C3 + h * D + c * 8) : bf16x8{};
      dr[i] = ok ? *reinterpret_cast<const bf16x8*>(dout + row * C + h * D + c * 8) : bf16x8{};
    }
    {
      // (threads past the first 256: row r >= 32, nothing to load)
      const int r = tid >> 3, part = tid & 7;
      const bool ok = r < 32 && qb + r < L;
      const long row = (long)n * L + (ok ? qb + r : 0);
#pragma unroll
      for (int k = 0; k < PER / 8; ++k) {
        orr[k] = ok ? *reinterpret_cast<const bf16x8*>(out + row * C + h * D + part * PER + 8 * k) : bf16x8{};
        drr[k] = ok ? *reinterpret_cast<const bf16x8*>(dout + row * C + h * D + part * PER + 8 * k) : bf16x8{};
      }
    }
    // unconditional load, used next step (a use inside a lane branch made
    // the compiler wait for every prefetch above at the branch's end)
    const int li = qb + (tid & 31);
    lse_ok = tid < 32 && li < L;
    lse_r = lse_nh[li < L ? li : 0];
  };
  fetch(0);

  for (int q0 = 0; q0 < L; q0 += 32) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      int idx = tid + i * NT;
      if (idx < 32 * CH) {
        int r = idx / CH, c = idx % CH;
        *reinterpret_cast<bf16x8*>(Qs + r * TS + c * 8) = qr[i];
        *reinterpret_cast<bf16x8*>(dOs + r * TS + c * 8) = dr[i];
      }
    }
    // query rows past L: lse = +inf makes their probabilities exactly 0
    if (tid < 32) lse_s[tid] = lse_ok ? lse_r * LOG2E : INFINITY;
    {
      // D[q] = sum_d dO[q, d] O[q, d]: 8 adjacent lanes per query row
      const int r = tid >> 3, part = tid & 7;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < PER / 8; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += (float)orr[k][j] * (float)drr[k][j];
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      acc += __shfl_xor(acc, 4, 64);
      if (part == 0 && r < 32) D_s[r] = acc;
    }
    if (q0 + 32 < L) fetch(q0 + 32);              // in flight during this tile's compute
    __syncthreads();
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      f32x4 p[2], ds[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          bf16x8 a = *reinterpret_cast<const bf16x8*>(Qs + (16 * qt + fr) * TS + 32 * kc + 8 * g);
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, kf[kg][kc], s, 0, 0, 0);
          bf16x8 b = *reinterpret_cast<const bf16x8*>(dOs + (16 * qt + fr) * TS + 32 * kc + 8 * g);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, vf[kg][kc], dp, 0, 0, 0);
        }
        // rows: q = 16qt + 4g + i ; column (lane): key
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int qi = 16 * qt + 4 * g + i;
          float pv = kok[kg] ? exp2f(s[i] * sl2 - lse_s[qi]) : 0.f;
          p[qt][i] = pv;
          ds[qt][i] = pv * (dp[i] - D_s[qi]);
        }
      }
      // dV += P^T dO ; dK += dS^T Q  (k-slots permuted: q = {4g+j, 16+4g+j})
      bf16x8 pa = pack8(p[0], p[1]);
      bf16x8 dsa = pack8(ds[0], ds[1]);
      int r1 = 4 * g + qq, r2 = 16 + 4 * g + qq;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        bf16x8 bo = tr8(dOs, TS, r1, r2, 16 * t + 4 * pc);
        dv[kg][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, bo, dv[kg][t], 0, 0, 0);
        bf16x8 bq = tr8(Qs, TS, r1, r2, 16 * t + 4 * pc);
        dk[kg][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsa, bq, dk[kg][t], 0, 0, 0);
      }
      // dS -> LDS [32 q][KW keys] for dQ = dS K
      // columns are stored in the permuted k-slot order of the tr-read K operand:
      // key u of a 32-key chunk -> slot 8*(u/4)+u%4 (u<16), 8*((u-16)/4)+4+u%4
      {
        const int kl = 16 * (w + NWV * kg) + fr, u = kl & 31;
        const int col = (kl & ~31) + (u < 16 ? 8 * (u >> 2) + (u & 3) : 8 * ((u - 16) >> 2) + 4 + (u & 3));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int i = 0; i < 4; ++i) dSs[(16 * qt + 4 * g + i) * SS + col] = (bf16)ds[qt][i];
      }
    }
    __syncthreads();
    // dQ tiles: 2 (q) x DT (d) tiles over the waves
    for (int tt = w; tt < 2 * DT; tt += NWV) {
      int qt = tt / DT, t = tt % DT;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KW / 32; ++kc) {   // KW keys = KW / 32 x 32
        bf16x8 a = *reinterpret_cast<const bf16x8*>(dSs + (16 * qt + fr) * SS + 32 * kc + 8 * g);
        bf16x8 b = tr8(Kt, TS, 32 * kc + 4 * g + qq, 32 * kc + 16 + 4 * g + qq, 16 * t + 4 * pc);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
      // acc rows: q = 16qt + 4g + i, col d = 16t + fr ... (A rows = q).
      // This key block's dQ contribution goes to its own slab (plain stores,
      // every element written once); dq_convert_k sums the slabs in key-block
      // order, so dQ is bitwise reproducible (fp32 atomics were not)
      if (direct_dq) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (q0 + 16 * qt + 4 * g + i >= L) continue;
          long row = (long)n * L + q0 + 16 * qt + 4 * g + i;
          dqkv[row * C3 + h * D + 16 * t + fr] = (bf16)(acc[i] * scale);
        }
      } else {
        float* slab = dq_acc + (long)kblk * gridDim.z * L * C;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (q0 + 16 * qt + 4 * g + i >= L) continue;
          long row = (long)n * L + q0 + 16 * qt + 4 * g + i;
          slab[row * C + h * D + 16 * t + fr] = acc[i] * scale;
        }
      }
    }
  }
  // write dK, dV for this wave's keys: dk[kg][t][i] = dK[key = 16 (w + NWV kg) + 4g+i][d = 16t+fr]
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = k0 + 16 * (w + NWV * kg) + 4 * g + i;
        if (kk >= L) continue;
        long row = (long)nkv * L + kk;
        dqkv[row * C3 + C + h * D + 16 * t + fr] = (bf16)(dk[kg][t][i] * scale);
        dqkv[row * C3 + 2 * C + h * D + 16 * t + fr] = (bf16)dv[kg][t][i];
      }
}

// dQ = sum over the kb key-block slabs (fixed order) -> bf16 q-columns of dqkv
__global__ void dq_convert_k(const float* __restrict__ dq, bf16* __restrict__ dqkv, long rows, int C, int kb) {
  const long total = rows * C / 8, slab = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long r = (i * 8) / C;
    int c = (int)((i * 8) % C);
    f32x8 s = ld8f(dq + i * 8);
    for (int k = 1; k < kb; ++k) s += ld8f(dq + k * slab + i * 8);
    st8(dqkv + r * 3L * C + c, s);
  }
}

}  // namespace

// qkv: [N, L, 3C] bf16; out: [N, L, C] bf16; lse: [N, heads, L] fp32.
// D = C/heads in {64, 128}; any L >= 1 (a ragged last 64-block is masked).
// One 16-wave workgroup per (image, head) for 64 < L <= 256 at head dim 64 once
// there are at least this many (image, head) pairs: bs128 (1024 pairs) +0.1%;
// at bs16 (128 pairs, half the CUs idle) the 64-query workgroups win by 0.5%.
static int g_attn_fwd_all_min = 512;
D3D_API void d3d_attn_fwd_cfg(int min_pairs) { g_attn_fwd_all_min = min_pairs; }
D3D_API int d3d_attn_fwd(const void* qkv, void* out, float* lse, int N, int L, int C, int heads, int cross,
                         float scale, hipStream_t st) {
  int D = C / heads;
  if (L < 1) return (int)hipErrorInvalidValue;
  if (D == 64 && L > 64 && L <= 256 && N * heads >= g_attn_fwd_all_min) {
    hipLaunchKernelGGL((attn_fwd_k<64, true>), dim3(1, heads, N), dim3(1024), 0, st, (const bf16*)qkv, (bf16*)out, lse,
                       L, C, heads, cross, scale);
    return (int)hipGetLastError();
  }
  dim3 grid((L + 63) / 64, heads, N);
  if (D == 64)
    hipLaunchKernelGGL(attn_fwd_k<64>, grid, dim3(256), 0, st, (const bf16*)qkv, (bf16*)out, lse, L, C, heads, cross,
                       scale);
  else if (D == 128)
    hipLaunchKernelGGL(attn_fwd_k<128>, grid, dim3(256), 0, st, (const bf16*)qkv, (bf16*)out, lse, L, C, heads,
                       cross, scale);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// KW = 256 (one workgroup per (image, head), dQ written directly) for
// head dim 64 and 64 < L <= 256 from g_attn_wide_min (image, head) pairs on
// (default: always -- +0.6 % at bs16 and bs128, +1.1 % at bs32, even with
// half the CUs busy at bs16's 128 pairs); else 64-key workgroups + fp32 dQ
// slabs.
static long g_attn_wide_min = 0;      // measured faster at bs16 / 32 / 128 (profiles/r6/attn_wide_bwd.txt)
D3D_API void d3d_attn_bwd_cfg(int wide_min_pairs) { g_attn_wide_min = wide_min_pairs; }
static bool attn_wide(int N, int L, int C, int heads) {
  return heads > 0 && C / heads == 64 && L > 64 && L <= 256 && (long)N * heads >= g_attn_wide_min;
}
// fp32 dQ slabs d3d_attn_bwd needs for this shape (0: dQ is written directly)
D3D_API int d3d_attn_bwd_slabs(int N, int L, int C, int heads) {
  return (L <= 64 || attn_wide(N, L, C, heads)) ? 0 : (L + 63) / 64;
}

// dq_acc: [d3d_attn_bwd_slabs(...), N, L, C] fp32 workspace (one slab per
// 64-key block, fully written; may be null when no slab is needed); dqkv:
// [N, L, 3C] bf16 output (every element written).
D3D_API int d3d_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* dq_acc,
                         void* dqkv, int N, int L, int C, int heads, int cross, float scale, hipStream_t st) {
  int D = C / heads;
  const int slabs = d3d_attn_bwd_slabs(N, L, C, heads);
  if (L < 1 || (slabs > 0 && dq_acc == nullptr)) return (int)hipErrorInvalidValue;
  if (attn_wide(N, L, C, heads)) {
    hipLaunchKernelGGL((attn_bwd_k<64, 256>), dim3(1, heads, N), dim3(512), 0, st, (const bf16*)qkv,
                       (const bf16*)dout, lse, (const bf16*)out, dq_acc, (bf16*)dqkv, L, C, heads, cross, scale);
    return (int)hipGetLastError();
  }
  const int kblocks = (L + 63) / 64;
  dim3 grid(kblocks, heads, N);
  if (D == 64)
    hipLaunchKernelGGL(attn_bwd_k<64>, grid, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse,
                       (const bf16*)out, dq_acc, (bf16*)dqkv, L, C, heads, cross, scale);
  else if (D == 128)
    hipLaunchKernelGGL(attn_bwd_k<128>, grid, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse,
                       (const bf16*)out, dq_acc, (bf16*)dqkv, L, C, heads, cross, scale);
  else
    return (int)hipErrorInvalidValue;
  if (L <= 64) return (int)hipGetLastError();
  long rows = (long)N * L;
  long g = (rows * C / 8 + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(dq_convert_k, dim3((int)g), dim3(256), 0, st, dq_acc, (bf16*)dqkv, rows, C, kblocks);
  return (int)hipGetLastError();
}
