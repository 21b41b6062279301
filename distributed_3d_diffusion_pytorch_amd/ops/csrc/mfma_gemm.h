// Shared pieces of the hand-written MFMA GEMM kernels (gemm.hip: the
// per-pixel dense layers; wgrad_gemm.hip: their weight gradients): inline-asm
// MFMAs on AGPR-constrained accumulators, LDS-DMA and buffer load / store
// helpers, and a compile-time loop.  The helpers are plain (non-template)
// device functions: the address-space cast and the buffer descriptor are
// device-only constructs that the host pass of a kernel template must never
// instantiate.
#pragma once
#include "common.h"

#include <utility>

namespace {
#define G_BAR()                        \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

__device__ __forceinline__ void g_mma(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void g_mma0(f32x4& c, const bf16x8& a, const bf16x8& b) {   // first K-tile: C = 0
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

// LDS-DMA of 16 bytes per lane from buffer (base, nrec bytes) at voff + soff
// into lds (wave-uniform base + lane * 16).  Plain (non-template) helpers:
// the address-space cast and the descriptor are device-only constructs that
// the host pass of a kernel template must never instantiate.
__device__ __forceinline__ void g_dma(const void* base, int nrec, void* lds, int voff, int soff) {
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000),
                                           (lds_void*)lds, 16, voff, soff, 0, 0);
}
// the same with a cache policy (CPOL: 1 sc0, 2 nt, 16 sc1) -- the streamed operand of the dense GEMM
template <int CPOL>
__device__ __forceinline__ void g_dma_cp(const void* base, int nrec, void* lds, int voff, int soff) {
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000),
                                           (lds_void*)lds, 16, voff, soff, 0, CPOL);
}
typedef unsigned g_u4 __attribute__((ext_vector_type(4)));
typedef unsigned g_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ g_u2 g_load8(const void* base, int nrec, int off) {
  return __builtin_amdgcn_raw_buffer_load_b64(__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000),
                                              off, 0, 0);
}
__device__ __forceinline__ void g_store16(const void* base, int nrec, g_u4 v, int off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000),
                                         off, 0, 0);
}

// Transposed LDS read (ds_read_b64_tr_b16): per 16-lane group, lane 4q + p
// addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane i receives
// column i of the 4 rows (row q in element q).
__device__ __forceinline__ g_u2 g_trd(const void* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s4 lds_s4;
  return __builtin_bit_cast(g_u2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)p));
}

// LDS-DMA issued from inline asm (buffer descriptor in SGPRs, M0 set inside):
// the compiler does not see an LDS write, so it inserts no conservative vmcnt
// wait before every later LDS read (it cannot tell the DMA's target buffer
// from the one being read) -- the kernel counts vmcnt itself.  s_nop 4: the
// descriptor / M0 operands may be fresh SGPR writes.
typedef int g_i4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ g_i4 g_desc(const void* base, int nrec) {
  const unsigned long a = (unsigned long)base;
  return g_i4{(int)(unsigned)a, (int)((a >> 32) & 0xffff), nrec, 0x00020000};
}
__device__ __forceinline__ unsigned g_lds_u32(const void* p) {
  typedef __attribute__((address_space(3))) const char lds_char;
  return (unsigned)(unsigned long)(lds_char*)p;
}
__device__ __forceinline__ void g_dma_asm(g_i4 desc, unsigned lds, int voff) {
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds), "v"(voff), "s"(desc)
               : "memory", "m0");
}

// base + step as an opaque VALU add: never hoisted out of a loop, so a per-piece
// offset costs one instruction at its use instead of a live register
__device__ __forceinline__ int g_vadd(int base, int step) {
  int r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "s"(step), "v"(base));
  return r;
}

template <int... I, typename F>
__device__ __forceinline__ void g_for(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

}  // namespace
