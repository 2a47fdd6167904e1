// attn_common.h -- device helpers shared by the attention kernels (k_attn.hip) and the fused
// QKV projection + decode attention (k_qkvattn.hip): MFMA operand swizzles, the P / V^T
// fragment builders, lane-group reductions and the loads the compiler cannot see.
#pragma once
#include "kernels.h"

namespace ms {

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ int k_swz(int row, int ch) { return row * 256 + ((ch ^ (row & 15)) << 4); }
// Q image of GB heads, rows interleaved ([row][head][256 B], K's chunk swizzle): the heads of
// one k-step sit 256 B apart, inside one ds_read_b128's immediate offset -- one address
// register per k-step instead of one per (head, k-step)
template <int GB>
__device__ __forceinline__ int q_swz(int row, int hh, int ch) { return row * (GB * 256) + hh * 256 + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_swz(int row, int ch) { return row * 256 + ((ch ^ ((row & 7) << 1)) << 4); }

// A operand of O^T += V^T P^T for d-tile dt, k-step ks: two transposed 4x16 reads.
__device__ __forceinline__ f16x8 load_vt(const char* vs, int dt, int ks, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r0 = 32 * ks + 4 * g + q, r1 = r0 + 16;
  const int ch = 2 * dt + (p >> 1), sub = (p & 1) * 8;
  typedef short s4 __attribute__((ext_vector_type(4)));
  s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4*)(vs + v_swz(r0, ch) + sub));
  s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4*)(vs + v_swz(r1, ch) + sub));
  // a vector concatenation (register adjacency): building the 8 shorts element by element
  // compiled to sdwa or/shift repacking, ~80 VALU instructions per attention tile
  return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// B operand P^T for k-step ks from the probabilities of m-tiles 2ks, 2ks+1, rounded to fp16
// (2^-11 relative): the rounding ggml applies to the softmax output before its F16 V.P matmul
// (DESIGN.md section 2).  Round 3 fed bf16 P as two halves (hi + lo, two MFMAs per V^T
// fragment) to keep P.V fp32-accurate; fp16 P needs one.
__device__ __forceinline__ f16x8 pack_p(const f32x4& a, const f32x4& b) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  u4 v = {pack2h(a[0], a[1]), pack2h(a[2], a[3]), pack2h(b[0], b[1]), pack2h(b[2], b[3])};
  return __builtin_bit_cast(f16x8, v);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// max / sum over the 4 lane groups of an MFMA column (lanes l, l^16, l^32, l^48) by
// v_permlane16_swap / v_permlane32_swap: two VALU swaps where __shfl_xor compiled to
// ds_bpermute LDS round trips on the softmax's critical path.  Same pairing and order as the
// xor-16-then-xor-32 shuffles (a + b is commutative), so the same bits.
__device__ __forceinline__ float grp_max(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float grp_sum(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// decode KV pages (plain loads: non-temporal ones measured slower, 2.45 vs 2.29 ms per decode
// step, profiles/r01 v5_nt_stream_ab_rejected)
__device__ __forceinline__ u32x4 ld_stream(const f16_t* p) { return *(const u32x4*)p; }

// One 16-B-per-lane LDS DMA (1 KiB per wave at lds + 16 * lane), issued where the compiler
// cannot see it: after a visible global_load_lds the compiler waits vmcnt(0) before every
// ds_read_b64_tr_b16 (it cannot prove the transposed V reads miss the DMA's LDS bytes), so the
// prefill's P.V of tile t waited for tile t+1's DMA to land.  Callers order the DMA themselves
// (s_waitcnt vmcnt(0) + barrier before the buffer is read).
__device__ __forceinline__ void dma16_opaque(const void* src, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS const char*)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"{m0}"(m0), "v"(src) : "memory");
}

// a barrier for LDS written by ds_write only: waits lgkmcnt, not vmcnt (the pages' loads and the
// V DMA stay in flight across it; gemv_common.h lds_sync)
__device__ __forceinline__ void attn2_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// loads the compiler cannot see (vmcnt retires in issue order, and the compiler's own waits
// only count the loads it sees): the prologue's small L2-resident operands are issued first
// through these, then the page's V DMA and K loads, and ONE manual s_waitcnt vmcnt(32) -- the
// page's 16 + 16 still in flight -- covers them, so the prologue runs while the page streams
__device__ __forceinline__ float ld_f32_opaque(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

}  // namespace ms
