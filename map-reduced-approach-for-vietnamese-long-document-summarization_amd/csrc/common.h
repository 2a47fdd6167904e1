// common.h -- shared device helpers for the gfx950 (CDNA4) map-phase kernels.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // storage type for bf16 in HBM
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))

namespace ms {

// Kernel-duration probe: when the engine's profiling mask selects a kernel class it points
// g_prof at an event pair; the next MS_LAUNCH then goes through hipExtLaunchKernelGGL, which
// timestamps exactly that dispatch (no extra stream commands between kernels).
struct ProfEvents {
  hipEvent_t start, stop;
};
extern thread_local ProfEvents* g_prof;

#define MS_LAUNCH(K, G, B, L, S, ...)                                                       \
  do {                                                                                      \
    if (::ms::g_prof) {                                                                     \
      hipExtLaunchKernelGGL(K, G, B, L, S, ::ms::g_prof->start, ::ms::g_prof->stop, 0,      \
                            __VA_ARGS__);                                                   \
      ::ms::g_prof = nullptr;                                                               \
    } else {                                                                                \
      hipLaunchKernelGGL(K, G, B, L, S, __VA_ARGS__);                                       \
    }                                                                                       \
  } while (0)

constexpr int kWave = 64;
constexpr int kHeadDim = 128;
constexpr int kPage = 64;  // KV page = 64 tokens = one attention K/V tile

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float((uint32_t)u << 16); }

// round-to-nearest-even; hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 (NaN-safe)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// one v_cvt_pk_bf16_f32 for the pair (same RNE rounding as f2bf): packing two f2bf results
// by shift + or compiled to two converts, a shift and an sdwa or
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){lo, hi}, b2));
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// In-launch hand-off words (cdna_hip_programming.md §6 Guideline 16, counter form with
// write-through payload): every handed-off word is stored and loaded sc1 (relaxed agent-scope
// atomics on GLOBAL pointers), every storing wave drains vmcnt before the workgroup barrier,
// one lane adds to the counter, the block whose add returns count-1 is the reducer.
typedef __attribute__((address_space(1))) unsigned gu32_t;
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gu32_t*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// all storing waves drained + one arrival; true in every thread of the last arriving block.
// flag: one LDS word no thread reads or writes otherwise during the call.
__device__ __forceinline__ bool arrive_last(unsigned* ticket, unsigned count, unsigned* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((gu32_t*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (t == count - 1) ? 1u : 0u;
  }
  __syncthreads();
  const bool last = *flag != 0u;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below
  return last;
}


}  // namespace ms
