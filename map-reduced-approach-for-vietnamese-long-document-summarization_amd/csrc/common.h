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

}  // namespace ms
