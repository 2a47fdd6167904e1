// common.h -- shared device helpers for the gfx950 (CDNA4) map-phase kernels.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

// The engine's 16-bit type is IEEE fp16 (numerics contract): the
// reference runs llama3.2:3b-instruct-fp16 on ggml's F16 path, and fp16 carries three more
// mantissa bits than bf16 at the same MFMA rate on gfx950 (v_mfma_f32_16x16x32_f16).
typedef uint16_t f16_t;  // storage type for fp16 in HBM
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
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

__device__ __forceinline__ float h2f(f16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
// the two fp16 halves of a packed word (low element first, as stored in memory)
__device__ __forceinline__ float h_lo(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w)[0]; }
__device__ __forceinline__ float h_hi(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w)[1]; }

// round-to-nearest-even (v_cvt_f16_f32; overflow -> inf, NaN stays NaN)
__device__ __forceinline__ f16_t f2h(float f) { return __builtin_bit_cast(f16_t, (_Float16)f); }

// one v_cvt_pk_f16_f32 for the pair (same RNE rounding as f2h)
__device__ __forceinline__ uint32_t pack2h(float lo, float hi) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){lo, hi}, f16x2));
}

__device__ __forceinline__ f16x8 as_f16x8(uint4 v) { return __builtin_bit_cast(f16x8, v); }

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
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
