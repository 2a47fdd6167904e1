// dma_probe.hip -- how many bytes must one CU keep in flight, and in which form, to stream HBM
// at speed on MI355X?  (Design probe for the persistent decode step, k_persist.hip.)
//
// 256 workgroups (one per CU) each stream their own 8 MiB slice of a 2 GiB buffer:
//   mode 0: LDS DMA (global_load_lds_dwordx4, 1 KiB per instruction) by `loaders` waves into a
//           ring in LDS, each wave keeping `depth` instructions in flight (s_waitcnt vmcnt(depth));
//   mode 1: global_load_dwordx4 into registers by `loaders` waves, `depth` 1-KiB wave loads in
//           flight per wave (the GEMV form), the data summed so the loads stay live.
// The other waves of the 256-thread workgroup idle.  Prints GB/s per configuration.
//   build: hipcc --offload-arch=gfx950 -O3 tools/dma_probe.hip -o tools/bin/dma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ void dma16(const void* src, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS const char*)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"{m0}"(m0), "v"(src) : "memory");
}

template <int DEPTH>
__device__ __forceinline__ void waitd() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DEPTH) : "memory");
}

constexpr size_t kSlice = 8u << 20;  // bytes per workgroup

template <int DEPTH>
__global__ __launch_bounds__(256, 1) void dma_stream(const char* __restrict__ buf, int loaders, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= loaders) return;
  const char* base = buf + (size_t)blockIdx.x * kSlice;
  const int n = (int)(kSlice / 1024);  // 1-KiB instructions per workgroup
  char* ring = smem + wave * 32768;      // 32 KiB per loader wave (content irrelevant)
  for (int i = wave; i < n; i += loaders) {
    dma16(base + (size_t)i * 1024 + lane * 16, ring + (i / loaders & 31) * 1024);
    waitd<DEPTH>();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && wave == 0 && sink) sink[blockIdx.x] = ((float*)smem)[0];
}

template <int DEPTH>
__global__ __launch_bounds__(256, 1) void reg_stream(const char* __restrict__ buf, int loaders, float* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= loaders) return;
  const char* base = buf + (size_t)blockIdx.x * kSlice;
  const int n = (int)(kSlice / 1024);
  uint4 acc = {0, 0, 0, 0};
  uint4 r[DEPTH];
  int i = wave;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) r[d] = *(const uint4*)(base + (size_t)(i + d * loaders) * 1024 + lane * 16);
  for (i += DEPTH * loaders; i < n; i += DEPTH * loaders) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc.x ^= r[d].x; acc.y ^= r[d].y; acc.z ^= r[d].z; acc.w ^= r[d].w;
      r[d] = *(const uint4*)(base + (size_t)(i + d * loaders) * 1024 + lane * 16);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) { acc.x ^= r[d].x; acc.y ^= r[d].y; }
  if (sink) sink[blockIdx.x * 256 + threadIdx.x] = (float)(acc.x ^ acc.y ^ acc.z ^ acc.w);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <class K>
static double run(K k, int loaders, const char* buf, float* sink, size_t lds) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(256), dim3(256), lds, 0, buf, loaders, sink);  // warm
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(256), lds, 0, buf, loaders, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return 5.0 * 256 * kSlice / (ms / 1e3) / 1e9;
}

int main() {
  char* buf;
  float* sink;
  CK(hipMalloc(&buf, 256 * kSlice));
  CK(hipMalloc(&sink, 256 * 256 * sizeof(float)));
  CK(hipMemset(buf, 1, 256 * kSlice));
  const size_t lds = 4 * 32768;
  printf("mode       loaders depth(KiB in flight per wave)  GB/s (chip)  GB/s per CU\n");
#define D(DEP)                                                                                      \
  for (int L = 1; L <= 4; L *= 2) {                                                                 \
    double g = run(dma_stream<DEP>, L, buf, sink, lds);                                             \
    printf("lds-dma    %d       %2d                            %7.0f     %6.1f\n", L, DEP, g, g / 256); \
  }
  D(8) D(16) D(32) D(48) D(62)
#define Rg(DEP)                                                                                     \
  for (int L = 1; L <= 4; L *= 2) {                                                                 \
    double g = run(reg_stream<DEP>, L, buf, sink, 0);                                               \
    printf("registers  %d       %2d                            %7.0f     %6.1f\n", L, DEP, g, g / 256); \
  }
  Rg(8) Rg(16) Rg(32)
  return 0;
}
