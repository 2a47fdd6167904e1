// Probe: how fast can a decode-attention-shaped read pattern pull K/V from cold HBM when the
// (sequence, kv head) groups are NOT split over CUs (no split-combine needed)?
//   * split4  : 256 blocks, each one distinct 288 KB range (the v2 kernel's shape: 4 splits/group)
//   * group64 : 64 blocks, each one whole group (36 pages x 32 KB = 1.15 MB)
//   * head192x: 192 blocks, one per (group, q head); the 3 blocks of a group on ONE XCD
//               (blockIdx % 8 equal), so the 2nd / 3rd reads can hit that XCD's L2
//   * head192s: same, the 3 blocks of a group spread over 3 XCDs (no L2 sharing)
// Every pattern reads 64 groups x 1.15 MB = 73.7 MB of unique bytes from a 2.5 GB buffer
// (cold: a 1 GB flush write between repetitions).  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// block b reads [base[b], base[b] + len) with its W waves; each lane U x 16 B in flight per step
template <int U>
__global__ void stream_kernel(const u32x4* __restrict__ src, const long* __restrict__ base, long len16,
                              unsigned* __restrict__ out) {
  const long b0 = base[blockIdx.x];
  const int nthr = blockDim.x;
  unsigned acc = 0;
  for (long i = threadIdx.x; i < len16; i += (long)nthr * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * nthr;
      v[u] = j < len16 ? __builtin_nontemporal_load(src + b0 + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// same, default cache policy (plain loads)
template <int U>
__global__ void stream_kernel_dp(const u32x4* __restrict__ src, const long* __restrict__ base, long len16,
                                 unsigned* __restrict__ out) {
  const long b0 = base[blockIdx.x];
  const int nthr = blockDim.x;
  unsigned acc = 0;
  for (long i = threadIdx.x; i < len16; i += (long)nthr * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * nthr;
      v[u] = j < len16 ? src[b0 + j] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void empty_kernel(unsigned* out) { if (threadIdx.x == 1023) out[blockIdx.x] = 0; }

__global__ void flush_kernel(u32x4* p, long n, unsigned s) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = u32x4{s, s, s, s};
}

int main() {
  const long group_bytes = 36L * 32768;            // one (sequence, kv head): 36 pages of K+V
  const long stride = 40L * 1024 * 1024;           // groups spread like a slot-major pool
  const long total = 64 * stride;                  // 2.5 GB
  u32x4 *src, *fl;
  unsigned* out;
  long* dbase;
  CK(hipMalloc(&src, total));
  CK(hipMalloc(&fl, 1L << 30));
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMalloc(&dbase, 4096 * sizeof(long)));
  CK(hipMemset(src, 1, total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  struct Pat { const char* name; int nblk; std::vector<long> base; long len; };
  std::vector<Pat> pats;
  {  // split4: block = split * 64 + group (v2's order), 288 KB each
    Pat p{"split4", 256, {}, group_bytes / 4};
    for (int blk = 0; blk < 256; ++blk) { int sp = blk / 64, g = blk % 64; p.base.push_back((g * stride + sp * (group_bytes / 4)) / 16); }
    pats.push_back(p);
  }
  {  // group64
    Pat p{"group64", 64, {}, group_bytes};
    for (int blk = 0; blk < 64; ++blk) p.base.push_back(blk * stride / 16);
    pats.push_back(p);
  }
  {  // head192x: block i -> xcd i%8, slot j = i/8 (0..23), group xcd*8 + j/3
    Pat p{"head192x", 192, {}, group_bytes};
    for (int blk = 0; blk < 192; ++blk) { int x = blk % 8, j = blk / 8; p.base.push_back((long)(x * 8 + j / 3) * stride / 16); }
    pats.push_back(p);
  }
  {  // head192s: group = i / 3 (consecutive blocks -> consecutive XCDs)
    Pat p{"head192s", 192, {}, group_bytes};
    for (int blk = 0; blk < 192; ++blk) p.base.push_back((long)(blk / 3) * stride / 16);
    pats.push_back(p);
  }
  {  // head192x with half-range: 384 blocks, (group, q head, half) -- still needs a 2-way merge
    Pat p{"head384x_half", 384, {}, group_bytes / 2};
    for (int blk = 0; blk < 384; ++blk) { int x = blk % 8, j = blk / 8; int gi = j / 6, rem = j % 6; p.base.push_back(((long)(x * 8 + gi) * stride + (rem & 1) * (group_bytes / 2)) / 16); }
    pats.push_back(p);
  }

  {  // event overhead: an empty 256-block launch between the same events
    std::vector<float> ts;
    for (int rep = 0; rep < 12; ++rep) {
      flush_kernel<<<2048, 256>>>(fl, (1L << 30) / 16, rep);
      CK(hipEventRecord(e0));
      empty_kernel<<<256, 64>>>(out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 2) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    printf("empty launch between events: %.2f us (median)\n", ts[ts.size() / 2]);
  }
  const int waves_list[] = {4, 8, 9, 12, 16};
  printf("pattern        waves U  policy   us_med   unique_TB/s\n");
  for (auto& p : pats) {
    CK(hipMemcpy(dbase, p.base.data(), p.base.size() * sizeof(long), hipMemcpyHostToDevice));
    for (int w : waves_list) {
      for (int U : {4, 8, 16}) {
        for (int pol = 0; pol < 2; ++pol) {
          std::vector<float> ts;
          for (int rep = 0; rep < 12; ++rep) {
            flush_kernel<<<2048, 256>>>(fl, (1L << 30) / 16, rep);
            CK(hipEventRecord(e0));
#define L(UU) do { if (pol) stream_kernel_dp<UU><<<p.nblk, 64 * w>>>(src, dbase, p.len / 16, out); else stream_kernel<UU><<<p.nblk, 64 * w>>>(src, dbase, p.len / 16, out); } while (0)
            if (U == 4) L(4); else if (U == 8) L(8); else L(16);
#undef L
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2) ts.push_back(ms * 1000.f);
          }
          std::sort(ts.begin(), ts.end());
          const float med = ts[ts.size() / 2];
          printf("%-14s %5d %2d  %-6s %8.2f   %6.2f\n", p.name, w, U, pol ? "plain" : "nt", med, 64.0 * group_bytes / (med * 1e-6) / 1e12);
          fflush(stdout);
        }
      }
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
