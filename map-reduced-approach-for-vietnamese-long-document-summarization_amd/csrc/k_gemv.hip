// k_gemv.hip -- decode projections of the map call: weight-streaming skinny GEMM.
//
// Replaces ggml mul_mat at decode time: every decode step
// multiplies the B <= 64 in-flight sequences' rows by every weight matrix once, so the
// step is HBM-bound on the 6.4 GB of bf16 weights.  Design for that:
//  * W is streamed exactly once per step, straight HBM -> VGPR (no LDS round trip:
//    cdna_hip_programming.md §5 'GEMV / M <= 16' row), 32 contiguous bytes per lane
//    per 64-wide K step, so a wave-instruction pair covers 16 full 128-B lines.
//  * the multiply runs on v_mfma_f32_16x16x32_bf16 with the sequences as MFMA rows
//    (M padded to 16*MT); X is tiny and served from L2.  Both operands use the same
//    permuted k order (lane group g holds k0+16g..+15), which leaves the dot
//    products unchanged.
//  * K is split over the 4 waves of a block (LDS reduce) and, to put >= 1024 blocks
//    on the 256 CUs even for N = 3072, over KSPLIT blocks; the last-arriving block of
//    a tile sums the fp32 slabs in fixed order (deterministic; agent-scope
//    release/acquire ticket of cdna_hip_programming.md §5 'In-launch split-K').
//  * epilogues: bf16 store (QKV), fp32 residual add (O, down), SwiGLU on
//    16-row-interleaved gate/up (W_gu), fp32 store (lm_head logits).
#include "kernels.h"

namespace ms {

struct GemvShape {
  int MT, NT, KSPLIT, tiles;
};

static GemvShape gemv_shape(int M, int N, int K, int epi) {
  GemvShape g;
  g.MT = (M + 15) / 16;
  g.NT = (epi == 2) ? 2 : 1;
  g.tiles = (N + 16 * g.NT - 1) / (16 * g.NT);
  const int units = K / 256;  // 4 waves x 64
  g.KSPLIT = 1;
  const int cand[] = {1, 2, 3, 4, 6, 8, 12, 16};
  for (int c : cand) {
    if (units % c) continue;
    g.KSPLIT = c;
    if (g.tiles * c >= 1024) break;
  }
  return g;
}

// workspace = [kTicketWords uint32 tickets, zeroed once][fp32 slabs]; tickets never alias slabs
constexpr int kTicketWords = 16384;

size_t gemv_workspace_bytes(int M, int N, int K) {
  size_t best = 0;
  for (int epi = 0; epi < 4; ++epi) {
    GemvShape g = gemv_shape(M, N, K, epi);
    size_t b = (size_t)g.tiles * g.KSPLIT * g.MT * g.NT * 256 * 4;
    best = b > best ? b : best;
  }
  return (size_t)kTicketWords * 4 + ((best + 255) & ~(size_t)255);
}

__device__ __forceinline__ uint4 ldg16(const bf16_t* p) { return *(const uint4*)p; }

template <int MT, int NT, int EPI>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ X,
                                                   const bf16_t* __restrict__ W,
                                                   void* __restrict__ out, int M, int N, int K,
                                                   int ldo, int KSPLIT, float* __restrict__ ws,
                                                   unsigned* __restrict__ tickets) {
  constexpr int ELEMS = MT * NT * 256;  // floats per block result [mt][nt][lane][j]
  __shared__ __attribute__((aligned(16))) float red[4 * ELEMS + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int tile = blockIdx.x / KSPLIT, ks = blockIdx.x % KSPLIT;
  const int n0 = tile * 16 * NT;
  const int kspan = K / KSPLIT / 4;
  const int kbeg = ks * (K / KSPLIT) + wave * kspan;

  const bf16_t* wp[NT];
  const bf16_t* xp[MT];
#pragma unroll
  for (int n = 0; n < NT; ++n) wp[n] = W + (size_t)min(n0 + n * 16 + fr, N - 1) * K + kbeg + 16 * fg;
#pragma unroll
  for (int m = 0; m < MT; ++m) xp[m] = X + (size_t)min(m * 16 + fr, M - 1) * K + kbeg + 16 * fg;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int U = (MT <= 2) ? 4 : 2;
  const int steps = kspan / 64;
  int st = 0;
  for (; st + U <= steps; st += U) {
    uint4 w[U][NT][2], x[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        w[u][n][0] = ldg16(wp[n] + (st + u) * 64);
        w[u][n][1] = ldg16(wp[n] + (st + u) * 64 + 8);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        x[u][m][0] = ldg16(xp[m] + (st + u) * 64);
        x[u][m][1] = ldg16(xp[m] + (st + u) * 64 + 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          acc[m][n] = mfma16(as_bf16x8(x[u][m][0]), as_bf16x8(w[u][n][0]), acc[m][n]);
          acc[m][n] = mfma16(as_bf16x8(x[u][m][1]), as_bf16x8(w[u][n][1]), acc[m][n]);
        }
  }
  for (; st < steps; ++st) {
    uint4 w[NT][2], x[MT][2];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      w[n][0] = ldg16(wp[n] + st * 64);
      w[n][1] = ldg16(wp[n] + st * 64 + 8);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      x[m][0] = ldg16(xp[m] + st * 64);
      x[m][1] = ldg16(xp[m] + st * 64 + 8);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        acc[m][n] = mfma16(as_bf16x8(x[m][0]), as_bf16x8(w[n][0]), acc[m][n]);
        acc[m][n] = mfma16(as_bf16x8(x[m][1]), as_bf16x8(w[n][1]), acc[m][n]);
      }
  }

  // in-block reduce over the 4 K-quarters
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
      *(f32x4*)&red[wave * ELEMS + ((m * NT + n) * 64 + lane) * 4] = acc[m][n];
  __syncthreads();

  float* slab = ws + (size_t)(tile * KSPLIT + ks) * ELEMS;
  if (KSPLIT > 1) {
    for (int e = tid; e < ELEMS; e += 256)
      slab[e] = red[e] + red[ELEMS + e] + red[2 * ELEMS + e] + red[3 * ELEMS + e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)&red[4 * ELEMS];
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&tickets[tile], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t == (unsigned)(KSPLIT - 1));
      if (last) {
        __hip_atomic_store(&tickets[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    const float* base = ws + (size_t)tile * KSPLIT * ELEMS;
    for (int e = tid; e < ELEMS; e += 256) {
      float v = 0.f;
      for (int k = 0; k < KSPLIT; ++k) v += base[(size_t)k * ELEMS + e];
      red[e] = v;
    }
  } else {
    for (int e = tid; e < ELEMS; e += 256)
      red[e] = red[e] + red[ELEMS + e] + red[2 * ELEMS + e] + red[3 * ELEMS + e];
  }
  __syncthreads();

  // epilogue: element e = ((m*NT + n)*64 + l)*4 + j -> row m*16 + 4*(l>>4) + j, col n0 + n*16 + (l&15)
  if constexpr (EPI == 2) {
    for (int e = tid; e < MT * 256; e += 256) {
      const int m = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int row = m * 16 + 4 * (l >> 4) + j;
      if (row >= M || n0 >= N) continue;
      const float g = red[((m * NT + 0) * 64 + l) * 4 + j];
      const float u = red[((m * NT + 1) * 64 + l) * 4 + j];
      const int f = (n0 >> 5) * 16 + (l & 15);
      ((bf16_t*)out)[(size_t)row * ldo + f] = f2bf(g / (1.0f + __expf(-g)) * u);
    }
  } else {
    for (int e = tid; e < ELEMS; e += 256) {
      const int mn = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int m = mn / NT, n = mn % NT;
      const int row = m * 16 + 4 * (l >> 4) + j;
      const int col = n0 + n * 16 + (l & 15);
      if (row >= M || col >= N) continue;
      const size_t o = (size_t)row * ldo + col;
      const float v = red[e];
      if constexpr (EPI == 0) ((bf16_t*)out)[o] = f2bf(v);
      else if constexpr (EPI == 1) ((float*)out)[o] += v;
      else ((float*)out)[o] = v;
    }
  }
}

template <int MT, int NT>
static void gemv_dispatch_epi(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K,
                              int ldo, int epi, const GemvShape& g, float* ws, unsigned* tk,
                              hipStream_t s) {
  const dim3 grid(g.tiles * g.KSPLIT), blk(256);
  switch (epi) {
    case 0: hipLaunchKernelGGL((gemv_kernel<MT, NT, 0>), grid, blk, 0, s, X, W, out, M, N, K, ldo, g.KSPLIT, ws, tk); break;
    case 1: hipLaunchKernelGGL((gemv_kernel<MT, NT, 1>), grid, blk, 0, s, X, W, out, M, N, K, ldo, g.KSPLIT, ws, tk); break;
    case 2: hipLaunchKernelGGL((gemv_kernel<MT, NT, 2>), grid, blk, 0, s, X, W, out, M, N, K, ldo, g.KSPLIT, ws, tk); break;
    default: hipLaunchKernelGGL((gemv_kernel<MT, NT, 3>), grid, blk, 0, s, X, W, out, M, N, K, ldo, g.KSPLIT, ws, tk); break;
  }
}

void launch_gemv(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo, int epi,
                 void* ws, hipStream_t s) {
  if (M <= 0) return;
  const GemvShape g = gemv_shape(M, N, K, epi);
  // tickets at the start of the workspace (zeroed once at allocation; last arriver resets)
  if (g.KSPLIT > 1 && g.tiles > kTicketWords) return;  // guarded by the caller (engine.cpp)
  unsigned* tk = (unsigned*)ws;
  float* wsf = (float*)((char*)ws + (size_t)kTicketWords * 4);
#define GV(MT_, NT_) gemv_dispatch_epi<MT_, NT_>(X, W, out, M, N, K, ldo, epi, g, wsf, tk, s)
  if (g.NT == 2) {
    switch (g.MT) { case 1: GV(1, 2); break; case 2: GV(2, 2); break; case 3: GV(3, 2); break; default: GV(4, 2); }
  } else {
    switch (g.MT) { case 1: GV(1, 1); break; case 2: GV(2, 1); break; case 3: GV(3, 1); break; default: GV(4, 1); }
  }
#undef GV
}

}  // namespace ms
