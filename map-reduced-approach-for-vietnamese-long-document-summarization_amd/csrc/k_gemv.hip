// k_gemv.hip -- decode projections of the map call: weight-streaming skinny GEMM.
//
// Replaces ggml mul_mat at decode time: every decode step
// multiplies the B <= 64 in-flight sequences' rows by every weight matrix once, so the
// step is HBM-bound on the 6.4 GB of bf16 weights.  Design for that:
//  * one block per 16*NT weight rows, the whole K range split over the block's WAVES
//    waves (reduced through LDS) -- no cross-block split-K, so no fences or tickets;
//  * every wave issues the loads of its whole K slice (U steps of 64) before its
//    first MFMA: W straight HBM -> VGPR (no LDS round trip, cdna_hip_programming.md
//    §5 'GEMV / M <= 16'), 32 contiguous bytes per lane per step, so a wave-instruction
//    pair covers 16 full 128-B lines; X (tiny, L2-resident) is staged once per block
//    into LDS and read back as MFMA fragments;
//  * v_mfma_f32_16x16x32_bf16 with the sequences as MFMA rows (M padded to 16*MT);
//    both operands use the same permuted k order (lane group g holds k0+16g..+15),
//    which leaves every dot product unchanged;
//  * epilogues: bf16 store (QKV), fp32 residual add (O, down), SwiGLU on
//    16-row-interleaved gate/up (W_gu), fp32 store (lm_head logits).
// The result is deterministic and independent of the batch composition: a row's
// sum order depends only on K and the launch shape chosen for (N, K).
#include "kernels.h"

namespace ms {

struct GemvPlan {
  int MT, NT, waves, U, tiles;
};

// shape heuristic: U steps of 64 per wave, waves*U*64 == K
static GemvPlan gemv_plan(int M, int N, int K, int epi, int force_waves = 0) {
  GemvPlan p;
  p.MT = (M + 15) / 16;
  p.NT = (epi == 2) ? 2 : 1;
  p.tiles = (N + 16 * p.NT - 1) / (16 * p.NT);
  const int steps = K / 64;
  int best_w = 0;
  if (force_waves > 0 && steps % force_waves == 0 && steps / force_waves <= 8) {
    best_w = force_waves;
  } else {
    // most waves (<= 16) that split K evenly with U <= 8 steps each: measured on MI355X
    // (tools/bench_kernels.py gemv) 16 waves beat 6-12 on every Llama-3.2-3B shape
    for (int w = 16; w >= 1; --w)
      if (steps % w == 0 && steps / w <= 8) { best_w = w; break; }
  }
  p.waves = best_w;
  p.U = best_w ? steps / best_w : 0;
  return p;
}

size_t gemv_workspace_bytes(int, int, int) { return 256; }

// staged X: the M real rows, row stride 2K+16 bytes (the 16-B skew makes the 16 rows of a
// fragment read land on different banks); X rows >= M alias row M-1 and are never stored.
static size_t gemv_x_lds(int M, int K) { return (size_t)M * (2 * (size_t)K + 16); }

static size_t gemv_lds_bytes(const GemvPlan& p, int M, int K, bool xlds) {
  const size_t xs = xlds ? gemv_x_lds(M, K) : 0;
  const size_t red = (size_t)p.waves * p.MT * p.NT * 256 * 4;  // per-wave partials
  return xs > red ? xs : red;
}

__device__ __forceinline__ uint4 ldg16(const bf16_t* p) { return *(const uint4*)p; }

template <int MT, int NT, int EPI, int U, bool XL>
__global__ __launch_bounds__(1024) void gemv_kernel(const bf16_t* __restrict__ X,
                                                    const bf16_t* __restrict__ W,
                                                    void* __restrict__ out, int M, int N, int K,
                                                    int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ELEMS = MT * NT * 256;  // floats per wave result [mt][nt][lane][j]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int kbeg = wave * U * 64;

  // 1. issue this wave's whole W stream first (HBM latency overlaps the X staging)
  uint4 w[U][NT][2];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const bf16_t* wp = W + (size_t)min(n0 + n * 16 + fr, N - 1) * K + kbeg + 16 * fg;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      w[u][n][0] = ldg16(wp + u * 64);
      w[u][n][1] = ldg16(wp + u * 64 + 8);
    }
  }
  // 2. stage the M rows of X into LDS (XL) -- or read fragments from L2 (large M*K)
  const size_t xstride = 2 * (size_t)K + 16;
  if constexpr (XL) {
    const int kch = K / 8;  // 16-B chunks per row
    for (int c = tid; c < M * kch; c += nthreads) {
      const int r = c / kch, k8 = c - r * kch;
      *(uint4*)(smem + r * xstride + k8 * 16) = ldg16(X + (size_t)r * K + k8 * 8);
    }
    __syncthreads();
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int xrow = min(m * 16 + fr, M - 1);
      bf16x8 x0, x1;
      if constexpr (XL) {
        const char* xr = smem + xrow * xstride + (kbeg + u * 64 + 16 * fg) * 2;
        x0 = *(const bf16x8*)xr;
        x1 = *(const bf16x8*)(xr + 16);
      } else {
        const bf16_t* xg = X + (size_t)xrow * K + kbeg + u * 64 + 16 * fg;
        x0 = as_bf16x8(ldg16(xg));
        x1 = as_bf16x8(ldg16(xg + 8));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        acc[m][n] = mfma16(x0, as_bf16x8(w[u][n][0]), acc[m][n]);
        acc[m][n] = mfma16(x1, as_bf16x8(w[u][n][1]), acc[m][n]);
      }
    }
  }
  __syncthreads();  // X image no longer needed: reuse LDS for the partials
  float* red = (float*)smem;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
      *(f32x4*)&red[wave * ELEMS + ((m * NT + n) * 64 + lane) * 4] = acc[m][n];
  __syncthreads();
  const int nw = nthreads >> 6;
  // epilogue: element e = ((m*NT + n)*64 + l)*4 + j -> row m*16 + 4*(l>>4) + j, col n0 + n*16 + (l&15)
  if constexpr (EPI == 2) {
    for (int e = tid; e < MT * 256; e += nthreads) {
      const int m = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int row = m * 16 + 4 * (l >> 4) + j;
      if (row >= M || n0 >= N) continue;
      const int eg = ((m * NT + 0) * 64 + l) * 4 + j, eu = ((m * NT + 1) * 64 + l) * 4 + j;
      float g = 0.f, u = 0.f;
      for (int v = 0; v < nw; ++v) { g += red[v * ELEMS + eg]; u += red[v * ELEMS + eu]; }
      const int f = (n0 >> 5) * 16 + (l & 15);
      ((bf16_t*)out)[(size_t)row * ldo + f] = f2bf(g / (1.0f + __expf(-g)) * u);
    }
  } else {
    for (int e = tid; e < ELEMS; e += nthreads) {
      const int mn = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int m = mn / NT, n = mn % NT;
      const int row = m * 16 + 4 * (l >> 4) + j;
      const int col = n0 + n * 16 + (l & 15);
      if (row >= M || col >= N) continue;
      float v = 0.f;
      for (int q = 0; q < nw; ++q) v += red[q * ELEMS + e];
      const size_t o = (size_t)row * ldo + col;
      if constexpr (EPI == 0) ((bf16_t*)out)[o] = f2bf(v);
      else if constexpr (EPI == 1) ((float*)out)[o] += v;
      else ((float*)out)[o] = v;
    }
  }
}

template <int MT, int NT, int U, bool XL>
static void gemv_launch_x(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo,
                          int epi, const GemvPlan& p, size_t lds, hipStream_t s) {
  const dim3 grid(p.tiles), blk(64 * p.waves);
  if constexpr (NT == 2) {  // only SwiGLU runs on row pairs
    hipLaunchKernelGGL((gemv_kernel<MT, 2, 2, U, XL>), grid, blk, lds, s, X, W, out, M, N, K, ldo);
  } else {
    switch (epi) {
      case 0: hipLaunchKernelGGL((gemv_kernel<MT, 1, 0, U, XL>), grid, blk, lds, s, X, W, out, M, N, K, ldo); break;
      case 1: hipLaunchKernelGGL((gemv_kernel<MT, 1, 1, U, XL>), grid, blk, lds, s, X, W, out, M, N, K, ldo); break;
      default: hipLaunchKernelGGL((gemv_kernel<MT, 1, 3, U, XL>), grid, blk, lds, s, X, W, out, M, N, K, ldo); break;
    }
  }
}

template <int MT, int NT, int U>
static void gemv_launch_u(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo,
                          int epi, const GemvPlan& p, size_t lds, bool xl, hipStream_t s) {
  if (xl) gemv_launch_x<MT, NT, U, true>(X, W, out, M, N, K, ldo, epi, p, lds, s);
  else gemv_launch_x<MT, NT, U, false>(X, W, out, M, N, K, ldo, epi, p, lds, s);
}

template <int MT, int NT>
static void gemv_launch_mn(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo,
                           int epi, const GemvPlan& p, size_t lds, bool xl, hipStream_t s) {
  switch (p.U) {
    case 1: gemv_launch_u<MT, NT, 1>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 2: gemv_launch_u<MT, NT, 2>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 3: gemv_launch_u<MT, NT, 3>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 4: gemv_launch_u<MT, NT, 4>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 5: gemv_launch_u<MT, NT, 5>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 6: gemv_launch_u<MT, NT, 6>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    case 7: gemv_launch_u<MT, NT, 7>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
    default: gemv_launch_u<MT, NT, 8>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s); break;
  }
}

constexpr size_t kMaxLds = 160 * 1024;

bool gemv_supported(int M, int N, int K, int epi) {
  if (M < 1 || M > 64 || K % 64) return false;
  const GemvPlan p = gemv_plan(M, N, K, epi);
  return p.waves > 0 && gemv_lds_bytes(p, M, K, false) <= kMaxLds;
}

void launch_gemv_waves(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo,
                       int epi, int force_waves, hipStream_t s) {
  if (M <= 0) return;
  const GemvPlan p = gemv_plan(M, N, K, epi, force_waves);
  if (p.waves == 0) return;  // callers check gemv_supported()
  const bool xl = gemv_lds_bytes(p, M, K, true) <= kMaxLds;
  const size_t lds = gemv_lds_bytes(p, M, K, xl);
  if (lds > kMaxLds) return;
#define GV(MT_, NT_) gemv_launch_mn<MT_, NT_>(X, W, out, M, N, K, ldo, epi, p, lds, xl, s)
  if (p.NT == 2) {
    switch (p.MT) { case 1: GV(1, 2); break; case 2: GV(2, 2); break; case 3: GV(3, 2); break; default: GV(4, 2); }
  } else {
    switch (p.MT) { case 1: GV(1, 1); break; case 2: GV(2, 1); break; case 3: GV(3, 1); break; default: GV(4, 1); }
  }
#undef GV
}

void launch_gemv(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int ldo, int epi,
                 void*, hipStream_t s) {
  launch_gemv_waves(X, W, out, M, N, K, ldo, epi, 0, s);
}

}  // namespace ms
