// k_gemm.hip -- prefill projections of the map call on MFMA (gfx950).
//
// Replaces ggml mul_mat for QKV / O / gate+up / down over the packed prompt tokens
// of every chunk in flight (SURVEY.md §2 "ggml op replaced", §8a row A8).
// out (epilogue) A[M][K] . W[N][K]^T ; A = activations (bf16, K-contiguous),
// W = nn.Linear weight [out][in] (bf16, K-contiguous): an "NT" GEMM, so both MFMA
// operands are read along K and no transpose is ever needed.
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16.  Both operands stream HBM->LDS with global_load_lds
// dwordx4 (1 KiB per wave-instruction, lane-linear); the LDS image is XOR-swizzled
// by pre-swizzling the per-lane SOURCE address (chunk ^ (row & 7)), so the
// ds_read_b128 fragment reads are conflict-free (cdna_hip_programming.md §5.4 rule 21,
// T2).  Two LDS stages: the next K-tile's DMA is in flight while the current one is
// multiplied.  Block order: group-M raster + bijective XCD remap (T1) so that the
// blocks sharing an A panel run on one XCD's L2.
// Epilogues fuse the residual add (O, down) and SwiGLU (gate/up rows interleaved
// per 16 on upload) so no extra HBM pass is spent on them.
#include "kernels.h"

namespace ms {

constexpr int GBM = 128, GBN = 128, GBK = 64;

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ float silu_mul(float g, float u) { return g / (1.0f + __expf(-g)) * u; }

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const bf16_t* __restrict__ A,
                                                     const bf16_t* __restrict__ W,
                                                     void* __restrict__ out, int M, int N, int K,
                                                     int ldo) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * GBM * GBK * 2];  // 64 KiB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = (M + GBM - 1) / GBM, tiles_n = (N + GBN - 1) / GBN;
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int grp = pid / (GM * tiles_n);
  const int first_m = grp * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_grp = pid % (GM * tiles_n);
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * GBM, n0 = tn * GBN;

  // per-lane DMA sources: wave-instruction i = wave*4+t covers tile rows 8i..8i+7
  const bf16_t* a_src[4];
  const bf16_t* b_src[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int r = (wave * 4 + t) * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (r & 7);
    a_src[t] = A + (size_t)min(m0 + r, M - 1) * K + gc * 8;
    b_src[t] = W + (size_t)min(n0 + r, N - 1) * K + gc * 8;
  }
  auto stage = [&](int st, int k0) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      char* da = smem + st * 32768 + (wave * 4 + t) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)(a_src[t] + k0), (LDS_AS void*)da, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(b_src[t] + k0), (LDS_AS void*)(da + 16384),
                                       16, 0, 0);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * GBK);
    const char* As = smem + cur * 32768;
    const char* Bs = As + 16384;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row = wm * 64 + m * 16 + fr;
        const int ch = (4 * s + fg) ^ (row & 7);
        af[m] = *(const bf16x8*)(As + row * 128 + ch * 16);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + fr;
        const int ch = (4 * s + fg) ^ (row & 7);
        bfr[n] = *(const bf16x8*)(Bs + row * 128 + ch * 16);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(af[m], bfr[n], acc[m][n]);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // epilogue: acc[m][n][j] = C[row 4*fg + j][col fr] of 16x16 tile (m, n)
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = m0 + wm * 64 + m * 16 + fg * 4 + j;
      if (row >= M) continue;
      if constexpr (EPI == 2) {  // SwiGLU: n even = gate, n odd = up of the same 16 features
#pragma unroll
        for (int n = 0; n < 4; n += 2) {
          const int col = n0 + wn * 64 + n * 16;  // multiple of 32
          if (col >= N) continue;
          const int f = (col >> 5) * 16 + fr;
          ((bf16_t*)out)[(size_t)row * ldo + f] = f2bf(silu_mul(acc[m][n][j], acc[m][n + 1][j]));
        }
      } else {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int col = n0 + wn * 64 + n * 16 + fr;
          if (col >= N) continue;
          const size_t o = (size_t)row * ldo + col;
          if constexpr (EPI == 0) ((bf16_t*)out)[o] = f2bf(acc[m][n][j]);
          else if constexpr (EPI == 1) ((float*)out)[o] += acc[m][n][j];
          else ((float*)out)[o] = acc[m][n][j];
        }
      }
    }
  }
}

void launch_gemm(const bf16_t* A, const bf16_t* W, void* out, int M, int N, int K, int ldo, int epi,
                 hipStream_t s) {
  if (M <= 0) return;
  const int grid = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  switch (epi) {
    case 0: MS_LAUNCH(gemm_kernel<0>, dim3(grid), dim3(256), 0, s, A, W, out, M, N, K, ldo); break;
    case 1: MS_LAUNCH(gemm_kernel<1>, dim3(grid), dim3(256), 0, s, A, W, out, M, N, K, ldo); break;
    case 2: MS_LAUNCH(gemm_kernel<2>, dim3(grid), dim3(256), 0, s, A, W, out, M, N, K, ldo); break;
    default: MS_LAUNCH(gemm_kernel<3>, dim3(grid), dim3(256), 0, s, A, W, out, M, N, K, ldo); break;
  }
}

}  // namespace ms
