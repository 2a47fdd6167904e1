// k_dgemm.hip -- decode projections at large batch: a skinny GEMM for 16 < M <= 256 rows.
//
// The continuous batch of BASELINE configs[2] keeps B = 64..256 sequences in flight per GPU
// ("B_max chosen to fit KV"), and every decode step multiplies those B rows
// by every weight matrix once (ggml mul_mat).  The weight-streaming
// GEMV (k_gemv.hip) owns 16 weight rows per block and re-reads all M x K activations per
// block: at M = 64 the gate/up launch reads 4x more X from L2 than W from HBM and stalls on
// L2.  Here a block owns 64 weight rows (4 waves x 16) and ALL M rows:
//  * X (M x 64 per K step) goes HBM/L2 -> LDS by global_load_lds (1 KiB per wave
//    instruction, source-side XOR swizzle chunk ^ (row & 7): conflict-free ds_read_b128),
//    double-buffered; the 4 waves share it, so X is read from L2 once per 64 weight rows;
//  * W streams straight to VGPRs, each wave its own 16 rows, PF K steps in flight
//    (32 contiguous bytes per lane per step, as in the GEMV);
//  * v_mfma_f32_16x16x32_bf16, the wave's 16 weight rows as MFMA columns, MT m-tiles;
//  * split-K over gridDim.y for the narrow projections (fp32 slabs, folded by the next
//    residual_rmsnorm / attention prologue exactly like the GEMV's).
// A row's sum order depends only on (K, split), never on M or on the other rows.
#include "gemv_common.h"

namespace ms {

constexpr int DBN = 64, DBK = 64, DPF = 3;

template <int MT, int EPI>
__global__ __launch_bounds__(256, 2) void dgemm_kernel(const bf16_t* __restrict__ X,
                                                      const bf16_t* __restrict__ W,
                                                      void* __restrict__ out, int M, int N, int K,
                                                      int ldk, int ldo) {
  constexpr int XB = 16 * MT * DBK * 2;  // one X stage: 16*MT rows x 128 B
  __shared__ __attribute__((aligned(16))) char smem[2 * XB > 4 * MT * 256 * 4 ? 2 * XB : 4 * MT * 256 * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * DBN;
  const int kb = blockIdx.y * K;  // this split's K range in rows of length ldk
  if constexpr (EPI == MS_GEMV_EPI_STORE_F32) out = (float*)out + (size_t)blockIdx.y * M * ldo;

  // X DMA: instruction i of a stage covers rows 4*(wave*MT/2... ) -- rows r = i*32 + tid/8,
  // chunk c = tid&7 written at LDS row r, chunk c, from global chunk c ^ (r & 7)
  constexpr int XI = (16 * MT * 8 + 255) / 256;  // 16-B DMA pieces per thread per stage
  auto stage_x = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = i * 32 + (tid >> 3);
      if (r < 16 * MT) {
        const int gc = (tid & 7) ^ (r & 7);
        const bf16_t* src = X + (size_t)min(r, M - 1) * ldk + kb + k0 + gc * 8;
        char* dst = smem + buf * XB + (i * 32 + (wave << 3)) * 128;  // wave's 8 rows of piece i
        __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)dst, 16, 0, 0);
      }
    }
  };
  // W: lane (fr, fg) holds k0 + 16 fg .. +15 of row n0 + 16 wave + fr (32 contiguous bytes),
  // a DPF-slot register ring; X: the same permuted k order from the LDS image
  const bf16_t* wrow = W + (size_t)min(n0 + 16 * wave + fr, N - 1) * ldk + kb + 16 * fg;
  uint4 wr[DPF][2];
  const int nk = K / DBK;
#pragma unroll
  for (int p = 0; p < DPF - 1; ++p)
    if (p < nk) {
      wr[p][0] = ldw16(wrow + p * DBK);
      wr[p][1] = ldw16(wrow + p * DBK + 8);
    }
  stage_x(0, 0);

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    // issue order per step: W(t+DPF-1) into the slot step t-1 consumed, then X(t+1); vmcnt is
    // in order, so X(t) -- and every older W, W(t) included -- has landed once at most the
    // ops issued after it are pending
    const bool wmore = t + DPF - 1 < nk, more = t + 1 < nk;
    if (wmore) {
      wr[(t + DPF - 1) % DPF][0] = ldw16(wrow + (t + DPF - 1) * DBK);
      wr[(t + DPF - 1) % DPF][1] = ldw16(wrow + (t + DPF - 1) * DBK + 8);
    }
    if (more) stage_x(buf ^ 1, (t + 1) * DBK);
    if (wmore) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 + XI));
    else if (more) __builtin_amdgcn_s_waitcnt(vmcnt_imm(XI));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    __syncthreads();
    const uint4 w0 = wr[t % DPF][0], w1 = wr[t % DPF][1];
    const char* xs = smem + buf * XB;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 16 + fr;
      const bf16x8 x0 = *(const bf16x8*)(xs + row * 128 + (((2 * fg) ^ (row & 7)) << 4));
      const bf16x8 x1 = *(const bf16x8*)(xs + row * 128 + (((2 * fg + 1) ^ (row & 7)) << 4));
      acc[m] = mfma16(x0, as_bf16x8(w0), acc[m]);
      acc[m] = mfma16(x1, as_bf16x8(w1), acc[m]);
    }
    __syncthreads();  // every wave is done with buf before X(t+2) overwrites it
  }

  // epilogue: acc[m][j] = C[row m*16 + 4 fg + j][col n0 + 16 wave + fr]
  const int col = n0 + 16 * wave + fr;
  if constexpr (EPI == MS_GEMV_EPI_SWIGLU) {
    // waves 2q / 2q+1 hold the gate / up tile of the same 16 features: pair through LDS
    float* xch = (float*)smem;  // [4 waves][MT][64 lanes][4]
#pragma unroll
    for (int m = 0; m < MT; ++m) *(f32x4*)&xch[((wave * MT + m) * 64 + lane) * 4] = acc[m];
    __syncthreads();
    if (wave & 1) return;
    const int f = (n0 >> 5) * 16 + (wave >> 1) * 16 + fr;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x4 u = *(const f32x4*)&xch[(((wave + 1) * MT + m) * 64 + lane) * 4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + 4 * fg + j;
        if (row < M && f < N / 2) {
          const float gte = acc[m][j];
          ((bf16_t*)out)[(size_t)row * ldo + f] = f2bf(gte / (1.0f + __expf(-gte)) * u[j]);
        }
      }
    }
  } else if constexpr (EPI == MS_GEMV_EPI_ARGMAX) {
    // {max, id} of the row over this wave's 16 columns (lanes fr share row 4 fg + j)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + 4 * fg + j;
        float v = (col < N) ? acc[m][j] : -INFINITY;
        if (!(v == v)) v = -INFINITY;
        int idx = col;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
        if (fr == 0 && row < M) ((float2*)out)[(size_t)row * ldo + (n0 >> 4) + wave] = make_float2(v, __int_as_float(idx));
      }
  } else {
    if (col >= N) return;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + 4 * fg + j;
        if (row >= M) continue;
        const size_t o = (size_t)row * ldo + col;
        if constexpr (EPI == MS_GEMV_EPI_STORE_BF16) ((bf16_t*)out)[o] = f2bf(acc[m][j]);
        else if constexpr (EPI == MS_GEMV_EPI_ADD_F32) ((float*)out)[o] += acc[m][j];
        else ((float*)out)[o] = acc[m][j];
      }
  }
}

bool dgemm_supported(int M, int N, int K, int S, int epi) {
  if (M < 1 || M > 256 || N % 64 || S < 1 || K % (S * DBK)) return false;
  if (epi == MS_GEMV_EPI_ROPE_KV) return false;
  if (S > 1 && epi != MS_GEMV_EPI_STORE_F32) return false;
  return true;
}

template <int MT>
static void dgemm_go(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int S, int ldo,
                     int epi, hipStream_t s) {
  const dim3 grid(N / DBN, S), blk(256);
  const int Ks = K / S;
  switch (epi) {
#define DG(E_) MS_LAUNCH((dgemm_kernel<MT, E_>), grid, blk, 0, s, X, W, out, M, N, Ks, K, ldo)
    case MS_GEMV_EPI_STORE_BF16: DG(MS_GEMV_EPI_STORE_BF16); break;
    case MS_GEMV_EPI_ADD_F32: DG(MS_GEMV_EPI_ADD_F32); break;
    case MS_GEMV_EPI_SWIGLU: DG(MS_GEMV_EPI_SWIGLU); break;
    case MS_GEMV_EPI_ARGMAX: DG(MS_GEMV_EPI_ARGMAX); break;
    default: DG(MS_GEMV_EPI_STORE_F32); break;
#undef DG
  }
}

void launch_dgemm(const bf16_t* X, const bf16_t* W, void* out, int M, int N, int K, int S, int ldo, int epi,
                  hipStream_t s) {
  if (!dgemm_supported(M, N, K, S, epi)) return;  // callers check
  const int mt = (M + 15) / 16;
  if (mt <= 1) dgemm_go<1>(X, W, out, M, N, K, S, ldo, epi, s);
  else if (mt <= 2) dgemm_go<2>(X, W, out, M, N, K, S, ldo, epi, s);
  else if (mt <= 4) dgemm_go<4>(X, W, out, M, N, K, S, ldo, epi, s);
  else if (mt <= 8) dgemm_go<8>(X, W, out, M, N, K, S, ldo, epi, s);
  else dgemm_go<16>(X, W, out, M, N, K, S, ldo, epi, s);
}

}  // namespace ms
