// k_gemm.hip -- prefill projections of the map call on MFMA (gfx950).
//
// Replaces ggml mul_mat for QKV / O / gate+up / down over the packed prompt tokens
// of every chunk in flight (SURVEY.md §2 "ggml op replaced", §8a row A8).
// out (epilogue) A[M][K] . W[N][K]^T ; A = activations (fp16, K-contiguous),
// W = nn.Linear weight [out][in] (fp16, K-contiguous): an "NT" GEMM, so both MFMA
// operands are read along K and no transpose is ever needed.
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_f16.  Both operands stream HBM->LDS with global_load_lds
// dwordx4 (1 KiB per wave-instruction, lane-linear); the LDS image is XOR-swizzled
// by pre-swizzling the per-lane SOURCE address (chunk ^ (row & 7)), so the
// ds_read_b128 fragment reads are conflict-free (cdna_hip_programming.md §5.4 rule 21,
// T2).  Two LDS stages: the next K-tile's DMA is in flight while the current one is
// multiplied.  Block order: group-M raster + bijective XCD remap (T1) so that the
// blocks sharing an A panel run on one XCD's L2.
// Epilogues fuse the residual add (O, down) and SwiGLU (gate/up rows interleaved
// per 16 on upload) so no extra HBM pass is spent on them; the normalised projections (QKV,
// gate/up, logits) scale each output row by its deferred RMSNorm factor (kernels.h RowScale,
// one tile: rs_rinv(ssq[row])).
#include "kernels.h"

namespace ms {

constexpr int GBM = 128, GBN = 128, GBK = 64;

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// SwiGLU of the prefill epilogues: silu(g) u with v_rcp_f32 (1 ulp) for the division -- the
// correctly rounded fp32 division's ~10-instruction sequence per element made the gate/up
// epilogue a visible share of the GEMM (128 elements per lane at one wave per SIMD)
__device__ __forceinline__ float silu_mul(float g, float u) {
  return g * __builtin_amdgcn_rcpf(1.0f + __expf(-g)) * u;
}

// ---- deferred-norm statistics of the consumers (epilogues 0, 2, 3).  One tile: the rows' sums
// of squares by LDS DMA straight into rinv_s; more (a residual epilogue's per-column-tile
// partials, [tiles][M]): staged, then folded in tile order into rinv_s before the epilogue.
// Issued ahead of the first K tile (no register: a register load here made the compiler drain
// vmcnt inside the K loop).
template <int BM, int NW>
__device__ __forceinline__ void gemm_rs_dma(const RowScale& rs, int M, int m0, float* rinv_s, float* stage) {
  if (!rs.ssq) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (rs.tiles == 1) {
    if (wave < BM / 64)
      __builtin_amdgcn_global_load_lds((const void*)(rs.ssq + min(m0 + wave * 64 + lane, M - 1)),
                                       (LDS_AS void*)(rinv_s + wave * 64), 4, 0, 0);
    return;
  }
  for (int p = wave; p < rs.tiles * (BM / 64); p += NW) {
    const int t = p / (BM / 64), r0 = (p % (BM / 64)) * 64;
    __builtin_amdgcn_global_load_lds((const void*)(rs.ssq + (size_t)t * M + min(m0 + r0 + lane, M - 1)),
                                     (LDS_AS void*)(stage + t * BM + r0), 4, 0, 0);
  }
}
// (every staged load issued before the first add; the adds in tile order)
template <int BM, int MAXT>
__device__ __forceinline__ void gemm_rs_fold(const RowScale& rs, float* rinv_s, const float* stage) {
  if (!rs.ssq || rs.tiles == 1) return;  // block-uniform
  __syncthreads();  // every wave is past its K loop (the DMA landed before the first tile)
  if ((int)threadIdx.x < BM) {
    float v[MAXT];
#pragma unroll
    for (int t = 0; t < MAXT; ++t) v[t] = t < rs.tiles ? stage[t * BM + threadIdx.x] : 0.f;
    float sum = v[0];
#pragma unroll
    for (int t = 1; t < MAXT; ++t)
      if (t < rs.tiles) sum += v[t];
    rinv_s[threadIdx.x] = sum;
  }
  __syncthreads();
}
// ---- the residual epilogue on the transposed accumulator (every GEMM tile): a lane holds
// x[row][c0 .. c0+3] as one f32x4 -- loaded as the accumulators' initial value, stored as one 16-B
// write, its f16(x*g*2^-4) as one 8-B write (the four fp32 products, then one rounding each, as
// gemm_resid_xg), and the four squares added into the lane's partial in column order
__device__ __forceinline__ void gemm_resid_x4(const GemmResid& gr, float* x, size_t o, f32x4 v, uint2 g, bool fuse,
                                              float& ss) {
  *(f32x4*)(x + o) = v;
  if (!fuse) return;
  const float gf[4] = {h_lo(g.x), h_hi(g.x), h_lo(g.y), h_hi(g.y)};  // the 4 gains, packed fp16
  float p[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p[j] = v[j] * gf[j] * kXgScale;
    asm volatile("" : "+v"(p[j]));
  }
  *(uint2*)(gr.xg + o) = uint2{pack2h(p[0], p[1]), pack2h(p[2], p[3])};
#pragma unroll
  for (int j = 0; j < 4; ++j) ss += v[j] * v[j];
}
// statistics of the transposed epilogue: per row and 128-column group, 8 lane partials -- the
// group's two 64-column halves h, in each the 4 lane groups fg (lane group fg of a half holds its
// columns 16n + 4fg .. +3, n = 0..3, summed in that order) -- added in (h, fg) order by one
// thread per (row, group).  red: [rows][groups][8] floats (the free tile buffers)
template <int BM, int GROUPS>
__device__ __forceinline__ void gemm_resid_ssq_t(float* red, int M, int N, int m0, int n0, const GemmResid& gr) {
  __syncthreads();
  for (int t = threadIdx.x; t < BM * GROUPS; t += blockDim.x) {
    const int row = t % BM, grp = t / BM;
    if (m0 + row >= M || n0 + grp * kGemmStatCols >= N) continue;
    const float* q = red + (row * GROUPS + grp) * 8;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += q[k];
    gr.ssq[(size_t)(n0 / kGemmStatCols + grp) * M + m0 + row] = sum;
  }
}
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const f16_t* __restrict__ A,
                                                     const f16_t* __restrict__ W,
                                                     void* __restrict__ out, int M, int N, int K,
                                                     int ldo, RowScale rs, GemmResid gr) {
  // 64 KiB of tiles + the tile rows' sums of squares (deferred-norm statistics: the folded sum,
  // then up to kGemmRsTiles staged partials).  ONE LDS object: with the DMA into a second array
  // the compiler drained vmcnt before every LDS read
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * GBM * GBK * 2 + GBM * 4 * (1 + kGemmRsTiles)];
  float* rinv_s = (float*)(smem + 2 * 2 * GBM * GBK * 2);
  float* rs_stage = rinv_s + GBM;
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
  const f16_t* a_src[4];
  const f16_t* b_src[4];
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
  // the transposed accumulator as gemm256_kernel's (the two tiles must give a prompt the same
  // bits: prefill packing invariance): C^T, 4 consecutive columns of one row per lane
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  // the rows' sums of squares by LDS DMA ahead of the first tile (no register: a register
  // load here made the compiler drain vmcnt inside the K loop); read at the epilogue
  gemm_rs_dma<GBM, 4>(rs, M, m0, rinv_s, rs_stage);
  // residual epilogue: x as the accumulators' initial value (as gemm256_kernel)
  uint2 g4[4] = {};  // the gains as packed fp16 bits, converted in the epilogue
  if constexpr (EPI == 1) {
    // transposed: acc[m][n] = x[row 16m + fr][cols 16n + 4fg .. +3], one 16-B load each
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = min(m0 + wm * 64 + m * 16 + fr, M - 1);
        const int col = min(n0 + wn * 64 + n * 16 + 4 * fg, N - 4);
        acc[m][n] = *(const f32x4*)((const float*)out + (size_t)row * ldo + col);
      }
    const f16_t* gp = gr.xg ? gr.gamma : (const f16_t*)A;  // unconditional load (no merge wait)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      g4[n] = *(const uint2*)(gp + min(n0 + wn * 64 + n * 16 + 4 * fg, N - 4));
    }
  }
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
      f16x8 af[4], bfr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row = wm * 64 + m * 16 + fr;
        const int ch = (4 * s + fg) ^ (row & 7);
        af[m] = *(const f16x8*)(As + row * 128 + ch * 16);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + fr;
        const int ch = (4 * s + fg) ^ (row & 7);
        bfr[n] = *(const f16x8*)(Bs + row * 128 + ch * 16);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = mfma16(bfr[n], af[m], acc[m][n]);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // epilogue: acc[m][n][j] = C[row 16m + fr][col 16n + 4fg + j] of the wave's 64x64
  if constexpr (EPI == 1) {  // residual add (x was the accumulators' initial value)
    const bool fuse = gr.xg != nullptr;
    float* red = (float*)smem;
    if (fuse) __syncthreads();  // every wave is past its K loop: the tile buffers are free
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = m0 + wm * 64 + m * 16 + fr;
      float ss = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = n0 + wn * 64 + n * 16 + 4 * fg;
        if (row < M && col < N) gemm_resid_x4(gr, (float*)out, (size_t)row * ldo + col, acc[m][n], g4[n], fuse, ss);
      }
      if (fuse) red[(wm * 64 + m * 16 + fr) * 8 + wn * 4 + fg] = ss;
    }
    if (fuse) gemm_resid_ssq_t<GBM, 1>(red, M, N, m0, n0, gr);
    return;
  }
  if constexpr (EPI == MS_GEMV_EPI_ARGMAX) {
    // greedy partials of the decode lm_head (MS_GEMV_EPI_ARGMAX's layout, finished by the decode
    // tail / ms_op_argmax_partials): {max, id} of each row over each 16-column tile, ties to the
    // lowest id, NaN never wins; no row scale (r > 0 keeps every row's order).  Lane (fr, fg)
    // holds columns 4fg .. 4fg+3 of the tile; the 4 lane groups merge by two xor swaps.
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = m0 + wm * 64 + m * 16 + fr;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int c0 = n0 + wn * 64 + n * 16;
        float v = -INFINITY;
        int idx = c0 + 4 * fg;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x = c0 + 4 * fg + j < N ? acc[m][n][j] : -INFINITY;
          if (!(x == x)) x = -INFINITY;
          if (x > v) { v = x; idx = c0 + 4 * fg + j; }
        }
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
          const float v2 = __shfl_xor(v, o, 64);
          const int i2 = __shfl_xor(idx, o, 64);
          if (v2 > v || (v2 == v && i2 < idx)) { v = v2; idx = i2; }
        }
        if (fg == 0 && row < M && c0 < N) ((float2*)out)[(size_t)row * ldo + (c0 >> 4)] = make_float2(v, __int_as_float(idx));
      }
    }
    return;
  }
  gemm_rs_fold<GBM, kGemmRsTiles>(rs, rinv_s, rs_stage);
  {
    // acc[m][n][j] = C[row 16m + fr][col 16n + 4fg + j] of the wave's 64x64
    float rv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) rv[m] = 1.f;
    if (rs.ssq) {
#pragma unroll
      for (int m = 0; m < 4; ++m) rv[m] = rs_rinv(rinv_s[wm * 64 + m * 16 + fr], rs);
    }
    const bool vec = (ldo & 3) == 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = m0 + wm * 64 + m * 16 + fr;
      if (row >= M) continue;
      if constexpr (EPI == 2) {
#pragma unroll
        for (int n = 0; n < 4; n += 2) {
          const int col = n0 + wn * 64 + n * 16;
          if (col >= N) continue;
          const int f = (col >> 5) * 16 + 4 * fg;
          float hv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) hv[j] = silu_mul(acc[m][n][j] * rv[m], acc[m][n + 1][j] * rv[m]);
          f16_t* o = (f16_t*)out + (size_t)row * ldo + f;
          if (vec) {
            *(uint2*)o = uint2{pack2h(hv[0], hv[1]), pack2h(hv[2], hv[3])};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = f2h(hv[j]);
          }
        }
      } else {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int col = n0 + wn * 64 + n * 16 + 4 * fg;
          if (col >= N) continue;
          const size_t o = (size_t)row * ldo + col;
          const f32x4 v = acc[m][n] * rv[m];
          if (vec && col + 3 < N) {
            if constexpr (EPI == 0) *(uint2*)((f16_t*)out + o) = uint2{pack2h(v[0], v[1]), pack2h(v[2], v[3])};
            else *(f32x4*)((float*)out + o) = v;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (col + j < N) {
                if constexpr (EPI == 0) ((f16_t*)out)[o + j] = f2h(v[j]);
                else ((float*)out)[o + j] = v[j];
              }
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ 256x256 8-phase tile
// The large-M prefill shapes (M = packed prompt tokens, thousands) run a 256x256x64 tile,
// 512 threads = 8 waves in 2 (M) x 4 (N), each wave a 128x64 output = 8x4 MFMA tiles
// (cdna_hip_programming.md §5 "The 256² 8-phase template"; our own schedule below).
// LDS: two K-tile buffers of 64 KiB (A image [256][128 B], B image [256][128 B]), filled
// by global_load_lds in 16-KiB "units" of 128 rows:
//   UAt = A rows {0..63, 128..191}   UAb = A rows {64..127, 192..255}
//   UBl = B rows {64w + 0..31}       UBr = B rows {64w + 32..63}   (w = 0..3)
// A K-tile is computed in 4 phases, one C quadrant each (wave-local 64x32):
//   phase 0: ds-read A top    + B left  -> MFMA (top, left)
//   phase 1: ds-read B right            -> MFMA (top, right)
//   phase 2: ds-read A bottom           -> MFMA (bottom, right)
//   phase 3: ds-read B left             -> MFMA (bottom, left)
// so UAt is last read in phase 0, UBr in 1, UAb in 2, UBl in 3.  A unit may be restaged
// two phases after its last read, and each phase issues exactly one unit:
//   phase 0: UAb(t+1)  phase 1: UBl(t+1)  phase 2: UAt(t+2)  phase 3: UBr(t+2)
// then phase 3 waits vmcnt(4): everything up to UBl(t+1) has landed while UAt/UBr(t+2)
// stay in flight across the barrier (never vmcnt(0) in the steady state).  Tile t+1 is
// first read in the next phase, after a barrier.  (A deeper form -- reads retired before each
// phase's first barrier, restaging one phase after the last read, vmcnt(6) with three units
// in flight -- measured neutral, 1284 vs 1280 TF/s at 8192^3: the loop is not latency-bound.
// On uniform random fp16 it runs 1286 TF/s at 8192^3 and 1706 on zero A (the clock under
// MFMA power), profiles/r04/v7_*.)  The two wave rows run one barrier apart
// (wave row 1 takes an extra s_barrier up front), so one row's MFMA cluster overlaps the
// other row's LDS reads and DMA issue.  LDS swizzle: row r holds global 16-B chunk
// c ^ ((r >> 1) & 7) at chunk c -- the 16 rows of a fragment read hit 16 distinct slots of
// the 256-B bank window (conflict-free); applied on the DMA source and on the read.
constexpr int TBM = 256, TBN = 256, TBK = 64;

__device__ __forceinline__ int swz2(int r) { return (r >> 1) & 7; }

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(const f16_t* __restrict__ A,
                                                        const f16_t* __restrict__ W,
                                                        void* __restrict__ out, int M, int N, int K,
                                                        int ldo, RowScale rs, GemmResid gr) {
  // two K-tile buffers + the tile rows' sums of squares (deferred-norm statistics: the folded
  // sum, then up to kGemmRsTiles staged partials).  ONE LDS object: with the DMA into a second
  // array the compiler drained vmcnt before every LDS read
  __shared__ __attribute__((aligned(16))) char smem[2 * 65536 + TBM * 4 * (1 + kGemmRsTiles)];
  float* rinv_s = (float*)(smem + 2 * 65536);
  float* rs_stage = rinv_s + TBM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = (M + TBM - 1) / TBM, tiles_n = (N + TBN - 1) / TBN;
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int grp = pid / (GM * tiles_n);
  const int first_m = grp * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_grp = pid % (GM * tiles_n);
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * TBM, n0 = tn * TBN;

  // DMA sources: unit u, instruction i -> local row lr = (2*wave + i)*8 + lane/8
  uint32_t src_off[4][2];
  int dst_row[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = (2 * wave + i) * 8 + (lane >> 3);
      int tr;
      if (u == 0) tr = lr < 64 ? lr : lr + 64;
      else if (u == 1) tr = lr < 64 ? lr + 64 : lr + 128;
      else tr = (lr >> 5) * 64 + (lr & 31) + (u == 3 ? 32 : 0);
      const int grow = u < 2 ? min(m0 + tr, M - 1) : min(n0 + tr, N - 1);
      src_off[u][i] = (uint32_t)grow * (uint32_t)K + (uint32_t)(((lane & 7) ^ swz2(tr)) * 8);
      dst_row[u][i] = tr - (lane >> 3);  // first row of the instruction's 8-row group
    }
  auto stage = [&](int buf, int u, int k0) {
    const f16_t* base = u < 2 ? A : W;
    char* img = smem + buf * 65536 + (u < 2 ? 0 : 32768);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(base + src_off[u][i] + k0),
                                       (LDS_AS void*)(img + dst_row[u][i] * 128), 16, 0, 0);
  };

  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fr >> 1;  // swz2(row) for every fragment row (rows = 16-aligned base + fr)
  // the MFMA computes C^T (W fragment as the A operand), so a lane holds 4 CONSECUTIVE columns
  // of one row -- the epilogues load / store 8 / 16 B per lane instead of one 2 / 4-B element
  // (every GEMM tile does the same: the prefill packing invariance needs one set of bits)
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 af[4][2], bfr[2][2];

  auto read_a = [&](int buf, int qa) {
    const char* img = smem + buf * 65536;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = wr * 128 + qa * 64 + m * 16 + fr;
        af[m][s2] = *(const f16x8*)(img + row * 128 + (((4 * s2 + fg) ^ sw) << 4));
      }
  };
  auto read_b = [&](int buf, int qb) {
    const char* img = smem + buf * 65536 + 32768;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = wc * 64 + qb * 32 + n * 16 + fr;
        bfr[n][s2] = *(const f16x8*)(img + row * 128 + (((4 * s2 + fg) ^ sw) << 4));
      }
  };
  auto mma = [&](int qa, int qb) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          acc[qa * 4 + m][qb * 2 + n] = mfma16(bfr[n][s2], af[m][s2], acc[qa * 4 + m][qb * 2 + n]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };

  const int nk = K / TBK;
  // the rows' sums of squares by LDS DMA ahead of the first tile (no register: a register
  // load here made the compiler drain vmcnt inside the K loop); read at the epilogue
  gemm_rs_dma<TBM, 8>(rs, M, m0, rinv_s, rs_stage);
  // residual epilogue: the tile's x is the accumulators' initial value, loaded ahead of the
  // first K tile (the prologue's vmcnt waits retire it with tile 0), so the MFMAs add A . W^T
  // onto x and the epilogue only stores -- no load round trips after the K loop
  uint2 g4[4] = {};  // the gains as packed fp16 bits: converted in the epilogue (a conversion here waited)
  if constexpr (EPI == 1) {
    // transposed: acc[mi][ni] = x[row 16mi + fr][cols 16ni + 4fg .. +3], one 16-B load each
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = min(m0 + wr * 128 + mi * 16 + fr, M - 1);
        const int col = min(n0 + wc * 64 + ni * 16 + 4 * fg, N - 4);
        acc[mi][ni] = *(const f32x4*)((const float*)out + (size_t)row * ldo + col);
      }
    // unconditional (a conditional load's merge made the wave wait for it right here)
    const f16_t* gp = gr.xg ? gr.gamma : (const f16_t*)A;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      g4[ni] = *(const uint2*)(gp + min(n0 + wc * 64 + ni * 16 + 4 * fg, N - 4));
    }
  }
  // prologue: tile 0 whole, then UAt/UBr of tile 1; tile 0 landed when <= 4 loads remain
  stage(0, 0, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  stage(0, 2, 0);
  // (compiler-visible waits: they also retire the residual epilogue's x loads, issued first,
  // so no extra vmcnt(0) is inserted ahead of the K loop for the accumulators)
  if (nk > 1) {
    stage(1, 0, TBK);
    stage(1, 3, TBK);
    __builtin_amdgcn_s_waitcnt((4 & 0xF) | (0x7 << 4) | (0xF << 8));  // vmcnt(4)
  } else {
    __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));  // vmcnt(0)
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the two wave rows by one barrier

  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1, nb = buf ^ 1;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    // phase 0
    read_b(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(buf, 0);
    if (has1) stage(nb, 1, (t + 1) * TBK);
    mma(0, 0);
    // phase 1
    read_b(buf, 1);
    if (has1) stage(nb, 2, (t + 1) * TBK);
    mma(0, 1);
    // phase 2
    read_a(buf, 1);
    if (has2) stage(buf, 0, (t + 2) * TBK);
    mma(1, 1);
    // phase 3
    read_b(buf, 0);
    if (has2) {
      stage(buf, 3, (t + 2) * TBK);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mma(1, 0);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger

  // epilogue: acc[mi][ni][j] = C[row 16mi + fr][col 16ni + 4fg + j] of the wave's 128x64
  if constexpr (EPI == 1) {
    // residual add (x was the accumulators' initial value): store x, and with gr.xg also the
    // next projection's input and its statistics
    const bool fuse = gr.xg != nullptr;
    float* red = (float*)smem;
    if (fuse) __syncthreads();  // every wave is past its K loop: the tile buffers are free
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int row = m0 + wr * 128 + mi * 16 + fr;
      float ss = 0.f;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + wc * 64 + ni * 16 + 4 * fg;
        if (row < M && col < N) gemm_resid_x4(gr, (float*)out, (size_t)row * ldo + col, acc[mi][ni], g4[ni], fuse, ss);
      }
      if (fuse) red[((wr * 128 + mi * 16 + fr) * 2 + (wc >> 1)) * 8 + (wc & 1) * 4 + fg] = ss;
    }
    if (fuse) gemm_resid_ssq_t<TBM, 2>(red, M, N, m0, n0, gr);
    return;
  }
  gemm_rs_fold<TBM, kGemmRsTiles>(rs, rinv_s, rs_stage);
  {
    // acc[mi][ni][j] = C[row 16mi + fr][col 16ni + 4fg + j] of the wave's 128x64: one row factor
    // per mi, the four columns of a (mi, ni) stored as one 8-B (fp16) / 16-B (fp32) write
    float rv[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) rv[mi] = 1.f;
    if (rs.ssq) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rv[mi] = rinv_s[wr * 128 + mi * 16 + fr];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rv[mi] = rs_rinv(rv[mi], rs);
    }
    const bool vec = (ldo & 3) == 0;  // block-uniform: 4-element groups stay aligned
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int row = m0 + wr * 128 + mi * 16 + fr;
      if (row >= M) continue;
      if constexpr (EPI == 2) {  // SwiGLU: ni even = gate, ni odd = up of the same 16 features
#pragma unroll
        for (int ni = 0; ni < 4; ni += 2) {
          const int col = n0 + wc * 64 + ni * 16;  // multiple of 32
          if (col >= N) continue;
          const int f = (col >> 5) * 16 + 4 * fg;
          float hv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) hv[j] = silu_mul(acc[mi][ni][j] * rv[mi], acc[mi][ni + 1][j] * rv[mi]);
          f16_t* o = (f16_t*)out + (size_t)row * ldo + f;
          if (vec) {
            *(uint2*)o = uint2{pack2h(hv[0], hv[1]), pack2h(hv[2], hv[3])};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = f2h(hv[j]);
          }
        }
      } else {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int col = n0 + wc * 64 + ni * 16 + 4 * fg;
          if (col >= N) continue;
          const size_t o = (size_t)row * ldo + col;
          const f32x4 v = acc[mi][ni] * rv[mi];
          if (vec && col + 3 < N) {
            if constexpr (EPI == 0) *(uint2*)((f16_t*)out + o) = uint2{pack2h(v[0], v[1]), pack2h(v[2], v[3])};
            else *(f32x4*)((float*)out + o) = v;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (col + j < N) {
                if constexpr (EPI == 0) ((f16_t*)out)[o + j] = f2h(v[j]);
                else ((float*)out)[o + j] = v[j];
              }
          }
        }
      }
    }
  }
}

// ---- 4-wave 256x256x64 variant (gemm variant 3; the default dispatch's kernel for the stored epilogues,
// variant 4): 256 threads in 2 x 2, each wave a 128 x 128
// output (8 x 8 MFMA tiles, the 256 accumulators pinned in AGPRs, one wave per SIMD) -- the library
// GEMM's geometry at this shape (hipBLASLt MT256x256x64_MI16x16 on 4 waves: 1455 vs 1215 TF/s on
// the gate/up shape, same box, profiles/r05/v8_*).  Per K-tile a wave reads 32 KB of fragments for
// 128 MFMAs (the 8-wave kernel: 24 KB for 64).  One barrier per K-tile, every LDS read and DMA
// instruction slotted between MFMAs (one per two, the library kernel's interleave): the MFMAs of
// k-step 0 carry the fragment reads of k-step 1; then vmcnt(0) + barrier (tile t+1 has landed
// everywhere, tile t is no longer read); the MFMAs of k-step 1 carry tile t+2's DMA into tile t's
// buffer and tile t+1's k-step-0 reads.  Same LDS image and swizzle as gemm256_kernel, same k order
// per output element (x as the initial accumulator of the residual epilogue, 32-k MFMAs in k
// order), same statistics order: every result is bit-identical to gemm256_kernel's
// (test_gemm_4wave_bit_exact).  Measured (profiles/r05/v9_*, v10_*): 1002-1415 TF/s against the
// 8-wave kernel's 1016-1327 -- ahead on square shapes, level on the prefill ones; a 4-slot ring of
// 32-k steps (three steps of DMA lookahead, 64-B row segments) was slower (1029-1259).  Not the
// default: the library kernel's remaining 15-25 % is not in this schedule.
template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(const f16_t* __restrict__ A,
                                                       const f16_t* __restrict__ W,
                                                       void* __restrict__ out, int M, int N, int K,
                                                       int ldo, RowScale rs, GemmResid gr) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 65536 + TBM * 4 * (1 + kGemmRsTiles)];
  float* rinv_s = (float*)(smem + 2 * 65536);
  float* rs_stage = rinv_s + TBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + TBM - 1) / TBM, tiles_n = (N + TBN - 1) / TBN;
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int grp = pid / (GM * tiles_n);
  const int first_m = grp * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_grp = pid % (GM * tiles_n);
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * TBM, n0 = tn * TBN;

  // DMA: each operand tile is 256 rows x 128 B = 32 instructions of 8 rows; wave w issues row
  // groups 8w .. 8w + 7 of A and of B.  Lane l of a group lands at row 8g + l / 8, LDS chunk l % 8,
  // so it loads the global chunk (l % 8) ^ swz2(row) (gemm256_kernel's image)
  uint32_t src_a[8], src_b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = (8 * wave + i) * 8 + (lane >> 3);
    const int ch = ((lane & 7) ^ swz2(r)) * 8;
    src_a[i] = (uint32_t)min(m0 + r, M - 1) * (uint32_t)K + (uint32_t)ch;
    src_b[i] = (uint32_t)min(n0 + r, N - 1) * (uint32_t)K + (uint32_t)ch;
  }
  // one 1-KiB DMA instruction (i < 8: A row group 8 wave + i, else B), issued where the compiler
  // cannot see it: with the builtin it waited vmcnt(0) before LDS reads it could not prove disjoint
  // from the DMA's bytes.  The loop orders the DMA itself (vmcnt + barrier before a buffer is read).
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS char*)smem);
  auto dma1 = [&](int buf, int k0, int i) {
    const f16_t* src = i < 8 ? A + src_a[i] + k0 : W + src_b[i - 8] + k0;
    const uint32_t dst = lds0 + buf * 65536 + (i < 8 ? 0 : 32768) + (8 * wave + (i & 7)) * 8 * 128;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"{m0}"(dst), "v"(src) : "memory");
  };

  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fr >> 1;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 af[2][8], bf[2][8];  // [k-step parity][tile]
  // fragment g of a k-step (g < 8: A tile g, else B tile g - 8) into register set p
  auto rd1 = [&](int buf, int s, int p, int g) {
    const char* img = smem + buf * 65536;
    if (g < 8) af[p][g] = *(const f16x8*)(img + (wr * 128 + g * 16 + fr) * 128 + (((4 * s + fg) ^ sw) << 4));
    else bf[p][g - 8] = *(const f16x8*)(img + 32768 + (wc * 128 + (g - 8) * 16 + fr) * 128 + (((4 * s + fg) ^ sw) << 4));
  };
  // MFMA i (m-major) of register set p, the accumulator pinned in place (AGPRs, "+a"): with the
  // builtin, hipcc rotated one 4-register tile through a spare AGPR slot every MFMA (184
  // v_accvgpr_mov per K-tile); dependent MFMAs on one accumulator are interlocked, the reads after
  // the loop wait below
  // the transposed accumulator (gemm256_kernel's): C^T, 4 consecutive columns of one row per lane
  auto mf1 = [&](int p, int i) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[i >> 3][i & 7]) : "v"(bf[p][i & 7]), "v"(af[p][i >> 3]));
  };

  const int nk = K / TBK;
  gemm_rs_dma<TBM, 4>(rs, M, m0, rinv_s, rs_stage);
  uint2 g8[8] = {};
  if constexpr (EPI == 1) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) {
        const int row = min(m0 + wr * 128 + mi * 16 + fr, M - 1);
        const int col = min(n0 + wc * 128 + ni * 16 + 4 * fg, N - 4);
        acc[mi][ni] = *(const f32x4*)((const float*)out + (size_t)row * ldo + col);
      }
    const f16_t* gp = gr.xg ? gr.gamma : (const f16_t*)A;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      g8[ni] = *(const uint2*)(gp + min(n0 + wc * 128 + ni * 16 + 4 * fg, N - 4));
    }
  }
  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere, its k-step-0 fragments read
  // (the x preload of the residual epilogue and the statistics DMA are compiler-visible: retired
  // here, long before the first MFMA)
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma1(0, 0, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma1(1, min(1, nk - 1) * TBK, i);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 16; ++g) rd1(0, 0, 0, g);
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): k-step 0's fragments (a builtin: the compiler sees it)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mf1(0, 4 * g);
      mf1(0, 4 * g + 1);
      rd1(cur, 1, 1, g);
      mf1(0, 4 * g + 2);
      mf1(0, 4 * g + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): k-step 1's fragments
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // tile t+1 landed (this wave's DMA)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // ... for every wave: tile t's buffer is free, tile t+1 is in LDS
    __builtin_amdgcn_s_setprio(1);
    // (unconditional: past the last tile the DMA re-loads tile nk-1 into the free buffer and the
    // reads fill the unused register set -- no branches inside the interleave)
    const int k2 = min(t + 2, nk - 1) * TBK;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mf1(1, 4 * g);
      dma1(cur, k2, g);
      mf1(1, 4 * g + 1);
      rd1(cur ^ 1, 0, 0, g);
      mf1(1, 4 * g + 2);
      mf1(1, 4 * g + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  // the last MFMAs' results before any other instruction reads the accumulators (the asm MFMAs
  // are invisible to the compiler's hazard recognizer)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  // epilogue: acc[mi][ni][j] = C[row 16mi + fr][col 16ni + 4fg + j] of the wave's 128x128
  if constexpr (EPI == 1) {
    const bool fuse = gr.xg != nullptr;
    float* red = (float*)smem;
    if (fuse) __syncthreads();  // every wave is past its K loop: the tile buffers hold the statistics
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int row = m0 + wr * 128 + mi * 16 + fr;
      float ss[2] = {0.f, 0.f};  // two 64-column halves (gemm256_kernel's wave columns 2wc, 2wc+1)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) {
        const int col = n0 + wc * 128 + ni * 16 + 4 * fg;
        if (row < M && col < N)
          gemm_resid_x4(gr, (float*)out, (size_t)row * ldo + col, acc[mi][ni], g8[ni], fuse, ss[ni >> 2]);
      }
      if (fuse)
#pragma unroll
        for (int h = 0; h < 2; ++h) red[((wr * 128 + mi * 16 + fr) * 2 + wc) * 8 + h * 4 + fg] = ss[h];
    }
    if (fuse) gemm_resid_ssq_t<TBM, 2>(red, M, N, m0, n0, gr);
    return;
  }
  gemm_rs_fold<TBM, kGemmRsTiles>(rs, rinv_s, rs_stage);
  {
    // acc[mi][ni][j] = C[row 16mi + fr][col 16ni + 4fg + j] of the wave's 128x128
    float rv[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) rv[mi] = 1.f;
    if (rs.ssq) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rv[mi] = rs_rinv(rinv_s[wr * 128 + mi * 16 + fr], rs);
    }
    const bool vec = (ldo & 3) == 0;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int row = m0 + wr * 128 + mi * 16 + fr;
      if (row >= M) continue;
      if constexpr (EPI == 2) {
#pragma unroll
        for (int ni = 0; ni < 8; ni += 2) {
          const int col = n0 + wc * 128 + ni * 16;
          if (col >= N) continue;
          const int f = (col >> 5) * 16 + 4 * fg;
          float hv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) hv[j] = silu_mul(acc[mi][ni][j] * rv[mi], acc[mi][ni + 1][j] * rv[mi]);
          f16_t* o = (f16_t*)out + (size_t)row * ldo + f;
          if (vec) {
            *(uint2*)o = uint2{pack2h(hv[0], hv[1]), pack2h(hv[2], hv[3])};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = f2h(hv[j]);
          }
        }
      } else {
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
          const int col = n0 + wc * 128 + ni * 16 + 4 * fg;
          if (col >= N) continue;
          const size_t o = (size_t)row * ldo + col;
          const f32x4 v = acc[mi][ni] * rv[mi];
          if (vec && col + 3 < N) {
            if constexpr (EPI == 0) *(uint2*)((f16_t*)out + o) = uint2{pack2h(v[0], v[1]), pack2h(v[2], v[3])};
            else *(f32x4*)((float*)out + o) = v;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (col + j < N) {
                if constexpr (EPI == 0) ((f16_t*)out)[o + j] = f2h(v[j]);
                else ((float*)out)[o + j] = v[j];
              }
          }
        }
      }
    }
  }
}

// 0: heuristic (8-wave big tile), 1: 128x128, 2: 256x256 8-wave, 3: 256x256 4-wave, 4 (default):
// the heuristic with the 4-wave kernel for the stored epilogues and the 8-wave one for the residual
// epilogue (the 4-wave residual form spills) -- QKV 437 -> 422 us, gate/up 1327 -> 1321 us per
// launch, prefill 87.0 -> 86.2 ms per configs[1] step (profiles/r05/v11_ab3_*, v11_prof_*).  Tests and sweeps set
// it (ms_set_gemm_variant, MS_GEMM_VARIANT); every variant gives the same bits
static int g_gemm_variant = [] { const char* e = getenv("MS_GEMM_VARIANT"); return e ? atoi(e) : 4; }();

void set_gemm_variant(int v) { g_gemm_variant = v; }

static bool gemm_big(int M, int N) {
  return g_gemm_variant == 2 || g_gemm_variant == 3 ||
         ((g_gemm_variant == 0 || g_gemm_variant == 4) && M >= 1024 && N >= 1024);
}
// the 4-wave tile for this launch: variant 3 always, 4 for the stored epilogues (the residual
// O at K = 3072 on it measured 333 vs 321 us in the engine, r05/v18_*)
static bool gemm_4wave(int epi) { return g_gemm_variant == 3 || (g_gemm_variant == 4 && epi != 1); }

int gemm_resid_tiles(int M, int N) {
  (void)M;
  return (N + kGemmStatCols - 1) / kGemmStatCols;
}

void launch_gemm(const f16_t* A, const f16_t* W, void* out, int M, int N, int K, int ldo, int epi,
                 hipStream_t s, const RowScale* rs_in, const GemmResid* gr_in) {
  if (M <= 0) return;
  if (epi == MS_GEMV_EPI_ARGMAX) {  // the decode lm_head's greedy partials: the 128x128 tile only, no row scale
    const int grid = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
    MS_LAUNCH(gemm_kernel<MS_GEMV_EPI_ARGMAX>, dim3(grid), dim3(256), 0, s, A, W, out, M, N, K, ldo, RowScale{},
              GemmResid{});
    return;
  }
  const bool big = gemm_big(M, N);
  RowScale rs{};
  if (rs_in && rs_in->ssq && epi != 1) {
    if (rs_in->tiles < 1 || rs_in->tiles > kGemmRsTiles) return;  // callers check
    rs = *rs_in;
  }
  GemmResid gr{};
  if (gr_in && epi == 1) gr = *gr_in;
#define GL(KERN, EPI_, BLK) MS_LAUNCH(KERN<EPI_>, dim3(grid), dim3(BLK), 0, s, A, W, out, M, N, K, ldo, rs, gr)
  if (big && gemm_4wave(epi) && K % TBK == 0) {
    const int grid = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
    switch (epi) {
      case 0: GL(gemm4w_kernel, 0, 256); break;
      case 1: GL(gemm4w_kernel, 1, 256); break;
      case 2: GL(gemm4w_kernel, 2, 256); break;
      default: GL(gemm4w_kernel, 3, 256); break;
    }
    return;
  }
  if (big) {
    const int grid = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
    switch (epi) {
      case 0: GL(gemm256_kernel, 0, 512); break;
      case 1: GL(gemm256_kernel, 1, 512); break;
      case 2: GL(gemm256_kernel, 2, 512); break;
      default: GL(gemm256_kernel, 3, 512); break;
    }
    return;
  }
  const int grid = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  switch (epi) {
    case 0: GL(gemm_kernel, 0, 256); break;
    case 1: GL(gemm_kernel, 1, 256); break;
    case 2: GL(gemm_kernel, 2, 256); break;
    default: GL(gemm_kernel, 3, 256); break;
  }
#undef GL
}

bool gemm_rs_tiles_ok(int M, int N, int tiles) {
  (void)M;
  (void)N;
  return tiles >= 1 && tiles <= kGemmRsTiles;
}

}  // namespace ms
