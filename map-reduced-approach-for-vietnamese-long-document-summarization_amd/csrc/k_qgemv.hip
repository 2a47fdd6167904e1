// k_qgemv.hip -- ggml K-quant weights on gfx950: bit-exact dequantisation and the
// dequant-fused decode GEMV (BASELINE.json config 5).
//
// Ollama's default llama3.2:3b is Q4_K_M: Q4_K (144 B / 256 weights) for most matrices,
// Q6_K (210 B / 256 weights) for some (EXT: llama.cpp).  The dequantisers restate
// llama.cpp's dequantize_row_q4_K / _q6_K (oracle/ggml_quants.c) with the non-contracted
// float forms  y = d1*q - m1  and  y = (d*sc)*q  (__fmul_rn/__fsub_rn), so the fp32 result
// is bit-identical to the C restatement.
//
// Storage (engine.cpp): every quantised matrix keeps both
//   * a fp16 copy = f16(dequant(blocks)) in the fused row layout, for prefill GEMMs
//     and the embedding gather (compute-bound; fp16 is what MFMA consumes), and
//   * the quantised rows for decode, which is HBM-bound: 4.5 / 6.56 bits per weight
//     instead of 16.  Q4_K blocks keep their 16-B ggml header (d, dmin, 12 scale bytes) and
//     144 B, but the 128 quant bytes are re-ordered so that lane group g of a wave reads one
//     dword per sub-block s holding weights 32s+8g .. +7 (byte i = q[k_i] | q[k_{i+4}] << 4),
//     sub-blocks 0-3 of the 4 groups in 64 contiguous bytes, then 4-7; Q6_K blocks are repacked to 224 B [ql 128 | qh 64 | scales
//     16 | d 2 + pad] so every field is 16-B aligned, the ql bytes regrouped so that a wave
//     load reads 64 contiguous bytes per row (quant_rows_kernel).
// The fused GEMV streams the blocks HBM -> VGPR (one super-block of 256 weights per row
// per wave-step) and feeds v_mfma_f32_16x16x32_f16:
//   * Q4_K, one MFMA per 32-weight sub-block: the nibbles become the fp16 subnormals q 2^-24
//     by a byte permute (exact; gfx950 MFMA keeps fp16 denormal operands), the MFMA gives
//     A_s = 2^-24 sum_k x_k q_k, and sum_k x_k y_k = (2^24 d_s) A_s - m_s X_s with d_s = d*sc_s,
//     m_s = dmin*m_s (ggml's
//     fp32 d1 / m1) and X_s = sum of the sub-block's x (one more MFMA, against ones, shared
//     by the weight tiles of the block) -- 2 FMAs per output
//     element per sub-block instead of dequantising every weight: the decode GEMV uses the
//     exact fp32 dequantised weights (no fp16 rounding of them, and no cancellation: a
//     1024 + q bias form cost ~7e-6 relative against fp64);
//   * Q6_K, dequantised in registers to the fp16 values of the fp16 copy.
#include <algorithm>
#include <cstdlib>

#include "gemv_common.h"

namespace ms {

__device__ __forceinline__ float h2f_lo(uint32_t h16) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(h16 & 0xFFFFu));
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int i) {  // i compile-time or not
  const uint32_t w = (i < 4) ? v.x : (i < 8) ? v.y : (i < 12) ? v.z : v.w;
  return (w >> (8 * (i & 3))) & 0xFFu;
}

// get_scale_min_k4 on the 12 scale bytes = header bytes 4..15 (v.y, v.z, v.w)
__device__ __forceinline__ void scale_min_k4(const uint4& hdr, int j, int& d, int& m) {
  auto q = [&](int i) { return (int)byte_of(hdr, 4 + i); };
  if (j < 4) {
    d = q(j) & 63;
    m = q(j + 4) & 63;
  } else {
    d = (q(j + 4) & 0xF) | ((q(j - 4) >> 6) << 4);
    m = (q(j + 4) >> 4) | ((q(j) >> 6) << 4);
  }
}

// ---------------------------------------------------------------- dequantisers
// one 256-thread block per super-block, thread t -> weight t (the C loop order)
__device__ __forceinline__ float deq_q4k_one(const uint8_t* b, int t) {
  const uint4 hdr = *(const uint4*)b;
  const float d = h2f_lo(hdr.x), dmin = h2f_lo(hdr.x >> 16);
  const int c = t >> 6, w = t & 63, h = w >> 5, l = w & 31;
  int sc, m;
  scale_min_k4(hdr, 2 * c + h, sc, m);
  const uint32_t qb = b[16 + c * 32 + l];
  const uint32_t q = h ? (qb >> 4) : (qb & 0xF);
  const float d1 = __fmul_rn(d, (float)sc), m1 = __fmul_rn(dmin, (float)m);
  return __fsub_rn(__fmul_rn(d1, (float)q), m1);
}

// raw ggml Q6_K block: ql[128] qh[64] scales[16] d
__device__ __forceinline__ float deq_q6k_one(const uint8_t* b, int t) {
  const int n = t >> 7, r = t & 127, k4 = r >> 5, l = r & 31;
  const uint32_t a = b[n * 64 + l + ((k4 & 1) ? 32 : 0)];
  const uint32_t hb = b[128 + n * 32 + l];
  const int q = (int)(((k4 >> 1) ? (a >> 4) : (a & 0xF)) | (((hb >> (2 * k4)) & 3) << 4)) - 32;
  const int sc = (int)(int8_t)b[192 + n * 8 + (l >> 4) + 2 * k4];
  const float d = h2f_lo((uint32_t)b[208] | ((uint32_t)b[209] << 8));
  return __fmul_rn(__fmul_rn(d, (float)sc), (float)q);
}

__global__ __launch_bounds__(256) void dequant_f32_kernel(int type, const uint8_t* __restrict__ blocks,
                                                          float* __restrict__ out) {
  const size_t sb = blockIdx.x;
  const int t = threadIdx.x;
  const float y = (type == MS_QT_Q4_K) ? deq_q4k_one(blocks + sb * kQ4KBytes, t)
                                       : deq_q6k_one(blocks + sb * kQ6KBytes, t);
  out[sb * 256 + t] = y;
}

void launch_dequant_f32(int type, const uint8_t* blocks, int64_t n_blocks, float* out, hipStream_t s) {
  if (n_blocks <= 0) return;
  MS_LAUNCH(dequant_f32_kernel, dim3((unsigned)n_blocks), dim3(256), 0, s, type, blocks, out);
}

// rows of raw blocks -> (a) fp16 rows of the fused matrix, (b) packed quantised rows
__global__ __launch_bounds__(256) void quant_rows_kernel(int type, const uint8_t* __restrict__ blocks,
                                                         int K, f16_t* __restrict__ dst_f16,
                                                         int map_mul, int map_add,
                                                         uint8_t* __restrict__ dst_q, int q_row_base) {
  const int r = blockIdx.y, sb = blockIdx.x, t = threadIdx.x;
  const int nsb = K / 256;
  const int braw = (type == MS_QT_Q4_K) ? kQ4KBytes : kQ6KBytes;
  const uint8_t* b = blocks + ((size_t)r * nsb + sb) * braw;
  const float y = (type == MS_QT_Q4_K) ? deq_q4k_one(b, t) : deq_q6k_one(b, t);
  const size_t drow = map_row(r, map_mul, map_add);
  dst_f16[drow * K + (size_t)sb * 256 + t] = f2h(y);
  if (dst_q) {
    const int bp = (type == MS_QT_Q4_K) ? kQ4KBytes : kQ6KPacked;
    uint8_t* q = dst_q + ((drow - q_row_base) * nsb + sb) * bp;
    if (type == MS_QT_Q4_K) {
      // header as is; quant byte 16 + 64(s >> 2) + 16g + 4(s & 3) + i = q[k] | q[k + 4] << 4,
      // k = 32s + 8g + i: lane group g's sub-blocks 0-3 at 16 + 16g, 4-7 at 80 + 16g, so one wave
      // load instruction reads 64 contiguous bytes of each row
      if (t < 16) q[t] = b[t];
      if (t < 128) {
        const int g = t >> 5, s_ = (t >> 2) & 7, i = t & 3;
        auto nib = [&](int k) {
          const uint32_t qb = b[16 + (k >> 6) * 32 + (k & 31)];
          return ((k & 63) >> 5) ? (qb >> 4) : (qb & 0xF);
        };
        const int k = 32 * s_ + 8 * g + i;
        q[16 + 64 * (s_ >> 2) + 16 * g + 4 * (s_ & 3) + i] = (uint8_t)(nib(k) | (nib(k + 4) << 4));
      }
    } else {
      // Q6_K: same fields (qh at 128, scales at 192, d at 208, tail padded), ql regrouped by the
      // GEMV's lane group g = 2 hh + p: its low-half 16 bytes (raw hh*64 + 16p ..) at 16g and its
      // high-half 16 bytes (raw hh*64 + 32 + 16p ..) at 64 + 16g -- one wave load instruction
      // then reads 64 contiguous bytes of each row (one 64-B line) instead of two half lines
      // (qh is already in that order: raw 128 + hh*32 + 16p = 128 + 16g)
      if (t < 128) {
        const int hh = t >> 6, half = (t >> 5) & 1, p = (t >> 4) & 1, i = t & 15;
        q[half * 64 + 16 * (2 * hh + p) + i] = b[t];
      } else if (t < braw) {
        q[t] = b[t];
      }
      if (t >= braw && t < kQ6KPacked) q[t] = 0;
    }
  }
}

void launch_quant_rows(int type, const uint8_t* blocks, int rows, int K, f16_t* dst_f16, int map_mul,
                       int map_add, uint8_t* dst_q, int q_row_base, hipStream_t s) {
  if (rows <= 0) return;
  MS_LAUNCH(quant_rows_kernel, dim3(K / 256, rows), dim3(256), 0, s, type, blocks, K, dst_f16,
            map_mul, map_add, dst_q, q_row_base);
}

// seeded random blocks (bench / config 5 synthetic weights): every byte from a counter
// hash, then the fp16 scale fields set so dequantised weights have std ~ `scale`
__device__ __forceinline__ uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void synth_qblocks_kernel(int type, uint8_t* __restrict__ blocks, int64_t n_blocks,
                                     uint64_t seed_h, float scale) {
  const int braw = (type == MS_QT_Q4_K) ? kQ4KBytes : kQ6KBytes;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_blocks;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t* b = blocks + i * braw;
    uint64_t h = smix((uint64_t)i ^ seed_h);
    for (int k = 0; k < braw; k += 8) {
      h = smix(h);
      for (int q = 0; q < 8 && k + q < braw; ++q) b[k + q] = (uint8_t)(h >> (8 * q));
    }
    const float u = 0.5f + (float)(smix(h) >> 40) * (1.0f / 16777216.0f);
    if (type == MS_QT_Q4_K) {
      const _Float16 d = (_Float16)(u * scale / 270.f);
      const _Float16 dm = (_Float16)((float)d * 7.5f);
      const uint16_t db = __builtin_bit_cast(uint16_t, d), dmb = __builtin_bit_cast(uint16_t, dm);
      b[0] = db & 0xFF; b[1] = db >> 8; b[2] = dmb & 0xFF; b[3] = dmb >> 8;
    } else {
      for (int k = 0; k < 16; ++k) b[192 + k] = (uint8_t)((int)(b[192 + k] & 0x7F) - 64);
      const _Float16 d = (_Float16)(u * scale / 680.f);
      const uint16_t db = __builtin_bit_cast(uint16_t, d);
      b[208] = db & 0xFF; b[209] = db >> 8;
    }
  }
}

void launch_synth_qblocks(int type, uint8_t* blocks, int64_t n_blocks, uint64_t seed, float scale,
                          hipStream_t s) {
  MS_LAUNCH(synth_qblocks_kernel, dim3(2048), dim3(256), 0, s, type, blocks, n_blocks,
            (uint64_t)smix_host(seed), scale);
}

// ---------------------------------------------------------------- dequant-fused GEMV
// One block per 16*NT rows, waves split the K/256 super-blocks (SBW per wave).  Lane
// group g = lane>>4 owns 64 weights of each super-block:
//   Q4_K: chunk g (qs bytes 32g..32g+31): low nibbles = weights 64g..64g+31 (sub-block
//         2g), high nibbles = 64g+32.. (sub-block 2g+1);
//   Q6_K: half h = g>>1, positions l in [16p, 16p+16), p = g&1, each giving the four
//         weights h*128 + {0,32,64,96} + l.
// MFMA t of a super-block takes 8 of those weights per lane and the X elements of the
// same k -- a k permutation applied to both operands, so every dot product is unchanged.
// XM: the X source (gemv_common.h kXGlobal / kXLds / kXRegs, as in k_gemv.hip)
template <int MT, int NT, int EPI, int SBW, int XM, bool RS>
__global__ __launch_bounds__(1024) void qgemv_kernel(const f16_t* __restrict__ X, QMat qm,
                                                     void* __restrict__ out, int M, int N, int K,
                                                     int ldo, int rinv_off, GemvArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float rsd = 0.f;  // the rows' deferred-norm statistics, ahead of every load
  if constexpr (RS) rsd = rs_begin<true>(smem, rinv_off, ga.rs, M);
  // split-K (fp32 slab epilogue only): block row y owns super-blocks [y*K/256, (y+1)*K/256)
  // of the full row, where K is the per-split length; X and out shift to that slab.
  const int ldx = K * gridDim.y, sbk = blockIdx.y * (K / 256);
  if constexpr (EPI == MS_GEMV_EPI_STORE_F32) {
    X += (size_t)blockIdx.y * K;
    out = (float*)out + (size_t)blockIdx.y * (ga.slab_rows > 0 ? ga.slab_rows : M) * ldo;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  // RESID_SSQ: ga.rt weight rows per tile (lanes fr >= rt load the last row again, never stored)
  constexpr bool RESID = EPI == MS_GEMV_EPI_RESID_SSQ;
  const int rt = RESID && ga.rt > 0 ? ga.rt : 16;
  const int n0 = RESID ? blockIdx.x * rt : blockIdx.x * 16 * NT;
  const int frw = RESID ? min(fr, rt - 1) : fr;  // this lane's weight row in the tile
  const ResidPre pre = resid_prefetch<EPI>(M, N, ldo, out, n0, ga);
  // the region holding this tile (regions are 16-row aligned; block-uniform)
  int type = qm.type0, row_bytes = qm.row_bytes0, rbase = n0 - qm.row0_0;
  const uint8_t* base = qm.base0;
  if (qm.n > 1 && n0 >= qm.row0_1) { type = qm.type1; row_bytes = qm.row_bytes1; rbase = n0 - qm.row0_1; base = qm.base1; }
  if (qm.n > 2 && n0 >= qm.row0_2) { type = qm.type2; row_bytes = qm.row_bytes2; rbase = n0 - qm.row0_2; base = qm.base2; }
  const int sb0 = wave * SBW;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool XL = XM == kXLds, XR = XM == kXRegs;
  // X first (LDS DMA of the block's rows, or this wave's super-blocks into registers), then
  // the weight stream: vmcnt retires in issue order
  if constexpr (XL) gemv_dma_x(smem, X, M, K, ldx);
  // Q4_K sub-block s of super-block j: lane group g's 8 weights at k = (j*8 + s)*32 + 8g;
  // Q6_K MFMA t: k = j*256 + hh*128 + (t>>1)*32 + 16p + 8(t&1)
  f16x8 xr[XR ? SBW : 1][XR ? 8 : 1][XR ? MT : 1];
  if constexpr (XR) {
    const bool q6 = type != MS_QT_Q4_K;
#pragma unroll
    for (int j = 0; j < SBW; ++j)
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int k = q6 ? (sb0 + j) * 256 + (g >> 1) * 128 + (t >> 1) * 32 + 16 * (g & 1) + 8 * (t & 1)
                           : ((sb0 + j) * 8 + t) * 32 + 8 * g;
          xr[j][t][m] = as_f16x8(ldg16(X + (size_t)min(m * 16 + fr, M - 1) * ldx + k));
        }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (type == MS_QT_Q4_K) {
    uint4 hq[SBW][NT], q0[SBW][NT], q1[SBW][NT];
#pragma unroll
    for (int j = 0; j < SBW; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const uint8_t* bp = base + (size_t)(rbase + n * 16 + frw) * row_bytes + (size_t)(sbk + sb0 + j) * kQ4KBytes;
        hq[j][n] = ldw16(bp);
        q0[j][n] = ldw16(bp + 16 + 16 * g);  // sub-blocks 0-3 (quant_rows_kernel's layout)
        q1[j][n] = ldw16(bp + 80 + 16 * g);  // sub-blocks 4-7
      }
    if constexpr (XL) {  // the X image has landed once at most the weight loads are pending
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * SBW * NT));
      __builtin_amdgcn_s_barrier();  // no fence: a fence would wait for the weight loads too
    }
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const f16x8 ones = __builtin_bit_cast(f16x8, u4v{0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u});
#pragma unroll
    for (int j = 0; j < SBW; ++j)
#pragma unroll
      for (int s_ = 0; s_ < 8; ++s_) {
        const int k = ((sb0 + j) * 8 + s_) * 32 + 8 * g;  // this lane group's 8 weights
        const int sh = 8 * (s_ & 3);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int xrow = min(m * 16 + fr, M - 1);
          const f16x8 xf = XR ? xr[XR ? j : 0][XR ? s_ : 0][XR ? m : 0]
                          : XL ? *(const f16x8*)(smem + x_lds(xrow, k, K))
                               : *(const f16x8*)(X + (size_t)xrow * ldx + k);
          // X_s = the sub-block's sum of each row's x: one more MFMA against ones, shared by
          // the NT weight tiles (no separate pass over X, no barrier)
          const f32x4 xs = mfma16(xf, ones, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            // get_scale_min_k4 of sub-block s_ from the 12 scale bytes (header words y, z, w)
            const uint4 h = hq[j][n];
            const uint32_t scw = s_ < 4 ? (h.y & 0x3F3F3F3Fu) : ((h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u));
            const uint32_t mw = s_ < 4 ? (h.z & 0x3F3F3F3Fu) : (((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u));
            const float d1 = __fmul_rn(h2f_lo(h.x), (float)((scw >> sh) & 0xFFu));        // ggml d1 = d * sc
            const float m1 = __fmul_rn(h2f_lo(h.x >> 16), (float)((mw >> sh) & 0xFFu));   // ggml m1 = dmin * m
            const float d1s = d1 * 16777216.0f;                                  // d1 * 2^24 (exact)
            const uint4 qq = s_ < 4 ? q0[j][n] : q1[j][n];
            const int si = s_ & 3;
            const uint32_t qw = si == 0 ? qq.x : si == 1 ? qq.y : si == 2 ? qq.z : qq.w;
            const uint32_t lo = qw & 0x0F0F0F0Fu, hi = (qw >> 4) & 0x0F0F0F0Fu;
            // bytes [q, 0, q', 0] = the fp16 subnormals q * 2^-24, q' * 2^-24 (exact): weights
            // k .. k+7 in order (perm selector 0x0C is the constant byte 0)
            const u4v pk = {__builtin_amdgcn_perm(0u, lo, 0x0C010C00u), __builtin_amdgcn_perm(0u, lo, 0x0C030C02u),
                            __builtin_amdgcn_perm(0u, hi, 0x0C010C00u), __builtin_amdgcn_perm(0u, hi, 0x0C030C02u)};
            const f32x4 A = mfma16(xf, __builtin_bit_cast(f16x8, pk), f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[m][n][i] = __fmaf_rn(-m1, xs[i], __fmaf_rn(d1s, A[i], acc[m][n][i]));
          }
        }
      }
  } else {  // Q6_K, packed 224-B blocks
    const int hh = g >> 1, p = g & 1;
    uint4 qa[SBW][NT], qb[SBW][NT], qh[SBW][NT], sc[SBW][NT];
    uint32_t dw[SBW][NT];
#pragma unroll
    for (int j = 0; j < SBW; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const uint8_t* bp = base + (size_t)(rbase + n * 16 + frw) * row_bytes + (size_t)(sbk + sb0 + j) * kQ6KPacked;
        qa[j][n] = ldw16(bp + 16 * g);  // raw ql hh*64 + 16p .. (quant_rows_kernel's regrouping)
        qb[j][n] = ldw16(bp + 64 + 16 * g);  // raw ql hh*64 + 32 + 16p ..
        qh[j][n] = ldw16(bp + 128 + hh * 32 + 16 * p);
        sc[j][n] = ldw16(bp + 192);
        dw[j][n] = *(const uint32_t*)(bp + 208);
      }
    if constexpr (XL) {  // the X image has landed once at most the weight loads are pending
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(5 * SBW * NT));
      __builtin_amdgcn_s_barrier();  // no fence: a fence would wait for the weight loads too
    }
#pragma unroll
    for (int j = 0; j < SBW; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const float d = h2f_lo(dw[j][n]);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int k4 = t >> 1, sub = t & 1;
          const int si = hh * 8 + p + 2 * k4;
          const float ds = __fmul_rn(d, (float)(int)(int8_t)byte_of(sc[j][n], si));
          const float nds = -32.0f * ds;  // exact (a power-of-two multiple of an fp16 x int8 product)
          // the 6-bit codes of 4 weights assembled as bytes of one word (nibble | 2 high bits
          // << 4), each byte converted straight to fp32 (v_cvt_f32_ubyte*), then
          // fma(ds, q, -32 ds) = ds * (q - 32) with the single rounding of ggml's product (only
          // the sign of an exact zero can differ); ~3 VALU per weight instead of ~7
          const uint4 qsrc = (k4 & 1) ? qb[j][n] : qa[j][n];
          uint32_t pk[4];
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const int wi = 2 * sub + w;  // weights li = 4 wi .. 4 wi + 3
            const uint32_t aw = wi == 0 ? qsrc.x : wi == 1 ? qsrc.y : wi == 2 ? qsrc.z : qsrc.w;
            const uint32_t hw = wi == 0 ? qh[j][n].x : wi == 1 ? qh[j][n].y : wi == 2 ? qh[j][n].z : qh[j][n].w;
            const uint32_t q4 = (((k4 >> 1) ? (aw >> 4) : aw) & 0x0F0F0F0Fu) | (((hw >> (2 * k4)) & 0x03030303u) << 4);
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 ds2 = {ds, ds}, nds2 = {nds, nds};  // two weights per v_pk_fma_f32
            const f2 y01 = __builtin_elementwise_fma(ds2, f2{(float)(q4 & 0xFFu), (float)((q4 >> 8) & 0xFFu)}, nds2);
            const f2 y23 = __builtin_elementwise_fma(ds2, f2{(float)((q4 >> 16) & 0xFFu), (float)(q4 >> 24)}, nds2);
            pk[2 * w] = pack2h(y01.x, y01.y);
            pk[2 * w + 1] = pack2h(y23.x, y23.y);
          }
          const f16x8 wf = __builtin_bit_cast(f16x8, pk);
          const int k = (sb0 + j) * 256 + hh * 128 + k4 * 32 + 16 * p + 8 * sub;
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int xrow = min(m * 16 + fr, M - 1);
            const f16x8 xf = XR ? xr[XR ? j : 0][XR ? t : 0][XR ? m : 0]
                            : XL ? *(const f16x8*)(smem + x_lds(xrow, k, K))
                                 : *(const f16x8*)(X + (size_t)xrow * ldx + k);
            acc[m][n] = mfma16(xf, wf, acc[m][n]);
          }
        }
      }
  }
  gemv_finish<MT, NT, EPI, RS>(acc, smem, rinv_off, M, N, ldo, out, n0, ga, pre, rsd);
}

// ---- the Q6_K lm_head (greedy argmax partials) as a grid-stride two-stage loop.  One-tile
// blocks (qgemv_kernel) each DMA the whole X image (M x K fp16: 48 KiB at M = 8 -- 385 MB over
// the vocabulary's 8016 tiles, more than the weights' 323 MB) and pay one exposed weight
// latency per tile.  Here 2 x 256 resident blocks stage X and the rows' norm factors once,
// then walk tiles b, b + G, ...: each wave issues the NEXT tile's weight loads (17 VGPRs)
// before it dequantises and multiplies the current one, and the per-tile cross-wave reduction
// uses LDS-only barriers so those loads stay in flight.  Per tile the arithmetic is
// qgemv_kernel<1, 1, ARGMAX, 1, LDS, true>'s exactly (same K split over waves, same MFMA order,
// same reduction order and epilogue): bit-identical partials.
struct Q6Regs {
  uint4 qa, qb, qh, sc;
  uint32_t dw;
};
__device__ __forceinline__ void q6_fetch(Q6Regs& r, const uint8_t* base, int row_bytes, int n0, int fr, int sb,
                                         int hh, int p) {
  const uint8_t* bp = base + (size_t)(n0 + fr) * row_bytes + (size_t)sb * kQ6KPacked;
  r.qa = ldw16(bp + 32 * hh + 16 * p);  // = 16 g: quant_rows_kernel's ql regrouping
  r.qb = ldw16(bp + 64 + 32 * hh + 16 * p);
  r.qh = ldw16(bp + 128 + hh * 32 + 16 * p);
  r.sc = ldw16(bp + 192);
  r.dw = *(const uint32_t*)(bp + 208);
}
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(6, 8))) void qgemv_q6_argmax_gs_kernel(const f16_t* __restrict__ X, QMat qm,
                                                                float2* __restrict__ out, int M, int N, int K,
                                                                int ldo, int red_off, int rinv_off, GemvArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ELEMS = 256;  // MT = NT = 1
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, g = lane >> 4, hh = g >> 1, p = g & 1;
  const int tiles = N / 16, G = gridDim.x;
  const uint8_t* base = qm.base0;
  const int row_bytes = qm.row_bytes0;
  // 0. row statistics and X once per block, then the first tile's weights
  const bool rs_on = ga.rs.ssq != nullptr;
  if (rs_on) rs_begin<false>(smem, rinv_off, ga.rs, M);
  gemv_dma_x(smem, X, M, K, K);
  __builtin_amdgcn_sched_barrier(0);
  Q6Regs cur, nxt;
  int t = blockIdx.x;
  q6_fetch(cur, base, row_bytes, t * 16, fr, wave, hh, p);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(5));  // X and the statistics landed (issued first)
  __builtin_amdgcn_s_barrier();
  float* rinv = (float*)(smem + rinv_off);
  if (rs_on) rs_finish<false>(smem, rinv_off, ga.rs, M, 0.f);
  lds_sync();
  float* red = (float*)(smem + red_off);
  for (; t < tiles; t += G) {
    const bool more = t + G < tiles;
    if (more) q6_fetch(nxt, base, row_bytes, (t + G) * 16, fr, wave, hh, p);
    __builtin_amdgcn_sched_barrier(0);
    if (more) __builtin_amdgcn_s_waitcnt(vmcnt_imm(5));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    // qgemv_kernel's Q6_K body, SBW = 1 (this wave's super-block = its index), MT = NT = 1
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const float d = h2f_lo(cur.dw);
#pragma unroll
    for (int tt = 0; tt < 8; ++tt) {
      const int k4 = tt >> 1, sub = tt & 1;
      const int si = hh * 8 + p + 2 * k4;
      const float ds = __fmul_rn(d, (float)(int)(int8_t)byte_of(cur.sc, si));
      const float nds = -32.0f * ds;
      const uint4 qsrc = (k4 & 1) ? cur.qb : cur.qa;
      uint32_t pk[4];
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const int wi = 2 * sub + w;
        const uint32_t aw = wi == 0 ? qsrc.x : wi == 1 ? qsrc.y : wi == 2 ? qsrc.z : qsrc.w;
        const uint32_t hw = wi == 0 ? cur.qh.x : wi == 1 ? cur.qh.y : wi == 2 ? cur.qh.z : cur.qh.w;
        const uint32_t q4 = (((k4 >> 1) ? (aw >> 4) : aw) & 0x0F0F0F0Fu) | (((hw >> (2 * k4)) & 0x03030303u) << 4);
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 ds2 = {ds, ds}, nds2 = {nds, nds};
        const f2 y01 = __builtin_elementwise_fma(ds2, f2{(float)(q4 & 0xFFu), (float)((q4 >> 8) & 0xFFu)}, nds2);
        const f2 y23 = __builtin_elementwise_fma(ds2, f2{(float)((q4 >> 16) & 0xFFu), (float)(q4 >> 24)}, nds2);
        pk[2 * w] = pack2h(y01.x, y01.y);
        pk[2 * w + 1] = pack2h(y23.x, y23.y);
      }
      const f16x8 wf = __builtin_bit_cast(f16x8, pk);
      const int k = wave * 256 + hh * 128 + k4 * 32 + 16 * p + 8 * sub;
      const int xrow = min(fr, M - 1);
      acc = mfma16(*(const f16x8*)(smem + x_lds(xrow, k, K)), wf, acc);
    }
    // cross-wave reduction (LDS-only barriers: the next tile's loads stay in flight)
    *(f32x4*)&red[wave * ELEMS + lane * 4] = acc;
    lds_sync();
    if ((int)threadIdx.x < ELEMS) {
      const int e = threadIdx.x, l = (e >> 2) & 63, j = e & 3;
      const int row = 4 * (l >> 4) + j, col = t * 16 + (l & 15);
      float v = -INFINITY;
      if (row < M && col < N) {
        float sum = 0.f;
        for (int q = 0; q < nw; ++q) sum += red[q * ELEMS + e];
        v = sum * (rs_on ? rinv[row] : 1.0f);
      }
      if (!(v == v)) v = -INFINITY;
      int idx = col;
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
      if ((l & 15) == 0 && row < M) out[(size_t)row * ldo + t] = make_float2(v, __int_as_float(idx));
    }
    lds_sync();  // red is rewritten by the next tile
    cur = nxt;
  }
}

// ---- the Q4_K gate/up projection (SwiGLU epilogue) in the same grid-stride form: 256 blocks
// of 12 waves (wave w = super-block w of the 3072-long rows) take X into registers ONCE (the
// one-tile kernel's 512 blocks each re-read the 8 x 3072 X -- 49 MB of L2 traffic against
// 28 MB of weights), then walk 32-row tiles (16 gate + 16 up rows) with the next tile's 6
// weight loads per lane in flight under the current tile's dequant.  Per tile the arithmetic
// is qgemv_kernel<1, 2, SWIGLU, 1, REGS, RS>'s exactly: bit-identical outputs.
struct Q4Regs {
  uint4 hq, q0, q1;
};
__device__ __forceinline__ void q4_fetch(Q4Regs& r, const uint8_t* base, int row_bytes, int row, int sb, int g) {
  const uint8_t* bp = base + (size_t)row * row_bytes + (size_t)sb * kQ4KBytes;
  r.hq = ldw16(bp);
  r.q0 = ldw16(bp + 16 + 16 * g);
  r.q1 = ldw16(bp + 80 + 16 * g);
}
__global__ __launch_bounds__(768) void qgemv_q4_swiglu_gs_kernel(const f16_t* __restrict__ X, QMat qm,
                                                                 f16_t* __restrict__ out, int M, int N, int K,
                                                                 int ldo, int rinv_off, GemvArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = 2, ELEMS = NT * 256;  // MT = 1
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int tiles = N / 32, G = gridDim.x;
  const uint8_t* base = qm.base0;
  const int row_bytes = qm.row_bytes0, row0 = qm.row0_0;
  const bool rs_on = ga.rs.ssq != nullptr;
  if (rs_on) rs_begin<false>(smem, rinv_off, ga.rs, M);
  // this wave's super-block of X (qgemv_kernel's kXRegs load, SBW = 1, MT = 1)
  f16x8 xr[8];
  const f16_t* xrow = X + (size_t)min(fr, M - 1) * K;
#pragma unroll
  for (int t = 0; t < 8; ++t) xr[t] = as_f16x8(ldg16(xrow + (wave * 8 + t) * 32 + 8 * g));
  __builtin_amdgcn_sched_barrier(0);
  Q4Regs cur[NT], nxt[NT];
  int t = blockIdx.x;
#pragma unroll
  for (int n = 0; n < NT; ++n) q4_fetch(cur[n], base, row_bytes, t * 32 - row0 + n * 16 + fr, wave, g);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * NT));  // X and the statistics landed (issued first)
  __builtin_amdgcn_s_barrier();
  const float* rinv = (const float*)(smem + rinv_off);
  if (rs_on) rs_finish<false>(smem, rinv_off, ga.rs, M, 0.f);
  lds_sync();
  float* red = (float*)smem;
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const f16x8 ones = __builtin_bit_cast(f16x8, u4v{0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u});
  for (; t < tiles; t += G) {
    const bool more = t + G < tiles;
    if (more) {
#pragma unroll
      for (int n = 0; n < NT; ++n) q4_fetch(nxt[n], base, row_bytes, (t + G) * 32 - row0 + n * 16 + fr, wave, g);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (more) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * NT));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    f32x4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s_ = 0; s_ < 8; ++s_) {
      const int sh = 8 * (s_ & 3);
      const f16x8 xf = xr[s_];
      const f32x4 xs = mfma16(xf, ones, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const uint4 h = cur[n].hq;
        const uint32_t scw = s_ < 4 ? (h.y & 0x3F3F3F3Fu) : ((h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u));
        const uint32_t mw = s_ < 4 ? (h.z & 0x3F3F3F3Fu) : (((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u));
        const float d1 = __fmul_rn(h2f_lo(h.x), (float)((scw >> sh) & 0xFFu));
        const float m1 = __fmul_rn(h2f_lo(h.x >> 16), (float)((mw >> sh) & 0xFFu));
        const float d1s = d1 * 16777216.0f;
        const uint4 qq = s_ < 4 ? cur[n].q0 : cur[n].q1;
        const int si = s_ & 3;
        const uint32_t qw = si == 0 ? qq.x : si == 1 ? qq.y : si == 2 ? qq.z : qq.w;
        const uint32_t lo = qw & 0x0F0F0F0Fu, hi = (qw >> 4) & 0x0F0F0F0Fu;
        const u4v pk = {__builtin_amdgcn_perm(0u, lo, 0x0C010C00u), __builtin_amdgcn_perm(0u, lo, 0x0C030C02u),
                        __builtin_amdgcn_perm(0u, hi, 0x0C010C00u), __builtin_amdgcn_perm(0u, hi, 0x0C030C02u)};
        const f32x4 A = mfma16(xf, __builtin_bit_cast(f16x8, pk), f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n][i] = __fmaf_rn(-m1, xs[i], __fmaf_rn(d1s, A[i], acc[n][i]));
      }
    }
    // cross-wave reduction and the SwiGLU epilogue (gemv_epilogue's order), LDS-only barriers
#pragma unroll
    for (int n = 0; n < NT; ++n) *(f32x4*)&red[wave * ELEMS + (n * 64 + lane) * 4] = acc[n];
    lds_sync();
    if ((int)threadIdx.x < 256) {
      const int e = threadIdx.x, l = (e >> 2) & 63, j = e & 3;
      const int row = 4 * (l >> 4) + j;
      if (row < M) {
        const float rv = rs_on ? rinv[row] : 1.0f;
        float gs = 0.f, us = 0.f;
        for (int q = 0; q < nw; ++q) gs += red[q * ELEMS + (0 * 64 + l) * 4 + j];
        for (int q = 0; q < nw; ++q) us += red[q * ELEMS + (1 * 64 + l) * 4 + j];
        const float gv = gs * rv, uv = us * rv;
        out[(size_t)row * ldo + t * 16 + (l & 15)] = f2h(gv / (1.0f + __expf(-gv)) * uv);
      }
    }
    lds_sync();  // red is rewritten by the next tile
#pragma unroll
    for (int n = 0; n < NT; ++n) cur[n] = nxt[n];
  }
}

// which K-quant GEMVs take the grid-stride form: MS_QGEMV_GS bit 0 the Q6_K lm_head argmax,
// bit 1 the Q4_K gate/up (default: both; ms_set_qgemv_gs(0): one-tile blocks everywhere).  The
// same form for the single-type split-K slab projections (O, down: X slice staged once per
// block) measured slower -- O 5.10 -> 6.04 us, down 8.89 -> 9.4-10.7 us, decode 1.806 -> 1.871
// ms per Q4_K_M step (profiles/r04/v25_*): those launches are one latency each, and fewer
// blocks leave fewer weight bytes in flight.
static int g_q_gs = -1;
void set_qgemv_gs(bool on) { g_q_gs = on ? 3 : 0; }
static int q_gs_mask() {
  if (g_q_gs < 0) {
    const char* e = getenv("MS_QGEMV_GS");
    g_q_gs = e ? atoi(e) : 3;
  }
  return g_q_gs;
}
static bool q6_gs_on() { return (q_gs_mask() & 1) != 0; }
static bool q4_gs_on() { return (q_gs_mask() & 2) != 0; }


struct QPlan {
  int MT, NT, SBW, waves, tiles;
};

static QPlan qplan(int M, int N, int K, int epi, int rt = 0) {  // K: per-split length
  QPlan p{};
  p.MT = (M + 15) / 16;
  p.NT = (epi == MS_GEMV_EPI_SWIGLU) ? 2 : 1;
  const int rows = epi == MS_GEMV_EPI_RESID_SSQ && rt > 0 ? rt : 16 * p.NT;
  p.tiles = (N + rows - 1) / rows;
  const int nsb = K / 256;
  p.SBW = nsb > 16 ? 2 : 1;
  p.waves = (nsb % p.SBW == 0) ? nsb / p.SBW : 0;
  if (p.waves > 16) p.waves = 0;
  return p;
}

static constexpr size_t kLdsCap = 160 * 1024;

// the X image is staged in LDS only when the whole block's LDS -- the image, the deferred-norm
// factors and the staged statistics (gemv_lds_total) -- fits; a shape whose image alone fits
// (M = 40 at K = 2048: exactly 160 KiB) takes the global-X path instead of being refused
// (a refused split once made one row group of a K-quant batch fall back to an unsplit slab
// while the others split 4 ways, and the residual fold then dropped slabs of every row)
static bool qx_in_lds(int M, int K, const RowScale& rs = RowScale{}) {
  return gemv_lds_total(gemv_x_lds_bytes(M, K), rs, M) <= kLdsCap;
}

static bool qx_in_regs(const QPlan& p) {
  const int m = qgemv_x_mode();
  const bool want = m == 0 || (m == 2 && p.NT == 2) || (m == 3 && p.NT != 2);
  return want && p.MT * p.SBW == 1;
}

static size_t qlds_main(const QPlan& p, int M, int K, const RowScale& rs = RowScale{}) {
  // X image (when it fits and X is not taken into registers)
  const size_t xs = (!qx_in_regs(p) && qx_in_lds(M, K, rs)) ? gemv_x_lds_bytes(M, K) : 0;
  const size_t red = (size_t)p.waves * p.MT * p.NT * 256 * 4;
  return xs > red ? xs : red;
}
static size_t qlds(const QPlan& p, int M, int K, const RowScale& rs = RowScale{}) {
  return gemv_lds_total(qlds_main(p, M, K, rs), rs, M);
}

bool qgemv_supported(int M, int N, int K, int epi, int rs_tiles) {
  if (M < 1 || M > 64 || K % 256 || N % 16) return false;
  if ((epi == MS_GEMV_EPI_ROPE_KV || epi == MS_GEMV_EPI_RESID_SSQ) && M > 16) return false;
  const QPlan p = qplan(M, N, K, epi);
  // the residual epilogue's prefetch covers one element per thread of a >= 256-thread block
  if (epi == MS_GEMV_EPI_RESID_SSQ && p.waves < 4) return false;
  RowScale rs{};
  if (rs_tiles > 0 && epi != MS_GEMV_EPI_ARGMAX && epi != MS_GEMV_EPI_ADD_F32) {  // qgemv_go drops it there
    if (!gemv_rs_supported(M, rs_tiles)) return false;
    rs = make_row_scale(reinterpret_cast<const float*>(16), rs_tiles, 1, 0.f);
  }
  return p.waves > 0 && qlds(p, M, K, rs) <= kLdsCap;
}

template <int MT, int NT, int EPI>
static void qgemv_go(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int ldo,
                     const QPlan& p, const GemvArgs& ga_in, hipStream_t s, int S = 1) {
  GemvArgs ga = ga_in;
  if (EPI == MS_GEMV_EPI_ARGMAX || EPI == MS_GEMV_EPI_ADD_F32) ga.rs = RowScale{};  // r > 0 keeps the order
  if (ga.rs.ssq && rs_stage_floats(ga.rs, M) == 0) return;  // callers check gemv_rs_supported
  const size_t lds = qlds(p, M, K, ga.rs);
  const int ro = (int)gemv_rinv_offset(qlds_main(p, M, K, ga.rs));
  const dim3 grid(p.tiles, S), blk(64 * p.waves);
  if constexpr ((EPI == MS_GEMV_EPI_ROPE_KV || EPI == MS_GEMV_EPI_RESID_SSQ) && MT != 1) {
    return;
  } else {
    const bool xl = qx_in_lds(M, K, ga.rs);
    constexpr bool kRsEpi = gemv_rs_epi<EPI>();
    const bool rs = kRsEpi && ga.rs.ssq != nullptr;
#define QL(SBW_, XM_)                                                                                         \
    do {                                                                                                      \
      if constexpr (kRsEpi) {                                                                                 \
        if (rs) {                                                                                             \
          MS_LAUNCH((qgemv_kernel<MT, NT, EPI, SBW_, XM_, true>), grid, blk, lds, s, X, q, out, M, N, K, ldo, ro, \
                    ga);                                                                                      \
          break;                                                                                              \
        }                                                                                                     \
      }                                                                                                       \
      MS_LAUNCH((qgemv_kernel<MT, NT, EPI, SBW_, XM_, false>), grid, blk, lds, s, X, q, out, M, N, K, ldo, ro, ga); \
    } while (0)
    if (p.SBW == 2 && xl) QL(2, kXLds);
    else if (p.SBW == 2) QL(2, kXGlobal);
    else if (xl && !qx_in_regs(p)) QL(1, kXLds);
    else if (!qx_in_regs(p)) QL(1, kXGlobal);
    else if constexpr (MT == 1) QL(1, kXRegs);
#undef QL
  }
}

template <int MT>
static void qgemv_go_mt(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int ldo, int epi,
                        const QPlan& p, const GemvArgs& ga, hipStream_t s) {
  switch (epi) {
    case MS_GEMV_EPI_STORE_F16: qgemv_go<MT, 1, MS_GEMV_EPI_STORE_F16>(X, q, out, M, N, K, ldo, p, ga, s); break;
    case MS_GEMV_EPI_ADD_F32: qgemv_go<MT, 1, MS_GEMV_EPI_ADD_F32>(X, q, out, M, N, K, ldo, p, ga, s); break;
    case MS_GEMV_EPI_SWIGLU: qgemv_go<MT, 2, MS_GEMV_EPI_SWIGLU>(X, q, out, M, N, K, ldo, p, ga, s); break;
    case MS_GEMV_EPI_ROPE_KV: qgemv_go<MT, 1, MS_GEMV_EPI_ROPE_KV>(X, q, out, M, N, K, ldo, p, ga, s); break;
    case MS_GEMV_EPI_ARGMAX: qgemv_go<MT, 1, MS_GEMV_EPI_ARGMAX>(X, q, out, M, N, K, ldo, p, ga, s); break;
    case MS_GEMV_EPI_RESID_SSQ: qgemv_go<MT, 1, MS_GEMV_EPI_RESID_SSQ>(X, q, out, M, N, K, ldo, p, ga, s); break;
    default: qgemv_go<MT, 1, MS_GEMV_EPI_STORE_F32>(X, q, out, M, N, K, ldo, p, ga, s); break;
  }
}

void launch_qgemv(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int ldo, int epi,
                  const GemvArgs* ga_in, hipStream_t s) {
  if (M <= 0) return;
  const QPlan p = qplan(M, N, K, epi, ga_in ? ga_in->rt : 0);
  if (p.waves == 0) return;  // callers check qgemv_supported()
  GemvArgs ga{};
  if (ga_in) ga = *ga_in;
  // (both grid-stride kernels finish a tile with one thread per element: >= 4 waves)
  if (epi == MS_GEMV_EPI_ARGMAX && q6_gs_on() && q.n == 1 && q.type0 == MS_QT_Q6_K && p.MT == 1 && p.SBW == 1 &&
      p.waves >= 4 && N % 16 == 0) {
    ga.rs = RowScale{};  // as qgemv_go: a row's positive scale never moves its argmax
    // LDS: [X image][per-wave partials][rinv][staged statistics]
    const int red_off = (int)((gemv_x_lds_bytes(M, K) + 15) / 16 * 16);
    const size_t main_bytes = (size_t)red_off + (size_t)p.waves * 256 * 4;
    const int ro = (int)gemv_rinv_offset(main_bytes);
    const size_t lds = gemv_lds_total(main_bytes, ga.rs, M);
    if (lds <= kLdsCap) {
      const int grid = std::min(N / 16, 512);  // two resident blocks per CU
      MS_LAUNCH(qgemv_q6_argmax_gs_kernel, dim3(grid), dim3(64 * p.waves), lds, s, X, q, (float2*)out, M, N, K, ldo,
                red_off, ro, ga);
      return;
    }
  }
  if (epi == MS_GEMV_EPI_SWIGLU && q4_gs_on() && q.n == 1 && q.type0 == MS_QT_Q4_K && p.MT == 1 && p.SBW == 1 &&
      p.NT == 2 && p.waves >= 4 && qx_in_regs(p) && N % 32 == 0) {
    if (ga.rs.ssq && rs_stage_floats(ga.rs, M) == 0) return;  // callers check gemv_rs_supported
    const size_t main_bytes = (size_t)p.waves * 2 * 256 * 4;  // the per-wave partials
    const int ro = (int)gemv_rinv_offset(main_bytes);
    const size_t lds = gemv_lds_total(main_bytes, ga.rs, M);
    if (lds <= kLdsCap) {
      const int grid = std::min(N / 32, 256);  // one 12-wave block per CU
      MS_LAUNCH(qgemv_q4_swiglu_gs_kernel, dim3(grid), dim3(64 * p.waves), lds, s, X, q, (f16_t*)out, M, N, K,
                ldo, ro, ga);
      return;
    }
  }
  switch (p.MT) {
    case 1: qgemv_go_mt<1>(X, q, out, M, N, K, ldo, epi, p, ga, s); break;
    case 2: qgemv_go_mt<2>(X, q, out, M, N, K, ldo, epi, p, ga, s); break;
    case 3: qgemv_go_mt<3>(X, q, out, M, N, K, ldo, epi, p, ga, s); break;
    default: qgemv_go_mt<4>(X, q, out, M, N, K, ldo, epi, p, ga, s); break;
  }
}

bool qgemv_split_supported(int M, int N, int K, int S, int rs_tiles) {
  if (S < 1 || K % (256 * S)) return false;
  return qgemv_supported(M, N, K / S, MS_GEMV_EPI_STORE_F32, rs_tiles);
}

// fp32 partial slabs [S][M][N] over S equal K ranges (super-block aligned); the caller
// folds them (residual_rmsnorm_kernel / the decode attention prologue)
void launch_qgemv_split(const f16_t* X, const QMat& q, float* slabs, int M, int N, int K, int S,
                        hipStream_t s, const GemvArgs* ga_in) {
  if (M <= 0) return;
  const int Ks = K / S;
  const QPlan p = qplan(M, N, Ks, MS_GEMV_EPI_STORE_F32);
  if (p.waves == 0) return;  // callers check qgemv_split_supported()
  GemvArgs ga{};
  if (ga_in) ga = *ga_in;
  switch (p.MT) {
    case 1: qgemv_go<1, 1, MS_GEMV_EPI_STORE_F32>(X, q, slabs, M, N, Ks, N, p, ga, s, S); break;
    case 2: qgemv_go<2, 1, MS_GEMV_EPI_STORE_F32>(X, q, slabs, M, N, Ks, N, p, ga, s, S); break;
    case 3: qgemv_go<3, 1, MS_GEMV_EPI_STORE_F32>(X, q, slabs, M, N, Ks, N, p, ga, s, S); break;
    default: qgemv_go<4, 1, MS_GEMV_EPI_STORE_F32>(X, q, slabs, M, N, Ks, N, p, ga, s, S); break;
  }
}

}  // namespace ms
