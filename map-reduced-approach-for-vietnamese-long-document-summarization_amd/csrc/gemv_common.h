// gemv_common.h -- pieces shared by the fp16 and the K-quant decode GEMVs.
#pragma once
#include "kernels.h"

namespace ms {

__device__ __forceinline__ uint4 ldg16(const void* p) { return *(const uint4*)p; }

// once-read decode weight streams: plain loads (non-temporal ones measured slower on the whole
// decode step, 2.45 vs 2.29 ms, profiles/r01 v5_nt_stream_ab_rejected)
// (re-measured round 5 on the current GEMVs: nt weight loads 2.30 vs 2.10 ms per decode step,
// profiles/r05/v4_attn_ticket_nt_ab3.txt)
__device__ __forceinline__ uint4 ldw16(const void* p) { return *(const uint4*)p; }

// s_waitcnt immediate for vmcnt(n) with expcnt/lgkmcnt left alone (gfx9 encoding)
__host__ __device__ constexpr int vmcnt_imm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

// __syncthreads() for LDS only: waits for this wave's LDS operations (lgkmcnt) but not for
// its global loads, so a register-staged weight stream stays in flight across the barrier
// (a full __syncthreads() fence drains vmcnt as well).  Not for LDS written by DMA.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// X rows [M][K] fp16 (row stride ldx elements) -> LDS image of M rows x 2K bytes, 16-B
// chunk c of row r stored at chunk c ^ (r & 7) (the rows of an MFMA fragment read land on
// different bank groups).  Copied by LDS DMA (global_load_lds, 1 KiB per wave instruction)
// and issued BEFORE the weight stream: vmcnt retires loads in issue order, so X loaded
// after the weights would hold the image -- and every wave of the block, at the barrier --
// until the block's whole weight stream had landed, serialising all the dequant / MFMA work
// behind the memory phase; the DMA needs no registers (a register copy cost the GEMVs
// occupancy).  The caller waits vmcnt(<its weight loads>) and synchronises.  K % 64 == 0;
// the image is padded to whole KiB (the last piece's spare lanes land there).
__host__ __device__ inline size_t gemv_x_lds_bytes(int M, int K) {
  return ((size_t)M * K * 2 + 1023) / 1024 * 1024;
}
__device__ __forceinline__ int x_lds(int r, int k, int K) { return r * 2 * K + (((k >> 3) ^ (r & 7)) << 4); }

__device__ __forceinline__ void gemv_dma_x(char* smem, const f16_t* __restrict__ X, int M, int K, int ldx) {
  const int kch = K >> 3, n = M * kch, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int p = threadIdx.x >> 6; p * 64 < n; p += nw) {
    const int P = min(p * 64 + lane, n - 1);
    const int r = P / kch, c = P - r * kch;
    __builtin_amdgcn_global_load_lds((const void*)(X + (size_t)r * ldx + ((c ^ (r & 7)) << 3)),
                                     (LDS_AS void*)(smem + (size_t)p * 1024), 16, 0, 0);
  }
}

// where a decode GEMV's MFMA takes its X fragments from (k_gemv.hip / k_qgemv.hip)
enum { kXGlobal = 0, kXLds = 1, kXRegs = 2 };

// The deferred RMSNorm scale of a GEMV block's output rows (kernels.h RowScale), compiled only
// into the instantiations that take one (template RS; the rest carry none of this code).  The
// partial sums [tiles][M] are copied into LDS by DMA at the very start of the kernel, ahead of
// the X copy and the weight stream (no registers: a register preload of 256 tiles cost the
// 1024-thread gate/up GEMV its second co-resident block), and folded into rinv[row], which the
// epilogue reads: wave w owns rows w, w + nw, ..; lane l adds tiles l, l + 64, .. in order,
// then the wave's xor tree.  At most kRsStage partial sums (host-checked).  HOLD kernels (the
// K-quant GEMV) take one-tile statistics straight into a register of wave 0 instead; the fp16
// GEMV stages them like any other: holding that register across the weight
// stream took the 1024-thread gate/up GEMV from 63 to 67 VGPRs and cost its second co-resident
// block (20.8 -> 22.4 us per launch, profiles/r03/v9_rs_hold_ab.txt).
constexpr int kRsStage = 4096;  // floats of partial sums a block stages in LDS (16 KiB)
__host__ __device__ inline int rs_stage_floats(const RowScale& rs, int M) {
  const int n = rs.tiles * M;
  return (rs.ssq && n <= kRsStage) ? (n + 63) / 64 * 64 : 0;
}
// LDS of a decode GEMV block: [main: the X image or the per-wave partials, whichever is larger]
// [rinv: 64 floats][staged partial sums]
__host__ __device__ inline size_t gemv_rinv_offset(size_t main_bytes) { return (main_bytes + 15) / 16 * 16; }
__host__ __device__ inline size_t gemv_lds_total(size_t main_bytes, const RowScale& rs, int M) {
  return gemv_rinv_offset(main_bytes) + 64 * 4 + (size_t)rs_stage_floats(rs, M) * 4;
}
// issued before every other load of the kernel: HOLD and one-tile statistics -> lane l of wave 0
// holds ssq[l] (returned); otherwise LDS DMA into the stage (returns 0)
template <bool HOLD>
__device__ __forceinline__ float rs_begin(char* smem, size_t rinv_off, const RowScale& rs, int M) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if constexpr (HOLD)
    if (rs.tiles == 1) return (wave == 0 && lane < M) ? rs.ssq[lane] : 0.f;
  const int nf = rs_stage_floats(rs, M), n = rs.tiles * M;
  float* stage = (float*)(smem + rinv_off) + 64;
  for (int p = wave; p * 64 < nf; p += nw)
    __builtin_amdgcn_global_load_lds((const void*)(rs.ssq + min(p * 64 + lane, n - 1)),
                                     (LDS_AS void*)(stage + p * 64), 4, 0, 0);
  return 0.f;
}
// every wave calls this after a barrier that follows the DMA's completion (vmcnt); rinv[row]
// for row < M once the caller's next barrier has passed.  (Callers check rs_stage_floats: the
// engine's are <= 256 tiles x 16 rows.)
template <bool HOLD>
__device__ __forceinline__ void rs_finish(const char* smem, size_t rinv_off, const RowScale& rs, int M,
                                          float direct) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float* rinv = (float*)(smem + rinv_off);
  if (HOLD && rs.tiles == 1) {  // one partial: the wave tree of {ssq, 0, ..} is ssq itself
    if (wave == 0 && lane < M) rinv[lane] = rs_rinv(direct, rs);
    return;
  }
  const float* stage = rinv + 64;
  for (int row = wave; row < M; row += nw) {
    float sum = 0.f;
    for (int t = lane; t < ((rs.tiles + 63) & ~63); t += 64) sum += t < rs.tiles ? stage[t * M + row] : 0.f;
    sum = wave_sum(sum);
    if (lane == 0) rinv[row] = rs_rinv(sum, rs);
  }
}

// the deferred row scale exists only for the epilogues of normalised projections
template <int EPI> constexpr bool gemv_rs_epi() {
  return EPI == MS_GEMV_EPI_STORE_F16 || EPI == MS_GEMV_EPI_SWIGLU || EPI == MS_GEMV_EPI_STORE_F32 ||
         EPI == MS_GEMV_EPI_ROPE_KV;
}

constexpr int kXRegsMaxFrags = 4;  // MT x (U or 8*SBW/8) fragment pairs a wave may hold (<= 32 VGPRs)
// X source per GEMV family, measured same-box on MI355X at B = 8 (profiles/r02/v14_x_regs_ab.txt):
// the K-quant GEMVs take X into registers (Q4_K_M decode 2.023 -> 1.950 ms/step: the dequant
// work of each wave starts as soon as its own bytes land, with no block barrier), the fp16
// GEMVs keep the LDS image (registers measured 2.25 -> 2.39 ms/step).  MS_GEMV_X=regs /
// MS_QGEMV_X (below) flip them (A/B tuning).
// fp16 X source (MS_GEMV_X): "lds" everywhere (default), "regs" everywhere (where MT x U fits),
// "f32" registers for the split-K slab GEMVs only, "resid" for the residual-epilogue GEMVs only,
// "both" for those two families
enum { kGxLds = 0, kGxRegs = 1, kGxF32 = 2, kGxResid = 3, kGxBoth = 4 };
inline int gemv_x_mode() {
  static const int v = [] {
    const char* e = getenv("MS_GEMV_X");
    if (!e) return kGxLds;
    const char c = e[0];
    return c == 'r' && e[1] == 'e' && e[2] == 'g' ? kGxRegs : c == 'f' ? kGxF32 : c == 'r' ? kGxResid
         : c == 'b' ? kGxBoth : kGxLds;
  }();
  return v;
}
inline bool gemv_x_regs_for(int epi) {
  const int m = gemv_x_mode();
  const bool f32 = epi == MS_GEMV_EPI_STORE_F32, resid = epi == MS_GEMV_EPI_RESID_SSQ;
  return m == kGxRegs || ((m == kGxF32 || m == kGxBoth) && f32) || ((m == kGxResid || m == kGxBoth) && resid);
}
// K-quant X source (MS_QGEMV_X): 0 registers everywhere ("regs"), 1 LDS everywhere ("lds"),
// 2 registers for the gate/up GEMV only ("gu", the default), 3 registers for all but gate/up
// ("slab").  Same box, Q4_K_M decode ms/step: regs 1.862, lds 1.892, gu 1.845, slab 1.909
// (profiles/r03/v15_qgemv_x_mode_ab.txt): the two-tile gate/up blocks start their dequant as
// their own X lands; the one-tile slab / lm_head blocks (80 / 70 VGPRs with X in registers)
// do better with the LDS image.
inline int qgemv_x_mode() {
  static const int v = [] {
    const char* e = getenv("MS_QGEMV_X");
    if (!e) return 2;
    return e[0] == 'r' ? 0 : e[0] == 'l' ? 1 : e[0] == 'g' ? 2 : e[0] == 's' ? 3 : 2;
  }();
  return v;
}

__device__ __forceinline__ void amax_merge_dev(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

// Cross-wave reduction of the per-wave MFMA accumulators through LDS and the epilogue.
// acc[m][n][j] = C[row m*16 + 4*(lane>>4) + j][col n0 + n*16 + (lane&15)].
// RESID_SSQ: the x and gamma element each epilogue thread updates, loaded at kernel start
// (ahead of the weight stream) so the epilogue itself waits on no memory
struct ResidPre {
  float x, g;
};
template <int MT, int NT, int EPI, bool RS>
__device__ __forceinline__ void gemv_epilogue(const float* red, const float* rinv, int M, int N, int ldo,
                                              void* __restrict__ out, int n0, const GemvArgs& ga,
                                              const ResidPre& pre);
// element e of a tile result [mt][nt][lane][j] -> (row, col) of the output
__device__ __forceinline__ void gemv_elem(int e, int NT, int n0, int& row, int& col, int& c) {
  const int mn = e >> 8, l = (e >> 2) & 63, j = e & 3;
  row = (mn / NT) * 16 + 4 * (l >> 4) + j;
  c = l & 15;
  col = n0 + (mn % NT) * 16 + c;
}
template <int EPI>
__device__ __forceinline__ ResidPre resid_prefetch(int M, int N, int ldo, const void* out, int n0,
                                                   const GemvArgs& ga) {
  ResidPre p{0.f, 0.f};
  if constexpr (EPI == MS_GEMV_EPI_RESID_SSQ) {
    const int rtv = ga.rt > 0 ? ga.rt : 16;
    if ((int)threadIdx.x < 256) {  // MT = NT = 1: one element per thread
      int row, col, c;
      gemv_elem(threadIdx.x, 1, n0, row, col, c);
      if (row < M && c < rtv && col < N) {
        p.x = ((const float*)out)[(size_t)row * ldo + col];
        if (ga.xg_out) p.g = h2f(ga.gamma[col]);
      }
    }
  }
  return p;
}

// RS: the block's output rows carry a deferred-norm scale (ga.rs, rs_begin); RS_DONE: the
// kernel already folded the factors (rs_finish right after its X barrier, under the weights);
// RS_HOLD: rs_begin held one-tile statistics in the register passed as rs_direct
template <int MT, int NT, int EPI, bool RS = false, bool RS_DONE = false, bool RS_HOLD = true>
__device__ __forceinline__ void gemv_finish(const f32x4 (&acc)[MT][NT], char* smem, size_t rinv_off,
                                            int M, int N, int ldo, void* __restrict__ out, int n0,
                                            const GemvArgs& ga, const ResidPre& pre = ResidPre{0.f, 0.f},
                                            float rs_direct = 0.f) {
  constexpr int ELEMS = MT * NT * 256;  // floats per wave result [mt][nt][lane][j]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* rinv = (const float*)(smem + rinv_off);
  if constexpr (RS && !RS_DONE) wait_vmcnt0();  // the staged partial sums (rs_begin's DMA) have landed
  __syncthreads();  // X image no longer needed: reuse LDS for the partials
  if constexpr (RS && !RS_DONE) rs_finish<RS_HOLD>(smem, rinv_off, ga.rs, M, rs_direct);
  float* red = (float*)smem;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
      *(f32x4*)&red[wave * ELEMS + ((m * NT + n) * 64 + lane) * 4] = acc[m][n];
  __syncthreads();
  gemv_epilogue<MT, NT, EPI, RS>(red, rinv, M, N, ldo, out, n0, ga, pre);
}

// The epilogue of a decode GEMV tile from the per-wave partials in LDS (red[wave][elem]).
template <int MT, int NT, int EPI, bool RS>
__device__ __forceinline__ void gemv_epilogue(const float* red, const float* rinv, int M, int N, int ldo,
                                              void* __restrict__ out, int n0, const GemvArgs& ga,
                                              const ResidPre& pre) {
  constexpr int ELEMS = MT * NT * 256;
  const int tid = threadIdx.x;
  const int nthreads = blockDim.x, nw = nthreads >> 6;
  auto rsc = [&](int row) { return RS ? rinv[row] : 1.0f; };
  // element e = ((m*NT + n)*64 + l)*4 + j -> row m*16 + 4*(l>>4) + j, col n0 + n*16 + (l&15)
  auto sum_e = [&](int e) {
    float v = 0.f;
    for (int q = 0; q < nw; ++q) v += red[q * ELEMS + e];
    return v;
  };
  if constexpr (EPI == MS_GEMV_EPI_SWIGLU) {
    for (int e = tid; e < MT * 256; e += nthreads) {
      const int m = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int row = m * 16 + 4 * (l >> 4) + j;
      if (row >= M || n0 >= N) continue;
      const float rv = rsc(row);
      const float g = sum_e(((m * NT + 0) * 64 + l) * 4 + j) * rv;
      const float u = sum_e(((m * NT + 1) * 64 + l) * 4 + j) * rv;
      const int f = (n0 >> 5) * 16 + (l & 15);
      ((f16_t*)out)[(size_t)row * ldo + f] = f2h(g / (1.0f + __expf(-g)) * u);
    }
  } else if constexpr (EPI == MS_GEMV_EPI_ROPE_KV) {
    static_assert(MT == 1 && NT == 1, "rope epilogue works on single 16-row tiles");
    // element of (row, col) in tile (0, 0): l = 16*(row>>2) + col, j = row & 3
    auto e_of = [](int row, int col) { return ((((row >> 2) << 4) + col) << 2) + (row & 3); };
    const int QD = ga.Hq * kHeadDim, KD = ga.Hk * kHeadDim;
    if (n0 < QD + KD) {  // Q or K head: tile t of head h holds dims 8t..8t+7 | 64+8t..64+8t+7
      const bool is_q = n0 < QD;
      const int h = is_q ? n0 / kHeadDim : (n0 - QD) / kHeadDim;
      const int t = (n0 % kHeadDim) / 16;
      for (int e = tid; e < M * 8; e += nthreads) {
        const int row = e >> 3, c = e & 7, i = 8 * t + c;
        const float rv = rsc(row);
        const float lo = h2f(f2h(sum_e(e_of(row, c)) * rv));      // q/k rounded to fp16, then
        const float hi = h2f(f2h(sum_e(e_of(row, c + 8)) * rv));  // rotated in fp32 (as prefill)
        const int pos = ga.tok_pos[row];
        const float cs = ga.cos_tab[(size_t)pos * 64 + i], sn = ga.sin_tab[(size_t)pos * 64 + i];
        const float ra = __fsub_rn(__fmul_rn(lo, cs), __fmul_rn(hi, sn));
        const float rb = __fadd_rn(__fmul_rn(hi, cs), __fmul_rn(lo, sn));
        f16_t* dst;
        if (is_q) {
          dst = (f16_t*)out + (size_t)row * ldo + h * kHeadDim;
        } else {
          const int slot = ga.tok_slot[row];
          const int page = ga.kv.block_table[(size_t)slot * ga.kv.max_pages + pos / kPage];
          dst = ga.kv.k + (((size_t)page * ga.kv.n_kv_heads + h) * kPage + pos % kPage) * kHeadDim;
        }
        dst[i] = f2h(ra);
        dst[64 + i] = f2h(rb);
      }
    } else {  // V head: natural order, straight into the cache
      const int h = (n0 - QD - KD) / kHeadDim, d0 = n0 % kHeadDim;
      for (int e = tid; e < M * 16; e += nthreads) {
        const int row = e >> 4, c = e & 15;
        const int pos = ga.tok_pos[row], slot = ga.tok_slot[row];
        const int page = ga.kv.block_table[(size_t)slot * ga.kv.max_pages + pos / kPage];
        ga.kv.v[(((size_t)page * ga.kv.n_kv_heads + h) * kPage + pos % kPage) * kHeadDim + d0 + c] =
            f2h(sum_e(e_of(row, c)) * rsc(row));
      }
    }
  } else if constexpr (EPI == MS_GEMV_EPI_RESID_SSQ) {
    static_assert(NT == 1, "residual epilogue works on single-column-tile plans");
    const int rtv = ga.rt > 0 ? ga.rt : 16;
    // a row's 16 columns sit in lanes 4c + j of one wave: reduce over lane bits 2..5
    for (int e = tid; e < ELEMS; e += nthreads) {
      const int m = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int row = m * 16 + 4 * (l >> 4) + j, c = l & 15, col = n0 + c;
      float q = 0.f;
      if (row < M && c < rtv && col < N) {
        float* px = (float*)out + (size_t)row * ldo + col;
        const float xo = (ELEMS <= 256 ? pre.x : *px) + sum_e(e);  // pre: resid_prefetch
        *px = xo;
        q = xo * xo;
        // the fp32 product, then its fp16 rounding (the oracle's f16(x * g), rmsnorm_kernel's
        // v_cvt_pk_f16_f32): left visible, the compiler fused x * g -> fp16 into one
        // v_fma_mixlo_f16, a single rounding of the exact product that differs at ties
        if (ga.xg_out) {
          float xg = xo * (ELEMS <= 256 ? pre.g : h2f(ga.gamma[col])) * kXgScale;
          asm volatile("" : "+v"(xg));
          ga.xg_out[(size_t)row * ldo + col] = f2h(xg);
        }
      }
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
      if (c == 0 && row < M) ga.ssq_out[(size_t)blockIdx.x * M + row] = q;
    }
  } else if constexpr (EPI == MS_GEMV_EPI_ARGMAX) {
    static_assert(NT == 1, "argmax epilogue works on 16-column tiles");
    // lanes sharing (m, l>>4, j) hold one row's 16 columns: they differ in lane bits 2..5
    for (int e = tid; e < ELEMS; e += nthreads) {
      const int m = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int row = m * 16 + 4 * (l >> 4) + j, col = n0 + (l & 15);
      float v = (row < M && col < N) ? sum_e(e) * rsc(row) : -INFINITY;
      if (!(v == v)) v = -INFINITY;  // NaN never wins
      int idx = col;
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
      if ((l & 15) == 0 && row < M)
        ((float2*)out)[(size_t)row * ldo + blockIdx.x] = make_float2(v, __int_as_float(idx));
    }
  } else {
    for (int e = tid; e < ELEMS; e += nthreads) {
      const int mn = e >> 8, l = (e >> 2) & 63, j = e & 3;
      const int m = mn / NT, n = mn % NT;
      const int row = m * 16 + 4 * (l >> 4) + j;
      const int col = n0 + n * 16 + (l & 15);
      if (row >= M || col >= N || (NT == 1 && ga.rt > 0 && (l & 15) >= ga.rt)) continue;
      const float v = sum_e(e);
      const size_t o = (size_t)row * ldo + col;
      if constexpr (EPI == MS_GEMV_EPI_STORE_F16) ((f16_t*)out)[o] = f2h(v * rsc(row));
      else if constexpr (EPI == MS_GEMV_EPI_ADD_F32) ((float*)out)[o] += v;
      else ((float*)out)[o] = v * rsc(row);
    }
  }
}

}  // namespace ms
