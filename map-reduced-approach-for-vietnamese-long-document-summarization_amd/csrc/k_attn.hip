// k_attn.hip -- causal GQA attention of the map call over the paged KV cache.
//
// Replaces ggml's attention (mul_mat+soft_max / flash_attn_ext) inside Ollama
// (SURVEY.md §2 'ggml op replaced', §8a rows A8/A9).  head_dim 128, any GQA group.
//
// KV cache: pool[page][kv_head][64 tokens][128] fp16, one page = one 64-key tile;
// a per-sequence block table maps logical tile -> page (engine.cpp owns the pages).
//
// Both kernels use the "swapped" orientation on v_mfma_f32_16x16x32_f16:
//   S^T = K . Q^T     (A = K rows from LDS/HBM, B = Q fragments held in VGPRs)
//   O^T += V^T . P^T  (A = V^T via ds_read_b64_tr_b16 from a row-major V tile,
//                      B = P^T taken straight from the S^T accumulators)
// so the query index sits on the MFMA column (lane & 15) in S^T, P^T and O^T alike:
// the online-softmax max/sum need only two lane-group swaps and the O rescale is
// lane-local.  The k order inside a PV step is permuted (keys 4g..4g+3 and
// 16+4g..16+4g+3 for lane group g), identically on both operands.
// LDS images: K rows swizzled chunk ^ (row & 15) (ds_read_b128, conflict-free);
// V rows swizzled chunk ^ ((row & 7) << 1) (tr reads conflict-free).
#include <algorithm>

#include "attn_common.h"

namespace ms {

// ============================================================ prefill (varlen, causal)
// 1-D grid over (q-block, head group), heaviest q-blocks first for every head group; block
// 512 = 8 waves x 16 query rows (kPrefillQRows = 128), GB q heads of ONE kv head (GQA group, or
// a divisor of it).  Each K fragment read from LDS feeds GB MFMAs (S^T of the GB heads) and each
// V^T fragment GB MFMAs (O^T of the GB heads), and each K/V tile is fetched once per 128 query
// rows x GB heads.  Two waves per SIMD (launch bounds 512, 1: <= 256 registers a wave, the O
// accumulators of the GB heads in AGPRs): one wave's softmax and LDS reads run under the other's
// MFMAs -- the round-3 kernel (4 waves x 16 rows, hi + lo bf16 P) held 240 VGPRs + 148 AGPRs at
// one wave per SIMD and could not hide its own QK -> softmax -> PV chain.  The online softmax
// works on raw scores (p = exp2(s*c - m*c), c = log2(e)/sqrt(d)) with a lazily moved reference
// max (below); the O rescale is skipped when no query column of the wave moved it; the causal /
// sequence-end mask is applied only on tiles that can cross it, and a wave skips the tiles that
// lie wholly after its last query.  K/V tiles reach LDS by DMA (global_load_lds, no register
// staging and no ds_write), two buffers: tile t+1 is in flight while tile t is multiplied, one
// barrier per tile.  The swizzles are applied on the DMA source (lane i of a 1-KiB piece lands
// at chunk i % 16 of row i / 16, so it loads the global chunk that belongs there); rows past
// the sequence load the last valid row instead (finite values under P = 0: never NaN * 0 in P.V).
template <int GB>
__global__ __launch_bounds__(512, 1) void attn_prefill_kernel(const f16_t* __restrict__ qkv,
                                                              f16_t* __restrict__ out, int Hq,
                                                              int Hk, KVView kv, PrefillAttnArgs a,
                                                              float scale_log2) {
  constexpr int QR = kPrefillQRows;  // 128 query rows per block
  // [K|V tile buffer 0][K|V tile buffer 1][Q of the GB heads, QR x 256 B each]: 160 KiB at GB = 3
  __shared__ __attribute__((aligned(16))) char smem[2 * 32768 + GB * QR * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int ngrp = Hq / GB;
  const int e = a.qblk[blockIdx.x / ngrp];
  const int h0 = (blockIdx.x % ngrp) * GB;
  const int sq = e >> 16, qb = e & 0xFFFF;
  const int qlen = a.seq_qlen[sq], kvlen = a.seq_kvlen[sq], qstart = a.seq_qstart[sq];
  const int slot = a.seq_slot[sq];
  const int kvh = h0 / (Hq / Hk);
  const int row_stride = (Hq + 2 * Hk) * kHeadDim;
  const int q0 = qb * QR + wave * 16;  // the wave's first query (sequence-relative)
  const int qi = q0 + r;
  const int qpos = kvlen - qlen + qi;
  const int wave_qpos0 = kvlen - qlen + q0;
  const int wave_qlast = kvlen - qlen + min(q0 + 15, qlen - 1);  // keys after it: nothing to do
  const bool wave_live = q0 < qlen;

  const int q_last = min(qb * QR + QR - 1, qlen - 1);
  const int kv_end = kvlen - qlen + q_last + 1;  // keys visible to the block's last query
  const int ntiles = (kv_end + 63) / 64;
  const int32_t* bt = kv.block_table + (size_t)slot * kv.max_pages;

  // this wave's 4 DMA pieces of a tile: piece J = 4*wave + i covers rows 4(J % 16) ..+3 of
  // K (J < 16) or V; lane -> row 4(J % 16) + lane / 16, LDS chunk lane % 16
  auto page_of = [&](int t) { return kv.slot_major ? (int)(bt - kv.block_table) + t : bt[t]; };
  // (waves 0-3 load K, 4-7 V: J >> 4 = wave >> 2; the source array is picked once, in scalar
  // registers -- a per-piece select reloaded the kernel argument by a vector load every tile)
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const bool dma_v = wave_u >= 4;
  const f16_t* dma_src = dma_v ? kv.v : kv.k;
  const int n_kv_heads = kv.n_kv_heads;
  auto dma_tile = [&](int pid, int t, int buf) {
    const f16_t* page = dma_src + ((size_t)pid * n_kv_heads + kvh) * kPage * kHeadDim;
    const int lim = kvlen - t * 64;  // rows >= lim are past the sequence
    char* img = smem + buf * 32768 + (dma_v ? 16384 : 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int J = 4 * wave_u + i;
      const int row = 4 * (J & 15) + (lane >> 4), c = lane & 15;
      const int srow = min(row, lim - 1);
      const int sch = dma_v ? (c ^ ((row & 7) << 1)) : (c ^ (row & 15));
      dma16_opaque(page + srow * kHeadDim + sch * 8, img + 4 * (J & 15) * 256);
    }
  };
  dma_tile(page_of(0), 0, 0);

  // tile 0's K/V DMA is issued before the Q prologue's loads: the two round trips overlap
  // (in-order vmcnt: the prologue's compiler-counted waits also cover these four pieces)
  // Q fragments live in LDS (each wave reads back only its own 16 rows, swizzled like K)
  char* qimg = smem + 2 * 32768;
  const int qrow_l = wave * 16 + r;
  {
    const int qr = min(qi, qlen - 1);
    const f16_t* qrow = qkv + (size_t)(qstart + qr) * row_stride + h0 * kHeadDim;
    if (a.cos_tab) {
      // Q straight from the GEMM: head dims in the rope-permuted order (the 16-element group
      // g8 holds dims 8 g8 .. +7, then 64 + 8 g8 .. +7), rotated here with rope_kv_kernel's
      // arithmetic (fp16 in, fp32 rotation, fp16 out) into natural chunks g8 and 8 + g8 --
      // which are this lane group's chunks 4s + g for s = t and 2 + t (g8 = 4t + g)
      const int pos = kvlen - qlen + qr;
      const float* ct = a.cos_tab + (size_t)pos * 64;
      const float* st = a.sin_tab + (size_t)pos * 64;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int g8 = 4 * t + g;
        const float4 c0 = *(const float4*)(ct + 8 * g8), c1 = *(const float4*)(ct + 8 * g8 + 4);
        const float4 s0 = *(const float4*)(st + 8 * g8), s1 = *(const float4*)(st + 8 * g8 + 4);
        const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int hh = 0; hh < GB; ++hh) {
          const uint4 lo = *(const uint4*)(qrow + hh * kHeadDim + 16 * g8);
          const uint4 hi = *(const uint4*)(qrow + hh * kHeadDim + 16 * g8 + 8);
          const uint32_t lw[4] = {lo.x, lo.y, lo.z, lo.w}, hw[4] = {hi.x, hi.y, hi.z, hi.w};
          uint32_t ra[4], rb[4];
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            float r0[2], r1[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const float av = e ? h_hi(lw[p]) : h_lo(lw[p]), bv = e ? h_hi(hw[p]) : h_lo(hw[p]);
              const float c = cc[2 * p + e], sn = ss[2 * p + e];
              r0[e] = __fsub_rn(__fmul_rn(av, c), __fmul_rn(bv, sn));
              r1[e] = __fadd_rn(__fmul_rn(bv, c), __fmul_rn(av, sn));
            }
            ra[p] = pack2h(r0[0], r0[1]);
            rb[p] = pack2h(r1[0], r1[1]);
          }
          *(uint4*)(qimg + q_swz<GB>(qrow_l, hh, 4 * t + g)) = uint4{ra[0], ra[1], ra[2], ra[3]};
          *(uint4*)(qimg + q_swz<GB>(qrow_l, hh, 4 * (2 + t) + g)) = uint4{rb[0], rb[1], rb[2], rb[3]};
        }
      }
    } else {
#pragma unroll
      for (int hh = 0; hh < GB; ++hh)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          *(uint4*)(qimg + q_swz<GB>(qrow_l, hh, 4 * s + g)) = *(const uint4*)(qrow + hh * kHeadDim + 32 * s + 8 * g);
    }
  }
  f32x4 o[GB][8];
  float m_run[GB], l_run[GB];
#pragma unroll
  for (int hh = 0; hh < GB; ++hh) {
    m_run[hh] = -INFINITY;
    l_run[hh] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[hh][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // Lockstep: every wave runs QK, softmax and PV of tile t between two barriers.  A staggered
  // schedule (wave groups w < 4 and w >= 4, which share SIMDs, one phase apart so one wave's
  // QK MFMAs run beside the other's softmax) measured slower: 356 vs 295 us per layer at
  // configs[1] (two barriers and half-tile DMA waits per tile; profiles/r04/v5_*).
  // page ids run one tile ahead of the DMAs: tile t+1's DMA never waits on a table load
  int pid_next = ntiles > 1 ? page_of(1) : 0;
  for (int t = 0; t < ntiles; ++t) {
    // tile t landed (its DMA and the next page id are the only global loads in flight), and
    // every wave is past tile t-1, whose buffer the next DMA overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 1 < ntiles) {
      dma_tile(pid_next, t + 1, (t + 1) & 1);
      pid_next = t + 2 < ntiles ? page_of(t + 2) : 0;
    }
    if (!wave_live || t * 64 > wave_qlast) continue;  // wave-uniform: keys after every query
    const char* ks_ = smem + (t & 1) * 32768;
    const char* vs_ = ks_ + 16384;

    // S^T by k-step s outermost: the 4 x GB accumulators of a step are independent MFMAs,
    // and step s+1's K / Q fragments are read from LDS under step s's
    f32x4 sc[GB][4];
    f16x8 kf[2][4], qf[2][GB];
    auto rd_step = [&](int s, int b) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) kf[b][mt] = *(const f16x8*)(ks_ + k_swz(mt * 16 + r, 4 * s + g));
#pragma unroll
      for (int hh = 0; hh < GB; ++hh) qf[b][hh] = *(const f16x8*)(qimg + q_swz<GB>(qrow_l, hh, 4 * s + g));
    };
    rd_step(0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s + 1 < 4) rd_step(s + 1, (s + 1) & 1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int hh = 0; hh < GB; ++hh)
          sc[hh][mt] = mfma16(kf[s & 1][mt], qf[s & 1][hh], s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : sc[hh][mt]);
    }
    // pin that order (the scheduler otherwise issues each read just before its MFMA and
    // waits on it): [reads s=0] then per step [reads s+1][4 GB MFMAs of s]
    __builtin_amdgcn_sched_group_barrier(0x100, 4 + GB, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s + 1 < 4) __builtin_amdgcn_sched_group_barrier(0x100, 4 + GB, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * GB, 0);
    }
    // keys past this query (causal) or past the sequence: only tiles reaching past the wave's
    // first query or the sequence end can hold any
    const bool masked = (t * 64 + 63 > wave_qpos0) || (t * 64 + 64 > kvlen);
    if (masked) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = t * 64 + mt * 16 + 4 * g + j;
          if (key > qpos || key >= kvlen)
#pragma unroll
            for (int hh = 0; hh < GB; ++hh) sc[hh][mt][j] = -INFINITY;
        }
    }
    f16x8 pf[GB][2];
    bool rescale = false;
    float alpha[GB];
#pragma unroll
    for (int hh = 0; hh < GB; ++hh) {
      float mx = -INFINITY;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, sc[hh][mt][j]);
      mx = grp_max(mx);
      // lazy rescale: the running max only moves when a tile's max exceeds it by more than
      // 8 in log2 units (p <= 2^8 is harmless in fp32 and in fp16 P), so after the first
      // tiles the O accumulators are rarely rescaled; O / l is unchanged by the choice of
      // reference max
      const float m_new = fmaxf(m_run[hh], mx);
      const bool grow = m_new != m_run[hh] && !((m_new - m_run[hh]) * scale_log2 <= 8.f);
      const float m_use = grow ? m_new : m_run[hh];
      alpha[hh] = grow ? __builtin_amdgcn_exp2f((m_run[hh] - m_new) * scale_log2) : 1.f;
      rescale |= grow;
      const float mc = (m_use == -INFINITY) ? 0.f : m_use * scale_log2;
      float rs = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __builtin_amdgcn_exp2f(__fmaf_rn(sc[hh][mt][j], scale_log2, -mc));
          sc[hh][mt][j] = p;
          rs += p;
        }
      rs = grp_sum(rs);
      l_run[hh] = l_run[hh] * alpha[hh] + rs;
      m_run[hh] = m_use;
      pf[hh][0] = pack_p(sc[hh][0], sc[hh][1]);
      pf[hh][1] = pack_p(sc[hh][2], sc[hh][3]);
    }
    // (an unconditional multiply -- alpha = 1 exactly unless the max moved -- measured
    // slower: 312 vs 297 us per layer, profiles/r04/v6_*; the exponent arguments and row sums
    // as v_pk_fma_f32 / v_pk_add_f32 pairs, 45 fewer VALU per tile: 276.9 vs 271.5 us, v20_*)
    if (__ballot(rescale) != 0) {
#pragma unroll
      for (int hh = 0; hh < GB; ++hh)
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[hh][dt] *= alpha[hh];
    }
#pragma unroll
    for (int kstep = 0; kstep < 2; ++kstep)
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const f16x8 vt = load_vt(vs_, dt, kstep, lane);
#pragma unroll
        for (int hh = 0; hh < GB; ++hh) o[hh][dt] = mfma16(vt, pf[hh][kstep], o[hh][dt]);
      }
  }
  // O / l through LDS, then stored as whole rows: a query's GB heads are one contiguous
  // GB * 256-B run of its output row, written by consecutive lanes in 16-B pieces (per-lane 8-B
  // stores at the row stride touched 16 rows per instruction).  Row stride GB * 256 + 16 B: the
  // 16 rows of a ds_write_b64 land on distinct banks.
  constexpr int OS = GB * 256 + 16;
  __syncthreads();  // every wave is past its last tile: the tile buffers and the Q image are free
  // lane indices recomputed here (v_mbcnt) rather than kept live across the tile loop, which
  // holds all 256 registers
  const int ln = __lane_id(), tid_e = wave_u * 64 + ln, row_e = wave_u * 16 + (ln & 15), g_e = ln >> 4;
  if (wave_live) {
#pragma unroll
    for (int hh = 0; hh < GB; ++hh) {
      const float inv = 1.0f / l_run[hh];  // rows past the sequence (l = 0) are never stored
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        uint2 w;
        w.x = pack2h(o[hh][dt][0] * inv, o[hh][dt][1] * inv);
        w.y = pack2h(o[hh][dt][2] * inv, o[hh][dt][3] * inv);
        *(uint2*)(smem + row_e * OS + hh * 256 + dt * 32 + 8 * g_e) = w;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = GB * 16;  // 16-B pieces per row
  const int rows = min(QR, qlen - qb * QR);
  f16_t* obase = out + (size_t)(qstart + qb * QR) * (Hq * kHeadDim) + h0 * kHeadDim;
  for (int c = tid_e; c < rows * CPR; c += 512) {
    const int row = c / CPR, col = c - row * CPR;
    *(uint4*)(obase + (size_t)row * (Hq * kHeadDim) + col * 8) = *(const uint4*)(smem + row * OS + col * 16);
  }
}

void launch_attn_prefill(const f16_t* qkv, f16_t* out, int Hq, int Hk, KVView kv,
                         PrefillAttnArgs a, hipStream_t s) {
  if (a.n_qblk <= 0) return;
  const float scale_log2 = kLog2e / sqrtf((float)kHeadDim);
  const int G = Hq / Hk;
  const int gb = (G % 3 == 0) ? 3 : (G % 2 == 0) ? 2 : 1;
  const dim3 grid(a.n_qblk * (Hq / gb));
#define AP(GB_) MS_LAUNCH(attn_prefill_kernel<GB_>, grid, dim3(512), 0, s, qkv, out, Hq, Hk, kv, a, scale_log2)
  if (gb == 3) AP(3);
  else if (gb == 2) AP(2);
  else AP(1);
#undef AP
}

// ============================================================ decode (split-K over keys)
// grid (B, Hk, nsplit); block 256 = 4 waves, each wave walking ppw 64-key pages (below) with
// a whole page (K as MFMA fragments + V rows, 32 KB) in flight before its first MFMA.  The G
// query heads of the kv head are MFMA columns 0..G-1.  Per-wave (m, l, O^T) are merged in LDS
// (reusing the waves' V images); each block writes one partial (m, l, o[128]) per (b, q head,
// split), and attn_decode_combine_kernel merges the nsplit partials into the fp16 output.
// With the deferred RMSNorm (kernels.h RowScale) the prologue also folds the row's norm
// statistics and scales q / k / v by r before rounding them.
//
// FROM_SLABS (the fused decode chain): the QKV projection arrives as S fp32 split-K slabs
// [S][B][(Hq+2Hk)*128] with Q/K rows rope-permuted (k_gemv.hip).  The prologue adds the
// slabs (slab order), rounds q/k/v to fp16, applies RoPE in fp32 and rounds again -- the
// arithmetic of rope_kv_kernel -- and the block that owns the new token's page writes its
// K/V into the cache (for later steps) and patches them into the page it holds in
// registers / LDS.  Otherwise q comes from fp16 qkv rows already roped (rope_kv_kernel).
constexpr int kSplitPages = 4;  // = waves per block
constexpr int kMaxGroup = 8;    // q heads per kv head
constexpr int kMaxSlabs = 8;    // QKV split-K slabs (engine kMaxSplit)

// Pages per wave (ppw) and splits per (sequence, kv head).  Every wave walks its pages with
// the next page's K and V in flight under the current page's math, so more pages per wave
// cost nothing but parallelism.  ppw is fixed per ENGINE from its max_batch and max_ctx
// (the split boundaries, at multiples of 4*ppw pages, set a sequence's summation order, so
// they must not move with the batch): ~2 blocks per CU in one round (512 blocks) at a full
// batch of max_ctx keys, at least 2 pages per wave.  B = 8 at 2304 keys -> ppw 2, 5 splits,
// 320 blocks; B = 128 -> ppw 16, 1 split, 1024 blocks: the per-block prologue (QKV slab
// fold, RoPE) and epilogue (merge, partial) are paid once per 36 pages instead of per 8.
// MS_ATTN_PPW pins ppw (tuning).
constexpr int kTargetBlocks = 512, kMaxPPW = 16;
static int decode_ppw_env() {
  static const int v = [] { const char* e = getenv("MS_ATTN_PPW"); return e ? atoi(e) : 0; }();
  return v;
}
int attn_decode_ppw(int max_batch, int Hk, int max_ctx) {
  const int np = (max_ctx + kPage - 1) / kPage;
  int ppw = decode_ppw_env();
  if (ppw <= 0) {
    const long want = ((long)np * max_batch * Hk + (long)kSplitPages * kTargetBlocks - 1) /
                      ((long)kSplitPages * kTargetBlocks);
    ppw = (int)std::max(2L, std::min((long)kMaxPPW, want));
  }
  return std::max(1, std::min(ppw, kMaxPPW));
}
static int decode_nsplit(int ppw, int max_len) {
  const int np = (max_len + kPage - 1) / kPage;
  return (np + kSplitPages * ppw - 1) / (kSplitPages * ppw);
}
// the most splits any B can get (ppw >= 1 under MS_ATTN_PPW, else >= 2)
static int decode_nsplit_max(int max_len) {
  const int np = (max_len + kPage - 1) / kPage;
  const int ppw_min = decode_ppw_env() > 0 ? 1 : 2;
  return (np + kSplitPages * ppw_min - 1) / (kSplitPages * ppw_min);
}

constexpr int kMaxSplits = 127;

// workspace: partials (b, q head, split) x 132 floats {m, l, o[128], pad}
size_t attn_decode_workspace_bytes(int B, int Hq, int max_len) {
  return (size_t)B * Hq * decode_nsplit_max(max_len) * 132 * sizeof(float);
}

bool attn_decode_supported(int B, int Hq, int Hk, int max_len) {
  (void)B;
  return Hk >= 1 && Hq % Hk == 0 && Hq / Hk <= kMaxGroup && decode_nsplit_max(max_len) <= kMaxSplits;
}

// PPWT = 2: the page loop unrolled for exactly 2 pages per wave (the B = 8 plan); 0: runtime
template <bool FROM_SLABS, int PPWT>
__global__ __launch_bounds__(256, 2) void attn_decode_kernel(DecodeQKV qa, int Hq, int Hk, KVView kv,
                                                          DecodeAttnArgs a, float* __restrict__ ws,
                                                          int nsplit, int ppw, float scale_log2) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 16384 + (kMaxGroup + 2) * kHeadDim * 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int b = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  const int G = Hq / Hk;
  const int len = a.seq_len[b];
  const int slot = a.seq_slot[b];
  const int row_stride = (Hq + 2 * Hk) * kHeadDim;
  char* vs_ = smem + wave * 16384;
  // this wave's pages: split*4*ppw + wave, +4, ... below pend (interleaved: waves stay balanced)
  const int pg0 = split * kSplitPages * ppw + wave;
  const int pend = min((split + 1) * kSplitPages * ppw, (len + kPage - 1) / kPage);
  const int pos = len - 1;               // the new token
  f16_t* qn = (f16_t*)(smem + 4 * 16384);  // [G][128] roped q
  f16_t* kn = qn + kMaxGroup * kHeadDim;     // [128] roped k of the new token
  f16_t* vn = kn + kHeadDim;                 // [128] v of the new token
  const int32_t* bt = kv.block_table + (size_t)slot * kv.max_pages;
  constexpr int NWB = kSplitPages;  // waves per block: a wave's pages are NWB apart

  // K fragments (16 rows x 64 B per instruction) and V rows (1 KB) of one page, by physical
  // page id
  u32x4 kf[4][4], vr[16];
  auto fetch_k = [&](int pid) {
    const size_t base = ((size_t)pid * kv.n_kv_heads + kvh) * kPage * kHeadDim;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        kf[mt][s4] = ld_stream(kv.k + base + (mt * 16 + r) * kHeadDim + 32 * s4 + 8 * g);
  };
  auto fetch_v = [&](int pid) {
    const size_t base = ((size_t)pid * kv.n_kv_heads + kvh) * kPage * kHeadDim;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      vr[i] = ld_stream(kv.v + base + (i * 4 + (lane >> 4)) * kHeadDim + (lane & 15) * 8);
  };
  // the block-table entries of the unrolled plan's two pages load together, before any
  // page: the second page's prefetch (issued under the first page's math) then needs no
  // table round trip of its own (vmcnt retires in order: a table load issued there would
  // also wait for everything before it)
  // (a slot-major pool needs no table at all)
  auto page_id = [&](int pg) { return kv.slot_major ? slot * kv.max_pages + pg : bt[pg]; };
  int pid_next = 0;
  if constexpr (PPWT == 2) pid_next = pg0 + NWB < pend ? page_id(pg0 + NWB) : 0;
  // the row's deferred-norm partial sums (every wave folds them itself: no extra barrier),
  // lane l holding tiles l + 64 i in order -- gemv_common.h rs_finish's summation order; loaded
  // before the pages, so the fold waits on no page (vmcnt retires in order)
  float rv[4] = {0.f, 0.f, 0.f, 0.f};
  if (FROM_SLABS && qa.rs.ssq) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = lane + 64 * i;
      rv[i] = t < qa.rs.tiles ? qa.rs.ssq[(size_t)t * a.B + b] : 0.f;
    }
  }
  // issue the first page first, so its HBM latency overlaps the q/k/v prologue
  if (pg0 < pend) {
    const int pid0 = page_id(pg0);
    fetch_k(pid0);
    fetch_v(pid0);
  }

  if constexpr (FROM_SLABS) {
    const bool owns_new = (pos / kPage) / (kSplitPages * ppw) == split;  // block-uniform
    float* raw = (float*)smem;  // [(G+2)][128] fp16-rounded sums; aliases wave 0's V image
    const size_t sstride = (size_t)a.B * row_stride;
    const float* src = qa.slabs + (size_t)b * row_stride;
    const float rcs = qa.cos_tab[(size_t)pos * 64 + (tid & 63)];  // this thread's rope pair i
    const float rsn = qa.sin_tab[(size_t)pos * 64 + (tid & 63)];
    const int nvec = (G + (owns_new ? 2 : 0)) * kHeadDim;
    constexpr int PER = ((kMaxGroup + 2) * kHeadDim + 255) / 256;
    float sv[PER][kMaxSlabs];  // every slab load of this thread in flight at once
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (i * 256 >= nvec) break;  // block-uniform
      const int e = min(tid + i * 256, nvec - 1);
      const int hh = e >> 7, j = e & 127;  // hh < G: q head kvh*G+hh; G: k; G+1: v
      const int col = hh < G ? (kvh * G + hh) * kHeadDim + j
                             : (hh == G ? (Hq + kvh) * kHeadDim + j : (Hq + Hk + kvh) * kHeadDim + j);
#pragma unroll
      for (int q = 0; q < kMaxSlabs; ++q) sv[i][q] = src[min(q, qa.S - 1) * sstride + col];
    }
    const float rrow = qa.rs.ssq ? rs_rinv(wave_sum(((rv[0] + rv[1]) + rv[2]) + rv[3]), qa.rs) : 1.0f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + i * 256;
      if (i * 256 >= nvec) break;
      float acc = sv[i][0];
#pragma unroll
      for (int q = 1; q < kMaxSlabs; ++q)
        if (q < qa.S) acc += sv[i][q];
      if (e < nvec) raw[e] = h2f(f2h(acc * rrow));
    }
    __syncthreads();
    const int nrot = (G + (owns_new ? 1 : 0)) * 64;  // (head, i) pairs: the q heads, then k
    for (int e = tid; e < nrot; e += 256) {
      const int hh = e >> 6, i = e & 63;  // i == tid & 63 for every e of this thread
      const float lo = raw[hh * kHeadDim + rope_perm(i)], hi = raw[hh * kHeadDim + rope_perm(64 + i)];
      const float cs = rcs, sn = rsn;
      const float ra = __fsub_rn(__fmul_rn(lo, cs), __fmul_rn(hi, sn));
      const float rb = __fadd_rn(__fmul_rn(hi, cs), __fmul_rn(lo, sn));
      f16_t* dst = hh < G ? qn + hh * kHeadDim : kn;
      dst[i] = f2h(ra);
      dst[64 + i] = f2h(rb);
    }
    if (owns_new && tid < kHeadDim) vn[tid] = f2h(raw[(G + 1) * kHeadDim + tid]);
    __syncthreads();  // raw consumed (wave 0 may stage V); qn/kn/vn ready
    if (owns_new && tid < kHeadDim) {  // the new token's K/V into the cache, for later steps
      const int page = page_id(pos / kPage);
      const size_t o = (((size_t)page * kv.n_kv_heads + kvh) * kPage + pos % kPage) * kHeadDim + tid;
      kv.k[o] = kn[tid];
      kv.v[o] = vn[tid];
    }
  }

  f32x4 o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  if (pg0 < pend) {
    f16x8 qf[4];
    {
      const int hl = min(r, G - 1);
      if constexpr (FROM_SLABS) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *(const f16x8*)(qn + hl * kHeadDim + 32 * s4 + 8 * g);
      } else {
        const f16_t* qrow = qa.qkv + (size_t)b * row_stride + (kvh * G + hl) * kHeadDim;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) qf[s4] = as_f16x8(*(const uint4*)(qrow + 32 * s4 + 8 * g));
      }
    }
    const int off = pos % kPage;
    constexpr int kUnrollPages = PPWT > 0 ? PPWT : 1;
#pragma unroll kUnrollPages
    for (int pp = 0; PPWT == 0 || pp < PPWT; ++pp) {
      const int pg = pg0 + pp * kSplitPages;
      if (pg >= pend) break;  // wave-uniform
      const bool more = pg + kSplitPages < pend;
      const bool patch = FROM_SLABS && pg == pos / kPage;  // wave-uniform: holds the new token
      if (patch) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            if (mt * 16 + r == off) kf[mt][s4] = *(const u32x4*)(kn + 32 * s4 + 8 * g);
      }
      f32x4 sc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) sc[mt] = mfma16(__builtin_bit_cast(f16x8, kf[mt][s4]), qf[s4], sc[mt]);
      }
      const int pid_n = PPWT == 2 ? pid_next : (more ? page_id(pg + kSplitPages) : 0);
      if (more) fetch_k(pid_n);  // K registers are free: next page's K in flight
      float mx = -INFINITY;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = pg * kPage + mt * 16 + 4 * g + j;
          const float v = (key >= len) ? -INFINITY : sc[mt][j] * scale_log2;
          sc[mt][j] = v;
          mx = fmaxf(mx, v);
        }
      mx = grp_max(mx);
      const float m_new = fmaxf(m_run, mx);  // finite: key pg*64 < len is always visible
      const float alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
      float rs = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = (sc[mt][j] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sc[mt][j] - m_new);
          sc[mt][j] = p;
          rs += p;
        }
      rs = grp_sum(rs);
      l_run = l_run * alpha + rs;
      m_run = m_new;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
      // V rows -> this wave's LDS image (rows past len zeroed: no stale V in P.V)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = i * 4 + (lane >> 4);
        if (pg * kPage + row >= len) vr[i] = u32x4{0, 0, 0, 0};
        if (patch && row == off) vr[i] = *(const u32x4*)(vn + (lane & 15) * 8);
        *(u32x4*)(vs_ + v_swz(row, lane & 15)) = vr[i];
      }
      if (more) fetch_v(pid_n);  // V registers are free: next page's V in flight
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the V image is in LDS
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int kstep = 0; kstep < 2; ++kstep) {
        const f16x8 pf = pack_p(sc[2 * kstep], sc[2 * kstep + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const f16x8 vt = load_vt(vs_, dt, kstep, lane);
          o[dt] = mfma16(vt, pf, o[dt]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
    }
  }
  // publish (m, l, O^T) of this wave's 16 columns into its own LDS region
  {
    float* mw = (float*)vs_;
    if (g == 0) { mw[r * 130 + 0] = m_run; mw[r * 130 + 1] = l_run; }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) mw[r * 130 + 2 + dt * 16 + 4 * g + j] = o[dt][j];
  }
  __syncthreads();
  // merged (m, l, O^T) of head c over the block's 4 waves: k = 0 -> m, 1 -> l, 2.. -> O[k - 2]
  auto merged = [&](int c, int k, float& M) {
    M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, ((const float*)(smem + w * 16384))[c * 130]);
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* mw = (const float*)(smem + w * 16384);
      const float m_w = mw[c * 130];
      const float f = (m_w == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_w - M);
      acc += (k == 0) ? 0.f : f * mw[c * 130 + k];
    }
    return acc;
  };
  for (int idx = tid; idx < G * 130; idx += 256) {
    const int c = idx / 130, k = idx % 130;
    float M;
    const float acc = merged(c, k, M);
    ws[(((size_t)b * Hq + kvh * G + c) * nsplit + split) * 132 + k] = (k == 0) ? M : acc;
  }
}

// split combine: out[b][hq*128 + d] = sum_s w_s o_s / sum_s w_s l_s, w_s = 2^(m_s - max m) --
// its own launch.  Merging in the attention kernel instead (the last split of each (b, kv head),
// told by an agent-scope ticket, sc1 partial stores) measured slower twice: 2.289 vs 2.294 ms per
// decode step with release / acquire fences (round 2), 2.24 vs 2.13 with write-through stores
// and one ticket per block (round 4, profiles/r04/v3_attn_fused_combine_rejected_ab.txt): every
// block's lifetime grows by the drain + ticket round trip.
// PRE: O values preloaded per thread (>= nsplit where it fits: no redundant loads).  GRP: a
// 1-D grid whose block L merges (b, kv head) group grp = L % (B * Hk), q head c = L / (B * Hk)
// of it -- so L % 8 == grp % 8, the XCD of that group's split blocks in launch_attn_decode2's
// grid (blockIdx = split * B * Hk + grp): the partials are read from the L2 they were written
// through (plain stores keep the line there; a kernel boundary writes back, it does not evict)
template <int PRE, bool GRP>
__global__ __launch_bounds__(128) void attn_decode_combine_kernel(const float* __restrict__ ws,
                                                                  f16_t* __restrict__ out, int Hq,
                                                                  int nsplit, int Hk, int B) {
  // one memory round trip: every (m_s, l_s) pair (wave 0, two splits per lane) and, for
  // nsplit <= PRE, every O value of this thread are loaded before the barrier (the O loads
  // do not depend on the split weights); sums keep the split order, so results are unchanged
  __shared__ float fw[128], lw[128];
  int b, hq;
  if constexpr (GRP) {
    const int BH = B * Hk, L = blockIdx.x;
    const int grp = L % BH, c = L / BH;
    b = grp / Hk;
    hq = (grp - b * Hk) * (Hq / Hk) + c;
  } else {
    b = blockIdx.x;
    hq = blockIdx.y;
  }
  const int d = threadIdx.x;
  const float* p = ws + ((size_t)b * Hq + hq) * nsplit * 132;
  const float* po = p + 2 + d;
  float ov[PRE];
#pragma unroll
  for (int q = 0; q < PRE; ++q) ov[q] = q < nsplit ? po[q * 132] : 0.f;
  if (d < 64) {
    const float m0 = d < nsplit ? p[d * 132] : -INFINITY;
    const float m1 = d + 64 < nsplit ? p[(d + 64) * 132] : -INFINITY;
    const float l0 = d < nsplit ? p[d * 132 + 1] : 0.f;
    const float l1 = d + 64 < nsplit ? p[(d + 64) * 132 + 1] : 0.f;
    float M = fmaxf(m0, m1);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o));
    fw[d] = m0 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m0 - M);
    fw[d + 64] = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - M);
    lw[d] = l0;
    lw[d + 64] = l1;
  }
  __syncthreads();
  float L = 0.f, O = 0.f;
#pragma unroll
  for (int q = 0; q < PRE; ++q) {
    if (q < nsplit) {
      L += fw[q] * lw[q];
      O += fw[q] * ov[q];
    }
  }
  for (int s = PRE; s < nsplit; ++s) {
    L += fw[s] * lw[s];
    O += fw[s] * po[s * 132];
  }
  out[(size_t)b * Hq * kHeadDim + hq * kHeadDim + d] = f2h(O / L);
}

// decode-attention tuning (MS_COMBINE_GRP / MS_A2_ORDER, or ms_set_attn_tuning): the combine's
// XCD-matched grid (placement only) and the v2 prologue form (3: the prologue wave); both give
// the same bits.  Read at launch: a captured decode graph keeps what it was captured with.
static int g_combine_grp = [] { const char* e = getenv("MS_COMBINE_GRP"); return e ? atoi(e) : 1; }();
void set_attn_tuning(int combine_grp, int order) {
  (void)order;  // the v2 prologue-wave form (order 3) was removed in round 6: one form remains
  g_combine_grp = combine_grp;
}
static bool combine_grp_ok(int B, int Hk) { return g_combine_grp != 0 && (B * Hk) % 8 == 0; }

// the combine launch: (B, Hq) grid, or with grp the 1-D XCD-matched grid of the v2 kernel
static void launch_combine(const float* ws, f16_t* out, int B, int Hq, int Hk, int nsplit, bool grp,
                           hipStream_t s) {
#define CB(P_)                                                                                          \
  do {                                                                                                  \
    if (grp)                                                                                            \
      MS_LAUNCH((attn_decode_combine_kernel<P_, true>), dim3(B * Hq), dim3(128), 0, s, ws, out, Hq,     \
                nsplit, Hk, B);                                                                         \
    else                                                                                                \
      MS_LAUNCH((attn_decode_combine_kernel<P_, false>), dim3(B, Hq), dim3(128), 0, s, ws, out, Hq,     \
                nsplit, Hk, B);                                                                         \
  } while (0)
  if (nsplit <= 4) CB(4);
  else if (nsplit <= 8) CB(8);
  else CB(16);
#undef CB
}

void launch_attn_decode(const DecodeQKV& qa, f16_t* out, int Hq, int Hk, KVView kv,
                        DecodeAttnArgs a, float* ws, hipStream_t s) {
  if (a.B <= 0) return;
  if (!attn_decode_supported(a.B, Hq, Hk, a.max_len)) return;  // callers check
  if (qa.slabs && (qa.S < 1 || qa.S > kMaxSlabs)) return;
  if (qa.slabs && qa.rs.ssq && (qa.rs.tiles < 1 || qa.rs.tiles > 256)) return;  // callers check
  const int ppw = a.ppw > 0 ? a.ppw : 2;
  const int nsplit = decode_nsplit(ppw, a.max_len);
  const float scale_log2 = kLog2e / sqrtf((float)kHeadDim);
  const dim3 grid(a.B, Hk, nsplit);
#define AD(SL)                                                                                              \
  do {                                                                                                      \
    if (ppw == 2)                                                                                           \
      MS_LAUNCH((attn_decode_kernel<SL, 2>), grid, dim3(256), 0, s, qa, Hq, Hk, kv, a, ws, nsplit, ppw,     \
                scale_log2);                                                                                \
    else                                                                                                    \
      MS_LAUNCH((attn_decode_kernel<SL, 0>), grid, dim3(256), 0, s, qa, Hq, Hk, kv, a, ws, nsplit, ppw,     \
                scale_log2);                                                                                \
  } while (0)
  if (qa.slabs) AD(true);
  else AD(false);
#undef AD
  launch_combine(ws, out, a.B, Hq, Hk, nsplit, false, s);
}

}  // namespace ms

namespace ms {

// ============================================================ decode, one page per wave (v2)
// For the small-batch regime (engines of <= 16 slots, the configs[1] bench at B = 8) the
// kernel above is latency-bound: each wave walks 2 pages and issues the second page only after
// the first has landed and been multiplied, and the block prologue (the QKV slab fold) waits
// for the first page (vmcnt retires in issue order).  Here every wave owns ONE page and issues
// it at once -- K into registers, V by LDS DMA straight into its V^T image (v_swz layout,
// applied on the DMA source) -- so a block's whole page range (ppb pages, 32 KB each) is in
// flight from its first microsecond and the chip requests all of a step's K/V in one burst.
// One block of ppb waves per (sequence, kv head, split) with ppb fixed per ENGINE (the split
// boundaries, multiples of ppb pages, set a sequence's summation order: batch invariance) and
// chosen so a full batch is ~one block per CU; the splits of one (sequence, kv head) share
// blockIdx % 8 (one XCD: their partials meet in one L2).  Waves merge (m, l, O^T) in LDS in
// wave order; the block writes the split's partial (attn_decode_combine_kernel merges them in
// split order) or, with a single split, the fp16 output itself.  Arithmetic per page is the
// kernel above's (same MFMA orientation, fp16 P, lazy-free online softmax per page).
constexpr int kPpbMin = 4, kPpbMax = 9;  // 9 x 16 KB V images + the prologue fit 160 KB of LDS

int attn_decode2_ppb(int max_batch, int Hk, int max_ctx) {
  const char* ev = getenv("MS_ATTN_PPB");  // read per engine (tests pin several values in one process)
  const int env = ev ? atoi(ev) : 0;
  if (env > 0) return std::max(kPpbMin, std::min(env, kPpbMax));
  const long np = (max_ctx + kPage - 1) / kPage;
  const long want = (np * max_batch * Hk + 255) / 256;  // ~one block per CU at a full batch
  return (int)std::max((long)kPpbMin, std::min((long)kPpbMax, want));
}

static size_t attn2_lds_bytes(int ppb, int G) {
  // + 16 B: the prologue wave's flag (PW)
  return (size_t)ppb * 16384 + (size_t)(G + 2) * kHeadDim * 4 + (size_t)(G + 2) * kHeadDim * 2 + 16;
}
bool attn_decode2_supported(int B, int Hq, int Hk, int max_len, int ppb) {
  (void)B;
  if (Hk < 1 || Hq % Hk || Hq / Hk > kMaxGroup || ppb < kPpbMin || ppb > kPpbMax) return false;
  const int np = (max_len + kPage - 1) / kPage;
  return (np + ppb - 1) / ppb <= kMaxSplits && attn2_lds_bytes(ppb, Hq / Hk) <= 160 * 1024;
}

size_t attn_decode2_workspace_bytes(int B, int Hq, int max_len, int ppb) {
  const int np = (max_len + kPage - 1) / kPage;
  return (size_t)B * Hq * ((np + ppb - 1) / ppb) * 132 * sizeof(float);
}

// TICKET: the splits of one (sequence, kv head) are merged inside the launch by the block that
// finishes last (an agent-scope arrival counter per group, cnt[B * Hk], zero between launches:
// the last arriver resets it), with attn_decode_combine_kernel's arithmetic in split order --
// the same bits as the second launch; the group's blocks share one XCD (blockIdx % 8), so the
// partials and the counter meet in one L2
// In-kernel timeline stamps (diagnostic, MS_A2_STAMPS=1, never in a timed run): per block of the
// latest launch, s_memrealtime (100 MHz) at [0] entry, [2] prologue done, [3 + w] wave w's S done
// (its K landed), [12 + w] its P.V done, [21] partial stored, [22] / [23] wave 0's / the last wave's
// prologue operands landed, [24] the last wave's entry, [25] / [26] the last wave's / wave 0's
// prologue loads issued; [1] = XCC_ID << 32 | HW_ID
// (tools/a2_stamps.py reads them through ms_debug_a2_stamps)
constexpr int kA2StampBlocks = 1024, kA2Stamps = 32;
__device__ unsigned long long g_a2_stamps[kA2StampBlocks * kA2Stamps];
#define A2_STAMP(k)                                                                               \
  do {                                                                                            \
    if (stamps && lane == 0 && blockIdx.x < kA2StampBlocks)                                       \
      stamps[blockIdx.x * kA2Stamps + (k)] = __builtin_amdgcn_s_memrealtime();                    \
  } while (0)

template <bool FROM_SLABS, int PPB, bool TICKET>
__global__ __launch_bounds__(64 * PPB) void attn_decode2_kernel(
    DecodeQKV qa, int Hq, int Hk, KVView kv, DecodeAttnArgs a, float* __restrict__ ws, f16_t* __restrict__ out,
    int nsplit, float scale_log2, unsigned* __restrict__ cnt, unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NTHR = 64 * PPB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int BH = a.B * Hk;
  const int split = blockIdx.x / BH, grp = blockIdx.x - split * BH;
  const int b = grp / Hk, kvh = grp - b * Hk;
  const int G = Hq / Hk;
  const int len = a.seq_len[b];
  const int slot = a.seq_slot[b];
  const int np = (len + kPage - 1) / kPage;
  const int pg = split * PPB + wave;  // this wave's page (none when >= np)
  const int pos = len - 1;            // the new token
  const int row_stride = (Hq + 2 * Hk) * kHeadDim;
  char* vs_ = smem + wave * 16384;
  float* raw = (float*)(smem + (size_t)PPB * 16384);  // [(G+2)][128] fp16-rounded sums
  f16_t* qn = (f16_t*)(raw + (G + 2) * kHeadDim);     // [G][128] roped q
  f16_t* kn = qn + G * kHeadDim;                       // [128] roped k of the new token
  f16_t* vn = kn + kHeadDim;                           // [128] v of the new token
  const bool has_page = pg < np;                       // wave-uniform
  if (wave == PPB - 1) A2_STAMP(24);
  if (stamps && wave == 0) {
    A2_STAMP(0);
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0 && blockIdx.x < kA2StampBlocks)
      stamps[blockIdx.x * kA2Stamps + 1] = ((unsigned long long)xcc << 32) | hw;
  }
  // slot-major pool (launch_attn_decode2 checks): page ids are arithmetic, no table load
  const size_t pbase = (((size_t)slot * kv.max_pages + pg) * kv.n_kv_heads + kvh) * kPage * kHeadDim;

  // 0. the prologue's operands: the row's deferred-norm partial sums, the QKV slab values and
  // this thread's rope pair (opaque loads, issued first)
  const bool owns_new = (pos / kPage) / PPB == split;  // block-uniform
  const int nvec = FROM_SLABS ? (G + (owns_new ? 2 : 0)) * kHeadDim : 0;
  constexpr int PER = ((kMaxGroup + 2) * kHeadDim + NTHR - 1) / NTHR;
  float rv[4] = {0.f, 0.f, 0.f, 0.f};
  float sv[PER][kMaxSlabs];
  float rcs = 0.f, rsn = 0.f;
  if constexpr (FROM_SLABS) {
    if (qa.rs.ssq) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = lane + 64 * i;
        if (64 * i < qa.rs.tiles) rv[i] = ld_f32_opaque(qa.rs.ssq + (size_t)min(t, qa.rs.tiles - 1) * a.B + b);
      }
    }
    const size_t sstride = (size_t)a.B * row_stride;
    const float* src = qa.slabs + (size_t)b * row_stride;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (i * NTHR < nvec) {  // block-uniform
        const int e = min(tid + i * NTHR, nvec - 1);
        const int hh = e >> 7, j = e & 127;  // hh < G: q head kvh*G+hh; G: k; G+1: v
        const int col = hh < G ? (kvh * G + hh) * kHeadDim + j
                               : (hh == G ? (Hq + kvh) * kHeadDim + j : (Hq + Hk + kvh) * kHeadDim + j);
#pragma unroll
        for (int q = 0; q < kMaxSlabs; ++q)
          if (q < qa.S) sv[i][q] = ld_f32_opaque(src + q * sstride + col);
      }
    }
    rcs = ld_f32_opaque(qa.cos_tab + (size_t)pos * 64 + (tid & 63));
    rsn = ld_f32_opaque(qa.sin_tab + (size_t)pos * 64 + (tid & 63));
    if (wave == 0) A2_STAMP(26);
    if (wave == PPB - 1) A2_STAMP(25);
  }
  // 1. this wave's page: V by LDS DMA into its V^T image (chunk c of row rr lands at
  // v_swz(rr, c): lane l of 1-KiB piece i covers row 4i + l / 16, LDS chunk l % 16, so it loads
  // the global chunk (l % 16) ^ ((row & 7) << 1)), then K into registers (16 rows x 64 B per
  // instruction, as the kernel above)
  u32x4 kf[4][4];
  if (has_page) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = 4 * i + (lane >> 4), ch = (lane & 15) ^ ((rr & 7) << 1);
      dma16_opaque(kv.v + pbase + rr * kHeadDim + ch * 8, vs_ + i * 1024);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        kf[mt][s4] = ld_stream(kv.k + pbase + (mt * 16 + r) * kHeadDim + 32 * s4 + 8 * g);
  }

  // 2. prologue: fold the slabs, the row scale, RoPE -> qn / kn / vn; the owner writes the new
  // token's K/V into the cache (rope_kv_kernel's arithmetic, as the kernel above)
  if constexpr (FROM_SLABS) {
    // the opaque loads above have landed once at most the page's 32 are in flight
    if (has_page) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave == 0) A2_STAMP(22);
    if (wave == PPB - 1) A2_STAMP(23);
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(rv[i]));
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
      for (int q = 0; q < kMaxSlabs; ++q) asm volatile("" : "+v"(sv[i][q]));
    asm volatile("" : "+v"(rcs), "+v"(rsn));
    float rsum = 0.f;
    if (qa.rs.ssq) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (!(lane + 64 * i < qa.rs.tiles)) rv[i] = 0.f;
      rsum = ((rv[0] + rv[1]) + rv[2]) + rv[3];
    }
    const float rrow = qa.rs.ssq ? rs_rinv(wave_sum(rsum), qa.rs) : 1.0f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + i * NTHR;
      if (i * NTHR >= nvec) break;
      float acc = sv[i][0];
#pragma unroll
      for (int q = 1; q < kMaxSlabs; ++q)
        if (q < qa.S) acc += sv[i][q];
      if (e < nvec) raw[e] = h2f(f2h(acc * rrow));
    }
    attn2_lds_sync();
    const int nrot = (G + (owns_new ? 1 : 0)) * 64;  // (head, i) pairs: the q heads, then k
    for (int e = tid; e < nrot; e += NTHR) {
      const int hh = e >> 6, i = e & 63;  // i == tid & 63 (NTHR % 64 == 0)
      const float lo = raw[hh * kHeadDim + rope_perm(i)], hi = raw[hh * kHeadDim + rope_perm(64 + i)];
      const float ra = __fsub_rn(__fmul_rn(lo, rcs), __fmul_rn(hi, rsn));
      const float rb = __fadd_rn(__fmul_rn(hi, rcs), __fmul_rn(lo, rsn));
      f16_t* dst = hh < G ? qn + hh * kHeadDim : kn;
      dst[i] = f2h(ra);
      dst[64 + i] = f2h(rb);
    }
    if (owns_new && tid < kHeadDim) vn[tid] = f2h(raw[(G + 1) * kHeadDim + tid]);
    attn2_lds_sync();
    if (owns_new && tid < kHeadDim) {
      const size_t o = ((((size_t)slot * kv.max_pages + pos / kPage) * kv.n_kv_heads + kvh) * kPage + pos % kPage) *
                           kHeadDim + tid;
      kv.k[o] = kn[tid];
      kv.v[o] = vn[tid];
    }
  }
  if (wave == 0) A2_STAMP(2);

  // 3. S^T = K Q^T, softmax over the page, O^T = V^T P^T
  f32x4 o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  if (has_page) {
    f16x8 qf[4];
    const int hl = min(r, G - 1);
    if constexpr (FROM_SLABS) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *(const f16x8*)(qn + hl * kHeadDim + 32 * s4 + 8 * g);
    } else {
      const f16_t* qrow = qa.qkv + (size_t)b * row_stride + (kvh * G + hl) * kHeadDim;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) qf[s4] = as_f16x8(*(const uint4*)(qrow + 32 * s4 + 8 * g));
    }
    const int off = pos % kPage;
    const bool patch = FROM_SLABS && pg == pos / kPage;  // wave-uniform: holds the new token
    if (patch) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          if (mt * 16 + r == off) kf[mt][s4] = *(const u32x4*)(kn + 32 * s4 + 8 * g);
    }
    f32x4 sc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) sc[mt] = mfma16(__builtin_bit_cast(f16x8, kf[mt][s4]), qf[s4], sc[mt]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = pg * kPage + mt * 16 + 4 * g + j;
        const float v = (key >= len) ? -INFINITY : sc[mt][j] * scale_log2;
        sc[mt][j] = v;
        mx = fmaxf(mx, v);
      }
    mx = grp_max(mx);  // finite: key pg*64 < len is always visible
    A2_STAMP(3 + wave);
    float rs = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = (sc[mt][j] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sc[mt][j] - mx);
        sc[mt][j] = p;
        rs += p;
      }
    l_run = grp_sum(rs);
    m_run = mx;
    // the V image has landed (its DMA was issued before the K loads the S MFMAs waited for)
    wait_vmcnt0();
    // rows past the sequence (last page) zeroed -- no stale V in P.V -- and the new token's row
    if (pg == np - 1) {
      const int first = len - pg * kPage;  // rows [first, 64) are past the sequence
      for (int e = first * 16 + lane; e < 64 * 16; e += 64)
        *(u32x4*)(vs_ + v_swz(e >> 4, e & 15)) = u32x4{0, 0, 0, 0};
    }
    if (patch && lane < 16) *(u32x4*)(vs_ + v_swz(off, lane)) = *(const u32x4*)(vn + lane * 8);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the patched rows are in LDS
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kstep = 0; kstep < 2; ++kstep) {
      const f16x8 pf = pack_p(sc[2 * kstep], sc[2 * kstep + 1]);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const f16x8 vt = load_vt(vs_, dt, kstep, lane);
        o[dt] = mfma16(vt, pf, o[dt]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    A2_STAMP(12 + wave);
  }
  // 4. publish (m, l, O^T) of this wave's 16 columns into its own LDS region, merge in wave order
  {
    float* mw = (float*)vs_;
    if (g == 0) { mw[r * 130 + 0] = m_run; mw[r * 130 + 1] = l_run; }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) mw[r * 130 + 2 + dt * 16 + 4 * g + j] = o[dt][j];
  }
  __syncthreads();
  for (int idx = tid; idx < G * 130; idx += NTHR) {
    const int c = idx / 130, k = idx - c * 130;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < PPB; ++w) M = fmaxf(M, ((const float*)(smem + w * 16384))[c * 130]);
    float acc = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < PPB; ++w) {
      const float* mw = (const float*)(smem + w * 16384);
      const float m_w = mw[c * 130];
      const float f = (m_w == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_w - M);
      acc += (k == 0) ? 0.f : f * mw[c * 130 + k];
      L += f * mw[c * 130 + 1];
    }
    if (nsplit == 1) {
      // a single split: O / L straight to the output (the combine's arithmetic with one
      // partial, whose weight 2^(M - M) is 1)
      if (k >= 2) out[(size_t)b * Hq * kHeadDim + (kvh * G + c) * kHeadDim + (k - 2)] = f2h(acc / L);
    } else if constexpr (TICKET) {
      // write-through (sc1) partial stores: the hand-off needs no release fence (an agent-scope
      // fence writes back and invalidates the L2 -- 64 us per launch, measured)
      __hip_atomic_store(ws + (((size_t)b * Hq + kvh * G + c) * nsplit + split) * 132 + k, (k == 0) ? M : acc,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      ws[(((size_t)b * Hq + kvh * G + c) * nsplit + split) * 132 + k] = (k == 0) ? M : acc;
    }
  }
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave == 0) A2_STAMP(21);
  }
  if constexpr (TICKET) {
    if (nsplit == 1) return;
    __shared__ unsigned last_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial stores are done
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(cnt + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = old == (unsigned)(nsplit - 1);
    }
    __syncthreads();
    if (!last_s) return;
    // the last block of the group: every split's partial, by sc1 loads (no stale cached copy),
    // merged as attn_decode_combine_kernel does (same order, same bits)
    auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int idx = tid; idx < G * kHeadDim; idx += NTHR) {
      const int c = idx >> 7, d = idx & 127;
      const float* p = ws + ((size_t)b * Hq + kvh * G + c) * nsplit * 132;
      float M = -INFINITY;
      for (int q = 0; q < nsplit; ++q) M = fmaxf(M, ld(p + q * 132));
      float L = 0.f, O = 0.f;
      for (int q = 0; q < nsplit; ++q) {
        const float m_q = ld(p + q * 132);
        const float f = m_q == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_q - M);
        L += f * ld(p + q * 132 + 1);
        O += f * ld(p + q * 132 + 2 + d);
      }
      out[(size_t)b * Hq * kHeadDim + (kvh * G + c) * kHeadDim + d] = f2h(O / L);
    }
    if (tid == 0) __hip_atomic_store(cnt + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

void launch_attn_decode2(const DecodeQKV& qa, f16_t* out, int Hq, int Hk, KVView kv, DecodeAttnArgs a,
                         float* ws, int ppb, hipStream_t s, unsigned* cnt) {
  if (a.B <= 0) return;
  if (!attn_decode2_supported(a.B, Hq, Hk, a.max_len, ppb) || !kv.slot_major) return;  // callers check
  if (qa.slabs && (qa.S < 1 || qa.S > kMaxSlabs)) return;
  if (qa.slabs && qa.rs.ssq && (qa.rs.tiles < 1 || qa.rs.tiles > 256)) return;
  const int np = (a.max_len + kPage - 1) / kPage;
  const int nsplit = (np + ppb - 1) / ppb;
  const float scale_log2 = kLog2e / sqrtf((float)kHeadDim);
  const dim3 grid(a.B * Hk * nsplit);
  const size_t lds = attn2_lds_bytes(ppb, Hq / Hk);
  static unsigned long long* stamps = [] {
    const char* e = getenv("MS_A2_STAMPS");
    void* p = nullptr;
    if (e && atoi(e)) (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_a2_stamps));
    return (unsigned long long*)p;
  }();
#define A2(P_)                                                                                                \
  case P_:                                                                                                    \
    if (qa.slabs && cnt)                                                                                      \
      MS_LAUNCH((attn_decode2_kernel<true, P_, true>), grid, dim3(64 * P_), lds, s, qa, Hq, Hk, kv, a, ws,    \
                out, nsplit, scale_log2, cnt, stamps);                                                        \
    else if (qa.slabs)                                                                                        \
      MS_LAUNCH((attn_decode2_kernel<true, P_, false>), grid, dim3(64 * P_), lds, s, qa, Hq, Hk, kv, a, ws,   \
                out, nsplit, scale_log2, cnt, stamps);                                                        \
    else                                                                                                      \
      MS_LAUNCH((attn_decode2_kernel<false, P_, false>), grid, dim3(64 * P_), lds, s, qa, Hq, Hk, kv, a, ws,  \
                out, nsplit, scale_log2, cnt, stamps);                                                        \
    break;
  switch (ppb) {
    A2(4) A2(5) A2(6) A2(7) A2(8) A2(9)
    default: return;
  }
#undef A2
  if (nsplit > 1 && !(qa.slabs && cnt)) launch_combine(ws, out, a.B, Hq, Hk, nsplit, combine_grp_ok(a.B, Hk), s);
}

}  // namespace ms

namespace ms {
// the split combine as its own launch (the fused QKV + attention kernel writes the same partials)
void attn2_stamps(unsigned long long* host, int n) {
  n = std::min(n, kA2StampBlocks * kA2Stamps);
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_a2_stamps), (size_t)n * sizeof(unsigned long long));
}

void launch_attn_combine(const float* ws, f16_t* out, int B, int Hq, int Hk, int nsplit, hipStream_t s) {
  if (B <= 0 || nsplit <= 1) return;
  launch_combine(ws, out, B, Hq, Hk, nsplit, combine_grp_ok(B, Hk), s);
}
}  // namespace ms
