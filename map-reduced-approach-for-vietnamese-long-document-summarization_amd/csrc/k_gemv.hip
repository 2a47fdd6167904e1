// k_gemv.hip -- decode projections of the map call: weight-streaming skinny GEMM.
//
// Replaces ggml mul_mat at decode time: every decode step
// multiplies the B <= 64 in-flight sequences' rows by every weight matrix once, so the
// step is HBM-bound on the 6.4 GB of fp16 weights.  Design for that:
//  * one block per 16*NT weight rows, the whole K range split over the block's waves
//    (reduced through LDS) -- no cross-block split-K, so no fences or tickets;
//  * every wave issues the loads of its whole K slice (U steps of 64) before its
//    first MFMA: W straight HBM -> VGPR (no LDS round trip, cdna_hip_programming.md
//    §5 'GEMV / M <= 16'), 32 contiguous bytes per lane per step, so a wave-instruction
//    pair covers 16 full 128-B lines; X (tiny, L2-resident) is staged once per block
//    into LDS (row stride 2K+16 B: conflict-free fragment reads) while W is in flight;
//  * v_mfma_f32_16x16x32_f16 with the sequences as MFMA rows (M padded to 16*MT);
//    both operands use the same permuted k order (lane group g holds k0+16g..+15),
//    which leaves every dot product unchanged.
// Fusions that remove whole launches from the decode step:
//  * the deferred RMSNorm (kernels.h RowScale): X is already f16(x * g), written by the
//    producer of x (RESID_SSQ epilogue or a norm kernel) with per-tile sums of x^2; the block
//    loads its rows' partial sums ahead of everything else and scales its output rows by
//    rinv in the epilogue -- no norm launch between the residual update and the projection
//    (recomputing the norm from the fp32 residual in each block measured slower: every block
//    re-read x before its weight stream, GU 19 -> 27 us, profiles/r03/v1_norm_fused_ab.txt);
//  * EPI_ROPE_KV (QKV): Q/K rows are uploaded rope-permuted (dims i and i+64 in one
//    16-row tile), so the epilogue applies RoPE, writes Q for attention and scatters
//    K/V into the paged cache;
//  * fp16 store, fp32 residual add (O, down), SwiGLU on 16-row-interleaved gate/up,
//    fp32 store (lm_head logits).
// Results are deterministic and independent of the batch composition: a row's sum
// order depends only on (N, K), never on M or on the other rows.
#include "gemv_common.h"

namespace ms {

struct GemvPlan {
  int MT, NT, waves, U, tiles;
};

static GemvPlan gemv_plan(int M, int N, int K, int epi, int force_waves = 0, int rt = 0) {
  GemvPlan p;
  p.MT = (M + 15) / 16;
  p.NT = (epi == MS_GEMV_EPI_SWIGLU) ? 2 : 1;
  const int rows = p.NT == 1 && rt > 0 ? rt : 16 * p.NT;
  p.tiles = (N + rows - 1) / rows;
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

constexpr size_t kMaxLds = 160 * 1024;

// LDS: the X image (gemv_x_lds_bytes, when staged) or the per-wave partials, whichever is
// larger, then the deferred-norm factors (gemv_lds_total)
static size_t gemv_lds_main(const GemvPlan& p, int M, int K, bool xlds) {
  size_t xs = xlds ? gemv_x_lds_bytes(M, K) : 0;
  const size_t red = (size_t)p.waves * p.MT * p.NT * 256 * 4;  // per-wave partials
  return xs > red ? xs : red;
}
static size_t gemv_lds_bytes(const GemvPlan& p, int M, int K, bool xlds, const RowScale& rs = RowScale{}) {
  return gemv_lds_total(gemv_lds_main(p, M, K, xlds), rs, M);
}

// Split-K (gridDim.y = S > 1, STORE_F32 only): block (x, y) covers k in [y*K, (y+1)*K) of
// rows of length ldk and writes its fp32 partial to slab y = out + y*M*ldo; the consumer
// (residual_rmsnorm_kernel) adds the S slabs in slab order -- deterministic, no atomics.
// XM = where the MFMA's X fragments come from:
//   kXGlobal: global loads inside the MFMA loop (large M*K: no room in LDS or registers);
//   kXLds:    the block's LDS image, copied by DMA ahead of the weight stream (gemv_dma_x);
//   kXRegs:   each wave loads its OWN k-slice of X (the only part it multiplies) straight
//             into registers ahead of its weight loads -- no LDS image, no block barrier,
//             every wave starts its MFMAs as soon as its own bytes have landed.
// rinv_off: LDS byte offset of the deferred-norm factors (gemv_rinv_offset).  (Two
// 1024-thread gate/up blocks share a CU at <= 64 VGPRs: 58 / 60 without / with the row scale.)
template <int MT, int NT, int EPI, int U, int XM, bool RS>
__global__ __launch_bounds__(1024) void gemv_kernel(const f16_t* __restrict__ X,
                                                    const f16_t* __restrict__ W,
                                                    void* __restrict__ out, int M, int N, int K,
                                                    int ldk, int ldo, int rinv_off, GemvArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  // NT = 1: ga.rt weight rows per tile (lanes fr >= rt duplicate the last row; never stored)
  const int rt = NT == 1 && ga.rt > 0 ? ga.rt : 16;
  const int n0 = blockIdx.x * (NT == 1 ? rt : 16 * NT);
  const int kbeg = wave * U * 64;
  if constexpr (EPI == MS_GEMV_EPI_STORE_F32) {
    X += (size_t)blockIdx.y * K;
    W += (size_t)blockIdx.y * K;
    out = (float*)out + (size_t)blockIdx.y * (ga.slab_rows > 0 ? ga.slab_rows : M) * ldo;
  }

  // 0. the output rows' deferred-norm partial sums, 1. X (LDS DMA of the block's rows or this
  // wave's slice into registers), then this wave's whole W stream: vmcnt retires in issue order
  // (row statistics always staged here: gemv_common.h rs_begin HOLD)
  constexpr bool kRsEarly = XM == kXLds && NT == 1;  // folds right after the X barrier
  if constexpr (RS) rs_begin<false>(smem, rinv_off, ga.rs, M);
  const ResidPre pre = resid_prefetch<EPI>(M, N, ldo, out, n0, ga);
  if constexpr (XM == kXLds) gemv_dma_x(smem, X, M, K, ldk);
  uint4 xr[XM == kXRegs ? U : 1][XM == kXRegs ? MT : 1][2];
  if constexpr (XM == kXRegs) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const f16_t* xg = X + (size_t)min(m * 16 + fr, M - 1) * ldk + kbeg + u * 64 + 16 * fg;
        xr[u][m][0] = ldg16(xg);
        xr[u][m][1] = ldg16(xg + 8);
      }
  }
  __builtin_amdgcn_sched_barrier(0);
  uint4 w[U][NT][2];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int wrow = NT == 1 ? n0 + min(fr, rt - 1) : n0 + n * 16 + fr;
    const f16_t* wp = W + (size_t)min(wrow, N - 1) * ldk + kbeg + 16 * fg;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      w[u][n][0] = ldw16(wp + u * 64);
      w[u][n][1] = ldw16(wp + u * 64 + 8);
    }
  }
  // 2. the X image (and the staged row statistics, issued before it) has landed once at most
  // the W loads are pending; the row factors are folded now, under the weight stream
  if constexpr (XM == kXLds) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(U * NT * 2));
    __builtin_amdgcn_s_barrier();  // no fence: a fence would wait for the W loads too
    // (two-tile plans fold them at the end: their 6 weight stages fill the 64 VGPRs)
    if constexpr (RS && NT == 1) rs_finish<false>(smem, rinv_off, ga.rs, M, 0.f);
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
      f16x8 x0, x1;
      if constexpr (XM == kXRegs) {
        x0 = as_f16x8(xr[u][m][0]);
        x1 = as_f16x8(xr[u][m][1]);
      } else if constexpr (XM == kXLds) {
        const int k0 = kbeg + u * 64 + 16 * fg;
        x0 = *(const f16x8*)(smem + x_lds(xrow, k0, K));
        x1 = *(const f16x8*)(smem + x_lds(xrow, k0 + 8, K));
      } else {
        const f16_t* xg = X + (size_t)xrow * ldk + kbeg + u * 64 + 16 * fg;
        x0 = as_f16x8(ldg16(xg));
        x1 = as_f16x8(ldg16(xg + 8));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        acc[m][n] = mfma16(x0, as_f16x8(w[u][n][0]), acc[m][n]);
        acc[m][n] = mfma16(x1, as_f16x8(w[u][n][1]), acc[m][n]);
      }
    }
  }
  gemv_finish<MT, NT, EPI, RS, kRsEarly, false>(acc, smem, rinv_off, M, N, ldo, out, n0, ga, pre);
}

template <int MT, int NT, int EPI, int U, bool RS>
static void gemv_go_rs(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                       const dim3& grid, const dim3& blk, size_t lds, int ro, int ldo, int xm,
                       const GemvArgs& ga, hipStream_t s) {
  if constexpr (MT * U <= kXRegsMaxFrags) {
    if (xm == kXRegs) {
      MS_LAUNCH((gemv_kernel<MT, NT, EPI, U, kXRegs, RS>), grid, blk, lds, s, X, W, out, M, N, K, ldk,
                ldo, ro, ga);
      return;
    }
  }
  if (xm == kXLds)
    MS_LAUNCH((gemv_kernel<MT, NT, EPI, U, kXLds, RS>), grid, blk, lds, s, X, W, out, M, N, K, ldk,
              ldo, ro, ga);
  else
    MS_LAUNCH((gemv_kernel<MT, NT, EPI, U, kXGlobal, RS>), grid, blk, lds, s, X, W, out, M, N, K, ldk,
              ldo, ro, ga);
}

template <int MT, int NT, int EPI, int U>
static void gemv_go(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                    int S, int ldo, const GemvPlan& p, size_t lds, int xm, const GemvArgs& ga,
                    hipStream_t s) {
  const dim3 grid(p.tiles, S), blk(64 * p.waves);
  const int ro = (int)gemv_rinv_offset(gemv_lds_main(p, M, K, xm == kXLds));
  if constexpr (EPI == MS_GEMV_EPI_ROPE_KV && MT != 1) {
    return;  // rope epilogue works on M <= 16 (checked by gemv_supported)
  } else if constexpr (gemv_rs_epi<EPI>()) {
    if (ga.rs.ssq) gemv_go_rs<MT, NT, EPI, U, true>(X, W, out, M, N, K, ldk, grid, blk, lds, ro, ldo, xm, ga, s);
    else gemv_go_rs<MT, NT, EPI, U, false>(X, W, out, M, N, K, ldk, grid, blk, lds, ro, ldo, xm, ga, s);
  } else {
    gemv_go_rs<MT, NT, EPI, U, false>(X, W, out, M, N, K, ldk, grid, blk, lds, ro, ldo, xm, ga, s);
  }
}

template <int MT, int NT, int EPI>
static void gemv_go_u(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                      int S, int ldo, const GemvPlan& p, size_t lds, int xm, const GemvArgs& ga,
                      hipStream_t s) {
#define GU(U_) gemv_go<MT, NT, EPI, U_>(X, W, out, M, N, K, ldk, S, ldo, p, lds, xm, ga, s)
  switch (p.U) {
    case 1: GU(1); break;
    case 2: GU(2); break;
    case 3: GU(3); break;
    case 4: GU(4); break;
    case 5: GU(5); break;
    case 6: GU(6); break;
    case 7: GU(7); break;
    default: GU(8); break;
  }
#undef GU
}

template <int MT>
static void gemv_go_mt(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                       int S, int ldo, int epi, const GemvPlan& p, size_t lds, int xm,
                       const GemvArgs& ga, hipStream_t s) {
#define GE(NT_, E_) gemv_go_u<MT, NT_, E_>(X, W, out, M, N, K, ldk, S, ldo, p, lds, xm, ga, s)
  switch (epi) {
    case MS_GEMV_EPI_STORE_F16: GE(1, MS_GEMV_EPI_STORE_F16); break;
    case MS_GEMV_EPI_ADD_F32: GE(1, MS_GEMV_EPI_ADD_F32); break;
    case MS_GEMV_EPI_SWIGLU: GE(2, MS_GEMV_EPI_SWIGLU); break;
    case MS_GEMV_EPI_ROPE_KV: GE(1, MS_GEMV_EPI_ROPE_KV); break;
    case MS_GEMV_EPI_ARGMAX: GE(1, MS_GEMV_EPI_ARGMAX); break;
    case MS_GEMV_EPI_RESID_SSQ: GE(1, MS_GEMV_EPI_RESID_SSQ); break;
    default: GE(1, MS_GEMV_EPI_STORE_F32); break;
  }
#undef GE
}

bool gemv_supported(int M, int N, int K, int epi, int rs_tiles) {
  if (M < 1 || M > 64 || K % 64) return false;
  if (epi == MS_GEMV_EPI_ROPE_KV && M > 16) return false;
  if (epi == MS_GEMV_EPI_ARGMAX && N % 16) return false;
  const GemvPlan p = gemv_plan(M, N, K, epi);
  if (p.waves == 0) return false;
  // the residual epilogue's prefetch covers one element per thread of a >= 256-thread block
  if (epi == MS_GEMV_EPI_RESID_SSQ && p.waves < 4) return false;
  if (epi == MS_GEMV_EPI_ROPE_KV && gemv_lds_bytes(p, M, K, true) > kMaxLds) return false;
  RowScale rs{};
  const bool takes_rs = epi != MS_GEMV_EPI_ARGMAX && epi != MS_GEMV_EPI_ADD_F32 && epi != MS_GEMV_EPI_RESID_SSQ;
  if (rs_tiles > 0 && takes_rs) {  // gemv_dispatch drops the scale for the other epilogues
    if (!gemv_rs_supported(M, rs_tiles)) return false;
    rs = make_row_scale(reinterpret_cast<const float*>(16), rs_tiles, 1, 0.f);
  }
  return gemv_lds_bytes(p, M, K, false, rs) <= kMaxLds;
}

static void gemv_dispatch(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                          int S, int ldo, int epi, const GemvArgs* ga_in, int force_waves,
                          hipStream_t s) {
  if (M <= 0) return;
  const int rt = ga_in ? ga_in->rt : 0;
  const GemvPlan p = gemv_plan(M, N, K, epi, force_waves, rt);
  if (p.waves == 0) return;  // callers check gemv_supported()
  GemvArgs ga{};
  if (ga_in) ga = *ga_in;
  if (epi == MS_GEMV_EPI_ARGMAX || epi == MS_GEMV_EPI_ADD_F32 || epi == MS_GEMV_EPI_RESID_SSQ)
    ga.rs = RowScale{};  // argmax: r > 0 keeps every row's order; the others take unnormalised X
  // the X image only when the block's whole LDS (image + factors + staged statistics) fits
  const bool xl = gemv_lds_bytes(p, M, K, true, ga.rs) <= kMaxLds;
  int xm = xl ? kXLds : kXGlobal;
  if (gemv_x_regs_for(epi) && p.MT * p.U <= kXRegsMaxFrags) xm = kXRegs;
  if (ga.rs.ssq && rs_stage_floats(ga.rs, M) == 0) return;  // callers check gemv_rs_supported
  const size_t lds = gemv_lds_bytes(p, M, K, xm == kXLds, ga.rs);
  if (lds > kMaxLds) return;
  switch (p.MT) {
    case 1: gemv_go_mt<1>(X, W, out, M, N, K, ldk, S, ldo, epi, p, lds, xm, ga, s); break;
    case 2: gemv_go_mt<2>(X, W, out, M, N, K, ldk, S, ldo, epi, p, lds, xm, ga, s); break;
    case 3: gemv_go_mt<3>(X, W, out, M, N, K, ldk, S, ldo, epi, p, lds, xm, ga, s); break;
    default: gemv_go_mt<4>(X, W, out, M, N, K, ldk, S, ldo, epi, p, lds, xm, ga, s); break;
  }
}

void launch_gemv_ex(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldo,
                    int epi, const GemvArgs* ga_in, int force_waves, hipStream_t s) {
  gemv_dispatch(X, W, out, M, N, K, K, 1, ldo, epi, ga_in, force_waves, s);
}

// tuning hook: W rows of stride ldk >= K elements (padded layouts: HBM channel spread)
void launch_gemv_strided(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                         int ldo, int epi, hipStream_t s) {
  gemv_dispatch(X, W, out, M, N, K, ldk, 1, ldo, epi, nullptr, 0, s);
}

bool gemv_rs_supported(int M, int tiles) { return M >= 1 && tiles >= 1 && tiles * M <= kRsStage; }

bool gemv_split_supported(int M, int N, int K, int S, int rs_tiles) {
  if (S < 1 || K % S) return false;
  return gemv_supported(M, N, K / S, MS_GEMV_EPI_STORE_F32, rs_tiles);
}

void launch_gemv_split(const f16_t* X, const f16_t* W, float* slabs, int M, int N, int K, int S,
                       int force_waves, hipStream_t s, const GemvArgs* ga) {
  gemv_dispatch(X, W, slabs, M, N, K / S, K, S, N, MS_GEMV_EPI_STORE_F32, ga, force_waves, s);
}

// ---------------------------------------------------------------- argmax of partials
// rows of {max, id} float2 partials (MS_GEMV_EPI_ARGMAX) -> greedy ids; ties -> lowest id
// whatever the merge order; -1 when the row has no finite maximum (a failed chunk)
__global__ __launch_bounds__(1024) void argmax_partials_kernel(const float2* __restrict__ part, int tiles,
                                                               int32_t* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const float2* p = part + (size_t)blockIdx.x * tiles;
  float v = -INFINITY;
  int idx = 0x7FFFFFFF;
  for (int t0 = 0; t0 < tiles; t0 += 8 * 1024) {  // 8 loads in flight per thread
    float2 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = t0 + i * 1024 + threadIdx.x;
      q[i] = t < tiles ? p[t] : make_float2(-INFINITY, __int_as_float(0x7FFFFFFF));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) amax_merge_dev(v, idx, q[i].x, __float_as_int(q[i].y));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = v; si[threadIdx.x >> 6] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) amax_merge_dev(v, idx, sv[w], si[w]);
    out[blockIdx.x] = (idx == 0x7FFFFFFF || !__builtin_isfinite(v)) ? -1 : idx;
  }
}

void launch_argmax_partials(const void* partials, int rows, int tiles, int32_t* out, hipStream_t s) {
  if (rows <= 0) return;
  MS_LAUNCH(argmax_partials_kernel, dim3(rows), dim3(1024), 0, s, (const float2*)partials, tiles, out);
}

void launch_gemv(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldo, int epi,
                 void*, hipStream_t s) {
  launch_gemv_ex(X, W, out, M, N, K, ldo, epi, nullptr, 0, s);
}

}  // namespace ms
