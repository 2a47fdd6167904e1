// k_dgemm.hip -- decode projections at large batch: a skinny GEMM for 16 < M <= 256 rows.
//
// The continuous batch of BASELINE configs[2] keeps B = 64..256 sequences in flight per GPU
// ("B_max chosen to fit KV"), and every decode step multiplies those B rows
// by every weight matrix once (ggml mul_mat).  The weight-streaming
// GEMV (k_gemv.hip) owns 16 weight rows per block and re-reads all M x K activations per
// block: at M = 64 the gate/up launch reads 4x more X from L2 than W from HBM and stalls on
// L2.  Here a block owns 64 weight rows (4 waves x 16) and ALL M rows:
//  * X (M x 64 per K step) is register-staged one step ahead into a double-buffered LDS
//    image (XOR swizzle chunk ^ (row & 7): conflict-free ds_read_b128); the 4 waves share
//    it, so X is read from L2 once per 64 weight rows;
//  * W streams straight to VGPRs, each wave its own 16 rows, DPF K steps in flight
//    (32 contiguous bytes per lane per step, as in the GEMV), and stays in flight across
//    the step's LDS-only barrier (an LDS-DMA X image would force a full vmcnt drain there);
//  * v_mfma_f32_16x16x32_f16, the wave's 16 weight rows as MFMA columns, MT m-tiles;
//  * split-K over gridDim.y for the narrow projections (fp32 slabs, folded by the next
//    residual_rmsnorm / attention prologue exactly like the GEMV's).
// A row's sum order depends only on (K, split), never on M or on the other rows.
#include "gemv_common.h"

namespace ms {

constexpr int DBK = 64;

// KH = 2: an 8-wave block whose waves 4..7 take the upper 64 k of every 128-k step for the
// same 64 weight rows, summed into waves 0..3 once at the end (acc(k half 0) + acc(k half 1),
// in that order for every M).  Two waves per SIMD on grids of <= 256 blocks (gate/up at
// N = 16384: 41.4 -> 34.9 us at M = 128), which otherwise leave one wave per SIMD to cover
// every X / W latency and every step barrier alone; the split projections measured as fast or
// faster on 4-wave blocks (profiles/r05/v20_*).  M <= 128 (MT = 16 spills at 2 waves/SIMD).
int g_dgemm_kh = [] {
  const char* v = getenv("MS_DGEMM_KH");
  return v && atoi(v) == 1 ? 1 : 2;
}();

void set_dgemm_kh(int kh) { g_dgemm_kh = kh == 2 ? 2 : 1; }
int dgemm_kh_setting() { return g_dgemm_kh; }
// WN = 8 (MS_DGEMM_WN, op-level tuning hook; engines pass it per launch): 8 weight-row groups,
// 128 rows per block sharing one X image -- half the X bytes per weight byte.  Same sum order
// as WN = 4 (every wave still covers its 16 rows over the whole K range in the same steps).
static int g_dgemm_wn = [] {
  const char* v = getenv("MS_DGEMM_WN");
  return v && atoi(v) == 8 ? 8 : 4;
}();
void set_dgemm_wn(int wn) { g_dgemm_wn = wn == 8 ? 8 : 4; }

// W ring depth: 3 K steps in flight at 2 blocks per CU; M > 128 (MT = 16) needs more
// registers than 2 blocks per CU allow, so 1 block per CU with a deeper ring
template <int MT, int KH> constexpr int dgemm_dpf() { return MT >= 16 || KH > 1 ? 6 : 3; }

template <int MT, int EPI, int KH, int WN>
__global__ __launch_bounds__(64 * WN * KH, MT >= 16 || KH * WN > 4 ? 1 : 2) void dgemm_kernel(const f16_t* __restrict__ X,
                                                      const f16_t* __restrict__ W,
                                                      void* __restrict__ out, int M, int N, int K,
                                                      int ldk, int ldo, RowScale rs) {
  constexpr int DPF = dgemm_dpf<MT, KH * WN / 4>();
  constexpr int NT = 64 * WN * KH, SK = DBK * KH;  // threads; k per step
  // one X stage: KH half-images of XR rows x 128 B (16*MT rounded up to whole 16-B chunks per thread)
  constexpr int XR = 16 * MT < 32 ? 32 : 16 * MT;
  constexpr int XH = XR * DBK * 2, XB = XH * KH;
  constexpr int XC = XR * 8 * KH, XI = (XC + NT - 1) / NT;  // 16-B chunks of one stage; per thread
  constexpr int XCH = WN * MT * 256 * 4;  // bytes of one [WN waves][MT][64 lanes][4] f32 exchange
  constexpr int SMEM = 2 * XB > KH * XCH ? 2 * XB : KH * XCH;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WN, kh = wave / WN;  // weight-row group, k half
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 16 * WN;
  const int kb = blockIdx.y * K;  // this split's K range in rows of length ldk
  if constexpr (EPI == MS_GEMV_EPI_STORE_F32) out = (float*)out + (size_t)blockIdx.y * M * ldo;
  const int nk = K / SK;

  // X is register-staged one K step ahead: chunk c = tid + NT i of a stage is row c/(8 KH),
  // 16-B chunk cc = c%(8 KH) (k half cc/8), stored at chunk (cc%8) ^ (row & 7) of its half-image
  // (conflict-free fragment reads).  Every wait is then a register dependency the compiler
  // counts itself, and the one barrier per step is LDS-only (lds_sync): the weight loads stay
  // in flight across it.
  uint4 xr[XI];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int c = min(tid + NT * i, XC - 1), r = c / (8 * KH);
      xr[i] = ldg16(X + (size_t)min(r, M - 1) * ldk + kb + k0 + (c % (8 * KH)) * 8);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int c = min(tid + NT * i, XC - 1), r = c / (8 * KH), cc = c % (8 * KH);
      *(uint4*)(smem + buf * XB + (cc >> 3) * XH + r * 128 + (((cc & 7) ^ (r & 7)) << 4)) = xr[i];
    }
  };
  // W: lane (fr, fg) holds k0 + 64 kh + 16 fg .. +15 of row n0 + 16 wn + fr (32 contiguous
  // bytes), a DPF-slot register ring, DPF K steps in flight; X: the same permuted k order from LDS
  const f16_t* wrow = W + (size_t)min(n0 + 16 * wn + fr, N - 1) * ldk + kb + DBK * kh + 16 * fg;
  uint4 wr[DPF][2];
  load_x(0);
  store_x(0);
  load_x(min(1, nk - 1) * SK);
#pragma unroll
  for (int p = 0; p < DPF; ++p) {
    wr[p][0] = ldw16(wrow + min(p, nk - 1) * SK);
    wr[p][1] = ldw16(wrow + min(p, nk - 1) * SK + 8);
  }
  lds_sync();

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // unrolled by DPF so every ring slot is a compile-time register set (a runtime-indexed
  // ring compiles to selects that wait for each load as soon as it is issued); past the
  // end the loads are clamped re-reads, never branched around
  for (int t0 = 0; t0 < nk; t0 += DPF) {
#pragma unroll
    for (int i = 0; i < DPF; ++i) {
      const int t = t0 + i;
      if (t >= nk) break;  // block-uniform
      const int buf = t & 1;
      // (a) X(t) x W(t)
      const char* xs = smem + buf * XB + kh * XH;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = m * 16 + fr;
        const f16x8 x0 = *(const f16x8*)(xs + row * 128 + (((2 * fg) ^ (row & 7)) << 4));
        const f16x8 x1 = *(const f16x8*)(xs + row * 128 + (((2 * fg + 1) ^ (row & 7)) << 4));
        acc[m] = mfma16(x0, as_f16x8(wr[i][0]), acc[m]);
        acc[m] = mfma16(x1, as_f16x8(wr[i][1]), acc[m]);
      }
      // (b) X(t+1) into the other stage (every wave finished reading it before the last sync)
      store_x(buf ^ 1);
      // (c) X(t+2) and W(t+DPF) (into the slot just consumed) in flight
      load_x(min(t + 2, nk - 1) * SK);
      wr[i][0] = ldw16(wrow + min(t + DPF, nk - 1) * SK);
      wr[i][1] = ldw16(wrow + min(t + DPF, nk - 1) * SK + 8);
      // (d) X(t+1) visible; every wave done with stage buf before X(t+2) overwrites it
      lds_sync();
    }
  }

  if constexpr (KH > 1) {
    // acc = ((acc(k part 0) + acc(part 1)) + acc(part 2)) + ...; the stages are free after the
    // loop's last sync
    float* kx = (float*)smem;  // [KH - 1][WN waves][MT][64 lanes][4]
    if (kh)
#pragma unroll
      for (int m = 0; m < MT; ++m) *(f32x4*)&kx[(((kh - 1) * WN + wn) * MT + m) * 256 + lane * 4] = acc[m];
    __syncthreads();
    if (!kh)
#pragma unroll
      for (int p = 0; p < KH - 1; ++p)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] += *(const f32x4*)&kx[((p * WN + wn) * MT + m) * 256 + lane * 4];
  }

  // epilogue (waves 0..3): acc[m][j] = C[row m*16 + 4 fg + j][col n0 + 16 wn + fr]; rows scaled
  // by the deferred RMSNorm factor (one-tile RowScale: rs_rinv(ssq[row]), as every consumer forms it)
  const int col = n0 + 16 * wn + fr;
  if (rs.ssq && !kh) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[m][j] *= rs_rinv(rs.ssq[min(m * 16 + 4 * fg + j, M - 1)], rs);
  }
  if constexpr (EPI == MS_GEMV_EPI_SWIGLU) {
    // waves 2q / 2q+1 hold the gate / up tile of the same 16 features: pair through LDS
    // (a region of its own: the k-half exchange may still be read by a slower wave)
    float* xch = (float*)(smem + (KH - 1) * XCH);  // [WN waves][MT][64 lanes][4]
    if (!kh)
#pragma unroll
      for (int m = 0; m < MT; ++m) *(f32x4*)&xch[((wn * MT + m) * 64 + lane) * 4] = acc[m];
    __syncthreads();
    if (kh || (wn & 1)) return;
    const int f = (n0 >> 5) * 16 + (wn >> 1) * 16 + fr;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x4 u = *(const f32x4*)&xch[(((wn + 1) * MT + m) * 64 + lane) * 4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + 4 * fg + j;
        if (row < M && f < N / 2) {
          const float gte = acc[m][j];
          ((f16_t*)out)[(size_t)row * ldo + f] = f2h(gte / (1.0f + __expf(-gte)) * u[j]);
        }
      }
    }
  } else if constexpr (EPI == MS_GEMV_EPI_ARGMAX) {
    if (kh) return;
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
        if (fr == 0 && row < M) ((float2*)out)[(size_t)row * ldo + (n0 >> 4) + wn] = make_float2(v, __int_as_float(idx));
      }
  } else {
    if (kh || col >= N) return;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + 4 * fg + j;
        if (row >= M) continue;
        const size_t o = (size_t)row * ldo + col;
        if constexpr (EPI == MS_GEMV_EPI_STORE_F16) ((f16_t*)out)[o] = f2h(acc[m][j]);
        else if constexpr (EPI == MS_GEMV_EPI_ADD_F32) ((float*)out)[o] += acc[m][j];
        else ((float*)out)[o] = acc[m][j];
      }
  }
}

// kh 0 = the library setting where it applies (M <= 128, K % (128 S) == 0), else 1
static int dgemm_kh_for(int M, int K, int S) { return g_dgemm_kh == 2 && M <= 128 && K % (S * 2 * DBK) == 0 ? 2 : 1; }
static int dgemm_wn_for(int M, int N, int kh) { return g_dgemm_wn == 8 && kh == 1 && M <= 128 && N % 128 == 0 ? 8 : 4; }

bool dgemm_supported(int M, int N, int K, int S, int epi, int kh, int wn) {
  if (!kh) kh = dgemm_kh_for(M, K, S);
  if (!wn) wn = dgemm_wn_for(M, N, kh);
  if (wn != 4 && (wn != 8 || kh != 1 || M > 128)) return false;
  if (M < 1 || M > (kh > 1 ? 128 : 256) || N % (16 * wn) || S < 1 || K % (S * DBK * kh)) return false;
  if (epi == MS_GEMV_EPI_ROPE_KV) return false;
  if (S > 1 && epi != MS_GEMV_EPI_STORE_F32) return false;
  return true;
}

template <int MT, int KH, int WN = 4>
static void dgemm_go(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int S, int ldo,
                     int epi, const RowScale& rs, hipStream_t s) {
  const dim3 grid(N / (16 * WN), S), blk(64 * WN * KH);
  const int Ks = K / S;
  switch (epi) {
#define DG(E_) MS_LAUNCH((dgemm_kernel<MT, E_, KH, WN>), grid, blk, 0, s, X, W, out, M, N, Ks, K, ldo, rs)
    case MS_GEMV_EPI_STORE_F16: DG(MS_GEMV_EPI_STORE_F16); break;
    case MS_GEMV_EPI_ADD_F32: DG(MS_GEMV_EPI_ADD_F32); break;
    case MS_GEMV_EPI_SWIGLU: DG(MS_GEMV_EPI_SWIGLU); break;
    case MS_GEMV_EPI_ARGMAX: DG(MS_GEMV_EPI_ARGMAX); break;
    default: DG(MS_GEMV_EPI_STORE_F32); break;
#undef DG
  }
}

// rs: the deferred RMSNorm scale of the output rows, one-tile partials only (or null)
void launch_dgemm(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int S, int ldo, int epi,
                  hipStream_t s, const RowScale* rs_in, int kh, int wn) {
  if (!kh) kh = dgemm_kh_for(M, K, S);
  if (!wn) wn = dgemm_wn_for(M, N, kh);
  if (!dgemm_supported(M, N, K, S, epi, kh, wn)) return;  // callers check
  RowScale rs{};
  if (rs_in && rs_in->ssq && epi != MS_GEMV_EPI_ARGMAX) {  // argmax: r > 0 keeps the order
    if (rs_in->tiles != 1) return;  // callers pass one-tile statistics (a norm kernel's)
    rs = *rs_in;
  }
  const int mt = (M + 15) / 16;
  if (wn == 8) {  // 128 weight rows per block (KH = 1, M <= 128)
    if (mt <= 1) dgemm_go<1, 1, 8>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else if (mt <= 2) dgemm_go<2, 1, 8>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else if (mt <= 4) dgemm_go<4, 1, 8>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else dgemm_go<8, 1, 8>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    return;
  }
  if (kh > 1) {  // the k-half block (M <= 128)
    if (mt <= 1) dgemm_go<1, 2>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else if (mt <= 2) dgemm_go<2, 2>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else if (mt <= 4) dgemm_go<4, 2>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    else dgemm_go<8, 2>(X, W, out, M, N, K, S, ldo, epi, rs, s);
    return;
  }
  if (mt <= 1) dgemm_go<1, 1>(X, W, out, M, N, K, S, ldo, epi, rs, s);
  else if (mt <= 2) dgemm_go<2, 1>(X, W, out, M, N, K, S, ldo, epi, rs, s);
  else if (mt <= 4) dgemm_go<4, 1>(X, W, out, M, N, K, S, ldo, epi, rs, s);
  else if (mt <= 8) dgemm_go<8, 1>(X, W, out, M, N, K, S, ldo, epi, rs, s);
  else dgemm_go<16, 1>(X, W, out, M, N, K, S, ldo, epi, rs, s);
}

}  // namespace ms
