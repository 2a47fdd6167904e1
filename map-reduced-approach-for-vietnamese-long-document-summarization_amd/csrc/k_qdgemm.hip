// k_qdgemm.hip -- decode projections of K-quant engines at large batch: the skinny GEMM of
// k_dgemm.hip with the weights streamed as their packed Q4_K / Q6_K rows and dequantised in
// registers, so a Q4_K_M engine of > 64 slots reads each quantised weight ONCE per decode step
// (1.9 GB instead of the fp16 copies' 6.4 GB; SURVEY.md §8a rows A9 / A10, BASELINE.json
// configs[4] at configs[2]'s batch).
//
// The K-quant GEMV (k_qgemv.hip) keeps the exact fp32 dequantised weights by scaling every
// 32-weight sub-block's MFMA partial with two FMAs per output element: at 16 rows that costs
// nothing, at 128 rows it is 16x the work, and its row groups of <= 64 rows re-stream the
// weights per group (Q4_K_M at 128 slots: 18.2 ms per decode step against fp16's 8.4,
// profiles/r06/v9_*).  Here each wave dequantises its 16 weight rows ONCE per 32-k MFMA column
// to fp16 -- the values of the engine's fp16 copy, f16(ggml dequant), the ones every prefill GEMM
// multiplies -- and feeds all M rows from the block's shared X image with them.
//  * block: 4 waves x 16 weight rows, all M <= 256 rows (MT m-tiles); X staged by LDS DMA into a
//    4-stage swizzled image three 64-k steps ahead, with counted vmcnt waits and fence-free step
//    barriers, so the weight ring and the later stages stay in flight across them (the time per
//    step grows with the X bytes every block re-reads -- the bound, not the weight bytes: the
//    same kernel on fp16 rows, kQdF16, runs gate/up at M = 128 in 33.7 us against 29.0 us on
//    Q4_K; profiles/r06/v10_*);
//  * W: one super-block (256 k) of the wave's 16 rows per ring slot, DPF super-blocks in flight
//    (Q4_K: header + sub-blocks 0-3 / 4-7, 48 B per lane; Q6_K: four 8-B ql pieces, two 8-B qh
//    pieces, the scales and d);
//  * MFMA column c of a super-block (v_mfma_f32_16x16x32_f16, 32 consecutive k): lane group g
//    holds k = 32c + 8g .. +7 of its row -- the packed Q4_K layout's own order (quant_rows_kernel)
//    and Q6_K's natural one -- and reads the same k of X;
//  * dequant: Q4_K y = fma(d*sc, q, -(dmin*m)) (the products are exact in fp32, so this is
//    ggml's d1*q - m1 with its single rounding), Q6_K y = fma(d*sc, q, -32 d*sc) (ggml's
//    (d*sc)*(q-32)), both rounded to fp16 by v_cvt_pk_f16_f32 (RNE, as the fp16 copy);
//  * epilogues as the skinny GEMM: fp32 split-K slabs (gridDim.y), SwiGLU on the 16-row
//    interleaved gate/up rows, greedy argmax partials; the rows' deferred-norm scale.
// A row's sum order depends only on (K, split), never on M: batch-invariant inside the regime.
#include "gemv_common.h"

namespace ms {

constexpr int QBK = 64;  // k per X stage: two 32-k MFMA columns

__device__ __forceinline__ float qd_h2f(uint32_t h16) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(h16 & 0xFFFFu));
}

struct QdQ4 {  // one packed Q4_K super-block of this lane's row: header, sub-blocks 0-3, 4-7
  uint4 h, q0, q1;
};
struct QdQ6 {  // one packed Q6_K super-block: ql pieces [k4 & 1][n], qh [n], scales, d
  uint2 ql[2][2], qh[2];
  uint4 sc;
  uint32_t d;
};
// fp16 rows through the same kernel (the large regime's fp16 projections): 256 k = 512 B of a row,
// MFMA column c's 8 weights of lane group g at 64 c + 16 g
constexpr int kQdF16 = 1;  // ggml_type F16
struct QdH {
  uint4 w[8];
};

__device__ __forceinline__ uint32_t qd_word(const uint4& v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// W loads: plain loads the compiler tracks (its own waits cover each ring slot's first use).
// Every byte a fetch loads is used, so none is dropped or narrowed and each fetch issues exactly
// kQdLoads instructions -- the counts the step waits assume (checked in the ISA).
__device__ __forceinline__ uint4 qd_ld16(const uint8_t* p) { return ldw16(p); }
__device__ __forceinline__ uint2 qd_ld8(const uint8_t* p) { return *(const uint2*)p; }
__device__ __forceinline__ uint32_t qd_ld4(const uint8_t* p) { return *(const uint32_t*)p; }

__device__ __forceinline__ void qd_fetch(QdQ4& r, const uint8_t* bp, int g) {
  r.h = qd_ld16(bp);
  r.q0 = qd_ld16(bp + 16 + 16 * g);
  r.q1 = qd_ld16(bp + 80 + 16 * g);
}
__device__ __forceinline__ void qd_fetch(QdH& r, const uint8_t* bp, int g) {
#pragma unroll
  for (int c = 0; c < 8; ++c) r.w[c] = qd_ld16(bp + 64 * c + 16 * g);
}
__device__ __forceinline__ void qd_fetch(QdQ6& r, const uint8_t* bp, int g) {
  // packed 224-B block (quant_rows_kernel): raw ql[n*64 + half*32 + l] at half*64 + 32n + 8g + i
  // for l = 8g + i; qh and the scales unmoved
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int n = 0; n < 2; ++n) r.ql[h][n] = qd_ld8(bp + h * 64 + 32 * n + 8 * g);
#pragma unroll
  for (int n = 0; n < 2; ++n) r.qh[n] = qd_ld8(bp + 128 + 32 * n + 8 * g);
  r.sc = qd_ld16(bp + 192);
  r.d = qd_ld4(bp + 208);
}

typedef float qd_f2 __attribute__((ext_vector_type(2)));

// four weights held as the bytes of q4 -> two packed fp16 pairs of fma(a, q, b)
__device__ __forceinline__ void qd_deq4(uint32_t q4, float a, float b, uint32_t& p0, uint32_t& p1) {
  const qd_f2 a2 = {a, a}, b2 = {b, b};
  const qd_f2 y01 = __builtin_elementwise_fma(a2, qd_f2{(float)(q4 & 0xFFu), (float)((q4 >> 8) & 0xFFu)}, b2);
  const qd_f2 y23 = __builtin_elementwise_fma(a2, qd_f2{(float)((q4 >> 16) & 0xFFu), (float)(q4 >> 24)}, b2);
  p0 = pack2h(y01.x, y01.y);
  p1 = pack2h(y23.x, y23.y);
}

// the fp16 weights k = 32c + 8g .. +7 of this lane's row (MFMA column c of the super-block)
__device__ __forceinline__ f16x8 qd_dequant(const QdQ4& r, int c, int g) {
  (void)g;
  const int sh = 8 * (c & 3);
  const uint32_t scw = c < 4 ? (r.h.y & 0x3F3F3F3Fu) : ((r.h.w & 0x0F0F0F0Fu) | ((r.h.y >> 2) & 0x30303030u));
  const uint32_t mw = c < 4 ? (r.h.z & 0x3F3F3F3Fu) : (((r.h.w >> 4) & 0x0F0F0F0Fu) | ((r.h.z >> 2) & 0x30303030u));
  const float d1 = __fmul_rn(qd_h2f(r.h.x), (float)((scw >> sh) & 0xFFu));       // ggml d1 = d * sc
  const float m1 = __fmul_rn(qd_h2f(r.h.x >> 16), (float)((mw >> sh) & 0xFFu));  // ggml m1 = dmin * m
  const uint32_t qw = qd_word(c < 4 ? r.q0 : r.q1, c & 3);  // byte i = q[k_i] | q[k_{i+4}] << 4
  uint32_t pk[4];
  qd_deq4(qw & 0x0F0F0F0Fu, d1, -m1, pk[0], pk[1]);
  qd_deq4((qw >> 4) & 0x0F0F0F0Fu, d1, -m1, pk[2], pk[3]);
  return __builtin_bit_cast(f16x8, pk);
}
__device__ __forceinline__ f16x8 qd_dequant(const QdH& r, int c, int g) {
  (void)g;
  return __builtin_bit_cast(f16x8, r.w[c]);
}
__device__ __forceinline__ f16x8 qd_dequant(const QdQ6& r, int c, int g) {
  const int n = c >> 2, k4 = c & 3;  // weights n*128 + k4*32 + l, l = 8g + i
  const float ds = __fmul_rn(qd_h2f(r.d), (float)(int)(int8_t)((qd_word(r.sc, 2 * n + (k4 >> 1)) >> (8 * ((g >> 1) + 2 * (k4 & 1)))) & 0xFFu));
  const uint2 a = r.ql[k4 & 1][n], hq = r.qh[n];
  const int ns = 4 * (k4 >> 1), hs = 2 * k4;
  uint32_t pk[4];
  qd_deq4(((a.x >> ns) & 0x0F0F0F0Fu) | (((hq.x >> hs) & 0x03030303u) << 4), ds, -32.0f * ds, pk[0], pk[1]);
  qd_deq4(((a.y >> ns) & 0x0F0F0F0Fu) | (((hq.y >> hs) & 0x03030303u) << 4), ds, -32.0f * ds, pk[2], pk[3]);
  return __builtin_bit_cast(f16x8, pk);
}

// the counted waits below hold only if every W load sits where the source puts it, between the
// step's X DMA and its wait: a memory clobber no load may cross (W is not __restrict__: a
// restrict / read-only pointer let the compiler sink loads past the clobber -- the Q6_K qh
// loads moved and the wait released early) and a scheduling barrier
__device__ __forceinline__ void qd_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// the step barrier: no fence -- a workgroup fence makes the compiler drain vmcnt (the LDS DMA
// writes LDS), which would wait for the W ring and the X stages in flight too.  Each wave has
// waited for its own DMA pieces (counted vmcnt) and consumed its LDS reads (the MFMAs wait on
// them) before it arrives; the empty asm keeps the compiler from moving LDS accesses across.
__device__ __forceinline__ void qd_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// steps s in [t - len + 1, t] with s % 4 == 3, for q = t % 4 (compile-time after unrolling)
__host__ __device__ constexpr int qd_fetches_in(int q, int len) {
  int n = 0;
  for (int i = 0; i < len; ++i) n += ((q - i) % 4 + 4) % 4 == 3;
  return n;
}

// s_waitcnt vmcnt(BASE + WF * (fetch steps in the window)) for q = t % 4 (the immediate must be a
// constant: one case per q, folded once the step loop is unrolled)
template <int BASE, int WF, int LEN>
__device__ __forceinline__ void qd_wait_steady(int q) {
  switch (q) {
    case 0: __builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE + WF * qd_fetches_in(0, LEN))); break;
    case 1: __builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE + WF * qd_fetches_in(1, LEN))); break;
    case 2: __builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE + WF * qd_fetches_in(2, LEN))); break;
    default: __builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE + WF * qd_fetches_in(3, LEN))); break;
  }
}

// vector memory instructions of one qd_fetch
template <int QT> constexpr int kQdLoads = QT == MS_QT_Q4_K ? 3 : QT == kQdF16 ? 8 : 8;

// the packed rows of one launch: up to three regions of one type (the fused QKV matrix's Q / K / V
// allocations), rows [0, r1) in b0, [r1, r2) in b1, [r2, N) in b2 -- each a multiple of 64 rows,
// so a block's rows never straddle two (flat fields: no runtime-indexed kernel-argument arrays)
struct QdSrc {
  const uint8_t *b0, *b1, *b2;
  int r1, r2, row_bytes;
};
__device__ __forceinline__ const uint8_t* qd_row(const QdSrc& s, int r) {
  return r >= s.r2 ? s.b2 + (size_t)(r - s.r2) * s.row_bytes
                   : r >= s.r1 ? s.b1 + (size_t)(r - s.r1) * s.row_bytes : s.b0 + (size_t)r * s.row_bytes;
}

template <int QT> struct QdRegs;
template <> struct QdRegs<MS_QT_Q4_K> { using T = QdQ4; static constexpr int kBytes = kQ4KBytes; };
template <> struct QdRegs<MS_QT_Q6_K> { using T = QdQ6; static constexpr int kBytes = kQ6KPacked; };
template <> struct QdRegs<kQdF16> { using T = QdH; static constexpr int kBytes = 512; };

// DPF: super-blocks of W in flight per wave, a divisor of the split's super-block count (the
// ring loop then has no early exit, whose merged paths made the compiler drain vmcnt at the
// loop head).  4 waves x 16 weight rows per block.
template <int MT, int EPI, int QT, int DPF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MT >= 16 ? 1 : 2, 2))) void qdgemm_kernel(
    const f16_t* __restrict__ X, QdSrc src, void* __restrict__ out, int M, int N, int K, int ldk, int ldo,
    RowScale rs) {
  using R = QdRegs<QT>;
  constexpr int WN = 4;
  constexpr int WF = kQdLoads<QT>;                  // vector memory instructions of one W fetch
  constexpr int XR = 16 * MT < 32 ? 32 : 16 * MT;  // X image rows (a KiB piece per wave at least)
  constexpr int XB = XR * QBK * 2;                  // one stage: XR rows x 128 B
  constexpr int PW = XB / 1024 / WN;                // 1-KiB DMA pieces of a stage per wave
  // X stages: three 64-k steps in flight (6 / 8 stages at <= 128 rows measured no faster, and cost
  // the 128-row form its second block per CU)
  constexpr int NS = 4;
  constexpr int XCH = WN * MT * 256 * 4;  // [WN waves][MT][64 lanes][4] f32: SwiGLU pairing
  constexpr int SMEM = NS * XB > XCH ? NS * XB : XCH;
  static_assert(PW >= 1 && PW * WN * 1024 == XB, "X stage pieces");
  // every counted wait assumes the wave never has more than vmcnt's 63 memory instructions in
  // flight (the W ring plus the X stages ahead): a saturated counter would release a wait early
  static_assert(DPF * WF + (NS - 1) * PW <= 63, "vector memory instructions in flight exceed vmcnt");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * WN;  // first weight row of the block
  const int kb = blockIdx.y * K;        // this split's K range in X rows of length ldk
  if constexpr (EPI == MS_GEMV_EPI_STORE_F32) out = (float*)out + (size_t)blockIdx.y * M * ldo;
  const int nk = K / QBK, nsb = K / 256;

  // X stage s (64 k) by LDS DMA, 1 KiB per wave instruction: lane l of piece p copies chunk
  // C = 64 p + l = row C / 8, chunk C % 8 of the image, i.e. the row's global chunk
  // (C % 8) ^ (row & 7) (the swizzle applied on the source side; conflict-free fragment
  // reads).  No registers, and issued three steps ahead: its waits are counted vmcnt
  // immediates that leave every later load (W fetches, later stages) in flight.
  auto dma_x = [&](int st, int t) {
    const int k0 = kb + min(t, nk - 1) * QBK;  // past the end: clamped re-reads
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int p = wn + WN * i, C = p * 64 + lane, r = C >> 3, c = C & 7;
      __builtin_amdgcn_global_load_lds((const void*)(X + (size_t)min(r, M - 1) * ldk + k0 + ((c ^ (r & 7)) << 3)),
                                       (LDS_AS void*)(smem + st * XB + p * 1024), 16, 0, 0);
    }
  };
  // this lane's weight row n0 + 16 wn + fr
  const uint8_t* wrow = qd_row(src, min(n0 + 16 * wn + fr, N - 1)) + (size_t)blockIdx.y * nsb * R::kBytes;
  typename R::T wr[DPF];
  auto fetch = [&](int sb, typename R::T& dst) { qd_fetch(dst, wrow + (size_t)min(sb, nsb - 1) * R::kBytes, g); };
  // the W ring first (older than every X stage, so no X wait ever counts it), then X(0..NS-2)
#pragma unroll
  for (int p = 0; p < DPF; ++p) fetch(p, wr[p]);
  qd_order();
#pragma unroll
  for (int a = 0; a < NS - 1; ++a) dma_x(a, a);
  qd_order();
  __builtin_amdgcn_s_waitcnt(vmcnt_imm((NS - 2) * PW));  // X(0) landed
  qd_barrier();

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // unrolled by DPF super-blocks so every ring slot is a compile-time register set, and by the
  // super-block's four 64-k steps so every vmcnt immediate is compile-time; past the end the
  // loads are clamped re-reads, never branched around (nsb % DPF == 0: host-checked)
  for (int j0 = 0; j0 < nsb; j0 += DPF) {
#pragma unroll
    for (int jj = 0; jj < DPF; ++jj) {
      const int j = j0 + jj;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // step t: X stage t % NS, MFMA columns 2q, 2q + 1
        const int t = 4 * j + q;
        const char* xs = smem + (t % NS) * XB;
        // every X fragment of the step read up front (the step's LDS round trip exposed once, not
        // once per MFMA); the dequant runs under the reads.  MFMA column c = 2q + h: k 32c + 8g ..
        f16x8 xf[2][MT];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int row = m * 16 + fr;
            xf[h][m] = *(const f16x8*)(xs + row * 128 + (((4 * h + g) ^ (row & 7)) << 4));
          }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f16x8 wf = qd_dequant(wr[jj], 2 * q + h, g);
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[m] = mfma16(xf[h][m], wf, acc[m]);
        }
        qd_order();
        dma_x((t + NS - 1) % NS, t + NS - 1);  // into the stage every wave finished reading in step t - 1
        qd_order();
        if (q == 3) fetch(j + DPF, wr[jj]);  // slot consumed
        qd_order();
        // X(t+1) landed: at most the instructions issued after its DMA pending -- the DMAs of
        // steps t-NS+3 .. t and the W fetches of steps t-NS+2 .. t (those with s % 4 == 3); before
        // step NS-2 its DMA came from the prologue (no fetch after it: the fetch-free count waits
        // at least as long)
        constexpr int kDmaAfter = (NS - 2) * PW;
        if (t >= NS - 2)
          qd_wait_steady<kDmaAfter, WF, NS - 1>(q);
        else
          __builtin_amdgcn_s_waitcnt(vmcnt_imm(kDmaAfter));
        qd_barrier();  // X(t+1) visible to every wave; its old stage free for the next DMA
      }
    }
  }
  wait_vmcnt0();  // the clamped tail DMAs land before the epilogue reuses the stages
  __syncthreads();

  // epilogue: acc[m][i] = C[row m*16 + 4g + i][col n0 + 16 wn + fr]; rows scaled by the deferred
  // RMSNorm factor (one-tile RowScale), as k_dgemm.hip
  const int col = n0 + 16 * wn + fr;
  if (rs.ssq) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[m][i] *= rs_rinv(rs.ssq[min(m * 16 + 4 * g + i, M - 1)], rs);
  }
  if constexpr (EPI == MS_GEMV_EPI_SWIGLU) {
    // waves 2p / 2p+1 hold the gate / up rows of the same 16 features (the fused matrix
    // interleaves them by 16 rows); the stages are free after the loop's last barrier
    float* xch = (float*)smem;
#pragma unroll
    for (int m = 0; m < MT; ++m) *(f32x4*)&xch[((wn * MT + m) * 64 + lane) * 4] = acc[m];
    __syncthreads();
    if (wn & 1) return;
    const int f = (n0 >> 5) * 16 + (wn >> 1) * 16 + fr;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x4 u = *(const f32x4*)&xch[(((wn + 1) * MT + m) * 64 + lane) * 4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m * 16 + 4 * g + i;
        if (row < M && f < N / 2) {
          const float gte = acc[m][i];
          ((f16_t*)out)[(size_t)row * ldo + f] = f2h(gte / (1.0f + __expf(-gte)) * u[i]);
        }
      }
    }
  } else if constexpr (EPI == MS_GEMV_EPI_ARGMAX) {
    // {max, id} of each row over this wave's 16 columns
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m * 16 + 4 * g + i;
        float v = (col < N) ? acc[m][i] : -INFINITY;
        if (!(v == v)) v = -INFINITY;
        int idx = col;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
        if (fr == 0 && row < M) ((float2*)out)[(size_t)row * ldo + (n0 >> 4) + wn] = make_float2(v, __int_as_float(idx));
      }
  } else {
    if (col >= N) return;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m * 16 + 4 * g + i;
        if (row < M) ((float*)out)[(size_t)row * ldo + col] = acc[m][i];
      }
  }
}

static constexpr int kQdRowAlign = 64;  // region rows: whole 64-row blocks

// the row range [r0, r1) of region i of q
static void qd_region(const QMat& q, int i, int N, int& r0, int& r1, const uint8_t*& base, int& type, int& rb) {
  const int row0[3] = {q.row0_0, q.row0_1, q.row0_2};
  const uint8_t* b[3] = {q.base0, q.base1, q.base2};
  const int ty[3] = {q.type0, q.type1, q.type2}, rbs[3] = {q.row_bytes0, q.row_bytes1, q.row_bytes2};
  r0 = row0[i];
  r1 = i + 1 < q.n ? row0[i + 1] : N;
  base = b[i];
  type = ty[i];
  rb = rbs[i];
}

// W super-blocks in flight: the largest of 4, 3, 2 dividing the split's super-block count
static int qd_dpf(int nsb) { return nsb % 4 == 0 ? 4 : nsb % 3 == 0 ? 3 : nsb % 2 == 0 ? 2 : 0; }

bool qdgemm_supported(int M, int N, int K, int S, int epi, const QMat& q) {
  if (M < 1 || M > 256 || S < 1 || K % (256 * S) || q.n < 1 || q.n > 3 || !qd_dpf(K / S / 256)) return false;
  if (epi != MS_GEMV_EPI_STORE_F32 && epi != MS_GEMV_EPI_SWIGLU && epi != MS_GEMV_EPI_ARGMAX) return false;
  if (S > 1 && epi != MS_GEMV_EPI_STORE_F32) return false;
  // the SwiGLU pairing and the argmax partial index need the whole matrix in one region
  if ((epi == MS_GEMV_EPI_SWIGLU || epi == MS_GEMV_EPI_ARGMAX) && (q.n != 1 || q.row0_0 != 0)) return false;
  if (q.row0_0 != 0) return false;
  for (int i = 0; i < q.n; ++i) {
    int r0, r1, type, rb;
    const uint8_t* base;
    qd_region(q, i, N, r0, r1, base, type, rb);
    if (r1 <= r0 || (r1 - r0) % kQdRowAlign || (type != MS_QT_Q4_K && type != MS_QT_Q6_K)) return false;
    if (type != q.type0) return false;  // one launch: one type
    if (rb != (K / 256) * qblock_bytes(type, true)) return false;
  }
  return true;
}

template <int MT, int QT, int DPF>
static void qdgemm_go(const f16_t* X, const QdSrc& src, void* out, int M, int Nr, int K, int S, int ldo,
                      int epi, const RowScale& rs, hipStream_t s) {
  const dim3 grid(Nr / 64, S), blk(256);
  const int Ks = K / S;
  switch (epi) {
#define QD(E_) MS_LAUNCH((qdgemm_kernel<MT, E_, QT, DPF>), grid, blk, 0, s, X, src, out, M, Nr, Ks, K, ldo, rs)
    case MS_GEMV_EPI_SWIGLU: QD(MS_GEMV_EPI_SWIGLU); break;
    case MS_GEMV_EPI_ARGMAX: QD(MS_GEMV_EPI_ARGMAX); break;
    default: QD(MS_GEMV_EPI_STORE_F32); break;
#undef QD
  }
}

template <int QT, int DPF>
static void qdgemm_mt(const f16_t* X, const QdSrc& src, void* out, int M, int Nr, int K, int S, int ldo,
                      int epi, const RowScale& rs, hipStream_t s) {
  const int mt = (M + 15) / 16;
  if (mt <= 1) qdgemm_go<1, QT, DPF>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
  else if (mt <= 2) qdgemm_go<2, QT, DPF>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
  else if (mt <= 4) qdgemm_go<4, QT, DPF>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
  else if (mt <= 8) qdgemm_go<8, QT, DPF>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
  else qdgemm_go<16, QT, DPF>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
}
template <int QT>
static void qdgemm_form(const f16_t* X, const QdSrc& src, void* out, int M, int Nr, int K, int S, int ldo,
                        int epi, const RowScale& rs, hipStream_t s) {
  if constexpr (QT == kQdF16) {  // 32 VGPRs a ring slot: at most 3 in flight, preferring 2
    const int nsb = K / S / 256;
    if (nsb % 2 == 0) qdgemm_mt<QT, 2>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
    else qdgemm_mt<QT, 3>(X, src, out, M, Nr, K, S, ldo, epi, rs, s);
    return;
  }
  switch (qd_dpf(K / S / 256)) {
    case 4: qdgemm_mt<QT, 4>(X, src, out, M, Nr, K, S, ldo, epi, rs, s); break;
    case 3: qdgemm_mt<QT, 3>(X, src, out, M, Nr, K, S, ldo, epi, rs, s); break;
    default: qdgemm_mt<QT, 2>(X, src, out, M, Nr, K, S, ldo, epi, rs, s); break;
  }
}

// out as launch_dgemm's (slabs [S][M][ldo] for STORE_F32, the region's columns at their place
// in the whole matrix); rs: one-tile statistics or null (dropped for the argmax)
void launch_qdgemm(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int S, int ldo, int epi,
                   hipStream_t s, const RowScale* rs_in) {
  if (!qdgemm_supported(M, N, K, S, epi, q)) return;  // callers check
  RowScale rs{};
  if (rs_in && rs_in->ssq && epi != MS_GEMV_EPI_ARGMAX) {  // argmax: r > 0 keeps the order
    if (rs_in->tiles != 1) return;
    rs = *rs_in;
  }
  // one launch over every region (all of one type, qdgemm_supported)
  QdSrc src{q.base0, q.n > 1 ? q.base1 : q.base0, q.n > 2 ? q.base2 : q.base0, q.n > 1 ? q.row0_1 : N,
            q.n > 2 ? q.row0_2 : N, q.row_bytes0};
  if (q.type0 == MS_QT_Q4_K) qdgemm_form<MS_QT_Q4_K>(X, src, out, M, N, K, S, ldo, epi, rs, s);
  else qdgemm_form<MS_QT_Q6_K>(X, src, out, M, N, K, S, ldo, epi, rs, s);
}

// the same kernel on fp16 rows W [N][K] (the engine's fp16 large-regime projections; tuning)
bool qdgemm_f16_supported(int M, int N, int K, int S, int epi) {
  const int nsb = S >= 1 && K % (256 * S) == 0 ? K / S / 256 : 0;
  if (M < 1 || M > 256 || N % kQdRowAlign || !(nsb % 2 == 0 || nsb % 3 == 0) || nsb == 0) return false;
  if (epi != MS_GEMV_EPI_STORE_F32 && epi != MS_GEMV_EPI_SWIGLU && epi != MS_GEMV_EPI_ARGMAX) return false;
  return S == 1 || epi == MS_GEMV_EPI_STORE_F32;
}
void launch_qdgemm_f16(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int S, int ldo, int epi,
                       hipStream_t s, const RowScale* rs_in) {
  if (!qdgemm_f16_supported(M, N, K, S, epi)) return;  // callers check
  RowScale rs{};
  if (rs_in && rs_in->ssq && epi != MS_GEMV_EPI_ARGMAX) {
    if (rs_in->tiles != 1) return;
    rs = *rs_in;
  }
  const uint8_t* b = (const uint8_t*)W;
  QdSrc src{b, b, b, N, N, K * 2};
  qdgemm_form<kQdF16>(X, src, out, M, N, K, S, ldo, epi, rs, s);
}

}  // namespace ms
