// k_qkvattn.hip -- the decode step's QKV projection and attention as ONE launch (small-regime
// engines of <= 8 slots, fp16 QKV weights, one KV page per wave: the configs[1] bench engine).
//
// Why.  Decode attention streams every sequence's cached K/V (71 MB per layer at 8 x 2176 keys)
// and needs q only for its math; the QKV projection before it streams 31.5 MB of weights at
// 3.9 TB/s and attention cannot issue a single page load until that launch has drained
// (8.2 + 18.4 us per layer as two launches, profiles/r05/v5_kernel_stats_f16.txt).  The pages do
// not depend on q.  Here every workgroup streams its share of the QKV weights, and the page waves
// put their K/V page in flight the moment their weight bytes have been multiplied: the K/V
// stream runs under the projection's tail, its publish and the hand-off, instead of after them
// (the reference's decode loop, /root/reference/run_full_evaluation_pipeline.py:90
// via Ollama, runs this once per generated token).
//
// Layout: 256 workgroups x 12 waves, one per CU (all resident: the hand-off needs it -- checked
// at engine creation, and every wait is bounded).  Workgroup j produces 20 rows of kv head
// hp = j % Hk's 640 QKV rows ([its G q heads | k | v], group-local rows 20 (j / Hk) ..) and
// runs attention item j of launch_attn_decode2's grid (split * B * Hk + b * Hk + kvh, so
// kvh = j % Hk = hp): the 32 producers and the 32 consumers of one kv head are the same
// workgroups (one XCD under round-robin placement -- speed only, never correctness).
//
// Arithmetic: bit-identical to gemv_kernel<1, 1, STORE_F32, 1, LDS> split 6 (K / 6 = 512 = 8 units
// of 64 k, one unit per wave, per-wave partials summed in wave order from 0) followed by the
// attention prologue's slab fold (s0 + s1 + .. + s5): wave w owns units 4w .. 4w+3 of both 10-row
// tiles (unit u = 64 k at k = 64 u; slab u / 8), each unit is the same two MFMAs from a zero
// accumulator, the even wave of a slab sums its four units from 0 (the first half of the GEMV's
// wave-order sum), the odd wave continues from that prefix through LDS, and the publishing wave
// adds the six slab sums in slab order -- qkv32 holds exactly the folded value, so the consumer
// prologue (v2's, S = 1) rounds the same bits.  Attention math, merge and partials are v2's.
//
// Measured (opt-in, MS_QKV_ATTN=1; profiles/r05/v6_*): 32.4-35.4 us per layer against 8.2 + 18.4
// for the two launches -- SLOWER.  In-kernel stamps (MS_QA_STAMPS, tools/qa_stamps.py) show why:
// the weights land at 6.4 us, but a CU's vector memory operations retire in order ACROSS its
// waves, so with the pages issued under the projection (MS_QA_ORDER=0) the publishing wave's own
// weight loads land at 17 us behind them; issued after the publish (1), the prologue's reads of
// the handed-off rows wait behind them (prologue done at 27 us); issued after the prologue (2,
// no overlap), publish -> poll alone takes 6-7 us (drain, arrival, the slowest of 32 producers)
// where a kernel boundary costs ~1.5 us.  The page stream cannot overlap the hand-off on one CU.
//
// Hand-off (cdna_hip_programming.md Guideline 16, as k_mlp.hip): the publishing wave (no page
// loads of its own in flight: vmcnt retires in order, a page wave's drain would wait for its
// page) stores its rows write-through (sc1), drains them, and adds 1 to its kv head's arrival
// counter; a helper wave polls its item's counter (relaxed, s_sleep, bounded by `spin`: a
// timeout sets *err and goes on -- never a hang); the prologue reads qkv32 with sc1 loads.  The
// last workgroup to depart resets the counters for the next launch (stream order).
#include "attn_common.h"
#include "gemv_common.h"

namespace ms {

constexpr int kQaBlocks = 256;                  // one workgroup per CU
constexpr int kQaWaves = 12;                    // PPB page waves + helpers
constexpr int kQaThreads = 64 * kQaWaves;
constexpr int kQaRt = 10;                       // weight rows per MFMA tile (lanes >= 10 duplicate row 9)
constexpr int kQaRows = 2 * kQaRt;              // QKV rows per workgroup: 256 x 20 = 5120
constexpr int kQaUnits = 4;                     // 64-k units per wave: 12 x 4 x 64 = 3072
constexpr int kQaSlabUnits = 8;                 // units per slab of the split-6 GEMV (512 / 64)
constexpr int kQaSlabs = kQaWaves * kQaUnits / kQaSlabUnits;  // 6
constexpr int kQaH = kQaWaves * kQaUnits * 64;  // 3072
constexpr int kQaMaxB = 8;                      // rows of the MFMA tile a lane group pair holds
constexpr int kQaRedBytes = kQaSlabs * 2 * 64 * 16;  // one f32x4 per lane per (slab, tile)
constexpr int kQaDepart = 16;                   // sync word of the departures
constexpr unsigned kQaSpin = 1u << 20;          // ~1 s of polls: a give-up, never a hang
constexpr int kMaxGroupQa = 8;                  // q heads per kv head (k_attn.hip kMaxGroup)

typedef __attribute__((address_space(1))) unsigned qa_gu32_t;

// In-kernel timeline stamps (diagnostic build switch MS_QA_STAMPS=1, never on in a timed run):
// s_memrealtime (100 MHz, chip-wide) at the phase boundaries of every workgroup of the latest
// launch, [kQaBlocks][kQaStamps]; read back with qkv_attn_stamps (tools/qa_stamps.py)
constexpr int kQaStamps = 16;
__device__ unsigned long long g_qa_stamps[kQaBlocks * kQaStamps];
#define QA_STAMP(k) \
  do { if (a.stamps && lane == 0) g_qa_stamps[blockIdx.x * kQaStamps + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

struct QkvAttnArgs {
  const f16_t* xb;    // [B][H] f16(x * attn_norm * 2^-4), the deferred-norm GEMM input
  const f16_t* wqkv;  // [QKVN][H], q / k rows rope-permuted
  float* qkv32;       // [B][QKVN] the projection, unscaled fp32 (the hand-off payload)
  unsigned* sync;     // [0, Hk) arrivals per kv head, [kQaDepart] departures
  unsigned* err;
  unsigned spin;
  DecodeQKV qa;       // rs: the rows' deferred-norm statistics (256 tiles); cos / sin tables
  KVView kv;
  DecodeAttnArgs da;
  float* ws;
  f16_t* out;
  int Hq, Hk, nsplit, n_items;
  float scale_log2;
  int order;  // where the page loads are issued (issue_pages)
  int stamps;
};

__device__ __forceinline__ void qa_store_wt(float* p, float v) {  // write-through (sc1)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float qa_load_wt(const float* p) {  // no stale cached copy (sc1)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int PPB>
__global__ __launch_bounds__(kQaThreads, 1) void qkv_attn_kernel(QkvAttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NH = kQaThreads - 64 * PPB;  // helper threads (waves PPB ..)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int g = fg, r = fr;
  const int Hq = a.Hq, Hk = a.Hk, G = Hq / Hk;
  const int B = a.da.B;
  const int QKVN = (Hq + 2 * Hk) * kHeadDim;
  const int j = blockIdx.x;
  char* red = smem + (size_t)PPB * 16384;  // the reduction exchange, later the prologue's q / k / v
  const bool helper = wave >= PPB;
  const int htid = tid - 64 * PPB;         // helper thread index (valid when helper)
  constexpr int kPubWave = kQaWaves - 1;   // publishes the rows, polls, departs

  // ---- the attention item (launch_attn_decode2's block index) and this wave's page
  const bool has_item = j < a.n_items;
  const int BH = B * Hk;
  const int split = j / BH, grp = j - split * BH;
  const int b = grp / Hk, kvh = grp - b * Hk;
  const int len = has_item ? a.da.seq_len[b] : 1;
  const int slot = has_item ? a.da.seq_slot[b] : 0;
  const int np = (len + kPage - 1) / kPage;
  const int pg = split * PPB + wave;
  const int pos = len - 1;
  const bool has_page = has_item && !helper && pg < np;  // wave-uniform
  const size_t pbase = (((size_t)slot * a.kv.max_pages + pg) * a.kv.n_kv_heads + kvh) * kPage * kHeadDim;
  char* vs_ = smem + (size_t)min(wave, PPB - 1) * 16384;

  if (wave == kQaWaves - 1) QA_STAMP(0);
  if (wave == 0) QA_STAMP(8);
  // the helpers' prologue operands: the row's deferred-norm partial sums (tile lane + 64 i, as
  // gemv_common.h rs_finish) and this thread's rope pair -- L2-resident, loaded first
  float rv[4] = {0.f, 0.f, 0.f, 0.f};
  float rcs = 0.f, rsn = 0.f;
  if (helper && has_item) {
    if (a.qa.rs.ssq) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = lane + 64 * i;
        rv[i] = a.qa.rs.ssq[(size_t)min(t, a.qa.rs.tiles - 1) * B + b];
      }
    }
    rcs = a.qa.cos_tab[(size_t)pos * 64 + (htid & 63)];
    rsn = a.qa.sin_tab[(size_t)pos * 64 + (htid & 63)];
  }

  // ---- 1. the projection: 20 rows of kv head hp, units 4 wave .. 4 wave + 3 of both tiles
  const int hp = j % Hk, sub = j / Hk;
  auto qkv_row = [&](int rl) {  // group-local row -> fused QKV row
    const int qr = G * kHeadDim;
    return rl < qr ? hp * qr + rl
                   : (rl < qr + kHeadDim ? (Hq + hp) * kHeadDim + (rl - qr) : (Hq + Hk + hp) * kHeadDim + (rl - qr - kHeadDim));
  };
  const bool odd = wave & 1;  // second half of slab wave / 2
  f32x4 part[2];              // even: the slab's prefix (units 0-3); odd: unused until the exchange
  f32x4 uo[kQaUnits][2];      // odd: the unit results, added onto the prefix in unit order
  {
    const int kb = wave * kQaUnits * 64 + 16 * fg;
    uint4 xr[kQaUnits][2], w[kQaUnits][2][2];
    const f16_t* xp = a.xb + (size_t)min(fr, B - 1) * kQaH + kb;
#pragma unroll
    for (int u = 0; u < kQaUnits; ++u) {
      xr[u][0] = ldg16(xp + u * 64);
      xr[u][1] = ldg16(xp + u * 64 + 8);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f16_t* wp = a.wqkv + (size_t)qkv_row(kQaRows * sub + kQaRt * t + min(fr, kQaRt - 1)) * kQaH + kb;
#pragma unroll
      for (int u = 0; u < kQaUnits; ++u) {
        w[u][t][0] = ldw16(wp + u * 64);
        w[u][t][1] = ldw16(wp + u * 64 + 8);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) part[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kQaUnits; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        acc = mfma16(as_f16x8(xr[u][0]), as_f16x8(w[u][t][0]), acc);
        acc = mfma16(as_f16x8(xr[u][1]), as_f16x8(w[u][t][1]), acc);
        if (odd) uo[u][t] = acc;
        else part[t] += acc;
      }
  }

  // ---- 2. this wave's K/V page in flight: V by LDS DMA into its V^T image, then K into
  // registers (launch_attn_decode2's loads).  Where (a.order, tuning): 0 under the projection's
  // exchange (the weight registers are free), 1 after the publish, 2 after the prologue -- loads a
  // CU has in flight delay every later memory operation of the CU, the hand-off's included
  u32x4 kf[4][4];
  auto issue_pages = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = 4 * i + (lane >> 4), ch = (lane & 15) ^ ((rr & 7) << 1);
      dma16_opaque(a.kv.v + pbase + rr * kHeadDim + ch * 8, vs_ + i * 1024);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        kf[mt][s4] = ld_stream(a.kv.k + pbase + (mt * 16 + r) * kHeadDim + 32 * s4 + 8 * g);
  };
  if (wave == kQaWaves - 1) QA_STAMP(1);   // (the MFMAs have consumed this wave's weight bytes)
  if (wave == 0) QA_STAMP(9);
  if (a.order == 0 && has_page) issue_pages();

  // ---- 3. the slab sums: even waves hand their prefix to the odd wave of the slab
  f32x4* xch = (f32x4*)red;  // [slab][tile][lane]
  if (!odd)
#pragma unroll
    for (int t = 0; t < 2; ++t) xch[((wave >> 1) * 2 + t) * 64 + lane] = part[t];
  lds_sync();
  if (odd) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 p = xch[((wave >> 1) * 2 + t) * 64 + lane];
#pragma unroll
      for (int u = 0; u < kQaUnits; ++u) p += uo[u][t];
      xch[((wave >> 1) * 2 + t) * 64 + lane] = p;
    }
  }
  lds_sync();
  // ---- 4. publish: the slabs in slab order, write-through stores, drain, arrive
  if (wave == kPubWave) {
    QA_STAMP(2);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 tot = xch[t * 64 + lane];
#pragma unroll
      for (int y = 1; y < kQaSlabs; ++y) tot += xch[(y * 2 + t) * 64 + lane];
      const int col = qkv_row(kQaRows * sub + kQaRt * t + fr);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int row = 4 * fg + jj;
        if (row < B && fr < kQaRt) qa_store_wt(a.qkv32 + (size_t)row * QKVN + col, tot[jj]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows reached L2 (write-through)
    if (lane == 0) __hip_atomic_fetch_add((qa_gu32_t*)&a.sync[hp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the arrival has landed before this workgroup can depart (relaxed atomics to different
    // words may reach L2 out of order: a departure must never let the reset overtake it)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    QA_STAMP(3);
  }
  if (a.order == 1) {  // workgroup-uniform
    lds_sync();
    if (has_page) issue_pages();
  }
  if (wave == kPubWave) {
    // wait for the item's kv head: its 256 / Hk producers
    if (has_item) {
      bool ok = false;
      const unsigned want = (unsigned)(kQaBlocks / Hk);
      for (unsigned it = 0; it < a.spin; ++it) {
        if (__hip_atomic_load((qa_gu32_t*)&a.sync[kvh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) {
          ok = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok && lane == 0) __hip_atomic_store((qa_gu32_t*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      QA_STAMP(4);
    }
    if (lane == 0) {  // every workgroup past its wait: the last one resets the counters
      const unsigned d =
          __hip_atomic_fetch_add((qa_gu32_t*)&a.sync[kQaDepart], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == kQaBlocks - 1) {
        for (int h = 0; h < Hk; ++h) __hip_atomic_store((qa_gu32_t*)&a.sync[h], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((qa_gu32_t*)&a.sync[kQaDepart], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (!has_item) return;  // workgroup-uniform: a producer only
  lds_sync();             // the item's q / k / v rows are published; the exchange region is free

  // ---- 5. prologue (helpers): q / k / v of (b, kvh) -> fp16 with the row scale, RoPE; the owner
  // writes the new token's K/V into the cache (launch_attn_decode2's arithmetic, one slab)
  float* raw = (float*)red;                        // [(G+2)][128] fp16-rounded sums
  f16_t* qn = (f16_t*)(raw + (G + 2) * kHeadDim);  // [G][128] roped q
  f16_t* kn = qn + G * kHeadDim;                   // [128] roped k of the new token
  f16_t* vn = kn + kHeadDim;                       // [128] v of the new token
  const bool owns_new = (pos / kPage) / PPB == split;  // workgroup-uniform
  if (helper) {
    const int nvec = (G + (owns_new ? 2 : 0)) * kHeadDim;
    float rsum = 0.f;
    if (a.qa.rs.ssq) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (!(lane + 64 * i < a.qa.rs.tiles)) rv[i] = 0.f;
      rsum = ((rv[0] + rv[1]) + rv[2]) + rv[3];
    }
    const float rrow = a.qa.rs.ssq ? rs_rinv(wave_sum(rsum), a.qa.rs) : 1.0f;
    const float* src = a.qkv32 + (size_t)b * QKVN;
    constexpr int PER = ((kMaxGroupQa + 2) * kHeadDim + NH - 1) / NH;
    float sv[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = min(htid + i * NH, nvec - 1);
      const int hh = e >> 7, jj = e & 127;
      const int col = hh < G ? (kvh * G + hh) * kHeadDim + jj
                             : (hh == G ? (Hq + kvh) * kHeadDim + jj : (Hq + Hk + kvh) * kHeadDim + jj);
      sv[i] = qa_load_wt(src + col);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = htid + i * NH;
      if (e < nvec) raw[e] = h2f(f2h(sv[i] * rrow));
    }
  }
  lds_sync();
  if (helper) {
    const int nrot = (G + (owns_new ? 1 : 0)) * 64;  // (head, i) pairs: the q heads, then k
    for (int e = htid; e < nrot; e += NH) {
      const int hh = e >> 6, i = e & 63;  // i == htid & 63 (NH % 64 == 0)
      const float lo = raw[hh * kHeadDim + rope_perm(i)], hi = raw[hh * kHeadDim + rope_perm(64 + i)];
      const float ra = __fsub_rn(__fmul_rn(lo, rcs), __fmul_rn(hi, rsn));
      const float rb = __fadd_rn(__fmul_rn(hi, rcs), __fmul_rn(lo, rsn));
      f16_t* dst = hh < G ? qn + hh * kHeadDim : kn;
      dst[i] = f2h(ra);
      dst[64 + i] = f2h(rb);
    }
    if (owns_new && htid < kHeadDim) vn[htid] = f2h(raw[(G + 1) * kHeadDim + htid]);
  }
  lds_sync();
  if (wave == kQaWaves - 1) QA_STAMP(5);
  if (a.order == 2 && has_page) issue_pages();
  if (helper && owns_new && htid < kHeadDim) {
    const size_t o = ((((size_t)slot * a.kv.max_pages + pos / kPage) * a.kv.n_kv_heads + kvh) * kPage + pos % kPage) *
                         kHeadDim + htid;
    a.kv.k[o] = kn[htid];
    a.kv.v[o] = vn[htid];
  }

  // ---- 6. S^T = K Q^T, softmax over the page, O^T = V^T P^T (launch_attn_decode2's math)
  f32x4 o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  if (has_page) {
    f16x8 qf[4];
    const int hl = min(r, G - 1);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *(const f16x8*)(qn + hl * kHeadDim + 32 * s4 + 8 * g);
    const int off = pos % kPage;
    const bool patch = pg == pos / kPage;  // wave-uniform: holds the new token
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
      for (int jj = 0; jj < 4; ++jj) {
        const int key = pg * kPage + mt * 16 + 4 * g + jj;
        const float v = (key >= len) ? -INFINITY : sc[mt][jj] * a.scale_log2;
        sc[mt][jj] = v;
        mx = fmaxf(mx, v);
      }
    mx = grp_max(mx);  // finite: key pg*64 < len is always visible
    float rs = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float p = (sc[mt][jj] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sc[mt][jj] - mx);
        sc[mt][jj] = p;
        rs += p;
      }
    l_run = grp_sum(rs);
    m_run = mx;
    if (wave == 0) QA_STAMP(10);  // K has landed (the S MFMAs waited for it)
    // the V image has landed (its DMA was issued before the K loads the S MFMAs waited for)
    wait_vmcnt0();
    if (pg == np - 1) {
      const int first = len - pg * kPage;  // rows [first, 64) are past the sequence
      for (int e = first * 16 + lane; e < 64 * 16; e += 64) *(u32x4*)(vs_ + v_swz(e >> 4, e & 15)) = u32x4{0, 0, 0, 0};
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
  }
  if (wave == 0) QA_STAMP(11);
  // ---- 7. publish (m, l, O^T) of each page wave's 16 columns, merge in wave order
  if (!helper) {
    float* mw = (float*)vs_;
    if (g == 0) { mw[r * 130 + 0] = m_run; mw[r * 130 + 1] = l_run; }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mw[r * 130 + 2 + dt * 16 + 4 * g + jj] = o[dt][jj];
  }
  __syncthreads();
  for (int idx = tid; idx < G * 130; idx += kQaThreads) {
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
    if (a.nsplit == 1) {
      if (k >= 2) a.out[(size_t)b * Hq * kHeadDim + (kvh * G + c) * kHeadDim + (k - 2)] = f2h(acc / L);
    } else {
      a.ws[(((size_t)b * Hq + kvh * G + c) * a.nsplit + split) * 132 + k] = (k == 0) ? M : acc;
    }
  }
  if (wave == 0) QA_STAMP(12);
}

static size_t qkv_attn_lds(int ppb, int G) {
  const size_t pro = (size_t)(G + 2) * kHeadDim * 4 + (size_t)(G + 2) * kHeadDim * 2;
  return (size_t)ppb * 16384 + std::max((size_t)kQaRedBytes, pro);
}

static bool qkv_attn_resident(int ppb) {
  // every workgroup must be resident at once (the hand-off waits on all producers of a kv head):
  // one per CU on a chip of >= 256 CUs
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  const size_t lds = qkv_attn_lds(ppb, 3);
  hipError_t e = hipErrorInvalidValue;
#define QO(P_) case P_: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, qkv_attn_kernel<P_>, kQaThreads, lds); break;
  switch (ppb) { QO(4) QO(5) QO(6) QO(7) QO(8) QO(9) default: return false; }
#undef QO
  return e == hipSuccess && (long)per * cus >= kQaBlocks;
}

bool qkv_attn_supported(int B, int max_batch, int H, int Hq, int Hk, int max_len, int ppb, int split_qkv) {
  if (B < 1 || B > max_batch || max_batch > kQaMaxB || H != kQaH || split_qkv != kQaSlabs) return false;
  if (Hk < 1 || Hq % Hk || Hq / Hk > kMaxGroupQa || kQaBlocks % Hk) return false;
  if ((Hq + 2 * Hk) * kHeadDim != kQaBlocks * kQaRows) return false;           // 256 x 20 rows
  if ((Hq / Hk + 2) * kHeadDim != (kQaBlocks / Hk) * kQaRows) return false;    // a kv head's rows on 256 / Hk workgroups
  if (ppb < 4 || ppb > 9 || kQaThreads - 64 * ppb < 192) return false;         // >= 3 helper waves
  if (qkv_attn_lds(ppb, Hq / Hk) > 160 * 1024) return false;
  const int np = (max_len + kPage - 1) / kPage;
  const int nsplit = (np + ppb - 1) / ppb;
  if ((long)max_batch * Hk * nsplit > kQaBlocks) return false;  // one item per workgroup
  static const int resident[10] = {-1, -1, -1, -1, qkv_attn_resident(4), qkv_attn_resident(5), qkv_attn_resident(6),
                                   qkv_attn_resident(7), qkv_attn_resident(8), qkv_attn_resident(9)};
  return resident[ppb] == 1;
}

void launch_qkv_attn(const f16_t* xb, const f16_t* wqkv, float* qkv32, const DecodeQKV& qa, f16_t* out, int Hq,
                     int Hk, KVView kv, DecodeAttnArgs da, float* ws, int ppb, unsigned* sync, unsigned* err,
                     hipStream_t s) {
  if (da.B <= 0 || !kv.slot_major) return;  // callers check qkv_attn_supported
  QkvAttnArgs a{};
  a.xb = xb;
  a.wqkv = wqkv;
  a.qkv32 = qkv32;
  a.sync = sync;
  a.err = err;
  // MS_QA_SPIN: the poll bound (0 forces the timeout path in tests)
  const char* sv = getenv("MS_QA_SPIN");
  a.spin = sv ? (unsigned)strtoul(sv, nullptr, 10) : kQaSpin;
  a.qa = qa;
  a.kv = kv;
  a.da = da;
  a.ws = ws;
  a.out = out;
  a.Hq = Hq;
  a.Hk = Hk;
  const int np = (da.max_len + kPage - 1) / kPage;
  a.nsplit = (np + ppb - 1) / ppb;
  a.n_items = da.B * Hk * a.nsplit;
  a.scale_log2 = kLog2e / sqrtf((float)kHeadDim);
  static const int order = [] { const char* e = getenv("MS_QA_ORDER"); return e ? atoi(e) : 1; }();
  a.order = order;
  static const int stamps = [] { const char* e = getenv("MS_QA_STAMPS"); return e ? atoi(e) : 0; }();
  a.stamps = stamps;
  const size_t lds = qkv_attn_lds(ppb, Hq / Hk);
#define QL(P_) case P_: MS_LAUNCH(qkv_attn_kernel<P_>, dim3(kQaBlocks), dim3(kQaThreads), lds, s, a); break;
  switch (ppb) { QL(4) QL(5) QL(6) QL(7) QL(8) QL(9) default: return; }
#undef QL
  launch_attn_combine(ws, out, da.B, Hq, Hk, a.nsplit, s);
}

void qkv_attn_stamps(unsigned long long* host, int n) {
  n = std::min(n, kQaBlocks * kQaStamps);
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qa_stamps), (size_t)n * sizeof(unsigned long long));
}

}  // namespace ms
