// k_persist.hip -- the decode step's transformer layers as ONE persistent launch (small-batch
// engines: <= 8 slots, fp16 weights, the Llama-3.2-3B shapes of the bench).
//
// Why.  At B = 8 a decode layer is six weight / KV streams (QKV, attention + its split combine,
// O, gate/up, down) of 3-16 us each, and every launch pays a fixed ramp and drain: the decode
// GEMVs fit t = 4.6 us + bytes / 6.25 TB/s, ~30 % of the step.  Nothing a
// phase STREAMS depends on the previous phase (weights, and the K/V pages of earlier positions,
// are known before the step starts); only what it COMPUTES does.  So one launch covers all
// layers, and on every CU (cdna_hip_programming.md section 5.6, MI355X_MICROARCH 'engine-vs-launches'):
//   * wave 0 is a LOADER: it walks the CU's fixed schedule of weight tiles and K/V pages and
//     streams them by LDS DMA (global_load_lds_dwordx4, 1 KiB per instruction) into a ring of
//     R = 6 slots of 16 KiB, running ahead of every dependency; it alone polls the chip-wide
//     arrival counters of a phase's input and then gathers that input (the hand-off vectors
//     x*g, attention output, h, the QKV slabs) into LDS with sc1 (coherent) DMA;
//   * waves 1-3 are CONSUMERS: they wait on LDS words only (FULL per slot, one per gather),
//     run the MFMAs out of LDS and release slots; results are published with write-through
//     (sc1) stores, drained, then counted on an agent-scope arrival counter (Guideline 16 R1).
//
// Arithmetic: bit-identical to the launches it replaces for these engines -- the split-6 QKV
// GEMV (k_gemv.hip, 8 waves x 1 step per 512-k slab), decode attention v2 with ppb pages per
// split and its combine (k_attn.hip), the O / down GEMVs with the residual + statistics epilogue
// on 12-row tiles (16 waves x 3 / 8 steps) and the gate/up GEMV + SwiGLU (16 waves x 3 steps, 32-row
// tiles).  Every output element is the same MFMA chain per "wave chunk" of K, summed over the
// chunks in the same order (here: in chunk order through an LDS ticket, there: over the waves in
// LDS), with the same epilogue expressions; pages skipped past a sequence's end contribute
// exact zeros there.  tests/test_gpu_persist.py compares the two paths bit for bit.
//
// Work per CU (c = blockIdx.x, 256 CUs): QKV units (16 rows x one 512-k slab; group g's 240 units
// on XCD g's 32 CUs, where the attention items of kv head g run too), attention items (sequence
// b, kv head g, split s) item idx = c + 256 n with idx = s * B * 8 + b * 8 + g, O tile c, gate/up
// tiles c and c + 256, down tile c.  The fp32 residual of tile c's 12 columns lives in LDS for
// the whole step (only this CU updates those columns).
//
// Every wait is bounded: a hand-off that never arrives (a workgroup not resident) sets *err and
// an abort word, every wave then leaves its loops, and the engine recomputes the run with the
// launches (engine.cpp decode_run) -- never a hang.
#include "attn_common.h"
#include "gemv_common.h"

namespace ms {
namespace pk {

constexpr int H = 3072, F = 8192, HQ = 24, HK = 8, G = 3, D = 128;
constexpr int QKVN = (HQ + 2 * HK) * D;  // 5120
constexpr int NCU = 256;
constexpr int NTHR = 256;  // waves 0-1 loaders, waves 2-3 consumers
constexpr int NLD = 2;     // loader waves: one wave issuing LDS DMA tops out at ~14 GB/s per CU, two
                           // reach ~23 (tools/dma_probe.hip, profiles/r06/dma_probe.txt)
constexpr int NCW = 2;
// DMA instructions (KiB) each loader keeps in flight: two loaders at 8 each already stream ~23 GB/s
// per CU (dma_probe), and a deeper queue only delays every other memory operation of the CU (a
// consumer's publish drain, a poll, a gather) behind it -- the CU serves them in order
constexpr int DEPTH = 12;
constexpr int MAXB = 8;
constexpr int R = 6;  // ring slots
constexpr int SLOT = 16384;
constexpr int RT = 12;                // O / down rows per tile (H / NCU)
constexpr int QS = 6;                 // QKV split-K slabs of 512 k
constexpr int QUG = 40 * QS;          // 240 units per kv group (on the 32 CUs of XCD g)
constexpr int PPB_MAX = 9;
// The weights in STREAM order (pack_layer_kernel): every ring slot of a layer is one contiguous
// block whose bytes are already in the slot's LDS order (chunk swizzle applied), so a fill is a
// straight 1-KiB-per-instruction copy -- read in [N][K] order a gate/up slot was 32 pieces of
// 384 B, 6 KiB apart, and streamed at half the rate of a contiguous K / V page
constexpr size_t PK_QKV = (size_t)8 * QUG * 16384;  // [kv group][unit][16 rows x 512 k]
constexpr size_t PK_O = (size_t)NCU * 8 * 9216;      // [cu][slot][12 rows x 384 k]
constexpr size_t PK_GU = (size_t)NCU * 32 * 12288;   // [cu][slot][32 rows x 192 k]
constexpr size_t PK_DN = (size_t)NCU * 16 * 12288;   // [cu][slot][12 rows x 512 k]
constexpr size_t PK_LAYER = PK_QKV + PK_O + PK_GU + PK_DN;

// LDS map (bytes)
constexpr int L_RING = 0;
constexpr int L_X = R * SLOT;               // X image [B][K] / attention scratch / h ring (3 x 16 KiB)
constexpr int XBYTES = 49152;
constexpr int L_SSQ = L_X + XBYTES;         // gate/up statistics stage [256][B] f32
constexpr int L_TOT = L_SSQ + 8192;         // tile totals: [256] gate (or O / down), [256] up
constexpr int L_XRES = L_TOT + 2048;        // residual of this CU's 12 columns [B][12] f32
constexpr int L_GAM = L_XRES + MAXB * RT * 4;  // gains of this CU's columns [layer][2][12] f16
constexpr int MAXL = 28;
constexpr int L_RINV = L_GAM + MAXL * 2 * RT * 2;
constexpr int L_SEQ = L_RINV + 32;          // len[8], slot[8], nsplit[8]
constexpr int L_CTL = L_SEQ + 96;
constexpr int L_PQ = L_CTL + 256;           // each loader's queue of issued fills: end, flag, value
constexpr int PQN = 16;
constexpr int L_END = L_PQ + NLD * PQN * 12;
static_assert(L_END <= 160 * 1024, "LDS");
// attention scratch inside the X region
constexpr int A_SL = 0;                     // gathered QKV slab values [6][(G+2)*128] f32
constexpr int A_RS = A_SL + QS * (G + 2) * D * 4;  // statistics of row b [256] f32
constexpr int A_CS = A_RS + 1024;           // cos [64], sin [64] f32 (+ 512 B DMA spill)
constexpr int A_RAW = A_CS + 1024;          // fp16-rounded sums [(G+2)*128] f32
constexpr int A_QN = A_RAW + (G + 2) * D * 4;  // qn [G][128], kn [128], vn [128] f16
constexpr int A_MW = A_QN + (G + 2) * D * 2;   // per page: [G][130] f32 (m, l, o[128])
constexpr int MWP = G * 130 * 4;
static_assert(A_MW + PPB_MAX * MWP <= XBYTES, "attention scratch");
// control words (ints at L_CTL)
// C_XCNT / C_HCNT count completed HALVES of the split fills (each loader wave adds one per fill);
// C_RDY: the latest chip-wide edge loader 0 saw (4 l + j), which loader 1 waits on instead of polling
enum {
  C_FULL = 0, C_FREE = R, C_XCNT = 2 * R, C_PROSEQ, C_PRODONE, C_ITEMDONE, C_QKVDONE, C_PAGESDONE,
  C_HCNT, C_HFREE = C_HCNT + 3, C_TICK = C_HFREE + 3, C_RINV, C_ABORT, C_LAST, C_RDY, C_NCTL
};
constexpr int kAddOne = -0x7fffffff;  // pending-queue value: atomically add 1 to the flag word
static_assert(C_NCTL * 4 <= 256, "control words");
// global sync words per layer
constexpr int SL = 128;
enum { S_QKV = 0, S_ATT = 8, S_O = 16, S_GU = 24, S_DN = 32, S_TKT = 64 };

constexpr unsigned kLdsSpin = 1u << 23;   // LDS polls (s_sleep 2 each) before giving up
constexpr int kStamps = 16;
__device__ unsigned long long g_pk_stamps[NCU * MAXL * kStamps];
// per-slot trace of one CU in one layer (diagnostic): [slot][0 issue, 1 FULL published, 2 consumer
// saw FULL, 3 consumer released]; layer kTraceLayer of CU 0
constexpr int kTraceLayer = 5, kTraceSlots = 160;
__device__ unsigned long long g_pk_trace[kTraceSlots * 4];
__device__ __forceinline__ void pk_trace(unsigned long long* st, int cu, int slot_rel, int layer, int k) {
  if (st && cu == 0 && layer == kTraceLayer && slot_rel >= 0 && slot_rel < kTraceSlots && (threadIdx.x & 63) == 0)
    g_pk_trace[slot_rel * 4 + k] = __builtin_amdgcn_s_memrealtime();
}
// timeline stamp k of layer l (diagnostic; one lane, s_memrealtime = 100 MHz)
#define PK_STAMP(l, k)                                                                              \
  do {                                                                                              \
    if (a.stamps && lane == 0) a.stamps[((size_t)c * MAXL + (l)) * kStamps + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

}  // namespace pk

namespace pk {

typedef __attribute__((address_space(1))) unsigned gu32_t;
#define PK_CTL(o) (*(volatile int*)(smem + L_CTL + 4 * (o)))

__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ void dma16(const void* src, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS const char*)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"{m0}"(m0), "v"(src) : "memory");
}
// the loader's throttle after each DMA instruction: at most `depth` in flight (wave-uniform; a
// scalar branch per instruction)
__device__ __forceinline__ void throttle(int depth) {
  if (depth <= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (depth <= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (depth <= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (depth <= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (depth <= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
  else if (depth <= 36) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
}
// coherent (sc1) DMA of bytes other workgroups wrote in this launch (behind their counters)
__device__ __forceinline__ void dma16c(const void* src, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS const char*)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1" ::"{m0}"(m0), "v"(src) : "memory");
}
__device__ __forceinline__ void dma4c(const void* src, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS_AS const char*)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dword %1, off sc1" ::"{m0}"(m0), "v"(src) : "memory");
}

// s_waitcnt vmcnt(n) for a run-time n (wave-uniform): the loader knows how many of its DMA
// instructions were issued after the group it waits for
__device__ __forceinline__ void wait_vm(int n) {
  // conservative: waits until at most 4 * floor(n / 4) are outstanding (the group n behind the
  // head, and up to 3 more, have landed); 16 cases keep the inlined copies small
  switch (n < 0 ? 0 : (n > 63 ? 15 : n >> 2)) {
#define PK_W(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k " * 4)" ::: "memory"); break;
    PK_W(0) PK_W(1) PK_W(2) PK_W(3) PK_W(4) PK_W(5) PK_W(6) PK_W(7) PK_W(8) PK_W(9) PK_W(10) PK_W(11)
    PK_W(12) PK_W(13) PK_W(14) PK_W(15)
#undef PK_W
  }
}

// ---------------------------------------------------------------- per-CU schedule
struct Sched {
  int c, B, nq, natt, ns, n_items, nsplit_max;
};
// QKV unit i of CU c: kv group g = c % 8 (XCD-local with that group's attention items), m = c / 8
__device__ __forceinline__ void qkv_unit(int c, int i, int& tile, int& slab, int& grp) {
  grp = c & 7;
  const int u = (c >> 3) + 32 * i;  // < 240
  const int tl = u / QS;
  slab = u - tl * QS;
  tile = tl < 24 ? 24 * grp + tl : (tl < 32 ? 192 + 8 * grp + (tl - 24) : 256 + 8 * grp + (tl - 32));
}
__device__ __forceinline__ int qkv_units(int c) { return ((c >> 3) < QUG - 32 * 7) ? 8 : 7; }

// item idx -> (b, g, s); false when the split is past the sequence
__device__ __forceinline__ bool item_of(const char* smem, int B, int idx, int& b, int& g, int& s) {
  const int BH = B * HK;
  s = idx / BH;
  const int grp = idx - s * BH;
  b = grp / HK;
  g = grp - b * HK;
  const int* nsp = (const int*)(smem + L_SEQ + 64);
  return s < nsp[b];
}
__device__ __forceinline__ int item_pages(const char* smem, int ppb, int b, int s) {
  const int len = ((const int*)(smem + L_SEQ))[b];
  const int np = (len + kPage - 1) / kPage;
  return min(ppb, np - s * ppb);
}

// ---------------------------------------------------------------- waits
__device__ __forceinline__ bool aborted(const char* smem) { return PK_CTL(C_ABORT) != 0; }
__device__ __forceinline__ void set_abort(char* smem, unsigned* err, unsigned code) {
  PK_CTL(C_ABORT) = 1;
  if ((threadIdx.x & 63) == 0) __hip_atomic_store((gu32_t*)err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// consumer wait on an LDS word (>= v); false on abort / timeout
__device__ __forceinline__ bool lds_wait(char* smem, int idx, int v, unsigned* err, unsigned code) {
  for (unsigned it = 0;; ++it) {
    if (PK_CTL(idx) >= v) {
      cbar();
      return true;
    }
    if (aborted(smem)) return false;
    if (it > kLdsSpin) {
      set_abort(smem, err, code);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// ---------------------------------------------------------------- loader
struct Loader {
  char* smem;
  unsigned* err;
  unsigned spin;
  int lane;
  int ldr;     // loader index: issues the ring slots k with k % NLD == ldr and instruction i % NLD == ldr of fills
  int depth;   // DMA instructions kept in flight by the throttle
  int issued;  // DMA instructions issued
  int head, tail;
  int k;         // next ring slot
  int done_end;  // every DMA instruction before this one has landed
  unsigned long long* st;  // diagnostic trace (stamps on)
  int cu, tbase;           // trace: this CU, the traced layer's first slot
  __device__ __forceinline__ int* pq() { return (int*)(smem + L_PQ + ldr * PQN * 12); }
  // keep the wave's outstanding DMA instructions <= 62 (vmcnt is 6 bits) before issuing n more
  __device__ __forceinline__ void make_room(int n) {
    while (head != tail && issued - done_end + n > 62) retire_one();
    if (issued - done_end + n > 62) {  // nothing pending to publish: plain drain
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      done_end = issued;
    }
  }
  __device__ __forceinline__ void push(int flag_idx, int val) {
    int* q = pq();
    const int e = tail & (PQN - 1);
    if (lane == 0) {
      q[3 * e] = issued;
      q[3 * e + 1] = flag_idx;
      q[3 * e + 2] = val;
    }
    tail += 1;
  }
  __device__ __forceinline__ void retire_one() {
    int* q = pq();
    const int e = head & (PQN - 1);
    const int end = __builtin_amdgcn_readfirstlane(q[3 * e]);
    const int fi = __builtin_amdgcn_readfirstlane(q[3 * e + 1]);
    const int val = __builtin_amdgcn_readfirstlane(q[3 * e + 2]);
    wait_vm(issued - end);
    cbar();
    if (lane == 0) {
      if (val == kAddOne) atomicAdd((int*)(smem + L_CTL + 4 * fi), 1);
      else PK_CTL(fi) = val;
    }
    head += 1;
    done_end = end;
    if (fi < R) pk_trace(st, cu, val - tbase, kTraceLayer, 1);
  }
  __device__ __forceinline__ void retire_all() {
    while (head != tail) retire_one();
  }
  // groups at least DEPTH instructions behind the issue head have landed (throttle): publish them
  __device__ __forceinline__ void retire_lag() {
    while (head != tail && issued - __builtin_amdgcn_readfirstlane(pq()[3 * (head & (PQN - 1))]) >= depth) retire_one();
    while (tail - head >= PQN - 2) retire_one();
  }
  // wait until LDS word idx >= v, publishing landed fills meanwhile
  __device__ __forceinline__ bool wait_lds(int idx, int v, unsigned code) {
    for (unsigned it = 0;; ++it) {
      if (PK_CTL(idx) >= v) {
        cbar();
        return true;
      }
      if (aborted(smem)) return false;
      if (head != tail) {
        retire_one();
        continue;
      }
      if (it > kLdsSpin) {
        set_abort(smem, err, code);
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // wait until the n counters p[0..n) are >= target (one lane each, sc1 loads)
  __device__ __forceinline__ bool wait_glb(const unsigned* p, int n, unsigned target, unsigned code) {
    retire_all();  // a poll load waits for every DMA issued before it anyway
    for (unsigned it = 0;; ++it) {
      bool ok = true;
      if (lane < n) ok = __hip_atomic_load((gu32_t*)(p + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__all(ok)) {
        cbar();
        return true;
      }
      if (aborted(smem)) return false;
      if (it >= spin || __hip_atomic_load((gu32_t*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        set_abort(smem, err, code);
        return false;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  // chip-wide edge e (4 l + j): loader 0 polls the n counters at p and publishes e in LDS; loader 1
  // waits for that word (one poller per CU: polling-cost)
  __device__ __forceinline__ bool wait_edge(int e, const unsigned* p, int n, unsigned target, unsigned code) {
    if (ldr == 0) {
      if (p && !wait_glb(p, n, target, code)) return false;
      cbar();
      if (lane == 0) PK_CTL(C_RDY) = e;
      return true;
    }
    return wait_lds(C_RDY, e, code + 0x10);
  }
  // ring slots are owned by parity: the other loader's slots are only counted
  __device__ __forceinline__ bool mine() const { return k % NLD == ldr; }
  __device__ __forceinline__ void skip() { k += 1; }
  // the next ring slot's position is free once slot k - R was released
  __device__ __forceinline__ char* ring_slot() {
    const int pos = k % R;
    wait_lds(C_FREE + pos, k - R, 0x101);
    return smem + L_RING + pos * SLOT;
  }
  __device__ __forceinline__ void ring_done(int ninst) {
    pk_trace(st, cu, k - tbase, kTraceLayer, 0);
    issued += ninst;
    push(C_FULL + k % R, k);
    k += 1;
    retire_lag();
  }
  // a packed weight slot (NI KiB, contiguous, already in LDS order) into the next ring position
  template <int NI>
  __device__ __forceinline__ void w_slot(const char* src) {
    if (!mine()) return skip();
    char* dst = ring_slot();
    if (aborted(smem)) return;
    make_room(NI);
#pragma unroll 4
    for (int i = 0; i < NI; ++i) {
      dma16(src + i * 1024 + lane * 16, dst + i * 1024);
      throttle(depth);
    }
    ring_done(NI);
  }
  // K page (k_swz layout) or V page (v_swz layout, k_attn.hip attn_decode2's DMA mapping)
  __device__ __forceinline__ void kv_slot(const f16_t* base, bool is_v) {
    if (!mine()) return skip();
    char* dst = ring_slot();
    if (aborted(smem)) return;
    make_room(16);
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int rr = 4 * i + (lane >> 4);
      const int ch = is_v ? ((lane & 15) ^ ((rr & 7) << 1)) : ((lane & 15) ^ (rr & 15));
      dma16(base + rr * D + ch * 8, dst + i * 1024);
      throttle(depth);
    }
    ring_done(16);
  }
  // this loader's half of the X image of rows [0, B) x k [k0, k0 + K) of a [B][ld] fp16 matrix
  // (gemv_common.h x_lds layout): instructions i % NLD == ldr.  Not throttled: a hand-off gather
  // sits on the edge's critical path and its coherent (sc1) reads take ~3 us each, so all of them
  // go out at once (one round trip; the weight slots keep DEPTH)
  __device__ __forceinline__ int x_fill(const f16_t* X, int B, int K, int ld, int k0, char* dst) {
    const int kch = K >> 3, n = B * kch, ni = (n + 63) / 64;
    const int mine_n = (ni - ldr + NLD - 1) / NLD;
    make_room(mine_n);
    for (int i = ldr; i < ni; i += NLD) {
      const int P = min(i * 64 + lane, n - 1);
      const int r = P / kch, c = P - r * kch;
      dma16c(X + (size_t)r * ld + k0 + ((c ^ (r & 7)) << 3), dst + i * 1024);
    }
    issued += mine_n;
    return mine_n;
  }
};

// ---------------------------------------------------------------- consumer helpers
__device__ __forceinline__ void lds_release(char* smem, int k) {
  cbar();
  if ((threadIdx.x & 63) == 0) PK_CTL(C_FREE + k % R) = k;
}
#define PK_TR(k_, w_) pk_trace(a.stamps, c, (k_) - kTraceLayer * NSL, kTraceLayer, (w_))
__device__ __forceinline__ f16x8 ldx(const char* xs, int xrow, int k, int K) {
  return *(const f16x8*)(xs + x_lds(xrow, k, K));
}
// weight fragment of slot row r, 16-B chunk C (chunk swizzle of Loader::w_slot)
template <int S>
__device__ __forceinline__ f16x8 ldw(const char* slot, int r, int C) {
  const int p = C ^ ((S % 16 == 0) ? (r & 15) : ((r >> 1) & 7));
  return *(const f16x8*)(slot + r * (S * 16) + (p << 4));
}
// ordered chunk sums: chunk q of a tile is added (tot = tot + acc; the first add is 0 + acc, as
// gemv_epilogue's sum over the waves) once the chunks before it are in
__device__ __forceinline__ bool tick_wait(char* smem, int t, unsigned* err) { return lds_wait(smem, C_TICK, t, err, 0x201); }
__device__ __forceinline__ void tick_add(char* smem, int off, const f32x4& acc, bool first, int lane) {
  f32x4* p = (f32x4*)(smem + off) + lane;
  *p = first ? (f32x4{0.f, 0.f, 0.f, 0.f} + acc) : (*p + acc);
}
__device__ __forceinline__ void tick_next(char* smem) {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's LDS ops are done
  cbar();
  if ((threadIdx.x & 63) == 0) PK_CTL(C_TICK) = PK_CTL(C_TICK) + 1;
}

__device__ __forceinline__ void st_f16_sc1(f16_t* p, f16_t v) {
  __hip_atomic_store((unsigned short*)p, (unsigned short)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_f32_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_f32_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// publish: this wave's sc1 stores are drained, then one lane counts the arrival
__device__ __forceinline__ void arrive(unsigned* p) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add((gu32_t*)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// O / down epilogue (gemv_epilogue RESID_SSQ on a 12-row tile): x += tot, xg = f16(x * g * 2^-4),
// per-tile sums of x^2 -- lanes hold (column c = lane >> 2, row 4 * half + (lane & 3))
__device__ __forceinline__ void resid_epilogue(char* smem, int B, int t, const f16_t* gam, f16_t* xg_out, float* ssq_out) {
  const int lane = threadIdx.x & 63;
  const float* tot = (const float*)(smem + L_TOT);
  float* xres = (float*)(smem + L_XRES);
  for (int half = 0; half < 2; ++half) {
    const int c = lane >> 2, row = 4 * half + (lane & 3), e = 64 * half + lane;
    float q = 0.f;
    if (row < B && c < RT) {
      const float xo = xres[row * RT + c] + tot[e];
      xres[row * RT + c] = xo;
      q = xo * xo;
      float xg = xo * h2f(gam[c]) * kXgScale;
      asm volatile("" : "+v"(xg));
      st_f16_sc1(xg_out + (size_t)row * H + t * RT + c, f2h(xg));
    }
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
    if (c == 0 && row < B) st_f32_sc1(ssq_out + (size_t)t * B + row, q);
  }
}

}  // namespace pk

using namespace pk;

__global__ __launch_bounds__(NTHR, 1) void decode_step_kernel(PkArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = blockIdx.x;
  const int B = a.B;
  const int fr = lane & 15, fg = lane >> 4;
  const int xrow = min(fr, B - 1);

  // ---- setup (every thread): control words, sequence table, residual columns, gains
  if (tid < 64) ((int*)(smem + L_CTL))[tid] = -1;
  if (tid < MAXB) {
    int* sq = (int*)(smem + L_SEQ);
    const int len = tid < B ? a.seq_len[tid] : 0;
    sq[tid] = len;
    sq[8 + tid] = tid < B ? a.seq_slot[tid] : 0;
    const int np = (len + kPage - 1) / kPage;
    sq[16 + tid] = tid < B ? (np + a.ppb - 1) / a.ppb : 0;
  }
  if (tid < B * RT) ((float*)(smem + L_XRES))[tid] = a.x[(size_t)(tid / RT) * H + c * RT + tid % RT];
  for (int i = tid; i < a.L * 2 * RT; i += NTHR) {
    const int l = i / (2 * RT), w = (i / RT) & 1, cc = i % RT;
    const f16_t* gp = w == 0 ? a.layers[l].ffn_norm : a.layers[l].g_next;
    ((f16_t*)(smem + L_GAM))[i] = gp[c * RT + cc];
  }
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < C_NCTL; ++i) PK_CTL(i) = -1;
    for (int p = 0; p < R; ++p) PK_CTL(C_FREE + p) = -1;
    PK_CTL(C_QKVDONE) = 0;
    PK_CTL(C_PAGESDONE) = 0;
    PK_CTL(C_XCNT) = 0;
    for (int p = 0; p < 3; ++p) PK_CTL(C_HFREE + p) = 0;
    for (int p = 0; p < 3; ++p) PK_CTL(C_HCNT + p) = 0;
    PK_CTL(C_TICK) = 0;
    PK_CTL(C_ABORT) = 0;
  }
  __syncthreads();

  // the per-CU schedule (identical in every wave)
  const int* sq = (const int*)(smem + L_SEQ);
  int nsplit_max = 0;
  for (int b = 0; b < B; ++b) nsplit_max = max(nsplit_max, sq[16 + b]);
  const int n_items = nsplit_max * B * HK;
  const int nq = qkv_units(c);
  int natt = 0, nit = 0;
  for (int idx = c; idx < n_items; idx += NCU) {
    int b, g, s;
    if (!item_of(smem, B, idx, b, g, s)) continue;
    natt += 2 * item_pages(smem, a.ppb, b, s);
    nit += 1;
  }
  const int NSL = nq + natt + 8 + 32 + 16;  // ring slots per layer
  const int tiles0 = a.rs0_tiles;

  if (wave < NLD) {
    // ================================================================ loaders
    Loader ld{smem, a.err, a.spin, lane, wave, a.depth, 0, 0, 0, 0, 0, a.stamps, c, kTraceLayer * NSL};
    for (int l = 0; l < a.L && !aborted(smem); ++l) {
      const PkLayer Ly = a.layers[l];
      unsigned* sy = a.sync + (size_t)l * SL;
      if (wave == 0) PK_STAMP(l, 0);
      // -- QKV: unit slots; the X image (xb) once the previous layer's down tiles are all in
      auto x_qkv = [&]() __attribute__((always_inline)) {
        if (!ld.wait_edge(4 * l, l > 0 ? a.sync + (size_t)(l - 1) * SL + S_DN : nullptr, 8, 32, 0x301)) return;
        if (wave == 0) PK_STAMP(l, 1);
        ld.x_fill(a.xb, B, H, H, 0, smem + L_X);
        ld.push(C_XCNT, kAddOne);
        ld.retire_lag();
      };
      for (int i = 0; i < nq; ++i) {
        if (i == min(R, nq)) x_qkv();
        int tile, slab, grp;
        qkv_unit(c, i, tile, slab, grp);
        ld.w_slot<16>(Ly.packed + ((size_t)(c & 7) * QUG + (c >> 3) + 32 * i) * 16384);
        (void)tile;
        (void)slab;
        (void)grp;
      }
      if (nq <= R) x_qkv();
      // -- attention items: K / V page slots; the item's QKV slab values (loader 0) once its group is in
      int it_ord = l * nit;
      for (int idx = c; idx < n_items; idx += NCU) {
        int b, g, s;
        if (!item_of(smem, B, idx, b, g, s)) continue;
        const int npg = item_pages(smem, a.ppb, b, s);
        const int slot = sq[8 + b], len = sq[b], pos = len - 1;
        auto gather = [&]() __attribute__((always_inline)) {
          if (wave != 0) return;
          // this CU's QKV units are done with the X image, and the previous item's prologue with
          // the slab area; then the group's 240 QKV units
          if (!ld.wait_lds(C_QKVDONE, nq * (l + 1), 0x102)) return;
          if (!ld.wait_lds(C_PRODONE, it_ord - 1, 0x103)) return;
          if (!ld.wait_glb(sy + S_QKV + g, 1, 32 * NCW, 0x302)) return;
          PK_STAMP(l, 2);
          char* ax = smem + L_X;
          const int tiles = l == 0 ? tiles0 : NCU;
          const int nrs = (tiles + 63) / 64;
          ld.make_room(15 + nrs + 1);
          // slab values: 6 x 640 floats, 4 per lane
#pragma unroll 3
          for (int i = 0; i < 15; ++i) {
            const int E = i * 256 + lane * 4, sl = E / 640, e = E - sl * 640;
            const int hh = e >> 7, j = e & 127;
            const int col = hh < G ? (g * G + hh) * D + j : (hh == G ? (HQ + g) * D + j : (HQ + HK + g) * D + j);
            dma16c(a.slabs + ((size_t)sl * B + b) * QKVN + col, ax + A_SL + i * 1024);
          }
          for (int i = 0; i < nrs; ++i)
            dma4c(a.ssq + (size_t)min(i * 64 + lane, tiles - 1) * B + b, ax + A_RS + i * 256);
          {
            const float* tab = lane < 16 ? a.cos_tab : a.sin_tab;
            dma16(tab + (size_t)pos * 64 + (lane & 15) * 4, ax + A_CS);
          }
          ld.issued += 15 + nrs + 1;
          ld.push(C_PROSEQ, it_ord);
        };
        const size_t pb0 = ((size_t)slot * a.max_pages + (size_t)s * a.ppb) * HK + g;
        for (int w = 0; w < 2 * npg; ++w) {
          if (w == min(R, 2 * npg)) gather();
          const size_t pbase = (pb0 + (size_t)(w >> 1) * HK) * kPage * D;
          ld.kv_slot(((w & 1) ? Ly.vc : Ly.kc) + pbase, w & 1);
        }
        if (2 * npg <= R) gather();
        it_ord += 1;
      }
      // -- O: tile c, 8 slots of 2 chunks; the attention output once every (b, g) is in
      for (int j = 0; j < 8; ++j) {
        if (j == min(R, 8)) {
          if (ld.wait_edge(4 * l + 1, sy + S_ATT, 1, (unsigned)(B * HK), 0x303)) {
            if (wave == 0) PK_STAMP(l, 3);
            ld.x_fill(a.attn, B, H, H, 0, smem + L_X);
            ld.push(C_XCNT, kAddOne);
            ld.retire_lag();
          }
        }
        ld.w_slot<9>(Ly.packed + PK_QKV + ((size_t)c * 8 + j) * 9216);
      }
      // -- gate/up: tiles c, c + 256, 16 chunks each; xg2 + statistics once every O tile is in
      for (int j = 0; j < 32; ++j) {
        if (j == R) {
          if (ld.wait_edge(4 * l + 2, sy + S_O, 8, 32, 0x304)) {
            if (wave == 0) PK_STAMP(l, 4);
            ld.x_fill(a.xg2, B, H, H, 0, smem + L_X);
            const int mine_b = (B - wave + NLD - 1) / NLD;
            ld.make_room(mine_b);
            for (int i = wave; i < B; i += NLD) dma16c(a.ssq2 + i * 256 + lane * 4, smem + L_SSQ + i * 1024);
            ld.issued += mine_b;
            ld.push(C_XCNT, kAddOne);
          }
        }
        ld.w_slot<12>(Ly.packed + PK_QKV + PK_O + ((size_t)c * 32 + j) * 12288);
      }
      // -- down: tile c, 16 chunks of 512 k; h through the 3-slot ring in the X region
      auto h_slot = [&](int i) __attribute__((always_inline)) {  // h columns [1024 i, +1024)
        const int hi = l * 8 + i, pos = hi % 3;
        if (!ld.wait_lds(C_HFREE + pos, 2 * (hi / 3), 0x104)) return;
        ld.x_fill(a.hbuf, B, 1024, F, 1024 * i, smem + L_X + pos * 16384);
        ld.push(C_HCNT + pos, kAddOne);
      };
      for (int j = 0; j < 16; ++j) {
        if (j == R) {
          if (ld.wait_edge(4 * l + 3, sy + S_GU, 8, 64, 0x305)) {
            if (wave == 0) PK_STAMP(l, 5);
            h_slot(0);
            h_slot(1);
            h_slot(2);
          }
        }
        if (j >= R && !(j & 1) && j / 2 >= 3) h_slot(j / 2);
        ld.w_slot<12>(Ly.packed + PK_QKV + PK_O + PK_GU + ((size_t)c * 16 + j) * 12288);
      }
      if (wave == 0) PK_STAMP(l, 6);
    }
    ld.retire_all();
  } else {
    // ================================================================ consumers
    const int cw = wave - NLD;
    int tick0 = 0;   // ordered chunks before this tile
    int pages_cum = 0;
    for (int l = 0; l < a.L && !aborted(smem); ++l) {
      const PkLayer Ly = a.layers[l];
      unsigned* sy = a.sync + (size_t)l * SL;
      const int base = l * NSL;
      const char* xs = smem + L_X;
      // ---------------- QKV units
      int ndone = 0;
      for (int i = cw; i < nq; i += NCW) {
        const int k = base + i;
        if (!lds_wait(smem, C_XCNT, NLD * (3 * l + 1), a.err, 0x401)) break;
        if (!lds_wait(smem, C_FULL + k % R, k, a.err, 0x402)) break;
        PK_TR(k, 2);
        int tile, slab, grp;
        qkv_unit(c, i, tile, slab, grp);
        const char* sl = smem + L_RING + (k % R) * SLOT;
        f32x4 tot = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const int kx = slab * 512 + 64 * st + 16 * fg;
          const f16x8 x0 = ldx(xs, xrow, kx, H), x1 = ldx(xs, xrow, kx + 8, H);
          const int c0 = 8 * st + 2 * fg;
          const f16x8 w0 = ldw<64>(sl, fr, c0), w1 = ldw<64>(sl, fr, c0 + 1);
          f32x4 p = {0.f, 0.f, 0.f, 0.f};
          p = mfma16(x0, w0, p);
          p = mfma16(x1, w1, p);
          tot = tot + p;
        }
        PK_TR(k, 3);
        lds_release(smem, k);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int b = 4 * fg + jj;
          if (b < B) st_f32_sc1(a.slabs + ((size_t)slab * B + b) * QKVN + 16 * tile + fr, tot[jj]);
        }
        ndone += 1;
      }
      // one arrival per consumer wave after all its units (every unit of CU c is kv group c % 8):
      // the group is complete only with its last unit anyway, and each drain waits behind the
      // CU's in-flight DMA
      if (ndone) arrive(sy + S_QKV + (c & 7));
      if (lane == 0 && ndone) atomicAdd((int*)(smem + L_CTL + 4 * C_QKVDONE), ndone);
      PK_STAMP(l, 7 + (cw == 0 ? 0 : 8));
      // ---------------- attention items
      int k = base + nq;
      int it_ord = l * nit;
      char* ax = smem + L_X;
      f16_t* qn = (f16_t*)(ax + A_QN);
      f16_t* kn = qn + G * D;
      f16_t* vn = kn + D;
      for (int idx = c; idx < n_items && !aborted(smem); idx += NCU) {
        int b, g, s;
        if (!item_of(smem, B, idx, b, g, s)) continue;
        const int npg = item_pages(smem, a.ppb, b, s);
        const int len = sq[b], slot = sq[8 + b], nsb = sq[16 + b];
        const int pos = len - 1, np = (len + kPage - 1) / kPage;
        const bool owns_new = (pos / kPage) / a.ppb == s;
        // prologue (consumer 0): fold the slabs, the row scale, RoPE -> qn / kn / vn; the owner
        // writes the new token's K / V (k_attn.hip attn_decode2's arithmetic)
        if (cw == 0 && lds_wait(smem, C_PROSEQ, it_ord, a.err, 0x403)) {
          const float* slv = (const float*)(ax + A_SL);
          const float* rsv = (const float*)(ax + A_RS);
          const float* cs = (const float*)(ax + A_CS);
          float* raw = (float*)(ax + A_RAW);
          const int tiles = l == 0 ? tiles0 : NCU;
          float rv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) rv[i] = (lane + 64 * i < tiles) ? rsv[lane + 64 * i] : 0.f;
          const float rsum = ((rv[0] + rv[1]) + rv[2]) + rv[3];
          const RowScale rs{nullptr, tiles, H, a.eps, a.inv_h};
          const float rrow = rs_rinv(wave_sum(rsum), rs);
          const int nvec = (G + (owns_new ? 2 : 0)) * D;
          for (int e = lane; e < nvec; e += 64) {
            float acc = slv[e];
#pragma unroll
            for (int q = 1; q < QS; ++q) acc += slv[q * (G + 2) * D + e];
            raw[e] = h2f(f2h(acc * rrow));
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_wave_barrier();
          const float rcs = cs[lane], rsn = cs[64 + lane];
          const int nh = G + (owns_new ? 1 : 0);
          for (int hh = 0; hh < nh; ++hh) {
            const float lo = raw[hh * D + rope_perm(lane)], hi = raw[hh * D + rope_perm(64 + lane)];
            const float ra = __fsub_rn(__fmul_rn(lo, rcs), __fmul_rn(hi, rsn));
            const float rb = __fadd_rn(__fmul_rn(hi, rcs), __fmul_rn(lo, rsn));
            f16_t* dst = hh < G ? qn + hh * D : kn;
            dst[lane] = f2h(ra);
            dst[64 + lane] = f2h(rb);
          }
          if (owns_new) {
            vn[lane] = f2h(raw[(G + 1) * D + lane]);
            vn[64 + lane] = f2h(raw[(G + 1) * D + 64 + lane]);
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_wave_barrier();
          if (owns_new) {
            const size_t o0 = ((((size_t)slot * a.max_pages + pos / kPage) * HK + g) * kPage + pos % kPage) * D;
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              Ly.kc[o0 + lane + 64 * h2] = kn[lane + 64 * h2];
              Ly.vc[o0 + lane + 64 * h2] = vn[lane + 64 * h2];
            }
          }
          cbar();
          if (lane == 0) PK_CTL(C_PRODONE) = it_ord;
          PK_STAMP(l, 8);
        }
        // pages (page w of the split by consumer w % 3)
        for (int w = cw; w < npg; w += NCW) {
          if (!lds_wait(smem, C_PRODONE, it_ord, a.err, 0x404)) break;
          const int kk = k + 2 * w, kv = kk + 1;
          if (!lds_wait(smem, C_FULL + kk % R, kk, a.err, 0x405)) break;
          PK_TR(kk, 2);
          if (!lds_wait(smem, C_FULL + kv % R, kv, a.err, 0x406)) break;
          PK_TR(kv, 2);
          const char* ks = smem + L_RING + (kk % R) * SLOT;
          char* vs = smem + L_RING + (kv % R) * SLOT;
          const int pg = s * a.ppb + w;
          const int r = fr, gq = fg;
          const int hl = min(r, G - 1);
          f16x8 qf[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *(const f16x8*)(qn + hl * D + 32 * s4 + 8 * gq);
          u32x4 kf[4][4];
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) kf[mt][s4] = *(const u32x4*)(ks + k_swz(mt * 16 + r, 4 * s4 + gq));
          const int off = pos % kPage;
          const bool patch = pg == pos / kPage;
          if (patch) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
              for (int s4 = 0; s4 < 4; ++s4)
                if (mt * 16 + r == off) kf[mt][s4] = *(const u32x4*)(kn + 32 * s4 + 8 * gq);
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
              const int key = pg * kPage + mt * 16 + 4 * gq + j;
              const float v = (key >= len) ? -INFINITY : sc[mt][j] * a.scale_log2;
              sc[mt][j] = v;
              mx = fmaxf(mx, v);
            }
          mx = grp_max(mx);
          float rsm = 0.f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float p = (sc[mt][j] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sc[mt][j] - mx);
              sc[mt][j] = p;
              rsm += p;
            }
          const float l_run = grp_sum(rsm);
          const float m_run = mx;
          if (pg == np - 1) {
            const int first = len - pg * kPage;
            for (int e = first * 16 + lane; e < 64 * 16; e += 64) *(u32x4*)(vs + v_swz(e >> 4, e & 15)) = u32x4{0, 0, 0, 0};
          }
          if (patch && lane < 16) *(u32x4*)(vs + v_swz(off, lane)) = *(const u32x4*)(vn + lane * 8);
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_wave_barrier();
          f32x4 o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kstep = 0; kstep < 2; ++kstep) {
            const f16x8 pf = pack_p(sc[2 * kstep], sc[2 * kstep + 1]);
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) o[dt] = mfma16(load_vt(vs, dt, kstep, lane), pf, o[dt]);
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          PK_TR(kk, 3);
          lds_release(smem, kk);
          PK_TR(kv, 3);
          lds_release(smem, kv);
          float* mw = (float*)(ax + A_MW + w * MWP);
          if (r < G) {
            if (gq == 0) {
              mw[r * 130 + 0] = m_run;
              mw[r * 130 + 1] = l_run;
            }
#pragma unroll
            for (int dt = 0; dt < 8; ++dt)
#pragma unroll
              for (int j = 0; j < 4; ++j) mw[r * 130 + 2 + dt * 16 + 4 * gq + j] = o[dt][j];
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          cbar();
          if (lane == 0) atomicAdd((int*)(smem + L_CTL + 4 * C_PAGESDONE), 1);
        }
        pages_cum += npg;
        // merge (consumer 0): pages in order, then the split partial / output
        if (cw == 0 && lds_wait(smem, C_PAGESDONE, pages_cum, a.err, 0x407)) {
          const int grp = b * HK + g;
          for (int id = lane; id < G * 130; id += 64) {
            const int cc = id / 130, kq = id - cc * 130;
            float M = -INFINITY;
            for (int w = 0; w < npg; ++w) M = fmaxf(M, ((const float*)(ax + A_MW + w * MWP))[cc * 130]);
            float acc = 0.f, Lsum = 0.f;
            for (int w = 0; w < npg; ++w) {
              const float* mw = (const float*)(ax + A_MW + w * MWP);
              const float m_w = mw[cc * 130];
              const float f = (m_w == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_w - M);
              acc += (kq == 0) ? 0.f : f * mw[cc * 130 + kq];
              Lsum += f * mw[cc * 130 + 1];
            }
            if (nsb == 1) {
              if (kq >= 2) st_f16_sc1(a.attn + (size_t)b * HQ * D + (g * G + cc) * D + (kq - 2), f2h(acc / Lsum));
            } else {
              st_f32_sc1(a.ws + (((size_t)b * HQ + g * G + cc) * a.nsplit_ws + s) * 132 + kq, kq == 0 ? M : acc);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          bool last = nsb == 1;
          if (nsb > 1) {
            unsigned old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add((gu32_t*)(sy + S_TKT + grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            old = __builtin_amdgcn_readfirstlane(old);
            last = old == (unsigned)(nsb - 1);
            if (last) {
              // (attn_decode_combine_kernel's arithmetic; every partial this lane needs is loaded
              // before the first is used: the loads queue behind the CU's DMA, one round trip)
              constexpr int QM = 8;
              for (int id = lane; id < G * D; id += 64) {
                const int cc = id >> 7, d = id & 127;
                const float* p = a.ws + ((size_t)b * HQ + g * G + cc) * a.nsplit_ws * 132;
                float mq[QM], lq[QM], oq[QM];
#pragma unroll
                for (int q = 0; q < QM; ++q) {
                  const int qq = min(q, nsb - 1);
                  mq[q] = ld_f32_sc1(p + qq * 132);
                  lq[q] = ld_f32_sc1(p + qq * 132 + 1);
                  oq[q] = ld_f32_sc1(p + qq * 132 + 2 + d);
                }
                float M = -INFINITY;
                for (int q = 0; q < nsb; ++q) M = fmaxf(M, q < QM ? mq[q] : ld_f32_sc1(p + q * 132));
                float Lq = 0.f, O = 0.f;
                for (int q = 0; q < nsb; ++q) {
                  const float m_q = q < QM ? mq[q] : ld_f32_sc1(p + q * 132);
                  const float f = m_q == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_q - M);
                  Lq += f * (q < QM ? lq[q] : ld_f32_sc1(p + q * 132 + 1));
                  O += f * (q < QM ? oq[q] : ld_f32_sc1(p + q * 132 + 2 + d));
                }
                st_f16_sc1(a.attn + (size_t)b * HQ * D + (g * G + cc) * D + d, f2h(O / Lq));
              }
            }
          }
          if (last) arrive(sy + S_ATT);
          cbar();
          if (lane == 0) PK_CTL(C_ITEMDONE) = it_ord;
          PK_STAMP(l, 9);
        }
        k += 2 * npg;
        it_ord += 1;
      }
      // ---------------- O tile c: 8 slots x 2 chunks (3 steps each)
      const f16_t* gam = (const f16_t*)(smem + L_GAM) + l * 2 * RT;
      for (int j = cw; j < 8; j += NCW) {
        const int kk = base + nq + natt + j;
        if (!lds_wait(smem, C_XCNT, NLD * (3 * l + 2), a.err, 0x411)) break;
        if (!lds_wait(smem, C_FULL + kk % R, kk, a.err, 0x412)) break;
        PK_TR(kk, 2);
        const char* sl = smem + L_RING + (kk % R) * SLOT;
        const int wr = min(fr, RT - 1);
        f32x4 acc[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          acc[h2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int st = 3 * h2 + u;
            const int kx = 384 * j + 64 * st + 16 * fg;
            const f16x8 x0 = ldx(xs, xrow, kx, H), x1 = ldx(xs, xrow, kx + 8, H);
            const int c0 = 8 * st + 2 * fg;
            acc[h2] = mfma16(x0, ldw<48>(sl, wr, c0), acc[h2]);
            acc[h2] = mfma16(x1, ldw<48>(sl, wr, c0 + 1), acc[h2]);
          }
        }
        PK_TR(kk, 3);
        lds_release(smem, kk);
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int q = 2 * j + h2;
          if (!tick_wait(smem, tick0 + q, a.err)) break;
          tick_add(smem, L_TOT, acc[h2], q == 0, lane);
          if (q == 15) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            resid_epilogue(smem, B, c, gam, a.xg2, a.ssq2);
            arrive(sy + S_O + (c & 7));
            PK_STAMP(l, 10);
          }
          tick_next(smem);
        }
      }
      tick0 += 16;
      // ---------------- gate/up tiles c, c + 256: 32 slots of one chunk (3 steps)
      if (cw == 0 && lds_wait(smem, C_XCNT, NLD * (3 * l + 3), a.err, 0x421)) {
        // the rows' deferred-norm factors from the 256 statistics tiles (gemv_common.h rs_finish)
        const float* st = (const float*)(smem + L_SSQ);
        const RowScale rs{nullptr, NCU, H, a.eps, a.inv_h};
        for (int row = 0; row < B; ++row) {
          float sum = 0.f;
          for (int t = lane; t < NCU; t += 64) sum += st[t * B + row];
          sum = wave_sum(sum);
          if (lane == 0) ((float*)(smem + L_RINV))[row] = rs_rinv(sum, rs);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        cbar();
        if (lane == 0) PK_CTL(C_RINV) = l;
      }
      for (int j = cw; j < 32; j += NCW) {
        const int kk = base + nq + natt + 8 + j;
        if (!lds_wait(smem, C_XCNT, NLD * (3 * l + 3), a.err, 0x422)) break;
        if (!lds_wait(smem, C_FULL + kk % R, kk, a.err, 0x423)) break;
        PK_TR(kk, 2);
        const char* sl = smem + L_RING + (kk % R) * SLOT;
        const int q = j & 15;
        f32x4 ag = {0.f, 0.f, 0.f, 0.f}, au = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int kx = 192 * q + 64 * u + 16 * fg;
          const f16x8 x0 = ldx(xs, xrow, kx, H), x1 = ldx(xs, xrow, kx + 8, H);
          const int c0 = 8 * u + 2 * fg;
          ag = mfma16(x0, ldw<24>(sl, fr, c0), ag);
          ag = mfma16(x1, ldw<24>(sl, fr, c0 + 1), ag);
          au = mfma16(x0, ldw<24>(sl, 16 + fr, c0), au);
          au = mfma16(x1, ldw<24>(sl, 16 + fr, c0 + 1), au);
        }
        PK_TR(kk, 3);
        lds_release(smem, kk);
        if (!tick_wait(smem, tick0 + j, a.err)) break;
        tick_add(smem, L_TOT, ag, q == 0, lane);
        tick_add(smem, L_TOT + 1024, au, q == 0, lane);
        if (q == 15) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          if (!lds_wait(smem, C_RINV, l, a.err, 0x424)) break;
          const float* tg_ = (const float*)(smem + L_TOT);
          const float* tu_ = (const float*)(smem + L_TOT + 1024);
          const float* rinv = (const float*)(smem + L_RINV);
          const int tg = c + NCU * (j >> 4);
          for (int e = lane; e < 128; e += 64) {
            const int ll = (e >> 2) & 63, jj = e & 3;
            const int row = 4 * (ll >> 4) + jj;
            if (row >= B) continue;
            const float rv = rinv[row];
            const float gv = tg_[e] * rv;
            const float uv = tu_[e] * rv;
            const int f = tg * 16 + (ll & 15);
            st_f16_sc1(a.hbuf + (size_t)row * F + f, f2h(gv / (1.0f + __expf(-gv)) * uv));
          }
          arrive(sy + S_GU + (c & 7));
          PK_STAMP(l, 11 + (j >> 4));
        }
        tick_next(smem);
      }
      tick0 += 32;
      // ---------------- down tile c: 16 slots of one chunk (8 steps); h from the X ring
      for (int j = cw; j < 16; j += NCW) {
        const int kk = base + nq + natt + 40 + j;
        const int hi = l * 8 + j / 2, hp = hi % 3;
        if (!lds_wait(smem, C_HCNT + hp, NLD * (hi / 3 + 1), a.err, 0x431)) break;
        if (!lds_wait(smem, C_FULL + kk % R, kk, a.err, 0x432)) break;
        PK_TR(kk, 2);
        const char* sl = smem + L_RING + (kk % R) * SLOT;
        const char* hs = smem + L_X + hp * 16384;
        const int wr = min(fr, RT - 1);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int kx = 512 * (j & 1) + 64 * u + 16 * fg;
          const f16x8 x0 = ldx(hs, xrow, kx, 1024), x1 = ldx(hs, xrow, kx + 8, 1024);
          const int c0 = 8 * u + 2 * fg;
          acc = mfma16(x0, ldw<64>(sl, wr, c0), acc);
          acc = mfma16(x1, ldw<64>(sl, wr, c0 + 1), acc);
        }
        PK_TR(kk, 3);
        lds_release(smem, kk);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        cbar();
        if (lane == 0) atomicAdd((int*)(smem + L_CTL + 4 * (C_HFREE + hp)), 1);
        if (!tick_wait(smem, tick0 + j, a.err)) break;
        tick_add(smem, L_TOT, acc, j == 0, lane);
        if (j == 15) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          resid_epilogue(smem, B, c, gam + RT, a.xb, a.ssq);
          arrive(sy + S_DN + (c & 7));
          PK_STAMP(l, 13);
        }
        tick_next(smem);
      }
      tick0 += 16;
    }
  }

  // ---- end: the residual columns back, then the last workgroup out resets the counters
  __syncthreads();
  if (tid < B * RT) a.x[(size_t)(tid / RT) * H + c * RT + tid % RT] = ((const float*)(smem + L_XRES))[tid];
  if (tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old =
        __hip_atomic_fetch_add((gu32_t*)(a.sync + (size_t)a.L * SL), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool bad = __hip_atomic_load((gu32_t*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    PK_CTL(C_LAST) = (old == NCU - 1 && !bad) ? 1 : 0;
  }
  __syncthreads();
  if (PK_CTL(C_LAST) == 1)
    for (int i = tid; i <= a.L * SL; i += NTHR) __hip_atomic_store((gu32_t*)(a.sync + i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- stream layout
// one 16-B chunk of the packed layer per thread: slot bytes in the LDS order Loader::w_slot's
// consumers read (ldw<S>: chunk C of row r at position C ^ (S % 16 ? (r >> 1) & 7 : r & 15))
__global__ __launch_bounds__(256) void pack_layer_kernel(const f16_t* __restrict__ wqkv, const f16_t* __restrict__ wo,
                                                         const f16_t* __restrict__ wgu, const f16_t* __restrict__ wdown,
                                                         char* __restrict__ out) {
  const size_t X = (size_t)blockIdx.x * 256 + threadIdx.x;  // output chunk
  if (X >= PK_LAYER / 16) return;
  size_t x = X * 16;
  const f16_t* src;
  if (x < PK_QKV) {
    const int slot = (int)(x / 16384), P = (int)(x % 16384) / 16;
    const int g = slot / QUG, u = slot % QUG, tl = u / QS, slab = u % QS;
    const int tile = tl < 24 ? 24 * g + tl : (tl < 32 ? 192 + 8 * g + (tl - 24) : 256 + 8 * g + (tl - 32));
    const int r = P / 64, ch = P % 64, C = ch ^ (r & 15);
    src = wqkv + (size_t)(16 * tile + r) * H + slab * 512 + C * 8;
  } else if ((x -= PK_QKV) < PK_O) {
    const int slot = (int)(x / 9216), P = (int)(x % 9216) / 16;
    const int cu = slot / 8, j = slot % 8;
    const int r = P / 48, ch = P % 48, C = ch ^ (r & 15);
    src = wo + (size_t)(RT * cu + r) * H + 384 * j + C * 8;
  } else if ((x -= PK_O) < PK_GU) {
    const int slot = (int)(x / 12288), P = (int)(x % 12288) / 16;
    const int cu = slot / 32, j = slot % 32, tg = cu + NCU * (j >> 4);
    const int r = P / 24, ch = P % 24, C = ch ^ ((r >> 1) & 7);
    src = wgu + (size_t)(32 * tg + r) * H + 192 * (j & 15) + C * 8;
  } else {
    x -= PK_GU;
    const int slot = (int)(x / 12288), P = (int)(x % 12288) / 16;
    const int cu = slot / 16, j = slot % 16;
    const int r = P / 64, ch = P % 64, C = ch ^ (r & 15);
    src = wdown + (size_t)(RT * cu + r) * F + 512 * j + C * 8;
  }
  *(uint4*)(out + X * 16) = *(const uint4*)src;
}

size_t persist_packed_bytes_per_layer() { return PK_LAYER; }

void launch_pack_layer(const f16_t* wqkv, const f16_t* wo, const f16_t* wgu, const f16_t* wdown, void* out,
                       hipStream_t s) {
  const size_t n = PK_LAYER / 16;
  MS_LAUNCH(pack_layer_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, wqkv, wo, wgu, wdown, (char*)out);
}

// ---------------------------------------------------------------- host
size_t persist_sync_words(int L) { return (size_t)L * SL + 1; }

bool persist_supported(int max_batch, int H_, int F_, int Hq, int Hk, int Dh, int L, int ppb, int n_cu) {
  return max_batch >= 1 && max_batch <= MAXB && H_ == H && F_ == F && Hq == HQ && Hk == HK && Dh == D && L >= 1 &&
         L <= MAXL && ppb >= 1 && ppb <= PPB_MAX && n_cu == NCU;
}

void launch_decode_step(const PkArgs& a, hipStream_t s) {
  if (a.B < 1 || a.B > MAXB || a.L < 1 || a.L > MAXL) return;  // callers check persist_supported
  // MS_PK_SPIN (tests; read per launch, a captured graph keeps it): 0 makes every hand-off that is
  // not ready at its first poll give up
  const char* e = getenv("MS_PK_SPIN");
  PkArgs b = a;
  b.spin = e ? (unsigned)strtoul(e, nullptr, 10) : (1u << 19);
  const char* dv = getenv("MS_PK_DEPTH");  // DMA instructions in flight per loader wave (tuning)
  b.depth = dv ? std::max(4, std::min(44, atoi(dv))) : DEPTH;
  static unsigned long long* stamps = [] {
    const char* e = getenv("MS_PK_STAMPS");
    void* p = nullptr;
    if (e && atoi(e)) (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_pk_stamps));
    return (unsigned long long*)p;
  }();
  b.stamps = stamps;
  MS_LAUNCH(decode_step_kernel, dim3(NCU), dim3(NTHR), L_END, s, b);
}

void persist_stamps(unsigned long long* host, int n) {
  // [0, NCU * MAXL * kStamps): the per-CU phase stamps; then the per-slot trace [kTraceSlots][4]
  const int ns = std::min(n, NCU * MAXL * kStamps);
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pk_stamps), (size_t)ns * sizeof(unsigned long long));
  if (n > NCU * MAXL * kStamps)
    (void)hipMemcpyFromSymbol(host + ns, HIP_SYMBOL(g_pk_trace),
                              (size_t)std::min(n - ns, kTraceSlots * 4) * sizeof(unsigned long long));
}

}  // namespace ms
