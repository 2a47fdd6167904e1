// engine.cpp -- libmapsum: the map-phase engine behind the C-ABI of include/mapsum.h.
//
// One engine = one GPU = one process.  It replaces, for every chunk the map node
// sends (runners/run_summarization_ollama_mapreduce.py:103-106 ->
// run_full_evaluation_pipeline.py:80-106 -> POST /api/generate), what Ollama does
// with the prompt ids: prefill, greedy decode until an end-of-turn id or
// num_predict.  Unlike the reference, whose blocking
// _acall (run_full_evaluation_pipeline.py:108-109) serialises the map fan-out,
// every submitted chunk joins one continuous batch:
//   ms_step = admit waiting chunks (slot + KV pages reserved for prompt+num_predict)
//             -> one packed varlen prefill pass over all admitted prompts
//             -> one decode step for every running sequence.
// Device memory is laid out once at ms_create for the configured max batch:
// fp16 weights (Q|K|V fused, gate/up interleaved per 16 rows), a paged fp16 KV
// pool [layer][page][kv_head][64][128], fp32 residual stream, fp16 activations.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <array>
#include <functional>
#include <map>
#include <tuple>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#if MS_HAVE_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#else  // no rocprofiler-sdk-roctx: the trace ranges compile to nothing
static inline int roctxRangePushA(const char*) { return 0; }
static inline int roctxRangePop() { return 0; }
#endif

#include "kernels.h"
#include "mapsum.h"

using namespace ms;

namespace {

thread_local std::string g_last_error;

// roctx ranges around the scheduler's phases (SURVEY.md §5 tracing): rocprofv3 --marker-trace
// separates admission, the packed prefill and each decode run on the timeline (host ranges;
// both phases end with a stream synchronisation, so they bracket the device work)
struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

struct MsError : std::runtime_error {
  int code;
  MsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_OK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw MsError(MS_EIO, std::string(#expr) + ": " + hipGetErrorString(e_));             \
  } while (0)

#define REQUIRE(cond, code, msg)                      \
  do {                                                \
    if (!(cond)) throw MsError((code), (msg));        \
  } while (0)

enum KClass { K_GEMM = 0, K_ATTN_PREFILL = 1, K_GEMV = 2, K_ATTN_DECODE = 3, K_LMHEAD = 4, K_MISC = 5, K_PERSIST = 6 };

struct Seq {
  uint64_t tag = 0;
  std::vector<int32_t> prompt;
  int32_t num_predict = 0;
  uint32_t flags = 0;
  int slot = -1;
  int len = 0;  // tokens whose K/V are in the cache
  std::vector<int32_t> out;
  std::vector<int32_t> pages;
  int finish = 0;
  // teacher forcing (ms_submit_forced, parity tests): decode step j is fed forced[j-1]
  // instead of the sequence's own previous choice; `out` keeps the engine's choices
  std::vector<int32_t> forced;
  int32_t next_input() const { return forced.empty() ? out.back() : forced[out.size() - 1]; }
};

struct Layer {
  f16_t *attn_norm = nullptr, *wqkv = nullptr, *wo = nullptr, *ffn_norm = nullptr,
         *wgu = nullptr, *wdown = nullptr;
};

// Quantised (ggml K-quant) copy of one fused matrix for the decode GEMV; `need` = the
// logical tensors that must all be loaded quantised before decode uses it.
struct QSlot {
  QMat m{};
  size_t bytes[3] = {0, 0, 0};  // device bytes of each region (weight broadcast)
  uint32_t loaded = 0, need = 0;
  bool ready() const { return need != 0 && loaded == need; }
};
enum { QS_QKV = 0, QS_O = 1, QS_GU = 2, QS_DOWN = 3 };

}  // namespace

struct ms_engine {
  ms_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  int H = 0, Hq = 0, Hk = 0, D = 128, F = 0, V = 0, L = 0, QKVN = 0;
  int max_pages = 0, n_pages = 0, Tmax = 0;
  bool slot_major = false;  // pool of max_batch x max_pages: slot s owns pages [s*max_pages, +max_pages)
  std::vector<void*> allocs;
  std::vector<Layer> layers;
  std::vector<std::array<QSlot, 4>> lq;  // per layer: QKV, O, gate/up, down
  QSlot lmq;                             // lm_head (the tied embedding when tie_embeddings)
  f16_t *embed = nullptr, *final_norm = nullptr, *lm_head = nullptr;
  float *cos_tab = nullptr, *sin_tab = nullptr;
  f16_t *kpool = nullptr, *vpool = nullptr;
  size_t layer_kv_elems = 0;
  int32_t* bt_d = nullptr;
  int32_t* bt_h = nullptr;  // pinned host copy of the block table (async row uploads)
  std::vector<int> free_pages, free_slots;
  float* x = nullptr;
  float* ssq = nullptr;
  f16_t *xb = nullptr, *qkv = nullptr, *attn = nullptr, *hbuf = nullptr;
  float* logits = nullptr;
  int32_t* ids_out_d = nullptr;
  void* gemv_ws = nullptr;
  float* attn_ws = nullptr;
  // decode O / down projections: split-K partial slabs [S][B][H] fp32, folded into the
  // residual by the next residual_rmsnorm launch (pending_split = S of the unfolded slabs)
  float* slabs = nullptr;
  int split_qkv = 6, split_o = 6, split_down = 4, pending_split = 0;
  // large-batch regime (BASELINE configs[2]): QKV / O / down / gate-up / lm_head on the skinny
  // GEMM (k_dgemm.hip, split 6 / 4 / 8 / 1 / 1).  The regime is chosen per ENGINE, from its
  // max_batch (>= dgemm_min), never from the rows of one step: every step of an engine then
  // runs one arithmetic whatever the number of sequences in flight (admission ramps, tails,
  // a chunk alone), so a chunk's summary never depends on its companions.  The crossover:
  // at M = 16 the GEMV and the skinny GEMM tie over a layer's four projections, at M = 32
  // the skinny GEMM takes 30 % less (profiles/r02/v7_dgemm_lds_sync_ab.txt).
  int dgemm_min = 24, dsplit_qkv = 6, dsplit_o = 4, dsplit_down = 8;
  // gate/up skinny-GEMM block form (k_dgemm.hip kh), fixed per engine like the regime: the
  // library setting (2, the default: k split over the two wave groups of an 8-wave block;
  // 41.4 -> 34.9 us at M = 128, profiles/r05/v20_*) for engines of <= 128 slots; the split
  // projections and the lm_head keep the 4-wave block (as fast or faster there)
  int dgemm_kh = 1;
  // weight-row groups per skinny-GEMM block (k_dgemm.hip wn) for launches of <= 128 rows: the
  // 128-row block for QKV, down and the lm_head (down 22.3 -> 20.4 us, lm_head 262 -> 241 us at
  // M = 128, profiles/r05/v21_*), 64 rows for O (15.6 vs 12.9 us at its split 4); bit-identical
  int dwn_qkv = 8, dwn_o = 4, dwn_down = 8, dwn_lm = 8;
  bool large_engine = false;
  int attn_ppw = 2;  // decode attention pages per wave, fixed per engine (k_attn.hip)
  // decode attention with one page per wave (k_attn.hip v2, MS_ATTN_V2), attn_ppb waves / pages
  // per block, fixed per engine like attn_ppw
  bool attn_v2 = false;
  int attn_ppb = 9;
  // v2's splits merged inside the launch by the last block of each group (MS_ATTN_TICKET)
  bool attn_ticket = false;
  unsigned* attn_cnt = nullptr;  // [max_batch * Hk] arrival counters, zero between launches
  bool attn2_ok(int B, int max_len) const {
    return attn_v2 && slot_major && attn_decode2_supported(B, Hq, Hk, max_len, attn_ppb);
  }
  void attn_decode(const DecodeQKV& qa, const KVView& kv, const DecodeAttnArgs& da) {
    prof_begin(K_ATTN_DECODE);
    if (attn2_ok(da.B, da.max_len))
      launch_attn_decode2(qa, attn, Hq, Hk, kv, da, attn_ws, attn_ppb, stream, attn_ticket ? attn_cnt : nullptr);
    else
      launch_attn_decode(qa, attn, Hq, Hk, kv, da, attn_ws, stream);
    prof_end(K_ATTN_DECODE);
  }
  // Residual-fused decode (small-regime engines, fp16 O / down): O and down run unsplit on
  // resid_rt-row tiles (3072 / 12 = 256 workgroups, one per CU) and their epilogue adds into
  // the fp32 residual and emits the next projection's input itself -- xb = f16(x * g_next)
  // and per-tile sums of x^2 (ssq [256][B]) -- so the decode layer has no residual_rmsnorm
  // launch: the deferred RMSNorm (kernels.h RowScale) scales the rows of the QKV / gate-up /
  // lm_head outputs instead.  Chosen per engine (MS_RESID_FUSED=0: split-K slabs + norm
  // launches, the large-regime form; K-quant engines take it too, below: qresid).
  bool resid_fuse = true, has_quant = false;
  // decode_tail_kernel: the step's greedy ids, argument advance and next embedding in one launch
  bool tail_fuse = true;
  // The decode step's layers as ONE persistent launch (k_persist.hip, MS_PERSIST / ms_set_persist;
  // off by default until it measures faster than the launches):
  // engines of <= 8 slots on fp16 Llama-3.2-3B weights in the residual-fused / v2-attention
  // regime, bit-identical to the per-layer launches below.  Chosen per engine (persist_ok at
  // ms_create) and per run (no profiling mask, no prefill overlap: every workgroup must be
  // resident); a hand-off timeout sets pk_err_d, and decode_run recomputes the run with the
  // launches and turns the persistent step off for the engine.
  bool persist = false, persist_ok = false, pk_used = false;
  int n_cu = 0, nsplit_ws = 1;
  unsigned* pk_sync = nullptr;   // [persist_sync_words(L)] zero between launches
  unsigned* pk_err_d = nullptr;  // timeout flag
  unsigned* pk_err_h = nullptr;  // pinned copy
  f16_t* pk_xg2 = nullptr;       // [max_batch][H] gate/up input
  float* pk_ssq2 = nullptr;      // [256][max_batch] its statistics
  // the layers' matrices in the step's stream order (launch_pack_layer; 201 MB per layer),
  // allocated at the first persistent run and rebuilt after any weight (re)load -- including a
  // broadcast into the regions ms_weight_regions hands out
  char* pk_packed = nullptr;
  mutable bool pk_packed_ok = false;
  bool persist_on(int B) const {
    return persist && persist_ok && !overlap && B >= 1 && B <= cfg.max_batch && !has_quant &&
           attn2_ok(B, max_pages * kPage) && attn_slabs && resid_fused(nullptr) && split_qkv == 6;
  }
  int resid_rt = 12;
  // K-quant O / down with the same epilogue (the Q-GEMV on resid_rt-row tiles; MS_QRESID=0:
  // split-K 4 + residual_rmsnorm): 1.785 vs 1.794 ms per Q4_K_M decode step -- O 5.8 vs 4.8 +
  // 4.7 us, down 12.8 vs 8.8 + 4.7 us, the gate/up folding 256 statistics tiles +0.9 us
  // (profiles/r04/v31_*; round 3 measured it even before the Q-GEMV rewrites)
  bool qresid = true;
  // the K-quant GEMVs this regime launches support its shapes (ms_create: RESID_SSQ on O / down
  // and the gate/up SwiGLU folding 256 statistics tiles); the launchers return silently on an
  // unsupported shape, so an engine whose quantised shapes fall outside the Q plan takes split-K
  // + residual_rmsnorm instead of skipping the residual update
  bool qresid_ok = true;
  bool resid_fused(const QSlot* q) const {
    if (!resid_fuse || large_engine) return false;
    if (has_quant && !qresid_ok) return false;
    return !(q && q->ready()) || qresid;
  }
  // the large-batch arithmetic (skinny GEMM) for engines of >= dgemm_min slots.  Engines with
  // K-quant weights keep the exact Q4_K / Q6_K GEMV up to qlarge_min - 1 slots (in row groups of
  // <= kMaxGemvRows above 64: a row's sum order does not depend on its group); from qlarge_min
  // (MS_QLARGE_MIN, default 65: the row groups' weight re-streams cost Q4_K_M 18.2 ms per decode
  // step at 128 slots, profiles/r06/v9_*) they take the large regime too, where every quantised
  // matrix streams its packed blocks once per step through the K-quant skinny GEMM
  // (k_qdgemm.hip, the fp16-copy values).  MS_QDGEMM selects which matrices: 1 (default) the
  // all-Q4_K ones -- a Q6_K matrix (the Q4_K_M lm_head, half of the down / V projections) runs
  // its fp16 copy through k_dgemm.hip, which measured faster there (its dequant is twice the
  // VALU; r06/v11_*) --, 2 every K-quant matrix, 0 none (the fp16 copies everywhere)
  int qlarge_min = 65;
  int qdgemm_mode = 1;
  // engines of >= lm_gemm_min slots run the large-regime lm_head (its greedy partials) on the
  // prefill GEMM's 128x128 tile (k_gemm.hip gemm_kernel, ~1000 blocks of 128 vocabulary rows)
  // instead of the skinny GEMM: 169 vs 252 us at 128 rows, 276 vs 429 at 256
  // (profiles/r06/v21_rows_dgemm_vs_gemm128.txt).  Per engine, so its arithmetic never changes
  // with the rows of a step; MS_LM_GEMM_MIN (0 = never) for A/B.
  int lm_gemm_min = 96;
  // fp16 engines of >= qdf_min slots (16-row-tile launches of up to 256 rows) run their skinny
  // GEMMs on k_qdgemm.hip's fp16-rows form (activations by LDS DMA three steps ahead) with
  // QKV / down split 3 / 4 instead of 6 / 8: at 256 rows gate/up 57.3 -> 50.4 us, QKV 30.2 ->
  // 22.6, down 43.3 -> 34.5, O 19.8 -> 19.2 (profiles/r06/v22_*).  Per engine (MS_QDF_MIN, 0 =
  // never): below it the tested 24-128-slot arithmetic is unchanged.
  int qdf_min = 192;
  bool qdf(int M, int N, int K, int S, int epi) const {
    return !has_quant && qdf_min > 0 && cfg.max_batch >= qdf_min && qdgemm_f16_supported(M, N, K, S, epi);
  }
  bool large(int) const { return large_engine && (!has_quant || cfg.max_batch >= qlarge_min); }
  // the K-quant skinny GEMM for this matrix (large regime)
  bool qd(const QSlot* q, int M, int N, int K, int S, int epi) const {
    if (!qdgemm_mode || !q || !q->ready()) return false;
    const QMat& m = q->m;
    const bool q4 = m.type0 == MS_QT_Q4_K && (m.n < 2 || m.type1 == MS_QT_Q4_K) && (m.n < 3 || m.type2 == MS_QT_Q4_K);
    return (q4 || qdgemm_mode == 2) && qdgemm_supported(M, N, K, S, epi, m);
  }
  bool row_groups(int B) const { return !large(B) && B > kMaxGemvRows; }
  // split count of every quantised slab projection (MS_QSPLIT; 0: as fp16): 4 measured best
  // for Q4_K_M at B = 8 -- 1.878 vs 1.900 ms/step with the fp16 splits (6 / 6 / 4), 2 / 3 / 8
  // slower (profiles/r02/v27_qsplit_sweep_q4_k_m.txt)
  int qsplit = 4;
  // decode attention variant (tuning): q/k/v from QKV split slabs (else the GEMV RoPE
  // epilogue, B <= 16)
  bool attn_slabs = true;
  // the deferred RMSNorm scale of the rows now in xb (set by whoever wrote xb)
  RowScale cur_rs{};
  int32_t* args_d = nullptr;
  int32_t* args_h = nullptr;  // pinned
  size_t args_cap = 0;
  // Prefill and decode each own a stream, activations, argument staging, first-token /
  // argmax buffers and timing events, so the prefill of newly admitted chunks runs on one
  // stream WHILE the decode run of the running chunks runs on the other (prefill is
  // MFMA-bound, decode HBM-bound: SURVEY.md §7 step 6 "admit prefill chunks while decoding").
  // use() points the working members (stream, x, xb, ..., ev_a/ev_b) at one of them; KV pages,
  // slots and weights are shared (a chunk's pages are only touched by its own phase).
  // Measured on MI355X (configs[2], 128 slots, profiles/r03/v3_overlap_*): the two phases
  // interfere -- the prefill GEMMs and the decode step's short launches share every CU, so
  // prefill took +28 % and a decode step +23 % -- and the whole job was 8 % SLOWER with a
  // 16-step run under each prefill (2.6 % slower with one-step runs), natural EOS or not.  So
  // the phases run one after the other by default; MS_OVERLAP=1 turns the overlap on.
  struct Ctx {
    hipStream_t stream = nullptr;
    float* x = nullptr;
    float* ssq = nullptr;  // sums of x^2 behind xb: [rows] (norm kernels) or [256][rows] (RESID)
    f16_t *xb = nullptr, *qkv = nullptr, *attn = nullptr, *hbuf = nullptr;
    float* logits = nullptr;
    int32_t* ids_out_d = nullptr;
    int32_t* args_d = nullptr;
    int32_t* args_h = nullptr;
    size_t args_cap = 0;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;
  } cp, cd;
  bool overlap = false;
  void use(const Ctx& c) {
    stream = c.stream; x = c.x; ssq = c.ssq; xb = c.xb; qkv = c.qkv; attn = c.attn; hbuf = c.hbuf;
    logits = c.logits; ids_out_d = c.ids_out_d; args_d = c.args_d; args_h = c.args_h;
    args_cap = c.args_cap; ev_a = c.ev_a; ev_b = c.ev_b;
  }
  std::vector<uint8_t> stop_set;  // ms_set_eos_ids: a stop-id bitmap replacing cfg.eos_ids
  std::deque<std::unique_ptr<Seq>> waiting;
  std::vector<std::unique_ptr<Seq>> running;
  std::vector<std::unique_ptr<Seq>> done, polled;
  ms_stats stats{};
  uint32_t prof_mask = 0;
  std::vector<std::pair<int, int>> ev_pending;  // (class, event pair index)
  size_t ev_used = 0;
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  // decode steps replay a captured hipGraph per (batch rows, attention splits): the
  // kernels' pointers and the step-argument layout depend on nothing else
  // key: (batch rows, attention split grid, decode steps captured in the graph)
  // (graph, last use) -- least recently used graphs are destroyed beyond kMaxGraphs, so ragged
  // or admission-ramp workloads with many distinct (B, length bucket) keys stay bounded
  std::map<std::tuple<int, int, int>, std::pair<hipGraphExec_t, uint64_t>> decode_graphs;
  uint64_t graph_clock = 0;
  static constexpr size_t kMaxGraphs = 64;
  // chained decode steps per graph launch (MS_GRAPH_STEPS): 16 measured 12.12 -> 12.20
  // chunks/s on configs[1], unchanged on the ragged level and configs[2]
  // (profiles/r02/v35_graph_steps_ab.txt); a run's remainder uses the one-step graph
  int graph_steps = 16;
  bool use_graphs = true;
  int32_t* ids_host = nullptr;  // pinned landing buffer: kMaxRun steps x <= 256 greedy ids
  int32_t* first_host = nullptr;  // pinned: the first greedy id of each prefilled prompt
  int32_t* ids_ring_d = nullptr;  // device ring of a decode run's ids (decode_advance)
  static constexpr int kMaxRun = 64;  // chained decode steps per host synchronisation
  int max_run = kMaxRun;              // MS_DECODE_RUN (1 = one step per ms_step)

  template <class T>
  T* dalloc(size_t n, bool zero = false) {
    void* p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess)
      throw MsError(MS_ENOMEM, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B) failed: " +
                                   hipGetErrorString(e));
    allocs.push_back(p);
    if (zero) HIP_OK(hipMemset(p, 0, n * sizeof(T)));
    return (T*)p;
  }

  // ---- profiling brackets -------------------------------------------------
  // prof_begin(cls) arms ms::g_prof with an event pair; the next kernel launch of the class
  // records its own start/stop (hipExtLaunchKernelGGL), so timings match rocprofv3.
  std::vector<ProfEvents> ev_pairs;
  void prof_begin(int cls) {
    if (!((prof_mask >> cls) & 1)) return;
    if (ev_used >= ev_pairs.size()) {
      for (int i = 0; i < 64; ++i) {
        ProfEvents pe;
        HIP_OK(hipEventCreate(&pe.start));
        HIP_OK(hipEventCreate(&pe.stop));
        ev_pairs.push_back(pe);
      }
    }
    ev_pending.push_back({cls, (int)ev_used});
    g_prof = &ev_pairs[ev_used];
    ev_used += 1;
  }
  void prof_end(int cls) {
    if (!((prof_mask >> cls) & 1)) return;
    g_prof = nullptr;
  }
  void prof_collect() {  // after a stream sync
    for (auto& pr : ev_pending) {
      float ms_ = 0.f;
      HIP_OK(hipEventElapsedTime(&ms_, ev_pairs[pr.second].start, ev_pairs[pr.second].stop));
      stats.kernel_ms[pr.first] += ms_;
      stats.kernel_launches[pr.first] += 1;
    }
    ev_pending.clear();
    ev_used = 0;
  }

  KVView kv_layer(int l) const {
    KVView v;
    v.k = kpool + (size_t)l * layer_kv_elems;
    v.v = vpool + (size_t)l * layer_kv_elems;
    v.block_table = bt_d;
    v.max_pages = max_pages;
    v.n_kv_heads = Hk;
    v.slot_major = slot_major ? 1 : 0;
    return v;
  }

  // the deferred RMSNorm scale of rows whose sums of squares a norm kernel wrote (one tile)
  RowScale norm_rs() const { return make_row_scale(ssq, 1, H, cfg.norm_eps); }

  // normalised (rs) or plain projection: the decode GEMV where it fits, else the MFMA GEMM
  void gemm_or_gemv(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldo,
                    int epi, bool decode, int cls, const RowScale* rs = nullptr) {
    prof_begin(cls);
    if (decode && gemv_supported(M, N, K, epi)) {
      GemvArgs ga{};
      if (rs) ga.rs = *rs;
      launch_gemv_ex(X, W, out, M, N, K, ldo, epi, &ga, 0, stream);
    } else {
      launch_gemm(X, W, out, M, N, K, ldo, epi, stream, rs);
    }
    prof_end(cls);
  }

  // decode projection: the K-quant stream when that matrix was loaded quantised; above
  // kMaxGemvRows rows (row groups) the rows go in groups, out elements of `esz` bytes
  void proj(const QSlot* q, const f16_t* X, const f16_t* W, void* out, int M, int N, int K,
            int ldo, int epi, const GemvArgs* ga, int cls, int esz = 0) {
    if (row_groups(M)) {
      for (int r0 = 0; r0 < M; r0 += kMaxGemvRows) {
        GemvArgs g = ga ? *ga : GemvArgs{};
        g.rs = rs_rows(g.rs, r0);
        proj(q, X + (size_t)r0 * K, W, (char*)out + (size_t)r0 * ldo * esz, std::min(M - r0, (int)kMaxGemvRows),
             N, K, ldo, epi, &g, cls, esz);
      }
      return;
    }
    prof_begin(cls);
    if (q && q->ready() && qgemv_supported(M, N, K, epi))
      launch_qgemv(X, q->m, out, M, N, K, ldo, epi, ga, stream);
    else
      launch_gemv_ex(X, W, out, M, N, K, ldo, epi, ga, 0, stream);
    prof_end(cls);
  }

  // decode with fused epilogues: QKV (split-K slabs, deferred norm scale) -> attention (folds
  // the slabs, RoPE, KV write) -> O -> gate/up + SwiGLU -> down, where O and down either add
  // into the residual and emit the next projection's input themselves (resid_fused) or write
  // split-K slabs that a residual_rmsnorm launch folds
  bool fused_decode(int B) const {
    if (large(B))
      return B <= kMaxSlabRows && attn_slabs && residual_rmsnorm_supported(kMaxSplit, H) &&
             dgemm_supported(B, QKVN, H, dsplit_qkv, MS_GEMV_EPI_STORE_F32, 1) &&
             dgemm_supported(B, H, Hq * D, dsplit_o, MS_GEMV_EPI_STORE_F32, 1) &&
             dgemm_supported(B, H, F, dsplit_down, MS_GEMV_EPI_STORE_F32, 1) &&
             dgemm_supported(B, 2 * F, H, 1, MS_GEMV_EPI_SWIGLU, dgemm_kh) && (2 * F) % 32 == 0 &&
             attn_decode_supported(B, Hq, Hk, max_pages * kPage);
    // row groups (K-quant engines above 64 rows): split-K slabs and SwiGLU only, no residual
    // epilogue (resid_fused is off in large engines), one residual_rmsnorm over all rows
    if (row_groups(B) && !(B <= kMaxSlabRows && attn_slabs && !resid_fused(nullptr))) return false;
    const int Bg = std::min(B, (int)kMaxGemvRows);
    // the gate/up GEMV folds the statistics its producer wrote: 256 tiles behind the residual
    // epilogue, one behind residual_rmsnorm
    const int gu_tiles = resid_fused(nullptr) ? H / resid_rt : 1;
    return residual_rmsnorm_supported(kMaxSplit, H) &&
           (attn_slabs ? gemv_split_supported(Bg, QKVN, H, 1) : gemv_supported(Bg, QKVN, H, MS_GEMV_EPI_ROPE_KV)) &&
           gemv_supported(Bg, 2 * F, H, MS_GEMV_EPI_SWIGLU, gu_tiles) &&
           gemv_split_supported(Bg, H, Hq * D, 1) && gemv_split_supported(Bg, H, F, 1) &&
           (!resid_fuse || (gemv_supported(Bg, H, Hq * D, MS_GEMV_EPI_RESID_SSQ) &&
                            gemv_supported(Bg, H, F, MS_GEMV_EPI_RESID_SSQ))) &&
           attn_decode_supported(B, Hq, Hk, max_pages * kPage);
  }
  // a row group's deferred-norm scale: one-tile statistics are per row ([M]), so the group
  // starts at its first row (multi-tile [tiles][M] statistics never reach row groups)
  static RowScale rs_rows(const RowScale& rs, int r0) {
    RowScale g = rs;
    if (g.ssq) g.ssq += r0;
    return g;
  }
  static constexpr int kMaxGemvRows = 64, kMaxSlabRows = 256, kMaxSplit = 8;

  // normalised projection into fp32 partial slabs [S][M][N], rows scaled by cur_rs; returns
  // the number of slabs written
  // dwn: the skinny GEMM's weight-row groups per block (k_dgemm.hip wn; 8 = 128-row blocks,
  // the same bits as 4) for launches of <= 128 rows
  int proj_split(const QSlot* q, const f16_t* X, const f16_t* W, int M, int N, int K, int S, int Sl,
                 const RowScale* rs, int dwn = 4) {
    if (row_groups(M)) {
      // every group must write the same number of slabs: the fold adds S slabs for all rows
      int used = 0;
      for (int r0 = 0; r0 < M; r0 += kMaxGemvRows) {
        const RowScale g = rs ? rs_rows(*rs, r0) : RowScale{};
        const int u = proj_split_rows(q, X + (size_t)r0 * K, W, std::min(M - r0, (int)kMaxGemvRows), N, K, S, Sl,
                                      rs ? &g : nullptr, slabs + (size_t)r0 * N, M, dwn);
        REQUIRE(used == 0 || u == used, MS_EIO, "row groups split a projection differently");
        used = u;
      }
      return used;
    }
    return proj_split_rows(q, X, W, M, N, K, S, Sl, rs, slabs, 0, dwn);
  }
  int proj_split_rows(const QSlot* q, const f16_t* X, const f16_t* W, int M, int N, int K, int S, int Sl,
                      const RowScale* rs, float* slabs, int slab_rows, int dwn) {
    prof_begin(K_GEMV);
    GemvArgs ga{};
    if (rs) ga.rs = *rs;
    ga.slab_rows = slab_rows;
    int used = 1;
    if (large(M)) {  // skinny GEMM: the packed K-quant blocks, or the fp16 weights
      if (qd(q, M, N, K, Sl, MS_GEMV_EPI_STORE_F32))
        launch_qdgemm(X, q->m, slabs, M, N, K, Sl, N, MS_GEMV_EPI_STORE_F32, stream, rs);
      else if (qdf(M, N, K, Sl, MS_GEMV_EPI_STORE_F32))
        launch_qdgemm_f16(X, W, slabs, M, N, K, Sl, N, MS_GEMV_EPI_STORE_F32, stream, rs);
      else
        launch_dgemm(X, W, slabs, M, N, K, Sl, N, MS_GEMV_EPI_STORE_F32, stream, rs, 1,
                     M <= 128 && N % 128 == 0 ? dwn : 4);
      used = Sl;
    } else if (q && q->ready() && qgemv_supported(M, N, K, MS_GEMV_EPI_STORE_F32)) {
      // Q4_K/Q6_K: same split-K as fp16 (a 16-row tile carries 3.6x fewer weight bytes, so
      // the unsplit grid -- 192 blocks for O/down -- is too thin to cover 256 CUs)
      const int Sq = qsplit > 0 ? qsplit : S;
      if (Sq > 1 && Sq <= kMaxSplit && qgemv_split_supported(M, N, K, Sq)) {
        launch_qgemv_split(X, q->m, slabs, M, N, K, Sq, stream, &ga);
        used = Sq;
      } else {
        launch_qgemv(X, q->m, slabs, M, N, K, N, MS_GEMV_EPI_STORE_F32, &ga, stream);
      }
    } else {
      if (!(S >= 1 && S <= kMaxSplit && gemv_split_supported(M, N, K, S))) S = 1;
      launch_gemv_split(X, W, slabs, M, N, K, S, 0, stream, &ga);
      used = S;
    }
    prof_end(K_GEMV);
    return used;
  }

  // fold pending slabs into x, then xb = f16(x * w) and its one-tile statistics
  void residual_norm(const f16_t* w, int B) {
    prof_begin(K_MISC);
    launch_residual_rmsnorm(x, slabs, pending_split, w, xb, ssq, B, H, stream);
    prof_end(K_MISC);
    pending_split = 0;
    cur_rs = norm_rs();
  }

  // the residual update of O / down: x += X . W^T, then the input of the next normalised
  // projection (gain g_next) -- in the GEMV epilogue (resid_fused: RESID_SSQ on resid_rt-row
  // tiles, 256 tiles of statistics) or as split-K slabs + one residual_rmsnorm launch
  void resid_update(const QSlot* q, const f16_t* X, const f16_t* W, int B, int K, int S, int Sl,
                    const f16_t* g_next, int dwn) {
    if (resid_fused(q)) {
      GemvArgs ga{};
      ga.rt = resid_rt;
      ga.ssq_out = ssq;
      ga.gamma = g_next;
      ga.xg_out = xb;
      prof_begin(K_GEMV);
      if (q && q->ready())
        launch_qgemv(X, q->m, x, B, H, K, H, MS_GEMV_EPI_RESID_SSQ, &ga, stream);
      else
        launch_gemv_ex(X, W, x, B, H, K, H, MS_GEMV_EPI_RESID_SSQ, &ga, 0, stream);
      prof_end(K_GEMV);
      pending_split = 0;
      cur_rs = make_row_scale(ssq, H / resid_rt, H, cfg.norm_eps);
    } else {
      pending_split = proj_split(q, X, W, B, H, K, S, Sl, nullptr, dwn);
      residual_norm(g_next, B);
    }
  }

  void run_layer_fused_decode(int l, int B, const int32_t* tok_pos, const int32_t* tok_slot,
                              const DecodeAttnArgs& da) {
    const Layer& Ly = layers[l];
    KVView kv = kv_layer(l);
    const auto& Q = lq[l];
    const RowScale rs_attn = cur_rs;
    DecodeQKV qa{nullptr, slabs, 0, cos_tab, sin_tab, rs_attn};
    if (attn_slabs) {
      // QKV -> unscaled slabs; attention adds them, applies the row's deferred-norm factor and
      // RoPE, and writes the new K/V (k_attn.hip): one factor per attention block, not per
      // QKV tile
      qa.S = proj_split(&Q[QS_QKV], xb, Ly.wqkv, B, QKVN, H, split_qkv, dsplit_qkv, nullptr, dwn_qkv);
    } else {
      // QKV GEMV epilogue: RoPE, q -> qkv rows, K/V -> paged cache
      GemvArgs ga{};
      ga.tok_pos = tok_pos;
      ga.tok_slot = tok_slot;
      ga.cos_tab = cos_tab;
      ga.sin_tab = sin_tab;
      ga.kv = kv;
      ga.Hq = Hq;
      ga.Hk = Hk;
      ga.rs = rs_attn;
      proj(&Q[QS_QKV], xb, Ly.wqkv, qkv, B, QKVN, H, QKVN, MS_GEMV_EPI_ROPE_KV, &ga, K_GEMV);
      qa = DecodeQKV{qkv, nullptr, 0, cos_tab, sin_tab, RowScale{}};
    }
    attn_decode(qa, kv, da);
    resid_update(&Q[QS_O], attn, Ly.wo, B, Hq * D, split_o, dsplit_o, Ly.ffn_norm, dwn_o);
    const RowScale rs_ffn = cur_rs;
    const f16_t* g_next = l + 1 < L ? layers[l + 1].attn_norm : final_norm;
    if (large(B)) {
      // gate/up + SwiGLU on the skinny GEMM (41 vs 55 us for the 128x128 GEMM at M = 128,
      // profiles/r02/v7_dgemm_lds_sync_ab.txt; fused_decode checked M <= 256)
      prof_begin(K_GEMV);
      if (qd(&Q[QS_GU], B, 2 * F, H, 1, MS_GEMV_EPI_SWIGLU))
        launch_qdgemm(xb, Q[QS_GU].m, hbuf, B, 2 * F, H, 1, F, MS_GEMV_EPI_SWIGLU, stream, &rs_ffn);
      else if (qdf(B, 2 * F, H, 1, MS_GEMV_EPI_SWIGLU))
        launch_qdgemm_f16(xb, Ly.wgu, hbuf, B, 2 * F, H, 1, F, MS_GEMV_EPI_SWIGLU, stream, &rs_ffn);
      else
        launch_dgemm(xb, Ly.wgu, hbuf, B, 2 * F, H, 1, F, MS_GEMV_EPI_SWIGLU, stream, &rs_ffn, dgemm_kh);
      prof_end(K_GEMV);
    } else {
      GemvArgs gg{};
      gg.rs = rs_ffn;
      proj(&Q[QS_GU], xb, Ly.wgu, hbuf, B, 2 * F, H, F, MS_GEMV_EPI_SWIGLU, &gg, K_GEMV, sizeof(f16_t));
    }
    resid_update(&Q[QS_DOWN], hbuf, Ly.wdown, B, F, split_down, dsplit_down, g_next, dwn_down);
  }

  // one transformer layer over T packed tokens (decode: T = B rows, one token each); on entry
  // xb = f16(x * attn_norm) with cur_rs, on exit xb = f16(x * g_next) with cur_rs
  // (tail = false: the last layer of a prefill whose caller normalises only the rows it needs)
  void run_layer(int l, int T, bool decode, const int32_t* tok_pos, const int32_t* tok_slot,
                 const PrefillAttnArgs& pa, const DecodeAttnArgs& da, bool tail = true) {
    if (decode && fused_decode(T)) {
      run_layer_fused_decode(l, T, tok_pos, tok_slot, da);
      return;
    }
    const Layer& Ly = layers[l];
    const int kc = decode ? K_GEMV : K_GEMM;
    const RowScale rs_attn = cur_rs;
    KVView kv = kv_layer(l);
    // (RoPE + the K / V scatter in the prefill QKV GEMM's epilogue measured slower than this
    // launch: 611 vs 423 + 58 us per layer, scattered 2-byte stores and per-element table loads,
    // profiles/r04/v5_prefill_fusions_prof_*.txt)
    gemm_or_gemv(xb, Ly.wqkv, qkv, T, QKVN, H, QKVN, MS_EPI_STORE_F16, decode, kc, &rs_attn);
    prof_begin(K_MISC);
    // prefill: K / V only -- the attention kernel rotates Q while staging it (pa.cos_tab)
    launch_rope_kv(qkv, T, Hq, Hk, tok_pos, tok_slot, cos_tab, sin_tab, kv, stream, decode || !pa.cos_tab);
    prof_end(K_MISC);
    if (decode) {
      attn_decode(DecodeQKV{qkv, nullptr, 0, cos_tab, sin_tab, RowScale{}}, kv, da);
    } else {
      prof_begin(K_ATTN_PREFILL);
      launch_attn_prefill(qkv, attn, Hq, Hk, kv, pa, stream);
      prof_end(K_ATTN_PREFILL);
    }
    const f16_t* g_next = l + 1 < L ? layers[l + 1].attn_norm : final_norm;
    if (decode) {
      gemm_or_gemv(attn, Ly.wo, x, T, H, Hq * D, H, MS_EPI_ADD_F32, decode, kc);
      norm_input(Ly.ffn_norm, T);
    } else {  // prefill: the O GEMM's residual epilogue emits the gate/up input and statistics
      prefill_resid(attn, Ly.wo, T, Hq * D, Ly.ffn_norm);
    }
    const RowScale rs_ffn = cur_rs;
    gemm_or_gemv(xb, Ly.wgu, hbuf, T, 2 * F, H, F, MS_EPI_SWIGLU, decode, kc, &rs_ffn);
    if (decode) {
      gemm_or_gemv(hbuf, Ly.wdown, x, T, H, F, H, MS_EPI_ADD_F32, decode, kc);
      if (tail) norm_input(g_next, T);
    } else if (tail) {
      prefill_resid(hbuf, Ly.wdown, T, F, g_next);
    } else {
      gemm_or_gemv(hbuf, Ly.wdown, x, T, H, F, H, MS_EPI_ADD_F32, decode, kc);
    }
  }

  // prefill residual update x += X . W^T whose GEMM epilogue also writes xb = f16(x * g_next)
  // and per-column-tile sums of x^2 (k_gemm.hip GemmResid): no norm launch between the
  // residual add and the next normalised projection
  // The path is picked BEFORE any launch: the epilogue writes [H / 128][T] statistics into ssq
  // (sized R * kGemmRsTiles), so hidden sizes above 24 * 128 take the plain residual add and
  // one rmsnorm launch instead (ms_create accepts any hidden % 256 == 0).
  bool prefill_resid_ok(int T) const {
    const int tiles = gemm_resid_tiles(T, H);
    return tiles <= kGemmRsTiles && gemm_rs_tiles_ok(T, QKVN, tiles) && gemm_rs_tiles_ok(T, 2 * F, tiles);
  }
  void prefill_resid(const f16_t* X, const f16_t* W, int T, int K, const f16_t* g_next) {
    if (!prefill_resid_ok(T)) {
      gemm_or_gemv(X, W, x, T, H, K, H, MS_EPI_ADD_F32, false, K_GEMM);
      norm_input(g_next, T);
      return;
    }
    GemmResid gr{g_next, xb, ssq};
    prof_begin(K_GEMM);
    launch_gemm(X, W, x, T, H, K, H, MS_EPI_ADD_F32, stream, nullptr, &gr);
    prof_end(K_GEMM);
    cur_rs = make_row_scale(ssq, gemm_resid_tiles(T, H), H, cfg.norm_eps);
  }

  // xb = f16(x * w), ssq = the rows' sums of squares (rmsnorm_kernel), cur_rs = their scale
  void norm_input(const f16_t* w, int T, const int32_t* row_idx = nullptr) {
    prof_begin(K_MISC);
    launch_rmsnorm(x, w, xb, ssq, T, H, row_idx, stream);
    prof_end(K_MISC);
    cur_rs = norm_rs();
  }

  // K-quant tensors loaded so far, (tensor, layer, ggml type) in load order: the manifest a
  // weight broadcast replays on the receiving ranks (ms_quant_manifest / ms_declare_weight_q)
  std::vector<std::array<int32_t, 3>> quant_manifest;
  void note_quant(int tensor, int layer, int type) {
    for (auto& q : quant_manifest)
      if (q[0] == tensor && q[1] == layer) { q[2] = type; return; }
    quant_manifest.push_back({tensor, layer, type});
  }
  // every device weight buffer, in a fixed order: fp16 matrices and norms, then the K-quant
  // regions (the payload of a weight broadcast, dist.broadcast_engine_weights)
  std::vector<std::pair<void*, size_t>> weight_regions() const {
    std::vector<std::pair<void*, size_t>> r;
    const size_t H2 = (size_t)H * 2;
    r.push_back({embed, (size_t)V * H2});
    if (!cfg.tie_embeddings) r.push_back({lm_head, (size_t)V * H2});
    r.push_back({final_norm, H2});
    for (const Layer& Ly : layers) {
      r.push_back({Ly.attn_norm, H2});
      r.push_back({Ly.ffn_norm, H2});
      r.push_back({Ly.wqkv, (size_t)QKVN * H2});
      r.push_back({Ly.wo, (size_t)Hq * D * H2});
      r.push_back({Ly.wgu, (size_t)2 * F * H2});
      r.push_back({Ly.wdown, (size_t)F * H2});
    }
    auto qs = [&](const QSlot& q) {
      const uint8_t* b[3] = {q.m.base0, q.m.base1, q.m.base2};
      for (int i = 0; i < 3; ++i)
        if (b[i]) r.push_back({(void*)b[i], q.bytes[i]});
    };
    qs(lmq);
    for (const auto& l : lq)
      for (const QSlot& q : l) qs(q);
    return r;
  }

  // Captured decode graphs bake in the weight form (fp16 vs K-quant stream) and the split
  // choices: any weight (re)load invalidates them.
  void drop_graphs() {
    pk_packed_ok = false;
    for (auto& kv : decode_graphs) (void)hipGraphExecDestroy(kv.second.first);
    decode_graphs.clear();
  }
  void evict_graphs() {  // keep at most kMaxGraphs - 1 before inserting one more
    while (decode_graphs.size() >= kMaxGraphs) {
      auto lru = decode_graphs.begin();
      for (auto it = decode_graphs.begin(); it != decode_graphs.end(); ++it)
        if (it->second.second < lru->second.second) lru = it;
      (void)hipGraphExecDestroy(lru->second.first);
      decode_graphs.erase(lru);
    }
  }

  int32_t* upload_args(const std::vector<int32_t>& a) {
    REQUIRE(a.size() <= args_cap, MS_EINVAL, "step arguments exceed the staging buffer");
    std::memcpy(args_h, a.data(), a.size() * sizeof(int32_t));
    HIP_OK(hipMemcpyAsync(args_d, args_h, a.size() * sizeof(int32_t), hipMemcpyHostToDevice, stream));
    return args_d;
  }
};

namespace {

int fail(ms_engine* e, const MsError& x) {
  if (e) e->err = x.what();
  g_last_error = x.what();
  return x.code;
}

template <class Fn>
int guarded(ms_engine* e, Fn&& fn) {
  try {
    return fn();
  } catch (const MsError& x) {
    return fail(e, x);
  } catch (const std::exception& x) {
    return fail(e, MsError(MS_EIO, x.what()));
  } catch (...) {
    return fail(e, MsError(MS_EIO, "unknown exception"));
  }
}

// llama3-scaled rotate-half tables (oracle/llama_ref.py rope_inv_freq restates this)
void rope_tables(const ms_config& c, int max_ctx, std::vector<float>& cs, std::vector<float>& sn) {
  const int half = c.head_dim / 2;
  std::vector<double> inv(half);
  for (int i = 0; i < half; ++i) {
    double f = 1.0 / std::pow((double)c.rope_theta, (2.0 * i) / c.head_dim);
    if (c.rope_factor > 0) {
      const double low_wl = c.rope_orig_ctx / (double)c.rope_low_freq_factor;
      const double high_wl = c.rope_orig_ctx / (double)c.rope_high_freq_factor;
      const double wl = 2.0 * M_PI / f;
      double out = wl > low_wl ? f / c.rope_factor : f;
      if (!(wl < high_wl) && !(wl > low_wl)) {
        const double smooth = (c.rope_orig_ctx / wl - c.rope_low_freq_factor) /
                              (c.rope_high_freq_factor - c.rope_low_freq_factor);
        out = (1.0 - smooth) * out / c.rope_factor + smooth * out;
      }
      f = out;
    }
    inv[i] = f;
  }
  cs.resize((size_t)max_ctx * half);
  sn.resize((size_t)max_ctx * half);
  for (int p = 0; p < max_ctx; ++p)
    for (int i = 0; i < half; ++i) {
      const double a = (double)p * inv[i];
      cs[(size_t)p * half + i] = (float)std::cos(a);
      sn[(size_t)p * half + i] = (float)std::sin(a);
    }
}

void validate_config(const ms_config& c) {
  REQUIRE(c.abi_version == MS_ABI_VERSION, MS_EINVAL, "abi_version mismatch");
  REQUIRE(c.head_dim == 128, MS_EINVAL, "head_dim must be 128");
  REQUIRE(c.n_layers > 0 && c.n_heads > 0 && c.n_kv_heads > 0 && c.n_heads % c.n_kv_heads == 0,
          MS_EINVAL, "bad head/layer counts");
  REQUIRE(c.n_heads / c.n_kv_heads <= 16, MS_EINVAL, "GQA group must be <= 16");
  REQUIRE(c.n_heads + c.n_kv_heads <= 64, MS_EINVAL, "at most 64 query+key heads");
  REQUIRE(c.hidden == c.n_heads * c.head_dim, MS_EINVAL, "hidden must equal n_heads*head_dim");
  REQUIRE(c.hidden % 256 == 0 && c.ffn % 256 == 0, MS_EINVAL, "hidden and ffn must be multiples of 256");
  REQUIRE(c.vocab % 16 == 0 && c.vocab > 0, MS_EINVAL, "vocab must be a multiple of 16");
  REQUIRE(c.max_batch >= 1 && c.max_batch <= 1024, MS_EINVAL, "max_batch must be in [1,1024]");
  REQUIRE(c.max_ctx >= 64 && c.max_ctx <= 131072, MS_EINVAL, "max_ctx must be in [64,131072]");
  REQUIRE(c.max_prefill_tokens >= 1, MS_EINVAL, "max_prefill_tokens must be >= 1");
  REQUIRE(c.n_eos >= 0 && c.n_eos <= 8, MS_EINVAL, "n_eos must be in [0,8]");
}

}  // namespace

// ============================================================================ C-ABI
extern "C" {

int ms_create(const ms_config* cfg, ms_engine** out) {
  if (!cfg || !out) {
    g_last_error = "ms_create: null argument";
    return MS_EINVAL;
  }
  *out = nullptr;
  auto e = std::make_unique<ms_engine>();
  int rc = guarded(nullptr, [&]() -> int {
    validate_config(*cfg);
    ms_engine& E = *e;
    E.cfg = *cfg;
    HIP_OK(hipSetDevice(cfg->device));
    for (ms_engine::Ctx* c : {&E.cp, &E.cd}) {
      HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      HIP_OK(hipEventCreate(&c->ev_a));
      HIP_OK(hipEventCreate(&c->ev_b));
    }
    E.use(E.cp);
    E.H = cfg->hidden; E.Hq = cfg->n_heads; E.Hk = cfg->n_kv_heads; E.D = cfg->head_dim;
    E.F = cfg->ffn; E.V = cfg->vocab; E.L = cfg->n_layers;
    E.QKVN = (E.Hq + 2 * E.Hk) * E.D;
    E.max_pages = (cfg->max_ctx + kPage - 1) / kPage;
    E.n_pages = cfg->n_pages > 0 ? cfg->n_pages : cfg->max_batch * E.max_pages;
    E.slot_major = E.n_pages == cfg->max_batch * E.max_pages && !getenv("MS_KV_PAGED");
    E.Tmax = std::max(cfg->max_prefill_tokens, cfg->max_batch);
    // weights
    E.embed = E.dalloc<f16_t>((size_t)E.V * E.H);
    E.lm_head = cfg->tie_embeddings ? E.embed : E.dalloc<f16_t>((size_t)E.V * E.H);
    E.final_norm = E.dalloc<f16_t>(E.H);
    E.layers.resize(E.L);
    E.lq.resize(E.L);
    for (auto& Ly : E.layers) {
      Ly.attn_norm = E.dalloc<f16_t>(E.H);
      Ly.ffn_norm = E.dalloc<f16_t>(E.H);
      Ly.wqkv = E.dalloc<f16_t>((size_t)E.QKVN * E.H);
      Ly.wo = E.dalloc<f16_t>((size_t)E.H * E.Hq * E.D);
      Ly.wgu = E.dalloc<f16_t>((size_t)2 * E.F * E.H);
      Ly.wdown = E.dalloc<f16_t>((size_t)E.H * E.F);
    }
    // rope tables
    std::vector<float> cs, sn;
    rope_tables(*cfg, cfg->max_ctx, cs, sn);
    E.cos_tab = E.dalloc<float>(cs.size());
    E.sin_tab = E.dalloc<float>(sn.size());
    HIP_OK(hipMemcpy(E.cos_tab, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(E.sin_tab, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
    // paged KV pool (zeroed: stale-page bytes are always finite)
    E.layer_kv_elems = (size_t)E.n_pages * E.Hk * kPage * E.D;
    E.kpool = E.dalloc<f16_t>(E.layer_kv_elems * E.L, true);
    E.vpool = E.dalloc<f16_t>(E.layer_kv_elems * E.L, true);
    HIP_OK(hipHostMalloc((void**)&E.bt_h, (size_t)cfg->max_batch * E.max_pages * sizeof(int32_t),
                         hipHostMallocDefault));
    std::memset(E.bt_h, 0, (size_t)cfg->max_batch * E.max_pages * sizeof(int32_t));
    E.bt_d = E.dalloc<int32_t>((size_t)cfg->max_batch * E.max_pages, true);
    for (int p = E.n_pages - 1; p >= 0; --p) E.free_pages.push_back(p);
    for (int s = cfg->max_batch - 1; s >= 0; --s) E.free_slots.push_back(s);
    // activations
    const size_t T = E.Tmax;
    for (ms_engine::Ctx* c : {&E.cp, &E.cd}) {  // prefill: T rows; decode: max_batch rows
      const size_t R = c == &E.cp ? T : (size_t)cfg->max_batch;
      c->x = E.dalloc<float>(R * E.H);
      // [rows] (norm kernels), [256][rows] (decode RESID epilogue), [tiles][rows] (prefill GEMM)
      c->ssq = E.dalloc<float>(std::max(R * kGemmRsTiles, (size_t)256 * cfg->max_batch), true);
      c->xb = E.dalloc<f16_t>(R * E.H);
      c->qkv = E.dalloc<f16_t>(R * E.QKVN);
      c->attn = E.dalloc<f16_t>(R * E.Hq * E.D);
      c->hbuf = E.dalloc<f16_t>(R * E.F);
      c->logits = E.dalloc<float>((size_t)cfg->max_batch * E.V);
      c->ids_out_d = E.dalloc<int32_t>(cfg->max_batch);
    }
    const int Md = std::min(cfg->max_batch, 64);
    size_t gws = 0;
    const int shapes[5][2] = {{E.QKVN, E.H}, {E.H, E.Hq * E.D}, {2 * E.F, E.H}, {E.H, E.F}, {E.V, E.H}};
    for (auto& sh : shapes) gws = std::max(gws, gemv_workspace_bytes(Md, sh[0], sh[1]));
    E.gemv_ws = E.dalloc<char>(gws, true);
    // decode attention: v2 (one page per wave) for engines of <= 16 slots (MS_ATTN_V2 overrides)
    E.attn_ppb = attn_decode2_ppb(cfg->max_batch, E.Hk, cfg->max_ctx);
    E.attn_v2 = cfg->max_batch <= 16;
    if (const char* v = getenv("MS_ATTN_V2")) E.attn_v2 = atoi(v) != 0;
    if (const char* v = getenv("MS_ATTN_TICKET")) E.attn_ticket = atoi(v) != 0;
    E.attn_cnt = E.dalloc<unsigned>((size_t)cfg->max_batch * E.Hk, true);
    // decode_run sets the split grid from the longest sequence rounded UP to 256 keys, which can
    // pass max_ctx when max_ctx is not a multiple of 256: size both attention
    // workspaces for the rounded context
    const int ws_ctx = (cfg->max_ctx + 255) / 256 * 256;
    E.attn_ws = (float*)E.dalloc<char>(std::max(attn_decode_workspace_bytes(cfg->max_batch, E.Hq, ws_ctx),
                                                attn_decode2_workspace_bytes(cfg->max_batch, E.Hq, ws_ctx,
                                                                             E.attn_ppb)),
                                       true);
    E.slabs = E.dalloc<float>((size_t)ms_engine::kMaxSplit * std::min(std::max(cfg->max_batch, 64), 256) *
                              std::max(E.QKVN, E.H));
    if (const char* v = getenv("MS_SPLIT_QKV")) E.split_qkv = atoi(v);
    if (const char* v = getenv("MS_ATTN_SLABS")) E.attn_slabs = atoi(v) != 0;
    if (const char* v = getenv("MS_SPLIT_O")) E.split_o = atoi(v);
    if (const char* v = getenv("MS_SPLIT_DOWN")) E.split_down = atoi(v);
    if (const char* v = getenv("MS_DGEMM_MIN")) E.dgemm_min = atoi(v);
    E.large_engine = cfg->max_batch >= E.dgemm_min;
    if (const char* v = getenv("MS_QLARGE_MIN")) E.qlarge_min = atoi(v);
    if (const char* v = getenv("MS_QDGEMM")) E.qdgemm_mode = atoi(v);
    if (const char* v = getenv("MS_LM_GEMM_MIN")) E.lm_gemm_min = atoi(v);
    // (the k-half block steps 128 k at a time: hidden sizes that are not a multiple of 128
    // keep the 4-wave block)
    E.dgemm_kh = cfg->max_batch <= 128 && E.H % 128 == 0 ? dgemm_kh_setting() : 1;
    if (const char* v = getenv("MS_QDF_MIN")) E.qdf_min = atoi(v);
    if (E.qdf_min > 0 && cfg->max_batch >= E.qdf_min) {  // splits measured at 256 rows (v22_*), any weights
      E.dsplit_qkv = 3;
      E.dsplit_down = 4;
    }
    if (const char* v = getenv("MS_DSPLIT_QKV")) E.dsplit_qkv = atoi(v);
    if (const char* v = getenv("MS_DSPLIT_O")) E.dsplit_o = atoi(v);
    if (const char* v = getenv("MS_DSPLIT_DOWN")) E.dsplit_down = atoi(v);
    if (const char* v = getenv("MS_DWN")) E.dwn_qkv = E.dwn_o = E.dwn_down = E.dwn_lm = atoi(v) == 8 ? 8 : 4;
    for (int* d : {&E.dsplit_qkv, &E.dsplit_o, &E.dsplit_down}) *d = std::min(std::max(*d, 1), (int)ms_engine::kMaxSplit);
    E.attn_ppw = attn_decode_ppw(cfg->max_batch, E.Hk, cfg->max_ctx);
    if (const char* v = getenv("MS_QSPLIT")) E.qsplit = atoi(v);
    if (const char* v = getenv("MS_RESID_FUSED")) E.resid_fuse = atoi(v) != 0;
    if (const char* v = getenv("MS_DECODE_TAIL")) E.tail_fuse = atoi(v) != 0;
    if (const char* v = getenv("MS_QRESID")) E.qresid = atoi(v) != 0;
    if (E.H % E.resid_rt || E.H / E.resid_rt > 256) E.resid_rt = 16;
    if (E.H % E.resid_rt || E.H / E.resid_rt > 256) E.resid_fuse = false;
    // the consumers stage the 256-tile statistics in LDS: engines of <= 16 slots (per engine,
    // so every step of it runs the same arithmetic)
    if (!gemv_rs_supported(cfg->max_batch, E.H / E.resid_rt)) E.resid_fuse = false;
    {
      const int Bg = std::min(cfg->max_batch, (int)ms_engine::kMaxGemvRows);
      E.qresid_ok = qgemv_supported(Bg, E.H, E.Hq * E.D, MS_GEMV_EPI_RESID_SSQ) &&
                    qgemv_supported(Bg, E.H, E.F, MS_GEMV_EPI_RESID_SSQ) &&
                    qgemv_supported(Bg, 2 * E.F, E.H, MS_GEMV_EPI_SWIGLU, E.H / E.resid_rt);
    }
    if (const char* v = getenv("MS_GRAPH_STEPS")) E.graph_steps = std::max(1, std::min(atoi(v), 16));
    for (ms_engine::Ctx* c : {&E.cp, &E.cd}) {
      c->args_cap = 8 * T + 64 * (size_t)cfg->max_batch + (size_t)cfg->max_batch * E.max_pages + 1024;
      c->args_d = E.dalloc<int32_t>(c->args_cap);
      HIP_OK(hipHostMalloc((void**)&c->args_h, c->args_cap * sizeof(int32_t), hipHostMallocDefault));
    }
    if (const char* v = getenv("MS_OVERLAP")) E.overlap = atoi(v) != 0;
    E.use(E.cp);
    HIP_OK(hipHostMalloc((void**)&E.ids_host, (size_t)ms_engine::kMaxRun * 256 * sizeof(int32_t),
                         hipHostMallocDefault));
    E.ids_ring_d = E.dalloc<int32_t>((size_t)ms_engine::kMaxRun * 256);
    // the persistent decode step (k_persist.hip)
    {
      int dev_cu = 0;
      HIP_OK(hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, cfg->device));
      E.n_cu = dev_cu;
      if (const char* v = getenv("MS_PERSIST")) E.persist = atoi(v) != 0;
      const int np_ws = (ws_ctx + kPage - 1) / kPage;
      E.nsplit_ws = (np_ws + E.attn_ppb - 1) / E.attn_ppb;
      E.persist_ok = persist_supported(cfg->max_batch, E.H, E.F, E.Hq, E.Hk, E.D, E.L, E.attn_ppb, E.n_cu) &&
                     E.slot_major && E.attn_v2 && E.resid_rt == 12;
      E.pk_sync = E.dalloc<unsigned>(persist_sync_words(E.L), true);
      E.pk_err_d = E.dalloc<unsigned>(4, true);
      HIP_OK(hipHostMalloc((void**)&E.pk_err_h, 64, hipHostMallocDefault));
      *E.pk_err_h = 0;
      E.pk_xg2 = E.dalloc<f16_t>((size_t)cfg->max_batch * E.H);
      E.pk_ssq2 = E.dalloc<float>((size_t)256 * cfg->max_batch, true);
    }
    HIP_OK(hipHostMalloc((void**)&E.first_host, (size_t)cfg->max_batch * sizeof(int32_t), hipHostMallocDefault));
    if (const char* v = getenv("MS_DECODE_RUN")) E.max_run = std::max(1, std::min(atoi(v), (int)ms_engine::kMaxRun));
    if (const char* ng = getenv("MAPSUM_NO_GRAPHS")) E.use_graphs = !(ng[0] == '1');
    HIP_OK(hipDeviceSynchronize());
    return MS_OK;
  });
  if (rc != MS_OK) {
    ms_destroy(e.release());
    return rc;
  }
  *out = e.release();
  return MS_OK;
}

int ms_destroy(ms_engine* e) {
  if (!e) return MS_OK;
  (void)hipSetDevice(e->cfg.device);
  for (ms_engine::Ctx* c : {&e->cp, &e->cd})
    if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : e->allocs) (void)hipFree(p);
  for (ms_engine::Ctx* c : {&e->cp, &e->cd})
    if (c->args_h) (void)hipHostFree(c->args_h);
  if (e->ids_host) (void)hipHostFree(e->ids_host);
  if (e->pk_err_h) (void)hipHostFree(e->pk_err_h);
  if (e->first_host) (void)hipHostFree(e->first_host);
  if (e->bt_h) (void)hipHostFree(e->bt_h);
  for (auto& kv : e->decode_graphs) (void)hipGraphExecDestroy(kv.second.first);
  for (auto& pe : e->ev_pairs) {
    (void)hipEventDestroy(pe.start);
    (void)hipEventDestroy(pe.stop);
  }
  for (ms_engine::Ctx* c : {&e->cp, &e->cd}) {
    if (c->ev_a) (void)hipEventDestroy(c->ev_a);
    if (c->ev_b) (void)hipEventDestroy(c->ev_b);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete e;
  return MS_OK;
}

const char* ms_last_error(const ms_engine* e) {
  if (e) return e->err.c_str();
  return g_last_error.c_str();
}

// where a logical tensor lives: fused fp16 destination + row map, and its K-quant slot
struct TensorDst {
  f16_t* dst = nullptr;
  int rows = 0, cols = 0, mul = 16, add = 0;
  QSlot* qs = nullptr;
  int qbit = 0, qneed = 0, qregion = 0, qrow0 = 0, qrows = 0;
};

static TensorDst tensor_dst(ms_engine& E, int tensor, int layer) {
  const bool per_layer = tensor != MS_T_EMBED && tensor != MS_T_FINAL_NORM && tensor != MS_T_LM_HEAD;
  REQUIRE(!per_layer || (layer >= 0 && layer < E.L), MS_EINVAL, "layer out of range");
  const int H = E.H, QD = E.Hq * E.D, KD = E.Hk * E.D;
  TensorDst t;
  auto q = [&](QSlot* s, int bit, int need, int region, int row0, int rows) {
    t.qs = s; t.qbit = bit; t.qneed = need; t.qregion = region; t.qrow0 = row0; t.qrows = rows;
  };
  switch (tensor) {
    case MS_T_EMBED:
      t.dst = E.embed; t.rows = E.V; t.cols = H;
      if (E.cfg.tie_embeddings) q(&E.lmq, 1, 1, 0, 0, E.V);
      break;
    case MS_T_LM_HEAD:
      REQUIRE(!E.cfg.tie_embeddings, MS_EINVAL, "lm_head is tied to the embedding");
      t.dst = E.lm_head; t.rows = E.V; t.cols = H; q(&E.lmq, 1, 1, 0, 0, E.V); break;
    case MS_T_FINAL_NORM: t.dst = E.final_norm; t.rows = 1; t.cols = H; break;
    case MS_T_ATTN_NORM: t.dst = E.layers[layer].attn_norm; t.rows = 1; t.cols = H; break;
    case MS_T_FFN_NORM: t.dst = E.layers[layer].ffn_norm; t.rows = 1; t.cols = H; break;
    case MS_T_WQ:  // rope-permuted rows (map_mul 0)
      t.dst = E.layers[layer].wqkv; t.rows = QD; t.cols = H; t.mul = 0;
      q(&E.lq[layer][QS_QKV], 1, 7, 0, 0, QD); break;
    case MS_T_WK:
      t.dst = E.layers[layer].wqkv; t.rows = KD; t.cols = H; t.mul = 0; t.add = QD;
      q(&E.lq[layer][QS_QKV], 2, 7, 1, QD, KD); break;
    case MS_T_WV:
      t.dst = E.layers[layer].wqkv; t.rows = KD; t.cols = H; t.add = QD + KD;
      q(&E.lq[layer][QS_QKV], 4, 7, 2, QD + KD, KD); break;
    case MS_T_WO:
      t.dst = E.layers[layer].wo; t.rows = H; t.cols = QD; q(&E.lq[layer][QS_O], 1, 1, 0, 0, H); break;
    case MS_T_WGATE:  // gate/up interleaved per 16 rows
      t.dst = E.layers[layer].wgu; t.rows = E.F; t.cols = H; t.mul = 32;
      q(&E.lq[layer][QS_GU], 1, 3, 0, 0, 2 * E.F); break;
    case MS_T_WUP:
      t.dst = E.layers[layer].wgu; t.rows = E.F; t.cols = H; t.mul = 32; t.add = 16;
      q(&E.lq[layer][QS_GU], 2, 3, 0, 0, 2 * E.F); break;
    case MS_T_WDOWN:
      t.dst = E.layers[layer].wdown; t.rows = H; t.cols = E.F; q(&E.lq[layer][QS_DOWN], 1, 1, 0, 0, H); break;
    default: throw MsError(MS_EINVAL, "unknown tensor id " + std::to_string(tensor));
  }
  return t;
}

int ms_load_weight(ms_engine* e, int32_t tensor, int32_t layer, const uint16_t* host, int64_t n) {
  if (!e) return MS_EINVAL;
  e->drop_graphs();
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    REQUIRE(host != nullptr, MS_EINVAL, "null weight buffer");
    HIP_OK(hipSetDevice(E.cfg.device));
    TensorDst t = tensor_dst(E, tensor, layer);
    REQUIRE(n == (int64_t)t.rows * t.cols, MS_EINVAL,
            "tensor " + std::to_string(tensor) + ": expected " + std::to_string((int64_t)t.rows * t.cols) +
                " elements, got " + std::to_string(n));
    if (t.qs) t.qs->loaded &= ~(uint32_t)t.qbit;  // a fp16 reload supersedes a quantised copy
    if (t.rows == 1) {
      HIP_OK(hipMemcpy(t.dst, host, (size_t)n * 2, hipMemcpyHostToDevice));
      return MS_OK;
    }
    void* tmp = nullptr;
    HIP_OK(hipMalloc(&tmp, (size_t)n * 2));
    hipError_t ce = hipMemcpy(tmp, host, (size_t)n * 2, hipMemcpyHostToDevice);
    if (ce == hipSuccess) {
      launch_scatter_rows((const f16_t*)tmp, t.dst, t.rows, t.cols, t.mul, t.add, E.stream);
      ce = hipStreamSynchronize(E.stream);
    }
    (void)hipFree(tmp);
    HIP_OK(ce);
    return MS_OK;
  });
}

static uint8_t* q_region(ms_engine& E, QSlot& s, int idx, int row0, int rows, int type, int K) {
  const uint8_t** base = idx == 0 ? &s.m.base0 : idx == 1 ? &s.m.base1 : &s.m.base2;
  int* rw0 = idx == 0 ? &s.m.row0_0 : idx == 1 ? &s.m.row0_1 : &s.m.row0_2;
  int* ty = idx == 0 ? &s.m.type0 : idx == 1 ? &s.m.type1 : &s.m.type2;
  int* rb = idx == 0 ? &s.m.row_bytes0 : idx == 1 ? &s.m.row_bytes1 : &s.m.row_bytes2;
  if (*base) {
    REQUIRE(*ty == type, MS_EINVAL, "tensors sharing a fused region (gate/up) need one quant type");
    return (uint8_t*)*base;
  }
  const int rowb = (K / 256) * qblock_bytes(type, true);
  uint8_t* p = E.dalloc<uint8_t>((size_t)rows * rowb);
  *base = p; *rw0 = row0; *ty = type; *rb = rowb;
  s.bytes[idx] = (size_t)rows * rowb;
  s.m.n = std::max(s.m.n, idx + 1);
  return p;
}

// device-resident raw ggml blocks of one logical tensor -> fp16 copy + quantised copy
static void load_quant(ms_engine& E, int tensor, int layer, int type, const uint8_t* dblocks) {
  TensorDst t = tensor_dst(E, tensor, layer);
  REQUIRE(t.rows > 1, MS_EINVAL, "RMSNorm weights are not quantised");
  REQUIRE(t.cols % 256 == 0, MS_EINVAL, "K-quant tensors need cols % 256 == 0");
  // an untied embedding is only gathered: its fp16 copy is all decode needs
  uint8_t* q = t.qs ? q_region(E, *t.qs, t.qregion, t.qrow0, t.qrows, type, t.cols) : nullptr;
  launch_quant_rows(type, dblocks, t.rows, t.cols, t.dst, t.mul, t.add, q, t.qrow0, E.stream);
  HIP_OK(hipGetLastError());
  E.has_quant = true;  // the K-quant decode GEMVs have no norm prologue: the unfused step
  if (t.qs) {
    t.qs->loaded |= (uint32_t)t.qbit;
    t.qs->need = (uint32_t)t.qneed;
  }
  E.note_quant(tensor, layer, type);
}

int ms_load_weight_q(ms_engine* e, int32_t tensor, int32_t layer, int32_t type, const void* host,
                     int64_t n_bytes) {
  if (!e) return MS_EINVAL;
  e->drop_graphs();
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    REQUIRE(host != nullptr, MS_EINVAL, "null block buffer");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K (12) or Q6_K (14)");
    HIP_OK(hipSetDevice(E.cfg.device));
    TensorDst t = tensor_dst(E, tensor, layer);
    const int64_t want = (int64_t)t.rows * (t.cols / 256) * qblock_bytes(type, false);
    REQUIRE(t.cols % 256 == 0 && n_bytes == want, MS_EINVAL,
            "tensor " + std::to_string(tensor) + ": expected " + std::to_string(want) + " bytes of blocks");
    void* tmp = nullptr;
    HIP_OK(hipMalloc(&tmp, (size_t)n_bytes));
    int rc = MS_OK;
    try {
      HIP_OK(hipMemcpy(tmp, host, (size_t)n_bytes, hipMemcpyHostToDevice));
      load_quant(E, tensor, layer, type, (const uint8_t*)tmp);
      HIP_OK(hipStreamSynchronize(E.stream));
    } catch (...) {
      (void)hipFree(tmp);
      throw;
    }
    (void)hipFree(tmp);
    return rc;
  });
}

int ms_declare_weight_q(ms_engine* e, int32_t tensor, int32_t layer, int32_t type) {
  if (!e) return MS_EINVAL;
  e->drop_graphs();
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K (12) or Q6_K (14)");
    HIP_OK(hipSetDevice(E.cfg.device));
    TensorDst t = tensor_dst(E, tensor, layer);
    REQUIRE(t.rows > 1 && t.cols % 256 == 0, MS_EINVAL, "not a K-quant matrix");
    E.has_quant = true;
    if (t.qs) {  // the layout of a quantised load, without its bytes (a broadcast fills them)
      q_region(E, *t.qs, t.qregion, t.qrow0, t.qrows, type, t.cols);
      t.qs->loaded |= (uint32_t)t.qbit;
      t.qs->need = (uint32_t)t.qneed;
    }
    E.note_quant(tensor, layer, type);
    return MS_OK;
  });
}

int ms_quant_manifest(const ms_engine* e, int32_t* triples, int32_t cap) {
  if (!e || cap < 0 || (cap > 0 && !triples)) return MS_EINVAL;
  const int n = (int)e->quant_manifest.size();
  for (int i = 0; i < std::min(n, (int)cap); ++i)
    for (int j = 0; j < 3; ++j) triples[3 * i + j] = e->quant_manifest[i][j];
  return n;
}

int ms_weight_regions(const ms_engine* e, void** ptrs, int64_t* bytes, int32_t cap) {
  if (!e || cap < 0 || (cap > 0 && (!ptrs || !bytes))) return MS_EINVAL;
  e->pk_packed_ok = false;  // the caller may write into the regions (weight broadcast)
  const auto r = e->weight_regions();
  for (int i = 0; i < std::min((int)r.size(), (int)cap); ++i) {
    ptrs[i] = r[i].first;
    bytes[i] = (int64_t)r[i].second;
  }
  return (int)r.size();
}

// Q4_K_M per-tensor mix (EXT llama.cpp; restated in oracle/quants.py q4_k_m_type)
static int q4_k_m_type(int tensor, int layer, int n_layers) {
  if (tensor == MS_T_EMBED || tensor == MS_T_LM_HEAD) return MS_QT_Q6_K;
  if (tensor == MS_T_WV || tensor == MS_T_WDOWN) {
    const bool more = layer < n_layers / 8 || layer >= 7 * n_layers / 8 ||
                      (layer - n_layers / 8) % 3 == 2;
    return more ? MS_QT_Q6_K : MS_QT_Q4_K;
  }
  return MS_QT_Q4_K;
}

int ms_init_synthetic_q(ms_engine* e, uint64_t seed, float scale, float jitter) {
  if (!e) return MS_EINVAL;
  e->drop_graphs();
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    HIP_OK(hipSetDevice(E.cfg.device));
    hipStream_t s = E.stream;
    size_t maxb = 0;
    const int mats[] = {MS_T_WQ, MS_T_WK, MS_T_WV, MS_T_WO, MS_T_WGATE, MS_T_WUP, MS_T_WDOWN};
    for (int tsr : mats) {
      TensorDst t = tensor_dst(E, tsr, 0);
      maxb = std::max(maxb, (size_t)t.rows * (t.cols / 256) * kQ6KBytes);
    }
    maxb = std::max(maxb, (size_t)E.V * (E.H / 256) * kQ6KBytes);
    void* tmp = nullptr;
    HIP_OK(hipMalloc(&tmp, maxb));
    try {
      auto one = [&](int tsr, int l) {
        TensorDst t = tensor_dst(E, tsr, l);
        const int ty = q4_k_m_type(tsr, l, E.L);
        launch_synth_qblocks(ty, (uint8_t*)tmp, (int64_t)t.rows * (t.cols / 256),
                             seed ^ ((uint64_t)tsr << 56) ^ ((uint64_t)l << 48), scale, s);
        load_quant(E, tsr, l, ty, (const uint8_t*)tmp);
      };
      one(E.cfg.tie_embeddings ? MS_T_EMBED : MS_T_LM_HEAD, 0);
      if (!E.cfg.tie_embeddings) one(MS_T_EMBED, 0);
      launch_synth_norm(E.final_norm, MS_T_FINAL_NORM, 0, E.H, seed, jitter, s);
      for (int l = 0; l < E.L; ++l) {
        launch_synth_norm(E.layers[l].attn_norm, MS_T_ATTN_NORM, l, E.H, seed, jitter, s);
        launch_synth_norm(E.layers[l].ffn_norm, MS_T_FFN_NORM, l, E.H, seed, jitter, s);
        for (int tsr : mats) one(tsr, l);
      }
      HIP_OK(hipStreamSynchronize(s));
    } catch (...) {
      (void)hipFree(tmp);
      throw;
    }
    (void)hipFree(tmp);
    return MS_OK;
  });
}

int ms_init_synthetic(ms_engine* e, uint64_t seed, float std_, float jitter) {
  if (!e) return MS_EINVAL;
  e->drop_graphs();
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    HIP_OK(hipSetDevice(E.cfg.device));
    const int H = E.H, QD = E.Hq * E.D, KD = E.Hk * E.D;
    hipStream_t s = E.stream;
    launch_synth_linear(E.embed, MS_T_EMBED, 0, E.V, H, seed, std_, 16, 0, s);
    if (!E.cfg.tie_embeddings) launch_synth_linear(E.lm_head, MS_T_LM_HEAD, 0, E.V, H, seed, std_, 16, 0, s);
    launch_synth_norm(E.final_norm, MS_T_FINAL_NORM, 0, H, seed, jitter, s);
    for (int l = 0; l < E.L; ++l) {
      Layer& Ly = E.layers[l];
      launch_synth_norm(Ly.attn_norm, MS_T_ATTN_NORM, l, H, seed, jitter, s);
      launch_synth_norm(Ly.ffn_norm, MS_T_FFN_NORM, l, H, seed, jitter, s);
      launch_synth_linear(Ly.wqkv, MS_T_WQ, l, QD, H, seed, std_, 0, 0, s);  // rope-permuted rows
      launch_synth_linear(Ly.wqkv, MS_T_WK, l, KD, H, seed, std_, 0, QD, s);
      launch_synth_linear(Ly.wqkv, MS_T_WV, l, KD, H, seed, std_, 16, QD + KD, s);
      launch_synth_linear(Ly.wo, MS_T_WO, l, H, QD, seed, std_, 16, 0, s);
      launch_synth_linear(Ly.wgu, MS_T_WGATE, l, E.F, H, seed, std_, 32, 0, s);
      launch_synth_linear(Ly.wgu, MS_T_WUP, l, E.F, H, seed, std_, 32, 16, s);
      launch_synth_linear(Ly.wdown, MS_T_WDOWN, l, H, E.F, seed, std_, 16, 0, s);
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(s));
    return MS_OK;
  });
}

static void submit_seq(ms_engine& E, const int32_t* ids, int32_t n, int32_t num_predict, uint32_t flags,
                       uint64_t tag, const int32_t* forced, int32_t n_forced) {
  REQUIRE(ids != nullptr && n >= 1, MS_EINVAL, "empty prompt");
  REQUIRE(num_predict >= 1, MS_EINVAL, "num_predict must be >= 1");
  REQUIRE((int64_t)n + num_predict <= E.cfg.max_ctx, MS_ENOSPC,
          "prompt (" + std::to_string(n) + ") + num_predict (" + std::to_string(num_predict) +
              ") exceeds max_ctx " + std::to_string(E.cfg.max_ctx));
  REQUIRE(n <= E.cfg.max_prefill_tokens, MS_ENOSPC, "prompt longer than max_prefill_tokens");
  const int need = (n + num_predict + kPage - 1) / kPage;
  REQUIRE(need <= E.n_pages, MS_ENOSPC, "request needs more KV pages than the pool holds");
  for (int i = 0; i < n; ++i)
    REQUIRE(ids[i] >= 0 && ids[i] < E.V, MS_EINVAL, "token id out of range at position " + std::to_string(i));
  auto s = std::make_unique<Seq>();
  if (forced) {
    REQUIRE(n_forced >= num_predict - 1, MS_EINVAL, "teacher forcing needs num_predict - 1 forced ids");
    for (int i = 0; i < num_predict - 1; ++i)
      REQUIRE(forced[i] >= 0 && forced[i] < E.V, MS_EINVAL, "forced id out of range at " + std::to_string(i));
    s->forced.assign(forced, forced + std::max(num_predict - 1, 0));
    s->forced.push_back(0);  // never fed: the last step's choice ends the sequence
  }
  s->tag = tag;
  s->prompt.assign(ids, ids + n);
  s->num_predict = num_predict;
  s->flags = flags;
  E.waiting.push_back(std::move(s));
}

int ms_submit(ms_engine* e, const int32_t* ids, int32_t n, int32_t num_predict, uint32_t flags,
              uint64_t tag) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    submit_seq(*e, ids, n, num_predict, flags, tag, nullptr, 0);
    return MS_OK;
  });
}

int ms_submit_forced(ms_engine* e, const int32_t* ids, int32_t n, const int32_t* forced, int32_t n_forced,
                     int32_t num_predict, uint32_t flags, uint64_t tag) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    REQUIRE(forced != nullptr || num_predict == 1, MS_EINVAL, "null forced ids");
    static const int32_t none = 0;
    submit_seq(*e, ids, n, num_predict, flags, tag, forced ? forced : &none, n_forced);
    return MS_OK;
  });
}

int ms_pending(const ms_engine* e) {
  if (!e) return MS_EINVAL;
  return (int)(e->waiting.size() + e->running.size());
}

static bool is_eos(const ms_engine& E, int32_t t) {
  if (!E.stop_set.empty()) return t >= 0 && t < (int)E.stop_set.size() && E.stop_set[t];
  for (int i = 0; i < E.cfg.n_eos; ++i)
    if (E.cfg.eos_ids[i] == t) return true;
  return false;
}

int ms_set_eos_ids(ms_engine* e, const int32_t* ids, int32_t n) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    REQUIRE(n >= 0 && (n == 0 || ids), MS_EINVAL, "bad stop-id list");
    std::vector<uint8_t> set;
    if (n > 0) {
      set.assign(E.V, 0);
      for (int i = 0; i < n; ++i) {
        REQUIRE(ids[i] >= 0 && ids[i] < E.V, MS_EINVAL, "stop id out of range");
        set[ids[i]] = 1;
      }
    }
    E.stop_set.swap(set);  // empty: back to the config's eos_ids
    return MS_OK;
  });
}

// returns true if the sequence finished with this token
static bool accept_token(ms_engine& E, Seq& s, int32_t t) {
  if (t < 0 || t >= E.V) {  // no finite logit (NaN/Inf in this chunk's activations)
    s.finish = MS_FINISH_ERROR;
    return true;
  }
  if (!(s.flags & MS_FLAG_IGNORE_EOS) && is_eos(E, t)) {
    s.finish = MS_FINISH_EOS;
    return true;
  }
  s.out.push_back(t);
  if ((int)s.out.size() >= s.num_predict) {
    s.finish = MS_FINISH_LENGTH;
    return true;
  }
  return false;
}

static void release(ms_engine& E, Seq& s) {
  for (int p : s.pages) E.free_pages.push_back(p);
  s.pages.clear();
  if (s.slot >= 0) E.free_slots.push_back(s.slot);
  s.slot = -1;
}

static void reserve(ms_engine& E, Seq& s, int tokens) {
  s.slot = E.free_slots.back();
  E.free_slots.pop_back();
  const int need = (tokens + kPage - 1) / kPage;
  for (int i = 0; i < need; ++i) {
    // slot-major pool: the free list only counts pages; the slot's own range is used
    s.pages.push_back(E.slot_major ? s.slot * E.max_pages + i : E.free_pages.back());
    E.free_pages.pop_back();
  }
  int32_t* row = &E.bt_h[(size_t)s.slot * E.max_pages];
  for (int i = 0; i < need; ++i) row[i] = s.pages[i];
  HIP_OK(hipMemcpyAsync(E.bt_d + (size_t)s.slot * E.max_pages, row, need * sizeof(int32_t),
                        hipMemcpyHostToDevice, E.stream));
}

// packed varlen prefill of `batch` (fresh sequences); writes K/V, returns first greedy ids.
// If n_layers_run < L: stops after that many layers (probe mode, no logits).
static void prefill(ms_engine& E, std::vector<Seq*>& batch, int n_layers_run, float* logits_all,
                    std::vector<int32_t>* first_ids) {
  const int S = (int)batch.size();
  int T = 0;
  for (Seq* s : batch) T += (int)s->prompt.size();
  std::vector<int32_t> a;
  a.reserve(4 * T + 8 * S + 64);
  const size_t o_ids = a.size();
  for (Seq* s : batch) a.insert(a.end(), s->prompt.begin(), s->prompt.end());
  const size_t o_pos = a.size();
  for (Seq* s : batch)
    for (int i = 0; i < (int)s->prompt.size(); ++i) a.push_back(s->len + i);
  const size_t o_slot = a.size();
  for (Seq* s : batch)
    for (int i = 0; i < (int)s->prompt.size(); ++i) a.push_back(s->slot);
  const size_t o_qstart = a.size();
  {
    int q = 0;
    for (Seq* s : batch) { a.push_back(q); q += (int)s->prompt.size(); }
  }
  const size_t o_qlen = a.size();
  for (Seq* s : batch) a.push_back((int)s->prompt.size());
  const size_t o_kvlen = a.size();
  for (Seq* s : batch) a.push_back(s->len + (int)s->prompt.size());
  const size_t o_sslot = a.size();
  for (Seq* s : batch) a.push_back(s->slot);
  const size_t o_last = a.size();
  {
    int q = 0;
    for (Seq* s : batch) { q += (int)s->prompt.size(); a.push_back(q - 1); }
  }
  // q-blocks, heaviest (latest positions) first
  std::vector<std::pair<int, int32_t>> qb;
  for (int i = 0; i < S; ++i) {
    const int n = (int)batch[i]->prompt.size();
    for (int b = 0; b < (n + kPrefillQRows - 1) / kPrefillQRows; ++b)
      qb.push_back({batch[i]->len + b * kPrefillQRows, (i << 16) | b});
  }
  std::stable_sort(qb.begin(), qb.end(), [](auto& x, auto& y) { return x.first > y.first; });
  const size_t o_qblk = a.size();
  for (auto& p : qb) a.push_back(p.second);
  int32_t* d = E.upload_args(a);

  PrefillAttnArgs pa;
  pa.seq_qstart = d + o_qstart;
  pa.seq_qlen = d + o_qlen;
  pa.seq_kvlen = d + o_kvlen;
  pa.seq_slot = d + o_sslot;
  pa.qblk = d + o_qblk;
  pa.n_qblk = (int)qb.size();
  pa.cos_tab = E.cos_tab;  // Q is rotated by the attention kernel as it stages it
  pa.sin_tab = E.sin_tab;
  DecodeAttnArgs da{};

  E.prof_begin(K_MISC);
  launch_embed(d + o_ids, T, E.embed, E.H, E.x, E.stream);
  E.prof_end(K_MISC);
  E.norm_input(E.layers[0].attn_norm, T);
  for (int l = 0; l < n_layers_run; ++l)
    E.run_layer(l, T, false, d + o_pos, d + o_slot, pa, da, l + 1 < E.L || logits_all);
  HIP_OK(hipGetLastError());
  if (n_layers_run < E.L) return;
  if (!logits_all && !first_ids) return;  // probe of the final residual only
  if (logits_all) {  // probe: logits of every position (xb = f16(x * final_norm), cur_rs)
    launch_gemm(E.xb, E.lm_head, logits_all, T, E.V, E.H, E.V, MS_EPI_STORE_F32, E.stream, &E.cur_rs);
    return;
  }
  E.norm_input(E.final_norm, S, d + o_last);
  // the first token goes through the decode lm_head GEMV in row groups of <= 64: its sum
  // order is then the decode steps' one whatever the number of admitted prompts
  for (int r0 = 0; r0 < S; r0 += ms_engine::kMaxGemvRows) {
    const int rows = std::min(S - r0, (int)ms_engine::kMaxGemvRows);
    const RowScale rs = make_row_scale(E.ssq + r0, 1, E.H, E.cfg.norm_eps);
    E.gemm_or_gemv(E.xb + (size_t)r0 * E.H, E.lm_head, E.logits + (size_t)r0 * E.V, rows, E.V, E.H, E.V,
                   MS_EPI_STORE_F32, true, K_LMHEAD, &rs);
  }
  E.prof_begin(K_MISC);
  launch_argmax(E.logits, S, E.V, E.ids_out_d, E.stream);
  E.prof_end(K_MISC);
  HIP_OK(hipGetLastError());
  // pinned landing buffer: a pageable destination would make this copy wait for the prefill
  // on the host, before the overlapping decode run is launched
  first_ids->resize(S);
  HIP_OK(hipMemcpyAsync(E.first_host, E.ids_out_d, S * sizeof(int32_t), hipMemcpyDeviceToHost, E.stream));
}

// the first layer's input of a decode step from the ids in the argument blob: x, xb = f16(x * g0)
// and its statistics (decode_run's first step; every later step gets them from the previous
// step's tail)
static void decode_head(ms_engine& E, int B, int32_t* d) {
  E.prof_begin(K_MISC);
  launch_embed(d, B, E.embed, E.H, E.x, E.stream, E.layers[0].attn_norm, E.xb, E.ssq);
  E.prof_end(K_MISC);
}

// argmax of the lm_head partials + decode_advance + the next step's decode_head, one launch
// (MS_DECODE_TAIL=0: the three launches; the same bits either way)
static void decode_tail(ms_engine& E, int B, int32_t* d, int tiles) {
  E.prof_begin(K_MISC);
  if (E.tail_fuse && B <= 256) {
    launch_decode_tail(E.logits, tiles, d, E.ids_out_d, E.ids_ring_d, B, E.V, E.embed, E.H, E.x,
                       E.layers[0].attn_norm, E.xb, E.ssq, E.stream);
    E.prof_end(K_MISC);
    return;
  }
  launch_argmax_partials(E.logits, B, tiles, E.ids_out_d, E.stream);
  E.prof_end(K_MISC);
  launch_decode_advance(d, E.ids_out_d, E.ids_ring_d, B, E.V, E.stream);
  decode_head(E, B, d);
}

// every layer of one decode step as the persistent launch (k_persist.hip): enters with layer 0's
// input in x / xb / ssq (one-tile statistics) and leaves the final norm's input in xb / ssq with
// 256 statistics tiles, like the per-layer launches it replaces
static void persist_layers(ms_engine& E, int B, const DecodeAttnArgs& da) {
  PkArgs a{};
  for (int l = 0; l < E.L; ++l) {
    const Layer& Ly = E.layers[l];
    const KVView kv = E.kv_layer(l);
    a.layers[l] = PkLayer{Ly.wqkv, Ly.wo, Ly.wgu, Ly.wdown, Ly.ffn_norm,
                          l + 1 < E.L ? E.layers[l + 1].attn_norm : E.final_norm, kv.k, kv.v,
                          E.pk_packed + (size_t)l * persist_packed_bytes_per_layer()};
  }
  a.L = E.L;
  a.B = B;
  a.seq_len = da.seq_len;
  a.seq_slot = da.seq_slot;
  a.max_pages = E.max_pages;
  a.ppb = E.attn_ppb;
  a.nsplit_ws = E.nsplit_ws;
  a.cos_tab = E.cos_tab;
  a.sin_tab = E.sin_tab;
  a.eps = E.cfg.norm_eps;
  a.inv_h = 1.0f / (float)E.H;
  a.scale_log2 = 1.4426950408889634f / sqrtf((float)E.D);
  a.rs0_tiles = E.cur_rs.tiles;
  a.x = E.x;
  a.xb = E.xb;
  a.ssq = E.ssq;
  a.slabs = E.slabs;
  a.ws = E.attn_ws;
  a.attn = E.attn;
  a.xg2 = E.pk_xg2;
  a.ssq2 = E.pk_ssq2;
  a.hbuf = E.hbuf;
  a.sync = E.pk_sync;
  a.err = E.pk_err_d;
  E.prof_begin(K_PERSIST);
  launch_decode_step(a, E.stream);
  E.prof_end(K_PERSIST);
  E.pending_split = 0;
  E.cur_rs = make_row_scale(E.ssq, E.H / E.resid_rt, E.H, E.cfg.norm_eps);
}

// kernels of one decode step (no host synchronisation: capturable into a hipGraph).  Enters
// with the step's layer-0 input in x / xb / ssq and leaves the NEXT step's there: the greedy
// ids, the argument advance and the next embedding gather are one launch (decode_tail_kernel)
// on the argmax-partials lm_head paths.
static void decode_body(ms_engine& E, int B, int32_t* d, const DecodeAttnArgs& da) {
  const size_t o_pos = B, o_slot = 2 * (size_t)B;
  PrefillAttnArgs pa{};
  E.pending_split = 0;
  E.cur_rs = E.norm_rs();
  if (E.persist_on(B)) {
    persist_layers(E, B, da);
  } else {
    // every layer leaves xb = f16(x * the next gain) with its deferred scale in cur_rs
    for (int l = 0; l < E.L; ++l) E.run_layer(l, B, true, d + o_pos, d + o_slot, pa, da);
  }
  const RowScale rs = E.cur_rs;
  if (E.large(B) && dgemm_supported(B, E.V, E.H, 1, MS_GEMV_EPI_ARGMAX, 1)) {
    const int tiles = E.V / 16;
    E.prof_begin(K_LMHEAD);
    // no row scale: r > 0 keeps every row's order (the logits themselves are never stored)
    // 4-wave blocks always: a 2004-block grid keeps two per CU (k_dgemm.hip kh)
    if (E.qd(&E.lmq, B, E.V, E.H, 1, MS_GEMV_EPI_ARGMAX))
      launch_qdgemm(E.xb, E.lmq.m, E.logits, B, E.V, E.H, 1, tiles, MS_GEMV_EPI_ARGMAX, E.stream, nullptr);
    else if (E.lm_gemm_min > 0 && E.cfg.max_batch >= E.lm_gemm_min && E.H % 64 == 0 && E.V % 16 == 0)
      launch_gemm(E.xb, E.lm_head, E.logits, B, E.V, E.H, tiles, MS_GEMV_EPI_ARGMAX, E.stream);
    else
      launch_dgemm(E.xb, E.lm_head, E.logits, B, E.V, E.H, 1, tiles, MS_GEMV_EPI_ARGMAX, E.stream, nullptr, 1,
                   B <= 128 && E.V % 128 == 0 ? E.dwn_lm : 4);
    E.prof_end(K_LMHEAD);
    decode_tail(E, B, d, tiles);
    return;
  } else if (gemv_supported(std::min(B, (int)ms_engine::kMaxGemvRows), E.V, E.H, MS_GEMV_EPI_ARGMAX) &&
             (B <= ms_engine::kMaxGemvRows || E.row_groups(B))) {
    // greedy argmax in the lm_head epilogue: {max, id} per 16-column tile, no logits row
    const int tiles = E.V / 16;
    E.proj(&E.lmq, E.xb, E.lm_head, E.logits, B, E.V, E.H, tiles, MS_GEMV_EPI_ARGMAX, nullptr, K_LMHEAD,
           sizeof(float2));
    decode_tail(E, B, d, tiles);
    return;
  }
  E.gemm_or_gemv(E.xb, E.lm_head, E.logits, B, E.V, E.H, E.V, MS_EPI_STORE_F32, true, K_LMHEAD, &rs);
  E.prof_begin(K_MISC);
  launch_argmax(E.logits, B, E.V, E.ids_out_d, E.stream);
  E.prof_end(K_MISC);
  // the next chained step's arguments on the device, then its input rows
  launch_decode_advance(d, E.ids_out_d, E.ids_ring_d, B, E.V, E.stream);
  decode_head(E, B, d);
}

// k chained greedy decode steps for every sequence of `batch` (B rows of one token each)
// with ONE host synchronisation: the arguments are uploaded once, each step's argmax ids
// feed the next step on the device (decode_advance), and each step's ids are copied to a
// pinned ring.  The caller picks k so that no sequence reaches num_predict inside the run
// and the split grid of decode attention (longest sequence rounded up to 256 keys) does not
// change; a sequence that stops early (EOS, failed row) keeps computing until the run ends
// and its extra tokens are dropped -- its reserved pages hold them, and no other row
// depends on it (batch-invariant kernels).  ids[j * B + i] = token of row i at step j.
static void decode_run(ms_engine& E, std::vector<Seq*>& batch, int k, std::vector<int32_t>& ids) {
  const int B = (int)batch.size();
  std::vector<int32_t> a;
  a.reserve(4 * B);
  int max_len = 0;
  for (Seq* s : batch) a.push_back(s->next_input());  // [0, B)   token ids
  for (Seq* s : batch) a.push_back(s->len);         // [B, 2B)  positions
  for (Seq* s : batch) a.push_back(s->slot);        // [2B, 3B) block-table rows
  for (Seq* s : batch) { a.push_back(s->len + 1); max_len = std::max(max_len, s->len + 1); }
  a.push_back(0);                                   // [4B]     step of the run (ring row)
  a.push_back(0);                                   // [4B+1]   decode_tail's arrival ticket
  // the persistent step runs (captured or eagerly) exactly when persist_on holds for this run;
  // toggling it drops the cached graphs (ms_set_persist, the timeout fallback below)
  E.pk_used = E.persist_on(B);
  if (E.pk_used && !E.pk_packed_ok) {
    // its weights in stream order: allocated once (the engine falls back to the launches if
    // the 5.6 GB do not fit), rebuilt from the [N][K] matrices after every weight (re)load
    if (!E.pk_packed) {
      void* p = nullptr;
      if (hipMalloc(&p, persist_packed_bytes_per_layer() * E.L) == hipSuccess) {
        E.pk_packed = (char*)p;
        E.allocs.push_back(p);
      } else {
        (void)hipGetLastError();
        E.persist = false;
        E.pk_used = false;
      }
    }
    if (E.pk_used) {
      for (int l = 0; l < E.L; ++l) {
        const Layer& Ly = E.layers[l];
        launch_pack_layer(Ly.wqkv, Ly.wo, Ly.wgu, Ly.wdown, E.pk_packed + (size_t)l * persist_packed_bytes_per_layer(),
                          E.stream);
      }
      HIP_OK(hipGetLastError());
      E.pk_packed_ok = true;
    }
  }
  HIP_OK(hipEventRecord(E.ev_a, E.stream));
  int32_t* d = E.upload_args(a);
  decode_head(E, B, d);  // the first step's input; each step's tail gathers the next one's
  DecodeAttnArgs da;
  da.seq_len = d + 3 * (size_t)B;
  da.seq_slot = d + 2 * (size_t)B;
  da.B = B;
  // the split grid only depends on the longest sequence rounded up to 256 keys
  da.max_len = ((max_len + k - 1 + 255) / 256) * 256;
  da.ppw = E.attn_ppw;
  auto graph = [&](int steps) {  // `steps` chained decode bodies in one graph
    const auto key = std::make_tuple(B, da.max_len, steps);
    auto it = E.decode_graphs.find(key);
    if (it == E.decode_graphs.end()) {
      E.evict_graphs();
      hipGraph_t g = nullptr;
      hipGraphExec_t ex = nullptr;
      HIP_OK(hipStreamBeginCapture(E.stream, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < steps; ++i) decode_body(E, B, d, da);
      HIP_OK(hipStreamEndCapture(E.stream, &g));
      HIP_OK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      HIP_OK(hipGraphDestroy(g));
      it = E.decode_graphs.emplace(key, std::make_pair(ex, (uint64_t)0)).first;
      E.stats.graphs_built += 1;
    }
    it->second.second = ++E.graph_clock;
    return it->second.first;
  };
  if (E.use_graphs && E.prof_mask == 0) {
    const int G = std::max(1, E.graph_steps);
    for (int j = 0; j + G <= k; j += G) HIP_OK(hipGraphLaunch(graph(G), E.stream));
    for (int j = 0; j < k % G; ++j) HIP_OK(hipGraphLaunch(graph(1), E.stream));
  } else {
    for (int j = 0; j < k; ++j) decode_body(E, B, d, da);
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(E.ev_b, E.stream));
  HIP_OK(hipMemcpyAsync(E.ids_host, E.ids_ring_d, (size_t)k * B * sizeof(int32_t), hipMemcpyDeviceToHost,
                        E.stream));
  if (E.pk_used)
    HIP_OK(hipMemcpyAsync(E.pk_err_h, E.pk_err_d, sizeof(unsigned), hipMemcpyDeviceToHost, E.stream));
  ids.resize((size_t)k * B);
  HIP_OK(hipStreamSynchronize(E.stream));
  if (E.pk_used && *E.pk_err_h) {
    // a hand-off of the persistent step timed out (a workgroup was not resident): never silent,
    // never a hang.  Turn the persistent step off for this engine, reset its counters and flag,
    // drop every graph that holds it, and recompute the whole run with the per-layer launches:
    // the run started from the sequences' own state (args above), and every K / V row it wrote
    // is at a position the recomputation writes again
    fprintf(stderr, "mapsum: persistent decode step timed out (code 0x%x); recomputing with the launches\n",
            *E.pk_err_h);
    E.persist = false;
    E.pk_used = false;
    HIP_OK(hipMemsetAsync(E.pk_sync, 0, persist_sync_words(E.L) * sizeof(unsigned), E.stream));
    HIP_OK(hipMemsetAsync(E.pk_err_d, 0, 4 * sizeof(unsigned), E.stream));
    HIP_OK(hipStreamSynchronize(E.stream));
    *E.pk_err_h = 0;
    E.drop_graphs();
    E.stats.persist_fallbacks += 1;
    decode_run(E, batch, k, ids);
    return;
  }
  if (E.pk_used) E.stats.persist_steps += k;
  E.pk_used = false;
  std::memcpy(ids.data(), E.ids_host, (size_t)k * B * sizeof(int32_t));
}

int ms_step(ms_engine* e) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    HIP_OK(hipSetDevice(E.cfg.device));
    // Profiling runs serialise the phases, so every bracketed launch runs alone on the chip.
    const bool ov = E.overlap && E.prof_mask == 0;
    TraceRange tr_step("mapsum.step");
    // 1. admit (the new slots' block-table rows go out on the prefill stream)
    E.use(E.cp);
    std::vector<Seq*> admitted;
    int budget = E.cfg.max_prefill_tokens;
    while (!E.waiting.empty() && !E.free_slots.empty()) {
      Seq& s = *E.waiting.front();
      const int n = (int)s.prompt.size();
      const int need = (n + s.num_predict + kPage - 1) / kPage;
      if (need > (int)E.free_pages.size() || n > budget) break;
      reserve(E, s, n + s.num_predict);
      budget -= n;
      admitted.push_back(&s);
      E.running.push_back(std::move(E.waiting.front()));
      E.waiting.pop_front();
    }
    // 2. prefill the admitted prompts on the prefill stream; with overlap the host does not
    // wait here: the decode run below proceeds on the decode stream meanwhile, and the new
    // chunks join the decode batch from the next step on
    std::vector<int32_t> first;
    auto finish_prefill = [&]() {
      HIP_OK(hipStreamSynchronize(E.cp.stream));
      float ms_ = 0.f;
      HIP_OK(hipEventElapsedTime(&ms_, E.cp.ev_a, E.cp.ev_b));
      E.stats.prefill_ms += ms_;
      E.stats.prefill_passes += 1;
      for (size_t i = 0; i < admitted.size(); ++i) {
        Seq& s = *admitted[i];
        s.len = (int)s.prompt.size();
        E.stats.prefill_tokens += s.len;
        accept_token(E, s, E.first_host[i]);
      }
    };
    if (!admitted.empty()) {
      TraceRange tr("mapsum.prefill");
      HIP_OK(hipEventRecord(E.cp.ev_a, E.cp.stream));
      prefill(E, admitted, E.L, nullptr, &first);
      HIP_OK(hipEventRecord(E.cp.ev_b, E.cp.stream));
      if (!ov) {
        finish_prefill();
        E.prof_collect();
      }
    }
    // 3. decode every running sequence that still needs tokens and has been prefilled: a run
    // of k chained steps (one host synchronisation), k bounded by the nearest num_predict, the
    // attention split grid and kMaxRun; k = 1 while admissible work waits for a free slot
    E.use(E.cd);
    std::vector<Seq*> batch;
    for (auto& s : E.running)
      if (!s->finish && s->len > 0) batch.push_back(s.get());
    for (size_t i0 = 0; i0 < batch.size(); i0 += 256) {
      std::vector<Seq*> sub(batch.begin() + i0, batch.begin() + std::min(batch.size(), i0 + 256));
      int k = (batch.size() > 256 || (!E.waiting.empty() && !E.free_slots.empty())) ? 1 : E.max_run;
      // chunks wait for a slot: a chunk that stops at EOS inside the run keeps its slot until
      // the run ends, so bound the run by one captured graph (<= 16 steps) instead of 64
      if (!E.waiting.empty()) k = std::min(k, std::max(1, E.graph_steps));
      // a prefill is in flight on the other stream: decode a whole graph of steps under it
      // (a one-step run would leave the prefill exposed)
      if (ov && !admitted.empty() && batch.size() <= 256) k = std::max(k, std::max(1, E.graph_steps));
      int max_len = 0;
      for (Seq* s : sub) {
        k = std::min(k, s->num_predict - (int)s->out.size());
        if (!s->forced.empty()) k = 1;  // the next input is the forced id, not this step's choice
        max_len = std::max(max_len, s->len + 1);
      }
      k = std::max(1, std::min(k, ((max_len + 255) / 256) * 256 - max_len + 1));
      std::vector<int32_t> ids;
      {
        TraceRange tr("mapsum.decode_run");
        decode_run(E, sub, k, ids);  // records ev_a/ev_b around its device work and syncs
      }
      float ms_ = 0.f;
      HIP_OK(hipEventElapsedTime(&ms_, E.ev_a, E.ev_b));
      E.stats.decode_ms += ms_;
      E.prof_collect();
      E.stats.decode_steps += k;
      E.stats.decode_tokens += (int64_t)sub.size() * k;
      for (int j = 0; j < k; ++j)
        for (size_t i = 0; i < sub.size(); ++i) {
          Seq& s = *sub[i];
          if (s.finish) continue;  // stopped earlier in the run: drop the rest
          E.stats.decode_kv_tokens += s.len + 1;
          s.len += 1;
          accept_token(E, s, ids[(size_t)j * sub.size() + i]);
        }
    }
    if (ov && !admitted.empty()) finish_prefill();
    E.use(E.cp);
    // 4. retire finished sequences
    for (auto it = E.running.begin(); it != E.running.end();) {
      if ((*it)->finish) {
        release(E, **it);
        E.stats.finished += 1;
        E.done.push_back(std::move(*it));
        it = E.running.erase(it);
      } else {
        ++it;
      }
    }
    return (int)(E.waiting.size() + E.running.size());
  });
}

int ms_poll(ms_engine* e, ms_result* out, int32_t cap) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    REQUIRE(cap >= 0 && (cap == 0 || out != nullptr), MS_EINVAL, "bad poll buffer");
    E.polled.clear();  // invalidates ids handed out by the previous poll
    const int n = std::min<int>(cap, (int)E.done.size());
    for (int i = 0; i < n; ++i) {
      Seq& s = *E.done[i];
      out[i].tag = s.tag;
      out[i].ids = s.out.data();
      out[i].n_ids = (int32_t)s.out.size();
      out[i].finish_reason = s.finish;
      out[i].n_prompt = (int32_t)s.prompt.size();
      out[i]._pad = 0;
    }
    for (int i = 0; i < n; ++i) E.polled.push_back(std::move(E.done[i]));
    E.done.erase(E.done.begin(), E.done.begin() + n);
    return n;
  });
}

int ms_trace_push(const char* name) {
  if (!name) return MS_EINVAL;
  roctxRangePushA(name);
  return MS_OK;
}

int ms_trace_pop(void) {
  roctxRangePop();
  return MS_OK;
}

int ms_get_stats(const ms_engine* e, ms_stats* out) {
  if (!e || !out) return MS_EINVAL;
  *out = e->stats;
  return MS_OK;
}

int ms_reset_stats(ms_engine* e) {
  if (!e) return MS_EINVAL;
  e->stats = ms_stats{};
  return MS_OK;
}

int ms_set_profiling(ms_engine* e, uint32_t mask) {
  if (!e) return MS_EINVAL;
  e->prof_mask = mask;
  return MS_OK;
}

int ms_set_persist(ms_engine* e, int32_t on) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    HIP_OK(hipStreamSynchronize(e->cd.stream));
    e->persist = on != 0;
    e->drop_graphs();
    return (e->persist_ok ? 1 : 0);
  });
}

int ms_debug_read(ms_engine* e, int32_t which, int64_t offset, void* host, int64_t bytes) {
  if (!e || !host || offset < 0 || bytes < 0) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    const void* base = nullptr;
    size_t cap = 0;
    switch (which) {
      case MS_DBG_KPOOL: base = E.kpool; cap = E.layer_kv_elems * E.L * sizeof(f16_t); break;
      case MS_DBG_VPOOL: base = E.vpool; cap = E.layer_kv_elems * E.L * sizeof(f16_t); break;
      case MS_DBG_DECODE_LOGITS: base = E.cd.logits; cap = (size_t)E.cfg.max_batch * E.V * sizeof(float); break;
      case MS_DBG_DECODE_X: base = E.cd.x; cap = (size_t)E.cfg.max_batch * E.H * sizeof(float); break;
      default: REQUIRE(false, MS_EINVAL, "ms_debug_read: unknown buffer");
    }
    REQUIRE((size_t)offset + (size_t)bytes <= cap, MS_EINVAL, "ms_debug_read: range past the buffer");
    HIP_OK(hipStreamSynchronize(E.cd.stream));
    HIP_OK(hipStreamSynchronize(E.cp.stream));
    HIP_OK(hipMemcpy(host, (const char*)base + offset, (size_t)bytes, hipMemcpyDeviceToHost));
    return MS_OK;
  });
}

int ms_debug_pk_stamps(uint64_t* out, int32_t n) {
  if (!out || n < 0) return MS_EINVAL;
  ms::persist_stamps(reinterpret_cast<unsigned long long*>(out), n);
  return MS_OK;
}

int ms_debug_a2_stamps(uint64_t* out, int32_t n) {
  if (!out || n < 0) return MS_EINVAL;
  ms::attn2_stamps(reinterpret_cast<unsigned long long*>(out), n);
  return MS_OK;
}

int ms_synchronize(ms_engine* e) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    HIP_OK(hipStreamSynchronize(e->cp.stream));
    HIP_OK(hipStreamSynchronize(e->cd.stream));
    return MS_OK;
  });
}

int ms_forward_packed(ms_engine* e, const int32_t* ids, const int32_t* lens, int32_t n_seqs,
                      int32_t n_layers_run, float* hidden_out, float* logits_out) {
  if (!e) return MS_EINVAL;
  return guarded(e, [&]() -> int {
    ms_engine& E = *e;
    HIP_OK(hipSetDevice(E.cfg.device));
    REQUIRE(E.waiting.empty() && E.running.empty(), MS_EBUSY, "ms_forward needs an idle engine");
    REQUIRE(ids && lens && n_seqs >= 1 && n_seqs <= (int)E.free_slots.size(), MS_EINVAL,
            "bad probe batch (1 <= n_seqs <= max_batch)");
    REQUIRE(n_layers_run >= 0 && n_layers_run <= E.L, MS_EINVAL, "n_layers_run out of range");
    REQUIRE(!logits_out || n_layers_run == E.L, MS_EINVAL, "logits need every layer");
    int64_t T = 0, pages = 0;
    for (int i = 0; i < n_seqs; ++i) {
      REQUIRE(lens[i] >= 1 && lens[i] <= E.cfg.max_ctx, MS_EINVAL, "bad probe length");
      T += lens[i];
      pages += (lens[i] + kPage - 1) / kPage;
    }
    REQUIRE(T <= E.cfg.max_prefill_tokens, MS_EINVAL, "probe longer than max_prefill_tokens");
    REQUIRE(pages <= (int64_t)E.free_pages.size(), MS_ENOSPC, "not enough KV pages");
    for (int64_t i = 0; i < T; ++i) REQUIRE(ids[i] >= 0 && ids[i] < E.V, MS_EINVAL, "token id out of range");
    E.use(E.cp);
    std::vector<Seq> seqs(n_seqs);
    std::vector<Seq*> b;
    int64_t off = 0;
    for (int i = 0; i < n_seqs; ++i) {
      seqs[i].prompt.assign(ids + off, ids + off + lens[i]);
      off += lens[i];
      reserve(E, seqs[i], lens[i]);
      b.push_back(&seqs[i]);
    }
    float* lg = nullptr;
    try {
      if (logits_out) HIP_OK(hipMalloc((void**)&lg, (size_t)T * E.V * sizeof(float)));
      prefill(E, b, n_layers_run, lg, nullptr);
      HIP_OK(hipStreamSynchronize(E.stream));
      if (hidden_out)
        HIP_OK(hipMemcpy(hidden_out, E.x, (size_t)T * E.H * sizeof(float), hipMemcpyDeviceToHost));
      if (logits_out)
        HIP_OK(hipMemcpy(logits_out, lg, (size_t)T * E.V * sizeof(float), hipMemcpyDeviceToHost));
    } catch (...) {
      if (lg) (void)hipFree(lg);
      for (Seq& s : seqs) release(E, s);
      throw;
    }
    if (lg) (void)hipFree(lg);
    for (Seq& s : seqs) release(E, s);
    E.ev_pending.clear();
    E.ev_used = 0;
    return MS_OK;
  });
}

int ms_forward(ms_engine* e, const int32_t* ids, int32_t n, int32_t n_layers_run, float* hidden_out,
               float* logits_out) {
  return ms_forward_packed(e, ids, &n, 1, n_layers_run, hidden_out, logits_out);
}

// ---------------------------------------------------------------------------- op entry points
static int op_guard(const std::function<void()>& fn) {
  try {
    fn();
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
      g_last_error = std::string("kernel launch failed: ") + hipGetErrorString(err);
      return MS_EIO;
    }
    return MS_OK;
  } catch (const MsError& x) {
    g_last_error = x.what();
    return x.code;
  }
}

// the deferred RMSNorm scale the next op calls of this thread apply (ms_op_set_row_scale)
static thread_local RowScale g_op_rs{};

int ms_op_set_row_scale(const float* ssq, int32_t tiles, int32_t hidden, float eps) {
  if (ssq && (tiles < 1 || hidden < 1)) return MS_EINVAL;
  g_op_rs = ssq ? make_row_scale(ssq, tiles, hidden, eps) : RowScale{};
  return MS_OK;
}

static int op_rs_tiles() { return g_op_rs.ssq ? g_op_rs.tiles : 0; }

static const GemvArgs* op_gemv_args(GemvArgs& ga) {
  ga = GemvArgs{};
  ga.rs = g_op_rs;
  return g_op_rs.ssq ? &ga : nullptr;
}

int ms_op_gemm(const void* A, const void* W, void* out, int32_t M, int32_t N, int32_t K, int32_t ldo,
               int32_t epi, void* stream) {
  return op_guard([&] {
    REQUIRE(A && W && out && M >= 1 && N >= 16 && K >= 64 && K % 64 == 0, MS_EINVAL, "bad gemm shape");
    REQUIRE(((epi >= 0 && epi <= 3) || epi == MS_EPI_ARGMAX) && (epi != MS_EPI_SWIGLU || N % 32 == 0), MS_EINVAL,
            "bad epilogue");
    REQUIRE(epi != MS_EPI_ADD_F32 || (N % 4 == 0 && ldo % 4 == 0), MS_EINVAL,
            "residual gemm: N and ldo multiples of 4 (16-B x rows)");
    // argmax: {max, id} float2 partials [M][ldo >= N / 16], the 128x128 tile, no row scale
    REQUIRE(epi != MS_EPI_ARGMAX || (N % 16 == 0 && ldo >= N / 16), MS_EINVAL, "gemm argmax: N % 16, ldo >= N / 16");
    // the epilogues store 4 consecutive columns per lane (8 B fp16, 16 B fp32)
    REQUIRE(((uintptr_t)out & ((epi == MS_EPI_ADD_F32 || epi == MS_EPI_STORE_F32) ? 15 : 7)) == 0, MS_EINVAL,
            "gemm: out must be 16-B (fp32) / 8-B (fp16) aligned");
    REQUIRE(!g_op_rs.ssq || gemm_rs_tiles_ok(M, N, g_op_rs.tiles), MS_EINVAL,
            "gemm row scale: at most 24 tiles of statistics (kGemmRsTiles, both GEMM tiles)");
    launch_gemm((const f16_t*)A, (const f16_t*)W, out, M, N, K, ldo, epi == MS_EPI_ARGMAX ? MS_GEMV_EPI_ARGMAX : epi,
                (hipStream_t)stream, &g_op_rs);
  });
}

int ms_op_gemm_resid(const void* A, const void* W, float* x, void* xg_out, const void* gamma, float* ssq_out,
                     int32_t M, int32_t N, int32_t K, void* stream) {
  return op_guard([&] {
    REQUIRE(A && W && x && xg_out && gamma && ssq_out && M >= 1 && N >= 16 && K >= 64 && K % 64 == 0, MS_EINVAL,
            "bad gemm_resid operands (K % 64 == 0)");
    REQUIRE(gemm_resid_tiles(M, N) <= kGemmRsTiles, MS_EINVAL, "gemm_resid: N over 24 column tiles");
    REQUIRE(N % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)xg_out & 7) == 0, MS_EINVAL,
            "gemm_resid: N a multiple of 4, x 16-B and xg 8-B aligned (vector rows)");
    GemmResid gr{(const f16_t*)gamma, (f16_t*)xg_out, ssq_out};
    launch_gemm((const f16_t*)A, (const f16_t*)W, x, M, N, K, N, MS_EPI_ADD_F32, (hipStream_t)stream, nullptr, &gr);
  });
}

int ms_gemm_resid_tiles(int32_t M, int32_t N) { return gemm_resid_tiles(M, N); }

int ms_set_gemm_variant(int32_t v) {
  if (v < 0 || v > 4) return MS_EINVAL;
  set_gemm_variant(v);
  return MS_OK;
}

int ms_set_attn_tuning(int32_t combine_grp, int32_t order) {
  if (combine_grp < 0 || combine_grp > 1 || (order != 0 && order != 3)) return MS_EINVAL;
  set_attn_tuning(combine_grp, order);
  return MS_OK;
}

int ms_set_dgemm_kh(int32_t kh) {
  if (kh != 1 && kh != 2) return MS_EINVAL;
  set_dgemm_kh(kh);
  return MS_OK;
}

int ms_set_dgemm_wn(int32_t wn) {
  if (wn != 4 && wn != 8) return MS_EINVAL;
  set_dgemm_wn(wn);
  return MS_OK;
}

int ms_set_qgemv_gs(int32_t on) {
  if (on < 0 || on > 1) return MS_EINVAL;
  set_qgemv_gs(on != 0);
  return MS_OK;
}

int64_t ms_op_gemv_workspace(int32_t M, int32_t N, int32_t K) {
  if (M < 1 || M > 64 || N < 16 || K < 64 || K % 64) return MS_EINVAL;
  return (int64_t)gemv_workspace_bytes(M, N, K);
}

int ms_op_gemv(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K, int32_t ldo,
               int32_t epi, void* ws, void* stream) {
  return ms_op_gemv_tuned(X, W, out, M, N, K, ldo, epi, ws, 0, stream);
}

int ms_op_gemv_tuned(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K,
                     int32_t ldo, int32_t epi, void* ws, int32_t waves, void* stream) {
  return op_guard([&] {
    REQUIRE(X && W && out && ws && N >= 16 && N % 16 == 0, MS_EINVAL, "bad gemv operands");
    REQUIRE(((epi >= 0 && epi <= 3) || epi == MS_EPI_ARGMAX) && (epi != MS_EPI_SWIGLU || N % 32 == 0),
            MS_EINVAL, "bad epilogue");
    REQUIRE(gemv_supported(M, N, K, epi, op_rs_tiles()), MS_EINVAL,
            "gemv shape unsupported (M<=64, K%64==0, K/64 split into <=16 waves of <=8 steps; "
            "row-scale statistics within kRsStage and LDS)");
    GemvArgs ga;
    launch_gemv_ex((const f16_t*)X, (const f16_t*)W, out, M, N, K, ldo, epi, op_gemv_args(ga), waves,
                   (hipStream_t)stream);
  });
}

int ms_op_gemv_strided(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K,
                       int32_t ldk, int32_t ldo, int32_t epi, void* stream) {
  return op_guard([&] {
    REQUIRE(X && W && out && N >= 16 && N % 16 == 0 && ldk >= K && ldk % 8 == 0, MS_EINVAL,
            "bad strided gemv operands");
    REQUIRE(epi >= 0 && epi <= 3 && epi != MS_EPI_SWIGLU, MS_EINVAL, "bad epilogue");
    REQUIRE(gemv_supported(M, N, K, epi), MS_EINVAL, "gemv shape unsupported");
    launch_gemv_strided((const f16_t*)X, (const f16_t*)W, out, M, N, K, ldk, ldo, epi, (hipStream_t)stream);
  });
}

int ms_op_gemv_resid(const void* X, const void* W, float* x, void* xg_out, const void* gamma,
                     float* ssq_out, int32_t M, int32_t N, int32_t K, int32_t rt, void* stream) {
  return op_guard([&] {
    REQUIRE(X && W && x && xg_out && gamma && ssq_out && rt >= 1 && rt <= 16 && N % rt == 0, MS_EINVAL,
            "bad gemv_resid operands");
    REQUIRE(gemv_supported(M, N, K, MS_GEMV_EPI_RESID_SSQ), MS_EINVAL, "gemv_resid shape unsupported");
    GemvArgs ga{};
    ga.rt = rt;
    ga.ssq_out = ssq_out;
    ga.gamma = (const f16_t*)gamma;
    ga.xg_out = (f16_t*)xg_out;
    launch_gemv_ex((const f16_t*)X, (const f16_t*)W, x, M, N, K, N, MS_GEMV_EPI_RESID_SSQ, &ga, 0,
                   (hipStream_t)stream);
  });
}

int ms_op_dgemm(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K, int32_t S,
                int32_t ldo, int32_t epi, void* stream) {
  return op_guard([&] {
    REQUIRE(X && W && out, MS_EINVAL, "bad dgemm operands");
    REQUIRE(((epi >= 0 && epi <= 3) || epi == MS_EPI_ARGMAX) && dgemm_supported(M, N, K, S, epi), MS_EINVAL,
            "dgemm shape unsupported (M <= 256, N % 64 == 0, K % (64 S) == 0, S > 1 only for fp32 slabs)");
    REQUIRE(!g_op_rs.ssq || g_op_rs.tiles == 1, MS_EINVAL, "dgemm row scale: one-tile statistics only");
    launch_dgemm((const f16_t*)X, (const f16_t*)W, out, M, N, K, S, ldo, epi, (hipStream_t)stream, &g_op_rs);
  });
}

int ms_op_gemv_split(const void* X, const void* W, float* slabs, int32_t M, int32_t N, int32_t K,
                     int32_t S, int32_t waves, void* stream) {
  return op_guard([&] {
    REQUIRE(X && W && slabs && N >= 16 && S >= 1, MS_EINVAL, "bad gemv_split operands");
    REQUIRE(gemv_split_supported(M, N, K, S, op_rs_tiles()), MS_EINVAL,
            "gemv_split shape unsupported (M<=64, (K/S)%64==0, row-scale statistics within kRsStage and LDS)");
    GemvArgs ga;
    launch_gemv_split((const f16_t*)X, (const f16_t*)W, slabs, M, N, K, S, waves, (hipStream_t)stream,
                      op_gemv_args(ga));
  });
}

int ms_op_residual_rmsnorm(float* x, const float* slabs, int32_t S, const void* w, void* y, float* ssq,
                           int32_t rows, int32_t hidden, void* stream) {
  return op_guard([&] {
    REQUIRE(x && w && y && ssq && rows >= 1 && hidden >= 4 && hidden % 4 == 0 && hidden <= 8192, MS_EINVAL,
            "bad residual_rmsnorm shape");
    REQUIRE(S == 0 || slabs, MS_EINVAL, "slabs missing");
    REQUIRE(residual_rmsnorm_supported(S, hidden) || (S == 0 && hidden <= 8192), MS_EINVAL,
            "residual_rmsnorm: S <= 8 and hidden <= 3072 (wider rows: S == 0 only)");
    launch_residual_rmsnorm(x, slabs, S, (const f16_t*)w, (f16_t*)y, ssq, rows, hidden,
                            (hipStream_t)stream);
  });
}

int ms_op_dequant(int32_t type, const void* blocks, int64_t n_blocks, float* out, void* stream) {
  return op_guard([&] {
    REQUIRE(blocks && out && n_blocks >= 1, MS_EINVAL, "bad dequant arguments");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K or Q6_K");
    launch_dequant_f32(type, (const uint8_t*)blocks, n_blocks, out, (hipStream_t)stream);
  });
}

int ms_op_quant_rows(int32_t type, const void* blocks, int32_t rows, int32_t K, void* f16_out,
                     void* packed_out, void* stream) {
  return op_guard([&] {
    REQUIRE(blocks && f16_out && rows >= 1 && K >= 256 && K % 256 == 0, MS_EINVAL, "bad quant_rows arguments");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K or Q6_K");
    launch_quant_rows(type, (const uint8_t*)blocks, rows, K, (f16_t*)f16_out, 16, 0,
                      (uint8_t*)packed_out, 0, (hipStream_t)stream);
  });
}

int ms_op_qgemv(const void* X, int32_t type, const void* packed, void* out, int32_t M, int32_t N,
                int32_t K, int32_t ldo, int32_t epi, void* stream) {
  return op_guard([&] {
    REQUIRE(X && packed && out && N >= 16, MS_EINVAL, "bad qgemv operands");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K or Q6_K");
    REQUIRE(((epi >= 0 && epi <= 3) || epi == MS_EPI_ARGMAX) && (epi != MS_EPI_SWIGLU || N % 32 == 0),
            MS_EINVAL, "bad epilogue");
    REQUIRE(qgemv_supported(M, N, K, epi, op_rs_tiles()), MS_EINVAL,
            "qgemv shape unsupported (M<=64, K%256==0, N%16==0, row-scale statistics within kRsStage and LDS)");
    QMat q{};
    q.n = 1;
    q.base0 = (const uint8_t*)packed;
    q.row0_0 = 0;
    q.type0 = type;
    q.row_bytes0 = (K / 256) * qblock_bytes(type, true);
    GemvArgs ga;
    launch_qgemv((const f16_t*)X, q, out, M, N, K, ldo, epi, op_gemv_args(ga), (hipStream_t)stream);
  });
}

int ms_op_qgemv_split(const void* X, int32_t type, const void* packed, float* slabs, int32_t M,
                      int32_t N, int32_t K, int32_t S, void* stream) {
  return op_guard([&] {
    REQUIRE(X && packed && slabs && N >= 16 && S >= 1, MS_EINVAL, "bad qgemv_split operands");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K, MS_EINVAL, "ggml type must be Q4_K or Q6_K");
    REQUIRE(qgemv_split_supported(M, N, K, S, op_rs_tiles()), MS_EINVAL,
            "qgemv_split shape unsupported (M<=64, K%(256*S)==0, row-scale statistics within kRsStage and LDS)");
    QMat q{};
    q.n = 1;
    q.base0 = (const uint8_t*)packed;
    q.row0_0 = 0;
    q.type0 = type;
    q.row_bytes0 = (K / 256) * qblock_bytes(type, true);
    GemvArgs ga;
    launch_qgemv_split((const f16_t*)X, q, slabs, M, N, K, S, (hipStream_t)stream, op_gemv_args(ga));
  });
}

int ms_op_qdgemm(const void* X, int32_t type, const void* packed, void* out, int32_t M, int32_t N, int32_t K,
                 int32_t S, int32_t ldo, int32_t epi, void* stream) {
  return op_guard([&] {
    REQUIRE(X && packed && out && N >= 64 && K >= 256 && S >= 1, MS_EINVAL, "bad qdgemm operands");
    REQUIRE(type == MS_QT_Q4_K || type == MS_QT_Q6_K || type == 1, MS_EINVAL, "ggml type must be Q4_K, Q6_K or F16");
    REQUIRE(!g_op_rs.ssq || g_op_rs.tiles == 1, MS_EINVAL, "qdgemm row scale: one-tile statistics only");
    if (type == 1) {  // fp16 rows [N][K] through the same kernel
      const int e = epi == MS_EPI_ARGMAX ? MS_GEMV_EPI_ARGMAX : epi;
      REQUIRE(qdgemm_f16_supported(M, N, K, S, e), MS_EINVAL, "qdgemm (fp16 rows) shape unsupported");
      launch_qdgemm_f16((const f16_t*)X, (const f16_t*)packed, out, M, N, K, S, ldo, e, (hipStream_t)stream, &g_op_rs);
      return;
    }
    QMat q{};
    q.n = 1;
    q.base0 = (const uint8_t*)packed;
    q.row0_0 = 0;
    q.type0 = type;
    q.row_bytes0 = (K / 256) * qblock_bytes(type, true);
    const int e = epi == MS_EPI_ARGMAX ? MS_GEMV_EPI_ARGMAX : epi;
    REQUIRE(qdgemm_supported(M, N, K, S, e, q), MS_EINVAL,
            "qdgemm shape unsupported (M <= 256, N % 64 == 0, K % (256 S) == 0, S > 1 only for fp32 slabs)");
    launch_qdgemm((const f16_t*)X, q, out, M, N, K, S, ldo, e, (hipStream_t)stream, &g_op_rs);
  });
}

int ms_op_rmsnorm(const void* x, const void* w, void* y, float* ssq, int32_t rows, int32_t hidden,
                  const int32_t* row_idx, void* stream) {
  return op_guard([&] {
    REQUIRE(x && w && y && ssq && rows >= 1 && hidden >= 4 && hidden % 4 == 0 && hidden <= 8192, MS_EINVAL,
            "bad rmsnorm shape");
    launch_rmsnorm((const float*)x, (const f16_t*)w, (f16_t*)y, ssq, rows, hidden, row_idx,
                   (hipStream_t)stream);
  });
}

int ms_op_argmax_partials(const void* partials, int32_t rows, int32_t tiles, int32_t* ids, void* stream) {
  return op_guard([&] {
    REQUIRE(partials && ids && rows >= 1 && tiles >= 1, MS_EINVAL, "bad argmax_partials shape");
    launch_argmax_partials(partials, rows, tiles, ids, (hipStream_t)stream);
  });
}

int ms_op_argmax(const void* logits, int32_t rows, int32_t n, int32_t* ids, void* stream) {
  return op_guard([&] {
    REQUIRE(logits && ids && rows >= 1 && n >= 1, MS_EINVAL, "bad argmax shape");
    launch_argmax((const float*)logits, rows, n, ids, (hipStream_t)stream);
  });
}

}  // extern "C"
