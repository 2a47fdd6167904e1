/*
 * mapsum.h -- C-ABI of libmapsum.so, the MI355X-native map-phase engine.
 *
 * What this replaces.  The reference has no native boundary: its
 * map call is one HTTP request per chunk,
 *     OllamaLLM._call(prompt) -> requests.post(f"{url}/api/generate",
 *         json={"model", "prompt", "stream": False, "options": {"num_predict": N}})
 *         -> resp.json()["response"]
 * (run_full_evaluation_pipeline.py:80-106; runner copies
 *  runners/run_summarization_ollama_mapreduce.py:37-49,
 *  runners/run_summarization_ollama_mapreduce_critique.py:63-79,
 *  runners/run_summarization_ollama_mapreduce_hierarchical.py:56-68).
 * Everything behind that request (template -> tokenize -> prefill -> decode ->
 * detokenize) happens inside Ollama.  libmapsum takes over the
 * prefill/decode part on ids: the Python host (mapsum/compat.py OllamaLLM) keeps
 * the prompt-in/summary-out contract and calls
 *     ms_submit (one per chunk)  ~ the body of one /api/generate request
 *     ms_step                    ~ one scheduler iteration (admit+prefill, decode)
 *     ms_poll                    ~ resp.json()["response"] (as ids)
 * Errors: every entry point returns an int status (0 = OK, < 0 errno-like) and
 * never throws across the ABI; ms_last_error() gives the text.  The Python
 * wrapper raises RuntimeError, mirroring resp.raise_for_status()
 * (run_full_evaluation_pipeline.py:91).
 * Ownership: input ids are copied at submit; result id buffers are owned by the
 * engine and stay valid until the next ms_poll / ms_destroy.  One engine per GPU
 * per process; an engine is not thread-safe.
 */
#ifndef MAPSUM_H
#define MAPSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MS_ABI_VERSION 3  /* 3: the 16-bit type is IEEE fp16 (weights, KV cache, activations) */

/* status codes */
#define MS_OK 0
#define MS_EIO -5       /* device / runtime failure                  */
#define MS_ENOMEM -12   /* device allocation failed                  */
#define MS_EBUSY -16    /* operation not allowed while work pending  */
#define MS_EINVAL -22   /* bad argument                              */
#define MS_ENOSPC -28   /* request can never fit (ctx / KV pages)    */

/* finish reasons (ms_result.finish_reason) -- Ollama's done_reason "stop"/"length" */
#define MS_FINISH_EOS 1
#define MS_FINISH_LENGTH 2
#define MS_FINISH_ERROR 3 /* this chunk only: no finite logit (NaN/Inf in its activations);
                             the other chunks of the batch are unaffected.  The reference has
                             no retry (run_full_evaluation_pipeline.py:627-638 marks the whole
                             model failed); the Python host re-queues such a chunk once. */

/* ms_submit flags */
#define MS_FLAG_IGNORE_EOS 1u /* bench mode: always generate num_predict tokens */

/* logical weight tensors for ms_load_weight ([rows][cols] row-major fp16, HF
 * nn.Linear layout [out][in]); the engine fuses Q|K|V and interleaves gate/up
 * on upload. */
enum ms_tensor {
  MS_T_EMBED = 0,      /* [vocab][hidden]          */
  MS_T_ATTN_NORM = 1,  /* [hidden]                 */
  MS_T_WQ = 2,         /* [n_heads*head_dim][hidden] */
  MS_T_WK = 3,         /* [n_kv*head_dim][hidden]  */
  MS_T_WV = 4,         /* [n_kv*head_dim][hidden]  */
  MS_T_WO = 5,         /* [hidden][n_heads*head_dim] */
  MS_T_FFN_NORM = 6,   /* [hidden]                 */
  MS_T_WGATE = 7,      /* [ffn][hidden]            */
  MS_T_WUP = 8,        /* [ffn][hidden]            */
  MS_T_WDOWN = 9,      /* [hidden][ffn]            */
  MS_T_FINAL_NORM = 10,/* [hidden]                 */
  MS_T_LM_HEAD = 11    /* [vocab][hidden]; only when tie_embeddings == 0 */
};

typedef struct ms_config {
  int32_t abi_version;          /* = MS_ABI_VERSION */
  /* model (Llama-3.2 family; head_dim must be 128) */
  int32_t n_layers, hidden, n_heads, n_kv_heads, head_dim, ffn, vocab;
  float rope_theta, rope_factor, rope_low_freq_factor, rope_high_freq_factor;
  int32_t rope_orig_ctx;
  float norm_eps;
  int32_t tie_embeddings;
  /* engine */
  int32_t device;               /* HIP device ordinal                         */
  int32_t max_batch;            /* sequences in flight (<= 1024).  Also fixes the
                                   engine's decode arithmetic (fp16 weights:
                                   1-16 residual-fused GEMV, 17-23 split GEMV +
                                   residual_rmsnorm, 24-95 skinny GEMM, 96-191
                                   + the lm_head on the 128x128 GEMM tile,
                                   >= 192 + the fp16-rows K-quant GEMM form;
                                   K-quant: 1-16 residual-fused Q-GEMV, 17-64
                                   split Q-GEMV + residual_rmsnorm, >= 65 the
                                   K-quant skinny GEMM, lm_head tile from 96); results
                                   are batch-invariant inside one engine, not
                                   across these boundaries */
  int32_t max_ctx;              /* prompt + generated tokens per sequence     */
  int32_t max_prefill_tokens;   /* packed prompt tokens per prefill pass      */
  int32_t n_pages;              /* KV pages of 64 tokens; 0 = enough for all  */
  int32_t n_eos;                /* end-of-turn ids (<|eot_id|> etc.)          */
  int32_t eos_ids[8];
} ms_config;

typedef struct ms_result {
  uint64_t tag;          /* the caller's tag from ms_submit                    */
  const int32_t* ids;    /* generated ids (EOS excluded); engine-owned          */
  int32_t n_ids;
  int32_t finish_reason; /* MS_FINISH_*                                         */
  int32_t n_prompt;
  int32_t _pad;
} ms_result;

typedef struct ms_stats {
  int64_t prefill_tokens;     /* prompt tokens processed                       */
  int64_t decode_tokens;      /* tokens produced by decode steps               */
  int64_t prefill_passes, decode_steps;
  int64_t finished;
  double prefill_ms, decode_ms; /* device time (events) when profiling is on   */
  double kernel_ms[8];          /* per kernel class, when profiling is on:
                                   0 gemm(prefill) 1 attn_prefill 2 gemv(decode)
                                   3 attn_decode 4 lm_head 5 norm/rope/misc
                                   6 persist (the decode step's layers as one
                                   persistent launch, <= 8-slot engines)        */
  int64_t kernel_launches[8];
  int64_t decode_kv_tokens;     /* sum over decode steps and rows of the keys attended
                                   (the KV-read term of SURVEY.md §8d's decode bytes)  */
  int64_t graphs_built;         /* decode hipGraphs captured + instantiated (the cache keeps
                                   at most 64, least recently used evicted)            */
  int64_t persist_fallbacks;    /* decode runs recomputed with the per-layer launches after a
                                   hand-off of the persistent step timed out (expected 0)  */
  int64_t persist_steps;        /* decode steps that ran the persistent launch             */
} ms_stats;

typedef struct ms_engine ms_engine;

/* ---- engine lifecycle ------------------------------------------------------ */
int ms_create(const ms_config* cfg, ms_engine** out);
int ms_destroy(ms_engine* e);
/* e == NULL returns the last error of a failed ms_create / op call */
const char* ms_last_error(const ms_engine* e);

/* ---- weights ---------------------------------------------------------------- */
int ms_load_weight(ms_engine* e, int32_t tensor, int32_t layer, const uint16_t* host_f16,
                   int64_t n_elems);
/* device-side counter-based N(0,std)-like init; restated in oracle/synth.py */
int ms_init_synthetic(ms_engine* e, uint64_t seed, float std, float norm_jitter);

/* ggml K-quant weights (Q4_K_M files: BASELINE.json config 5).  `blocks` are the tensor's
 * rows as raw ggml blocks (Q4_K = 144 B, Q6_K = 210 B per 256 weights).  The engine keeps
 * f16(dequant) for prefill and the blocks for the dequant-fused decode GEMV.  RMSNorm
 * weights stay fp16 (ms_load_weight). */
#define MS_GGML_Q4_K 12
#define MS_GGML_Q6_K 14
int ms_load_weight_q(ms_engine* e, int32_t tensor, int32_t layer, int32_t ggml_type,
                     const void* host_blocks, int64_t n_bytes);
/* random Q4_K/Q6_K blocks with the Q4_K_M per-tensor type mix (bench) */
int ms_init_synthetic_q(ms_engine* e, uint64_t seed, float scale, float norm_jitter);

/* ---- weight broadcast (one process per GPU: rank 0 loads, the others receive over RCCL) -- */
/* every device weight buffer in a fixed order (fp16 matrices and norms, then K-quant
   regions); returns the count, fills up to cap (ptr, bytes) pairs */
int ms_weight_regions(const ms_engine* e, void** ptrs, int64_t* bytes, int32_t cap);
/* the (tensor, layer, ggml_type) triples of the K-quant tensors loaded so far; returns the count */
int ms_quant_manifest(const ms_engine* e, int32_t* triples, int32_t cap);
/* lay out a K-quant tensor as ms_load_weight_q would, without its bytes (a broadcast fills
   the regions afterwards) */
int ms_declare_weight_q(ms_engine* e, int32_t tensor, int32_t layer, int32_t ggml_type);

/* ---- request path (replaces one /api/generate per chunk) -------------------- */
int ms_submit(ms_engine* e, const int32_t* ids, int32_t n, int32_t num_predict,
              uint32_t flags, uint64_t tag);
/* replace the config's end-of-turn ids by a larger stop set (0 <= ids < vocab; n = 0 restores
   cfg.eos_ids).  Ollama's `stop` option; bench.py --eos uses a synthetic set so that random-init
   weights finish chunks at natural, varied lengths (slot turnover). */
int ms_set_eos_ids(ms_engine* e, const int32_t* ids, int32_t n);
/* one scheduler iteration: admit + prefill, then a decode run of up to 64 chained greedy
   steps with one host synchronisation (fewer when a chunk reaches num_predict, the
   attention split grid changes, or admissible work waits for a slot); a chunk that meets
   EOS mid-run stops there.  Returns sequences still waiting or running (>= 0).
   MS_DECODE_RUN=1 in the environment restores one decode step per call. */
int ms_step(ms_engine* e);
/* copies up to cap finished results; returns the number copied */
int ms_poll(ms_engine* e, ms_result* out, int32_t cap);
int ms_pending(const ms_engine* e);
int ms_get_stats(const ms_engine* e, ms_stats* out);
int ms_reset_stats(ms_engine* e);
/* bit mask of kernel classes to bracket with HIP events (0 = off) */
int ms_set_profiling(ms_engine* e, uint32_t class_mask);
/* roctx ranges (rocprofv3 --marker-trace).  ms_step brackets itself ("mapsum.step") and its
   phases ("mapsum.prefill", "mapsum.decode_run"); these let the host mark its own phases
   (dist.gather_summaries: "mapsum.gather").  Nest; no-ops unless a profiler is attached. */
int ms_trace_push(const char* name);
int ms_trace_pop(void);
int ms_synchronize(ms_engine* e);
/* the decode step's layers as ONE persistent launch (k_persist.hip; engines of <= 8 slots on
   fp16 Llama-3.2-3B weights, bit-identical to the per-layer launches): on (1, the default, also
   MS_PERSIST) or off (0).  Returns 1 when this engine supports it, 0 when it never runs it. */
int ms_set_persist(ms_engine* e, int32_t on);
/* test hook: copy `bytes` from byte `offset` of an engine buffer to host memory (after the
   engine's streams are idle) */
#define MS_DBG_KPOOL 0          /* K cache [layer][page][kv_head][64][head_dim] fp16 */
#define MS_DBG_VPOOL 1          /* V cache, same layout */
#define MS_DBG_DECODE_LOGITS 2  /* the decode lm_head output (argmax partials {max, id} per 16 columns) */
#define MS_DBG_DECODE_X 3       /* the decode residual [max_batch][hidden] fp32 */
int ms_debug_read(ms_engine* e, int32_t which, int64_t offset, void* host, int64_t bytes);
/* diagnostic: the persistent step's in-kernel timeline of its latest launch, [256][28][16]
   s_memrealtime ticks (100 MHz), recorded only under MS_PK_STAMPS=1 (tools/pk_stamps.py) */
int ms_debug_pk_stamps(uint64_t* out, int32_t n);
/* diagnostic: decode attention v2's per-block phase stamps of its latest launch, [1024][32]
   (entry, XCC / HW id, prologue, per-wave S and P.V done, partial stored), recorded only under
   MS_A2_STAMPS=1 (tools/a2_stamps.py) */
int ms_debug_a2_stamps(uint64_t* out, int32_t n);

/* ---- parity probe (tests): one prompt through the prefill path -------------- */
/* hidden_out: [n][hidden] fp32 residual after `n_layers_run` layers (or NULL);
   logits_out: [n][vocab] fp32 logits of every position (or NULL; needs
   n_layers_run == n_layers). */
int ms_forward(ms_engine* e, const int32_t* ids, int32_t n, int32_t n_layers_run,
               float* hidden_out, float* logits_out);
/* the same over n_seqs prompts packed into ONE varlen prefill pass (the ragged batches of
   the hierarchical runner, runners/run_summarization_ollama_mapreduce_hierarchical.py:242-274):
   ids = the prompts back to back, lens[i] = length of prompt i; hidden_out / logits_out rows
   follow the packed order ([sum lens][hidden], [sum lens][vocab]). */
int ms_forward_packed(ms_engine* e, const int32_t* ids, const int32_t* lens, int32_t n_seqs,
                      int32_t n_layers_run, float* hidden_out, float* logits_out);
/* teacher forcing through the DECODE path (parity tests): as ms_submit, but decode step j
   (j >= 1) is fed forced[j-1] instead of the engine's own previous choice, so the result ids
   are the engine's greedy choices after a context the caller fixes (e.g. the oracle's own
   greedy tokens).  n_forced >= num_predict - 1.  Such a sequence decodes one step per run. */
int ms_submit_forced(ms_engine* e, const int32_t* ids, int32_t n, const int32_t* forced,
                     int32_t n_forced, int32_t num_predict, uint32_t flags, uint64_t tag);

/* ---- op-level entry points (device pointers; stream = hipStream_t or NULL) -- */
#define MS_EPI_STORE_F16 0  /* out fp16 [M][ldo]                              */
#define MS_EPI_ADD_F32 1     /* out fp32 [M][ldo] += acc  (residual add)       */
#define MS_EPI_SWIGLU 2      /* W rows interleaved gate/up per 16; out fp16 [M][N/2] */
#define MS_EPI_STORE_F32 3   /* out fp32 [M][ldo]                              */
#define MS_EPI_ARGMAX 5      /* decode GEMV only: out {max, id} float2 [M][ldo = N/16], one per
                                16-column tile (ties -> lowest id; NaN never wins); finish the
                                rows with ms_op_argmax_partials                          */
/* prefill GEMM: out[M][N] (op) A[M][K] . W[N][K]^T ; K % 64 == 0.  MS_EPI_ARGMAX (the large
   decode regime's lm_head): {max, id} float2 partials [M][ldo >= N/16] per 16-column tile on the
   128x128 tile, no row scale, N % 16 == 0 */
int ms_op_gemm(const void* A, const void* W, void* out, int32_t M, int32_t N, int32_t K,
               int32_t ldo, int32_t epilogue, void* stream);
/* prefill O / down with the residual update fused (the engine's prefill layer): x fp32 [M][N] +=
   A . W^T, and the input of the next normalised projection: xg_out fp16 [M][N] = f16(x * gamma * 2^-4),
   ssq_out fp32 [tiles][M] = per-128-column sums of the new x^2 (tiles = ms_gemm_resid_tiles(M, N) = N / 128),
   the deferred RMSNorm statistics the next ms_op_gemm takes through ms_op_set_row_scale */
int ms_op_gemm_resid(const void* A, const void* W, float* x, void* xg_out, const void* gamma, float* ssq_out,
                     int32_t M, int32_t N, int32_t K, void* stream);
int ms_gemm_resid_tiles(int32_t M, int32_t N);
/* tuning/test hook: prefill GEMM tile (0 heuristic, 1 = 128x128, 2 = 256x256 8-phase,
   3 = 256x256 on 4 waves, 4 = 3 for the stored epilogues and 2 for the residual one; every
   variant gives the same bits) */
int ms_set_gemm_variant(int32_t variant);
/* tuning/test hook: the K-quant GEMVs that have a grid-stride two-stage form (the Q6_K lm_head
   argmax, the Q4_K gate/up SwiGLU) take it (1, the default) or run one-tile blocks (0); the
   two give bit-identical outputs */
int ms_set_qgemv_gs(int32_t on);
/* tuning/test hook: decode attention's split combine on the XCD-matched grid (1, default) or the
   (B, Hq) grid (0), and the v2 prologue form (0 default, 3 a dedicated prologue wave); every
   setting gives the same bits.  Engines capture their decode graphs with the current setting. */
int ms_set_attn_tuning(int32_t combine_grp, int32_t order);
/* tuning/test hook: the large-batch decode skinny GEMM on 4-wave blocks (1) or on 8-wave
   blocks that split each 128-k step in two k halves (2, the default); the two sum in
   different orders, each independent of the batch rows.  Engines of <= 128 slots take the
   setting for their gate/up launch at creation (set it before ms_engine_create);
   ms_op_dgemm takes it where it applies (M <= 128, K % (128 S) == 0). */
int ms_set_dgemm_kh(int32_t kh);
/* tuning/test hook: ms_op_dgemm's weight rows per block, 64 (4 row groups, the default) or 128
   (8; 4-wave-group blocks only, M <= 128, N % 128 == 0, else 64) -- the same bits either way.
   Engines choose per projection (128 for QKV, down and the lm_head at <= 128 rows). */
int ms_set_dgemm_wn(int32_t wn);
/* decode skinny GEMM (M <= 64): same contract; workspace >= ms_op_gemv_workspace() bytes */
int64_t ms_op_gemv_workspace(int32_t M, int32_t N, int32_t K);
int ms_op_gemv(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K,
               int32_t ldo, int32_t epilogue, void* workspace, void* stream);
/* tuning hook: as ms_op_gemv with the K-splitting wave count forced (0 = heuristic) */
int ms_op_gemv_tuned(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K,
                     int32_t ldo, int32_t epilogue, void* workspace, int32_t waves, void* stream);
/* tuning hook: ms_op_gemv over X [M][ldk] and W [N][ldk] (row stride ldk >= K elements) */
int ms_op_gemv_strided(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K,
                       int32_t ldk, int32_t ldo, int32_t epilogue, void* stream);
/* decode O / down with the residual update fused (the engine's small-regime layer): x fp32
   [M][N] += X . W^T on rt-row tiles (N % rt == 0, tiles = N / rt <= 256), and the input of the
   next normalised projection: xg_out fp16 [M][N] = f16(x * gamma * 2^-4), ssq_out fp32 [tiles][M] =
   per-tile sums of the new x^2 (its deferred RMSNorm statistics, see ms_op_set_row_scale) */
int ms_op_gemv_resid(const void* X, const void* W, float* x, void* xg_out, const void* gamma,
                     float* ssq_out, int32_t M, int32_t N, int32_t K, int32_t rt, void* stream);
/* the deferred RMSNorm of the numerics contract: the next ms_op_gemm /
   ms_op_gemv / ms_op_gemv_split / ms_op_dgemm / ms_op_qgemv / ms_op_qgemv_split calls of the
   calling thread scale output row r by 16/sqrt(sum_t ssq[t][r] / hidden + eps) -- 16 undoes the
   2^-4 the producers pre-scale their fp16 output by (ssq [tiles][M];
   gemm / dgemm: tiles == 1); ssq = NULL turns the scale off.  Test hook: the engine passes the
   scale with each launch. */
int ms_op_set_row_scale(const float* ssq, int32_t tiles, int32_t hidden, float eps);
/* large-batch decode GEMM (M <= 256 rows; 64 weight rows per block, X shared via LDS): the
   ms_op_gemv epilogues (plus MS_EPI_ARGMAX); S > 1: split-K fp32 slabs [S][M][N] with
   epilogue MS_EPI_STORE_F32; N % 64 == 0, K % (64 S) == 0 */
int ms_op_dgemm(const void* X, const void* W, void* out, int32_t M, int32_t N, int32_t K, int32_t S,
                int32_t ldo, int32_t epilogue, void* stream);
/* decode split-K: slabs fp32 [S][M][N], slab s = X[:, sK/S:(s+1)K/S] . W[:, same]^T;
   waves = 0 picks the heuristic (tuning hook otherwise) */
int ms_op_gemv_split(const void* X, const void* W, float* slabs, int32_t M, int32_t N, int32_t K,
                     int32_t S, int32_t waves, void* stream);
/* x fp32 [rows][hidden] += slab_0 + ... + slab_{S-1} (slab order); then the input of the
   normalised projection that follows: y fp16 = f16(x * w * 2^-4), ssq[r] = sum of x[r]^2 (one tile) */
int ms_op_residual_rmsnorm(float* x, const float* slabs, int32_t S, const void* w, void* y, float* ssq,
                           int32_t rows, int32_t hidden, void* stream);
/* K-quant ops: raw ggml blocks -> fp32 (bit-exact restatement of llama.cpp's
   dequantize_row_q4_K/q6_K); raw rows -> fp16 rows + packed rows (Q6_K repacked to 224 B);
   dequant-fused GEMV over packed rows (same epilogues as ms_op_gemv) */
int ms_op_dequant(int32_t ggml_type, const void* blocks, int64_t n_blocks, float* out, void* stream);
int ms_op_quant_rows(int32_t ggml_type, const void* blocks, int32_t rows, int32_t K, void* f16_out,
                     void* packed_out, void* stream);
int ms_op_qgemv(const void* X, int32_t ggml_type, const void* packed_rows, void* out, int32_t M,
                int32_t N, int32_t K, int32_t ldo, int32_t epilogue, void* stream);
/* dequant-fused split-K: slabs fp32 [S][M][N] over S equal, super-block aligned K ranges
   (the quantised counterpart of ms_op_gemv_split; K % (256*S) == 0) */
int ms_op_qgemv_split(const void* X, int32_t ggml_type, const void* packed_rows, float* slabs,
                      int32_t M, int32_t N, int32_t K, int32_t S, void* stream);
/* large-batch K-quant decode GEMM (M <= 256 rows): ms_op_dgemm over the packed rows, each weight
   dequantised in registers to its fp16-copy value f16(ggml dequant); epilogues MS_EPI_STORE_F32
   (S > 1: split-K slabs [S][M][N]), MS_EPI_SWIGLU, MS_EPI_ARGMAX; N % 64 == 0, K % (256 S) == 0
   with K / (256 S) even or a multiple of 3 (the engine's K-quant decode projections in engines
   of >= 65 slots) */
int ms_op_qdgemm(const void* X, int32_t ggml_type, const void* packed_rows, void* out, int32_t M,
                 int32_t N, int32_t K, int32_t S, int32_t ldo, int32_t epilogue, void* stream);
/* the input of a normalised projection: y fp16 [rows][hidden] = f16(x * w * 2^-4) and ssq[r] = sum
   of x[r]^2 over x fp32 [.][hidden] rows (row_idx optional gather); the projection then scales
   its output rows by 16/sqrt(ssq / hidden + eps) (ms_op_set_row_scale).  The 2^-4 pre-scale
   (exact) keeps un-normalised residual rows up to ~1e6 inside fp16 (kernels.h kXgScale). */
int ms_op_rmsnorm(const void* x, const void* w, void* y, float* ssq, int32_t rows, int32_t hidden,
                  const int32_t* row_idx, void* stream);
/* ids[r] = argmax_j logits[r][j] (ties -> lowest j; -1 when no logit of the row is finite) */
int ms_op_argmax(const void* logits, int32_t rows, int32_t n, int32_t* ids, void* stream);
/* ids[r] = the lowest id of the largest {max, id} partial of row r (MS_EPI_ARGMAX output) */
int ms_op_argmax_partials(const void* partials, int32_t rows, int32_t tiles, int32_t* ids, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAPSUM_H */
