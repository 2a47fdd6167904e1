// kernels.h -- launchers for the gfx950 map-phase kernels (host-callable).
#pragma once
#include "common.h"

namespace ms {

// Where the K/V of one layer live: pool[page][kv_head][64 tokens][128] fp16.
struct KVView {
  f16_t* k;
  f16_t* v;
  const int32_t* block_table;  // [slots][max_pages]
  int32_t max_pages;           // row stride of block_table
  int32_t n_kv_heads;
  // 1: slot-major pool (the engine's default sizing, max_batch x max_pages pages): logical
  // page p of slot s is page s*max_pages + p, so decode attention needs no table lookup
  int32_t slot_major;
};

// Prefill attention work description (device arrays, see engine.cpp StepArgs).
constexpr int kPrefillQRows = 128;  // query rows per prefill attention block (8 waves x 16)
struct PrefillAttnArgs {
  const int32_t* seq_qstart;  // [S] row of the sequence's first query token in qkv
  const int32_t* seq_qlen;    // [S]
  const int32_t* seq_kvlen;   // [S] keys visible to the last query (= cached + qlen)
  const int32_t* seq_slot;    // [S] block-table row
  const int32_t* qblk;        // [NQB] (seq << 16) | q_block (kPrefillQRows rows), heaviest first
  int32_t n_qblk;
  // non-null: Q arrives straight from the QKV GEMM (rope-permuted, not rotated) and the kernel
  // applies RoPE while staging it (rope_kv_kernel's arithmetic); null: Q already rotated
  const float* cos_tab;
  const float* sin_tab;
};

struct DecodeAttnArgs {
  const int32_t* seq_len;   // [B] keys incl. the new token
  const int32_t* seq_slot;  // [B]
  int32_t B;
  int32_t max_len;          // upper bound over the batch (sets the split grid)
  int32_t ppw;              // pages per wave, fixed per engine (attn_decode_ppw); 0 = 2
};

// The deferred RMSNorm of the numerics contract (oracle/llama_ref.py): a
// normalised projection (QKV, gate/up, lm_head) multiplies the fp16 GEMM input f16(x * g) by
// W and scales output row r by rinv(r) = rsq(sum_t ssq[t][r] / H + eps), where ssq holds
// partial sums of x[r]^2 [tiles][rows] written by the producer of x (a norm kernel: one tile;
// a RESID_SSQ GEMV epilogue: one per column tile).  Every consumer forms the sum in the same
// order (tile t = lane + 64 i added in i order per lane, then the wave's xor tree; with one
// tile that is ssq[0][r] exactly), so a row's factor depends only on (tiles, H) -- never on
// the number of rows or on the kernel.  ssq == nullptr: no scale.
struct RowScale {
  const float* ssq;
  int tiles, H;
  float eps;
  float inv_h;  // 1 / H
};
inline RowScale make_row_scale(const float* ssq, int tiles, int H, float eps) {
  return RowScale{ssq, tiles, H, eps, 1.0f / (float)H};
}
// The producers store the GEMM input pre-scaled by an exact power of two, xg = f16(x * g * 2^-4),
// and every consumer folds 2^4 into the row factor: r' = 16 rsq(...).  Both scalings are exact
// in fp32, and f16(v * 2^-4) = f16(v) * 2^-4 wherever v is a normal fp16 value, so the products
// r' * (xg . W) are bit-identical to r * (f16(x * g) . W) there -- but the un-normalised residual
// (massive activations of real checkpoints reach 1e3-1e4 in a few channels; x * g is NOT
// normalised before the rounding) now overflows fp16 only beyond |x * g| = 16 * 65504 ~ 1e6
// instead of 65504.  Below |x * g| = 2^-10 the value lands in fp16's subnormals,
// whose absolute step 2^-20 is the normal step at that magnitude: no precision is lost where
// it matters for a dot product.
constexpr float kXgScale = 0.0625f, kXgUnscale = 16.0f;
// rinv = 16 rsq(sum / H + eps): one v_rsq_f32 (1 ulp) and an exact power-of-two multiply -- the
// same instruction sequence in every consumer, so every kernel derives the identical factor
// from the identical sum
__device__ __forceinline__ float rs_rinv(float sum, const RowScale& rs) {
  return __builtin_amdgcn_rsqf(__fmaf_rn(sum, rs.inv_h, rs.eps)) * kXgUnscale;
}

// x = the embedding rows; with gamma also xg = f16(x * gamma) and ssq = per-row sums of x^2
// (the first normalised projection's input, one-tile RowScale)
void launch_embed(const int32_t* ids, int T, const f16_t* emb, int H, float* x, hipStream_t s,
                  const f16_t* gamma = nullptr, f16_t* xg = nullptr, float* ssq = nullptr);
// chained decode: next ids <- this step's argmax (clamped into [0, V)), positions and key
// counts += 1 in the step-argument blob [ids | positions | slots | key counts | step], and the
// raw ids appended to ring row `step` (B <= 256)
void launch_decode_advance(int32_t* args, const int32_t* ids_out, int32_t* ring, int B, int V,
                           hipStream_t s);
// launch_argmax_partials + launch_decode_advance + the next step's launch_embed (with gamma) as
// one launch, bit-identical; the blob carries a ticket word args[4B + 1] (zero between steps)
void launch_decode_tail(const void* partials, int tiles, int32_t* args, int32_t* ids_out, int32_t* ring, int B,
                        int V, const f16_t* emb, int H, float* x, const f16_t* gamma, f16_t* xg, float* ssq,
                        hipStream_t s);
// the GEMM input of a normalised projection: y[r] = f16(x[row_idx[r]] * w), ssq[r] = sum of
// x[row_idx[r]]^2 (one-tile RowScale); row_idx optional (gather)
void launch_rmsnorm(const float* x, const f16_t* w, f16_t* y, float* ssq, int rows, int H,
                    const int32_t* row_idx, hipStream_t s);
// RoPE on Q (in place, rope-permuted -> natural dim order) and K; K,V scattered into the
// paged cache.  Q/K heads arrive in the rope-permuted row order of the fused weights.
// rope_q = false: K and V only (prefill: the attention kernel rotates Q as it stages it)
void launch_rope_kv(f16_t* qkv, int T, int Hq, int Hk, const int32_t* tok_pos,
                    const int32_t* tok_slot, const float* cos_tab, const float* sin_tab,
                    KVView kv, hipStream_t s, bool rope_q = true);
void launch_argmax(const float* logits, int rows, int n, int32_t* out, hipStream_t s);

// out (epi) A[M][K] . W[N][K]^T, MFMA 16x16x32 fp16, K % 64 == 0; rs (<= kGemmRsTiles tiles of
// statistics, or null): the deferred RMSNorm scale of the output rows (epilogues 0, 2, 3).
// gr (epilogue 1, the residual add of O / down): the GEMM also writes the next normalised
// projection's input, gr->xg = f16(x_new * gr->gamma) [M][N], and per-tile sums of x_new^2,
// gr->ssq [N / 128][M] (gemm_resid_tiles) -- no norm launch.
struct GemmResid {
  const f16_t* gamma;
  f16_t* xg;
  float* ssq;
};
constexpr int kGemmRsTiles = 24;     // statistics tiles a consumer GEMM folds (H / 128 at H = 3072)
constexpr int kGemmStatCols = 128;  // columns per statistics tile, on both GEMM tiles
// statistics tiles the residual epilogue writes for an M x N GEMM: N / 128 whatever the tile,
// so a packed prompt's rows get the same statistics at any packing (batch invariance)
int gemm_resid_tiles(int M, int N);
// whether an M x N GEMM's row scale can fold `tiles` statistics tiles (launch_gemm skips otherwise)
bool gemm_rs_tiles_ok(int M, int N, int tiles);
void launch_gemm(const f16_t* A, const f16_t* W, void* out, int M, int N, int K, int ldo,
                 int epi, hipStream_t s, const RowScale* rs = nullptr, const GemmResid* gr = nullptr);
// tile choice: 0 = heuristic (256x256 8-phase for M, N >= 1024), 1 = 128x128, 2 = 256x256,
// 3 = 256x256 on 4 waves, 4 (default) = the heuristic with 3 for the stored epilogues
void set_gemm_variant(int v);
// the Q6_K lm_head argmax GEMV: grid-stride two-stage loop (default) or one-tile blocks
void set_qgemv_gs(bool on);
// decode attention: the combine's XCD-matched grid (1, default) or the (B, Hq) grid (0) --
// placement only, the same bits (order: 0; the prologue-wave form was removed in round 6)
void set_attn_tuning(int combine_grp, int order);
// large-batch skinny GEMM: 1 = 4-wave blocks, 2 = 8-wave blocks with the K step split in halves
// (S = 1 launches; a different but M-independent sum order)
void set_dgemm_kh(int kh);
// op-level skinny GEMM: weight-row groups per block (4 or 8; engines choose per launch)
void set_dgemm_wn(int wn);
// M <= 64 decode variant (weight streaming); gemv_supported() says whether a shape fits.
// Epilogues: the four of launch_gemm plus ROPE_KV (QKV with rope-permuted Q/K rows).
enum {
  MS_GEMV_EPI_STORE_F16 = 0,
  MS_GEMV_EPI_ADD_F32 = 1,
  MS_GEMV_EPI_SWIGLU = 2,
  MS_GEMV_EPI_STORE_F32 = 3,
  MS_GEMV_EPI_ROPE_KV = 4,
  // greedy argmax partials: out = {max, id} float2 [M][tiles] of each 16-column tile
  // (ties -> lowest id, NaN never wins); launch_argmax_partials finishes the rows
  MS_GEMV_EPI_ARGMAX = 5,
  // residual update + the next RMSNorm's inputs (decode O / down, no split-K): out = x fp32
  // [M][ldo], x[r][c] += acc; ga.ssq_out[tile][r] = sum over the tile's columns of the new
  // x[r][c]^2 (a fixed lane tree) and ga.xg_out[r][c] = f16(x[r][c] * ga.gamma[c]): the next
  // projection's GEMM input and its deferred row scale (RowScale), with no norm launch
  MS_GEMV_EPI_RESID_SSQ = 6
};
struct GemvArgs {
  // ROPE_KV epilogue: Q -> out[row][h*128..] (ld = ldo), K/V -> paged cache
  const int32_t* tok_pos;
  const int32_t* tok_slot;
  const float* cos_tab;
  const float* sin_tab;
  KVView kv;
  int Hq, Hk;
  // weight rows per tile (NT = 1 plans; 0 = 16): 12 puts the 3072-row O / down projections on
  // exactly 256 workgroups (one per CU) without split-K
  int rt;
  // RESID_SSQ epilogue: per-tile sums of squares [tiles][M], the next norm's gain [ldo] and
  // the fp16 GEMM input it feeds [M][ldo]
  float* ssq_out;
  const f16_t* gamma;
  f16_t* xg_out;
  // deferred RMSNorm scale of the output rows (STORE_F16 / STORE_F32 / SWIGLU / ROPE_KV /
  // ARGMAX epilogues)
  RowScale rs;
  // split-K slabs: rows between consecutive slabs (0 = M).  A row group of a larger batch
  // writes its rows into the batch's [S][B][N] slabs (slab_rows = B, out = slab 0, row r0)
  int slab_rows;
};
// split-K into S fp32 slabs [S][M][N] (slab s = partial over k in [s*K/S, (s+1)*K/S)); the
// consumer adds them in slab order (launch_residual_rmsnorm / the decode attention prologue)
bool gemv_split_supported(int M, int N, int K, int S, int rs_tiles = 0);
// whether a decode GEMV / Q-GEMV can take a deferred-norm scale of `tiles` partial sums per row
// (staged in LDS: tiles * M <= 4096)
bool gemv_rs_supported(int M, int tiles);
void launch_gemv_split(const f16_t* X, const f16_t* W, float* slabs, int M, int N, int K, int S,
                       int force_waves, hipStream_t s, const GemvArgs* ga = nullptr);
// X [M][ldk] and W [N][ldk] rows of stride ldk >= K (tuning hook: padded weight layouts)
void launch_gemv_strided(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldk,
                         int ldo, int epi, hipStream_t s);
// rows of {max, id} partials [rows][tiles] -> ids (-1: no finite maximum)
void launch_argmax_partials(const void* partials, int rows, int tiles, int32_t* out, hipStream_t s);

// x[r] += slab[0][r] + ... + slab[S-1][r] (left to right, then added to x); y = f16(x * w)
// and ssq[r] = sum of x[r]^2 (the one-tile RowScale of the projection y feeds).  S = 0: no
// slabs.  Supported: S <= 8, H <= 3072 (H > 3072 only with S = 0).
bool residual_rmsnorm_supported(int S, int H);
void launch_residual_rmsnorm(float* x, const float* slabs, int S, const f16_t* w, f16_t* y,
                             float* ssq, int rows, int H, hipStream_t s);
size_t gemv_workspace_bytes(int M, int N, int K);
// rs_tiles > 0: the call carries deferred-norm statistics of that many tiles (RowScale), which
// the staged-partials LDS and kRsStage must also fit
bool gemv_supported(int M, int N, int K, int epi, int rs_tiles = 0);
void launch_gemv(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldo,
                 int epi, void* ws, hipStream_t s);
// ga: prologue/epilogue arguments (or null); force_waves: tuning hook (0 = heuristic)
void launch_gemv_ex(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int ldo,
                    int epi, const GemvArgs* ga, int force_waves, hipStream_t s);

// large-batch decode projections (k_dgemm.hip): 64 weight rows x all M <= 256 rows per block,
// X shared through LDS; S > 1 = split-K fp32 slabs [S][M][N] (STORE_F32 only).  Epilogues as
// the GEMV's except ROPE_KV; N % 64 == 0, K % (64 S) == 0.
// kh: 1 = 4-wave blocks, 2 = 8-wave blocks splitting each 128-k step in two k halves (then
// K % (128 S) == 0 and M <= 128), 0 = the library setting (set_dgemm_kh) where it applies
// (M <= 128, K % (128 S) == 0), else 1
// wn: weight-row groups per block, 4 (64 rows) or 8 (128 rows; kh 1, M <= 128, N % 128 == 0;
// the same bits as 4), 0 = the op-level setting (MS_DGEMM_WN) where it applies, else 4
bool dgemm_supported(int M, int N, int K, int S, int epi, int kh = 0, int wn = 0);
void launch_dgemm(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int S, int ldo, int epi,
                  hipStream_t s, const RowScale* rs = nullptr, int kh = 0, int wn = 0);
int dgemm_kh_setting();

// ---- ggml K-quant weights (k_qgemv.hip)
enum { MS_QT_Q4_K = 12, MS_QT_Q6_K = 14 };  // ggml_type ids
constexpr int kQ4KBytes = 144, kQ6KBytes = 210, kQ6KPacked = 224;
// up to 3 row regions of one fused matrix, each of a single K-quant type (flat fields:
// no runtime-indexed kernel-argument arrays)
struct QMat {
  int n;
  const uint8_t* base0; int row0_0, type0, row_bytes0;
  const uint8_t* base1; int row0_1, type1, row_bytes1;
  const uint8_t* base2; int row0_2, type2, row_bytes2;
};
// large-batch K-quant decode projections (k_qdgemm.hip): the skinny GEMM with the weights
// streamed as packed Q4_K / Q6_K rows and dequantised in registers to their fp16-copy values;
// each region launched on its own (rows % 64 == 0 per region, first region at row 0), SwiGLU /
// argmax need one region; S > 1 = fp32 split-K slabs; K % (256 S) == 0, M <= 256
bool qdgemm_supported(int M, int N, int K, int S, int epi, const QMat& q);
void launch_qdgemm(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int S, int ldo, int epi,
                   hipStream_t s, const RowScale* rs = nullptr);
bool qdgemm_f16_supported(int M, int N, int K, int S, int epi);
void launch_qdgemm_f16(const f16_t* X, const f16_t* W, void* out, int M, int N, int K, int S, int ldo, int epi,
                       hipStream_t s, const RowScale* rs = nullptr);

inline uint64_t smix_host(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline int qblock_bytes(int type, bool packed) {
  return type == MS_QT_Q4_K ? kQ4KBytes : (packed ? kQ6KPacked : kQ6KBytes);
}
void launch_dequant_f32(int type, const uint8_t* blocks, int64_t n_blocks, float* out, hipStream_t s);
// raw ggml rows [rows][K/256 blocks] -> fp16 rows of a fused matrix (map_row) and, if dst_q,
// packed quantised rows at (map_row(r) - q_row_base)
void launch_quant_rows(int type, const uint8_t* blocks, int rows, int K, f16_t* dst_f16,
                       int map_mul, int map_add, uint8_t* dst_q, int q_row_base, hipStream_t s);
void launch_synth_qblocks(int type, uint8_t* blocks, int64_t n_blocks, uint64_t seed, float scale,
                          hipStream_t s);
bool qgemv_supported(int M, int N, int K, int epi, int rs_tiles = 0);
bool qgemv_split_supported(int M, int N, int K, int S, int rs_tiles = 0);
void launch_qgemv_split(const f16_t* X, const QMat& q, float* slabs, int M, int N, int K, int S,
                        hipStream_t s, const GemvArgs* ga = nullptr);
void launch_qgemv(const f16_t* X, const QMat& q, void* out, int M, int N, int K, int ldo, int epi,
                  const GemvArgs* ga, hipStream_t s);

void launch_attn_prefill(const f16_t* qkv, f16_t* out, int Hq, int Hk, KVView kv,
                         PrefillAttnArgs a, hipStream_t s);
// decode attention input: either fp16 qkv rows already roped with K/V in the cache
// (slabs == nullptr), or S fp32 split-K slabs of the QKV projection (rope-permuted Q/K rows):
// the kernel then adds the slabs, applies RoPE and writes the new token's K/V itself.
// With slabs, rs is the deferred RMSNorm scale of the QKV rows (tiles <= 256): the kernel
// rounds q/k/v = f16(rinv(b) * sum of the slabs).
struct DecodeQKV {
  const f16_t* qkv;
  const float* slabs;
  int S;
  const float* cos_tab;
  const float* sin_tab;
  RowScale rs;
};
// split partials of decode attention (combined by a second launch)
size_t attn_decode_workspace_bytes(int B, int Hq, int max_len);
bool attn_decode_supported(int B, int Hq, int Hk, int max_len);
// pages per wave of an engine's decode attention (from its max_batch / max_ctx, never from
// one step's batch: the split boundaries set a sequence's summation order)
int attn_decode_ppw(int max_batch, int Hk, int max_ctx);
void launch_attn_decode(const DecodeQKV& qa, f16_t* out, int Hq, int Hk, KVView kv,
                        DecodeAttnArgs a, float* ws, hipStream_t s);
// one page per wave, ppb waves per block (k_attn.hip "v2"): pages per block fixed per engine
// from its max_batch / max_ctx (the split boundaries set a sequence's summation order)
int attn_decode2_ppb(int max_batch, int Hk, int max_ctx);
bool attn_decode2_supported(int B, int Hq, int Hk, int max_len, int ppb);
size_t attn_decode2_workspace_bytes(int B, int Hq, int max_len, int ppb);
// cnt (optional, [B * Hk] zeroed unsigned): merge the splits inside the launch (the last block of
// each (sequence, kv head) combines, bit-identical to the second launch); null: combine kernel
void launch_attn_decode2(const DecodeQKV& qa, f16_t* out, int Hq, int Hk, KVView kv, DecodeAttnArgs a,
                         float* ws, int ppb, hipStream_t s, unsigned* cnt = nullptr);

// merge nsplit decode-attention partials (launch_attn_decode2's workspace layout) into out
void launch_attn_combine(const float* ws, f16_t* out, int B, int Hq, int Hk, int nsplit, hipStream_t s);

// decode attention v2's per-block phase stamps of its latest launch (MS_A2_STAMPS=1), [1024][32]
void attn2_stamps(unsigned long long* host, int n);

// ---- the decode step's layers as ONE persistent launch (k_persist.hip): engines of <= 8 slots
// on fp16 Llama-3.2-3B weights (persist_supported), bit-identical to the per-layer launches
struct PkLayer {
  const f16_t* wqkv;
  const f16_t* wo;
  const f16_t* wgu;
  const f16_t* wdown;
  const f16_t* ffn_norm;
  const f16_t* g_next;  // the next layer's attn_norm, or the final norm
  f16_t* kc;            // this layer's K / V pools (slot-major pages)
  f16_t* vc;
  const char* packed;   // the layer's matrices in stream order (launch_pack_layer)
};

struct PkArgs {
  PkLayer layers[28];  // kernel arguments: scalar loads, nothing queued behind the loader's DMA
  int L, B;
  const int32_t* seq_len;   // [B] keys incl. the new token
  const int32_t* seq_slot;  // [B]
  int max_pages, ppb, nsplit_ws;
  const float* cos_tab;
  const float* sin_tab;
  float eps, inv_h, scale_log2;
  int rs0_tiles;  // statistics tiles behind layer 0's xb (1: the embedding kernel)
  float* x;       // [B][H] residual
  f16_t* xb;      // [B][H] QKV input; the down epilogue writes the next one
  float* ssq;     // [tiles][B]
  float* slabs;   // [6][B][QKVN]
  float* ws;      // attention split partials [B][HQ][nsplit_ws][132]
  f16_t* attn;    // [B][H]
  f16_t* xg2;     // [B][H] gate/up input
  float* ssq2;    // [256][B]
  f16_t* hbuf;    // [B][F]
  unsigned* sync;  // [L * SL + 1] counters (zero between launches: the last workgroup resets them)
  unsigned* err;   // set on a hand-off timeout (never cleared here)
  unsigned spin;   // global polls before a hand-off gives up (MS_PK_SPIN; tests force 0)
  unsigned long long* stamps;  // diagnostic timeline (MS_PK_STAMPS=1): [256][L][16] s_memrealtime
  int depth;                   // DMA instructions each loader wave keeps in flight (MS_PK_DEPTH)
};
// the persistent step's in-kernel timeline of its latest launch (MS_PK_STAMPS=1), [256][L][16]
void persist_stamps(unsigned long long* host, int n);

size_t persist_sync_words(int L);
// the layer's QKV / O / gate-up / down weights in the persistent step's stream order (every ring slot
// contiguous, LDS swizzle applied): persist_packed_bytes_per_layer() bytes per layer
size_t persist_packed_bytes_per_layer();
void launch_pack_layer(const f16_t* wqkv, const f16_t* wo, const f16_t* wgu, const f16_t* wdown, void* out,
                       hipStream_t s);
bool persist_supported(int max_batch, int H, int F, int Hq, int Hk, int Dh, int L, int ppb, int n_cu);
void launch_decode_step(const PkArgs& a, hipStream_t s);

// synthetic weights (oracle/synth.py restates this generator)
// row maps: dst_row = (r >> 4) * map_mul + (r & 15) + map_add, or with map_mul == 0 the
// rope permutation dst_row = (r & ~127) + rope_perm(r & 127) + map_add
__host__ __device__ inline int rope_perm(int i) {
  return i < 64 ? 16 * (i >> 3) + (i & 7) : 16 * ((i - 64) >> 3) + 8 + ((i - 64) & 7);
}
__host__ __device__ inline size_t map_row(int r, int map_mul, int map_add) {
  if (map_mul == 0) return (size_t)(r & ~127) + rope_perm(r & 127) + map_add;
  return (size_t)(r >> 4) * map_mul + (r & 15) + map_add;
}
void launch_synth_linear(f16_t* dst, int kind, int layer, int rows, int cols, uint64_t seed,
                         float std, int map_mul, int map_add, hipStream_t s);
void launch_synth_norm(f16_t* dst, int kind, int layer, int n, uint64_t seed, float jitter,
                       hipStream_t s);
// scatter a logical [rows][cols] tensor into a fused/interleaved physical layout
void launch_scatter_rows(const f16_t* src, f16_t* dst, int rows, int cols, int map_mul,
                         int map_add, hipStream_t s);

}  // namespace ms
