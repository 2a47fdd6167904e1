// k_misc.hip -- HBM-bound helper kernels of the map call: embedding gather, RMSNorm,
// RoPE + paged-KV scatter, greedy argmax, synthetic weights.
//
// Reference semantics (EXT, inside Ollama for one /api/generate, SURVEY.md §2 table
// "ggml op replaced"): get_rows, rms_norm+mul, rope (llama3 freq factors), the greedy
// sampler.  Numerics contract restated in oracle/llama_ref.py.
#include "gemv_common.h"

namespace ms {

thread_local ProfEvents* g_prof = nullptr;

// ---------------------------------------------------------------- embedding
// x[t][:] = float(E[ids[t]][:]) ; 16-B loads, 32-B stores.  With gamma (a decode step's first
// layer): also xg[t] = f16(x[t] * gamma) and ssq[t] = sum of x[t]^2 (a fixed order)
// -- the first QKV projection's input and deferred-norm statistics, with no norm launch.
__global__ __launch_bounds__(256) void embed_kernel(const int32_t* __restrict__ ids,
                                                    const f16_t* __restrict__ emb, int H,
                                                    float* __restrict__ x, const f16_t* __restrict__ gamma,
                                                    f16_t* __restrict__ xg, float* __restrict__ ssq) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  const f16_t* row = emb + (size_t)ids[t] * H;
  float* xo = x + (size_t)t * H;
  float ss = 0.f;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    uint4 v = *(const uint4*)(row + c * 8);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float4 a, b;
    a.x = h_lo(w[0]); a.y = h_hi(w[0]);
    a.z = h_lo(w[1]); a.w = h_hi(w[1]);
    b.x = h_lo(w[2]); b.y = h_hi(w[2]);
    b.z = h_lo(w[3]); b.w = h_hi(w[3]);
    *(float4*)(xo + c * 8) = a;
    *(float4*)(xo + c * 8 + 4) = b;
    if (gamma) {  // block-uniform
      const uint4 gv = *(const uint4*)(gamma + c * 8);
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
      uint4 o;
      o.x = pack2h(a.x * h_lo(gw[0]) * kXgScale, a.y * h_hi(gw[0]) * kXgScale);
      o.y = pack2h(a.z * h_lo(gw[1]) * kXgScale, a.w * h_hi(gw[1]) * kXgScale);
      o.z = pack2h(b.x * h_lo(gw[2]) * kXgScale, b.y * h_hi(gw[2]) * kXgScale);
      o.w = pack2h(b.z * h_lo(gw[3]) * kXgScale, b.w * h_hi(gw[3]) * kXgScale);
      *(uint4*)(xg + (size_t)t * H + c * 8) = o;
      ss += (a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w);
    }
  }
  if (!gamma) return;
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssq[t] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Chained decode steps (engine.cpp decode_run): the step's argmax ids become the next
// step's input ids (an id outside [0, V) -- a failed row, already finished on the host --
// is fed as 0 so no gather leaves the table), every position / key count advances by one,
// and the raw ids are appended to the run's device ring at row `step` (args[4B], then
// incremented), which the host copies back once per run.  Args blob layout:
// [ids | positions | slots | key counts] (B each) + [step].  One block: B <= 256.
__global__ __launch_bounds__(256) void decode_advance_kernel(int32_t* __restrict__ args,
                                                             const int32_t* __restrict__ ids_out,
                                                             int32_t* __restrict__ ring, int B, int V) {
  const int b = threadIdx.x;
  const int step = args[4 * B];
  if (b < B) {
    const int id = ids_out[b];
    ring[(size_t)step * B + b] = id;
    args[b] = (id >= 0 && id < V) ? id : 0;
    args[B + b] += 1;
    args[3 * B + b] += 1;
  }
  __syncthreads();  // every thread has read `step`
  if (b == 0) args[4 * B] = step + 1;
}

void launch_decode_advance(int32_t* args, const int32_t* ids_out, int32_t* ring, int B, int V,
                           hipStream_t s) {
  if (B <= 0 || B > 256) return;  // callers chain sub-batches of <= 256 rows
  MS_LAUNCH(decode_advance_kernel, dim3(1), dim3(256), 0, s, args, ids_out, ring, B, V);
}

// One decode step's tail and the next step's head as ONE launch (three before): block b
// finishes row b's greedy id from the lm_head's {max, id} partials (argmax_partials_kernel's
// loop and merge: the same id), advances row b's arguments as decode_advance_kernel does, and
// gathers the next input row -- x[b] = E[id], xg[b] = f16(x * gamma), ssq[b] -- with
// embed_kernel's arithmetic on threads 0-255 (the same sums in the same order).  The run's
// step counter args[4B] moves once, by the last block to arrive on the ticket args[4B + 1]
// (every block has read it before its ticket), which that block zeroes again.
__global__ __launch_bounds__(1024) void decode_tail_kernel(const float2* __restrict__ part, int tiles,
                                                           int32_t* __restrict__ args, int32_t* __restrict__ ids_out,
                                                           int32_t* __restrict__ ring, int B, int V,
                                                           const f16_t* __restrict__ emb, int H, float* __restrict__ x,
                                                           const f16_t* __restrict__ gamma, f16_t* __restrict__ xg,
                                                           float* __restrict__ ssq) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int next_id;
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float2* p = part + (size_t)b * tiles;
  float v = -INFINITY;
  int idx = 0x7FFFFFFF;
  for (int t0 = 0; t0 < tiles; t0 += 8 * 1024) {
    float2 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = t0 + i * 1024 + tid;
      q[i] = t < tiles ? p[t] : make_float2(-INFINITY, __int_as_float(0x7FFFFFFF));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) amax_merge_dev(v, idx, q[i].x, __float_as_int(q[i].y));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax_merge_dev(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  if ((tid & 63) == 0) { sv[tid >> 6] = v; si[tid >> 6] = idx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 16; ++w) amax_merge_dev(v, idx, sv[w], si[w]);
    const int id = (idx == 0x7FFFFFFF || !__builtin_isfinite(v)) ? -1 : idx;
    ids_out[b] = id;
    const int step = args[4 * B];
    ring[(size_t)step * B + b] = id;
    const int in = (id >= 0 && id < V) ? id : 0;
    args[b] = in;
    args[B + b] += 1;
    args[3 * B + b] += 1;
    next_id = in;
    __threadfence();  // this block's read of the step counter precedes its ticket
    typedef __attribute__((address_space(1))) unsigned gu32_t;
    const unsigned arrived =
        __hip_atomic_fetch_add((gu32_t*)&args[4 * B + 1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == (unsigned)B - 1) {
      args[4 * B + 1] = 0;
      args[4 * B] = step + 1;
    }
  }
  __syncthreads();
  if (tid < 256) {
    const f16_t* row = emb + (size_t)next_id * H;
    float* xo = x + (size_t)b * H;
    float ss = 0.f;
    for (int c = tid; c < H / 8; c += 256) {
      uint4 e = *(const uint4*)(row + c * 8);
      const uint32_t w[4] = {e.x, e.y, e.z, e.w};
      float4 a, bb;
      a.x = h_lo(w[0]); a.y = h_hi(w[0]);
      a.z = h_lo(w[1]); a.w = h_hi(w[1]);
      bb.x = h_lo(w[2]); bb.y = h_hi(w[2]);
      bb.z = h_lo(w[3]); bb.w = h_hi(w[3]);
      *(float4*)(xo + c * 8) = a;
      *(float4*)(xo + c * 8 + 4) = bb;
      const uint4 gv = *(const uint4*)(gamma + c * 8);
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
      uint4 o;
      o.x = pack2h(a.x * h_lo(gw[0]) * kXgScale, a.y * h_hi(gw[0]) * kXgScale);
      o.y = pack2h(a.z * h_lo(gw[1]) * kXgScale, a.w * h_hi(gw[1]) * kXgScale);
      o.z = pack2h(bb.x * h_lo(gw[2]) * kXgScale, bb.y * h_hi(gw[2]) * kXgScale);
      o.w = pack2h(bb.z * h_lo(gw[3]) * kXgScale, bb.w * h_hi(gw[3]) * kXgScale);
      *(uint4*)(xg + (size_t)b * H + c * 8) = o;
      ss += (a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w) + (bb.x * bb.x + bb.y * bb.y + bb.z * bb.z + bb.w * bb.w);
    }
    ss = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
  }
  __syncthreads();
  if (tid == 0) ssq[b] = ((red[0] + red[1]) + red[2]) + red[3];
}

void launch_decode_tail(const void* partials, int tiles, int32_t* args, int32_t* ids_out, int32_t* ring, int B,
                        int V, const f16_t* emb, int H, float* x, const f16_t* gamma, f16_t* xg, float* ssq,
                        hipStream_t s) {
  if (B <= 0 || tiles <= 0) return;
  MS_LAUNCH(decode_tail_kernel, dim3(B), dim3(1024), 0, s, (const float2*)partials, tiles, args, ids_out, ring, B, V,
            emb, H, x, gamma, xg, ssq);
}

void launch_embed(const int32_t* ids, int T, const f16_t* emb, int H, float* x, hipStream_t s,
                  const f16_t* gamma, f16_t* xg, float* ssq) {
  if (T <= 0) return;
  MS_LAUNCH(embed_kernel, dim3(T), dim3(256), 0, s, ids, emb, H, x, gamma, xg, ssq);
}

// ---------------------------------------------------------------- RMSNorm
// The GEMM input of a normalised projection (deferred RMSNorm, kernels.h RowScale):
// y = f16(x * w) and ssq[r] = sum of x^2 (per thread, the wave tree, then the 4 waves in
// order), one 256-thread block per row; the row is read once (<= 8 float4 per thread kept in
// registers, H <= 8192).  The projection scales its output rows by rs_rinv(ssq[r]).
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* __restrict__ x,
                                                      const f16_t* __restrict__ w,
                                                      f16_t* __restrict__ y, float* __restrict__ ssq,
                                                      int H, const int32_t* __restrict__ row_idx) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  const int src = row_idx ? row_idx[r] : r;
  const float* xr = x + (size_t)src * H;
  const int n4 = H / 4;
  float4 v[8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = min(threadIdx.x + k * 256, n4 - 1);  // clamped, never predicated
    v[k] = *(const float4*)(xr + c * 4);
    if (threadIdx.x + k * 256 < n4) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  }
  f16_t* yr = y + (size_t)r * H;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c >= n4) break;
    uint2 wv = *(const uint2*)(w + c * 4);
    float g0 = h_lo(wv.x), g1 = h_hi(wv.x);
    float g2 = h_lo(wv.y), g3 = h_hi(wv.y);
    uint2 o;
    o.x = pack2h(v[k].x * g0 * kXgScale, v[k].y * g1 * kXgScale);
    o.y = pack2h(v[k].z * g2 * kXgScale, v[k].w * g3 * kXgScale);
    *(uint2*)(yr + c * 4) = o;
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssq[r] = ((red[0] + red[1]) + red[2]) + red[3];
}

void launch_rmsnorm(const float* x, const f16_t* w, f16_t* y, float* ssq, int rows, int H,
                    const int32_t* row_idx, hipStream_t s) {
  if (rows <= 0) return;
  MS_LAUNCH(rmsnorm_kernel, dim3(rows), dim3(256), 0, s, x, w, y, ssq, H, row_idx);
}

// Decode: the residual update of a split-K projection fused with the next norm's input.
// x[r] += (slab_0[r] + slab_1[r] + ... + slab_{S-1}[r]), then y[r] = f16(x[r] * w) and
// ssq[r] = sum of x[r]^2 (rmsnorm_kernel's order): the next projection's deferred RowScale.
// The summation order is fixed (slab order), so the result does not depend on timing or on
// the other rows.  One block per row; every load (x, w, all S slabs) is issued before the
// first add (S is a template parameter: a runtime trip count serialises the loads).
template <int S>
__global__ __launch_bounds__(256) void residual_rmsnorm_kernel(float* __restrict__ x,
                                                               const float* __restrict__ slabs,
                                                               int rows,
                                                               const f16_t* __restrict__ w,
                                                               f16_t* __restrict__ y,
                                                               float* __restrict__ ssq, int H) {
  constexpr int KMAX = 3;  // float4 per thread: H <= 3072
  __shared__ float red[4];
  const int r = blockIdx.x;
  float* xr = x + (size_t)r * H;
  const int n4 = H / 4;
  const size_t slab = (size_t)rows * H;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  f32x4 v[KMAX], p[KMAX][S > 0 ? S : 1];
  u32x2 wv[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int c = min((int)threadIdx.x + k * 256, n4 - 1);
    v[k] = *(const f32x4*)(xr + c * 4);
    wv[k] = *(const u32x2*)(w + c * 4);
#pragma unroll
    for (int q = 0; q < S; ++q) p[k][q] = *(const f32x4*)(slabs + q * slab + (size_t)r * H + c * 4);
  }
  // every load above is in flight before the first add (one memory round trip), and the
  // residual stores wait until after the row reduction (on gfx9 stores count in vmcnt, so a
  // store between the loads and their last use makes the reduction wait for it too).  The
  // empty asm statements make every loaded value opaque here, so no add is hoisted between
  // the loads (the compiler otherwise interleaves them and issues the loads in three waves).
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    asm volatile("" : "+v"(v[k]));
    asm volatile("" : "+v"(wv[k]));
#pragma unroll
    for (int q = 0; q < S; ++q) asm volatile("" : "+v"(p[k][q]));
  }
  if constexpr (S > 0) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      f32x4 acc = p[k][0];
#pragma unroll
      for (int q = 1; q < S; ++q) acc += p[k][q];
      v[k] += acc;
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (threadIdx.x + k * 256 < n4) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  f16_t* yr = y + (size_t)r * H;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c >= n4) break;
    if constexpr (S > 0) *(f32x4*)(xr + c * 4) = v[k];
    const float g0 = h_lo(wv[k].x), g1 = h_hi(wv[k].x);
    const float g2 = h_lo(wv[k].y), g3 = h_hi(wv[k].y);
    uint2 o;
    o.x = pack2h(v[k].x * g0 * kXgScale, v[k].y * g1 * kXgScale);
    o.y = pack2h(v[k].z * g2 * kXgScale, v[k].w * g3 * kXgScale);
    *(uint2*)(yr + c * 4) = o;
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssq[r] = ((red[0] + red[1]) + red[2]) + red[3];
}

bool residual_rmsnorm_supported(int S, int H) { return S >= 0 && S <= 8 && H % 4 == 0 && H <= 3072; }

void launch_residual_rmsnorm(float* x, const float* slabs, int S, const f16_t* w, f16_t* y,
                             float* ssq, int rows, int H, hipStream_t s) {
  if (rows <= 0) return;
  if (H > 3072) {  // wider models: the plain kernel (S = 0 only)
    launch_rmsnorm(x, w, y, ssq, rows, H, nullptr, s);
    return;
  }
#define RN(S_)                                                                                 \
  case S_:                                                                                     \
    MS_LAUNCH(residual_rmsnorm_kernel<S_>, dim3(rows), dim3(256), 0, s, x, slabs, rows, w, y, ssq, H); \
    break;
  switch (S) { RN(0) RN(1) RN(2) RN(3) RN(4) RN(5) RN(6) RN(7) RN(8) }
#undef RN
}

// ---------------------------------------------------------------- RoPE + KV scatter
// qkv row layout: [Q heads | K heads | V heads] x 128, Q/K heads rope-permuted (the fused
// weight rows are uploaded in rope_perm order so a 16-row GEMV tile holds dims i and i+64).
// rotate-half pairs (i, i+64).  One block per token; the token's Q|K part is staged in LDS
// first because Q is rewritten in place in natural dim order.
__global__ __launch_bounds__(256) void rope_kv_kernel(f16_t* __restrict__ qkv, int Hq, int Hk,
                                                      const int32_t* __restrict__ tok_pos,
                                                      const int32_t* __restrict__ tok_slot,
                                                      const float* __restrict__ cos_tab,
                                                      const float* __restrict__ sin_tab,
                                                      KVView kv, int h_begin) {
  __shared__ __attribute__((aligned(16))) f16_t st[64 * kHeadDim];  // <= 64 Q+K heads
  const int t = blockIdx.x;
  const int pos = tok_pos[t];
  const int slot = tok_slot[t];
  const int page = kv.block_table[(size_t)slot * kv.max_pages + pos / kPage];
  const int off = pos % kPage;
  const int row_elems = (Hq + 2 * Hk) * kHeadDim;
  f16_t* row = qkv + (size_t)t * row_elems;
  // heads h_begin.. (0: Q, K and V; Hq: K and V only)
  const int qk_elems = (Hq + Hk) * kHeadDim, e0 = h_begin * kHeadDim;
  for (int c = threadIdx.x; c < (qk_elems - e0) / 8; c += blockDim.x)
    *(uint4*)(st + e0 + c * 8) = *(const uint4*)(row + e0 + c * 8);
  __syncthreads();
  const int items = (Hq + 2 * Hk - h_begin) * 16;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int head = h_begin + (it >> 4);
    const int i0 = (it & 15) * 4;  // dims i0..i0+3 and 64+i0..64+i0+3
    uint2 olo, ohi;
    if (head < Hq + Hk) {  // Q or K: rotate (from the permuted staging copy)
      const f16_t* hp = st + head * kHeadDim;
      const uint2 lo = *(const uint2*)(hp + rope_perm(i0));
      const uint2 hi = *(const uint2*)(hp + rope_perm(64 + i0));
      const float4 c = *(const float4*)(cos_tab + (size_t)pos * 64 + i0);
      const float4 sn = *(const float4*)(sin_tab + (size_t)pos * 64 + i0);
      float a[4] = {h_lo(lo.x), h_hi(lo.x),
                    h_lo(lo.y), h_hi(lo.y)};
      float b[4] = {h_lo(hi.x), h_hi(hi.x),
                    h_lo(hi.y), h_hi(hi.y)};
      const float cc[4] = {c.x, c.y, c.z, c.w};
      const float ss[4] = {sn.x, sn.y, sn.z, sn.w};
      float ra[4], rb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ra[j] = __fsub_rn(__fmul_rn(a[j], cc[j]), __fmul_rn(b[j], ss[j]));
        rb[j] = __fadd_rn(__fmul_rn(b[j], cc[j]), __fmul_rn(a[j], ss[j]));
      }
      olo.x = pack2h(ra[0], ra[1]); olo.y = pack2h(ra[2], ra[3]);
      ohi.x = pack2h(rb[0], rb[1]); ohi.y = pack2h(rb[2], rb[3]);
    } else {  // V: natural order, copied as is
      const f16_t* hp = row + head * kHeadDim;
      olo = *(const uint2*)(hp + i0);
      ohi = *(const uint2*)(hp + i0 + 64);
    }
    if (head < Hq) {
      f16_t* hp = row + head * kHeadDim;
      *(uint2*)(hp + i0) = olo;
      *(uint2*)(hp + i0 + 64) = ohi;
    } else {
      const bool is_k = head < Hq + Hk;
      const int kh = is_k ? head - Hq : head - Hq - Hk;
      f16_t* dst = (is_k ? kv.k : kv.v) +
                    (((size_t)page * kv.n_kv_heads + kh) * kPage + off) * kHeadDim;
      *(uint2*)(dst + i0) = olo;
      *(uint2*)(dst + i0 + 64) = ohi;
    }
  }
}

void launch_rope_kv(f16_t* qkv, int T, int Hq, int Hk, const int32_t* tok_pos,
                    const int32_t* tok_slot, const float* cos_tab, const float* sin_tab,
                    KVView kv, hipStream_t s, bool rope_q) {
  if (T <= 0) return;
  MS_LAUNCH(rope_kv_kernel, dim3(T), dim3(256), 0, s, qkv, Hq, Hk, tok_pos, tok_slot,
                     cos_tab, sin_tab, kv, rope_q ? 0 : Hq);
}

// ---------------------------------------------------------------- greedy argmax
// Ollama T=0 / top_k=1 semantics; ties resolve to the lowest id (oracle: np.argmax).
__device__ __forceinline__ void amax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ logits, int n,
                                                      int32_t* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const float* row = logits + (size_t)blockIdx.x * n;
  float v = -INFINITY;
  int idx = 0x7FFFFFFF;
  const int n4 = n / 4;
  for (int c = threadIdx.x; c < n4; c += 1024) {
    float4 q = *(const float4*)(row + c * 4);
    amax_merge(v, idx, q.x, c * 4);
    amax_merge(v, idx, q.y, c * 4 + 1);
    amax_merge(v, idx, q.z, c * 4 + 2);
    amax_merge(v, idx, q.w, c * 4 + 3);
  }
  for (int c = n4 * 4 + threadIdx.x; c < n; c += 1024) amax_merge(v, idx, row[c], c);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float v2 = __shfl_xor(v, o, 64);
    int i2 = __shfl_xor(idx, o, 64);
    amax_merge(v, idx, v2, i2);
  }
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = v; si[threadIdx.x >> 6] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) amax_merge(v, idx, sv[w], si[w]);
    // no finite maximum (a NaN/Inf row): -1 tells the engine this chunk failed
    out[blockIdx.x] = (idx == 0x7FFFFFFF || !__builtin_isfinite(v)) ? -1 : idx;
  }
}

void launch_argmax(const float* logits, int rows, int n, int32_t* out, hipStream_t s) {
  if (rows <= 0) return;
  MS_LAUNCH(argmax_kernel, dim3(rows), dim3(1024), 0, s, logits, n, out);
}

// ---------------------------------------------------------------- synthetic weights
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int limb_sum(uint64_t seed_h, int kind, int layer, int r, int c) {
  const uint64_t key = ((uint64_t)kind << 58) | ((uint64_t)layer << 50) | ((uint64_t)r << 20) |
                       (uint64_t)c;
  const uint64_t h = splitmix64(key ^ seed_h);
  return (int)((h & 0xFFFF) + ((h >> 16) & 0xFFFF) + ((h >> 32) & 0xFFFF) + ((h >> 48) & 0xFFFF)) -
         131070;
}

// the generator's values are bf16-rounded (integer RNE, finite inputs only), as oracle/synth.py
// restates; the engine stores them as fp16 (exact for |v| >= 2^-17: a bf16 significand has 8
// bits; smaller magnitudes are rounded to fp16's subnormal grid, as llama.cpp's F16 converter
// would round them)
__device__ __forceinline__ f16_t rne_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return f2h(__uint_as_float((u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u));
}

__global__ void synth_linear_kernel(f16_t* dst, int kind, int layer, int rows, int cols,
                                    uint64_t seed_h, float scale, int map_mul, int map_add) {
  const size_t n = (size_t)rows * cols;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / cols), c = (int)(e % cols);
    const float v = __fmul_rn((float)limb_sum(seed_h, kind, layer, r, c), scale);
    dst[map_row(r, map_mul, map_add) * cols + c] = rne_bits(v);
  }
}

__global__ void synth_norm_kernel(f16_t* dst, int kind, int layer, int n, uint64_t seed_h,
                                  float scale) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const float v = __fadd_rn(1.0f, __fmul_rn((float)limb_sum(seed_h, kind, layer, 0, c), scale));
    dst[c] = rne_bits(v);
  }
}

static uint64_t host_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void launch_synth_linear(f16_t* dst, int kind, int layer, int rows, int cols, uint64_t seed,
                         float std, int map_mul, int map_add, hipStream_t s) {
  // scale = float32(std*sqrt(3)/65536), computed in double then rounded once (as numpy does)
  const float scale = (float)((double)std * 1.7320508075688772 / 65536.0);
  MS_LAUNCH(synth_linear_kernel, dim3(2048), dim3(256), 0, s, dst, kind, layer, rows,
                     cols, host_splitmix64(seed), scale, map_mul, map_add);
}

void launch_synth_norm(f16_t* dst, int kind, int layer, int n, uint64_t seed, float jitter,
                       hipStream_t s) {
  const float scale = (float)((double)jitter / 131070.0);
  MS_LAUNCH(synth_norm_kernel, dim3(16), dim3(256), 0, s, dst, kind, layer, n,
                     host_splitmix64(seed), scale);
}

__global__ void scatter_rows_kernel(const f16_t* __restrict__ src, f16_t* __restrict__ dst,
                                    int rows, int cols, int map_mul, int map_add) {
  const int r = blockIdx.x;
  const size_t dr = map_row(r, map_mul, map_add);
  for (int c = threadIdx.x; c < cols; c += blockDim.x) dst[dr * cols + c] = src[(size_t)r * cols + c];
}

void launch_scatter_rows(const f16_t* src, f16_t* dst, int rows, int cols, int map_mul,
                         int map_add, hipStream_t s) {
  MS_LAUNCH(scatter_rows_kernel, dim3(rows), dim3(256), 0, s, src, dst, rows, cols,
                     map_mul, map_add);
}

}  // namespace ms
