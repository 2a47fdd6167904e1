// k_mlp.hip -- the decode MLP of one layer as ONE launch (small-regime engines, fp16 weights,
// B <= 8 rows): gate/up GEMV + SwiGLU, a chip-wide hand-off of h, then the down GEMV with
// the residual epilogue.
//
// Why.  In the decode step every projection is its own launch, and a launch of a weight
// stream pays a fixed ramp -- dispatch, the first loads' latency, the tail -- that the kernel
// before it cannot hide (the next launch starts only when the previous one has drained).
// Here the down projection's weights do not depend on h, so each workgroup issues its whole
// down-weight slice (12 rows x 8192, 192 KiB per CU, held in registers) BEFORE it waits for
// the other workgroups' h: the down stream is already in flight when the hand-off completes.
//
// Arithmetic: bit-identical to the two launches it replaces (k_gemv.hip gemv_kernel<1, 2,
// SWIGLU, 3, LDS, RS> on 512 32-row tiles, then gemv_kernel<1, 1, RESID_SSQ, 8, LDS> on 256
// 12-row tiles): the same per-wave K ranges (16 waves), the same MFMA order, the same
// cross-wave reduction order and epilogues (gemv_common.h).  Each of the 256 workgroups (one
// per CU, all resident) takes gate/up tiles b and b + 256, then down tile b.
//
// Hand-off (cdna_hip_programming.md Guideline 16, R1): h is stored write-through (sc1, agent
// scope), every storing wave drains its stores (s_waitcnt vmcnt(0)) before the workgroup's
// barrier, then ONE lane adds to an agent-scope arrival counter; every wave then issues its
// down slice, and one wave polls the word
// (relaxed, bounded: after kSpinLimit polls it records a timeout and goes on -- never a hang);
// h is then read with sc1 loads straight into registers (no stale L1/L2 copy can be read,
// no acquire fence) and staged into the LDS image the down MFMAs read.  The last workgroup
// past the poll resets both counters for the next launch (stream order makes that visible).
#include "gemv_common.h"

namespace ms {

constexpr int kMlpBlocks = 256;       // one workgroup per CU: all resident (the hand-off needs it)
constexpr int kMlpWaves = 16;         // as the unfused GEMVs' plans at K = 3072 / 8192
constexpr int kMlpGuU = 3;            // 3072 / 64 / 16
constexpr int kMlpDnU = 8;            // 8192 / 64 / 16
constexpr int kMlpRt = 12;            // down rows per tile: 3072 / 12 = 256 tiles
constexpr unsigned kSpinLimit = 1u << 20;  // ~1 s of polls: a give-up, never a hang
constexpr int kMlpPollWave = 0;       // the wave that polls the arrival counter

typedef __attribute__((address_space(1))) unsigned gu32_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlp_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

struct MlpArgs {
  const f16_t* xb;     // [M][H] f16(x * ffn_norm): the gate/up input (deferred-norm rows)
  const f16_t* wgu;    // [2F][H], gate/up interleaved per 16 rows
  const f16_t* wdown;  // [H][F]
  f16_t* h;            // [M][F] SwiGLU output (the hand-off payload)
  float* x;            // [M][H] fp32 residual
  unsigned* sync;      // [2]: arrivals, departures (zero between launches)
  unsigned* err;       // timeout flag (set, never cleared by the kernel)
  unsigned spin;       // polls before the hand-off gives up (kSpinLimit; MS_MLP_SPIN for tests)
  GemvArgs gu;         // .rs: the gate/up rows' deferred-norm statistics
  GemvArgs dn;         // .rt = 12, .ssq_out / .gamma / .xg_out: the residual epilogue
  int M, H, F, rinv_off;
};

__global__ __launch_bounds__(1024) void mlp_decode_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int MT = 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, H = a.H, F = a.F;
  const int b = blockIdx.x;
  // the down phase: this wave's 12-row x (U x 64) slice of Wdown, and the residual prefetch
  constexpr int UD = kMlpDnU;
  const int n0 = b * kMlpRt;
  const int kbd = wave * UD * 64;
  uint4 wd[UD][2];
  auto issue_down = [&]() {
    const f16_t* wp = a.wdown + (size_t)(n0 + min(fr, kMlpRt - 1)) * F + kbd + 16 * fg;
#pragma unroll
    for (int u = 0; u < UD; ++u) {
      wd[u][0] = ldw16(wp + u * 64);
      wd[u][1] = ldw16(wp + u * 64 + 8);
    }
  };
  // the residual element and gain this thread's epilogue updates (gemv_common.h resid_prefetch,
  // one element per thread of waves 0..3): loaded first, the gain kept as raw fp16 bits so no
  // conversion waits for it here
  // (unconditional, clamped: a conditional load's merge made every wave wait for it here)
  float pre_x;
  unsigned short pre_g;
  {
    int row, col, c;
    gemv_elem(tid & 255, 1, n0, row, col, c);
    pre_x = a.x[(size_t)min(row, M - 1) * H + min(col, H - 1)];
    pre_g = *(const unsigned short*)(a.dn.gamma + min(col, H - 1));
  }

  // ---------------------------------------------------------------- phase 1: gate/up
  {
    constexpr int NT = 4;  // tiles b and b + 256, two 16-row (gate, up) halves each
    constexpr int U = kMlpGuU;
    const int kbeg = wave * U * 64;
    rs_begin<false>(smem, a.rinv_off, a.gu.rs, M);
    gemv_dma_x(smem, a.xb, M, H, H);
    __builtin_amdgcn_sched_barrier(0);
    uint4 w[U][NT][2];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int tile = n < 2 ? b : b + kMlpBlocks;
      const f16_t* wp = a.wgu + (size_t)(tile * 32 + (n & 1) * 16 + fr) * H + kbeg + 16 * fg;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        w[u][n][0] = ldw16(wp + u * 64);
        w[u][n][1] = ldw16(wp + u * 64 + 8);
      }
    }
    // the X image and the staged row statistics (issued first) have landed once at most the
    // weight loads are pending
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(U * NT * 2));
    __builtin_amdgcn_s_barrier();
    f32x4 acc[MT][NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int xrow = min(fr, M - 1);
      const int k0 = kbeg + u * 64 + 16 * fg;
      const f16x8 x0 = *(const f16x8*)(smem + x_lds(xrow, k0, H));
      const f16x8 x1 = *(const f16x8*)(smem + x_lds(xrow, k0 + 8, H));
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        acc[0][n] = mfma16(x0, as_f16x8(w[u][n][0]), acc[0][n]);
        acc[0][n] = mfma16(x1, as_f16x8(w[u][n][1]), acc[0][n]);
      }
    }
    // the gate/up weight registers are free: every wave but the storing one puts its down
    // slice in flight now, under the epilogue and the hand-off (the storing wave must drain its
    // h stores with vmcnt(0) first, so it issues its slice after publishing)
    // gemv_finish's steps: rinv from the staged statistics, per-wave partials -> LDS
    constexpr int ELEMS = MT * NT * 256;
    __syncthreads();
    rs_finish<false>(smem, a.rinv_off, a.gu.rs, M, 0.f);
    float* red = (float*)smem;
#pragma unroll
    for (int n = 0; n < NT; ++n) *(f32x4*)&red[wave * ELEMS + (n * 64 + lane) * 4] = acc[0][n];
    __syncthreads();
    // SwiGLU of both tiles (gemv_epilogue's sums, in wave order) -> the block's h tile in LDS,
    // hs[row][32]: columns 0..15 tile b, 16..31 tile b + 256
    const float* rinv = (const float*)(smem + a.rinv_off);
    if (tid < 2 * 256) {
      const int p = tid >> 8, e = tid & 255, l = (e >> 2) & 63, j = e & 3;
      const int row = 4 * (l >> 4) + j;
      if (row < M) {
        float g = 0.f, u = 0.f;
        for (int q = 0; q < kMlpWaves; ++q) g += red[q * ELEMS + ((2 * p) * 64 + l) * 4 + j];
        for (int q = 0; q < kMlpWaves; ++q) u += red[q * ELEMS + ((2 * p + 1) * 64 + l) * 4 + j];
        const float rv = rinv[row];
        g *= rv;
        u *= rv;
        const int tile = p == 0 ? b : b + kMlpBlocks;
        const f16_t hv = f2h(g / (1.0f + __expf(-g)) * u);
        __hip_atomic_store((unsigned short*)(a.h + (size_t)row * F + tile * 16 + (l & 15)), (unsigned short)hv,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through (sc1)
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its h stores
    __syncthreads();
  }

  // ---------------------------------------------------------------- hand-off
  if (tid == 0) __hip_atomic_fetch_add((gu32_t*)&a.sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the down weights do not depend on h: every wave's slice goes in flight before the wait
  // (issued under the gate/up epilogue instead, the down stream slowed the gate/up stragglers
  // every workgroup waits for: 42.7 vs 34.0 us per layer, profiles/r04/v13_*)
  issue_down();
  if (wave == kMlpPollWave) {
    bool ok = false;
    for (unsigned it = 0; it < a.spin; ++it) {
      if (__hip_atomic_load((gu32_t*)&a.sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= kMlpBlocks) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok && lane == 0) __hip_atomic_store((gu32_t*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // h -> the LDS image (x_lds layout), by sc1 loads into registers (16 B per lane per load)
  {
    const __amdgpu_buffer_rsrc_t hr = mlp_rsrc(a.h, (unsigned)((size_t)M * F * 2));
    const int kch = F >> 3, n = M * kch;
    for (int c = tid; c < n; c += 1024) {
      const int r = c / kch, k = (c - r * kch) << 3;
      typedef uint32_t u4v __attribute__((ext_vector_type(4)));
      const u4v v = __builtin_amdgcn_raw_buffer_load_b128(hr, (r * F + k) * 2, 0, 16);
      *(u4v*)(smem + x_lds(r, k, F)) = v;
    }
  }
  __syncthreads();
  if (tid == 0) {  // every workgroup is past the poll once all have departed: reset for the next launch
    const unsigned d = __hip_atomic_fetch_add((gu32_t*)&a.sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == kMlpBlocks - 1) {
      __hip_atomic_store((gu32_t*)&a.sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32_t*)&a.sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // ---------------------------------------------------------------- phase 2: down + residual
  wait_vmcnt0();
  f32x4 acc[MT][1];
  acc[0][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < UD; ++u) {
    const int xrow = min(fr, M - 1);
    const int k0 = kbd + u * 64 + 16 * fg;
    const f16x8 x0 = *(const f16x8*)(smem + x_lds(xrow, k0, F));
    const f16x8 x1 = *(const f16x8*)(smem + x_lds(xrow, k0 + 8, F));
    acc[0][0] = mfma16(x0, as_f16x8(wd[u][0]), acc[0][0]);
    acc[0][0] = mfma16(x1, as_f16x8(wd[u][1]), acc[0][0]);
  }
  const ResidPre pre{pre_x, h2f(pre_g)};
  gemv_finish<MT, 1, MS_GEMV_EPI_RESID_SSQ, false, false, false>(acc, smem, a.rinv_off, M, H, H, a.x, n0, a.dn,
                                                                pre);
}

// LDS: phase 1 [max(X image, per-wave partials)][rinv][staged statistics]; phase 2 the h image
static size_t mlp_lds(int M, int H, int F, const RowScale& rs, int* rinv_off) {
  const size_t main1 = std::max(gemv_x_lds_bytes(M, H), (size_t)kMlpWaves * 4 * 256 * 4);
  *rinv_off = (int)gemv_rinv_offset(main1);
  const size_t p1 = gemv_lds_total(main1, rs, M);
  const size_t p2 = std::max(gemv_x_lds_bytes(M, F), (size_t)kMlpWaves * 256 * 4);
  return std::max(p1, p2);
}

bool mlp_decode_supported(int M, int H, int F, int rs_tiles) {
  if (M < 1 || M > 8 || H != kMlpBlocks * kMlpRt || F != 2 * kMlpBlocks * 16) return false;
  if (H != kMlpWaves * kMlpGuU * 64 || F != kMlpWaves * kMlpDnU * 64) return false;
  if (!gemv_rs_supported(M, rs_tiles)) return false;
  int ro;
  const RowScale rs = make_row_scale(reinterpret_cast<const float*>(16), rs_tiles, H, 0.f);
  return mlp_lds(M, H, F, rs, &ro) <= 160 * 1024;
}

void launch_mlp_decode(const f16_t* xb, const f16_t* wgu, const f16_t* wdown, f16_t* h, float* x, int M, int H,
                       int F, const RowScale& rs, float* ssq_out, const f16_t* gamma_next, f16_t* xg_out,
                       unsigned* sync, unsigned* err, hipStream_t s) {
  if (!mlp_decode_supported(M, H, F, rs.tiles)) return;  // callers check
  MlpArgs a{};
  a.xb = xb;
  a.wgu = wgu;
  a.wdown = wdown;
  a.h = h;
  a.x = x;
  a.sync = sync;
  a.err = err;
  // MS_MLP_SPIN: the poll bound (0 forces the timeout path: test_fused_decode_mlp_timeout_recovers)
  const char* sv = getenv("MS_MLP_SPIN");  // read per launch (host side; graphs capture it once)
  a.spin = sv ? (unsigned)strtoul(sv, nullptr, 10) : kSpinLimit;
  a.gu.rs = rs;
  a.dn.rt = kMlpRt;
  a.dn.ssq_out = ssq_out;
  a.dn.gamma = gamma_next;
  a.dn.xg_out = xg_out;
  a.M = M;
  a.H = H;
  a.F = F;
  const size_t lds = mlp_lds(M, H, F, rs, &a.rinv_off);
  MS_LAUNCH(mlp_decode_kernel, dim3(kMlpBlocks), dim3(64 * kMlpWaves), lds, s, a);
}

}  // namespace ms
