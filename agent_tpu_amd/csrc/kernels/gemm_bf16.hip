// bf16 MFMA GEMM with fused epilogues for the BERT/T5 encoder hot path
// (QKV projection, attention out-proj + residual,
// FFN1 + GELU, FFN2 + residual; pooler + tanh).
//
//   C[M,N] = epi( A[M,K] · Bt[N,K]ᵀ )      A, Bt, C, R bf16; bias fp32
//   epi(x) = act(x + bias[n]) + R[m,n]      act ∈ {id, erf-GELU, tanh}
//
// Weights are stored [N][K] (K contiguous, = torch nn.Linear.weight), so both
// operand tiles are K-contiguous rows and every MFMA fragment is one 16-byte
// ds_read_b128.
//
// CDNA4 structure (cdna_hip_programming.md §5):
//  * v_mfma_f32_16x16x32_bf16, 64-wide waves, 4 waves as 2x2, 64x64 per wave.
//  * A/B tiles staged global -> LDS with global_load_lds_dwordx4 (no VGPR
//    round trip), two LDS buffers so tile k+1 streams in while tile k computes.
//  * LDS image XOR-swizzled on the 16-B chunk: chunk' = chunk ^ ((row>>1)&7).
//    128-B rows put two rows in one 256-B bank row; the swizzle makes the 16
//    rows a ds_read_b128 lane group touches land on 16 distinct 16-B slots
//    (conflict-free). glds writes lane-linearly, so the permutation is applied
//    to the per-lane GLOBAL source address and inverted on the read (rule 21).
//  * MFMA operands swapped (Bt as "A", A as "B") so each lane's accumulator
//    holds 4 consecutive output columns of one row -> 8-byte vector stores and
//    16-byte bias loads in the epilogue.
//  * Tile order: bijective XCD remap, N-fastest within a row panel, so the
//    blocks that share an A panel run on one XCD and hit its L2.
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/l2_prefetch.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#ifndef ATPU_GEMM_SYNC_EPI
#define ATPU_GEMM_SYNC_EPI 1
#endif

namespace atpu {
namespace {

constexpr int kBK = 64;          // K per LDS stage
constexpr int kRowBytes = kBK * 2;  // 128 B per staged row

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// SPLIT: split-K. blockIdx.y = K slice (length K); the slice stores its fp32
// partial tile in ws[slice][M][N] and splitk_reduce_kernel sums the slices in
// order (deterministic) with the epilogue fused. (An in-kernel "last block
// reduces" fixup was measured 10x slower: the device-scope fence it needs
// writes back the XCD's whole L2 on gfx950.)
// KvScatter destination (decode QKV GEMM writes K|V straight into the KV cache)
struct KvOut {
  bf16* cache = nullptr;
  int ld = 0, T = 0, col0 = 0;
  const int32_t* step = nullptr;
};

// RowRms (EPI & kEpiRowRms): every lane sums the squares of the A fragments it reads
// (v_dot2c_f32_bf16); the 4 lanes of a row (its 4 k-chunks) complete the row's sum over
// the whole K loop, and the accumulator of that row is scaled by rsqrt(mean + eps).
// MFMA operands are swapped (Bt as "A"), so an accumulator's row is the lane's A
// fragment row: no transposition of the statistics.
__device__ __forceinline__ float sumsq_bf16x8(bf16x8 a, float acc) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2_t p = bf16x2_t{a[2 * e], a[2 * e + 1]};
    acc = __builtin_amdgcn_fdot2_f32_bf16(p, p, acc, false);
  }
  return acc;
}
// sum of the 8 values of a 16-B chunk (fdot2 against ones), fp32
__device__ __forceinline__ float sum_bf16x8(bf16x8 a, float acc) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t one = bf16x2_t{(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
  for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{a[2 * e], a[2 * e + 1]}, one, acc, false);
  return acc;
}


// Decode LayerNorm folding (kEpiRowLn / kEpiResLn / kEpiRowStats; GemmArgs fields of the
// same names). A row's statistics travel as partial (sum, sumsq) per 32-column slab, written
// by the epilogue of the GEMM that produced the row (RowStats) and summed by its consumers:
// no K-loop VALU work in the consumers, no LayerNorm pass between them.
struct LnDec {
  const float* colsum = nullptr;    // RowLn: [N] column sums of the gamma-folded weights
  const float* in_part = nullptr;   // RowLn: [K/32][M][2] partials of A's rows
  const float* res_part = nullptr;  // ResLn: [N/32][M][2] partials of R's rows
  const float* gamma = nullptr;     // ResLn: [N] LN gamma of R
  float* part_out = nullptr;        // RowStats: [N/32][M][2] partials of C's rows (bf16-rounded values)
};

// Row partials of a width <= 1024 row (<= 32 slots): the 4 lanes of the row (fchunk 0-3)
// take slots fchunk, fchunk + 4, ... Loaded at kernel start (every load in flight at once,
// landing under the K loop), reduced in the epilogue.
constexpr int kPartPerLane = 8;
__device__ __forceinline__ void part_prefetch(float2 (&v)[kPartPerLane], const float* part, int slots, int M, int m,
                                              int fchunk) {
  // unconditional loads (a clamped slot; part_ln drops the extras): a conditional load per
  // slot became a branch per slot and hipcc drained vmcnt at the joins
  const size_t mc = min(m, M - 1);
#pragma unroll
  for (int t = 0; t < kPartPerLane; ++t) {
    const int k = min(fchunk + 4 * t, slots - 1);
    v[t] = *reinterpret_cast<const float2*>(part + 2 * ((size_t)k * M + mc));
  }
}
// (rstd, rstd*mu) of the row from its prefetched partials; every lane of the row gets it.
// Variance as E[x^2] - mu^2 in fp32, clamped at 0. Call with all 4 lanes of the row active.
__device__ __forceinline__ float2 part_ln(const float2 (&v)[kPartPerLane], int slots, int fchunk, float eps) {
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int t = 0; t < kPartPerLane; ++t) {
    const bool in = fchunk + 4 * t < slots;
    s += in ? v[t].x : 0.f;
    q += in ? v[t].y : 0.f;
  }
  const float inv = 1.f / (32 * slots);
  const float mu = lane_rows_sum(s) * inv;
  const float var = fmaxf(lane_rows_sum(q) * inv - mu * mu, 0.f);
  const float rs = __builtin_amdgcn_rsqf(var + eps);
  return float2{rs, rs * mu};
}

template <int BM, int BN, int WM, int WN, int EPI, int SPLIT = 0>
__global__ __launch_bounds__(WM* WN * 64, 2) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K,
    float* __restrict__ ws = nullptr, float rms_eps = 0.f, KvOut kvo = {}, LnDec ln = {}) {
  static_assert(!(SPLIT && (EPI & (kEpiRowRms | kEpiRowLn | kEpiResLn))), "row statistics need the whole K loop");
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int A_BYTES = BM * kRowBytes;
  constexpr int B_BYTES = BN * kRowBytes;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "stage split");
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (N + BN - 1) / BN;
  const int ntm = (M + BM - 1) / BM;
  if constexpr (SPLIT) {
    A += (size_t)blockIdx.y * K;
    Bt += (size_t)blockIdx.y * K;
  }
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * BM;
  const int n0 = (tile % ntn) * BN;

  // ---- per-lane staging addresses (row, swizzled chunk) ----
  // wave-instruction i of this wave covers staged rows [(i*NW+wave)*8, +8)
  const int srow = lane >> 3, spos = lane & 7;
  const bf16* a_src[BM / 8 / NW];
  const bf16* b_src[BN / 8 / NW];
#pragma unroll
  for (int i = 0; i < BM / 8 / NW; ++i) {
    const int r = (i * NW + wave) * 8 + srow;
    const int gr = min(m0 + r, M - 1);
    a_src[i] = A + (size_t)gr * lda + swz(r, spos) * 8;
  }
#pragma unroll
  for (int i = 0; i < BN / 8 / NW; ++i) {
    const int r = (i * NW + wave) * 8 + srow;
    const int gr = min(n0 + r, N - 1);
    b_src[i] = Bt + (size_t)gr * ldb + swz(r, spos) * 8;
  }

  auto stage = [&](int kt, int buf) {
    char* base = lds + buf * STAGE_BYTES;
    const int koff = kt * kBK;
#pragma unroll
    for (int i = 0; i < BM / 8 / NW; ++i) glds16(a_src[i] + koff, base + (i * NW + wave) * 8 * kRowBytes);
#pragma unroll
    for (int i = 0; i < BN / 8 / NW; ++i)
      glds16(b_src[i] + koff, base + A_BYTES + (i * NW + wave) * 8 * kRowBytes);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int arow0 = wm * (BM / WM), brow0 = wn * (BN / WN);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fchunk = lane >> 4;
  // RowLn / ResLn: the rows' partials, loaded before the K loop
  constexpr bool kPart = EPI & (kEpiRowLn | kEpiResLn);
  float2 pv[kPart ? TM : 1][kPartPerLane];
  const int pslots = (EPI & kEpiRowLn) ? K / 32 : N / 32;
  if constexpr (kPart) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
      part_prefetch(pv[i], (EPI & kEpiRowLn) ? ln.in_part : ln.res_part, pslots, M, m0 + arow0 + i * 16 + frow, fchunk);
  }
  float ssq[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) ssq[i] = 0.f;
  auto compute = [&](int buf) {
    const char* base = lds + buf * STAGE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = arow0 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
        if constexpr (EPI & kEpiRowRms) ssq[i] = sumsq_bf16x8(af[i], ssq[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = brow0 + j * 16 + frow;
        bfg[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = K / kBK;
  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    compute(cur);
    wait_vmcnt0();
    __syncthreads();
  }

  if constexpr (SPLIT) {
    const size_t slab = (size_t)M * N;
    float* mine = ws + blockIdx.y * slab;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + arow0 + i * 16 + frow;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + brow0 + j * 16 + fchunk * 4;
        if (m < M && n < N) *reinterpret_cast<f32x4*>(mine + (size_t)m * N + n) = acc[i][j];
      }
    }
    return;
  }

  // ---- epilogue: lane owns C[m][n..n+3] for each (i, j) fragment ----
  const int kv_pos = (EPI & kEpiKvScatter) ? max(*kvo.step, 0) : 0;
  float rstd[TM], rmu[TM];
  float2 rfs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    rstd[i] = (EPI & kEpiRowRms) ? __builtin_amdgcn_rsqf(lane_rows_sum(ssq[i]) * (1.f / K) + rms_eps) : 1.f;
    rmu[i] = 0.f;
    rfs[i] = float2{1.f, 0.f};
    if constexpr (EPI & kEpiRowLn) {
      const float2 st = part_ln(pv[i], pslots, fchunk, rms_eps);
      rstd[i] = st.x;
      rmu[i] = st.y;
    }
    if constexpr (EPI & kEpiResLn) rfs[i] = part_ln(pv[i], pslots, fchunk, rms_eps);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + arow0 + i * 16 + frow;
    if (m >= M) continue;
    const float2 rf = rfs[i];
    float ps[(TN + 1) / 2], pss[(TN + 1) / 2];  // RowStats: this lane's share of each 32-column slab
#pragma unroll
    for (int h = 0; h < (TN + 1) / 2; ++h) ps[h] = pss[h] = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + brow0 + j * 16 + fchunk * 4;
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI & kEpiRowRms) v *= rstd[i];
      if constexpr (EPI & kEpiRowLn) {
        const f32x4 cs = *reinterpret_cast<const f32x4*>(ln.colsum + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(v[e], rstd[i], -rmu[i] * cs[e]);
      }
      if constexpr (EPI & kEpiBias) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n);
        v += b;
      }
      if constexpr (EPI & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_poly1(v[e]);
      }
      if constexpr (EPI & kEpiTanh) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
      }
      if constexpr (EPI & kEpiRelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (EPI & kEpiResidual) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n);
        if constexpr (EPI & kEpiResLn) {
          const f32x4 g = *reinterpret_cast<const f32x4*>(ln.gamma + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaf(fmaf(bf2f(r[e]), rf.x, -rf.y), g[e], v[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(r[e]);
        }
      }
      if constexpr (EPI & kEpiOutF32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = v;
      } else {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        if (EPI & kEpiKvScatter) {
          // the tile is all Q or all K|V (host: kv_col0 % 128 == 0)
          // a step past the cache (caller bug) drops the K|V write instead of writing out of bounds
          if (n < kvo.col0)
            *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
          else if (kv_pos < kvo.T)
            *reinterpret_cast<bf16x4*>(kvo.cache + ((size_t)m * kvo.T + kv_pos) * kvo.ld + (n - kvo.col0)) = o;
        } else {
          *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
        }
        if constexpr (EPI & kEpiRowStats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float f = bf2f(o[e]);
            ps[j / 2] += f;
            pss[j / 2] = fmaf(f, f, pss[j / 2]);
          }
        }
      }
    }
    if constexpr (EPI & kEpiRowStats) {
#pragma unroll
      for (int h = 0; h < (TN + 1) / 2; ++h) {
        const float S = lane_rows_sum(ps[h]), Q = lane_rows_sum(pss[h]);
        const int col = n0 + brow0 + h * 32;
        if (fchunk == 0 && col < N) *reinterpret_cast<float2*>(ln.part_out + 2 * ((size_t)(col / 32) * M + m)) = float2{S, Q};
      }
    }
  }
}

// ============================================================================
// 256x256 tile, 8 waves, FULL-LINE staging (the retired "256b" schedule, git history;
// docs/PERF_NOTES.md). Its staging constants (g2) are shared by the kernels below.
//
// The ablation of the ring kernel showed the LDS-DMA instructions themselves
// costing ~40 % of the MFMA rate; its k-half chunks had 64-byte rows, so every
// 1 KiB DMA instruction touched 16 half-used 128-byte lines. Here a K-tile
// (BK = 64) is split by ROWS into four 16 KiB chunks [A rows 0-127 | A rows
// 128-255 | B rows 0-127 | B rows 128-255] of 128-byte rows: one DMA
// instruction = 8 full lines. Row swizzle c ^ ((r>>1)&7) (conflict-free for the
// ds_read_b128 lane groups, see gemm_bf16 128x128 kernel). Wave (wm, wn) reads
// only chunk A[wm] and chunk B[wn>>1].
// Schedule per K-tile t (buffer t&1, two 64 KiB buffers):
//   SYNC(t): vmcnt(0) + barrier  -> tile t landed, every wave done with t-1
//   issue tile t+1 (8 DMA/wave) into the other buffer, interleaved into R1
//   R1..R4: 4 MFMA clusters of 16 with the next cluster's fragment reads
//           interleaved (k32 step x row half of the wave tile)
// ============================================================================
namespace g2 {
constexpr int kChunk = 16384;    // 128 rows x 128 B
constexpr int kTile = 4 * kChunk;
__device__ __forceinline__ int sw(int r, int c) { return c ^ ((r >> 1) & 7); }
}  // namespace g2


// ============================================================================
// 256x256 tile, 8 waves, PING-PONG schedule (kernel "256p").
//
// Two wave groups (wave row wm = 0 / 1; every SIMD hosts one wave of each) run
// staggered by one barrier: between two consecutive s_barriers one group
// issues its 16 MFMAs while the other issues its LDS fragment reads and LDS-DMA
// staging, so the SIMD's matrix core never waits for the issue of memory ops
// (the cost the 256b ablation exposed). Each K-tile is 4 phases (quadrants of
// the wave's 128x64 output):
//   p0: read A-top, B-left  -> MFMA (top, left)      stage quarter 0 of t+1
//   p1: read B-right        -> MFMA (top, right)     stage quarter 1 of t+1
//   p2: read A-bottom       -> MFMA (bottom, right)  stage quarter 2 of t+1
//   p3: (registers only)    -> MFMA (bottom, left)   stage quarter 3 of t+1
// Quarters are ROW sets of the 128-B-row images in the order they are first
// read: Q0 = A-top rows {0-63,128-191}, Q1 = B-left rows {32-row blocks 0,2,4,6},
// Q2 = B-right rows {blocks 1,3,5,7}, Q3 = A-bottom rows {64-127,192-255}.
// Phase program: R (ds_read) ; G (2 DMA/wave) ; vmcnt(4) ; s_barrier ;
// lgkmcnt(0) ; setprio(1) MFMA x16 setprio(0) ; s_barrier.
// Hazards (checked for both stagger orders): with vmcnt(4) before the first
// barrier a quarter issued at phase r is visible to every reader at phase
// >= r+3 (each is issued >= 3 phases before its first read), and a restage at
// phase r is safe after reads at phase <= r-2 (every restage is >= 2 phases
// after the quarter's last read in the previous K-tile).
// ============================================================================
// Epilogue of the 256x256 kernels: wave (wm, wn) owns C rows m0+wm*128 .. +128,
// columns n0+wn*64 .. +64; acc[i][j] = the 16x16 fragment (row block i, col block j).
// FULL: every row of the tile is < M (no per-store bounds test; the persistent
// kernel also relies on every wave issuing exactly 16 stores).
// ABL (timing-only ablations, results WRONG): 1 = all VALU work, no stores;
// 2 = stores of the raw accumulator bits, no VALU work.
// lds_bias: when non-null, the tile's 256 bias values staged in LDS (read
// there instead of global memory: no exposed load round trip in the tail).
template <int EPI, bool FULL = false, int ABL = 0, bool NT = false>
__device__ __forceinline__ void epilogue_256(const f32x4 (&acc)[8][4], int m0, int n0, int wm, int wn, int lane,
                                             bf16* __restrict__ C, int ldc, const float* __restrict__ bias,
                                             const bf16* __restrict__ R, int ldr, int M,
                                             const float* lds_bias = nullptr) {
  const int fr = lane & 15, fc = lane >> 4;
  // ---- epilogue, widened (guide T21 for the 16x16 layout). Lane (fr, fc) owns
  // rows (2p)*16+fr and (2p+1)*16+fr, columns j*16+fc*4..+3 of fragments
  // (2p, j), (2p+1, j). Bias, activation and residual are applied there in
  // fp32, both fragments are packed to bf16 pairs, and ONE v_permlane16_swap
  // per dword pair leaves every lane 8 consecutive bf16 columns of one row
  // (even fc: row 2p, odd fc: row 2p+1; probed: tools/probes/permlane_probe.hip)
  // -> one 16-B store. Swapping packed bf16 pairs instead of fp32 values halves
  // the swaps and needs no operand laundering (distinct scalars, "+v").
  const int hi = fc & 1, cq = (fc >> 1) * 8;  // stored row parity, stored column half
  // residual: loaded as 16-B rows in the STORED layout (one row pair ahead of
  // its use: 2 x 16 VGPRs live, the persistent kernel keeps its staging state
  // through the epilogue), then taken to the fragment layout by the same
  // (involutive) dword swap the outputs go through
  u32x4 res[4][4];
  auto load_res = [&](int pp) {
    if constexpr (EPI & kEpiResidual) {
      const int m = min(m0 + wm * 128 + (2 * pp + hi) * 16 + fr, M - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        res[pp][j] = *reinterpret_cast<const u32x4*>(R + (size_t)m * ldr + n0 + wn * 64 + j * 16 + cq);
    }
  };
  load_res(0);
  f32x4 b4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = wn * 64 + j * 16 + fc * 4;
    if constexpr (EPI & kEpiBias) {
      b4[j] = lds_bias ? *reinterpret_cast<const f32x4*>(lds_bias + c) : *reinterpret_cast<const f32x4*>(bias + n0 + c);
    } else {
      b4[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const bool full_tile = m0 + 256 <= M;  // uniform: no per-store bounds branch
  // row pair outer, column fragment inner: the 4 consecutive 16-B stores of a
  // lane cover its row's whole 128-B line segment (write combining in L2)
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) {
    const int m = m0 + wm * 128 + (2 * pp + hi) * 16 + fr;
    if (pp + 1 < 4) load_res(pp + 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + cq;
      if constexpr (ABL == 2) {
        // both fragments feed the store (else half the MFMAs are dead code)
        const u32x4 a = __builtin_bit_cast(u32x4, acc[2 * pp][j]) ^ __builtin_bit_cast(u32x4, acc[2 * pp + 1][j]);
        *reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n) = a;
        continue;
      }
      float v[8];  // [0..3] row 2p, [4..7] row 2p+1, columns fc*4..+3
      const f32x4 lo4 = acc[2 * pp][j] + b4[j], hi4 = acc[2 * pp + 1][j] + b4[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = lo4[e], v[4 + e] = hi4[e];
      if constexpr (EPI & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_poly1(v[e]);
      }
      if constexpr (EPI & kEpiTanh) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = tanhf(v[e]);
      }
      if constexpr (EPI & kEpiRelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (EPI & kEpiResidual) {
        unsigned r0 = res[pp][j][0], r1 = res[pp][j][1], r2 = res[pp][j][2], r3 = res[pp][j][3];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
        const unsigned rr[4] = {r0, r1, r2, r3};  // row 2p cols 0-3 | row 2p+1 cols 0-3
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __builtin_bit_cast(float, rr[e] << 16);
          v[2 * e + 1] += __builtin_bit_cast(float, rr[e] & 0xffff0000u);
        }
      }
      unsigned l0 = pack_bf16x2(v[0], v[1]), l1 = pack_bf16x2(v[2], v[3]);
      unsigned h0 = pack_bf16x2(v[4], v[5]), h1 = pack_bf16x2(v[6], v[7]);
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                   : "+v"(l0), "+v"(l1), "+v"(h0), "+v"(h1));
      if constexpr (ABL == 1) {
        asm volatile("" ::"v"(l0), "v"(l1), "v"(h0), "v"(h1));
        continue;
      }
      if (FULL || full_tile || m < M) {
        u32x4* cp = reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n);
        if constexpr (NT) __builtin_nontemporal_store(u32x4{l0, l1, h0, h1}, cp);
        else *cp = u32x4{l0, l1, h0, h1};
      }
    }
  }
}

// DBG (timing-only ablation, results WRONG): 1 = skip the epilogue (acc kept live)
template <int EPI, int DBG = 0>
__global__ __launch_bounds__(512, 1) void gemm256p_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K) {
  using namespace g2;
  constexpr int kImg = 256 * 128;  // one operand image (256 rows x 128 B)
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kImg];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = N / 256, ntm = (M + 255) / 256;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;
  const int wm = wave >> 2, wn = wave & 3;

  // ---- staging: quarter q, instruction i of this wave covers quarter-local
  // rows ql = (i*8 + wave)*8 + (lane>>3), 16-B chunk (lane&7) of each row ----
  const int spos = lane & 7;
  const bf16* src[4][2];
  int dst[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ql0 = (i * 8 + wave) * 8;  // first quarter-local row of this instruction
      const int ql = ql0 + (lane >> 3);
      int r, r0;  // image row of this lane / of the instruction's first row
      if (q == 0 || q == 3) {
        const int off = q == 3 ? 64 : 0;
        r = (ql & 63) + (ql >> 6) * 128 + off;
        r0 = (ql0 & 63) + (ql0 >> 6) * 128 + off;
      } else {
        const int off = q == 2 ? 32 : 0;
        r = (ql & 31) + (ql >> 5) * 64 + off;
        r0 = (ql0 & 31) + (ql0 >> 5) * 64 + off;
      }
      const bool is_a = (q == 0 || q == 3);
      src[q][i] = is_a ? A + (size_t)min(m0 + r, M - 1) * lda + sw(r, spos) * 8
                       : Bt + (size_t)(n0 + r) * ldb + sw(r, spos) * 8;
      dst[q][i] = (is_a ? 0 : kImg) + r0 * 128;
    }
  auto stage = [&](int q, int kt) {
    char* base = lds + (kt & 1) * 2 * kImg;
    const int koff = kt * 64;
    glds16(src[q][0] + koff, base + dst[q][0]);
    glds16(src[q][1] + koff, base + dst[q][1]);
  };

  const int fr = lane & 15, fc = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][4], bl[2][2], br[2][2];  // [kstep][frag]
  auto read_a = [&](int buf, int qm) {
    const char* img = lds + buf * 2 * kImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 128 + qm * 64 + i * 16 + fr;
        af[ks][i] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
      }
  };
  auto read_b = [&](bf16x8 (&f)[2][2], int buf, int qn) {
    const char* img = lds + buf * 2 * kImg + kImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 64 + qn * 32 + j * 16 + fr;
        f[ks][j] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
      }
  };
  auto mma = [&](const bf16x8 (&bf)[2][2], int qm, int qn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
  };

  const int nk = K / 64;
  // prologue: K-tile 0 fully staged and visible
#pragma unroll
  for (int q = 0; q < 4; ++q) stage(q, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

#define ATPU_PP_SYNC_MMA(BF, QM, QN)                         \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_setprio(1);                            \
  mma(BF, QM, QN);                                          \
  __builtin_amdgcn_s_setprio(0);                            \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  __builtin_amdgcn_sched_barrier(0)

  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const bool more = t + 1 < nk;
    // p0
    read_a(buf, 0);
    read_b(bl, buf, 0);
    if (more) {
      stage(0, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    ATPU_PP_SYNC_MMA(bl, 0, 0);
    // p1
    read_b(br, buf, 1);
    if (more) {
      stage(1, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    ATPU_PP_SYNC_MMA(br, 0, 1);
    // p2
    read_a(buf, 1);
    if (more) {
      stage(2, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    ATPU_PP_SYNC_MMA(br, 1, 1);
    // p3
    if (more) {
      stage(3, t + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    ATPU_PP_SYNC_MMA(bl, 1, 0);
  }
#undef ATPU_PP_SYNC_MMA
  if (wm == 0) __builtin_amdgcn_s_barrier();  // close the stagger (equal barrier counts)
  if constexpr (DBG & 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  epilogue_256<EPI>(acc, m0, n0, wm, wn, lane, C, ldc, bias, R, ldr, M);
}

void launch_256p(const GemmArgs& g, hipStream_t s) {
  const int nb = ((g.M + 255) / 256) * (g.N / 256);
#define ATPU_G256P(E)                                                                                     \
  case E:                                                                                                 \
    hipLaunchKernelGGL((gemm256p_kernel<E>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, g.ldc, \
                       g.bias, g.R, g.ldr, g.M, g.N, g.K);                                                \
    break;
  switch (g.epi) {
    ATPU_G256P(0)
    ATPU_G256P(kEpiBias)
    ATPU_G256P(kEpiBias | kEpiGelu)
    ATPU_G256P(kEpiBias | kEpiTanh)
    ATPU_G256P(kEpiBias | kEpiResidual)
    ATPU_G256P(kEpiResidual)
    ATPU_G256P(kEpiGelu)
    ATPU_G256P(kEpiRelu)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_G256P
}



// 16-B global load the compiler does not track: its waitcnt pass treats the
// counter as out of order once loads, stores and LDS-DMA are all pending and
// waits vmcnt(0) at the first use; the line epilogue counts its own waits
__device__ __forceinline__ u32x4 load16_untracked(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// Full-line epilogue of the persistent kernel ("line"): the wave's 128 x 64
// output (one 128-B line per row) goes out as 16 stores of 8 rows x 128 B
// FULL lines, after an LDS transpose through a private 2 KiB scratch per wave
// (16 rows x 128 B, 16-B chunks XOR-swizzled by row & 7). Per 16-row block i:
//   residual: 2 x 16-B full-line loads (all 8 blocks issued up front) -> LDS ->
//             8-B reads in the fragment layout -> added in fp32
//   output:   acc + bias (+act) (+res) -> bf16 -> 4 x ds_write_b64 in the
//             fragment layout -> 2 x ds_read_b128 in line layout -> 2 stores
// The fragment-layout 8-B accesses are 2-way bank conflicted (rows r, r+8
// share a swizzle), the line-layout ones conflict-free. DS ops of one wave
// execute in order, so the scratch needs no barrier, only lgkmcnt waits.
// VMEM accounting of the line epilogue (per wave). s_waitcnt vmcnt(N) waits
// until all but the wave's N youngest vector-memory ops are done; on gfx950
// loads, stores and LDS-DMA of the global/buffer kinds all count on vmcnt and
// retire IN ISSUE ORDER (MI355X_MICROARCH.md, s_waitcnt paragraph; CDNA4 ISA
// "Data dependency resolution": only flat_* returns out of order, and the
// epilogue issues none). Each 16-row block i has kLineLoadsPerBlock residual
// loads and kLineStoresPerBlock output stores (distinct rows: never merged).
// Younger than block i's loads when it waits: the loads of blocks i+1..7 and
// the stores of blocks 0..i-1, i.e. L*(7-i) + S*i, which is the same for
// every i only because L == S. kLineResWait is that count.
constexpr int kLineBlocks = 8;
constexpr int kLineLoadsPerBlock = 2;
constexpr int kLineStoresPerBlock = 2;
constexpr int kLineResWait = kLineLoadsPerBlock * (kLineBlocks - 1);
static_assert(kLineLoadsPerBlock == kLineStoresPerBlock,
              "vmcnt(kLineResWait) is exact for every block only when each block issues as many stores as loads");
static_assert(kLineResWait == 14, "the counted residual wait assumes 8 blocks x 2 loads");
static_assert(kLineResWait < 64, "vmcnt field is 6 bits on gfx950");

// Sum of x over the 4 lanes l, l^16, l^32, l^48 (one 16-lane row each), in registers:
// v_permlane16_swap of two copies leaves row pairs (0,1) and (2,3) exchanged across the
// copies, so their sum is x + x^16; v_permlane32_swap does the same for the halves.
// The copies are made inside the asm into early-clobber outputs: as plain copies of one
// value hipcc allocated both operands to ONE register (docs/PERF_NOTES.md, permlane).
// Same bits on all 4 lanes ((a+b)+(c+d) in either operand order). Replaces 2 LDS
// round trips (ds_bpermute) per value on the epilogue's dependency chain.
__device__ __forceinline__ float sum_lane_rows(float x) { return lane_rows_sum(x); }

// LayerNorm folding state of the line epilogue, all in the kernel's LDS array:
//   fin[256][2]  (rstd, rstd*mu) of the tile's rows: of A (InNorm) or of R (ResNorm)
//   col[256]     colsum of the folded weights (InNorm) or the residual's gamma (ResNorm)
//   st[4][256][2] per-wave-column partial (sum, sumsq) of the output rows (StatsOut),
//                slot wn written by wave (wm, wn) for its 128 rows; summed in slot
//                order when flushed (deterministic, no atomics)
struct LnLds {
  const float* fin = nullptr;
  const float* col = nullptr;
  float* st = nullptr;
};

// IN_ACC (InNorm): the caller started the accumulators at -mu*colsum (else the
// epilogue applies -rstd*mu*colsum itself, from LDS colsum)
// NOST (timing-only ablation, results WRONG): the output values are computed but not stored
template <int EPI, bool NT, bool IN_ACC = true, int GM = 0, bool NOST = false>
__device__ __forceinline__ void epilogue_256_line(const f32x4 (&acc)[8][4], int m0, int n0, int wm, int wn, int lane,
                                                  bf16* __restrict__ C, int ldc, const bf16* __restrict__ R, int ldr,
                                                  const float* lds_bias, char* scratch,
                                                  const u32x4 (&pre)[2][2], LnLds ln = {}) {
  constexpr int kResWait = kLineResWait;
  constexpr bool kIn = EPI & kEpiInNorm, kRes = EPI & kEpiResNorm, kSt = EPI & kEpiStatsOut;
  const int fr = lane & 15, fc = lane >> 4;
  // per-column LDS vectors (bias, colsum, gamma) at this lane's 4 columns of fragment j
  auto col4 = [&](const float* v, int j) {
    return *reinterpret_cast<const f32x4*>(v + wn * 64 + j * 16 + fc * 4);
  };
  f32x4 b4[4], g4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    b4[j] = (EPI & kEpiBias) ? col4(lds_bias, j) : f32x4{0.f, 0.f, 0.f, 0.f};
    // ResNorm: gamma (its caller adds the bias in the accumulator init); InNorm without
    // IN_ACC: colsum
    if constexpr (kRes || (kIn && !IN_ACC)) g4[j] = col4(ln.col, j);
  }
  // (rstd, rstd*mu) of the lane's row in block i, read one block ahead: the residual
  // wait (asm with a memory clobber) would otherwise pin each read behind it
  auto row_fin = [&](int i) {
    return (kIn || kRes) ? *reinterpret_cast<const f32x2*>(ln.fin + (wm * 128 + i * 16 + fr) * 2) : f32x2{1.f, 0.f};
  };
  f32x2 rsm_next = row_fin(0);
  // line layout: lane -> row lr (+8 for the second half), 16-B chunk lc
  const int lr = lane >> 3, lc = lane & 7;
  const int line_off0 = lr * 128 + ((lc ^ (lr & 7)) << 4);
  const int line_off1 = (lr + 8) * 128 + ((lc ^ ((lr + 8) & 7)) << 4);
  // fragment layout: row fr, bytes j*32 + fc*8 (16-B chunk j*2 + fc/2, half fc&1)
  auto frag_off = [&](int j) { return fr * 128 + (((j * 2 + (fc >> 1)) ^ (fr & 7)) << 4) + (fc & 1) * 8; };
  const size_t row0 = (size_t)(m0 + wm * 128);
  const int col = n0 + wn * 64 + lc * 8;
  // all 16 residual loads go out at once (64 VGPRs: the operand fragments are
  // dead here). Loading one 16-row block ahead left every other block waiting
  // a full memory latency (~4 latencies per tile: o-proj ran 38 % over its main
  // loop); now only the first block waits.
  // blocks 0-1 were issued by the caller during the last MMA phase (pre)
  u32x4 res[8][2];
  if constexpr (EPI & kEpiResidual) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      res[i][0] = pre[i][0];
      res[i][1] = pre[i][1];
    }
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      const bf16* rp = R + (row0 + i * 16 + lr) * ldr + col;
      res[i][0] = load16_untracked(rp);
      res[i][1] = load16_untracked(rp + 8 * (size_t)ldr);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float v[4][4];
    const int lrow = wm * 128 + i * 16 + fr;  // tile-local row of this lane's fragment row
    const f32x2 rsm = rsm_next;               // (rstd, rstd*mu) of that row (InNorm / ResNorm)
    if (i + 1 < 8) rsm_next = row_fin(i + 1);
    // the LN math runs on value PAIRS (v_pk_fma_f32 with the row scalars broadcast):
    // written per element, hipcc packed it with a v_mov per operand pair
    const f32x2 rs2 = f32x2{rsm[0], rsm[0]}, nrm2 = f32x2{-rsm[1], -rsm[1]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 t;
      if constexpr (kIn) {
        // LN(a) . W = rstd * (a . (gamma o W) - mu * colsum(gamma o W)) + beta . W (in the bias);
        // IN_ACC: the caller started acc at -mu * colsum
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x2 c2 = f32x2{b4[j][2 * h], b4[j][2 * h + 1]};
          if constexpr (!IN_ACC) c2 = __builtin_elementwise_fma(nrm2, f32x2{g4[j][2 * h], g4[j][2 * h + 1]}, c2);
          const f32x2 o = __builtin_elementwise_fma(f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]}, rs2, c2);
          t[2 * h] = o[0];
          t[2 * h + 1] = o[1];
        }
      } else {
        t = acc[i][j] + b4[j];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = t[e];
    }
    if constexpr (EPI & kEpiGelu) gelu_poly16(*reinterpret_cast<float(*)[16]>(&v[0][0]));
    if constexpr (EPI & kEpiTanh) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = tanhf(v[j][e]);
    }
    if constexpr (EPI & kEpiRelu) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = fmaxf(v[j][e], 0.f);
    }
    if constexpr (EPI & kEpiResidual) {
      // block i's two loads have landed once at most 14 younger VMEM ops are
      // pending: blocks 0-1 (issued in the last MMA phase) are followed by the
      // other pre load pair and 12 loads; block i >= 2 by 2 (7 - i) loads; and
      // every earlier block added its 2 stores -> 14 for every i
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(res[i][0]), "+v"(res[i][1]) : "n"(kResWait) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      *reinterpret_cast<u32x4*>(scratch + line_off0) = res[i][0];
      *reinterpret_cast<u32x4*>(scratch + line_off1) = res[i][1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(scratch + frag_off(j));
        if constexpr (kRes) {
          // residual = LN(r) = (r*rstd - rstd*mu) * gamma (+ beta, folded into the bias)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x2 t2 = __builtin_elementwise_fma(f32x2{bf2f(r[2 * h]), bf2f(r[2 * h + 1])}, rs2, nrm2);
            const f32x2 o = __builtin_elementwise_fma(t2, f32x2{g4[j][2 * h], g4[j][2 * h + 1]},
                                                      f32x2{v[j][2 * h], v[j][2 * h + 1]});
            v[j][2 * h] = o[0];
            v[j][2 * h + 1] = o[1];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[j][e] += bf2f(r[e]);
        }
      }
    }
    if constexpr (kSt) {
      // row partials over this wave's 64 columns: 16 values per lane, then the 4
      // lanes sharing the row (fc = 0..3: lanes fr, fr+16, fr+32, fr+48), fixed order
      f32x2 s1 = f32x2{0.f, 0.f}, s2 = f32x2{0.f, 0.f};  // over value pairs: packed add / fma
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 p2 = f32x2{v[j][2 * h], v[j][2 * h + 1]};
          s1 += p2;
          s2 = __builtin_elementwise_fma(p2, p2, s2);
        }
      const f32x2 s = f32x2{sum_lane_rows(s1[0] + s1[1]), sum_lane_rows(s2[0] + s2[1])};
      if (fc == 0) *reinterpret_cast<f32x2*>(ln.st + (wn * 256 + lrow) * 2) = s;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned p0 = pack_bf16x2(v[j][0], v[j][1]), p1 = pack_bf16x2(v[j][2], v[j][3]);
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(scratch + frag_off(j)) = u32x2{p0, p1};
    }
    const u32x4 o0 = *reinterpret_cast<const u32x4*>(scratch + line_off0);
    const u32x4 o1 = *reinterpret_cast<const u32x4*>(scratch + line_off1);
    u32x4* cp = reinterpret_cast<u32x4*>(C + (row0 + i * 16 + lr) * ldc + col);
    u32x4* cp1 = reinterpret_cast<u32x4*>(C + (row0 + i * 16 + lr + 8) * ldc + col);
    if constexpr (NOST) {
      asm volatile("" ::"v"(o0), "v"(o1), "v"(cp), "v"(cp1));
    } else if constexpr (NT) {
      __builtin_nontemporal_store(o0, cp);
      __builtin_nontemporal_store(o1, cp1);
    } else {
      *cp = o0;
      *cp1 = o1;
    }
  }
}

// ============================================================================
// 256x256 PERSISTENT ping-pong kernel ("256s"): the 256p schedule with one
// workgroup per CU walking its tiles, and the LDS-DMA stream running on from
// the last K-tile of a tile into K-tile 0 of the next. What that buys over one
// launch per tile (hipBLASLt's stream-K kernels do the same at these shapes):
//  * K-tile 0 of tile i+1 is staged during the last K-tile of tile i and lands
//    while tile i's epilogue runs: no exposed prologue per tile;
//  * the epilogue's 16 stores per wave stay in flight into the first phases
//    of tile i+1: the waits of its phases 0-1 allow them (vmcnt counts every
//    VMEM op of the wave in issue order, and K-tile 0 was issued before them);
//  * no workgroup launch / drain per tile.
// Tile walk: virtual block v = blockIdx.x + it * gridDim.x (gridDim.x % 8 == 0
// keeps v % 8 = the XCD), tile = xcd_remap(v, tiles): each XCD walks a
// contiguous tile range, N-fastest, exactly as the one-launch-per-tile grid.
// The phase/quarter program and its hazard argument are those of 256p; the
// epilogue has no barrier, so the two wave groups stay staggered across tiles.
// ============================================================================
// Kernel arguments of the LayerNorm folding epilogues (GemmArgs fields of the same names).
struct LnFold {
  const float* in_fin;
  const float* colsum;
  const float* res_fin;
  const float* gamma;
  float* part_out;
};

// DBG (timing-only ablation, results WRONG): 1 = skip the epilogue (acc kept live)
//
// LayerNorm folding (EPI & (kEpiInNorm | kEpiResNorm | kEpiStatsOut), LINE only, K >= 256):
//  * K-tile 1, phase 0: the tile's per-row / per-column LN data is staged by 4-byte
//    LDS-DMA (as the bias is at K-tile 0): the finalized (rstd, rstd*mu) of the 256
//    A rows (InNorm) or R rows (ResNorm), and colsum (InNorm) or gamma (ResNorm) of
//    columns n0..+256. Every wave issues the same op count; the later counted waits
//    only get stricter. Single buffers: by K-tile 1 both (staggered) wave groups
//    have left the previous tile's epilogue. K-tiles 0-1 are peeled, so the K loop
//    itself has no branch.
//  * StatsOut: the epilogue writes per-wave row partials to LDS; K-tile 1 of the
//    NEXT tile (or a barrier after the loop, for the last tile) sums the 4 column
//    slots in order and stores the tile's 256 (sum, sumsq) pairs. The statistics are
//    finalized between the kernels (ln_stats_finalize, norm_embed.hip).
template <int EPI, int DBG = 0, bool NT = false, bool LINE = false>
__global__ __launch_bounds__(512, 1) void gemm256s_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K, LnFold lf) {
  using namespace g2;
  constexpr int kImg = 256 * 128;
  // VMEM ops per wave the epilogue leaves in flight: its 16-B stores (every residual load
  // has been waited for by then). The relaxed phase-0/1 waits below add this to their count.
  constexpr int kEpiOps = kLineBlocks * kLineStoresPerBlock;
  static_assert(kEpiOps == 16, "epilogue store count changed: re-derive the relaxed waits");
  constexpr int kBiasOff = 2 * 2 * kImg;  // [2 tiles][256] fp32 bias after the operand buffers
  // ONE __shared__ array: a second LDS object makes hipcc drain vmcnt before ds_reads
  constexpr int kEpiOff = kBiasOff + 2 * 256 * 4;  // LINE epilogue: 2 KiB scratch per wave
  constexpr bool kIn = EPI & kEpiInNorm, kRes = EPI & kEpiResNorm, kSt = EPI & kEpiStatsOut;
  static_assert(!(kIn || kRes || kSt) || LINE, "LayerNorm folding needs the full-line epilogue");
  static_assert(!(kIn && (kRes || kSt)), "InNorm and ResNorm/StatsOut do not share one kernel (LDS budget)");
  constexpr int kXOff = kEpiOff + (LINE ? 8 * 2048 : 0);
  constexpr int kFinOff = kXOff;                                    // [2 tiles (InNorm)][256][2] (rstd, rstd*mu)
  constexpr int kColOff = kFinOff + (kIn ? 4096 : kRes ? 2048 : 0); // [256] colsum | gamma
  constexpr int kStOff = kColOff + ((kIn || kRes) ? 1024 : 0);      // StatsOut: [4][256][2]
  constexpr int kLdsBytes = kStOff + (kSt ? 4 * 2048 : 0);
  static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = N / 256, ntm = (M + 255) / 256, ntiles = ntm * ntn;
  const int G = gridDim.x;
  const int wm = wave >> 2, wn = wave & 3;
  int v = blockIdx.x;
  if (v >= ntiles) return;

  // staging rows of quarter q / instruction i (same map as 256p); the lane's
  // row is recomputed per tile (registers are the budget here), the LDS
  // destination is wave-uniform (scalar)
  const int spos = lane & 7;
  auto qrow = [&](int q, int ql) {
    return (q == 0 || q == 3) ? (ql & 63) + (ql >> 6) * 128 + (q == 3 ? 64 : 0)
                              : (ql & 31) + (ql >> 5) * 64 + (q == 2 ? 32 : 0);
  };
  int dst[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) dst[q][i] = (q == 0 || q == 3 ? 0 : kImg) + qrow(q, (i * 8 + wave) * 8) * 128;
  // lane ids are made opaque per use (recomputed by mbcnt, never hoisted): with the
  // LayerNorm-folding epilogues the per-lane staging rows kept live across the tile
  // loop spilled, and a scratch reload is a VMEM load the waitcnt pass drains the
  // LDS-DMA stream for (vmcnt(0) in the last K-tile)
  auto opaque_lane = [] {
    int l = __lane_id();
    asm volatile("" : "+v"(l));
    return l;
  };
  // staging sources: 64-bit per-lane pointers, or (LN-folding variants, whose
  // epilogue is the register peak) 32-bit byte offsets from the uniform A / Bt
  // base, which the DMA takes in its saddr form: 8 VGPRs instead of 16 live over
  // the whole tile loop (host: A and Bt each < 4 GiB)
  constexpr bool kFold = kIn || kRes || kSt;
  // epilogues of the two wave groups side by side (see the end of the K loop);
  // (bench.py A/B, same box: 47.13k -> 48.17k rows/s); ATPU_GEMM_SYNC_EPI=0 builds the staggered form
  constexpr bool kSyncEpi = ATPU_GEMM_SYNC_EPI && !(DBG & 128);
  // InNorm: statistics and colsum staged at K-tile 1 (peeled), the epilogue applies
  // rstd*acc - rstd*mu*colsum + bias (two packed FMAs per value pair). DBG & 16 (A/B
  // variant, gemm_ablate(8)): statistics staged ahead of the tile and the accumulators
  // started at -mu*colsum, one FMA in the epilogue; measured slower (tools/bench_fold.py:
  // qkv +9.4 vs +4.7 us, ffn1 +13 vs +6 us over the plain kernel), the extra LDS reads
  // sit on the tile-start path
  constexpr bool kInAcc = kIn && (DBG & 16);
  constexpr bool kPeel = kRes || kSt || (kIn && !kInAcc);
  // ResNorm / StatsOut variants start each tile's accumulators at the bias (read from
  // LDS, where the previous tile's last K-tile staged it) instead of adding it in the
  // epilogue: 16 fewer VGPRs and one op fewer per value pair on the epilogue chain
  constexpr bool kBiasAcc = (kRes || kSt) && (EPI & kEpiBias);
  const bf16* src[4][2];
  uint32_t soff[4][2];
  auto set_src = [&](int tm0, int tn0) {
    const int ln = kFold ? opaque_lane() : lane;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = qrow(q, (i * 8 + wave) * 8 + (ln >> 3));
        const size_t e = (q == 0 || q == 3) ? (size_t)min(tm0 + r, M - 1) * lda + sw(r, ln & 7) * 8
                                            : (size_t)(tn0 + r) * ldb + sw(r, ln & 7) * 8;
        if constexpr (kFold) soff[q][i] = (uint32_t)(e * 2);
        else src[q][i] = ((q == 0 || q == 3) ? A : Bt) + e;
      }
  };
  auto stage = [&](int q, int kt, int buf) {
    char* base = lds + buf * 2 * kImg;
    const int koff = kt * 64;
    if constexpr (kFold) {
      const char* g = reinterpret_cast<const char*>((q == 0 || q == 3) ? A : Bt) + koff * 2;
      glds16(g + soff[q][0], base + dst[q][0]);
      glds16(g + soff[q][1], base + dst[q][1]);
    } else {
      glds16(src[q][0] + koff, base + dst[q][0]);
      glds16(src[q][1] + koff, base + dst[q][1]);
    }
  };

  const int fr = lane & 15, fc = lane >> 4;
  f32x4 acc[8][4];
  bf16x8 af[2][4], bl[2][2], br[2][2];
  auto read_a = [&](int buf, int qm) {
    const char* img = lds + buf * 2 * kImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 128 + qm * 64 + i * 16 + fr;
        af[ks][i] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
      }
  };
  auto read_b = [&](bf16x8 (&f)[2][2], int buf, int qn) {
    const char* img = lds + buf * 2 * kImg + kImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 64 + qn * 32 + j * 16 + fr;
        f[ks][j] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
      }
  };
  auto mma = [&](const bf16x8 (&bf)[2][2], int qm, int qn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
  };

  const int nk = K / 64;
  // ---- LayerNorm folding (see the kernel comment) ----
  // LN data staging: uniform base + 32-bit lane offset (saddr form, no 64-bit
  // per-lane address kept live)
  auto glds4 = [&](const float* ubase, char* ldst) {
    const uint32_t lo = (uint32_t)opaque_lane() * 4u;
    __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)(reinterpret_cast<const char*>(ubase) + lo),
                                     (ATPU_LDS_AS void*)ldst, 4, 0, 0);
  };
  auto ln_stage = [&](int tm0, int tn0) {  // ResNorm (and InNorm without kInAcc), at K-tile 1
    if constexpr (kRes || (kIn && !kInAcc)) {
      glds4((kRes ? lf.res_fin : lf.in_fin) + (size_t)tm0 * 2 + wave * 64, lds + kFinOff + wave * 256);
      glds4((kRes ? lf.gamma : lf.colsum) + tn0 + (wave & 3) * 64, lds + kColOff + (wave & 3) * 256);
    }
  };
  // InNorm: a tile's row statistics and colsum are staged ahead of the tile (prologue,
  // or the previous tile's last K-tile, like kBiasAcc's bias): the accumulators start
  // at -mu*colsum, so the epilogue is one packed FMA per value pair, rstd*acc + bias.
  // The statistics are double-buffered (the epilogue of the tile before reads its own).
  auto ln_stage_in = [&](int tm0, int tn0, int par) {
    if constexpr (kInAcc) {
      glds4(lf.in_fin + (size_t)tm0 * 2 + wave * 64, lds + kFinOff + par * 2048 + wave * 256);
      glds4(lf.colsum + tn0 + (wave & 3) * 64, lds + kColOff + (wave & 3) * 256);
    }
  };
  auto ln_flush = [&](int fm0, int fn0) {
    if constexpr (kSt) {
      const int l = opaque_lane();
      if (l < 32) {
        const int r = wave * 32 + l;
        f32x2 s = f32x2{0.f, 0.f};
#pragma unroll
        for (int w = 0; w < 4; ++w) s += *reinterpret_cast<const f32x2*>(lds + kStOff + (w * 256 + r) * 8);
        float* ub = lf.part_out + ((size_t)(fn0 >> 8) * M + fm0 + wave * 32) * 2;
        *reinterpret_cast<f32x2*>(reinterpret_cast<char*>(ub) + (uint32_t)l * 8u) = s;
      }
    }
  };
  int pm0 = 0, pn0 = 0;  // StatsOut: the tile whose row partials sit in LDS

  int tile = xcd_remap(v, ntiles);
  int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;
  set_src(m0, n0);
  if constexpr (kBiasAcc) glds4(bias + n0 + (wave & 3) * 64, lds + kBiasOff + (wave & 3) * 256);
  ln_stage_in(m0, n0, 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) stage(q, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

#define ATPU_PS_SYNC_MMA(BF, QM, QN)                         \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_setprio(1);                            \
  mma(BF, QM, QN);                                          \
  __builtin_amdgcn_s_setprio(0);                            \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  __builtin_amdgcn_sched_barrier(0)

  int buf = 0;        // LDS buffer of the current K-tile (global K-tile parity)
  int tile_par = 0;   // bias buffer of the current tile
  bool first = true;  // no epilogue stores in flight before the first tile
  for (;;) {
    if constexpr (kBiasAcc) {
      // this tile's bias landed before a barrier of the previous tile's last K-tile
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(lds + kBiasOff + (wn * 64 + j * 16 + fc * 4) * 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] = b;
      }
    } else if constexpr (kInAcc) {
      // acc = -mu * colsum: rstd * acc_final = rstd*(a.W') - rstd*mu*colsum(W').
      // LDS offsets from an opaque lane id (the hoisted lane-derived offsets spilled)
      const int ol = opaque_lane();
      f32x4 c4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        c4[j] = *reinterpret_cast<const f32x4*>(lds + kColOff + (wn * 64 + j * 16 + (ol >> 4) * 4) * 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x2 f = *reinterpret_cast<const f32x2*>(lds + kFinOff + tile_par * 2048 +
                                                        (wm * 128 + i * 16 + (ol & 15)) * 8);
        const float nmu = -f[1] * __builtin_amdgcn_rcpf(f[0]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = c4[j] * nmu;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int vn = v + G;
    const bool has_next = vn < ntiles;
    const int cm0 = m0, cn0 = n0;
    u32x4 pre[2][2];  // LINE + residual: epilogue residual blocks 0-1, issued in the last phase
    // one K-tile; the last one is a separate instantiation so that pre[] is
    // live only from its p3 to the epilogue (assigned in a loop iteration it
    // would be live around the whole K loop and spill)
    // peel_c: std::integral_constant<int, P>; P >= 0 = this is K-tile P (compile time,
    // the ResNorm/StatsOut variants peel K-tiles 0-1 so no per-tile branch sits in the K loop),
    // -1 = a K-tile >= 2 of a peeled loop, -2 = runtime t (non-folding variants)
    auto kstep = [&](int t, auto last_c, auto peel_c) {
      constexpr bool last = decltype(last_c)::value;
      constexpr int P = decltype(peel_c)::value;
      const bool is_t0 = P == -2 ? t == 0 : P == 0;
      const bool more = !last || has_next;
      int kn = t + 1;  // K-tile staged during this one
      if (last && has_next) {
        // the stream runs on into K-tile 0 of the next tile
        tile = xcd_remap(vn, ntiles);
        m0 = (tile / ntn) * 256;
        n0 = (tile % ntn) * 256;
        set_src(m0, n0);
        kn = 0;
      }
      const bool relax = is_t0 && !first;  // epilogue stores of the previous tile may be in flight
      // p0
      read_a(buf, 0);
      read_b(bl, buf, 0);
      if constexpr (kBiasAcc) {
        // the next tile's bias, ahead of its K-tile 0 (older than every quarter of
        // it, so retired by the waits that retire them; single buffer: this tile's
        // bias was consumed by the accumulator init)
        if (last && has_next) glds4(bias + n0 + (wave & 3) * 64, lds + kBiasOff + (wave & 3) * 256);
      } else if ((EPI & kEpiBias) && is_t0) {
        // this tile's bias -> LDS (waves w, w+4 write the same 256 B: every wave
        // issues the same op count). Only makes the waits below stricter.
        const int bl_lane = (kIn || kRes || kSt) ? opaque_lane() : lane;
        __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)(bias + cn0 + (wave & 3) * 64 + bl_lane),
                                         (ATPU_LDS_AS void*)(lds + kBiasOff + (tile_par * 256 + (wave & 3) * 64) * 4),
                                         4, 0, 0);
      }
      if constexpr (kInAcc) {
        if (last && has_next) ln_stage_in(m0, n0, tile_par ^ 1);
      }
      if constexpr (kPeel) {
        if constexpr (P == 1) {
          ln_stage(cm0, cn0);
          if (!first) ln_flush(pm0, pn0);
        }
      }
      if (more) {
        stage(0, kn, buf ^ 1);
        if (relax) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + kEpiOps) : "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      ATPU_PS_SYNC_MMA(bl, 0, 0);
      // p1
      read_b(br, buf, 1);
      if (more) {
        stage(1, kn, buf ^ 1);
        if (relax) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + kEpiOps) : "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      ATPU_PS_SYNC_MMA(br, 0, 1);
      // p2
      read_a(buf, 1);
      if (more) {
        stage(2, kn, buf ^ 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      ATPU_PS_SYNC_MMA(br, 1, 1);
      // p3
      if (more) {
        stage(3, kn, buf ^ 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      if constexpr (LINE && (EPI & kEpiResidual)) {
        // the first two 16-row residual blocks of the line epilogue go out now
        // (into br's registers, dead after p2) and land under this phase's MMAs:
        // the tail then starts without a full memory latency
        if constexpr (last) {
          // buffer loads: scalar base, one 32-bit lane offset (recomputed from
          // the lane id, opaque so it is not hoisted and kept live), row steps
          // as scalar offsets - the 64-bit address math spilled
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<bf16*>(R + (size_t)(cm0 + wm * 128) * ldr + cn0 + wn * 64), 0, 0x7fffffff, 0x00020000);
          int l2 = __lane_id();
          asm volatile("" : "+v"(l2));
          const int vo = ((l2 >> 3) * ldr + (l2 & 7) * 8) * 2;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int so = (i * 16 + h * 8) * ldr * 2;
              // untracked (see load16_untracked); the epilogue waits for it
              asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(pre[i][h]) : "v"(vo), "s"(rs), "s"(so) : "memory");
            }
        }
      }
      ATPU_PS_SYNC_MMA(bl, 1, 0);
      buf ^= 1;
    };
    if constexpr (kPeel) {  // host: K >= 256, so K-tiles 0-1 are never the last
      kstep(0, std::false_type{}, std::integral_constant<int, 0>{});
      kstep(1, std::false_type{}, std::integral_constant<int, 1>{});
      for (int t = 2; t + 1 < nk; ++t) kstep(t, std::false_type{}, std::integral_constant<int, -1>{});
      kstep(nk - 1, std::true_type{}, std::integral_constant<int, -1>{});
    } else {
      for (int t = 0; t + 1 < nk; ++t) kstep(t, std::false_type{}, std::integral_constant<int, -2>{});
      kstep(nk - 1, std::true_type{}, std::integral_constant<int, -2>{});
    }
    // Both wave groups run the epilogue TOGETHER: group 0 waits one barrier (group 1's
    // last MMA phase) before it, group 1 takes one after it, so the stagger resumes at
    // the next tile with equal barrier counts. A wave alone issues VALU at half the
    // SIMD's rate and sits out its LDS / store latencies; two epilogues side by side
    // fill each other's gaps, where the staggered form ran them back to back (each
    // beside only one 16-MFMA phase of the partner).
    if constexpr (kSyncEpi) {
      __builtin_amdgcn_sched_barrier(0);
      if (wm == 0) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DBG & 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else {
      // DBG & 8 (timing-only ablation of the LN-folding variants): their staging and
      // tile-loop structure, the plain epilogue (no LN math, no statistics)
      constexpr int kEpiRun0 = kBiasAcc ? (EPI & ~kEpiBias) : EPI;
      constexpr int kEpiRun = (DBG & 8) ? (kEpiRun0 & ~(kEpiInNorm | kEpiResNorm | kEpiStatsOut)) : kEpiRun0;
      if constexpr (LINE)
        epilogue_256_line<kEpiRun, NT, kInAcc, ((DBG >> 5) & 3), bool(DBG & 256)>(
            acc, cm0, cn0, wm, wn, (kIn || kRes || kSt) ? opaque_lane() : lane, C, ldc, R, ldr,
            reinterpret_cast<const float*>(lds + kBiasOff) + tile_par * 256, lds + kEpiOff + wave * 2048, pre,
            LnLds{reinterpret_cast<const float*>(lds + kFinOff + (kInAcc ? tile_par * 2048 : 0)),
                  reinterpret_cast<const float*>(lds + kColOff), reinterpret_cast<float*>(lds + kStOff)});
      else
        epilogue_256<EPI, true, (DBG >> 1), NT>(acc, cm0, cn0, wm, wn, lane, C, ldc, bias, R, ldr, M,
                                            reinterpret_cast<const float*>(lds + kBiasOff) + tile_par * 256);
    }
    if constexpr (kSyncEpi) {
      __builtin_amdgcn_sched_barrier(0);
      if (wm == 1) __builtin_amdgcn_s_barrier();
    }
    pm0 = cm0;
    pn0 = cn0;
    if (!has_next) break;
    v = vn;
    first = false;
    tile_par ^= 1;
  }
#undef ATPU_PS_SYNC_MMA
  if (wm == 0) __builtin_amdgcn_s_barrier();  // close the stagger (equal barrier counts)
  if constexpr (kSt) {
    // the last tile's row partials: every wave's epilogue LDS writes done, then flushed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    ln_flush(pm0, pn0);
  }
}


}  // namespace

static int g_cu_budget = 0;

int cu_budget(int set) {
  if (set >= 0) g_cu_budget = set;
  return g_cu_budget;
}

int num_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      cus = 256;
    return cus > 0 ? cus : 256;
  }();
  // persistent grids are sized for the CUs a launch can use: a CU-masked stream
  // (ClassifyEngine's split mode) sees only its share of the chip
  return g_cu_budget > 0 ? std::min(g_cu_budget, n) : n;
}

int64_t make_cu_mask_stream(int first_bit, int nbits) {
  // CU mask bits are dealt round-robin over the XCDs (bit i -> XCD i % 8), so a
  // contiguous bit range is an even share of every XCD (and of its L2)
  uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = first_bit; b < first_bit + nbits && b < 256; ++b) mask[b / 32] |= 1u << (b % 32);
  hipStream_t s = nullptr;
  ATPU_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, 8, mask));
  return reinterpret_cast<int64_t>(s);
}

namespace {

template <bool NT, bool LINE = false>
void launch_256s(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + 255) / 256) * (g.N / 256);
  // one workgroup per CU; a multiple of 8 so v % 8 keeps naming the XCD
  int nb = std::min(tiles, num_cus());
  if (nb >= 8) nb &= ~7;
  const LnFold lf{g.in_fin, g.colsum, g.res_fin, g.gamma, g.part_out};
#define ATPU_G256S(E)                                                                                          \
  case E:                                                                                                      \
    hipLaunchKernelGGL((gemm256s_kernel<E, 0, NT, LINE>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, g.ldc, \
                       g.bias, g.R, g.ldr, g.M, g.N, g.K, lf);                                                 \
    break;
  if constexpr (LINE) {
    switch (g.epi) {
      ATPU_G256S(kEpiBias | kEpiInNorm)
      ATPU_G256S(kEpiBias | kEpiInNorm | kEpiGelu)
      ATPU_G256S(kEpiBias | kEpiResidual | kEpiStatsOut)
      ATPU_G256S(kEpiBias | kEpiResidual | kEpiResNorm | kEpiStatsOut)
      default:
        break;
    }
    if (g.epi & (kEpiInNorm | kEpiResNorm | kEpiStatsOut)) return;
  }
  switch (g.epi) {
    ATPU_G256S(0)
    ATPU_G256S(kEpiBias)
    ATPU_G256S(kEpiBias | kEpiGelu)
    ATPU_G256S(kEpiBias | kEpiTanh)
    ATPU_G256S(kEpiBias | kEpiResidual)
    ATPU_G256S(kEpiResidual)
    ATPU_G256S(kEpiGelu)
    ATPU_G256S(kEpiRelu)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_G256S
}





// ============================================================================
// Skinny-M GEMM ("dec"): decode steps (M = docs x beams, ~256-2048 rows) and
// the CLS-only last encoder layer. The 128x128 kernel underfills the chip at
// these M (48 tiles for [1024 x 768]) and its two-buffer loop waits one full
// L2/HBM round trip per K-tile, so even split 6 ways it ran ~12 us + a 5 us
// reduce for a 1.2 GFLOP problem. Here:
//  * 64x64 tiles, 4 waves (2x2, 32x32 each): 4x the blocks of 128x128;
//  * an NST-deep LDS ring fed by LDS-DMA keeps NST-1 K-tiles in flight
//    (counted vmcnt, one barrier per K-tile), so the loop runs at L2->LDS
//    bandwidth instead of latency;
//  * M-fastest tile order under the XCD remap: the blocks of one XCD share
//    weight panels, so each XCD's L2 pulls a distinct slice of the weights.
// Same swizzle, fragment layout and epilogue as the 128x128 kernel.
// ============================================================================
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One row's share of a 64x64 "dec" tile epilogue (also the exact few-row kernel's): the lane holds
// row m, columns nb + j*16 + fchunk*4 .. +3 of fragments j < NJ (nb = the wave's first column;
// with RowStats NJ = 2, nb a 32-column slab). Every operation and its order are shared, so the
// two kernels produce the same bits for a row (batch invariance).
template <int EPI, int NJ>
__device__ __forceinline__ void dec_row_vals(const f32x4 (&acc)[NJ], int m, int nb, int fchunk, int N, float rstd,
                                             float rmu, float2 rf, bf16* __restrict__ C, int ldc,
                                             const float* __restrict__ bias, const bf16* __restrict__ R, int ldr,
                                             const KvOut& kvo, const LnDec& ln, int kv_pos, bf16x4 (&ov)[NJ]) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = nb + j * 16 + fchunk * 4;
    if (n >= N) continue;
    f32x4 v = acc[j];
    if constexpr (EPI & kEpiRowRms) v *= rstd;
    if constexpr (EPI & kEpiRowLn) {
      const f32x4 cs = *reinterpret_cast<const f32x4*>(ln.colsum + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaf(v[e], rstd, -rmu * cs[e]);
    }
    if constexpr (EPI & kEpiBias) v += *reinterpret_cast<const f32x4*>(bias + n);
    if constexpr (EPI & kEpiGelu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_poly1(v[e]);
    }
    if constexpr (EPI & kEpiTanh) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
    }
    if constexpr (EPI & kEpiRelu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if constexpr (EPI & kEpiResidual) {
      const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n);
      if constexpr (EPI & kEpiResLn) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(ln.gamma + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(fmaf(bf2f(r[e]), rf.x, -rf.y), g[e], v[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bf2f(r[e]);
      }
    }
    if constexpr (EPI & kEpiOutF32) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = v;
    } else {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      ov[j] = o;
      if (EPI & kEpiKvScatter) {
        // the tile is all Q or all K|V (host: kv_col0 % 128 == 0)
        // a step past the cache (caller bug) drops the K|V write instead of writing out of bounds
        if (n < kvo.col0)
          *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
        else if (kv_pos < kvo.T)
          *reinterpret_cast<bf16x4*>(kvo.cache + ((size_t)m * kvo.T + kv_pos) * kvo.ld + (n - kvo.col0)) = o;
      } else {
        *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
      }
    }
  }
}

// RowStats: the (sum, sum of squares) of the row's stored (bf16) outputs over the 32-column slab
// at nb, this lane's 2 x 4 values in column order, then over the slab's 4 lanes of the row
__device__ __forceinline__ void dec_row_stats(const bf16x4 (&ov)[2], int m, int nb, int fchunk, int M, int N,
                                              const LnDec& ln) {
  float ps = 0.f, pss = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (nb + j * 16 + fchunk * 4 >= N) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float f = bf2f(ov[j][e]);
      ps += f;
      pss = fmaf(f, f, pss);
    }
  }
  const float S = lane_rows_sum(ps), Q = lane_rows_sum(pss);
  if (fchunk == 0 && nb < N) *reinterpret_cast<float2*>(ln.part_out + 2 * ((size_t)(nb / 32) * M + m)) = float2{S, Q};
}

// One row's share of a 64x64 "dec" tile epilogue (also the exact few-row kernel's): the lane holds
// row m, columns nb + j*16 + fchunk*4 .. +3 of fragments j < NJ (nb = the wave's first column;
// with RowStats NJ = 2, nb a 32-column slab). Every operation and its order are shared, so the
// two kernels produce the same bits for a row (batch invariance).
template <int EPI, int NJ>
__device__ __forceinline__ void dec_row_out(const f32x4 (&acc)[NJ], int m, int nb, int fchunk, int M, int N,
                                            float rstd, float rmu, float2 rf, bf16* __restrict__ C, int ldc,
                                            const float* __restrict__ bias, const bf16* __restrict__ R, int ldr,
                                            const KvOut& kvo, const LnDec& ln, int kv_pos) {
  static_assert(!(EPI & kEpiRowStats) || NJ == 2, "RowStats: a 32-column slab per wave");
  if (m >= M) return;
  bf16x4 ov[NJ];
  dec_row_vals<EPI, NJ>(acc, m, nb, fchunk, N, rstd, rmu, rf, C, ldc, bias, R, ldr, kvo, ln, kv_pos, ov);
  if constexpr (EPI & kEpiRowStats) dec_row_stats(ov, m, nb, fchunk, M, N, ln);
}

template <int EPI, int NST, int SPLIT>
__global__ __launch_bounds__(256, 2) void gemm_dec_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                          int ldc, const float* __restrict__ bias,
                                                          const bf16* __restrict__ R, int ldr, int M, int N, int K,
                                                          float* __restrict__ ws, float rms_eps = 0.f,
                                                          KvOut kvo = {}, LnDec ln = {}) {
  static_assert(!(SPLIT && (EPI & (kEpiRowRms | kEpiRowLn | kEpiResLn))), "row statistics need the whole K loop");
  constexpr int BM = 64, BN = 64;
  constexpr int STAGE = (BM + BN) * kRowBytes;  // 16 KiB: A rows 0-63, B rows 64-127
  constexpr int LPS = (BM + BN) / 8 / 4;        // DMA instructions per wave per stage (4)
  __shared__ __attribute__((aligned(16))) char lds[NST * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (M + BM - 1) / BM;
  const int ntn = (N + BN - 1) / BN;
  if constexpr (SPLIT) {
    A += (size_t)blockIdx.y * K;
    Bt += (size_t)blockIdx.y * K;
  }
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile % ntm) * BM;
  const int n0 = (tile / ntm) * BN;

  const int srow = lane >> 3, spos = lane & 7;
  const bf16* src[LPS];
#pragma unroll
  for (int i = 0; i < LPS; ++i) {
    const int r = (i * 4 + wave) * 8 + srow;  // staged row 0..127 (wave-uniform half)
    if (r < BM) {
      src[i] = A + (size_t)min(m0 + r, M - 1) * lda + swz(r, spos) * 8;
    } else {
      src[i] = Bt + (size_t)min(n0 + r - BM, N - 1) * ldb + swz(r, spos) * 8;
    }
  }
  auto stage = [&](int kt, int slot) {
    char* base = lds + slot * STAGE;
#pragma unroll
    for (int i = 0; i < LPS; ++i) glds16(src[i] + kt * kBK, base + (i * 4 + wave) * 8 * kRowBytes);
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int frow = lane & 15, fchunk = lane >> 4;
  // RowLn / ResLn: the rows' partials, loaded before the K loop
  constexpr bool kPart = EPI & (kEpiRowLn | kEpiResLn);
  float2 pv[kPart ? 2 : 1][kPartPerLane];
  const int pslots = (EPI & kEpiRowLn) ? K / 32 : N / 32;
  if constexpr (kPart) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      part_prefetch(pv[i], (EPI & kEpiRowLn) ? ln.in_part : ln.res_part, pslots, M, m0 + wm * 32 + i * 16 + frow, fchunk);
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float ssq[2] = {0.f, 0.f};  // RowRms: this lane's share of its A rows' sum of squares
  auto compute = [&](int slot) {
    const char* base = lds + slot * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfg[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm * 32 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
        if constexpr (EPI & kEpiRowRms) ssq[i] = sumsq_bf16x8(af[i], ssq[i]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = BM + wn * 32 + j * 16 + frow;
        bfg[j] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = K / kBK;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) stage(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    // stages issued so far: min(nk, kt + NST - 1); stage kt must have landed
    if (kt + NST - 1 <= nk)
      wait_vmcnt<(NST - 2) * LPS>();
    else
      wait_vmcnt0();
    // raw s_barrier: __syncthreads() would add a vmcnt(0) fence and drain the ring.
    // After the counted wait every wave's DMA for stage kt has landed; the
    // barrier publishes that and frees slot (kt-1)%NST (its ds_reads retired
    // before the MFMAs that consumed them).
    asm volatile("s_barrier" ::: "memory");
    if (kt + NST - 1 < nk) stage(kt + NST - 1, (kt + NST - 1) % NST);
    compute(kt % NST);
  }

  if constexpr (SPLIT) {
    float* mine = ws + blockIdx.y * (size_t)M * N;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + wm * 32 + i * 16 + frow;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 32 + j * 16 + fchunk * 4;
        if (m < M && n < N) *reinterpret_cast<f32x4*>(mine + (size_t)m * N + n) = acc[i][j];
      }
    }
    return;
  }
  const int kv_pos = (EPI & kEpiKvScatter) ? max(*kvo.step, 0) : 0;
  float rstd[2], rmu[2];
  float2 rfs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rstd[i] = (EPI & kEpiRowRms) ? __builtin_amdgcn_rsqf(lane_rows_sum(ssq[i]) * (1.f / K) + rms_eps) : 1.f;
    rmu[i] = 0.f;
    rfs[i] = float2{1.f, 0.f};
    if constexpr (EPI & kEpiRowLn) {
      const float2 st = part_ln(pv[i], pslots, fchunk, rms_eps);
      rstd[i] = st.x;
      rmu[i] = st.y;
    }
    if constexpr (EPI & kEpiResLn) rfs[i] = part_ln(pv[i], pslots, fchunk, rms_eps);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
    dec_row_out<EPI, 2>(acc[i], m0 + wm * 32 + i * 16 + frow, n0 + wn * 32, fchunk, M, N, rstd[i], rmu[i], rfs[i],
                        C, ldc, bias, R, ldr, kvo, ln, kv_pos);
}

// ============================================================================
// Exact few-row GEMM (M <= 16, batch-invariant mode: ATPU_BATCH_INVARIANT). The <= 4-row GEMV
// sums K with v_dot2 partials spread over lanes, so a 1-document decode step would round
// differently from the same document inside a batch (the dec / 128 / 256 kernels). This kernel
// computes each output exactly as gemm_dec_kernel does -- ONE v_mfma_f32_16x16x32_bf16 chain over
// K in ascending 32-wide k-steps with the same fragment layout (lane (fr, fc): row fr, k fc*8..+8),
// the RowRms sum of squares in the same lane order, and the shared epilogue (dec_row_out) -- but
// with no LDS ring: one wave owns 16 x 16 outputs and streams its operands straight into MFMA
// fragment registers, RD k-steps per round, the next round's loads in flight under this round's
// MFMAs (two register sets). N / 16 compute waves, one per workgroup (two per workgroup for
// RowStats: a 32-column slab whose statistics wave 0 forms from both halves' stored outputs, in
// the 64x64 kernel's order), plus (PF) the GEMV's L2 prefetch wave for the next GEMM's weight rows.
// ============================================================================
template <int EPI, int RD, bool PF>
__global__ __launch_bounds__(64 * (((EPI & kEpiRowStats) ? 2 : 1) + PF)) void gemm_few_exact_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K, float rms_eps, KvOut kvo,
    LnDec ln, L2Pf pf) {
  // compute waves, one 16-column fragment each: 2 for RowStats (a 32-column slab, whose statistics
  // wave 0 forms from both halves in dec_row_out's order)
  constexpr int NCW = (EPI & kEpiRowStats) ? 2 : 1;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (PF) {
    __shared__ __attribute__((aligned(16))) char pf_scratch[256];
    if (w == NCW) {  // (takes the compute waves' barriers)
      l2_prefetch_rows<NCW - 1>(pf, threadIdx.x & 63, pf_scratch, blockIdx.x, gridDim.x);
      return;
    }
  }
  const int lane = threadIdx.x & 63, fr = lane & 15, fc = lane >> 4;
  const int nb = (blockIdx.x * NCW + w) * 16;  // this wave's first column
  const bf16* ar = A + (size_t)min(fr, M - 1) * lda + fc * 8;
  const bf16* br = Bt + (size_t)min(nb + fr, N - 1) * ldb + fc * 8;
  constexpr bool kPart = EPI & (kEpiRowLn | kEpiResLn);
  float2 pv[kPartPerLane];
  const int pslots = (EPI & kEpiRowLn) ? K / 32 : N / 32;
  if constexpr (kPart) part_prefetch(pv, (EPI & kEpiRowLn) ? ln.in_part : ln.res_part, pslots, M, fr, fc);
  f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
  float ssq = 0.f;
  const int nks = K / 32;
  bf16x8 a0[RD], b0[RD], a1[RD], b1[RD];
  auto load = [&](bf16x8 (&a)[RD], bf16x8 (&b)[RD], int r0) {
#pragma unroll
    for (int u = 0; u < RD; ++u) {
      const int ks = min(r0 + u, nks - 1);  // clamped: a tail round's extra k-steps are never used
      a[u] = *reinterpret_cast<const bf16x8*>(ar + ks * 32);
      b[u] = *reinterpret_cast<const bf16x8*>(br + ks * 32);
    }
  };
  auto mma = [&](const bf16x8 (&a)[RD], const bf16x8 (&b)[RD], int r0) {
#pragma unroll
    for (int u = 0; u < RD; ++u) {
      if (r0 + u < nks) {  // uniform
        if constexpr (EPI & kEpiRowRms) ssq = sumsq_bf16x8(a[u], ssq);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[u], a[u], acc[0], 0, 0, 0);
      }
    }
  };
  load(a0, b0, 0);
  for (int r0 = 0; r0 < nks; r0 += 2 * RD) {
    if (r0 + RD < nks) load(a1, b1, r0 + RD);
    mma(a0, b0, r0);
    if (r0 + RD < nks) {
      if (r0 + 2 * RD < nks) load(a0, b0, r0 + 2 * RD);
      mma(a1, b1, r0 + RD);
    }
  }
  const int kv_pos = (EPI & kEpiKvScatter) ? max(*kvo.step, 0) : 0;
  float rstd = (EPI & kEpiRowRms) ? __builtin_amdgcn_rsqf(lane_rows_sum(ssq) * (1.f / K) + rms_eps) : 1.f;
  float rmu = 0.f;
  float2 rf = float2{1.f, 0.f};
  if constexpr (EPI & kEpiRowLn) {
    const float2 st = part_ln(pv, pslots, fc, rms_eps);
    rstd = st.x;
    rmu = st.y;
  }
  if constexpr (EPI & kEpiResLn) rf = part_ln(pv, pslots, fc, rms_eps);
  if constexpr (NCW == 1) {
    dec_row_out<EPI, 1>(acc, fr, nb, fc, M, N, rstd, rmu, rf, C, ldc, bias, R, ldr, kvo, ln, kv_pos);
  } else {
    __shared__ bf16x4 xch[64];  // wave 1's stored outputs, for wave 0's slab statistics
    bf16x4 ov[1];
    if (fr < M) {
      dec_row_vals<EPI & ~kEpiRowStats, 1>(acc, fr, nb, fc, N, rstd, rmu, rf, C, ldc, bias, R, ldr, kvo, ln, kv_pos, ov);
      if (w == 1) xch[lane] = ov[0];
    }
    __syncthreads();
    if (w == 0 && fr < M) {
      const bf16x4 both[2] = {ov[0], xch[lane]};
      dec_row_stats(both, fr, nb, fc, M, N, ln);
    }
  }
}

// The long-K few-row case (K = 2048 / 3072: T5's FF-out, M <= 8): the register kernel above needs K / 512
// dependent load rounds per wave (8.1 us for T5 wo against the GEMV's 5). Here the workgroup's 4 waves
// put the wave's whole B slab (16 weight rows x K) and the M activation rows into LDS with LDS-DMA, every
// load in flight at once, and wave 0 runs the same MFMA chain (same fragments, same order, same epilogue)
// from LDS; wave 3 then issues the next GEMM's L2 prefetch. Bit-identical to gemm_few_exact_kernel.
template <int EPI, int NKS>
__global__ __launch_bounds__(256) void gemm_few_dma_kernel(const bf16* __restrict__ A, int lda,
                                                           const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                           int ldc, const float* __restrict__ bias,
                                                           const bf16* __restrict__ R, int ldr, int M, int N, int K,
                                                           KvOut kvo, LnDec ln, L2Pf pf, int pf_on) {
  static_assert(!(EPI & (kEpiRowStats | kEpiRowLn | kEpiResLn | kEpiRowRms)), "plain / bias / residual epilogues");
  constexpr int kApitch = NKS * 64 + 16;  // bytes per staged A row (padded: rows land 4 banks apart)
  constexpr int kApieces = NKS / 16;      // 1-KiB DMA pieces per A row
  __shared__ __attribute__((aligned(16))) char sB[NKS * 1024];  // k-step ks: lane (fr, fc)'s 16 B at ks*1024 + 16*lane
  __shared__ __attribute__((aligned(16))) char sA[8 * kApitch];
  __shared__ __attribute__((aligned(16))) char pf_scratch[256];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int fr = lane & 15, fc = lane >> 4;
  const int nb = blockIdx.x * 16;
  const bf16* br = Bt + (size_t)min(nb + fr, N - 1) * ldb + fc * 8;
  for (int ks = w; ks < NKS; ks += 4) glds16(br + ks * 32, sB + ks * 1024);
  for (int p = w; p < M * kApieces; p += 4) {
    const int r = p / kApieces, i = p - r * kApieces;
    glds16(A + (size_t)r * lda + i * 512 + lane * 8, sA + r * kApitch + i * 1024);
  }
  wait_vmcnt0();
  __syncthreads();
  if (w != 0) {
    if (w == 3 && pf_on) l2_prefetch_rows<0>(pf, lane, pf_scratch, blockIdx.x, gridDim.x);
    return;
  }
  const char* ap = sA + min(fr, M - 1) * kApitch + fc * 16;
  const char* bp = sB + lane * 16;
  f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 8
  for (int ks = 0; ks < NKS; ++ks) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(ap + ks * 64);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(bp + ks * 1024);
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[0], 0, 0, 0);
  }
  dec_row_out<EPI, 1>(acc, fr, nb, fc, M, N, 1.f, 0.f, float2{1.f, 0.f}, C, ldc, bias, R, ldr, kvo, ln, 0);
}

// the DMA form's cases (launch_few_exact); false: the register kernel
bool launch_few_dma(const GemmArgs& g, hipStream_t s, bool pf, const L2Pf& pfa) {
  static const bool on = [] {
    const char* f = std::getenv("ATPU_FEW_DMA");
    return !(f && f[0] == '0');
  }();
  if (!on || g.M > 8 || (g.K != 2048 && g.K != 3072) || g.N % 16) return false;
  const KvOut kvo{g.kv_cache, g.kv_ld, g.kv_T, g.kv_col0, g.kv_step};
  const LnDec ln{g.colsum, g.in_part, g.res_part, g.gamma, g.part_out};
#define ATPU_FD(E, NKS)                                                                                          \
  hipLaunchKernelGGL((gemm_few_dma_kernel<E, NKS>), dim3(g.N / 16), dim3(256), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, \
                     g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, kvo, ln, pfa, pf ? 1 : 0)
#define ATPU_FD_CASE(E)   \
  case E:                 \
    if (g.K == 2048) {    \
      ATPU_FD(E, 64);     \
    } else {              \
      ATPU_FD(E, 96);     \
    }                     \
    return true;
  switch (g.epi) {
    ATPU_FD_CASE(0)
    ATPU_FD_CASE(kEpiBias)
    ATPU_FD_CASE(kEpiResidual)
    ATPU_FD_CASE(kEpiBias | kEpiResidual)
    default:
      return false;
  }
#undef ATPU_FD_CASE
#undef ATPU_FD
}

bool few_exact_ok(const GemmArgs& g) {
  // batch-invariant mode: every <= 16-row GEMM; otherwise the 5-16-row ones (2-4 documents x 4 beams), where
  // it replaces the 64x64 kernel's few-workgroup grid with the same bits (ATPU_FEW_ROWS=0: off). <= 4 rows
  // keep the GEMV there.
  static const bool rows_on = [] {
    const char* f = std::getenv("ATPU_FEW_ROWS");
    return !(f && f[0] == '0');
  }();
  const bool inv = batch_invariant(-1) != 0;
  return (inv || (rows_on && g.M > 4)) && g.M <= 16 && g.N % 32 == 0 && g.K % 32 == 0 &&
         gemm_force_tile(-1) == 0 && !(g.epi & (kEpiInNorm | kEpiResNorm | kEpiStatsOut));
}

void launch_few_exact(const GemmArgs& g, hipStream_t s) {
  const KvOut kvo{g.kv_cache, g.kv_ld, g.kv_T, g.kv_col0, g.kv_step};
  const LnDec ln{g.colsum, g.in_part, g.res_part, g.gamma, g.part_out};
  // the GEMV's prefetch rule (ATPU_GEMV_PREFETCH, not from RowStats launches)
  static const bool pf_on = [] {
    const char* f = std::getenv("ATPU_GEMV_PREFETCH");
    return !(f && f[0] == '0');
  }();
  const bool pf = pf_on && g.pf_w && g.pf_n > 0 && g.pf_k > 0 && !(g.epi & kEpiRowStats);
  const L2Pf pfa{g.pf_w, g.pf_ld, g.pf_k, g.pf_n, g.pf_rpb > 0 ? g.pf_rpb : 16};
  if (launch_few_dma(g, s, pf, pfa)) return;
  // K >= 2048 (T5 wo, BART fc2): 16 k-steps per round, half the dependent load rounds
#define ATPU_FEW_GO1(E, RD, P)                                                                                    \
  hipLaunchKernelGGL((gemm_few_exact_kernel<E, RD, P>), dim3(g.N / (16 * kNcw)), dim3(64 * (kNcw + (P))), 0, s,   \
                     g.A, g.lda, g.Bt, g.ldb, g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, g.rms_eps, kvo, ln, pfa)
#define ATPU_FEW_CASE(E)                                    \
  case E: {                                                 \
    constexpr int kNcw = ((E) & kEpiRowStats) ? 2 : 1;      \
    if (pf && g.K >= 2048) {                                \
      ATPU_FEW_GO1(E, 16, true);                            \
    } else if (pf) {                                        \
      ATPU_FEW_GO1(E, 8, true);                             \
    } else if (g.K >= 2048) {                               \
      ATPU_FEW_GO1(E, 16, false);                           \
    } else {                                                \
      ATPU_FEW_GO1(E, 8, false);                            \
    }                                                       \
    break;                                                  \
  }
  switch (g.epi) {
    ATPU_FEW_CASE(kEpiRowLn | kEpiBias | kEpiKvScatter)
    ATPU_FEW_CASE(kEpiRowLn | kEpiBias)
    ATPU_FEW_CASE(kEpiRowLn | kEpiBias | kEpiGelu)
    ATPU_FEW_CASE(kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats)
    ATPU_FEW_CASE(kEpiBias | kEpiResidual | kEpiRowStats)
    ATPU_FEW_CASE(kEpiBias | kEpiResidual | kEpiResLn)
    ATPU_FEW_CASE(kEpiRowRms | kEpiKvScatter)
    ATPU_FEW_CASE(kEpiBias | kEpiKvScatter)
    ATPU_FEW_CASE(kEpiRowRms)
    ATPU_FEW_CASE(kEpiRowRms | kEpiRelu)
    ATPU_FEW_CASE(kEpiRowRms | kEpiOutF32)
    ATPU_FEW_CASE(0)
    ATPU_FEW_CASE(kEpiBias)
    ATPU_FEW_CASE(kEpiBias | kEpiGelu)
    ATPU_FEW_CASE(kEpiBias | kEpiTanh)
    ATPU_FEW_CASE(kEpiBias | kEpiResidual)
    ATPU_FEW_CASE(kEpiResidual)
    ATPU_FEW_CASE(kEpiGelu)
    ATPU_FEW_CASE(kEpiRelu)
    ATPU_FEW_CASE(kEpiOutF32)
    ATPU_FEW_CASE(kEpiBias | kEpiOutF32)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_FEW_CASE
#undef ATPU_FEW_GO1
}

// Ring depth 4 (64 KiB LDS, 2 blocks/CU). 8 stages measured the same on the
// decode shapes (tools/bench_decode_gemm.py), so the loop is not bound by
// bytes in flight per CU.
constexpr int kDecStages = 4;

void launch_dec(const GemmArgs& g, hipStream_t s) {
  const dim3 grid(((g.M + 63) / 64) * ((g.N + 63) / 64)), block(256);
#define ATPU_DEC_CASE(E)                                                                                       \
  case E:                                                                                                      \
    hipLaunchKernelGGL((gemm_dec_kernel<E, kDecStages, 0>), grid, block, 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, \
                       g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, nullptr, g.rms_eps,                          \
                       KvOut{g.kv_cache, g.kv_ld, g.kv_T, g.kv_col0, g.kv_step},                              \
                       LnDec{g.colsum, g.in_part, g.res_part, g.gamma, g.part_out});                        \
    break;
  switch (g.epi) {
    ATPU_DEC_CASE(kEpiRowLn | kEpiBias | kEpiKvScatter)
    ATPU_DEC_CASE(kEpiRowLn | kEpiBias)
    ATPU_DEC_CASE(kEpiRowLn | kEpiBias | kEpiGelu)
    ATPU_DEC_CASE(kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats)
    ATPU_DEC_CASE(kEpiBias | kEpiResidual | kEpiRowStats)
    ATPU_DEC_CASE(kEpiBias | kEpiResidual | kEpiResLn)
    ATPU_DEC_CASE(kEpiRowRms | kEpiKvScatter)
    ATPU_DEC_CASE(kEpiBias | kEpiKvScatter)
    ATPU_DEC_CASE(kEpiRowRms)
    ATPU_DEC_CASE(kEpiRowRms | kEpiRelu)
    ATPU_DEC_CASE(kEpiRowRms | kEpiOutF32)
    ATPU_DEC_CASE(0)
    ATPU_DEC_CASE(kEpiBias)
    ATPU_DEC_CASE(kEpiBias | kEpiGelu)
    ATPU_DEC_CASE(kEpiBias | kEpiTanh)
    ATPU_DEC_CASE(kEpiBias | kEpiResidual)
    ATPU_DEC_CASE(kEpiResidual)
    ATPU_DEC_CASE(kEpiGelu)
    ATPU_DEC_CASE(kEpiRelu)
    ATPU_DEC_CASE(kEpiOutF32)
    ATPU_DEC_CASE(kEpiBias | kEpiOutF32)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_DEC_CASE
}

// Sum the split-K fp32 partials [splits][M][N] in slice order and apply the epilogue.
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, bf16* __restrict__ C,
                                                            int ldc, const float* __restrict__ bias,
                                                            const bf16* __restrict__ R, int ldr, int M, int N) {
  const int nq = N / 4;
  const size_t slab = (size_t)M * N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M * nq; i += gridDim.x * blockDim.x) {
    const int m = i / nq, n = (i % nq) * 4;
    const float* src = ws + (size_t)m * N + n;
    f32x4 v = *reinterpret_cast<const f32x4*>(src);
    for (int z = 1; z < splits; ++z) v += *reinterpret_cast<const f32x4*>(src + z * slab);
    if constexpr (EPI & kEpiBias) v += *reinterpret_cast<const f32x4*>(bias + n);
    if constexpr (EPI & kEpiGelu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_poly1(v[e]);
    }
    if constexpr (EPI & kEpiTanh) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
    }
    if constexpr (EPI & kEpiRelu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if constexpr (EPI & kEpiResidual) {
      const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += bf2f(r[e]);
    }
    if constexpr (EPI & kEpiOutF32) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = v;
    } else {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
    }
  }
}

void launch_splitk(const GemmArgs& g, int splits, bool dec, hipStream_t s) {
  const int kc = g.K / splits;
  if (dec) {
    const int nb = ((g.M + 63) / 64) * ((g.N + 63) / 64);
    hipLaunchKernelGGL((gemm_dec_kernel<0, kDecStages, 1>), dim3(nb, splits), dim3(256), 0, s, g.A, g.lda, g.Bt,
                       g.ldb, nullptr, 0, nullptr, nullptr, 0, g.M, g.N, kc, g.ws);
  } else {
    constexpr int BM = 128, BN = 128;
    const int nb = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, 2, 2, 0, 1>), dim3(nb, splits), dim3(256), 0, s, g.A, g.lda, g.Bt,
                       g.ldb, nullptr, 0, nullptr, nullptr, 0, g.M, g.N, kc, g.ws);
  }
  const int work = g.M * (g.N / 4);
  const dim3 rg(std::max(1, std::min(2048, (work + 255) / 256))), rb(256);
#define ATPU_RED(E)                                                                                          \
  case E:                                                                                                    \
    hipLaunchKernelGGL((splitk_reduce_kernel<E>), rg, rb, 0, s, g.ws, splits, g.C, g.ldc, g.bias, g.R, g.ldr, \
                       g.M, g.N);                                                                            \
    break;
  switch (g.epi) {
    ATPU_RED(0)
    ATPU_RED(kEpiBias)
    ATPU_RED(kEpiBias | kEpiGelu)
    ATPU_RED(kEpiBias | kEpiTanh)
    ATPU_RED(kEpiBias | kEpiResidual)
    ATPU_RED(kEpiResidual)
    ATPU_RED(kEpiGelu)
    ATPU_RED(kEpiRelu)
    ATPU_RED(kEpiOutF32)
    ATPU_RED(kEpiBias | kEpiOutF32)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_RED
}

template <int BM, int BN, int WM, int WN>
void launch_tile(const GemmArgs& g, hipStream_t s) {
  const int nb = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(nb), block(WM * WN * 64);
#define ATPU_GEMM_CASE(E)                                                                             \
  case E:                                                                                             \
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, E>), grid, block, 0, s, g.A, g.lda, g.Bt, g.ldb, \
                       g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, nullptr, g.rms_eps,              \
                       KvOut{g.kv_cache, g.kv_ld, g.kv_T, g.kv_col0, g.kv_step},                      \
                       LnDec{g.colsum, g.in_part, g.res_part, g.gamma, g.part_out});                \
    break;
  switch (g.epi) {
    ATPU_GEMM_CASE(kEpiRowLn | kEpiBias | kEpiKvScatter)
    ATPU_GEMM_CASE(kEpiRowLn | kEpiBias)
    ATPU_GEMM_CASE(kEpiRowLn | kEpiBias | kEpiGelu)
    ATPU_GEMM_CASE(kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats)
    ATPU_GEMM_CASE(kEpiBias | kEpiResidual | kEpiRowStats)
    ATPU_GEMM_CASE(kEpiBias | kEpiResidual | kEpiResLn)
    ATPU_GEMM_CASE(kEpiRowRms | kEpiKvScatter)
    ATPU_GEMM_CASE(kEpiBias | kEpiKvScatter)
    ATPU_GEMM_CASE(kEpiRowRms)
    ATPU_GEMM_CASE(kEpiRowRms | kEpiRelu)
    ATPU_GEMM_CASE(kEpiRowRms | kEpiOutF32)
    ATPU_GEMM_CASE(0)
    ATPU_GEMM_CASE(kEpiBias)
    ATPU_GEMM_CASE(kEpiBias | kEpiGelu)
    ATPU_GEMM_CASE(kEpiBias | kEpiTanh)
    ATPU_GEMM_CASE(kEpiBias | kEpiResidual)
    ATPU_GEMM_CASE(kEpiResidual)
    ATPU_GEMM_CASE(kEpiGelu)
    ATPU_GEMM_CASE(kEpiRelu)
    ATPU_GEMM_CASE(kEpiOutF32)
    ATPU_GEMM_CASE(kEpiBias | kEpiOutF32)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_GEMM_CASE
}

}  // namespace

int gemm_256_variant(int set) {
  // 256x256 schedule (ATPU_GEMM_256=p|l|n):
  //   1 "256p" ping-pong, one launch per tile
  //   3 "256l" persistent, full-line LDS-transposed epilogue
  //   4 "256n" = 256l with non-temporal stores (default; docs/PERF_NOTES.md)
  //   (0 "256b" and 2 "256s" with the permlane epilogue are retired: git history)
  static int v = [] {
    const char* f = std::getenv("ATPU_GEMM_256");
    if (!f) return 4;
    switch (f[0]) {
      case 'p': return 1;
      case 'l': return 3;
      default: return 4;
    }
  }();
  if (set >= 0) {
    ATPU_CHECK(set == 1 || set == 3 || set == 4, "gemm_256_variant: schedules 1 (256p), 3 (256l), 4 (256n)");
    v = set;
  }
  return v;
}

int gemm_force_tile(int set) {
  // kernel family override (benchmarks / tests): 0 = auto, 64 = skinny "dec", 128, 256; ATPU_GEMM_TILE
  static int v = [] {
    const char* f = std::getenv("ATPU_GEMM_TILE");
    return f ? std::atoi(f) : 0;
  }();
  if (set >= 0) v = set;
  return v;
}

int gemm_dec_mode(int set) {
  // skinny-M path: 1 = 64x64 multi-stage "dec" kernel (default), 0 = 128x128 split-K; ATPU_GEMM_DEC=0|1
  static int v = [] {
    const char* f = std::getenv("ATPU_GEMM_DEC");
    return (f && f[0] == '0') ? 0 : 1;
  }();
  if (set >= 0) v = set;
  return v;
}

namespace {
// problems the 128x128 grid would leave under two blocks per CU
// Kernel family by how well each fills the 256 CUs (tools/bench_tile_choice.py, decode
// shapes at M = 1024 / 2048 / 4096): the 64x64 "dec" kernel while the 128x128 grid is
// small, the 128x128 kernel above that, the persistent 256x256 kernel once it has at
// more than half a tile per CU (e.g. N = 768 at M = 4096 is 48 tiles: 20 us there, 13.7 us
// on 128x128; at M = 2048 the dec kernel takes 8.7 us).
bool skinny(int M, int N) { return ((M + 127) / 128) * ((N + 127) / 128) < (M <= 1024 ? 512 : 192); }
bool big_fills(int M, int N) { return 2 * ((M + 255) / 256) * (N / 256) > num_cus(); }
}  // namespace

int batch_invariant(int set) {
  // Batch-invariant kernel selection (ATPU_BATCH_INVARIANT=1, the agent's default): a row's
  // result must not depend on how many rows share its launch. Off: the <= 4-row GEMV (v_dot2
  // partial sums) and split-K (fp32 slices summed by a second kernel) run where they are faster;
  // both change a row's K-summation order with the batch's row count. On: every GEMM row is one
  // MFMA 16x16x32 chain over K in ascending order on the 64x64 / 128x128 / 256x256 kernels,
  // which compute a row identically (the same chain, the same epilogue arithmetic and GELU);
  // decode attention and the LM head likewise keep their per-row kernels (decode.hip, lm_head.hip).
  static int v = [] {
    const char* f = std::getenv("ATPU_BATCH_INVARIANT");
    return (f && f[0] == '1') ? 1 : 0;
  }();
  if (set == 0 || set == 1) v = set;
  return v;
}

int gemm_splitk_splits(int M, int N, int K) {
  // Skinny problems (decode: M = beams x docs) leave most of the 256 CUs idle.
  // dec kernel: split K only when even 64x64 tiles give < 64 blocks AND the
  // K loop is long (>= 32 K-tiles): the reduce launch costs ~4 us, which a
  // 12-16 K-tile loop does not win back (measured, tools/bench_decode_gemm.py);
  // at 96-192 blocks (512-1024 rows) unsplit measured faster too (round 5:
  // tools/bench_dec_splitk.py at 1024 rows, T5 256-doc summarize at 2 x 512 rows).
  // 128x128 kernel: split so the grid reaches ~2 blocks per CU, >= 2 K-tiles per split.
  static const int forced = [] {
    const char* f = std::getenv("ATPU_GEMM_SPLITK");
    return f ? std::atoi(f) : -1;
  }();
  const int nk = K / kBK;
  if (batch_invariant(-1)) return 1;
  int want;
  if (gemm_dec_mode(-1) == 1 && skinny(M, N)) {
    const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
    want = forced >= 0 ? forced : (tiles >= 64 || nk < 32 ? 1 : (256 + tiles - 1) / tiles);
    want = std::max(1, std::min({want, nk / 8, 16}));
  } else {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    want = forced >= 0 ? forced : (M > 1024 || tiles >= 256 ? 1 : (512 + tiles - 1) / tiles);
    want = std::max(1, std::min({want, nk / 2, 16}));
  }
  while (want > 1 && nk % want) --want;
  return want;
}

namespace {

// ============================================================================
// Decode GEMV (M <= 4 rows: one document x 4 beams, the reference's job shape).
// The 64x64 "dec" kernel walks K through a chain of LDS-DMA round trips (a ~5.5 us
// floor at 12 K-tiles) and covers N = 768 with 12 workgroups; at 4 rows the GEMM is
// a weight stream. Here a wave owns 4 output columns and its 64 lanes split K in
// 16-B chunks (lane l: chunks l, l+64, ...): each round issues kGemvU chunks' weight
// and A loads at once (every load of K <= 1536 in one round), accumulates with
// v_dot2 in fp32, and the lanes are reduced by wave sums. 4 waves = 16 columns per
// workgroup (N = 768: 48 workgroups, 3072: 192). Epilogue as the other kernels:
// RowRms scale, bias, GELU / ReLU, residual, bf16 store (KvScatter: K|V columns into
// the cache row m*T + step). No split-K, no workspace.
// ============================================================================
constexpr int kGemvRows = 4;
// chunks per lane in flight per round (template U): 3 up to K = 1536, 6 up to K = 3072, so
// every K of the T5 / BART decoders but BART's fc2 (4096: two rounds) issues all of its loads
// in ONE round (two rounds serialised two memory latencies: 7.5 vs 4.5 us at K = 3072 cold,
// tools/probe_gemv_l2.py)
constexpr int gemv_u(int K) { return K <= 64 * 8 * 3 ? 3 : 6; }

// Prefetch of the next GEMV's weight (PF): one extra wave per workgroup (l2_prefetch.h). A 4-row
// GEMV on L2-resident weights ran 3.6-4.5 us against 4.9-7.5 us from HBM.
using GemvPf = L2Pf;
// tuning constants (python -m agent_tpu_amd.csrc.build -D NAME=V --out ...)
#ifndef ATPU_GEMV_NWV
#define ATPU_GEMV_NWV 4  // waves (4-column groups) per workgroup of the unsplit GEMVs but RowStats
#endif
constexpr int kGemvNwv = ATPU_GEMV_NWV;
#ifndef ATPU_GEMV_KS_NWV
#define ATPU_GEMV_KS_NWV 1  // column groups per K-split workgroup (x KS slices + the prefetch wave)
#endif
#ifndef ATPU_GEMV_KS
#define ATPU_GEMV_KS 2  // K slices of the split GEMV
#endif
#ifndef ATPU_GEMV_KS_MINK
#define ATPU_GEMV_KS_MINK 512  // split K above this
#endif
constexpr int kGemvKs = ATPU_GEMV_KS, kGemvKsU = 4096 / (512 * ATPU_GEMV_KS);  // K = 4096: one round
constexpr int kKsNwv = ATPU_GEMV_KS_NWV;

// BART's LayerNorm folding (RowLn / ResLn / RowStats, see LnDec): the row statistics come
// from the <= 32 slab partials (lane = slab, wave sums); RowStats workgroups are 8 waves =
// one 32-column slab, summed across the waves through LDS.
// KS > 1 (epilogues without row statistics taken from A, K > 512: the attention-out and FF-out
// GEMVs): KS waves per column group, each over 1/KS of K, their partials summed through LDS.
// One column group per workgroup (N/4 workgroups + the prefetch wave): 1-doc BART 11.1 -> 12.2,
// T5 14.6 -> 15.4 docs/s against the unsplit 4-wave workgroups (and K = 4096 no longer takes two
// serialised load rounds); profiles/gemv_ksplit_ab_r04.txt.
template <int EPI, int NWV, int U, bool PF, int KS = 1>
__global__ __launch_bounds__((NWV * KS + PF) * 64) void gemv_kernel(const bf16* __restrict__ A, int lda,
                                                              const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                              int ldc, const float* __restrict__ bias,
                                                              const bf16* __restrict__ R, int ldr, int M, int N, int K,
                                                              float rms_eps, KvOut kvo, LnDec ln, GemvPf pf) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  static_assert(!(EPI & kEpiRowStats) || NWV == 8, "RowStats: one 32-column slab per workgroup");
  static_assert(KS == 1 || !(EPI & kEpiRowStats), "K split: one barrier, not with the slab sum");
  constexpr int kGemvU = U;
  __shared__ float2 st_red[NWV][kGemvRows];
  __shared__ float ks_red[KS > 1 ? KS - 1 : 1][NWV][16];
  __shared__ float2 ks_row[KS > 1 ? KS - 1 : 1][NWV][kGemvRows];
  __shared__ __attribute__((aligned(16))) char pf_scratch[PF ? 256 : 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if constexpr (PF) {
    if (w == NWV * KS) {
      // RowStats workgroups have one barrier (the slab sum), K-split ones one (the half sum),
      // taken with the loads in flight
      l2_prefetch_rows<((EPI & kEpiRowStats) != 0 || KS > 1) ? 1 : 0>(pf, lane, pf_scratch, blockIdx.x, gridDim.x);
      return;
    }
  }
  const int cg = KS > 1 ? w % NWV : w, ks = KS > 1 ? w / NWV : 0;  // column group, K slice
  const int n0 = (blockIdx.x * NWV + cg) * 4;                      // this wave's 4 columns
  const int nch = K / (8 * KS), c0 = ks * nch;                     // its 16-B chunks of K
  // lanes 16 mo + 4 jo finish output (mo, n0 + jo). With LayerNorm folding (BART) its
  // epilogue operands (bias, residual, LN column sums / gamma, the row-statistics partials)
  // are loaded before the main loop and arrive under it instead of as a dependent round trip
  // after the reductions: BART 1-doc 8.5 -> 8.8 docs/s; for the T5 epilogues (RowRms, ReLU,
  // residual, KV scatter) the same early loads measured slower (12.3 -> 11.7), so those load
  // in the epilogue (profiles/summarize_1doc_gemv_early_loads_r04.txt; issued right after the
  // first round's loads instead: also slower, profiles/summarize_1doc_gemv_mid_loads_ab_r04.txt)
  constexpr bool kEarly = (EPI & (kEpiRowLn | kEpiResLn)) != 0;
  const int mo = lane >> 4, jo = (lane >> 2) & 3;  // the reduction's output lanes (below)
  const bool mine = mo < M && (lane & 3) == 0;
  const int om = min(mo, M - 1), n = n0 + jo;  // (clamped) output row
  float e_bias = 0.f, e_res = 0.f, e_col = 0.f, e_gam = 0.f;
  int e_step = 0;
  auto epi_loads = [&] {
    if (!mine) return;
    if constexpr (EPI & kEpiBias) e_bias = bias[n];
    if constexpr (EPI & kEpiResidual) e_res = bf2f(R[(size_t)om * ldr + n]);
    if constexpr (EPI & kEpiRowLn) e_col = ln.colsum[n];
    if constexpr (EPI & kEpiResLn) e_gam = ln.gamma[n];
    if constexpr (EPI & kEpiKvScatter) e_step = *kvo.step;
  };
  if constexpr (kEarly) epi_loads();
  // (sum, sum of squares) per row, lane-partial: RowLn takes its A rows' statistics from the A
  // chunks it loads anyway (the whole row: K is the LN width), so it needs no producer partials;
  // ResLn reads the slab partials of its residual rows
  float2 e_part[kGemvRows];
#pragma unroll
  for (int r = 0; r < kGemvRows; ++r) e_part[r] = float2{0.f, 0.f};
  if constexpr ((EPI & kEpiResLn) && !(EPI & kEpiRowLn)) {
    const int slots = N / 32;
#pragma unroll
    for (int r = 0; r < kGemvRows; ++r)
      e_part[r] = lane < slots ? *reinterpret_cast<const float2*>(ln.res_part + 2 * ((size_t)lane * M + min(r, M - 1)))
                               : float2{0.f, 0.f};
  }
  float acc[kGemvRows][4], ssq[kGemvRows];
#pragma unroll
  for (int m = 0; m < kGemvRows; ++m) {
    ssq[m] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[m][j] = 0.f;
  }
  for (int base = 0; base < nch; base += 64 * kGemvU) {
    bf16x8 wv[kGemvU][4], av[kGemvU][kGemvRows];
#pragma unroll
    for (int u = 0; u < kGemvU; ++u) {
      const int c = c0 + min(base + u * 64 + lane, nch - 1);  // clamped: its products are dropped below
#pragma unroll
      for (int j = 0; j < 4; ++j) wv[u][j] = *reinterpret_cast<const bf16x8*>(Bt + (size_t)(n0 + j) * ldb + c * 8);
#pragma unroll
      for (int m = 0; m < kGemvRows; ++m)
        av[u][m] = *reinterpret_cast<const bf16x8*>(A + (size_t)min(m, M - 1) * lda + c * 8);
    }
    // every load of the round is issued before the first use: left alone, the scheduler issued
    // them in groups of 8 with a full wait in between (U serialised memory latencies)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kGemvU; ++u) {
      const bool ok = base + u * 64 + lane < nch;
#pragma unroll
      for (int m = 0; m < kGemvRows; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float d = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            d = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{av[u][m][2 * e], av[u][m][2 * e + 1]},
                                                bf16x2_t{wv[u][j][2 * e], wv[u][j][2 * e + 1]}, d, false);
          acc[m][j] += ok ? d : 0.f;
        }
        if constexpr (EPI & kEpiRowRms) ssq[m] += ok ? sumsq_bf16x8(av[u][m], 0.f) : 0.f;
        if constexpr (EPI & kEpiRowLn) {
          e_part[m].x += ok ? sum_bf16x8(av[u][m], 0.f) : 0.f;
          e_part[m].y += ok ? sumsq_bf16x8(av[u][m], 0.f) : 0.f;
        }
      }
    }
  }
  // the 16 partials (m, j) summed over the wave by a butterfly that halves the values each
  // step (two permlane swaps, then xor shuffles): 17 cross-lane ops instead of 16 x 6, and
  // lanes 4i..4i+3 end with output i = m*4 + j (RowRms: lanes 16m.. with row m's sum of squares)
  float v, rs = 0.f;
  {
    float a16[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a16[i] = acc[i >> 2][i & 3];
    v = wave_bfly<16>(a16, OpAdd{});
    if constexpr (EPI & kEpiRowRms) rs = wave_bfly<kGemvRows>(ssq, OpAdd{});  // row lane >> 4
  }
  // (sum, sum of squares) of A's rows (RowLn) or R's rows (ResLn), row mo
  float S = 0.f, Q = 0.f;
  if constexpr (EPI & (kEpiRowLn | kEpiResLn)) {
    {
      // the 8 sums (row r: S = 2r, Q = 2r + 1) by the same butterfly as the outputs: lane l
      // ends with sum l >> 3, i.e. row l >> 4 (= mo), its partner lane l ^ 8 the other one
      float a8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a8[i] = i & 1 ? e_part[i >> 1].y : e_part[i >> 1].x;
      const float h = wave_bfly<8>(a8, OpAdd{});
      const float o = dppf<kDppMirror>(h);  // a lane of the other bit-3 half of the row
      const bool b3 = lane & 8;
      S = b3 ? o : h;
      Q = b3 ? h : o;
    }
  }
  if constexpr (KS > 1) {
    // the upper K slices hand their 16 sums (and A-row statistics) to slice 0's wave: one barrier
    if (ks > 0) {
      if ((lane & 3) == 0) ks_red[ks - 1][cg][lane >> 2] = v;
      if ((lane & 15) == 0) ks_row[ks - 1][cg][mo] = float2{(EPI & kEpiRowRms) ? rs : S, Q};
    }
    __syncthreads();
    if (ks > 0) return;
#pragma unroll
    for (int i = 0; i < KS - 1; ++i) {
      v += ks_red[i][cg][lane >> 2];
      const float2 t = ks_row[i][cg][mo];
      if constexpr (EPI & kEpiRowRms) rs += t.x;
      if constexpr (EPI & kEpiRowLn) {
        S += t.x;
        Q += t.y;
      }
    }
  }
  // (rstd, rstd*mu) of A's rows (RowLn) or R's rows (ResLn)
  float2 lnst = float2{1.f, 0.f};
  if constexpr (EPI & (kEpiRowLn | kEpiResLn)) {
    const float inv = 1.f / ((EPI & kEpiRowLn) ? K : N);
    const float mu = S * inv, var = fmaxf(Q * inv - mu * mu, 0.f);
    const float rr = __builtin_amdgcn_rsqf(var + rms_eps);
    lnst = float2{rr, rr * mu};
    if constexpr (EPI & kEpiRowLn) {
      // part_out (optional): A's rows in the [K/32][M][2] partial format of a RowStats producer,
      // the row totals in slot 0 and zeros elsewhere, for the ResLn GEMV that adds LN(A) as its
      // residual (workgroup 0, wave 0; lanes 16 r hold row r)
      if (ln.part_out && blockIdx.x == 0 && w == 0) {
        const int slots = K / 32;
        float2 tot[kGemvRows];
#pragma unroll
        for (int r = 0; r < kGemvRows; ++r)
          tot[r] = float2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(S), 16 * r)),
                          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Q), 16 * r))};
        for (int i = lane; i < slots * M; i += 64) {
          const int sl = i / M, r = i - sl * M;
          float2 val = float2{0.f, 0.f};
#pragma unroll
          for (int rr2 = 0; rr2 < kGemvRows; ++rr2) val = (sl == 0 && r == rr2) ? tot[rr2] : val;
          *reinterpret_cast<float2*>(ln.part_out + 2 * (size_t)i) = val;
        }
      }
    }
  }
  if constexpr (!kEarly) epi_loads();
  float f = 0.f;  // RowStats: the stored (bf16-rounded) value
  if (mine) {
    if constexpr (EPI & kEpiRowRms) v *= __builtin_amdgcn_rsqf(rs * (1.f / K) + rms_eps);
    if constexpr (EPI & kEpiRowLn) v = fmaf(v, lnst.x, -lnst.y * e_col);
    if constexpr (EPI & kEpiBias) v += e_bias;
    if constexpr (EPI & kEpiGelu) v = gelu_poly1(v);
    if constexpr (EPI & kEpiRelu) v = fmaxf(v, 0.f);
    if constexpr (EPI & kEpiResidual) {
      if constexpr (EPI & kEpiResLn) v = fmaf(fmaf(e_res, lnst.x, -lnst.y), e_gam, v);
      else v += e_res;
    }
    const bf16 o = f2bf(v);
    f = bf2f(o);
    if constexpr (EPI & kEpiKvScatter) {
      const int pos = max(e_step, 0);
      if (n < kvo.col0)
        C[(size_t)om * ldc + n] = o;
      else if (pos < kvo.T)  // a step past the cache (caller bug) drops the write
        kvo.cache[((size_t)om * kvo.T + pos) * kvo.ld + (n - kvo.col0)] = o;
    } else {
      C[(size_t)om * ldc + n] = o;
    }
  }
  if constexpr (EPI & kEpiRowStats) {
    // this wave's 4 columns of row m (lanes 16m + 4j), then the 8 waves of the slab
    float s1 = f, s2 = f * f;
    s1 += __shfl_xor(s1, 4);
    s2 += __shfl_xor(s2, 4);
    s1 += __shfl_xor(s1, 8);
    s2 += __shfl_xor(s2, 8);
    if (mine && jo == 0) st_red[w][mo] = float2{s1, s2};
    __syncthreads();
    if (w == 0 && lane < M) {
      float2 t = float2{0.f, 0.f};
#pragma unroll
      for (int x = 0; x < NWV; ++x) {
        t.x += st_red[x][lane].x;
        t.y += st_red[x][lane].y;
      }
      *reinterpret_cast<float2*>(ln.part_out + 2 * ((size_t)blockIdx.x * M + lane)) = t;
    }
  }
}

constexpr int kGemvEpis =
    kEpiBias | kEpiGelu | kEpiRelu | kEpiResidual | kEpiRowRms | kEpiKvScatter | kEpiRowLn | kEpiResLn | kEpiRowStats;

bool gemv_ok(const GemmArgs& g) {
  static const bool on = [] {
    const char* f = std::getenv("ATPU_GEMV");
    return !(f && f[0] == '0');
  }();
  return on && !batch_invariant(-1) && g.M <= kGemvRows && g.N % 16 == 0 && !(g.epi & ~kGemvEpis) &&
         gemm_force_tile(-1) == 0;
}

void launch_gemv(const GemmArgs& g, hipStream_t s) {
  if (g.epi & kEpiKvScatter)
    ATPU_CHECK(g.kv_cache && g.kv_step && g.kv_T > 0 && g.kv_col0 > 0 && g.kv_col0 < g.N && g.kv_ld >= g.N - g.kv_col0,
               "gemm: KvScatter needs a cache, a device step and kv_ld >= N - kv_col0");
  ATPU_CHECK(!(g.epi & (kEpiRowRms | kEpiRowLn | kEpiResLn)) || g.rms_eps > 0.f, "gemm: RowRms / RowLn / ResLn need eps > 0");
  // RowLn: the statistics come from A itself (in_part unused); part_out, if given, receives them
  ATPU_CHECK(!(g.epi & kEpiRowLn) || (g.colsum && g.K <= 1024 && g.K % 32 == 0), "gemm: RowLn needs colsum, K <= 1024");
  ATPU_CHECK(!(g.epi & kEpiResLn) || (g.res_part && g.gamma && g.N <= 1024 && g.N % 32 == 0),
             "gemm: ResLn needs res_part, gamma, N <= 1024");
  ATPU_CHECK(!(g.epi & kEpiRowStats) || (g.part_out && g.N % 32 == 0), "gemm: RowStats needs part_out and N % 32 == 0");
  const KvOut kvo{g.kv_cache, g.kv_ld, g.kv_T, g.kv_col0, g.kv_step};
  const LnDec ln{g.colsum, g.in_part, g.res_part, g.gamma, g.part_out};
  static const bool pf_on = [] {
    const char* f = std::getenv("ATPU_GEMV_PREFETCH");
    return !(f && f[0] == '0');
  }();
  // not from RowStats GEMVs (measured: BART 1-doc 8.20 -> 7.98 docs/s with it, round 4): their
  // 32 workgroups would stream the next weight alone, and the kernel ends only when the
  // prefetch waves do
  const bool pf = pf_on && g.pf_w && g.pf_n > 0 && g.pf_k > 0 && !(g.epi & kEpiRowStats);
  const GemvPf pfa{g.pf_w, g.pf_ld, g.pf_k, g.pf_n, g.pf_rpb > 0 ? g.pf_rpb : 16};
  const bool u6 = gemv_u(g.K) == 6;
  static const bool ks_on = [] {
    const char* f = std::getenv("ATPU_GEMV_KSPLIT");
    return !(f && f[0] == '0');
  }();
  // K split (KS slices, up to 4096 / (512 KS) chunks per lane and slice in one round)
  const bool ks2 = ks_on && g.K > ATPU_GEMV_KS_MINK && g.K % (8 * kGemvKs) == 0;
  const bool ks_u1 = g.K <= 512 * kGemvKs;  // one chunk per lane and slice
#define ATPU_GEMV_GO(E, UU, P)                                                                                   \
  hipLaunchKernelGGL((gemv_kernel<E, nwv, UU, P>), dim3(g.N / (4 * nwv)), dim3(64 * (nwv + P)), 0, s, g.A, g.lda, \
                     g.Bt, g.ldb, g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, g.rms_eps, kvo, ln, pfa)
// K-split epilogues (no A-row statistics) launch <E, nwv, 4, P, 2>; for the others the same
// expression names their existing <E, nwv, 3, P, 1> instantiation (never launched with ks2)
#define ATPU_GEMV_GO_KS(E, UU, P)                                                                                \
  hipLaunchKernelGGL((gemv_kernel<E, kKs ? kKsNwv : nwv, kKs ? UU : 3, P, kKs ? kGemvKs : 1>),                  \
                     dim3(g.N / (4 * (kKs ? kKsNwv : nwv))), dim3(64 * (kKs ? kGemvKs * kKsNwv : nwv) + 64 * P), 0, s, \
                     g.A,                                                                                        \
                     g.lda, g.Bt, g.ldb, g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, g.rms_eps, kvo, ln, pfa)
// (E) parenthesised: for E = kEpiBias | kEpiResidual, `E & kEpiRowStats` parsed as
// kEpiBias | (kEpiResidual & kEpiRowStats) and gave 8-wave workgroups to every multi-flag
// epilogue (round 3). The 8-wave RowStats kernels keep 3 chunks per lane in flight: with the
// prefetch wave (9 waves, <= 168 VGPRs) 6 spilled.
#define ATPU_GEMV_CASE(E)                                                                                       \
  case E: {                                                                                                     \
    constexpr int nwv = ((E) & kEpiRowStats) ? 8 : kGemvNwv;                                                    \
    constexpr int kU6 = nwv < 8 ? 6 : 3;                                                                        \
    constexpr bool kKs = !((E) & (kEpiRowStats | kEpiRowRms | kEpiRowLn));                                      \
    if (kKs && ks2) {                                                                                           \
      if (pf) {                                                                                                 \
        if (ks_u1) ATPU_GEMV_GO_KS(E, 1, true);                                                                 \
        else ATPU_GEMV_GO_KS(E, kGemvKsU, true);                                                                \
      } else {                                                                                                  \
        if (ks_u1) ATPU_GEMV_GO_KS(E, 1, false);                                                                \
        else ATPU_GEMV_GO_KS(E, kGemvKsU, false);                                                               \
      }                                                                                                         \
    } else if (pf) {                                                                                            \
      if (u6) ATPU_GEMV_GO(E, kU6, true);                                                                       \
      else ATPU_GEMV_GO(E, 3, true);                                                                            \
    } else {                                                                                                    \
      if (u6) ATPU_GEMV_GO(E, kU6, false);                                                                      \
      else ATPU_GEMV_GO(E, 3, false);                                                                           \
    }                                                                                                           \
    break;                                                                                                      \
  }
  switch (g.epi) {
    ATPU_GEMV_CASE(0)
    ATPU_GEMV_CASE(kEpiBias)
    ATPU_GEMV_CASE(kEpiResidual)
    ATPU_GEMV_CASE(kEpiBias | kEpiResidual)
    ATPU_GEMV_CASE(kEpiRelu)
    ATPU_GEMV_CASE(kEpiBias | kEpiRelu)
    ATPU_GEMV_CASE(kEpiBias | kEpiGelu)
    ATPU_GEMV_CASE(kEpiRowRms)
    ATPU_GEMV_CASE(kEpiRowRms | kEpiRelu)
    ATPU_GEMV_CASE(kEpiRowRms | kEpiKvScatter)
    ATPU_GEMV_CASE(kEpiBias | kEpiKvScatter)
    ATPU_GEMV_CASE(kEpiRowLn | kEpiBias)
    ATPU_GEMV_CASE(kEpiRowLn | kEpiBias | kEpiGelu)
    ATPU_GEMV_CASE(kEpiRowLn | kEpiBias | kEpiKvScatter)
    ATPU_GEMV_CASE(kEpiBias | kEpiResidual | kEpiRowStats)
    ATPU_GEMV_CASE(kEpiBias | kEpiResidual | kEpiResLn)
    ATPU_GEMV_CASE(kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats)
    default:
      throw std::invalid_argument("atpu: unsupported GEMV epilogue " + std::to_string(g.epi));
  }
#undef ATPU_GEMV_CASE
#undef ATPU_GEMV_GO_KS
#undef ATPU_GEMV_GO
  ATPU_HIP_CHECK(hipGetLastError());
}

bool gemv_has_case(int epi) {
  switch (epi) {
    case 0: case kEpiBias: case kEpiResidual: case kEpiBias | kEpiResidual: case kEpiRelu: case kEpiBias | kEpiRelu:
    case kEpiBias | kEpiGelu: case kEpiRowRms: case kEpiRowRms | kEpiRelu: case kEpiRowRms | kEpiKvScatter:
    case kEpiBias | kEpiKvScatter: case kEpiRowLn | kEpiBias: case kEpiRowLn | kEpiBias | kEpiGelu:
    case kEpiRowLn | kEpiBias | kEpiKvScatter: case kEpiBias | kEpiResidual | kEpiRowStats:
    case kEpiBias | kEpiResidual | kEpiResLn: case kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats:
      return true;
    default:
      return false;
  }
}

}  // namespace

bool gemv_selected(int M, int N, int epi) {
  GemmArgs g;
  g.M = M;
  g.N = N;
  g.epi = epi;
  return gemv_ok(g) && gemv_has_case(epi);
}

void gemm_bf16(const GemmArgs& g, hipStream_t stream) {
  ATPU_CHECK(g.M > 0 && g.N > 0 && g.K > 0, "gemm: empty problem");
  ATPU_CHECK(g.K % kBK == 0, "gemm: K must be a multiple of 64");
  ATPU_CHECK(g.N % 4 == 0, "gemm: N must be a multiple of 4");
  ATPU_CHECK(g.lda % 8 == 0 && g.ldb % 8 == 0 && g.ldc % 4 == 0, "gemm: leading dims must keep 16-B rows");
  ATPU_CHECK(!((g.epi & kEpiRelu) && (g.epi & (kEpiGelu | kEpiTanh))), "gemm: one activation at most");
  ATPU_CHECK((reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.Bt) & 15) == 0,
             "gemm: A/Bt must be 16-byte aligned");
  ATPU_CHECK(!(g.epi & kEpiBias) || g.bias, "gemm: bias epilogue without bias");
  ATPU_CHECK(!(g.epi & kEpiResidual) || (g.R && g.ldr % 4 == 0), "gemm: residual epilogue without R");
  // 256x256 tiles once the grid fills the chip several times over; the 128x128
  // kernel (2 blocks/CU) covers small M (pooler, decode) and odd N.
  // 256x256 full-line-staged kernel once the grid fills the chip several
  // times over; the 128x128 kernel (2 blocks/CU) covers small M and odd N.
  // ATPU_GEMM_TILE=128|256 forces one (benchmarks/tests).
  const int forced = gemm_force_tile(-1);
  if (few_exact_ok(g) && !(g.epi & kEpiRowLn && !(g.epi & kEpiRowStats) && g.part_out)) {
    // batch-invariant mode, <= 16 rows: the dec kernel's exact arithmetic without its LDS ring
    if (g.epi & kEpiKvScatter)
      ATPU_CHECK(g.kv_cache && g.kv_step && g.kv_T > 0 && g.kv_col0 % 128 == 0 && g.kv_col0 > 0 && g.kv_col0 < g.N &&
                     g.kv_ld >= g.N - g.kv_col0 && g.kv_ld % 4 == 0,
                 "gemm: KvScatter needs a cache, a device step, kv_col0 % 128 == 0 and kv_ld >= N - kv_col0");
    ATPU_CHECK(!(g.epi & (kEpiRowRms | kEpiRowLn | kEpiResLn)) || g.rms_eps > 0.f, "gemm: RowRms / RowLn / ResLn need eps > 0");
    ATPU_CHECK(!(g.epi & kEpiRowLn) || (g.colsum && g.in_part && g.K <= 1024), "gemm: RowLn needs colsum, in_part, K <= 1024");
    ATPU_CHECK(!(g.epi & kEpiResLn) || (g.res_part && g.gamma && g.N <= 1024), "gemm: ResLn needs res_part, gamma, N <= 1024");
    ATPU_CHECK(!(g.epi & kEpiRowStats) || g.part_out, "gemm: RowStats needs part_out");
    launch_few_exact(g, stream);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  if (gemv_ok(g) && gemv_has_case(g.epi)) {  // <= 4 rows: weight-streaming GEMV (no split-K)
    launch_gemv(g, stream);
    return;
  }
  // the A-row statistics output of a RowLn GEMV (ops.linear row_ln_out) exists on the GEMV only
  ATPU_CHECK(!((g.epi & kEpiRowLn) && !(g.epi & kEpiRowStats) && g.part_out),
             "gemm: RowLn with an A-statistics output runs on the <= 4-row GEMV only");
  if (g.splits > 1) {
    ATPU_CHECK(!(g.epi & (kEpiRowRms | kEpiKvScatter | kEpiRowLn | kEpiResLn | kEpiRowStats)),
               "gemm: RowRms / RowLn / ResLn / KvScatter cannot split K");
    ATPU_CHECK(g.ws && (g.K / kBK) % g.splits == 0, "gemm: split-K needs a workspace and K/64 % splits == 0");
    launch_splitk(g, g.splits, gemm_dec_mode(-1) == 1 && skinny(g.M, g.N), stream);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  const int kernel256 = gemm_256_variant(-1);
  const bool big_ok = g.N % 256 == 0 && g.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0 &&
                      (!(g.epi & kEpiResidual) || (g.ldr % 8 == 0 && (reinterpret_cast<uintptr_t>(g.R) & 15) == 0));
  if (g.epi & (kEpiInNorm | kEpiResNorm | kEpiStatsOut)) {
    // LayerNorm folding: persistent full-line kernel only (ops.linear checks the same
    // conditions and falls back to a materialised LayerNorm)
    const int fe = g.epi;
    ATPU_CHECK(fe == (kEpiBias | kEpiInNorm) || fe == (kEpiBias | kEpiInNorm | kEpiGelu) ||
                   fe == (kEpiBias | kEpiResidual | kEpiStatsOut) ||
                   fe == (kEpiBias | kEpiResidual | kEpiResNorm | kEpiStatsOut),
               "gemm: unsupported LayerNorm-folding epilogue " + std::to_string(fe));
    ATPU_CHECK(big_ok && g.M % 256 == 0 && g.K % 256 == 0 && g.K >= 256, "gemm: LN folding needs M, N, K % 256 == 0");
    ATPU_CHECK(kernel256 >= 3, "gemm: LN folding needs the full-line 256x256 kernel (ATPU_GEMM_256=n|l)");
    ATPU_CHECK(!(fe & kEpiInNorm) || (g.in_fin && g.colsum), "gemm: InNorm needs in_fin and colsum");
    // staging offsets are 32-bit byte offsets from A / Bt
    ATPU_CHECK((size_t)g.M * g.lda * 2 < (1ull << 32) && (size_t)g.N * g.ldb * 2 < (1ull << 32),
               "gemm: LN folding needs A and Bt under 4 GiB");
    ATPU_CHECK(!(fe & kEpiResNorm) || (g.res_fin && g.gamma), "gemm: ResNorm needs res_fin and gamma");
    ATPU_CHECK(!(fe & kEpiStatsOut) || g.part_out, "gemm: StatsOut needs part_out");
    if (kernel256 == 3) launch_256s<false, true>(g, stream);
    else launch_256s<true, true>(g, stream);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  if (g.epi & kEpiKvScatter) {
    // decode QKV straight into the KV cache (128x128 / dec kernels; every 64- and
    // 128-column tile must be all Q or all K|V)
    const int fe = g.epi & ~kEpiKvScatter;
    ATPU_CHECK(fe == kEpiRowRms || fe == kEpiBias || fe == (kEpiRowLn | kEpiBias),
               "gemm: unsupported KvScatter epilogue " + std::to_string(g.epi));
    ATPU_CHECK(g.kv_cache && g.kv_step && g.kv_T > 0 && g.kv_col0 % 128 == 0 && g.kv_col0 > 0 && g.kv_col0 < g.N &&
                   g.kv_ld >= g.N - g.kv_col0 && g.kv_ld % 4 == 0,
               "gemm: KvScatter needs a cache, a device step, kv_col0 % 128 == 0 and kv_ld >= N - kv_col0");
  }
  if (g.epi & (kEpiRowLn | kEpiResLn | kEpiRowStats)) {
    // decode LayerNorm folding (BART decoder steps): producers write per-row partials
    // (RowStats), RowLn consumers normalise their A rows and ResLn consumers their
    // residual rows from those partials
    const int fe = g.epi & ~kEpiKvScatter;
    ATPU_CHECK(fe == (kEpiRowLn | kEpiBias) || fe == (kEpiRowLn | kEpiBias | kEpiGelu) ||
                   (!(g.epi & kEpiKvScatter) && (fe == (kEpiBias | kEpiResidual | kEpiResLn | kEpiRowStats) ||
                                                 fe == (kEpiBias | kEpiResidual | kEpiRowStats) ||
                                                 fe == (kEpiBias | kEpiResidual | kEpiResLn))),
               "gemm: unsupported decode LayerNorm-folding epilogue " + std::to_string(g.epi));
    ATPU_CHECK(!(fe & kEpiRowLn) || (g.colsum && g.in_part && g.K <= 1024), "gemm: RowLn needs colsum, in_part, K <= 1024");
    ATPU_CHECK(!(fe & kEpiResLn) || (g.res_part && g.gamma && g.N <= 1024 && g.N % 32 == 0),
               "gemm: ResLn needs res_part, gamma, N <= 1024");
    ATPU_CHECK(!(fe & (kEpiRowLn | kEpiResLn)) || g.rms_eps > 0.f, "gemm: RowLn / ResLn need eps > 0");
    ATPU_CHECK(!(fe & kEpiRowStats) || (g.part_out && g.N % 32 == 0), "gemm: RowStats needs part_out and N % 32 == 0");
  }
  if (g.epi & (kEpiRowRms | kEpiKvScatter | kEpiRowLn | kEpiResLn | kEpiRowStats)) {
    // RMSNorm / LayerNorm folded into the GEMM (T5 / BART decoder steps): the 128x128 and
    // skinny kernels sum the A rows' statistics over their whole K loop (no split-K)
    const int fe = g.epi & ~(kEpiRowRms | kEpiKvScatter);
    ATPU_CHECK(fe == 0 || fe == kEpiRelu || fe == kEpiOutF32 || fe == kEpiBias ||
                   (g.epi & (kEpiRowLn | kEpiResLn | kEpiRowStats)),
               "gemm: unsupported RowRms / KvScatter epilogue " + std::to_string(g.epi));
    ATPU_CHECK(!(g.epi & kEpiRowRms) || g.rms_eps > 0.f, "gemm: RowRms needs rms_eps > 0");
    if (forced == 64 || (forced != 128 && gemm_dec_mode(-1) == 1 && skinny(g.M, g.N)))
      launch_dec(g, stream);
    else
      launch_tile<128, 128, 2, 2>(g, stream);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  const bool use_big = !(g.epi & kEpiOutF32) &&
                       (forced ? (forced == 256 && big_ok) : (g.M >= 2048 && big_ok && big_fills(g.M, g.N)));
  // 256s counts its epilogue's stores in the next tile's waits: whole row tiles only
  const bool persistent_ok = g.M % 256 == 0;
  if (use_big && persistent_ok && kernel256 >= 2) {
    if (kernel256 == 3) launch_256s<false, true>(g, stream);
    else launch_256s<true, true>(g, stream);
  } else if (use_big && kernel256 != 0)
    launch_256p(g, stream);  // M % 256 != 0 (or the per-tile schedule forced)
  else if ((forced == 64 || (!forced && gemm_dec_mode(-1) == 1 && skinny(g.M, g.N))))
    launch_dec(g, stream);
  else
    launch_tile<128, 128, 2, 2>(g, stream);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
