// Fused decode LM head + beam top-k (replaces the fp32-logit
// GEMM + beam_topk_rows pair of decode.hip for the device-selection decode loop).
//
// The LM head of a beam-search step is [rows, d] x [V, d]^T (rows = docs x beams,
// V = 32128 / 50264): 50-105 GFLOP whose output only feeds a per-row log-softmax
// normaliser and the row's top-2nb tokens. Writing the fp32 logits (206 MB per
// BART step) and reading them back in a separate top-k pass cost 175 + 74 us.
// Here the logits never leave the CU:
//
//  lm_head_topk_kernel  one 128x128 (rows x vocab) tile per workgroup, K in full:
//    * 4 waves, each 32 rows x 128 vocab columns (2 x 8 MFMA 16x16x32 fragments),
//      so all 128 values of a row sit in the 4 lanes l, l^16, l^32, l^48 of ONE
//      wave: every row reduction is two register permlane swaps, no LDS;
//    * NST-deep LDS ring fed by LDS-DMA (counted vmcnt, one raw barrier per K-tile),
//      M-fastest tile order under the XCD remap: the M tiles of one vocab panel
//      run on one XCD, so each weight panel comes from HBM once;
//    * epilogue per (row, tile): max and sum exp(x - max) over every column (the
//      log-softmax normaliser covers banned tokens, as HF applies the processors
//      after log_softmax), then the candidate set: values >= L, where L is the
//      8th largest of the 16 lane-local top-4 values (v_med3 insertion, 4 VALU
//      per value, no indices). Any 8 values >= L prove that the tile's 8 best
//      allowed values are >= L, so the set holds the tile's exact top 8
//      (ties at L included). It has 8.1 values on average and more than 16 with
//      probability < 1e-5 on Gaussian logits; then (or on massive ties) the
//      wave falls back to 8 exact argmax rounds over (value desc, index asc).
//      Banned tokens (a per-row bitmap, built once per step by ban_bitmap_kernel
//      from the ban list and the device token history) and the min-length EOS
//      mask only drop values from the candidate set.
//    Output per (row, tile): {max, sumexp, count} + up to 16 (value, token) pairs.
//  lm_head_merge_kernel  one workgroup per row: log-sum-exp over the tiles and
//    the exact top-K (K <= 8) of the candidates, written exactly like
//    beam_topk_rows (score = logit - lse + beam score), so beam_select consumes
//    it unchanged.
//
// Measured (tools/bench_kernels.py --only lm_bart,lm_t5, 1024 rows): BART 50264 x 1024
// 187 us against 223 us for the logits GEMM + beam_topk_rows pair (the GEMM alone
// 170 us: the epilogue is nearly free, hidden by the second workgroup per CU); T5
// 32128 x 768 110 vs 135 us. The mainloop is the limit (~0.6 PF): the persistent
// 256x256 kernel reaches 1 PF on this shape with bf16 output, but with this epilogue
// (~12 VALU per logit, barrier-locked with the ping-pong partner) it ran 267 us, and
// 256-row tiles / deeper rings / 2x2 wave grids here were all slower (dev builds,
// ATPU_LM_CFG 1-5; docs/PERF_NOTES.md).
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/topk.h"

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <utility>

namespace atpu {
namespace {

constexpr int kBN = 128, kBK = 64;          // vocab columns per tile (= per wave), K per stage
constexpr int kRowB = kBK * 2;                // 128-B staged row
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue of one 16-row fragment of a wave's WC = 16 TN vocabulary columns (lane (frow,
// fchunk): row m, columns c0 + j*16 + fchunk*4 + e): RMS scale / bias, the row's max and
// sum exp over every column, bans / EOS mask / past-V columns out of the candidates, then
// the slab's header and candidate set (tile_row_emit).
template <bool RMS, bool BIAS, bool BANS, int TN>
__device__ __forceinline__ void lm_row_emit(const f32x4 (&acc)[TN], float ssq, int m, int fchunk, int c0, int M, int V,
                                            int K, const float* __restrict__ bias, float rms_eps,
                                            const uint32_t* __restrict__ ban_bits, int ban_ld, int eos, int mask_eos,
                                            int nslab, float4* __restrict__ hdr, float2* __restrict__ cand) {
  constexpr int WC = TN * 16;
  const int slab = c0 / WC;
  const bool tail = c0 + WC > V;
  const bool eos_here = mask_eos && eos >= c0 && eos < c0 + WC;
  f32x4 bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = c0 + j * 16 + fchunk * 4;
    bv[j] = (BIAS && n < V) ? *reinterpret_cast<const f32x4*>(bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  {
    const bool live = m < M;
    const float rs = RMS ? __builtin_amdgcn_rsqf(lane_rows_sum(ssq) * (1.f / K) + rms_eps) : 1.f;
    float v[TN][4];
    float mx = -FLT_MAX;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = acc[j][e];
        if constexpr (RMS) x *= rs;
        if constexpr (BIAS) x += bv[j][e];
        if (tail && c0 + j * 16 + fchunk * 4 + e >= V) x = -FLT_MAX;
        v[j][e] = x;
        mx = fmaxf(mx, x);
      }
    const float rmax = lane_rows_max(mx);
    const float mb = rmax * kLog2e;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += __builtin_amdgcn_exp2f(fmaf(v[j][e], kLog2e, -mb));
    s = lane_rows_sum(s);

    // selection values: banned / masked EOS / past-V columns -> -FLT_MAX
    if constexpr (BANS) {
      // the slab's WC / 32 bitmap words of row m (16-B rows, 8-B aligned slabs)
      uint32_t wd[WC / 32];
      const uint32_t* bp = ban_bits + (size_t)min(m, M - 1) * ban_ld + c0 / 32;
      if constexpr (WC == 128) {
        const uint4 q = *reinterpret_cast<const uint4*>(bp);
        wd[0] = q.x, wd[1] = q.y, wd[2] = q.z, wd[3] = q.w;
      } else {
        const uint2 q = *reinterpret_cast<const uint2*>(bp);
        wd[0] = q.x, wd[1] = q.y;
      }
      uint32_t any = 0u;
#pragma unroll
      for (int w = 0; w < WC / 32; ++w) any |= wd[w];
      if (__ballot(any != 0u)) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if ((wd[j >> 1] >> ((j & 1) * 16 + fchunk * 4 + e)) & 1u) v[j][e] = -FLT_MAX;
      }
    }
    if (eos_here) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c0 + j * 16 + fchunk * 4 + e == eos) v[j][e] = -FLT_MAX;
    }
    const size_t slot = (size_t)m * nslab + slab;
    tile_row_emit<TN>(v, c0, fchunk, live, rmax, s, hdr + slot, cand + slot * kTileCand);
  }
}

template <bool RMS, bool BIAS, bool BANS, int BM, int NST, int WN>
__global__ __launch_bounds__(BM / 32 * 64, (BM + kBN) * kRowB * NST <= 80 * 1024 ? 2 : 1) void lm_head_topk_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ W, int ldw, const float* __restrict__ bias,
    float rms_eps, int M, int V, int K, const uint32_t* __restrict__ ban_bits, int ban_ld, int eos, int mask_eos,
    float4* __restrict__ hdr, float2* __restrict__ cand) {
  constexpr int NW = BM / 32;                 // waves
  constexpr int WM = NW / WN;                 // wave grid WM x WN
  constexpr int WR = BM / WM, WC = kBN / WN;  // rows x vocab columns per wave (= one partial slab)
  constexpr int TM = WR / 16, TN = WC / 16;
  constexpr int kStage = (BM + kBN) * kRowB;  // ring slot: A rows 0..BM-1, vocab rows BM..
  constexpr int kLps = (BM + kBN) / 8 / NW;   // LDS-DMA instructions per wave per slot
  static_assert((BM + kBN) % (8 * NW) == 0 && BM % (8 * NW) == 0 && NW % WN == 0, "stage split");
  __shared__ __attribute__((aligned(16))) char lds[NST * kStage];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = (M + BM - 1) / BM;
  const int ntn = (V + kBN - 1) / kBN;
  const int nslab = (V + WC - 1) / WC;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile % ntm) * BM;
  const int n0 = (tile / ntm) * kBN;

  // staged rows 0..BM-1: A rows m0.., BM..BM+127: vocab rows n0.. (clamped; masked in the epilogue)
  const int srow = lane >> 3, spos = lane & 7;
  const bf16* src[kLps];
#pragma unroll
  for (int i = 0; i < kLps; ++i) {
    const int r = (i * NW + wave) * 8 + srow;  // A rows for i < BM / (8 NW) (wave-uniform)
    src[i] = r < BM ? A + (size_t)min(m0 + r, M - 1) * lda + swz(r, spos) * 8
                    : W + (size_t)min(n0 + r - BM, V - 1) * ldw + swz(r, spos) * 8;
  }
  auto stage = [&](int kt, int slot) {
    char* base = lds + slot * kStage;
#pragma unroll
    for (int i = 0; i < kLps; ++i) glds16(src[i] + kt * kBK, base + (i * NW + wave) * 8 * kRowB);
  };

  const int frow = lane & 15, fchunk = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssq[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) ssq[i] = 0.f;
  auto compute = [&](int slot) {
    const char* base = lds + slot * kStage;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WR + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowB + swz(r, ks * 4 + fchunk) * 16);
        if constexpr (RMS) ssq[i] = sumsq_chunk(af[i], ssq[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = BM + wn * WC + j * 16 + frow;
        bw[j] = *reinterpret_cast<const bf16x8*>(base + r * kRowB + swz(r, ks * 4 + fchunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = K / kBK;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) stage(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NST - 1 <= nk)
      wait_vm<(NST - 2) * kLps>();
    else
      wait_vm<0>();
    // raw barrier: __syncthreads() would add a vmcnt(0) and drain the ring. Every wave's
    // DMA for slot kt has landed; slot (kt-1) % NST is free (its reads fed retired MFMAs).
    asm volatile("s_barrier" ::: "memory");
    if (kt + NST - 1 < nk) stage(kt + NST - 1, (kt + NST - 1) % NST);
    compute(kt % NST);
  }

  // ------------------------------------------------------------------ epilogue
  // lane (frow, fchunk) holds rows wm*WR + i*16 + frow, columns c0 + j*16 + fchunk*4 + e
  const int c0 = n0 + wn * WC;  // this wave's slab
  if (c0 >= V) return;          // wholly past the vocabulary (wave-uniform)
#pragma unroll
  for (int i = 0; i < TM; ++i)
    lm_row_emit<RMS, BIAS, BANS, TN>(acc[i], ssq[i], m0 + wm * WR + i * 16 + frow, fchunk, c0, M, V, K, bias, rms_eps,
                                     ban_bits, ban_ld, eos, mask_eos, nslab, hdr, cand);
}

// Few rows (<= 16: a 1-document decode step) and <= one panel per CU: lm_head_topk_kernel streams each 128-column
// panel through a 2-slot LDS ring, one 64-deep K-tile per barrier, with the A tile's 128
// staged rows mostly copies of the 4 real ones -- 20 us per T5 step for 49 MB of weights.
// Here 8 waves split K (K / 8 = 96 or 128 per wave) and every lane issues ALL its operand
// loads at once, straight from global memory into MFMA fragment registers (no LDS, no
// barrier in the loop): 16-B weight chunks of the panel's 128 rows, the A rows from L2.
// Each wave's [16 rows x 128 columns] partial goes through LDS, wave w sums column block w
// over the 8 waves (fixed order), and wave 0 runs the same epilogue (lm_row_emit) on the
// one 16-row fragment: the same slab format, so lm_head_merge* take it unchanged.
constexpr int kFewRows = 16, kFewWaves = 8, kFewKs = 4;  // rows, waves (K split), max k-steps of 32 per wave

template <bool RMS, bool BIAS, bool BANS>
__global__ __launch_bounds__(kFewWaves * 64) void lm_head_few_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ W, int ldw, const float* __restrict__ bias,
    float rms_eps, int M, int V, int K, const uint32_t* __restrict__ ban_bits, int ban_ld, int eos, int mask_eos,
    float4* __restrict__ hdr, float2* __restrict__ cand) {
  constexpr int TN = kBN / 16;
  __shared__ f32x4 red[kFewWaves][TN][64];  // 64 KiB
  __shared__ float rsq[kFewWaves][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fchunk = lane >> 4;
  const int n0 = blockIdx.x * kBN;
  const int kw = K / kFewWaves;  // host: K % (32 * kFewWaves) == 0, kw <= 32 * kFewKs
  const int k0 = wave * kw + fchunk * 8;
  const bf16* ar = A + (size_t)min(frow, M - 1) * lda + k0;
  bf16x8 af[kFewKs], bw[kFewKs][TN];
#pragma unroll
  for (int ks = 0; ks < kFewKs; ++ks) {
    if (ks * 32 < kw) {  // wave-uniform
      af[ks] = *reinterpret_cast<const bf16x8*>(ar + ks * 32);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[ks][j] = *reinterpret_cast<const bf16x8*>(W + (size_t)min(n0 + j * 16 + frow, V - 1) * ldw + k0 + ks * 32);
    }
  }
  f32x4 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssq = 0.f;
#pragma unroll
  for (int ks = 0; ks < kFewKs; ++ks) {
    if (ks * 32 < kw) {
      if constexpr (RMS) ssq = sumsq_chunk(af[ks], ssq);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks][j], af[ks], acc[j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) red[wave][j][lane] = acc[j];
  if constexpr (RMS) rsq[wave][lane] = ssq;
  __syncthreads();
  {  // column block j = wave, summed over the waves in order
    f32x4 t = red[0][wave][lane];
#pragma unroll
    for (int x = 1; x < kFewWaves; ++x) t += red[x][wave][lane];
    red[0][wave][lane] = t;
  }
  __syncthreads();
  if (wave != 0 || n0 >= V) return;
#pragma unroll
  for (int j = 0; j < TN; ++j) acc[j] = red[0][j][lane];
  if constexpr (RMS) {
    ssq = rsq[0][lane];
#pragma unroll
    for (int x = 1; x < kFewWaves; ++x) ssq += rsq[x][lane];
  }
  lm_row_emit<RMS, BIAS, BANS, TN>(acc, ssq, frow, fchunk, n0, M, V, K, bias, rms_eps, ban_bits, ban_ld, eos, mask_eos,
                                   (V + kBN - 1) / kBN, hdr, cand);
}

constexpr int kMergeThreads = 256;

__global__ __launch_bounds__(kMergeThreads) void lm_head_merge_kernel(const float4* __restrict__ hdr,
                                                                       const float2* __restrict__ cand, int ntn,
                                                                       const float* __restrict__ beam_scores, int K,
                                                                       float* __restrict__ out_score,
                                                                       int32_t* __restrict__ out_token) {
  constexpr int NW = kMergeThreads / 64;
  static_assert(NW * kTileSel <= 64, "wave 0 merges every wave's top kTileSel in one pass");
  __shared__ float wm[NW], wsum[NW];
  __shared__ float cv[NW * kTileSel];
  __shared__ int ci[NW * kTileSel];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float4* h = hdr + (size_t)row * ntn;
  const float2* c = cand + (size_t)row * ntn * kTileCand;
  float mx = -FLT_MAX, sm = 0.f;
  float tv[kTileSel];
  int ti[kTileSel];
#pragma unroll
  for (int r = 0; r < kTileSel; ++r) {
    tv[r] = -FLT_MAX;
    ti[r] = 0x7fffffff;
  }
  // two tiles per thread per round, every load of a round in flight at once: both headers
  // and all 16 candidate slots of each tile (16-B loads). A per-candidate load loop
  // serialised one memory latency per candidate (43 us per BART step).
  const float4* c4 = reinterpret_cast<const float4*>(c);
  for (int t0 = tid; t0 < ntn; t0 += 2 * kMergeThreads) {
    const int t1 = t0 + kMergeThreads;
    const float4 p0 = h[t0];
    const float4 p1 = t1 < ntn ? h[t1] : float4{-FLT_MAX, 0.f, 0.f, 0.f};
    const int n0 = __float_as_int(p0.z), n1 = __float_as_int(p1.z);
    float4 e0[kTileCand / 2], e1[kTileCand / 2];
    // slots 0-7 unconditionally (slots past the count hold stale data, masked below), 8-15
    // in one block only when a tile has more than 8 (~9 % of tiles): a load under `2q < n`
    // per slot became a branch with a vmcnt(0) at each join (39 us per step)
    const size_t b0 = (size_t)t0 * (kTileCand / 2), b1 = (size_t)min(t1, ntn - 1) * (kTileCand / 2);
#pragma unroll
    for (int q = 0; q < kTileCand / 4; ++q) {
      e0[q] = c4[b0 + q];
      e1[q] = c4[b1 + q];
    }
#pragma unroll
    for (int q = kTileCand / 4; q < kTileCand / 2; ++q) e0[q] = e1[q] = float4{-FLT_MAX, 0.f, -FLT_MAX, 0.f};
    if (n0 > kTileCand / 2 || n1 > kTileCand / 2) {
#pragma unroll
      for (int q = kTileCand / 4; q < kTileCand / 2; ++q) {
        e0[q] = c4[b0 + q];
        e1[q] = c4[b1 + q];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float4 p = u ? p1 : p0;
      if (p.x > mx) {
        sm = sm * __expf(mx - p.x) + p.y;
        mx = p.x;
      } else if (p.x > -FLT_MAX) {
        sm += p.y * __expf(p.x - mx);
      }
    }
#pragma unroll
    for (int q = 0; q < kTileCand; ++q) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 e = u ? e1[q / 2] : e0[q / 2];
        const int n = u ? n1 : n0;
        const float x = (q & 1) ? e.z : e.x;
        const int id = __float_as_int((q & 1) ? e.w : e.y);
        if (q < n && better(x, id, tv[kTileSel - 1], ti[kTileSel - 1])) list_insert<kTileSel>(tv, ti, x, id);
      }
    }
  }
  const float gm0 = wave_max(mx);
  float sa = (mx == -FLT_MAX) ? 0.f : sm * __expf(mx - gm0);
  sa = wave_sum(sa);
  float rv;
  int ri;
  wave_topk<kTileSel>(tv, ti, rv, ri);
  if (lane == 0) {
    wm[w] = gm0;
    wsum[w] = sa;
  }
  if (lane < kTileSel) {
    cv[w * kTileSel + lane] = rv;
    ci[w * kTileSel + lane] = ri;
  }
  __syncthreads();
  if (w == 0) {
    float gm = -FLT_MAX;
#pragma unroll
    for (int x = 0; x < NW; ++x) gm = fmaxf(gm, wm[x]);
    float gs = 0.f;
#pragma unroll
    for (int x = 0; x < NW; ++x) gs += wsum[x] * __expf(wm[x] - gm);
    const float shift = beam_scores[row] - gm - __logf(gs);
#pragma unroll
    for (int r = 0; r < kTileSel; ++r) {
      tv[r] = -FLT_MAX;
      ti[r] = 0x7fffffff;
    }
    if (lane < NW * kTileSel) list_insert<kTileSel>(tv, ti, cv[lane], ci[lane]);
    wave_topk<kTileSel>(tv, ti, rv, ri);
    if (lane < K) {
      out_score[(size_t)row * K + lane] = rv == -FLT_MAX ? -FLT_MAX : rv + shift;
      out_token[(size_t)row * K + lane] = ri;
    }
  }
}

// Few rows (a 1-document step: 4-32 rows, one workgroup each on an idle chip): the merge above
// is a dependent chain per thread (16-32 candidate insertions of 8 compare-selects, then two
// 8-round wave arg-max passes at one wave per SIMD) -- 14.6-16.3 us per call. Here 16 waves
// per row and 4 threads per tile, each inserting its tile's 4 candidate slots: the
// insertion chain is 4 long; the per-wave passes run side by side; wave 0 merges the 16
// waves' top kTileSel (two per lane). Same selection (value desc, token asc) and output.
constexpr int kMergeFewThreads = 1024;
constexpr int kMergeFewRows = 32;  // rows up to which lm_head_topk merges with it

__global__ __launch_bounds__(kMergeFewThreads) void lm_head_merge_few_kernel(const float4* __restrict__ hdr,
                                                                              const float2* __restrict__ cand, int ntn,
                                                                              const float* __restrict__ beam_scores,
                                                                              int K, float* __restrict__ out_score,
                                                                              int32_t* __restrict__ out_token) {
  constexpr int NW = kMergeFewThreads / 64;
  constexpr int kPart = kTileCand / 4;  // candidate slots per thread
  static_assert(NW * kTileSel == 128, "wave 0 merges two per lane");
  __shared__ float wm[NW], wsum[NW];
  __shared__ float cv[NW * kTileSel];
  __shared__ int ci[NW * kTileSel];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int part = tid & 3;
  const float4* h = hdr + (size_t)row * ntn;
  const float4* c4 = reinterpret_cast<const float4*>(cand + (size_t)row * ntn * kTileCand);
  float mx = -FLT_MAX, sm = 0.f;
  float tv[kTileSel];
  int ti[kTileSel];
#pragma unroll
  for (int r = 0; r < kTileSel; ++r) {
    tv[r] = -FLT_MAX;
    ti[r] = 0x7fffffff;
  }
  for (int t = tid >> 2; t < ntn; t += kMergeFewThreads / 4) {
    const float4 p = h[t];
    // slots part*4 .. part*4+3: two 16-B loads, issued with the header's
    const float4 e0 = c4[(size_t)t * (kTileCand / 2) + part * 2];
    const float4 e1 = c4[(size_t)t * (kTileCand / 2) + part * 2 + 1];
    const int n = __float_as_int(p.z);
    if (part == 0) {
      if (p.x > mx) {
        sm = sm * __expf(mx - p.x) + p.y;
        mx = p.x;
      } else if (p.x > -FLT_MAX) {
        sm += p.y * __expf(p.x - mx);
      }
    }
#pragma unroll
    for (int q = 0; q < kPart; ++q) {
      const float4 e = q < 2 ? e0 : e1;
      const float x = (q & 1) ? e.z : e.x;
      const int id = __float_as_int((q & 1) ? e.w : e.y);
      if (part * kPart + q < n && better(x, id, tv[kTileSel - 1], ti[kTileSel - 1])) list_insert<kTileSel>(tv, ti, x, id);
    }
  }
  const float gm0 = wave_max(mx);
  float sa = (mx == -FLT_MAX) ? 0.f : sm * __expf(mx - gm0);
  sa = wave_sum(sa);
  float rv;
  int ri;
  wave_topk<kTileSel>(tv, ti, rv, ri);
  if (lane == 0) {
    wm[w] = gm0;
    wsum[w] = sa;
  }
  if (lane < kTileSel) {
    cv[w * kTileSel + lane] = rv;
    ci[w * kTileSel + lane] = ri;
  }
  __syncthreads();
  if (w == 0) {
    float gm = -FLT_MAX;
#pragma unroll
    for (int x = 0; x < NW; ++x) gm = fmaxf(gm, wm[x]);
    float gs = 0.f;
#pragma unroll
    for (int x = 0; x < NW; ++x) gs += wsum[x] * __expf(wm[x] - gm);
    const float shift = beam_scores[row] - gm - __logf(gs);
#pragma unroll
    for (int r = 0; r < kTileSel; ++r) {
      tv[r] = -FLT_MAX;
      ti[r] = 0x7fffffff;
    }
    list_insert<kTileSel>(tv, ti, cv[lane], ci[lane]);
    list_insert<kTileSel>(tv, ti, cv[lane + 64], ci[lane + 64]);
    wave_topk<kTileSel>(tv, ti, rv, ri);
    if (lane < K) {
      out_score[(size_t)row * K + lane] = rv == -FLT_MAX ? -FLT_MAX : rv + shift;
      out_token[(size_t)row * K + lane] = ri;
    }
  }
}

// Per-row ban bitmap (bit t of row r set = token t banned): the explicit ban list
// (-1 padded) and/or the no-repeat-n-gram bans of the device token history, built
// in LDS and written out whole (rows of ban_ld words, zero past V).
__global__ __launch_bounds__(256) void ban_bitmap_kernel(int V, int ban_ld, const int32_t* __restrict__ bans,
                                                         int nbmax, const int32_t* __restrict__ seq, int seq_stride,
                                                         int cur, int ngram, uint32_t* __restrict__ bits) {
  extern __shared__ uint32_t bb[];
  const int row = blockIdx.x, tid = threadIdx.x;
  for (int w = tid; w < ban_ld; w += 256) bb[w] = 0u;
  __syncthreads();
  for (int b = tid; b < nbmax; b += 256) {
    const int t = bans[(size_t)row * nbmax + b];
    if (t >= 0 && t < V) atomicOr(&bb[t >> 5], 1u << (t & 31));
  }
  if (ngram > 0 && cur >= ngram) {
    const int32_t* sr = seq + (size_t)row * seq_stride;
    for (int i = tid; i + ngram <= cur; i += 256) {
      bool eq = true;
      for (int e = 0; e + 1 < ngram; ++e) eq = eq && sr[i + e] == sr[cur - ngram + 1 + e];
      const int t = sr[i + ngram - 1];
      if (eq && t >= 0 && t < V) atomicOr(&bb[t >> 5], 1u << (t & 31));
    }
  }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(bits + (size_t)row * ban_ld);
  for (int w = tid; w < ban_ld / 4; w += 256) dst[w] = uint4{bb[4 * w], bb[4 * w + 1], bb[4 * w + 2], bb[4 * w + 3]};
}

int ban_ld_words(int V) { return ((V + 31) / 32 + 3) & ~3; }  // 16-B rows

}  // namespace

int lm_head_stages(int set) {
  // fused LM head tile / LDS ring / wave grid (rows x vocab per workgroup). Release builds
  // run config 0; dev builds (python -m agent_tpu_amd.csrc.build --dev) also the measured
  // alternatives (ATPU_LM_CFG, tools/bench_kernels.py --only lm_bart,lm_t5; docs/PERF_NOTES.md):
  //   0: 128x128, 2 slots (64 KiB, two workgroups per CU), 4 waves of 32 rows x 128 columns
  //   1: 128x128, 4 slots (128 KiB)   2: 256x128, 2 slots (96 KiB)   3: 256x128, 3 slots (144 KiB)
  //   4: as 0 with 2x2 waves of 64 x 64 (fewer LDS fragment reads per MFMA; 64-column slabs)
  //   5: as 2 with 4x2 waves of 64 x 64
  (void)set;
  return 0;
}

// workspace: per-slab headers and candidates (slabs of 64 columns at the finest), the ban bitmap
size_t lm_head_ws_bytes(int M, int V) {
  const size_t slabs = (size_t)M * ((V + 63) / 64);
  return slabs * sizeof(float4) + slabs * kTileCand * sizeof(float2) + (size_t)M * ban_ld_words(V) * 4;
}

void lm_head_topk(const bf16* A, int lda, const bf16* W, int ldw, const float* bias, float rms_eps, int M, int V,
                  int K, int topk, const float* beam_scores, int eos, int mask_eos, const int32_t* bans, int nbmax,
                  const int32_t* seq, int seq_stride, int cur, int ngram, void* ws, float* out_score,
                  int32_t* out_token, hipStream_t stream) {
  ATPU_CHECK(M > 0 && V > 0 && K > 0 && K % kBK == 0, "lm_head_topk: K must be a positive multiple of 64");
  ATPU_CHECK(V % 4 == 0, "lm_head_topk: V must be a multiple of 4");
  ATPU_CHECK(topk >= 1 && topk <= kTileSel && topk <= V, "lm_head_topk: 1 <= k <= 8");
  ATPU_CHECK(lda % 8 == 0 && ldw % 8 == 0 && lda >= K && ldw >= K, "lm_head_topk: 16-B rows of at least K");
  ATPU_CHECK((reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(bias) & 15) == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0,
             "lm_head_topk: A, W, bias and the workspace must be 16-byte aligned");
  ATPU_CHECK(ws && beam_scores && out_score && out_token, "lm_head_topk: null buffer");
  ATPU_CHECK(nbmax >= 0 && (nbmax == 0 || bans), "lm_head_topk: ban list");
  ATPU_CHECK(ngram <= 0 || (seq && cur <= seq_stride), "lm_head_topk: n-gram bans need the token history [rows, >= cur]");
  const int cfg = lm_head_stages(-1);
  const int wc = (cfg >= 4) ? 64 : 128;  // vocabulary columns per partial slab (the wave's columns)
  const int nslab = (V + wc - 1) / wc;
  const int ntn = (V + kBN - 1) / kBN;
  ATPU_CHECK((long long)((M + 127) / 128) * ntn < (1ll << 31), "lm_head_topk: grid too large");
  if (ngram > 0 && cur < ngram) ngram = 0;
  const bool any_bans = nbmax > 0 || ngram > 0;
  const int ld = ban_ld_words(V);
  const size_t slabs = (size_t)M * ((V + 63) / 64);
  float4* hdr = reinterpret_cast<float4*>(ws);
  float2* cand = reinterpret_cast<float2*>(hdr + slabs);
  uint32_t* bits = reinterpret_cast<uint32_t*>(cand + slabs * kTileCand);
  if (any_bans) {
    ATPU_CHECK((size_t)ld * 4 <= 64 * 1024, "lm_head_topk: vocabulary too large for the ban bitmap");
    hipLaunchKernelGGL(ban_bitmap_kernel, dim3(M), dim3(256), (size_t)ld * 4, stream, V, ld, bans, nbmax, seq,
                       seq_stride, cur, ngram, bits);
  }
  const bool rms = rms_eps > 0.f, has_bias = bias != nullptr;
  ATPU_CHECK(!(rms && has_bias), "lm_head_topk: RMSNorm folding and a bias together are not instantiated");
  // few rows, and one workgroup per CU covers the vocabulary (T5's 251 panels; BART's 393 would
  // run in two rounds at one 8-wave workgroup per CU: 44 vs 40 us per call, measured)
  // (batch_invariant: the per-row tiles of lm_head_topk_kernel and the one merge kernel for every M)
  const bool inv = batch_invariant(-1) != 0;
  const bool few = !inv && M <= kFewRows && K % (32 * kFewWaves) == 0 && K <= 32 * kFewWaves * kFewKs &&
                   wc == kBN && ntn <= num_cus();
  if (few) {
#define ATPU_LMF(R, B, X)                                                                                             \
  hipLaunchKernelGGL((lm_head_few_kernel<R, B, X>), dim3(ntn), dim3(kFewWaves * 64), 0, stream, A, lda, W, ldw, bias, \
                     rms_eps, M, V, K, bits, ld, eos, mask_eos, hdr, cand)
    if (rms) {
      if (any_bans) ATPU_LMF(true, false, true); else ATPU_LMF(true, false, false);
    } else if (has_bias) {
      if (any_bans) ATPU_LMF(false, true, true); else ATPU_LMF(false, true, false);
    } else {
      if (any_bans) ATPU_LMF(false, false, true); else ATPU_LMF(false, false, false);
    }
#undef ATPU_LMF
  } else {
#define ATPU_LM(R, B, X, BM, N, WN)                                                                              \
  hipLaunchKernelGGL((lm_head_topk_kernel<R, B, X, BM, N, WN>), dim3(((M + BM - 1) / BM) * ntn), dim3(BM / 32 * 64), \
                     0, stream, A, lda, W, ldw, bias, rms_eps, M, V, K, bits, ld, eos, mask_eos, hdr, cand)
  // (a 4-slot ring for the one-row-tile step measured within noise for T5 and slower for BART,
  // profiles/lm_head_small_ring_ab_r04.txt)
#define ATPU_LM_CFG(R, B, X) ATPU_LM(R, B, X, 128, 2, 1);
#define ATPU_LM_BANS(R, B)        \
  if (any_bans) {                 \
    ATPU_LM_CFG(R, B, true)       \
  } else {                        \
    ATPU_LM_CFG(R, B, false)      \
  }
  if (rms) {
    ATPU_LM_BANS(true, false)
  } else if (has_bias) {
    ATPU_LM_BANS(false, true)
  } else {
    ATPU_LM_BANS(false, false)
  }
#undef ATPU_LM_BANS
#undef ATPU_LM_CFG
#undef ATPU_LM
  }
  if (M <= kMergeFewRows && !inv)
    hipLaunchKernelGGL(lm_head_merge_few_kernel, dim3(M), dim3(kMergeFewThreads), 0, stream, hdr, cand, nslab,
                       beam_scores, topk, out_score, out_token);
  else
    hipLaunchKernelGGL(lm_head_merge_kernel, dim3(M), dim3(kMergeThreads), 0, stream, hdr, cand, nslab, beam_scores,
                       topk, out_score, out_token);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
