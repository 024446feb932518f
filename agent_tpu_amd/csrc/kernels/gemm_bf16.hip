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

#include <cstdlib>
#include <string>
#include <type_traits>

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
template <int BM, int BN, int WM, int WN, int EPI, int SPLIT = 0>
__global__ __launch_bounds__(WM* WN * 64, 2) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K,
    float* __restrict__ ws = nullptr) {
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
  auto compute = [&](int buf) {
    const char* base = lds + buf * STAGE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = arow0 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
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
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + arow0 + i * 16 + frow;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + brow0 + j * 16 + fchunk * 4;
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI & kEpiBias) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n);
        v += b;
      }
      if constexpr (EPI & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_fast(v[e]);
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
}

// ============================================================================
// 256x256 tile, 8 waves, FULL-LINE staging (kernel "256b").
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

// DBG: timing-only ablation builds (results are WRONG): 1 = no vmcnt/barrier
// waits, 2 = no global->LDS DMA. See docs/PERF_NOTES.md.
template <int EPI, int DBG = 0>
__global__ __launch_bounds__(512, 2) void gemm256b_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K) {
  using namespace g2;
  __shared__ __attribute__((aligned(16))) char lds[2 * kTile];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = N / 256, ntm = (M + 255) / 256;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;

  // staging: chunk q (0..3) = (A|B) x (row half); this wave issues
  // instructions i = wave, wave + 8 of each chunk (8 rows x 128 B each)
  const int srow = lane >> 3, spos = lane & 7;
  const int lr0 = wave * 8 + srow, lr1 = (wave + 8) * 8 + srow;  // local rows 0..127
  const bf16* src[4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    src[h][0] = A + (size_t)min(m0 + h * 128 + lr0, M - 1) * lda + sw(lr0, spos) * 8;
    src[h][1] = A + (size_t)min(m0 + h * 128 + lr1, M - 1) * lda + sw(lr1, spos) * 8;
    src[2 + h][0] = Bt + (size_t)(n0 + h * 128 + lr0) * ldb + sw(lr0, spos) * 8;
    src[2 + h][1] = Bt + (size_t)(n0 + h * 128 + lr1) * ldb + sw(lr1, spos) * 8;
  }
  auto issue_tile = [&](int kt, int buf) {
    if constexpr (DBG & 2) return;
    char* base = lds + buf * kTile;
    const int koff = kt * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      glds16(src[q][0] + koff, base + q * kChunk + wave * 1024);
      glds16(src[q][1] + koff, base + q * kChunk + (wave + 8) * 1024);
    }
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fc = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_b = [&](bf16x8 (&f)[4], int buf, int ks) {
    const char* img = lds + buf * kTile + (2 + (wn >> 1)) * kChunk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (wn & 1) * 64 + j * 16 + fr;
      f[j] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
    }
  };
  auto load_a = [&](bf16x8 (&f)[4], int buf, int ks, int qm) {
    const char* img = lds + buf * kTile + wm * kChunk;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = qm * 64 + i * 16 + fr;
      f[i] = *reinterpret_cast<const bf16x8*>(img + r * 128 + sw(r, ks * 4 + fc) * 16);
    }
  };
  auto mma = [&](const bf16x8 (&bfr)[4], const bf16x8 (&afr)[4], int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[qm * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], afr[i], acc[qm * 4 + i][j], 0, 0, 0);
  };
#define ATPU_INTERLEAVE(NREAD)                                           \
  _Pragma("unroll") for (int q = 0; q < (NREAD); ++q) {                  \
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                   \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                   \
  }                                                                      \
  __builtin_amdgcn_sched_group_barrier(0x008, 16 - (NREAD), 0)

  const int nk = K / 64;
  bf16x8 b0[4], b1[4], a00[4], a01[4], a10[4], a11[4];
  issue_tile(0, 0);
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if constexpr (!(DBG & 1)) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    load_b(b0, cur, 0);
    load_a(a00, cur, 0, 0);
    if (t + 1 < nk) issue_tile(t + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(b0, a00, 0);
    load_a(a01, cur, 0, 1);
    ATPU_INTERLEAVE(4);
    __builtin_amdgcn_sched_barrier(0);
    mma(b0, a01, 1);
    load_b(b1, cur, 1);
    load_a(a10, cur, 1, 0);
    ATPU_INTERLEAVE(8);
    __builtin_amdgcn_sched_barrier(0);
    mma(b1, a10, 0);
    load_a(a11, cur, 1, 1);
    ATPU_INTERLEAVE(4);
    __builtin_amdgcn_sched_barrier(0);
    mma(b1, a11, 1);
    __builtin_amdgcn_sched_barrier(0);
  }
#undef ATPU_INTERLEAVE

  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + fc * 4;
    if constexpr (EPI & kEpiBias) bv[j] = *reinterpret_cast<const f32x4*>(bias + n);
    else bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    bf16x4 res[4][4];
    if constexpr (EPI & kEpiResidual) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int m = min(m0 + wm * 128 + (half * 4 + ii) * 16 + fr, M - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          res[ii][j] = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n0 + wn * 64 + j * 16 + fc * 4);
      }
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = half * 4 + ii;
      const int m = m0 + wm * 128 + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + fc * 4;
        f32x4 v = acc[i][j] + bv[j];
        if constexpr (EPI & kEpiGelu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gelu_fast(v[e]);
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
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(res[ii][j][e]);
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        if (m < M) *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
      }
    }
  }
}


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
  // the last MFMAs' results are read by inline-asm v_permlane below, which the
  // hazard recognizer cannot see: pad the MFMA-write -> VALU-read window
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue, widened (guide T21 for the 16x16 layout): v_permlane16_swap
  // of fragments (2p, j) and (2p+1, j) leaves every lane with 8 consecutive
  // fp32 columns of ONE row -> 16-B residual loads and 16-B stores (half the
  // VMEM instructions of the 8-B row-per-lane tail) ----
  const int hi = fc & 1, cq = (fc >> 1) * 8;  // row parity within the pair, column half
  bf16x8 res[4][4];
  if constexpr (EPI & kEpiResidual) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) {
        const int m = min(m0 + wm * 128 + (2 * pp + hi) * 16 + fr, M - 1);
        res[j][pp] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldr + n0 + wn * 64 + j * 16 + cq);
      }
  }
  f32x4 bias8[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + cq;
    if constexpr (EPI & kEpiBias) {
      bias8[j][0] = *reinterpret_cast<const f32x4*>(bias + n);
      bias8[j][1] = *reinterpret_cast<const f32x4*>(bias + n + 4);
    } else {
      bias8[j][0] = bias8[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const bool full_tile = m0 + 256 <= M;  // uniform: no per-store bounds branch
  // row pair outer, column fragment inner: the 4 consecutive 16-B stores of a
  // lane cover its row's whole 128-B line segment (write combining in L2)
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) {
    const int m = m0 + wm * 128 + (2 * pp + hi) * 16 + fr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + cq;
      const f32x4 lo4 = acc[2 * pp][j], hi4 = acc[2 * pp + 1][j];
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // v_permlane16_swap (odd 16-lane rows of x <-> even rows of y): the
        // even lane keeps row 2p (own cols 0-3 + partner's 4-7), the odd lane
        // row 2p+1 (semantics probed: tools/probes/permlane_probe.hip).
        // Operands are laundered through v_mov into fresh early-clobber
        // registers: handing element extracts of the accumulator tuples to
        // the swap directly got both operands allocated to one register.
        unsigned x, y;
        asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3\n\ts_nop 1\n\tv_permlane16_swap_b32 %0, %1"
                     : "=&v"(x), "=&v"(y)
                     : "v"(lo4[e]), "v"(hi4[e]));
        v[e] = __builtin_bit_cast(float, x) + bias8[j][0][e];
        v[4 + e] = __builtin_bit_cast(float, y) + bias8[j][1][e];
      }
      if constexpr (EPI & kEpiGelu) gelu_fast8(v);
      if constexpr (EPI & kEpiTanh) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = tanhf(v[e]);
      }
      if constexpr (EPI & kEpiRelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (EPI & kEpiResidual) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf2f(res[j][pp][e]);
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
      if (full_tile || m < M) *reinterpret_cast<bf16x8*>(C + (size_t)m * ldc + n) = o;
    }
  }
}

void launch_256p(const GemmArgs& g, hipStream_t s) {
  const int nb = ((g.M + 255) / 256) * (g.N / 256);
  static const int ablate = [] {
    const char* f = std::getenv("ATPU_GEMM_ABLATE");
    return f ? std::atoi(f) : 0;
  }();
  if (ablate == 4) {  // no epilogue (timing only)
    hipLaunchKernelGGL((gemm256p_kernel<kEpiBias, 1>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C,
                       g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K);
    return;
  }
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

void launch_256b(const GemmArgs& g, hipStream_t s) {
  const int nb = ((g.M + 255) / 256) * (g.N / 256);
  static const int ablate = [] {
    const char* f = std::getenv("ATPU_GEMM_ABLATE");
    return f ? std::atoi(f) : 0;
  }();
  if (ablate && g.epi == (kEpiBias | kEpiResidual)) {
#define ATPU_ABL(D)                                                                                              \
  case D:                                                                                                        \
    hipLaunchKernelGGL((gemm256b_kernel<kEpiBias | kEpiResidual, D>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, \
                       g.ldb, g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K);                                   \
    return;
    switch (ablate) {
      ATPU_ABL(1) ATPU_ABL(2) ATPU_ABL(3)
      default: break;
    }
#undef ATPU_ABL
  }
#define ATPU_G256B(E)                                                                                     \
  case E:                                                                                                 \
    hipLaunchKernelGGL((gemm256b_kernel<E>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, g.ldc, \
                       g.bias, g.R, g.ldr, g.M, g.N, g.K);                                                \
    break;
  switch (g.epi) {
    ATPU_G256B(0)
    ATPU_G256B(kEpiBias)
    ATPU_G256B(kEpiBias | kEpiGelu)
    ATPU_G256B(kEpiBias | kEpiTanh)
    ATPU_G256B(kEpiBias | kEpiResidual)
    ATPU_G256B(kEpiResidual)
    ATPU_G256B(kEpiGelu)
    ATPU_G256B(kEpiRelu)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_G256B
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

template <int EPI, int NST, int SPLIT>
__global__ __launch_bounds__(256, 2) void gemm_dec_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                          int ldc, const float* __restrict__ bias,
                                                          const bf16* __restrict__ R, int ldr, int M, int N, int K,
                                                          float* __restrict__ ws) {
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
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const char* base = lds + slot * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfg[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm * 32 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
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
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 32 + i * 16 + frow;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + fchunk * 4;
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI & kEpiBias) v += *reinterpret_cast<const f32x4*>(bias + n);
      if constexpr (EPI & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_fast(v[e]);
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
                       g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K, nullptr);                                    \
    break;
  switch (g.epi) {
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
      for (int e = 0; e < 4; ++e) v[e] = gelu_fast(v[e]);
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
                       g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K);                                 \
    break;
  switch (g.epi) {
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
  // 256x256 schedule: 1 = ping-pong "256p" (default), 0 = "256b"; ATPU_GEMM_256=b|p
  static int v = [] {
    const char* f = std::getenv("ATPU_GEMM_256");
    return (f && f[0] == 'b') ? 0 : 1;
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
bool skinny(int M, int N) { return M <= 2048 && ((M + 127) / 128) * ((N + 127) / 128) < 512; }
}  // namespace

int gemm_splitk_splits(int M, int N, int K) {
  // Skinny problems (decode: M = beams x docs) leave most of the 256 CUs idle.
  // dec kernel: split K only when even 64x64 tiles give < 128 blocks AND the
  // K loop is long (>= 32 K-tiles): the reduce launch costs ~4 us, which a
  // 12-16 K-tile loop does not win back (measured, tools/bench_decode_gemm.py).
  // 128x128 kernel: split so the grid reaches ~2 blocks per CU, >= 2 K-tiles per split.
  static const int forced = [] {
    const char* f = std::getenv("ATPU_GEMM_SPLITK");
    return f ? std::atoi(f) : -1;
  }();
  const int nk = K / kBK;
  int want;
  if (gemm_dec_mode(-1) == 1 && skinny(M, N)) {
    const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
    want = forced >= 0 ? forced : (tiles >= 128 || nk < 32 ? 1 : (256 + tiles - 1) / tiles);
    want = std::max(1, std::min({want, nk / 8, 16}));
  } else {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    want = forced >= 0 ? forced : (M > 1024 || tiles >= 256 ? 1 : (512 + tiles - 1) / tiles);
    want = std::max(1, std::min({want, nk / 2, 16}));
  }
  while (want > 1 && nk % want) --want;
  return want;
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
  static const int forced = [] {
    const char* f = std::getenv("ATPU_GEMM_TILE");
    return f ? std::atoi(f) : 0;
  }();
  if (g.splits > 1) {
    ATPU_CHECK(g.ws && (g.K / kBK) % g.splits == 0, "gemm: split-K needs a workspace and K/64 % splits == 0");
    launch_splitk(g, g.splits, gemm_dec_mode(-1) == 1 && skinny(g.M, g.N), stream);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  const int kernel256 = gemm_256_variant(-1);
  const bool big_ok = g.N % 256 == 0 && g.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0 &&
                      (!(g.epi & kEpiResidual) || (g.ldr % 8 == 0 && (reinterpret_cast<uintptr_t>(g.R) & 15) == 0));
  const bool use_big = !(g.epi & kEpiOutF32) && (forced ? (forced == 256 && big_ok) : (g.M >= 2048 && big_ok));
  if (use_big && kernel256 == 1)
    launch_256p(g, stream);
  else if (use_big)
    launch_256b(g, stream);
  else if (!forced && gemm_dec_mode(-1) == 1 && skinny(g.M, g.N))
    launch_dec(g, stream);
  else
    launch_tile<128, 128, 2, 2>(g, stream);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
