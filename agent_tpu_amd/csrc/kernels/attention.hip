// Fused masked multi-head attention (T5 encoder/cross
// attention reuses it with an additive position bias and scale 1).
//
//   O[b,q,h,:] = softmax_k( scale * Q[b,q,h]·K[b,k,h] + bias[h,q,k] ) · V[b,k,h,:]
//   keys k >= lens[b] are masked; causal=1 additionally masks k > q.
//
// D = 64 (BERT-base/large, T5-base). Workgroup = 8 waves = 128 queries of one
// (batch, head); each wave owns 16 queries (one MFMA column tile), which keeps
// a wave at <= 128 VGPRs: 2 workgroups = 4 waves/SIMD per CU to hide the
// staging latency (the 4-wave/32-query layout needed 251 VGPRs, 2 waves/SIMD). Keys are processed in chunks of
// 128 with an fp32 online softmax, so any Skv works; BERT (S=128) is one chunk.
//
// CDNA4 mapping (cdna_hip_programming.md §3, App. B "Fused attention"):
//  * S^T = K·Q^T on v_mfma_f32_16x16x32_bf16: the KEY index sits in the
//    accumulator rows and the QUERY on the lane, so every lane owns whole
//    score columns -> row max / row sum are in-register plus two xor-shuffles,
//    and the P^T tile is ALREADY the B operand of O^T = V^T·P^T (the k order
//    inside a 32-key step is permuted identically on both operands).
//  * K chunk staged by global_load_lds (16 B/lane) into a row-swizzled image
//    (chunk ^ ((row>>1)&7)) read conflict-free with ds_read_b128.
//  * V chunk staged ROW-major by global_load_lds like K (no VGPR round trip),
//    16-B chunks swizzled chunk ^ (((row>>1)&3)<<1); the PV A operand (8 keys
//    of one d column per lane) is gathered with ds_read_b64_tr_b16 (guide
//    T10): a 16-lane group reads a 4-key x 16-d block and lane i receives
//    column i. The chunk-pair swizzle puts the 8 rows a 32-lane half reads in
//    8 distinct 32-B bank groups -> conflict-free.
//  * Q fragments go global -> VGPR directly (read once per wave).
#include "atpu/common.h"
#include "atpu/kernels.h"

#include <algorithm>
#include <cstdlib>

namespace atpu {
namespace {

constexpr int kD = 64;
constexpr int kKC = 128;  // keys per chunk
constexpr int kQB = 128;  // queries per workgroup
constexpr int kKRowB = kD * 2;     // 128 B per K row
constexpr int kVRowB = kD * 2;     // 128 B per V row
constexpr int kLdsK = kKC * kKRowB;  // 16 KiB
constexpr int kLdsV = kKC * kVRowB;  // 16 KiB

__device__ __forceinline__ int kswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int vswz(int row, int chunk) { return chunk ^ (((row >> 1) & 3) << 1); }

typedef short v4s __attribute__((vector_size(8)));
// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, elements
// 4p..4p+3 of a 4x16 block; lane i gets column i of the 4 rows (row q -> elem q)
__device__ __forceinline__ bf16x4 lds_read_tr16(const char* p) {
  const v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
  return __builtin_bit_cast(bf16x4, r);
}

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;

template <bool HAS_BIAS, bool CAUSAL>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(HAS_BIAS ? 2 : 4))) void attention_fwd_kernel(
    const bf16* __restrict__ Q, int ldq, const bf16* __restrict__ Kp, int ldk, const bf16* __restrict__ V, int ldv,
    bf16* __restrict__ O, int ldo, const int32_t* __restrict__ lens, const float* __restrict__ bias, int Sq, int Skv,
    int H, float scale) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsK + kLdsV];
  char* ldsK = lds;
  char* ldsV = lds + kLdsK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int len = lens ? min(lens[b], Skv) : Skv;
  const int fr = lane & 15, fg = lane >> 4;

  const bf16* Qb = Q + (size_t)b * Sq * ldq + h * kD;
  const bf16* Kb = Kp + (size_t)b * Skv * ldk + h * kD;
  const bf16* Vb = V + (size_t)b * Skv * ldv + h * kD;

  // ---- this wave's Q fragments: 16 queries x 2 d-steps, 16 B each ----
  const int qw = qblk * kQB + wave * 16;
  bf16x8 qf[2];
  {
    const int q = min(qw + fr, Sq - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[ds] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)q * ldq + ds * 32 + fg * 8);
  }

  float m_run = -1e30f, l_run = 0.f;
  f32x4 o[4];  // O^T tiles [d-tile] for the wave's 16 queries
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kv_end = CAUSAL ? min(len, qblk * kQB + kQB) : len;
  for (int kc = 0; kc < kv_end; kc += kKC) {
    __syncthreads();  // previous chunk fully consumed
    // ---- stage K chunk: 16 wave-instructions of 8 rows (4 per wave) ----
    {
      const int srow = lane >> 3, spos = lane & 7;
#pragma unroll
      for (int i = 0; i < 16 / kWaves; ++i) {
        const int r = (i * kWaves + wave) * 8 + srow;
        const int key = min(kc + r, Skv - 1);
        glds16(Kb + (size_t)key * ldk + kswz(r, spos) * 8, ldsK + (i * kWaves + wave) * 8 * kKRowB);
      }
    }
    // ---- stage V chunk row-major (same DMA pattern as K, V swizzle) ----
    {
      const int srow = lane >> 3, spos = lane & 7;
#pragma unroll
      for (int i = 0; i < 16 / kWaves; ++i) {
        const int r = (i * kWaves + wave) * 8 + srow;
        const int key = min(kc + r, Skv - 1);
        glds16(Vb + (size_t)key * ldv + vswz(r, spos) * 8, ldsV + (i * kWaves + wave) * 8 * kVRowB);
      }
    }
    wait_vmcnt0();
    __syncthreads();

    // ---- S^T = K·Q^T : s[kt] holds keys kt*16 + fg*4 + r, query fr ----
    f32x4 s[8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = kt * 16 + fr;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ldsK + r * kKRowB + kswz(r, ds * 4 + fg) * 16);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], s[kt], 0, 0, 0);
      }
    }

    // ---- scale, bias, mask, online softmax (per query column) ----
    {
      const int q = qw + fr;
      const int qc = min(q, Sq - 1);
      float cmax = -1e30f;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        const int key0 = kc + kt * 16 + fg * 4;
        f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (HAS_BIAS) {
          // Skv % 4 == 0 is enforced on the host for the bias path
          if (key0 < Skv) bv = *reinterpret_cast<const f32x4*>(bias + ((size_t)h * Sq + qc) * Skv + key0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = key0 + r;
          float x = s[kt][r] * scale + bv[r];
          const bool dead = key >= len || (CAUSAL && key > q);
          x = dead ? -1e30f : x;
          s[kt][r] = x;
          cmax = fmaxf(cmax, x);
        }
      }
      cmax = lane_rows_max(cmax);  // l, l^16, l^32, l^48 by permlane swaps
      const float m_new = fmaxf(m_run, cmax);
      const float alpha = __expf(m_run - m_new);
      float psum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = s[kt][r];
          const float p = x <= -1e29f ? 0.f : __expf(x - m_new);
          s[kt][r] = p;
          psum += p;
        }
      psum = lane_rows_sum(psum);
      l_run = l_run * alpha + psum;
      m_run = m_new;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    }

    // ---- O^T += V^T · P^T over 4 key-steps of 32 ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pf[e] = f2bf(s[2 * ks][e]);
        pf[4 + e] = f2bf(s[2 * ks + 1][e]);
      }
      const int tq = fr >> 2, tp = fr & 3;  // transposed-read lane roles
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int klo = ks * 32 + fg * 4 + tq, khi = klo + 16;
        const int c = dt * 2 + (tp >> 1);
        const bf16x4 lo = lds_read_tr16(ldsV + klo * kVRowB + vswz(klo, c) * 16 + (tp & 1) * 8);
        const bf16x4 hi = lds_read_tr16(ldsV + khi * kVRowB + vswz(khi, c) * 16 + (tp & 1) * 8);
        bf16x8 vf;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vf[e] = lo[e];
          vf[4 + e] = hi[e];
        }
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }
  }

  // ---- normalise and store: lane holds O[q][dt*16 + fg*4 + 0..3] ----
  {
    const int q = qw + fr;
    if (q < Sq) {
      const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
      bf16* orow = O + ((size_t)b * Sq + q) * ldo + h * kD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][e] * inv);
        *reinterpret_cast<bf16x4*>(orow + dt * 16 + fg * 4) = v;
      }
    }
  }
}


// ============================================================================
// Long-sequence encoder attention (SURVEY.md §2.6 K4/K8 at S = 512 / 1024: the
// summarizer's encoder, the reference truncating at 1024 tokens, ref
// ops/map_summarize.py:49). Same 8-wave x 16-query tile and MFMA / transposed-V
// math as attention_fwd_kernel, restructured for many key chunks per query block:
//  * K/V chunks double-buffered by LDS-DMA: chunk c+1 is in flight while chunk c
//    is computed (counted vmcnt(4): every wave issues exactly 4 LDS-DMA pieces
//    per chunk), instead of a full HBM round trip per chunk;
//  * T5 relative-position bias by DISTANCE: bias[h,q,k] depends only on k - q,
//    so the head's [Sq + Skv - 1] row is staged in LDS once (pre-scaled by
//    log2 e) instead of streaming a dense [H, S, S] fp32 tensor from L2/HBM
//    (4 B per score: at S = 1024 that was 12.9 GB per call);
//  * softmax in the exp2 domain with scale*log2(e) folded into one multiply;
//    the key-length mask is applied only in the last (partial) chunk;
//  * XCD-aware block order: the query blocks of one (batch, head) run on one XCD,
//    so its K/V chunks are fetched into that XCD's L2 once, not once per XCD.
// ============================================================================
constexpr int kFlashTab = 4096;  // Sq + Skv - 1 <= 4096 distance-bias entries (16 KiB)
constexpr float kLog2e = 1.4426950408889634f;

template <bool DIST>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void attention_flash_kernel(
    const bf16* __restrict__ Q, int ldq, const bf16* __restrict__ Kp, int ldk, const bf16* __restrict__ V, int ldv,
    bf16* __restrict__ O, int ldo, const int32_t* __restrict__ lens, const float* __restrict__ bias_dist, int Sq,
    int Skv, int H, float scale_log2, int nq, int nblocks) {
  constexpr int kTab = DIST ? kFlashTab * 4 : 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * (kLdsK + kLdsV) + kTab];
  float* tab = reinterpret_cast<float*>(lds + 2 * (kLdsK + kLdsV));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = xcd_remap(blockIdx.x, nblocks);
  const int qblk = t % nq, bh = t / nq, h = bh % H, b = bh / H;
  const int len = lens ? min(lens[b], Skv) : Skv;
  const int fr = lane & 15, fg = lane >> 4;

  const bf16* Qb = Q + (size_t)b * Sq * ldq + h * kD;
  const bf16* Kb = Kp + (size_t)b * Skv * ldk + h * kD;
  const bf16* Vb = V + (size_t)b * Skv * ldv + h * kD;

  const int qw = qblk * kQB + wave * 16;
  bf16x8 qf[2];
  {
    const int q = min(qw + fr, Sq - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[ds] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)q * ldq + ds * 32 + fg * 8);
  }
  const int ntab = Sq + Skv - 1;
  if constexpr (DIST) {
    const float* row = bias_dist + (size_t)h * ntab;
    for (int j = tid; j < ntab; j += kThreads) tab[j] = row[j] * kLog2e;
  }

  // 4 LDS-DMA pieces per wave per chunk: 2 for K, 2 for V
  auto stage = [&](int kc, int buf) {
    char* lk = lds + buf * (kLdsK + kLdsV);
    char* lv = lk + kLdsK;
    const int srow = lane >> 3, spos = lane & 7;
#pragma unroll
    for (int i = 0; i < 16 / kWaves; ++i) {
      const int r = (i * kWaves + wave) * 8 + srow;
      const int key = min(kc + r, Skv - 1);
      glds16(Kb + (size_t)key * ldk + kswz(r, spos) * 8, lk + (i * kWaves + wave) * 8 * kKRowB);
    }
#pragma unroll
    for (int i = 0; i < 16 / kWaves; ++i) {
      const int r = (i * kWaves + wave) * 8 + srow;
      const int key = min(kc + r, Skv - 1);
      glds16(Vb + (size_t)key * ldv + vswz(r, spos) * 8, lv + (i * kWaves + wave) * 8 * kVRowB);
    }
  };

  const int nch = (len + kKC - 1) / kKC;
  if (nch > 0) stage(0, 0);
  wait_vmcnt0();
  __syncthreads();  // Q fragments, distance table and chunk 0 are in place

  // VALU per score (the kernel was VALU-bound, MFMA busy 18 %: profiles/pmc_flash_attention_t5_src1024.txt):
  // the distance bias comes from ONE per-lane LDS base per chunk with immediate offsets (no
  // per-value index math or clamp: entries past the table's used part are only read for keys
  // >= Skv, which the tail mask drops), scale and bias are one FMA, and the row sums come from
  // the MFMA (P times a ones block, o[4]) instead of VALU adds and a cross-lane sum -- the sum
  // of the same bf16-rounded P the context is made of.
  float m_run = -1e30f;
  f32x4 o[5];
#pragma unroll
  for (int dt = 0; dt < 5; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q = qw + fr;
  const int qc = min(q, Sq - 1);
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;

  for (int c = 0; c < nch; ++c) {
    const int kc = c * kKC;
    const int buf = c & 1;
    if (c + 1 < nch) {
      stage(kc + kKC, buf ^ 1);  // buffer buf^1 was released by the barrier closing chunk c-1
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      wait_vmcnt0();
    }
    __syncthreads();  // chunk c landed for every wave
    const char* ldsK = lds + buf * (kLdsK + kLdsV);
    const char* ldsV = ldsK + kLdsK;

    f32x4 s[8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = kt * 16 + fr;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ldsK + r * kKRowB + kswz(r, ds * 4 + fg) * 16);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], s[kt], 0, 0, 0);
      }
    }

    const bool tail = kc + kKC > len;
    // this lane's scores: keys kc + kt*16 + fg*4 + r -> distance-table entry
    // kc + kt*16 + fg*4 + r - qc + Sq - 1 = tb[kt*16 + r]
    const float* tb = tab + (kc + fg * 4 - qc + Sq - 1);
    float cmax = -1e30f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x;
        if constexpr (DIST) x = fmaf(s[kt][r], scale_log2, tb[kt * 16 + r]);
        else x = s[kt][r] * scale_log2;
        s[kt][r] = x;
      }
      if (tail) {
        const int key0 = kc + kt * 16 + fg * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][r] = key0 + r >= len ? -1e30f : s[kt][r];
      }
      cmax = fmaxf(cmax, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
    }
    cmax = lane_rows_max(cmax);  // l, l^16, l^32, l^48 by permlane swaps
    const float m_new = fmaxf(m_run, cmax);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = s[kt][r];
        float p = __builtin_amdgcn_exp2f(x - m_new);
        if (tail) p = x <= -1e29f ? 0.f : p;
        s[kt][r] = p;
      }
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < 5; ++dt) o[dt] *= alpha;

#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pf[e] = f2bf(s[2 * ks][e]);
        pf[4 + e] = f2bf(s[2 * ks + 1][e]);
      }
      const int tq = fr >> 2, tp = fr & 3;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int klo = ks * 32 + fg * 4 + tq, khi = klo + 16;
        const int cc = dt * 2 + (tp >> 1);
        const bf16x4 lo = lds_read_tr16(ldsV + klo * kVRowB + vswz(klo, cc) * 16 + (tp & 1) * 8);
        const bf16x4 hi = lds_read_tr16(ldsV + khi * kVRowB + vswz(khi, cc) * 16 + (tp & 1) * 8);
        bf16x8 vf;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vf[e] = lo[e];
          vf[4 + e] = hi[e];
        }
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
      o[4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf, o[4], 0, 0, 0);  // row sums
    }
    __syncthreads();  // every wave is done with buffer buf before chunk c+2 is staged into it
  }

  if (q < Sq) {
    const float l_run = o[4][0];  // every element of the ones block holds the query's row sum
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16* orow = O + ((size_t)b * Sq + q) * ldo + h * kD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][e] * inv);
      *reinterpret_cast<bf16x4*>(orow + dt * 16 + fg * 4) = v;
    }
  }
}


// ============================================================================
// Persistent packed-QKV attention (BERT encoder: no bias, not causal, S <= 128,
// so one key chunk per (batch, head) item). The one-item-per-workgroup kernel
// above waits a full HBM round trip for K/V/Q before every item and only
// 2 workgroups per CU (98 VGPRs) overlap those waits. Here each workgroup walks
// items b*H + h = blockIdx.x + i * gridDim.x and prefetches item i+1 while it
// computes item i, everything by LDS-DMA (no VGPR loads the compiler would
// drain with vmcnt(0)):
//   top:   s_waitcnt vmcnt(2) -> K/V(i), Q(i) landed; only the previous item's
//          2 output stores may still be in flight (vmcnt(0) for the first item).
//          barrier.
//   Q(i) fragments LDS -> VGPR (the wave's private 2 KiB Q image), lgkmcnt(0)
//   issue: K/V(i+1) -> the other 32 KiB buffer, Q(i+1) -> the wave's Q image
//   compute item i (same MFMA / softmax / transposed-V code as above); O is
//   staged through the K half of the buffer (free after a barrier following
//   QK^T) and stored as whole 128-B rows
// A K/V buffer is restaged one barrier after the compute that read it; the Q
// image is private to its wave and restaged after that wave's reads retired.
// LDS 80 KiB -> two workgroups per CU.
// ============================================================================
constexpr int kQImg = 16 * kKRowB;  // one wave's 16 query rows

__device__ __forceinline__ bf16x4 lds_read_tr16_asm(const char* p) {
  v4s r;
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return __builtin_bit_cast(bf16x4, r);
}

// HOT (timing-only diagnostic, results WRONG): every item reads batch row 0's Q/K/V (L2-resident)
// PL: row max / sum over the 4 lanes of a query by v_permlane16/32_swap (registers
// only) instead of the ds_bpermute round trips __shfl_xor compiles to
template <int CPOL, bool HOT = false, bool PL = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void attention_packed_persist_kernel(
    const bf16* __restrict__ QKV, int ldq, bf16* __restrict__ O, int ldo, const int32_t* __restrict__ lens, int S,
    int H, int items, float scale) {
  __shared__ __attribute__((aligned(16))) char lds[2 * (kLdsK + kLdsV) + kWaves * kQImg];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int srow = lane >> 3, spos = lane & 7;
  const int hd = H * kD;
  char* qimg = lds + 2 * (kLdsK + kLdsV) + wave * kQImg;
  int item = blockIdx.x;
  if (item >= items) return;

  auto stage = [&](int it, int buf) {
    const int b = HOT ? 0 : __builtin_amdgcn_readfirstlane(it / H), h = __builtin_amdgcn_readfirstlane(it % H);
    // buffer resource over this item's rows (scalar base + 32-bit lane offsets,
    // guide T8): one VGPR per DMA. The lane offsets are recomputed per item from
    // the lane id (v_mbcnt, rematerialisable): kept live across the loop they were
    // spilled (the compute phase needs ~120 VGPRs under the 128 cap of 2 groups/CU).
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(QKV + (size_t)b * S * ldq + h * kD), 0, S * ldq * 2, 0x00020000);
    int l = __lane_id();
    asm volatile("" : "+v"(l));  // opaque per call: no loop-invariant offsets to keep live (or spill)
    const int sr = l >> 3, sp = l & 7;
    char* ldsK = lds + buf * (kLdsK + kLdsV);
    char* ldsV = ldsK + kLdsK;
    auto dma = [&](uint32_t off, char* dst) {
      // CPOL 2 = nt: Q/K/V are read exactly once, stream them past L2/MALL so the
      // residual and the next GEMM's operands stay resident
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (ATPU_LDS_AS void*)dst, 16, off, 0, 0, CPOL);
    };
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (i * kWaves + wave) * 8 + sr;
      const uint32_t row = (uint32_t)min(r, S - 1) * (uint32_t)ldq;
      dma((row + hd + kswz(r, sp) * 8) * 2, ldsK + (i * kWaves + wave) * 8 * kKRowB);
      dma((row + 2 * hd + vswz(r, sp) * 8) * 2, ldsV + (i * kWaves + wave) * 8 * kVRowB);
    }
    // this wave's 16 query rows (swizzled like K: conflict-free fragment reads)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = i * 8 + sr;
      dma(((uint32_t)min(wave * 16 + r, S - 1) * (uint32_t)ldq + kswz(r, sp) * 8) * 2, qimg + i * 8 * kKRowB);
    }
  };

  stage(item, 0);
  int buf = 0;
  bool first = true;
  for (;;) {
    const int next = item + gridDim.x;
    const bool has_next = next < items;
    // K/V/Q(item) are older than the previous item's 2 output stores (none
    // before the first item: its 6 DMAs are the newest ops)
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    first = false;
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 qf[2];
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[ds] = *reinterpret_cast<const bf16x8*>(qimg + fr * kKRowB + kswz(fr, ds * 4 + fg) * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Q image read before it is restaged
    __builtin_amdgcn_sched_barrier(0);
    if (has_next) stage(next, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    const char* ldsK = lds + buf * (kLdsK + kLdsV);
    const char* ldsV = ldsK + kLdsK;
    const int len = min(lens[item / H], S);

    f32x4 s[8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = kt * 16 + fr;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ldsK + r * kKRowB + kswz(r, ds * 4 + fg) * 16);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], s[kt], 0, 0, 0);
      }
    }
    // every wave's K reads have retired (its MFMAs consumed them): the K half
    // of this buffer becomes the O staging area below
    __builtin_amdgcn_s_barrier();
    // softmax over the keys (unscaled scores: scale > 0, so max(s)*scale = max(s*scale)).
    // exp((s - max)*scale) = exp2(s*c - max*c), c = scale*log2(e): one FMA + v_exp per
    // score. When all 128 key slots are valid keys (S == 128 and a full-length row) the
    // wave-uniform branch skips the per-score mask compares and selects; for S < 128 the
    // slots past S hold clamped duplicate rows and are always masked.
    const float c = scale * 1.4426950408889634f;
    float mx = -1e30f, psum = 0.f;
    if (len >= 8 * 16) {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) mx = fmaxf(mx, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
      if constexpr (PL) {
        mx = lane_rows_max(mx);
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      const float moff = mx * c;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][r], c, -moff));
          s[kt][r] = p;
          psum += p;
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + fg * 4 + r;
          const float x = key < len ? s[kt][r] : -1e30f;
          s[kt][r] = x;
          mx = fmaxf(mx, x);
        }
      if constexpr (PL) {
        mx = lane_rows_max(mx);
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      const float moff = mx * c;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = s[kt][r];
          const float p = x <= -1e29f ? 0.f : __builtin_amdgcn_exp2f(fmaf(x, c, -moff));
          s[kt][r] = p;
          psum += p;
        }
    }
    if constexpr (PL) {
      psum = lane_rows_sum(psum);
    } else {
      psum += __shfl_xor(psum, 16, 64);
      psum += __shfl_xor(psum, 32, 64);
    }

    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pf[e] = f2bf(s[2 * ks][e]);
        pf[4 + e] = f2bf(s[2 * ks + 1][e]);
      }
      const int tq = fr >> 2, tp = fr & 3;
      // transposed V reads by inline asm: the builtin form makes hipcc's waitcnt
      // pass assume it may alias the LDS-DMA in flight to the other buffer and
      // drain it (vmcnt(0)) right here, which serialises the prefetch
#pragma unroll
      for (int dh = 0; dh < 4; dh += 2) {  // two d-tiles per wait: 8 VGPRs of V fragments live
        bf16x4 lo[2], hi[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const int klo = ks * 32 + fg * 4 + tq, khi = klo + 16;
          const int c = (dh + d) * 2 + (tp >> 1);
          lo[d] = lds_read_tr16_asm(ldsV + klo * kVRowB + vswz(klo, c) * 16 + (tp & 1) * 8);
          hi[d] = lds_read_tr16_asm(ldsV + khi * kVRowB + vswz(khi, c) * 16 + (tp & 1) * 8);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // keep the reads' consumers below the wait (guide §5.4 rule 18)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          bf16x8 vf;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            vf[e] = lo[d][e];
            vf[4 + e] = hi[d][e];
          }
          o[dh + d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dh + d], 0, 0, 0);
        }
      }
    }
    {
      // O goes out through LDS (this wave's 2 KiB of the K half of the buffer,
      // free since the barrier after QK^T; 16-B chunks XOR-swizzled by row) so
      // each store writes whole 128-B head rows: 8 rows x 128 B per
      // wave-instruction instead of 16 rows x 32 B (partial-line stores were
      // most of the GEMM tail's cost, docs/PERF_NOTES.md).
      const float inv = psum > 0.f ? 1.f / psum : 0.f;
      char* ost = const_cast<char*>(ldsK) + wave * 16 * kKRowB;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][e] * inv);
        const int ch = dt * 2 + (fg >> 1);
        *reinterpret_cast<bf16x4*>(ost + fr * kKRowB + ((ch ^ (fr & 7)) << 4) + (fg & 1) * 8) = v;
      }
      // rows past S (S = 64: waves 4-7) computed query S-1 (clamped Q rows)
      // and rewrite its identical values; S % 16 == 0 (host check): every lane
      // stores, so each wave issues exactly 2 stores per item (the count the
      // top-of-loop vmcnt(2) relies on)
      int l2 = __lane_id();
      asm volatile("" : "+v"(l2));
      const int lr = l2 >> 3, lc = l2 & 7;
      const bf16* obase0 = O + (size_t)(item / H) * S * ldo + (item % H) * kD + lc * 8;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = lr + hh * 8;
        const u32x4 val = *reinterpret_cast<const u32x4*>(ost + r * kKRowB + ((lc ^ (r & 7)) << 4));
        *reinterpret_cast<u32x4*>(const_cast<bf16*>(obase0) + (size_t)min(wave * 16 + r, S - 1) * ldo) = val;
      }
    }
    if (!has_next) break;
    buf ^= 1;
    item = next;
  }
}

}  // namespace

int attention_persist_mode(int set) {
  // packed BERT case: 2 = persistent kernel with register-only row reductions (default),
  // 1 = persistent kernel with ds_bpermute reductions, 0 = one item per workgroup
  static int v = [] {
    const char* f = std::getenv("ATPU_ATTN_PERSIST");
    return (f && (f[0] == '0' || f[0] == '1')) ? f[0] - '0' : 2;
  }();
  if (set >= 0) v = set;
  return v;
}

int attention_flash_mode(int set) {
  // encoder attention with many key chunks: 1 = double-buffered flash kernel (default), 0 = attention_fwd_kernel
  static int v = [] {
    const char* f = std::getenv("ATPU_ATTN_FLASH");
    return (f && f[0] == '0') ? 0 : 1;
  }();
  if (set >= 0) v = set;
  return v;
}

void attention_fwd_strided(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv, bf16* out,
                           int ldo, const int32_t* lens, const float* bias, int B, int Sq, int Skv, int H, int D,
                           float scale, int causal, hipStream_t stream, const float* bias_dist) {
  ATPU_CHECK(D == kD, "attention: head dim must be 64");
  ATPU_CHECK(!(bias && bias_dist), "attention: dense bias and distance bias are exclusive");
  if (bias_dist) {
    ATPU_CHECK(!causal && Sq + Skv - 1 <= kFlashTab, "attention: distance bias needs !causal and Sq + Skv <= 4097");
  }
  ATPU_CHECK(B > 0 && Sq > 0 && Skv > 0 && H > 0, "attention: empty problem");
  ATPU_CHECK(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "attention: row strides must be 16-B");
  ATPU_CHECK(!bias || Skv % 4 == 0, "attention: bias path needs Skv % 4 == 0");
  // packed BERT layout (q | k | v column blocks of one [rows, 3*H*64] tensor),
  // one key chunk, whole 16-query tiles: the persistent prefetching kernel
  const bool packed = k == q + H * kD && v == k + H * kD && ldk == ldq && ldv == ldq;
  if (packed && !bias && !causal && lens && Sq == Skv && Sq <= kKC && Sq % 16 == 0 &&
      attention_persist_mode(-1) >= 1) {
    const int nb = 2 * num_cus();  // two workgroups per CU (80 KiB LDS each)

    const int items = B * H;
    // ATPU_ATTN_NT=0: Q/K/V loads with the default cache policy (kept in L2 / the Infinity
    // Cache) instead of streaming nt loads: for batches whose QKV fits the 256 MiB MALL
    static const bool nt = [] {
      const char* f = std::getenv("ATPU_ATTN_NT");
      return !(f && f[0] == '0');
    }();
    if (attention_persist_mode(-1) == 2) {
      if (nt)
        hipLaunchKernelGGL((attention_packed_persist_kernel<2, false, true>), dim3(std::min(items, nb)),
                           dim3(kThreads), 0, stream, q, ldq, out, ldo, lens, Sq, H, items, scale);
      else
        hipLaunchKernelGGL((attention_packed_persist_kernel<0, false, true>), dim3(std::min(items, nb)),
                           dim3(kThreads), 0, stream, q, ldq, out, ldo, lens, Sq, H, items, scale);
      ATPU_HIP_CHECK(hipGetLastError());
      return;
    }
    static const bool hot = [] {
      const char* f = std::getenv("ATPU_ATTN_HOT");
      return f && f[0] == '1';
    }();
    if (hot)
      hipLaunchKernelGGL((attention_packed_persist_kernel<2, true>), dim3(std::min(items, nb)), dim3(kThreads), 0,
                         stream, q, ldq, out, ldo, lens, Sq, H, items, scale);
    else if (nt)
      hipLaunchKernelGGL(attention_packed_persist_kernel<2>, dim3(std::min(items, nb)), dim3(kThreads), 0, stream, q,
                         ldq, out, ldo, lens, Sq, H, items, scale);
    else
      hipLaunchKernelGGL(attention_packed_persist_kernel<0>, dim3(std::min(items, nb)), dim3(kThreads), 0, stream, q,
                         ldq, out, ldo, lens, Sq, H, items, scale);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  if (bias_dist || (!bias && !causal && Skv > kKC && attention_flash_mode(-1) == 1)) {
    ATPU_CHECK(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0, "attention: 16-B rows required");
    const int nq = (Sq + kQB - 1) / kQB;
    const long long nb = (long long)nq * H * B;
    ATPU_CHECK(nb < (1LL << 31), "attention: grid too large");
    const float sl2 = scale * kLog2e;
    if (bias_dist)
      hipLaunchKernelGGL(attention_flash_kernel<true>, dim3((unsigned)nb), dim3(kThreads), 0, stream, q, ldq, k, ldk,
                         v, ldv, out, ldo, lens, bias_dist, Sq, Skv, H, sl2, nq, (int)nb);
    else
      hipLaunchKernelGGL(attention_flash_kernel<false>, dim3((unsigned)nb), dim3(kThreads), 0, stream, q, ldq, k, ldk,
                         v, ldv, out, ldo, lens, nullptr, Sq, Skv, H, sl2, nq, (int)nb);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid((Sq + kQB - 1) / kQB, H, B);
#define ATPU_ATTN(HB, CA)                                                                                   \
  hipLaunchKernelGGL((attention_fwd_kernel<HB, CA>), grid, dim3(kThreads), 0, stream, q, ldq, k, ldk, v, ldv, out, \
                     ldo, lens, bias, Sq, Skv, H, scale)
  if (bias && causal)
    ATPU_ATTN(true, true);
  else if (bias)
    ATPU_ATTN(true, false);
  else if (causal)
    ATPU_ATTN(false, true);
  else
    ATPU_ATTN(false, false);
#undef ATPU_ATTN
  ATPU_HIP_CHECK(hipGetLastError());
}

void attention_fwd(const bf16* qkv, const int32_t* lens, const float* bias, bf16* out, int B, int S, int H, int D,
                   float scale, hipStream_t stream) {
  const int hd = H * D;
  attention_fwd_strided(qkv, 3 * hd, qkv + hd, 3 * hd, qkv + 2 * hd, 3 * hd, out, hd, lens, bias, B, S, S, H, D,
                        scale, 0, stream);
}

}  // namespace atpu
