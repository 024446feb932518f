// BERT encoder QKV projection on 256 x 192 tiles: one tile = the Q | K | V columns of ONE
// head (192 = 3 x 64) for 256 rows = two 128-token sequences, so a tile holds everything
// the head's attention needs for both sequences.
//
// Persistent ping-pong schedule of the 256 x 256 "256s" kernel (gemm_bf16.hip), adapted to a
// 192-column B tile: wave (wm, wn) owns rows wm*128..+128 (sequence wm of the tile) and
// columns wn*48..+48 (3 MFMA column fragments). Per 64-deep K-tile, four phases:
//   p0: read A-top (4 frags) + B frags 0-1 -> MFMA (top, 0-1)    16 MFMA   stage Q0, Q1 (4 DMA)
//   p1: read B frag 2                     -> MFMA (top, 2)       8 MFMA   stage Q2 (1 DMA)
//   p2: read A-bottom                     -> MFMA (bottom, 2)    8 MFMA   stage Q3 (2 DMA)
//   p3: (registers only)                  -> MFMA (bottom, 0-1) 16 MFMA
// Quarters = row sets of the 128-B-row images of the NEXT K-tile, by the phase that first
// reads them: Q0 = A rows {0-63, 128-191}, Q1 = B rows wn*48 + {0..31} (both read at p0),
// Q2 = B rows wn*48 + {32..47} (p1), Q3 = A rows {64-127, 192-255} (p2). A quarter is staged
// the phase its buffer half was read one K-tile earlier, and retired by the wait of the phase
// before its first read (a wait before phase p's barrier covers reads in phase p+1, for both
// staggered wave groups): Q0/Q1 at p3 (vmcnt 3), Q2 at p0 (6), Q3 at p1 (5) - 32, 32 and 40
// MFMAs of the wave after their issue, at least the 256s kernel's 32.
//
// MODE 0 stores Q|K|V (bf16) like the general GEMM; MODE 1 is a timing-only build with no
// epilogue (accumulators kept live). EPI: bias, optionally InNorm (the QKV of BERT layers
// >= 1 consumes LN2 of the previous layer folded into the weights, as gemm256s).
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/lds_ops.h"

#include <algorithm>

namespace atpu {
namespace {

constexpr int kHImgA = 256 * 128;             // A image: 256 rows x 128 B
constexpr int kHImgB = 192 * 128;             // B image: 192 rows x 128 B
constexpr int kHBuf = kHImgA + kHImgB;        // one K-tile
constexpr int kHStores = 24;                  // MODE 0 epilogue stores per wave (8 row x 3 col fragments)

// image row of staging round i (of the quarter) for the wave's 8-row group g8 = (i*8 + wave)*8
__device__ __forceinline__ int hq_row(int q, int ql) {
  switch (q) {
    case 0: return (ql & 63) + (ql >> 6) * 128;
    case 3: return (ql & 63) + (ql >> 6) * 128 + 64;
    case 1: return (ql >> 5) * 48 + (ql & 31);
    default: return (ql >> 4) * 48 + 32 + (ql & 15);
  }
}
constexpr int hq_rounds(int q) { return q == 2 ? 1 : 2; }

constexpr int kAImg = kAttnImg;  // attention images (MODE 2): lds_ops.h

template <int EPI, int MODE>
__global__ __launch_bounds__(512, 1) void gemm256h_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ Bt, int ldb,
                                                          bf16* __restrict__ C, int ldc,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ in_fin,
                                                          const float* __restrict__ colsum, int M, int N, int K,
                                                          const int32_t* __restrict__ lens, float scale) {
  constexpr bool kIn = EPI & kEpiInNorm;
  // MODE 2: the 6 attention images (96 KiB) start at operand buffer 1, which holds the last
  // K-tile of every tile (host: K / 64 even), and run 40 KiB past it
  constexpr int kImgOff = kHBuf;
  constexpr int kBiasOff = MODE == 2 ? kImgOff + 6 * kAImg : 2 * kHBuf;  // [2 tiles][4 x 64] fp32 (wn-padded)
  constexpr int kFinOff = kBiasOff + 2 * 1024;  // [256][2] (rstd, rstd*mu) of the tile's rows
  constexpr int kColOff = kFinOff + 2048;       // [4 x 64] colsum (wn-padded)
  constexpr int kLds = kColOff + 1024;
  // VMEM ops a tile's epilogue leaves in flight: C stores (MODE 0) or context stores (MODE 2)
  constexpr int kEpiOps = MODE == 0 ? kHStores : MODE == 2 ? 4 : 0;
  constexpr int kLn1 = kIn ? 2 : 0;
  static_assert(kLds <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntn = N / 192, ntiles = (M / 256) * ntn;
  const int G = gridDim.x;
  int v = blockIdx.x;
  if (v >= ntiles) return;

  auto opaque_lane = [] {
    int l = __lane_id();
    asm volatile("" : "+v"(l));
    return l;
  };
  // per (quarter, round): wave-uniform LDS destination and 32-bit byte offset of the lane's source
  int dst[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dst[q][i] = (q == 0 || q == 3 ? 0 : kHImgA) + hq_row(q, (i * 8 + wave) * 8) * 128;
  uint32_t soff[4][2];
  auto set_src = [&](int tm0, int tn0) {
    const int ln = opaque_lane();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < hq_rounds(q); ++i) {
        const int r = hq_row(q, (i * 8 + wave) * 8 + (ln >> 3));
        const size_t e = (q == 0 || q == 3) ? (size_t)(tm0 + r) * lda + hsw(r, ln & 7) * 8
                                            : (size_t)(tn0 + r) * ldb + hsw(r, ln & 7) * 8;
        soff[q][i] = (uint32_t)(e * 2);
      }
  };
  auto stage = [&](int q, int kt, int buf) {
    char* base = lds + buf * kHBuf;
    const char* g = reinterpret_cast<const char*>((q == 0 || q == 3) ? A : Bt) + kt * 128;
#pragma unroll
    for (int i = 0; i < hq_rounds(q); ++i) glds16(g + soff[q][i], base + dst[q][i]);
  };
  // 4-byte LDS-DMA of 64 floats per wave: wn-padded [4][64] rows, lanes past 48 clamped
  // (their copies land in the padding)
  auto glds4 = [&](const float* ubase, int nvalid, char* ldst) {
    const int l = opaque_lane();
    __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)(ubase + min(l, nvalid - 1)),
                                     (ATPU_LDS_AS void*)ldst, 4, 0, 0);
  };

  const int fr = lane & 15, fc = lane >> 4;
  f32x4 acc[8][3];
  bf16x8 af[2][4], b01[2][2], b2[2];
  auto read_a = [&](int buf, int qm) {
    const char* img = lds + buf * kHBuf;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 128 + qm * 64 + i * 16 + fr;
        af[ks][i] = *reinterpret_cast<const bf16x8*>(img + r * 128 + hsw(r, ks * 4 + fc) * 16);
      }
  };
  auto read_b01 = [&](int buf) {
    const char* img = lds + buf * kHBuf + kHImgA;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 48 + j * 16 + fr;
        b01[ks][j] = *reinterpret_cast<const bf16x8*>(img + r * 128 + hsw(r, ks * 4 + fc) * 16);
      }
  };
  auto read_b2 = [&](int buf) {
    const char* img = lds + buf * kHBuf + kHImgA;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r = wn * 48 + 32 + fr;
      b2[ks] = *reinterpret_cast<const bf16x8*>(img + r * 128 + hsw(r, ks * 4 + fc) * 16);
    }
  };
  auto mma01 = [&](int qm) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b01[ks][j], af[ks][i], acc[qm * 4 + i][j], 0, 0, 0);
  };
  auto mma2 = [&](int qm) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[qm * 4 + i][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2[ks], af[ks][i], acc[qm * 4 + i][2], 0, 0, 0);
  };

  // ---- MODE 2: attention of sequence wm of the tile, head h, query rows wn*32..+32 ----
  // Two 16-query blocks share every K / V fragment read. S = K.Q^T per 16 x 16 block (lane:
  // query fr, keys 4fc..+4), row max over the 4 lanes of a query in registers, exp2 with the
  // scale folded, P as the A operand of P.V in the key order of its two score blocks, V
  // through transposed reads. Loads are issued in batches far ahead of their use (the
  // accumulator registers are free by now): Q and all of K before the first QK^T MFMA
  // (counted waits from the compiler), all of V right after QK^T so it lands under the
  // softmax. The row sums come from the MFMA too: P times a ones tile (one extra 16-column
  // output block), so every lane holds its query's sum of the same bf16-rounded P the context
  // is made of, with no VALU adds or cross-lane reduction. The context goes out through the
  // wave's own Q rows (free once read) as whole 128-B rows.
  auto attend = [&](int tm0, int h, int len) {
    const char* qi = lds + kImgOff + wm * 3 * kAImg;
    const char* ki = qi + kAImg;
    const char* vi = qi + 2 * kAImg;
    bf16x8 qf[2][2], kf[8][2];
#pragma unroll
    for (int qp = 0; qp < 2; ++qp)
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = wn * 32 + qp * 16 + fr;
        qf[qp][ds] = ds_read128(qi + r * 128 + asw(r, ds * 4 + fc) * 16);
      }
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = kt * 16 + fr;
        kf[kt][ds] = ds_read128(ki + r * 128 + asw(r, ds * 4 + fc) * 16);
      }
    // 20 reads in flight, retired in issue order: K-tile kt's MFMAs wait for lgkmcnt(14 - 2 kt).
    // Phase A: S(qp 0) = K.Q0^T, counted waits.
    f32x4 s[2][8];
    auto qk0 = [&](auto kt_c) {
      constexpr int kt = decltype(kt_c)::value;
      if constexpr (kt == 0) {
        lgkm_wait<14>(qf[0][0], qf[0][1]);
        asm volatile("" : "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(kf[0][0]), "+v"(kf[0][1]));
      } else {
        lgkm_wait<14 - 2 * kt>(kf[kt][0], kf[kt][1]);
      }
      s[0][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[0][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      s[0][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[0][1], s[0][kt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // K-tile kt's MFMAs before the next wait
    };
    qk0(std::integral_constant<int, 0>{});
    qk0(std::integral_constant<int, 1>{});
    qk0(std::integral_constant<int, 2>{});
    qk0(std::integral_constant<int, 3>{});
    qk0(std::integral_constant<int, 4>{});
    qk0(std::integral_constant<int, 5>{});
    qk0(std::integral_constant<int, 6>{});
    qk0(std::integral_constant<int, 7>{});
    const float cl = scale * 1.4426950408889634f;
    bf16x8 pf[2][4];  // P in bf16, A operand of key step ks
    // softmax of query block qp -> pf[qp] (VALU; interleaved below with the other block's MFMAs)
    // Keys >= len: scores set to -1e30 by a small separate block (mask(qp)), so the softmax
    // itself is branch-free, one basic block the scheduler can interleave with MFMAs (exp2 of
    // the masked scores underflows to 0; len == 0 is caught at the normalisation).
    auto mask = [&](int qp) {
      if (len < 128) {
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (kt * 16 + (opaque_lane() >> 4) * 4 + e >= len) s[qp][kt][e] = -1e30f;
      }
    };
    auto softmax = [&](int qp) {
      {
        float mx = -1e30f;
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
          mx = fmaxf(mx, fmaxf(fmaxf(s[qp][kt][0], s[qp][kt][1]), fmaxf(s[qp][kt][2], s[qp][kt][3])));
        const float moff = lane_rows_max(mx) * cl;
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) s[qp][kt][e] = __builtin_amdgcn_exp2f(fmaf(s[qp][kt][e], cl, -moff));
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pf[qp][ks][e] = f2bf(s[qp][2 * ks][e]);
          pf[qp][ks][4 + e] = f2bf(s[qp][2 * ks + 1][e]);
        }
    };
    f32x4 o[2][5];  // [4] = row sums (P times ones)
    unsigned xw[4][2];
    bf16x4 vlo[4][4], vhi[4][4];
    mask(0);
    // Phase B: S(qp 1) MFMAs beside softmax(qp 0) VALU (one wave's MFMA leaves the SIMD's
    // vector issue free for half its cycles)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[1][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[1][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      s[1][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[1][1], s[1][kt], 0, 0, 0);
    }
    softmax(0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // V fragments of key step ks (lane (tq, tp) of each 16-lane row addresses key row
    // ks*32 + fc*4 + tq (+16), columns 4tp.. of d-tile dt), all 32 reads issued now (K is
    // dead); addresses from an opaque lane id (hoisted, the per-step addresses spilled)
    {
      const int l = opaque_lane();
      const int tq = (l >> 2) & 3, tp = l & 3;
      const int k0 = (l >> 4) * 4 + tq;  // (k0 + ks*32 (+16)) & 7 == k0 & 7
      const char* row = vi + k0 * 128 + (tp & 1) * 8;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int c = asw(k0, dt * 2 + (tp >> 1)) * 16;
          vlo[ks][dt] = tr16(row + ks * 32 * 128 + c);
          vhi[ks][dt] = tr16(row + (ks * 32 + 16) * 128 + c);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
    auto vfrag = [&](int ks, int dt) {
      bf16x8 vf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vf[e] = vlo[ks][dt][e];
        vf[4 + e] = vhi[ks][dt][e];
      }
      return vf;
    };
    mask(1);
    __builtin_amdgcn_sched_barrier(0);
    // Phase C: P0.V MFMAs beside softmax(qp 1); key step ks waits for its 8 V reads (the
    // lgkmcnt field holds at most 15: steps 0-1 wait for 17 of the 32 reads)
    softmax(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks == 0) asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(vlo[0][0]), "+v"(vlo[0][1]), "+v"(vlo[0][2]), "+v"(vlo[0][3]),
                                "+v"(vhi[0][0]), "+v"(vhi[0][1]), "+v"(vhi[0][2]), "+v"(vhi[0][3])::"memory");
      if (ks == 1) asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(vlo[1][0]), "+v"(vlo[1][1]), "+v"(vlo[1][2]), "+v"(vlo[1][3]),
                                "+v"(vhi[1][0]), "+v"(vhi[1][1]), "+v"(vhi[1][2]), "+v"(vhi[1][3])::"memory");
      if (ks == 2) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(vlo[2][0]), "+v"(vlo[2][1]), "+v"(vlo[2][2]), "+v"(vlo[2][3]),
                                "+v"(vhi[2][0]), "+v"(vhi[2][1]), "+v"(vhi[2][2]), "+v"(vhi[2][3])::"memory");
      if (ks == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[3][0]), "+v"(vlo[3][1]), "+v"(vlo[3][2]), "+v"(vlo[3][3]),
                                "+v"(vhi[3][0]), "+v"(vhi[3][1]), "+v"(vhi[3][2]), "+v"(vhi[3][3])::"memory");
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfrag(ks, dt), pf[0][ks],
                                                             ks ? o[0][dt] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      o[0][4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[0][ks], ks ? o[0][4] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 20; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    // Phase D: P1.V MFMAs beside the scaling / packing of the qp 0 context
    const float inv0 = len > 0 && o[0][4][0] > 0.f ? 1.f / o[0][4][0] : 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      xw[dt][0] = pack_bf16x2(o[0][dt][0] * inv0, o[0][dt][1] * inv0);
      xw[dt][1] = pack_bf16x2(o[0][dt][2] * inv0, o[0][dt][3] * inv0);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfrag(ks, dt), pf[1][ks],
                                                             ks ? o[1][dt] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      o[1][4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[1][ks], ks ? o[1][4] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // context -> this wave's 32 Q rows (asw image layout), one 16-B write per lane per d-tile
    // (qp 0 / 1 fragments paired by swap16), then whole 128-B lines out
    char* ost = const_cast<char*>(qi) + wn * 32 * 128;
    const float inv1 = len > 0 && o[1][4][0] > 0.f ? 1.f / o[1][4][0] : 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      unsigned x0 = xw[dt][0], x1 = xw[dt][1];
      unsigned y0 = pack_bf16x2(o[1][dt][0] * inv1, o[1][dt][1] * inv1);
      unsigned y1 = pack_bf16x2(o[1][dt][2] * inv1, o[1][dt][3] * inv1);
      swap16(x0, y0);
      swap16(x1, y1);
      const int ro = (fc & 1) * 16 + fr, ch = dt * 2 + (fc >> 1);
      *reinterpret_cast<u32x4*>(ost + ro * 128 + asw(ro, ch) * 16) = u32x4{x0, x1, y0, y1};
    }
    const int l2 = opaque_lane();
    const int lr = l2 >> 3, lc8 = l2 & 7;
    bf16* obase = C + (size_t)(tm0 + wm * 128 + wn * 32 + lr) * ldc + h * 64 + lc8 * 8;
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
      const int ro = hh * 8 + lr;
      const u32x4 val = *reinterpret_cast<const u32x4*>(ost + ro * 128 + asw(ro, lc8) * 16);
      u32x4* dst = reinterpret_cast<u32x4*>(obase + (size_t)(hh * 8) * ldc);
      *dst = val;
    }
  };

  const int nk = K / 64;
  int tile = xcd_remap(v, ntiles);
  int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 192;
  set_src(m0, n0);
#pragma unroll
  for (int q = 0; q < 4; ++q) stage(q, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

#define ATPU_H_SYNC_MMA(MMA)                                \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_setprio(1);                            \
  MMA;                                                      \
  __builtin_amdgcn_s_setprio(0);                            \
  __builtin_amdgcn_sched_barrier(0);                        \
  __builtin_amdgcn_s_barrier();                             \
  __builtin_amdgcn_sched_barrier(0)

  int buf = 0, tile_par = 0;
  bool first = true;
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int vn = v + G;
    const bool has_next = vn < ntiles;
    const int cm0 = m0, cn0 = n0;
    // P: K-tile 0 / 1 (compile time: bias / LN staging) or -1
    auto kstep = [&](int t, auto last_c, auto peel_c) {
      constexpr bool last = decltype(last_c)::value;
      constexpr int P = decltype(peel_c)::value;
      const bool more = !last || has_next;
      int kn = t + 1;
      if (last && has_next) {  // the stream runs on into K-tile 0 of the next tile
        tile = xcd_remap(vn, ntiles);
        m0 = (tile / ntn) * 256;
        n0 = (tile % ntn) * 192;
        set_src(m0, n0);
        kn = 0;
      }
      // VMEM ops (oldest first) a wait may leave in flight. K-tile 0 of a tile after the
      // first: the previous tile's epilogue stores (kEpiOps) sit between the last quarters
      // of this K-tile and the next K-tile's; they are retired with Q0/Q1 at p3. Extra ops
      // are issued after the phase-0 staging: this tile's bias at K-tile 0 (1) and the LN
      // data at K-tile 1 (kLn1, 2 with InNorm); the counts below include them (kX) and they
      // retire at the next K-tile's p0, long before the epilogue reads them.
      const bool relax = P == 0 && !first;
      constexpr int kX = P == 0 ? 1 : (P == 1 ? kLn1 : 0);
      // p0
      read_a(buf, 0);
      read_b01(buf);
      if (more) {
        stage(0, kn, buf ^ 1);
        stage(1, kn, buf ^ 1);
        if constexpr (P == 0) {
          // this tile's bias -> LDS (every wave issues one op; waves w and w+4 write the same bytes)
          glds4(bias + cn0 + wn * 48, 48, lds + kBiasOff + tile_par * 1024 + wn * 256);
        }
        if constexpr (P == 1 && kIn) {
          glds4(in_fin + (size_t)cm0 * 2 + wave * 64, 64, lds + kFinOff + wave * 256);
          glds4(colsum + cn0 + wn * 48, 48, lds + kColOff + wn * 256);
        }
        // retires Q2 (read at p1); Q3 (2) + epilogue stores + Q0/Q1 (4) + extras may fly
        if (relax) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + kEpiOps + kX) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + kX) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // Q2 landed, Q3 (2) may fly
      }
      ATPU_H_SYNC_MMA(mma01(0));
      // p1
      read_b2(buf);
      if (more) {
        stage(2, kn, buf ^ 1);
        // retires Q3 (read at p2)
        if (relax) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 + kEpiOps + kX) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 + kX) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      ATPU_H_SYNC_MMA(mma2(0));
      // p2
      read_a(buf, 1);
      if (more) stage(3, kn, buf ^ 1);
      ATPU_H_SYNC_MMA(mma2(1));
      // p3: retires Q0/Q1 of the next K-tile (read at its p0) and everything older
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 + kX) : "memory");
      ATPU_H_SYNC_MMA(mma01(1));
      buf ^= 1;
    };
    kstep(0, std::false_type{}, std::integral_constant<int, 0>{});
    kstep(1, std::false_type{}, std::integral_constant<int, 1>{});
    for (int t = 2; t + 1 < nk; ++t) kstep(t, std::false_type{}, std::integral_constant<int, -1>{});
    kstep(nk - 1, std::true_type{}, std::integral_constant<int, -1>{});
    // both wave groups run the epilogue side by side (as gemm256s)
    __builtin_amdgcn_sched_barrier(0);
    if (wm == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else {
      const int ol = kIn ? opaque_lane() : lane;
      const int ofr = ol & 15, ofc = ol >> 4;
      const float* lb = reinterpret_cast<const float*>(lds + kBiasOff + tile_par * 1024 + wn * 256);
      const float* lc = reinterpret_cast<const float*>(lds + kColOff + wn * 256);
      // MODE 2: the sequence length (scalar load), consumed here: an SMEM load still in flight
      // at the attention would turn every counted LDS wait there into lgkmcnt(0)
      int len = 0;
      if constexpr (MODE == 2) {
        len = min(lens[(cm0 >> 7) + wm], 128);
        asm volatile("" : "+s"(len));
      }
      // the tile's per-column (bias, colsum) and per-row (rstd, rstd*mu) vectors, read from LDS
      // in one batch (read per fragment, each read's latency was exposed on its own)
      f32x4 bv[3], cv[3];
      f32x2 rf[8];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        bv[j] = *reinterpret_cast<const f32x4*>(lb + j * 16 + ofc * 4);
        if constexpr (kIn) cv[j] = *reinterpret_cast<const f32x4*>(lc + j * 16 + ofc * 4);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        rf[i] = kIn ? *reinterpret_cast<const f32x2*>(lds + kFinOff + (wm * 128 + i * 16 + ofr) * 8) : f32x2{1.f, 0.f};
      // value pairs of fragment (i, j) as packed bf16: (acc*rstd - rstd*mu*colsum + bias), the LN
      // math on pairs (v_pk_fma_f32, row scalars broadcast)
      auto frag = [&](int i, int j, unsigned& p0, unsigned& p1) {
        const f32x4 b4 = bv[j];
        f32x4 t;
        if constexpr (kIn) {
          const f32x4 c4 = cv[j];
          const f32x2 rs2 = f32x2{rf[i][0], rf[i][0]}, nrm2 = f32x2{-rf[i][1], -rf[i][1]};
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const f32x2 c2 = __builtin_elementwise_fma(nrm2, f32x2{c4[2 * hh], c4[2 * hh + 1]},
                                                       f32x2{b4[2 * hh], b4[2 * hh + 1]});
            const f32x2 o = __builtin_elementwise_fma(f32x2{acc[i][j][2 * hh], acc[i][j][2 * hh + 1]}, rs2, c2);
            t[2 * hh] = o[0];
            t[2 * hh + 1] = o[1];
          }
        } else {
          t = acc[i][j] + b4;
        }
        p0 = pack_bf16x2(t[0], t[1]);
        p1 = pack_bf16x2(t[2], t[3]);
      };
      if constexpr (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            unsigned p0, p1;
            frag(i, j, p0, p1);
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u32x2*>(C + (size_t)(cm0 + wm * 128 + i * 16 + ofr) * ldc + cn0 + wn * 48 + j * 16 +
                                      ofc * 4) = u32x2{p0, p1};
          }
        }
      } else {
        // Q / K / V images of sequence wm: fragments of row blocks i, i+1 paired by swap16, one
        // 16-B write per lane (lane row G: block i + (G & 1), 8 columns (G >> 1)). 16-column
        // fragments never straddle Q | K | V (48 = 3 x 16): the image is wave-uniform.
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            unsigned x0, x1, y0, y1;
            frag(i, j, x0, x1);
            frag(i + 1, j, y0, y1);
            swap16(x0, y0);
            swap16(x1, y1);
            const int cb = wn * 48 + j * 16, typ = cb >> 6;
            const int r = (i + (ofc & 1)) * 16 + ofr, ch = ((cb & 63) >> 3) + (ofc >> 1);
            *reinterpret_cast<u32x4*>(lds + kImgOff + (wm * 3 + typ) * kAImg + r * 128 + asw(r, ch) * 16) =
                u32x4{x0, x1, y0, y1};
          }
        }
      }
      if constexpr (MODE == 2) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // the images of both sequences are complete
        __builtin_amdgcn_sched_barrier(0);
        attend(cm0, cn0 / 192, len);
        // every wave's image reads are done before group 0 runs ahead into the next tile,
        // whose K-tile 1 is staged into operand buffer 1 (= part of the images)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (wm == 1) __builtin_amdgcn_s_barrier();
    if (!has_next) break;
    v = vn;
    first = false;
    tile_par ^= 1;
  }
#undef ATPU_H_SYNC_MMA
  if (wm == 0) __builtin_amdgcn_s_barrier();  // close the stagger (equal barrier counts)
}

}  // namespace

static void launch_256h(const GemmArgs& g, int mode, const int32_t* lens, float scale, hipStream_t s) {
  ATPU_CHECK(g.N % 192 == 0 && g.M % 256 == 0 && g.K % 64 == 0 && g.K >= 256,
             "gemm256h: N % 192, M % 256 == 0, K % 64 == 0 and K >= 256");
  ATPU_CHECK(g.epi == kEpiBias || g.epi == (kEpiBias | kEpiInNorm), "gemm256h: epilogue bias or bias|InNorm");
  ATPU_CHECK(!(g.epi & kEpiInNorm) || (g.in_fin && g.colsum), "gemm256h: InNorm needs in_fin and colsum");
  ATPU_CHECK(g.bias && g.ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(g.C) & 7) == 0, "gemm256h: bias, 8-B rows");
  ATPU_CHECK((size_t)g.M * g.lda * 2 < (1ull << 32) && (size_t)g.N * g.ldb * 2 < (1ull << 32),
             "gemm256h: A and Bt under 4 GiB (32-bit staging offsets)");
  ATPU_CHECK(mode >= 0 && mode <= 2, "gemm256h: mode 0 (store), 1 (timing only) or 2 (attention)");
  if (mode == 2) {
    // the images live in operand buffer 1: the last K-tile of every tile must be staged there
    ATPU_CHECK((g.K / 64) % 2 == 0, "qkv_attention: K / 64 must be even");
    ATPU_CHECK(lens && g.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0,
               "qkv_attention: lens and 16-B aligned context rows");
  }
  const int tiles = (g.M / 256) * (g.N / 192);
  int nb = std::min(tiles, num_cus());
  if (nb >= 8) nb &= ~7;
#define ATPU_GH(E, MD)                                                                                          \
  hipLaunchKernelGGL((gemm256h_kernel<E, MD>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, g.ldc, \
                     g.bias, g.in_fin, g.colsum, g.M, g.N, g.K, lens, scale)
  if (g.epi & kEpiInNorm) {
    if (mode == 0) ATPU_GH(kEpiBias | kEpiInNorm, 0);
    else if (mode == 1) ATPU_GH(kEpiBias | kEpiInNorm, 1);
    else ATPU_GH(kEpiBias | kEpiInNorm, 2);
  } else {
    if (mode == 0) ATPU_GH(kEpiBias, 0);
    else if (mode == 1) ATPU_GH(kEpiBias, 1);
    else ATPU_GH(kEpiBias, 2);
  }
#undef ATPU_GH
  ATPU_HIP_CHECK(hipGetLastError());
}

void gemm256h(const GemmArgs& g, int mode, hipStream_t s) {
  ATPU_CHECK(mode == 0 || mode == 1, "gemm256h: mode 0 (store) or 1 (timing only, no epilogue)");
  launch_256h(g, mode, nullptr, 0.f, s);
}

void qkv_attention(const GemmArgs& g, const int32_t* lens, float scale, hipStream_t s) {
  launch_256h(g, 2, lens, scale, s);
}

}  // namespace atpu
