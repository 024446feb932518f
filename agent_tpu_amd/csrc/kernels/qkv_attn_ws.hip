// BERT QKV projection + self-attention, wave-specialised ("give the
// attention to one wave group while the other runs the next tile"), and the same structure
// as a GEMM whose epilogue leaves through dedicated waves ("dedicated epilogue waves").
// DEV BUILD ONLY (-DATPU_DEV_BUILD, build.py --dev): measured slower than the release kernels
// (QKV+attention 489 vs 479 us, FFN1 693 vs 592 us at the bench shape; docs/PERF_NOTES.md
// "Wave-specialised kernels"), kept as the recorded experiment; the release .so has stubs.
//
// qkv_attn.hip runs the attention of a tile in its epilogue with all 8 waves, so the MFMA
// pipes idle for the image writes, the softmax and the context stores (~35 % of that kernel).
// Here a tile is ONE sequence x one head (128 rows x 192 columns: the head's Q | K | V) and
// the 8 waves of the workgroup have two roles:
//  * MMA waves 0-3: the main loop only. Wave (wm, wn) owns rows wm*64..+64, columns
//    wn*96..+96 (4 x 6 MFMA fragments). Per 64-deep K-tile: read the k-step-1 fragments,
//    MFMAs of k-step 0, wait, workgroup barrier, read k-step 0 of the next K-tile, MFMAs of
//    k-step 1 - the fragment reads of one k-step fly under the other's 24 MFMAs. No
//    LDS-DMA issue on these waves. After the last K-tile: bias (+ InNorm) -> bf16 Q, K, V
//    images of the sequence in LDS, barrier, next tile.
//  * loader/attention waves 4-7: between two barriers ("slots") they issue the LDS-DMA of the
//    K-tiles ahead into the ring slots the barrier just freed, run one piece of the PREVIOUS
//    tile's attention (each wave 32 queries; the math of qkv_attn.hip's attend()), and wait
//    for their DMA before arriving at the next barrier.
// Barriers per tile: one per K-tile (KB_t: K-tile t's ring slots free, K-tile t+1 landed) and
// one after the image writes (EB). Slots of the loader waves, tile T (NK K-tiles):
//   slot -1 (EB(T-1) .. KB_0): vectors (bias, colsum, fin) of T; attention piece 1 of T-1
//   slot s  (KB_s .. KB_s+1 / EB): DMA of B K-tile s+2 and A K-tile s+AS (past NK: the next
//           tile's); pieces 2-10 of T-1 in slots 0-8, its context stores in slot 9
// The A operand ring is AS deep (2, or 3 with ws_variant bit 3 at K = 768: the activation
// tiles, first touched in HBM, get two slots of latency), the B (weight) ring 2 deep. The
// attention of T-1 is over (its LDS reads retired) before KB_NK-1 of T, after which the MMA
// waves overwrite the images. The last tile's attention runs after the final barrier.
//
// LDS: A ring AS x 16 KiB, B ring 2 x 24 KiB, 3 attention images (48 KiB), bias / colsum / fin
// (2.5 KiB): 130.5 / 146.5 KiB, one workgroup per CU.
// MODE 0 stores Q|K|V (bf16, head order) instead of attention (exactness of the GEMM part);
// MODE 1 is timing-only (no epilogue). MODE 3 / 4: a plain GEMM (N % 192) whose output
// leaves through the loader waves (MODE 3 with GELU: BERT's FFN1), the MMA waves' epilogue
// only the bias / InNorm image. NK = K / 64: 12 (BERT-base), 16 (BERT-large).
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/lds_ops.h"

#include <algorithm>
#include <vector>

namespace atpu {
#ifdef ATPU_DEV_BUILD
namespace {

constexpr int kWImgA = 128 * 128;  // A operand image: 128 rows x 128 B
constexpr int kWImgB = 192 * 128;  // B operand image: 192 rows x 128 B
// LDS layout for AS A-stages: A ring, B ring (2), Q/K/V images, bias / colsum / fin
template <int AS>
struct WsLds {
  static constexpr int kB = AS * kWImgA;
  static constexpr int kAttn = kB + 2 * kWImgB;
  static constexpr int kBias = kAttn + 3 * kAttnImg;  // [192] fp32
  static constexpr int kCol = kBias + 768;            // [192] fp32 colsum
  static constexpr int kFin = kCol + 768;             // [128][2] fp32 (rstd, rstd*mu)
  static constexpr int kSize = kFin + 1024;
  static_assert(kSize <= 160 * 1024, "LDS budget");
};

// Diagnostic build only (-DATPU_WS_STAMPS, a separate .so; the release kernel has no stamps):
// s_memtime cycle sums per workgroup, written with vector stores to a buffer of their own that
// no output reads. MMA wave 0: [0] K-tile barrier waits, [1] image-barrier waits, [2] image
// writes, [3] total, [4] tiles; loader wave 4: [5] barrier waits, [6] DMA waits, [7] total,
// [16 + c] attention piece c (1..11). 32 words per workgroup.
#ifdef ATPU_WS_STAMPS
__device__ unsigned long long g_ws_stamps[1024 * 32];
#define WS_NOW() __builtin_amdgcn_s_memtime()
#define WS_T(v)                         \
  __builtin_amdgcn_sched_barrier(0);    \
  const uint64_t v = WS_NOW();          \
  __builtin_amdgcn_sched_barrier(0)
#define WS_ACC(i, t0)                   \
  __builtin_amdgcn_sched_barrier(0);    \
  st[i] += WS_NOW() - (t0);             \
  __builtin_amdgcn_sched_barrier(0)
#else
#define WS_T(v)
#define WS_ACC(i, t0)
#endif

template <int EPI, int MODE, int NK, int AS>
__global__ __launch_bounds__(512, 1) void qkv_ws_kernel(const bf16* __restrict__ A, int lda,
                                                        const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                        int ldc, const float* __restrict__ bias,
                                                        const float* __restrict__ in_fin,
                                                        const float* __restrict__ colsum, int M, int N,
                                                        const int32_t* __restrict__ lens, float scale, int var) {
  static_assert(NK % 2 == 0 && NK % AS == 0 && NK >= 11,
                "K-tiles: whole rings per tile (every tile starts in stage 0), 11 attention slots");
  constexpr bool kIn = EPI & kEpiInNorm;
  using L = WsLds<AS>;
  constexpr int kWAttn = L::kAttn, kWBias = L::kBias, kWCol = L::kCol, kWFin = L::kFin;
  __shared__ __attribute__((aligned(16))) char lds[L::kSize];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = N / 192, ntiles = (M / 128) * ntn;
  const int G = gridDim.x;
  int v = blockIdx.x;
  if (v >= ntiles) return;
  // tile order: consecutive tiles (one XCD's concurrent set, xcd_remap) walk groups of GM
  // row blocks x all column tiles, the GM row blocks fastest (var bits 5-6: GM = 1, 2, 4, 8).
  // GM = 1 is the column-fastest order; with GM = 4 an XCD's 32 concurrent tiles need 4 A and
  // 8 B panels (3.2 MB at K = 768) instead of every B panel (4.7 MB for FFN1's N = 3072).
  const int mt = M / 128, gm_log = (var >> 5) & 3;
  auto tile_of = [&](int vv, int& m0, int& n0) {
    const int t = xcd_remap(vv, ntiles);
    const int gsz = ntn << gm_log, g = t / gsz, r = t - g * gsz;
    const int gm = min(1 << gm_log, mt - (g << gm_log));
    m0 = ((g << gm_log) + r % gm) * 128;
    n0 = (r / gm) * 192;
  };
  auto opaque_lane = [] {
    int l = __lane_id();
    asm volatile("" : "+v"(l));
    return l;
  };
  const int fr = lane & 15, fc = lane >> 4;
#ifdef ATPU_WS_STAMPS
  uint64_t st[32] = {};
  const uint64_t st_start = WS_NOW();
  auto st_flush = [&](int lo, int hi) {
    st[lo == 0 ? 3 : 7] = WS_NOW() - st_start;
    if (lane == 0)
      for (int i = lo; i < hi; ++i) g_ws_stamps[blockIdx.x * 32 + i] = st[i];
  };
#endif

  if (wave < 4) {
    // =============================== MMA waves ===============================
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[4][6];
    bf16x8 a0[4], b0[6], a1[4], b1[6];
    // K-tile t: A image in ring slot t % AS, B image in t & 1
    auto read_ks = [&](int t, int ks, bf16x8(&af)[4], bf16x8(&bf)[6]) {
      const char* ia = lds + (t % AS) * kWImgA;
      const char* ib = lds + L::kB + (t & 1) * kWImgB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(ia + r * 128 + hsw(r, ks * 4 + fc) * 16);
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int r = wn * 96 + j * 16 + fr;
        bf[j] = *reinterpret_cast<const bf16x8*>(ib + r * 128 + hsw(r, ks * 4 + fc) * 16);
      }
    };
    auto mma = [&](bf16x8(&af)[4], bf16x8(&bf)[6]) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    };
    if (var & 1) __builtin_amdgcn_s_setprio(2);
    __builtin_amdgcn_s_barrier();  // K-tiles 0 and 1 of the first tile landed
    __builtin_amdgcn_sched_barrier(0);
    for (;;) {
      int m0, n0;
      tile_of(v, m0, n0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      read_ks(0, 0, a0, b0);
#pragma unroll
      for (int t = 0; t < NK; ++t) {
        // the reads of one k-step are issued before the other k-step's 24 MFMAs (left to the
        // scheduler, they sank among the last MFMAs and their latency showed at the next group)
        read_ks(t, 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        WS_T(t_kb);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // KB_t
        WS_ACC(0, t_kb);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < NK) read_ks(t + 1, 0, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
      }
      WS_T(t_epi);
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 6; ++j) asm volatile("" ::"v"(acc[i][j]));
      } else {
        // bias / colsum per column, (rstd, rstd*mu) per row, from LDS in one batch
        const float* lb = reinterpret_cast<const float*>(lds + kWBias) + wn * 96;
        const float* lc = reinterpret_cast<const float*>(lds + kWCol) + wn * 96;
        f32x4 bv[6], cv[6];
        f32x2 rf[4];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          bv[j] = *reinterpret_cast<const f32x4*>(lb + j * 16 + fc * 4);
          if constexpr (kIn) cv[j] = *reinterpret_cast<const f32x4*>(lc + j * 16 + fc * 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          rf[i] = kIn ? *reinterpret_cast<const f32x2*>(lds + kWFin + (wm * 64 + i * 16 + fr) * 8) : f32x2{1.f, 0.f};
        // value pairs of fragment (i, j) as packed bf16: acc*rstd - rstd*mu*colsum + bias
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
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
              unsigned p0, p1;
              frag(i, j, p0, p1);
              *reinterpret_cast<u32x2*>(C + (size_t)(m0 + wm * 64 + i * 16 + fr) * ldc + n0 + wn * 96 + j * 16 +
                                        fc * 4) = u32x2{p0, p1};
            }
        } else {
          // Q / K / V images: row blocks i, i+1 paired by swap16, one 16-B write per lane (lane
          // row G: block i + (G & 1), 8 columns (G >> 1)); a 16-column fragment never straddles
          // Q | K | V, so the image is wave-uniform
#pragma unroll
          for (int i = 0; i < 4; i += 2)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
              unsigned x0, x1, y0, y1;
              frag(i, j, x0, x1);
              frag(i + 1, j, y0, y1);
              swap16(x0, y0);
              swap16(x1, y1);
              const int cb = wn * 96 + j * 16, typ = cb >> 6;
              const int r = wm * 64 + (i + (fc & 1)) * 16 + fr, ch = ((cb & 63) >> 3) + (fc >> 1);
              *reinterpret_cast<u32x4*>(lds + kWAttn + typ * kAttnImg + r * 128 + asw(r, ch) * 16) =
                  u32x4{x0, x1, y0, y1};
            }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      WS_ACC(2, t_epi);
      WS_T(t_eb);
      __builtin_amdgcn_s_barrier();  // EB: the images are complete
      WS_ACC(1, t_eb);
      __builtin_amdgcn_sched_barrier(0);
#ifdef ATPU_WS_STAMPS
      st[4] += 1;
#endif
      v += G;
      if (v >= ntiles) break;
    }
#ifdef ATPU_WS_STAMPS
    if (wave == 0) st_flush(0, 5);
#endif
    return;
  }

  // ============================ loader / attention waves ============================
  const int l = wave - 4;
  if (var & 16) __builtin_amdgcn_s_setprio(1);
  // LDS-DMA: this wave stages A rows l*32..+32 (4 x 8 rows) and B rows l*48..+48 (6 x 8 rows)
  // of a K-tile; the lane's 32-bit source offsets carry the swizzle (the DMA writes lane-linear)
  uint32_t soffA[4], soffB[6];
  auto set_srcA = [&](int m0) {
    const int ln = opaque_lane();
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int r = l * 32 + a * 8 + (ln >> 3);
      soffA[a] = (uint32_t)(((size_t)(m0 + r) * lda + hsw(r, ln & 7) * 8) * 2);
    }
  };
  auto set_srcB = [&](int n0) {
    const int ln = opaque_lane();
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int r = l * 48 + b * 8 + (ln >> 3);
      soffB[b] = (uint32_t)(((size_t)(n0 + r) * ldb + hsw(r, ln & 7) * 8) * 2);
    }
  };
  auto stageA = [&](int kt, int slot) {
    const char* ga = reinterpret_cast<const char*>(A) + kt * 128;
#pragma unroll
    for (int a = 0; a < 4; ++a) glds16(ga + soffA[a], lds + slot * kWImgA + (l * 32 + a * 8) * 128);
  };
  auto stageB = [&](int kt, int slot) {
    const char* gb = reinterpret_cast<const char*>(Bt) + kt * 128;
#pragma unroll
    for (int b = 0; b < 6; ++b) glds16(gb + soffB[b], lds + L::kB + slot * kWImgB + (l * 48 + b * 8) * 128);
  };
  auto glds4 = [&](const float* ubase, char* ldst) {
    __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)(ubase + opaque_lane()), (ATPU_LDS_AS void*)ldst, 4,
                                     0, 0);
  };
  // the tile's epilogue vectors: bias / colsum [n0..+192], fin rows [m0..+128]
  auto stage_vec = [&](int m0, int n0) {
    if constexpr (MODE != 1) {
      if (l < 3) {
        glds4(bias + n0 + l * 64, lds + kWBias + l * 256);
        if constexpr (kIn) glds4(colsum + n0 + l * 64, lds + kWCol + l * 256);
      }
      if constexpr (kIn) glds4(in_fin + (size_t)m0 * 2 + l * 64, lds + kWFin + l * 256);
    }
  };

  // end of a slot: its DMA landed (with AS = 3 the A ring's 4 ops, issued last, may fly one
  // slot longer: vmcnt(4)), its LDS work retired, barrier
  auto slot_end = [&](auto fly_c) {
    constexpr int fly = decltype(fly_c)::value;
    __builtin_amdgcn_sched_barrier(0);
    WS_T(t_vm);
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(fly) : "memory");
    WS_ACC(6, t_vm);
    WS_T(t_bar);
    __builtin_amdgcn_s_barrier();
    WS_ACC(5, t_bar);
    __builtin_amdgcn_sched_barrier(0);
  };
  using Fly0 = std::integral_constant<int, 0>;
  using FlyA = std::integral_constant<int, AS == 3 ? 4 : 0>;
  int m0, n0;
  tile_of(v, m0, n0);
  set_srcA(m0);
  set_srcB(n0);
  stageB(0, 0);
  stageB(1, 1);
#pragma unroll
  for (int k = 0; k < AS; ++k) stageA(k, k);
  slot_end(Fly0{});  // the first tile's B K-tiles 0-1 and A K-tiles 0..AS-1 landed
  int pm0 = 0, ph = 0, pn0 = 0;
  // one tile of the loader waves; ATT: the previous tile's attention runs in its slots (a
  // compile-time flag - a runtime `if (pending)` around every piece made the attention state
  // of both paths live at each join: ~100 VGPRs of spills). Returns false after the last tile.
  auto tile_body = [&](auto att_c) -> bool {
    constexpr bool pending = decltype(att_c)::value && MODE >= 2;
    const int vn = v + G;
    const bool has_next = vn < ntiles;
    int nm0 = 0, nn0 = 0;
    if (has_next) tile_of(vn, nm0, nn0);
    // ---- attention of the previous tile (pm0, head ph), queries l*32..+32, in pieces; the
    // state is local to one tile (declared outside the tile loop it was loop-carried: spills)
    const char* qi = lds + kWAttn;
    const char* ki = qi + kAttnImg;
    const char* vi = qi + 2 * kAttnImg;
    const float cl = scale * 1.4426950408889634f;
    int len = 0;
    bf16x8 qf[2][2], kf[8][2];
    f32x4 s[2][8];
    bf16x8 pf[2][4];
    f32x4 o[2][5];
    unsigned xw[4][2];
    bf16x4 vlo[4][4], vhi[4][4];
    bf16x8 ones;
  #pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
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
    auto vfrag = [&](int ks, int dt) {
      bf16x8 vf;
  #pragma unroll
      for (int e = 0; e < 4; ++e) {
        vf[e] = vlo[ks][dt][e];
        vf[4 + e] = vhi[ks][dt][e];
      }
      return vf;
    };
    // The attention in 11 pieces, one per slot (slots -1 .. 9), each well under the MMA waves'
    // K-tile: the measured (stamped) chunks of a 5- and an 8-way split ran 550-1300 cycles under
    // the main loop's LDS and MFMA traffic, and every one longer than the MMA waves' ~1170-cycle
    // K-tile held them at the next barrier (29 % of their cycles).
    //  1: len (scalar load, consumed before any counted LDS wait), Q and K fragment reads,
    //     S(qp 0) of key tiles 0-3 with counted waits;  2: key tiles 4-7, mask;
    //  3: S(qp 1);  4: softmax(qp 0), mask(qp 1);  5: the 32 transposed V reads, softmax(qp 1);
    //  6, 7: P0.V (key steps 0-1, 2-3);  8, 9: the qp 0 context packed, P1.V;
    //  10: context -> this wave's 32 Q rows (free once read) and back as whole 128-B rows;
    //  11: the global stores (issued at the start of slot 9, before its DMA).
    // LDS addresses come from an opaque lane id inside each piece: from `lane` they are
    // loop-invariant, and hoisted out of the tile loop they held ~60 VGPRs (spills).
    u32x4 cval[4];
    auto qk0 = [&](auto kt_c) {
      constexpr int kt = decltype(kt_c)::value;
      if constexpr (kt == 0) {
        lgkm_wait<14>(qf[0][0], qf[0][1]);
        asm volatile("" : "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(kf[0][0]), "+v"(kf[0][1]));
      } else if constexpr (kt < 4) {
        lgkm_wait<14 - 2 * kt>(kf[kt][0], kf[kt][1]);
      } else {
        lgkm_wait<0>(kf[kt][0], kf[kt][1]);  // landed at the slot end: pins only
      }
      s[0][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[0][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      s[0][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[0][1], s[0][kt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    // the V reads retired (slot end, or here for the last tile) and their registers pinned
    // after the wait: the tr16 asm outputs look available to the compiler at issue
    auto v_landed = [&]() {
  #pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[ks][0]), "+v"(vlo[ks][1]), "+v"(vlo[ks][2]), "+v"(vlo[ks][3]),
                     "+v"(vhi[ks][0]), "+v"(vhi[ks][1]), "+v"(vhi[ks][2]), "+v"(vhi[ks][3])::"memory");
    };
    auto pv = [&](int qp, int ks0) {
  #pragma unroll
      for (int ks = ks0; ks < ks0 + 2; ++ks) {
  #pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          o[qp][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfrag(ks, dt), pf[qp][ks],
                                                              ks ? o[qp][dt] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        o[qp][4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qp][ks], ks ? o[qp][4] : f32x4{0.f, 0.f, 0.f, 0.f},
                                                           0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    // 1 / (row sum of the bf16 P): v_rcp_f32 (1 ulp) before the bf16 rounding of the context
    auto inv_sum = [&](int qp) { return len > 0 && o[qp][4][0] > 0.f ? __builtin_amdgcn_rcpf(o[qp][4][0]) : 0.f; };
    auto piece_impl = [&](int c) {
      if (c == 1) {
        len = min(lens[pm0 >> 7], 128);
        asm volatile("" : "+s"(len));
        const int ln = opaque_lane(), fr = ln & 15, fc = ln >> 4;
  #pragma unroll
        for (int qp = 0; qp < 2; ++qp)
  #pragma unroll
          for (int ds = 0; ds < 2; ++ds) {
            const int r = l * 32 + qp * 16 + fr;
            qf[qp][ds] = ds_read128(qi + r * 128 + asw(r, ds * 4 + fc) * 16);
          }
  #pragma unroll
        for (int kt = 0; kt < 8; ++kt)
  #pragma unroll
          for (int ds = 0; ds < 2; ++ds) {
            const int r = kt * 16 + fr;
            kf[kt][ds] = ds_read128(ki + r * 128 + asw(r, ds * 4 + fc) * 16);
          }
        qk0(std::integral_constant<int, 0>{});
        qk0(std::integral_constant<int, 1>{});
        qk0(std::integral_constant<int, 2>{});
        qk0(std::integral_constant<int, 3>{});
      } else if (c == 2) {
        qk0(std::integral_constant<int, 4>{});
        qk0(std::integral_constant<int, 5>{});
        qk0(std::integral_constant<int, 6>{});
        qk0(std::integral_constant<int, 7>{});
        mask(0);
      } else if (c == 3) {
  #pragma unroll
        for (int kt = 0; kt < 8; ++kt) {
          s[1][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[1][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          s[1][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[1][1], s[1][kt], 0, 0, 0);
        }
      } else if (c == 4) {
        softmax(0);
        mask(1);
      } else if (c == 5) {
        const int ln = opaque_lane();
        const int tq = (ln >> 2) & 3, tp = ln & 3;
        const int k0 = (ln >> 4) * 4 + tq;
        const char* row = vi + k0 * 128 + (tp & 1) * 8;
  #pragma unroll
        for (int ks = 0; ks < 4; ++ks)
  #pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const int cc = asw(k0, dt * 2 + (tp >> 1)) * 16;
            vlo[ks][dt] = tr16(row + ks * 32 * 128 + cc);
            vhi[ks][dt] = tr16(row + (ks * 32 + 16) * 128 + cc);
          }
        __builtin_amdgcn_sched_barrier(0);
        softmax(1);
      } else if (c == 6) {
        v_landed();
        pv(0, 0);
      } else if (c == 7) {
        pv(0, 2);
      } else if (c == 8) {
        const float inv0 = inv_sum(0);
  #pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          xw[dt][0] = pack_bf16x2(o[0][dt][0] * inv0, o[0][dt][1] * inv0);
          xw[dt][1] = pack_bf16x2(o[0][dt][2] * inv0, o[0][dt][3] * inv0);
        }
        pv(1, 0);
      } else if (c == 9) {
        pv(1, 2);
      } else if (c == 10) {
        const int ln = opaque_lane(), fr = ln & 15, fc = ln >> 4;
        char* ost = const_cast<char*>(qi) + l * 32 * 128;
        const float inv1 = inv_sum(1);
  #pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          unsigned x0 = xw[dt][0], x1 = xw[dt][1];
          unsigned y0 = pack_bf16x2(o[1][dt][0] * inv1, o[1][dt][1] * inv1);
          unsigned y1 = pack_bf16x2(o[1][dt][2] * inv1, o[1][dt][3] * inv1);
          swap16(x0, y0);
          swap16(x1, y1);
          const int ro = (fc & 1) * 16 + fr, ch = dt * 2 + (fc >> 1);
          ds_write128(ost + ro * 128 + asw(ro, ch) * 16, u32x4{x0, x1, y0, y1});
        }
        const int lr = ln >> 3, lc8 = ln & 7;
  #pragma unroll
        for (int hh = 0; hh < 4; ++hh) {
          const int ro = hh * 8 + lr;
          cval[hh] = ds_read128u(ost + ro * 128 + asw(ro, lc8) * 16);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cval[0]), "+v"(cval[1]), "+v"(cval[2]), "+v"(cval[3])::"memory");
      } else if (c == 11) {
        const int ln = opaque_lane();
        const int lr = ln >> 3, lc8 = ln & 7;
        bf16* obase = C + (size_t)(pm0 + l * 32 + lr) * ldc + ph * 64 + lc8 * 8;
  #pragma unroll
        for (int hh = 0; hh < 4; ++hh) *reinterpret_cast<u32x4*>(obase + (size_t)(hh * 8) * ldc) = cval[hh];
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    // MODE 3 / 4 (a GEMM whose output leaves through the loader waves): piece c = 1..6 takes
    // 16 rows (two 8-row blocks) of image (c - 1) >> 1 of this wave's 32 rows, applies GELU
    // (MODE 3, on the bf16-rounded pre-activation, as the bf16 model's gelu(linear(x))) and
    // stores whole 128-B rows, non-temporal
    auto store_piece = [&](int c) {
      const int typ = (c - 1) >> 1, rb = (c - 1) & 1;
      const int ln = opaque_lane(), ch = ln & 7;
      u32x4 v[2];
      int row[2];
  #pragma unroll
      for (int h = 0; h < 2; ++h) {
        row[h] = l * 32 + rb * 16 + h * 8 + (ln >> 3);
        v[h] = ds_read128u(qi + typ * kAttnImg + row[h] * 128 + asw(row[h], ch) * 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1])::"memory");
      if constexpr (MODE == 3) {
        float f[16];
  #pragma unroll
        for (int h = 0; h < 2; ++h)
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[h * 8 + 2 * e] = __uint_as_float(v[h][e] << 16);
            f[h * 8 + 2 * e + 1] = __uint_as_float(v[h][e] & 0xffff0000u);
          }
        gelu_poly16_v<1>(f);  // scalar FMAs: packed ones beside the MMA waves' MFMAs cost ~3x (MICROARCH)
  #pragma unroll
        for (int h = 0; h < 2; ++h)
  #pragma unroll
          for (int e = 0; e < 4; ++e) v[h][e] = pack_bf16x2(f[h * 8 + 2 * e], f[h * 8 + 2 * e + 1]);
      }
  #pragma unroll
      for (int h = 0; h < 2; ++h)
        __builtin_nontemporal_store(v[h], reinterpret_cast<u32x4*>(C + (size_t)(pm0 + row[h]) * ldc + pn0 + typ * 64 +
                                                                   ch * 8));
      __builtin_amdgcn_sched_barrier(0);
    };
    auto piece = [&](int c) {
      WS_T(t_c);
      if constexpr (MODE == 2) piece_impl(c);
      if constexpr (MODE >= 3) store_piece(c);
#ifdef ATPU_WS_STAMPS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      st[16 + c] += WS_NOW() - t_c;
#endif
    };
    // slot -1: the tile's epilogue vectors, piece 1
    stage_vec(m0, n0);
    if constexpr (pending) piece(1);
    if constexpr (pending && MODE >= 3) slot_end(std::integral_constant<int, 2>{});  // KB_0; stores fly
    else slot_end(Fly0{});  // KB_0
    // slots 0 .. NK-1: the DMA of B K-tile s + 2 and A K-tile s + AS (past NK: the next tile's,
    // its offsets switched at its K-tile 0). MODE 2: pieces 2-10 in slots 0-8, the stores in
    // slot 9; MODE 3 / 4: pieces 2-6 in slots 0-4, after the DMA
    constexpr int kLast = MODE == 2 ? 10 : 6;
#pragma unroll
    for (int sl = 0; sl < NK; ++sl) {
      if (sl == 9 && MODE == 2) {
        if constexpr (pending) piece(11);
      }
      const int kb = sl + 2, ka = sl + AS;
      if (kb < NK) {
        stageB(kb, kb & 1);
      } else if (has_next) {
        if (kb == NK) set_srcB(nn0);
        stageB(kb - NK, (kb - NK) & 1);
      }
      if (ka < NK) {
        stageA(ka, ka % AS);
      } else if (has_next) {
        if (ka == NK) set_srcA(nm0);
        stageA(ka - NK, ka % AS);
      }
      if (sl + 2 <= kLast) {
        if constexpr (pending) piece(sl + 2);
      }
      // MODE 3 / 4: the piece's 2 stores, issued after the DMA, may fly one slot longer
      constexpr bool st2 = MODE >= 3 && pending;
      if (st2 && sl + 2 <= kLast) {
        if (ka < NK || has_next) slot_end(std::integral_constant<int, FlyA::value + 2>{});
        else slot_end(std::integral_constant<int, 2>{});
      } else {
        if (ka < NK || has_next) slot_end(FlyA{});  // KB_sl+1, or EB after the last slot
        else slot_end(Fly0{});
      }
    }
    pm0 = m0;
    ph = n0 / 192;
    pn0 = n0;
    if (!has_next) {
      // the last tile's attention, after the final barrier
      if constexpr (MODE >= 3) {
        piece(1);
        piece(2);
        piece(3);
        piece(4);
        piece(5);
        piece(6);
      }
      if constexpr (MODE == 2) {
        piece(1);
        piece(2);
        piece(3);
        piece(4);
        piece(5);
        piece(6);
        piece(7);
        piece(8);
        piece(9);
        piece(10);
        piece(11);
      }
      return false;
    }
    v = vn;
    m0 = nm0;
    n0 = nn0;
    return true;
  };
  if (tile_body(std::false_type{}))
    while (tile_body(std::true_type{})) {
    }
#ifdef ATPU_WS_STAMPS
  if (wave == 4) st_flush(5, 32);
#endif
}

}  // namespace

#ifdef ATPU_WS_STAMPS
std::vector<unsigned long long> ws_stamps(int nblocks) {
  std::vector<unsigned long long> out((size_t)nblocks * 32);
  ATPU_HIP_CHECK(hipMemcpyFromSymbol(out.data(), HIP_SYMBOL(g_ws_stamps), out.size() * 8, 0, hipMemcpyDeviceToHost));
  return out;
}
#else
std::vector<unsigned long long> ws_stamps(int) { return {}; }
#endif

static int g_ws_variant = 0;
// experiment knob (benchmarks): bit 0 = MMA waves at s_setprio 2; bit 3 = a 3-deep A ring
// (K = 768); bit 4 = loader waves at s_setprio 1; bits 5-6 = log2 of the row blocks per tile
// group (tile_of); set >= 0 switches, returns the current
int ws_variant(int set) {
  if (set >= 0) g_ws_variant = set;
  return g_ws_variant;
}

bool qkv_attention_ws_ok(int M, int N, int K) {
  return N % 192 == 0 && M % 128 == 0 && (K == 768 || K == 1024) && (size_t)M * K * 2 < (1ull << 32) &&
         (size_t)N * K * 2 < (1ull << 32);
}

void qkv_attention_ws(const GemmArgs& g, int mode, const int32_t* lens, float scale, hipStream_t s) {
  ATPU_CHECK(qkv_attention_ws_ok(g.M, g.N, g.K) && g.lda >= g.K && g.ldb >= g.K,
             "qkv_attention_ws: N % 192 == 0, M % 128 == 0, K 768 or 1024, A and Bt under 4 GiB");
  ATPU_CHECK(g.epi == kEpiBias || g.epi == (kEpiBias | kEpiInNorm), "qkv_attention_ws: epilogue bias or bias|InNorm");
  ATPU_CHECK(!(g.epi & kEpiInNorm) || (g.in_fin && g.colsum), "qkv_attention_ws: InNorm needs in_fin and colsum");
  ATPU_CHECK(g.bias && g.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0,
             "qkv_attention_ws: bias, 16-B aligned output rows");
  ATPU_CHECK(mode >= 0 && mode <= 4,
             "qkv_attention_ws: mode 0 (store QKV), 1 (timing only), 2 (attention), 3 (GELU GEMM), 4 (GEMM)");
  ATPU_CHECK(mode != 2 || lens, "qkv_attention_ws: lens");
  const int tiles = (g.M / 128) * (g.N / 192);
  int nb = std::min(tiles, num_cus());
  if (nb >= 8) nb &= ~7;
  const int var = ws_variant(-1);
#define ATPU_WS(E, MD, NKV, ASV)                                                                              \
  hipLaunchKernelGGL((qkv_ws_kernel<E, MD, NKV, ASV>), dim3(nb), dim3(512), 0, s, g.A, g.lda, g.Bt, g.ldb, g.C, \
                     g.ldc, g.bias, g.in_fin, g.colsum, g.M, g.N, lens, scale, var)
#define ATPU_WS_NK(E, MD)                    \
  if (g.K == 768 && (var & 8)) ATPU_WS(E, MD, 12, 3); \
  else if (g.K == 768) ATPU_WS(E, MD, 12, 2); \
  else ATPU_WS(E, MD, 16, 2)
#define ATPU_WS_MODE(E)                \
  if (mode == 0) { ATPU_WS_NK(E, 0); } \
  else if (mode == 1) { ATPU_WS_NK(E, 1); } \
  else if (mode == 2) { ATPU_WS_NK(E, 2); } \
  else if (mode == 3) { ATPU_WS_NK(E, 3); } \
  else { ATPU_WS_NK(E, 4); }
  if (g.epi & kEpiInNorm) {
    ATPU_WS_MODE(kEpiBias | kEpiInNorm);
  } else {
    ATPU_WS_MODE(kEpiBias);
  }
#undef ATPU_WS_MODE
#undef ATPU_WS_NK
#undef ATPU_WS
  ATPU_HIP_CHECK(hipGetLastError());
}

#else  // release build: the measured-slower experiment is not compiled (docs/PERF_NOTES.md)
std::vector<unsigned long long> ws_stamps(int) { return {}; }
int ws_variant(int) { return 0; }
bool qkv_attention_ws_ok(int, int, int) { return false; }
void qkv_attention_ws(const GemmArgs&, int, const int32_t*, float, hipStream_t) {
  ATPU_CHECK(false, "qkv_attention_ws: wave-specialised kernels are in the dev build only (build.py --dev)");
}
#endif  // ATPU_DEV_BUILD

}  // namespace atpu
