// BERT QKV projection + self-attention, wave-specialised ("give the
// attention to one wave group while the other runs the next tile").
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
//    K-tile two ahead into the operand stage the barrier just freed, run one chunk of the
//    PREVIOUS tile's attention (each wave 32 queries, the schedule of qkv_attn.hip's attend()),
//    and wait for their DMA before arriving at the next barrier.
// Barriers per tile: one per K-tile (KB_t: stage of K-tile t free, K-tile t+1 landed) and one
// after the image writes (EB). Slots of the loader waves, tile T (NK K-tiles):
//   slot -1 (EB(T-1) .. KB_0): vectors (bias, colsum, fin) of T; attention chunk 1 of T-1
//   slot s  (KB_s .. KB_s+1), s = 0..NK-2: DMA of K-tile s+2 (s = NK-2: K-tile 0 of T+1);
//           chunks 2, 3, 4+5 of T-1 in slots 0-2, its context stores in slot 3
//   slot NK-1 (KB_NK-1 .. EB(T)): DMA of K-tile 1 of T+1
// The attention of T-1 is over (its LDS reads retired) before KB_NK-1 of T, after which the
// MMA waves overwrite the images. The last tile's attention runs after the final barrier.
//
// LDS: 2 operand stages x 40 KiB (A 128 x 128 B + B 192 x 128 B), 3 attention images
// (48 KiB), bias / colsum / fin (2.5 KiB): 130.5 KiB, one workgroup per CU.
// MODE 0 stores Q|K|V (bf16, head order) instead of attention (exactness of the GEMM part);
// MODE 1 is timing-only (no epilogue). NK = K / 64: 12 (BERT-base), 16 (BERT-large).
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/lds_ops.h"

#include <algorithm>

namespace atpu {
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

template <int EPI, int MODE, int NK, int AS>
__global__ __launch_bounds__(512, 1) void qkv_ws_kernel(const bf16* __restrict__ A, int lda,
                                                        const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C,
                                                        int ldc, const float* __restrict__ bias,
                                                        const float* __restrict__ in_fin,
                                                        const float* __restrict__ colsum, int M, int N,
                                                        const int32_t* __restrict__ lens, float scale, int var) {
  static_assert(NK % 2 == 0 && NK % AS == 0 && NK >= 8,
                "K-tiles: whole rings per tile (every tile starts in stage 0), >= 8 (attention slots)");
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
  auto tile_of = [&](int vv, int& m0, int& n0) {
    const int t = xcd_remap(vv, ntiles);
    m0 = (t / ntn) * 128;
    n0 = (t % ntn) * 192;
  };
  auto opaque_lane = [] {
    int l = __lane_id();
    asm volatile("" : "+v"(l));
    return l;
  };
  const int fr = lane & 15, fc = lane >> 4;

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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // KB_t
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < NK) read_ks(t + 1, 0, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
      }
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
      __builtin_amdgcn_s_barrier();  // EB: the images are complete
      __builtin_amdgcn_sched_barrier(0);
      v += G;
      if (v >= ntiles) break;
    }
    return;
  }

  // ============================ loader / attention waves ============================
  const int l = wave - 4;
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
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(fly) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using Fly0 = std::integral_constant<int, 0>;
  using FlyA = std::integral_constant<int, AS == 3 ? 4 : 0>;
  // the DMA of slot s (s >= 0): B of K-tile s + 2, A of K-tile s + AS (runtime s: this tile)
  auto slot_dma = [&](int sl) {
    stageB(sl + 2, sl & 1);
    stageA(sl + AS, (sl + AS) % AS);
  };

  int m0, n0;
  tile_of(v, m0, n0);
  set_srcA(m0);
  set_srcB(n0);
  stageB(0, 0);
  stageB(1, 1);
#pragma unroll
  for (int k = 0; k < AS; ++k) stageA(k, k);
  slot_end(Fly0{});  // the first tile's B K-tiles 0-1 and A K-tiles 0..AS-1 landed
  int pm0 = 0, ph = 0;
  // one tile of the loader waves; ATT: the previous tile's attention runs in its slots (a
  // compile-time flag - a runtime `if (pending)` around every chunk made the attention state
  // of both paths live at each join: ~100 VGPRs of spills). Returns false after the last tile.
  auto tile_body = [&](auto att_c) -> bool {
    constexpr bool pending = decltype(att_c)::value && MODE == 2;
    const int vn = v + G;
    const bool has_next = vn < ntiles;
    int nm0 = 0, nn0 = 0;
    if (has_next) tile_of(vn, nm0, nn0);
    // ---- attention of the previous tile (pm0, head ph), queries l*32..+32, in chunks; the
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
    // chunk 1: the sequence length (scalar load, consumed before any counted LDS wait), Q and K
    // fragment reads, S(qp 0) = K.Q0^T with counted waits, mask
    // LDS addresses from an opaque lane id inside each chunk: from `lane` they are loop-invariant,
    // and hoisted out of the tile loop they held ~60 VGPRs for its whole length (spills)
    auto chunk1 = [&]() {
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
        __builtin_amdgcn_sched_barrier(0);
      };
      qk0(std::integral_constant<int, 0>{});
      qk0(std::integral_constant<int, 1>{});
      qk0(std::integral_constant<int, 2>{});
      qk0(std::integral_constant<int, 3>{});
      qk0(std::integral_constant<int, 4>{});
      qk0(std::integral_constant<int, 5>{});
      qk0(std::integral_constant<int, 6>{});
      qk0(std::integral_constant<int, 7>{});
      mask(0);
    };
    // chunk 2: S(qp 1) MFMAs beside softmax(qp 0)
    auto chunk2 = [&]() {
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
      mask(1);
    };
    // chunk 3: all 32 transposed V reads, P0.V beside softmax(qp 1); key step ks waits for its
    // 8 V reads (the lgkmcnt field holds at most 15: steps 0-1 wait for 17 of the 32)
    auto chunk3 = [&]() {
      {
        const int ln = opaque_lane();
        const int tq = (ln >> 2) & 3, tp = ln & 3;
        const int k0 = (ln >> 4) * 4 + tq;
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
    };
    // chunk 4: P1.V MFMAs beside the scaling / packing of the qp 0 context
    auto chunk4 = [&]() {
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
    };
    // chunk 5: context -> this wave's 32 Q rows (free once read) and back as whole 128-B rows
    // (cval); chunk 6: the global stores, issued at the start of the next slot before its DMA
    u32x4 cval[4];
    auto chunk5 = [&]() {
      const int ln = opaque_lane(), fr = ln & 15, fc = ln >> 4;
      char* ost = const_cast<char*>(qi) + l * 32 * 128;
      const float inv1 = len > 0 && o[1][4][0] > 0.f ? 1.f / o[1][4][0] : 0.f;
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
      const int l2 = opaque_lane();
      const int lr = l2 >> 3, lc8 = l2 & 7;
  #pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        const int ro = hh * 8 + lr;
        cval[hh] = ds_read128u(ost + ro * 128 + asw(ro, lc8) * 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cval[0]), "+v"(cval[1]), "+v"(cval[2]), "+v"(cval[3])::"memory");
    };
    auto chunk6 = [&]() {
      const int l2 = opaque_lane();
      const int lr = l2 >> 3, lc8 = l2 & 7;
      bf16* obase = C + (size_t)(pm0 + l * 32 + lr) * ldc + ph * 64 + lc8 * 8;
  #pragma unroll
      for (int hh = 0; hh < 4; ++hh) *reinterpret_cast<u32x4*>(obase + (size_t)(hh * 8) * ldc) = cval[hh];
    };
    auto chunk = [&](int c) {
      if constexpr (MODE == 2) {
        if (c == 1) chunk1();
        if (c == 2) chunk2();
        if (c == 3) chunk3();
        if (c == 4) chunk4();
        if (c == 5) chunk5();
        if (c == 6) chunk6();
      }
    };
    // slots -1 .. 3: the previous tile's attention beside the DMA of K-tiles 2 .. 5 (+1 for
    // A with AS = 3); the context stores go out at the start of slot 3, before its DMA
    stage_vec(m0, n0);
    if constexpr (pending) chunk(1);
    slot_end(Fly0{});  // KB_0
    slot_dma(0);
    if constexpr (pending) chunk(2);
    slot_end(FlyA{});
    slot_dma(1);
    if constexpr (pending) chunk(3);
    slot_end(FlyA{});
    slot_dma(2);
    if constexpr (pending) {
      chunk(4);
      chunk(5);
    }
    slot_end(FlyA{});
    if constexpr (pending) chunk(6);
    slot_dma(3);
    slot_end(FlyA{});  // KB_4
#pragma unroll 1
    for (int sl = 4; sl + AS < NK; ++sl) {
      slot_dma(sl);
      if (var & 4) {  // diagnostic (results wrong): no DMA wait in these slots (drained later)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        slot_end(FlyA{});
      }
    }
    // the last AS slots run into the next tile: B of K-tile s + 2 and A of K-tile s + AS, past
    // NK taken from the next tile (its offsets switched at its K-tile 0)
#pragma unroll
    for (int sl = NK - AS; sl < NK; ++sl) {
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
      if (has_next) slot_end(FlyA{});  // KB_sl+1, or EB after the last slot
      else slot_end(Fly0{});
    }
    pm0 = m0;
    ph = n0 / 192;
    if (!has_next) {
      // the last tile's attention, after the final barrier
      chunk(1);
      chunk(2);
      chunk(3);
      chunk(4);
      chunk(5);
      chunk(6);
      return false;
    }
    v = vn;
    m0 = nm0;
    n0 = nn0;
    return true;
  };
  if (!tile_body(std::false_type{})) return;
  while (tile_body(std::true_type{})) {
  }
}

}  // namespace

static int g_ws_variant = 0;
// experiment knob (benchmarks): bit 0 = MMA waves at s_setprio 2; bit 2 = diagnostic, no DMA wait in
// the middle slots (results wrong); bit 3 = a 3-deep A ring (K = 768); set >= 0 switches
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
  ATPU_CHECK(mode >= 0 && mode <= 2, "qkv_attention_ws: mode 0 (store QKV), 1 (timing only) or 2 (attention)");
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
  else { ATPU_WS_NK(E, 2); }
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

}  // namespace atpu
