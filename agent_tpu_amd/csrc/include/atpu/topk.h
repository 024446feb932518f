// Small register top-K helpers shared by the beam-search kernels (decode.hip
// beam_topk / beam_select, lm_head.hip fused LM head + top-k merge).
// Order: value descending, then token index ascending (HF / torch.topk on ties
// keep the lower index first, which the host reference reproduces).
#pragma once

#include "atpu/common.h"

#include <cfloat>

namespace atpu {

// (value desc, index asc) ordering
__device__ __forceinline__ bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

// insert (val, id) into a sorted register list; compile-time indices only
template <int KM>
__device__ __forceinline__ void list_insert(float (&tv)[KM], int (&ti)[KM], float val, int id) {
#pragma unroll
  for (int r = 0; r < KM; ++r) {
    const bool sw = better(val, id, tv[r], ti[r]);
    const float ov = tv[r];
    const int oi = ti[r];
    tv[r] = sw ? val : ov;
    ti[r] = sw ? id : oi;
    val = sw ? ov : val;
    id = sw ? oi : id;
  }
}

// KM rounds of wave argmax over the lanes' list heads; results in lane r (< KM)
template <int KM>
__device__ __forceinline__ void wave_topk(float (&tv)[KM], int (&ti)[KM], float& res_v, int& res_i) {
  const int lane = threadIdx.x & 63;
  res_v = -FLT_MAX;
  res_i = 0x7fffffff;
#pragma unroll
  for (int r = 0; r < KM; ++r) {
    float bv = tv[0];
    int bi = ti[0];
    // partners l ^ 32, l ^ 16 by permlane swaps, then the 16-lane row by DPP (l ^ 15, l ^ 7,
    // l ^ 2, l ^ 1): register and VALU only, no ds_bpermute round trips
    auto step = [&](float ov, int oi) {
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    };
    step(xor32f(bv), xor32i(bi));
    step(xor16f(bv), xor16i(bi));
    step(dppf<kDppMirror>(bv), dppi<kDppMirror>(bi));
    step(dppf<kDppHalfMirror>(bv), dppi<kDppHalfMirror>(bi));
    step(dppf<kDppXor2>(bv), dppi<kDppXor2>(bi));
    step(dppf<kDppXor1>(bv), dppi<kDppXor1>(bi));
    if (lane == r) { res_v = bv; res_i = bi; }
    if (ti[0] == bi && tv[0] == bv && bi != 0x7fffffff) {  // owner pops its head
#pragma unroll
      for (int x = 0; x + 1 < KM; ++x) { tv[x] = tv[x + 1]; ti[x] = ti[x + 1]; }
      tv[KM - 1] = -FLT_MAX;
      ti[KM - 1] = 0x7fffffff;
    }
  }
}

// ---------------------------------------------------------------------------
// Per-row tile reduction of the fused LM head (lm_head.hip, gemm_bf16.hip 256x256
// top-k epilogue). A row's values of one vocabulary tile sit in the 4 lanes
// l, l^16, l^32, l^48 of one wave (MFMA 16x16 fragment layout, operands swapped):
// lane (fr, fc) holds columns c0 + j*16 + fc*4 + e. The tile's exact top kTileSel
// (value desc, index asc) is contained in the candidate set {x >= L}, L = the
// kTileSel-th largest of the 4 lanes' top-4 values (any kTileSel values >= L bound
// the tile's kTileSel-th best from below).
constexpr int kTileCand = 16;  // candidate slots per (row, tile)
constexpr int kTileSel = 8;    // exact per tile: the top 8 (>= any K2 = 2 x beams <= 8)

// sorted (descending) top-4 of the values seen, values only: t0 >= t1 >= t2 >= t3
__device__ __forceinline__ void top4_push(float (&t)[4], float x) {
  const float n3 = __builtin_amdgcn_fmed3f(t[2], t[3], x);
  const float n2 = __builtin_amdgcn_fmed3f(t[1], t[2], x);
  const float n1 = __builtin_amdgcn_fmed3f(t[0], t[1], x);
  t[0] = fmaxf(t[0], x);
  t[1] = n1;
  t[2] = n2;
  t[3] = n3;
}

__device__ __forceinline__ void ce_desc(float& a, float& b) {
  const float hi = fmaxf(a, b), lo = fminf(a, b);
  a = hi;
  b = lo;
}

// 8th largest of the row's 4 lanes x top-4 (every lane of the row gets the same value)
__device__ __forceinline__ float row_kth8(const float (&t)[4]) {
  float u[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    u[k] = t[k];
    u[7 - k] = xor16f(t[k]);  // partner's list reversed: u is bitonic
  }
#pragma unroll
  for (int st = 4; st > 0; st >>= 1)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if ((i & st) == 0) ce_desc(u[i], u[i + st]);
  float q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q[k] = xor32f(u[k]);
  // 8th largest of two sorted 8-lists: max_i min(u_i, q_{8-i}), u_0 = q_0 = +inf
  float L = fmaxf(u[7], q[7]);
#pragma unroll
  for (int i = 1; i < 8; ++i) L = fmaxf(L, fminf(u[i - 1], q[7 - i]));
  return L;
}

// One row of one tile: sel[j][e] = selection value of column c0 + j*16 + fc*4 + e
// (-FLT_MAX: banned, masked or past the vocabulary); rmax / sumexp = the row's
// log-softmax partial over the tile. Writes hdr = {rmax, sumexp, count} and count
// (value, token) candidates to cb (kTileCand slots) when `live`. Whole wave, all
// lanes (the exact fallback is taken wave-uniformly).
template <int J>
__device__ __forceinline__ void tile_row_emit(const float (&sel)[J][4], int c0, int fc, bool live, float rmax,
                                              float sumexp, float4* hdr, float2* cb) {
  float t4[4] = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) top4_push(t4, sel[j][e]);
  const float L = row_kth8(t4);
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cnt += (sel[j][e] >= L && sel[j][e] > -FLT_MAX) ? 1 : 0;
  const int x1 = xor16i(cnt), x2 = xor32i(cnt), x3 = xor32i(x1);  // lanes l ^ 16, l ^ 32, l ^ 48
  int total = cnt + x1 + x2 + x3;
  const int pre = ((fc & 1) ? x1 : 0) + ((fc & 2) ? x2 + x3 : 0);  // lanes of lower fc first
  if (__ballot(live && total > kTileCand) == 0) {
    int k = pre;
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (sel[j][e] >= L && sel[j][e] > -FLT_MAX) {
          if (live) cb[k] = float2{sel[j][e], __int_as_float(c0 + j * 16 + fc * 4 + e)};
          ++k;
        }
  } else {
    // exact: kTileSel rounds of row argmax over (value desc, index asc) below the last pick
    float pv = __builtin_inff();
    int pi = -1;
    total = 0;
    for (int r = 0; r < kTileSel; ++r) {
      float bv = -FLT_MAX;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = sel[j][e];
          const int id = c0 + j * 16 + fc * 4 + e;
          if (x > -FLT_MAX && better(pv, pi, x, id) && better(x, id, bv, bi)) {
            bv = x;
            bi = id;
          }
        }
      {
        const float ov = xor16f(bv);
        const int oi = xor16i(bi);
        if (better(ov, oi, bv, bi)) {
          bv = ov;
          bi = oi;
        }
      }
      {
        const float ov = xor32f(bv);
        const int oi = xor32i(bi);
        if (better(ov, oi, bv, bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (bv > -FLT_MAX) {
        if (live && fc == 0) cb[r] = float2{bv, __int_as_float(bi)};
        total = r + 1;
      }
      pv = bv;
      pi = bi;
    }
  }
  if (live && fc == 0) *hdr = float4{rmax, sumexp, __int_as_float(total), 0.f};
}

// RowRms statistics exactly as the 128x128 / fused kernels accumulate them (per lane
// fdot2 over its 16-B A chunks in K order, then the 4-lane permlane sum), so a kernel
// that takes rstd from here produces the same logits bits
__device__ __forceinline__ float sumsq_chunk(bf16x8 a, float acc) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2_t p = bf16x2_t{a[2 * e], a[2 * e + 1]};
    acc = __builtin_amdgcn_fdot2_f32_bf16(p, p, acc, false);
  }
  return acc;
}

}  // namespace atpu
