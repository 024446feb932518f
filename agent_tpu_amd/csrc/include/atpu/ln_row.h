// Half-wave-per-row LayerNorm of one row, shared by the LayerNorm kernels (norm_embed.hip) and
// the decode-step state advance that also embeds the next tokens (decode.hip).
#pragma once

#include "atpu/common.h"

namespace atpu {

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Half-wave-per-row LayerNorm: 32 lanes own one row, each lane NG chunks of 8
// contiguous bf16 (16-byte loads/stores), so one wave instruction moves two
// 512-byte row segments instead of one 512-byte segment with 8-byte accesses.
// Half the memory instructions of layernorm_kernel for the same bytes; the
// statistics stay fp32 two-pass, reduced over the half wave.
// one row of the half-wave LayerNorm: LN(x_row (+ res_row)) -> out_row (rows of N = 256 NG)
template <int NG, bool NTL>
__device__ __forceinline__ void ln_hw_row(const bf16* __restrict__ xrow, const bf16* __restrict__ rrow,
                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                          bf16* __restrict__ orow_base, bool live, float eps, int hl) {
  constexpr int N = NG * 256;
  const bf16* xr = xrow + hl * 8;
  float v[NG * 8];
  bf16x8 xv[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    // NTL: the pre-norm input is dead after this pass; stream it past the caches
    if constexpr (NTL) xv[g] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(xr + g * 256));
    else xv[g] = *reinterpret_cast<const bf16x8*>(xr + g * 256);
  }
  if (rrow) {
    const bf16* rr = rrow + hl * 8;
    bf16x8 rv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) rv[g] = *reinterpret_cast<const bf16x8*>(rr + g * 256);
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[g * 8 + e] = bf2f(xv[g][e]) + bf2f(rv[g][e]);
  } else {
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[g * 8 + e] = bf2f(xv[g][e]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NG * 8; ++i) s += v[i];
  const float mean = half_sum(s) * (1.0f / N);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NG * 8; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(half_sum(q) * (1.0f / N) + eps);
  if (!live) return;
  bf16* orow = orow_base + hl * 8;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = g * 256 + hl * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + c + 4);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = f2bf((v[g * 8 + e] - mean) * rstd * g0[e] + b0[e]);
      o[e + 4] = f2bf((v[g * 8 + e + 4] - mean) * rstd * g1[e] + b1[e]);
    }
    *reinterpret_cast<bf16x8*>(orow + g * 256) = o;
  }
}


}  // namespace atpu
