// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace atpu {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

#define ATPU_GLOBAL_AS __attribute__((address_space(1)))
#define ATPU_LDS_AS __attribute__((address_space(3)))

// Async 16-byte global -> LDS copy (global_load_lds_dwordx4). `lds` must be
// wave-uniform: lane i lands at lds + 16*i.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds) {
  __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)gsrc, (ATPU_LDS_AS void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// erf-GELU with erf from Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7, far below
// bf16 output resolution): one v_rcp + one v_exp + 6 FMAs instead of the
// branchy libm erff, which dominated the FFN1 epilogue.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float erf_abs = 1.0f - p * t * __expf(-z * z);
  const float erf_x = copysignf(erf_abs, x);
  return 0.5f * x * (1.0f + erf_x);
}

// gelu_fast over 8 independent values, written stage by stage so the
// transcendental results (v_rcp, v_exp) are consumed several instructions
// after they are produced: the per-element form left hipcc padding every
// trans->use pair with s_nop. Same A&S 7.1.26 erf, exp folded into exp2.
__device__ __forceinline__ void gelu_fast8(float (&v)[8]) {
  float t[8], ex[8], p[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = fmaf(0.3275911f * 0.70710678118654752f, fabsf(v[e]), 1.0f);
#pragma unroll
  for (int e = 0; e < 8; ++e) ex[e] = v[e] * v[e];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = __builtin_amdgcn_rcpf(t[e]);
#pragma unroll
  for (int e = 0; e < 8; ++e) ex[e] = __builtin_amdgcn_exp2f(ex[e] * (-0.5f * 1.4426950408889634f));
#pragma unroll
  for (int e = 0; e < 8; ++e) p[e] = fmaf(1.061405429f, t[e], -1.453152027f);
#pragma unroll
  for (int e = 0; e < 8; ++e) p[e] = fmaf(p[e], t[e], 1.421413741f);
#pragma unroll
  for (int e = 0; e < 8; ++e) p[e] = fmaf(p[e], t[e], -0.284496736f);
#pragma unroll
  for (int e = 0; e < 8; ++e) p[e] = fmaf(p[e], t[e], 0.254829592f);
#pragma unroll
  for (int e = 0; e < 8; ++e) p[e] = fmaf(-p[e] * t[e], ex[e], 1.0f);  // |erf(x/sqrt2)|
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float half_x = 0.5f * v[e];
    v[e] = fmaf(half_x, copysignf(p[e], v[e]), half_x);
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// erf-GELU on 16 values with NO transcendental: erf(z) = z * P(t) on the
// clamped z = clamp(x/sqrt2, -3.5, 3.5), t = 2 z^2 / 3.5^2 - 1 in [-1, 1], P a
// degree-12 least-squares Chebyshev fit (monomial in t; tools/gelu_fit.py).
// Evaluated here in x-space (clamp x to +-3.5*sqrt2, 1/sqrt2 folded into the
// coefficients). Max |gelu error| <= 3.4e-6 over all x (<= 8.7e-7 for
// |x| < 4) in fp32. The Horner chain runs on float2 -> v_pk_fma_f32, two values
// per instruction; the A&S form (gelu_fast8) spends a v_rcp and a v_exp per
// value, each a quarter-rate transcendental. In the FFN1 epilogue, whose VALU
// issue is not hidden behind MFMAs, this is ~40 % fewer VALU cycles.
__device__ __forceinline__ void gelu_poly16(float (&v)[16]) {
  constexpr float kC[13] = {2.855813205e-01f,  -1.419170350e-01f, 1.037684307e-01f,  -8.104421943e-02f,
                            6.250595301e-02f,  -4.579368234e-02f, 3.184378892e-02f,  -2.125407569e-02f,
                            1.203811448e-02f,  -5.087599624e-03f, 3.172110533e-03f,  -2.829871373e-03f,
                            1.047181780e-03f};
  constexpr float kClamp = 4.949747562e+00f;  // 3.5 * sqrt(2)
  constexpr float kT = 8.16326513886e-02f;    // 1 / 3.5^2
  f32x2 xc[8], t[8], p[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    xc[e] = f32x2{__builtin_amdgcn_fmed3f(v[2 * e], -kClamp, kClamp),
                  __builtin_amdgcn_fmed3f(v[2 * e + 1], -kClamp, kClamp)};
    t[e] = __builtin_elementwise_fma(xc[e] * xc[e], f32x2{kT, kT}, f32x2{-1.f, -1.f});
    p[e] = f32x2{kC[12], kC[12]};
  }
#pragma unroll
  for (int k = 11; k >= 0; --k)
#pragma unroll
    for (int e = 0; e < 8; ++e) p[e] = __builtin_elementwise_fma(p[e], t[e], f32x2{kC[k], kC[k]});
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const f32x2 hx = f32x2{v[2 * e], v[2 * e + 1]} * 0.5f;
    const f32x2 g = __builtin_elementwise_fma(hx, xc[e] * p[e], hx);  // 0.5x (1 + erf)
    v[2 * e] = g[0];
    v[2 * e + 1] = g[1];
  }
}

__device__ __forceinline__ float bf2f(bf16 x) { return static_cast<float>(x); }
__device__ __forceinline__ bf16 f2bf(float x) { return static_cast<bf16>(x); }

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// two fp32 -> one dword of bf16 (RNE; one v_cvt_pk_bf16_f32), lo in bits 0-15
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, bf16x2{f2bf(lo), f2bf(hi)});
}

// Bijective XCD-aware block remap (guide §5 "XCD swizzle must be bijective"):
// blocks that the dispatcher places on one XCD (b % 8 equal) get a contiguous
// range of logical tile ids, so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

}  // namespace atpu

#define ATPU_HIP_CHECK(expr)                                                              \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                \
  } while (0)

#define ATPU_CHECK(cond, msg)                                                   \
  do {                                                                          \
    if (!(cond)) throw std::invalid_argument(std::string("atpu: ") + (msg));    \
  } while (0)
