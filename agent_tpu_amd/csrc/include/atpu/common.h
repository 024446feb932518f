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

// DPP lane permutations inside a 16-lane row, VALU only (no ds_bpermute round trip through
// the LDS crossbar, which is what __shfl_xor compiles to): row_mirror pairs lane l with
// l ^ 15, row_half_mirror with l ^ 7, the quad perms with l ^ 2 and l ^ 1. The masks
// 15, 7, 2, 1 span the 4 row bits, so a butterfly over them reduces all 16 lanes.
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
constexpr int kDppMirror = 0x140, kDppHalfMirror = 0x141, kDppXor2 = 0x4E, kDppXor1 = 0xB1;

__device__ __forceinline__ float lane_rows_sum(float x);
__device__ __forceinline__ float lane_rows_max(float x);

// whole-wave reductions: the 4 lane rows by permlane swaps (lane_rows_*), then the 16 lanes
// of a row by DPP; every lane gets the result
__device__ __forceinline__ float wave_sum(float v) {
  v = lane_rows_sum(v);
  v += dppf<kDppMirror>(v);
  v += dppf<kDppHalfMirror>(v);
  v += dppf<kDppXor2>(v);
  return v + dppf<kDppXor1>(v);
}

__device__ __forceinline__ float wave_max(float v) {
  v = lane_rows_max(v);
  v = fmaxf(v, dppf<kDppMirror>(v));
  v = fmaxf(v, dppf<kDppHalfMirror>(v));
  v = fmaxf(v, dppf<kDppXor2>(v));
  return fmaxf(v, dppf<kDppXor1>(v));
}

// Reductions over the 4 lanes l, l^16, l^32, l^48 (the 4 lane rows holding one
// MFMA 16x16 fragment row/column), registers only: v_permlane16_swap then
// v_permlane32_swap, no ds_bpermute round trips. Every lane gets the result.
// The operands are laundered through v_mov into early-clobber outputs: the
// two-result builtin let hipcc allocate both to ONE register (ROCm 7.2).
__device__ __forceinline__ float lane_rows_sum(float x) {
  float a, b, c, d;
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %2\n\ts_nop 1\n\tv_permlane16_swap_b32 %0, %1"
               : "=&v"(a), "=&v"(b) : "v"(x));
  const float y = a + b;
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %2\n\ts_nop 1\n\tv_permlane32_swap_b32 %0, %1"
               : "=&v"(c), "=&v"(d) : "v"(y));
  return c + d;
}

__device__ __forceinline__ float lane_rows_max(float x) {
  float a, b, c, d;
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %2\n\ts_nop 1\n\tv_permlane16_swap_b32 %0, %1"
               : "=&v"(a), "=&v"(b) : "v"(x));
  const float y = fmaxf(a, b);
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %2\n\ts_nop 1\n\tv_permlane32_swap_b32 %0, %1"
               : "=&v"(c), "=&v"(d) : "v"(y));
  return fmaxf(c, d);
}

// v_permlane32_swap / v_permlane16_swap of two values (x's upper 32 lanes <-> y's lower 32;
// x's odd 16-lane rows <-> y's even rows), laundered into early-clobber outputs as above
__device__ __forceinline__ float2 pl32_swap(float x, float y) {
  float a, b;
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3\n\ts_nop 1\n\tv_permlane32_swap_b32 %0, %1"
               : "=&v"(a), "=&v"(b)
               : "v"(x), "v"(y));
  return float2{a, b};
}
__device__ __forceinline__ float2 pl16_swap(float x, float y) {
  float a, b;
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3\n\ts_nop 1\n\tv_permlane16_swap_b32 %0, %1"
               : "=&v"(a), "=&v"(b)
               : "v"(x), "v"(y));
  return float2{a, b};
}

// the value of lane l ^ 16 / l ^ 32 (exact partner, by one permlane swap and a select)
__device__ __forceinline__ float xor16f(float x) {
  const float2 p = pl16_swap(x, x);
  return (threadIdx.x & 16) ? p.x : p.y;
}
__device__ __forceinline__ float xor32f(float x) {
  const float2 p = pl32_swap(x, x);
  return (threadIdx.x & 32) ? p.x : p.y;
}
__device__ __forceinline__ int xor16i(int x) { return __float_as_int(xor16f(__int_as_float(x))); }
__device__ __forceinline__ int xor32i(int x) { return __float_as_int(xor32f(__int_as_float(x))); }
template <int CTRL>
__device__ __forceinline__ int dppi(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}

// Butterfly all-reduce of N (1..16, a power of two) per-lane values over the wave: every step
// halves the values (a permlane32 swap pairs i / i + N/2 across the lane halves, a permlane16
// swap the 16-lane rows, then xor shuffles), the lane bits left over are reduced as a plain
// xor tree. Lane l ends with the reduction of value l >> (6 - log2 N) (N + 5 - log2 N
// cross-lane ops instead of 6 N independent wave reductions).
template <int N, class Op>
__device__ __forceinline__ float wave_bfly(const float (&v)[N], Op op) {
  static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16, "wave_bfly: N in 1..16, power of two");
  const int lane = threadIdx.x & 63;
  float a[N];
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = v[i];
  if constexpr (N >= 2) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float2 p = pl32_swap(a[i], a[i + N / 2]);
      a[i] = op(p.x, p.y);
    }
  }
  if constexpr (N >= 4) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const float2 p = pl16_swap(a[i], a[i + N / 4]);
      a[i] = op(p.x, p.y);
    }
  }
  // inside the 16-lane rows by DPP: partners l ^ 15 (splitting on bit 3), l ^ 7 (bit 2), then
  // l ^ 2, l ^ 1; each splitting partner has the other value of the bit, and the rest share it
  if constexpr (N >= 8) {
    const bool b = lane & 8;
#pragma unroll
    for (int i = 0; i < N / 8; ++i) a[i] = op(b ? a[i + N / 8] : a[i], dppf<kDppMirror>(b ? a[i] : a[i + N / 8]));
  }
  if constexpr (N >= 16) {
    const bool b = lane & 4;
    a[0] = op(b ? a[1] : a[0], dppf<kDppHalfMirror>(b ? a[0] : a[1]));
  }
  float x = a[0];
  if constexpr (N < 2) {
    const float2 p = pl32_swap(x, x);
    x = op(p.x, p.y);
  }
  if constexpr (N < 4) {
    const float2 p = pl16_swap(x, x);
    x = op(p.x, p.y);
  }
  if constexpr (N < 8) x = op(x, dppf<kDppMirror>(x));
  if constexpr (N < 16) x = op(x, dppf<kDppHalfMirror>(x));
  x = op(x, dppf<kDppXor2>(x));
  return op(x, dppf<kDppXor1>(x));
}
struct OpAdd {
  __device__ float operator()(float a, float b) const { return a + b; }
};
struct OpMax {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};

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

// erf-GELU on 16 values with NO transcendental:
//   xc = clamp(x, -A, A),  w = xc^2 - A^2/2,  gelu(x) = x * (0.5 + xc * Q(w))
// Q ~= erf(xc/sqrt2) / (2 xc), a degree-10 least-squares Chebyshev fit on
// |xc| <= A = 3.25*sqrt2, rescaled to monomials in the CENTRED w: as well
// conditioned as the Chebyshev interval, and w is one FMA (tools/gelu_fit.py).
// fp32 max |gelu error| 1.7e-5 over all x, 3.6e-6 for |x| < 4 (bf16 output
// resolution at 1.0 is 3.9e-3). Per pair of values: 2 v_med3 + 13 packed ops
// (v_pk_fma_f32 / v_pk_mul_f32); the A&S form (gelu_fast8) spends a v_rcp and a
// v_exp per value, each a quarter-rate transcendental. The FFN1 epilogue's VALU
// issue is not hidden behind MFMAs, so this count is its tail cost.
__device__ __forceinline__ void gelu_poly16(float (&v)[16]) {
  constexpr int kDeg = 10;
  constexpr float kQ[kDeg + 1] = {1.536687613e-01f,  -7.178471889e-03f, 4.856055602e-04f, -3.426085095e-05f,
                                  2.347781901e-06f,  -1.526724844e-07f, 8.713541888e-09f, -4.079194205e-10f,
                                  2.366933385e-11f,  -1.725522828e-12f, 5.926992431e-14f};
  constexpr float kH = 1.056250000e+01f;  // A^2 / 2, A = 3.25 * sqrt(2) (the fit interval |x| <= A)
  // Phi(x) = 0.5 + x * p(x^2 - A^2/2) on |x| <= A. Outside the fit interval the degree-10
  // polynomial runs away with the sign of x (x * p >= 0.49999 for x >= A, <= -0.5 + 2e-6 for
  // x <= -A, up to +-inf for huge |x|; never NaN: every Horner step is inf * w + c with w > 0),
  // so the [0, 1] output clamp of the last packed FMA (VOP3P clamp bit) saturates Phi exactly
  // where the old input clamp did: two v_med3 per value pair fewer (13 VALU per pair, was 15).
  f32x2 x[8], w[8], p[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    x[e] = f32x2{v[2 * e], v[2 * e + 1]};
    w[e] = __builtin_elementwise_fma(x[e], x[e], f32x2{-kH, -kH});
    p[e] = f32x2{kQ[kDeg], kQ[kDeg]};
  }
#pragma unroll
  for (int k = kDeg - 1; k >= 0; --k)
#pragma unroll
    for (int e = 0; e < 8; ++e) p[e] = __builtin_elementwise_fma(p[e], w[e], f32x2{kQ[k], kQ[k]});
  const f32x2 half = f32x2{0.5f, 0.5f};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    f32x2 phi;
    asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(phi) : "v"(x[e]), "v"(p[e]), "v"(half));
    const f32x2 g = x[e] * phi;
    v[2 * e] = g[0];
    v[2 * e + 1] = g[1];
  }
}

// gelu_poly16's arithmetic on ONE value, operation for operation (a v_pk_fma_f32 lane is the
// same correctly rounded fp32 FMA as v_fma_f32; the clamp is the same [0, 1] output modifier):
// every GEMM family (64x64 dec, 128x128, 256x256, GEMV, split-K reduce) applies this GELU, so
// a row's FFN output does not depend on which kernel the batch size selected (batch invariance).
__device__ __forceinline__ float gelu_poly1(float x) {
  constexpr int kDeg = 10;
  constexpr float kQ[kDeg + 1] = {1.536687613e-01f,  -7.178471889e-03f, 4.856055602e-04f, -3.426085095e-05f,
                                  2.347781901e-06f,  -1.526724844e-07f, 8.713541888e-09f, -4.079194205e-10f,
                                  2.366933385e-11f,  -1.725522828e-12f, 5.926992431e-14f};
  constexpr float kH = 1.056250000e+01f;
  const float w = fmaf(x, x, -kH);
  float p = kQ[kDeg];
#pragma unroll
  for (int k = kDeg - 1; k >= 0; --k) p = fmaf(p, w, kQ[k]);
  float phi;
  asm("v_fma_f32 %0, %1, %2, %3 clamp" : "=v"(phi) : "v"(x), "v"(p), "v"(0.5f));
  return x * phi;
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
