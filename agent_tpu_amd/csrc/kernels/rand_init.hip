// Seeded random init of model parameters on the GPU (atpu/rand.h; CPU twin in
// runtime/rand_host.cpp). A cache miss in the agent (ops/_gpu_runtime.py) used to pay a
// host torch.randn of the whole pack (2.0 s for BERT-base, 6.3 s for BERT-large) plus a
// first host -> HBM copy; here every element is a pure function of (seed, stream, index),
// written straight into the device ParamPack: a store-bound pass at HBM rate.
//
// One thread per 8 elements (a 16-B bf16 or 2 x 16-B fp32 store), grid-stride. Elements
// [0, n0) take scale0, the rest scale1 (T5 folds the attention scale into the q rows).
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/rand.h"

namespace atpu {
namespace {

template <bool F32>
__global__ __launch_bounds__(256) void rand_fill_kernel(void* __restrict__ dst, int64_t n, uint64_t key, float scale0,
                                                        int64_t n0, float scale1) {
  const int64_t nv = (n + 7) / 8;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = v * 8;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t i = i0 + e;
      f[e] = (float)rnd::ih4(key, (uint64_t)i) * (i < n0 ? scale0 : scale1);
    }
    if (i0 + 8 <= n) {
      if constexpr (F32) {
        float4* p = reinterpret_cast<float4*>(static_cast<float*>(dst) + i0);
        p[0] = float4{f[0], f[1], f[2], f[3]};
        p[1] = float4{f[4], f[5], f[6], f[7]};
      } else {
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (uint32_t)rnd::f2bf_rne(f[2 * e]) | ((uint32_t)rnd::f2bf_rne(f[2 * e + 1]) << 16);
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(dst) + i0) = uint4{w[0], w[1], w[2], w[3]};
      }
    } else {
      for (int e = 0; e < 8 && i0 + e < n; ++e) {
        if constexpr (F32) static_cast<float*>(dst)[i0 + e] = f[e];
        else static_cast<uint16_t*>(dst)[i0 + e] = rnd::f2bf_rne(f[e]);
      }
    }
  }
}

}  // namespace

void rand_fill(void* dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0, float scale1,
               hipStream_t stream) {
  ATPU_CHECK(n >= 0, "rand_fill: negative size");
  if (n == 0) return;
  ATPU_CHECK((reinterpret_cast<uintptr_t>(dst) & 15) == 0, "rand_fill: destination must be 16-byte aligned");
  const uint64_t key = rnd::stream_key(seed, sid);
  const int64_t nv = (n + 7) / 8;
  const int blocks = (int)std::min<int64_t>((nv + 255) / 256, 8 * num_cus());
  if (f32)
    hipLaunchKernelGGL(rand_fill_kernel<true>, dim3(blocks), dim3(256), 0, stream, dst, n, key, scale0, n0, scale1);
  else
    hipLaunchKernelGGL(rand_fill_kernel<false>, dim3(blocks), dim3(256), 0, stream, dst, n, key, scale0, n0, scale1);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
