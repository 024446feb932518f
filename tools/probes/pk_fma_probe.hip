#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, float mm, float cc) {
  const float s = threadIdx.x * 1e-3f; mm += s * 1e-7f; cc += s * 1e-9f;
  if constexpr (MODE == 0) {  // packed f32
    f32x2 a[16], m{mm, mm}, c{cc, -cc};
    for (int i = 0; i < 16; ++i) a[i] = f32x2{s + i, s - i};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_fma(a[i], m, c);
    float r = 0; for (int i = 0; i < 16; ++i) r += a[i][0] + a[i][1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
  } else if constexpr (MODE == 1) {  // packed f16
    f16x2 a[16], m{(_Float16)mm, (_Float16)mm}, c{(_Float16)cc, (_Float16)-cc};
    for (int i = 0; i < 16; ++i) a[i] = f16x2{(_Float16)(s + i), (_Float16)(s - i)};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_fma(a[i], m, c);
    float r = 0; for (int i = 0; i < 16; ++i) r += (float)a[i][0] + (float)a[i][1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
  } else if constexpr (MODE == 2) {  // scalar f32
    float a[16];
    for (int i = 0; i < 16; ++i) a[i] = s + i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = fmaf(a[i], mm, cc);
    float r = 0; for (int i = 0; i < 16; ++i) r += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
  } else {  // packed bf16 (if the target has it)
    bf16x2 a[16], m{(__bf16)mm, (__bf16)mm}, c{(__bf16)cc, (__bf16)-cc};
    for (int i = 0; i < 16; ++i) a[i] = bf16x2{(__bf16)(s + i), (__bf16)(s - i)};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_fma(a[i], m, c);
    float r = 0; for (int i = 0; i < 16; ++i) r += (float)a[i][0] + (float)a[i][1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
  }
}
template <int MODE> double run(float* d, int blocks, int iters) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 1e-4f);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 1e-4f);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}
int main() {
  float* d; hipMalloc(&d, 256 * 8192 * 4);
  const int blocks = 256 * 8, iters = 4096;
  const double ops = (double)blocks * 256 * iters * 16;  // instructions x lanes
  for (int r = 0; r < 2; ++r) {
    double t0 = run<0>(d, blocks, iters), t1 = run<1>(d, blocks, iters), t2 = run<2>(d, blocks, iters), t3 = run<3>(d, blocks, iters);
    printf("pk_f32 %.3f ms (%.1f Ginstr-lanes/ms) | pk_f16 %.3f ms | f32 %.3f ms | pk_bf16 %.3f ms\n", t0, ops / t0 / 1e9, t1, t2, t3);
  }
  return 0;
}
