// v_permlane16_swap semantics: builtin vs inline asm, and an epilogue-like use
// on MFMA results (does the swapped data match the expected lane mapping?).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__global__ void k(unsigned* out, float* mf) {
  const unsigned l = threadIdx.x;
  unsigned x = 1000 + l, y = 2000 + l;
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  unsigned a = 1000 + l, b = 2000 + l;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  out[128 + l] = a;
  out[192 + l] = b;
  // MFMA result: D = A·B with A = identity-ish so D[i][j] = lane-tagged values
  bf16x8 av, bv;
  for (int e = 0; e < 8; ++e) { av[e] = (__bf16)(((l & 15) == ((l >> 4) * 8 + e) % 16) ? 1.f : 0.f); bv[e] = (__bf16)(float)((l & 15) * 16 + (l >> 4) * 8 + e); }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  unsigned p, q;
  asm volatile("s_nop 7\n\ts_nop 7\n\tv_mov_b32 %0, %1" : "=v"(p) : "v"(acc[0]));
  asm volatile("v_mov_b32 %0, %1" : "=v"(q) : "v"(acc[1]));
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p), "+v"(q));
  mf[l] = acc[0]; mf[64 + l] = acc[1];
  mf[128 + l] = __builtin_bit_cast(float, p); mf[192 + l] = __builtin_bit_cast(float, q);
}
int main() {
  unsigned* d; float* m;
  unsigned h[256]; float hm[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&m, sizeof(hm)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(hm, m, sizeof(hm), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l : {0, 5, 16, 21, 32, 48}) std::printf("lane %2d builtin r0=%u r1=%u | asm a=%u b=%u\n", l, h[l], h[64 + l], h[128 + l], h[192 + l]);
  for (int l : {0, 5, 16, 21, 32, 48}) std::printf("lane %2d mfma e0=%g e1=%g | swapped p=%g q=%g\n", l, hm[l], hm[64 + l], hm[128 + l], hm[192 + l]);
  return 0;
}
