// Probe: how fast can G workgroups of 16 waves stream a weight slice each (all loads in flight,
// 16-B per lane, summed so nothing is dead)? The fused few-row QKV + self-attention design puts
// one head's 192 x 768 bf16 QKV rows (295 KB) on one workgroup (12 workgroups for T5-base).
// Standalone: hipcc --offload-arch=gfx950 -O3 tools/probes/few_cu_stream.hip -o /tmp/fcs && /tmp/fcs
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LOADS>
__global__ __launch_bounds__(1024) void stream_kernel(const u16x8* __restrict__ w, size_t per_wg, float* out) {
  // workgroup g reads per_wg 16-B chunks starting at g * per_wg; thread t its LOADS chunks t, t + 1024, ...
  const u16x8* base = w + (size_t)blockIdx.x * per_wg;
  u16x8 v[LOADS];
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const size_t c = (size_t)threadIdx.x + (size_t)i * 1024;
    v[i] = c < per_wg ? base[c] : u16x8{};
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < LOADS; ++i) s += v[i][0] ^ v[i][7];
  if (s == 0x12345678u) out[blockIdx.x] = (float)s;  // keeps the loads live
}

int main() {
  const size_t per_wg = 192 * 768 * 2 / 16;  // 16-B chunks of one head's QKV rows (18432)
  const int G_list[] = {12, 24, 48, 144};
  u16x8* w;
  float* out;
  const size_t slice = per_wg * 12;  // 16-B chunks of all 12 heads (3.5 MB); 64 copies rotate (L2-cold)
  CK(hipMalloc(&w, slice * 16 * 64));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(w, 1, slice * 16 * 64));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode)
  for (int G : G_list) {
    // the same 12 slices' bytes (3.5 MB) over G workgroups: per_wg scaled down
    const size_t pw = per_wg * 12 / G;
    int copy = 0;
    bool rotate = false;
    auto launch = [&]() {
      const u16x8* src = w + (rotate ? (size_t)(copy++ % 64) * slice : 0);
      hipLaunchKernelGGL(stream_kernel<18>, dim3(G), dim3(1024), 0, st, src, pw, out);
    };
    rotate = mode == 1;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 50; ++i) launch();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("{\"workgroups\": %d, \"bytes_per_wg\": %zu, \"weights\": \"%s\", \"us_per_launch\": %.2f}\n", G, pw * 16,
           rotate ? "64 rotating copies (L2-cold)" : "one copy (L2-hot)", best * 1000.f / 50);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // reference: an empty-ish launch (1 workgroup, 1 load per thread)
  return 0;
}
