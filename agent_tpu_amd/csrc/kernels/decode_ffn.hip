// Persistent-launch prototype: a T5-base decoder FFN block for <= 4 rows
// (one document x 4 beams) as ONE launch with one in-launch grid barrier, against today's two
// GEMV launches (gemm_bf16.hip gemv_kernel: RowRms|ReLU wi, then the K-split residual wo):
//
//   h = relu(rsqrt(mean(x^2) + eps) * (x . wi'^T))      wi' = wi with the RMSNorm gamma folded
//   y = x + h . wo^T
//
// 192 workgroups of 4 waves (T5-base: d = 768, d_ff = 3072):
//  * stage 1: wave (g, w) owns wi columns (4g + w) * 4 .. +4: its lanes split K = 768 in 16-B
//    chunks (two per lane), dot2 in fp32, the RMS sum of squares from the same x chunks, one
//    butterfly for the 16 (row, column) sums and one for the 4 row sums; h (bf16) is stored;
//  * before waiting at the barrier every wave issues its stage-2 weight loads (wo rows
//    4g .. 4g + 3, K quarter w): they land while the grid converges (the prefetch credit a
//    kernel boundary cannot give);
//  * grid barrier (placement-independent, MI355X_MICROARCH.md visibility rules): every storing
//    wave drains, workgroup barrier, ONE lane releases (agent fence) and adds to an arrival
//    counter; the last arriver resets the counter and bumps a generation word (release), the
//    others poll the generation with relaxed agent loads and s_sleep, bounded (a give-up sets
//    an error word); then ONE agent acquire and a workgroup barrier before any h load;
//  * stage 2: each wave dots its K quarter of h against the prefetched weights, a butterfly
//    per wave, the 4 quarters summed through LDS, + residual, bf16 store.
// The barrier words (count, generation, error) persist across launches and replays: a launch
// leaves the counter at 0, so only the allocation zeroes them (no per-call memset node).
#include "atpu/common.h"
#include "atpu/kernels.h"

namespace atpu {
namespace {

constexpr int kFfnRows = 4;
constexpr int kFfnD = 768;                   // T5-base d_model (stage-1 K, stage-2 columns / 4 waves ...)
constexpr int kFfnF = 3072;                  // d_ff
constexpr int kFfnG = kFfnD / 4;             // workgroups: 4 output columns each in stage 2
static_assert(kFfnF / 16 == kFfnG, "stage 1: 4 waves x 4 columns per workgroup cover d_ff");
constexpr int kCh1 = kFfnD / 8;              // stage-1 16-B chunks of K (96)
constexpr int kCh2 = kFfnF / 4 / 8;          // stage-2 chunks per wave (its K quarter, 96)

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 b, float acc) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{a[2 * e], a[2 * e + 1]}, bf16x2_t{b[2 * e], b[2 * e + 1]}, acc,
                                          false);
  return acc;
}

// grid barrier; returns false when this workgroup gave up waiting (error word set)
__device__ __forceinline__ bool ffn_grid_sync(unsigned* count, unsigned* gen, unsigned* err, unsigned G, int tid,
                                              int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its stores are done
  __syncthreads();
  if (tid == 0) {
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ROCm 7.2 can drop the fence's own wait
    const unsigned old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    if (old == G - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g0 + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {  // ~ a second: a lost workgroup, never a hang
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *flag_lds = ok;
  }
  __syncthreads();
  return *flag_lds != 0;
}

__global__ __launch_bounds__(256) void t5_ffn_fused_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wi,
                                                          const bf16* __restrict__ wo, bf16* __restrict__ y,
                                                          bf16* __restrict__ h, int M, float eps, unsigned* sync) {
  __shared__ float red[4][16];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = blockIdx.x;
  const bool c1ok = lane + 64 < kCh1;  // the second chunk of the lane (96 = 64 + 32)
  // ---- stage 1: wi columns n1 = (4g + w) * 4 .. +4
  const int n1 = (g * 4 + w) * 4;
  bf16x8 xa[kFfnRows][2], wa[4][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = min(lane + c * 64, kCh1 - 1);
#pragma unroll
    for (int m = 0; m < kFfnRows; ++m) xa[m][c] = *reinterpret_cast<const bf16x8*>(x + (size_t)min(m, M - 1) * kFfnD + ch * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[j][c] = *reinterpret_cast<const bf16x8*>(wi + (size_t)(n1 + j) * kFfnD + ch * 8);
  }
  float acc[16], ssq[kFfnRows];
#pragma unroll
  for (int m = 0; m < kFfnRows; ++m) {
    ssq[m] = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bool ok = c == 0 || c1ok;
      ssq[m] += ok ? dot8(xa[m][c], xa[m][c], 0.f) : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = dot8(xa[m][c], wa[j][c], 0.f);
        acc[m * 4 + j] = (c == 0 ? 0.f : acc[m * 4 + j]) + (ok ? d : 0.f);
      }
    }
  }
  const float v = wave_bfly<16>(acc, OpAdd{});      // lane l: (row l >> 4, column (l >> 2) & 3)
  const float rs = wave_bfly<kFfnRows>(ssq, OpAdd{});  // lane l: row l >> 4
  const int mo = lane >> 4, jo = (lane >> 2) & 3;
  if ((lane & 3) == 0 && mo < M) {
    const float hv = fmaxf(v * __builtin_amdgcn_rsqf(rs * (1.f / kFfnD) + eps), 0.f);
    h[(size_t)mo * kFfnF + n1 + jo] = f2bf(hv);
  }
  // ---- stage-2 weights, issued before the barrier: wo rows n2 .. n2 + 3, K quarter w
  const int n2 = g * 4, k0 = w * (kFfnF / 4);
  bf16x8 wb[4][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = min(lane + c * 64, kCh2 - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[j][c] = *reinterpret_cast<const bf16x8*>(wo + (size_t)(n2 + j) * kFfnF + k0 + ch * 8);
  }
  if (!ffn_grid_sync(sync, sync + 1, sync + 2, gridDim.x, tid, &flag)) return;
  // ---- stage 2: this wave's K quarter of h
  bf16x8 ha[kFfnRows][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = min(lane + c * 64, kCh2 - 1);
#pragma unroll
    for (int m = 0; m < kFfnRows; ++m)
      ha[m][c] = *reinterpret_cast<const bf16x8*>(h + (size_t)min(m, M - 1) * kFfnF + k0 + ch * 8);
  }
#pragma unroll
  for (int m = 0; m < kFfnRows; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = dot8(ha[m][0], wb[j][0], 0.f);
      s += c1ok ? dot8(ha[m][1], wb[j][1], 0.f) : 0.f;
      acc[m * 4 + j] = s;
    }
  const float v2 = wave_bfly<16>(acc, OpAdd{});
  if ((lane & 3) == 0) red[w][lane >> 2] = v2;
  __syncthreads();
  if (w == 0 && lane < 16) {
    const int m = lane >> 2, j = lane & 3;
    if (m < M) {
      const float s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
      y[(size_t)m * kFfnD + n2 + j] = f2bf(s + bf2f(x[(size_t)m * kFfnD + n2 + j]));
    }
  }
}

}  // namespace

size_t t5_ffn_fused_ws_bytes() { return (size_t)kFfnRows * kFfnF * 2; }

void t5_ffn_fused(const bf16* x, const bf16* wi, const bf16* wo, bf16* y, int M, int d, int f, float eps, bf16* h_ws,
                  unsigned* sync, hipStream_t stream) {
  ATPU_CHECK(M >= 1 && M <= kFfnRows, "t5_ffn_fused: 1..4 rows");
  ATPU_CHECK(d == kFfnD && f == kFfnF, "t5_ffn_fused: the T5-base FFN (d 768, d_ff 3072) only");
  ATPU_CHECK(h_ws && sync && x != y, "t5_ffn_fused: workspace, zeroed sync words, out-of-place output");
  ATPU_CHECK(kFfnG <= 8 * num_cus(), "t5_ffn_fused: the grid must be resident");
  hipLaunchKernelGGL(t5_ffn_fused_kernel, dim3(kFfnG), dim3(256), 0, stream, x, wi, wo, y, h_ws, M, eps, sync);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
