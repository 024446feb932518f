// bf16 MFMA GEMM with fused epilogues for the BERT/T5 encoder hot path
// (QKV projection, attention out-proj + residual,
// FFN1 + GELU, FFN2 + residual; pooler + tanh).
//
//   C[M,N] = epi( A[M,K] · Bt[N,K]ᵀ )      A, Bt, C, R bf16; bias fp32
//   epi(x) = act(x + bias[n]) + R[m,n]      act ∈ {id, erf-GELU, tanh}
//
// Weights are stored [N][K] (K contiguous, = torch nn.Linear.weight), so both
// operand tiles are K-contiguous rows and every MFMA fragment is one 16-byte
// ds_read_b128.
//
// CDNA4 structure (cdna_hip_programming.md §5):
//  * v_mfma_f32_16x16x32_bf16, 64-wide waves, 4 waves as 2x2, 64x64 per wave.
//  * A/B tiles staged global -> LDS with global_load_lds_dwordx4 (no VGPR
//    round trip), two LDS buffers so tile k+1 streams in while tile k computes.
//  * LDS image XOR-swizzled on the 16-B chunk: chunk' = chunk ^ ((row>>1)&7).
//    128-B rows put two rows in one 256-B bank row; the swizzle makes the 16
//    rows a ds_read_b128 lane group touches land on 16 distinct 16-B slots
//    (conflict-free). glds writes lane-linearly, so the permutation is applied
//    to the per-lane GLOBAL source address and inverted on the read (rule 21).
//  * MFMA operands swapped (Bt as "A", A as "B") so each lane's accumulator
//    holds 4 consecutive output columns of one row -> 8-byte vector stores and
//    16-byte bias loads in the epilogue.
//  * Tile order: bijective XCD remap, N-fastest within a row panel, so the
//    blocks that share an A panel run on one XCD and hit its L2.
#include "atpu/common.h"
#include "atpu/kernels.h"

namespace atpu {
namespace {

constexpr int kBK = 64;          // K per LDS stage
constexpr int kRowBytes = kBK * 2;  // 128 B per staged row

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(WM* WN * 64, 2) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb, bf16* __restrict__ C, int ldc,
    const float* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int A_BYTES = BM * kRowBytes;
  constexpr int B_BYTES = BN * kRowBytes;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "stage split");
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (N + BN - 1) / BN;
  const int ntm = (M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * BM;
  const int n0 = (tile % ntn) * BN;

  // ---- per-lane staging addresses (row, swizzled chunk) ----
  // wave-instruction i of this wave covers staged rows [(i*NW+wave)*8, +8)
  const int srow = lane >> 3, spos = lane & 7;
  const bf16* a_src[BM / 8 / NW];
  const bf16* b_src[BN / 8 / NW];
#pragma unroll
  for (int i = 0; i < BM / 8 / NW; ++i) {
    const int r = (i * NW + wave) * 8 + srow;
    const int gr = min(m0 + r, M - 1);
    a_src[i] = A + (size_t)gr * lda + swz(r, spos) * 8;
  }
#pragma unroll
  for (int i = 0; i < BN / 8 / NW; ++i) {
    const int r = (i * NW + wave) * 8 + srow;
    const int gr = min(n0 + r, N - 1);
    b_src[i] = Bt + (size_t)gr * ldb + swz(r, spos) * 8;
  }

  auto stage = [&](int kt, int buf) {
    char* base = lds + buf * STAGE_BYTES;
    const int koff = kt * kBK;
#pragma unroll
    for (int i = 0; i < BM / 8 / NW; ++i) glds16(a_src[i] + koff, base + (i * NW + wave) * 8 * kRowBytes);
#pragma unroll
    for (int i = 0; i < BN / 8 / NW; ++i)
      glds16(b_src[i] + koff, base + A_BYTES + (i * NW + wave) * 8 * kRowBytes);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int arow0 = wm * (BM / WM), brow0 = wn * (BN / WN);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fchunk = lane >> 4;
  auto compute = [&](int buf) {
    const char* base = lds + buf * STAGE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = arow0 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = brow0 + j * 16 + frow;
        bfg[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * kRowBytes + swz(r, ks * 4 + fchunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = K / kBK;
  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    compute(cur);
    wait_vmcnt0();
    __syncthreads();
  }

  // ---- epilogue: lane owns C[m][n..n+3] for each (i, j) fragment ----
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + arow0 + i * 16 + frow;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + brow0 + j * 16 + fchunk * 4;
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI & kEpiBias) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n);
        v += b;
      }
      if constexpr (EPI & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      if constexpr (EPI & kEpiTanh) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
      }
      if constexpr (EPI & kEpiResidual) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldr + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bf2f(r[e]);
      }
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
    }
  }
}

template <int BM, int BN, int WM, int WN>
void launch_tile(const GemmArgs& g, hipStream_t s) {
  const int nb = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(nb), block(WM * WN * 64);
#define ATPU_GEMM_CASE(E)                                                                             \
  case E:                                                                                             \
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, E>), grid, block, 0, s, g.A, g.lda, g.Bt, g.ldb, \
                       g.C, g.ldc, g.bias, g.R, g.ldr, g.M, g.N, g.K);                                 \
    break;
  switch (g.epi) {
    ATPU_GEMM_CASE(0)
    ATPU_GEMM_CASE(kEpiBias)
    ATPU_GEMM_CASE(kEpiBias | kEpiGelu)
    ATPU_GEMM_CASE(kEpiBias | kEpiTanh)
    ATPU_GEMM_CASE(kEpiBias | kEpiResidual)
    ATPU_GEMM_CASE(kEpiResidual)
    ATPU_GEMM_CASE(kEpiGelu)
    default:
      throw std::invalid_argument("atpu: unsupported GEMM epilogue " + std::to_string(g.epi));
  }
#undef ATPU_GEMM_CASE
}

}  // namespace

void gemm_bf16(const GemmArgs& g, hipStream_t stream) {
  ATPU_CHECK(g.M > 0 && g.N > 0 && g.K > 0, "gemm: empty problem");
  ATPU_CHECK(g.K % kBK == 0, "gemm: K must be a multiple of 64");
  ATPU_CHECK(g.N % 4 == 0, "gemm: N must be a multiple of 4");
  ATPU_CHECK(g.lda % 8 == 0 && g.ldb % 8 == 0 && g.ldc % 4 == 0, "gemm: leading dims must keep 16-B rows");
  ATPU_CHECK((reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.Bt) & 15) == 0,
             "gemm: A/Bt must be 16-byte aligned");
  ATPU_CHECK(!(g.epi & kEpiBias) || g.bias, "gemm: bias epilogue without bias");
  ATPU_CHECK(!(g.epi & kEpiResidual) || (g.R && g.ldr % 4 == 0), "gemm: residual epilogue without R");
  launch_tile<128, 128, 2, 2>(g, stream);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
