// Row normalisation + embedding kernels (T5 RMSNorm).
//
// One 64-wide wave per row; a row of N = 256*NG elements is held in registers
// (NG groups of 4 per lane, 8-byte vector loads/stores), so statistics are a
// register pass plus one wave butterfly — a single HBM read and write per row.
// fp32 statistics, two-pass (mean, then centred variance) for accuracy.
#include <cstdlib>
#include <string>

#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/ln_row.h"

namespace atpu {
namespace {

template <int NG>
__device__ __forceinline__ void load_row(const bf16* p, float (&v)[NG * 4], int lane) {
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const bf16x4 x = *reinterpret_cast<const bf16x4*>(p + g * 256 + lane * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[g * 4 + e] = bf2f(x[e]);
  }
}

template <int NG>
__device__ __forceinline__ void add_row(const bf16* p, float (&v)[NG * 4], int lane) {
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const bf16x4 x = *reinterpret_cast<const bf16x4*>(p + g * 256 + lane * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[g * 4 + e] += bf2f(x[e]);
  }
}

template <int NG>
__device__ __forceinline__ void ln_store(float (&v)[NG * 4], const float* gamma, const float* beta, bf16* out,
                                         int N, float eps, int lane) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) s += v[i];
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = g * 256 + lane * 4;
    const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 bt = *reinterpret_cast<const f32x4*>(beta + c);
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf((v[g * 4 + e] - mean) * rstd * gm[e] + bt[e]);
    *reinterpret_cast<bf16x4*>(out + c) = o;
  }
}

template <int NG>
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, bf16* __restrict__ out,
                                                        int rows, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int N = NG * 256;
  float v[NG * 4];
  load_row<NG>(x + (size_t)row * N, v, lane);
  if (res) add_row<NG>(res + (size_t)row * N, v, lane);
  ln_store<NG>(v, gamma, beta, out + (size_t)row * N, N, eps, lane);
}

template <int NG, bool NTL>
__global__ __launch_bounds__(256) void layernorm_hw_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, bf16* __restrict__ out,
                                                           int rows, float eps) {
  const int hl = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool live = row < rows;
  const int r = live ? row : rows - 1;  // dead half-waves read a valid row, never store
  constexpr int N = NG * 256;
  ln_hw_row<NG, NTL>(x + (size_t)r * N, res ? res + (size_t)r * N : nullptr, gamma, beta, out + (size_t)row * N,
                     live, eps, hl);
}

// Decoder input of a learned-position model at one device-side step (BART): LN(table[ids[r]] +
// pos[*step + pos_off]) per row, the layernorm_hw math on the gathered rows, so the output equals
// embed_gather + the position row + layernorm_bf16(residual=) bit for bit in one launch (the
// position index never leaves the device: no host sync, graph-capturable).
template <int NG>
__global__ __launch_bounds__(256) void embed_pos_ln_kernel(const int32_t* __restrict__ ids,
                                                           const bf16* __restrict__ table,
                                                           const bf16* __restrict__ pos,
                                                           const int32_t* __restrict__ step, int pos_off, int npos,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, bf16* __restrict__ out,
                                                           int rows, int vocab, float eps) {
  const int hl = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool live = row < rows;
  const int r = live ? row : rows - 1;
  constexpr int N = NG * 256;
  int id = ids[r];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  int pi = *step + pos_off;
  pi = pi < 0 ? 0 : (pi >= npos ? npos - 1 : pi);
  ln_hw_row<NG, false>(table + (size_t)id * N, pos + (size_t)pi * N, gamma, beta, out + (size_t)row * N, live, eps,
                       hl);
}

template <int NG>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                      bf16* __restrict__ out, int rows, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int N = NG * 256;
  float v[NG * 4];
  load_row<NG>(x + (size_t)row * N, v, lane);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) q += v[i] * v[i];
  const float r = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = g * 256 + lane * 4;
    const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c);
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(v[g * 4 + e] * r * gm[e]);
    *reinterpret_cast<bf16x4*>(out + (size_t)row * N + c) = o;
  }
}

template <int NG>
__global__ __launch_bounds__(256) void embed_ln_kernel(const int32_t* __restrict__ ids,
                                                       const int32_t* __restrict__ type_ids,
                                                       const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                       const bf16* __restrict__ type, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, bf16* __restrict__ out,
                                                       int tokens, int S, int vocab, int type_vocab, float eps) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tokens) return;
  constexpr int N = NG * 256;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  int tt = type_ids ? type_ids[t] : 0;  // clamped like the word id: a bad type id never reads past the table
  tt = tt < 0 ? 0 : (tt >= type_vocab ? type_vocab - 1 : tt);
  float v[NG * 4];
  load_row<NG>(word + (size_t)id * N, v, lane);
  add_row<NG>(pos + (size_t)(t % S) * N, v, lane);
  add_row<NG>(type + (size_t)tt * N, v, lane);
  ln_store<NG>(v, gamma, beta, out + (size_t)t * N, N, eps, lane);
}

template <int NG>
__global__ __launch_bounds__(256) void embed_gather_kernel(const int32_t* __restrict__ ids,
                                                           const bf16* __restrict__ table, bf16* __restrict__ out,
                                                           int tokens, int vocab) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tokens) return;
  constexpr int N = NG * 256;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = g * 256 + lane * 4;
    *reinterpret_cast<bf16x4*>(out + (size_t)t * N + c) = *reinterpret_cast<const bf16x4*>(table + (size_t)id * N + c);
  }
}

#define ATPU_NG_DISPATCH(N, CALL)                                    \
  switch ((N) / 256) {                                               \
    case 1: { constexpr int NG = 1; CALL; break; }                   \
    case 2: { constexpr int NG = 2; CALL; break; }                   \
    case 3: { constexpr int NG = 3; CALL; break; }                   \
    case 4: { constexpr int NG = 4; CALL; break; }                   \
    case 6: { constexpr int NG = 6; CALL; break; }                   \
    case 8: { constexpr int NG = 8; CALL; break; }                   \
    default: throw std::invalid_argument("atpu: unsupported row width " + std::to_string(N)); \
  }

// LayerNorm folding: one thread per row turns the GEMM StatsOut partials
// (sum, sumsq per 256-column tile, slots summed in order) into (rstd, rstd*mu).
// 8 B in + 8 B out per slot and row: a few microseconds at BERT sizes.
__global__ __launch_bounds__(256) void ln_stats_finalize_kernel(const float* __restrict__ part, int slots, int M,
                                                                 float inv_k, float eps, float* __restrict__ fin) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  f32x2 s = *reinterpret_cast<const f32x2*>(part + (size_t)m * 2);
  for (int k = 1; k < slots; ++k) s += *reinterpret_cast<const f32x2*>(part + ((size_t)k * M + m) * 2);
  const float mu = s[0] * inv_k;
  const float rs = rsqrtf(fmaxf(s[1] * inv_k - mu * mu, 0.f) + eps);
  *reinterpret_cast<f32x2*>(fin + (size_t)m * 2) = f32x2{rs, rs * mu};
}

inline void check_width(int N) { ATPU_CHECK(N % 256 == 0 && N <= 2048, "row width must be a multiple of 256, <= 2048"); }

}  // namespace

void layernorm_bf16(const bf16* x, const bf16* res, const float* gamma, const float* beta, bf16* out, int rows, int N,
                    float eps, hipStream_t stream) {
  check_width(N);
  if (rows <= 0) return;
  // ATPU_LN_KERNEL=wave selects the wave-per-row kernel (A/B against the default half-wave kernel).
  static const int mode = [] {
    const char* e = std::getenv("ATPU_LN_KERNEL");
    const std::string m = e ? e : "";
    return m == "wave" ? 1 : (m == "hw" ? 2 : 0);
  }();
  const bool wave_per_row = mode == 1;
  if (wave_per_row) {
    const dim3 grid((rows + 3) / 4);
    ATPU_NG_DISPATCH(N, hipLaunchKernelGGL(layernorm_kernel<NG>, grid, dim3(256), 0, stream, x, res, gamma, beta, out,
                                           rows, eps));
  } else {
    const dim3 grid((rows + 7) / 8);
    if (mode == 2) {
      ATPU_NG_DISPATCH(N, hipLaunchKernelGGL((layernorm_hw_kernel<NG, false>), grid, dim3(256), 0, stream, x, res,
                                             gamma, beta, out, rows, eps));
    } else {
      ATPU_NG_DISPATCH(N, hipLaunchKernelGGL((layernorm_hw_kernel<NG, true>), grid, dim3(256), 0, stream, x, res,
                                             gamma, beta, out, rows, eps));
    }
  }
  ATPU_HIP_CHECK(hipGetLastError());
}

void rmsnorm_bf16(const bf16* x, const float* gamma, bf16* out, int rows, int N, float eps, hipStream_t stream) {
  check_width(N);
  if (rows <= 0) return;
  const dim3 grid((rows + 3) / 4);
  ATPU_NG_DISPATCH(N, hipLaunchKernelGGL(rmsnorm_kernel<NG>, grid, dim3(256), 0, stream, x, gamma, out, rows, eps));
  ATPU_HIP_CHECK(hipGetLastError());
}

void embed_layernorm(const int32_t* ids, const int32_t* type_ids, const bf16* word, const bf16* pos, const bf16* type,
                     const float* gamma, const float* beta, bf16* out, int B, int S, int N, int vocab, int type_vocab,
                     float eps, hipStream_t stream) {
  check_width(N);
  ATPU_CHECK(vocab > 0 && type_vocab > 0, "embedding tables must be non-empty");
  const int tokens = B * S;
  if (tokens <= 0) return;
  const dim3 grid((tokens + 3) / 4);
  ATPU_NG_DISPATCH(N, hipLaunchKernelGGL(embed_ln_kernel<NG>, grid, dim3(256), 0, stream, ids, type_ids, word, pos,
                                         type, gamma, beta, out, tokens, S, vocab, type_vocab, eps));
  ATPU_HIP_CHECK(hipGetLastError());
}

void ln_stats_finalize(const float* part, int slots, int M, int K, float eps, float* fin, hipStream_t stream) {
  ATPU_CHECK(slots >= 1 && K > 0, "ln_stats_finalize: bad shape");
  if (M <= 0) return;
  hipLaunchKernelGGL(ln_stats_finalize_kernel, dim3((M + 255) / 256), dim3(256), 0, stream, part, slots, M,
                     1.0f / static_cast<float>(K), eps, fin);
  ATPU_HIP_CHECK(hipGetLastError());
}

void embed_pos_layernorm(const int32_t* ids, const bf16* table, const bf16* pos, const int32_t* step, int pos_off,
                         int npos, const float* gamma, const float* beta, bf16* out, int rows, int N, int vocab,
                         float eps, hipStream_t stream) {
  check_width(N);
  ATPU_CHECK(vocab > 0 && npos > 0 && step, "embed_pos_layernorm: empty table or no step");
  if (rows <= 0) return;
  const dim3 grid((rows + 7) / 8);
  ATPU_NG_DISPATCH(N, hipLaunchKernelGGL(embed_pos_ln_kernel<NG>, grid, dim3(256), 0, stream, ids, table, pos, step,
                                         pos_off, npos, gamma, beta, out, rows, vocab, eps));
  ATPU_HIP_CHECK(hipGetLastError());
}

void embed_gather(const int32_t* ids, const bf16* table, bf16* out, int tokens, int N, int vocab, hipStream_t stream) {
  check_width(N);
  if (tokens <= 0) return;
  const dim3 grid((tokens + 3) / 4);
  ATPU_NG_DISPATCH(N, hipLaunchKernelGGL(embed_gather_kernel<NG>, grid, dim3(256), 0, stream, ids, table, out, tokens,
                                         vocab));
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
