// Classify head + softmax + top-k and the streaming
// count/sum/min/max reduction behind risk_accumulate (K12).
#include "atpu/common.h"
#include "atpu/kernels.h"

#include <algorithm>
#include <cfloat>

namespace atpu {
namespace {

constexpr int kMaxClasses = 4096;
constexpr int kMaxK = 64;

// One wave per row. pooled row staged in LDS; lane j owns classes j, j+64, ...
// Top-k = k rounds of a wave-wide argmax on (prob desc, index asc), so ties
// resolve to the lower class index deterministically (ref _topk:
// /root/reference/ops/map_classify_tpu.py:15-19 orders by descending score).
__global__ __launch_bounds__(64) void head_topk_kernel(const bf16* __restrict__ pooled, int ldp,
                                                       const bf16* __restrict__ Wc, const float* __restrict__ bc,
                                                       float* __restrict__ logits, int32_t* __restrict__ topk_idx,
                                                       float* __restrict__ topk_score, int N, int C, int k) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* x = reinterpret_cast<float*>(smem);       // [N]
  float* z = x + N;                                 // [C]
  const int lane = threadIdx.x, row = blockIdx.x;
  const bf16* p = pooled + (size_t)row * ldp;
  for (int i = lane; i < N; i += 64) x[i] = bf2f(p[i]);
  __syncthreads();
  float mx = -FLT_MAX;
  for (int c = lane; c < C; c += 64) {
    const bf16* w = Wc + (size_t)c * N;
    float acc = bc ? bc[c] : 0.f;
    for (int i = 0; i < N; i += 8) {
      const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + i);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += x[i + e] * bf2f(wv[e]);
    }
    z[c] = acc;
    logits[(size_t)row * C + c] = acc;
    mx = fmaxf(mx, acc);
  }
  mx = wave_max(mx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(z[c] - mx);
  se = wave_sum(se);
  const float inv = 1.f / se;
  __syncthreads();
  for (int r = 0; r < k; ++r) {
    float best = -FLT_MAX;
    int bi = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float v = z[c];
      if (v > best || (v == best && c < bi)) { best = v; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) {
      topk_idx[(size_t)row * k + r] = bi;
      topk_score[(size_t)row * k + r] = __expf(best - mx) * inv;
      z[bi] = -FLT_MAX;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- K12
constexpr int kRedThreads = 256;

struct RedAcc {
  double cnt = 0, sum = 0, comp = 0, lo = DBL_MAX, hi = -DBL_MAX;
  __device__ __forceinline__ void add(double v) {
    // Neumaier-compensated running sum: keeps fp64 sums within an ulp or two of
    // the reference's sequential Python sum for well-conditioned data
    const double t = sum + v;
    comp += fabs(sum) >= fabs(v) ? (sum - t) + v : (v - t) + sum;
    sum = t;
    lo = fmin(lo, v);
    hi = fmax(hi, v);
    cnt += 1;
  }
};

// 16-B vector loads (2 doubles / 4 floats per lane), four chunks in flight per
// iteration; elements before the first 16-B boundary and after the last full
// chunk take the scalar path. HBM-bound: ~8 B/lane loads left it at ~60 % of
// the chip's bandwidth.
template <typename T>
__global__ __launch_bounds__(kRedThreads) void reduce_stats_kernel(const T* __restrict__ x, int64_t n,
                                                                   double* __restrict__ partial) {
  constexpr int kPer = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(kPer)));
  __shared__ double sh[4][kRedThreads / 64];
  RedAcc a;
  const int64_t tid = (int64_t)blockIdx.x * kRedThreads + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kRedThreads;
  // head: up to the first 16-B aligned element
  const int64_t mis = (reinterpret_cast<uintptr_t>(x) & 15) / sizeof(T);
  const int64_t head = mis ? std::min<int64_t>(n, kPer - mis) : 0;
  if (tid < head) a.add((double)x[tid]);
  const vec_t* xv = reinterpret_cast<const vec_t*>(x + head);
  const int64_t nv = (n - head) / kPer;
  int64_t i = tid;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    vec_t u[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) u[c] = __builtin_nontemporal_load(xv + i + c * stride);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < kPer; ++e) a.add((double)u[c][e]);
  }
  for (; i < nv; i += stride) {
    const vec_t u = __builtin_nontemporal_load(xv + i);
#pragma unroll
    for (int e = 0; e < kPer; ++e) a.add((double)u[e]);
  }
  // tail
  const int64_t t0 = head + nv * kPer;
  if (t0 + tid < n) a.add((double)x[t0 + tid]);
  double cnt = a.cnt, sum = a.sum + a.comp, lo = a.lo, hi = a.hi;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    sum += __shfl_xor(sum, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = cnt; sh[1][w] = sum; sh[2][w] = lo; sh[3][w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kRedThreads / 64; ++i) {
      sh[0][0] += sh[0][i]; sh[1][0] += sh[1][i];
      sh[2][0] = fmin(sh[2][0], sh[2][i]); sh[3][0] = fmax(sh[3][0], sh[3][i]);
    }
    partial[4 * blockIdx.x + 0] = sh[0][0];
    partial[4 * blockIdx.x + 1] = sh[1][0];
    partial[4 * blockIdx.x + 2] = sh[2][0];
    partial[4 * blockIdx.x + 3] = sh[3][0];
  }
}

__global__ __launch_bounds__(64) void reduce_finalize_kernel(const double* __restrict__ partial, int blocks,
                                                             double* __restrict__ out) {
  double cnt = 0, sum = 0, lo = DBL_MAX, hi = -DBL_MAX;
  for (int i = threadIdx.x; i < blocks; i += 64) {
    cnt += partial[4 * i];
    sum += partial[4 * i + 1];
    lo = fmin(lo, partial[4 * i + 2]);
    hi = fmax(hi, partial[4 * i + 3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    sum += __shfl_xor(sum, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  if (threadIdx.x == 0) {
    out[0] = cnt; out[1] = sum; out[2] = lo; out[3] = hi;
  }
}

// accumulate one launch's block partials into a running device total (streamed
// reduces: one call per chunk, in chunk order -> deterministic)
__global__ __launch_bounds__(64) void reduce_accumulate_kernel(const double* __restrict__ partial, int blocks,
                                                               double* __restrict__ acc, int first) {
  double cnt = 0, sum = 0, lo = DBL_MAX, hi = -DBL_MAX;
  for (int i = threadIdx.x; i < blocks; i += 64) {
    cnt += partial[4 * i];
    sum += partial[4 * i + 1];
    lo = fmin(lo, partial[4 * i + 2]);
    hi = fmax(hi, partial[4 * i + 3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    sum += __shfl_xor(sum, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  if (threadIdx.x == 0) {
    if (first) {
      acc[0] = cnt; acc[1] = sum; acc[2] = lo; acc[3] = hi;
    } else {
      acc[0] += cnt; acc[1] += sum; acc[2] = fmin(acc[2], lo); acc[3] = fmax(acc[3], hi);
    }
  }
}

// ---------------------------------------------------------------- K13 + K12
// Streamed risk reduce over a raw CSV chunk (runtime/risk_stream.cpp): the host ships
// the chunk's record bytes and per-record offsets; one thread per record finds field
// `col` and parses it, and the values are reduced as in reduce_stats_kernel.

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

__device__ __forceinline__ bool csv_blank(int c) { return c == ' ' || c == '\t' || c == '\v' || c == '\f'; }
__device__ __forceinline__ bool csv_digit(int c) { return c >= '0' && c <= '9'; }

// Field `col` of the record [i, e) as a double by the exact fast path (Clinger): at most 19
// significant digits whose integer value w <= 2^53 and a decimal exponent |q| <= 22 give
// w * 10^q (or w / 10^-q) in ONE correctly rounded IEEE operation on two exact operands,
// i.e. the double strtod returns. Everything else (a quote before or in the field, more
// digits, a larger exponent, inf / nan / hex, bad syntax, a missing field) returns false
// and the host re-parses that record with strtod (CsvTable::parse_double): the same value,
// or the same error.
__device__ bool csv_field_number(const uint8_t* __restrict__ t, uint32_t i, uint32_t e, int col, double* out) {
  for (int f = 0; f < col; ++f) {
    for (;;) {
      if (i >= e) return false;
      const int c = t[i++];
      if (c == ',') break;
      if (c == '"' || c == '\n' || c == '\r') return false;
    }
  }
  while (i < e && csv_blank(t[i])) ++i;
  bool neg = false;
  if (i < e && (t[i] == '+' || t[i] == '-')) neg = t[i++] == '-';
  uint64_t w = 0;
  int nd = 0, frac = 0;
  bool any = false;
  for (; i < e && csv_digit(t[i]); ++i) {
    const int d = t[i] - '0';
    any = true;
    if (w || d) {
      if (++nd > 19) return false;
      w = w * 10 + d;
    }
  }
  if (i < e && t[i] == '.') {
    for (++i; i < e && csv_digit(t[i]); ++i) {
      const int d = t[i] - '0';
      any = true;
      ++frac;
      if (w || d) {
        if (++nd > 19) return false;
        w = w * 10 + d;
      }
    }
  }
  if (!any) return false;
  int ex = 0;
  if (i < e && (t[i] == 'e' || t[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < e && (t[i] == '+' || t[i] == '-')) eneg = t[i++] == '-';
    int ed = 0;
    for (; i < e && csv_digit(t[i]); ++i) {
      if (++ed > 4) return false;
      ex = ex * 10 + (t[i] - '0');
    }
    if (!ed) return false;
    if (eneg) ex = -ex;
  }
  while (i < e && csv_blank(t[i])) ++i;
  if (i < e && !(t[i] == ',' || t[i] == '\n' || t[i] == '\r')) return false;
  const int q = ex - frac;
  double v;
  if (w == 0) {
    v = 0.0;
  } else if (w <= (1ull << 53) && q >= -22 && q <= 22) {
    v = q >= 0 ? (double)w * kPow10[q] : (double)w / kPow10[-q];
  } else {
    return false;
  }
  *out = neg ? -v : v;
  return true;
}

__global__ __launch_bounds__(kRedThreads) void csv_parse_reduce_kernel(
    const uint8_t* __restrict__ text, const uint32_t* __restrict__ offs, int n, int col, int64_t row0,
    double* __restrict__ partial, int* __restrict__ fb_count, int64_t* __restrict__ fb_rows, int fb_cap) {
  __shared__ double sh[4][kRedThreads / 64];
  RedAcc a;
  for (int r = blockIdx.x * kRedThreads + threadIdx.x; r < n; r += gridDim.x * kRedThreads) {
    double v;
    if (csv_field_number(text, offs[r], offs[r + 1], col, &v)) {
      a.add(v);
    } else {
      const int k = atomicAdd(fb_count, 1);  // vector atomic, returns the slot
      if (k < fb_cap) fb_rows[k] = row0 + r;
    }
  }
  double cnt = a.cnt, sum = a.sum + a.comp, lo = a.lo, hi = a.hi;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    sum += __shfl_xor(sum, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = cnt; sh[1][w] = sum; sh[2][w] = lo; sh[3][w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kRedThreads / 64; ++i) {
      sh[0][0] += sh[0][i]; sh[1][0] += sh[1][i];
      sh[2][0] = fmin(sh[2][0], sh[2][i]); sh[3][0] = fmax(sh[3][0], sh[3][i]);
    }
    partial[4 * blockIdx.x + 0] = sh[0][0];
    partial[4 * blockIdx.x + 1] = sh[1][0];
    partial[4 * blockIdx.x + 2] = sh[2][0];
    partial[4 * blockIdx.x + 3] = sh[3][0];
  }
}

}  // namespace

void classify_head_topk(const bf16* pooled, int ldp, const bf16* Wc, const float* bc, float* logits,
                        int32_t* topk_idx, float* topk_score, int B, int N, int C, int k, hipStream_t stream) {
  ATPU_CHECK(C >= 1 && C <= kMaxClasses, "head: 1 <= classes <= 4096");
  ATPU_CHECK(k >= 1 && k <= C && k <= kMaxK, "head: 1 <= k <= min(C, 64)");
  ATPU_CHECK(N % 8 == 0, "head: hidden size must be a multiple of 8");
  if (B <= 0) return;
  const size_t shm = (size_t)(N + C) * sizeof(float);
  hipLaunchKernelGGL(head_topk_kernel, dim3(B), dim3(64), shm, stream, pooled, ldp, Wc, bc, logits, topk_idx,
                     topk_score, N, C, k);
  ATPU_HIP_CHECK(hipGetLastError());
}

int reduce_stats_blocks(int64_t n) {
  const int64_t want = (n + kRedThreads * 16 - 1) / (kRedThreads * 16);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, 4096));
}

void reduce_stats_f64(const double* x, int64_t n, double* partial, int blocks, hipStream_t stream) {
  hipLaunchKernelGGL(reduce_stats_kernel<double>, dim3(blocks), dim3(kRedThreads), 0, stream, x, n, partial);
  ATPU_HIP_CHECK(hipGetLastError());
}

void reduce_stats_f32(const float* x, int64_t n, double* partial, int blocks, hipStream_t stream) {
  hipLaunchKernelGGL(reduce_stats_kernel<float>, dim3(blocks), dim3(kRedThreads), 0, stream, x, n, partial);
  ATPU_HIP_CHECK(hipGetLastError());
}

void reduce_stats_finalize(const double* partial, int blocks, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(reduce_finalize_kernel, dim3(1), dim3(64), 0, stream, partial, blocks, out);
  ATPU_HIP_CHECK(hipGetLastError());
}

int csv_parse_blocks(int64_t n) {
  // ~16 records per thread, at most 2048 blocks (kCsvMaxBlocks: the partial buffers' size)
  const int64_t want = (n + kRedThreads * 16 - 1) / (kRedThreads * 16);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, kCsvMaxBlocks));
}

void csv_parse_reduce(const uint8_t* text, const uint32_t* offs, int n, int col, int64_t row0, double* partial,
                      int blocks, int* fb_count, int64_t* fb_rows, int fb_cap, hipStream_t stream) {
  ATPU_CHECK(blocks >= 1 && blocks <= kCsvMaxBlocks && col >= 0, "csv_parse_reduce: bad launch");
  hipLaunchKernelGGL(csv_parse_reduce_kernel, dim3(blocks), dim3(kRedThreads), 0, stream, text, offs, n, col, row0,
                     partial, fb_count, fb_rows, fb_cap);
  ATPU_HIP_CHECK(hipGetLastError());
}

void reduce_stats_accumulate(const double* partial, int blocks, double* acc, bool first, hipStream_t stream) {
  hipLaunchKernelGGL(reduce_accumulate_kernel, dim3(1), dim3(64), 0, stream, partial, blocks, acc, first ? 1 : 0);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
