// Seq2seq decode kernels for map_summarize.
//
//  * decode_attention: one query token per row against a KV cache. Self
//    attention reads the beam's own cache rows [0, t]; cross attention reads
//    the ENCODER K/V of the row's batch item (rows / group), masked by the
//    source length. Optional T5 relative-position bias indexed by distance.
//    One 64-wide wave per (row, head): q lives in registers, lane j scores key
//    j of each 64-key chunk (128-B row reads), the softmax is a wave
//    reduction, and lane d accumulates output dim d over keys (coalesced V
//    rows).
//  * kv_append: write the new token's K/V (from the fused QKV GEMM output)
//    into the cache at step t (t read from device memory -> graph friendly).
//  * gather_rows: beam reorder, dst[r] = src[parent[r]] for the first n rows
//    of every cache slab.
//  * beam_topk_rows: per beam row, log-softmax(logits) + beam score (+ EOS
//    mask while below min_length) and its top-k candidates; the union over a
//    batch item's beams contains that item's global top-k (merge on host).
#include "atpu/common.h"
#include "atpu/kernels.h"

#include <cfloat>

namespace atpu {
namespace {

constexpr int kD = 64;
constexpr int kMaxKeys = 2048;

__global__ __launch_bounds__(64) void decode_attention_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, int group, const int32_t* __restrict__ lens, const int32_t* __restrict__ step_dev,
    const float* __restrict__ bias_dist, int bias_stride, bf16* __restrict__ out, int ldo, float scale) {
  __shared__ float p[kMaxKeys];
  const int row = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int seq = row / group;
  int len = lens ? lens[seq] : (*step_dev + 1);
  len = min(len, kMaxKeys);
  // q row -> registers (fp32)
  float qv[kD];
  const bf16* qr = q + (size_t)row * ldq + h * kD;
#pragma unroll
  for (int c = 0; c < kD / 8; ++c) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(qr + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[c * 8 + e] = bf2f(x[e]) * scale;
  }
  const size_t base = (size_t)seq * seq_stride;
  float mx = -FLT_MAX;
  for (int j0 = 0; j0 < len; j0 += 64) {
    const int j = j0 + lane;
    float s = -FLT_MAX;
    if (j < len) {
      const bf16* kr = k + (base + j) * ldkv + h * kD;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < kD / 8; ++c) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(kr + c * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += qv[c * 8 + e] * bf2f(x[e]);
      }
      if (bias_dist) acc += bias_dist[h * bias_stride + (len - 1 - j)];
      s = acc;
      p[j] = s;
    }
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < len; j += 64) {
    const float e = __expf(p[j] - mx);
    p[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  // lane d accumulates output dim d
  float o = 0.f;
  const bf16* vcol = v + base * ldkv + h * kD + lane;
  int j = 0;
  for (; j + 4 <= len; j += 4) {
    const float v0 = bf2f(vcol[(size_t)(j + 0) * ldkv]);
    const float v1 = bf2f(vcol[(size_t)(j + 1) * ldkv]);
    const float v2 = bf2f(vcol[(size_t)(j + 2) * ldkv]);
    const float v3 = bf2f(vcol[(size_t)(j + 3) * ldkv]);
    o += p[j] * v0 + p[j + 1] * v1 + p[j + 2] * v2 + p[j + 3] * v3;
  }
  for (; j < len; ++j) o += p[j] * bf2f(vcol[(size_t)j * ldkv]);
  out[(size_t)row * ldo + h * kD + lane] = f2bf(o * inv);
}

// cache[row][t][0:ncols] = src[row][col0 : col0+ncols]
__global__ __launch_bounds__(256) void kv_append_kernel(const bf16* __restrict__ src, int lds, int col0, int ncols,
                                                        bf16* __restrict__ cache, int seq_stride, int ldc,
                                                        const int32_t* __restrict__ step_dev, int rows) {
  const int t = *step_dev;
  const int per_row = ncols / 8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows * per_row; i += gridDim.x * blockDim.x) {
    const int r = i / per_row, c = (i % per_row) * 8;
    *reinterpret_cast<bf16x8*>(cache + ((size_t)r * seq_stride + t) * ldc + c) =
        *reinterpret_cast<const bf16x8*>(src + (size_t)r * lds + col0 + c);
  }
}

// dst[slab][r][0:n_rows_used][:] = src[slab][parent[r]][...]
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                          const int32_t* __restrict__ parent, int nrows,
                                                          int seq_stride, int ldc, const int32_t* __restrict__ step_dev,
                                                          int slabs, size_t slab_elems) {
  const int used = *step_dev + 1;
  const int per_tok = ldc / 8;
  const size_t per_row = (size_t)used * per_tok;
  const size_t total = (size_t)slabs * nrows * per_row;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t slab = i / (nrows * per_row);
    const size_t rem = i % (nrows * per_row);
    const int r = (int)(rem / per_row);
    const size_t w = rem % per_row;
    const int tok = (int)(w / per_tok), c = (int)(w % per_tok) * 8;
    const size_t so = slab * slab_elems + ((size_t)parent[r] * seq_stride + tok) * ldc + c;
    const size_t d = slab * slab_elems + ((size_t)r * seq_stride + tok) * ldc + c;
    *reinterpret_cast<bf16x8*>(dst + d) = *reinterpret_cast<const bf16x8*>(src + so);
  }
}

constexpr int kTopkThreads = 256;
constexpr int kMaxBeamK = 16;

// one block per beam row: log-softmax + beam score, then top-K (value desc,
// index asc) via per-thread sorted lists and K rounds of block argmax
__global__ __launch_bounds__(kTopkThreads) void beam_topk_kernel(const float* __restrict__ logits, int V,
                                                                 const float* __restrict__ beam_scores, int eos,
                                                                 int mask_eos, int K, float* __restrict__ out_score,
                                                                 int32_t* __restrict__ out_token) {
  __shared__ float red[kTopkThreads / 64];
  __shared__ float cand_v[kTopkThreads];
  __shared__ int cand_i[kTopkThreads];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* x = logits + (size_t)row * V;
  float mx = -FLT_MAX;
  // normaliser over ALL tokens; the min-length EOS mask applies to selection
  // only (HF applies MinLengthLogitsProcessor after log_softmax)
  for (int i = tid; i < V; i += kTopkThreads) mx = fmaxf(mx, x[i]);
  mx = wave_max(mx);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float se = 0.f;
  for (int i = tid; i < V; i += kTopkThreads) se += __expf(x[i] - mx);
  se = wave_sum(se);
  if (lane == 0) red[w] = se;
  __syncthreads();
  se = red[0] + red[1] + red[2] + red[3];
  const float shift = beam_scores[row] - mx - __logf(se);
  // per-thread sorted top-K
  float tv[kMaxBeamK];
  int ti[kMaxBeamK];
#pragma unroll
  for (int r = 0; r < kMaxBeamK; ++r) { tv[r] = -FLT_MAX; ti[r] = 0x7fffffff; }
  for (int i = tid; i < V; i += kTopkThreads) {
    const float val = (mask_eos && i == eos) ? -FLT_MAX : x[i];
    if (val > tv[K - 1]) {
      int pos = K - 1;
      while (pos > 0 && val > tv[pos - 1]) {
        tv[pos] = tv[pos - 1];
        ti[pos] = ti[pos - 1];
        --pos;
      }
      tv[pos] = val;
      ti[pos] = i;
    }
  }
  int head = 0;
  for (int r = 0; r < K; ++r) {
    cand_v[tid] = head < K ? tv[head] : -FLT_MAX;
    cand_i[tid] = head < K ? ti[head] : 0x7fffffff;
    __syncthreads();
    for (int s = kTopkThreads / 2; s > 0; s >>= 1) {
      if (tid < s) {
        const float a = cand_v[tid], b = cand_v[tid + s];
        const int ia = cand_i[tid], ib = cand_i[tid + s];
        if (b > a || (b == a && ib < ia)) { cand_v[tid] = b; cand_i[tid] = ib; }
      }
      __syncthreads();
    }
    const int win = cand_i[0];
    const float wv = cand_v[0];
    if (tid == 0) {
      out_score[(size_t)row * K + r] = wv == -FLT_MAX ? -FLT_MAX : wv + shift;
      out_token[(size_t)row * K + r] = win;
    }
    if (head < K && ti[head] == win && tv[head] == wv) ++head;  // owner advances
    __syncthreads();
  }
}

}  // namespace

void decode_attention(const bf16* q, int ldq, const bf16* k, const bf16* v, int ldkv, int seq_stride, int group,
                      const int32_t* lens, const int32_t* step_dev, const float* bias_dist, int bias_stride, bf16* out,
                      int ldo, int rows, int H, float scale, hipStream_t stream) {
  ATPU_CHECK(rows > 0 && H > 0 && group >= 1, "decode_attention: bad shape");
  ATPU_CHECK(lens || step_dev, "decode_attention: need lens or a device step");
  ATPU_CHECK(ldq % 8 == 0 && ldkv % 8 == 0, "decode_attention: 16-B rows required");
  hipLaunchKernelGGL(decode_attention_kernel, dim3(rows, H), dim3(64), 0, stream, q, ldq, k, v, ldkv, seq_stride, group,
                     lens, step_dev, bias_dist, bias_stride, out, ldo, scale);
  ATPU_HIP_CHECK(hipGetLastError());
}

void kv_append(const bf16* src, int lds, int col0, int ncols, bf16* cache, int seq_stride, int ldc,
               const int32_t* step_dev, int rows, hipStream_t stream) {
  ATPU_CHECK(ncols % 8 == 0 && lds % 8 == 0 && ldc % 8 == 0 && col0 % 8 == 0, "kv_append: 16-B alignment");
  const int work = rows * ncols / 8;
  hipLaunchKernelGGL(kv_append_kernel, dim3(std::max(1, std::min(1024, (work + 255) / 256))), dim3(256), 0, stream,
                     src, lds, col0, ncols, cache, seq_stride, ldc, step_dev, rows);
  ATPU_HIP_CHECK(hipGetLastError());
}

void gather_rows(const bf16* src, bf16* dst, const int32_t* parent, int nrows, int seq_stride, int ldc,
                 const int32_t* step_dev, int slabs, size_t slab_elems, hipStream_t stream) {
  ATPU_CHECK(ldc % 8 == 0, "gather_rows: 16-B rows required");
  hipLaunchKernelGGL(gather_rows_kernel, dim3(2048), dim3(256), 0, stream, src, dst, parent, nrows, seq_stride, ldc,
                     step_dev, slabs, slab_elems);
  ATPU_HIP_CHECK(hipGetLastError());
}

void beam_topk_rows(const float* logits, int rows, int V, const float* beam_scores, int eos, int mask_eos, int K,
                    float* out_score, int32_t* out_token, hipStream_t stream) {
  ATPU_CHECK(K >= 1 && K <= kMaxBeamK && K <= V, "beam_topk: 1 <= K <= 16");
  hipLaunchKernelGGL(beam_topk_kernel, dim3(rows), dim3(kTopkThreads), 0, stream, logits, V, beam_scores, eos, mask_eos,
                     K, out_score, out_token);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
