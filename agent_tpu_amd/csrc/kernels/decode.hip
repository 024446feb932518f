// Seq2seq decode kernels for map_summarize.
//
//  * decode_attention: one query token per row against a KV cache.
//      - cross attention (lens != null): ONE workgroup per (batch item, head)
//        serves all `group` beam rows of that item, so the encoder K/V of the
//        item is streamed from HBM once per step instead of once per beam
//        (it is the dominant byte stream of a decode step).
//      - self attention (step_dev != null): key j of row r lives in the cache
//        of physical row hist[r][j] (beam backpointers, see beam_reorder_hist)
//        except the current position, which is the row's own; no cache copy
//        on beam reorder. Optional T5 relative-position bias by distance.
//    Scores: lane = key (full 128-B K row per lane, queries broadcast from
//    LDS); softmax with block reductions; P·V with lane = (key-sub, 8 dims):
//    one 16-B load per lane covers 8 keys x 128 B, fully coalesced.
//  * kv_append: write the new token's K/V (from the fused QKV GEMM output)
//    into the cache at step t (t read from device memory -> graph friendly).
//  * beam_reorder_hist: hist'[r][j] = hist[parent[r]][j] (j < t), hist'[r][t]
//    = parent[r]; the O(rows*T) int gather replaces an O(rows*T*L*2d) copy.
//    The same kernel keeps the running beams' token history (n-gram bans).
//  * gather_rows: explicit cache reorder (kept for callers without hist).
//  * beam_topk_rows: per beam row, ONE pass over the logits computes the
//    online max / sum-exp (log-softmax normaliser) and each wave's exact top-K
//    (candidates >= a rising threshold kept in LDS, cut back when full), then
//    wave-level argmax rounds merge the waves; the union over an item's beams
//    contains the item's global top-k (beam_select).
//  * beam_select: per item, the global top-2nb and the next running beams.
#include "atpu/common.h"
#include "atpu/kernels.h"
#include "atpu/l2_prefetch.h"
#include "atpu/ln_row.h"
#include "atpu/topk.h"

#include <cfloat>
#include <cstdlib>

namespace atpu {
namespace {

constexpr int kD = 64;
constexpr int kMaxKeys = 2048;

// Memory-level parallelism: a decode step is a latency-bound stream of short
// K/V rows, so both loops issue U independent tiles' loads before consuming
// any (one round trip per U tiles instead of per tile), and the self-attention
// backpointer rows are resolved once into LDS (phase 1) and reused by P.V.
constexpr int kUnrollS = 4;  // 16-key score tiles in flight per wave
constexpr int kUnrollV = 4;  // 8-key V slabs in flight per wave

// o[8] summed over the 8 key subs (lane bits 3-5) by butterfly: two permlane swaps and one
// xor-8 shuffle (7 cross-lane ops instead of 24); lane l ends with element l >> 3 of its sum
__device__ __forceinline__ float wave_bfly_rows8(const float (&o)[8]) {
  const int lane = threadIdx.x & 63;
  float a[4], b2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float2 p = pl32_swap(o[i], o[i + 4]);
    a[i] = p.x + p.y;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float2 p = pl16_swap(a[i], a[i + 2]);
    b2[i] = p.x + p.y;
  }
  const bool b3 = lane & 8;
  return (b3 ? b2[1] : b2[0]) + __shfl_xor(b3 ? b2[0] : b2[1], 8);
}


template <int GM, int NW>
__global__ __launch_bounds__(NW * 64) void decode_attention_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, int group, int nrows, const int32_t* __restrict__ lens, const int32_t* __restrict__ step_dev,
    const int32_t* __restrict__ hist, int hist_stride, const float* __restrict__ bias_dist, int bias_stride,
    bf16* __restrict__ out, int ldo, float scale) {
  // scores / probabilities, GM rows of pst = seq_stride rounded to 4 (dynamic: sized
  // to the cache, not kMaxKeys -- 32 KiB static held the cross-attention launch to 4
  // workgroups per CU)
  extern __shared__ float p_dyn[];
  const int pst = (seq_stride + 3) & ~3;
  auto P = [&](int g, int j) -> float& { return p_dyn[g * pst + j]; };
  __shared__ float po[NW][GM][kD];
  __shared__ float red[NW][16];
  __shared__ int prow[GM == 1 ? kMaxKeys : 1];  // self attention: physical cache row of key j
  // self attention: the beams of one item mostly share their history (backpointers
  // to the same physical cache rows), so consecutive rows go to ONE XCD (bijective
  // remap of the row index, guide T1) and re-read each other's K/V rows from its L2
  const int seq = (GM == 1 && hist) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int G = min(group, nrows - seq * group);
  int len = lens ? lens[seq] : (*step_dev + 1);
  len = min(len, seq_stride);  // <= kMaxKeys (host check)
  const bool use_hist = GM == 1 && hist != nullptr;
  auto row_of = [&](int j) -> int {
    return (use_hist && j < len - 1) ? hist[(size_t)seq * hist_stride + j] : seq;
  };
  auto at = [&](int r, int j) -> size_t { return ((size_t)r * seq_stride + j) * ldkv + h * kD; };
  // ---- scores on MFMA: S^T[16 keys x 16 queries] = K[16 x 64] . Q^T[64 x 16] ----
  // A operand = K rows (lane&15 = key, (lane>>4)*8 = dims), B operand = the
  // group's queries zero-padded to 16 (loop invariant, 8 VGPRs). Lane l gets
  // S[key (l>>4)*4 + e][query l&15].
  const int li = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 qb0, qb1;
  if (li < G) {
    const bf16* qr = q + (size_t)(seq * group + li) * ldq + h * kD;
    qb0 = *reinterpret_cast<const bf16x8*>(qr + kq);
    qb1 = *reinterpret_cast<const bf16x8*>(qr + 32 + kq);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) { qb0[e] = f2bf(0.f); qb1[e] = f2bf(0.f); }
  }
  // (8 tiles / slabs in flight per wave for cross attention measured the same as 4)
  constexpr int US = kUnrollS;
  constexpr int UV = kUnrollV;
  float mxl = -FLT_MAX;
  for (int t0 = w; t0 * 16 < len; t0 += NW * US) {
    bf16x8 a0[US], a1[US];
    int rr[US];
#pragma unroll
    for (int u = 0; u < US; ++u) rr[u] = row_of(min((t0 + u * NW) * 16 + li, len - 1));
#pragma unroll
    for (int u = 0; u < US; ++u) {
      const bf16* kr = k + at(rr[u], min((t0 + u * NW) * 16 + li, len - 1));
      a0[u] = *reinterpret_cast<const bf16x8*>(kr + kq);
      a1[u] = *reinterpret_cast<const bf16x8*>(kr + 32 + kq);
    }
#pragma unroll
    for (int u = 0; u < US; ++u) {
      const int t = t0 + u * NW;
      if (t * 16 >= len) break;
      if (GM == 1 && lane < 16 && t * 16 + lane < len) prow[t * 16 + lane] = rr[u];
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], qb0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], qb1, acc, 0, 0, 0);
      if (li < G) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = t * 16 + (lane >> 4) * 4 + e;
          if (j < len) {
            const float sj = acc[e] * scale + (bias_dist ? bias_dist[h * bias_stride + (len - 1 - j)] : 0.f);
            P(li, j) = sj;
            mxl = fmaxf(mxl, sj);
          }
        }
      }
    }
  }
  mxl = lane_rows_max(mxl);  // lanes l, l^16, l^32, l^48 by permlane swaps
  if (lane < 16) red[w][lane] = mxl;
  __syncthreads();
  // ---- P·V operands: lane = (key sub 0..7, dims (lane&7)*8 .. +8) ----
  const int ksub = lane >> 3, dc = (lane & 7) * 8;
  bf16x8 vv[UV];
  auto load_v = [&](int j0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int j = min(j0 + u * NW * 8 + ksub, len - 1);
      const int r = use_hist ? prow[j] : seq;
      vv[u] = *reinterpret_cast<const bf16x8*>(v + at(r, j) + dc);
    }
  };
  load_v(w * 8);  // in flight under the softmax
  float mx[GM];
#pragma unroll
  for (int g = 0; g < GM; ++g) {
    float m = red[0][g];
#pragma unroll
    for (int x = 1; x < NW; ++x) m = fmaxf(m, red[x][g]);
    mx[g] = m;
  }
  __syncthreads();
  float sm[GM];
#pragma unroll
  for (int g = 0; g < GM; ++g) sm[g] = 0.f;
  for (int j = tid; j < len; j += NW * 64) {
#pragma unroll
    for (int g = 0; g < GM; ++g) {
      if (g < G) {
        const float e = __expf(P(g, j) - mx[g]);
        P(g, j) = e;
        sm[g] += e;
      }
    }
  }
#pragma unroll
  for (int g = 0; g < GM; ++g) {
    const float s = wave_sum(sm[g]);
    if (lane == 0) red[w][g] = s;
  }
  __syncthreads();
  // ---- P·V ----
  float o[GM][8];
#pragma unroll
  for (int g = 0; g < GM; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[g][e] = 0.f;
  for (int j0 = w * 8; j0 < len; j0 += NW * 8 * UV) {
    if (j0 != w * 8) load_v(j0);
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int j = j0 + u * NW * 8 + ksub;
      if (j < len) {
#pragma unroll
        for (int g = 0; g < GM; ++g) {
          if (g < G) {
            const float pj = P(g, j);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[g][e] += pj * bf2f(vv[u][e]);
          }
        }
      }
    }
  }
  // reduce the 8 key-subgroups of the wave (lanes with equal lane&7) by butterfly: lane l
  // keeps dimension dc + ksub of each beam
#pragma unroll
  for (int g = 0; g < GM; ++g) po[w][g][dc + ksub] = wave_bfly_rows8(o[g]);
  __syncthreads();
  for (int i = tid; i < G * kD; i += NW * 64) {
    const int g = i / kD, d = i % kD;
    float s = 0.f, acc = 0.f;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
      s += red[x][g];
      acc += po[x][g][d];
    }
    out[(size_t)(seq * group + g) * ldo + h * kD + d] = f2bf(s > 0.f ? acc / s : 0.f);
  }
}

// ----------------------------------------------------------------------------
// Self-attention decode step, ONE workgroup per sequence row for ALL heads
// (default; ATPU_DEC_SELF=0 restores decode_attention_kernel<1, 4>).
// The per-(row, head) kernel above spends a 16-key MFMA tile and three block
// barriers on ~65 keys of one query, and every one of its rows x heads blocks
// walks the same dependent chain: backpointer load -> K row -> barrier ->
// V row -> barrier (206 us per call at 4096 rows, far from any bandwidth
// bound). Here the backpointer row is resolved once into LDS for all heads,
// and each wave owns whole heads, so nothing crosses waves after that:
//   scores : lane = key, the key's 128-B K row in 8 x 16-B loads, 32 v_dot2
//            with the (uniform) query, wave max / sum reductions;
//   P.V    : lane = (key sub 0..7, 8 dims), probabilities through a per-wave
//            LDS row, 16-B V loads kUnrollV deep, xor-reduce over key subs.
// ----------------------------------------------------------------------------
template <int NW>
__global__ __launch_bounds__(NW * 64) void decode_self_attention_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, const int32_t* __restrict__ step_dev, const int32_t* __restrict__ hist, int hist_stride,
    const float* __restrict__ bias_dist, int bias_stride, bf16* __restrict__ out, int ldo, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const int seq = xcd_remap(blockIdx.x, gridDim.x);  // beams of one item on one XCD (shared history rows)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int len = min(*step_dev + 1, seq_stride);
  const int cap = (seq_stride + 3) & ~3;
  int* prow = reinterpret_cast<int*>(dsm);                  // physical cache row of key j
  float* pw = reinterpret_cast<float*>(dsm) + cap * (1 + w);  // this wave's scores / probabilities
  for (int j = tid; j < len; j += NW * 64) prow[j] = (hist && j < len - 1) ? hist[(size_t)seq * hist_stride + j] : seq;
  __syncthreads();
  auto at = [&](int r, int j, int h) -> size_t { return ((size_t)r * seq_stride + j) * ldkv + h * kD; };
  const int ksub = lane >> 3, dc = (lane & 7) * 8;
  // gridDim.y > 1 (few rows: a grid of `rows` workgroups leaves the chip idle): workgroup y
  // takes heads y*NW + w, y*NW + w + NW*gridDim.y, ... (every workgroup resolves prow itself)
  for (int h = blockIdx.y * NW + w; h < H; h += NW * gridDim.y) {
    bf16x8 qq[8];  // the head's query, identical in every lane
    const bf16* qr = q + (size_t)seq * ldq + h * kD;
#pragma unroll
    for (int c = 0; c < 8; ++c) qq[c] = *reinterpret_cast<const bf16x8*>(qr + c * 8);
    float mx = -FLT_MAX;
    for (int j0 = 0; j0 < len; j0 += 64) {
      const int j = j0 + lane;
      if (j < len) {
        const bf16* kr = k + at(prow[j], j, h);
        bf16x8 kk[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) kk[c] = *reinterpret_cast<const bf16x8*>(kr + c * 8);
        float d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            d[e & 3] = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{kk[c][2 * e], kk[c][2 * e + 1]},
                                                       bf16x2_t{qq[c][2 * e], qq[c][2 * e + 1]}, d[e & 3], false);
        const float sj = ((d[0] + d[1]) + (d[2] + d[3])) * scale +
                         (bias_dist ? bias_dist[h * bias_stride + (len - 1 - j)] : 0.f);
        pw[j] = sj;
        mx = fmaxf(mx, sj);
      }
    }
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < len; j += 64) {
      const float e = __expf(pw[j] - mx);
      pw[j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    for (int j0 = 0; j0 < len; j0 += 8 * kUnrollV) {
      bf16x8 vv[kUnrollV];
#pragma unroll
      for (int u = 0; u < kUnrollV; ++u) {
        const int j = min(j0 + u * 8 + ksub, len - 1);
        vv[u] = *reinterpret_cast<const bf16x8*>(v + at(prow[j], j, h) + dc);
      }
#pragma unroll
      for (int u = 0; u < kUnrollV; ++u) {
        const int j = j0 + u * 8 + ksub;
        const float pj = j < len ? pw[j] : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pj * bf2f(vv[u][e]);
      }
    }
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    // key subs reduced by butterfly: lane l holds dim dc + ksub (one 2-B store per lane)
    out[(size_t)seq * ldo + h * kD + dc + ksub] = f2bf(wave_bfly_rows8(o) * inv);
  }
}

// ----------------------------------------------------------------------------
// Cross attention in 64-key chunks ("flash decoding"). The split kernel runs one wave per
// (item, head, chunk) for grids the per-(item, head) kernel leaves idle: 1 document x 12
// heads is 12 workgroups on 256 CUs, each walking 1024 keys through dependent load rounds
// (23 us per call where the K/V bytes take < 1 us). Per chunk:
//   scores : lane = key, its 128-B K row in 8 x 16-B loads, v_dot2 with each of the
//            item's G beam queries (LDS), butterfly max / sum over the beams;
//   P.V    : lane = (key sub 0..7, 8 dims), all 8 V slabs' loads in flight at once,
//            probabilities through LDS, xor-reduce over the key subs;
//   record : per (row, chunk) {max, sum, o[64]} (o unnormalised).
// decode_attn_combine_kernel rescales a row's chunks to the global max and divides. The
// chunked kernel runs the SAME chunk and combine code with the records in LDS, one workgroup
// per (item, head) (no record traffic; for many items), so both forms give the same bits
// and batch-invariant mode can pick either by the grid size.
// ----------------------------------------------------------------------------
constexpr int kSplitKeys = 64;
constexpr int kSplitRec = 2 + kD;  // floats per (row, head, chunk): max, sum, o[64]
constexpr int kMaxSplits = kMaxKeys / kSplitKeys;

struct XsArgs {  // one (item, head) of the cross attention
  const bf16* q;
  const bf16* k;
  const bf16* v;
  const float* bias_dist;
  int ldq, ldkv, seq_stride, group, bias_stride, seq, h, G, len;
  float scale;
};

template <bool B>
struct XsRegs {  // one chunk's operands: K (MFMA A fragments of the 4 16-key tiles), V slabs, bias
  bf16x8 ka[4], kb[4];  // tile t: key jb + 16 t + (lane & 15), dims (lane >> 4) * 8 (+32 in kb)
  bf16x8 vv[kSplitKeys / 8];
  float bj[B ? 4 : 1][4];  // (B) T5-style distance bias of key jb + 16 t + 4 (lane >> 4) + e
};

struct XsQ {  // the item's beam queries as the MFMA B operand: query lane & 15 (zero past G)
  bf16x8 q0, q1;
};

// The row is clamped and the padding zeroed by a select, not a predicated load: a load under
// `li < G` merged with an undefined value may be speculated for every lane by the compiler,
// i.e. read past the last item's rows (it was, and faulted on a small q).
__device__ __forceinline__ XsQ xs_q(const XsArgs& a) {
  const int lane = threadIdx.x & 63, li = lane & 15, kq = (lane >> 4) * 8;
  const bf16* qr = a.q + (size_t)(a.seq * a.group + min(li, a.G - 1)) * a.ldq + a.h * kD;
  XsQ r{*reinterpret_cast<const bf16x8*>(qr + kq), *reinterpret_cast<const bf16x8*>(qr + 32 + kq)};
  if (li >= a.G) {
#pragma unroll
    for (int e = 0; e < 8; ++e) r.q0[e] = r.q1[e] = f2bf(0.f);
  }
  return r;
}

// every load of chunk [jb, jb + n), n >= 1, issued at once (B: with the distance bias)
template <bool B>
__device__ __forceinline__ void xs_load(const XsArgs& a, int jb, int n, XsRegs<B>& r) {
  const int lane = threadIdx.x & 63, li = lane & 15, kq = (lane >> 4) * 8;
  auto at = [&](int j) -> size_t { return ((size_t)a.seq * a.seq_stride + j) * a.ldkv + a.h * kD; };
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16* kr = a.k + at(jb + min(t * 16 + li, n - 1));
    r.ka[t] = *reinterpret_cast<const bf16x8*>(kr + kq);
    r.kb[t] = *reinterpret_cast<const bf16x8*>(kr + 32 + kq);
  }
  const int ksub = lane >> 3, dc = (lane & 7) * 8;
#pragma unroll
  for (int u = 0; u < kSplitKeys / 8; ++u)
    r.vv[u] = *reinterpret_cast<const bf16x8*>(a.v + at(jb + min(u * 8 + ksub, n - 1)) + dc);
  if constexpr (B) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = jb + min(t * 16 + (lane >> 4) * 4 + e, n - 1);
        r.bj[t][e] = a.bias_dist[a.h * a.bias_stride + (a.len - 1 - j)];
      }
  }
}

// chunk [jb, jb + n) of the loaded operands -> the G rows' records rec(g) (one wave; pl is the
// wave's own probability rows):
//   scores : S^T[16 keys x 16 queries] per 16-key tile on MFMA (2 x 16x16x32 each); lane l
//            holds keys 4 (l >> 4) + e of each tile for query l & 15; max and sum of the query
//            over its lanes l, l^16, l^32, l^48 (lane_rows_*), in a fixed order;
//   P.V    : lane = (key sub 0..7, 8 dims), probabilities through LDS, xor-reduce over the subs.
// Every multiply-add here and in xs_combine is an explicit fma or an unfusable product, so the
// split and chunked kernels (different surrounding code) cannot differ in contraction.
template <int GM, bool B, class Rec>
__device__ __forceinline__ void xs_compute(const XsArgs& a, int n, const XsRegs<B>& r, const XsQ& q,
                                           float (&pl)[GM][kSplitKeys], Rec rec) {
  const int lane = threadIdx.x & 63, li = lane & 15, kg = lane >> 4, G = a.G;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.ka[t], q.q0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.kb[t], q.q1, acc[t], 0, 0, 0);
  }
  float sv[4][4], m = -FLT_MAX;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = t * 16 + kg * 4 + e;
      sv[t][e] = j < n ? __builtin_fmaf(acc[t][e], a.scale, B ? r.bj[B ? t : 0][e] : 0.f) : -FLT_MAX;
      m = fmaxf(m, sv[t][e]);
    }
  m = lane_rows_max(m);
  float sum = 0.f;
  f32x4 pv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pv[t][e] = t * 16 + kg * 4 + e < n ? __expf(sv[t][e] - m) : 0.f;
      sum += pv[t][e];
    }
  sum = lane_rows_sum(sum);
  if (li < G) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<f32x4*>(&pl[li][t * 16 + kg * 4]) = pv[t];
  }
  __builtin_amdgcn_wave_barrier();  // (one wave: LDS ops complete in order)
  const int ksub = lane >> 3, dc = (lane & 7) * 8;
  float o[GM][8];
#pragma unroll
  for (int g = 0; g < GM; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[g][e] = 0.f;
#pragma unroll
  for (int u = 0; u < kSplitKeys / 8; ++u) {
    const int jl = u * 8 + ksub;
#pragma unroll
    for (int g = 0; g < GM; ++g) {
      if (g < G) {
        const float pj = jl < n ? pl[g][jl] : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[g][e] = __builtin_fmaf(pj, bf2f(r.vv[u][e]), o[g][e]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < GM; ++g) {
    if (g < G) {
      float* rp = rec(g);
      // the 8 dims over the key subs (lane bits 3-5) by butterfly: lane l ends with dim dc + ksub
      rp[2 + dc + ksub] = wave_bfly_rows8(o[g]);
      if (lane == g) {  // query g's max and sum (lanes l & 15 == g hold them)
        rp[0] = m;
        rp[1] = sum;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // pl is rewritten by the wave's next chunk
}

// a chunk past the item's source length contributes nothing
template <class Rec>
__device__ __forceinline__ void xs_empty(int G, Rec rec) {
  for (int i = threadIdx.x & 63; i < G * kSplitRec; i += 64) {
    const int g = i / kSplitRec, e = i % kSplitRec;
    rec(g)[e] = e == 0 ? -FLT_MAX : 0.f;
  }
}

// out[h*64 + d] of one row = sum_c o_c[d] e^(m_c - M) / sum_c l_c e^(m_c - M), M = max_c m_c,
// from the row's NS records r[c * kSplitRec] (one wave): lane c < NS takes chunk c's (max, sum)
// and the weights are reduced across lanes; then lane = dimension sums the chunks' o with
// every load issued before the first add (a loop of dependent rounds took 8 us per call).
// NSM >= NS record slots are read (16 covers 1024-token sources).
template <int NSM>
__device__ __forceinline__ void xs_combine(const float* r, int NS, bf16* __restrict__ out_row) {
  const int lane = threadIdx.x & 63;
  float ov[NSM];
#pragma unroll
  for (int c = 0; c < NSM; ++c) ov[c] = r[min(c, NS - 1) * kSplitRec + 2 + lane];
  const float mr = r[min(lane, NS - 1) * kSplitRec], lr = r[min(lane, NS - 1) * kSplitRec + 1];  // (in bounds)
  const float m = lane < NS ? mr : -FLT_MAX;
  const float l = lane < NS ? lr : 0.f;
  const float M = wave_max(m);
  const float w = lane < NS ? __expf(m - M) : 0.f;  // 0 for an empty chunk (max -FLT_MAX)
  float wl = w * l;
  asm volatile("" : "+v"(wl));  // a rounded product: never fused into the reduction's first add
  const float L = wave_sum(wl);
  float o = 0.f;
#pragma unroll
  for (int c = 0; c < NSM; ++c)
    o = __builtin_fmaf(c < NS ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), c)) : 0.f, ov[c], o);
  out_row[lane] = f2bf(L > 0.f ? o / L : 0.f);
}

__device__ __forceinline__ void xs_combine_any(const float* r, int NS, bf16* __restrict__ out_row) {
  if (NS <= 16)
    xs_combine<16>(r, NS, out_row);
  else
    xs_combine<kMaxSplits>(r, NS, out_row);
}

template <int GM, bool B>
__global__ __launch_bounds__(64) void decode_cross_split_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, int group, int nrows, const int32_t* __restrict__ lens, const float* __restrict__ bias_dist,
    int bias_stride, float* __restrict__ ws, int H, float scale) {
  __shared__ __attribute__((aligned(16))) float pl[GM][kSplitKeys];
  const int seq = blockIdx.x, h = blockIdx.y, c = blockIdx.z, NS = gridDim.z;
  const int G = min(group, nrows - seq * group);
  const int len = min(lens[seq], seq_stride);
  const XsArgs a{q, k, v, bias_dist, ldq, ldkv, seq_stride, group, bias_stride, seq, h, G, len, scale};
  const int jb = c * kSplitKeys, n = max(0, min(kSplitKeys, len - jb));
  auto rec = [&](int g) { return ws + (((size_t)(seq * group + g) * H + h) * NS + c) * kSplitRec; };
  if (n == 0) {
    xs_empty(G, rec);
    return;
  }
  // every load before any use: the beams' queries, the K tiles, the V slabs (and the bias)
  const XsQ qr = xs_q(a);
  XsRegs<B> r;
  xs_load<B>(a, jb, n, r);
  xs_compute<GM, B>(a, n, r, qr, pl, rec);
}

// one wave per (row, head)
__global__ __launch_bounds__(64) void decode_attn_combine_kernel(const float* __restrict__ ws, int NS, int H,
                                                                 bf16* __restrict__ out, int ldo) {
  const int row = blockIdx.x, h = blockIdx.y;
  xs_combine_any(ws + ((size_t)row * H + h) * NS * kSplitRec, NS, out + (size_t)row * ldo + h * kD);
}

// One workgroup per (item, head): wave w takes chunks w, w + NW, ..., the next chunk's loads in
// flight under the current one's arithmetic, records into LDS ([GM][NSX] x kSplitRec floats,
// NS <= NSX), then wave g % NW combines beam row g.
template <int GM, int NW, int NSX, bool B>
__global__ __launch_bounds__(NW * 64) void decode_cross_chunked_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, int group, int nrows, const int32_t* __restrict__ lens, const float* __restrict__ bias_dist,
    int bias_stride, bf16* __restrict__ out, int ldo, int NS, float scale) {
  __shared__ float recs[GM][NSX][kSplitRec];
  __shared__ __attribute__((aligned(16))) float pl[NW][GM][kSplitKeys];
  const int seq = blockIdx.x, h = blockIdx.y, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = min(group, nrows - seq * group);
  const int len = min(lens[seq], seq_stride);
  const XsArgs a{q, k, v, bias_dist, ldq, ldkv, seq_stride, group, bias_stride, seq, h, G, len, scale};
  const int nch = min(NS, (len + kSplitKeys - 1) / kSplitKeys);  // chunks holding keys
  auto nkeys = [&](int c) { return min(kSplitKeys, len - c * kSplitKeys); };
  const XsQ qr = xs_q(a);
  XsRegs<B> r0;
  {  // (unconditional on a clamped chunk: see xs_q)
    const int c0 = min(w, max(nch - 1, 0));
    xs_load<B>(a, c0 * kSplitKeys, max(1, nkeys(c0)), r0);
  }
  for (int c = nch + w; c < NS; c += NW) {  // chunks past the source length
    auto rec = [&](int g) { return &recs[g][c][0]; };
    xs_empty(G, rec);
  }
  // one register set (168 VGPRs: three waves per SIMD) -- the other resident waves hide a chunk's
  // load latency; two sets (236 VGPRs, two waves per SIMD) ran 256-doc T5 at 542 vs 593 docs/s
  for (int c = w; c < nch; c += NW) {
    if (c != w) xs_load<B>(a, c * kSplitKeys, nkeys(c), r0);
    auto rec0 = [&](int g) { return &recs[g][c][0]; };
    xs_compute<GM, B>(a, nkeys(c), r0, qr, pl[w], rec0);
  }
  __syncthreads();
  for (int g = w; g < G; g += NW)
    xs_combine_any(&recs[g][0][0], NS, out + (size_t)(seq * group + g) * ldo + h * kD);
}

// ----------------------------------------------------------------------------
// Self attention of few rows (the 1-document job: 4 beam rows) with a short cache
// (T <= 64 KC keys): ONE wave per (row, head), 48 waves over 48 CUs, two memory round
// trips in all. Round 1: the step, the row's backpointers (every key the cache can hold,
// masked by the length later) and the head's query; round 2: the K row of every key
// (lane = key, KC chunks) and the V slabs of every key (lane = (key sub, 8 dims)), all
// issued before the first use. decode_self_attention_kernel walks the same keys in up to
// 3 + 5 dependent load rounds per head (6.3 us per call at 4 rows x 12 heads).
// ----------------------------------------------------------------------------
template <int KC>
__global__ __launch_bounds__(64) void decode_self_few_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ k, const bf16* __restrict__ v, int ldkv,
    int seq_stride, const int32_t* __restrict__ step_dev, const int32_t* __restrict__ hist, int hist_stride,
    const float* __restrict__ bias_dist, int bias_stride, bf16* __restrict__ out, int ldo, float scale) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  constexpr int NK = KC * 64, NV = NK / 8;
  __shared__ int prow[NK];
  __shared__ float pw[NK];
  const int seq = xcd_remap(blockIdx.x, gridDim.x), h = blockIdx.y, lane = threadIdx.x;
  const int ksub = lane >> 3, dc = (lane & 7) * 8;
  // round 1
  const int stp = *step_dev;
  int hv[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int j = c * 64 + lane;
    hv[c] = (hist && j < hist_stride) ? hist[(size_t)seq * hist_stride + j] : seq;
  }
  bf16x8 qq[8];
  const bf16* qr = q + (size_t)seq * ldq + h * kD;
#pragma unroll
  for (int e = 0; e < 8; ++e) qq[e] = *reinterpret_cast<const bf16x8*>(qr + e * 8);
  const int len = min(stp + 1, seq_stride);
  auto at = [&](int r, int j) -> size_t { return ((size_t)r * seq_stride + j) * ldkv + h * kD; };
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int j = c * 64 + lane;
    hv[c] = (hist && j < len - 1) ? hv[c] : seq;
    prow[j] = hv[c];
  }
  __syncthreads();  // one wave: orders the prow writes before the V address reads
  // round 2: every K row and V slab of the cache's first len keys
  bf16x8 kk[KC][8], vv[NV];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    if (c * 64 < len) {  // wave-uniform
      const int j = min(c * 64 + lane, len - 1);
      const bf16* kr = k + at(j == c * 64 + lane ? hv[c] : prow[j], j);
#pragma unroll
      for (int e = 0; e < 8; ++e) kk[c][e] = *reinterpret_cast<const bf16x8*>(kr + e * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    if (u * 8 < len) {
      const int j = min(u * 8 + ksub, len - 1);
      vv[u] = *reinterpret_cast<const bf16x8*>(v + at(prow[j], j) + dc);
    }
  }
  float mx = -FLT_MAX;
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int j = c * 64 + lane;
    if (c * 64 < len) {
      float d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          d[t] = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{kk[c][e][2 * t], kk[c][e][2 * t + 1]},
                                                 bf16x2_t{qq[e][2 * t], qq[e][2 * t + 1]}, d[t], false);
      const float sj = j < len ? ((d[0] + d[1]) + (d[2] + d[3])) * scale +
                                     (bias_dist ? bias_dist[h * bias_stride + (len - 1 - j)] : 0.f)
                               : -FLT_MAX;
      pw[j] = sj;
      mx = fmaxf(mx, sj);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int j = c * 64 + lane;
    if (c * 64 < len) {
      const float e = j < len ? __expf(pw[j] - mx) : 0.f;
      pw[j] = e;
      sum += e;
    }
  }
  sum = wave_sum(sum);
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    if (u * 8 < len) {
      const int j = u * 8 + ksub;
      const float pj = j < len ? pw[j] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pj * bf2f(vv[u][e]);
    }
  }
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  // key subs reduced by the row kernel's butterfly (bit-identical to it)
  out[(size_t)seq * ldo + h * kD + dc + ksub] = f2bf(wave_bfly_rows8(o) * inv);
}

// hist'[r][j] = hist[parent[r]][j] for j < t; hist'[r][t] = last ? last[r] : parent[r],
// t = *step_dev + off (token histories: last = the new tokens, off = 1)
__global__ __launch_bounds__(256) void beam_reorder_hist_kernel(const int32_t* __restrict__ src,
                                                                int32_t* __restrict__ dst,
                                                                const int32_t* __restrict__ parent, int rows,
                                                                int stride, const int32_t* __restrict__ step_dev,
                                                                const int32_t* __restrict__ last, int off) {
  const int t = min(*step_dev + off, stride - 1);
  const int n = rows * (t + 1);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / (t + 1), j = i % (t + 1);
    const int pr = parent[r];
    dst[(size_t)r * stride + j] = j < t ? src[(size_t)pr * stride + j] : (last ? last[r] : pr);
  }
}

// The whole per-step state advance of a small beam search in ONE workgroup (1-document decode:
// it replaced 2 reorders, 3 copies and the step increment, ~4.5 us of launch each):
//   hist[r][:t] = hist[par[r]][:t], hist[r][t] = par[r]                (t = step)
//   seq[r][:t+1] = seq[par[r]][:t+1], seq[r][t+1] = tok[r]   (optional, n-gram bans)
//   tokens[r] = tok[r];  step += 1
// in place: every row is gathered into LDS before any is written back.
// NG > 0: also the decoder input of the new tokens, rows of N = 256 NG (the next step's first
// launch folded in): xout[r] = emb[tok[r]] (T5), or with gamma LN(emb[tok[r]] + pos[step + 1 +
// pos_off]) (BART: embed_pos_ln_kernel's math, ln_hw_row), one half wave per row.
template <int NG>
__global__ __launch_bounds__(256) void decode_advance_kernel(int32_t* __restrict__ hist, int32_t* __restrict__ seq,
                                                             int rows, int stride, const int32_t* __restrict__ par,
                                                             const int32_t* __restrict__ tok,
                                                             int32_t* __restrict__ tokens, int32_t* step_dev,
                                                             DecEmbed em) {
  extern __shared__ int32_t adv_sh[];  // [rows][stride] hist, then [rows][stride] seq
  const int tid = threadIdx.x;
  const int step = *step_dev;
  const int th = min(step, stride - 1), ts = min(step + 1, stride - 1);
  for (int i = tid; i < rows * th; i += blockDim.x) {
    const int r = i / th, j = i - r * th;
    adv_sh[r * stride + j] = hist[(size_t)par[r] * stride + j];
  }
  if (seq)
    for (int i = tid; i < rows * ts; i += blockDim.x) {
      const int r = i / ts, j = i - r * ts;
      adv_sh[(rows + r) * stride + j] = seq[(size_t)par[r] * stride + j];
    }
  __syncthreads();  // every source row read before any row is overwritten (and step read by all)
  for (int i = tid; i < rows * (th + 1); i += blockDim.x) {
    const int r = i / (th + 1), j = i - r * (th + 1);
    hist[(size_t)r * stride + j] = j < th ? adv_sh[r * stride + j] : par[r];
  }
  if (seq)
    for (int i = tid; i < rows * (ts + 1); i += blockDim.x) {
      const int r = i / (ts + 1), j = i - r * (ts + 1);
      seq[(size_t)r * stride + j] = j < ts ? adv_sh[(rows + r) * stride + j] : tok[r];
    }
  for (int r = tid; r < rows; r += blockDim.x) tokens[r] = tok[r];
  if (tid == 0) *step_dev = step + 1;
  if constexpr (NG > 0) {
    constexpr int N = NG * 256;
    const int hl = tid & 31;
    for (int r = tid >> 5; r < rows; r += 8) {  // 8 half waves
      int id = tok[r];
      id = id < 0 ? 0 : (id >= em.vocab ? em.vocab - 1 : id);
      const bf16* er = em.table + (size_t)id * N;
      if (em.gamma) {
        int pi = step + 1 + em.pos_off;
        pi = pi < 0 ? 0 : (pi >= em.npos ? em.npos - 1 : pi);
        ln_hw_row<NG, false>(er, em.pos ? em.pos + (size_t)pi * N : nullptr, em.gamma, em.beta, em.out + (size_t)r * N,
                             true, em.eps, hl);
      } else {
#pragma unroll
        for (int g = 0; g < NG; ++g)
          *reinterpret_cast<bf16x8*>(em.out + (size_t)r * N + g * 256 + hl * 8) =
              *reinterpret_cast<const bf16x8*>(er + g * 256 + hl * 8);
      }
    }
  }
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
constexpr int kTopkWaves = kTopkThreads / 64;
constexpr int kMaxBeamK = 16;
constexpr int kMaxBans = 512;  // banned tokens per row (beam_topk_rows); more -> the caller's exact path

template <int K, bool BANS>
__global__ __launch_bounds__(kTopkThreads) void beam_topk_kernel(const float* __restrict__ logits, int V,
                                                                 const float* __restrict__ beam_scores, int eos,
                                                                 int mask_eos, float* __restrict__ out_score,
                                                                 int32_t* __restrict__ out_token, int vec4,
                                                                 const int32_t* __restrict__ bans, int nbmax,
                                                                 const int32_t* __restrict__ seq, int seq_stride,
                                                                 int cur, int ngram) {
  __shared__ float wm[kTopkWaves], ws[kTopkWaves];
  constexpr int KM = K;
  __shared__ float cv[kTopkWaves * KM];
  __shared__ int ci[kTopkWaves * KM];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* x = logits + (size_t)row * V;
  float tv[KM];
  int ti[KM];
#pragma unroll
  for (int r = 0; r < KM; ++r) { tv[r] = -FLT_MAX; ti[r] = 0x7fffffff; }
  // normaliser over ALL tokens; the min-length EOS mask applies to selection
  // only (HF applies MinLengthLogitsProcessor after log_softmax).
  // 16-B loads, 4 per thread in flight per round (the scalar, branchy loop ran at
  // ~1 TB/s); the running (max, sum) is rescaled once per 16 values.
  // no-repeat-n-gram bans: the row's banned token ids (-1 padded) become a V-bit LDS
  // bitmap, tested (one ds_read) only for a value that would enter the candidates,
  // so the kernel returns the top K among the allowed tokens (HF applies the processor
  // after log_softmax: the normaliser still covers every token). A per-candidate scan of
  // the ban list diverged: some lane of a wave inserts at almost every value, so every
  // wave ran the whole scan per value (584 us per BART step).
  extern __shared__ uint32_t ban_bits[];  // (V + 31) / 32 words when nbmax > 0
  if (BANS) {
    const int nw = (V + 31) / 32;
    for (int w2 = tid; w2 < nw; w2 += kTopkThreads) ban_bits[w2] = 0u;
    __syncthreads();
    for (int b = tid; b < nbmax; b += kTopkThreads) {
      const int t = bans[(size_t)row * nbmax + b];
      if (t >= 0 && t < V) atomicOr(&ban_bits[t >> 5], 1u << (t & 31));
    }
    // no-repeat-n-gram from the device token history (HF NoRepeatNGramLogitsProcessor):
    // the row's first cur tokens; window i bans its last token when its first n-1
    // match the row's last n-1
    if (ngram > 0 && cur >= ngram) {
      const int32_t* sr = seq + (size_t)row * seq_stride;
      for (int i = tid; i + ngram <= cur; i += kTopkThreads) {
        bool eq = true;
        for (int e = 0; e + 1 < ngram; ++e) eq = eq && sr[i + e] == sr[cur - ngram + 1 + e];
        const int t = sr[i + ngram - 1];
        if (eq && t >= 0 && t < V) atomicOr(&ban_bits[t >> 5], 1u << (t & 31));
      }
    }
    __syncthreads();
  }
  float m = -FLT_MAX, s = 0.f;
  // Selection (per wave, exact): a value enters the wave's candidate buffer (LDS,
  // ballot + mbcnt compaction) only if it is >= thr, a lower bound of the wave's K-th
  // best allowed value: every value below thr has K strictly better ones. thr starts
  // at the K-th largest lane maximum of the first 16 values per lane and rises when a
  // nearly full buffer is cut back to the candidates >= the K-th largest of their
  // per-lane maxima. A float4 costs a max, a compare and a ballot unless one of the
  // wave's is a candidate. The per-lane sorted-list insert this replaces ran on every
  // value some lane of the wave inserted (60 of 90 us per 1024 x 32128 step); a
  // sorted cut-back (list insert + K-round wave top-K) per refill cost as much again.
  constexpr int kBuf = 16 * 64 + 64;
  __shared__ float bufv[kTopkWaves][kBuf];
  __shared__ int bufi[kTopkWaves][kBuf];
  float* bv = bufv[w];
  int* bi = bufi[w];
  float thr = -FLT_MAX;
  int cnt = 0;  // wave-uniform
  float rv;
  int ri;
  // K-th largest of one value per lane (duplicates count), -FLT_MAX if fewer than K
  auto kth_lane_max = [&](float x) __attribute__((always_inline)) -> float {
    float t = -FLT_MAX;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      t = wave_max(x);
      const unsigned long long hit = __ballot(x == t);
      if (lane == (int)__builtin_ctzll(hit | (1ull << 63))) x = -FLT_MAX;
    }
    return t;
  };
  // sorted top K of the buffer -> (rv, ri) in lanes 0..K-1, buffer = those K
  auto exact_cut = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < KM; ++r) { tv[r] = -FLT_MAX; ti[r] = 0x7fffffff; }
    for (int c = lane; c < cnt; c += 64) list_insert<KM>(tv, ti, bv[c], bi[c]);
    wave_topk<KM>(tv, ti, rv, ri);
    __builtin_amdgcn_wave_barrier();
    if (lane < K) { bv[lane] = rv; bi[lane] = ri; }
    thr = fmaxf(thr, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rv), K - 1)));
    cnt = K;
    __builtin_amdgcn_wave_barrier();
  };
  // room for one more chunk (1024 values): raise thr, keep the candidates >= thr
  auto make_room = [&]() __attribute__((always_inline)) {
    if (cnt <= kBuf - 16 * 64) return;
    float lmx = -FLT_MAX;
    for (int c = lane; c < cnt; c += 64) lmx = fmaxf(lmx, bv[c]);
    thr = fmaxf(thr, kth_lane_max(lmx));
    int n = 0;
    for (int c0 = 0; c0 < cnt; c0 += 64) {  // in place: round r writes below (r + 1) * 64
      const int c = c0 + lane;
      const bool in = c < cnt;
      const float val = in ? bv[c] : -FLT_MAX;
      const int id = in ? bi[c] : 0;
      const bool keep = in && val >= thr;
      const unsigned long long bal = __ballot(keep);
      __builtin_amdgcn_wave_barrier();
      if (keep) {
        const int pos = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        bv[pos] = val;
        bi[pos] = id;
      }
      __builtin_amdgcn_wave_barrier();
      n += __popcll(bal);
    }
    cnt = n;
    if (cnt > kBuf - 16 * 64) exact_cut();  // candidates held by fewer than K lanes
  };
  auto push = [&](float sel, int i, bool p) __attribute__((always_inline)) {
    if (BANS && p) p = !((ban_bits[i >> 5] >> (i & 31)) & 1u);
    const unsigned long long bal = __ballot(p);
    if (bal == 0) return;
    if (p) {
      const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      bv[pos] = sel;
      bi[pos] = i;
    }
    cnt += __popcll(bal);
  };
  // Loops run over block-uniform ranges (ballots and cut-backs need the whole wave).
  // Two register sets alternate: loads are unconditional (index clamped, value
  // masked), so the next 16 values per lane are in flight under the current 16 and
  // the compiler's counted waits stay exact (a conditional or copied prefetch made
  // it wait for everything).
  const int nv4 = vec4 ? V / 4 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int eos4 = mask_eos ? (eos >> 2) : -1;
  auto load4 = [&](float4 (&dst)[4], int jb) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = x4[min(jb + tid + u * kTopkThreads, nv4 - 1)];
  };
  auto process = [&](const float4 (&src)[4], int jb) __attribute__((always_inline)) {
    make_room();
    float4 v[4];
    float lm[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = jb + tid + u * kTopkThreads < nv4;
      v[u] = ok ? src[u] : make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX);
      lm[u] = fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
    }
    const float cm = fmaxf(m, fmaxf(fmaxf(lm[0], lm[1]), fmaxf(lm[2], lm[3])));
    s *= __expf(m - cm);  // m == -FLT_MAX: s is 0 either way
    m = cm;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      s += (__expf(v[u].x - m) + __expf(v[u].y - m)) + (__expf(v[u].z - m) + __expf(v[u].w - m));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (__builtin_expect(jb + tid + u * kTopkThreads == eos4, 0)) {  // selection only: the normaliser keeps EOS
        const int c = eos & 3;
        if (c == 0) v[u].x = -FLT_MAX;
        if (c == 1) v[u].y = -FLT_MAX;
        if (c == 2) v[u].z = -FLT_MAX;
        if (c == 3) v[u].w = -FLT_MAX;
        lm[u] = fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
      }
    }
    // first chunk: no candidates yet; K lanes hold allowed values >= the K-th largest
    // lane maximum (banned values are dropped from this chunk's selection first)
    if (jb == 0) {
      if (BANS) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = 4 * (jb + tid + u * kTopkThreads);
          auto banned = [&](int t) { return t < V && ((ban_bits[t >> 5] >> (t & 31)) & 1u); };
          if (banned(i)) v[u].x = -FLT_MAX;
          if (banned(i + 1)) v[u].y = -FLT_MAX;
          if (banned(i + 2)) v[u].z = -FLT_MAX;
          if (banned(i + 3)) v[u].w = -FLT_MAX;
          lm[u] = fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
        }
      }
      thr = kth_lane_max(fmaxf(fmaxf(lm[0], lm[1]), fmaxf(lm[2], lm[3])));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // a float4 of the wave enters the per-value path only if one of its values can
      // be a candidate
      if (__ballot(lm[u] >= thr) == 0) continue;
      const bool ok = jb + tid + u * kTopkThreads < nv4;
      const int i = 4 * (jb + tid + u * kTopkThreads);
      push(v[u].x, i, ok && v[u].x >= thr);
      push(v[u].y, i + 1, ok && v[u].y >= thr);
      push(v[u].z, i + 2, ok && v[u].z >= thr);
      push(v[u].w, i + 3, ok && v[u].w >= thr);
    }
  };
  if (nv4 > 0) {
    float4 ra[4], rb[4];
    load4(ra, 0);
    for (int jb = 0; jb < nv4; jb += 8 * kTopkThreads) {  // an odd chunk count runs one masked chunk
      load4(rb, jb + 4 * kTopkThreads);
      process(ra, jb);
      load4(ra, jb + 8 * kTopkThreads);
      process(rb, jb + 4 * kTopkThreads);
    }
  }
  for (int ib = 4 * nv4; ib < V; ib += kTopkThreads) {  // tail (or every element without vec4)
    if (cnt > kBuf - 64) exact_cut();
    const int i = ib + tid;
    const bool ok = i < V;
    const float val = ok ? x[i] : -FLT_MAX;
    if (ok) {
      if (val > m) {
        s = s * __expf(m - val) + 1.f;
        m = val;
      } else {
        s += __expf(val - m);
      }
    }
    const float sel = (mask_eos && i == eos) ? -FLT_MAX : val;
    push(sel, i, ok && sel >= thr);
  }
  exact_cut();  // lanes 0..K-1: the wave's top K in (rv, ri)
  // block log-sum-exp
  const float wmax = wave_max(m);
  float sa = (m == -FLT_MAX) ? 0.f : s * __expf(m - wmax);
  sa = wave_sum(sa);
  if (lane == 0) { wm[w] = wmax; ws[w] = sa; }
  if (lane < K) { cv[w * KM + lane] = rv; ci[w * KM + lane] = ri; }
  __syncthreads();
  if (w == 0) {
    float gm = -FLT_MAX;
#pragma unroll
    for (int x2 = 0; x2 < kTopkWaves; ++x2) gm = fmaxf(gm, wm[x2]);
    float gs = 0.f;
#pragma unroll
    for (int x2 = 0; x2 < kTopkWaves; ++x2) gs += ws[x2] * __expf(wm[x2] - gm);
    const float shift = beam_scores[row] - gm - __logf(gs);
    // merge kTopkWaves sorted lists of K: lane l takes candidates l, l+64, ...
#pragma unroll
    for (int r = 0; r < KM; ++r) { tv[r] = -FLT_MAX; ti[r] = 0x7fffffff; }
    for (int c = lane; c < kTopkWaves * K; c += 64) {
      const int ww = c / K, rr = c % K;
      list_insert<KM>(tv, ti, cv[ww * KM + rr], ci[ww * KM + rr]);
    }
    wave_topk<KM>(tv, ti, rv, ri);
    if (lane < K) {
      out_score[(size_t)row * K + lane] = rv == -FLT_MAX ? -FLT_MAX : rv + shift;
      out_token[(size_t)row * K + lane] = ri;
    }
  }
}

// ----------------------------------------------------------------------------
// Beam selection on the device (one workgroup per batch item): from each beam
// row's top K2 continuations (beam_topk_rows) pick the item's global top K2 by
// (score desc, beam*V + token asc), mark hits (EOS, or the last position), keep
// the best nb non-hits (stable) as the next running beams and write the next
// step's inputs straight into the device staging row [parent rows | tokens |
// running scores]. The host gets a per-item record [top score bits K2 | top
// tokens K2 | top beams K2 | kept slots nb] by async D2H for its finished-
// hypothesis bookkeeping, so the next decoder step is enqueued without a host
// round trip (runtime/summarize.py, device selection).
// ----------------------------------------------------------------------------
constexpr int kSelMax = 256;  // nb * K2 candidates per item
__global__ __launch_bounds__(kSelMax) void beam_select_kernel(const float* __restrict__ sc,
                                                              const int32_t* __restrict__ tk, int nb, int K2, int V,
                                                              int eos, int hit_all, float neg,
                                                              int32_t* __restrict__ stage, int rows,
                                                              int32_t* __restrict__ rec) {
  __shared__ float cs[kSelMax];
  __shared__ long long cf[kSelMax];
  __shared__ int ctok[kSelMax];
  __shared__ float ts[kSelMax];
  __shared__ int tt[kSelMax], tb[kSelMax];
  __shared__ float rc[kSelMax];
  const int b = blockIdx.x, c = threadIdx.x, n = nb * K2;
  if (c < n) {
    const size_t src = (size_t)b * n + c;  // rows b*nb .. b*nb+nb-1, K2 each: contiguous
    cs[c] = sc[src];
    ctok[c] = tk[src];
    cf[c] = (long long)(c / K2) * V + tk[src];
  }
  __syncthreads();
  if (c < n) {
    const float s = cs[c];
    const long long f = cf[c];
    int rank = 0;
    // (score desc, flat asc, candidate index asc): np.lexsort's order, total even for
    // duplicate (score, token) pairs
    for (int o = 0; o < n; ++o) rank += (cs[o] > s || (cs[o] == s && (cf[o] < f || (cf[o] == f && o < c)))) ? 1 : 0;
    if (rank < K2) {
      ts[rank] = s;
      tt[rank] = ctok[c];
      tb[rank] = c / K2;
    }
  }
  __syncthreads();
  if (c < K2) {
    const bool hit = hit_all || tt[c] == eos;
    rc[c] = hit ? ts[c] + neg : ts[c];
  }
  __syncthreads();
  int32_t* r = rec + (size_t)b * (3 * K2 + nb);
  if (c < K2) {
    const float x = rc[c];
    int rank = 0;
    for (int o = 0; o < K2; ++o) rank += (rc[o] > x || (rc[o] == x && o < c)) ? 1 : 0;
    if (rank < nb) {
      const int row = b * nb + rank;
      stage[row] = b * nb + tb[c];
      stage[rows + row] = tt[c];
      stage[2 * rows + row] = __float_as_int(x);
      r[3 * K2 + rank] = c;
    }
    r[c] = __float_as_int(ts[c]);
    r[K2 + c] = tt[c];
    r[2 * K2 + c] = tb[c];
  }
}

}  // namespace

int decode_self_few(int set) {
  // few-row self attention: one wave per (row, head), all loads in two rounds
  // (decode_self_few_kernel); ATPU_DEC_SELF_FEW=0 or decode_self_few(0) turns it off
  static int v = [] {
    const char* f = std::getenv("ATPU_DEC_SELF_FEW");
    return (f && f[0] == '0') ? 0 : 1;
  }();
  if (set == 0 || set == 1) v = set;
  return v;
}

int decode_attention_splits(int rows, int group, int H, int seq_stride, bool cross) {
  // key chunks of the split cross attention while the per-(item, head) grid (items x heads)
  // cannot cover the chip twice, else 0 (decode_cross_chunked_kernel under batch invariance: the
  // same bits; decode_attention_kernel otherwise)
  if (!cross || group < 1 || group > 8 || seq_stride < 2 * kSplitKeys) return 0;
  const int nseq = (rows + group - 1) / group;
  if (nseq * H >= 512) return 0;
  return (seq_stride + kSplitKeys - 1) / kSplitKeys;
}

size_t decode_attention_ws_floats(int rows, int group, int H, int seq_stride, bool cross) {
  const int ns = decode_attention_splits(rows, group, H, seq_stride, cross);
  return ns ? (size_t)rows * H * ns * kSplitRec : 0;
}

void decode_attention(const bf16* q, int ldq, const bf16* k, const bf16* v, int ldkv, int seq_stride, int group,
                      const int32_t* lens, const int32_t* step_dev, const int32_t* hist, int hist_stride,
                      const float* bias_dist, int bias_stride, bf16* out, int ldo, int rows, int H, float scale,
                      hipStream_t stream, float* ws) {
  ATPU_CHECK(rows > 0 && H > 0 && group >= 1, "decode_attention: bad shape");
  ATPU_CHECK(lens || step_dev, "decode_attention: need lens or a device step");
  ATPU_CHECK(!hist || (step_dev && group == 1), "decode_attention: hist is for self attention (group 1)");
  ATPU_CHECK(ldq % 8 == 0 && ldkv % 8 == 0, "decode_attention: 16-B rows required");
  ATPU_CHECK((reinterpret_cast<uintptr_t>(k) & 15) == 0 && (reinterpret_cast<uintptr_t>(v) & 15) == 0,
             "decode_attention: K/V must be 16-byte aligned");
  static const bool row_kernel = [] {
    const char* f = std::getenv("ATPU_DEC_SELF");
    return !(f && f[0] == '0');
  }();
  if (group == 1 && step_dev && !lens && row_kernel) {
    ATPU_CHECK(seq_stride <= kMaxKeys, "decode_attention: cache length above 2048");
    ATPU_CHECK(!hist || hist_stride >= seq_stride, "decode_attention: hist rows shorter than the cache");
    ATPU_CHECK(ldo % 8 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (reinterpret_cast<uintptr_t>(q) & 15) == 0,
               "decode_attention: q / out need 16-B rows");
    // batch invariance: the few-row kernel (one wave per (row, head)) at any row count while the
    // cache fits it, so a row never switches kernels with the batch size
    if (seq_stride <= 192 && decode_self_few(-1) && (rows * H <= num_cus() || batch_invariant(-1))) {
#define ATPU_SF(KC)                                                                                                \
  hipLaunchKernelGGL((decode_self_few_kernel<KC>), dim3(rows, H), dim3(64), 0, stream, q, ldq, k, v, ldkv, seq_stride, \
                     step_dev, hist, hist_stride, bias_dist, bias_stride, out, ldo, scale)
      if (seq_stride <= 64) {
        ATPU_SF(1);
      } else if (seq_stride <= 128) {
        ATPU_SF(2);
      } else {
        ATPU_SF(3);
      }
#undef ATPU_SF
      ATPU_HIP_CHECK(hipGetLastError());
      return;
    }
    constexpr int NW = 4;
    const size_t smem = (size_t)((seq_stride + 3) & ~3) * 4 * (1 + NW);
    // few rows: head groups over grid.y (one head per wave) so the launch covers more CUs
    const int hg = rows < 128 ? (H + NW - 1) / NW : 1;
    hipLaunchKernelGGL((decode_self_attention_kernel<NW>), dim3(rows, hg), dim3(NW * 64), smem, stream, q, ldq, k, v, ldkv,
                       seq_stride, step_dev, hist, hist_stride, bias_dist, bias_stride, out, ldo, H, scale);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  ATPU_CHECK(seq_stride <= kMaxKeys, "decode_attention: cache length above 2048");
  const int nseq = (rows + group - 1) / group;
  const int ns = decode_attention_splits(rows, group, H, seq_stride, lens != nullptr && !hist);
  if (ns > 0 && ws) {
    static_assert(kMaxSplits * kSplitKeys >= kMaxKeys, "combine kernel chunk count");
    ATPU_CHECK(ldq % 8 == 0 && (reinterpret_cast<uintptr_t>(q) & 15) == 0, "decode_attention: q needs 16-B rows");
    ATPU_CHECK((reinterpret_cast<uintptr_t>(ws) & 15) == 0, "decode_attention: ws must be 16-byte aligned");
#define ATPU_DS1(GM, B)                                                                                         \
  hipLaunchKernelGGL((decode_cross_split_kernel<GM, B>), dim3(nseq, H, ns), dim3(64), 0, stream, q, ldq, k, v,  \
                     ldkv, seq_stride, group, rows, lens, bias_dist, bias_stride, ws, H, scale)
#define ATPU_DS(GM)          \
  if (bias_dist) {           \
    ATPU_DS1(GM, true);      \
  } else {                   \
    ATPU_DS1(GM, false);     \
  }
    if (group == 1) {
      ATPU_DS(1);
    } else if (group <= 4) {
      ATPU_DS(4);
    } else {
      ATPU_DS(8);
    }
#undef ATPU_DS
#undef ATPU_DS1
    ATPU_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(decode_attn_combine_kernel, dim3(rows, H), dim3(64), 0, stream, ws, ns, H, out, ldo);
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
  // batch invariance: a grid too large to split runs the split form's chunk and combine arithmetic
  // in one workgroup per (item, head), so an item rounds the same in a launch of any size
  if (lens && !hist && group <= 8 && seq_stride >= 2 * kSplitKeys && batch_invariant(-1)) {
    ATPU_CHECK(ldq % 8 == 0 && (reinterpret_cast<uintptr_t>(q) & 15) == 0, "decode_attention: q needs 16-B rows");
    const int ns = (seq_stride + kSplitKeys - 1) / kSplitKeys;
#define ATPU_DC1(GM, NSX, B)                                                                                    \
  hipLaunchKernelGGL((decode_cross_chunked_kernel<GM, 4, NSX, B>), dim3(nseq, H), dim3(256), 0, stream, q, ldq, k, \
                     v, ldkv, seq_stride, group, rows, lens, bias_dist, bias_stride, out, ldo, ns, scale)
#define ATPU_DC(GM, NSX)        \
  if (bias_dist) {              \
    ATPU_DC1(GM, NSX, true);    \
  } else {                      \
    ATPU_DC1(GM, NSX, false);   \
  }
#define ATPU_DC_NS(GM)  \
  if (ns <= 16) {       \
    ATPU_DC(GM, 16);    \
  } else {              \
    ATPU_DC(GM, 32);    \
  }
    if (group == 1) {
      ATPU_DC_NS(1)
    } else if (group <= 4) {
      ATPU_DC_NS(4)
    } else {
      ATPU_DC_NS(8)
    }
#undef ATPU_DC_NS
#undef ATPU_DC
#undef ATPU_DC1
    ATPU_HIP_CHECK(hipGetLastError());
    return;
  }
#define ATPU_DA(GM, NW)                                                                                          \
  hipLaunchKernelGGL((decode_attention_kernel<GM, NW>), dim3(nseq, H), dim3(NW * 64),                           \
                     (size_t)GM * ((seq_stride + 3) & ~3) * sizeof(float), stream, q, ldq, k, v, ldkv,          \
                     seq_stride, group, rows, lens, step_dev, hist, hist_stride, bias_dist, bias_stride, out, ldo, \
                     scale)
  if (group == 1)
    ATPU_DA(1, 4);
  else if (group <= 4)
    ATPU_DA(4, 4);
  else if (group <= 8)
    ATPU_DA(8, 4);
  else
    ATPU_CHECK(false, "decode_attention: group (beams) must be <= 8");
#undef ATPU_DA
  ATPU_HIP_CHECK(hipGetLastError());
}

size_t decode_advance_lds(int rows, int stride, bool seq) { return (size_t)rows * stride * (seq ? 2 : 1) * 4; }

void decode_advance(int32_t* hist, int32_t* seq, int rows, int stride, const int32_t* par, const int32_t* tok,
                    int32_t* tokens, int32_t* step_dev, hipStream_t stream, const DecEmbed& em, int N) {
  ATPU_CHECK(rows > 0 && stride > 0 && hist && par && tok && tokens && step_dev, "decode_advance: bad arguments");
  const size_t lds = decode_advance_lds(rows, stride, seq != nullptr);
  ATPU_CHECK(lds <= 64 * 1024, "decode_advance: rows x stride too large for one workgroup (use beam_reorder_hist)");
  if (!em.table) {
    hipLaunchKernelGGL(decode_advance_kernel<0>, dim3(1), dim3(256), lds, stream, hist, seq, rows, stride, par, tok,
                       tokens, step_dev, em);
  } else {
    ATPU_CHECK(em.out && em.vocab > 0 && (!em.gamma || (em.beta && (!em.pos || em.npos > 0))),
               "decode_advance: embedding needs table, out, vocab (and beta / positions with gamma)");
    ATPU_CHECK((reinterpret_cast<uintptr_t>(em.table) & 15) == 0 && (reinterpret_cast<uintptr_t>(em.out) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(em.pos) & 15) == 0 && (reinterpret_cast<uintptr_t>(em.gamma) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(em.beta) & 15) == 0,
               "decode_advance: embedding operands must be 16-byte aligned");
    switch (N) {
      case 512:
        hipLaunchKernelGGL(decode_advance_kernel<2>, dim3(1), dim3(256), lds, stream, hist, seq, rows, stride, par, tok,
                           tokens, step_dev, em);
        break;
      case 768:
        hipLaunchKernelGGL(decode_advance_kernel<3>, dim3(1), dim3(256), lds, stream, hist, seq, rows, stride, par, tok,
                           tokens, step_dev, em);
        break;
      case 1024:
        hipLaunchKernelGGL(decode_advance_kernel<4>, dim3(1), dim3(256), lds, stream, hist, seq, rows, stride, par, tok,
                           tokens, step_dev, em);
        break;
      default:
        throw std::invalid_argument("decode_advance: embedding width must be 512, 768 or 1024");
    }
  }
  ATPU_HIP_CHECK(hipGetLastError());
}

void beam_reorder_hist(const int32_t* src, int32_t* dst, const int32_t* parent, int rows, int stride,
                       const int32_t* step_dev, hipStream_t stream, const int32_t* last, int off) {
  ATPU_CHECK(rows > 0 && stride > 0 && off >= 0, "beam_reorder_hist: bad shape");
  const int blocks = std::max(1, std::min(1024, (rows * stride + 255) / 256));
  hipLaunchKernelGGL(beam_reorder_hist_kernel, dim3(blocks), dim3(256), 0, stream, src, dst, parent, rows, stride,
                     step_dev, last, off);
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
                    float* out_score, int32_t* out_token, hipStream_t stream, const int32_t* bans, int nbmax,
                    const int32_t* seq, int seq_stride, int cur, int ngram) {
  ATPU_CHECK(K >= 1 && K <= kMaxBeamK && K <= V, "beam_topk: 1 <= K <= 16");
  ATPU_CHECK(nbmax >= 0 && nbmax <= kMaxBans && (nbmax == 0 || bans), "beam_topk: 0 <= banned tokens per row <= 512");
  ATPU_CHECK(ngram <= 0 || (seq && cur <= seq_stride), "beam_topk: n-gram bans need the token history [rows, >= cur]");
  if (ngram > 0 && cur < ngram) ngram = 0;
  const bool any_bans = nbmax > 0 || ngram > 0;
  const int vec4 = V % 4 == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
  const size_t smem = any_bans ? (size_t)((V + 31) / 32) * 4 : 0;
  ATPU_CHECK(smem <= 64 * 1024, "beam_topk: vocabulary too large for the ban bitmap (2M tokens)");
#define ATPU_TK(KK)                                                                                             \
  case KK:                                                                                                      \
    if (any_bans)                                                                                               \
      hipLaunchKernelGGL((beam_topk_kernel<KK, true>), dim3(rows), dim3(kTopkThreads), smem, stream, logits, V, \
                         beam_scores, eos, mask_eos, out_score, out_token, vec4, bans, nbmax, seq, seq_stride,  \
                         cur, ngram);                                                                           \
    else                                                                                                        \
      hipLaunchKernelGGL((beam_topk_kernel<KK, false>), dim3(rows), dim3(kTopkThreads), smem, stream, logits,   \
                         V, beam_scores, eos, mask_eos, out_score, out_token, vec4, bans, nbmax, seq,           \
                         seq_stride, cur, ngram);                                                               \
    break;
  switch (K) {
    ATPU_TK(1) ATPU_TK(2) ATPU_TK(3) ATPU_TK(4) ATPU_TK(5) ATPU_TK(6) ATPU_TK(7) ATPU_TK(8)
    ATPU_TK(9) ATPU_TK(10) ATPU_TK(11) ATPU_TK(12) ATPU_TK(13) ATPU_TK(14) ATPU_TK(15) ATPU_TK(16)
    default: break;
  }
#undef ATPU_TK
  ATPU_HIP_CHECK(hipGetLastError());
}

uintptr_t host_device_ptr(uintptr_t host, size_t bytes) {
  // the device address of a pinned (hipHostMalloc'd / registered) host buffer, checked on the
  // host before any kernel writes there: an unmapped address would fault the GPU
  hipPointerAttribute_t a{};
  ATPU_HIP_CHECK(hipPointerGetAttributes(&a, reinterpret_cast<void*>(host)));
  ATPU_CHECK(a.type == hipMemoryTypeHost && a.devicePointer != nullptr,
             "host_device_ptr: not a device-mapped pinned host buffer");
  // the whole range must lie in the same mapping
  hipPointerAttribute_t b{};
  ATPU_HIP_CHECK(hipPointerGetAttributes(&b, reinterpret_cast<void*>(host + (bytes ? bytes - 1 : 0))));
  ATPU_CHECK(b.type == hipMemoryTypeHost && b.devicePointer != nullptr &&
                 reinterpret_cast<uintptr_t>(b.devicePointer) - reinterpret_cast<uintptr_t>(a.devicePointer) ==
                     (bytes ? bytes - 1 : 0),
             "host_device_ptr: the range is not one pinned mapping");
  return reinterpret_cast<uintptr_t>(a.devicePointer);
}

void beam_select(const float* sc, const int32_t* tk, int B, int nb, int K2, int V, int eos, int hit_all, float neg,
                 int32_t* stage, int32_t* rec, hipStream_t stream) {
  ATPU_CHECK(B > 0 && nb >= 1 && K2 >= nb && nb * K2 <= kSelMax, "beam_select: need nb <= K2 and nb*K2 <= 256");
  hipLaunchKernelGGL(beam_select_kernel, dim3(B), dim3(kSelMax), 0, stream, sc, tk, nb, K2, V, eos, hit_all, neg,
                     stage, B * nb, rec);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
