// Host-side launch API for every hand-written gfx950 kernel in csrc/kernels.
// All launchers are asynchronous on the given stream and graph-capturable
// (no allocation, no synchronisation inside).
#pragma once
#include <vector>

#include <hip/hip_runtime.h>

#include <cstdint>

namespace atpu {

typedef __bf16 bf16;

// ---------------------------------------------------------------- random init (atpu/rand.h)
// dst[i] = Irwin-Hall(4) value of (seed, sid, i) x (i < n0 ? scale0 : scale1), bf16 (RNE) or fp32;
// bit-identical to rand_fill_host (runtime.h)
void rand_fill(void* dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0, float scale1,
               hipStream_t stream);

// ---------------------------------------------------------------- GEMM (K3/K5/K6)
enum GemmEpilogue : int {
  kEpiBias = 1,
  kEpiGelu = 2,
  kEpiTanh = 4,
  kEpiResidual = 8,
  kEpiRelu = 16,
  kEpiOutF32 = 32,  // C is float* (128x128 kernel only; LM-head logits)
  // LayerNorm folding (post-LN encoders; persistent 256x256 full-line kernel only,
  // M, N, K multiples of 256). LN(x) = (x - mu) * rstd * gamma + beta is never
  // materialised: its producer emits row statistics, its consumers apply them.
  kEpiInNorm = 64,     // A rows are raw LN inputs, gamma folded into Bt, beta into bias:
                       //   C = rstd*acc - rstd*mu*colsum + bias    (rstd, mu from in_fin)
  kEpiResNorm = 128,   // R rows are raw LN inputs (beta folded into bias):
                       //   C = ... + (R*rstd - rstd*mu) * gamma     (rstd, mu from res_fin)
  kEpiStatsOut = 256,  // also write per-row partial (sum, sum of squares) of C, one per 256 columns
  kEpiKvScatter = 1024,  // decode QKV: columns >= kv_col0 (K|V) go to the KV cache at row m*kv_T + *kv_step
                         //   (leading dim kv_ld), columns < kv_col0 (Q) to C (128x128 / "dec" kernels)
  kEpiRowRms = 512,    // A rows are raw RMSNorm inputs (gamma folded into Bt): the kernel sums A^2
                       //   over its K loop, C = rsqrt(mean_k A^2 + rms_eps) * (A . Bt^T) ... (128x128 and
                       //   skinny "dec" kernels, no split-K; T5 decoder steps)
  // LayerNorm folding for decode steps (post-LN decoders, BART; 128x128 and "dec" kernels,
  // no split-K). Row statistics travel as partial (sum, sumsq) per 32-column slab:
  kEpiRowLn = 2048,     // A rows are raw LN inputs, gamma folded into Bt, beta into bias:
                        //   C = rstd*acc - rstd*mu*colsum + bias, (mu, rstd) of A's rows from in_part
                        //   [K/32][M][2] (eps in rms_eps)
  kEpiResLn = 4096,     // R rows are raw LN inputs (beta folded into bias), stats from res_part
                        //   [N/32][M][2]: C = ... + (R*rstd - rstd*mu) * gamma
  kEpiRowStats = 8192,  // also write part_out [N/32][M][2]: (sum, sumsq) of the bf16-rounded C
                        //   values of each row's 32-column slabs
};

struct GemmArgs {
  const bf16* A = nullptr;  // [M, K] row-major, leading dim lda
  int lda = 0;
  const bf16* Bt = nullptr;  // [N, K] row-major (nn.Linear.weight layout)
  int ldb = 0;
  bf16* C = nullptr;  // [M, N], leading dim ldc
  int ldc = 0;
  const float* bias = nullptr;  // [N] fp32
  const bf16* R = nullptr;      // residual [M, N], leading dim ldr
  int ldr = 0;
  int M = 0, N = 0, K = 0;
  int epi = 0;
  // split-K (skinny M): splits > 1 needs ws = fp32 [splits, M, N]
  int splits = 1;
  float* ws = nullptr;
  // LayerNorm folding (see kEpiInNorm / kEpiResNorm / kEpiStatsOut)
  const float* in_fin = nullptr;   // InNorm: [M][2] (rstd, rstd*mu) of A's rows
  const float* colsum = nullptr;   // InNorm: [N] fp32, colsum[n] = sum_k Bt[n][k]
  const float* res_fin = nullptr;  // ResNorm: [M][2] (rstd, rstd*mu) of R's rows
  const float* gamma = nullptr;    // ResNorm: [N] LN gamma of R
  float* part_out = nullptr;       // StatsOut: [N/256][M][2] partial (sum, sumsq) of C's rows (fp32 values)
  const float* in_part = nullptr;   // RowLn: [K/32][M][2] (sum, sumsq) partials of A's rows (+ colsum)
  const float* res_part = nullptr;  // ResLn: [N/32][M][2] partials of R's rows (+ gamma); RowStats: part_out
  float rms_eps = 0.f;             // RowRms
  bf16* kv_cache = nullptr;        // KvScatter: cache [rows * kv_T, kv_ld]
  int kv_ld = 0, kv_T = 0, kv_col0 = 0;
  const int32_t* kv_step = nullptr;  // device scalar: the position being written
  // GEMV (<= 4 rows) only: the weight [pf_n, pf_k] (row stride pf_ld) of the NEXT GEMV of a
  // decode chain, pulled into the L2 of the XCD that will read it (ATPU_GEMV_PREFETCH)
  const bf16* pf_w = nullptr;
  int pf_ld = 0, pf_k = 0, pf_n = 0;
  int pf_rpb = 16;  // weight rows per workgroup of that next GEMV (32 when it writes RowStats)
};
void gemm_bf16(const GemmArgs& g, hipStream_t stream);
// true when gemm_bf16 runs an [M, N] problem with epilogue `epi` on the <= 4-row GEMV (the
// same test it applies: ATPU_GEMV, ATPU_GEMM_TILE, N % 16, an instantiated epilogue)
bool gemv_selected(int M, int N, int epi);
// split count the library picks for an [M,N,K] problem (1 = no split-K)
int gemm_splitk_splits(int M, int N, int K);
// skinny-M selector (benchmarks): 1 = 64x64 multi-stage dec kernel, 0 = 128x128 split-K
int gemm_dec_mode(int set);
// batch-invariant kernel selection (ATPU_BATCH_INVARIANT): no GEMV / split-K GEMMs, no split
// cross attention / few-row self attention, no few-row LM head or merge; set 0/1, -1 reads
int batch_invariant(int set);
// kernel family override (benchmarks/tests): 0 auto, 64 dec, 128, 256; -1 reads
int gemm_force_tile(int set);
// 256x256 schedule selector (benchmarks): set >= 0 switches; returns the current
int gemm_256_variant(int set);
// persistent 256 x 192 GEMM (qkv_attn.hip; one BERT head's Q|K|V per tile): epi = Bias or
// Bias|InNorm; mode 0 stores C, 1 = timing only (no epilogue, C untouched)
void gemm256h(const GemmArgs& g, int mode, hipStream_t stream);
// BERT QKV projection + self-attention in one persistent kernel (S = 128, head dim 64):
// Bt = the QKV weight with rows in [head][Q 64 | K 64 | V 64] order (bias / colsum likewise),
// g.C = the context [M, N / 3] (row stride g.ldc), lens[M / 128] the sequence lengths
void qkv_attention(const GemmArgs& g, const int32_t* lens, float scale, hipStream_t stream);
int attention_persist_mode(int set);  // packed BERT attention: 1 persistent (default), 0 per-item
int num_cus();                        // CUs a persistent grid is sized for (device count, or the budget below)
int cu_budget(int set);               // >0: size persistent grids for this many CUs (CU-masked streams)
int64_t make_cu_mask_stream(int first_bit, int nbits);  // hipStream_t over CU-mask bits [first, first+n)

// ------------------------------------------------------------ decode (K9-K11)
// One query row per (row, head) against a KV cache. Cross attention (lens set):
// key j of row r lives at k/v + ((r / group) * seq_stride + j) * ldkv + h*64,
// length lens[r / group]; one workgroup serves the `group` rows of a sequence.
// Self attention (step_dev set, group 1): length *step_dev + 1; key j < len-1
// of row r lives in physical row hist[r * hist_stride + j] when hist is given
// (beam backpointers), else in row r. bias_dist (fp32 [H, bias_stride]) adds
// bias_dist[h][len-1-j] (T5 decoder relative position bias).
void decode_attention(const bf16* q, int ldq, const bf16* k, const bf16* v, int ldkv, int seq_stride, int group,
                      const int32_t* lens, const int32_t* step_dev, const int32_t* hist, int hist_stride,
                      const float* bias_dist, int bias_stride, bf16* out, int ldo, int rows, int H, float scale,
                      hipStream_t stream, float* ws = nullptr);
// Cross attention (lens) over a grid of few items splits the keys into 64-key chunks
// (flash decoding) when given a workspace of this many floats (0: no split for the shape).
int decode_attention_splits(int rows, int group, int H, int seq_stride, bool cross);
size_t decode_attention_ws_floats(int rows, int group, int H, int seq_stride, bool cross);
int decode_self_few(int set);  // 1: few-row self attention one wave per (row, head), T <= 192 (default); -1 reads
// one-workgroup state advance of a small beam search (rows x stride x 4 B x (seq ? 2 : 1) <= 64 KiB):
// hist / seq reordered in place by par (as beam_reorder_hist, seq with last = tok, off 1),
// tokens = tok, *step_dev += 1
size_t decode_advance_lds(int rows, int stride, bool seq);
// decoder input of the new tokens, written by decode_advance (table == nullptr: none):
// out[r] = table[tok[r]], or with gamma LN(table[tok[r]] + pos[step + 1 + pos_off])
struct DecEmbed {
  const bf16* table = nullptr;
  int vocab = 0;
  const bf16* pos = nullptr;
  int pos_off = 0, npos = 0;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float eps = 0.f;
  bf16* out = nullptr;
};
void decode_advance(int32_t* hist, int32_t* seq, int rows, int stride, const int32_t* par, const int32_t* tok,
                    int32_t* tokens, int32_t* step_dev, hipStream_t stream, const DecEmbed& em = DecEmbed{},
                    int N = 0);
// dst[r][j] = src[parent[r]][j] (j < t), dst[r][t] = last ? last[r] : parent[r]; t = *step_dev + off
// device beam selection (runtime/summarize.py): item top-K2 over its beams' candidates, hits,
// next running beams -> stage [parents | tokens | score bits] and a host record per item
// device address of a pinned host buffer of `bytes` (checked with hipPointerGetAttributes)
uintptr_t host_device_ptr(uintptr_t host, size_t bytes);
void beam_select(const float* sc, const int32_t* tk, int B, int nb, int K2, int V, int eos, int hit_all, float neg,
                 int32_t* stage, int32_t* rec, hipStream_t stream);
void beam_reorder_hist(const int32_t* src, int32_t* dst, const int32_t* parent, int rows, int stride,
                       const int32_t* step_dev, hipStream_t stream, const int32_t* last = nullptr, int off = 0);
void kv_append(const bf16* src, int lds, int col0, int ncols, bf16* cache, int seq_stride, int ldc,
               const int32_t* step_dev, int rows, hipStream_t stream);
void gather_rows(const bf16* src, bf16* dst, const int32_t* parent, int nrows, int seq_stride, int ldc,
                 const int32_t* step_dev, int slabs, size_t slab_elems, hipStream_t stream);
void beam_topk_rows(const float* logits, int rows, int V, const float* beam_scores, int eos, int mask_eos, int K,
                    float* out_score, int32_t* out_token, hipStream_t stream,
                    const int32_t* bans = nullptr, int nbmax = 0, const int32_t* seq = nullptr, int seq_stride = 0,
                    int cur = 0, int ngram = 0);
// Fused LM head + beam top-k (lm_head.hip): the result of beam_topk_rows over the logits
// (A[M,K] . W[V,K]^T) * rstd(A rows, when rms_eps > 0) + bias (when given), without the
// fp32 logits. topk <= 8. ws: lm_head_ws_bytes(M, V) bytes, 16-B aligned (per-tile partials
// and the per-row ban bitmap).
size_t lm_head_ws_bytes(int M, int V);
int lm_head_stages(int set);  // tile / ring / wave-grid config 0-5 (dev builds; release: 0); -1 reads
void lm_head_topk(const bf16* A, int lda, const bf16* W, int ldw, const float* bias, float rms_eps, int M, int V,
                  int K, int topk, const float* beam_scores, int eos, int mask_eos, const int32_t* bans, int nbmax,
                  const int32_t* seq, int seq_stride, int cur, int ngram, void* ws, float* out_score,
                  int32_t* out_token, hipStream_t stream);

// ------------------------------------------------------------- attention (K4)
// qkv: [B*S, 3*H*D] packed per token as [q(H*D) | k(H*D) | v(H*D)];
// lens: [B] valid key count per row (keys >= len masked); bias: optional
// additive fp32 [H, S, S] (T5 relative-position bias), may be null.
// out: [B*S, H*D]. D must be 64; S <= 512.
void attention_fwd(const bf16* qkv, const int32_t* lens, const float* bias, bf16* out, int B, int S, int H,
                   int D, float scale, hipStream_t stream);

// ------------------------------------------------------- normalisation (K2/K6b)
// out = LN(x (+ res)) * gamma + beta, rows of width N; fp32 statistics.
void layernorm_bf16(const bf16* x, const bf16* res, const float* gamma, const float* beta, bf16* out, int rows,
                    int N, float eps, hipStream_t stream);
// out = x * rsqrt(mean(x^2) + eps) * gamma (T5 RMSNorm, no mean subtraction)
void rmsnorm_bf16(const bf16* x, const float* gamma, bf16* out, int rows, int N, float eps,
                  hipStream_t stream);
// Fused BERT embedding: out[t] = LN(word[ids[t]] + pos[t % S] + type[tt[t]]); ids clamped to
// [0, vocab), type ids to [0, type_vocab).
void embed_layernorm(const int32_t* ids, const int32_t* type_ids, const bf16* word, const bf16* pos,
                     const bf16* type, const float* gamma, const float* beta, bf16* out, int B, int S, int N,
                     int vocab, int type_vocab, float eps, hipStream_t stream);
// LayerNorm folding: fin[m] = (rstd, rstd*mu) of rows of width K from the StatsOut
// partials part[slots][M][2] (sum, sumsq), slots summed in order (deterministic)
void ln_stats_finalize(const float* part, int slots, int M, int K, float eps, float* fin, hipStream_t stream);
// Plain embedding gather (T5 encoder/decoder input): out[t] = table[ids[t]] * scale
// LN(table[ids[r]] + pos[*step + pos_off]) per row (decoder input of a learned-position model at a
// device-side step; the layernorm_bf16 math, bit for bit)
void embed_pos_layernorm(const int32_t* ids, const bf16* table, const bf16* pos, const int32_t* step, int pos_off,
                         int npos, const float* gamma, const float* beta, bf16* out, int rows, int N, int vocab,
                         float eps, hipStream_t stream);
void embed_gather(const int32_t* ids, const bf16* table, bf16* out, int tokens, int N, int vocab,
                  hipStream_t stream);

// ----------------------------------------------------------- tokenizer (K1)
// Deterministic hash word-piece tokenizer (see agent_tpu_amd/tokenizer.py for
// the exact spec and the CPU twin). text: packed UTF-8 bytes; offsets[B+1].
void tokenize_hash(const uint8_t* text, const int32_t* offsets, int32_t* ids, int32_t* lens, int B, int S,
                   int vocab, int max_row_bytes, hipStream_t stream,
                   long long text_bytes);

// ------------------------------------------------ classify head + top-k (K7)
// logits[b, c] = pooled[b] · Wc[c] + bc[c]; probs = softmax(logits);
// writes top-k (descending prob, ties -> lower index) and the full logits.
void classify_head_topk(const bf16* pooled, int ldp, const bf16* Wc, const float* bc, float* logits,
                        int32_t* topk_idx, float* topk_score, int B, int N, int C, int k, hipStream_t stream);

// ---------------------------------------------------- streaming reduce (K12)
// partial[4*blocks] doubles {count, sum, min, max}; finalize on host or via
// reduce_stats_finalize into out[4].
int reduce_stats_blocks(int64_t n);
void reduce_stats_f64(const double* x, int64_t n, double* partial, int blocks, hipStream_t stream);
void reduce_stats_f32(const float* x, int64_t n, double* partial, int blocks, hipStream_t stream);
void reduce_stats_finalize(const double* partial, int blocks, double* out, hipStream_t stream);
// acc[4] (+)= the reduction of a launch's block partials (first: overwrite); streamed reduces
void reduce_stats_accumulate(const double* partial, int blocks, double* acc, bool first, hipStream_t stream);
// K13+K12 over raw CSV records (runtime/risk_stream.cpp): record r is text[offs[r], offs[r+1]);
// field `col` parsed on the device (exact fast path), block partials [blocks][4] like
// reduce_stats_*; records the fast path cannot take are appended (global row row0 + r) to
// fb_rows (first fb_cap of them; *fb_count counts all) for the host to parse.
constexpr int kCsvMaxBlocks = 2048;
int csv_parse_blocks(int64_t n);
void csv_parse_reduce(const uint8_t* text, const uint32_t* offs, int n, int col, int64_t row0, double* partial,
                      int blocks, int* fb_count, int64_t* fb_rows, int fb_cap, hipStream_t stream);

}  // namespace atpu

namespace atpu {
// General strided form (T5 cross/causal attention): q rows b*Sq+t, k/v rows
// b*Skv+t; head h at column h*D of each row. ``bias`` is a dense fp32 [H, Sq, Skv]
// additive bias; ``bias_dist`` (exclusive with it) a bias by key-query distance,
// fp32 [H, Sq+Skv-1] with entry k - q + Sq - 1 (T5's relative position bias).
void attention_fwd_strided(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv, bf16* out,
                           int ldo, const int32_t* lens, const float* bias, int B, int Sq, int Skv, int H, int D,
                           float scale, int causal, hipStream_t stream, const float* bias_dist = nullptr);
// 1 = long-sequence encoder attention on the double-buffered flash kernel (default), 0 = per-chunk kernel
int attention_flash_mode(int set);
}  // namespace atpu
