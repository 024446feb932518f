// pybind11 module `_atpu`: the Python face of the native MI355X runtime.
//
// Device buffers are owned by PyTorch (caching allocator); kernels receive raw
// device pointers and the hipStream_t of torch's current stream as integers,
// so every launch is graph-capturable through torch.cuda.CUDAGraph (hipGraph).
// Python-side wrappers with shape/dtype checks live in agent_tpu_amd/ops/.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "atpu/comm.h"
#include "atpu/common.h"
#include "atpu/csv.h"
#include "atpu/kernels.h"
#include "atpu/l2_prefetch.h"
#include "atpu/risk_stream.h"
#include "atpu/runtime.h"

namespace py = pybind11;
using namespace atpu;

namespace {

template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::str decode(const std::string& s) {
  PyObject* o = PyUnicode_DecodeUTF8(s.data(), static_cast<Py_ssize_t>(s.size()), "strict");
  if (!o) throw py::error_already_set();
  return py::reinterpret_steal<py::str>(o);
}

py::dict make_row(const std::vector<std::string>& header, const std::vector<std::string>& row) {
  // csv.DictReader semantics: zip(fieldnames, row); extra -> key None (list);
  // missing -> value None.
  py::dict d;
  const size_t nf = header.size(), nr = row.size();
  for (size_t i = 0; i < std::min(nf, nr); ++i)
    d[py::str(header[i])] = decode(row[i]);
  if (nr > nf) {
    py::list extra;
    for (size_t i = nf; i < nr; ++i) extra.append(decode(row[i]));
    d[py::none()] = extra;
  } else {
    for (size_t i = nr; i < nf; ++i) d[py::str(header[i])] = py::none();
  }
  return d;
}

}  // namespace

PYBIND11_MODULE(_atpu, m) {
  m.doc() = "agent_tpu_amd native runtime: gfx950 HIP kernels + C++ host runtime";
  m.attr("ARCH") = "gfx950";

  // ------------------------------------------------------------- kernels
  m.def(
      "gemm",
      [](uintptr_t A, int lda, uintptr_t Bt, int ldb, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R, int ldr, int M,
         int N, int K, int epi, uintptr_t stream, int splits, uintptr_t ws, float rms_eps, uintptr_t kv_cache,
         int kv_ld, int kv_T, int kv_col0, uintptr_t kv_step, uintptr_t colsum, uintptr_t in_part,
         uintptr_t res_part, uintptr_t gamma, uintptr_t part_out, uintptr_t pf_w, int pf_ld, int pf_k, int pf_n,
         int pf_rpb) {
        GemmArgs g;
        g.A = P<const bf16>(A); g.lda = lda; g.Bt = P<const bf16>(Bt); g.ldb = ldb; g.C = P<bf16>(C); g.ldc = ldc;
        g.bias = P<const float>(bias); g.R = P<const bf16>(R); g.ldr = ldr; g.M = M; g.N = N; g.K = K; g.epi = epi;
        g.splits = splits; g.ws = P<float>(ws); g.rms_eps = rms_eps;
        g.kv_cache = P<bf16>(kv_cache); g.kv_ld = kv_ld; g.kv_T = kv_T; g.kv_col0 = kv_col0;
        g.kv_step = P<const int32_t>(kv_step);
        g.colsum = P<const float>(colsum); g.in_part = P<const float>(in_part);
        g.res_part = P<const float>(res_part); g.gamma = P<const float>(gamma); g.part_out = P<float>(part_out);
        g.pf_w = P<const bf16>(pf_w); g.pf_ld = pf_ld; g.pf_k = pf_k; g.pf_n = pf_n; g.pf_rpb = pf_rpb;
        gemm_bf16(g, S(stream));
      },
      "bf16 MFMA GEMM C = epi(A @ Bt^T)", py::arg("A"), py::arg("lda"), py::arg("Bt"), py::arg("ldb"), py::arg("C"),
      py::arg("ldc"), py::arg("bias"), py::arg("R"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("epi"), py::arg("stream"), py::arg("splits") = 1, py::arg("ws") = 0, py::arg("rms_eps") = 0.f,
      py::arg("kv_cache") = 0, py::arg("kv_ld") = 0, py::arg("kv_T") = 0, py::arg("kv_col0") = 0,
      py::arg("kv_step") = 0, py::arg("colsum") = 0, py::arg("in_part") = 0, py::arg("res_part") = 0,
      py::arg("gamma") = 0, py::arg("part_out") = 0, py::arg("pf_w") = 0, py::arg("pf_ld") = 0, py::arg("pf_k") = 0,
      py::arg("pf_n") = 0, py::arg("pf_rpb") = 16);
  m.def(
      "gemm_ln",
      [](uintptr_t A, int lda, uintptr_t Bt, int ldb, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R, int ldr, int M,
         int N, int K, int epi, uintptr_t in_fin, uintptr_t colsum, uintptr_t res_fin, uintptr_t gamma,
         uintptr_t part_out, uintptr_t stream) {
        GemmArgs g;
        g.A = P<const bf16>(A); g.lda = lda; g.Bt = P<const bf16>(Bt); g.ldb = ldb; g.C = P<bf16>(C); g.ldc = ldc;
        g.bias = P<const float>(bias); g.R = P<const bf16>(R); g.ldr = ldr; g.M = M; g.N = N; g.K = K; g.epi = epi;
        g.in_fin = P<const float>(in_fin); g.colsum = P<const float>(colsum); g.res_fin = P<const float>(res_fin);
        g.gamma = P<const float>(gamma); g.part_out = P<float>(part_out);
        gemm_bf16(g, S(stream));
      },
      "bf16 MFMA GEMM with LayerNorm folding epilogues (InNorm / ResNorm / StatsOut)", py::arg("A"), py::arg("lda"),
      py::arg("Bt"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("bias"), py::arg("R"), py::arg("ldr"),
      py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("in_fin"), py::arg("colsum"),
      py::arg("res_fin"), py::arg("gamma"), py::arg("part_out"), py::arg("stream"));
  m.def(
      "gemm256h",
      [](uintptr_t A, int lda, uintptr_t Bt, int ldb, uintptr_t C, int ldc, uintptr_t bias, int M, int N, int K,
         int epi, uintptr_t in_fin, uintptr_t colsum, int mode, uintptr_t stream) {
        GemmArgs g;
        g.A = P<const bf16>(A); g.lda = lda; g.Bt = P<const bf16>(Bt); g.ldb = ldb; g.C = P<bf16>(C); g.ldc = ldc;
        g.bias = P<const float>(bias); g.M = M; g.N = N; g.K = K; g.epi = epi;
        g.in_fin = P<const float>(in_fin); g.colsum = P<const float>(colsum);
        gemm256h(g, mode, S(stream));
      },
      "persistent 256x192 bf16 GEMM (one head's Q|K|V per tile); mode 1 = timing only", py::arg("A"),
      py::arg("lda"), py::arg("Bt"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("bias"), py::arg("M"),
      py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("in_fin"), py::arg("colsum"), py::arg("mode"),
      py::arg("stream"));
  m.def(
      "qkv_attention",
      [](uintptr_t A, int lda, uintptr_t Bt, int ldb, uintptr_t ctx, int ldo, uintptr_t bias, int M, int N, int K,
         int epi, uintptr_t in_fin, uintptr_t colsum, uintptr_t lens, float scale, uintptr_t stream) {
        GemmArgs g;
        g.A = P<const bf16>(A); g.lda = lda; g.Bt = P<const bf16>(Bt); g.ldb = ldb; g.C = P<bf16>(ctx); g.ldc = ldo;
        g.bias = P<const float>(bias); g.M = M; g.N = N; g.K = K; g.epi = epi;
        g.in_fin = P<const float>(in_fin); g.colsum = P<const float>(colsum);
        qkv_attention(g, P<const int32_t>(lens), scale, S(stream));
      },
      "BERT QKV projection + self-attention (S = 128) in one persistent kernel; Bt rows per head [Q|K|V]",
      py::arg("A"), py::arg("lda"), py::arg("Bt"), py::arg("ldb"), py::arg("ctx"), py::arg("ldo"), py::arg("bias"),
      py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("in_fin"), py::arg("colsum"),
      py::arg("lens"), py::arg("scale"), py::arg("stream"));
  m.def(
      "ln_stats_finalize",
      [](uintptr_t part, int slots, int M, int K, float eps, uintptr_t fin, uintptr_t stream) {
        ln_stats_finalize(P<const float>(part), slots, M, K, eps, P<float>(fin), S(stream));
      },
      "fin[m] = (rstd, rstd*mu) from StatsOut partials [slots][M][2]", py::arg("part"), py::arg("slots"),
      py::arg("M"), py::arg("K"), py::arg("eps"), py::arg("fin"), py::arg("stream"));
  m.def("trace_enabled", &trace_enabled, "roctx tracing active (MI355X_TRACE=1 and roctx loadable)");
  m.def("trace_push", [](const std::string& n) { trace_push(n.c_str()); });
  m.def("trace_pop", &trace_pop);
  m.def("trace_mark", [](const std::string& n) { trace_mark(n.c_str()); });
  m.def("gemm_splitk_splits", &gemm_splitk_splits, "split-K factor chosen for an [M,N,K] GEMM");
  m.def(
      "rand_fill",
      [](uintptr_t dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0, float scale1,
         uintptr_t stream) { rand_fill(P<void>(dst), n, f32, seed, sid, scale0, n0, scale1, S(stream)); },
      py::arg("dst"), py::arg("n"), py::arg("f32"), py::arg("seed"), py::arg("sid"), py::arg("scale0"), py::arg("n0"),
      py::arg("scale1"), py::arg("stream"), "seeded random init of a device tensor (atpu/rand.h)");
  m.def(
      "rand_fill_host",
      [](uintptr_t dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0, float scale1,
         int threads) {
        py::gil_scoped_release nogil;
        rand_fill_host(P<void>(dst), n, f32, seed, sid, scale0, n0, scale1, threads);
      },
      py::arg("dst"), py::arg("n"), py::arg("f32"), py::arg("seed"), py::arg("sid"), py::arg("scale0"), py::arg("n0"),
      py::arg("scale1"), py::arg("threads") = 8, "CPU twin of rand_fill (bit-identical values)");
  m.def("gemv_selected", &gemv_selected, py::arg("M"), py::arg("N"), py::arg("epi"),
        "true when gemm_bf16 runs this [M, N] problem / epilogue on the <= 4-row GEMV");
  m.def("batch_invariant", &batch_invariant, py::arg("set") = -1,
        "batch-invariant kernel selection (ATPU_BATCH_INVARIANT): 1 on, 0 off, -1 reads; returns the current");
  m.def("gemm_force_tile", &gemm_force_tile, py::arg("set") = -1, "GEMM kernel family override: 0 auto, 64, 128, 256");
  m.def("gemm_dec_mode", &gemm_dec_mode, py::arg("set") = -1,
        "skinny-M GEMM path: 1 = 64x64 multi-stage dec kernel, 0 = 128x128 split-K; returns the current");
  m.def("gemm_256_variant", &gemm_256_variant, py::arg("set") = -1,
        "256x256 GEMM schedule: 1 = 256p ping-pong, 3 = 256l persistent full-line epilogue, "
        "4 = 256n full-line + nt stores (default); set >= 0 switches, returns the current");
  m.def("cu_budget", &cu_budget, py::arg("set") = -1,
        "get/set the CU count persistent grids are sized for (0 = the device's; set it to the CU share of "
        "CU-masked streams)");
  m.def("num_cus", &num_cus, "CUs persistent grids are sized for");
  m.def("make_cu_mask_stream", &make_cu_mask_stream, py::arg("first_bit"), py::arg("nbits"),
        "create a HIP stream restricted to CU-mask bits [first_bit, first_bit+nbits) (bit i -> XCD i % 8); "
        "returns the hipStream_t as an int (wrap with torch.cuda.ExternalStream)");
  m.def("attention_persist_mode", &attention_persist_mode, py::arg("set") = -1,
        "packed BERT attention: 1 = persistent prefetching kernel (default), 0 = one item per workgroup");
  m.attr("EPI_BIAS") = static_cast<int>(kEpiBias);
  m.attr("EPI_GELU") = static_cast<int>(kEpiGelu);
  m.attr("EPI_TANH") = static_cast<int>(kEpiTanh);
  m.attr("EPI_RESIDUAL") = static_cast<int>(kEpiResidual);
  m.attr("EPI_RELU") = static_cast<int>(kEpiRelu);
  m.attr("EPI_OUT_F32") = static_cast<int>(kEpiOutF32);
  m.def("decode_attention", [](uintptr_t q, int ldq, uintptr_t k, uintptr_t v, int ldkv, int seq_stride, int group,
                               uintptr_t lens, uintptr_t step_dev, uintptr_t hist, int hist_stride, uintptr_t bias,
                               int bias_stride, uintptr_t out, int ldo, int rows, int H, float scale, uintptr_t stream,
                               uintptr_t ws) {
    decode_attention(P<const bf16>(q), ldq, P<const bf16>(k), P<const bf16>(v), ldkv, seq_stride, group,
                     P<const int32_t>(lens), P<const int32_t>(step_dev), P<const int32_t>(hist), hist_stride,
                     P<const float>(bias), bias_stride, P<bf16>(out), ldo, rows, H, scale, S(stream), P<float>(ws));
  }, py::arg("q"), py::arg("ldq"), py::arg("k"), py::arg("v"), py::arg("ldkv"), py::arg("seq_stride"), py::arg("group"),
     py::arg("lens"), py::arg("step_dev"), py::arg("hist"), py::arg("hist_stride"), py::arg("bias"), py::arg("bias_stride"),
     py::arg("out"), py::arg("ldo"), py::arg("rows"), py::arg("H"), py::arg("scale"), py::arg("stream"), py::arg("ws") = 0);
  m.def("decode_attention_ws_floats", [](int rows, int group, int H, int seq_stride, bool cross) {
    return decode_attention_ws_floats(rows, group, H, seq_stride, cross);
  });
  m.def("host_device_ptr", &host_device_ptr, "device address of a pinned host buffer (checked)", py::arg("host"),
        py::arg("bytes"));
  m.def("beam_select", [](uintptr_t sc, uintptr_t tk, int B, int nb, int K2, int V, int eos, int hit_all, float neg,
                          uintptr_t stage, uintptr_t rec, uintptr_t stream) {
    beam_select(P<const float>(sc), P<const int32_t>(tk), B, nb, K2, V, eos, hit_all, neg, P<int32_t>(stage),
                P<int32_t>(rec), S(stream));
  });
  m.def(
      "decode_advance",
      [](uintptr_t hist, uintptr_t seq, int rows, int stride, uintptr_t par, uintptr_t tok, uintptr_t tokens,
         uintptr_t step_dev, uintptr_t stream, uintptr_t emb, int vocab, int N, uintptr_t pos, int pos_off, int npos,
         uintptr_t gamma, uintptr_t beta, float eps, uintptr_t out) {
        DecEmbed em;
        em.table = P<const bf16>(emb);
        em.vocab = vocab;
        em.pos = P<const bf16>(pos);
        em.pos_off = pos_off;
        em.npos = npos;
        em.gamma = P<const float>(gamma);
        em.beta = P<const float>(beta);
        em.eps = eps;
        em.out = P<bf16>(out);
        decode_advance(P<int32_t>(hist), P<int32_t>(seq), rows, stride, P<const int32_t>(par), P<const int32_t>(tok),
                       P<int32_t>(tokens), P<int32_t>(step_dev), S(stream), em, N);
      },
      "one-workgroup beam state advance: hist/seq reordered in place, tokens = tok, step += 1 (emb: the new "
      "tokens' decoder input into out, LayerNorm with gamma)",
      py::arg("hist"), py::arg("seq"), py::arg("rows"), py::arg("stride"), py::arg("par"), py::arg("tok"),
      py::arg("tokens"), py::arg("step"), py::arg("stream"), py::arg("emb") = 0, py::arg("vocab") = 0,
      py::arg("N") = 0, py::arg("pos") = 0, py::arg("pos_off") = 0, py::arg("npos") = 0, py::arg("gamma") = 0,
      py::arg("beta") = 0, py::arg("eps") = 0.f, py::arg("out") = 0);
  m.def("decode_advance_lds", &decode_advance_lds, py::arg("rows"), py::arg("stride"), py::arg("seq"));
  m.def(
      "beam_reorder_hist",
      [](uintptr_t src, uintptr_t dst, uintptr_t parent, int rows, int stride, uintptr_t step_dev, uintptr_t stream,
         uintptr_t last, int off) {
        beam_reorder_hist(P<const int32_t>(src), P<int32_t>(dst), P<const int32_t>(parent), rows, stride,
                          P<const int32_t>(step_dev), S(stream), P<const int32_t>(last), off);
      },
      py::arg("src"), py::arg("dst"), py::arg("parent"), py::arg("rows"), py::arg("stride"), py::arg("step_dev"),
      py::arg("stream"), py::arg("last") = 0, py::arg("off") = 0);
  m.def("kv_append", [](uintptr_t src, int lds, int col0, int ncols, uintptr_t cache, int seq_stride, int ldc,
                        uintptr_t step_dev, int rows, uintptr_t stream) {
    kv_append(P<const bf16>(src), lds, col0, ncols, P<bf16>(cache), seq_stride, ldc, P<const int32_t>(step_dev), rows,
              S(stream));
  });
  m.def("gather_rows", [](uintptr_t src, uintptr_t dst, uintptr_t parent, int nrows, int seq_stride, int ldc,
                          uintptr_t step_dev, int slabs, size_t slab_elems, uintptr_t stream) {
    gather_rows(P<const bf16>(src), P<bf16>(dst), P<const int32_t>(parent), nrows, seq_stride, ldc,
                P<const int32_t>(step_dev), slabs, slab_elems, S(stream));
  });
  m.def(
      "beam_topk_rows",
      [](uintptr_t logits, int rows, int V, uintptr_t beam_scores, int eos, int mask_eos, int K, uintptr_t out_score,
         uintptr_t out_token, uintptr_t stream, uintptr_t bans, int nbmax, uintptr_t seq, int seq_stride, int cur,
         int ngram) {
        beam_topk_rows(P<const float>(logits), rows, V, P<const float>(beam_scores), eos, mask_eos, K,
                       P<float>(out_score), P<int32_t>(out_token), S(stream), P<const int32_t>(bans), nbmax,
                       P<const int32_t>(seq), seq_stride, cur, ngram);
      },
      py::arg("logits"), py::arg("rows"), py::arg("V"), py::arg("beam_scores"), py::arg("eos"), py::arg("mask_eos"),
      py::arg("K"), py::arg("out_score"), py::arg("out_token"), py::arg("stream"), py::arg("bans") = 0,
      py::arg("nbmax") = 0, py::arg("seq") = 0, py::arg("seq_stride") = 0, py::arg("cur") = 0, py::arg("ngram") = 0);
  m.def("lm_head_ws_bytes", &lm_head_ws_bytes);
  m.def("lm_head_stages", &lm_head_stages, py::arg("set") = -1);
  m.def("decode_self_few", &decode_self_few, py::arg("set") = -1);
  m.def(
      "lm_head_topk",
      [](uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t bias, float rms_eps, int M, int V, int K, int topk,
         uintptr_t beam_scores, int eos, int mask_eos, uintptr_t bans, int nbmax, uintptr_t seq, int seq_stride,
         int cur, int ngram, uintptr_t ws, uintptr_t out_score, uintptr_t out_token, uintptr_t stream) {
        lm_head_topk(P<const bf16>(A), lda, P<const bf16>(W), ldw, P<const float>(bias), rms_eps, M, V, K, topk,
                     P<const float>(beam_scores), eos, mask_eos, P<const int32_t>(bans), nbmax, P<const int32_t>(seq),
                     seq_stride, cur, ngram, reinterpret_cast<void*>(ws), P<float>(out_score), P<int32_t>(out_token),
                     S(stream));
      });

  m.def("attention", [](uintptr_t qkv, uintptr_t lens, uintptr_t bias, uintptr_t out, int B, int Sq, int H, int D,
                        float scale, uintptr_t stream) {
    attention_fwd(P<const bf16>(qkv), P<const int32_t>(lens), P<const float>(bias), P<bf16>(out), B, Sq, H, D, scale,
                  S(stream));
  });
  m.def("attention_strided", [](uintptr_t q, int ldq, uintptr_t k, int ldk, uintptr_t v, int ldv, uintptr_t out,
                                int ldo, uintptr_t lens, uintptr_t bias, int B, int Sq, int Skv, int H, int D,
                                float scale, int causal, uintptr_t stream, uintptr_t bias_dist) {
    attention_fwd_strided(P<const bf16>(q), ldq, P<const bf16>(k), ldk, P<const bf16>(v), ldv, P<bf16>(out), ldo,
                          P<const int32_t>(lens), P<const float>(bias), B, Sq, Skv, H, D, scale, causal, S(stream),
                          P<const float>(bias_dist));
  }, py::arg("q"), py::arg("ldq"), py::arg("k"), py::arg("ldk"), py::arg("v"), py::arg("ldv"), py::arg("out"),
     py::arg("ldo"), py::arg("lens"), py::arg("bias"), py::arg("B"), py::arg("Sq"), py::arg("Skv"), py::arg("H"),
     py::arg("D"), py::arg("scale"), py::arg("causal"), py::arg("stream"), py::arg("bias_dist") = 0);
  m.def("attention_flash_mode", &attention_flash_mode, py::arg("set") = -1,
        "long-sequence encoder attention: 1 = double-buffered flash kernel (default), 0 = per-chunk kernel");
  m.def("layernorm", [](uintptr_t x, uintptr_t res, uintptr_t g, uintptr_t b, uintptr_t out, int rows, int N,
                        float eps, uintptr_t stream) {
    layernorm_bf16(P<const bf16>(x), P<const bf16>(res), P<const float>(g), P<const float>(b), P<bf16>(out), rows, N,
                   eps, S(stream));
  });
  m.def("rmsnorm", [](uintptr_t x, uintptr_t g, uintptr_t out, int rows, int N, float eps, uintptr_t stream) {
    rmsnorm_bf16(P<const bf16>(x), P<const float>(g), P<bf16>(out), rows, N, eps, S(stream));
  });
  m.def("embed_layernorm", [](uintptr_t ids, uintptr_t tt, uintptr_t word, uintptr_t pos, uintptr_t type, uintptr_t g,
                              uintptr_t b, uintptr_t out, int B, int Sq, int N, int vocab, int type_vocab, float eps,
                              uintptr_t stream) {
    embed_layernorm(P<const int32_t>(ids), P<const int32_t>(tt), P<const bf16>(word), P<const bf16>(pos),
                    P<const bf16>(type), P<const float>(g), P<const float>(b), P<bf16>(out), B, Sq, N, vocab,
                    type_vocab, eps, S(stream));
  });
  m.def("embed_gather", [](uintptr_t ids, uintptr_t table, uintptr_t out, int tokens, int N, int vocab,
                           uintptr_t stream) {
    embed_gather(P<const int32_t>(ids), P<const bf16>(table), P<bf16>(out), tokens, N, vocab, S(stream));
  });
  m.def("embed_pos_layernorm", [](uintptr_t ids, uintptr_t table, uintptr_t pos, uintptr_t step, int pos_off, int npos,
                                  uintptr_t gamma, uintptr_t beta, uintptr_t out, int rows, int N, int vocab, float eps,
                                  uintptr_t stream) {
    embed_pos_layernorm(P<const int32_t>(ids), P<const bf16>(table), P<const bf16>(pos), P<const int32_t>(step),
                        pos_off, npos, P<const float>(gamma), P<const float>(beta), P<bf16>(out), rows, N, vocab, eps,
                        S(stream));
  });
  m.def("tokenize", [](uintptr_t text, uintptr_t offsets, uintptr_t ids, uintptr_t lens, int B, int Sq, int vocab,
                       int max_row_bytes, uintptr_t stream, long long text_bytes) {
    tokenize_hash(P<const uint8_t>(text), P<const int32_t>(offsets), P<int32_t>(ids), P<int32_t>(lens), B, Sq, vocab,
                  max_row_bytes, S(stream), text_bytes);
  });
  m.def("head_topk", [](uintptr_t pooled, int ldp, uintptr_t Wc, uintptr_t bc, uintptr_t logits, uintptr_t idx,
                        uintptr_t score, int B, int N, int C, int k, uintptr_t stream) {
    classify_head_topk(P<const bf16>(pooled), ldp, P<const bf16>(Wc), P<const float>(bc), P<float>(logits),
                       P<int32_t>(idx), P<float>(score), B, N, C, k, S(stream));
  });
  m.def("reduce_stats_blocks", &reduce_stats_blocks);
  m.def("reduce_stats_f64", [](uintptr_t x, int64_t n, uintptr_t partial, int blocks, uintptr_t stream) {
    reduce_stats_f64(P<const double>(x), n, P<double>(partial), blocks, S(stream));
  });
  m.def("reduce_stats_f32", [](uintptr_t x, int64_t n, uintptr_t partial, int blocks, uintptr_t stream) {
    reduce_stats_f32(P<const float>(x), n, P<double>(partial), blocks, S(stream));
  });
  m.def("reduce_stats_finalize", [](uintptr_t partial, int blocks, uintptr_t out, uintptr_t stream) {
    reduce_stats_finalize(P<const double>(partial), blocks, P<double>(out), S(stream));
  });

  // ------------------------------------------------------- host runtime
  m.def(
      "tokenize_host",
      [](py::array_t<uint8_t, py::array::c_style> text, py::array_t<int32_t, py::array::c_style> offsets, int Sq,
         int vocab, int max_row_bytes) {
        const int B = static_cast<int>(offsets.size()) - 1;
        ATPU_CHECK(B >= 0, "tokenize_host: offsets must have B+1 entries");
        py::array_t<int32_t> ids({B, Sq});
        py::array_t<int32_t> lens(B);
        {
          py::gil_scoped_release nogil;
          tokenize_host(text.data(), offsets.data(), ids.mutable_data(), lens.mutable_data(), B, Sq, vocab,
                        max_row_bytes);
        }
        return py::make_tuple(ids, lens);
      },
      py::arg("text"), py::arg("offsets"), py::arg("seq_len"), py::arg("vocab"), py::arg("max_row_bytes"));
  m.def(
      "word_maps_host",
      [](py::array_t<uint8_t, py::array::c_style> text, py::array_t<int64_t, py::array::c_style> offsets, int vocab,
         int cap) {
        const int B = static_cast<int>(offsets.size()) - 1;
        ATPU_CHECK(B >= 0, "word_maps_host: offsets must have B+1 entries");
        std::vector<int32_t> ids;
        std::vector<int64_t> word_of, doc_off;
        {
          py::gil_scoped_release nogil;
          word_maps_host(text.data(), offsets.data(), B, vocab, cap, ids, word_of, doc_off);
        }
        return py::make_tuple(py::array_t<int32_t>(ids.size(), ids.data()),
                              py::array_t<int64_t>(word_of.size(), word_of.data()),
                              py::array_t<int64_t>(doc_off.size(), doc_off.data()));
      },
      "per document (words joined by single spaces): distinct token ids ascending, first word index of each, "
      "document offsets [B+1]",
      py::arg("text"), py::arg("offsets"), py::arg("vocab"), py::arg("cap"));

  m.def("risk_stats_list",
        [](py::list values, int mode, py::object field, bool keep) -> py::object {
          RiskStats st{};
          std::vector<double> vals;
          if (!risk_stats_pylist(values.ptr(), mode, field.ptr(), &st, keep ? &vals : nullptr))
            throw py::error_already_set();
          py::object arr = py::none();
          if (keep) {
            py::array_t<double> a(static_cast<py::ssize_t>(vals.size()));
            std::memcpy(a.mutable_data(), vals.data(), vals.size() * sizeof(double));
            arr = a;
          }
          return py::make_tuple(st.count, st.sum, st.min, st.max, arr);
        },
        "risk_accumulate over a JSON list: (count, sum, min, max, values f64 | None); mode 0 values, 1 items[field]",
        py::arg("values"), py::arg("mode") = 0, py::arg("field") = py::str("risk"), py::arg("keep") = false);
  m.def("topk_json",
        [](int64_t start_row, py::array_t<int32_t, py::array::c_style | py::array::forcecast> idx,
           py::array_t<float, py::array::c_style | py::array::forcecast> score, int mode) {
          if (idx.ndim() != 2 || score.ndim() != 2 || idx.shape(0) != score.shape(0) || idx.shape(1) != score.shape(1))
            throw std::invalid_argument("topk_json: idx and score must be [n, k]");
          std::string s;
          const int32_t* ip = idx.data();
          const float* sp = score.data();
          const int64_t n = idx.shape(0);
          const int k = static_cast<int>(idx.shape(1));
          {
            py::gil_scoped_release nogil;
            s = topk_json(start_row, ip, sp, n, k, mode);
          }
          return py::bytes(s);
        },
        "top-k [n,k] -> JSON bytes (0 rows, 1 index columns, 2 score columns)", py::arg("start_row"),
        py::arg("idx"), py::arg("score"), py::arg("mode") = 0);
  m.def("device_query", [](int mem_of) {
    if (mem_of < 0) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      mem_of = cur;
    }
    py::list out;
    for (const auto& d : device_query(mem_of)) {
      py::dict x;
      x["index"] = d.index; x["name"] = d.name; x["arch"] = d.arch; x["total_memory_bytes"] = d.total_bytes;
      x["free_memory_bytes"] = d.free_bytes; x["compute_units"] = d.cus; x["clock_khz"] = d.clock_khz;
      x["free_memory_known"] = d.index == mem_of;
      out.append(x);
    }
    return out;
  }, "every visible device; free HBM only for device mem_of (-1: current)", py::arg("mem_of") = -1);

  py::class_<CsvTable, std::shared_ptr<CsvTable>>(m, "CsvTable")
      .def(py::init([](const std::string& path) {
             py::gil_scoped_release nogil;
             return std::make_shared<CsvTable>(path);
           }),
           py::arg("path"))
      .def_property_readonly("path", &CsvTable::path)
      .def_property_readonly("num_rows", &CsvTable::num_rows)
      .def_property_readonly("file_size", &CsvTable::file_size)
      .def_property_readonly("mtime_ns", &CsvTable::mtime_ns)
      .def_property_readonly("header",
                             [](const CsvTable& t) {
                               py::list h;
                               for (const auto& s : t.header()) h.append(decode(s));
                               return h;
                             })
      .def_property_readonly("index_from_cache", &CsvTable::index_from_cache)
      .def("column_index", &CsvTable::column_index)
      .def("parse_double", [](const CsvTable& t, size_t row, int col) { return t.parse_double(row, col); },
           "field col of data record row as a float (extract_doubles' parse; ValueError on a bad value)")
      .def("release_pages", &CsvTable::release_pages)
      .def("row",
           [](const CsvTable& t, size_t i) {
             std::vector<std::string> f;
             t.parse_row(i, f);
             py::list out;
             for (const auto& s : f) out.append(decode(s));
             return out;
           })
      .def("dict_rows",
           [](const CsvTable& t, size_t start, size_t n) {
             py::list out;
             if (start >= t.num_rows()) return out;
             n = std::min(n, t.num_rows() - start);
             std::vector<std::string> f;
             for (size_t r = start; r < start + n; ++r) {
               t.parse_row(r, f);
               out.append(make_row(t.header(), f));
             }
             return out;
           })
      .def("float_column",
           [](const CsvTable& t, size_t start, size_t n, int col, int threads) {
             if (start > t.num_rows()) start = t.num_rows();
             n = std::min(n, t.num_rows() - start);
             py::array_t<double> out(n);
             {
               py::gil_scoped_release nogil;
               t.extract_doubles(start, n, col, out.mutable_data(), threads);
             }
             return out;
           },
           py::arg("start"), py::arg("n"), py::arg("col"), py::arg("threads") = 8)
      .def("extract_doubles_into",
           [](const CsvTable& t, size_t start, size_t n, int col, py::array_t<double, py::array::c_style> out,
              int threads) {
             if (start > t.num_rows()) start = t.num_rows();
             n = std::min(n, t.num_rows() - start);
             if (static_cast<size_t>(out.size()) < n) throw std::invalid_argument("extract_doubles_into: out too small");
             double* dst = out.mutable_data();
             {
               py::gil_scoped_release nogil;
               t.extract_doubles(start, n, col, dst, threads);
               if (n) t.release_pages(t.row_begin(start), t.row_end(start + n - 1));  // streamed: drop consumed pages
             }
             return n;
           },
           py::arg("start"), py::arg("n"), py::arg("col"), py::arg("out"), py::arg("threads") = 8,
           "float_column into a caller-owned buffer (chunked streaming without per-chunk allocations)")
      .def("extract_column",
           [](const CsvTable& t, size_t start, size_t n, int col, size_t max_bytes, int threads) {
             if (start > t.num_rows()) start = t.num_rows();
             n = std::min(n, t.num_rows() - start);
             py::array_t<int32_t> offs(n + 1);
             // capacity bound: each value is at most max_bytes
             std::vector<uint8_t> buf(std::max<size_t>(1, n * max_bytes));
             int64_t bytes;
             {
               py::gil_scoped_release nogil;
               bytes = t.extract_column(start, n, col, buf.data(), buf.size(), offs.mutable_data(), max_bytes, threads);
             }
             py::array_t<uint8_t> text(bytes);
             std::memcpy(text.mutable_data(), buf.data(), bytes);
             return py::make_tuple(text, offs);
           },
           py::arg("start"), py::arg("n"), py::arg("col"), py::arg("max_bytes"), py::arg("threads") = 8);

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](int world, int rank, py::bytes uid, int device) {
             std::string u = uid;
             py::gil_scoped_release nogil;  // ncclCommInitRank blocks until every rank joined
             return std::make_shared<RcclComm>(world, rank, u, device);
           }),
           py::arg("world"), py::arg("rank"), py::arg("uid"), py::arg("device"))
      .def_static("unique_id", [] { return py::bytes(RcclComm::unique_id()); })
      .def_static("init_all", &RcclComm::init_all, py::arg("devices"))
      .def("broadcast",
           [](RcclComm& c, uintptr_t buf, size_t count, int dtype, int root, uintptr_t stream) {
             py::gil_scoped_release nogil;
             c.broadcast(P<void>(buf), count, dtype, root, S(stream));
           })
      .def("all_gather",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t stream) {
             py::gil_scoped_release nogil;
             c.all_gather(P<const void>(send), P<void>(recv), count, dtype, S(stream));
           })
      .def("all_reduce",
           [](RcclComm& c, uintptr_t buf, size_t count, int dtype, int op, uintptr_t stream) {
             py::gil_scoped_release nogil;
             c.all_reduce(P<void>(buf), count, dtype, op, S(stream));
           })
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device);
  m.def("rccl_group_start", &rccl_group_start);
  m.def("rccl_group_end", &rccl_group_end);
  m.def("rccl_version", &rccl_version);

  py::class_<RiskStream>(m, "RiskStream")
      .def(py::init<size_t, size_t, int>(), py::arg("slot_bytes"), py::arg("slot_rows"), py::arg("fallback_cap"))
      .def("run",
           [](RiskStream& r, std::shared_ptr<CsvTable> t, size_t start, size_t n, int col, uintptr_t copy_stream,
              uintptr_t compute_stream, int threads) {
             RiskStream::Result res;
             {
               py::gil_scoped_release nogil;
               res = r.run(*t, start, n, col, S(copy_stream), S(compute_stream), threads);
             }
             py::dict d;
             d["count"] = res.count;
             d["sum"] = res.sum;
             d["min"] = res.min;
             d["max"] = res.max;
             d["host_rows"] = py::array_t<int64_t>(res.host_rows.size(), res.host_rows.data());
             d["fallback_total"] = res.fallback_total;
             d["overflow"] = res.overflow;
             d["chunks"] = res.chunks;
             d["bytes"] = res.bytes;
             return d;
           })
      .def_property_readonly("slot_bytes", &RiskStream::slot_bytes)
      .def_property_readonly("slot_rows", &RiskStream::slot_rows);

  py::class_<HostStager>(m, "HostStager")
      .def(py::init<int, size_t, int>(), py::arg("slots"), py::arg("text_capacity"), py::arg("max_rows"))
      .def("submit",
           [](HostStager& s, int slot, std::shared_ptr<CsvTable> t, size_t start, size_t n, int col, size_t max_bytes,
              int threads) { s.submit(slot, t.get(), start, n, col, max_bytes, threads); },
           py::keep_alive<1, 3>())
      .def("upload",
           [](HostStager& s, int slot, uintptr_t dev_text, size_t cap, uintptr_t dev_off, uintptr_t copy_stream,
              uintptr_t compute_stream) {
             py::gil_scoped_release nogil;
             return s.upload(slot, P<void>(dev_text), cap, P<void>(dev_off), S(copy_stream), S(compute_stream));
           })
      .def("wait",
           [](HostStager& s, int slot) {
             py::gil_scoped_release nogil;
             return s.wait(slot);
           })
      .def("release", [](HostStager& s, int slot, uintptr_t stream) { s.release(slot, S(stream)); })
      .def("take_h2d_ms",
           [](HostStager& s) {
             py::gil_scoped_release nogil;
             return s.take_h2d_ms();
           },
           "(device ms of the H2D copies since the last call, number of uploads)")
      .def_property_readonly("slots", &HostStager::slots)
      .def_property_readonly("text_capacity", &HostStager::text_capacity);
}
