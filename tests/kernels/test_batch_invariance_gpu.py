"""Batch invariance on the GPU: under ``ATPU_BATCH_INVARIANT`` (the agent's
default) a row's result is bit-identical whatever the number of rows that share its launch.

* every GEMM family (64x64 dec, 128x128, 256x256 persistent / per-tile) computes a row the same way
  (one MFMA 16x16x32 chain over K in order, the same epilogue arithmetic and GELU);
* decode GEMMs at 4 rows (where the GEMV runs by default) equal the same rows inside 512;
* decode attention (cross and self) and the fused LM head + top-k: 1 item vs many;
* summarize (T5 and BART): N one-document jobs one by one == batched (sequences and scores);
* classify: 1-row ``input`` jobs one by one == stacked (top-k indices and scores).
Reference numerics are pinned by the per-kernel fp32 tests elsewhere; these tests pin equality.
"""
import pytest
import torch

from agent_tpu_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture
def invariant():
    prev = ops.set_batch_invariant(True)
    yield
    ops.set_batch_invariant(prev)


def _r(shape, dev, scale=1.0, seed=0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dev, dtype)


def _tile(nat, t):
    prev = nat.gemm_force_tile(-1)
    nat.gemm_force_tile(t)
    return prev


@pytest.mark.parametrize("epi", ["bias_gelu", "bias_res", "plain", "rms_relu", "bias_tanh"])
def test_gemm_families_compute_a_row_identically(gpu, nat, invariant, epi):
    M, K, N = 512, 768, 768
    x = _r((M, K), gpu, 1.0, 1)
    w = _r((N, K), gpu, 0.04, 2)
    b = (torch.randn(N, generator=torch.Generator().manual_seed(3)) * 0.1).to(gpu)
    res = _r((M, N), gpu, 1.0, 4)
    kw = {"bias_gelu": dict(bias=b, act="gelu"), "bias_res": dict(bias=b, residual=res), "plain": {},
          "rms_relu": dict(act="relu", rms_eps=1e-6), "bias_tanh": dict(bias=b, act="tanh")}[epi]
    tiles = (64, 128) if epi == "rms_relu" else (64, 128, 256)
    outs = {}
    for t in tiles:
        prev = _tile(nat, t)
        try:
            outs[t] = ops.linear(x, w, **kw)
        finally:
            nat.gemm_force_tile(prev)
    torch.cuda.synchronize()
    for t in tiles[1:]:
        assert torch.equal(outs[tiles[0]], outs[t]), (epi, t)
    # a different row count picks a different family / grid: the shared rows do not move
    few = ops.linear(x[:4].contiguous(), w, **{k: (v[:4].contiguous() if k == "residual" else v) for k, v in kw.items()})
    mid = ops.linear(x[:40].contiguous(), w, **{k: (v[:40].contiguous() if k == "residual" else v) for k, v in kw.items()})
    assert torch.equal(few, outs[64][:4]) and torch.equal(mid, outs[64][:40])


def test_gemm_256_per_tile_schedule_matches(gpu, nat, invariant):
    """M % 256 != 0 at M >= 2048 runs the per-tile 256p schedule (permlane epilogue)."""
    M, K, N = 2048 + 128, 768, 768
    x = _r((M, K), gpu, 1.0, 5)
    w = _r((N, K), gpu, 0.04, 6)
    b = (torch.randn(N, generator=torch.Generator().manual_seed(7)) * 0.1).to(gpu)
    prev = _tile(nat, 256)
    try:
        big = ops.linear(x, w, b, act="gelu")
    finally:
        nat.gemm_force_tile(prev)
    small = ops.linear(x[:64].contiguous(), w, b, act="gelu")
    assert torch.equal(big[:64], small)


def test_decode_gemm_epilogues_rows_4_vs_512(gpu, invariant):
    """The decoder's fused epilogues (RowRms + KV scatter, RowLn / ResLn / RowStats) at 4 rows
    (the 1-document step) equal the same rows of a 512-row step."""
    from agent_tpu_amd.ops.linear import row_parts_ref

    M, d, T = 512, 768, 16
    x = _r((M, d), gpu, 1.0, 11)
    w = _r((3 * d, d), gpu, 0.04, 12)
    step = torch.tensor([5], dtype=torch.int32, device=gpu)
    outs = []
    for m in (M, 4):
        cache = torch.zeros((m * T, 2 * d), dtype=torch.bfloat16, device=gpu)
        q = ops.linear(x[:m].contiguous(), w, rms_eps=1e-6, kv_cache=(cache, T, step, d))
        outs.append((q, cache.view(m, T, 2 * d)[:, 5].clone()))
    assert torch.equal(outs[0][0][:4], outs[1][0]) and torch.equal(outs[0][1][:4], outs[1][1])
    # BART-style LayerNorm folding: RowStats producer, RowLn consumer, ResLn residual
    wo = _r((d, d), gpu, 0.04, 13)
    bo = (torch.randn(d, generator=torch.Generator().manual_seed(14)) * 0.1).to(gpu)
    res = _r((M, d), gpu, 1.0, 15)
    colsum = wo.float().sum(1).contiguous()
    gamma = (1 + 0.1 * torch.randn(d, generator=torch.Generator().manual_seed(16))).to(gpu)
    got = []
    for m in (M, 4):
        part = torch.empty((d // 32, m, 2), dtype=torch.float32, device=gpu)
        y = ops.linear(x[:m].contiguous(), wo, bo, residual=res[:m].contiguous(), stats_out=part)
        inp = row_parts_ref(res[:m]).contiguous()
        z = ops.linear(y, wo, bo, row_ln=(1e-5, colsum, part))
        u = ops.linear(y, wo, bo, residual=res[:m].contiguous(), res_ln=(1e-5, inp, gamma))
        got.append((y, part, z, u))
    for a_, b_ in zip(got[0], got[1]):
        if a_.dim() == 3:
            assert torch.equal(a_[:, :4], b_)
        else:
            assert torch.equal(a_[:4], b_)


def test_decode_attention_one_item_vs_many(gpu, invariant):
    H, d, S, group = 12, 768, 1024, 4
    items = 40
    q = _r((items * group, d), gpu, 1.0, 21)
    kv = _r((items * S, 2 * d), gpu, 1.0, 22)
    lens = torch.randint(300, S + 1, (items,), generator=torch.Generator().manual_seed(23), dtype=torch.int32).to(gpu)
    many = ops.decode_attention(q, kv[:, :d], kv[:, d:], H, S, group, lens=lens)
    one = ops.decode_attention(q[:group].contiguous(), kv[:S, :d], kv[:S, d:], H, S, group, lens=lens[:1])
    assert torch.equal(many[:group], one)
    # self attention with beam backpointers: 4 rows (few-row kernel by default) vs 64
    T, rows = 130, 64
    cache = _r((rows * T, 2 * d), gpu, 1.0, 24)
    qs = _r((rows, d), gpu, 1.0, 25)
    hist = torch.randint(0, 4, (rows, T), generator=torch.Generator().manual_seed(26), dtype=torch.int32).to(gpu)
    step = torch.tensor([70], dtype=torch.int32, device=gpu)
    bias = torch.randn(H, T, generator=torch.Generator().manual_seed(27)).to(gpu)
    big = ops.decode_attention(qs, cache[:, :d], cache[:, d:], H, T, 1, step=step, bias_dist=bias, hist=hist)
    small = ops.decode_attention(qs[:4].contiguous(), cache[:4 * T, :d], cache[:4 * T, d:], H, T, 1, step=step,
                                 bias_dist=bias, hist=hist[:4].contiguous())
    assert torch.equal(big[:4], small)


@pytest.mark.parametrize("group,S,H,items", [(4, 1024, 12, 64), (8, 2048, 16, 40), (1, 700, 12, 50),
                                              (3, 256, 12, 200)])
def test_cross_attention_chunked_equals_split(gpu, invariant, group, S, H, items):
    """Past the split grid (items x heads >= 512) batch-invariant mode runs decode_cross_chunked_kernel
    (the split form's chunk and combine code, one workgroup per (item, head), records in LDS):
    every item equals its own one-item split launch bit for bit, and the reference to rounding."""
    from agent_tpu_amd.ops.decode import _decode_attention_ref

    d = H * 64
    rows = items * group
    q = _r((rows, 3 * d), gpu, 1.0, 81)[:, :d]  # strided like the fused QKV output
    kv = _r((items * S, 2 * d), gpu, 1.0, 82)
    lens = torch.randint(1, S + 1, (items,), generator=torch.Generator().manual_seed(83), dtype=torch.int32)
    lens[0], lens[-1] = S, 37  # a full source and one shorter than a chunk
    lens = lens.to(gpu)
    bias = _r((H, S), gpu, 1.0, 84, torch.float32)
    many = ops.decode_attention(q, kv[:, :d], kv[:, d:], H, S, group, lens=lens, bias_dist=bias, scale=0.125)
    for i in (0, 1, items // 2, items - 1):
        one = ops.decode_attention(q[i * group:(i + 1) * group], kv[i * S:(i + 1) * S, :d], kv[i * S:(i + 1) * S, d:],
                                   H, S, group, lens=lens[i:i + 1], bias_dist=bias, scale=0.125)
        assert torch.equal(many[i * group:(i + 1) * group], one), i
    sub = slice(0, 3 * group)
    ref = _decode_attention_ref(q[sub].cpu(), kv[:3 * S, :d].cpu(), kv[:3 * S, d:].cpu(), H, S, group, lens[:3].cpu(),
                                None, bias.cpu(), 0.125, None)
    assert (many[sub].float().cpu() - ref.float()).abs().max().item() < 2e-2 * max(1.0, ref.float().abs().max().item())


@pytest.mark.parametrize("V,d,rms,bias", [(32128, 768, True, False), (50264, 1024, False, True)])
def test_lm_head_topk_rows_4_vs_64(gpu, invariant, V, d, rms, bias):
    w = _r((V, d), gpu, d ** -0.5, 31)
    x = _r((64, d), gpu, 1.0, 32)
    b = (torch.randn(V, generator=torch.Generator().manual_seed(33)) * 0.5).to(gpu) if bias else None
    bs = torch.randn(64, generator=torch.Generator().manual_seed(34)).to(gpu)
    eps = 1e-6 if rms else 0.0
    s64, t64 = ops.lm_head_topk(x, w, bs, 8, 1, False, bias=b, rms_eps=eps)
    s4, t4 = ops.lm_head_topk(x[:4].contiguous(), w, bs[:4].contiguous(), 8, 1, False, bias=b, rms_eps=eps)
    assert torch.equal(s64[:4], s4) and torch.equal(t64[:4], t4)


@pytest.mark.parametrize("family", ["t5-base", "bart-large-cnn"])
def test_summarize_one_doc_jobs_equal_batched(gpu, invariant, family):
    """N single-document jobs one by one == the same documents as one batch (and through the
    in-flight SummarizeStream): identical token sequences and beam scores."""
    from agent_tpu_amd.runtime.summarize import GenConfig, SummarizeEngine, SummarizeStream, build_model
    from agent_tpu_amd.utils.synthetic import make_text_rows

    model, _ = build_model(family, device=gpu, seed=0)
    eng = SummarizeEngine(model, 1024)
    docs = make_text_rows(5, words_per_row=700, seed=41)
    gen = GenConfig(num_beams=4, max_length=40, min_length=10)
    singles = [eng.run(*eng.encode_texts([t], with_maps=False)[:2], gen) for t in docs]
    batched = eng.run(*eng.encode_texts(docs, with_maps=False)[:2], gen)
    for i, s in enumerate(singles):
        assert s.sequences[0] == batched.sequences[i], (family, i)
        assert s.scores[0] == batched.scores[i], (family, i)
    st = SummarizeStream(eng, max_searches=2, part_max=3)
    for i, t in enumerate(docs):
        st.submit(i, [t], gen)
    got = {}
    for tag, _, scores, _ in st.drain():
        got[tag] = scores[0]
    assert got == {i: s.scores[0] for i, s in enumerate(singles)}


def test_classify_single_rows_equal_stacked(gpu, invariant):
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine

    cfg = config_for("bert-base", num_labels=4)
    eng = ClassifyEngine(cfg, init_random(cfg, seed=0, device=gpu), gpu, batch_rows=64, seq_len=128, topk=4)
    g = torch.Generator().manual_seed(51)
    n = 37
    lens = torch.randint(10, 129, (n,), generator=g, dtype=torch.int32)
    ids = torch.randint(1000, 30000, (n, 128), generator=g, dtype=torch.int32)
    ids[:, 0] = 101
    for i in range(n):
        ids[i, int(lens[i]):] = 0
    stacked = eng.classify_ids(ids, lens, 4)
    for i in (0, 5, 36):
        one = eng.classify_ids(ids[i:i + 1], lens[i:i + 1], 4)
        assert torch.equal(one.idx[0], stacked.idx[i]) and torch.equal(one.score[0], stacked.score[i]), i


@pytest.mark.parametrize("epi", ["rms_kv", "rms_relu", "bias_res", "res", "plain", "bias_gelu", "row_ln", "res_ln_stats",
                                 "out_f32"])
@pytest.mark.parametrize("M,K", [(1, 768), (4, 3072), (8, 2048), (16, 1024)])
def test_few_row_exact_kernel_equals_dec(gpu, nat, invariant, epi, M, K):
    """Under batch invariance <= 16 rows run gemm_few_exact_kernel (no LDS ring; K = 2048 / 3072 at
    <= 8 rows: gemm_few_dma_kernel); it must give the dec kernel's bits (ATPU_GEMM_TILE=64 forces the
    dec kernel on the same rows)."""
    from agent_tpu_amd.ops.linear import row_parts_ref

    N = 1024 if epi in ("row_ln", "res_ln_stats") else 768
    if epi == "row_ln":
        K = min(K, 1024)  # RowLn rows are <= 1024 wide
    x = _r((M, K), gpu, 1.0, 61)
    w = _r((N, K), gpu, K ** -0.5, 62)
    b = (torch.randn(N, generator=torch.Generator().manual_seed(63)) * 0.1).to(gpu)
    res = _r((M, N), gpu, 1.0, 64)

    def run():
        if epi == "rms_kv":
            T = 8
            cache = torch.zeros((M * T, 2 * N), dtype=torch.bfloat16, device=gpu)
            w3 = _r((3 * N, K), gpu, K ** -0.5, 65)
            q = ops.linear(x, w3, rms_eps=1e-6, kv_cache=(cache, T, torch.tensor([3], dtype=torch.int32,
                                                                                   device=gpu), N))
            return [q, cache]
        if epi == "rms_relu":
            return [ops.linear(x, w, act="relu", rms_eps=1e-6)]
        if epi == "bias_res":
            return [ops.linear(x, w, b, residual=res)]
        if epi == "res":  # T5's FF-out (K = 3072: the LDS-DMA form at <= 8 rows)
            return [ops.linear(x, w, residual=res)]
        if epi == "plain":
            return [ops.linear(x, w)]
        if epi == "bias_gelu":
            return [ops.linear(x, w, b, act="gelu")]
        if epi == "out_f32":
            return [ops.linear(x, w, out_f32=True, rms_eps=1e-6)]
        if epi == "row_ln":
            part = row_parts_ref(x).contiguous()
            return [ops.linear(x, w, b, act="gelu", row_ln=(1e-5, w.float().sum(1).contiguous(), part))]
        part = torch.empty((N // 32, M, 2), dtype=torch.float32, device=gpu)
        gam = (1 + 0.1 * torch.randn(N, generator=torch.Generator().manual_seed(66))).to(gpu)
        y = ops.linear(x, w, b, residual=res, res_ln=(1e-5, row_parts_ref(res).contiguous(), gam), stats_out=part)
        return [y, part]

    got = run()
    prev = _tile(nat, 64)
    try:
        ref = run()
    finally:
        nat.gemm_force_tile(prev)
    torch.cuda.synchronize()
    for a_, b_ in zip(got, ref):
        assert torch.equal(a_, b_), epi
