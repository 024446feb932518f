"""Decode kernels (K9-K11) and the T5 HIP path vs the fp32 CPU references."""
import numpy as np
import pytest
import torch

from agent_tpu_amd import ops
from agent_tpu_amd.ops.decode import _decode_attention_ref

pytestmark = pytest.mark.gpu


def _r(shape, dev, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dtype).to(dev)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("rows,group,S,H", [(8, 4, 37, 12), (3, 1, 130, 4), (16, 4, 512, 12)])
def test_decode_attention_cross(gpu, rows, group, S, H):
    nseq = rows // group
    q = _r((rows, H * 64), gpu, seed=1)
    kv = _r((nseq * S, 2 * H * 64), gpu, seed=2)
    lens = torch.tensor([S - 5 * i for i in range(nseq)], dtype=torch.int32).clamp(min=1)
    out = ops.decode_attention(q, kv[:, :H * 64], kv[:, H * 64:], H, S, group, lens=lens.to(gpu))
    ref = _decode_attention_ref(q.cpu(), kv.cpu()[:, :H * 64], kv.cpu()[:, H * 64:], H, S, group, lens, None, None,
                                1.0, None)
    assert _rel(out, ref) < 2e-2


@pytest.mark.parametrize("lens,group,S,H,scale", [([1, 63, 64, 65, 128, 1024], 4, 1024, 12, 1.0),
                                                   ([1000], 4, 1024, 12, 0.125), ([130, 7], 1, 130, 16, 1.0),
                                                   ([700, 3, 640], 8, 704, 12, 1.0), ([200, 199], 3, 256, 12, 1.0)])
def test_decode_cross_split_keys(gpu, lens, group, S, H, scale):
    # few items: the keys are split into 64-key chunks (flash decoding) over workgroups and
    # combined by a second kernel; chunks past an item's length, a 1-key item, partial last
    # chunks, 1-8 beams
    from agent_tpu_amd._native import native

    nat = native()
    nseq = len(lens)
    rows = nseq * group - (1 if group > 2 else 0)  # a short last item
    assert nat.decode_attention_ws_floats(rows, group, H, S, True) > 0
    q = _r((rows, 3 * H * 64), gpu, seed=41)[:, :H * 64]  # strided like the fused QKV output
    kv = _r((nseq * S, 2 * H * 64), gpu, seed=42)
    lt = torch.tensor(lens, dtype=torch.int32)
    for bias in (None, _r((H, S), gpu, 1.0, torch.float32, seed=43)):
        out = ops.decode_attention(q, kv[:, :H * 64], kv[:, H * 64:], H, S, group, lens=lt.to(gpu),
                                   bias_dist=bias, scale=scale)
        ref = _decode_attention_ref(q.cpu(), kv.cpu()[:, :H * 64], kv.cpu()[:, H * 64:], H, S, group, lt, None,
                                    None if bias is None else bias.cpu(), scale, None)
        assert _rel(out, ref) < 2e-2


@pytest.mark.parametrize("rows,H,T,t", [(4, 12, 130, 70), (1, 12, 130, 0), (8, 16, 300, 299)])
def test_decode_self_head_groups(gpu, rows, H, T, t):
    # few rows: the per-row self-attention kernel spreads the heads over grid.y
    d = H * 64
    cache = _r((rows * T, 2 * d), gpu, seed=51)
    q = _r((rows, d), gpu, seed=52)
    g = torch.Generator().manual_seed(6)
    hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32)
    step = torch.tensor([t], dtype=torch.int32)
    bias = _r((H, T), gpu, 1.0, torch.float32, seed=53)
    out = ops.decode_attention(q, cache[:, :d], cache[:, d:], H, T, 1, step=step.to(gpu), bias_dist=bias,
                               hist=hist.to(gpu))
    ref = _decode_attention_ref(q.cpu(), cache.cpu()[:, :d], cache.cpu()[:, d:], H, T, 1, None, step, bias.cpu(), 1.0,
                                None, hist)
    assert _rel(out, ref) < 2e-2


@pytest.mark.parametrize("rows,H,T,t,hist_on", [(4, 12, 130, 70, True), (4, 12, 130, 129, True), (1, 12, 130, 0, True),
                                                (4, 12, 64, 63, False), (3, 16, 100, 64, True), (4, 12, 192, 150, True)])
def test_decode_self_few_matches_row_kernel(gpu, rows, H, T, t, hist_on):
    # few rows, T <= 192: one wave per (row, head) with every load in two rounds
    # (decode_self_few_kernel) against the per-row kernel: same key / dimension order of
    # every sum, so bit-identical; KC = 1-3 key chunks, a step at the cache end, no hist
    nat = __import__("agent_tpu_amd._native", fromlist=["native"]).native()
    d = H * 64
    cache = _r((rows * T, 2 * d), gpu, seed=61)
    q = _r((rows, 3 * d), gpu, seed=62)[:, :d]
    g = torch.Generator().manual_seed(7)
    hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32).to(gpu) if hist_on else None
    step = torch.tensor([t], dtype=torch.int32, device=gpu)
    bias = _r((H, T), gpu, 1.0, torch.float32, seed=63)
    prev = nat.decode_self_few(-1)
    try:
        outs = []
        for few in (1, 0):
            nat.decode_self_few(few)
            outs.append(ops.decode_attention(q, cache[:, :d], cache[:, d:], H, T, 1, step=step, bias_dist=bias, hist=hist))
    finally:
        nat.decode_self_few(prev)
    assert torch.equal(outs[0], outs[1])
    ref = _decode_attention_ref(q.cpu(), cache.cpu()[:, :d], cache.cpu()[:, d:], H, T, 1, None, step.cpu(), bias.cpu(),
                                1.0, None, None if hist is None else hist.cpu())
    assert _rel(outs[0], ref) < 2e-2


def test_decode_self_with_bias_append_gather(gpu):
    rows, H, T = 6, 4, 20
    d = H * 64
    cache = torch.zeros((rows * T, 2 * d), dtype=torch.bfloat16, device=gpu)
    step = torch.zeros(1, dtype=torch.int32, device=gpu)
    bias = _r((H, T), gpu, 1.0, torch.float32, seed=3)
    for t in range(7):
        step.fill_(t)
        qkv = _r((rows, 3 * d), gpu, seed=10 + t)
        ops.kv_append(qkv, d, 2 * d, cache, T, step)
        out = ops.decode_attention(qkv[:, :d], cache[:, :d], cache[:, d:], H, T, 1, step=step, bias_dist=bias)
        ref = _decode_attention_ref(qkv.cpu(), cache.cpu()[:, :d], cache.cpu()[:, d:], H, T, 1, None,
                                    step.cpu(), bias.cpu(), 1.0, None)
        assert _rel(out, ref) < 2e-2
    parent = torch.tensor([2, 2, 0, 5, 1, 3], dtype=torch.int32, device=gpu)
    dst = torch.zeros_like(cache)
    ops.gather_rows(cache.view(1, rows * T, 2 * d), dst.view(1, rows * T, 2 * d), parent, rows, T, step)
    c3, d3 = cache.view(rows, T, 2 * d).cpu(), dst.view(rows, T, 2 * d).cpu()
    assert torch.equal(d3[:, :7], c3[parent.long().cpu(), :7])


def test_decode_self_hist_backpointers(gpu):
    rows, H, T, t = 8, 4, 24, 13
    d = H * 64
    cache = _r((rows * T, 2 * d), gpu, seed=21)
    q = _r((rows, d), gpu, seed=22)
    g = torch.Generator().manual_seed(3)
    hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32)
    step = torch.tensor([t], dtype=torch.int32)
    bias = _r((H, T), gpu, 1.0, torch.float32, seed=23)
    out = ops.decode_attention(q, cache[:, :d], cache[:, d:], H, T, 1, step=step.to(gpu), bias_dist=bias,
                               hist=hist.to(gpu))
    ref = _decode_attention_ref(q.cpu(), cache.cpu()[:, :d], cache.cpu()[:, d:], H, T, 1, None, step, bias.cpu(), 1.0,
                                None, hist)
    assert _rel(out, ref) < 2e-2
    # reorder kernel vs CPU reference
    parent = torch.tensor([3, 3, 0, 7, 1, 2, 2, 5], dtype=torch.int32)
    dst = torch.zeros_like(hist)
    ops.beam_reorder_hist(hist, dst, parent, step)
    dgpu = torch.zeros_like(hist).to(gpu)
    ops.beam_reorder_hist(hist.to(gpu), dgpu, parent.to(gpu), step.to(gpu))
    assert torch.equal(dgpu.cpu()[:, :t + 1], dst[:, :t + 1])
    assert torch.equal(dst[:, t], parent) and torch.equal(dst[:, :t], hist[parent.long(), :t])


@pytest.mark.parametrize("rows,H,T,t,scale", [(9, 16, 300, 257, 0.125), (64, 12, 130, 64, 1.0), (5, 12, 131, 0, 1.0),
                                              (3, 2, 2048, 2047, 0.125)])
def test_decode_self_rows_all_heads(gpu, rows, H, T, t, scale):
    # per-row all-heads self-attention kernel: > 64 keys (several score passes), 16 heads over 4 waves,
    # the first step (one key), the longest cache; random backpointers, no bias / T5 bias
    d = H * 64
    cache = _r((rows * T, 2 * d), gpu, seed=31)
    q = _r((rows, 3 * d), gpu, seed=32)[:, :d]  # strided like the fused QKV output
    g = torch.Generator().manual_seed(5)
    hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32)
    step = torch.tensor([t], dtype=torch.int32)
    for bias in (None, _r((H, T), gpu, 1.0, torch.float32, seed=33)):
        out = ops.decode_attention(q, cache[:, :d], cache[:, d:], H, T, 1, step=step.to(gpu), bias_dist=bias,
                                   hist=hist.to(gpu), scale=scale)
        ref = _decode_attention_ref(q.cpu(), cache.cpu()[:, :d], cache.cpu()[:, d:], H, T, 1, None, step,
                                    None if bias is None else bias.cpu(), scale, None, hist)
        assert _rel(out, ref) < 2e-2


@pytest.mark.parametrize("rows,group,seqlen", [(256, 4, 512), (40, 4, 100), (24, 8, 7), (9, 3, 2048), (10, 4, 64),
                                               (13, 5, 300)])
def test_decode_cross_grouped_shapes(gpu, rows, group, seqlen):
    H = 12
    nseq = (rows + group - 1) // group
    q = _r((rows, H * 64), gpu, seed=31)
    kv = _r((nseq * seqlen, 2 * H * 64), gpu, seed=32)
    g = torch.Generator().manual_seed(4)
    lens = torch.randint(1, seqlen + 1, (nseq,), generator=g, dtype=torch.int32)
    out = ops.decode_attention(q, kv[:, :H * 64], kv[:, H * 64:], H, seqlen, group, lens=lens.to(gpu))
    ref = _decode_attention_ref(q.cpu(), kv.cpu()[:, :H * 64], kv.cpu()[:, H * 64:], H, seqlen, group, lens, None, None,
                                1.0, None)
    assert _rel(out, ref) < 2e-2


@pytest.mark.parametrize("V,k,mask", [(4096, 8, False), (32128, 8, True), (50, 2, False), (32128, 16, False),
                                      (1000, 1, True), (70000, 5, False)])
def test_beam_topk_rows(gpu, V, k, mask):
    R = 12
    logits = _r((R, V), gpu, 3.0, torch.float32, seed=4)
    bs = _r((R,), gpu, 1.0, torch.float32, seed=5)
    sc, idx = ops.beam_topk_rows(logits, bs, k, eos=1, mask_eos=mask)
    rsc, ridx = ops.beam_topk_rows(logits.cpu(), bs.cpu(), k, eos=1, mask_eos=mask)
    torch.testing.assert_close(sc.cpu(), rsc, atol=2e-4, rtol=1e-5)
    assert torch.equal(idx.cpu(), ridx)
    if mask:
        assert not (idx == 1).any()


@pytest.mark.parametrize("V,k", [(32128, 8), (50264, 16), (1002, 4), (7, 5)])
def test_beam_topk_rows_ties(gpu, V, k):
    # coarse logits: many exact ties at the top; the order is (value desc, index asc)
    R = 9
    logits = (_r((R, V), gpu, 3.0, torch.float32, seed=8) * 2).round() / 2
    logits[3] = 1.0  # a row of one value
    bs = _r((R,), gpu, 1.0, torch.float32, seed=9)
    sc, idx = ops.beam_topk_rows(logits, bs, k, eos=1, mask_eos=True)
    rsc, _ = ops.beam_topk_rows(logits.cpu(), bs.cpu(), k, eos=1, mask_eos=True)
    torch.testing.assert_close(sc.cpu(), rsc, atol=2e-4, rtol=1e-5)
    x = logits.cpu().numpy().copy()
    x[:, 1] = -np.inf
    for r in range(R):
        want = np.lexsort((np.arange(V), -x[r]))[:k]
        assert idx[r].tolist() == want.tolist(), r


@pytest.mark.parametrize("n,cur", [(3, 40), (3, 2), (2, 17), (4, 64)])
def test_beam_topk_rows_device_ngram(gpu, n, cur):
    # n-gram bans computed in the kernel from the device token history == host processor;
    # tokens drawn from a tiny alphabet so every row repeats its n-grams
    R, V, T = 12, 4096, 70
    logits = _r((R, V), gpu, 3.0, torch.float32, seed=51)
    bs = _r((R,), gpu, 1.0, torch.float32, seed=52)
    g = torch.Generator().manual_seed(53)
    seq = torch.randint(0, 6, (R, T), generator=g, dtype=torch.int32)
    logits[:, :6] += 20.0  # the banned candidates are the best raw ones
    sc, idx = ops.beam_topk_rows(logits, bs, 8, eos=1, mask_eos=False, ngram=(seq.to(gpu), cur, n))
    rsc, ridx = ops.beam_topk_rows(logits.cpu(), bs.cpu(), 8, eos=1, mask_eos=False, ngram=(seq, cur, n))
    torch.testing.assert_close(sc.cpu(), rsc, atol=2e-4, rtol=1e-5)
    assert torch.equal(idx.cpu(), ridx)


def test_beam_reorder_token_history(gpu):
    R, T = 10, 16
    g = torch.Generator().manual_seed(3)
    src = torch.randint(0, 100, (R, T), generator=g, dtype=torch.int32)
    parent = torch.randint(0, R, (R,), generator=g, dtype=torch.int32)
    tok = torch.randint(0, 100, (R,), generator=g, dtype=torch.int32)
    for step in (0, 5, T - 2, T - 1):
        st = torch.tensor([step], dtype=torch.int32)
        want = torch.full((R, T), -7, dtype=torch.int32)
        ops.beam_reorder_hist(src, want, parent, st, last=tok, off=1)
        got = torch.full((R, T), -7, dtype=torch.int32, device=gpu)
        ops.beam_reorder_hist(src.to(gpu), got, parent.to(gpu), st.to(gpu), last=tok.to(gpu), off=1)
        assert torch.equal(got.cpu(), want), step


@pytest.mark.parametrize("V,k,nb", [(50264, 8, 12), (32128, 8, 1), (4096, 3, 300)])
def test_beam_topk_rows_bans(gpu, V, k, nb):
    # per-row banned tokens filtered inside the kernel: equal to the CPU path, and the
    # best raw candidates of each row are banned on purpose (so the filter must act)
    R = 16
    logits = _r((R, V), gpu, 3.0, torch.float32, seed=41)
    bs = _r((R,), gpu, 1.0, torch.float32, seed=42)
    g = torch.Generator().manual_seed(6)
    bans = torch.randint(0, V, (R, nb), generator=g, dtype=torch.int32)
    top = torch.topk(logits.cpu(), min(nb, 4), dim=-1).indices.to(torch.int32)
    bans[:, :top.shape[1]] = top
    bans[::3, -1] = -1  # padding
    sc, idx = ops.beam_topk_rows(logits, bs, k, eos=1, mask_eos=True, bans=bans.to(gpu))
    rsc, ridx = ops.beam_topk_rows(logits.cpu(), bs.cpu(), k, eos=1, mask_eos=True, bans=bans)
    torch.testing.assert_close(sc.cpu(), rsc, atol=2e-4, rtol=1e-5)
    assert torch.equal(idx.cpu(), ridx)
    for r in range(R):
        assert not set(idx[r].tolist()) & set(b for b in bans[r].tolist() if b >= 0)


def _lm_case(R, V, d, rms, bias, gpu, seed, scale=1.0):
    x = _r((R, d), gpu, 1.0, seed=seed)
    w = _r((V, d), gpu, scale / d ** 0.5, seed=seed + 1)
    b = _r((V,), gpu, 0.5, torch.float32, seed=seed + 2) if bias else None
    bs = _r((R,), gpu, 1.0, torch.float32, seed=seed + 3)
    return ops.LmHead(x, w, b, 1e-6 if rms else 0.0), bs


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])  # release builds run 0 whatever is set
@pytest.mark.parametrize("R,V,d,rms,bias,k,mask", [(12, 32128, 768, True, False, 8, True), (300, 50264, 1024, False, True, 8, False),
                                                   (4, 1000, 64, False, False, 2, True), (1024, 32128, 768, True, False, 8, False),
                                                   (130, 4100, 128, False, True, 5, True), (512, 50264, 1024, False, True, 8, True),
                                                   (256, 1000, 128, True, False, 8, False),
                                                   # <= 16 rows, <= one 128-column panel per CU: lm_head_few_kernel
                                                   (8, 20000, 1024, False, True, 8, True), (16, 32128, 768, True, False, 8, False),
                                                   (1, 32128, 768, True, False, 8, True)])
def test_lm_head_topk_matches_logits_path(gpu, cfg, R, V, d, rms, bias, k, mask):
    # fused LM head + top-k == fp32-logit GEMM + beam_topk_rows: the same MFMA accumulation
    # order gives bit-identical logits, so the tokens match exactly; the normaliser is summed
    # in another order (scores to ~1e-6)
    nat = __import__("agent_tpu_amd._native", fromlist=["native"]).native()
    prev = nat.lm_head_stages(-1)
    nat.lm_head_stages(cfg)
    try:
        head, bs = _lm_case(R, V, d, rms, bias, gpu, seed=R + V)
        sc, idx = head.topk(bs, k, eos=1, mask_eos=mask)
        rsc, ridx = ops.beam_topk_rows(head.logits(), bs, k, eos=1, mask_eos=mask)
    finally:
        nat.lm_head_stages(prev)
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(sc.cpu(), rsc.cpu(), atol=1e-4, rtol=1e-5)
    if mask:
        assert not (idx == 1).any()


def test_lm_head_topk_matches_cpu(gpu):
    head, bs = _lm_case(8, 2000, 256, False, True, gpu, seed=5)
    sc, idx = head.topk(bs, 8, eos=1, mask_eos=True)
    cpu = ops.LmHead(head.x.cpu(), head.w.cpu(), head.bias.cpu(), 0.0)
    rsc, ridx = cpu.topk(bs.cpu(), 8, eos=1, mask_eos=True)
    assert torch.equal(idx.cpu(), ridx)
    torch.testing.assert_close(sc.cpu(), rsc, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("V,k,R", [(32128, 8, 20), (1000, 3, 20), (32128, 8, 256), (1000, 8, 512)])
def test_lm_head_topk_ties_take_the_exact_path(gpu, V, k, R):
    # identical vocabulary rows: every logit of a row ties, every tile overflows its 16
    # candidate slots and falls back to the exact argmax rounds -> lowest token ids first
    # (R % 256 == 0: the persistent 256x256 path)
    d = 128
    x = _r((R, d), gpu, 1.0, seed=3)
    w = _r((1, d), gpu, 0.1, seed=4).expand(V, d).contiguous()
    w[V // 2:V // 2 + 3] *= 2  # a few distinct values inside the ties
    bs = _r((R,), gpu, 1.0, torch.float32, seed=5)
    head = ops.LmHead(x, w, None, 0.0)
    sc, idx = head.topk(bs, k, eos=1, mask_eos=True)
    rsc, ridx = ops.beam_topk_rows(head.logits(), bs, k, eos=1, mask_eos=True)
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(sc.cpu(), rsc.cpu(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("n,cur,R", [(3, 40, 12), (3, 2, 12), (2, 17, 12), (3, 40, 256)])
def test_lm_head_topk_device_ngram(gpu, n, cur, R):
    V, d, T = 4096, 128, 70
    head, bs = _lm_case(R, V, d, False, True, gpu, seed=60)
    g = torch.Generator().manual_seed(61)
    seq = torch.randint(0, 6, (R, T), generator=g, dtype=torch.int32).to(gpu)
    head.bias[:6] += 20.0  # the banned candidates are the best raw ones
    sc, idx = head.topk(bs, 8, eos=1, mask_eos=False, ngram=(seq, cur, n))
    rsc, ridx = ops.beam_topk_rows(head.logits(), bs, 8, eos=1, mask_eos=False, ngram=(seq, cur, n))
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(sc.cpu(), rsc.cpu(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("R,V", [(16, 50264), (256, 50264), (4, 20000)])  # (4, 20000): the few-row kernel
def test_lm_head_topk_ban_list(gpu, R, V):
    d, nb = 256, 12
    head, bs = _lm_case(R, V, d, False, True, gpu, seed=70)
    logits = head.logits()
    g = torch.Generator().manual_seed(71)
    bans = torch.randint(0, V, (R, nb), generator=g, dtype=torch.int32)
    bans[:, :4] = torch.topk(logits.cpu(), 4, dim=-1).indices.to(torch.int32)
    bans[::3, -1] = -1
    sc, idx = ops.lm_head_topk(head.x, head.w, bs, 8, 1, True, bias=head.bias, bans=bans.to(gpu))
    rsc, ridx = ops.beam_topk_rows(logits, bs, 8, eos=1, mask_eos=True, bans=bans.to(gpu))
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(sc.cpu(), rsc.cpu(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("M,N,K,act,res,bias", [(256, 768, 3072, None, True, False), (256, 3072, 768, "relu", False, False),
                                                (256, 2304, 768, None, False, True), (96, 768, 768, "gelu", False, True),
                                                (512, 768, 768, None, True, False)])
@pytest.mark.parametrize("mode", [0, 1])
def test_gemm_splitk_skinny(gpu, M, N, K, act, res, bias, mode):
    """mode 0: 128x128 split-K partials + reduce; mode 1: the 64x64 multi-stage
    dec kernel (split-K only when even its grid is small)."""
    from agent_tpu_amd._native import native
    from agent_tpu_amd.ops.linear import _splits, linear_ref

    prev = native().gemm_dec_mode(mode)
    _splits.cache_clear()
    try:
        x = _r((M, K), gpu, seed=41)
        w = _r((N, K), gpu, 0.05, seed=42)
        r = _r((M, N), gpu, seed=43) if res else None
        b = _r((N,), gpu, 1.0, torch.float32, seed=44) if bias else None
        y = ops.linear(x, w, bias=b, act=act, residual=r)
        ref = linear_ref(x.cpu(), w.cpu(), None if b is None else b.cpu(), act, None if r is None else r.cpu(),
                         out_f32=True)
        if mode == 0:
            assert _splits(M, N, K) > 1
        assert _rel(y, ref) < 2e-2
    finally:
        native().gemm_dec_mode(1)
        _splits.cache_clear()


@pytest.mark.parametrize("M,N,K", [(300, 200, 64 * 13), (1024, 768, 768), (64, 64, 64), (70, 132, 128),
                                   (2000, 1000, 3072), (256, 768, 3072), (96, 256, 64 * 40)])
def test_gemm_dec_exact_integers(gpu, M, N, K):
    """{-1,0,1} operands: exact in fp32 and bf16, so the dec kernel (ragged
    M/N edges, ring tails for K-tile counts around the stage depth, split-K
    for the small grids) must match bit for bit."""
    from agent_tpu_amd.ops.linear import _splits

    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randint(-1, 2, (M, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-1, 2, (N, K), generator=g).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = ops.linear(x.to(gpu), w.to(gpu), out_f32=True)
    assert torch.equal(y.cpu(), ref), (M, N, K, _splits(M, N, K))
    yb = ops.linear(x.to(gpu), w.to(gpu))
    assert torch.equal(yb.cpu().float(), ref.to(torch.bfloat16).float())


def test_gemm_relu_and_f32_out(gpu):
    x = _r((96, 256), gpu, seed=6)
    w = _r((512, 256), gpu, 0.1, seed=7)
    y = ops.linear(x, w, act="relu")
    ref = torch.relu(x.cpu().float() @ w.cpu().float().t())
    assert _rel(y, ref) < 2e-2 and (y >= 0).all()
    y32 = ops.linear(x, w, out_f32=True)
    assert y32.dtype == torch.float32 and _rel(y32, x.cpu().float() @ w.cpu().float().t()) < 1e-3
    big = _r((4096, 768), gpu, seed=8)
    w2 = _r((1024, 768), gpu, 0.05, seed=9)
    assert _rel(ops.linear(big, w2, act="relu"), torch.relu(big.cpu().float() @ w2.cpu().float().t())) < 2e-2


def test_t5_step_and_generate_gpu(gpu):
    from agent_tpu_amd.models.t5 import T5Model, config_for, init_random
    from agent_tpu_amd.runtime.summarize import GenConfig, generate

    cfg = config_for("t5-tiny")
    pack = init_random(cfg, seed=1)
    cpu_m, gpu_m = T5Model(cfg, pack, fp32=True), T5Model(cfg, pack.to(gpu))
    B, S = 2, 24
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(2, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([24, 17], dtype=torch.int32)
    ec, kc = cpu_m.encode(ids, lens)
    eg, kg = gpu_m.encode(ids.to(gpu), lens.to(gpu))
    assert _rel(eg[:S], ec[:S]) < 3e-2
    T = 8
    cc, cg = cpu_m.new_cache(B, T), gpu_m.new_cache(B, T)
    tok = torch.zeros(B, dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int32)
    lc = cpu_m.step(tok, step, cc, T, kc, lens, S, 1)
    lg = gpu_m.step(tok.to(gpu), step.to(gpu), cg, T, kg, lens.to(gpu), S, 1)
    assert _rel(lg, lc) < 5e-2
    r1 = generate(gpu_m, ids.to(gpu), lens.to(gpu), GenConfig(num_beams=4, max_length=16, min_length=4))
    r2 = generate(gpu_m, ids.to(gpu), lens.to(gpu), GenConfig(num_beams=4, max_length=16, min_length=4))
    r3 = generate(gpu_m, ids.to(gpu), lens.to(gpu), GenConfig(num_beams=4, max_length=16, min_length=4,
                                                              use_graph=False))
    assert r1.sequences == r2.sequences == r3.sequences
    assert all(2 <= len(s) <= 16 and s[0] == 0 for s in r1.sequences)


@pytest.mark.parametrize("family,S", [("t5", 1024), ("t5", 600), ("bart", 1024)])
def test_encoder_long_source_matches_cpu(gpu, family, S):
    """Encoder at the reference's 1024-token source truncation (ref ops/map_summarize.py:49):
    GPU (flash attention, T5 distance bias) vs the fp32 CPU oracle, ragged lengths."""
    if family == "t5":
        from agent_tpu_amd.models.t5 import T5Model as M, config_for, init_random
        name = "t5-tiny"
    else:
        from agent_tpu_amd.models.bart import BartModel as M, config_for, init_random
        name = "bart-tiny"
    cfg = config_for(name)
    if family == "bart":
        import dataclasses
        cfg = dataclasses.replace(cfg, max_positions=1024)
    pack = init_random(cfg, seed=3)
    cpu_m, gpu_m = M(cfg, pack, fp32=True), M(cfg, pack.to(gpu))
    B = 2
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(5, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([S, S - 301], dtype=torch.int32)
    ec, kc = cpu_m.encode(ids, lens)
    eg, kg = gpu_m.encode(ids.to(gpu), lens.to(gpu))
    for b in range(B):
        n = int(lens[b])
        assert _rel(eg[b * S:b * S + n], ec[b * S:b * S + n]) < 3e-2
        assert _rel(kg[b * S:b * S + n], kc[b * S:b * S + n]) < 3e-2


def test_bart_encoder_ln_fold_matches_unfolded(gpu):
    """The LN-folded BART encoder (BartModel._encode_folded: BERT's fold scheme, StatsOut
    partials + InNorm / ResNorm GEMMs) against the LayerNorm-pass encoder and the fp32 CPU
    oracle, at a width the folding GEMMs take (d = 256, d_ff = 1024, 2 x 1024 tokens)."""
    import dataclasses

    from agent_tpu_amd.models.bart import BartModel, config_for, init_random

    cfg = dataclasses.replace(config_for("bart-tiny"), d_model=256, heads=4, d_ff=1024, enc_layers=3,
                              max_positions=1024)
    pack = init_random(cfg, seed=5)
    cpu_m, gpu_m = BartModel(cfg, pack, fp32=True), BartModel(cfg, pack.to(gpu))
    B, S = 2, 1024
    g = torch.Generator().manual_seed(6)
    ids = torch.randint(5, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([S, S - 301], dtype=torch.int32)
    assert gpu_m._enc_fold_ok(B * S)
    ef, kf = gpu_m.encode(ids.to(gpu), lens.to(gpu))
    gpu_m.enc_ln_fold = False
    eu, ku = gpu_m.encode(ids.to(gpu), lens.to(gpu))
    ec, kc = cpu_m.encode(ids, lens)
    for b in range(B):
        r = slice(b * S, b * S + int(lens[b]))
        assert _rel(ef[r], eu[r]) < 2e-2 and _rel(kf[r], ku[r]) < 2e-2
        assert _rel(ef[r], ec[r]) < 3e-2 and _rel(kf[r], kc[r]) < 3e-2


def test_map_summarize_op_gpu(gpu, monkeypatch):
    import importlib

    monkeypatch.setenv("SUMMARIZE_MODEL", "t5-tiny")
    import ops.map_summarize as ms

    ms = importlib.reload(ms)
    out = ms.handle({"texts": ["the quick brown fox jumps over the lazy dog " * 5, "MI355X summarize test."],
                     "max_length": 20, "min_length": 5})
    assert out["ok"] and out["device"] == "cuda" and len(out["summaries"]) == 2
    assert ms.handle({}) == {"ok": False, "error": "empty payload"}


def test_bart_step_and_generate_gpu(gpu):
    from agent_tpu_amd.models.bart import BartModel, config_for, init_random
    from agent_tpu_amd.runtime.summarize import GenConfig, generate

    cfg = config_for("bart-tiny")
    pack = init_random(cfg, seed=2, std=0.1)
    cpu_m, gpu_m = BartModel(cfg, pack, fp32=True), BartModel(cfg, pack.to(gpu))
    B, S = 2, 24
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([24, 17], dtype=torch.int32)
    ec, kc = cpu_m.encode(ids, lens)
    eg, kg = gpu_m.encode(ids.to(gpu), lens.to(gpu))
    assert _rel(eg[:S], ec[:S]) < 3e-2 and _rel(kg, kc) < 3e-2
    T = 8
    cc, cg = cpu_m.new_cache(B, T), gpu_m.new_cache(B, T)
    step = torch.zeros(1, dtype=torch.int32)
    tok = torch.full((B,), 2, dtype=torch.int32)
    for t in range(3):
        step.fill_(t)
        lc = cpu_m.step(tok, step, cc, T, kc, lens, S, 1)
        lg = gpu_m.step(tok.to(gpu), step.to(gpu), cg, T, kg, lens.to(gpu), S, 1)
        assert _rel(lg, lc) < 5e-2, t
        tok = lc.argmax(-1).to(torch.int32)
    gen = GenConfig(num_beams=4, max_length=20, min_length=6)
    r1 = generate(gpu_m, ids.to(gpu), lens.to(gpu), gen)
    r2 = generate(gpu_m, ids.to(gpu), lens.to(gpu), GenConfig(num_beams=4, max_length=20, min_length=6,
                                                              use_graph=False))
    assert r1.sequences == r2.sequences
    assert all(s[0] == 2 and s[1] == 0 and len(s) <= 20 for s in r1.sequences)


@pytest.mark.parametrize("M,N,K,act,out_f32", [(1024, 2304, 768, None, False), (1024, 3072, 768, "relu", False),
                                               (256, 768, 768, None, False), (4096, 768, 768, None, False),
                                               (1024, 32128, 768, None, True), (77, 192, 256, "relu", False)])
def test_gemm_row_rms_fold(gpu, M, N, K, act, out_f32):
    # RMSNorm folded into the GEMM (skinny dec kernel, 128x128 kernel, LM-head fp32 out):
    # rsqrt(mean(x^2) + eps) * (x @ (w*gamma).T) against the fp32 norm-then-linear reference
    x = _r((M, K), gpu, 2.0, seed=21)
    w = _r((N, K), gpu, 0.05, seed=22)
    gamma = 1 + _r((K,), gpu, 0.3, torch.float32, seed=23)
    eps = 1e-6
    wf = ops.fold_rms_into_linear(w, gamma)
    y = ops.linear(x, wf, act=act, out_f32=out_f32, rms_eps=eps)
    xf = x.cpu().float()
    xn = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * gamma.cpu()
    ref = xn @ w.cpu().float().t()
    if act == "relu":
        ref = torch.relu(ref)
    assert y.dtype == (torch.float32 if out_f32 else torch.bfloat16)
    assert _rel(y, ref) < 2e-2


def test_t5_step_rms_fold_matches_unfolded(gpu):
    # non-trivial RMSNorm gammas: the folded decoder step vs the rmsnorm + linear step (GPU) and the fp32 oracle
    from agent_tpu_amd.models.t5 import T5Model, config_for, init_random

    cfg = config_for("t5-tiny")
    pack = init_random(cfg, seed=3)
    g = torch.Generator().manual_seed(4)
    for n in pack.names():
        if n.split(".")[-1].startswith("ln"):
            pack[n].copy_(1 + 0.3 * torch.randn(pack[n].shape, generator=g))
    cpu_m = T5Model(cfg, pack, fp32=True)
    gp = pack.to(gpu)
    fold_m, plain_m = T5Model(cfg, gp), T5Model(cfg, gp)
    plain_m.rms_fold = False
    assert fold_m.rms_fold
    B, S, T = 3, 16, 8
    ids = torch.randint(2, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([16, 9, 12], dtype=torch.int32)
    _, kc = cpu_m.encode(ids, lens)
    _, kg = fold_m.encode(ids.to(gpu), lens.to(gpu))
    tok = torch.randint(2, cfg.vocab_size, (B,), generator=g, dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int32)
    lc = cpu_m.step(tok, step, cpu_m.new_cache(B, T), T, kc, lens, S, 1)
    lf = fold_m.step(tok.to(gpu), step.to(gpu), fold_m.new_cache(B, T), T, kg, lens.to(gpu), S, 1)
    lp = plain_m.step(tok.to(gpu), step.to(gpu), plain_m.new_cache(B, T), T, kg, lens.to(gpu), S, 1)
    assert _rel(lf, lc) < 5e-2 and _rel(lp, lc) < 5e-2
    assert _rel(lf, lp) < 3e-2


@pytest.mark.parametrize("M,N,K,act,kv", [(1024, 1024, 1024, None, False), (1024, 4096, 1024, "gelu", False),
                                          (4096, 1024, 1024, None, False), (2048, 4096, 1024, "gelu", False),
                                          (1024, 3072, 1024, None, True), (4096, 3072, 1024, None, True),
                                          (77, 192, 256, "gelu", False),
                                          # <= 4 rows: the GEMV (RowStats producer, RowLn / ResLn consumers)
                                          (4, 1024, 1024, None, False), (4, 4096, 1024, "gelu", False),
                                          (1, 3072, 1024, None, True), (3, 1024, 1024, "gelu", False)])
def test_gemm_row_ln_fold(gpu, M, N, K, act, kv):
    # decode LayerNorm folding (dec and 128x128 kernels): a producer GEMM writes the row
    # partials of its bf16 output (RowStats), a RowLn consumer and a ResLn consumer normalise
    # from them; against the fp32 LayerNorm-then-linear reference
    import torch.nn.functional as F

    ctx0 = _r((M, 256), gpu, 1.0, seed=60)
    w0 = _r((K, 256), gpu, 0.05, seed=59)
    b0 = _r((K,), gpu, 0.1, torch.float32, seed=58)
    res0 = _r((M, K), gpu, 2.0, seed=61) + 0.25
    part = torch.full((K // 32, M, 2), float("nan"), dtype=torch.float32, device=gpu)
    x = ops.linear(ctx0, w0, b0, residual=res0, stats_out=part)
    torch.testing.assert_close(part.cpu(), ops.row_parts_ref(x.cpu()), rtol=1e-4, atol=1e-2)
    w = _r((N, K), gpu, 0.05, seed=62)
    b = _r((N,), gpu, 0.1, torch.float32, seed=63)
    gam = 1 + _r((K,), gpu, 0.3, torch.float32, seed=64)
    bet = _r((K,), gpu, 0.2, torch.float32, seed=65)
    eps = 1e-5
    wf, cs, bf = ops.fold_ln_into_linear(w, b, gam, bet)
    xf = x.cpu().float()
    xn = F.layer_norm(xf, (K,), gam.cpu(), bet.cpu(), eps)
    ref = xn @ w.cpu().float().t() + b.cpu()
    if act == "gelu":
        ref = F.gelu(ref)
    if kv:
        d = N // 3
        T, t = 5, 3
        cache = torch.zeros((M * T, 2 * d), dtype=torch.bfloat16, device=gpu)
        step = torch.tensor([t], dtype=torch.int32, device=gpu)
        q = ops.linear(x, wf, bf, kv_cache=(cache, T, step, d), row_ln=(eps, cs, part))
        assert _rel(q, ref[:, :d]) < 2e-2
        assert _rel(cache.view(M, T, 2 * d)[:, t], ref[:, d:]) < 2e-2
    else:
        y = ops.linear(x, wf, bf, act=act, row_ln=(eps, cs, part))
        assert _rel(y, ref) < 2e-2
    # residual consumer (o-proj / FFN2 of the folded step): ctx @ Wo.T + (bo + beta) + LN(x)
    ctx = _r((M, 256), gpu, 1.0, seed=66)
    wo = _r((K, 256), gpu, 0.05, seed=67)
    bo = _r((K,), gpu, 0.1, torch.float32, seed=68)
    z = ops.linear(ctx, wo, (bo + bet).contiguous(), residual=x, res_ln=(eps, part, gam))
    zref = ctx.cpu().float() @ wo.cpu().float().t() + bo.cpu() + xn
    assert _rel(z, zref) < 2e-2


@pytest.mark.parametrize("M,K,N,act,kv", [(4, 1024, 1024, None, False), (1, 1024, 4096, "gelu", False),
                                          (3, 1024, 3072, None, True), (2, 768, 768, None, False)])
def test_gemv_row_ln_self_stats(gpu, M, K, N, act, kv):
    # <= 4 rows: the RowLn GEMV takes x's LayerNorm statistics from the rows it loads (no
    # producer partials) and hands them on (row_ln_out: totals in slot 0) to the ResLn GEMV
    # that adds LN(x) as its residual; against the fp32 LayerNorm references
    import torch.nn.functional as F

    x = _r((M, K), gpu, 2.0, seed=90) + 0.3
    w = _r((N, K), gpu, 0.05, seed=91)
    b = _r((N,), gpu, 0.1, torch.float32, seed=92)
    gam = 1 + _r((K,), gpu, 0.3, torch.float32, seed=93)
    bet = _r((K,), gpu, 0.2, torch.float32, seed=94)
    eps = 1e-5
    wf, cs, bf = ops.fold_ln_into_linear(w, b, gam, bet)
    out_parts = torch.full((K // 32, M, 2), float("nan"), dtype=torch.float32, device=gpu)
    xf = x.cpu().float()
    xn = F.layer_norm(xf, (K,), gam.cpu(), bet.cpu(), eps)
    ref = xn @ w.cpu().float().t() + b.cpu()
    if act == "gelu":
        ref = F.gelu(ref)
    if kv:
        d = N // 3
        T, t = 5, 2
        cache = torch.zeros((M * T, 2 * d), dtype=torch.bfloat16, device=gpu)
        step = torch.tensor([t], dtype=torch.int32, device=gpu)
        q = ops.linear(x, wf, bf, kv_cache=(cache, T, step, d), row_ln=(eps, cs, None), row_ln_out=out_parts)
        assert _rel(q, ref[:, :d]) < 2e-2
        assert _rel(cache.view(M, T, 2 * d)[:, t], ref[:, d:]) < 2e-2
    else:
        y = ops.linear(x, wf, bf, act=act, row_ln=(eps, cs, None), row_ln_out=out_parts)
        assert _rel(y, ref) < 2e-2
    torch.testing.assert_close(out_parts.cpu(), ops.row_totals_parts_ref(x.cpu()), rtol=1e-4, atol=1e-2)
    # the residual consumer reads the handed-on statistics (the fc1 -> fc2 shape: K = 4096 runs
    # the K-split GEMV)
    kc = N if act == "gelu" else 256
    ctx = _r((M, kc), gpu, 1.0, seed=95)
    wo = _r((K, kc), gpu, 0.05, seed=96)
    bo = _r((K,), gpu, 0.1, torch.float32, seed=97)
    z = ops.linear(ctx, wo, (bo + bet).contiguous(), residual=x, res_ln=(eps, out_parts, gam))
    zref = ctx.cpu().float() @ wo.cpu().float().t() + bo.cpu() + xn
    assert _rel(z, zref) < 2e-2


def test_bart_step_ln_fold_matches_unfolded(gpu):
    # non-trivial LayerNorm gammas / betas: the folded BART decoder step vs the layernorm +
    # linear step (GPU) and the fp32 oracle
    from agent_tpu_amd.models.bart import BartModel, config_for, init_random

    cfg = config_for("bart-tiny")
    pack = init_random(cfg, seed=2, std=0.1)
    g = torch.Generator().manual_seed(4)
    for n in pack.names():
        base = n.split(".")[-1]
        if base.startswith("ln") and base.endswith("_g"):
            pack[n].copy_(1 + 0.3 * torch.randn(pack[n].shape, generator=g))
        elif base.startswith("ln") and base.endswith("_b"):
            pack[n].copy_(0.2 * torch.randn(pack[n].shape, generator=g))
    cpu_m = BartModel(cfg, pack, fp32=True)
    gp = pack.to(gpu)
    fold_m, plain_m = BartModel(cfg, gp), BartModel(cfg, gp)
    plain_m.ln_fold = False
    assert fold_m.ln_fold
    B, S, T = 3, 16, 8
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([16, 9, 12], dtype=torch.int32)
    _, kc = cpu_m.encode(ids, lens)
    _, kg = fold_m.encode(ids.to(gpu), lens.to(gpu))
    tok = torch.randint(3, cfg.vocab_size, (B,), generator=g, dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int32)
    caches = [cpu_m.new_cache(B, T), fold_m.new_cache(B, T), plain_m.new_cache(B, T)]
    for t in range(3):
        step.fill_(t)
        lc = cpu_m.step(tok, step, caches[0], T, kc, lens, S, 1)
        lf = fold_m.step(tok.to(gpu), step.to(gpu), caches[1], T, kg, lens.to(gpu), S, 1)
        lp = plain_m.step(tok.to(gpu), step.to(gpu), caches[2], T, kg, lens.to(gpu), S, 1)
        assert _rel(lf, lc) < 5e-2 and _rel(lp, lc) < 5e-2, t
        assert _rel(lf, lp) < 3e-2, t
        tok = lc.argmax(-1).to(torch.int32)


def test_bart_step_folded_with_forced_tile(gpu):
    """with ATPU_GEMM_TILE forcing a tile kernel, <= 4-row folded BART steps must
    plan for the tile kernels (producer partials), not the GEMV (which would throw)."""
    from agent_tpu_amd._native import native
    from agent_tpu_amd.models.bart import BartModel, config_for, init_random

    cfg = config_for("bart-tiny")
    gp = init_random(cfg, seed=2, std=0.1).to(gpu)
    m = BartModel(cfg, gp)
    g = torch.Generator().manual_seed(5)
    B, S, T = 3, 16, 8
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32).to(gpu)
    lens = torch.tensor([16, 9, 12], dtype=torch.int32).to(gpu)
    _, kg = m.encode(ids, lens)
    tok = torch.randint(3, cfg.vocab_size, (B,), generator=g, dtype=torch.int32).to(gpu)
    step = torch.zeros(1, dtype=torch.int32, device=gpu)
    outs = []
    prev = native().gemm_force_tile(-1)
    for tile in (0, 128):
        native().gemm_force_tile(tile)
        try:
            assert m._gemv_path(B) == (tile == 0)
            outs.append(m.step(tok, step, m.new_cache(B, T), T, kg, lens, S, 1))
        finally:
            native().gemm_force_tile(prev)
    assert _rel(outs[1], outs[0]) < 3e-2


@pytest.mark.parametrize("M,d,rms", [(1024, 768, True), (256, 1024, False), (4096, 768, True), (77, 256, False)])
def test_gemm_kv_scatter(gpu, M, d, rms):
    # decode QKV GEMM writing K|V into the cache row m*T + step and Q into out, vs the plain GEMM
    T, t = 9, 5
    x = _r((M, d), gpu, 1.0, seed=51)
    w = _r((3 * d, d), gpu, 0.05, seed=52)
    b = None if rms else _r((3 * d,), gpu, 0.1, torch.float32, seed=53)
    cache = torch.zeros((M * T, 2 * d), dtype=torch.bfloat16, device=gpu)
    step = torch.tensor([t], dtype=torch.int32, device=gpu)
    eps = 1e-6 if rms else None
    q = ops.linear(x, w, b, rms_eps=eps, kv_cache=(cache, T, step, d))
    full = ops.linear(x, w, b, rms_eps=eps)
    assert torch.equal(q, full[:, :d])
    kv = cache.view(M, T, 2 * d)
    assert torch.equal(kv[:, t], full[:, d:])
    assert kv[:, :t].abs().sum().item() == 0 and kv[:, t + 1:].abs().sum().item() == 0


@pytest.mark.parametrize("B,nb,K2", [(7, 4, 8), (64, 4, 8), (3, 8, 16), (5, 1, 2)])
def test_beam_select_kernel(gpu, B, nb, K2):
    # device beam selection vs the host reference, with many exact score ties (the
    # (score desc, beam*V + token asc) order and the stable non-hit ranking must agree)
    V, eos = 1000, 1
    g = torch.Generator().manual_seed(B * 10 + nb)
    sc = (torch.randint(-6, 1, (B * nb, K2), generator=g).float() * 0.5).contiguous()
    tk = torch.randint(0, 40, (B * nb, K2), generator=g, dtype=torch.int32)
    tk[::3, 0] = eos
    for hit_all in (False, True):
        st_g = torch.zeros(3 * B * nb, dtype=torch.int32, device=gpu)
        rec_g = torch.zeros((B, 3 * K2 + nb), dtype=torch.int32, device=gpu)
        ops.beam_select(sc.to(gpu), tk.to(gpu), nb, V, eos, hit_all, -1e9, st_g, rec_g)
        st_c = torch.zeros(3 * B * nb, dtype=torch.int32)
        rec_c = torch.zeros((B, 3 * K2 + nb), dtype=torch.int32)
        ops.beam_select(sc, tk, nb, V, eos, hit_all, -1e9, st_c, rec_c)
        assert torch.equal(rec_g.cpu(), rec_c) and torch.equal(st_g.cpu(), st_c)
        # the record written by the kernel straight into pinned host memory (the search loop's form)
        rec_h = torch.full((B, 3 * K2 + nb), -7, dtype=torch.int32).pin_memory()
        ops.beam_select(sc.to(gpu), tk.to(gpu), nb, V, eos, hit_all, -1e9, st_g, rec_h)
        ev = torch.cuda.Event()
        ev.record()
        ev.synchronize()
        assert torch.equal(rec_h, rec_c)


@pytest.mark.parametrize("d,ln,rows", [(768, False, 4), (1024, True, 4), (1024, True, 20), (512, False, 9)])
def test_decode_advance_embeds_the_new_tokens(gpu, d, ln, rows):
    # the state advance's embedding == the stand-alone embed op at the advanced step, bit for bit
    T, V, P = 40, 3000, 140
    g = torch.Generator().manual_seed(d + rows)
    table = (torch.randn(V, d, generator=g) * 0.1).to(gpu, torch.bfloat16)
    pos = (torch.randn(P, d, generator=g) * 0.1).to(gpu, torch.bfloat16) if ln else None
    gam = (1 + 0.1 * torch.randn(d, generator=g)).to(gpu) if ln else None
    bet = (0.1 * torch.randn(d, generator=g)).to(gpu) if ln else None
    emb = ops.DecEmbed(table, pos, 2, gam, bet, 1e-5)
    hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32).to(gpu)
    par = torch.randint(0, rows, (rows,), generator=g, dtype=torch.int32).to(gpu)
    tok = torch.randint(0, V, (rows,), generator=g, dtype=torch.int32).to(gpu)
    tok[0] = V + 3  # clamped
    tokens = torch.zeros(rows, dtype=torch.int32, device=gpu)
    step = torch.tensor([7], dtype=torch.int32, device=gpu)
    h2, t2, s2 = hist.clone(), tokens.clone(), step.clone()
    out = torch.empty((rows, d), dtype=torch.bfloat16, device=gpu)
    ops.decode_advance(hist, None, par, tok, tokens, step, embed=emb, out=out)
    ops.decode_advance(h2, None, par, tok, t2, s2)
    assert torch.equal(hist, h2) and torch.equal(tokens, t2) and int(step) == 8 == int(s2)
    assert torch.equal(out, emb.apply(tokens, step))


def test_beam_select_host_record_must_be_pinned(gpu):
    sc = torch.zeros((4, 8), device=gpu)
    tk = torch.zeros((4, 8), dtype=torch.int32, device=gpu)
    st = torch.zeros(12, dtype=torch.int32, device=gpu)
    with pytest.raises(ValueError, match="pinned"):
        ops.beam_select(sc, tk, 4, 100, 1, False, -1e9, st, torch.zeros((1, 28), dtype=torch.int32))


@pytest.mark.parametrize("family", ["t5-tiny", "bart-tiny"])
def test_generate_device_select_matches_host(gpu, family):
    # the device-selection beam loop (host bookkeeping one step behind) returns exactly the
    # host-selection loop's sequences and scores (BART: n-gram bans, forced BOS/EOS)
    from agent_tpu_amd.runtime.summarize import GenConfig, build_model, generate

    model, _ = build_model(family, device=gpu, seed=3)
    g = torch.Generator().manual_seed(7)
    B, S = 5, 32
    ids = torch.randint(5, model.cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([32, 20, 31, 9, 27], dtype=torch.int32)
    for ml, nbm, mn in ((24, 4, 5), (40, 4, 5), (2, 4, 0), (3, 2, 1), (12, 1, 3)):
        a = generate(model, ids.to(gpu), lens.to(gpu), GenConfig(num_beams=nbm, max_length=ml, min_length=mn))
        b = generate(model, ids.to(gpu), lens.to(gpu),
                     GenConfig(num_beams=nbm, max_length=ml, min_length=mn, device_select=False))
        # device selection runs the fused LM head: same tokens, the log-softmax normaliser
        # summed in another order (scores to float rounding)
        assert a.sequences == b.sequences and a.steps == b.steps, (ml, nbm)
        np.testing.assert_allclose(a.scores, b.scores, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("family", ["t5-tiny", "bart-tiny"])
def test_generate_device_select_unfused_is_exact(gpu, family, monkeypatch):
    # ATPU_LM_FUSED=0: the device loop consumes the same logits + top-k kernels as the host loop
    from agent_tpu_amd.runtime import summarize
    from agent_tpu_amd.runtime.summarize import GenConfig, build_model, generate

    monkeypatch.setattr(summarize, "LM_FUSED", False)
    model, _ = build_model(family, device=gpu, seed=3)
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(5, model.cfg.vocab_size, (5, 32), generator=g, dtype=torch.int32)
    lens = torch.tensor([32, 20, 31, 9, 27], dtype=torch.int32)
    gen = dict(num_beams=4, max_length=24, min_length=5)
    a = generate(model, ids.to(gpu), lens.to(gpu), GenConfig(**gen))
    b = generate(model, ids.to(gpu), lens.to(gpu), GenConfig(**gen, device_select=False))
    assert a.sequences == b.sequences and a.scores == b.scores and a.steps == b.steps


@pytest.mark.parametrize("family", ["t5-tiny", "bart-tiny"])
def test_generate_concurrent_matches_serial(gpu, family):
    # two (or three) batches searched concurrently on their own streams, host loops
    # interleaved, return exactly what one search per batch returns
    from agent_tpu_amd.runtime.summarize import GenConfig, build_model, generate, generate_concurrent

    model, _ = build_model(family, device=gpu, seed=5)
    g = torch.Generator().manual_seed(11)
    B, S = 9, 40
    ids = torch.randint(5, model.cfg.vocab_size, (B, S), generator=g, dtype=torch.int32).to(gpu)
    lens = torch.tensor([40, 12, 33, 9, 27, 40, 3, 18, 25], dtype=torch.int32).to(gpu)
    for cuts, (ml, nbm, mn) in (((0, 4, 9), (30, 4, 5)), ((0, 2, 5, 9), (20, 2, 1)), ((0, 5, 9), (3, 4, 0))):
        gen = GenConfig(num_beams=nbm, max_length=ml, min_length=mn)
        parts = [(ids[a:b], lens[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
        ref = [generate(model, i, l, gen) for i, l in parts]
        got = generate_concurrent(model, parts, gen)
        for r, o in zip(ref, got):
            assert r.sequences == o.sequences and r.scores == o.scores and r.steps == o.steps, (cuts, ml)


@pytest.mark.parametrize("streams", [2, 3])
def test_engine_stream_split_matches_single(gpu, monkeypatch, streams):
    # SummarizeEngine.run split over two / three streams (3 is the default): same output as one search
    from agent_tpu_amd.runtime.summarize import GenConfig, SummarizeEngine, build_model

    model, _ = build_model("t5-tiny", device=gpu, seed=2)
    eng = SummarizeEngine(model, 64)
    g = torch.Generator().manual_seed(4)
    B, S = 70, 24
    ids = torch.randint(5, model.cfg.vocab_size, (B, S), generator=g, dtype=torch.int32).to(gpu)
    lens = torch.randint(2, S + 1, (B,), generator=g, dtype=torch.int32).to(gpu)
    gen = GenConfig(num_beams=4, max_length=16, min_length=2)
    monkeypatch.setenv("ATPU_SUMM_STREAMS", "1")
    a = eng.run(ids, lens, gen)
    monkeypatch.setenv("ATPU_SUMM_STREAMS", str(streams))
    monkeypatch.setenv("ATPU_SUMM_PART_MIN", "20")
    b = eng.run(ids, lens, gen)
    assert a.sequences == b.sequences and a.scores == b.scores


@pytest.mark.parametrize("family", ["t5-tiny", "bart-tiny"])
def test_decoder_graph_cache_reuse_is_exact(gpu, family, monkeypatch):
    # a second search of the same shape replays the first one's captured decoder step on the
    # same buffers (cross K/V, cache, histories reset): bit-identical to capturing per call
    from agent_tpu_amd.runtime import summarize
    from agent_tpu_amd.runtime.summarize import GenConfig, build_model, generate, slot_cache

    model, _ = build_model(family, device=gpu, seed=3)
    g = torch.Generator().manual_seed(9)
    B = 5
    gen = GenConfig(num_beams=4, max_length=20, min_length=3)
    inputs = []
    for S, lens in ((128, [128, 90, 31, 9, 127]), (100, [100, 12, 77, 64, 5]), (120, [3, 120, 40, 41, 99])):
        ids = torch.randint(5, model.cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
        inputs.append((ids, torch.tensor(lens, dtype=torch.int32)))
    monkeypatch.setattr(summarize, "GRAPH_CACHE", False)
    ref = []
    for ids, lens in inputs:  # uncached, source padded to the bucket by hand
        pad = torch.full((B, 128 - ids.shape[1]), model.cfg.pad_id, dtype=torch.int32)
        ref.append(generate(model, torch.cat([ids, pad], 1).to(gpu), lens.to(gpu), gen))
    monkeypatch.setattr(summarize, "GRAPH_CACHE", True)
    sc = slot_cache(model)
    for rnd in range(2):
        for (ids, lens), r in zip(inputs, ref):
            o = generate(model, ids.to(gpu), lens.to(gpu), gen)
            assert o.sequences == r.sequences and o.scores == r.scores and o.steps == r.steps
    assert sc.misses == 1 and sc.hits == 5 and len(sc.slots) == 1 and not sc.slots[0].busy
    # another shape (max_length) is another slot; a full cache evicts the idle LRU slot
    monkeypatch.setattr(sc, "max_slots", 1)
    generate(model, inputs[0][0].to(gpu), inputs[0][1].to(gpu), GenConfig(num_beams=4, max_length=12, min_length=3))
    assert len(sc.slots) == 1 and sc.slots[0].key[2] == 12


def test_decoder_graph_cache_concurrent_parts(gpu, monkeypatch):
    # three equal parts on three streams take three slots of one key; the next call reuses them
    from agent_tpu_amd.runtime import summarize
    from agent_tpu_amd.runtime.summarize import GenConfig, build_model, generate, generate_concurrent, slot_cache

    monkeypatch.setattr(summarize, "GRAPH_CACHE", True)
    model, _ = build_model("t5-tiny", device=gpu, seed=5)
    g = torch.Generator().manual_seed(12)
    ids = torch.randint(5, model.cfg.vocab_size, (9, 40), generator=g, dtype=torch.int32).to(gpu)
    lens = torch.tensor([40, 12, 33, 9, 27, 40, 3, 18, 25], dtype=torch.int32).to(gpu)
    gen = GenConfig(num_beams=4, max_length=16, min_length=2)
    parts = [(ids[a:a + 3], lens[a:a + 3]) for a in (0, 3, 6)]
    ref = [generate(model, i, l, gen) for i, l in parts]
    sc = slot_cache(model)
    h0 = sc.hits
    for _ in range(2):
        got = generate_concurrent(model, parts, gen)
        for r, o in zip(ref, got):
            assert r.sequences == o.sequences and r.scores == o.scores and r.steps == o.steps
    assert len(sc.slots) == 3 and sc.hits - h0 >= 3 and not any(s.busy for s in sc.slots)


@pytest.mark.parametrize("M", [1, 3, 4])
@pytest.mark.parametrize("N,K,epi", [(768, 768, "plain"), (768, 3072, "bias_res"), (3072, 768, "relu"),
                                     (4096, 1024, "bias_gelu"), (2304, 768, "rms"), (3072, 768, "rms_relu"),
                                     (1024, 1024, "res"), (1024, 4096, "bias_res"), (512, 6144, "plain")])
def test_gemv_few_rows(gpu, M, N, K, epi):
    # <= 4 rows (1 document x 4 beams) run the weight-streaming GEMV; vs the fp32 reference and
    # vs the 64x64 decode kernel (forced)
    from agent_tpu_amd._native import native

    x = _r((M, 2 * K), gpu, 1.5, seed=61)[:, :K]  # strided rows
    w = _r((N, K), gpu, 0.05, seed=62)
    b = _r((N,), gpu, 0.1, torch.float32, seed=63) if "bias" in epi else None
    res = _r((M, N), gpu, 1.0, seed=64) if "res" in epi else None
    act = "relu" if "relu" in epi else "gelu" if "gelu" in epi else None
    eps = 1e-6 if "rms" in epi else None
    if eps is not None:
        gamma = 1 + _r((K,), gpu, 0.3, torch.float32, seed=65)
        wf = ops.fold_rms_into_linear(w, gamma)
        xf = x.cpu().float()
        xin = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * gamma.cpu()
    else:
        wf, xin = w, x.cpu().float()
    y = ops.linear(x, wf, b, act=act, residual=res, rms_eps=eps)
    ref = xin @ w.cpu().float().t()
    if b is not None:
        ref = ref + b.cpu()
    ref = torch.relu(ref) if act == "relu" else torch.nn.functional.gelu(ref) if act == "gelu" else ref
    if res is not None:
        ref = ref + res.cpu().float()
    assert _rel(y, ref) < 2e-2
    prev = native().gemm_force_tile(-1)
    native().gemm_force_tile(64)
    try:
        y64 = ops.linear(x, wf, b, act=act, residual=res, rms_eps=eps)
    finally:
        native().gemm_force_tile(prev)
    assert _rel(y, y64) < 1e-2


@pytest.mark.parametrize("M,rms", [(4, True), (1, False), (3, True)])
def test_gemv_kv_scatter(gpu, M, rms):
    # decode QKV at <= 4 rows through the GEMV: K|V into cache row m*T + step, Q into out
    d, T, t = 768, 9, 4
    x = _r((M, d), gpu, 1.0, seed=71)
    w = _r((3 * d, d), gpu, 0.05, seed=72)
    b = None if rms else _r((3 * d,), gpu, 0.1, torch.float32, seed=73)
    cache = torch.zeros((M * T, 2 * d), dtype=torch.bfloat16, device=gpu)
    step = torch.tensor([t], dtype=torch.int32, device=gpu)
    eps = 1e-6 if rms else None
    q = ops.linear(x, w, b, rms_eps=eps, kv_cache=(cache, T, step, d))
    full = ops.linear(x, w, b, rms_eps=eps)
    assert torch.equal(q, full[:, :d])
    kv = cache.view(M, T, 2 * d)
    assert torch.equal(kv[:, t], full[:, d:])
    assert kv[:, :t].abs().sum().item() == 0 and kv[:, t + 1:].abs().sum().item() == 0


@pytest.mark.parametrize("rows,T,with_seq", [(4, 130, True), (4, 130, False), (8, 200, True), (1, 7, True)])
def test_decode_advance_matches_reorder_path(gpu, rows, T, with_seq):
    """The one-workgroup state advance == beam_reorder_hist + copies + add, at several steps
    (including the clamped last position)."""
    g = torch.Generator().manual_seed(rows * 1000 + T)
    for step in (0, 1, T // 2, T - 2, T - 1):
        hist = torch.randint(0, rows, (rows, T), generator=g, dtype=torch.int32)
        seq = torch.randint(0, 50000, (rows, T), generator=g, dtype=torch.int32) if with_seq else None
        par = torch.randint(0, rows, (rows,), generator=g, dtype=torch.int32)
        tok = torch.randint(0, 50000, (rows,), generator=g, dtype=torch.int32)
        st = torch.tensor([step], dtype=torch.int32)
        # reference: the multi-launch path on the CPU twin
        h_ref, s_ref = hist.clone(), (seq.clone() if with_seq else None)
        alt = torch.empty_like(h_ref)
        ops.beam_reorder_hist(h_ref, alt, par, st)
        h_ref = alt
        if with_seq:
            alt2 = torch.empty_like(s_ref)
            ops.beam_reorder_hist(s_ref, alt2, par, st, last=tok, off=1)
            s_ref = alt2
        hd, sd = hist.to(gpu), (seq.to(gpu) if with_seq else None)
        tokens = torch.zeros(rows, dtype=torch.int32, device=gpu)
        std = st.to(gpu)
        ops.decode_advance(hd, sd, par.to(gpu), tok.to(gpu), tokens, std)
        torch.cuda.synchronize()
        t = min(step, T - 1)
        assert torch.equal(hd.cpu()[:, :t + 1], h_ref[:, :t + 1]), step
        if with_seq:
            t2 = min(step + 1, T - 1)
            assert torch.equal(sd.cpu()[:, :t2 + 1], s_ref[:, :t2 + 1]), step
        assert torch.equal(tokens.cpu(), tok) and int(std.item()) == step + 1
