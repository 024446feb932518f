"""LayerNorm folding algebra (CPU reference path of ops.linear_ln, the oracle of the GPU epilogues).

A post-LN encoder never materialises its LayerNorms on the GPU: producers emit row
partial (sum, sumsq), consumers apply (rstd, mu) to folded weights or to the residual.
These tests pin the algebra in fp32 against the plain LayerNorm formulation.
"""
import torch
import torch.nn.functional as F

from agent_tpu_amd import ops
from agent_tpu_amd.models.bert import BertClassifier, config_for, init_random


def _ln(x, g, b, eps):
    return F.layer_norm(x, (x.shape[1],), g, b, eps)


def test_partials_and_finalize_match_layernorm_stats():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 768, generator=g) * 3 + 0.5
    part = ops.ln_partials_ref(x)
    assert part.shape == (3, 64, 2)
    fin = ops.ln_finalize(part, 768, 1e-12)
    mu, var = x.mean(1), x.var(1, unbiased=False)
    torch.testing.assert_close(fin[:, 0], torch.rsqrt(var + 1e-12), rtol=1e-4, atol=0)
    torch.testing.assert_close(fin[:, 1], torch.rsqrt(var + 1e-12) * mu, rtol=1e-4, atol=1e-6)


def test_input_norm_fold_equals_ln_then_linear():
    g = torch.Generator().manual_seed(1)
    M, K, N, eps = 32, 512, 256, 1e-12
    x = torch.randn(M, K, generator=g) * 2 + 1.0
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    gam = 1 + 0.2 * torch.randn(K, generator=g)
    bet = 0.1 * torch.randn(K, generator=g)
    ref = _ln(x, gam, bet, eps) @ w.t() + b
    wf, colsum, bf = ops.fold_ln_into_linear(w, b, gam, bet)
    fin = ops.ln_finalize(ops.ln_partials_ref(x), K, eps)
    y = ops.linear_ln(x, wf, bf, in_fin=fin, colsum=colsum)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    yg = ops.linear_ln(x, wf, bf, act="gelu", in_fin=fin, colsum=colsum)
    torch.testing.assert_close(yg, F.gelu(ref), rtol=1e-4, atol=1e-4)


def test_residual_norm_and_stats_out():
    g = torch.Generator().manual_seed(2)
    M, K, N, eps = 16, 256, 512, 1e-5
    ctx = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    r = torch.randn(M, N, generator=g) * 1.5 - 0.3  # raw pre-LN residual stream
    gam = 1 + 0.2 * torch.randn(N, generator=g)
    bet = 0.1 * torch.randn(N, generator=g)
    fin = ops.ln_finalize(ops.ln_partials_ref(r), N, eps)
    part = torch.empty(N // 256, M, 2)
    y = ops.linear_ln(ctx, w, b + bet, residual=r, res_fin=fin, res_gamma=gam, part_out=part)
    ref = ctx @ w.t() + b + _ln(r, gam, bet, eps)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(part, ops.ln_partials_ref(ref), rtol=1e-4, atol=1e-3)


def test_folded_encoder_equals_layernorm_encoder_fp32():
    """The whole folded BERT encoder (CPU fp32) == the LayerNorm encoder, incl. the
    [CLS]-only last layer, with non-trivial LN gamma/beta."""
    cfg = config_for("bert-tiny", num_labels=3)  # hidden 256, intermediate 1024
    pack = init_random(cfg, seed=5, bias_std=0.02)
    g = torch.Generator().manual_seed(7)
    for name in pack.names():
        if name.endswith("_g"):
            pack[name].copy_(1 + 0.1 * torch.randn(pack[name].shape, generator=g))
        elif name.endswith("ln_b") or name.endswith("ln1_b") or name.endswith("ln2_b"):
            pack[name].copy_(0.05 * torch.randn(pack[name].shape, generator=g))
    m = BertClassifier(cfg, pack, fp32=True)
    B, S = 4, 32
    ids = torch.randint(1000, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([32, 20, 9, 32], dtype=torch.int32)
    for cls_only in (False, True):
        ref = m.encode(ids, lens, cls_only_last=cls_only)
        got = m.encode_folded(ids, lens, cls_only_last=cls_only)
        torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-4)


def test_decode_row_ln_and_res_ln_equal_ln_then_linear():
    # decode LayerNorm folding (ops.linear stats_out / row_ln / res_ln, the BART decoder
    # step): the producer writes per-32-column row partials, both consumers normalise from them
    g = torch.Generator().manual_seed(7)
    M, K, N = 12, 256, 96
    ctx0, W0, b0 = torch.randn(M, 64, generator=g), torch.randn(K, 64, generator=g) * 0.05, torch.zeros(K)
    res = torch.randn(M, K, generator=g) * 2 + 0.3
    part = torch.empty(K // 32, M, 2)
    x = ops.linear(ctx0, W0, b0, residual=res, stats_out=part)  # producer of the raw rows
    torch.testing.assert_close(part.sum(0)[:, 0], x.sum(1), rtol=1e-5, atol=1e-4)
    gam, bet = 1 + 0.3 * torch.randn(K, generator=g), 0.2 * torch.randn(K, generator=g)
    w, b = torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g) * 0.1
    wf, cs, bf = ops.fold_ln_into_linear(w, b, gam, bet)
    y = ops.linear(x, wf, bf, act="gelu", row_ln=(1e-5, cs, part))
    torch.testing.assert_close(y, F.gelu(_ln(x, gam, bet, 1e-5) @ w.t() + b), rtol=1e-4, atol=1e-4)
    # residual consumer: ctx @ Wo.T + bo + LN(x), with beta in the bias
    Wo, bo = torch.randn(K, 64, generator=g) * 0.05, torch.randn(K, generator=g) * 0.1
    ctx = torch.randn(M, 64, generator=g)
    z = ops.linear(ctx, Wo, bo + bet, residual=x, res_ln=(1e-5, part, gam))
    torch.testing.assert_close(z, ctx @ Wo.t() + bo + _ln(x, gam, bet, 1e-5), rtol=1e-4, atol=1e-4)


def test_bart_folded_decoder_step_equals_unfolded():
    from agent_tpu_amd.models.bart import BartModel, config_for as bart_config, init_random as bart_init

    cfg = bart_config("bart-tiny")
    pack = bart_init(cfg, seed=2, std=0.1)
    g = torch.Generator().manual_seed(4)
    for n in pack.names():  # non-trivial LayerNorm gammas and betas
        base = n.split(".")[-1]
        if base.startswith("ln") and base.endswith("_g"):
            pack[n].copy_(1 + 0.3 * torch.randn(pack[n].shape, generator=g))
        elif base.startswith("ln") and base.endswith("_b"):
            pack[n].copy_(0.2 * torch.randn(pack[n].shape, generator=g))
    plain, fold = BartModel(cfg, pack, fp32=True), BartModel(cfg, pack, fp32=True)
    fold.ln_fold = True
    assert not plain.ln_fold
    B, S, T = 3, 16, 8
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([16, 9, 12], dtype=torch.int32)
    _, kv = plain.encode(ids, lens)
    tok = torch.randint(3, cfg.vocab_size, (B,), generator=g, dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int32)
    c1, c2 = plain.new_cache(B, T), fold.new_cache(B, T)
    for t in range(3):
        step.fill_(t)
        l1 = plain.step(tok, step, c1, T, kv, lens, S, 1)
        l2 = fold.step(tok, step, c2, T, kv, lens, S, 1)
        torch.testing.assert_close(l2, l1, rtol=1e-4, atol=1e-4)
        tok = l1.argmax(-1).to(torch.int32)


def test_decode_ln_fold_argument_checks():
    import pytest

    M, K = 4, 64
    x, w, b = torch.randn(M, K), torch.randn(32, K), torch.zeros(32)
    cs, part = torch.zeros(32), torch.zeros(K // 32, M, 2)
    with pytest.raises(ValueError, match="row_ln in_part"):
        ops.linear(x, w, b, row_ln=(1e-5, cs, torch.zeros(1, M, 2)))
    with pytest.raises(ValueError, match="row_ln takes a bias"):
        ops.linear(x, w, None, row_ln=(1e-5, cs, part))
    with pytest.raises(ValueError, match="res_ln takes a bias and a residual"):
        ops.linear(x, w, b, res_ln=(1e-5, torch.zeros(1, M, 2), torch.ones(32)))
    with pytest.raises(ValueError, match="stats_out"):
        ops.linear(x, w, b, residual=torch.zeros(M, 32), stats_out=torch.zeros(2, M, 2, dtype=torch.float64))
    wide = torch.randn(M, 2048)
    with pytest.raises(ValueError, match="<= 1024"):
        ops.linear(wide, torch.randn(32, 2048), b, row_ln=(1e-5, cs, torch.zeros(64, M, 2)))
