"""BART encoder-decoder + beam search vs transformers' BartForConditionalGeneration.generate.

The reference summarizer (``/root/reference/ops/map_summarize.py:53-59``) is
BART-large-CNN, whose generation config adds no_repeat_ngram_size=3,
length_penalty=2.0, forced_bos_token_id=0 and forced_eos_token_id=2 to the
call's num_beams/max_length/min_length/early_stopping. Identical random
weights (bf16-rounded matrices), CPU fp32 reference path of every op;
sequences must match HF token for token. A "hot" token set makes hypotheses
repeat so the n-gram bans are exercised.
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from agent_tpu_amd.models.bart import BartModel, config_for, from_hf_state_dict  # noqa: E402
from agent_tpu_amd.runtime.summarize import GenConfig, generate, ngram_bans  # noqa: E402


def _models(eos_boost: float, hot: float):
    cfg = config_for("bart-tiny")
    hc = transformers.BartConfig(vocab_size=cfg.vocab_size, d_model=cfg.d_model, encoder_layers=cfg.enc_layers,
                                 decoder_layers=cfg.dec_layers, encoder_attention_heads=cfg.heads,
                                 decoder_attention_heads=cfg.heads, encoder_ffn_dim=cfg.d_ff,
                                 decoder_ffn_dim=cfg.d_ff, max_position_embeddings=cfg.max_positions,
                                 activation_function="gelu", scale_embedding=False, dropout=0.0,
                                 attention_dropout=0.0, activation_dropout=0.0, pad_token_id=1, bos_token_id=0,
                                 eos_token_id=2, decoder_start_token_id=2, forced_bos_token_id=0,
                                 forced_eos_token_id=2, tie_word_embeddings=True)
    torch.manual_seed(0)
    m = transformers.BartForConditionalGeneration(hc).eval()
    sd = m.state_dict()
    g = torch.Generator().manual_seed(5)
    for k in sd:
        t = sd[k]
        if t.dim() == 2:
            scale = 2.0 if ("shared" in k or "embed" in k) else 1.2
            sd[k] = (torch.randn(t.shape, generator=g) * scale / t.shape[-1] ** 0.5).to(torch.bfloat16).float()
        elif k.endswith("layer_norm.weight") or k.endswith("layernorm_embedding.weight"):
            sd[k] = 1 + 0.1 * torch.randn(t.shape, generator=g)
        elif t.dim() == 1 and "bias" in k:
            sd[k] = 0.05 * torch.randn(t.shape, generator=g)
    flb = torch.zeros(1, cfg.vocab_size)
    if hot:
        flb[0, 100:108] = hot  # a few favoured tokens -> repeated n-grams
    if eos_boost:
        flb[0, 2] = eos_boost
    sd["final_logits_bias"] = flb
    sd["lm_head.weight"] = sd["model.shared.weight"]
    sd["model.encoder.embed_tokens.weight"] = sd["model.shared.weight"]
    sd["model.decoder.embed_tokens.weight"] = sd["model.shared.weight"]
    m.load_state_dict(sd)
    return cfg, m, BartModel(cfg, from_hf_state_dict(cfg, m.state_dict()), fp32=True)


@pytest.mark.parametrize("eos_boost,hot", [(0.0, 0.0), (0.0, 9.0), (7.0, 6.0)])
@pytest.mark.parametrize("nb,max_len,min_len", [(1, 14, 0), (4, 18, 5), (4, 24, 10)])
def test_generate_matches_hf(eos_boost, hot, nb, max_len, min_len):
    cfg, hf, ours = _models(eos_boost, hot)
    B, S = 2, 16
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([16, 11], dtype=torch.int32)
    ids[:, 0] = 0
    ids[0, 15] = 2
    ids[1, 10] = 2
    ids[1, 11:] = 1
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    kw = dict(num_beams=nb, max_length=max_len, min_length=min_len, do_sample=False, early_stopping=True,
              length_penalty=2.0, no_repeat_ngram_size=3, forced_bos_token_id=0, forced_eos_token_id=2,
              decoder_start_token_id=2)
    with torch.no_grad():
        ref = hf.generate(input_ids=ids.long(), attention_mask=mask, **kw)
    res = generate(ours, ids, lens, GenConfig(num_beams=nb, max_length=max_len, min_length=min_len))
    for b in range(B):
        r, o = ref[b].tolist(), res.sequences[b]
        assert r[:len(o)] == o and all(x == 1 for x in r[len(o):]), (b, r, o)
        assert o[0] == 2 and o[1] == 0  # decoder start, forced BOS


def test_ngram_bans_vectorized():
    seq = torch.tensor([[2, 0, 5, 6, 7, 5, 6], [2, 0, 1, 2, 3, 4, 5], [2, 0, 9, 9, 9, 9, 9]])
    r, t = ngram_bans(seq, 3)
    got = sorted(zip(r.tolist(), t.tolist()))
    assert got == [(0, 7), (2, 9), (2, 9), (2, 9)]
    r, t = ngram_bans(seq[:, :2], 3)
    assert r.numel() == 0
