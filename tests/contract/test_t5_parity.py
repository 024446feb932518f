"""T5 encoder-decoder + beam search vs transformers' T5ForConditionalGeneration.generate.

Identical random weights (bf16-rounded matrices), CPU fp32 reference path of
every op; sequences must match token for token (greedy and 4-beam, with and
without EOS pressure, min_length masking).
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from agent_tpu_amd.models.t5 import T5Model, config_for, from_hf_state_dict  # noqa: E402
from agent_tpu_amd.runtime.summarize import GenConfig, generate  # noqa: E402


def _models(eos_boost: float):
    cfg = config_for("t5-tiny")
    hc = transformers.T5Config(vocab_size=cfg.vocab_size, d_model=cfg.d_model, d_kv=64, d_ff=cfg.d_ff,
                               num_layers=cfg.enc_layers, num_decoder_layers=cfg.dec_layers, num_heads=cfg.heads,
                               relative_attention_num_buckets=32, relative_attention_max_distance=128,
                               feed_forward_proj="relu", tie_word_embeddings=True, decoder_start_token_id=0,
                               pad_token_id=0, eos_token_id=1, dropout_rate=0.0)
    torch.manual_seed(0)
    m = transformers.T5ForConditionalGeneration(hc).eval()
    sd = m.state_dict()
    g = torch.Generator().manual_seed(11)
    for k in sd:
        if sd[k].dim() == 2:
            scale = 3.0 if ("shared" in k or "relative" in k) else 1.5
            sd[k] = torch.randn(sd[k].shape, generator=g) * scale / sd[k].shape[-1] ** 0.5
            if "relative" not in k:
                sd[k] = sd[k].to(torch.bfloat16).float()
        elif "layer_norm" in k:
            sd[k] = 1 + 0.1 * torch.randn(sd[k].shape, generator=g)
    if eos_boost:
        # tilt the (tied) output embedding toward EOS so hypotheses finish
        sd["shared.weight"][1] = (sd["shared.weight"][1] * eos_boost).to(torch.bfloat16).float()
    sd["lm_head.weight"] = sd["shared.weight"]
    m.load_state_dict(sd)
    return cfg, m, T5Model(cfg, from_hf_state_dict(cfg, m.state_dict()), fp32=True)


@pytest.mark.parametrize("eos_boost", [0.0, 6.0])
@pytest.mark.parametrize("nb,max_len,min_len", [(1, 12, 0), (4, 16, 4), (4, 20, 9)])
def test_generate_matches_hf(eos_boost, nb, max_len, min_len):
    cfg, hf, ours = _models(eos_boost)
    B, S = 2, 16
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(2, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.tensor([16, 11], dtype=torch.int32)
    ids[1, 11:] = 0
    ids[0, 15] = 1
    ids[1, 10] = 1
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    with torch.no_grad():
        ref = hf.generate(input_ids=ids.long(), attention_mask=mask, num_beams=nb, max_length=max_len,
                          min_length=min_len, do_sample=False, length_penalty=1.0, early_stopping=True)
    res = generate(ours, ids, lens, GenConfig(num_beams=nb, max_length=max_len, min_length=min_len))
    for b in range(B):
        r, o = ref[b].tolist(), res.sequences[b]
        # HF fills finished rows with `pad_token_id or eos` (pad=0 is falsy -> eos)
        assert r[:len(o)] == o and all(x in (0, 1) for x in r[len(o):]), (b, r, o)
        assert len(o) >= min(min_len, max_len) or o[-1] != 1
