"""BERT oracle vs transformers ``BertForSequenceClassification`` with identical
random-init weights: logits of our fp32 reference path —
the same graph the HIP kernels implement (tests/kernels/test_bert_gpu.py pins
GPU vs this oracle) — equal HF's on CPU."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from agent_tpu_amd.models.bert import BertClassifier, config_for, from_hf_state_dict  # noqa: E402


@pytest.mark.parametrize("labels,k", [(3, 3), (7, 5)])
def test_logits_match_hf(labels, k):
    hcfg = transformers.BertConfig(vocab_size=4096, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                   intermediate_size=1024, max_position_embeddings=512, type_vocab_size=2,
                                   num_labels=labels, hidden_act="gelu", layer_norm_eps=1e-12,
                                   attn_implementation="eager")
    torch.manual_seed(labels)
    hf = transformers.BertForSequenceClassification(hcfg).eval()
    with torch.no_grad():
        for p in hf.parameters():  # our pack stores bf16 weights: give HF the same values
            p.copy_(p.bfloat16().float())
    cfg = config_for("bert-tiny", num_labels=labels)
    ours = BertClassifier(cfg, from_hf_state_dict(cfg, hf.state_dict()), fp32=True)
    B, S = 4, 64
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, 4096, (B, S), generator=g)
    lens = torch.tensor([64, 40, 7, 2])
    mask = (torch.arange(S).view(1, S) < lens.view(B, 1)).long()
    ids = ids * mask
    ids[:, 0] = 101
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).logits
        logits, idx, prob = ours.forward(ids.to(torch.int32), lens.to(torch.int32), k)
    torch.testing.assert_close(logits.float(), ref, atol=2e-4, rtol=1e-4)
    p_ref = torch.softmax(ref, -1)
    top = torch.topk(p_ref, k, -1)
    torch.testing.assert_close(prob.float(), top.values, atol=1e-4, rtol=1e-4)
    assert torch.equal(idx.long(), top.indices)
