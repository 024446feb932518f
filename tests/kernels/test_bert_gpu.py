"""End-to-end BERT classify on the GPU vs the fp32 CPU oracle (same weights)."""
import pytest
import torch

from agent_tpu_amd.models.bert import BertClassifier, config_for, init_random
from agent_tpu_amd.runtime.classify import ClassifyEngine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,B,S", [("bert-tiny", 8, 128), ("bert-base", 4, 128), ("bert-base", 3, 64)])
def test_bert_gpu_vs_fp32_oracle(gpu, preset, B, S):
    cfg = config_for(preset, num_labels=7)
    pack = init_random(cfg, seed=3, bias_std=0.02)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    ids[:, 0] = 101
    lens = torch.tensor([S - 5 * i for i in range(B)], dtype=torch.int32).clamp(min=2)
    oracle = BertClassifier(cfg, pack, fp32=True)
    rl, ri, rs = oracle.forward(ids, lens, k=3)
    dev = BertClassifier(cfg, pack.to(gpu))
    gl, gi, gs = dev.forward(ids.to(gpu), lens.to(gpu), k=3)
    err = (gl.cpu() - rl).abs().max().item()
    assert err < 0.05 * rl.abs().max().item(), err
    # top-1 must agree where the oracle's margin is clear
    margin = rs[:, 0] - rs[:, 1]
    ok = margin > 0.02
    assert torch.equal(gi.cpu()[ok, 0], ri[ok, 0])


def test_engine_table_graph_vs_eager_vs_texts(gpu, tmp_path, nat):
    from agent_tpu_amd.utils.synthetic import write_csv

    cfg = config_for("bert-tiny", num_labels=5)
    pack = init_random(cfg, seed=0)
    path = write_csv(str(tmp_path / "rows.csv"), 300, words_per_row=60, seed=9)
    table = nat.CsvTable(path)
    col = table.column_index("text")
    eng_g = ClassifyEngine(cfg, pack, gpu, batch_rows=64, seq_len=128, topk=3, use_graph=True)
    eng_e = ClassifyEngine(cfg, pack, gpu, batch_rows=64, seq_len=128, topk=3, use_graph=False)
    ig, sg, st = eng_g.classify_table(table, 10, 250, col)
    ie, se, _ = eng_e.classify_table(table, 10, 250, col)
    assert st.rows == 250 and st.batches == 4
    assert torch.equal(ig.cpu(), ie.cpu())
    torch.testing.assert_close(sg.cpu(), se.cpu())
    # same rows through the in-memory text path
    import csv
    with open(path, newline="", encoding="utf-8") as f:
        rows = [r["text"] for r in csv.DictReader(f)][10:260]
    res = eng_e.classify_texts(rows)
    assert torch.equal(res.idx, ie.cpu())


def test_cls_only_last_layer_matches_full(gpu):
    """Pruned last layer ([CLS] rows only) == full last layer, on the GPU and vs the CPU oracle."""
    import torch

    from agent_tpu_amd.models.bert import BertClassifier, config_for, init_random

    cfg = config_for("bert-base", num_labels=4)
    pack = init_random(cfg, seed=3, bias_std=0.02)
    B, S = 16, 128
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(1000, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    lens = torch.randint(8, S + 1, (B,), generator=g, dtype=torch.int32)
    ids[torch.arange(S).view(1, S) >= lens.view(B, 1)] = 0
    dev = pack.to(gpu)
    pruned = BertClassifier(cfg, dev, cls_only_last=True)
    full = BertClassifier(cfg, dev, cls_only_last=False)
    lp, ip, pp = pruned.forward(ids.to(gpu), lens.to(gpu), 4)
    lf, if_, pf = full.forward(ids.to(gpu), lens.to(gpu), 4)
    assert (lp - lf).abs().max().item() < 3e-2 * lf.abs().max().item()
    oracle = BertClassifier(cfg, pack, fp32=True, cls_only_last=False)
    lo, _, _ = oracle.forward(ids, lens, 4)
    assert (lp.cpu() - lo).abs().max().item() < 5e-2 * lo.abs().max().item()


def test_bert_base_production_batch(gpu, nat):
    """The bench shape (B=64, S=128: M=8192 rows) runs the persistent GEMM and
    persistent attention kernels; compare against the per-tile GEMM + per-item
    attention kernels on the same batch, and against the fp32 oracle."""
    cfg = config_for("bert-base", num_labels=5)
    pack = init_random(cfg, seed=11, bias_std=0.02)
    B, S = 64, 128
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(1000, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    ids[:, 0] = 101
    lens = torch.randint(16, S + 1, (B,), generator=g, dtype=torch.int32)
    ids[torch.arange(S).view(1, S) >= lens.view(B, 1)] = 0
    dev = BertClassifier(cfg, pack.to(gpu))
    gl, gi, gs = dev.forward(ids.to(gpu), lens.to(gpu), k=3)
    pv, pa = nat.gemm_256_variant(-1), nat.attention_persist_mode(-1)
    try:
        nat.gemm_256_variant(1)
        nat.attention_persist_mode(0)
        bl, bi, bs = dev.forward(ids.to(gpu), lens.to(gpu), k=3)
    finally:
        nat.gemm_256_variant(pv)
        nat.attention_persist_mode(pa)
    # two bf16 pipelines 12 layers apart in rounding (LN-folded GEMMs + fused QKV/attention vs
    # unfolded per-tile GEMMs + separate LayerNorms + per-item attention; one GELU since round 6)
    assert (gl - bl).abs().max().item() < 5e-2 * bl.abs().max().item()
    margin = bs[:, 0] - bs[:, 1]
    ok = margin > 0.02
    assert torch.equal(gi[ok, 0], bi[ok, 0])
    oracle = BertClassifier(cfg, pack, fp32=True)
    rl, _, _ = oracle.forward(ids[:4], lens[:4], k=3)
    assert (gl[:4].cpu() - rl).abs().max().item() < 5e-2 * rl.abs().max().item()
