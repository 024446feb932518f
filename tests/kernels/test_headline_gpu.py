"""The exact headline path (bench.py) as a tested path.

ClassifyEngine at the bench configuration: BERT-base, 1024 rows x 128 tokens per batch,
two staging slots on two concurrent compute streams, hipGraph replay, LayerNorm folded
into the GEMMs, last layer on the [CLS] rows only; 4 batches (+ a ragged tail) of a
synthetic CSV through the native stager. Checked against

* a serial eager run of the SAME rows with none of those optimisations (one stream, no
  graphs, LayerNorm passes, full last layer): top-1 equal wherever the margin is clear,
  probabilities to 1e-2 on EVERY row;
* the fp32 CPU oracle (BertClassifier(fp32=True), same weights, CPU twin of the GPU
  tokenizer) on 64 sampled rows: logits within 5 % of the logit scale (no floor).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, S, NB = 1024, 128, 4


@pytest.fixture(scope="module")
def headline(tmp_path_factory):
    from agent_tpu_amd._native import native
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from agent_tpu_amd.utils.synthetic import write_csv

    dev = torch.device("cuda", 0)
    cfg = config_for("bert-base", num_labels=2)
    pack = init_random(cfg, seed=0, bias_std=0.02)
    n = NB * B + 77  # ragged tail batch
    path = write_csv(str(tmp_path_factory.mktemp("hl") / "rows.csv"), n, 150, seed=5)
    table = native().CsvTable(path)
    col = table.column_index("text")
    eng = ClassifyEngine(cfg, pack, dev, batch_rows=B, seq_len=S, topk=2, use_graph=True, slots=2)
    assert eng.concurrent and eng.use_graph and eng.model.cls_only_last and eng.model.can_fold(B, S)
    idx, sc, st = eng.classify_table(table, 0, n, col)
    torch.cuda.synchronize()
    assert st.rows == n and st.batches == NB + 1
    return dict(cfg=cfg, pack=pack, table=table, col=col, n=n, dev=dev, eng=eng, idx=idx.cpu(), sc=sc.cpu())


def test_headline_engine_vs_serial_eager_every_row(headline):
    from agent_tpu_amd.runtime.classify import ClassifyEngine

    h = headline
    # two staging slots (the stager's pipeline needs them) but ONE compute stream, eager
    ref = ClassifyEngine(h["cfg"], h["pack"], h["dev"], batch_rows=B, seq_len=S, topk=2, use_graph=False,
                         slots=2, concurrent=False)
    assert not ref.concurrent and not ref.use_graph
    ref.model.ln_fold = False
    ref.model.cls_only_last = False
    ri, rs, _ = ref.classify_table(h["table"], 0, h["n"], h["col"])
    ri, rs = ri.cpu(), rs.cpu()
    gi, gs = h["idx"], h["sc"]
    assert gi.shape == ri.shape == (h["n"], 2)
    # probabilities of both classes on every row (top-2 of 2 = the full distribution)
    p_g = torch.zeros(h["n"], 2).scatter_(1, gi.long(), gs)
    p_r = torch.zeros(h["n"], 2).scatter_(1, ri.long(), rs)
    err = (p_g - p_r).abs().max().item()
    assert err < 1e-2, err
    clear = (rs[:, 0] - rs[:, 1]) > 0.02
    assert clear.float().mean() > 0.2  # the check below covers a real share of the rows
    assert torch.equal(gi[clear, 0], ri[clear, 0])


def test_headline_engine_vs_fp32_oracle_sampled(headline):
    from agent_tpu_amd._native import native
    from agent_tpu_amd.models.bert import BertClassifier
    from agent_tpu_amd.tokenizer import DEFAULT_MAX_ROW_BYTES, pack_rows

    h = headline
    rng = np.random.default_rng(0)
    rows = np.sort(rng.choice(h["n"], 64, replace=False))
    texts = [h["table"].row(int(r))[h["col"]] for r in rows]
    text, offs = pack_rows(t.encode("utf-8")[:DEFAULT_MAX_ROW_BYTES] for t in texts)
    ids, lens = native().tokenize_host(text, offs, S, h["cfg"].vocab_size, DEFAULT_MAX_ROW_BYTES)
    oracle = BertClassifier(h["cfg"], h["pack"], fp32=True, cls_only_last=False)
    logits, _, _ = oracle.forward(torch.from_numpy(ids), torch.from_numpy(lens), k=2)
    # engine probabilities -> logit differences (2 classes: p1 = sigmoid(l1 - l0))
    p = torch.zeros(len(rows), 2).scatter_(1, h["idx"][rows].long(), h["sc"][rows])
    d_eng = torch.log(p[:, 1] / p[:, 0])
    d_ref = (logits[:, 1] - logits[:, 0]).float()
    scale = d_ref.abs().max().item()
    err = (d_eng - d_ref).abs().max().item()
    assert scale > 1e-3
    assert err < 0.05 * scale, (err, scale)
    p_ref = torch.softmax(logits.float(), -1)
    assert (p - p_ref).abs().max().item() < 1e-2
