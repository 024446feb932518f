"""CPU twins of the decoder-input ops (the GPU kernels are checked against them bit for bit in
tests/kernels/test_decode_gpu.py and tests/kernels/test_kernels_gpu.py)."""
import torch
import torch.nn.functional as F

from agent_tpu_amd import ops


def _tables(V=50, P=20, d=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    table = (torch.randn(V, d, generator=g) * 0.1).bfloat16()
    pos = (torch.randn(P, d, generator=g) * 0.1).bfloat16()
    gam, bet = 1 + 0.1 * torch.randn(d, generator=g), 0.1 * torch.randn(d, generator=g)
    return table, pos, gam, bet


def test_embed_pos_layernorm_cpu_is_token_plus_position_layernorm():
    table, pos, gam, bet = _tables()
    ids = torch.tensor([3, 0, 49, 70, -2], dtype=torch.int32)  # out-of-range ids clamp
    for st, off in ((0, 2), (5, 2), (30, 2), (4, 0)):
        y = ops.embed_pos_layernorm(ids, table, pos, torch.tensor([st], dtype=torch.int32), off, gam, bet, 1e-5)
        x = table.float()[ids.long().clamp(0, 49)] + pos.float()[min(st + off, 19)]
        ref = F.layer_norm(x, (64,), gam, bet, 1e-5).bfloat16()
        assert torch.equal(y, ref), (st, off)


def test_decode_advance_cpu_writes_the_next_input():
    table, pos, gam, bet = _tables()
    rows, T = 4, 12
    hist = torch.arange(rows * T, dtype=torch.int32).view(rows, T) % rows
    par = torch.tensor([1, 1, 0, 3], dtype=torch.int32)
    tok = torch.tensor([5, 6, 7, 8], dtype=torch.int32)
    for emb in (ops.DecEmbed(table), ops.DecEmbed(table, pos, 2, gam, bet, 1e-5)):
        tokens = torch.zeros(rows, dtype=torch.int32)
        step = torch.tensor([3], dtype=torch.int32)
        out = torch.empty(rows, 64, dtype=torch.bfloat16)
        ops.decode_advance(hist.clone(), None, par, tok, tokens, step, embed=emb, out=out)
        assert torch.equal(tokens, tok) and int(step) == 4
        if emb.gamma is None:
            assert torch.equal(out, table[tok.long()])
        else:
            ref = ops.embed_pos_layernorm(tok, table, pos, step, 2, gam, bet, 1e-5)
            assert torch.equal(out, ref)
