"""Numerics of every hand-written HIP kernel vs a plain PyTorch fp32 reference.

Run on a MI355X (``pytest -m gpu``). Tolerances: bf16 I/O with fp32
accumulation -> compare relative to the output scale.
"""
import math

import numpy as np
import pytest
import torch

from agent_tpu_amd import ops
from agent_tpu_amd.ops.attention import attention_ref
from agent_tpu_amd.ops.linear import linear_ref

pytestmark = pytest.mark.gpu


def _rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def _rand(shape, dev, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dtype).to(dev)


# ------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(256, 768, 768), (300, 2304, 768), (128, 100, 64), (512, 768, 3072),
                                   (1000, 3072, 768), (4096, 768, 768), (2500, 2304, 768), (2048, 768, 3072),
                                   (3000, 3072, 768), (2304, 256, 128)])
@pytest.mark.parametrize("act,use_bias,use_res", [(None, True, False), ("gelu", True, False),
                                                  ("tanh", True, False), (None, True, True), (None, False, False)])
def test_gemm_epilogues(gpu, M, N, K, act, use_bias, use_res):
    x = _rand((M, K), gpu, seed=1)
    w = _rand((N, K), gpu, 0.05, seed=2)
    b = _rand((N,), gpu, 0.1, torch.float32, seed=3) if use_bias else None
    r = _rand((M, N), gpu, seed=4) if use_res else None
    y = ops.linear(x, w, b, act=act, residual=r)
    ref = linear_ref(x.cpu(), w.cpu(), None if b is None else b.cpu(), act, None if r is None else r.cpu())
    assert _rel_err(y, ref) < 2e-2


def test_gemm_exact_integers_asymmetric(gpu):
    # {-1,0,1} operands: every partial sum is an exact small integer in fp32 and bf16
    g = torch.Generator().manual_seed(7)
    M, N, K = 256, 384, 192
    x = torch.randint(-1, 2, (M, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-1, 2, (N, K), generator=g).to(torch.bfloat16)
    y = ops.linear(x.to(gpu), w.to(gpu)).cpu().float()
    assert torch.equal(y, x.float() @ w.float().t())
    # A = I picks rows of W^T: catches row/col swaps in the C write
    eye = torch.eye(128).to(torch.bfloat16)
    w2 = torch.arange(256 * 128).remainder(17).sub(8).view(256, 128).to(torch.bfloat16)
    y2 = ops.linear(eye.to(gpu), w2.to(gpu)).cpu().float()
    assert torch.equal(y2, w2.float().t())


def test_gemm256_exact_integers(gpu):
    # the 256x256 pipelined kernel on exact data: M not a multiple of 256, many K-tiles
    g = torch.Generator().manual_seed(8)
    M, N, K = 2600, 512, 1024
    x = torch.randint(-1, 2, (M, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-1, 2, (N, K), generator=g).to(torch.bfloat16)
    b = torch.randint(-4, 5, (N,), generator=g).float()
    r = torch.randint(-3, 4, (M, N), generator=g).to(torch.bfloat16)
    y = ops.linear(x.to(gpu), w.to(gpu), b.to(gpu), residual=r.to(gpu)).cpu().float()
    ref = (x.float() @ w.float().t() + b + r.float()).to(torch.bfloat16).float()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("variant", [1, 3, 4])  # 256p, 256l, 256n (256b / 256s: dev builds only)
@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (65536, 768, 768), (16384, 768, 3072), (4096, 3072, 64)])
def test_gemm256_variants_exact(gpu, nat, variant, M, N, K):
    # every 256x256 schedule on exact data; the persistent kernel walks several
    # tiles per workgroup here (tiles > CUs), so a mis-counted wait across the
    # tile boundary shows up as wrong tiles
    g = torch.Generator().manual_seed(9)
    x = torch.randint(-1, 2, (M, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-1, 2, (N, K), generator=g).to(torch.bfloat16)
    b = torch.randint(-4, 5, (N,), generator=g).float()
    r = torch.randint(-3, 4, (M, N), generator=g).to(torch.bfloat16)
    xg, wg, bg, rg = x.to(gpu), w.to(gpu), b.to(gpu), r.to(gpu)
    exact = (x.float() @ w.float().t() + b)
    prev = nat.gemm_256_variant(-1)
    try:
        nat.gemm_256_variant(variant)
        for _ in range(3):  # repeated launches: races are intermittent
            y = ops.linear(xg, wg, bg, residual=rg).cpu().float()
            assert torch.equal(y, (exact + r.float()).to(torch.bfloat16).float())
            y = ops.linear(xg, wg, bg).cpu().float()
            assert torch.equal(y, exact.to(torch.bfloat16).float())
        yg = ops.linear(xg, wg, bg, act="gelu").cpu().float()
        ref = torch.nn.functional.gelu(exact).to(torch.bfloat16).float()
        assert (yg - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    finally:
        nat.gemm_256_variant(prev)


@pytest.mark.parametrize("variant", [1, 4])  # 256p (per tile, A&S erf), 256n (persistent, polynomial)
def test_gemm_gelu_accuracy(gpu, nat, variant):
    # W = I: the accumulator is x exactly, so the output is bf16(gelu_epilogue(x)).
    # 3M bf16 inputs in [-8, 8]: within one bf16 ulp (+3e-5 absolute) of the exact
    # erf-GELU everywhere, and equal to bf16(exact) for nearly all |x| < 4
    M, N = 4096, 768
    x = torch.linspace(-8, 8, M * N).to(torch.bfloat16).view(M, N)
    eye = torch.eye(N).to(torch.bfloat16)
    b = torch.zeros(N)
    exact = 0.5 * x.double() * (1 + torch.erf(x.double() / math.sqrt(2)))
    prev = nat.gemm_256_variant(-1)
    try:
        nat.gemm_256_variant(variant)
        y = ops.linear(x.to(gpu), eye.to(gpu), b.to(gpu), act="gelu").cpu()
    finally:
        nat.gemm_256_variant(prev)
    ref = exact.to(torch.bfloat16)
    diff = (y.double() - exact).abs()
    ulp = ref.double().abs() * 2.0 ** -7
    assert (diff <= ulp + 3e-5).all(), diff.max().item()
    inner = x.abs() < 4
    assert (y[inner] != ref[inner]).double().mean().item() < 0.08


def test_gemm_strided_rows(gpu):
    # pooler case: A rows taken every S rows (CLS tokens) of a [B*S, H] tensor
    B, S, H = 37, 128, 768
    h = _rand((B * S, H), gpu, seed=5)
    cls = h.view(B, S, H)[:, 0, :]
    w = _rand((H, H), gpu, 0.05, seed=6)
    b = _rand((H,), gpu, 0.1, torch.float32, seed=7)
    y = ops.linear(cls, w, b, act="tanh")
    ref = linear_ref(cls.cpu(), w.cpu(), b.cpu(), "tanh")
    assert _rel_err(y, ref) < 2e-2


# -------------------------------------------------------------- attention
@pytest.mark.parametrize("B,S,H", [(3, 128, 12), (2, 64, 4), (2, 200, 2), (1, 512, 2)])
def test_attention_packed(gpu, B, S, H):
    qkv = _rand((B * S, 3 * H * 64), gpu, seed=11)
    lens = torch.tensor([S - 7 * i for i in range(B)], dtype=torch.int32).clamp(min=2)
    out = ops.attention_packed(qkv, lens.to(gpu), B, S, H)
    hd = H * 64
    qc = qkv.cpu()
    ref = attention_ref(qc[:, :hd], qc[:, hd:2 * hd], qc[:, 2 * hd:], lens, B, S, S, H, 1 / math.sqrt(64))
    assert _rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("mode", [1, 2])  # ds_bpermute / permlane row reductions
@pytest.mark.parametrize("S", [128, 64])
def test_attention_persistent_matches_per_item(gpu, nat, S, mode):
    # the persistent prefetching kernel walks several (batch, head) items per
    # workgroup here (B*H > 2 workgroups per CU), with ragged key lengths
    B, H = 96, 12
    qkv = _rand((B * S, 3 * H * 64), gpu, seed=16)
    lens = torch.randint(2, S + 1, (B,), generator=torch.Generator().manual_seed(3), dtype=torch.int32).to(gpu)
    prev = nat.attention_persist_mode(-1)
    try:
        nat.attention_persist_mode(0)
        ref = ops.attention_packed(qkv, lens, B, S, H)
        nat.attention_persist_mode(mode)
        for _ in range(3):
            out = ops.attention_packed(qkv, lens, B, S, H)
            # the persistent kernel's softmax is exp2(s*c - max*c) (FMA form), the per-item
            # kernel's exp(s*scale - max): bf16 outputs differ by rounding flips only
            assert _rel_err(out, ref) < 2e-3
    finally:
        nat.attention_persist_mode(prev)
    hd = H * 64
    qc = qkv[: 4 * S].cpu()
    r32 = attention_ref(qc[:, :hd], qc[:, hd:2 * hd], qc[:, 2 * hd:], lens[:4].cpu(), 4, S, S, H, 1 / math.sqrt(64))
    assert _rel_err(out[: 4 * S], r32) < 2e-2


def test_attention_spike_forces_rescale(gpu):
    # one huge key late in the sequence forces the online-softmax rescale branch
    B, S, H = 1, 256, 1
    qkv = _rand((B * S, 3 * 64), gpu, 0.5, seed=12).float()
    qkv[:, :64] = 1.0
    qkv[200, 64:128] = 8.0  # key 200 dominates every query in chunk 2
    qkv = qkv.to(torch.bfloat16)
    lens = torch.tensor([S], dtype=torch.int32)
    out = ops.attention_packed(qkv, lens.to(gpu), B, S, H)
    qc = qkv.cpu()
    ref = attention_ref(qc[:, :64], qc[:, 64:128], qc[:, 128:], lens, B, S, S, H, 1 / 8)
    assert _rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("causal", [False, True])
def test_attention_strided_bias_causal(gpu, causal):
    B, Sq, Skv, H = 2, 96, 160, 3
    q = _rand((B * Sq, H * 64), gpu, seed=13)
    kv = _rand((B * Skv, 2 * H * 64), gpu, seed=14)
    k, v = kv[:, :H * 64], kv[:, H * 64:]
    bias = _rand((H, Sq, Skv), gpu, 1.0, torch.float32, seed=15)
    lens = torch.tensor([Skv, 100], dtype=torch.int32)
    out = ops.attention(q, k, v, lens.to(gpu), B, Sq, Skv, H, scale=1.0, bias=bias, causal=causal)
    ref = attention_ref(q.cpu(), k.cpu(), v.cpu(), lens, B, Sq, Skv, H, 1.0, bias.cpu(), causal)
    assert _rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("B,S,H,dist", [(2, 1024, 3, True), (3, 1000, 2, True), (2, 256, 2, True),
                                        (2, 1024, 3, False), (3, 640, 2, False)])
def test_attention_flash_long(gpu, nat, B, S, H, dist):
    """Long-sequence encoder attention (double-buffered flash kernel), with the T5
    distance-indexed bias or none, ragged key lengths (a partial last chunk) vs fp32."""
    from agent_tpu_amd.ops.attention import dist_to_dense

    q = _rand((B * S, H * 64), gpu, seed=31)
    kv = _rand((B * S, 2 * H * 64), gpu, seed=32)
    k, v = kv[:, :H * 64], kv[:, H * 64:]
    bd = _rand((H, 2 * S - 1), gpu, 2.0, torch.float32, seed=33) if dist else None
    lens = torch.tensor([S - 37 * i for i in range(B)], dtype=torch.int32).clamp(min=5)
    assert nat.attention_flash_mode(-1) == 1
    out = ops.attention(q, k, v, lens.to(gpu), B, S, S, H, scale=0.125, bias_dist=bd)
    dense = dist_to_dense(bd.cpu(), S, S) if dist else None
    ref = attention_ref(q.cpu(), k.cpu(), v.cpu(), lens, B, S, S, H, 0.125, dense)
    assert _rel_err(out, ref) < 2e-2
    if not dist:  # the per-chunk kernel computes the same attention
        prev = nat.attention_flash_mode(-1)
        nat.attention_flash_mode(0)
        try:
            old = ops.attention(q, k, v, lens.to(gpu), B, S, S, H, scale=0.125)
        finally:
            nat.attention_flash_mode(prev)
        assert _rel_err(out, old) < 1e-2


def test_attention_dist_bias_matches_dense(gpu):
    """bias_dist == the same bias expanded dense (old dense-bias kernel path)."""
    from agent_tpu_amd.ops.attention import dist_to_dense

    B, S, H = 2, 384, 4
    qkv = _rand((B * S, 3 * H * 64), gpu, seed=34)
    bd = _rand((H, 2 * S - 1), gpu, 1.0, torch.float32, seed=35)
    lens = torch.tensor([S, 200], dtype=torch.int32).to(gpu)
    a = ops.attention(qkv[:, :256], qkv[:, 256:512], qkv[:, 512:], lens, B, S, S, H, scale=1.0, bias_dist=bd)
    b = ops.attention(qkv[:, :256], qkv[:, 256:512], qkv[:, 512:], lens, B, S, S, H, scale=1.0,
                      bias=dist_to_dense(bd, S, S).contiguous())
    assert _rel_err(a, b) < 1e-2


# ------------------------------------------------------------ norms/embed
@pytest.mark.parametrize("N,rows", [(256, 1000), (768, 1000), (768, 1003), (1024, 1000), (2048, 77)])
def test_layernorm_residual(gpu, N, rows):
    # rows=1003/77: the last 8-row block of the half-wave kernel is partial
    x = _rand((rows, N), gpu, 2.0, seed=21)
    r = _rand((rows, N), gpu, seed=22)
    g = _rand((N,), gpu, 1.0, torch.float32, seed=23)
    b = _rand((N,), gpu, 1.0, torch.float32, seed=24)
    y = ops.layernorm(x, g, b, 1e-12, residual=r)
    ref = torch.nn.functional.layer_norm(x.cpu().float() + r.cpu().float(), (N,), g.cpu(), b.cpu(), 1e-12)
    assert _rel_err(y, ref) < 1e-2


def test_rmsnorm(gpu):
    x = _rand((333, 768), gpu, 3.0, seed=25)
    g = _rand((768,), gpu, 1.0, torch.float32, seed=26)
    y = ops.rmsnorm(x, g, 1e-6)
    xf = x.cpu().float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * g.cpu()
    assert _rel_err(y, ref) < 1e-2


def test_embed_layernorm_and_gather(gpu):
    V, N, B, S = 1000, 768, 4, 128
    word, pos, typ = _rand((V, N), gpu, seed=31), _rand((512, N), gpu, seed=32), _rand((2, N), gpu, seed=33)
    g = _rand((N,), gpu, 1.0, torch.float32, seed=34)
    b = _rand((N,), gpu, 1.0, torch.float32, seed=35)
    ids = torch.randint(0, V, (B, S), dtype=torch.int32)
    y = ops.embed_layernorm(ids.to(gpu), word, pos, typ, g, b, 1e-12)
    ref = ops.embed_layernorm(ids, word.cpu().float(), pos.cpu().float(), typ.cpu().float(), g.cpu(), b.cpu(), 1e-12)
    assert _rel_err(y, ref) < 1e-2
    e = ops.embed_gather(ids.to(gpu), word)
    assert torch.equal(e.cpu(), word.cpu()[ids.view(-1).long()])


@pytest.mark.parametrize("N,rows,off", [(1024, 4, 2), (768, 13, 0), (1024, 64, 2)])
def test_embed_pos_layernorm_matches_the_three_op_path(gpu, N, rows, off):
    # BART's decoder input: one launch == embed_gather + position row + layernorm(residual=), bit for bit,
    # with the position index read on the device (step past the table end clamps)
    V, P = 3000, 140
    table, pos = _rand((V, N), gpu, seed=41), _rand((P, N), gpu, seed=42)
    g = _rand((N,), gpu, 1.0, torch.float32, seed=43)
    b = _rand((N,), gpu, 1.0, torch.float32, seed=44)
    ids = torch.randint(0, V, (rows,), dtype=torch.int32).to(gpu)
    ids[0] = V + 5  # clamped like embed_gather
    for st in (0, 7, P - off - 1, P + 3):
        step = torch.tensor([st], dtype=torch.int32, device=gpu)
        y = ops.embed_pos_layernorm(ids, table, pos, step, off, g, b, 1e-5)
        pr = pos[min(st + off, P - 1)].view(1, N).expand(rows, N).contiguous()
        ref = ops.layernorm(ops.embed_gather(ids, table), g, b, 1e-5, residual=pr)
        assert torch.equal(y, ref), st
        cpu = ops.embed_pos_layernorm(ids.cpu(), table.cpu(), pos.cpu(), step.cpu(), off, g.cpu(), b.cpu(), 1e-5)
        assert _rel_err(y, cpu.float()) < 1e-2


# -------------------------------------------------------------- tokenizer
def test_tokenizer_gpu_matches_python_and_host(gpu, nat):
    from agent_tpu_amd import tokenizer as T
    from agent_tpu_amd.utils.synthetic import make_text_rows

    rows = make_text_rows(300, words_per_row=40, seed=3)
    rows += ["", "   ", "Hello, WORLD!!", "x" * 100, "naïve café — 東京 ok", "a\tb\nc\x01d", "(" * 300]
    # words of every length 1..130 at every offset mod 64 (the 128-bit ballot window, the 64+
    # byte walk, 24-byte pieces), upper case, and rows of random bytes
    rng = np.random.default_rng(7)
    for L in list(range(1, 72)) + [95, 96, 97, 127, 128, 129, 130]:
        for off in (0, 1, 3, 23, 40, 61, 62, 63):
            rows.append(" " * off + "".join(chr(65 + (k * 7 + L) % 26) for k in range(L)) + ",ab " + "Q" * (L % 30))
    for _ in range(40):
        rows.append(bytes(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)).decode("latin-1"))
    text, offs = T.pack_rows(rows)
    for S in (8, 128):
        ids_py, lens_py = T.tokenize_rows([r.encode() for r in rows], S, 30522, 2048)
        ids_h, lens_h = nat.tokenize_host(text, offs, S, 30522, 2048)
        ids_g, lens_g = ops.tokenize(torch.from_numpy(text).to(gpu), torch.from_numpy(offs).to(gpu), S, 30522, 2048)
        np.testing.assert_array_equal(ids_h, ids_py)
        np.testing.assert_array_equal(lens_h, lens_py)
        np.testing.assert_array_equal(ids_g.cpu().numpy(), ids_py)
        np.testing.assert_array_equal(lens_g.cpu().numpy(), lens_py)


# ------------------------------------------------------------------- head
@pytest.mark.parametrize("C,k", [(2, 2), (10, 5), (1000, 5), (3, 1)])
def test_head_topk(gpu, C, k):
    B, N = 50, 768
    pooled = _rand((B, N), gpu, seed=41)
    Wc = _rand((C, N), gpu, 0.05, seed=42)
    bc = _rand((C,), gpu, 0.1, torch.float32, seed=43)
    logits, idx, sc = ops.classify_head_topk(pooled, Wc, bc, k)
    rl, ri, rs = ops.classify_head_topk(pooled.cpu(), Wc.cpu(), bc.cpu(), k)
    assert _rel_err(logits, rl) < 1e-3
    torch.testing.assert_close(sc.cpu(), rs, atol=2e-4, rtol=1e-3)
    # indices equal wherever the top-k scores are well separated
    gap_ok = (rs[:, :-1] - rs[:, 1:]).abs().min(dim=1).values > 1e-3 if k > 1 else torch.ones(B, dtype=torch.bool)
    assert torch.equal(idx.cpu()[gap_ok], ri[gap_ok])


def test_head_ties_lower_index_first(gpu):
    B, N, C = 2, 64, 6
    pooled = torch.zeros((B, N), dtype=torch.bfloat16, device=gpu)
    Wc = torch.zeros((C, N), dtype=torch.bfloat16, device=gpu)
    bc = torch.tensor([0.0, 1.0, 1.0, 0.5, 1.0, 0.0], device=gpu)
    _, idx, _ = ops.classify_head_topk(pooled, Wc, bc, 4)
    assert idx.cpu().tolist() == [[1, 2, 4, 3]] * 2


# ----------------------------------------------------------------- reduce
@pytest.mark.parametrize("n", [1, 1000, 3_000_001])
def test_reduce_stats(gpu, n):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g, dtype=torch.float64) * 10 + 3
    out = ops.reduce_stats_tensor(x.to(gpu)).cpu()
    assert out[0].item() == n
    assert math.isclose(out[1].item(), x.sum().item(), rel_tol=1e-12, abs_tol=1e-9)
    assert out[2].item() == x.min().item() and out[3].item() == x.max().item()
    out32 = ops.reduce_stats_tensor(x.float().to(gpu)).cpu()
    assert math.isclose(out32[1].item(), x.float().double().sum().item(), rel_tol=1e-10, abs_tol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("off,n", [(0, 1), (1, 5), (3, 1000), (1, 4099), (2, 1 << 20), (0, (1 << 21) + 3)])
def test_reduce_stats_vector_paths(gpu, dtype, off, n):
    """16-B vector body + misaligned head + tail of the K12 kernel vs fp64 torch."""
    from agent_tpu_amd.ops.reduce import reduce_stats_tensor

    g = torch.Generator().manual_seed(n)
    base = (torch.rand(off + n, generator=g, dtype=torch.float64) * 200 - 100).to(dtype)
    x = base.to(gpu)[off:]
    got = reduce_stats_tensor(x).cpu().tolist()
    ref = base[off:].double()
    assert got[0] == n
    assert abs(got[1] - float(ref.sum())) <= 1e-9 * max(1.0, float(ref.abs().sum()))
    assert got[2] == float(ref.min()) and got[3] == float(ref.max())


def test_release_gemm_ignores_ablate_env(gpu):
    """ATPU_GEMM_ABLATE=4 (skip the epilogue in a dev build) must not change a release GEMM."""
    import os
    import subprocess
    import sys

    code = ("import torch; from agent_tpu_amd import ops; g = torch.Generator().manual_seed(1); "
            "x = torch.randint(-1, 2, (4096, 768), generator=g).to(torch.bfloat16); "
            "w = torch.randint(-1, 2, (768, 768), generator=g).to(torch.bfloat16); b = torch.ones(768); "
            "y = ops.linear(x.cuda(), w.cuda(), b.cuda()).cpu().float(); "
            "print(bool(torch.equal(y, (x.float() @ w.float().t() + b).to(torch.bfloat16).float())))")
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, ATPU_GEMM_ABLATE="4")
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "True"
