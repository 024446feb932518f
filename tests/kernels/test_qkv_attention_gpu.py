"""Fused QKV projection + attention (csrc/kernels/qkv_attn.hip) against
* an fp32 PyTorch reference of the same op (projection in fp32, attention_ref), and
* the unfused production path (QKV GEMM + packed attention kernel),
with ragged sequence lengths, the plain and the LayerNorm-folded (InNorm) input, and grids of
one to several persistent tiles per CU. The 256 x 192 GEMM alone (mode 0) is checked too.
"""
import math

import pytest
import torch

from agent_tpu_amd import ops
from agent_tpu_amd.ops.attention import attention_ref

H, D, K = 12, 64, 768


def _case(B, seed, innorm):
    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda", 0)
    M = B * 128
    x = (torch.randn(M, K, generator=g) * 1.5 + 0.2).to(torch.bfloat16)
    w = (torch.randn(3 * H * D, K, generator=g) * 0.04).to(torch.bfloat16)
    b = torch.randn(3 * H * D, generator=g) * 0.1
    lens = torch.randint(1, 129, (B,), generator=g, dtype=torch.int32)
    lens[0] = 128
    if B > 1:
        lens[1] = 1
    fin = col = None
    if innorm:
        xf = x.float()
        rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-12)
        fin = torch.stack([rstd, rstd * xf.mean(1)], 1).contiguous()
        col = w.float().sum(1).contiguous()
    return dev, M, x, w, b, lens, fin, col


def _ref(x, w, b, lens, fin, col, B):
    y = x.float() @ w.float().t()
    if fin is not None:
        y = y * fin[:, :1] - fin[:, 1:] * col.unsqueeze(0)
    qkv = (y + b).to(torch.bfloat16)
    hd = H * D
    return attention_ref(qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:], lens, B, 128, 128, H,
                         1.0 / math.sqrt(D)).float()


@pytest.mark.gpu
@pytest.mark.parametrize("B,innorm", [(2, False), (2, True), (32, True), (130, False), (258, True)])
def test_fused_matches_fp32_reference(B, innorm):
    dev, M, x, w, b, lens, fin, col = _case(B, 10 + B, innorm)
    p = ops.qkv_head_order(H)
    w_h, b_h = w[p].contiguous(), b[p].contiguous()
    col_h = col[p].contiguous() if innorm else None
    got = ops.qkv_attention(x.to(dev), w_h.to(dev), b_h.to(dev), lens.to(dev), H,
                            in_fin=fin.to(dev) if innorm else None, colsum_h=col_h.to(dev) if innorm else None)
    torch.cuda.synchronize()
    ref = _ref(x, w, b, lens, fin, col, B)
    err = (got.float().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert scale > 1e-2
    assert err < 2e-2 * max(scale, 1.0), (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("innorm", [False, True])
def test_fused_matches_unfused_kernels(innorm):
    B = 64
    dev, M, x, w, b, lens, fin, col = _case(B, 3, innorm)
    xd, wd, bd, ld = x.to(dev), w.to(dev), b.to(dev), lens.to(dev)
    if innorm:
        qkv = ops.linear_ln(xd, wd, bd, in_fin=fin.to(dev), colsum=col.to(dev))
    else:
        qkv = ops.linear(xd, wd, bd)
    ref = ops.attention_packed(qkv, ld, B, 128, H)
    p = ops.qkv_head_order(H, dev)
    got = ops.qkv_attention(xd, wd[p].contiguous(), bd[p].contiguous(), ld, H,
                            in_fin=fin.to(dev) if innorm else None,
                            colsum_h=col.to(dev)[p].contiguous() if innorm else None)
    torch.cuda.synchronize()
    # same bf16 QKV rounding on both sides up to accumulation order; the fused kernel normalises
    # by the sum of the bf16-rounded P (an MFMA row sum), the unfused one by the fp32 sum: the
    # contexts differ by at most ~2 bf16 ulps of the largest magnitude
    err = (got.float() - ref.float()).abs().max().item()
    assert err <= 2.0 ** -7 * ref.float().abs().max().item(), err
    assert (got.float() - ref.float()).abs().mean().item() < 1e-3


def test_cpu_reference_path_matches_unfused():
    """The CPU path of ops.qkv_attention (un-permutes the head-ordered weights); no GPU."""
    B = 2
    _, M, x, w, b, lens, fin, col = _case(B, 7, True)
    p = ops.qkv_head_order(H)
    got = ops.qkv_attention(x, w[p], b[p], lens, H, in_fin=fin, colsum_h=col[p])
    ref = _ref(x, w, b, lens, fin, col, B)
    assert (got.float() - ref).abs().max().item() < 1e-2


@pytest.mark.gpu
def test_fused_bert_large_shape():
    """16 heads, hidden 1024 (K / 64 = 16): the bert-large encoder runs the fused kernel too."""
    Hl, Kl, B = 16, 1024, 34
    g = torch.Generator().manual_seed(21)
    dev = torch.device("cuda", 0)
    M = B * 128
    x = (torch.randn(M, Kl, generator=g) * 1.2).to(torch.bfloat16)
    w = (torch.randn(3 * Hl * D, Kl, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(3 * Hl * D, generator=g) * 0.1
    lens = torch.randint(1, 129, (B,), generator=g, dtype=torch.int32)
    xf = x.float()
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-12)
    fin = torch.stack([rstd, rstd * xf.mean(1)], 1).contiguous()
    col = w.float().sum(1).contiguous()
    assert ops.qkv_attention_ok(M, 3 * Hl * D, Kl, 128)
    p = ops.qkv_head_order(Hl)
    got = ops.qkv_attention(x.to(dev), w[p].contiguous().to(dev), b[p].contiguous().to(dev), lens.to(dev), Hl,
                            in_fin=fin.to(dev), colsum_h=col[p].contiguous().to(dev))
    torch.cuda.synchronize()
    y = (xf @ w.float().t()) * fin[:, :1] - fin[:, 1:] * col.unsqueeze(0) + b
    qkv = y.to(torch.bfloat16)
    hd = Hl * D
    ref = attention_ref(qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:], lens, B, 128, 128, Hl, 1.0 / math.sqrt(D)).float()
    err = (got.float().cpu() - ref).abs().max().item()
    assert err < 2e-2 * max(ref.abs().max().item(), 1.0), err


@pytest.mark.gpu
def test_gemm256h_store_mode_exact():
    """Mode 0 of the 256 x 192 persistent GEMM: C = A.Bt^T + bias against fp32."""
    from agent_tpu_amd._native import native

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    M, N = 8192, 2304
    a = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    native().gemm256h(a.data_ptr(), K, w.data_ptr(), K, c.data_ptr(), N, b.data_ptr(), M, N, K, 1, 0, 0, 0,
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t() + b
    err = ((c.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
    assert err < 1.6e-2, err
