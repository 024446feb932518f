"""The wave-specialised GEMM (csrc/kernels/qkv_attn_ws.hip modes 3 / 4; ops.linear.gemm_ws):
BERT's FFN1 (InNorm-folded input, bias, GELU) and the plain input-normalising GEMM against an
fp32 PyTorch reference of the same op and against the 256 x 256 production kernel, at odd
tile counts, both K (768: 12 K-tiles, 1024: 16) and every schedule variant. Dev build only."""
import pytest
import torch
import torch.nn.functional as F

from agent_tpu_amd import ops
from agent_tpu_amd.ops.linear import gemm_ws, ws_gemm_ok


@pytest.fixture(autouse=True)
def _dev_build_only(request):
    """The ws kernels are compiled in the dev build only (measured slower than release)."""
    if request.node.get_closest_marker("gpu"):
        from agent_tpu_amd._native import native

        if not native().DEV_BUILD:
            pytest.skip("wave-specialised kernels: dev build of the extension only (build.py --dev)")


def _case(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(M, K, generator=g) * 1.5 + 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.04).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    xf = x.float()
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-12)
    fin = torch.stack([rstd, rstd * xf.mean(1)], 1).contiguous()
    col = w.float().sum(1).contiguous()
    pre = (xf @ w.float().t()) * fin[:, :1] - fin[:, 1:] * col.unsqueeze(0) + b
    return x, w, b, fin, col, pre


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,gelu", [(128 * 37, 3072, 768, True), (128 * 37, 1536, 768, False),
                                        (4096, 3072, 768, True), (128 * 5, 4032, 1024, True)])
def test_gemm_ws_matches_fp32(M, N, K, gelu):
    dev = torch.device("cuda", 0)
    x, w, b, fin, col, pre = _case(M, N, K, M + N)
    assert ws_gemm_ok(M, N, K)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    gemm_ws(x.to(dev), w.to(dev), b.to(dev), out, gelu=gelu, in_fin=fin.to(dev), colsum=col.to(dev))
    torch.cuda.synchronize()
    # reference of the same op: the pre-activation rounded to bf16 (the image), GELU in fp32
    ref = pre.to(torch.bfloat16).float()
    if gelu:
        ref = F.gelu(ref)
    got = out.float().cpu()
    assert torch.isfinite(got).all()
    err = ((got - ref).abs() / (ref.abs() + 1.0)).max().item()
    assert err < 1.6e-2, err


@pytest.mark.gpu
def test_gemm_ws_matches_production_ffn1(monkeypatch):
    """linear_ln with ATPU_GEMM_WS=1 routes FFN1 to the ws kernel; it agrees with the 256 x 256
    kernel to ~2 bf16 ulps (GELU of the bf16-rounded pre-activation vs of the fp32 one)."""
    dev = torch.device("cuda", 0)
    M, N, K = 8192, 3072, 768
    x, w, b, fin, col, _ = _case(M, N, K, 5)
    args = (x.to(dev), w.to(dev), b.to(dev))
    kw = dict(act="gelu", in_fin=fin.to(dev), colsum=col.to(dev))
    monkeypatch.setenv("ATPU_GEMM_WS", "0")
    ref = ops.linear_ln(*args, **kw)
    monkeypatch.setenv("ATPU_GEMM_WS", "1")
    got = ops.linear_ln(*args, **kw)
    torch.cuda.synchronize()
    d = (got.float() - ref.float()).abs()
    assert d.max().item() <= 2.0 ** -6 * max(ref.float().abs().max().item(), 1.0), d.max().item()
    assert d.mean().item() < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("var", [1, 8, 24, 72, 104])
def test_gemm_ws_schedule_variants_exact(var):
    from agent_tpu_amd._native import native

    dev = torch.device("cuda", 0)
    M, N, K = 128 * 67, 3072, 768
    x, w, b, fin, col, _ = _case(M, N, K, 9)
    xd, wd, bd, fd, cd = x.to(dev), w.to(dev), b.to(dev), fin.to(dev), col.to(dev)
    nat = native()
    old = nat.ws_variant(-1)
    try:
        nat.ws_variant(0)
        ref = gemm_ws(xd, wd, bd, torch.empty(M, N, dtype=torch.bfloat16, device=dev), gelu=True, in_fin=fd, colsum=cd)
        nat.ws_variant(var)
        got = gemm_ws(xd, wd, bd, torch.empty(M, N, dtype=torch.bfloat16, device=dev), gelu=True, in_fin=fd, colsum=cd)
        torch.cuda.synchronize()
    finally:
        nat.ws_variant(old)
    assert torch.equal(got, ref)
