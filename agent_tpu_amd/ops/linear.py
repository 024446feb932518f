"""Fused linear layer on the bf16 MFMA GEMM (K3/K5/K6).

``y = act(x @ w.T + bias) + residual`` with ``w`` in ``nn.Linear.weight``
layout ``[N, K]``. Native kernel: ``csrc/kernels/gemm_bf16.hip``. Skinny
problems (decode steps, M = beams x docs) run split-K: fp32 partials in a
caching-allocator workspace, summed in slice order by a reduce kernel that
applies the epilogue.
"""
from __future__ import annotations

import functools
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev, row_stride, same_device

EPI_BIAS, EPI_GELU, EPI_TANH, EPI_RESIDUAL, EPI_RELU, EPI_OUT_F32 = 1, 2, 4, 8, 16, 32
_ACTS = {None: 0, "none": 0, "gelu": EPI_GELU, "tanh": EPI_TANH, "relu": EPI_RELU}


EPI_ROW_RMS = 512
EPI_KV_SCATTER = 1024
EPI_ROW_LN, EPI_RES_LN, EPI_ROW_STATS = 2048, 4096, 8192


def row_parts_ref(y: torch.Tensor) -> torch.Tensor:
    """[N/32, M, 2] per-row (sum, sum of squares) of ``y`` over each 32-column slab (fp32)."""
    M, N = y.shape
    t = y.float().view(M, N // 32, 32).transpose(0, 1)
    return torch.stack([t.sum(-1), (t * t).sum(-1)], -1).contiguous()


def row_ln_from_parts_ref(part: torch.Tensor, eps: float) -> torch.Tensor:
    """[M, 2] (rstd, rstd*mu) of rows of width 32 * slots from their partials (as the kernels)."""
    s = part.float().sum(0)
    K = 32 * part.shape[0]
    mu = s[:, 0] / K
    rs = torch.rsqrt((s[:, 1] / K - mu * mu).clamp_min(0.0) + eps)
    return torch.stack([rs, rs * mu], -1)


def row_totals_parts_ref(x: torch.Tensor) -> torch.Tensor:
    """The ``row_ln_out`` format: ``[K/32, M, 2]`` with each row's (sum, sum of squares) in slot 0
    and zeros elsewhere (summing the slots gives the row totals, as partials do)."""
    M, K = x.shape
    xf = x.float()
    out = torch.zeros((K // 32, M, 2), dtype=torch.float32, device=x.device)
    out[0, :, 0] = xf.sum(-1)
    out[0, :, 1] = (xf * xf).sum(-1)
    return out


def linear_ref(x, w, bias=None, act=None, residual=None, out_f32=False, rms_eps=None, row_ln=None, res_ln=None,
               stats_out=None, row_ln_out=None):
    y = x.float() @ w.float().t()
    if rms_eps is not None:
        y = y * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + rms_eps)
    if row_ln is not None:
        eps, colsum, in_part = row_ln
        st = row_ln_from_parts_ref(in_part if in_part is not None else row_totals_parts_ref(x), eps)
        y = y * st[:, :1] - st[:, 1:] * colsum.float().unsqueeze(0)
        if row_ln_out is not None:
            row_ln_out.copy_(row_totals_parts_ref(x))
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y)
    elif act == "tanh":
        y = torch.tanh(y)
    elif act == "relu":
        y = torch.relu(y)
    if residual is not None:
        r = residual.float()
        if res_ln is not None:
            eps, res_part, gamma = res_ln
            st = row_ln_from_parts_ref(res_part, eps)
            r = (r * st[:, :1] - st[:, 1:]) * gamma.float().unsqueeze(0)
        y = y + r
    y = y if out_f32 else y.to(x.dtype)
    if stats_out is not None:
        stats_out.copy_(row_parts_ref(y))
    return y


@functools.lru_cache(maxsize=4096)
def _splits_cached(M: int, N: int, K: int, inv: bool) -> int:
    return native().gemm_splitk_splits(M, N, K)


def _splits(M: int, N: int, K: int) -> int:
    return _splits_cached(M, N, K, batch_invariant())


_splits.cache_clear = _splits_cached.cache_clear  # (tools and tests re-read the split rule)


def batch_invariant() -> bool:
    """Batch-invariant kernel selection (``ATPU_BATCH_INVARIANT``; the agent turns it on): a
    row's result never depends on how many rows share its launch -- no GEMV / split-K GEMMs,
    no split cross attention or few-row self attention, no few-row LM head, and the engines
    keep batches on their folded / padded paths (docs/ARCHITECTURE.md "Batch invariance")."""
    try:
        return bool(native().batch_invariant(-1))
    except Exception:  # no extension (CPU-only oracle paths): nothing to select
        return False


def set_batch_invariant(on: bool) -> bool:
    """Switch batch-invariant selection; returns the previous setting."""
    prev = batch_invariant()
    native().batch_invariant(1 if on else 0)
    return prev


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
           residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           out_f32: bool = False, rms_eps: Optional[float] = None, kv_cache=None, row_ln=None,
           res_ln=None, stats_out: Optional[torch.Tensor] = None,
           prefetch: Optional[torch.Tensor] = None, row_ln_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual``; ``out_f32`` returns fp32 (LM-head logits).

    ``rms_eps``: ``x`` rows are raw RMSNorm inputs and ``w`` carries the norm's gamma
    (:func:`fold_rms_into_linear`): ``y = rsqrt(mean(x^2) + eps) * (x @ w.T)``, the row
    statistics summed inside the GEMM's K loop (no bias / residual with it).

    ``kv_cache = (cache, T, step, col0)`` (decode QKV): output columns ``>= col0`` (K|V)
    are written to ``cache[m*T + step, :]`` (``step`` a 1-element int32 device tensor),
    the Q columns to ``out [M, col0]``, which is returned (no kv_append pass).

    Decode LayerNorm folding (post-LN decoder steps; :func:`fold_ln_into_linear`). Row
    statistics travel as partial (sum, sumsq) per 32-column slab, ``[width/32, M, 2]`` fp32:
    ``stats_out``: write the partials of the (bf16-rounded) output rows;
    ``row_ln = (eps, colsum, in_part)``: ``x`` rows are raw LN inputs with partials ``in_part``,
    ``w``/``bias`` folded: ``y = rstd*(x @ w.T) - rstd*mu*colsum + bias``;
    ``res_ln = (eps, res_part, gamma)``: ``residual`` rows are raw LN inputs with partials
    ``res_part``, added as ``(r - mu)*rstd*gamma`` (beta folded into ``bias``).
    On <= 4 rows (the decode GEMV) a ``row_ln`` GEMV takes the statistics of ``x`` from the
    rows it reads anyway (``in_part`` may be None) and ``row_ln_out`` receives them in the
    partial format (totals in slot 0) for a later ``res_ln`` GEMV on the same rows, so no
    producer needs ``stats_out`` (its 8-wave, 32-column-slab workgroups).

    ``prefetch``: the weight of the NEXT linear of a decode chain (or ``(weight, 32)`` when that
    linear writes ``stats_out``: 32 weight rows per workgroup). A <= 4-row GEMV (or, batch-invariant,
    the <= 16-row exact kernel) pulls it into the L2 of the XCDs that will read it while it runs
    (a hint; ignored elsewhere and on CPU)."""
    check(act in _ACTS, f"unknown activation {act!r}")
    M0, N0 = x.shape[0], w.shape[0]

    def parts(t, width, name):
        check(t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == (width // 32, M0, 2),
              f"linear: {name} must be contiguous fp32 [{width // 32}, {M0}, 2]")

    if row_ln is not None:
        eps, colsum, in_part = row_ln
        check(rms_eps is None and residual is None and bias is not None and act in (None, "none", "gelu")
              and not out_f32 and stats_out is None, "linear: row_ln takes a bias, no residual, at most a GELU")
        check(eps > 0, "linear: row_ln eps must be > 0")
        check(colsum.dtype == torch.float32 and colsum.is_contiguous() and colsum.numel() == N0,
              "linear: row_ln colsum must be contiguous fp32 [N]")
        if in_part is not None:
            parts(in_part, x.shape[1], "row_ln in_part")
        else:
            check(M0 <= 4 or not x.is_cuda, "linear: row_ln without in_part runs on <= 4 rows (the GEMV) only")
        check(x.shape[1] <= 1024, "linear: row_ln rows must be <= 1024 wide")
    if row_ln_out is not None:
        check(row_ln is not None and (M0 <= 4 or not x.is_cuda), "linear: row_ln_out needs row_ln on <= 4 rows")
        parts(row_ln_out, x.shape[1], "row_ln_out")
    if res_ln is not None:
        eps, res_part, gamma = res_ln
        check(residual is not None and bias is not None and act in (None, "none") and kv_cache is None
              and rms_eps is None and row_ln is None and not out_f32, "linear: res_ln takes a bias and a residual only")
        check(eps > 0, "linear: res_ln eps must be > 0")
        parts(res_part, N0, "res_ln res_part")
        check(N0 <= 1024, "linear: res_ln rows must be <= 1024 wide")
        check(gamma.dtype == torch.float32 and gamma.is_contiguous() and gamma.numel() == N0,
              "linear: res_ln gamma must be contiguous fp32 [N]")
    if stats_out is not None:
        check(residual is not None and bias is not None and act in (None, "none") and kv_cache is None
              and rms_eps is None and not out_f32 and N0 % 32 == 0, "linear: stats_out takes a bias and a residual only")
        parts(stats_out, N0, "stats_out")
    if kv_cache is not None:
        cache, T, step, col0 = kv_cache
        N0 = w.shape[0]
        check(residual is None and act in (None, "none") and not out_f32, "linear: kv_cache takes no residual / act")
        check(0 < col0 < N0 and col0 % 128 == 0, "linear: kv_cache col0 must be a positive multiple of 128 below N")
        check(cache.dim() == 2 and cache.shape[1] >= N0 - col0 and cache.shape[0] == x.shape[0] * T
              and cache.dtype == torch.bfloat16, "linear: cache must be bf16 [M*T, >= N-col0]")
        if not x.is_cuda:
            y = linear_ref(x, w, bias, act, None, False, rms_eps, row_ln, row_ln_out=row_ln_out)
            rows = torch.arange(x.shape[0]) * T + int(step.reshape(-1)[0])
            cache[rows, :N0 - col0] = y[:, col0:]
            q = y[:, :col0]
            return out.copy_(q) if out is not None else q.contiguous()
    if rms_eps is not None:
        check(bias is None and residual is None and act in (None, "none", "relu"),
              "linear: rms_eps takes no bias / residual and only a ReLU")
        check(rms_eps > 0, "linear: rms_eps must be > 0")
    if not x.is_cuda:
        y = linear_ref(x, w, bias, act, residual, out_f32, rms_eps, row_ln, res_ln, stats_out, row_ln_out)
        if out is not None:
            out.copy_(y)
            return out
        return y
    check_bf16_dev(x, "x")
    check_bf16_dev(w, "w")
    same_device(x, w, bias, residual, out)
    M, K = x.shape
    N, K2 = w.shape
    check(K == K2, f"inner dims differ: x {tuple(x.shape)} w {tuple(w.shape)}")
    lda, ldb = row_stride(x, "x"), row_stride(w, "w")
    epi = _ACTS[act]
    if bias is not None:
        check(bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N, "bias must be fp32 [N]")
        epi |= EPI_BIAS
    ldr = 0
    if residual is not None:
        check_bf16_dev(residual, "residual")
        check(tuple(residual.shape) == (M, N), "residual must be [M, N]")
        ldr = row_stride(residual, "residual")
        epi |= EPI_RESIDUAL
    if out_f32:
        epi |= EPI_OUT_F32
    odt = torch.float32 if out_f32 else torch.bfloat16
    NC = kv_cache[3] if kv_cache is not None else N  # columns that land in ``out``
    if out is None:
        out = torch.empty((M, NC), dtype=odt, device=x.device)
    check(tuple(out.shape) == (M, NC) and out.dtype == odt, "out must be [M, N] of the output dtype")
    ldc = row_stride(out, "out")
    kv_args = ()
    if kv_cache is not None:
        cache, T, step, col0 = kv_cache
        same_device(x, cache, step)
        check(step.dtype == torch.int32, "linear: kv step must be an int32 device tensor")
        epi |= EPI_KV_SCATTER
        kv_args = (ptr(cache), row_stride(cache, "cache"), int(T), int(col0), ptr(step))
    ln_args = [0, 0, 0, 0, 0]  # colsum, in_part, res_part, gamma, part_out
    eps_arg = float(rms_eps or 0.0)
    if row_ln is not None:
        eps, colsum, in_part = row_ln
        same_device(x, colsum)
        epi |= EPI_ROW_LN
        eps_arg = float(eps)
        ln_args[0], ln_args[1] = ptr(colsum), ptr(in_part)
        if row_ln_out is not None:
            same_device(x, row_ln_out)
            ln_args[4] = ptr(row_ln_out)
    if res_ln is not None:
        eps, res_part, gamma = res_ln
        same_device(x, res_part, gamma)
        epi |= EPI_RES_LN
        eps_arg = float(eps)
        ln_args[2], ln_args[3] = ptr(res_part), ptr(gamma)
    if stats_out is not None:
        same_device(x, stats_out)
        epi |= EPI_ROW_STATS
        ln_args[4] = ptr(stats_out)
    if rms_eps is not None or kv_cache is not None or row_ln is not None or res_ln is not None or stats_out is not None:
        if rms_eps is not None:
            epi |= EPI_ROW_RMS
        splits = 1
    else:
        splits = _splits(M, N, K)
    ws = torch.empty(splits * M * N, dtype=torch.float32, device=x.device) if splits > 1 else None
    if not kv_args:
        kv_args = (0, 0, 0, 0, 0)
    pf_args = (0, 0, 0, 0, 16)
    if prefetch is not None and M <= 16:  # the <= 4-row GEMV and the batch-invariant few-row kernel
        pw, rpb = prefetch if isinstance(prefetch, tuple) else (prefetch, 16)
        if pw.is_cuda and pw.dim() == 2 and pw.stride(1) == 1:
            pf_args = (ptr(pw), pw.stride(0), pw.shape[1], pw.shape[0], int(rpb))
    native().gemm(ptr(x), lda, ptr(w), ldb, ptr(out), ldc, ptr(bias), ptr(residual), ldr, M, N, K, epi,
                  launch_stream(x), splits, ptr(ws), eps_arg, *kv_args, *ln_args, *pf_args)
    return out


def fold_rms_into_linear(w: torch.Tensor, gamma: torch.Tensor) -> torch.Tensor:
    """``RMSNorm(x; gamma) @ w.T == rstd(x) * (x @ (w * gamma).T)``: the folded weight (``w``'s dtype)."""
    return (w.float() * gamma.float().unsqueeze(0)).to(w.dtype).contiguous()


# ---------------------------------------------------------------- LayerNorm folding
# A post-LN encoder's LayerNorm never materialised (kernel: gemm256s with the
# kEpiInNorm / kEpiResNorm / kEpiStatsOut epilogues, csrc/kernels/gemm_bf16.hip):
#   producer (attention out-proj, FFN2):  C = raw pre-LN sum, plus per-row partial
#       (sum, sumsq) of C for each 256-column tile          -> part  [N/256, M, 2]
#   ln_finalize (norm_embed.hip): part -> (rstd, rstd*mu)    -> fin   [M, 2]
#   consumer of LN(x) as GEMM input (QKV, FFN1):  gamma folded into the weight,
#       beta into the bias:  LN(x).W^T = rstd*(x.W'^T) - rstd*mu*colsum(W') + b'
#   consumer of LN(x) as the residual (out-proj, FFN2 of the next step):
#       + (x*rstd - rstd*mu)*gamma, beta folded into the bias
EPI_IN_NORM, EPI_RES_NORM, EPI_STATS_OUT = 64, 128, 256


def ln_partials_ref(y: torch.Tensor) -> torch.Tensor:
    """[N/256, M, 2] per-row (sum, sum of squares) of ``y`` over each 256-column tile (fp32)."""
    M, N = y.shape
    t = y.float().view(M, N // 256, 256).transpose(0, 1)
    return torch.stack([t.sum(-1), (t * t).sum(-1)], -1).contiguous()


def ln_finalize(part: torch.Tensor, K: int, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[M, 2] (rstd, rstd*mu) of rows of width K from their StatsOut partials ``part [slots, M, 2]``."""
    slots, M, two = part.shape
    check(two == 2 and part.dtype == torch.float32 and part.is_contiguous(), "part must be contiguous fp32 [S, M, 2]")
    if out is None:
        out = torch.empty((M, 2), dtype=torch.float32, device=part.device)
    check(tuple(out.shape) == (M, 2) and out.dtype == torch.float32 and out.is_contiguous(), "out must be fp32 [M, 2]")
    if not part.is_cuda:
        s = part.sum(0)
        mu = s[:, 0] * (1.0 / K)
        rs = torch.rsqrt((s[:, 1] * (1.0 / K) - mu * mu).clamp_min(0.0) + eps)
        return out.copy_(torch.stack([rs, rs * mu], -1))
    same_device(part, out)
    native().ln_stats_finalize(ptr(part), slots, M, int(K), float(eps), ptr(out), launch_stream(part))
    return out


def fold_ln_into_linear(w: torch.Tensor, b: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor):
    """``LN(x) @ w.T + b == rstd*(x @ w_f.T) - rstd*mu*colsum + b_f`` -> ``(w_f, colsum fp32, b_f fp32)``.

    ``colsum`` is taken over the (bf16-rounded) ``w_f`` the GEMM multiplies with."""
    wf = (w.float() * gamma.float().unsqueeze(0)).to(w.dtype)
    colsum = wf.float().sum(1).contiguous()
    # w @ beta as a broadcast product + row sum, not a GEMV: a torch matmul here was the
    # first rocBLAS call of the process (~100 ms of library initialisation on a cold load)
    bf = (b.float() + (w.float() * beta.float().unsqueeze(0)).sum(1)).contiguous()
    return wf.contiguous(), colsum, bf


def fold_ok(M: int, N: int, K: int) -> bool:
    """Shapes (and GEMM build) the LN-folding epilogues support."""
    if M % 256 or N % 256 or K % 256 or M < 2048:
        return False
    try:
        return native().gemm_256_variant(-1) >= 3
    except Exception:
        return False


def linear_ln(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, *, act: Optional[str] = None,
              in_fin: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None,
              residual: Optional[torch.Tensor] = None, res_fin: Optional[torch.Tensor] = None,
              res_gamma: Optional[torch.Tensor] = None, part_out: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Linear layer of a LayerNorm-folded encoder (see the block comment above).

    * ``in_fin [M, 2]`` (+ ``colsum``): ``x`` holds raw LN inputs whose (rstd, rstd*mu)
      are ``in_fin``; ``w``/``bias`` are folded (:func:`fold_ln_into_linear`).
    * ``res_fin`` + ``res_gamma``: ``residual`` holds raw LN inputs; the bias carries beta.
    * ``part_out [N/256, M, 2]``: row partials of the output (fp32, before bf16 rounding).
    """
    in_norm, res_norm = in_fin is not None, res_fin is not None
    check(act in (None, "gelu"), f"linear_ln: activation {act!r} not supported")
    check(not (in_norm and (res_norm or part_out is not None or residual is not None)),
          "linear_ln: an input-normalising GEMM has no residual / output statistics")
    check(not res_norm or residual is not None, "linear_ln: res_fin needs a residual")
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:
        y = x.float() @ w.float().t()
        if in_norm:
            y = y * in_fin[:, :1] - in_fin[:, 1:] * colsum.float().unsqueeze(0)
        y = y + bias.float()
        if act == "gelu":
            y = F.gelu(y)
        if residual is not None:
            r = residual.float()
            if res_norm:
                r = (r * res_fin[:, :1] - res_fin[:, 1:]) * res_gamma.float().unsqueeze(0)
            y = y + r
        if part_out is not None:
            part_out.copy_(ln_partials_ref(y))
        y = y.to(x.dtype)
        return out.copy_(y) if out is not None else y
    check_bf16_dev(x, "x")
    check_bf16_dev(w, "w")
    same_device(x, w, bias, residual, in_fin, colsum, res_fin, res_gamma, part_out, out)
    check(w.shape[1] == K, f"inner dims differ: x {tuple(x.shape)} w {tuple(w.shape)}")
    check(fold_ok(M, N, K), f"linear_ln: unsupported shape M={M} N={N} K={K} (needs multiples of 256, M >= 2048)")

    def f32(t, shape, name):
        check(t is not None and t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == tuple(shape),
              f"linear_ln: {name} must be contiguous fp32 {list(shape)}")

    f32(bias, (N,), "bias")
    epi = EPI_BIAS | (EPI_GELU if act == "gelu" else 0)
    if in_norm:
        f32(in_fin, (M, 2), "in_fin")
        f32(colsum, (N,), "colsum")
        epi |= EPI_IN_NORM
    ldr = 0
    if residual is not None:
        check_bf16_dev(residual, "residual")
        check(tuple(residual.shape) == (M, N), "residual must be [M, N]")
        ldr = row_stride(residual, "residual")
        epi |= EPI_RESIDUAL
    if res_norm:
        f32(res_fin, (M, 2), "res_fin")
        f32(res_gamma, (N,), "res_gamma")
        epi |= EPI_RES_NORM
    if part_out is not None:
        f32(part_out, (N // 256, M, 2), "part_out")
        epi |= EPI_STATS_OUT
    check(epi in (EPI_BIAS | EPI_IN_NORM, EPI_BIAS | EPI_IN_NORM | EPI_GELU,
                  EPI_BIAS | EPI_RESIDUAL | EPI_STATS_OUT, EPI_BIAS | EPI_RESIDUAL | EPI_RES_NORM | EPI_STATS_OUT),
          f"linear_ln: unsupported epilogue combination {epi}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    check(tuple(out.shape) == (M, N) and out.dtype == torch.bfloat16, "out must be bf16 [M, N]")
    native().gemm_ln(ptr(x), row_stride(x, "x"), ptr(w), row_stride(w, "w"), ptr(out), row_stride(out, "out"),
                     ptr(bias), ptr(residual), ldr, M, N, K, epi, ptr(in_fin), ptr(colsum), ptr(res_fin),
                     ptr(res_gamma), ptr(part_out), launch_stream(x))
    return out
