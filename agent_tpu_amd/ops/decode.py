"""Seq2seq decode ops (K9-K11). Native kernels: ``csrc/kernels/decode.hip``.

* :func:`decode_attention` — one query row per (row, head) vs a KV cache
  (self: the row's cache up to step t, optionally through beam backpointers
  ``hist``; cross: the encoder K/V of batch item ``row // group`` masked by its
  source length, one workgroup per item so beams share the K/V stream),
  optional T5 distance bias.
* :func:`kv_append` — write step t's K/V into the cache (t on device).
* :func:`beam_reorder_hist` — beam reorder of the backpointer table.
* :func:`gather_rows` — explicit beam reorder of cache slabs.
* :func:`beam_topk_rows` — log-softmax + beam score (+ EOS mask) + top-k per row.
* :func:`lm_head_topk` — the LM-head GEMM fused with :func:`beam_topk_rows`
  (``csrc/kernels/lm_head.hip``): no fp32 logits in HBM.
"""
from __future__ import annotations

import math
from typing import NamedTuple, Optional, Tuple

import numpy as np

import torch

from .._native import native, ptr, launch_stream
from ._util import check, check_bf16_dev, row_stride, same_device

HEAD_DIM = 64


def decode_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, H: int, seq_stride: int, group: int = 1,
                     lens: Optional[torch.Tensor] = None, step: Optional[torch.Tensor] = None,
                     bias_dist: Optional[torch.Tensor] = None, scale: float = 1.0,
                     out: Optional[torch.Tensor] = None, hist: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q [R, >=H*64]; k/v 2-D row views with ``seq_stride`` rows per sequence.

    ``hist`` (int32 [R, T], self attention only): key j < t of row r lives in
    the cache of row ``hist[r, j]``.
    """
    R = q.shape[0]
    if not q.is_cuda:
        return _decode_attention_ref(q, k, v, H, seq_stride, group, lens, step, bias_dist, scale, out, hist)
    check_bf16_dev(q, "q")
    check_bf16_dev(k, "k")
    check(lens is not None or step is not None, "need lens or step")
    if bias_dist is not None:
        check(bias_dist.dtype == torch.float32 and bias_dist.is_contiguous() and bias_dist.dim() == 2,
              "bias_dist must be fp32 [H, T]")
    if hist is not None:
        check(lens is None and group == 1, "hist is for self attention (group 1)")
        check(hist.dtype == torch.int32 and hist.is_contiguous() and hist.shape[0] == R, "hist must be int32 [R, T]")
    out = torch.empty((R, H * HEAD_DIM), dtype=torch.bfloat16, device=q.device) if out is None else out
    # few items: the keys are split over workgroups (flash decoding) into this workspace
    # (allocated per call: concurrent searches on other streams never share it; inside a
    # captured decoder step it comes from the graph's pool)
    nws = native().decode_attention_ws_floats(R, group, H, seq_stride, lens is not None and hist is None)
    ws = torch.empty(nws, dtype=torch.float32, device=q.device) if nws else None
    native().decode_attention(ptr(q), row_stride(q, "q"), ptr(k), ptr(v), row_stride(k, "k"), seq_stride, group,
                              ptr(lens), ptr(step), ptr(hist), 0 if hist is None else hist.shape[1], ptr(bias_dist),
                              0 if bias_dist is None else bias_dist.shape[1], ptr(out), row_stride(out, "out"), R, H,
                              float(scale), launch_stream(q), ptr(ws))
    return out


def _decode_attention_ref(q, k, v, H, seq_stride, group, lens, step, bias_dist, scale, out, hist=None):
    R = q.shape[0]
    D = HEAD_DIM
    res = torch.zeros((R, H * D), dtype=torch.float32)
    for r in range(R):
        s = r // group
        n = int(lens[s]) if lens is not None else int(step.reshape(-1)[0]) + 1
        if hist is not None:
            src_rows = torch.cat([hist[r, :n - 1].long().cpu(), torch.tensor([r])])
            rows_idx = src_rows * seq_stride + torch.arange(n)
            kk = k[rows_idx, :H * D].float().view(n, H, D)
            vv = v[rows_idx, :H * D].float().view(n, H, D)
        else:
            kk = k[s * seq_stride:s * seq_stride + n, :H * D].float().view(n, H, D)
            vv = v[s * seq_stride:s * seq_stride + n, :H * D].float().view(n, H, D)
        qq = q[r, :H * D].float().view(H, D) * scale
        sc = torch.einsum("hd,nhd->hn", qq, kk)
        if bias_dist is not None:
            dist = (n - 1 - torch.arange(n))
            sc = sc + bias_dist.float()[:, dist]
        p = torch.softmax(sc, dim=-1)
        res[r] = torch.einsum("hn,nhd->hd", p, vv).reshape(-1)
    y = res.to(q.dtype)
    return out.copy_(y) if out is not None else y


def kv_append(src: torch.Tensor, col0: int, ncols: int, cache: torch.Tensor, seq_stride: int,
              step: torch.Tensor) -> None:
    """cache rows (r*seq_stride + t) <- src[r, col0:col0+ncols]; cache is 2-D [R*seq_stride, ncols]."""
    R = src.shape[0]
    if not src.is_cuda:
        t = int(step.reshape(-1)[0])
        cache.view(R, seq_stride, -1)[:, t, :ncols] = src[:, col0:col0 + ncols]
        return
    native().kv_append(ptr(src), row_stride(src, "src"), col0, ncols, ptr(cache), seq_stride,
                       row_stride(cache, "cache"), ptr(step), R, launch_stream(src))


def beam_reorder_hist(src: torch.Tensor, dst: torch.Tensor, parent: torch.Tensor, step: torch.Tensor,
                      last: Optional[torch.Tensor] = None, off: int = 0) -> None:
    """dst[r, :t] = src[parent[r], :t]; dst[r, t] = last[r] if given else parent[r];
    t = step + off (clamped to T - 1); [R, T] int32. Cache backpointers: last None, off 0;
    token histories: last = the new tokens, off 1."""
    R, T = src.shape
    if not src.is_cuda:
        t = min(int(step.reshape(-1)[0]) + off, T - 1)
        pl = parent.long().cpu()
        dst[:, :t] = src[pl, :t]
        dst[:, t] = (last if last is not None else parent).to(dst.dtype)
        return
    check(src.dtype == torch.int32 and dst.dtype == torch.int32 and parent.dtype == torch.int32,
          "hist/parent must be int32")
    check(src.is_contiguous() and dst.is_contiguous() and tuple(dst.shape) == (R, T), "hist must be contiguous [R, T]")
    check(last is None or (last.dtype == torch.int32 and last.is_cuda and last.numel() >= R), "last: int32 [R] on device")
    native().beam_reorder_hist(ptr(src), ptr(dst), ptr(parent), R, T, ptr(step), launch_stream(src),
                               ptr(last) if last is not None else 0, int(off))


def decode_advance_ok(rows: int, T: int, seq: bool) -> bool:
    """The one-workgroup :func:`decode_advance` takes this beam batch (<= 64 KiB of LDS)."""
    return rows * T * 4 * (2 if seq else 1) <= 64 * 1024


def decode_advance(hist: torch.Tensor, seq: Optional[torch.Tensor], parent: torch.Tensor, tok: torch.Tensor,
                   tokens: torch.Tensor, step: torch.Tensor, embed: Optional[DecEmbed] = None,
                   out: Optional[torch.Tensor] = None) -> None:
    """A small beam search's per-step state advance in ONE launch, in place: ``hist`` reordered
    by ``parent`` (:func:`beam_reorder_hist`, t = step), ``seq`` likewise with the new tokens
    (off 1), ``tokens = tok``, ``step += 1`` (replaces 2 reorders, 3 copies and an add).

    ``embed`` (a model's :class:`DecEmbed`) with ``out`` [rows, d]: the same launch also writes
    the new tokens' decoder input into ``out`` (the next step's embedding launch folded in):
    ``table[tok]`` or, with a LayerNorm, ``LN(table[tok] + pos[step + pos_off])`` at the
    advanced step -- bit for bit :func:`embed_gather` / :func:`embed_pos_layernorm`."""
    R, T = hist.shape
    if not hist.is_cuda:
        alt = torch.empty_like(hist)
        beam_reorder_hist(hist, alt, parent, step)
        hist.copy_(alt)
        if seq is not None:
            alt = torch.empty_like(seq)
            beam_reorder_hist(seq, alt, parent, step, last=tok, off=1)
            seq.copy_(alt)
        tokens.copy_(tok)
        step.add_(1)
        if embed is not None:
            out.copy_(embed.apply(tokens, step))
        return
    for t, n in ((hist, "hist"), (parent, "parent"), (tok, "tok"), (tokens, "tokens"), (step, "step")):
        check(t.dtype == torch.int32 and t.is_cuda and t.is_contiguous(), f"decode_advance: {n} must be int32 on device")
    check(seq is None or (seq.dtype == torch.int32 and tuple(seq.shape) == (R, T) and seq.is_contiguous()),
          "decode_advance: seq must be int32 [R, T]")
    check(decode_advance_ok(R, T, seq is not None), "decode_advance: batch too large for one workgroup")
    if embed is None:
        native().decode_advance(ptr(hist), ptr(seq), R, T, ptr(parent), ptr(tok), ptr(tokens), ptr(step),
                                launch_stream(hist))
        return
    V, d = embed.table.shape
    check(embed.table.is_cuda and embed.table.dtype == torch.bfloat16 and embed.table.is_contiguous(),
          "decode_advance: embedding table must be contiguous bf16 on device")
    check(out is not None and tuple(out.shape) == (R, d) and out.dtype == torch.bfloat16 and out.is_contiguous(),
          f"decode_advance: out must be bf16 [{R}, {d}]")
    check(d in (512, 768, 1024), "decode_advance: embedding width 512 / 768 / 1024")
    if embed.gamma is not None:
        check(embed.gamma.dtype == torch.float32 and embed.gamma.numel() == d and embed.beta is not None
              and embed.beta.numel() == d, "decode_advance: fp32 gamma / beta [d]")
    if embed.pos is not None:
        check(embed.pos.dtype == torch.bfloat16 and embed.pos.is_contiguous() and embed.pos.shape[1] == d,
              "decode_advance: positions bf16 [P, d]")
    native().decode_advance(ptr(hist), ptr(seq), R, T, ptr(parent), ptr(tok), ptr(tokens), ptr(step),
                            launch_stream(hist), ptr(embed.table), V, d, ptr(embed.pos), int(embed.pos_off),
                            embed.pos.shape[0] if embed.pos is not None else 0, ptr(embed.gamma), ptr(embed.beta),
                            float(embed.eps), ptr(out))


class DecEmbed:
    """A decoder's input embedding, for :func:`decode_advance` to produce the next step's input:
    ``table[tok]`` (T5), or ``LN(table[tok] + pos[step + pos_off])`` with ``gamma`` (BART)."""

    def __init__(self, table: torch.Tensor, pos: Optional[torch.Tensor] = None, pos_off: int = 0,
                 gamma: Optional[torch.Tensor] = None, beta: Optional[torch.Tensor] = None, eps: float = 0.0):
        self.table, self.pos, self.pos_off, self.gamma, self.beta, self.eps = table, pos, pos_off, gamma, beta, eps

    def apply(self, tokens: torch.Tensor, step: torch.Tensor) -> torch.Tensor:
        """The same input through the stand-alone ops (the models' own path)."""
        from .norm import embed_gather, embed_pos_layernorm

        if self.gamma is None:
            return embed_gather(tokens, self.table)
        return embed_pos_layernorm(tokens, self.table, self.pos, step, self.pos_off, self.gamma, self.beta, self.eps)


def gather_rows(src: torch.Tensor, dst: torch.Tensor, parent: torch.Tensor, nrows: int, seq_stride: int,
                step: torch.Tensor, slabs: int = 1) -> None:
    """dst[slab, r, :t+1] = src[slab, parent[r], :t+1]; tensors [slabs, nrows*seq_stride, C]."""
    if not src.is_cuda:
        t = int(step.reshape(-1)[0]) + 1
        s4 = src.view(slabs, nrows, seq_stride, -1)
        dst.view(slabs, nrows, seq_stride, -1)[:, :, :t] = s4[:, parent.long(), :t]
        return
    check(parent.dtype == torch.int32 and parent.is_cuda, "parent must be int32 on device")
    C = src.shape[-1]
    native().gather_rows(ptr(src), ptr(dst), ptr(parent), nrows, seq_stride, C, ptr(step), slabs,
                         nrows * seq_stride * C, launch_stream(src))


MAX_BANS = 512  # banned tokens per row the kernel filters (decode.hip kMaxBans)


def ngram_bans(seq: torch.Tensor, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """HF NoRepeatNGramLogitsProcessor for every row of ``seq`` [R, cur] at once.

    Returns ``(rows, tokens)``: token t is banned for row r when the row's last
    n-1 tokens followed by t already occur in the row.
    """
    R, cur = seq.shape
    if n <= 0 or cur + 1 < n or cur < n:
        return torch.empty(0, dtype=torch.long), torch.empty(0, dtype=torch.long)
    if n == 1:
        rows = torch.arange(R).repeat_interleave(cur)
        return rows, seq.reshape(-1)
    ng = seq.unfold(1, n, 1)  # [R, cur-n+1, n]
    prefix = seq[:, cur - n + 1:]  # [R, n-1]
    match = (ng[:, :, :n - 1] == prefix.unsqueeze(1)).all(-1)
    r, c = match.nonzero(as_tuple=True)
    return r, ng[r, c, n - 1]


def beam_topk_rows(logits: torch.Tensor, beam_scores: torch.Tensor, k: int, eos: int, mask_eos: bool,
                   bans: Optional[torch.Tensor] = None,
                   ngram: Optional[Tuple[torch.Tensor, int, int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per row: top-k of ``log_softmax(logits) + beam_score`` (EOS masked if asked).

    ``bans`` (int32 ``[R, nb]``, -1 padded): token ids excluded from row r's selection
    (no-repeat-n-gram processor; the log-softmax normaliser still covers every token).
    ``ngram = (seq, cur, n)``: the same processor computed in the kernel from the
    device token history ``seq`` (int32 ``[R, T]``, the first ``cur`` columns valid)."""
    R, V = logits.shape
    nbmax = 0 if bans is None else int(bans.shape[1])
    if not logits.is_cuda:
        lp = torch.log_softmax(logits.float(), dim=-1)
        if mask_eos:
            lp[:, eos] = float("-inf")
        if nbmax:
            b = bans.to(torch.int64).cpu()
            r = torch.arange(R).view(-1, 1).expand_as(b)
            ok = b >= 0
            lp[r[ok], b[ok]] = float("-inf")
        if ngram is not None:
            seq, cur, n = ngram
            br, bt = ngram_bans(seq[:, :cur].cpu().long(), int(n))
            lp[br, bt] = float("-inf")
        lp = lp + beam_scores.float().view(-1, 1)
        sc, idx = torch.topk(lp, k, dim=-1)
        return sc, idx.to(torch.int32)
    check(logits.dtype == torch.float32 and logits.is_contiguous(), "logits must be contiguous fp32")
    if nbmax:
        check(nbmax <= MAX_BANS, f"beam_topk_rows: at most {MAX_BANS} banned tokens per row")
        check(bans.dtype == torch.int32 and bans.is_contiguous() and bans.shape[0] == R and bans.device == logits.device,
              "bans must be contiguous int32 [R, n] on the logits' device")
    sc = torch.empty((R, k), dtype=torch.float32, device=logits.device)
    idx = torch.empty((R, k), dtype=torch.int32, device=logits.device)
    seq_p, seq_stride, cur, n = 0, 0, 0, 0
    if ngram is not None:
        seq, cur, n = ngram
        check(seq.dtype == torch.int32 and seq.is_contiguous() and seq.shape[0] == R and seq.device == logits.device
              and 0 <= int(cur) <= seq.shape[1], "ngram: token history must be contiguous int32 [R, >= cur] on device")
        seq_p, seq_stride, cur, n = ptr(seq), int(seq.shape[1]), int(cur), int(n)
    native().beam_topk_rows(ptr(logits), R, V, ptr(beam_scores), int(eos), int(mask_eos), int(k), ptr(sc), ptr(idx),
                            launch_stream(logits), ptr(bans) if nbmax else 0, nbmax, seq_p, seq_stride, cur, n)
    return sc, idx


LM_HEAD_MAX_K = 8  # lm_head.hip / topk.h kTileSel


class LmHead(NamedTuple):
    """A decoder step's LM-head input (``model.step(..., logits=False)``): the rows ``x``,
    the vocabulary weights ``w`` [V, d], the logit bias and the folded RMSNorm eps."""
    x: torch.Tensor
    w: torch.Tensor
    bias: Optional[torch.Tensor]
    rms_eps: float

    def logits(self) -> torch.Tensor:
        from .linear import linear

        if self.rms_eps > 0:
            return linear(self.x, self.w, self.bias, out_f32=True, rms_eps=self.rms_eps)
        return linear(self.x, self.w, self.bias, out_f32=True)

    def topk(self, beam_scores: torch.Tensor, k: int, eos: int, mask_eos: bool,
             ngram: Optional[Tuple[torch.Tensor, int, int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        return lm_head_topk(self.x, self.w, beam_scores, k, eos, mask_eos, bias=self.bias, rms_eps=self.rms_eps,
                            ngram=ngram)


def lm_head(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], rms_eps: float, logits: bool):
    """End of a decoder step: fp32 logits, or the :class:`LmHead` for :func:`lm_head_topk`."""
    head = LmHead(x, w, bias, float(rms_eps))
    return head.logits() if logits else head


def lm_head_topk(x: torch.Tensor, w: torch.Tensor, beam_scores: torch.Tensor, k: int, eos: int, mask_eos: bool,
                 bias: Optional[torch.Tensor] = None, rms_eps: float = 0.0, bans: Optional[torch.Tensor] = None,
                 ngram: Optional[Tuple[torch.Tensor, int, int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused decode LM head + beam top-k (``csrc/kernels/lm_head.hip``, K10).

    The result of :func:`beam_topk_rows` over ``logits = (x @ w.T) * rstd(x) + bias``
    (``rstd`` = RMSNorm of the rows of ``x`` when ``rms_eps > 0``, its gamma folded
    into ``w``), computed without writing the fp32 logits: the GEMM's epilogue
    reduces every 128-token tile of a row to its log-softmax partials and exact
    top-8 candidates, a merge kernel finishes each row. ``k <= 8``."""
    R, Kd = x.shape
    V = int(w.shape[0])
    if not x.is_cuda:
        xf = x.float()
        if rms_eps > 0:
            xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + rms_eps)
        logits = xf @ w.float().t()
        if bias is not None:
            logits = logits + bias.float().view(1, -1)
        return beam_topk_rows(logits, beam_scores, k, eos, mask_eos, bans=bans, ngram=ngram)
    check_bf16_dev(x, "x")
    check_bf16_dev(w, "w")
    same_device(x, w, beam_scores)
    check(1 <= k <= LM_HEAD_MAX_K, f"lm_head_topk: 1 <= k <= {LM_HEAD_MAX_K}")
    check(w.shape[1] == Kd and x.stride(1) == 1 and w.stride(1) == 1, "lm_head_topk: x [R, d], w [V, d], unit column stride")
    check(not (bias is not None and rms_eps > 0), "lm_head_topk: bias and RMSNorm folding together are not supported")
    if bias is not None:
        check(bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == V and bias.device == x.device,
              "lm_head_topk: bias must be contiguous fp32 [V] on the device")
    check(beam_scores.dtype == torch.float32 and beam_scores.is_contiguous() and beam_scores.numel() == R,
          "lm_head_topk: beam_scores must be contiguous fp32 [R]")
    nbmax = 0 if bans is None else int(bans.shape[1])
    if nbmax:
        check(bans.dtype == torch.int32 and bans.is_contiguous() and bans.shape[0] == R and bans.device == x.device,
              "bans must be contiguous int32 [R, n] on the device")
    seq_p, seq_stride, cur, n = 0, 0, 0, 0
    if ngram is not None:
        seq, cur, n = ngram
        check(seq.dtype == torch.int32 and seq.is_contiguous() and seq.shape[0] == R and seq.device == x.device
              and 0 <= int(cur) <= seq.shape[1], "ngram: token history must be contiguous int32 [R, >= cur] on device")
        seq_p, seq_stride, cur, n = ptr(seq), int(seq.shape[1]), int(cur), int(n)
    nat = native()
    ws = torch.empty(int(nat.lm_head_ws_bytes(R, V)), dtype=torch.uint8, device=x.device)
    sc = torch.empty((R, k), dtype=torch.float32, device=x.device)
    idx = torch.empty((R, k), dtype=torch.int32, device=x.device)
    nat.lm_head_topk(ptr(x), row_stride(x, "x"), ptr(w), row_stride(w, "w"), ptr(bias), float(rms_eps), R, V, Kd,
                     int(k), ptr(beam_scores), int(eos), int(bool(mask_eos)), ptr(bans) if nbmax else 0, nbmax, seq_p,
                     seq_stride, cur, n, ptr(ws), ptr(sc), ptr(idx), launch_stream(x))
    return sc, idx


def beam_select_ref(sc: np.ndarray, tk: np.ndarray, nb: int, V: int, eos: int, hit_all: bool, neg: float):
    """Host reference of the device beam selection for ``B`` items.

    ``sc``/``tk`` [B*nb, K2]: each beam row's top continuations (accumulated score, token).
    Returns ``(top_sc [B,K2] f32, top_tok [B,K2], top_beam [B,K2], nxt [B,nb])``: the item's top K2 by
    (score desc, beam*V + token asc), and the K2 slots of the next running beams (best nb after hits
    get ``+neg``, stable)."""
    rows, K2 = sc.shape
    B = rows // nb
    s = np.ascontiguousarray(sc, dtype=np.float32).reshape(B, nb * K2)
    t = np.asarray(tk).astype(np.int64).reshape(B, nb * K2)
    beam_of = np.broadcast_to(np.repeat(np.arange(nb, dtype=np.int64), K2)[None, :], (B, nb * K2))
    rb = np.arange(B)[:, None]
    order = np.lexsort((beam_of * V + t, -s), axis=1)[:, :K2]
    top_sc, top_tok, top_beam = s[rb, order], t[rb, order], beam_of[rb, order]
    hits = (top_tok == eos) | bool(hit_all)
    run_cand = np.where(hits, top_sc + np.float32(neg), top_sc)
    nxt = np.argsort(-run_cand, axis=1, kind="stable")[:, :nb]
    return top_sc, top_tok, top_beam, nxt


def beam_select(sc: torch.Tensor, tk: torch.Tensor, nb: int, V: int, eos: int, hit_all: bool, neg: float,
                stage: torch.Tensor, rec: torch.Tensor) -> None:
    """Device beam selection (kernel ``beam_select_kernel``) for ``B = rows / nb`` items.

    Writes the next step's inputs into ``stage`` (int32 [3*rows]: parent rows | tokens | running-score
    bits) and per item ``rec`` (int32 [B, 3*K2 + nb]: top score bits | top tokens | top beams | kept
    slots) — the values of :func:`beam_select_ref`."""
    rows, K2 = sc.shape
    B = rows // nb
    check(rows % nb == 0 and K2 >= nb and tuple(tk.shape) == (rows, K2), "beam_select: sc/tk must be [B*nb, K2]")
    check(stage.numel() == 3 * rows and stage.dtype == torch.int32 and stage.is_contiguous(), "stage: int32 [3*rows]")
    check(tuple(rec.shape) == (B, 3 * K2 + nb) and rec.dtype == torch.int32 and rec.is_contiguous(),
          "rec: int32 [B, 3*K2 + nb]")
    if not sc.is_cuda:
        top_sc, top_tok, top_beam, nxt = beam_select_ref(sc.numpy(), tk.numpy(), nb, V, eos, hit_all, neg)
        rb = np.arange(B)[:, None]
        hits = (top_tok == eos) | bool(hit_all)
        run_cand = np.where(hits, top_sc + np.float32(neg), top_sc)
        st = stage.numpy()
        st[:rows] = (rb * nb + top_beam[rb, nxt]).reshape(-1)
        st[rows:2 * rows] = top_tok[rb, nxt].reshape(-1)
        st[2 * rows:] = run_cand[rb, nxt].astype(np.float32).reshape(-1).view(np.int32)
        r = rec.numpy()
        r[:, :K2] = top_sc.astype(np.float32).view(np.int32)
        r[:, K2:2 * K2] = top_tok
        r[:, 2 * K2:3 * K2] = top_beam
        r[:, 3 * K2:] = nxt
        return
    check(sc.dtype == torch.float32 and tk.dtype == torch.int32 and sc.is_contiguous() and tk.is_contiguous(),
          "beam_select: sc fp32 / tk int32, contiguous")
    if rec.device.type == "cpu":
        # the record straight into pinned host memory (no device buffer + D2H copy launch): the
        # host reads it after an event recorded behind this kernel
        check(rec.is_pinned(), "beam_select: a host rec must be pinned")
        same_device(sc, tk, stage)
        rec_p = native().host_device_ptr(ptr(rec), rec.numel() * 4)
    else:
        same_device(sc, tk, stage, rec)
        rec_p = ptr(rec)
    native().beam_select(ptr(sc), ptr(tk), B, nb, K2, int(V), int(eos), int(bool(hit_all)), float(neg), ptr(stage),
                         rec_p, launch_stream(sc))
