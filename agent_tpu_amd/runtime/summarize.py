"""Batched beam-search summarisation on the T5 HIP path (map_summarize).

Semantics follow HF transformers' (5.x) vectorised beam search, which the
reference invokes through ``model.generate(num_beams=4, max_length=130,
min_length=30, early_stopping=True)`` (``/root/reference/ops/map_summarize.py:53-59``):

* per step keep the top ``2*num_beams`` continuations of every batch item over
  ``num_beams x vocab`` accumulated log-probs (the fused K10 kernel returns
  each beam row's top ``2*num_beams``; their union holds the item's global top);
* a continuation "hits" when it emits EOS or reaches ``max_length``; the best
  ``num_beams`` non-hit continuations keep running, and hits among the top
  ``num_beams`` candidates enter the finished set scored
  ``logprob / generated_len ** length_penalty``;
* ``early_stopping=True`` freezes an item once ``num_beams`` hypotheses have
  finished; the loop ends when no item can improve;
* EOS is masked (after log-softmax) while the sequence is shorter than
  ``min_length``;
* BART's generation defaults (facebook/bart-large-cnn generation_config, which
  the reference's generate() call inherits): ``no_repeat_ngram_size`` bans (a
  token that would repeat an n-gram of the hypothesis), ``forced_bos`` at
  length 1 and ``forced_eos`` at ``max_length - 1`` (the only allowed token
  gets log-prob 0), ``length_penalty`` 2.0.

Device work per step: the decoder step (L layers of GEMMs, KV-cache appends,
single-query attention), then the LM head fused with K10 (``ops.lm_head_topk``: per
128-token tile log-softmax partials and exact top-8 candidates in the GEMM epilogue,
no fp32 logits) or, on the host-selection path, the LM-head GEMM and K10. Host work: bookkeeping on
``[B, 2*num_beams]`` tensors. Beam reorder never copies the KV cache: each
row's history is a backpointer table ``hist[row, pos]`` (physical cache row of
position ``pos``) and only that int table is gathered by parent beam (K11).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..tokenizer import pack_rows
from ..utils.trace import span

NEG = -1.0e9
# the device beam selection writes each step's record straight into the pinned host slot the
# search loop reads (no device record + D2H copy launch per step); ATPU_REC_ZERO_COPY=0: copy
REC_ZERO_COPY = os.environ.get("ATPU_REC_ZERO_COPY", "1") != "0"
# a small search's state advance also writes the next step's decoder input (one launch fewer
# per step); ATPU_ADVANCE_EMBED=0: the step embeds its tokens itself
ADVANCE_EMBED = os.environ.get("ATPU_ADVANCE_EMBED", "1") != "0"
# host-side step timing (tools/host_prof_summ.py): a dict to accumulate into, or None
HOST_PROF: Optional[Dict[str, float]] = None
# device selection runs the fused LM head + top-k (ops.lm_head_topk, csrc/kernels/lm_head.hip)
# instead of the fp32-logit GEMM + beam_topk_rows pair; ATPU_LM_FUSED=0 restores the pair
LM_FUSED = os.getenv("ATPU_LM_FUSED", "1").strip().lower() not in ("0", "false", "no")
# decoder-step hipGraphs (and the buffers they were captured on) kept across calls of the
# same shape (ATPU_SUMM_GRAPH_CACHE=0: capture per call); see _SlotCache. Same-box A/B: T5-base 256 docs
# 545 -> 550 docs/s, 1-doc jobs through the agent 7.46 -> 7.67 docs/s (profiles/summarize_graph_cache_r03.jsonl)
GRAPH_CACHE = os.getenv("ATPU_SUMM_GRAPH_CACHE", "1").strip().lower() not in ("0", "false", "no")
# source length buckets of a cached graph: ids are padded up to a multiple of this
# (masked by src_lens in the encoder and the cross attention: the outputs do not change)
SRC_BUCKET = 128


class _Slot:
    """One captured decoder step and every device buffer it reads or writes.

    The graph replays on fixed addresses, so a later search of the same shape reuses the
    buffers: the encoder writes its cross K/V into ``ckv``, the call's source lengths are
    copied into ``lens``, the per-search state (histories, tokens, step, staging) is
    reset. ``keep`` pins the model's lazily built tensors the graph read (a regrown
    decoder bias must not free the memory a replay reads). ``ev``: recorded on the
    search's stream when it releases the slot, waited for by the next user's stream."""

    def __init__(self, key):
        self.key = key
        self.bufs: Dict[str, torch.Tensor] = {}
        self.graph = None
        self.out = None
        self.keep: List[torch.Tensor] = []
        self.busy = False
        self.ev = None
        self.last = 0.0

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.bufs.values())


class _SlotCache:
    """Per-model LRU of :class:`_Slot` (a model attribute: dropping the model drops them).

    At most ``ATPU_SUMM_GRAPH_SLOTS`` (default 6) slots and ``ATPU_SUMM_GRAPH_CACHE_GB``
    (default 48) GiB of buffers; an acquire that would exceed them evicts idle slots in
    LRU order, and runs uncached if that is not enough. Capturing + instantiating a step
    graph cost 3.1 / 5.8 ms per T5 / BART call (docs/PERF_NOTES.md)."""

    def __init__(self):
        self.slots: List[_Slot] = []
        self.max_slots = int(os.getenv("ATPU_SUMM_GRAPH_SLOTS", "6"))
        self.max_bytes = int(float(os.getenv("ATPU_SUMM_GRAPH_CACHE_GB", "48")) * (1 << 30))
        self.hits = 0
        self.misses = 0

    def acquire(self, key) -> Optional[_Slot]:
        for sl in self.slots:
            if sl.key == key and not sl.busy and sl.graph is not None:
                sl.busy, sl.last = True, time.perf_counter()
                self.hits += 1
                if sl.ev is not None:
                    torch.cuda.current_stream().wait_event(sl.ev)
                return sl
        self.misses += 1
        return None

    def admit(self, sl: _Slot) -> bool:
        """Keep a newly captured slot if it fits (evicting idle LRU slots)."""
        need = sl.nbytes()
        if need > self.max_bytes:
            return False
        idle = sorted((s for s in self.slots if not s.busy), key=lambda s: s.last)
        while idle and (len(self.slots) >= self.max_slots or self.nbytes() + need > self.max_bytes):
            victim = idle.pop(0)
            # its last replay may still run on another stream (a host-selection search can
            # stop with a speculative step in flight): the caching allocator must not hand
            # its buffers to a new allocation before that replay has finished
            if victim.ev is not None:
                victim.ev.synchronize()
            self.slots.remove(victim)
        if len(self.slots) >= self.max_slots or self.nbytes() + need > self.max_bytes:
            return False
        sl.busy, sl.last = True, time.perf_counter()
        self.slots.append(sl)
        return True

    def release(self, sl: _Slot) -> None:
        ev = torch.cuda.Event()
        ev.record()
        sl.ev, sl.busy, sl.last = ev, False, time.perf_counter()

    def nbytes(self) -> int:
        return sum(s.nbytes() for s in self.slots)


def slot_cache(model) -> _SlotCache:
    sc = getattr(model, "_atpu_graph_slots", None)
    if sc is None:
        sc = _SlotCache()
        model._atpu_graph_slots = sc
    return sc


@dataclass
class GenConfig:
    num_beams: int = 4
    max_length: int = 130
    min_length: int = 30
    length_penalty: Optional[float] = None  # None -> model default (T5 1.0, bart-large-cnn 2.0)
    early_stopping: bool = True
    no_repeat_ngram_size: Optional[int] = None  # None -> model default (bart-large-cnn 3)
    forced_bos_id: Optional[int] = None  # None -> model default (bart-large-cnn 0)
    forced_eos_id: Optional[int] = None  # None -> model default (bart-large-cnn 2)
    use_graph: bool = True  # replay the decoder step as one hipGraph (device runs only)
    device_select: bool = True  # beam selection on the device, host bookkeeping one step behind

    def resolved(self, cfg) -> "GenConfig":
        def pick(v, name, default):
            return v if v is not None else getattr(cfg, name, default)

        return GenConfig(self.num_beams, self.max_length, self.min_length,
                         float(pick(self.length_penalty, "length_penalty", 1.0)), self.early_stopping,
                         int(pick(self.no_repeat_ngram_size, "no_repeat_ngram_size", 0) or 0),
                         pick(self.forced_bos_id, "forced_bos_id", None),
                         pick(self.forced_eos_id, "forced_eos_id", None), self.use_graph, self.device_select)


ngram_bans = ops.ngram_bans  # (re-exported: HF NoRepeatNGramLogitsProcessor, vectorised)


@dataclass
class GenResult:
    sequences: List[List[int]]
    scores: List[float]
    steps: int
    timing_ms: Dict[str, float] = field(default_factory=dict)


def _select(logits: torch.Tensor, run_scores: torch.Tensor, K2: int, cfg, gen: GenConfig, cur: int, T: int,
            run_seq: torch.Tensor, scores_dev: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Host selection path: per beam row, the top ``K2`` continuations ``(score [rows, K2],
    token [rows, K2])`` after log-softmax and the logits processors (min-length EOS mask,
    n-gram bans from the host sequences, forced BOS/EOS), returned on the host."""
    rows, V = logits.shape
    forced = None
    if gen.forced_bos_id is not None and cur == 1:
        forced = int(gen.forced_bos_id)
    elif gen.forced_eos_id is not None and cur == T - 1:
        forced = int(gen.forced_eos_id)
    if forced is not None:  # the only allowed token gets log-prob 0
        sc = torch.full((rows, K2), float("-inf"))
        sc[:, 0] = run_scores.view(-1)
        tk = torch.arange(K2).view(1, -1).expand(rows, -1).clone()
        tk[:, 1:] += (tk[:, 1:] >= forced).long()  # placeholders distinct from the forced token
        tk[:, 0] = forced
        return sc, tk
    mask_eos = cur < gen.min_length
    br, bt = ngram_bans(run_seq.view(rows, -1)[:, :cur], gen.no_repeat_ngram_size)
    counts = torch.bincount(br, minlength=rows) if br.numel() else None
    nban = int(counts.max()) if counts is not None else 0
    if scores_dev is None:  # the caller keeps a device copy of the running scores when it can
        scores_dev = run_scores.view(-1).to(logits.device)
    if logits.is_cuda and 0 < nban <= ops.MAX_BANS:
        # the kernel skips each row's banned tokens itself: exactly K2 per row come back
        starts = torch.cumsum(counts, 0) - counts
        bans = torch.full((rows, nban), -1, dtype=torch.int32)
        bans[br, torch.arange(br.numel()) - starts[br]] = bt.to(torch.int32)
        sc, tk = ops.beam_topk_rows(logits, scores_dev, K2, cfg.eos_id, mask_eos, bans=bans.to(logits.device))
        both = torch.cat([sc, tk.view(torch.float32)], 1).cpu()
        return both[:, :K2].contiguous(), both[:, K2:].contiguous().view(torch.int32).long()
    if K2 + nban <= 16:
        sc, tk = ops.beam_topk_rows(logits, scores_dev, K2 + nban, cfg.eos_id, mask_eos)
        if sc.is_cuda:  # one D2H copy (one sync) for scores and token ids
            both = torch.cat([sc, tk.view(torch.float32)], 1).cpu()
            sc, tk = both[:, :K2 + nban].contiguous(), both[:, K2 + nban:].contiguous().view(torch.int32).long()
        else:
            sc, tk = sc.cpu(), tk.cpu().long()
        if nban:
            key = br * V + bt
            flat = torch.arange(rows).view(-1, 1) * V + tk
            banned = torch.isin(flat, key)
            sc = sc.masked_fill(banned, float("-inf"))
            # keep the K2 best per row, ties -> lower token id (stable sort over token order)
            order = torch.argsort(tk, dim=1)
            sc, tk = torch.gather(sc, 1, order), torch.gather(tk, 1, order)
            top = torch.sort(sc, dim=1, descending=True, stable=True).indices[:, :K2]
            sc, tk = torch.gather(sc, 1, top), torch.gather(tk, 1, top)
        return sc, tk
    # many bans in one row: exact torch path for this step
    lp = torch.log_softmax(logits.float(), dim=-1)
    if mask_eos:
        lp[:, cfg.eos_id] = float("-inf")
    lp[br.to(lp.device), bt.to(lp.device)] = float("-inf")
    sc, tk = torch.topk(lp + scores_dev.view(-1, 1), K2, dim=-1)
    return sc.cpu(), tk.cpu().long()


def generate(model, src_ids: torch.Tensor, src_lens: torch.Tensor, gen: GenConfig) -> GenResult:
    """Beam search for a batch. ``src_ids`` [B, S] int32 (on the model device)."""
    return _drive([_generate_iter(model, src_ids, src_lens, gen)])[0]


def generate_concurrent(model, parts: Sequence[Tuple[torch.Tensor, torch.Tensor]], gen: GenConfig) -> List[GenResult]:
    """Beam search for several batches at once, each on its own HIP stream.

    A decode step of one batch is a chain of small latency-bound launches (skinny GEMMs,
    per-row attention) next to one bandwidth-bound kernel (cross attention); two batches
    on two streams fill each other's gaps (two 128-doc T5 runs side by side: 779 docs/s
    against 666 for one 256-doc run). The host interleaves the runs' device-selection
    loops: each yields before it waits for its own step's record."""
    dev = model.device
    caller = torch.cuda.current_stream(dev)
    prep = getattr(model, "prepare_decode", None)
    if prep is not None:  # lazily built weights / biases: once, before the streams fork
        for ids, _ in parts:
            prep(int(ids.shape[1]), int(gen.resolved(model.cfg).max_length))
    streams = [torch.cuda.Stream(dev) for _ in parts]
    for st in streams:  # the inputs were produced on the caller's stream
        st.wait_stream(caller)
    try:
        return _drive([_generate_iter(model, ids, lens, gen, stream=st) for (ids, lens), st in zip(parts, streams)])
    finally:
        torch.cuda.set_stream(caller)
        for st in streams:
            caller.wait_stream(st)


def _drive(iters) -> List[GenResult]:
    """Run generate iterators round robin until each returns its GenResult."""
    results: List[Optional[GenResult]] = [None] * len(iters)
    active = list(range(len(iters)))
    while active:
        for i in list(active):
            try:
                next(iters[i])
            except StopIteration as stop:
                results[i] = stop.value
                active.remove(i)
    return results  # type: ignore[return-value]


def _generate_iter(model, src_ids: torch.Tensor, src_lens: torch.Tensor, gen: GenConfig, stream=None):
    """:func:`generate` as a generator: yields where it would wait for its device step
    (device selection only), returns the GenResult. ``stream``: the HIP stream to run on.
    A cached decoder-step graph (:class:`_SlotCache`) is released when the search ends."""
    held: List[_Slot] = []
    try:
        return (yield from _generate_body(model, src_ids, src_lens, gen, stream, held))
    finally:
        for sl in held:
            slot_cache(model).release(sl)


def _generate_body(model, src_ids: torch.Tensor, src_lens: torch.Tensor, gen: GenConfig, stream, held: List[_Slot]):
    def on_stream():
        if stream is not None:
            torch.cuda.set_stream(stream)

    on_stream()
    cfg = model.cfg
    gen = gen.resolved(cfg)
    dev = model.device
    B, S = src_ids.shape
    nb = max(1, int(gen.num_beams))
    K2 = 2 * nb
    V = cfg.vocab_size
    T = int(gen.max_length)
    rows = B * nb
    pin = dev.type == "cuda"
    # Every step input is a static device buffer (tokens, step, cache, hist), so
    # after one eager step the whole decoder step (~13 launches x L layers) is
    # captured once and replayed: the host loop issues 1 launch per step.
    use_graph = gen.use_graph and pin
    # device selection with the fused LM head (lm_head.hip): the step ends at the LM-head
    # input and lm_head_topk produces the per-row top-K2 without fp32 logits
    fused = pin and gen.device_select and K2 <= ops.LM_HEAD_MAX_K and LM_FUSED
    ngram_dev = pin and bool(gen.device_select) and bool(gen.no_repeat_ngram_size)
    t0 = time.perf_counter()
    # device-side stage clocks (hipEvent pairs on this search's stream): encoder, decode loop
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if pin else None

    # graph cache: the source is padded to a length bucket (keys past src_lens are masked
    # in the encoder and the cross attention), the buffers of a previous search of this
    # shape are reused, and its captured step replays from the first launch
    # (padded on every device run with the cache on, graph or not: the padded source takes
    # other kernel paths -- split cross attention past 128 keys -- and a search's tokens
    # must not depend on whether its step was captured)
    slot, new_slot = None, None
    if pin and GRAPH_CACHE:
        Sb = -(-S // SRC_BUCKET) * SRC_BUCKET
        if Sb != S:
            src_ids = torch.nn.functional.pad(src_ids, (0, Sb - S), value=int(cfg.pad_id))
            S = Sb
    if use_graph and GRAPH_CACHE:
        key = (B, S, T, nb, fused, ngram_dev, bool(gen.device_select))
        slot = slot_cache(model).acquire(key)
        if slot is not None:
            held.append(slot)
            slot.bufs["lens"].copy_(src_lens)
        else:
            new_slot = _Slot(key)
            new_slot.bufs["lens"] = src_lens.to(torch.int32).clone()
        src_lens = (slot or new_slot).bufs["lens"]

    if evs:
        evs[0].record()  # after the host-side source prep: the window holds the encoder only
    with span("encode"):
        if slot is not None:
            _, ckv = model.encode(src_ids, src_lens, ckv_out=slot.bufs["ckv"])
        else:
            _, ckv = model.encode(src_ids, src_lens)
    if evs:
        evs[1].record()
    t_enc = time.perf_counter()
    if slot is not None:
        b = slot.bufs
        cache, hist, hist_alt, step_dev = b["cache"], b["hist"], b["hist_alt"], b["step"]
        hist.zero_()
        hist_alt.zero_()
    else:
        cache = model.new_cache(rows, T)
        hist = torch.zeros((rows, T), dtype=torch.int32, device=dev)
        hist_alt = torch.zeros_like(hist)
        step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        if new_slot is not None:
            new_slot.bufs.update(ckv=ckv, cache=cache, hist=hist, hist_alt=hist_alt, step=step_dev)

    # Host beam state lives in numpy: the per-step bookkeeping is ~40 tiny
    # array ops, ~4x cheaper than torch CPU ops, and everything that is not
    # needed to launch the next step (sequence copies, finished-hypothesis
    # merge, early-stop test) runs after that launch, under the GPU step.
    # sequences are int32 and only their first cur+1 columns are ever copied (the rest
    # stays pad): at 1024 docs x 4 beams the full-width int64 gathers were ~30 MB of host
    # memory traffic per step, longer than the GPU step. Two running buffers alternate.
    run_seq = np.full((B, nb, T), cfg.pad_id, dtype=np.int32)
    run_seq[:, :, 0] = cfg.decoder_start_id
    run_alt = run_seq.copy()
    run_scores = np.zeros((B, nb), dtype=np.float32)
    run_scores[:, 1:] = NEG
    fin_seq = run_seq.copy()
    fin_scores = np.full((B, nb), NEG, dtype=np.float32)
    fin_done = np.zeros((B, nb), dtype=bool)
    fin_len = np.ones((B, nb), dtype=np.int64)
    unsat = np.ones((B, 1), dtype=bool)
    top_mask = np.arange(K2) < nb
    rowsB = np.arange(B)[:, None]
    neg = np.float32(NEG)
    # per-item retirement: an item whose finished hypotheses can no longer change (HF's
    # BeamHypotheses.is_done with early_stopping, or the early-stop heuristic said no running
    # beam can beat its worst finished one: every later candidate is pushed down by NEG) is
    # reported at the search's next yield as (item, sequence, score), before the search ends
    reported = np.zeros(B, dtype=bool)
    done_q: List[Tuple[int, List[int], float]] = []

    def take_done() -> List[Tuple[int, List[int], float]]:
        out = list(done_q)
        done_q.clear()
        return out
    # one pinned staging row per step: [parent rows | new tokens | running beam scores]
    # -> ONE async H2D; everything after it (history reorder, token copy, step advance,
    # decoder step) is a single graph replay, and the next top-k finds the beam scores
    # already on the device (no synchronous pageable copy in front of it)
    stage_host = torch.empty(3 * rows, dtype=torch.int32, pin_memory=pin)
    seq_dev = seq_alt = None  # device token history (device selection with n-gram bans)
    if slot is not None:
        tokens, stage_dev = slot.bufs["tokens"], slot.bufs["stage"]
        tokens.fill_(cfg.decoder_start_id)
        if ngram_dev:
            seq_dev, seq_alt = slot.bufs["seq"], slot.bufs["seq_alt"]
    else:
        tokens = torch.full((rows,), cfg.decoder_start_id, dtype=torch.int32, device=dev)
        stage_dev = torch.zeros(3 * rows, dtype=torch.int32, device=dev)
        if ngram_dev:
            seq_dev = torch.empty((rows, T), dtype=torch.int32, device=dev)
            seq_alt = torch.zeros_like(seq_dev)
        if new_slot is not None:
            new_slot.bufs.update(tokens=tokens, stage=stage_dev)
            if ngram_dev:
                new_slot.bufs.update(seq=seq_dev, seq_alt=seq_alt)
    par_dev, tok_dev = stage_dev[:rows], stage_dev[rows:2 * rows]
    score_dev = stage_dev[2 * rows:].view(torch.float32)
    score_dev.copy_(torch.from_numpy(run_scores.reshape(-1)).to(dev))
    lp = float(gen.length_penalty)
    graph, g_logits = (slot.graph, slot.out) if slot is not None else (None, None)

    small = dev.type == "cuda" and ops.decode_advance_ok(rows, T, seq_dev is not None)
    # the same launch also embeds the new tokens (the step's first launch folded in)
    emb = model.dec_embed() if small and ADVANCE_EMBED and hasattr(model, "dec_embed") else None
    x0 = None
    if emb is not None:
        if slot is not None and "x0" in slot.bufs:
            x0 = slot.bufs["x0"]
        else:
            x0 = torch.empty((rows, emb.table.shape[1]), dtype=torch.bfloat16, device=dev)
            if new_slot is not None:
                new_slot.bufs["x0"] = x0

    def advance() -> torch.Tensor:
        """Histories follow their parent beams (backpointers, no KV copy), new tokens in,
        position + 1, decoder step -> logits. Static buffers only (graph-capturable)."""
        if small:  # one launch for the whole state advance (1-document searches)
            ops.decode_advance(hist, seq_dev, par_dev, tok_dev, tokens, step_dev, embed=emb, out=x0)
            if x0 is not None:
                return model.step(tokens, step_dev, cache, T, ckv, src_lens, S, nb, hist=hist, logits=not fused,
                                  x0=x0)
        else:
            ops.beam_reorder_hist(hist, hist_alt, par_dev, step_dev)
            hist.copy_(hist_alt)  # keep the captured buffer address
            if seq_dev is not None:  # token history for the in-kernel n-gram bans
                ops.beam_reorder_hist(seq_dev, seq_alt, par_dev, step_dev, last=tok_dev, off=1)
                seq_dev.copy_(seq_alt)
            tokens.copy_(tok_dev)
            step_dev.add_(1)
        return model.step(tokens, step_dev, cache, T, ckv, src_lens, S, nb, hist=hist, logits=not fused)

    def launch_next() -> torch.Tensor:
        nonlocal graph, g_logits
        if graph is not None:
            graph.replay()
            return g_logits
        out = advance()
        if use_graph:
            # capture records without executing: the state stays at the eager step's.
            # capture_graph skips torch.cuda.graph's device-wide synchronize + empty_cache,
            # which stalled the sibling searches' streams
            from .graphs import capture_graph

            graph, g_logits = capture_graph(advance)
            if new_slot is not None:
                new_slot.graph, new_slot.out = graph, g_logits
                # the lazily built model tensors the step read (a regrown one must not be freed)
                new_slot.keep = [t for t in (getattr(model, "_dec_bias", None),) if t is not None]
                if slot_cache(model).admit(new_slot):
                    held.append(new_slot)
        return out

    def apply(cur: int, top_sc, top_tok, top_beam, nxt) -> bool:
        """Fold step ``cur``'s selection into the host state (sequences, finished
        hypotheses); True when the search is over (HF's stopping rules)."""
        nonlocal run_seq, run_alt, run_scores, fin_seq, fin_scores, fin_done, fin_len, unsat
        hits = (top_tok == cfg.eos_id) | (cur + 1 >= T)
        run_cand = np.where(hits, top_sc + neg, top_sc)
        parent = top_beam[rowsB, nxt]  # beam index within the item
        new_tok = top_tok[rowsB, nxt]
        run_scores = run_cand[rowsB, nxt]
        prev_seq, run_seq = run_seq, run_alt
        run_alt = prev_seq
        run_seq[:, :, :cur] = prev_seq[rowsB, parent, :cur]
        run_seq[:, :, cur] = new_tok
        did = hits & top_mask[None, :]
        fin_cand = top_sc / np.float32(float(cur) ** lp)  # generated length = cur + 1 - prompt(1)
        full = fin_done.all(axis=1, keepdims=True) & bool(gen.early_stopping)
        fin_cand = fin_cand + full * neg + (~unsat) * neg + (~did) * neg
        m_sc = np.concatenate([fin_scores, fin_cand.astype(np.float32)], 1)
        keep = np.argsort(-m_sc, axis=1, kind="stable")[:, :nb]
        from_fin = keep < nb
        kc = np.maximum(keep - nb, 0)
        cand_rows = prev_seq[rowsB, top_beam[rowsB, kc], :cur + 1]
        cand_rows[:, :, cur] = top_tok[rowsB, kc]
        # columns past cur are pad in every finished hypothesis (all are at most cur long)
        fin_seq[:, :, :cur + 1] = np.where(from_fin[:, :, None], fin_seq[rowsB, np.minimum(keep, nb - 1), :cur + 1],
                                           cand_rows)
        fin_scores = m_sc[rowsB, keep]
        fin_done = np.where(from_fin, fin_done[rowsB, np.minimum(keep, nb - 1)], did[rowsB, kc])
        fin_len = np.where(from_fin, fin_len[rowsB, np.minimum(keep, nb - 1)], cur + 1)
        if cur + 1 >= T:
            return True
        # early-stop heuristic (early_stopping=True: best running at current length)
        best_run = run_scores[:, :1] / np.float32(float(cur) ** lp)
        worst_fin = np.where(fin_done, fin_scores.min(axis=1, keepdims=True), neg)
        unsat = unsat & (best_run > worst_fin).any(axis=1, keepdims=True)
        item_done = ~unsat[:, 0]
        if gen.early_stopping:
            item_done |= fin_done.all(axis=1)
        new = np.flatnonzero(item_done & ~reported)
        if new.size:
            reported[new] = True
            for b in new.tolist():
                done_q.append((b, fin_seq[b, 0, :int(fin_len[b, 0])].tolist(), float(fin_scores[b, 0])))
        open_beam = not (bool(fin_done.all()) and bool(gen.early_stopping))
        return not (bool(unsat.any()) and open_beam and not bool(hits.all()))

    def prof(tp0, tp1, tp2):
        if HOST_PROF is not None:  # (select incl. the wait for the GPU, select -> next launch, after launch)
            tp3 = time.perf_counter()
            for key, dt in (("select", tp1 - tp0), ("to_launch", tp2 - tp1), ("after_launch", tp3 - tp2)):
                HOST_PROF[key] = HOST_PROF.get(key, 0.0) + dt
            HOST_PROF["steps"] = HOST_PROF.get("steps", 0) + 1

    cur = 1  # sequence length so far (decoder start token included)
    steps = 0
    step_dev.fill_(0)
    logits = model.step(tokens, step_dev, cache, T, ckv, src_lens, S, nb, hist=hist, logits=not fused)
    if pin and gen.device_select:
        yield []  # let other runs start their encoders / first steps
        on_stream()
        # Device selection: nothing the GPU needs for step t comes from the host (n-gram
        # bans read the device token history, forced tokens the device beam scores), so
        # top-k(t) -> beam_select(t) -> decoder step t+1 are enqueued FIRST and the host
        # then folds step t-1's record into its state: the GPU always has a step queued
        # behind the one it runs. Two pinned record slots alternate.
        rec_dev = torch.empty((B, 3 * K2 + nb), dtype=torch.int32, device=dev)
        rec_host = [torch.empty((B, 3 * K2 + nb), dtype=torch.int32, pin_memory=True) for _ in range(2)]
        rec_ev = [torch.cuda.Event(), torch.cuda.Event()]
        forced_tk = {}
        for fid in (gen.forced_bos_id, gen.forced_eos_id):
            if fid is not None:
                tk = torch.arange(K2).view(1, -1).expand(rows, -1).clone()
                tk[:, 1:] += (tk[:, 1:] >= int(fid)).long()  # placeholders distinct from the forced token
                tk[:, 0] = int(fid)
                forced_tk[int(fid)] = tk.to(device=dev, dtype=torch.int32)

        def select_dev(cur: int):
            forced = None
            if gen.forced_bos_id is not None and cur == 1:
                forced = int(gen.forced_bos_id)
            elif gen.forced_eos_id is not None and cur == T - 1:
                forced = int(gen.forced_eos_id)
            if forced is not None:  # the only allowed token gets log-prob 0
                sc = torch.full((rows, K2), float("-inf"), device=dev)
                sc[:, 0] = score_dev
                return sc, forced_tk[forced]
            ngram = (seq_dev, cur, gen.no_repeat_ngram_size) if seq_dev is not None else None
            if fused:  # logits is the step's ops.LmHead
                return logits.topk(score_dev, K2, cfg.eos_id, cur < gen.min_length, ngram=ngram)
            return ops.beam_topk_rows(logits, score_dev, K2, cfg.eos_id, cur < gen.min_length, ngram=ngram)

        def record(slot: int):
            r = rec_host[slot].numpy()
            return (r[:, :K2].copy().view(np.float32), r[:, K2:2 * K2].astype(np.int64),
                    r[:, 2 * K2:3 * K2].astype(np.int64), r[:, 3 * K2:].astype(np.int64))

        if seq_dev is not None:
            # running beams' tokens [rows, T], reordered by parents in advance() (graph)
            seq_dev.fill_(cfg.pad_id)
            seq_dev[:, 0] = cfg.decoder_start_id
            seq_alt.zero_()
        pending, slot = None, 0
        while True:
            tp0 = time.perf_counter()
            with span("beam_select"):
                sc_d, tk_d = select_dev(cur)
                if REC_ZERO_COPY:  # the kernel writes the pinned record itself
                    ops.beam_select(sc_d, tk_d, nb, V, cfg.eos_id, cur + 1 >= T, NEG, stage_dev, rec_host[slot])
                else:
                    ops.beam_select(sc_d, tk_d, nb, V, cfg.eos_id, cur + 1 >= T, NEG, stage_dev, rec_dev)
                    rec_host[slot].copy_(rec_dev, non_blocking=True)
                rec_ev[slot].record()
            if cur + 1 < T:
                logits = launch_next()
            tp1 = time.perf_counter()
            if pending is not None:
                # other runs enqueue their steps while this one's record is folded in; the items
                # the previous fold retired go to the caller (SummarizeStream posts them)
                yield take_done()
                on_stream()
                rec_ev[pending[1]].synchronize()  # passed already: it precedes the running step
                steps += 1
                if apply(pending[0], *record(pending[1])):
                    break
            tp2 = time.perf_counter()
            prof(tp0, tp1, tp2)
            pending, slot = (cur, slot), slot ^ 1
            cur += 1
            if cur >= T:  # the last selection: fold it in and stop
                rec_ev[pending[1]].synchronize()
                steps += 1
                apply(pending[0], *record(pending[1]))
                break
        # an early stop leaves up to two speculatively launched steps in flight: let them
        # drain before their graph and buffers go out of scope
        torch.cuda.current_stream(dev).synchronize()
    else:
        stage_ev = None  # stage_host is rewritten only after its last H2D retired
        while True:
            tp0 = time.perf_counter()
            with span("beam_select"):
                sc_t, tk_t = _select(logits, torch.from_numpy(run_scores), K2, cfg, gen, cur, T,
                                     torch.from_numpy(run_seq), scores_dev=score_dev if pin else None)
            tp1 = time.perf_counter()
            top_sc, top_tok, top_beam, nxt = ops.beam_select_ref(sc_t.numpy(), tk_t.numpy(), nb, V, cfg.eos_id,
                                                                 cur + 1 >= T, NEG)
            steps += 1
            if cur + 1 < T:
                # enqueue step cur+1 NOW (the staging row is free: the top-k D2H of this
                # step synchronised past its previous H2D)
                hits = (top_tok == cfg.eos_id) | (cur + 1 >= T)
                run_cand = np.where(hits, top_sc + neg, top_sc)
                if stage_ev is not None:
                    stage_ev.synchronize()  # the previous step's async H2D has read stage_host
                st = stage_host.numpy()
                st[:rows] = (rowsB * nb + top_beam[rowsB, nxt]).reshape(-1)
                st[rows:2 * rows] = top_tok[rowsB, nxt].reshape(-1)
                st[2 * rows:] = run_cand[rowsB, nxt].reshape(-1).view(np.int32)
                stage_dev.copy_(stage_host, non_blocking=True)
                if pin:
                    stage_ev = torch.cuda.Event()
                    stage_ev.record()
                logits = launch_next()
            tp2 = time.perf_counter()
            stop = apply(cur, top_sc, top_tok, top_beam, nxt)  # under the GPU step
            prof(tp0, tp1, tp2)
            cur += 1
            if stop:
                break
            if done_q:
                yield take_done()  # retired items (host selection: a caller-paced search too)
    t_dec = time.perf_counter()
    seqs = [fin_seq[b, 0, :int(fin_len[b, 0])].tolist() for b in range(B)]
    scores = [float(fin_scores[b, 0]) for b in range(B)]
    # encode_ms / decode_ms: GPU time between hipEvents (encoder kernels; encoder end -> the
    # last decode step's work); host_*: the host clock of the enqueue / the search loop
    tm = {"host_encode_enqueue_ms": (t_enc - t0) * 1e3, "host_decode_loop_ms": (t_dec - t_enc) * 1e3}
    if evs:
        evs[2].record()
        evs[2].synchronize()
        tm["encode_ms"] = evs[0].elapsed_time(evs[1])
        tm["decode_ms"] = evs[1].elapsed_time(evs[2])
    else:
        tm["encode_ms"], tm["decode_ms"] = tm["host_encode_enqueue_ms"], tm["host_decode_loop_ms"]
    return GenResult(seqs, scores, steps, tm)


def build_model(name: str, pack=None, device: Optional[torch.device] = None, seed: int = 0, fp32: bool = False,
                broadcast: bool = False):
    """``t5-*`` / ``bart-*`` preset name -> (model, pack); random init when no pack.

    Random init is built on ``device`` itself (``params.rand_fill``: a kernel, no host pass or
    H2D copy) and is bit-identical on every rank, so a DP group needs no broadcast for it.
    ``broadcast`` with a given ``pack``: rank 0's weights reach every rank in ONE RCCL
    broadcast of the flat ParamPack (C1)."""
    from ..models import bart, t5

    fam = family_of(name)
    mod = bart if fam == "bart" else t5
    cfg = mod.config_for(name)
    if pack is None:
        dev = device if device is not None else torch.device("cpu")
        if broadcast:
            from ..parallel.dp_ops import load_collectively

            # every rank builds the same bits; the exchange fails the job on all ranks together
            pack = load_collectively(lambda: mod.init_random(cfg, seed=seed, device=dev), lambda p: p)
        else:
            pack = mod.init_random(cfg, seed=seed, device=dev)
    elif broadcast:
        from ..models.params import ParamPack
        from ..parallel.dp import broadcast_pack, world
        from ..parallel.dp_ops import load_collectively

        dev = device if device is not None else torch.device("cpu")
        src = pack

        def local():  # rank 0: its pack on the device; others: the destination buffer (either may OOM)
            if world()[0] == 0:
                return src if src.buffer.device == dev else src.to(dev)
            return ParamPack(mod.param_specs(cfg), device=dev)

        pack = load_collectively(local, lambda p: broadcast_pack(p, cfg, dev, builder=mod.param_specs))
    if device is not None and pack.buffer.device != device:
        pack = pack.to(device)
    cls = bart.BartModel if fam == "bart" else t5.T5Model
    return cls(cfg, pack, fp32=fp32), pack


def family_of(name: str) -> str:
    key = name.split("/")[-1].lower()
    if key.startswith("bart"):
        return "bart"
    if key.startswith("t5"):
        return "t5"
    raise ValueError(f"unknown summarization model {name!r} (t5-* or bart-*)")


@dataclass
class WordMap:
    """Sorted token ids, index of the first word producing each, the words."""
    ids: np.ndarray
    word_of: np.ndarray
    words: List[str]


class SummarizeEngine:
    """Texts -> summaries with a device-resident T5 or BART (batched beam search)."""

    def __init__(self, model, max_source_len: int = 512, max_batch_docs: Optional[int] = None):
        self.model = model
        self.cfg = model.cfg
        self.device = model.device
        self.max_src = int(max_source_len)
        # documents per device batch: what worker_sizing advertises for this model and HBM
        # (KV cache + cross K/V + encoder activations per document); run() splits larger calls
        self.max_batch_docs = int(max_batch_docs) if max_batch_docs else self._sized_batch_docs()

    def _sized_batch_docs(self) -> int:
        from worker_sizing import summarize_batch_docs

        c = self.cfg
        dims = (c.d_model, c.d_ff, c.enc_layers, c.dec_layers, c.vocab_size)
        if self.device.type == "cuda":
            total = torch.cuda.get_device_properties(self.device).total_memory
        else:
            total = 288 * (1 << 30)
        return summarize_batch_docs(total, dims, self.max_src)

    def encode_texts(self, texts: Sequence[str], with_maps: bool = True, to_device: bool = True
                     ) -> Tuple[torch.Tensor, torch.Tensor, List[Dict[int, str]]]:
        """Hash-tokenize (same spec as K1, the model's vocab), wrap with the
        model's specials (T5: ``toks </s>``; BART: ``<s> toks </s>``), pad to S % 8 == 0.
        Array ops only: the per-token Python loop cost ~35 ms per 256 documents."""
        from .._native import native

        text, offs = pack_rows(texts)
        ids, lens = native().tokenize_host(text, offs, self.max_src + 1, self.cfg.vocab_size, 1 << 16)
        wrapped = self.model.wrap_source([-1])
        cut = wrapped.index(-1)
        pre, post = wrapped[:cut], wrapped[cut + 1:]
        P = len(pre)
        ntok = np.minimum(lens.astype(np.int64) - 2, self.max_src - len(pre) - len(post))
        L = P + ntok + len(post)
        B = len(texts)
        S = max(8, (int(L.max()) + 7) // 8 * 8) if B else 8
        arr = np.full((B, S), self.cfg.pad_id, dtype=np.int32)
        arr[:, :P] = pre
        cols = np.arange(S)[None, :]
        src = np.take_along_axis(ids, np.clip(cols - P + 1, 0, ids.shape[1] - 1).repeat(B, 0), 1)
        tok = (cols >= P) & (cols < P + ntok[:, None])
        arr[tok] = src[tok]
        for k, t in enumerate(post):
            arr[np.arange(B), P + ntok + k] = t
        lens_t = torch.from_numpy(L.astype(np.int32))
        vocab_maps = self.word_maps(texts) if with_maps else []
        if not to_device:
            return torch.from_numpy(arr), lens_t, vocab_maps
        return torch.from_numpy(arr).to(self.device), lens_t.to(self.device), vocab_maps

    def _reverse_map(self, text: str) -> Dict[int, str]:
        """Python oracle of :meth:`word_maps` (first source word producing each id)."""
        from .. import tokenizer as T

        out: Dict[int, str] = {}
        for word in text.split():
            for tok_id in T.token_ids(word.encode("utf-8"), self.cfg.vocab_size, 64):
                out.setdefault(tok_id, word)
        return out

    def word_maps(self, texts: Sequence[str]) -> List["WordMap"]:
        """Per text: sorted token ids -> the first whitespace word producing each.

        ONE native call over all texts (``word_maps_host``: each text's ``str.split()``
        words re-joined by single spaces, tokenized word by word, deduplicated in C++);
        per-word Python packing and per-document ``np.unique`` cost ~200 ms per 256
        documents on the dev host."""
        from .._native import native

        words = [t.split() for t in texts]
        blobs = [" ".join(ws).encode("utf-8") for ws in words]
        offs = np.zeros(len(blobs) + 1, dtype=np.int64)
        if blobs:
            offs[1:] = np.cumsum([len(b) for b in blobs])
        text = np.frombuffer(b"".join(blobs), dtype=np.uint8) if blobs else np.zeros(0, np.uint8)
        ids, word_of, doc = native().word_maps_host(text, offs, self.cfg.vocab_size, 64)
        return [WordMap(ids[doc[i]:doc[i + 1]], word_of[doc[i]:doc[i + 1]], ws) for i, ws in enumerate(words)]

    def detokenize(self, seq: List[int], vmap: "WordMap") -> str:
        special = {self.cfg.pad_id, self.cfg.eos_id, self.cfg.decoder_start_id, getattr(self.cfg, "bos_id", -1)}
        keep = [t for t in seq if t not in special]
        if not keep:
            return ""
        q = np.asarray(keep, dtype=np.int64)
        i = np.minimum(np.searchsorted(vmap.ids, q), max(len(vmap.ids) - 1, 0))
        hit = (vmap.ids[i] == q) if len(vmap.ids) else np.zeros(len(q), bool)
        return " ".join(vmap.words[vmap.word_of[j]] if h else f"<{t}>" for t, j, h in zip(keep, i, hit))

    def run(self, ids: torch.Tensor, lens: torch.Tensor, gen: GenConfig) -> GenResult:
        """Beam search over a tokenized batch. On a GPU with device selection the batch is
        split into ``ATPU_SUMM_STREAMS`` (default 3) contiguous parts searched concurrently
        on their own streams (:func:`generate_concurrent`), each part >= ``ATPU_SUMM_PART_MIN``
        (default 128). Two parts ran bimodally (T5, 1024 docs: 708 / 989 / 987 and 575 / 645 docs/s in
        separate processes), three held 980-990 (tools/gpu_summ_streams.sh).
        One host thread runs every part's bookkeeping, so the split pays once a part's GPU step
        outlasts the other parts' host work: at the reference's 1024-token sources 256 docs as
        2 x 128 beat one search (T5-base 568 -> 576-583, BART-large-CNN 411 -> 423-428 docs/s;
        3 x 85 no better, docs/PERF_NOTES.md "Summarize: two searches at 256 documents")."""
        B = int(ids.shape[0])
        cap = self.max_batch_docs
        if cap and B > cap:  # HBM-sized device batches, searched one after another
            outs = [self.run(ids[a:a + cap], lens[a:a + cap], gen) for a in range(0, B, cap)]
            timing: Dict[str, float] = {}
            for o in outs:
                for k, v in o.timing_ms.items():
                    timing[k] = timing.get(k, 0.0) + v
            return GenResult([s for o in outs for s in o.sequences], [s for o in outs for s in o.scores],
                             max(o.steps for o in outs), timing)
        n = int(os.getenv("ATPU_SUMM_STREAMS", "3"))
        n = max(1, min(n, B // max(1, int(os.getenv("ATPU_SUMM_PART_MIN", "128")))))
        if n < 2 or self.device.type != "cuda" or not gen.device_select:
            return generate(self.model, ids, lens, gen)
        cuts = [B * i // n for i in range(n + 1)]
        parts = [(ids[a:b], lens[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
        t0 = time.perf_counter()
        outs = generate_concurrent(self.model, parts, gen)
        wall = (time.perf_counter() - t0) * 1e3
        # the parts run side by side: each stage is as long as its longest part
        tm = {k: max(o.timing_ms[k] for o in outs) for k in outs[0].timing_ms}
        tm["host_search_wall_ms"] = wall
        return GenResult([s for o in outs for s in o.sequences], [s for o in outs for s in o.scores],
                         max(o.steps for o in outs), tm)

    def generate_ids(self, texts: Sequence[str], gen: GenConfig) -> GenResult:
        """Token sequences only (a DP rank's shard; rank 0 detokenizes)."""
        ids, lens, _ = self.encode_texts(texts, with_maps=False)
        return self.run(ids, lens, gen)

    def detokenize_all(self, texts: Sequence[str], seqs: List[List[int]]) -> List[str]:
        return [self.detokenize(s, m) for s, m in zip(seqs, self.word_maps(texts))]

    def summarize(self, texts: Sequence[str], gen: GenConfig) -> Tuple[List[str], GenResult]:
        t0 = time.perf_counter()
        ids, lens, _ = self.encode_texts(texts, with_maps=False)
        t_prep = (time.perf_counter() - t0) * 1e3
        if self.device.type == "cuda" and os.getenv("ATPU_SUMM_MAPS_OVERLAP", "1") not in ("0", "false", "no"):
            # the detokenization maps are built on a worker thread while the GPU decodes
            # (the native part releases the GIL; the decode loop mostly waits on events)
            fut = _host_pool().submit(self.word_maps, texts)
            res = self.run(ids, lens, gen)
            maps = fut.result()
        else:
            res = self.run(ids, lens, gen)
            maps = self.word_maps(texts)
        t1 = time.perf_counter()
        out = [self.detokenize(s, m) for s, m in zip(res.sequences, maps)]
        res.timing_ms["host_prepare_ms"] = t_prep  # host tokenization + source staging
        res.timing_ms["host_detokenize_ms"] = (time.perf_counter() - t1) * 1e3
        return out, res


_POOL = None


def _host_pool():
    """One long-lived worker thread for host work overlapped with GPU decoding."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="atpu-summ-host")
    return _POOL


class SummarizeStream:
    """Continuous (in-flight) batching for single-document jobs.

    Jobs are :meth:`submit`-ted at any time and :meth:`pump`-ed by the caller's loop. Up to
    ``max_searches`` beam searches run side by side, each on its own HIP stream (the
    :func:`generate_concurrent` pairing, generalised): every :meth:`pump` advances each running
    search by one decode step (their launches interleave, so one search's host bookkeeping runs
    under another's GPU step), and new documents are ADMITTED at that step boundary as a new
    search of up to ``part_max`` documents whenever a search slot is free -- they never wait for
    the running searches to finish. An item is RETIRED (its job completed) the step its
    hypotheses can no longer change (``_generate_body``'s per-item retirement), not when its
    whole search ends.

    Documents are grouped by (generation settings, source-length bucket of ``SRC_BUCKET``
    tokens): a document's padded source length depends on its own length only, never on the
    documents it is batched with. A job's documents (``texts`` form) stay in one search.
    ``pump`` returns ``[(tag, sequences, scores, info)]`` for the jobs completed by that call.
    """

    def __init__(self, engine: "SummarizeEngine", max_searches: Optional[int] = None,
                 part_max: Optional[int] = None):
        self.eng = engine
        # two searches of up to 256 documents measured best through the agent (T5-base 1-doc jobs:
        # 513 docs/s vs 388 at three of 128; docs/PERF_NOTES.md "In-flight search shape")
        self.max_searches = int(max_searches or os.getenv("ATPU_INFLIGHT_SEARCHES", "2"))
        self.part_max = int(part_max or os.getenv("ATPU_INFLIGHT_PART_MAX", "256"))
        self.part_max = max(1, min(self.part_max, engine.max_batch_docs or self.part_max))
        self._queues: Dict[tuple, List[tuple]] = {}  # (gen key, bucket) -> [(tag, texts, ids rows, lens, t_submit)]
        self._active: List[dict] = []
        self._streams: List[torch.cuda.Stream] = []
        self.admitted = 0
        self.searches = 0

    # ------------------------------------------------------------------ admission
    @staticmethod
    def _gen_key(gen: GenConfig) -> tuple:
        return (gen.num_beams, gen.max_length, gen.min_length, gen.length_penalty, gen.early_stopping,
                gen.no_repeat_ngram_size, gen.forced_bos_id, gen.forced_eos_id, gen.use_graph, gen.device_select)

    def submit(self, tag: Any, texts: Sequence[str], gen: GenConfig) -> None:
        """Queue one job (``texts``: its documents, at least one)."""
        ids, lens, _ = self.eng.encode_texts(list(texts), with_maps=False, to_device=False)
        L = int(lens.max())
        bucket = -(-L // SRC_BUCKET) * SRC_BUCKET
        self._queues.setdefault((self._gen_key(gen), bucket), []).append(
            (tag, list(texts), ids, lens, gen, time.perf_counter()))

    def pending(self) -> int:
        return sum(len(q) for q in self._queues.values())

    def busy(self) -> bool:
        return bool(self._active) or self.pending() > 0

    def _stream(self, i: int):
        while len(self._streams) <= i:
            self._streams.append(torch.cuda.Stream(self.eng.device))
        return self._streams[i]

    def _start(self) -> None:
        """Admit queued jobs as new searches while search slots are free (oldest queue first)."""
        while len(self._active) < self.max_searches and self._queues:
            key = min(self._queues, key=lambda k: self._queues[k][0][5])
            q = self._queues[key]
            take, ndocs = [], 0
            while q and (not take or ndocs + len(q[0][1]) <= self.part_max):
                it = q.pop(0)
                take.append(it)
                ndocs += len(it[1])
            if not q:
                del self._queues[key]
            gen = take[0][4]
            dev = self.eng.device
            # the part's width: its longest source (<= the bucket); on the device the search pads
            # every source to the bucket itself (SRC_BUCKET: generate's graph-cache padding)
            S = max(int(it[2].shape[1]) for it in take)
            rows = []
            for _, _, ids, lens, _, _ in take:
                pad = torch.full((ids.shape[0], S), int(self.eng.cfg.pad_id), dtype=ids.dtype)
                pad[:, :ids.shape[1]] = ids
                rows.append((pad, lens))
            ids = torch.cat([r[0] for r in rows]).to(dev)
            lens = torch.cat([r[1] for r in rows]).to(dev)
            texts = [t for it in take for t in it[1]]
            owners = [(it[0], len(it[1])) for it in take]
            used = {a["slot"] for a in self._active}
            slot = next(i for i in range(self.max_searches) if i not in used)
            on_gpu = dev.type == "cuda"
            st = self._stream(slot) if on_gpu else None
            if on_gpu:
                st.wait_stream(torch.cuda.current_stream(dev))  # the inputs were copied on the caller's stream
                prep = getattr(self.eng.model, "prepare_decode", None)
                if prep is not None:
                    prep(int(ids.shape[1]), int(gen.resolved(self.eng.cfg).max_length))
            maps = _host_pool().submit(self.eng.word_maps, texts)
            it = _generate_iter(self.eng.model, ids, lens, gen, stream=st)
            # per-document result slots; a job completes when all of its documents have
            starts, pos = [], 0
            for _, n in owners:
                starts.append(pos)
                pos += n
            self._active.append({"it": it, "slot": slot, "owners": owners, "starts": starts, "maps": maps,
                                 "texts": texts, "seq": [None] * len(texts), "score": [None] * len(texts),
                                 "left": [n for _, n in owners], "t0": time.perf_counter(),
                                 "t_submit": [x[5] for x in take]})
            self.admitted += len(take)
            self.searches += 1

    # ------------------------------------------------------------------ stepping
    def _deliver(self, a: dict, items, out: list, steps: Optional[int] = None) -> None:
        maps = None
        for b, seq, score in items:
            if a["seq"][b] is not None:
                continue
            a["seq"][b], a["score"][b] = seq, score
            # the job owning document b
            j = max(i for i, s0 in enumerate(a["starts"]) if s0 <= b)
            a["left"][j] -= 1
            if a["left"][j] == 0:
                if maps is None:
                    maps = a["maps"].result()
                s0, n = a["starts"][j], a["owners"][j][1]
                summaries = [self.eng.detokenize(a["seq"][k], maps[k]) for k in range(s0, s0 + n)]
                info = {"batched_docs": len(a["texts"]), "batched_jobs": len(a["owners"]),
                        "queue_ms": (a["t0"] - a["t_submit"][j]) * 1e3,
                        "search_ms": (time.perf_counter() - a["t0"]) * 1e3,
                        "retired_early": steps is None}
                if steps is not None:
                    info["decode_steps"] = steps
                out.append((a["owners"][j][0], summaries, [a["score"][k] for k in range(s0, s0 + n)], info))

    def pump(self) -> List[tuple]:
        """Admit what fits, advance every running search one step, return completed jobs."""
        out: List[tuple] = []
        self._start()
        dev = self.eng.device
        caller = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        try:
            for a in list(self._active):
                try:
                    items = next(a["it"])
                except StopIteration as stop:
                    res: GenResult = stop.value
                    self._deliver(a, [(b, s, sc) for b, (s, sc) in enumerate(zip(res.sequences, res.scores))], out,
                                  steps=res.steps)
                    self._active.remove(a)
                    continue
                if items:
                    self._deliver(a, items, out)
        finally:
            if caller is not None:
                torch.cuda.set_stream(caller)
        return out

    def cancel_queued(self) -> List[Any]:
        """Drop every job not yet admitted to a search; returns their tags."""
        tags = [it[0] for q in self._queues.values() for it in q]
        self._queues.clear()
        return tags

    def abort(self) -> List[Any]:
        """Forget everything (after a device fault): the tags of every queued and running job."""
        tags = self.cancel_queued()
        for a in self._active:
            done = {j for j, left in enumerate(a["left"]) if left == 0}
            tags += [o[0] for j, o in enumerate(a["owners"]) if j not in done]
            try:
                a["it"].close()
            except Exception:
                pass
        self._active.clear()
        return tags

    def drain(self) -> List[tuple]:
        """Run every queued and running search to completion."""
        out: List[tuple] = []
        while self.busy():
            out.extend(self.pump())
        return out
