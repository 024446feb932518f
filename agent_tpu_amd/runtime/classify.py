"""ClassifyEngine: rows of text -> top-k classes on one MI355X.

The device-side replacement for the reference's single-tensor
``set_tensor / invoke / get_tensor`` (``/root/reference/ops/map_classify_tpu.py:71-74``),
batched and pipelined:

  host (C++ HostStager thread)        copy stream              compute stream
  CSV rows -> pinned slot s   ──►  hipMemcpyAsync(slot s) ──►  tokenize (K1)
                                                                BERT encoder (K2-K6)
                                                                pooler + head/top-k (K7)
                                                                D2H top-k (pinned)

Two staging slots alternate, so extraction of batch i+1 (host threads), its
H2D copy (side stream) and the encoder of batch i (compute stream) overlap.
The whole device step for a full batch (tokenize -> top-k) is captured once per
slot into a hipGraph (``torch.cuda.CUDAGraph``) and replayed: one launch per
batch instead of ~100.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from .._native import native
from ..models.bert import BertClassifier, BertConfig
from ..models.params import ParamPack
from ..tokenizer import DEFAULT_MAX_ROW_BYTES, pack_rows
from ..utils.trace import DeviceStages, span
from .graphs import capture_graph


@dataclass
class BatchResult:
    rows: int
    idx: torch.Tensor    # [rows, k] int32 (host)
    score: torch.Tensor  # [rows, k] fp32 (host)


@dataclass
class RunStats:
    rows: int = 0
    batches: int = 0
    wall_s: float = 0.0
    timing_ms: Dict[str, float] = field(default_factory=dict)

    @property
    def rows_per_sec(self) -> float:
        return self.rows / self.wall_s if self.wall_s > 0 else 0.0


class ClassifyEngine:
    def __init__(self, cfg: BertConfig, pack: ParamPack, device: torch.device, batch_rows: int = 512,
                 seq_len: int = 128, topk: int = 5, max_row_bytes: int = DEFAULT_MAX_ROW_BYTES,
                 use_graph: bool = True, slots: int = 2, concurrent: Optional[bool] = None):
        if pack.buffer.device != device:
            pack = pack.to(device)
        self.cfg, self.pack, self.device = cfg, pack, device
        self.model = BertClassifier(cfg, pack)
        self.B, self.S = int(batch_rows), int(seq_len)
        self.k = max(1, min(int(topk), cfg.num_labels))
        self.max_row_bytes = int(max_row_bytes)
        self.use_graph = use_graph and device.type == "cuda"
        self.n_slots = slots
        cap = self.B * self.max_row_bytes
        self.text = [torch.empty(cap, dtype=torch.uint8, device=device) for _ in range(slots)]
        self.offs = [torch.zeros(self.B + 1, dtype=torch.int32, device=device) for _ in range(slots)]
        # per-slot token buffers: with concurrent slots two batches are in flight at once
        self.ids_s = [torch.zeros((self.B, self.S), dtype=torch.int32, device=device) for _ in range(slots)]
        self.lens_s = [torch.zeros(self.B, dtype=torch.int32, device=device) for _ in range(slots)]
        self.ids, self.lens = self.ids_s[0], self.lens_s[0]
        self.copy_stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        # Concurrent slots: batch i runs on compute stream i % slots, so the
        # encoders of two consecutive batches overlap on the GPU. A GEMM block
        # fills a CU (128 KiB LDS, full register file), so overlap happens at CU
        # granularity: the memory-bound kernels (attention, LayerNorm, GEMM store
        # tails) of one batch run on some CUs while the other batch's GEMM main
        # loops run on the rest, instead of every CU alternating between regimes.
        if concurrent is None:
            concurrent = os.getenv("ATPU_CONCURRENT_SLOTS", "1") not in ("0", "false", "no")
        self.concurrent = bool(concurrent) and device.type == "cuda" and slots > 1
        self.compute_streams = [torch.cuda.Stream(device) for _ in range(slots)] if self.concurrent else None
        # CU split (ATPU_CU_SPLIT=1): slot i's stream is CU-masked to an even 1/slots share of every
        # XCD, and persistent grids are sized for that share (process-wide cu_budget). Without it a
        # persistent GEMM holds every CU (146 KiB LDS per workgroup) and the other batch's kernels
        # only slot in at kernel boundaries.
        self.cu_split = self.concurrent and os.getenv("ATPU_CU_SPLIT", "0") not in ("0", "false", "no")
        if self.cu_split:
            nat = native()
            nat.cu_budget(0)
            share = (nat.num_cus() // slots) // 8 * 8
            self.compute_streams = [torch.cuda.ExternalStream(nat.make_cu_mask_stream(i * share, share), device=device)
                                    for i in range(slots)]
            nat.cu_budget(share)
        if device.type == "cuda" and self.model.can_fold(self.B, self.S):
            self.model.folded()  # build the LN-folded weights now, so memory_bytes() counts them
        self._graphs: Dict[int, Tuple["torch.cuda.CUDAGraph", Tuple[torch.Tensor, ...]]] = {}
        # stage-timed replay: the same step as three graphs (tokenize | encoder | head) with
        # hipEvents between them, so timing_ms carries device time per stage
        self._staged: Dict[int, Tuple[Tuple["torch.cuda.CUDAGraph", ...], Tuple[torch.Tensor, ...]]] = {}
        self._stager = None

    # ------------------------------------------------------------ device step
    def _step(self, slot: int, rows: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        ids, lens = self.ids_s[slot], self.lens_s[slot]
        ops.tokenize(self.text[slot], self.offs[slot], self.S, self.cfg.vocab_size, self.max_row_bytes,
                     ids=ids, lens=lens, rows=rows)
        return self.model.forward(ids[:rows], lens[:rows], self.k)

    def _graph_step(self, slot: int):
        if slot not in self._graphs:
            if not self._graphs:  # once per engine: the other slots' steps take the same kernels
                s = torch.cuda.Stream(self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):  # warm up allocator + code objects off-graph
                    self._step(slot, self.B)
                torch.cuda.current_stream(self.device).wait_stream(s)
            g, outs = capture_graph(lambda: self._step(slot, self.B))
            self._graphs[slot] = (g, outs)
        g, outs = self._graphs[slot]
        g.replay()
        return outs

    def _stage_fns(self, slot: int, rows: int):
        ids, lens = self.ids_s[slot], self.lens_s[slot]
        box = {}

        def tok():
            ops.tokenize(self.text[slot], self.offs[slot], self.S, self.cfg.vocab_size, self.max_row_bytes,
                         ids=ids, lens=lens, rows=rows)

        def enc():
            box["h"] = self.model.encoder(ids[:rows], lens[:rows])

        def head():
            box["out"] = self.model.head(box["h"], rows, self.S, self.k)
            return box["out"]

        return tok, enc, head

    def _staged_graphs(self, slot: int):
        if slot not in self._staged:
            tok, enc, head = self._stage_fns(slot, self.B)
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):  # warm-up off-graph
                tok(), enc(), head()
            torch.cuda.current_stream(self.device).wait_stream(s)
            pool = torch.cuda.graph_pool_handle()
            gs = []
            outs = None
            for fn in (tok, enc, head):
                g, r = capture_graph(fn, pool=pool)
                gs.append(g)
                outs = r if r is not None else outs
            self._staged[slot] = (tuple(gs), outs)
        return self._staged[slot]

    def run_slot(self, slot: int, rows: int, stages: Optional[DeviceStages] = None, stream=None):
        if rows < self.B and ops.batch_invariant():
            # batch invariance: a partial batch (a shard's tail) runs the full-batch step like every
            # other batch -- an M-sized eager step could take other kernels (the folded encoder needs
            # M >= 2048 and whole 256-row tiles) -- its extra rows empty strings, their results unused
            offs = self.offs[slot]
            offs[rows + 1:].copy_(offs[rows:rows + 1].expand(self.B - rows))
            rows = self.B
        if stages is None:
            if self.use_graph and rows == self.B:
                return self._graph_step(slot)
            return self._step(slot, rows)
        ev = DeviceStages.event
        if self.use_graph and rows == self.B:
            gs, outs = self._staged_graphs(slot)
            fns = [g.replay for g in gs]
        else:
            fns, outs = list(self._stage_fns(slot, rows)), None
        marks = [ev(stream)]
        res = None
        for fn in fns:
            r = fn()
            res = r if r is not None else res
            marks.append(ev(stream))
        for name, a, b in zip(("tokenize", "encoder", "head"), marks, marks[1:]):
            stages.add(name, a, b)
        return outs if outs is not None else res

    # -------------------------------------------------------------- host APIs
    # ------------------------------------------------- small jobs (texts / input)
    # The per-job forms (the reference's one-row ``input`` job, short ``texts`` lists)
    # replay a captured graph too: rows are padded up to a power-of-two bucket (8 .. B),
    # so a job costs one H2D from pinned staging, one graph launch and one D2H instead
    # of ~100 eager launches (padding rows are empty and their results dropped).
    def _bucket(self, n: int) -> int:
        # batch invariance: at least 16 rows (2048 tokens), so every bucket takes the LayerNorm-
        # folded encoder (ops.fold_ok: M >= 2048, whole 256-row tiles) that the big batches take
        b = 16 if ops.batch_invariant() else 8
        while b < n:
            b *= 2
        return min(b, self.B)

    def _pinned(self):
        if getattr(self, "_pin", None) is None:
            self._pin = {
                "ids": torch.zeros((self.B, self.S), dtype=torch.int32, pin_memory=True),
                "lens": torch.ones(self.B, dtype=torch.int32, pin_memory=True),
                "text": torch.zeros(self.B * self.max_row_bytes, dtype=torch.uint8, pin_memory=True),
                "offs": torch.zeros(self.B + 1, dtype=torch.int32, pin_memory=True),
            }
            self._bpool = torch.cuda.graph_pool_handle()
            self._bgraphs = {}
        return self._pin

    def _bucket_graph(self, kind: str, bucket: int):
        key = (kind, bucket)
        if key not in self._bgraphs:
            ids, lens = self.ids_s[0][:bucket], self.lens_s[0][:bucket]

            def fn():
                if kind == "text":
                    ops.tokenize(self.text[0], self.offs[0], self.S, self.cfg.vocab_size, self.max_row_bytes,
                                 ids=self.ids_s[0], lens=self.lens_s[0], rows=bucket)
                return self.model.forward(ids, lens, self.k)

            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):  # warm-up off-graph
                fn()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._bgraphs[key] = capture_graph(fn, pool=self._bpool)
        return self._bgraphs[key]

    def _run_bucket(self, kind: str, m: int, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        bk = self._bucket(m)
        if self.use_graph:
            g, (_, idx, sc) = self._bucket_graph(kind, bk)
            g.replay()
        else:
            if kind == "text":
                ops.tokenize(self.text[0], self.offs[0], self.S, self.cfg.vocab_size, self.max_row_bytes,
                             ids=self.ids_s[0], lens=self.lens_s[0], rows=bk)
            _, idx, sc = self.model.forward(self.ids_s[0][:bk], self.lens_s[0][:bk], self.k)
        both = torch.cat([idx[:m, :k].view(torch.float32), sc[:m, :k]], 1).cpu()  # one D2H, one sync
        return both[:, :k].contiguous().view(torch.int32), both[:, k:].contiguous()

    def classify_ids(self, ids: torch.Tensor, lens: torch.Tensor, k: Optional[int] = None) -> BatchResult:
        """Pre-tokenized rows ``ids [n, S]`` / ``lens [n]`` (host tensors) -> top-k on the host."""
        k = self.k if k is None else max(1, min(int(k), self.k))
        n = int(ids.shape[0])
        if self.device.type != "cuda":
            _, idx, sc = self.model.forward(ids.to(torch.int32), lens.to(torch.int32), k)
            return BatchResult(n, idx[:, :k].cpu(), sc[:, :k].cpu())
        pin = self._pinned()
        idx_all, sc_all = [], []
        for c0 in range(0, n, self.B):
            m = min(self.B, n - c0)
            bk = self._bucket(m)
            pin["ids"][:m].copy_(ids[c0:c0 + m])
            pin["ids"][m:bk].zero_()
            pin["lens"][:m].copy_(lens[c0:c0 + m])
            pin["lens"][m:bk].fill_(1)
            self.ids_s[0][:bk].copy_(pin["ids"][:bk], non_blocking=True)
            self.lens_s[0][:bk].copy_(pin["lens"][:bk], non_blocking=True)
            i, s_ = self._run_bucket("ids", m, k)  # its D2H synchronizes: the pinned rows are free again
            idx_all.append(i)
            sc_all.append(s_)
        if not idx_all:
            return BatchResult(0, torch.zeros((0, k), dtype=torch.int32), torch.zeros((0, k)))
        return BatchResult(n, torch.cat(idx_all), torch.cat(sc_all))

    def classify_texts(self, rows: Sequence, k: Optional[int] = None) -> BatchResult:
        """Classify an in-memory list of strings (small jobs; no CSV)."""
        k = self.k if k is None else max(1, min(int(k), self.cfg.num_labels))
        idx_all, sc_all = [], []
        for b0 in range(0, len(rows), self.B):
            chunk = rows[b0:b0 + self.B]
            text, offs = pack_rows(r[:self.max_row_bytes] if isinstance(r, (bytes, bytearray)) else
                                   r.encode("utf-8")[:self.max_row_bytes] for r in chunk)
            n = len(chunk)
            if self.device.type == "cuda":
                pin = self._pinned()
                bk = self._bucket(n)
                pin["text"][:text.size].copy_(torch.from_numpy(text))
                pin["offs"][:n + 1].copy_(torch.from_numpy(offs))
                pin["offs"][n + 1:bk + 1].fill_(int(offs[-1]))  # padding rows: empty strings
                if text.size:
                    self.text[0][:text.size].copy_(pin["text"][:text.size], non_blocking=True)
                self.offs[0][:bk + 1].copy_(pin["offs"][:bk + 1], non_blocking=True)
                i, s_ = self._run_bucket("text", n, min(k, self.k))
                idx_all.append(i)
                sc_all.append(s_)
            else:
                ids, lens = ops.tokenize(torch.from_numpy(text), torch.from_numpy(offs), self.S,
                                         self.cfg.vocab_size, self.max_row_bytes)
                logits, idx, sc = self.model.forward(ids, lens, k)
                idx_all.append(idx.cpu())
                sc_all.append(sc.cpu())
        if not idx_all:
            return BatchResult(0, torch.zeros((0, k), dtype=torch.int32), torch.zeros((0, k)))
        return BatchResult(len(rows), torch.cat(idx_all), torch.cat(sc_all))

    def _get_stager(self):
        if self._stager is None:
            self._stager = native().HostStager(self.n_slots, self.B * self.max_row_bytes, self.B)
        return self._stager

    def classify_table(self, table, start: int, n: int, col: int, host_threads: Optional[int] = None,
                       out_idx: Optional[torch.Tensor] = None, out_score: Optional[torch.Tensor] = None,
                       stage_timing: bool = False) -> Tuple[torch.Tensor, torch.Tensor, RunStats]:
        """Pipelined classification of CSV rows ``[start, start+n)``.

        Returns device tensors ``idx[n,k]`` / ``score[n,k]`` (left on the GPU
        so a DP caller can all-gather them without a host round trip).
        ``stats.timing_ms``: ``host_*_ms`` host-side spans (stager waits, launch
        enqueue, the final drain); with ``stage_timing`` also ``device_*_ms``, GPU
        time per stage from hipEvent pairs (h2d: the copies on the copy stream,
        timed by the native stager after its wait for the slot's consumer;
        tokenize / encoder / head replayed as three graphs; the top-k copy-out),
        and ``device_span_ms`` (see :class:`DeviceStages`).
        """
        assert self.device.type == "cuda", "classify_table needs a ROCm device"
        if host_threads is None:
            from ..parallel.placement import host_threads as budget

            host_threads = budget(8)  # this rank's NUMA share (placement.py), at most the tuned 8
        n = max(0, min(int(n), table.num_rows - int(start)))
        dev = self.device
        out_idx = torch.empty((n, self.k), dtype=torch.int32, device=dev) if out_idx is None else out_idx
        out_score = torch.empty((n, self.k), dtype=torch.float32, device=dev) if out_score is None else out_score
        stats = RunStats()
        if n == 0:
            return out_idx, out_score, stats
        st = self._get_stager()
        caller = torch.cuda.current_stream(dev)
        streams = self.compute_streams or [caller] * self.n_slots
        for s in streams:
            if s is not caller:
                s.wait_stream(caller)  # out_* and earlier work were enqueued on the caller's stream
        cs = int(self.copy_stream.cuda_stream)
        nb = (n + self.B - 1) // self.B
        t0 = time.perf_counter()
        tm = stats.timing_ms  # host_* spans (+ roctx ranges under MI355X_TRACE=1); device_* from hipEvents
        dst = DeviceStages() if stage_timing else None
        ev = DeviceStages.event
        with span("host_csv_stage_ms", tm):
            st.submit(0, table, start, min(self.B, n), col, self.max_row_bytes, host_threads)
        def stage_next(i: int) -> None:
            if i + 1 < nb:
                b1 = start + (i + 1) * self.B
                with span("host_csv_stage_ms", tm):
                    st.submit((i + 1) % self.n_slots, table, b1, min(self.B, start + n - b1), col,
                              self.max_row_bytes, host_threads)

        for i in range(nb):
            slot = i % self.n_slots
            if self.n_slots > 1:  # batch i+1 stages into the other slot while batch i runs
                stage_next(i)
            stream = streams[slot]
            ks = int(stream.cuda_stream)
            with torch.cuda.stream(stream):
                with span("host_stager_wait_ms", tm):
                    rows, _ = st.upload(slot, self.text[slot].data_ptr(), self.text[slot].numel(),
                                        self.offs[slot].data_ptr(), cs, ks)
                with span("host_launch_ms", tm):
                    _, idx, sc = self.run_slot(slot, int(rows), dst, stream)
                st.release(slot, ks)
                if self.n_slots == 1:  # one slot: the next batch stages once this one released it
                    stage_next(i)
                r0 = i * self.B
                c0 = ev(stream) if dst else None
                out_idx[r0:r0 + rows].copy_(idx[:rows], non_blocking=True)
                out_score[r0:r0 + rows].copy_(sc[:rows], non_blocking=True)
                if dst:
                    dst.add("copy_out", c0, ev(stream))
            stats.batches += 1
        for s in streams:
            if s is not caller:
                caller.wait_stream(s)
        with span("host_drain_ms", tm):
            torch.cuda.synchronize(dev)
        h2d_ms, _ = st.take_h2d_ms()  # hipEvent pairs around the copies (native stager)
        if dst:
            dst.resolve(tm)
            tm["device_h2d_ms"] = round(h2d_ms, 3)
        stats.rows = n
        stats.wall_s = time.perf_counter() - t0
        return out_idx, out_score, stats

    def memory_bytes(self) -> int:
        """Resident device bytes: weights, the LayerNorm-folded weight copies once built
        (they are ~45 % of the encoder weights), staging and token buffers."""
        folded = getattr(self.model, "_folded", None) or {}
        extra = sum(t.numel() * t.element_size() for t in folded.values())
        return (self.pack.nbytes + extra + sum(t.numel() for t in self.text)
                + sum(t.numel() * 4 for t in self.ids_s) + sum(t.numel() * 4 for t in self.offs))


def activation_bytes_per_row(cfg: BertConfig, seq_len: int) -> int:
    """Peak transient device bytes per batch row (bf16 activations, one layer live)."""
    H, I, S = cfg.hidden, cfg.intermediate, seq_len
    per_tok = 2 * (H * 4 + 3 * H + I)  # h, h1, ctx, h2 + qkv + ffn (bf16)
    return S * per_tok + DEFAULT_MAX_ROW_BYTES + 8 * S
