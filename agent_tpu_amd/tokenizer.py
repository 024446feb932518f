"""atpu-hash-wordpiece v1 — the tokenizer the GPU K1 kernel implements.

There is no subword vocabulary in the reference: ``map_tokenize`` is character
chunking (``/root/reference/ops/map_tokenize.py:6-9``) and ``map_classify_tpu``
consumes pre-tokenized ids (``map_classify_tpu.CONTRACT.md:7-8,23``). With
random-init weights a deterministic hash tokenizer is the contractually
honest choice. Spec:

* bytes 0x09-0x0D and 0x20 separate tokens; other control bytes (<0x20, 0x7F)
  are dropped and also separate;
* each ASCII punctuation byte is a token of its own (BERT BasicTokenizer);
* every other byte (ASCII alnum, UTF-8 >= 0x80) is a word byte, A-Z folded
  to lower case;
* a word is cut into pieces of at most 24 bytes; piece 0 hashes from the
  FNV-1a-32 offset basis, later pieces from the FNV state after "##";
* ``id = 1000 + fnv % (vocab - 1000)``; ``[CLS]=101 … [SEP]=102`` then
  ``[PAD]=0`` up to ``seq_len``; ``len = tokens + 2``.

Three implementations must agree bit-for-bit: :func:`tokenize_rows` (pure
Python, this file), ``_atpu.tokenize_host`` (C++) and the HIP kernel.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np

CLS_ID, SEP_ID, PAD_ID = 101, 102, 0
FIRST_HASH_ID = 1000
PIECE_BYTES = 24
DEFAULT_MAX_ROW_BYTES = 2048
_BASIS, _PRIME = 2166136261, 16777619


def _byte_class(c: int) -> int:
    if c == 0x20 or 0x09 <= c <= 0x0D or c < 0x20 or c == 0x7F:
        return 0
    if 0x21 <= c <= 0x2F or 0x3A <= c <= 0x40 or 0x5B <= c <= 0x60 or 0x7B <= c <= 0x7E:
        return 1
    return 2


_CLASS = bytes(_byte_class(c) for c in range(256))


def _fnv(h: int, data: bytes) -> int:
    for c in data:
        if 0x41 <= c <= 0x5A:
            c += 32
        h = ((h ^ c) * _PRIME) & 0xFFFFFFFF
    return h


_CONT = _fnv(_BASIS, b"##")


def token_ids(row: bytes, vocab: int, cap: int) -> List[int]:
    """Hash-token ids of one row (no specials), at most ``cap`` of them."""
    mod = vocab - FIRST_HASH_ID
    out: List[int] = []
    i, n = 0, len(row)
    while i < n and len(out) < cap:
        k = _CLASS[row[i]]
        if k == 0:
            i += 1
            continue
        if k == 1:
            out.append(FIRST_HASH_ID + _fnv(_BASIS, row[i:i + 1]) % mod)
            i += 1
            continue
        j = i
        while j < n and _CLASS[row[j]] == 2:
            j += 1
        for p, b0 in enumerate(range(i, j, PIECE_BYTES)):
            if len(out) >= cap:
                break
            h = _fnv(_BASIS if p == 0 else _CONT, row[b0:min(j, b0 + PIECE_BYTES)])
            out.append(FIRST_HASH_ID + h % mod)
        i = j
    return out


def tokenize_rows(rows: Sequence[bytes], seq_len: int, vocab: int,
                  max_row_bytes: int = DEFAULT_MAX_ROW_BYTES) -> Tuple[np.ndarray, np.ndarray]:
    """Pure-Python reference: returns ``ids[B, seq_len]`` and ``lens[B]`` (int32)."""
    ids = np.zeros((len(rows), seq_len), dtype=np.int32)
    lens = np.zeros(len(rows), dtype=np.int32)
    for r, row in enumerate(rows):
        toks = token_ids(bytes(row[:max_row_bytes]), vocab, seq_len - 2)
        ids[r, 0] = CLS_ID
        ids[r, 1:1 + len(toks)] = toks
        ids[r, 1 + len(toks)] = SEP_ID
        lens[r] = len(toks) + 2
    return ids, lens


def pack_rows(rows: Iterable) -> Tuple[np.ndarray, np.ndarray]:
    """Pack str/bytes rows into (uint8 text, int32 offsets[B+1])."""
    blobs = [r.encode("utf-8") if isinstance(r, str) else bytes(r) for r in rows]
    offsets = np.zeros(len(blobs) + 1, dtype=np.int32)
    if blobs:
        offsets[1:] = np.cumsum([len(b) for b in blobs])
    text = np.frombuffer(b"".join(blobs), dtype=np.uint8).copy() if blobs else np.zeros(0, np.uint8)
    return text, offsets
