"""Synthetic CSV shards for benchmarks and tests (no datasets are downloadable).

Rows look like ``id,text,risk`` (the column set of the reference's csv_shard
probes). ``text`` is a sentence of random words from a
fixed synthetic vocabulary, with punctuation and some quoting, long enough by
default to fill a 128-token BERT window.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

_SYLL = ["ka", "lo", "mi", "ra", "ten", "vo", "qua", "zi", "ber", "nox", "al", "pe", "dru", "sim", "ox", "ul"]
_PUNCT = [",", ".", ";", "!", "?", "-", "(", ")"]


def _vocab(rng: np.random.Generator, size: int = 4096):
    words = set()
    while len(words) < size:
        n = int(rng.integers(1, 5))
        words.add("".join(rng.choice(_SYLL, n)))
    return sorted(words)


def make_text_rows(n: int, words_per_row: int = 150, seed: int = 0):
    rng = np.random.default_rng(seed)
    vocab = np.array(_vocab(rng), dtype=object)
    out = []
    for _ in range(n):
        w = vocab[rng.integers(0, len(vocab), words_per_row)]
        toks = []
        for j, word in enumerate(w):
            toks.append(word.capitalize() if j == 0 else word)
            if rng.random() < 0.06:
                toks.append(_PUNCT[int(rng.integers(0, len(_PUNCT)))])
        out.append(" ".join(toks))
    return out


def write_csv(path: str, n: int, words_per_row: int = 150, seed: int = 0, quote_every: int = 7) -> str:
    """Write ``n`` rows; every ``quote_every``-th text is quoted with an embedded comma/quote/newline."""
    import csv

    rows = make_text_rows(n, words_per_row, seed)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w", encoding="utf-8", newline="") as f:
        w = csv.writer(f, lineterminator="\n")  # excel dialect, QUOTE_MINIMAL
        w.writerow(["id", "text", "risk"])
        for i, t in enumerate(rows):
            if quote_every and i % quote_every == 3:
                t = t + ', said "x"\nend'
            w.writerow([i, t, (i % 1000) / 1000.0])
    os.replace(tmp, path)
    return path


def ensure_csv(path: str, n: int, words_per_row: int = 150, seed: int = 0) -> str:
    if not os.path.exists(path):
        write_csv(path, n, words_per_row, seed)
    return path
