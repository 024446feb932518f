#!/usr/bin/env python3
"""Does the cross-attention K/V layout matter? (decode step, T5-base shapes, src 1024)

The encoder's cross K/V live as ``[docs*S, L*2d]`` rows (one GEMM writes every layer's
K|V): one head's 128-B slice of consecutive keys sits 36.9 KB apart. This times the
grouped cross-attention kernel on (a) that layout (layer 0 slice, 12 heads) and (b) the
same bytes laid out head-major (``H = 1`` over 12x the documents, keys contiguous:
one 128 KiB block per (doc, head)), to decide whether a head-major cross-KV layout is
worth a scatter epilogue.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_tpu_amd import ops  # noqa: E402


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    docs, S, H, L, nb = 256, 1024, 12, 12, 4
    d = H * 64
    ckv = torch.randn(docs * S, L * 2 * d, device=dev).to(torch.bfloat16)
    lens = torch.full((docs,), S, dtype=torch.int32, device=dev)
    q = torch.randn(docs * nb, d, device=dev).to(torch.bfloat16)
    a = t(lambda: ops.decode_attention(q, ckv[:, :d], ckv[:, d:2 * d], H, S, nb, lens=lens))
    kv_b = torch.randn(docs * H * S, 2 * 64, device=dev).to(torch.bfloat16)  # head-major, K|V per key
    lens_b = torch.full((docs * H,), S, dtype=torch.int32, device=dev)
    q_b = torch.randn(docs * H * nb, 64, device=dev).to(torch.bfloat16)
    b = t(lambda: ops.decode_attention(q_b, kv_b[:, :64], kv_b[:, 64:], 1, S, nb, lens=lens_b))
    kv_c = torch.randn(docs * S, 2 * d, device=dev).to(torch.bfloat16)  # one layer's K|V rows only (3 KB rows)
    c = t(lambda: ops.decode_attention(q, kv_c[:, :d], kv_c[:, d:], H, S, nb, lens=lens))
    gb = docs * S * d * 2 * 2 / 1e9
    print(json.dumps({"bytes_GB": round(gb, 3),
                      "rows_all_layers_us": round(a, 1), "TBps_a": round(gb / a * 1e3, 2),
                      "head_major_us": round(b, 1), "TBps_b": round(gb / b * 1e3, 2),
                      "rows_one_layer_us": round(c, 1), "TBps_c": round(gb / c * 1e3, 2)}))


if __name__ == "__main__":
    main()
