#!/usr/bin/env python3
"""Where the wave-specialised QKV+attention kernel spends its cycles (diagnostic).

Needs the stamp build of the extension (``python agent_tpu_amd/csrc/build.py -D ATPU_WS_STAMPS
--out abso/_atpu_stamps.so`` and ``ATPU_NATIVE_PATH`` pointing at it): the kernel sums s_memtime
spans per workgroup (qkv_attn_ws.hip, ``g_ws_stamps``). After ~2 s of back-to-back launches on
random data (the clock the chip holds under load), one more launch is read back; per mode and
variant one JSON line with the per-tile means in cycles and as a share of the total.
Usage: python tools/ws_stamps.py [--variants 8] [--rows 131072]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from agent_tpu_amd._native import native  # noqa: E402
from agent_tpu_amd import ops  # noqa: E402
from agent_tpu_amd.ops.qkv_attention import qkv_ws  # noqa: E402

M_KEYS = ["kb_wait", "eb_wait", "image_writes", "total", "tiles"]
L_KEYS = ["bar_wait", "dma_wait", "total", "chunk8"] + [f"chunk{c}" for c in range(1, 8)]  # slots 5..15


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--variants", default="8")
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    nat = native()
    dev = torch.device("cuda", 0)
    M, K, N = a.rows, 768, 2304
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.1
    fin = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
    col = w.float().sum(1).contiguous()
    lens = torch.full((M // 128,), 128, dtype=torch.int32, device=dev)
    ctx = torch.empty(M, N // 3, dtype=torch.bfloat16, device=dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    nb = min((M // 128) * (N // 192), torch.cuda.get_device_properties(dev).multi_processor_count) & ~7
    for var in [int(v) for v in a.variants.split(",")]:
        nat.ws_variant(var)
        for mode in (2, 1):
            def run():
                if mode == 2:
                    ops.qkv_attention(x, w, b, lens, N // 192, in_fin=fin, colsum_h=col, out=ctx, kernel="ws")
                else:
                    qkv_ws(x, w, b, out, 1, in_fin=fin, colsum_h=col)
            run()
            torch.cuda.synchronize()
            t0 = time.time()
            n = 0
            while time.time() - t0 < a.seconds:
                run()
                n += 1
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            st = torch.tensor(nat.ws_stamps(nb), dtype=torch.float64).view(nb, 16)
            tiles = st[:, 4].clamp(min=1)
            rec = {"mode": mode, "variant": var, "us": round(e0.elapsed_time(e1) * 1e3, 1), "warm_launches": n,
                   "blocks": nb, "tiles_per_block": round(tiles.mean().item(), 2)}
            tot_m = st[:, 3].mean().item()
            rec["clock_ghz_est"] = round(tot_m / (e0.elapsed_time(e1) * 1e6), 3)
            per_tile = {}
            for i, k in enumerate(M_KEYS[:4]):
                per_tile["mma_" + k] = round((st[:, i] / tiles).mean().item())
            for j, k in enumerate(L_KEYS):
                per_tile["ld_" + k] = round((st[:, 5 + j] / tiles).mean().item())
            rec["cycles_per_tile"] = per_tile
            rec["mma_share"] = {k: round(per_tile["mma_" + k] / max(per_tile["mma_total"], 1), 3)
                                for k in M_KEYS[:3]}
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
