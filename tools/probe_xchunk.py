"""Chunked vs split cross attention under batch invariance: where do they differ?
(one GPU process; prints one line per configuration)."""
import sys

import torch

sys.path.insert(0, ".")
from agent_tpu_amd import ops  # noqa: E402


def _r(shape, dev, scale=1.0, seed=0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dev, dtype)


def main():
    dev = torch.device("cuda:0")
    ops.set_batch_invariant(True)
    for group, S, H, items, L in [(8, 2048, 16, 40, 1560), (8, 1024, 16, 40, 1000), (4, 2048, 16, 40, 1560),
                                  (8, 2048, 16, 40, 2048), (8, 2048, 12, 48, 1560), (4, 1024, 12, 64, 536),
                                  (8, 2048, 16, 40, 1600), (8, 2048, 16, 40, 64 * 20)]:
        d = H * 64
        q = _r((items * group, 3 * d), dev, 1.0, 81)[:, :d]
        kv = _r((items * S, 2 * d), dev, 1.0, 82)
        lens = torch.randint(1, S + 1, (items,), generator=torch.Generator().manual_seed(L), dtype=torch.int32).to(dev)
        lens[0] = L
        bias = _r((H, S), dev, 1.0, 84, torch.float32)
        many = ops.decode_attention(q, kv[:, :d], kv[:, d:], H, S, group, lens=lens, bias_dist=bias, scale=0.125)
        ones = [ops.decode_attention(q[i * group:(i + 1) * group], kv[i * S:(i + 1) * S, :d],
                                     kv[i * S:(i + 1) * S, d:], H, S, group, lens=lens[i:i + 1], bias_dist=bias,
                                     scale=0.125) for i in range(items)]
        a = many.float()
        b = torch.cat(ones).float()
        diff = (a != b)
        print(f"group {group} S {S} H {H} items {items} len {L}: mismatches {int(diff.sum())} of {diff.numel()} "
              f"maxdiff {float((a - b).abs().max()):.3g}", flush=True)


if __name__ == "__main__":
    main()
