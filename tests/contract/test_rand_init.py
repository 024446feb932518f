"""Counter-based random init (csrc/include/atpu/rand.h, models/params.rand_fill): the CPU twin
is deterministic, independent of the thread count and of the other tensors of a pack, and
N(0, std^2)-like; the GPU kernel's bits are pinned against it in
tests/kernels/test_runtime_gpu.py::test_rand_fill_gpu_matches_host."""
import torch

from agent_tpu_amd.models.params import rand_fill


def test_rand_fill_host_deterministic_and_thread_independent():
    a = torch.empty(300_001, dtype=torch.bfloat16)
    b = torch.empty_like(a)
    rand_fill(a, 7, "l0.qkv_w", 0.02)
    torch.set_num_threads(1)
    try:
        rand_fill(b, 7, "l0.qkv_w", 0.02)
    finally:
        torch.set_num_threads(8)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    c = torch.empty_like(a)
    rand_fill(c, 8, "l0.qkv_w", 0.02)  # another seed
    d = torch.empty_like(a)
    rand_fill(d, 7, "l1.qkv_w", 0.02)  # another tensor
    assert (a != c).float().mean() > 0.9 and (a != d).float().mean() > 0.9


def test_rand_fill_distribution_and_split_scale():
    x = torch.empty(1 << 20, dtype=torch.float32)
    rand_fill(x, 0, "w", 1.0)
    assert abs(x.mean().item()) < 5e-3 and abs(x.std().item() - 1.0) < 5e-3
    assert x.abs().max().item() <= 3.47  # Irwin-Hall(4) support: +-sqrt(12)
    y = torch.empty(1000, dtype=torch.float32)
    rand_fill(y, 0, "w", 0.5, n0=400, std1=2.0)
    z = torch.empty(1000, dtype=torch.float32)
    rand_fill(z, 0, "w", 1.0)
    torch.testing.assert_close(y[:400], z[:400] * 0.5, rtol=0, atol=0)
    torch.testing.assert_close(y[400:], z[400:] * 2.0, rtol=0, atol=0)


def test_bert_pack_built_the_same_twice():
    from agent_tpu_amd.models.bert import config_for, init_random

    cfg = config_for("bert-tiny", num_labels=3)
    p1, p2 = init_random(cfg, seed=3), init_random(cfg, seed=3)
    assert torch.equal(p1.buffer, p2.buffer)
    assert p1["l0.ln1_g"].eq(1).all() and p1["l0.qkv_b"].eq(0).all() and p1["l0.qkv_w"].float().std() > 0.015
