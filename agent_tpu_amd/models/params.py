"""ParamPack: every model parameter as a typed view into ONE flat byte buffer.

One buffer per model means model load / switch is a single
``dist.broadcast`` (219 MB for BERT-base bf16) instead of
hundreds of small collectives, and a single H2D copy. Views are 256-byte
aligned so every kernel operand satisfies the 16-byte load alignment.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, Tuple

import torch

_ALIGN = 256


class ParamPack:
    def __init__(self, specs: Iterable[Tuple[str, Tuple[int, ...], torch.dtype]], device="cpu"):
        self.specs = list(specs)
        self.layout: "OrderedDict[str, Tuple[int, Tuple[int, ...], torch.dtype]]" = OrderedDict()
        off = 0
        for name, shape, dtype in self.specs:
            n = 1
            for d in shape:
                n *= d
            nbytes = n * torch.empty((), dtype=dtype).element_size()
            self.layout[name] = (off, tuple(shape), dtype)
            off += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        self.nbytes = off
        self.buffer = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self._views = self._make_views()

    def _make_views(self) -> Dict[str, torch.Tensor]:
        views = {}
        for name, (off, shape, dtype) in self.layout.items():
            n = 1
            for d in shape:
                n *= d
            esz = torch.empty((), dtype=dtype).element_size()
            views[name] = self.buffer[off:off + n * esz].view(dtype).view(shape)
        return views

    def __getitem__(self, name: str) -> torch.Tensor:
        return self._views[name]

    def __contains__(self, name: str) -> bool:
        return name in self._views

    def names(self):
        return list(self.layout)

    def adopt(self, buffer: torch.Tensor) -> "ParamPack":
        """A pack with this layout over ``buffer`` (a copy of this pack's bytes, e.g. on a GPU)."""
        assert buffer.numel() == self.nbytes and buffer.dtype == torch.uint8
        out = ParamPack.__new__(ParamPack)
        out.specs, out.layout, out.nbytes = self.specs, self.layout, self.nbytes
        out.buffer = buffer
        out._views = out._make_views()
        return out

    def to(self, device) -> "ParamPack":
        out = ParamPack.__new__(ParamPack)
        out.specs, out.layout, out.nbytes = self.specs, self.layout, self.nbytes
        # pageable host -> HBM (a checkpoint load; random init is built on the device instead,
        # params.rand_fill). bench/cold_load.py --h2d: the FIRST copy of a process pays ~140 ms
        # of one-time HIP copy-path setup (a 4 KiB copy takes it all) and a never-copied source
        # buffer ~6-15 ms of page registration; a repeat copy of a 219 MB buffer runs at 56 GB/s
        # (as fast as from pinned memory; two-slot pinned staging measured 40 GB/s)
        out.buffer = self.buffer.to(device)
        out._views = out._make_views()
        return out

    def with_dtype(self, float_dtype: torch.dtype) -> Dict[str, torch.Tensor]:
        """Plain dict of copies with floating params cast (CPU oracle uses fp32)."""
        return {k: (v.to(float_dtype) if v.is_floating_point() else v.clone()) for k, v in self._views.items()}


def _sid(name: str) -> int:
    """Stream id of a parameter: FNV-1a-64 of its name (adding a tensor shifts no other)."""
    h = 0xCBF29CE484222325
    for b in name.encode():
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def rand_fill(t: torch.Tensor, seed: int, name: str, std: float, n0: int = -1, std1: float = 0.0) -> None:
    """Seeded N(0, std^2)-like init of ``t`` in place (Irwin-Hall(4), ``csrc/include/atpu/rand.h``):
    on a GPU tensor the ``rand_fill`` kernel writes it where it lives, on a CPU tensor the native
    twin does; both give the same bits. Elements ``[n0, numel)`` take ``std1`` when ``n0 >= 0``."""
    from .._native import native

    assert t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32), (t.dtype, t.shape)
    nat = native()
    n = t.numel()
    norm = 2.6428997921303014e-05  # atpu::rnd::kIh4Norm
    s0 = float(std * norm)
    s1 = float(std1 * norm) if n0 >= 0 else s0
    n0 = n if n0 < 0 else n0
    args = (t.data_ptr(), n, t.dtype == torch.float32, int(seed) & 0xFFFFFFFFFFFFFFFF, _sid(name), s0, n0, s1)
    if t.is_cuda:
        with torch.cuda.device(t.device):
            nat.rand_fill(*args, torch.cuda.current_stream(t.device).cuda_stream)
    else:
        nat.rand_fill_host(*args, max(1, min(8, torch.get_num_threads())))
