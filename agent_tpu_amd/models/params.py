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
        # a pageable host -> HBM copy runs at ~56 GB/s on MI355X (tools/probe_h2d.py: as fast as
        # from pinned memory; two-slot pinned staging measured 40 GB/s), so no staging here
        out.buffer = self.buffer.to(device)
        out._views = out._make_views()
        return out

    def with_dtype(self, float_dtype: torch.dtype) -> Dict[str, torch.Tensor]:
        """Plain dict of copies with floating params cast (CPU oracle uses fp32)."""
        return {k: (v.to(float_dtype) if v.is_floating_point() else v.clone()) for k, v in self._views.items()}
