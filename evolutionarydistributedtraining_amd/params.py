"""Parameter arenas: a model's parameters as ONE flat, contiguous HBM buffer.

The reference walks `model.parameters()` tensor by tensor in Python (EDT_LM/diloco.py:240-250);
on MI355X the whole population state lives in flat arenas instead, one per replica, laid out in
`parameters()` order (the index order torch.optim state uses). A fused kernel then sweeps an
arena in one launch, and a module whose parameters are re-pointed into an arena
(`bind_module_`) is updated in place by that launch with no gather/scatter copies.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch


@dataclass
class ParamLayout:
    """Shapes and flat offsets of a parameter list (in order)."""
    shapes: list[torch.Size]
    names: list[str] = field(default_factory=list)

    def __post_init__(self):
        self.numels = [int(torch.Size(s).numel()) for s in self.shapes]
        self.offsets = [0]
        for n in self.numels:
            self.offsets.append(self.offsets[-1] + n)

    @property
    def total(self) -> int:
        return self.offsets[-1]

    def __len__(self) -> int:
        return len(self.shapes)

    @classmethod
    def of(cls, tensors, names=None) -> "ParamLayout":
        return cls([t.shape for t in tensors], list(names or []))

    @classmethod
    def of_module(cls, module: torch.nn.Module) -> "ParamLayout":
        named = list(module.named_parameters())
        return cls([p.shape for _, p in named], [n for n, _ in named])

    def views(self, flat: torch.Tensor) -> list[torch.Tensor]:
        return [flat[a:a + n].view(s) for a, n, s in zip(self.offsets, self.numels, self.shapes)]


class ParamArena:
    """One flat device buffer holding a whole parameter list."""

    def __init__(self, layout: ParamLayout, dtype: torch.dtype, device, flat: torch.Tensor | None = None):
        self.layout = layout
        if flat is None:
            flat = torch.empty(layout.total, dtype=dtype, device=device)
        if flat.numel() != layout.total or not flat.is_contiguous():
            raise ValueError("arena buffer does not match the layout")
        self.flat = flat

    @property
    def dtype(self) -> torch.dtype:
        return self.flat.dtype

    @property
    def device(self) -> torch.device:
        return self.flat.device

    def views(self) -> list[torch.Tensor]:
        return self.layout.views(self.flat)

    def load_(self, tensors) -> "ParamArena":
        """Copy a tensor list into the arena (dtype cast = torch copy_ rounding)."""
        for v, t in zip(self.views(), tensors):
            v.copy_(t)
        return self

    @classmethod
    def from_tensors(cls, tensors, dtype=None, device=None) -> "ParamArena":
        tensors = list(tensors)
        layout = ParamLayout.of(tensors)
        dtype = dtype or tensors[0].dtype
        device = device or tensors[0].device
        return cls(layout, dtype, device).load_(tensors)


def bind_module_(module: torch.nn.Module, arena: ParamArena, copy: bool = True) -> ParamArena:
    """Re-point every parameter of `module` at its slice of `arena` (optionally copying the
    current values in first). Afterwards kernels that update the arena update the module."""
    params = list(module.parameters())
    if len(params) != len(arena.layout) or any(p.shape != s for p, s in zip(params, arena.layout.shapes)):
        raise ValueError("module parameters do not match the arena layout")
    views = arena.views()
    with torch.no_grad():
        for p, v in zip(params, views):
            if copy:
                v.copy_(p)
            p.data = v
    return arena


def arena_of_module(module: torch.nn.Module, dtype=None, device=None) -> ParamArena:
    """Allocate an arena for `module`, copy its parameters in and bind the module to it."""
    params = list(module.parameters())
    layout = ParamLayout.of_module(module)
    arena = ParamArena(layout, dtype or params[0].dtype, device or params[0].device)
    return bind_module_(module, arena, copy=True)


def flat_view(tensors) -> torch.Tensor | None:
    """If `tensors` are consecutive, contiguous views of one buffer (e.g. an arena), return the
    flat view spanning them; otherwise None."""
    tensors = list(tensors)
    if not tensors:
        return None
    t0 = tensors[0]
    dt, dev = t0.dtype, t0.device
    es = t0.element_size()
    storage = t0.untyped_storage().data_ptr()
    expect = t0.data_ptr()
    total = 0
    for t in tensors:
        if t.dtype != dt or t.device != dev or not t.is_contiguous():
            return None
        if t.untyped_storage().data_ptr() != storage or t.data_ptr() != expect:
            return None
        expect += t.numel() * es
        total += t.numel()
    start = (t0.data_ptr() - storage) // es
    base = torch.empty(0, dtype=dt, device=dev).set_(t0.untyped_storage(), start, (total,), (1,))
    return base


def pack(tensors, dtype=None, device=None) -> torch.Tensor:
    """Flat copy of a tensor list (used when the caller's tensors are not arena views)."""
    tensors = list(tensors)
    dtype = dtype or tensors[0].dtype
    device = device or tensors[0].device
    out = torch.empty(sum(t.numel() for t in tensors), dtype=dtype, device=device)
    off = 0
    for t in tensors:
        n = t.numel()
        out[off:off + n].copy_(t.reshape(-1))
        off += n
    return out


def unpack_(flat: torch.Tensor, tensors) -> None:
    """Copy a flat buffer back into a tensor list (in place)."""
    off = 0
    with torch.no_grad():
        for t in tensors:
            n = t.numel()
            t.copy_(flat[off:off + n].view(t.shape))
            off += n
