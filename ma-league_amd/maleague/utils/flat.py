"""Flat views of parameter lists (one fp32 buffer holding every parameter back to back, as FlatParams builds)."""
from __future__ import annotations

import torch


def flat_view(params) -> torch.Tensor | None:
    """The 1-D fp32 tensor spanning ``params`` when they are contiguous fp32 views laid out back to back in one
    storage (a learner's FlatParams), else None. Reads and writes through it touch the parameters themselves."""
    params = list(params)
    if not params or not all(p.dtype == torch.float32 and p.is_contiguous() for p in params):
        return None
    p0 = params[0]
    base = p0.untyped_storage().data_ptr()
    off = p0.data_ptr()
    for p in params:
        if p.data_ptr() != off or p.untyped_storage().data_ptr() != base:
            return None
        off += 4 * p.numel()
    n = sum(p.numel() for p in params)
    return p0.detach().new_empty(0).set_(p0.untyped_storage(), p0.storage_offset(), (n,), (1,))


def module_flat_view(module) -> torch.Tensor | None:
    """flat_view of ``module.parameters()``, cached on the module by the parameters' addresses (the cached view
    keeps its storage alive, so equal addresses mean the same layout in the same buffer)."""
    params = list(module.parameters())
    key = tuple(p.data_ptr() for p in params)
    hit = getattr(module, "_mlg_flat_view", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    flat = flat_view(params)
    object.__setattr__(module, "_mlg_flat_view", (key, flat))
    return flat
