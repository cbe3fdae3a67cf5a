"""EpisodeBatch -> MlgBatch (device pointers + sizes) for the C ABI."""
from __future__ import annotations

import torch

from .. import _native

KEYS = ("state", "obs", "actions", "avail_actions", "reward", "terminated", "actions_onehot", "filled")
DTYPES = {"state": torch.float32, "obs": torch.float32, "actions": torch.int64, "avail_actions": torch.int32,
          "reward": torch.float32, "terminated": torch.uint8, "actions_onehot": torch.float32, "filled": torch.int64}


def _time_stride_ok(t: torch.Tensor, T1: int) -> bool:
    """[B, T, *inner] view whose memory is [B][T1][*inner] with T <= T1 (a time slice starting at 0 is)."""
    inner = 1
    for s in t.shape[2:]:
        inner *= s
    want = [T1 * inner, inner]
    exp = []
    acc = 1
    for d in range(t.dim() - 1, 1, -1):
        exp.insert(0, acc)
        acc *= t.shape[d]
    return list(t.stride()[:2]) == want and all(
        t.shape[d] == 1 or t.stride(d) == exp[d - 2] for d in range(2, t.dim()))


def _sampled_view(batch) -> bool:
    """A SampledEpisodeBatch not yet materialised: kernels read the buffer through its slot map."""
    return getattr(batch, "host_rows", None) is not None and getattr(batch, "_data", None) is None


def mlg_batch(batch, required=KEYS, device_rows=True):
    """Build an MlgBatch for `batch` (EpisodeBatch), making tensors contiguous when the layout is not
    a plain [B][T1][...] array. Returns (MlgBatch, keepalive-list). With device_rows=False a sampled view's
    slot map is left out (MlgBatch.rows = NULL): the caller hands its host copy to the kernel instead."""
    rows = None
    if _sampled_view(batch):
        # sampled view of a replay buffer: point at the buffer itself, episodes through the slot map
        rows = batch.rows if device_rows else None
        data = batch.ring.data.transition_data
    else:
        data = batch.data.transition_data
    B = batch.batch_size
    ref = data["obs"]
    T1 = ref.stride(0) // max(1, ref.stride(1)) if ref.dim() > 1 and ref.stride(1) > 0 else ref.shape[1]
    tensors = {}
    for k in KEYS:
        if k not in data:
            if k in required:
                raise KeyError(f"EpisodeBatch lacks {k!r} needed by the kernel")
            tensors[k] = None
            continue
        t = data[k]
        if t.dtype != DTYPES[k]:
            raise TypeError(f"EpisodeBatch[{k!r}] has dtype {t.dtype}, kernel expects {DTYPES[k]}")
        if not t.is_cuda:
            raise _native.NativeError(f"EpisodeBatch[{k!r}] is on {t.device}; kernels need device tensors")
        tensors[k] = t
    if not all(t is None or _time_stride_ok(t, T1) for t in tensors.values()):
        tensors = {k: (None if t is None else t.contiguous()) for k, t in tensors.items()}
        T1 = batch.max_seq_length
    p = lambda k: None if tensors[k] is None else tensors[k].data_ptr()  # noqa: E731
    mb = _native.MlgBatch(p("state"), p("obs"), p("actions"), p("avail_actions"), p("reward"), p("terminated"),
                          p("actions_onehot"), p("filled"), B, T1, 0, 0, 0, None if rows is None else rows.data_ptr())
    return mb, list(tensors.values()) + [rows]


ENTITY_KEYS = ("entities", "obs_mask", "entity_mask", "actions", "avail_actions", "reward", "terminated",
               "actions_onehot", "filled")
ENTITY_DTYPES = {"entities": torch.float32, "obs_mask": torch.uint8, "entity_mask": torch.uint8,
                 "actions": torch.int64, "avail_actions": torch.int32, "reward": torch.float32,
                 "terminated": torch.uint8, "actions_onehot": torch.float32, "filled": torch.int64}


def mlg_entity_batch(batch, device_rows=True):
    """Entity-scheme EpisodeBatch (REFIL, config 5) -> MlgEntityBatch. Returns (MlgEntityBatch, keepalive).
    device_rows=False: a sampled view's slot map is left out (rows = NULL), as in mlg_batch."""
    rows = None
    if _sampled_view(batch):
        rows = batch.rows if device_rows else None
        data = batch.ring.data.transition_data
    else:
        data = batch.data.transition_data
    B = batch.batch_size
    ref = data["entities"]
    T1 = ref.stride(0) // max(1, ref.stride(1)) if ref.dim() > 1 and ref.stride(1) > 0 else ref.shape[1]
    tensors = {}
    for k in ENTITY_KEYS:
        if k not in data:
            raise KeyError(f"entity EpisodeBatch lacks {k!r} needed by the kernel")
        t = data[k]
        if t.dtype != ENTITY_DTYPES[k]:
            raise TypeError(f"EpisodeBatch[{k!r}] has dtype {t.dtype}, kernel expects {ENTITY_DTYPES[k]}")
        if not t.is_cuda:
            raise _native.NativeError(f"EpisodeBatch[{k!r}] is on {t.device}; kernels need device tensors")
        tensors[k] = t
    if not all(_time_stride_ok(t, T1) for t in tensors.values()):
        tensors = {k: t.contiguous() for k, t in tensors.items()}
        T1 = batch.max_seq_length
    p = lambda k: tensors[k].data_ptr()  # noqa: E731
    mb = _native.MlgEntityBatch(p("entities"), p("obs_mask"), p("entity_mask"), p("actions"), p("avail_actions"),
                                p("reward"), p("terminated"), p("actions_onehot"), p("filled"), B, T1, 0, 0, 0,
                                None if rows is None else rows.data_ptr())
    return mb, list(tensors.values()) + [rows]
