"""Scheme-driven episode storage (API of src/marl/components/episode_batch.py:57-248).

Dense tensors [batch, time, (group,) *vshape] per scheme key on one device (HBM for the GPU path),
a reserved ``filled`` mask, preprocess transforms (``actions`` -> ``actions_onehot``), slicing that
returns views, and ``max_t_filled``. The HIP rollout kernel writes straight into these tensors; their
dtypes and layout are the reference's so learners and checkpoints interoperate.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch

_INDEX_TYPES = (list, np.ndarray, torch.Tensor)


def _as_slices(item):
    """Normalise an index into [batch_index, time_index] (ints become length-1 slices)."""
    if isinstance(item, (slice, int)) or isinstance(item, _INDEX_TYPES):
        item = (item, slice(None))
    if isinstance(item[1], list):
        raise IndexError("Indexing across Time must be contiguous")
    out = []
    for it in item:
        out.append(slice(it, it + 1) if isinstance(it, int) else it)
    return out


def _count(index, size):
    if isinstance(index, slice):
        start, stop, step = index.indices(size)
        return max(0, 1 + (stop - start - 1) // step)
    return len(index)


def _safe_view_check(value: torch.Tensor, dest: torch.Tensor, key):
    """The reference refuses reshapes that are not plain (unit-dimension) views of the destination."""
    i = value.dim() - 1
    for s in reversed(dest.shape):
        if value.shape[i] != s:
            if s != 1:
                raise ValueError(f"Unsafe reshape of {tuple(value.shape)} to {tuple(dest.shape)} at Key: {key}")
        else:
            i -= 1


class EpisodeBatch:
    def __init__(self, scheme, groups, batch_size, max_seq_length, data=None, preprocess=None, device="cpu"):
        self.scheme = dict(scheme)
        self.groups = groups
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.preprocess = preprocess or {}
        self.device = device
        if data is not None:
            self.data = data
        else:
            self.data = SimpleNamespace(transition_data={}, episode_data={})
            self._setup_data(self.scheme, self.groups, batch_size, max_seq_length, self.preprocess)

    # -------------------------------------------------------------------------------------------
    def _setup_data(self, scheme, groups, batch_size, max_seq_length, preprocess):
        for src_key, (dst_key, transforms) in (preprocess or {}).items():
            assert src_key in scheme
            vshape, dtype = self.scheme[src_key]["vshape"], self.scheme[src_key]["dtype"]
            for tr in transforms:
                vshape, dtype = tr.infer_output_info(vshape, dtype)
            entry = {"vshape": vshape, "dtype": dtype}
            for carried in ("group", "episode_const"):
                if carried in self.scheme[src_key]:
                    entry[carried] = self.scheme[src_key][carried]
            self.scheme[dst_key] = entry
        assert "filled" not in scheme, '"filled" is a reserved key for masking.'
        scheme["filled"] = {"vshape": (1,), "dtype": torch.long}
        for key, info in scheme.items():
            assert "vshape" in info, f"Scheme must define vshape for {key}"
            vshape = info["vshape"]
            vshape = (vshape,) if isinstance(vshape, int) else tuple(vshape)
            group = info.get("group")
            if group:
                assert group in groups, f"Group {group} must have its number of members defined in _groups_"
                vshape = (groups[group],) + vshape
            dtype = info.get("dtype", torch.float32)
            if info.get("episode_const", False):
                self.data.episode_data[key] = torch.zeros((batch_size,) + vshape, dtype=dtype, device=self.device)
            else:
                self.data.transition_data[key] = torch.zeros((batch_size, max_seq_length) + vshape, dtype=dtype,
                                                             device=self.device)

    def extend(self, scheme, groups=None):
        self._setup_data(scheme, self.groups if groups is None else groups, self.batch_size, self.max_seq_length,
                         None)

    def to(self, device):
        for store in (self.data.transition_data, self.data.episode_data):
            for k in store:
                store[k] = store[k].to(device)
        self.device = device

    # -------------------------------------------------------------------------------------------
    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True):
        b_idx, t_idx = _as_slices((bs, ts))
        for key, value in data.items():
            if key in self.data.transition_data:
                store, index = self.data.transition_data, (b_idx, t_idx)
                if mark_filled:
                    store["filled"][index] = 1
                    mark_filled = False
            elif key in self.data.episode_data:
                store, index = self.data.episode_data, b_idx
            else:
                raise KeyError(f"{key} not found in transition or episode data")
            dtype = self.scheme[key].get("dtype", torch.float32)
            if isinstance(value, list):
                value = torch.tensor(value, dtype=dtype, device=self.device)
            else:
                value = value.to(dtype=dtype, device=self.device)
            dest = store[key][index]
            _safe_view_check(value, dest, key)
            store[key][index] = value.view_as(dest)
            if key in self.preprocess:
                dst_key, transforms = self.preprocess[key]
                out = store[key][index]
                for tr in transforms:
                    out = tr.transform(out)
                dest = store[dst_key][index]
                _safe_view_check(out, dest, key)
                store[dst_key][index] = out.view_as(dest)

    def __getitem__(self, item):
        if isinstance(item, str):
            if item in self.data.episode_data:
                return self.data.episode_data[item]
            if item in self.data.transition_data:
                return self.data.transition_data[item]
            raise ValueError(item)
        if isinstance(item, tuple) and all(isinstance(k, str) for k in item):
            sub = SimpleNamespace(transition_data={}, episode_data={})
            for k in item:
                if k in self.data.transition_data:
                    sub.transition_data[k] = self.data.transition_data[k]
                elif k in self.data.episode_data:
                    sub.episode_data[k] = self.data.episode_data[k]
                else:
                    raise KeyError(f"Unrecognised key {k}")
            sub_scheme = {k: self.scheme[k] for k in item}
            sub_groups = {self.scheme[k]["group"]: self.groups[self.scheme[k]["group"]]
                          for k in item if "group" in self.scheme[k]}
            return EpisodeBatch(sub_scheme, sub_groups, self.batch_size, self.max_seq_length, data=sub,
                                device=self.device)
        b_idx, t_idx = _as_slices(item)
        if isinstance(t_idx, torch.Tensor) and t_idx.dim() == 0:
            t_idx = int(t_idx)
        sub = SimpleNamespace(transition_data={k: v[b_idx, t_idx] for k, v in self.data.transition_data.items()},
                              episode_data={k: v[b_idx] for k, v in self.data.episode_data.items()})
        return EpisodeBatch(self.scheme, self.groups, _count(b_idx, self.batch_size),
                            _count(t_idx, self.max_seq_length), data=sub, device=self.device)

    def max_t_filled(self):
        return torch.sum(self.data.transition_data["filled"], 1).max(0)[0]

    def __repr__(self):
        return (f"EpisodeBatch. Batch Size:{self.batch_size} Max_seq_len:{self.max_seq_length} "
                f"Keys:{self.scheme.keys()} Groups:{self.groups.keys()}")
