"""Circular episode replay buffer (API of src/marl/components/replay_buffers/replay_buffer.py:6-59).

Lives on the training device (HBM) so sampling and training never cross PCIe.
"""
from __future__ import annotations

import weakref
from types import SimpleNamespace

import numpy as np
import torch

from .episode_batch import EpisodeBatch


class ReplayBuffer(EpisodeBatch):
    def __init__(self, scheme, groups, buffer_size: int, max_seq_length: int, preprocess=None, device="cpu"):
        super().__init__(scheme, groups, buffer_size, max_seq_length, preprocess=preprocess, device=device)
        self.buffer_size = buffer_size
        self.buffer_index = 0
        self.episodes_in_buffer = 0
        self._outstanding = []  # weakrefs to RingEpisodeBatches written into the ring but not inserted yet
        # per slot: exclusive end of the rows that may hold non-zero data (max_seq_length = unknown). Rollouts in
        # full-write ring mode zero only [L + 1, extent) of a slot they rewrite and record L + 1 (MlgBatch.slot_extent);
        # every other write into the buffer (insert by copy) marks its slots unknown again.
        self.slot_extent = (torch.full((buffer_size,), max_seq_length, dtype=torch.int32, device=device)
                            if torch.device(device).type == "cuda" else None)

    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True):
        super().update(data, bs, ts, mark_filled)
        self.invalidate_extents(bs)

    def extent_ptr(self):
        """Device pointer of the slot extents (None without them)."""
        ext = getattr(self, "slot_extent", None)
        return None if ext is None else ext.data_ptr()

    def invalidate_extents(self, slots=None):
        """Slots written by anything but a full-write rollout: their rows past any episode end are unknown."""
        if getattr(self, "slot_extent", None) is not None:
            if slots is None:
                self.slot_extent.fill_(self.max_seq_length)
            else:
                self.slot_extent[slots] = self.max_seq_length

    def has_outstanding(self) -> bool:
        """True while a rollout's episodes sit in the ring's next slots uncommitted (written in place, not yet
        passed to insert_episode_batch). A stepper must not write another run there: that would overwrite them,
        while the reference leaves the buffer untouched until insert."""
        self._outstanding = [r for r in getattr(self, "_outstanding", []) if r() is not None and r().attached]
        return bool(self._outstanding)

    def _register(self, ring_batch: "RingEpisodeBatch"):
        if not hasattr(self, "_outstanding"):
            self._outstanding = []
        self._outstanding.append(weakref.ref(ring_batch))

    def _detach_outstanding(self):
        """Give every uncommitted ring batch its own copy before a plain insert overwrites its slots."""
        for r in getattr(self, "_outstanding", []):
            rb = r()
            if rb is not None and rb.attached:
                rb.detach()
        self._outstanding = []

    def insert_episode_batch(self, ep_batch: EpisodeBatch):
        if isinstance(ep_batch, RingEpisodeBatch) and ep_batch.attached and ep_batch.ring is self:
            if ep_batch.slot0 != self.buffer_index:
                raise RuntimeError("ring episodes must be inserted in the order they were written")
            self._advance(ep_batch.batch_size)
            ep_batch.committed = True
            return
        self._detach_outstanding()
        room = self.buffer_size - self.buffer_index
        if ep_batch.batch_size > room:
            # split at the wrap point and insert both halves (replay_buffer.py:37-41)
            self.insert_episode_batch(ep_batch[0:room, :])
            self.insert_episode_batch(ep_batch[room:, :])
            return
        dst = slice(self.buffer_index, self.buffer_index + ep_batch.batch_size)
        self._copy_in(ep_batch, dst)
        self.invalidate_extents(dst)
        self.buffer_index += ep_batch.batch_size
        self.episodes_in_buffer = max(self.episodes_in_buffer, self.buffer_index)
        self.buffer_index %= self.buffer_size
        assert self.buffer_index < self.buffer_size

    def _advance(self, n: int):
        """Index bookkeeping of inserting n episodes at buffer_index (same as the split insert)."""
        room = self.buffer_size - self.buffer_index
        if n > room:
            self._advance(room)
            self._advance(n - room)
            return
        self.buffer_index += n
        self.episodes_in_buffer = max(self.episodes_in_buffer, self.buffer_index)
        self.buffer_index %= self.buffer_size

    def _copy_in(self, ep_batch: EpisodeBatch, dst: slice):
        """Same result as update(..., mark_filled=False) of every key: the preprocessed keys that the
        source already carries are copied rather than recomputed (their recomputed value is overwritten
        by the copy in the reference as well)."""
        t = slice(0, ep_batch.max_seq_length)
        src = ep_batch.data.transition_data
        derived = {v[0] for v in self.preprocess.values()}
        for key, value in src.items():
            if key not in self.data.transition_data:
                raise KeyError(f"{key} not found in transition or episode data")
            if key in self.preprocess and self.preprocess[key][0] in src:
                self.data.transition_data[key][dst, t] = value.to(self.data.transition_data[key].dtype)
                continue
            if key in derived or key not in self.preprocess:
                self.data.transition_data[key][dst, t] = value.to(self.data.transition_data[key].dtype)
            else:
                self.update({key: value}, dst, t, mark_filled=False)
        if ep_batch.data.episode_data:
            self.update(ep_batch.data.episode_data, dst)

    def can_sample(self, batch_size: int) -> bool:
        return self.episodes_in_buffer >= batch_size

    def sample(self, batch_size: int, view: bool = False) -> EpisodeBatch:
        """replay_buffer.py:50-57. view=True (device buffers): return a SampledEpisodeBatch that the kernels
        read in place through a slot map instead of a gathered copy -- valid until those slots are rewritten."""
        assert self.can_sample(batch_size)
        if self.episodes_in_buffer == batch_size:
            ep_ids = np.arange(batch_size)
            if not view:
                return self[:batch_size]
        else:
            ep_ids = np.random.choice(self.episodes_in_buffer, batch_size, replace=False)
        if view and torch.device(self.device).type == "cuda":
            return SampledEpisodeBatch(self, ep_ids)
        return self[ep_ids]

    def __repr__(self):
        return (f"ReplayBuffer. {self.episodes_in_buffer}/{self.buffer_size} episodes. "
                f"Keys:{self.scheme.keys()} Groups:{self.groups.keys()}")


class RingEpisodeBatch(EpisodeBatch):
    """The B episodes one rollout wrote straight into replay-buffer slots [slot0, slot0 + B) mod size
    (zero-copy insert). Reads materialise views (or a gathered copy when the range wraps); the content
    is valid until the ring slots are written again."""

    def __init__(self, ring: ReplayBuffer, slot0: int, batch_size: int):
        self.ring, self.slot0, self.committed = ring, slot0, False
        self.scheme, self.groups, self.preprocess = ring.scheme, ring.groups, ring.preprocess
        self.batch_size, self.max_seq_length, self.device = batch_size, ring.max_seq_length, ring.device
        self._data = None
        ring._register(self)

    @property
    def attached(self) -> bool:
        """Still backed by (uncommitted) ring slots: insert_episode_batch only advances the ring's indices."""
        return self.ring is not None and not self.committed

    def detach(self):
        """Materialise the episodes into their own tensors (the ring slots are about to be reused); the batch
        then behaves like a plain EpisodeBatch (insert copies it)."""
        d = self.data
        self._data = SimpleNamespace(transition_data={k: v.clone() for k, v in d.transition_data.items()},
                                     episode_data={k: v.clone() for k, v in d.episode_data.items()})
        self.ring = None

    @property
    def data(self):
        if self._data is None:
            size, B = self.ring.buffer_size, self.batch_size
            if self.slot0 + B <= size:
                sel = lambda v: v[self.slot0:self.slot0 + B]  # noqa: E731
            else:
                idx = (torch.arange(B, device=self.device) + self.slot0) % size
                sel = lambda v: v.index_select(0, idx)  # noqa: E731
            self._data = SimpleNamespace(
                transition_data={k: sel(v) for k, v in self.ring.data.transition_data.items()},
                episode_data={k: sel(v) for k, v in self.ring.data.episode_data.items()})
        return self._data

    @data.setter
    def data(self, value):
        self._data = value


class SampledEpisodeBatch(EpisodeBatch):
    """`batch_size` episodes of a device ReplayBuffer, addressed through a slot map (MlgBatch.rows): the
    learner kernels read the buffer in place, nothing is gathered. Host reads materialise a gathered copy.
    The episodes keep the buffer's full length (max_seq_length); the filled mask makes the steps past each
    episode inert in QLearner.train, exactly like the reference's [:, :max_t_filled] truncation."""

    def __init__(self, ring: ReplayBuffer, ep_ids):
        self.ring = ring
        self.scheme, self.groups, self.preprocess = ring.scheme, ring.groups, ring.preprocess
        self.batch_size, self.max_seq_length, self.device = len(ep_ids), ring.max_seq_length, ring.device
        self.ep_ids = np.asarray(ep_ids, dtype=np.int64)
        self.host_rows = np.ascontiguousarray(self.ep_ids, dtype=np.int32)  # kernel-argument slot map
        self._rows = None
        self._data = None

    @property
    def rows(self) -> torch.Tensor:
        """The slot map on the device (int32 [B]); copied on first use only."""
        if self._rows is None:
            host = torch.from_numpy(self.host_rows)
            if torch.device(self.device).type == "cuda":
                host = host.pin_memory()
            self._rows = host.to(self.device, non_blocking=True)
        return self._rows

    @property
    def data(self):
        if self._data is None:
            idx = self.rows.long()
            self._data = SimpleNamespace(
                transition_data={k: v.index_select(0, idx) for k, v in self.ring.data.transition_data.items()},
                episode_data={k: v.index_select(0, idx) for k, v in self.ring.data.episode_data.items()})
        return self._data

    @data.setter
    def data(self, value):
        self._data = value
