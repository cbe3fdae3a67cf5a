"""One-learner-per-GPU league exchange over torch.distributed (RCCL on ROCm; gloo for CPU tests).

Replaces the reference's process topology (src/league/processes/*: AgentPool queues, a shared-memory payoff
tensor incremented racily from every process, Barrier.wait -- SURVEY §2.1 table) with three collectives per
league iteration:
  * all_gather of each rank's flat agent parameters + [trained_steps, checkpoint flag]
    (AgentParamsUpdate/AgentPoolGet/AgentCheckpointAdd, agent_pool_instance.py:84-128)
  * all_reduce(SUM) of each rank's local payoff delta (payoff_entry.py:50-51, central_worker.py:63)
  * barrier                                           (league_experiment_process.py:83)
They run once per league iteration (play_time_mins), never on the per-step data path. The payoff table and
the agent pool (current parameters of every player + historical snapshots) are replicated on every rank, so
matchmaking is local and needs no coordinator process.

The collectives run whenever a process group exists, world size 1 included (``torchrun --nproc-per-node 1``
exercises the RCCL branch on one GPU); without one (plain ``python``) the pool degenerates to local copies.
The historical pool has a fixed capacity (its slots are payoff rows / columns); when it is full the oldest
snapshot of the parent holding the most snapshots is evicted -- its slot, payoff row and column reused by the
new snapshot -- identically on every rank (the reference appends HistoricalPlayers without bound,
players.py:32-60, agent_pool_instance.py:94-103).
"""
from __future__ import annotations

import logging
from typing import List

import numpy as np
import torch
import torch.distributed as dist

from .payoff import PayoffEntry, PayoffWrapper, PFSPSampling

log = logging.getLogger(__name__)


class DistributedLeague:
    def __init__(self, n_players: int, device, reference_compat: bool = False, seed: int = 0,
                 max_historical: int = 0, player_id: int = None):
        """``player_id`` (no process group only): this process plays that pid of an ``n_players`` league whose other
        players' parameters are fixed replicas installed with set_player_params (e.g. a main exploiter trained on one
        GPU against a main player loaded from its checkpoint)."""
        self._dist = dist.is_available() and dist.is_initialized()
        if player_id is not None and (self._dist or not 0 <= player_id < n_players):
            raise ValueError(f"player_id={player_id}: only without a process group, and < n_players={n_players}")
        self._pid = player_id
        self.rank = dist.get_rank() if self._dist else 0
        self.world = dist.get_world_size() if self._dist else 1
        self.n = n_players
        self.capacity = n_players + max_historical  # payoff rows/cols: players, then historical snapshots
        self.device = torch.device(device)
        self.payoff = PayoffWrapper(torch.zeros(self.capacity, self.capacity, 5, device=self.device), reference_compat)
        self._delta = torch.zeros_like(self.payoff.tensor)
        self.sampling = PFSPSampling(np.random.RandomState(seed + self.rank))
        # agent pool (replicated): current parameters of every player, historical snapshots
        self.current = None            # [n_players, n_params]
        self.historical = None         # [max_historical, n_params]
        self.historical_meta: List[tuple] = []  # (pid, parent pid, trained_steps), oldest first
        self.evictions = 0  # snapshots evicted to make room for newer ones (pool full)
        self.payoff_host = None  # host copy of the payoff taken by host_snapshot() (what matchmaking reads)
        self._installed = set()  # players whose parameters set_player_params installed (no process group)

    def player(self) -> int:
        return self.rank % self.n if self._pid is None else self._pid

    def set_player_params(self, pid: int, flat: torch.Tensor):
        """Install player ``pid``'s current parameters (a fixed replica; league without a process group)."""
        if self._dist:
            raise RuntimeError("set_player_params: the process group's all_gather owns the pool")
        flat = flat.detach().reshape(-1).to(torch.float32)
        self._alloc_pool(flat.numel(), flat.device)
        self.current[pid].copy_(flat)
        self._installed.add(pid)

    def _alloc_pool(self, n_p: int, device):
        if self.current is None:
            self.current = torch.zeros(self.n, n_p, dtype=torch.float32, device=device)
            self.historical = torch.empty(max(self.capacity - self.n, 0), n_p, dtype=torch.float32, device=device)

    # ---- payoff ------------------------------------------------------------------------------------------
    def record(self, home: int, away: int, result: PayoffEntry, n: int = 1):
        """Local, race-free accumulation; published by sync_payoff()."""
        d = PayoffWrapper(self._delta, self.payoff.reference_compat)
        d.record_result(home, away, result, n)

    def record_match(self, home: int, away: int):
        self._delta[home, away, PayoffEntry.MATCHES].add_(1)  # one in-place kernel on a view

    def record_runs(self, home: int, away: int, won: torch.Tensor, draw: torch.Tensor):
        """Episode results of one batched run, on the device (no host sync): _extract_result +
        _update_payoff (league_experiment_process.py:85-105) for every env. won [B, 2] (policy team first),
        draw [B]; DRAW if the env says so or if both / no team won, else WIN / LOSS by won[:, 0]. Device tensors: one
        mlg_league_record_runs launch; host tensors (CPU rehearsals / tests): the same reduction in torch."""
        if self._delta.is_cuda:
            from .. import _native
            B = int(won.shape[0])
            # the kernel reads int32 rows: [B, 2] won (policy team first) and [B] draw, from device memory or from a
            # pinned (device-accessible) summary slot written by the rollout (zero-copy, ParallelStepper)
            reach = lambda x: x.is_cuda or (x.device.type == "cpu" and x.is_pinned())  # noqa: E731
            if won.dtype != torch.int32 or draw.dtype != torch.int32 or tuple(won.shape) != (B, 2) or \
                    tuple(draw.shape) != (B,) or not reach(won) or not reach(draw):
                raise ValueError(f"record_runs: won must be int32 [B, 2] and draw int32 [B] on the device or pinned, "
                                 f"got {won.dtype} {tuple(won.shape)} / {draw.dtype} {tuple(draw.shape)}")
            entry = self._delta[home, away]
            dptr = lambda x: _native.ptr(x) if x.is_cuda else x.data_ptr()  # noqa: E731  (pinned: device-accessible)
            _native.call("mlg_league_record_runs", dptr(won.contiguous()), dptr(draw.contiguous()),
                         int(won.shape[0]), entry.data_ptr(), int(not self.payoff.reference_compat),
                         _native.stream_ptr(self.device))
            return
        w0, w1 = won[:, 0] != 0, won[:, 1] != 0
        d = (draw != 0) | (w0 == w1)
        win = ~d & w0
        counts = torch.stack([win.sum(), (~d & ~w0).sum(), d.sum()]).to(self._delta.dtype)
        self._delta[home, away, PayoffEntry.WIN:PayoffEntry.DRAW + 1] += counts
        if not self.payoff.reference_compat:
            self._delta[home, away, PayoffEntry.GAMES] += won.shape[0]

    def _host_staged(self) -> bool:
        """gloo (CPU tests, single-GPU rehearsals) reduces host tensors; RCCL reduces device tensors in place."""
        return self.device.type == "cuda" and dist.get_backend() == "gloo"

    @property
    def backend(self) -> str:
        return dist.get_backend() if self._dist else "local"

    def sync_payoff(self):
        if self._dist:
            if self._host_staged():
                d = self._delta.cpu()
                dist.all_reduce(d, op=dist.ReduceOp.SUM)
                self._delta.copy_(d)
            else:
                dist.all_reduce(self._delta, op=dist.ReduceOp.SUM)
        self.payoff.tensor.add_(self._delta)
        self._delta.zero_()
        self.payoff_host = None  # stale now: host_snapshot() is the only thing that installs a host copy
        return self.payoff.tensor

    def host_snapshot(self, counter: torch.Tensor = None):
        """ONE device -> host read per league iteration: the (reduced) payoff table, plus ``counter`` (a player's
        device-side trained-steps count) in the same copy. Matchmaking and the checkpoint decisions then read win
        rates from ``payoff_host`` with no further device round trips. Returns the counter's value (or None)."""
        flat = self.payoff.tensor.reshape(-1).to(torch.float64)
        if counter is not None:
            flat = torch.cat([flat, counter.reshape(1).to(device=flat.device, dtype=torch.float64)])
        host = flat.cpu()
        n = self.payoff.tensor.numel()
        self.payoff_host = PayoffWrapper(host[:n].to(torch.float32).reshape(self.payoff.tensor.shape),
                                         self.payoff.reference_compat)
        return float(host[n]) if counter is not None else None

    # ---- agent pool --------------------------------------------------------------------------------------
    def share_params(self, flat: torch.Tensor):
        """Every rank's flat parameter vector (index = rank)."""
        flat = flat.detach().contiguous()
        if not self._dist:
            return [flat.clone()]
        if self._host_staged():
            host = flat.cpu()
            out = [torch.empty_like(host) for _ in range(self.world)]
            dist.all_gather(out, host)
            return [o.to(flat.device) for o in out]
        out = [torch.empty_like(flat) for _ in range(self.world)]
        dist.all_gather(out, flat)
        return out

    def exchange(self, flat: torch.Tensor, trained_steps: int, checkpoint: bool):
        """all_gather [params | trained_steps | checkpoint flag | range flag] of every player; refresh the
        replicated pool and append a historical snapshot for every player that asked for a checkpoint (in player
        order, so every rank assigns the same historical pids). trained_steps travels as two float32 halves (steps
        mod 2^24 and steps >> 24), exact up to 2^48 (the reference's checkpoint thresholds are 2e9 / 4e9 steps); a
        value outside that range is flagged in the message and every rank raises after the gather (a rank raising
        before it would leave the others blocked in the collective). When the pool is full the oldest snapshot of
        the parent with the most snapshots is evicted (``_evict``). Returns the list of new (historical pid,
        parent pid)."""
        n_p = flat.numel()
        steps = int(trained_steps)
        bad = not 0 <= steps < 2 ** 48
        s = min(max(steps, 0), 2 ** 48 - 1)
        meta_in = [float(s & 0xFFFFFF), float(s >> 24), 1.0 if checkpoint else 0.0, 1.0 if bad else 0.0]
        if self._dist:
            msg = torch.cat([flat.detach().reshape(-1).to(torch.float32), torch.tensor(meta_in, device=flat.device)])
            gathered = self.share_params(msg)
            allm = torch.stack(gathered)[: self.n]
            params = allm[:, :n_p]
            meta = allm[:, n_p:].detach().cpu().numpy().astype(np.int64)
        else:  # nothing to gather: the message stays on the host, the parameters on the device; the other players
            # (player_id leagues) keep their installed replicas and never ask for checkpoints
            missing = [p for p in range(self.n) if p != self.player() and p not in self._installed]
            if missing:  # their pool rows would silently be zeros
                raise ValueError(f"league exchange without a process group: players {missing} have no parameters "
                                 "(DistributedLeague(player_id=...) + set_player_params for every other player)")
            meta = np.zeros((self.n, 4), dtype=np.int64)
            meta[self.player()] = np.asarray(meta_in, dtype=np.float32).astype(np.int64)
            params = None
        if meta[:, 3].any():
            raise ValueError(f"trained_steps outside the exchange's exact range [0, 2^48) on player(s) "
                             f"{np.nonzero(meta[:, 3])[0].tolist()} (this player: {steps})")
        self._alloc_pool(n_p, flat.device)
        if params is not None:
            self.current.copy_(params)
        else:
            self.current[self.player()].copy_(flat.detach().reshape(-1))
        new = []
        for pid in range(self.n):
            if meta[pid, 2] > 0:
                if self.historical.shape[0] == 0:
                    continue  # no historical capacity at all (max_historical = 0)
                if len(self.historical_meta) < self.historical.shape[0]:
                    hp = self.n + len(self.historical_meta)
                else:
                    hp = self._evict()
                self.historical[hp - self.n].copy_(self.current[pid])
                self.historical_meta.append((hp, pid, int(meta[pid, 0] + (meta[pid, 1] << 24))))
                new.append((hp, pid))
        return new

    def _evict(self) -> int:
        """Free a historical slot: the oldest snapshot of the parent that holds the most snapshots (ties: the
        parent whose oldest snapshot is older). Its payoff row and column are zeroed so the new snapshot starts
        with no games. Deterministic in the replicated state, hence identical on every rank."""
        counts = {}
        for _, parent, _ in self.historical_meta:
            counts[parent] = counts.get(parent, 0) + 1
        most = max(counts.values())
        idx = next(i for i, (_, parent, _) in enumerate(self.historical_meta) if counts[parent] == most)
        hp = self.historical_meta.pop(idx)[0]
        for t in (self.payoff.tensor, self._delta) + ((self.payoff_host.tensor,) if self.payoff_host else ()):
            t[hp, :, :] = 0
            t[:, hp, :] = 0
        self.evictions += 1
        log.info("league: historical pool full (%d snapshots): evicted snapshot %d", len(self.historical_meta) + 1, hp)
        return hp

    def params_of(self, pid: int) -> torch.Tensor:
        if pid < self.n:
            return self.current[pid]
        return self.historical[pid - self.n]

    def pfsp_opponent(self, weighting: str = "squared", exclude_self: bool = False) -> int:
        """PFSPMatchmaking.get_match / SimplePlayer.get_match (matchmaker.py:64-72, simple_player.py:24-37)."""
        me = self.player()
        opponents = [i for i in range(self.n) if not (exclude_self and i == me)]
        wr = self.payoff.win_rates(me, opponents).cpu().numpy()
        return self.sampling.sample(opponents, prio_measure=wr, weighting=weighting)

    def barrier(self):
        if self._dist:
            dist.barrier()
