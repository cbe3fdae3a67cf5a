"""One-learner-per-GPU league exchange over torch.distributed (RCCL on ROCm; gloo for CPU tests).

Replaces the reference's process topology (src/league/processes/*: AgentPool queues, a shared-memory payoff
tensor incremented racily from every process, Barrier.wait -- SURVEY §2.1 table) with three collectives per
league iteration:
  * all_gather of each rank's flat agent parameters  (AgentParamsUpdate/AgentPoolGet, agent_pool_instance.py:115-128)
  * all_reduce(SUM) of each rank's local payoff delta (payoff_entry.py:50-51, central_worker.py:63)
  * barrier                                           (league_experiment_process.py:83)
They run once per league iteration (play_time_mins), never on the per-step data path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .payoff import PayoffEntry, PayoffWrapper, PFSPSampling


class DistributedLeague:
    def __init__(self, n_players: int, device, reference_compat: bool = False, seed: int = 0):
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.n = n_players
        self.device = torch.device(device)
        self.payoff = PayoffWrapper(torch.zeros(n_players, n_players, 5, device=self.device), reference_compat)
        self._delta = torch.zeros_like(self.payoff.tensor)
        import numpy as np
        self.sampling = PFSPSampling(np.random.RandomState(seed + self.rank))

    def player(self) -> int:
        return self.rank % self.n

    def record(self, home: int, away: int, result: PayoffEntry, n: int = 1):
        """Local, race-free accumulation; published by sync_payoff()."""
        d = PayoffWrapper(self._delta, self.payoff.reference_compat)
        d.record_result(home, away, result, n)

    def record_match(self, home: int, away: int):
        self._delta[home, away, PayoffEntry.MATCHES] += 1

    def sync_payoff(self):
        if self.world > 1:
            dist.all_reduce(self._delta, op=dist.ReduceOp.SUM)
        self.payoff.tensor.add_(self._delta)
        self._delta.zero_()
        return self.payoff.tensor

    def share_params(self, flat: torch.Tensor):
        """Every rank's flat parameter vector (index = rank)."""
        flat = flat.detach().contiguous()
        if self.world == 1:
            return [flat.clone()]
        out = [torch.empty_like(flat) for _ in range(self.world)]
        dist.all_gather(out, flat)
        return out

    def pfsp_opponent(self, weighting: str = "squared", exclude_self: bool = False) -> int:
        """PFSPMatchmaking.get_match / SimplePlayer.get_match (matchmaker.py:64-72, simple_player.py:24-37)."""
        me = self.player()
        opponents = [i for i in range(self.n) if not (exclude_self and i == me)]
        wr = self.payoff.win_rates(me, opponents).cpu().numpy()
        return self.sampling.sample(opponents, prio_measure=wr, weighting=weighting)

    def barrier(self):
        if self.world > 1:
            dist.barrier()
