"""Action selection (API of src/marl/components/action_selectors.py:40-68), on the GPU.

EpsilonGreedyActionSelector.select masks unavailable actions to -inf, takes the first-index argmax
(torch.max semantics) and, with probability epsilon per agent, a uniformly random available action.
Randomness comes from the counter-based stream of the env spec instead of torch's
global generator, so CPU oracle and GPU kernel draw identical numbers; greedy picks are bit-exact
with the reference.
"""
from __future__ import annotations

import torch

from .epsilon_schedules import DecayThenFlatSchedule


class EpsilonGreedyActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.seed = int(getattr(args, "seed", 0) or 0)
        self._calls = 0

    def select(self, agent_inputs, avail_actions, t_env, test_mode=False):
        self.epsilon = self.schedule.eval(t_env)
        eps = 0.0 if test_mode else float(self.epsilon)
        if test_mode:
            self.epsilon = 0.0
        q = agent_inputs.float().contiguous()
        B, N, A = q.shape
        av = avail_actions.to(device=q.device, dtype=torch.int32).contiguous()
        keys = (torch.arange(B, dtype=torch.int64, device=q.device) + (self.seed << 32)).contiguous()
        episodes = torch.full((B,), self._calls & 0x7FFFFFFF, dtype=torch.int32, device=q.device)
        self._calls += 1
        from ..ops import select_actions
        return select_actions(q, av, keys, episodes, 0, eps)


class MultinomialActionSelector:
    """COMA's policy sampler -- outside the QMIX hot path (OUT OF SCOPE)."""

    def __init__(self, args):
        raise NotImplementedError("multinomial action selection (COMA) is out of scope for this build")


REGISTRY = {"epsilon_greedy": EpsilonGreedyActionSelector, "multinomial": MultinomialActionSelector}
