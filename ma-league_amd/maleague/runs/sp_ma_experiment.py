"""Self-play training loop (API of src/runs/train/sp_ma_experiment.py:12-101 and the league's
LeagueExperiment, src/runs/train/league_experiment.py:6-24).

The opposing team is a second, frozen policy instead of the scripted AI: both MACs act in the same
fused rollout launch (SelfPlayParallelStepper), only the home learner trains (sp_ma_experiment.py:81).
"""
from __future__ import annotations

from typing import OrderedDict

import torch

from ..controllers import REGISTRY as mac_REGISTRY
from ..learners.q_learner import FlatParams
from ..utils.flat import module_flat_view
from ..steppers import SELF_REGISTRY as self_steppers_REGISTRY
from .ma_experiment import MultiAgentExperiment


def agent_vector(mac) -> torch.Tensor:
    """The MAC's agent parameters as one flat vector (named_parameters order): a view of them when they are back
    to back in one buffer (a learner's FlatParams -- callers copy what they keep), else a concatenated copy."""
    flat = module_flat_view(mac.agent)
    if flat is not None:
        return flat.detach()
    return torch.nn.utils.parameters_to_vector(mac.agent.parameters()).detach()


@torch.no_grad()
def load_agent_vector(mac, vec: torch.Tensor):
    """In-place copy (keeps a learner's flat-parameter views valid; bumps versions -> weights repacked)."""
    flat = module_flat_view(mac.agent)
    if flat is not None:  # parameters back to back in one buffer: one copy
        if flat.numel() != vec.numel():
            raise ValueError(f"parameter vector of {vec.numel()} floats for an agent of {flat.numel()}")
        flat.copy_(vec.reshape(-1))
        mac.agent.mark_dirty()  # writes through the flat view bump no parameter version: repack explicitly
        return
    params = list(mac.agent.parameters())
    n = sum(p.numel() for p in params)
    if n != vec.numel():
        raise ValueError(f"parameter vector of {vec.numel()} floats for an agent of {n}")
    off = 0
    for p in params:
        k = p.numel()
        p.copy_(vec[off:off + k].view_as(p))
        off += k


class SelfPlayMultiAgentExperiment(MultiAgentExperiment):
    def __init__(self, args, logger, on_episode_end=None, log_start_t=0):
        super().__init__(args, logger, on_episode_end=on_episode_end, log_start_t=log_start_t)
        # the away agent uses the home buffer's scheme (sp_ma_experiment.py:24-25)
        self.away_mac = mac_REGISTRY[self.args.mac](self.home_buffer.scheme, self.groups, self.args)
        # the frozen opponent's parameters as views of one flat buffer: an opponent swap is one copy
        FlatParams(self.away_mac.agent.parameters(), self.args.device)

    def load_adversary(self, agent: OrderedDict):
        """Frozen opponent parameters (a DRQN state_dict), sp_ma_experiment.py:27-29."""
        self.away_mac.load_state_dict(agent=agent)
        del agent

    def load_adversary_vector(self, vec: torch.Tensor):
        """Opponent parameters as a flat vector (the league's agent pool, exchanged over RCCL)."""
        load_agent_vector(self.away_mac, vec)

    def _integrate_env_info(self):
        total_n_agents = int(self.env_info["n_agents"])
        if total_n_agents % 2:
            raise ValueError(f"A total of {total_n_agents} agents in the env do not fit in the symmetric two-team "
                             "scenario. Ensure the Self-Play scenario has two team set to is_scripted=False")
        env_scheme = {"n_agents": total_n_agents // 2, "n_actions": int(self.env_info["n_actions"]),
                      "state_shape": int(self.env_info["state_shape"]), "total_n_agents": total_n_agents}
        self._update_args(env_scheme)
        self.stepper.args = self.args
        return env_scheme

    def _build_stepper(self, log_start_t=0):
        return self_steppers_REGISTRY[self.args.runner](args=self.args, logger=self.logger, log_start_t=log_start_t)

    def _init_stepper(self):
        # (re)initialised every call like the reference (sp_ma_experiment.py:54-58): the away MAC may change
        self.stepper.initialize(scheme=self.scheme, groups=self.groups, preprocess=self.preprocess,
                                home_mac=self.home_mac, away_mac=self.away_mac)
        if getattr(self.args, "zero_copy_insert", True):
            self.stepper.attach_replay(self.home_buffer)

    def _train_episode(self, episode_num):
        home_batch, _, env_info = self.stepper.run(test_mode=False)
        if self.on_episode_end is not None:
            self.on_episode_end(env_info)
        self.home_buffer.insert_episode_batch(home_batch)
        # only the learning (home) agent trains, never its frozen adversary (sp_ma_experiment.py:81)
        self._train_home(episode_num)

    def evaluate_mean_returns(self, episode_n=1):
        """Mean home / away episode returns over episode_n test runs (sp_ma_experiment.py:86-101)."""
        home = torch.zeros(episode_n)
        away = torch.zeros(episode_n)
        self._init_stepper()
        for i in range(episode_n):
            hb, ab, _ = self.stepper.run(test_mode=True)
            home[i] = hb["reward"].sum().item() / hb.batch_size
            away[i] = ab["reward"].sum().item() / ab.batch_size
        self.stepper.close_env()
        return home.mean(), away.mean()


class LeagueExperiment(SelfPlayMultiAgentExperiment):
    """league_experiment.py:6-24: self-play training whose home agent can be replaced between matches."""

    def _test(self, n_test_runs):
        self.last_test_T = self.stepper.t_env  # tests skipped in the league to save compute (:17-19)

    def load_home_agent(self, agent: OrderedDict):
        self.home_mac.load_state_dict(agent=agent)
        del agent

    def configure_match(self, home, away=None):
        """LeagueExperimentInstance._configure_experiment(home, away, ai=False) (league_experiment_process.py:57-62):
        plan team 0 = the home team's roster, team 1 = the adversary's (the home roster mirrored when ``away`` is
        None). ``home`` / ``away``: league Teams or match_build_plan unit lists. The reference builds a new
        LeagueExperiment (env, buffer, optimizer) per match; here the stepper swaps the env spec in place."""
        from ..league.teams import match_plan
        self.stepper.set_match_build_plan(match_plan(home, away))
