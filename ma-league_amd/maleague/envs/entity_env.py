"""The entity ("refil") variant of the synthetic battle for the REFIL path (config 5).

REFIL consumes an entity scheme instead of per-agent obs / global state (src/marl/controllers/entity_controller.py:
11-30, src/marl/learners/refil_learner.py:81-100): ``entities`` [n_entities, entity_shape], ``obs_mask``
[n_entities, n_entities], ``entity_mask`` [n_entities], with the agents as the first ``n_agents`` entities. The
reference ships no env producing it (REFIL is vendored, unwired) and ma-env is absent (§0.2), so the
build defines one on top of spec v1: S unit slots per team (policy team = entities 0..S-1, scripted basic-AI
team = S..2S-1), k ~ U{min_agents..max_agents} active slots per team per episode, absent slots padded and
masked. Executed by the HIP kernel mlg_refil_rollout; checked bit-exact against oracle/env_ref.c.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

from .. import _native
from .plans import builtin_composition
from .teams_env import ATTACK_IDS, DEFAULT_EPISODE_LIMIT, ROLE_IDS, _enum_name, load_match_build_plan

ENTITY_SHAPE = 8


@dataclass
class EntityEnvSpec:
    roles: List[int]   # per slot (both teams use the same composition)
    melees: List[int]
    min_agents: int = 3
    max_agents: int = 8
    grid: int = 20
    episode_limit: int = DEFAULT_EPISODE_LIMIT
    stochastic: bool = True
    seed: int = 0

    @classmethod
    def from_env_args(cls, env_args: dict, config_dir: str | None = None) -> "EntityEnvSpec":
        plan = env_args.get("match_build_plan", "refil_8")
        if isinstance(plan, str) and plan in ("refil_8",):
            units = builtin_composition(plan)
        else:
            teams = load_match_build_plan(plan, config_dir)
            home = next((t for t in teams if not t.get("is_scripted", False)), teams[0])
            units = [(_enum_name(u["role"]), _enum_name(u.get("attack_type", "RANGED"))) for u in home["units"]]
        roles = [ROLE_IDS[r] for r, _ in units]
        melees = [ATTACK_IDS[a] for _, a in units]
        S = len(roles)
        if not 1 <= S <= 8:
            raise ValueError(f"entity env supports 1..8 unit slots per team, got {S}")
        kmax = int(env_args.get("max_agents", S))
        kmin = int(env_args.get("min_agents", min(3, kmax)))
        if not 1 <= kmin <= kmax <= S:
            raise ValueError(f"need 1 <= min_agents <= max_agents <= {S}, got {kmin}, {kmax}")
        return cls(roles=roles, melees=melees, min_agents=kmin, max_agents=kmax,
                   grid=int(env_args.get("grid_size", 20)),
                   episode_limit=int(env_args.get("episode_limit", DEFAULT_EPISODE_LIMIT)),
                   stochastic=bool(env_args.get("stochastic_spawns", True)), seed=int(env_args.get("seed", 0) or 0))

    @property
    def S(self) -> int:
        return len(self.roles)

    @property
    def U(self) -> int:
        return 2 * self.S

    @property
    def n_agents(self) -> int:
        return self.S

    @property
    def n_entities(self) -> int:
        return self.U

    @property
    def n_actions(self) -> int:
        return 5 + self.U

    policy_team = 0

    def env_info(self) -> dict:
        return {"n_agents": self.n_agents, "n_actions": self.n_actions, "n_entities": self.n_entities,
                "entity_shape": ENTITY_SHAPE, "episode_limit": self.episode_limit,
                "obs_shape": ENTITY_SHAPE, "state_shape": ENTITY_SHAPE * self.n_entities}

    def to_c(self) -> _native.MlgEntityEnvSpec:
        c = _native.MlgEntityEnvSpec()
        s = c.base
        S = self.S
        s.U, s.n_agents, s.n_actions = self.U, S, self.n_actions
        s.grid, s.episode_limit, s.stochastic = self.grid, self.episode_limit, int(self.stochastic)
        s.policy_team, s.n_policy_teams = 0, 1
        for u in range(self.U):
            s.team[u] = 0 if u < S else 1
            s.role[u] = self.roles[u % S]
            s.melee[u] = self.melees[u % S]
        for a in range(S):
            s.agent_unit[a] = a
        s.scripted[0], s.scripted[1] = 0, 1
        s.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        c.min_agents, c.max_agents = self.min_agents, self.max_agents
        return c
