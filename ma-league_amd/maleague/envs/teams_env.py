"""The "ma" environment: synthetic N-vs-N team battle, spec v1, on gfx950.

The reference constructs ``maenv.environment.TeamsEnv(**env_args)`` (src/envs/__init__.py:5-9), an
external package that is not available here. This module keeps its consumed interface
(SURVEY Appendix B): ``get_env_info()``, ``reset()``, ``step(actions)``, ``get_obs()``, ``get_state()``,
``get_avail_actions()``, ``close()``, built from the same ``env_args`` (match_build_plan, grid_size,
stochastic_spawns, seed, ...). The arithmetic is the build's frozen spec, executed by the HIP kernels
of libmaleague (mlg_env_* / mlg_rollout).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import List

import torch

from .. import _native

ROLE_IDS = {"TANK": 0, "HEALER": 1, "ADC": 2}
ATTACK_IDS = {"RANGED": 0, "MELEE": 1}
DEFAULT_EPISODE_LIMIT = 100


def _enum_name(v) -> str:
    """Accepts {"__enum__": "RoleTypes.TANK"}, "RoleTypes.TANK", "TANK" or an Enum member."""
    if isinstance(v, dict) and "__enum__" in v:
        v = v["__enum__"]
    if hasattr(v, "name") and not isinstance(v, str):
        v = v.name
    return str(v).split(".")[-1].upper()


def load_match_build_plan(plan, config_dir: str | None = None):
    """Resolve env_args["match_build_plan"]: a list of team dicts, or the name of config/teams/<name>.json
    (utils/main_utils.py:21-30 of the reference)."""
    if isinstance(plan, (list, tuple)):
        return [dict(t) for t in plan]
    plan = str(plan)
    candidates = [plan] if plan.endswith(".json") else []
    if config_dir is not None:
        candidates.append(os.path.join(config_dir, "teams", f"{plan}.json"))
    for path in candidates:
        if os.path.exists(path):
            with open(path) as f:
                return json.load(f)
    from .plans import builtin_plan
    try:
        return builtin_plan(plan)
    except KeyError:
        raise FileNotFoundError(f"match_build_plan {plan!r} not found (searched {candidates} and built-ins)")


@dataclass
class TeamsEnvSpec:
    """Host mirror of MlgEnvSpec."""
    team: List[int]
    role: List[int]
    melee: List[int]
    scripted: List[bool]
    grid: int = 20
    episode_limit: int = DEFAULT_EPISODE_LIMIT
    stochastic: bool = True
    seed: int = 0
    agent_unit: List[int] = field(default_factory=list)

    @classmethod
    def from_env_args(cls, env_args: dict, config_dir: str | None = None) -> "TeamsEnvSpec":
        plan = load_match_build_plan(env_args["match_build_plan"], config_dir)
        if len(plan) != 2:
            raise ValueError(f"match_build_plan must hold exactly two teams, got {len(plan)}")
        team, role, melee = [], [], []
        for tid, t in enumerate(plan):
            for u in t["units"]:
                team.append(tid)
                r = _enum_name(u["role"])
                a = _enum_name(u.get("attack_type", "RANGED"))
                if r not in ROLE_IDS:
                    raise ValueError(f"unknown role {r}")
                if a not in ATTACK_IDS:
                    raise ValueError(f"unknown attack type {a}")
                role.append(ROLE_IDS[r])
                melee.append(ATTACK_IDS[a])
        scripted = [bool(t.get("is_scripted", False)) for t in plan]
        if all(scripted):
            raise ValueError("match_build_plan needs at least one non-scripted (policy) team")
        if len(team) > _native.MAXU:
            raise ValueError(f"at most {_native.MAXU} units supported, got {len(team)}")
        agent_unit = [u for u in range(len(team)) if not scripted[team[u]]]
        return cls(team=team, role=role, melee=melee, scripted=scripted,
                   grid=int(env_args.get("grid_size", 20)),
                   episode_limit=int(env_args.get("episode_limit", DEFAULT_EPISODE_LIMIT)),
                   stochastic=bool(env_args.get("stochastic_spawns", True)),
                   seed=int(env_args.get("seed", 0) or 0),
                   agent_unit=agent_unit)

    @property
    def U(self) -> int:
        return len(self.team)

    @property
    def n_agents(self) -> int:
        return len(self.agent_unit)

    @property
    def n_actions(self) -> int:
        return 5 + self.U

    @property
    def policy_team(self) -> int:
        return self.scripted.index(False)

    @property
    def n_policy_teams(self) -> int:
        return sum(1 for s in self.scripted if not s)

    def env_info(self) -> dict:
        return {"n_agents": self.n_agents, "n_actions": self.n_actions, "state_shape": 6 * self.U,
                "obs_shape": 8 * self.U, "episode_limit": self.episode_limit}

    def to_c(self) -> _native.MlgEnvSpec:
        s = _native.MlgEnvSpec()
        s.U, s.n_agents, s.n_actions = self.U, self.n_agents, self.n_actions
        s.grid, s.episode_limit, s.stochastic = self.grid, self.episode_limit, int(self.stochastic)
        s.policy_team, s.n_policy_teams = self.policy_team, self.n_policy_teams
        for u in range(self.U):
            s.team[u], s.role[u], s.melee[u] = self.team[u], self.role[u], self.melee[u]
        for a, u in enumerate(self.agent_unit):
            s.agent_unit[a] = u
        s.scripted[0], s.scripted[1] = int(self.scripted[0]), int(self.scripted[1])
        s.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        return s


class VecEnvState:
    """Device-resident SoA state of B envs (x, y, hp [B, U] int32; t [B]; episode counters [B])."""

    def __init__(self, spec: TeamsEnvSpec, B: int, device):
        self.spec, self.B, self.device = spec, B, torch.device(device)
        U = spec.U
        self.x = torch.zeros(B, U, dtype=torch.int32, device=self.device)
        self.y = torch.zeros(B, U, dtype=torch.int32, device=self.device)
        self.hp = torch.zeros(B, U, dtype=torch.int32, device=self.device)
        self.t = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.episode = torch.zeros(B, dtype=torch.int32, device=self.device)  # read as uint32 by the kernels

    def to_c(self) -> _native.MlgEnvState:
        p = _native.ptr
        return _native.MlgEnvState(p(self.x), p(self.y), p(self.hp), p(self.t), p(self.episode), self.B)


class TeamsEnv:
    """Single-env TeamsEnv API (what EnvWorker drives, env_worker_process.py:27-71), on the GPU."""

    def __init__(self, device="cuda", config_dir: str | None = None, **env_args):
        self.spec = TeamsEnvSpec.from_env_args(env_args, config_dir)
        self.device = torch.device(device)
        self._cspec = self.spec.to_c()
        self.state = VecEnvState(self.spec, 1, self.device)
        self.episode_limit = self.spec.episode_limit
        U, N, A = self.spec.U, self.spec.n_agents, self.spec.n_actions
        self._obs = torch.zeros(1, N, 8 * U, device=self.device)
        self._st = torch.zeros(1, 6 * U, device=self.device)
        self._avail = torch.zeros(1, N, A, dtype=torch.int32, device=self.device)
        self._reward = torch.zeros(1, self.spec.n_policy_teams, device=self.device)
        self._done = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._won = torch.zeros(1, 2, dtype=torch.int32, device=self.device)
        self._draw = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._fresh = False

    def get_env_info(self) -> dict:
        return self.spec.env_info()

    def _observe(self):
        st = self.state.to_c()
        _native.call("mlg_env_observe", _native.byref(self._cspec), _native.byref(st), _native.ptr(self._obs),
                     _native.ptr(self._st), _native.ptr(self._avail), _native.stream_ptr())
        self._fresh = True

    def reset(self):
        st = self.state.to_c()
        _native.call("mlg_env_reset", _native.byref(self._cspec), _native.byref(st), _native.stream_ptr())
        self._observe()
        return self.get_obs()

    def step(self, actions):
        a = torch.as_tensor(actions).to(device=self.device, dtype=torch.int64).reshape(1, self.spec.n_agents)
        a = a.contiguous()
        st = self.state.to_c()
        _native.call("mlg_env_step", _native.byref(self._cspec), _native.byref(st), _native.ptr(a),
                     _native.ptr(self._reward), _native.ptr(self._done), _native.ptr(self._won),
                     _native.ptr(self._draw), _native.stream_ptr())
        self._observe()
        done = bool(self._done.item())
        info = {"battle_won": [bool(v) for v in self._won[0].tolist()], "draw": bool(self._draw.item())}
        n_teams = 2
        return self.get_obs(), self._reward[0].tolist(), [done] * n_teams, info

    def get_obs(self):
        return self._obs[0].tolist()

    def get_state(self):
        return self._st[0].tolist()

    def get_avail_actions(self):
        return self._avail[0].tolist()

    def render(self):
        pass

    def close(self):
        pass
