"""ctypes wrapper of oracle/env_ref.c -- the CPU restatement of the synthetic TeamsEnv spec v1.

TEST INFRASTRUCTURE ONLY (the checker / the timed CPU baseline). Env arithmetic is PARITY UNPINNED
against the reference's external ma-env (not in the container); this is the build's own
frozen spec, against which the HIP kernels must be bit-exact.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libenvref.so")
MAXU = 64


class CSpec(ctypes.Structure):
    _fields_ = [("U", ctypes.c_int), ("n_agents", ctypes.c_int), ("grid", ctypes.c_int),
                ("episode_limit", ctypes.c_int), ("stochastic", ctypes.c_int), ("team", ctypes.c_int * MAXU),
                ("role", ctypes.c_int * MAXU), ("melee", ctypes.c_int * MAXU), ("scripted", ctypes.c_int * 2),
                ("agent_unit", ctypes.c_int * MAXU), ("team_size", ctypes.c_int * 2), ("team_first", ctypes.c_int * 2),
                ("policy_team", ctypes.c_int)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        assert L.envref_sizeof_spec() == ctypes.sizeof(CSpec), "CSpec layout mismatch"
        P, I, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.envref_splitmix64.restype = U64
        L.envref_splitmix64.argtypes = [U64]
        L.envref_rng.restype = U64
        L.envref_rng.argtypes = [U64, U64]
        L.envref_ctr.restype = U64
        L.envref_ctr.argtypes = [ctypes.c_uint32] * 4
        L.envref_u01.restype = ctypes.c_float
        L.envref_u01.argtypes = [U64]
        L.envref_reset.argtypes = [P, U64, ctypes.c_uint32, P, P, P]
        L.envref_step.argtypes = [P, I, P, P, P, P, P, P, P, P]
        L.envref_obs.argtypes = [P, P, P, P, P]
        L.envref_state.argtypes = [P, P, P, P, P]
        L.envref_avail.argtypes = [P, P, P, P, P]
        L.envref_ai_action.argtypes = [P, P, P, P, I]
        _lib = L
    return _lib


def env_key(seed: int, env: int) -> int:
    return ((seed << 32) + env) & 0xFFFFFFFFFFFFFFFF


def ctr(episode: int, t: int, purpose: int, idx: int) -> int:
    return lib().envref_ctr(episode, t, purpose, idx)


def rng(key: int, c: int) -> int:
    return lib().envref_rng(key, c)


def u01(r: int) -> float:
    return float(np.float32((r >> 40) * (1.0 / 16777216.0)))


def random_available(avail_row, r: int) -> int:
    """k-th available action, k = ((r >> 40) * n) >> 24 (spec §3.7)."""
    idx = [a for a, v in enumerate(avail_row) if v]
    if not idx:
        return 0
    k = (((r >> 40) * len(idx)) >> 24)
    return idx[k]


class RefEnv:
    """One env of the spec (team/role/melee lists in plan unit order)."""

    def __init__(self, team, role, melee, scripted, grid=20, episode_limit=100, stochastic=True, seed=0, env_index=0):
        s = CSpec()
        U = len(team)
        s.U, s.grid, s.episode_limit, s.stochastic = U, grid, episode_limit, int(stochastic)
        for u in range(U):
            s.team[u], s.role[u], s.melee[u] = team[u], role[u], melee[u]
        s.scripted[0], s.scripted[1] = int(scripted[0]), int(scripted[1])
        agents = [u for u in range(U) if not scripted[team[u]]]
        s.n_agents = len(agents)
        for a, u in enumerate(agents):
            s.agent_unit[a] = u
        for tm in range(2):
            members = [u for u in range(U) if team[u] == tm]
            s.team_size[tm] = len(members)
            s.team_first[tm] = members[0] if members else 0
        s.policy_team = list(scripted).index(False)
        self.spec, self.U, self.N, self.A = s, U, len(agents), 5 + U
        self.key = env_key(seed, env_index)
        self.episode = 0
        self.t = 0
        self.x = np.zeros(U, np.int32)
        self.y = np.zeros(U, np.int32)
        self.hp = np.zeros(U, np.int32)
        self.scripted = list(scripted)
        self.policy_team = s.policy_team

    def _p(self, a):
        return a.ctypes.data_as(ctypes.c_void_p)

    def reset(self):
        lib().envref_reset(ctypes.byref(self.spec), self.key, self.episode, self._p(self.x), self._p(self.y),
                           self._p(self.hp))
        self.cur_episode = self.episode
        self.episode += 1
        self.t = 0

    def set_state(self, x, y, hp, t=0):
        self.x[:] = x
        self.y[:] = y
        self.hp[:] = hp
        self.t = t

    def step(self, actions):
        acts = np.ascontiguousarray(np.asarray(actions, dtype=np.int64).reshape(self.N))
        rewards = np.zeros(2, np.float32)
        done, draw = ctypes.c_int(0), ctypes.c_int(0)
        won = np.zeros(2, np.int32)
        lib().envref_step(ctypes.byref(self.spec), self.t, self._p(acts), self._p(self.x), self._p(self.y),
                          self._p(self.hp), self._p(rewards), ctypes.byref(done), self._p(won), ctypes.byref(draw))
        self.t += 1
        pt = self.policy_team
        reward_list = [float(rewards[tm]) for tm in range(2) if not self.scripted[tm]]
        info = {"battle_won": [bool(won[pt]), bool(won[1 - pt])], "draw": bool(draw.value)}
        return reward_list, bool(done.value), info

    def obs(self):
        o = np.zeros((self.N, 8 * self.U), np.float32)
        lib().envref_obs(ctypes.byref(self.spec), self._p(self.x), self._p(self.y), self._p(self.hp), self._p(o))
        return o

    def state(self):
        s = np.zeros(6 * self.U, np.float32)
        lib().envref_state(ctypes.byref(self.spec), self._p(self.x), self._p(self.y), self._p(self.hp), self._p(s))
        return s

    def avail(self):
        a = np.zeros((self.N, self.A), np.int32)
        lib().envref_avail(ctypes.byref(self.spec), self._p(self.x), self._p(self.y), self._p(self.hp), self._p(a))
        return a


class RefEntityEnv(RefEnv):
    """The entity ("refil") variant of the spec (env_ref.c envref_reset_entity / envref_entities): S slots per
    team, policy team = units 0..S-1 (the agents), scripted team = S..2S-1, k ~ U{kmin..kmax} active per team
    per episode."""

    def __init__(self, roles, melees, kmin, kmax, grid=20, episode_limit=100, stochastic=True, seed=0, env_index=0):
        S = len(roles)
        super().__init__([0] * S + [1] * S, list(roles) * 2, list(melees) * 2, [False, True], grid=grid,
                         episode_limit=episode_limit, stochastic=stochastic, seed=seed, env_index=env_index)
        self.kmin, self.kmax = int(kmin), int(kmax)
        self.k = None

    def reset(self):
        L = lib()
        L.envref_reset_entity.restype = ctypes.c_int
        L.envref_reset_entity.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        self.k = L.envref_reset_entity(ctypes.byref(self.spec), self.key, self.episode, self.kmin, self.kmax,
                                       self._p(self.x), self._p(self.y), self._p(self.hp))
        self.cur_episode = self.episode
        self.episode += 1
        self.t = 0

    def entities(self):
        U = self.U
        ent = np.zeros((U, 8), np.float32)
        om = np.zeros((U, U), np.uint8)
        em = np.zeros(U, np.uint8)
        L = lib()
        L.envref_entities.argtypes = [ctypes.c_void_p] * 7
        L.envref_entities(ctypes.byref(self.spec), self._p(self.x), self._p(self.y), self._p(self.hp), self._p(ent),
                          self._p(om), self._p(em))
        return ent, om, em
