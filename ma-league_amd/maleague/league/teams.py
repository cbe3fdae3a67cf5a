"""League team compositions: ``Team`` and ``TeamComposer`` (src/league/components/team_composer.py:18-181).

The reference enumerates every unit over the characteristic enums (``itertools.product(RoleTypes,
UnitAttackTypes)``, uid = position, :144-150), every team as a multiset of ``team_size`` units
(``combinations_with_replacement``, tid = position, :125-142) minus the all-healer teams (which can never win,
:136-138), samples ``league_size`` teams containing the forced unit (``random.sample``, :116-123) and sorts
each team's units by distance of their uid to the forced uid, so the forced unit comes first (:152-162;
``central_worker.py:44-50``). Team ``i`` belongs to league player ``i`` (``central_worker.py:84-93``), and each
match puts the home team against the adversary's team (``matchmaking_league_instance.py:52``,
``league_experiment_process.py:57-62``): ``match_plan``.

``RoleTypes`` / ``UnitAttackTypes`` come from maenv (``maenv.core``), which is absent here. The
enums below carry the build's order -- the role / attack ids of the env spec (TANK 0, HEALER 1,
ADC 2; RANGED 0, MELEE 1) -- so uids and tids follow from it; maenv's own member order is unpinned. The
algorithm (enumeration, filter, sampling, sorting, swap distance) is pinned bit-for-bit against the
reference's team_composer.py run with these enums (tests/golden/make_team_golden.py).

Sampling takes an explicit ``random.Random`` (``rng``): the reference draws from the process-global ``random``
module, which no one seeds; the league seeds one generator per league so every rank samples the same teams.
``random.Random(s).sample`` equals ``random.seed(s); random.sample`` draw for draw.
"""
from __future__ import annotations

import enum
import itertools
import math
import random
from collections import Counter
from functools import reduce
from typing import Dict, List, Optional, Sequence, Union

import numpy as np


class RoleTypes(enum.Enum):
    """maenv.core.RoleTypes members used by the configs (config/teams/*.json); value["id"] is read by Team."""
    TANK = {"id": 0}
    HEALER = {"id": 1}
    ADC = {"id": 2}


class UnitAttackTypes(enum.Enum):
    RANGED = {"id": 0}
    MELEE = {"id": 1}


def _enum(cls, v):
    """An enum member from a member, its name ("HEALER"), "RoleTypes.HEALER" or the JSON {"__enum__": ...} form."""
    if isinstance(v, cls):
        return v
    if isinstance(v, dict) and "__enum__" in v:
        v = v["__enum__"]
    return cls[str(v).split(".")[-1].upper()]


class Team:
    """team_composer.py:18-79. ``units``: dicts {uid, role, attack_type} (role / attack_type enum members)."""

    def __init__(self, tid: int, units: Sequence[Dict], is_scripted: bool = False):
        self.tid = tid
        self.units: List[Dict] = list(units)
        self._uids: List[int] = [u["uid"] for u in self.units]
        self._rids: List[int] = [u["role"].value["id"] for u in self.units]
        self.is_scripted = is_scripted

    def get_team_ids(self, query_ids: List[int]):
        """Positions in the team (as np.where's tuple) of units whose uid is one of ``query_ids`` (:26-33)."""
        uids = np.array(self._uids)
        mask = reduce(lambda x, y: x | y, [(uids == q) for q in query_ids])
        return np.where(mask)

    def contains(self, unit_ids: Union[List[int], int], unique: bool = False) -> bool:
        """At least one unit with one of ``unit_ids``; with ``unique`` exactly one (:35-47)."""
        if isinstance(unit_ids, int):
            unit_ids = [unit_ids]
        hits = sum(1 for u in self._uids if u in unit_ids)
        return hits == 1 if unique else hits > 0

    @property
    def roles(self):
        return {u["role"] for u in self.units}

    def __hash__(self):
        return self.tid

    def __eq__(self, other):
        return other is not None and isinstance(other, Team) and self.tid == other.tid

    def __str__(self):
        return f"Team #{self.tid}"

    __repr__ = __str__

    def difference(self, team: "Team") -> float:
        """Swap distance to ``team`` (:67-79): units this team has more of, weighted by how many kinds differ."""
        mine, theirs = Counter(self._uids), Counter(team._uids)
        diff = [mine[u] - theirs[u] if u in theirs else mine[u] for u in mine]
        surplus = [d for d in diff if d > 0]
        return sum(surplus) * (len(surplus) / sum(mine.values()))

    # ---- env plan ------------------------------------------------------------------------------------
    def plan_units(self) -> List[Dict]:
        """The units as match_build_plan entries (the config/teams/*.json form: EnumEncoder's {"__enum__"})."""
        return [{"role": {"__enum__": f"RoleTypes.{u['role'].name}"},
                 "attack_type": {"__enum__": f"UnitAttackTypes.{u['attack_type'].name}"}} for u in self.units]

    def codes(self) -> str:
        """Compact form, one "RA" pair per unit (role T/H/A, attack R/M), e.g. "HR TR TR AM AR"."""
        return " ".join(u["role"].name[0] + u["attack_type"].name[0] for u in self.units)

    def to_json(self) -> Dict:
        """AssetManager.save_team form (asset_manager.py:76-80): tid, is_scripted, units with enum names."""
        return {"tid": self.tid, "is_scripted": self.is_scripted, "units": self.plan_units()}


class TeamComposer:
    """team_composer.py:82-181."""

    def __init__(self, team_size: int, characteristics: Sequence[type] = (RoleTypes, UnitAttackTypes)):
        if not characteristics:
            raise ValueError("Please supply characteristics to create units from.")
        self.characteristics = list(characteristics)
        self.team_size = team_size
        self.teams: List[Team] = []
        self._compose_unique_teams(team_size)

    def __getitem__(self, item) -> Team:
        return self.teams[item]

    def __len__(self):
        return len(self.teams)

    def get_uids(self, type: enum.Enum, capability: str) -> List[int]:  # noqa: A002 (reference argument name)
        if capability not in ("role", "attack_type"):
            raise ValueError("Unknown capability")
        return [u["uid"] for u in self.units if u[capability] == type]

    def get_unique_uid(self, role_type, attack_type) -> int:
        if role_type is None or attack_type is None:
            raise ValueError("Please supply all characteristics to search unit ids.")
        role_type, attack_type = _enum(RoleTypes, role_type), _enum(UnitAttackTypes, attack_type)
        uid = [u["uid"] for u in self.units if u["role"] == role_type and u["attack_type"] == attack_type]
        if len(uid) != 1:
            raise ValueError(f"Consistency error: {len(uid)} units are {role_type.name}/{attack_type.name}.")
        return uid[0]

    def candidates(self, contains=None, unique: bool = False) -> List[Team]:
        return [t for t in self.teams if contains is None or t.contains(contains, unique)]

    def sample(self, k: int, contains=None, unique: bool = False, rng: Optional[random.Random] = None) -> List[Team]:
        """``k`` distinct teams, uniformly without replacement, among those containing ``contains`` (:116-123).
        Returns Team copies (their unit lists may then be re-sorted without touching the composer's teams)."""
        pool = self.candidates(contains, unique)
        picked = (rng or random).sample(pool, k=k)
        return [Team(t.tid, t.units, t.is_scripted) for t in picked]

    def _compose_unique_teams(self, team_size: int) -> List[Team]:
        units = list(self._compose_unique_units())
        self.units = units
        comps = itertools.combinations_with_replacement(units, team_size)
        plans = [{"tid": tid, "is_scripted": False, "units": comp} for tid, comp in enumerate(comps)]
        healers = self.get_uids(type=RoleTypes.HEALER, capability="role")
        plans = [p for p in plans if not all(u["uid"] in healers for u in p["units"])]
        self.build_plans = plans
        self.teams = [Team(**p) for p in plans]
        return self.teams

    def _compose_unique_units(self):
        return ({"uid": uid, "role": c[0], "attack_type": c[1]}
                for uid, c in enumerate(itertools.product(*self.characteristics)))

    @staticmethod
    def sort_team_units(teams: List[Team], uid: int = 0) -> List[Team]:
        """Stable sort of every team's units by |unit uid - uid| (:152-162): the forced unit first."""
        for team in teams:
            team.units.sort(key=lambda u: math.fabs(u["uid"] - uid))
            team._uids = [u["uid"] for u in team.units]
            team._rids = [u["role"].value["id"] for u in team.units]
        return teams


def compose_league_teams(team_size: int, league_size: int, role=None, attack=None, unique: bool = True,
                         seed: int = 0) -> List[Team]:
    """CentralWorker.run's team setup (central_worker.py:44-50): ``league_size`` sampled teams containing the forced
    unit (``force-unit --role --attack``), that unit sorted first. Without a forced unit every composition is a
    candidate (the reference then fails on the missing ``args.role``; here: no constraint, sorted around uid 0)."""
    composer = TeamComposer(team_size=team_size)
    uid = composer.get_unique_uid(role, attack) if role is not None and attack is not None else None
    teams = composer.sample(k=league_size, contains=uid, unique=unique, rng=random.Random(seed))
    return composer.sort_team_units(teams, uid=uid if uid is not None else 0)


def match_plan(home: Union[Team, Sequence[Dict]], away: Union[Team, Sequence[Dict], None] = None,
               ai: bool = False) -> List[Dict]:
    """LeagueExperimentInstance._configure_experiment (league_experiment_process.py:57-62): plan team 0 = the home
    (policy) team, team 1 = the away team -- its mirror when ``away`` is None -- scripted iff ``ai``."""
    def units(t):
        return t.plan_units() if isinstance(t, Team) else [dict(u) for u in t]
    home_u = units(home)
    away_u = home_u if away is None else units(away)
    return [{"is_scripted": False, "units": [dict(u) for u in home_u]},
            {"is_scripted": bool(ai), "units": [dict(u) for u in away_u]}]


def team_of_plan_units(units: Sequence[Dict], tid: int = -1) -> Team:
    """A Team from match_build_plan units (any accepted enum form); uids follow the composer's unit table."""
    roles, attacks = list(RoleTypes), list(UnitAttackTypes)
    out = []
    for u in units:
        r, a = _enum(RoleTypes, u["role"]), _enum(UnitAttackTypes, u.get("attack_type", "RANGED"))
        out.append({"uid": roles.index(r) * len(attacks) + attacks.index(a), "role": r, "attack_type": a})
    return Team(tid, out)


__all__ = ["RoleTypes", "UnitAttackTypes", "Team", "TeamComposer", "compose_league_teams", "match_plan",
           "team_of_plan_units"]

