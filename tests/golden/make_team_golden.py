"""Generate the TeamComposer golden fixture (tests/golden/teams.json) from the reference's own team_composer.py.

TEST INFRASTRUCTURE ONLY. Runs in the build container, where the reference is mounted read-only at /root/reference.
It loads /root/reference/src/league/components/team_composer.py as a standalone module (importing the `league`
package would pull in torch.multiprocessing / maenv / sacred) with ONE probe shim: a `maenv.core` module exposing
RoleTypes / UnitAttackTypes -- maenv is absent here, so the enums are the build's own
(maleague.league.teams: TANK, HEALER, ADC / RANGED, MELEE). The fixture records data only (uids, tids, sampled
tids, sorted unit orders, swap distances); no reference source text.

Recorded (team_composer.py line ranges):
  units         _compose_unique_units              :144-150
  teams         _compose_unique_teams (+ healer filter) :125-142, team_size 1..5
  samples       random.seed(s); sample(k, contains=uid, unique) :116-123 -> tids, then sort_team_units(uid) :152-162
                -> per team the uid order
  contains      Team.contains(uids, unique)         :35-47
  difference    Team.difference                      :67-79
  team_ids      Team.get_team_ids                    :26-33

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_team_golden.py
"""
import importlib.util
import json
import os
import random
import sys
import types

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ma-league_amd"))
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "teams.json")
REF = "/root/reference/src/league/components/team_composer.py"

from maleague.league.teams import RoleTypes, UnitAttackTypes  # noqa: E402


def load_reference():
    maenv = types.ModuleType("maenv")
    core = types.ModuleType("maenv.core")
    core.RoleTypes, core.UnitAttackTypes = RoleTypes, UnitAttackTypes
    maenv.core = core
    sys.modules["maenv"], sys.modules["maenv.core"] = maenv, core
    spec = importlib.util.spec_from_file_location("ref_team_composer", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ref = load_reference()
    out = {"enum_order": {"RoleTypes": [m.name for m in RoleTypes],
                          "UnitAttackTypes": [m.name for m in UnitAttackTypes]},
           "compositions": {}, "samples": [], "contains": [], "difference": [], "team_ids": []}
    for size in (1, 2, 3, 4, 5):
        comp = ref.TeamComposer(team_size=size, characteristics=[RoleTypes, UnitAttackTypes])
        out["compositions"][str(size)] = {
            "units": [[u["uid"], u["role"].name, u["attack_type"].name] for u in comp.units],
            "teams": [[t.tid, [u["uid"] for u in t.units]] for t in comp.teams],
        }
    comp5 = ref.TeamComposer(team_size=5, characteristics=[RoleTypes, UnitAttackTypes])
    comp3 = ref.TeamComposer(team_size=3, characteristics=[RoleTypes, UnitAttackTypes])
    for comp, size in ((comp5, 5), (comp3, 3)):
        for role, attack in ((RoleTypes.HEALER, UnitAttackTypes.RANGED), (RoleTypes.TANK, UnitAttackTypes.RANGED),
                             (RoleTypes.ADC, UnitAttackTypes.MELEE)):
            uid = comp.get_unique_uid(role_type=role, attack_type=attack)
            for unique in (True, False):
                for seed, k in ((0, 2), (1, 4), (7, 8), (123, 5)):
                    random.seed(seed)
                    teams = comp.sample(k=k, contains=uid, unique=unique)
                    tids = [t.tid for t in teams]
                    # the reference sorts the composer's own Team objects' unit lists in place: copy the order out
                    import copy
                    teams = [copy.copy(t) for t in teams]
                    for t in teams:
                        t.units = list(t.units)
                    comp.sort_team_units(teams, uid=uid)
                    out["samples"].append({"team_size": size, "role": role.name, "attack": attack.name, "uid": uid,
                                           "unique": unique, "seed": seed, "k": k, "tids": tids,
                                           "sorted_uids": [[u["uid"] for u in t.units] for t in teams]})
    rng = random.Random(42)
    teams = comp5.teams
    for _ in range(60):
        t = teams[rng.randrange(len(teams))]
        q = rng.sample(range(6), rng.randint(1, 3))
        for unique in (True, False):
            out["contains"].append({"tid": t.tid, "query": q, "unique": unique, "result": bool(t.contains(q, unique))})
        out["team_ids"].append({"tid": t.tid, "query": q, "result": [int(i) for i in t.get_team_ids(q)[0]]})
    for _ in range(60):
        a, b = teams[rng.randrange(len(teams))], teams[rng.randrange(len(teams))]
        out["difference"].append({"a": a.tid, "b": b.tid, "result": float(a.difference(b))})
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {OUT}: {len(out['samples'])} samples, {sum(len(c['teams']) for c in out['compositions'].values())} "
          f"teams")


if __name__ == "__main__":
    main()
