"""TeamComposer / Team (maleague.league.teams) against the reference's team_composer.py (tests/golden/teams.json,
written by tests/golden/make_team_golden.py with the build's RoleTypes / UnitAttackTypes enums -- maenv's own enum
order is unpinned), plus the league-facing helpers (compose_league_teams, match_plan -> TeamsEnvSpec)."""
import json
import os
import random

import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(GOLDEN, "teams.json")) as f:
        return json.load(f)


def test_enum_order_matches_fixture(fx):
    from maleague.league.teams import RoleTypes, UnitAttackTypes
    assert fx["enum_order"] == {"RoleTypes": [m.name for m in RoleTypes],
                                "UnitAttackTypes": [m.name for m in UnitAttackTypes]}


@pytest.mark.parametrize("size", [1, 2, 3, 4, 5])
def test_compositions_match_reference(fx, size):
    """_compose_unique_units / _compose_unique_teams (team_composer.py:125-150): uids, tids (all-healer teams
    filtered out after numbering), unit multisets in enumeration order."""
    from maleague.league.teams import TeamComposer
    c = TeamComposer(team_size=size)
    ref = fx["compositions"][str(size)]
    assert [[u["uid"], u["role"].name, u["attack_type"].name] for u in c.units] == ref["units"]
    assert [[t.tid, [u["uid"] for u in t.units]] for t in c.teams] == ref["teams"]


def test_sample_and_sort_match_reference(fx):
    """sample(k, contains=uid, unique) after random.seed(s) (team_composer.py:116-123) picks the same tids with a
    seeded random.Random; sort_team_units(uid) (:152-162) gives the same unit order (forced unit first)."""
    from maleague.league.teams import TeamComposer
    comps = {5: TeamComposer(5), 3: TeamComposer(3)}
    for s in fx["samples"]:
        c = comps[s["team_size"]]
        assert c.get_unique_uid(s["role"], s["attack"]) == s["uid"]
        teams = c.sample(k=s["k"], contains=s["uid"], unique=s["unique"], rng=random.Random(s["seed"]))
        assert [t.tid for t in teams] == s["tids"], s
        c.sort_team_units(teams, uid=s["uid"])
        assert [[u["uid"] for u in t.units] for t in teams] == s["sorted_uids"], s
        if s["unique"]:
            assert all(t.units[0]["uid"] == s["uid"] for t in teams)


def test_team_queries_match_reference(fx):
    from maleague.league.teams import TeamComposer
    c = TeamComposer(5)
    by_tid = {t.tid: t for t in c.teams}
    for q in fx["contains"]:
        assert by_tid[q["tid"]].contains(q["query"], q["unique"]) == q["result"], q
    for q in fx["team_ids"]:
        assert [int(i) for i in by_tid[q["tid"]].get_team_ids(q["query"])[0]] == q["result"], q
    for q in fx["difference"]:
        assert by_tid[q["a"]].difference(by_tid[q["b"]]) == pytest.approx(q["result"], abs=0, rel=0), q


def test_sample_does_not_mutate_composer():
    from maleague.league.teams import TeamComposer
    c = TeamComposer(5)
    before = [[u["uid"] for u in t.units] for t in c.teams]
    uid = c.get_unique_uid("HEALER", "RANGED")
    teams = c.sample(k=6, contains=uid, unique=True, rng=random.Random(3))
    c.sort_team_units(teams, uid=uid)
    assert [[u["uid"] for u in t.units] for t in c.teams] == before
    assert all(t.units[0]["uid"] == uid and t.get_team_ids([uid])[0].tolist() == [0] for t in teams)


def test_compose_league_teams_and_match_plan_spec():
    """central_worker.py:44-50 (force-unit HEALER / RANGED, unique): league_size distinct teams, each holding the
    forced unit exactly once, first; match_plan (league_experiment_process.py:57-62) -> an env spec whose team-0
    units are the home roster and team-1 units the away roster (both policy-controlled)."""
    from maleague.envs.teams_env import ATTACK_IDS, ROLE_IDS, TeamsEnvSpec
    from maleague.league.teams import compose_league_teams, match_plan
    teams = compose_league_teams(team_size=5, league_size=8, role="HEALER", attack="RANGED", seed=0)
    assert len({t.tid for t in teams}) == 8
    for t in teams:
        assert t.codes().split()[0] == "HR" and t.codes().split().count("HR") == 1
    assert [t.tid for t in compose_league_teams(5, 8, "HEALER", "RANGED", seed=0)] == [t.tid for t in teams]
    home, away = teams[0], teams[3]
    spec = TeamsEnvSpec.from_env_args({"match_build_plan": match_plan(home, away)})
    assert spec.n_agents == 10 and spec.n_policy_teams == 2 and spec.U == 10
    for side, t in ((0, home), (1, away)):
        for j, u in enumerate(t.units):
            assert spec.team[5 * side + j] == side
            assert spec.role[5 * side + j] == ROLE_IDS[u["role"].name]
            assert spec.melee[5 * side + j] == ATTACK_IDS[u["attack_type"].name]
    ai = TeamsEnvSpec.from_env_args({"match_build_plan": match_plan(home, ai=True)})
    assert ai.n_agents == 5 and ai.role[5:] == ai.role[:5] and ai.scripted == [False, True]


def test_team_json_roundtrip():
    from maleague.league.teams import TeamComposer, team_of_plan_units
    t = TeamComposer(5).teams[100]
    back = team_of_plan_units(json.loads(json.dumps(t.to_json()))["units"], tid=t.tid)
    assert [u["uid"] for u in back.units] == [u["uid"] for u in t.units] and back == t
