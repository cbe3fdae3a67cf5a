"""Built-in match build plans, keyed like the reference's src/config/teams/<name>.json.

A plan is two teams [scripted AI team, policy team]; each unit is (role, attack type). Compact codes:
role T=TANK H=HEALER A=ADC; attack R=RANGED M=MELEE. A user's own config/teams/*.json files (the
reference format with {"__enum__": "RoleTypes.X"} fields) are read directly by load_match_build_plan
when a config directory is given; these built-ins make the package self-contained.
"""
from __future__ import annotations

_ROLE = {"T": "TANK", "H": "HEALER", "A": "ADC"}
_ATK = {"R": "RANGED", "M": "MELEE"}

_COMPOSITIONS = {
    "small": "TR TR TR",
    "medium": "TR TR TR TR TR",
    "medium_1h_4t": "TR TR HR TR TR",
    "medium_1h_4a": "AR AR HR AR AR",
    "medium_1h_2t_2a": "TR TR HR AR AR",
    "medium_1h_2t_2a_melee": "TM TM HM AM AM",
    "large": " ".join(["TR"] * 25),
    # entity env (REFIL, config 5): 8 slots per team, the first k in play; every k >= 3 fields a healer
    "refil_8": "TR AR HR AR TM AR HR AM",
}


def team_from_codes(codes: str, is_scripted: bool) -> dict:
    units = [{"role": {"__enum__": f"RoleTypes.{_ROLE[c[0]]}"},
              "attack_type": {"__enum__": f"UnitAttackTypes.{_ATK[c[1]]}"}} for c in codes.split()]
    return {"is_scripted": is_scripted, "units": units}


def builtin_plan(name: str, self_play: bool = False):
    """Team plan list for a built-in name; self_play makes both teams policy-controlled."""
    codes = _COMPOSITIONS[name]
    return [team_from_codes(codes, not self_play), team_from_codes(codes, False)]


def available() -> list:
    return sorted(_COMPOSITIONS)


def mirror_plan(plan, ai: bool, config_dir=None):
    """LeagueExperimentInstance._configure_experiment (league_experiment_process.py:57-62) with no away team:
    team 0 = the home (policy) team, team 1 = its mirror, scripted iff ``ai``."""
    from .teams_env import load_match_build_plan
    teams = load_match_build_plan(plan, config_dir)
    home = next((t for t in teams if not t.get("is_scripted", False)), teams[0])
    return [{"is_scripted": False, "units": list(home["units"])},
            {"is_scripted": bool(ai), "units": list(home["units"])}]


def builtin_composition(name: str):
    """[(ROLE, ATTACK), ...] unit slots of a built-in composition."""
    return [(_ROLE[c[0]], _ATK[c[1]]) for c in _COMPOSITIONS[name].split()]
