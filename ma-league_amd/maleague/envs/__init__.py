"""Env registry (reference: src/envs/__init__.py:9 -- REGISTRY["ma"])."""
from .entity_env import EntityEnvSpec
from .teams_env import TeamsEnv, TeamsEnvSpec, VecEnvState, load_match_build_plan


def ma_env(**kwargs) -> TeamsEnv:
    return TeamsEnv(**kwargs)


REGISTRY = {"ma": ma_env}

__all__ = ["EntityEnvSpec", "REGISTRY", "TeamsEnv", "TeamsEnvSpec", "VecEnvState", "load_match_build_plan"]
