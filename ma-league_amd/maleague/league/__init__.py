from .distributed import DistributedLeague
from .instance import LeagueInstance, league_roles_for
from .matchmaking import REGISTRY as MATCHMAKING_REGISTRY
from .payoff import (REGISTRY, FSPSampling, PayoffEntry, PayoffWrapper, PFSPSampling, SPSampling,
                     episode_result)
from .roles import (ROLES, LeagueExploiter, LeagueView, MainExploiter, MainPlayer, SimplePlayer, alphastar_roles,
                    remove_monotonic_suffix)

__all__ = ["DistributedLeague", "LeagueInstance", "league_roles_for", "MATCHMAKING_REGISTRY", "PayoffEntry",
           "PayoffWrapper", "PFSPSampling", "FSPSampling", "SPSampling", "REGISTRY", "episode_result", "ROLES",
           "LeagueView", "MainPlayer", "MainExploiter", "LeagueExploiter", "SimplePlayer", "alphastar_roles",
           "remove_monotonic_suffix"]
