from .ma_experiment import MultiAgentExperiment
from .sp_ma_experiment import LeagueExperiment, SelfPlayMultiAgentExperiment

REGISTRY = {"normal": MultiAgentExperiment, "self": SelfPlayMultiAgentExperiment, "league": LeagueExperiment}

__all__ = ["MultiAgentExperiment", "SelfPlayMultiAgentExperiment", "LeagueExperiment", "REGISTRY"]
