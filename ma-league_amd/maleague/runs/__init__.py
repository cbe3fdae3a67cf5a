from .ma_experiment import MultiAgentExperiment

REGISTRY = {"normal": MultiAgentExperiment}

__all__ = ["MultiAgentExperiment", "REGISTRY"]
