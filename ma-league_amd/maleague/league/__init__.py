from .distributed import DistributedLeague
from .payoff import (REGISTRY, FSPSampling, PayoffEntry, PayoffWrapper, PFSPSampling, SPSampling,
                     episode_result)

__all__ = ["DistributedLeague", "PayoffEntry", "PayoffWrapper", "PFSPSampling", "FSPSampling", "SPSampling",
           "REGISTRY", "episode_result"]
