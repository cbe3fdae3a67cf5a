"""Stepper registries (reference: src/steppers/__init__.py:6-12)."""
from .parallel_stepper import EnvStepper, EpisodeStepper, ParallelStepper
from .self_play_stepper import SelfPlayParallelStepper, SelfPlayStepper

REGISTRY = {"episode": EpisodeStepper, "parallel": ParallelStepper}
SELF_REGISTRY = {"episode": SelfPlayStepper, "parallel": SelfPlayParallelStepper}

__all__ = ["EnvStepper", "EpisodeStepper", "ParallelStepper", "SelfPlayParallelStepper", "SelfPlayStepper",
           "REGISTRY", "SELF_REGISTRY"]
