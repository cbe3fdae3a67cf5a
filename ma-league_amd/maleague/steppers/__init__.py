"""Stepper registries (reference: src/steppers/__init__.py:6-12)."""
from .parallel_stepper import EnvStepper, EpisodeStepper, ParallelStepper

REGISTRY = {"episode": EpisodeStepper, "parallel": ParallelStepper}
SELF_REGISTRY = {}

__all__ = ["EnvStepper", "EpisodeStepper", "ParallelStepper", "REGISTRY", "SELF_REGISTRY"]
