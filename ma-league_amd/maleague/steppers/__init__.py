"""Stepper registries (reference: src/steppers/__init__.py:6-12). With ``entity_scheme`` (REFIL, config 5) the
same keys resolve to the entity-env steppers (see build_stepper)."""
from .entity_stepper import EntityEpisodeStepper, EntityParallelStepper
from .parallel_stepper import EnvStepper, EpisodeStepper, ParallelStepper
from .self_play_stepper import SelfPlayParallelStepper, SelfPlayStepper

REGISTRY = {"episode": EpisodeStepper, "parallel": ParallelStepper}
SELF_REGISTRY = {"episode": SelfPlayStepper, "parallel": SelfPlayParallelStepper}
ENTITY_REGISTRY = {"episode": EntityEpisodeStepper, "parallel": EntityParallelStepper}


def build_stepper(args, logger, log_start_t=0):
    reg = ENTITY_REGISTRY if getattr(args, "entity_scheme", False) else REGISTRY
    return reg[args.runner](args=args, logger=logger, log_start_t=log_start_t)


__all__ = ["EnvStepper", "EpisodeStepper", "ParallelStepper", "SelfPlayParallelStepper", "SelfPlayStepper",
           "EntityParallelStepper", "EntityEpisodeStepper", "REGISTRY", "SELF_REGISTRY", "ENTITY_REGISTRY",
           "build_stepper"]
