"""Learner registry (reference: src/marl/learners/__init__.py:5-9; COMA/SFS are out of scope; "refil" =
REFILLearner, unregistered in the reference)."""
from .q_learner import Learner, QLearner
from .refil_learner import REFILLearner

REGISTRY = {"q": QLearner, "refil": REFILLearner}

__all__ = ["Learner", "QLearner", "REFILLearner", "REGISTRY"]
