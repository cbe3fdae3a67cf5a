"""Learner registry (reference: src/marl/learners/__init__.py:5-9; COMA/SFS are out of scope)."""
from .q_learner import Learner, QLearner

REGISTRY = {"q": QLearner}

__all__ = ["Learner", "QLearner", "REGISTRY"]
