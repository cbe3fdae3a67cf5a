"""Agent registry (reference: src/marl/modules/agents/__init__.py:5-8)."""
from .drqn_agent import AgentNetwork, DRQNAgentNetwork

REGISTRY = {"rnn": DRQNAgentNetwork}

__all__ = ["AgentNetwork", "DRQNAgentNetwork", "REGISTRY"]
