"""Agent registry (reference: src/marl/modules/agents/__init__.py:5-8; the REFIL agents, unregistered in the
reference, are registered under their REFIL names)."""
from .drqn_agent import AgentNetwork, DRQNAgentNetwork
from .entity_agent import EntityAttentionRNNAgent, ImagineEntityAttentionRNNAgent

REGISTRY = {"rnn": DRQNAgentNetwork, "entity_attend_rnn": EntityAttentionRNNAgent,
            "imagine_entity_attend_rnn": ImagineEntityAttentionRNNAgent}

__all__ = ["AgentNetwork", "DRQNAgentNetwork", "EntityAttentionRNNAgent", "ImagineEntityAttentionRNNAgent",
           "REGISTRY"]
