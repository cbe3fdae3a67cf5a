"""MAC registry (reference: src/marl/controllers/__init__.py:6-11; "entity" = EntityMAC, unregistered in the
reference)."""
from .basic_controller import BasicMAC, MultiAgentController
from .entity_controller import EntityMAC

REGISTRY = {"basic": BasicMAC, "entity": EntityMAC}

__all__ = ["BasicMAC", "EntityMAC", "MultiAgentController", "REGISTRY"]
