"""MAC registry (reference: src/marl/controllers/__init__.py:6-11; only the QMIX-path "basic" MAC is built)."""
from .basic_controller import BasicMAC, MultiAgentController

REGISTRY = {"basic": BasicMAC}

__all__ = ["BasicMAC", "MultiAgentController", "REGISTRY"]
