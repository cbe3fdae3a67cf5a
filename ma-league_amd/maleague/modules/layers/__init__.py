"""Entity layers (reference: src/marl/modules/layers/attention.py)."""
from .attention import EntityAttentionLayer

__all__ = ["EntityAttentionLayer"]
