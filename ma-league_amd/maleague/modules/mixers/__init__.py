from .flex_qmix import AttentionHyperNet, FlexQMixer
from .qmix import QMixer
from .vdn import VDNMixer

__all__ = ["AttentionHyperNet", "FlexQMixer", "QMixer", "VDNMixer"]
