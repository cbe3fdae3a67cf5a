from .qmix import QMixer
from .vdn import VDNMixer

__all__ = ["QMixer", "VDNMixer"]
