"""maleague -- MI355X-native (gfx950) rebuild of the PMatthaei/ma-league QMIX hot path.

The package mirrors the reference's plugin registries (steppers, controllers, agents, learners,
mixers, env) so YAML configs select the same keys; every hot-path op runs in libmaleague.so
(hand-written HIP kernels, C ABI in include/maleague.h). See DESIGN.md.
"""
__version__ = "0.1.0"

from . import ops  # noqa: E402,F401  (registers torch.ops.maleague.*)
