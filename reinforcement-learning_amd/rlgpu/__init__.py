"""rlgpu -- MI355X-native rollout engine for the GigaLearnCPP / RLGymCPP hot path.

Python mirror of the reference's operator surface over the C ABI in include/*.h.
"""
from ._lib import RLGPUError, LIB_PATH  # noqa: F401
from .gae import GAE  # noqa: F401
