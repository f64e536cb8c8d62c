"""recommender_amd — MI355X-native (gfx950) sparse-embedding and feature-interaction engine.

Hot path in hand-written HIP behind the C-ABI of include/recsys_hip.h (librecsys_hip.so);
host side mirrors the reference's Keras layer/model call surfaces (neoyinyao/Recommender).
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
