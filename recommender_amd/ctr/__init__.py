"""ctr sub-repo surface: DLRM and DeepFM (reference ctr/layers.py, ctr/model.py, ctr/util.py)."""
from .layers import MLP, DotInteraction
from .model import DLRM, DeepFM

__all__ = ["MLP", "DotInteraction", "DLRM", "DeepFM"]
