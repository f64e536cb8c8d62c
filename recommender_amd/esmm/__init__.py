"""esmm sub-repo surface: BaseModel, ESMM, MMOE over per-feature tables (reference
esmm/layers.py, esmm/base.py, esmm/esmm.py, esmm/mmoe.py)."""
from .base import BaseModel
from .esmm import ESMM
from .layers import MLP
from .mmoe import MMOE

FEAT_VOCAB = {  # esmm/train.py:197-215 (Ali-CCP per-feature vocabularies, ids 1..n, OOV 0)
    "101": 238635, "121": 98, "122": 14, "124": 3, "125": 8, "126": 4, "127": 4, "128": 3,
    "129": 5, "205": 467298, "206": 6929, "207": 263942, "216": 106399, "508": 5888,
    "509": 104830, "702": 51878, "853": 37148, "301": 4,
}

__all__ = ["BaseModel", "ESMM", "MMOE", "MLP", "FEAT_VOCAB"]
