"""dien sub-repo surface: BaseModel, DIN, DIEN (reference dien/layers.py, dien/model.py)."""
from .model import DIEN, DIN, BaseModel

__all__ = ["BaseModel", "DIN", "DIEN"]
