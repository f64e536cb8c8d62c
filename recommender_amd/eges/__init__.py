"""EGES / GES / DeepWalk(BGE) surfaces (reference eges/model.py)."""
from .model import EGES, GES, Base, DeepWalk

__all__ = ["Base", "DeepWalk", "GES", "EGES"]
