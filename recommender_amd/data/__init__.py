"""Data paths either side of the hot path: Criteo TSV → device id batches."""
from .criteo import CriteoVocab, read_criteo_tsv

__all__ = ["CriteoVocab", "read_criteo_tsv"]
