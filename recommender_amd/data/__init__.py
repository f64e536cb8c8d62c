"""Data paths either side of the hot path: Criteo TSV and TFRecord, Ali-CCP CSV and
Amazon (DIEN) text → device-resident id batches."""
from .aliccp import ALICCP_COLUMNS, AliCCPVocab, aliccp_join, click_rows, subsample_impressions
from .amazon import DienVocab, read_dien_text
from .criteo import CriteoVocab, read_criteo_tsv
from .tfrecord import encode_tsv, read_tfrecord, write_tfrecord

__all__ = ["ALICCP_COLUMNS", "AliCCPVocab", "CriteoVocab", "DienVocab", "aliccp_join",
           "click_rows", "encode_tsv", "read_criteo_tsv", "read_dien_text", "read_tfrecord",
           "subsample_impressions", "write_tfrecord"]
