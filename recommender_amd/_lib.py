"""ctypes binding of librecsys_hip.so (include/recsys_hip.h).

This is the only place Python touches the C-ABI. There is no CPU fallback: if the library is
missing, or no gfx950 device is visible when a kernel is called, the call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "_lib" / "librecsys_hip.so"
HEADER = _PKG.parent / "include" / "recsys_hip.h"

RS_ID_I32 = 0
RS_ID_I64 = 1
RS_OPT_SGD = 0
RS_OPT_LAZY_ADAM = 1
RS_OPT_KERAS_ADAM = 2
RS_DEDUP_TILE = 32
RS_ERRBIT_OOB = 1
RS_ERRBIT_FORMAT = 2
RS_ERRBIT_RANGE = 4
RS_DIEN_SKIP_MASKED_ROWS = 1


class AdamParams(C.Structure):
    _fields_ = [("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float),
                ("one_minus_beta1", C.c_float), ("one_minus_beta2", C.c_float),
                ("epsilon", C.c_float)]


class DlrmTailArgs(C.Structure):
    """include/recsys_hip.h rs_dlrm_tail_args."""
    _fields_ = [("top_k", C.c_void_p * 3), ("top_b", C.c_void_p * 3), ("top_rows", C.c_void_p),
                ("top_inv", C.c_void_p), ("top_n_full0", C.c_int32), ("top_n0", C.c_int32),
                ("top_n1", C.c_int32), ("top_n2", C.c_int32), ("top_A", C.c_void_p),
                ("top_s", C.c_void_p), ("top_dk", C.c_void_p * 3), ("top_db", C.c_void_p * 3),
                ("top_q", C.c_void_p), ("top_c", C.c_void_p), ("bot_k", C.c_void_p * 3),
                ("bot_b", C.c_void_p * 3), ("bot_n0", C.c_int32), ("bot_n1", C.c_int32),
                ("bot_n2", C.c_int32), ("bot_n3", C.c_int32), ("bot_P", C.c_void_p),
                ("bot_comp2", C.c_void_p), ("bot_dk2", C.c_void_p), ("bot_dk3", C.c_void_p),
                ("bot_P2", C.c_void_p), ("bot_P1", C.c_void_p), ("bot_comp2_next", C.c_void_p),
                ("bot_comp3_next", C.c_void_p), ("lr", C.c_float)]


_p, _i32, _i64, _sz = C.c_void_p, C.c_int32, C.c_int64, C.c_size_t
_u32, _u64 = C.c_uint32, C.c_uint64
_SIGS = {
    "rs_last_error": (C.c_char_p, []),
    "rs_build_id": (C.c_char_p, []),
    "rs_version": (_i32, []),
    "rs_device_count": (_i32, []),
    "rs_stream_copy": (_i32, [_p, _p, _sz, _p]),
    "rs_event_create": (_p, []),
    "rs_event_destroy": (_i32, [_p]),
    "rs_event_record": (_i32, [_p, _p]),
    "rs_stream_wait_event": (_i32, [_p, _p]),
    "rs_embedding_fwd": (_i32, [_p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p, _p, _p]),
    "rs_embedding_fwd_strided": (_i32, [_p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p, _i64, _p, _p]),
    "rs_sort_ids_workspace_size": (_sz, [_i64]),
    "rs_sort_ids": (_i32, [_p, _i32, _i64, _p, _i32, _i64, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_sort_ids_masked": (_i32, [_p, _i32, _i64, _p, _p, _i32, _i64, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_sort_ids_runs": (_i32, [_p, _i64, _i32, _i64, _p, _p, _p, _p]),
    "rs_sort_ids_slots": (_i32, [_p, _i32, _i64, _p, _p, _i32, _i64, _i64, _p, _p, _p, _p, _p, _sz,
                                 _p]),
    "rs_sort_ids_sharded": (_i32, [_p, _i32, _i64, _p, _i32, _i64, _i32, _p, _p, _p, _p, _p, _sz,
                                   _p]),
    "rs_unique_inverse": (_i32, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_dedup_workspace_size": (_sz, [_i64, _i32]),
    "rs_embedding_grad_dense_small_workspace_size": (_sz, [_i64, _i64, _i32]),
    "rs_keras_adam_flat": (_i32, [_p, _p, _p, _p, _i64, _p, _p, C.POINTER(AdamParams), _p]),
    "rs_embedding_grad_dense_small": (_i32, [_p, _i32, _i64, _p, _i32, _i64, _p, _p, _p, _sz, _p]),
    "rs_embedding_dedup_grad": (_i32, [_p, _p, _i64, _p, _i32, _i64, _p, _p, _p, _sz, _p]),
    "rs_embedding_dedup_grad_scaled": (_i32, [_p, _p, _i64, _p, _p, _i32, _i32, _i64, _p, _p, _p,
                                              _sz, _p]),
    "rs_embedding_dedup_grad_mapped": (_i32, [_p, _p, _i64, _p, _p, _i32, _i32, _i64, _p, _p,
                                              _p, _p, _sz, _p]),
    "rs_embedding_dedup_grad_mapped_range": (_i32, [_p, _p, _i64, _p, _p, _i32, _i32, _i64, _u32,
                                                    _u32, _i32, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_unique_inverse_workspace_size": (_sz, [_i64]),
    "rs_exchange_pack": (_i32, [_p, _p, _p, _i32, _i64, _i64, _p, _i64, _p, _p, _p, _p, _p]),
    "rs_exchange_excess": (_i32, [_p, _i32, _i64, _p, _p]),
    "rs_exchange_pack_spill": (_i32, [_p, _p, _p, _i32, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p,
                                      _p]),
    "rs_gather_rows_padded": (_i32, [_p, _i64, _i32, _p, _i64, _p, _p]),
    "rs_exchange_mark": (_i32, [_p, _i64, _p, _i64, _i32, _p]),
    "rs_exchange_classify": (_i32, [_p, _i32, _i64, _p, _i64, _i32, _p, _p, _p, _p]),
    "rs_exchange_scatter_late": (_i32, [_p, _p, _i32, _i64, _i64, _i32, _p, _p]),
    "rs_embedding_grad_dense": (_i32, [_p, _p, _i64, _p, _i32, _i64, _p, _p, _sz, _p]),
    "rs_embedding_grad_dense_segs": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _i32, _i64, _p, _p,
                                            _sz, _p]),
    "rs_apply_workspace_size": (_sz, [_i64, _i32]),
    "rs_embedding_apply": (_i32, [_i32, _p, _p, _p, _i64, _i32, _p, _p, _i64, _p,
                                  C.POINTER(AdamParams), _p, _p, _sz, _p]),
    "rs_embedding_apply_scaled": (_i32, [_i32, _p, _p, _p, _i64, _i32, _p, _p, _i64, _p, _p,
                                         _i32, C.POINTER(AdamParams), _p, _p, _sz, _p]),
    "rs_keras_adam_dense_sweep": (_i32, [_p, _p, _p, _i64, _i32, C.POINTER(AdamParams), _p, _p]),
    "rs_keras_adam_catchup": (_i32, [_p, _p, _p, _p, _i64, _i32, _p, _i64, _p, _i32,
                                     C.POINTER(AdamParams), _p]),
    "rs_keras_adam_materialize": (_i32, [_p, _p, _p, _p, _i64, _i32, _p, _i32,
                                         C.POINTER(AdamParams), _p]),
    "rs_dot_interaction_fwd": (_i32, [_p, _i64, _i32, _i32, _i32, _i32, _p, _i64, _p]),
    "rs_dot_interaction_bwd": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _i32, _i64, _p, _p]),
    "rs_dlrm_interaction_fwd": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64, _i32, _p,
                                       _i64, _p, _p]),
    "rs_dlrm_interaction_bwd": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64, _i32, _p,
                                       _i64, _p, _p, _p]),
    "rs_fm_fwd": (_i32, [_p, _i64, _i32, _i32, _p, _p]),
    "rs_fm_bwd": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p]),
    "rs_bce_workspace_size": (_sz, [_i64]),
    "rs_bce_fwd": (_i32, [_p, _p, _i64, C.c_float, _i32, _p, _p, _sz, _p]),
    "rs_bce_bwd": (_i32, [_p, _p, _i64, C.c_float, _i32, _p, _p, _p]),
    "rs_gru_fwd": (_i32, [_p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_gru_bwd": (_i32, [_p, _p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _i32, _p]),
    "rs_augru_fwd": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _p, _i32, _p]),
    "rs_augru_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _i32, _p]),
    "rs_dien_attention_fwd": (_i32, [_p, _p, _p, _i64, _i32, _i32, _p, _p]),
    "rs_dien_attention_bwd": (_i32, [_p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_dien_aux_workspace_size": (_sz, [_i64, _i32, _i32, _i32]),
    "rs_valid_rows_workspace_size": (_sz, [_i64]),
    "rs_valid_rows": (_i32, [_p, _i64, _p, _p, _p, _sz, _p]),
    "rs_masked_proj": (_i32, [_p, _i64, _p, _p, _p, _p, _i64, _i32, _i32, _p, _i64, _p]),
    "rs_masked_dx": (_i32, [_p, _i64, _p, _p, _p, _p, _i64, _i32, _i32, _p, _i64, _p]),
    "rs_gemm_x3_workspace_size": (_sz, [_i64, _i64, _i32, _i32]),
    "rs_gemm_x3": (_i32, [_i32, _i32, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _p, _i64,
                          _i64, _i32, _p, _i64, _i32, _i32, _p, _sz, _p]),
    "rs_masked_dx_acc": (_i32, [_p, _i64, _p, _p, _p, _p, _i64, _i32, _i32, _p, _i64, _p, _i64,
                                _p]),
    "rs_masked_wgrad_workspace_size": (_sz, [_i32, _i32]),
    "rs_masked_wgrad": (_i32, [_p, _i64, _i32, _p, _i64, _p, _p, _i32, _i32, _p, _p, _p, _sz, _p]),
    "rs_dien_aux_fwd": (_i32, [_p, _p, _p, _p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                               _p, _p]),
    "rs_dien_aux_bwd": (_i32, [_p, _p, _p, _p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                               _p, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_dien_aux_bwd_acc": (_i32, [_p, _p, _p, _p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                                   _p, _p, _i32, _p, _p, _p, _p, _sz, _p]),
    "rs_act_bwd_colsum_workspace_size": (_sz, [_i64, _i32]),
    "rs_batch_norm_workspace_size": (_sz, [_i64, _i32]),
    "rs_batch_norm_fwd": (_i32, [_p, _i64, _i32, _p, _p, C.c_float, C.c_float, _i32, _p, _p,
                                 _p, _p, _p, _p, _sz, _p]),
    "rs_batch_norm_bwd": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _i32, _p, _p, _p, _p, _sz, _p]),
    "rs_act_bwd_colsum": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p, _p, _sz, _p]),
    "rs_act_bwd_colsum_groups": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _p, _p, _p, _sz, _p]),
    "rs_act_bwd_colsum_ld": (_i32, [_p, _i64, _p, _i64, _i64, _i32, _i32, _p, _i64, _p, _p,
                                    _sz, _p]),
    "rs_philox4x32_10": (_i32, [_p, _i64, _u32, _u32, _p, _p]),
    "rs_metapath_walk": (_i32, [_p, _p, _p, _p, _p, _i64, _i32, _i32, C.c_float, _u64, _u32,
                                _u32, _p, _p]),
    "rs_item_pairs_workspace_size": (_sz, [_i32]),
    "rs_item_pairs": (_i32, [_p, _p, _p, _p, _i32, _i64, _i32, _u64, _u32, _p, _p, _p, _p, _p,
                             _sz, _p]),
    "rs_item_pairs_at": (_i32, [_p, _p, _p, _p, _i32, _i64, _i32, _u64, _p, _p, _p, _p, _p, _p,
                                _sz, _p]),
    "rs_pinsage_neighbors_at": (_i32, [_p, _p, _p, _p, _p, _i64, _i32, _i32, C.c_float, _u64, _p,
                                       _u32, _i32, _p, _i64, _p, _p, _p]),
    "rs_pair_set_build": (_i32, [_p, _p, _i64, _p, _i64, _p]),
    "rs_pinsage_neighbors": (_i32, [_p, _p, _p, _p, _p, _i64, _i32, _i32, C.c_float, _u64, _u32,
                                    _u32, _i32, _p, _i64, _p, _p, _p]),
    "rs_unique_first_workspace_size": (_sz, [_i64, _i64]),
    "rs_unique_first": (_i32, [_p, _i64, _i64, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_pinsage_block_workspace_size": (_sz, [_i64, _i32]),
    "rs_pinsage_block": (_i32, [_p, _p, _i64, _i32, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _sz,
                                _p]),
    "rs_weighted_mean_agg_fwd": (_i32, [_p, _i64, _i32, _p, _p, _p, _i64, _p, _p, _p]),
    "rs_weighted_mean_agg_bwd": (_i32, [_p, _i32, _p, _p, _p, _p, _p, _i64, _p, _p]),
    "rs_frobenius_workspace_size": (_sz, [_i64]),
    "rs_frobenius_normalize_fwd": (_i32, [_p, _i64, _p, _p, _p, _sz, _p]),
    "rs_frobenius_normalize_bwd": (_i32, [_p, _p, _p, _i64, _p, _p, _sz, _p]),
    "rs_frobenius_normalize_rows_fwd": (_i32, [_p, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "rs_frobenius_normalize_rows_bwd": (_i32, [_p, _p, _p, _i64, _i32, _p, _p, _p, _sz, _p]),
    "rs_match_logits_fwd": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _i64, _p, _p, _p]),
    "rs_match_logits_bwd": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64, _p, _p, _p]),
    "rs_side_pool_fwd_strided": (_i32, [_p, _i64, _i64, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_side_pool_bwd_strided": (_i32, [_p, _i64, _i64, _p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_pair_margin_workspace_size": (_sz, [_i64]),
    "rs_multihot_mean_fwd": (_i32, [_p, _i32, _i32, _p, _i32, _i64, _p, _i64, _p, _p, _p]),
    "rs_multihot_mean_bwd_workspace_size": (_sz, [_i64, _i32, _i32]),
    "rs_multihot_mean_bwd": (_i32, [_p, _i32, _i64, _p, _i64, _p, _i32, _i32, _p, _p, _p, _sz,
                                    _p]),
    "rs_index_add_rows_workspace_size": (_sz, [_i64, _i32]),
    "rs_index_add_rows": (_i32, [_p, _i32, _i64, _p, _p, _i32, _i64, _p, _p, _p, _sz, _p]),
    "rs_pair_margin_fwd": (_i32, [_p, _i64, _i32, _i64, _p, _p, _p, _p, _i64, C.c_float, _p, _p,
                                  _p, _p, _p, _p, _p, _sz, _p]),
    "rs_pair_margin_bwd_workspace_size": (_sz, [_i64, _i32]),
    "rs_pair_margin_bwd": (_i32, [_p, _i64, _i32, _i64, _p, _p, _p, _p, _i64, C.c_float, _p, _p,
                                  _p, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_side_pool_fwd_multi": (_i32, [_p, _i64, _i64, _i64, _i32, _i32, _i32, _p, _i64, _p, _p,
                                      _p, _p]),
    "rs_side_pool_bwd_multi": (_i32, [_p, _i64, _i64, _i64, _i32, _i32, _i32, _p, _p, _p, _p,
                                      _i64, _p]),
    "rs_side_pool_fwd": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_side_pool_bwd": (_i32, [_p, _p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_auc_update": (_i32, [_p, _p, _i64, _p, _i32, _p, _p, _p]),
    "rs_line_index_workspace_size": (_sz, [_i64]),
    "rs_line_index": (_i32, [_p, _i64, _p, _p, _p, _sz, _p]),
    "rs_criteo_parse": (_i32, [_p, _i64, _p, _i64, _i32, _i32, _p, _p, _p, _p, _p]),
    "rs_crc32c_masked": (_i32, [_p, _i64, _p]),
    "rs_dlrm_train_workspace_size": (_sz, [_i64]),
    "rs_keras_adam_mark": (_i32, [_p, _i64, _p, _i64, _i32, _p]),
    "rs_dlrm_dense_tail_workspace_size": (_sz, [_i32, _i32, _i32]),
    "rs_dlrm_dense_tail": (_i32, [C.POINTER(DlrmTailArgs), _p, _sz, _p]),
    "rs_dlrm_train_step_fwd_unit": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _p, _i32, _p,
                                           _i64, _p, _p, C.c_float, C.c_float, _p, _p, _p, _p, _p,
                                           _sz, _p, _p]),
    "rs_dlrm_train_step_fwd_unit_nofold": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _p, _i32,
                                                  _p, _i64, _p, _p, C.c_float, C.c_float, _p, _p,
                                                  _p, _p, _sz, _p, _p]),
    "rs_dlrm_train_fold": (_i32, [_p, _sz, _i64, _i32, _i32, _p, _p]),
    "rs_tfrecord_index": (_i32, [_p, _i64, _i32, _p, _p, _i64, _p]),
    "rs_tfrecord_parse_criteo": (_i32, [_p, _p, _p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p]),
    "rs_vocab_count": (_i32, [_p, _i64, _i64, _p, _p, _p, _i64, _p, _p]),
    "rs_vocab_collect_workspace_size": (_sz, [_i64]),
    "rs_vocab_collect": (_i32, [_p, _p, _p, _i64, _u32, _p, _p, _p, _p, _sz, _p]),
    "rs_vocab_assign": (_i32, [_p, _i64, _p, _p]),
    "rs_vocab_lookup": (_i32, [_p, _i64, _p, _p, _i64, _p, _p]),
    "rs_latest_item": (_i32, [_p, _p, _p, _i64, _p, _p, _p]),
    "rs_masked_topk": (_i32, [_p, _i64, _i32, _i32, _i64, _p, _p, _i32, _p, _p, _p]),
    "rs_hit_flags": (_i32, [_p, _i64, _i32, _i64, _p, _p, _p, _p]),
    "rs_csr_weight_prefix": (_i32, [_p, _p, _i64, _p, _p]),
    "rs_eges_walks": (_i32, [_p, _p, _p, _i32, _i64, _i32, _i32, _u64, _u32, _p, _p]),
    "rs_skipgram_workspace_size": (_sz, [_i32, _i32, _i32]),
    "rs_skipgram_pairs": (_i32, [_p, _i32, _i32, _i32, _p, _p, _p, _p, _sz, _p]),
    "rs_log_uniform_sample": (_i32, [_p, _i32, _i64, _i32, _i32, _u64, _u32, _p, _p, _p]),
    "rs_dlrm_interaction_bwd_rank1": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64, _p, _p,
                                             _i64, _p, _p, _p]),
    "rs_dlrm_interaction_fwd_head": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64, _p,
                                            _i64, _p, _p, _i32, _p, _p, _p]),
    "rs_dlrm_interaction_fwd_head_dx": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p, _p, _i64,
                                               _p, _i64, _p, _p, _i32, _p, _p, _p, _p, _p]),
    "rs_chain3_vec_compose": (_i32, [_p, _p, _i32, _p, _p, _p, _p, _p, _i32, _i32, _p, _p, _p,
                                     _sz, _p]),
    "rs_chain_aug_product": (_i32, [_p, _i32, _i32, _p, _p, _i32, _i32, _p, _p, _p]),
    "rs_affine_narrow_fwd": (_i32, [_p, _i64, _i64, _i32, _p, _i32, _i32, _p, _i64, _p]),
    "rs_rowdot_act": (_i32, [_p, _i64, _i64, _i32, _p, _p, _i32, _p, _p]),
    "rs_chain_rt_product": (_i32, [_p, _i32, _p, _i32, _i32, _p, _p]),
    "rs_chain_outer": (_i32, [_p, _i32, _i32, _p, _i32, _p, _i32, _p, _p]),
    "rs_chain_reduce_workspace_size": (_sz, [_i64, _i32, _i32]),
    "rs_chain_reduce": (_i32, [_p, _i64, _i32, _p, _p, _i32, _i32, _i64, _p, _p, _p, _sz, _p]),
    "rs_chain3_vec_grads": (_i32, [_p, _p, _p, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p, _p,
                                   _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "rs_sparse_workspace_size": (_sz, [_i64, _i32]),
    "rs_embedding_bwd_dedup": (_i32, [_p, _i32, _i64, _p, _i32, _i64, _p, _i32, _p, _p, _p, _p, _p,
                                      _sz, _p]),
    "rs_apply_sgd": (_i32, [_p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p, C.c_float, _p, _p, _sz,
                            _p]),
    "rs_apply_lazy_adam": (_i32, [_p, _p, _p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p,
                                  C.POINTER(AdamParams), _p, _p, _sz, _p]),
    "rs_apply_keras_dense_adam": (_i32, [_p, _p, _p, _i64, _i32, _p, _i32, _i64, _p, _i32, _p,
                                         C.POINTER(AdamParams), _p, _p, _p, _sz, _p]),
    "rs_vocab_count_masked": (_i32, [_p, _p, _i64, _i64, _p, _p, _p, _i64, _p, _p]),
    "rs_kv_parse": (_i32, [_p, _i64, _p, _i64, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _p, _p,
                           _p, _p]),
    "rs_map_insert": (_i32, [_p, _i64, _p, _p, _i64, _p, _p]),
    "rs_aliccp_join_workspace_size": (_sz, [_i64]),
    "rs_aliccp_join": (_i32, [_p, _i64, _i32, _p, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _p,
                              _p, _p, _p, _sz, _p]),
    "rs_vocab_regroup": (_i32, [_p, _i64, _i32, _i64, _p, _p, _p]),
    "rs_vocab_assign_grouped": (_i32, [_p, _p, _p, _i64, _i32, _p, _p]),
    "rs_vocab_lookup_i32": (_i32, [_p, _i64, _p, _p, _i64, _i32, _i32, _p, _p, _p]),
    "rs_dien_parse": (_i32, [_p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "rs_dien_item_cat_workspace_size": (_sz, [_i64]),
    "rs_dien_item_cat": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p, _p, _i64, _p, _p, _i64, _p, _p,
                                _sz, _p]),
    "rs_dien_encode": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p, _p, _i64, _i32, _p, _p, _i64,
                              _i32, _p, _i32, _u64, _i64, _p, _p, _p, _p, _p, _p, _p, _p]),
}

_lib = None


class RecsysError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Every rs_* function declared in include/recsys_hip.h."""
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rs_\w+)\s*\(", text, re.M)))


def load(path: str | os.PathLike | None = None):
    """Load the library (no GPU needed). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    # RS_LIB: A/B runs of a variant build (recommender_amd/build.py --variant)
    p = Path(path) if path else Path(os.environ.get("RS_LIB", LIB_PATH))
    if not p.exists():
        raise RecsysError(f"{p} not built: run `python -m recommender_amd.build` "
                          "(or __graft_entry__.build())")
    lib = C.CDLL(str(p))
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    check_build_id(lib, p)
    _lib = lib
    return lib


def check_build_id(lib, path) -> None:
    """Refuse a library built from other sources than the csrc/ + include/ next to it (the .so
    travels prebuilt, untracked: without this a GPU box could test a stale build of a changed
    kernel with no signal). Skipped when the sources are absent (a library shipped alone)."""
    from .build import CSRC, source_hash

    if not CSRC.is_dir() or os.environ.get("RS_SKIP_BUILD_ID") == "1":
        return
    built, want = lib.rs_build_id().decode(), source_hash()
    if built != want:
        raise RecsysError(f"{path} was built from other sources (build id {built}, sources "
                          f"{want}): rebuild with `python -m recommender_amd.build`")


def lib():
    return _lib if _lib is not None else load()


def check(status: int, fn: str):
    if status != 0:
        msg = lib().rs_last_error().decode(errors="replace")
        raise RecsysError(f"{fn} failed with status {status}: {msg}")


class KernelTimer:
    """Records HIP events around the C-ABI calls named in `names` (on the current stream, the
    stream every kernel is launched on) while enabled; bench.py uses it for per-kernel time."""

    def __init__(self, names):
        self.names = set(names)
        self.events: dict[str, list] = {n: [] for n in self.names}
        self.enabled = False

    def totals_ms(self):
        """{name: (total ms, launches)} over the recorded (eagerly launched) calls."""
        torch.cuda.synchronize()
        return {n: (sum(s.elapsed_time(e) for s, e in ev), len(ev)) for n, ev in self.events.items()}


_timer: KernelTimer | None = None


def set_timer(t: KernelTimer | None):
    global _timer
    _timer = t


def call(fn: str, *args):
    """Invoke a kernel entry point; raises on a non-zero status."""
    f = getattr(lib(), fn)
    t = _timer
    # no events while a stream is being captured: a graph replay does not re-record them, so
    # their elapsed_time would be read off events that never completed (hipErrorInvalidHandle)
    if (t is not None and t.enabled and fn in t.names
            and not torch.cuda.is_current_stream_capturing()):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        st = f(*args)
        e.record()
        t.events[fn].append((s, e))
        check(st, fn)
        return
    check(f(*args), fn)


def require_device(t: torch.Tensor, name: str = "tensor"):
    if not t.is_cuda:
        raise RecsysError(f"{name} must be a GPU tensor (librecsys_hip has no CPU path)")


def ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# Stream ordering with device-scope events (rs_event_*): on by default, RS_DEVICE_EVENTS=0 uses
# torch's default events (a system-scope release at every record) everywhere.
DEVICE_EVENTS = os.environ.get("RS_DEVICE_EVENTS", "1") == "1"


class DeviceEvent:
    """A HIP event whose record is a device-scope release (rs_event_create): it orders the
    engine's own streams of one device without the system-scope cache write-back of a default
    event. Never used for host synchronisation, other devices or other processes. Re-recording
    is allowed once the waits on the previous record are enqueued (a wait binds the record that
    precedes it; on an in-order stream a later record only orders more work)."""
    __slots__ = ("h",)

    def __init__(self):
        h = lib().rs_event_create()
        if not h:
            raise RecsysError(f"rs_event_create: {lib().rs_last_error().decode()}")
        self.h = h

    def record(self, stream):
        call("rs_event_record", C.c_void_p(self.h), C.c_void_p(stream.cuda_stream))

    def wait_by(self, stream):
        call("rs_stream_wait_event", C.c_void_p(stream.cuda_stream), C.c_void_p(self.h))

    def __del__(self):
        try:
            lib().rs_event_destroy(C.c_void_p(self.h))
        except Exception:  # interpreter teardown
            pass


def stream_wait_event(stream, ev):
    """`stream` waits for the record of `ev` (a DeviceEvent or a torch.cuda.Event)."""
    if isinstance(ev, DeviceEvent):
        ev.wait_by(stream)
    else:
        stream.wait_event(ev)


def record_event(stream, ev=None):
    """An event recorded on `stream` now: a DeviceEvent (reused when given) unless device events
    are off or a graph is being captured, else a torch event."""
    if not DEVICE_EVENTS or torch.cuda.is_current_stream_capturing():
        e = torch.cuda.Event()
        e.record(stream)
        return e
    e = ev if isinstance(ev, DeviceEvent) else DeviceEvent()
    e.record(stream)
    return e


def stream_wait_stream(waiter, src, ev=None):
    """`waiter` waits for everything queued on `src` so far (torch's wait_stream, device-scope
    unless device events are off or a graph is being captured); ev: a DeviceEvent to reuse."""
    if waiter == src:
        return
    if not DEVICE_EVENTS or torch.cuda.is_current_stream_capturing():
        waiter.wait_stream(src)
        return
    e = ev if ev is not None else DeviceEvent()
    e.record(src)
    e.wait_by(waiter)


def id_dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.int64:
        return RS_ID_I64
    if t.dtype == torch.int32:
        return RS_ID_I32
    raise RecsysError(f"ids must be int32 or int64, got {t.dtype}")
