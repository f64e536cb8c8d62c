"""dien/model.py surface (reference dien/model.py:7-80): item / category tables with
mask_zero=True (dien/model.py:11-12), flat embeddings item‖cat (:14-19), BASE (masked history
mean), DIN (local activation), DIEN (GRU + aux loss, attention, AUGRU; returns
(prob [B,1], aux [B])).

DIEN's head BatchNormalization mode (`head_bn_mode`, parity unpinned): the reference calls
`self.mlp(embedding)` without `training` (dien/model.py:79) inside a model called with
training=True (dien/train.py:17). TF 2.2's `Layer.__call__` fills an unpassed `training` from the
enclosing call's context [3p], so during a train step the head BN normalises by the batch
statistics and updates its moving averages — "propagate", the default. "inference" is the
literal reading of the line (moving statistics, no update), kept as the alternative; both are
tested against oracle/dien.py."""
from __future__ import annotations

import torch
from torch import nn

from ..embedding import Embedding
from ..functional import embedding_lookup_concat
from .layers import (MLP, DIENAttention, InterestEvolve, InterestExtract, LocalActivationUnit,
                     attention_evolve, compute_his_average)


class BaseModel(nn.Module):
    def __init__(self, item_vocab_size, item_embedding_size, cat_vocab_size, cat_embedding_size,
                 mlp_units, device=None, generator=None):
        super().__init__()
        D = item_embedding_size + cat_embedding_size
        self.embedding_dim = D
        self.mlp = MLP(mlp_units, "sigmoid", 2 * D, device, generator)
        self.item_embedding = Embedding(item_vocab_size, item_embedding_size, mask_zero=True,
                                        device=device, generator=generator)
        self.cat_embedding = Embedding(cat_vocab_size, cat_embedding_size, mask_zero=True,
                                       device=device, generator=generator)

    def compute_flat_embedding(self, inputs, grad_mask=None):
        """grad_mask: the history mask when every consumer skips the masked steps (DIEN), so
        the tables' densified gradients leave those positions out (Embedding grad_mask)."""
        item, cat = inputs
        # one output, each lookup gathering into its column block (no concat pass)
        return embedding_lookup_concat(self.item_embedding, item, self.cat_embedding, cat, grad_mask)

    def compute_prob(self, inputs):
        return self.forward(inputs)

    def forward(self, inputs, training=False, mask=None):
        mask = self.item_embedding.compute_mask(inputs["pos_his_item"])
        target = self.compute_flat_embedding((inputs["target_item"], inputs["target_cat"])).squeeze(1)
        his = self.compute_flat_embedding((inputs["pos_his_item"], inputs["pos_his_cat"]))
        rep = compute_his_average(his, mask)
        return self.mlp(torch.cat([target, rep], -1), training=training)

    call = forward


class DIN(BaseModel):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.local_activation_unit = LocalActivationUnit(self.embedding_dim, kwargs.get("device"),
                                                         kwargs.get("generator"))

    def forward(self, inputs, training=False, mask=None):
        mask = self.item_embedding.compute_mask(inputs["pos_his_item"])
        target = self.compute_flat_embedding((inputs["target_item"], inputs["target_cat"]))
        his = self.compute_flat_embedding((inputs["pos_his_item"], inputs["pos_his_cat"]))
        rep = self.local_activation_unit((target, his), mask=mask)
        return self.mlp(torch.cat([target.squeeze(1), rep], -1), training=training)

    call = forward


class DIEN(BaseModel):
    def __init__(self, interest_extract_gru_units, interest_evolve_gru_units,
                 head_bn_mode="propagate", **kwargs):
        super().__init__(**kwargs)
        if head_bn_mode not in ("propagate", "inference"):
            raise ValueError("head_bn_mode must be 'propagate' or 'inference'")
        self.head_bn_mode = head_bn_mode
        dev, gen = kwargs.get("device"), kwargs.get("generator")
        D = self.embedding_dim
        self.interest_extract_layer = InterestExtract(interest_extract_gru_units, D, dev, gen)
        self.attention = DIENAttention(interest_extract_gru_units, D, dev, gen)
        self.interest_evolve = InterestEvolve(interest_evolve_gru_units, interest_extract_gru_units, dev, gen)
        if interest_evolve_gru_units != D:
            raise ValueError("the MLP input is [target (D), evolved interest]; the reference uses "
                             "36 units with 18+18 embeddings")

    def compute_prob(self, inputs):
        prob, _ = self.forward(inputs)
        return prob

    def forward(self, inputs, training=False, mask=None):
        mask = self.item_embedding.compute_mask(inputs["pos_his_item"])
        # as uint8 once: the lookups' gradient flags and every layer's kernels read this form
        mask = mask.to(torch.uint8)
        target = self.compute_flat_embedding((inputs["target_item"], inputs["target_cat"]))
        # masked history steps carry no gradient: the GRU / AUGRU skip them (their input rows'
        # gradient is written 0), the attention gives them weight exactly 0 and the aux loss
        # reads pos / neg only at steps t + 1 with m = 1
        pos = self.compute_flat_embedding((inputs["pos_his_item"], inputs["pos_his_cat"]), mask)
        neg = self.compute_flat_embedding((inputs["neg_his_item"], inputs["neg_his_cat"]), mask)
        hidden, aux = self.interest_extract_layer((pos, neg), training, mask)
        # attention then AUGRU as one node (the attention's hidden gradient summed in-kernel)
        rep = attention_evolve(self.attention, self.interest_evolve, target, hidden, mask)
        # dien/model.py:79 passes no `training`: TF 2.2 propagates the call's (head_bn_mode)
        bn_training = bool(training) and self.head_bn_mode == "propagate"
        prob = self.mlp(torch.cat([target.squeeze(1), rep], -1), training=bn_training)
        return prob, aux

    call = forward
