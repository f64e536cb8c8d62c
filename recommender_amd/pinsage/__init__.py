"""PinSage on the engine (reference pinsage/train/).

Surfaces kept from the reference: PinSageModel(full_graph, itype, num_layers, embedding_size,
conv_hidden_size, conv_output_size) with call(pos_graph, neg_graph, blocks) / get_repr(blocks)
(pinsage/train/model.py:8-39); Convolve, SageNet, FeatureProjector (pinsage/train/layers.py);
PinSageSampler / item2item_batch_sampler (pinsage/train/data_loader.py); margin_loss
(pinsage/train/train.py:17-20). DGL objects are replaced by the engine's device-resident
HeteroGraph / Block / PairGraph (CSR + NID arrays)."""
from .graph import NID, Block, HeteroGraph, PairGraph
from .layers import Convolve, FeatureProjector, SageNet
from .model import PinSageModel, margin_loss
from .sampler import PinSageSampler, item2item_batch_sampler

__all__ = ["NID", "Block", "HeteroGraph", "PairGraph", "Convolve", "FeatureProjector", "SageNet",
           "PinSageModel", "margin_loss", "PinSageSampler", "item2item_batch_sampler"]
