"""Device-resident graph structures standing in for the DGL objects of pinsage/train/.

HeteroGraph: the user–item heterograph built by pinsage/train/graph_builder.py:4-99 —
  CSR item→user and user→item (int64 indptr, int32 ids) in HBM, plus item node data
  ('year', 'genre', 'id') as `g.nodes[itype].data[...]` (pinsage/train/layers.py:52-79).
Block:      dgl.to_block output (pinsage/train/data_loader.py:40): src nodes (dst nodes first),
  CSR by dst with edge weights (visit counts, edata['weight']) and the src-major transpose.
PairGraph:  compacted pos/neg pair graph (compact_graphs, data_loader.py:48).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

NID = "_ID"  # dgl.NID


class _NodeView:
    def __init__(self, data: dict):
        self.data = data


class HeteroGraph:
    def __init__(self, users, items, n_users: int, n_items: int, device="cuda",
                 item_data: dict | None = None, utype: str = "user", itype: str = "movie",
                 edge_data: dict | None = None):
        """users/items: the rating edges (numpy or torch int). Builds both CSRs on device.
        edge_data: per-edge columns (e.g. {'timestamp': ...}), kept in u2i CSR order as
        `g.u2i_edata[name]` (the 'watched' etype's edata, graph_builder.py)."""
        dev = torch.device(device)
        u = torch.as_tensor(np.asarray(users), dtype=torch.int64, device=dev)
        i = torch.as_tensor(np.asarray(items), dtype=torch.int64, device=dev)
        self.utype, self.itype = utype, itype
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.n_edges = int(u.numel())
        self.device = dev
        key_u = u * self.n_items + i
        _, o = torch.sort(key_u, stable=True)
        self.u2i = i[o].to(torch.int32).contiguous()
        self.u2i_edata = {k: torch.as_tensor(np.asarray(v), device=dev)[o].contiguous()
                          for k, v in (edge_data or {}).items()}
        self.u2i_indptr = self._indptr(u, self.n_users)
        key_i = i * self.n_users + u
        _, o = torch.sort(key_i, stable=True)
        self.i2u = u[o].to(torch.int32).contiguous()
        self.i2u_indptr = self._indptr(i, self.n_items)
        data = {k: torch.as_tensor(np.asarray(v), device=dev) for k, v in (item_data or {}).items()}
        data.setdefault("id", torch.arange(self.n_items, device=dev))
        self.nodes = {itype: _NodeView(data), utype: _NodeView({})}

    @staticmethod
    def _indptr(keys: torch.Tensor, n: int) -> torch.Tensor:
        counts = torch.bincount(keys, minlength=n)
        ptr = torch.zeros(n + 1, dtype=torch.int64, device=keys.device)
        ptr[1:] = torch.cumsum(counts, 0)
        return ptr

    def number_of_nodes(self, ntype: str | None = None) -> int:
        if ntype == self.utype:
            return self.n_users
        return self.n_items

    def csr_args(self):
        return (self.i2u_indptr, self.i2u, self.u2i_indptr, self.u2i)

    def hbm_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.csr_args())


@dataclass
class Block:
    src_nodes: torch.Tensor   # [n_src] int32 global item ids; the first n_dst are the dst nodes
    n_dst: int
    indptr: torch.Tensor      # [n_dst+1] int32
    edge_src: torch.Tensor    # [cap] int32 local src id per edge (first n_edges valid)
    edge_dst: torch.Tensor    # [cap] int32
    edge_w: torch.Tensor      # [cap] float32 visit count
    n_edges: torch.Tensor     # [1] int32 (device)
    t_indptr: torch.Tensor    # [n_src+1] int32
    t_edge: torch.Tensor      # [cap] int32 edge ids grouped by src
    # capacity-shaped (sync-free) blocks: live dst / src counts [1] int32 on the device; rows
    # past them are padding (src id -1, no edges). None: every row is live.
    n_dst_live: torch.Tensor | None = None
    n_src_live: torch.Tensor | None = None

    @property
    def n_src(self) -> int:
        return int(self.src_nodes.numel())

    def num_dst_nodes(self) -> int:
        return self.n_dst

    def num_src_nodes(self) -> int:
        return self.n_src

    @property
    def srcdata(self):
        return {NID: self.src_nodes}

    @property
    def dstdata(self):
        return {NID: self.src_nodes[: self.n_dst]}


@dataclass
class PairGraph:
    """Edges src → dst in the compacted node space (ndata[NID] = the seed items)."""
    src: torch.Tensor
    dst: torch.Tensor
    nodes: torch.Tensor
    # capacity-shaped pair graphs: valid [E] bool (padding pairs have src/dst -1) and the live
    # count n_valid [1] int32 on the device. None: every edge is live.
    valid: torch.Tensor | None = None
    n_valid: torch.Tensor | None = None

    @property
    def ndata(self):
        return {NID: self.nodes}

    def num_edges(self) -> int:
        return int(self.src.numel())
