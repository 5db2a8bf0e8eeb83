"""The pooling-operator nets of the reference's kernel/ benchmark on mgcn.

Each keeps the reference's ``Net(dataset, num_layers, hidden)`` surface,
``reset_parameters()`` and ``forward(data) -> log_softmax`` over graphs:

=====================  ====================================  ==============================
net                    reference                             coarsening
=====================  ====================================  ==============================
TopK                   kernel/top_k.py:8-51                  TopKPooling after convs 0, 2, ..
SAGPool                kernel/sag_pool.py:8-51               SAGPooling after convs 0, 2, ..
EdgePool               kernel/edge_pool.py:8-51              EdgePooling after convs 0, 2, ..
Graclus                kernel/graclus.py:9-47                graclus + max_pool
HardPool               kernel/hard_pool.py:14-57             HardPooling (gcn_meta)
TopKNew                kernel/top_k_new.py:8-45              GCNConv, TopKPooling after each
SAGPoolNew             kernel/sag_pool_new.py:9-46           GCNConv, SAGPooling after each
GlobalAttentionNet     kernel/global_attention.py:7-38       SAGEConv + GlobalAttention
Set2SetNet             kernel/set2set.py:7-38                SAGEConv + Set2Set(4 steps)
SortPool               kernel/sort_pool.py:7-37              SAGEConv + global_sort_pool(k=10)
DiffPool               kernel/diff_pool.py:33-85             dense blocks + dense_diff_pool
=====================  ====================================  ==============================

(The _new files name their classes TopK / SAGPool too; here they are
TopKNew / SAGPoolNew.)  The jumping-knowledge nets share one skeleton:
``conv1``, then each conv followed by a graph mean read-out, and a
coarsening step after every even conv except the last; read-outs are
concatenated (JK 'cat') into lin1 -> ReLU -> dropout 0.5 -> lin2.
kernel/edge_pool.py:40 unpacks six values from EdgePooling, which returns
four in PyG; the net here unpacks four.
"""
from __future__ import annotations

from math import ceil

import torch
import torch.nn.functional as F

from ..models import Linear
from ..pool import (DenseSAGEConv, EdgePooling, GlobalAttention, HardPooling, SAGPooling,
                    Set2Set, TopKPooling, dense_diff_pool, global_sort_pool, graclus, max_pool)
from ..pyg import GCNConv, GraphConv, JumpingKnowledge, SAGEConv, global_mean_pool
from .data import Batch


def _head(model, x):
    x = F.relu(model.lin1(x))
    x = F.dropout(x, p=0.5, training=model.training)
    return F.log_softmax(model.lin2(x), dim=-1)


class _JKPoolNet(torch.nn.Module):
    """GraphConv(mean) stack with a graph read-out after every conv and a
    coarsening step (``_coarsen``) after convs 0, 2, 4, ... but the last."""

    n_pools = None  # pools built: num_layers // 2 (the reference builds that many)

    def __init__(self, dataset, num_layers, hidden):
        super().__init__()
        self.conv1 = GraphConv(dataset.num_features, hidden, aggr='mean')
        self.convs = torch.nn.ModuleList([GraphConv(hidden, hidden, aggr='mean')
                                          for _ in range(num_layers - 1)])
        self.pools = torch.nn.ModuleList([self._make_pool(hidden)
                                          for _ in range(num_layers // 2)])
        self.jump = JumpingKnowledge(mode='cat')
        self.lin1 = Linear(num_layers * hidden, hidden)
        self.lin2 = Linear(hidden, dataset.num_classes)

    def _make_pool(self, hidden):
        raise NotImplementedError

    def _coarsen(self, k, x, edge_index, batch):
        x, edge_index, _, batch, _, _ = self.pools[k](x, edge_index, batch=batch)
        return x, edge_index, batch

    def reset_parameters(self):
        self.conv1.reset_parameters()
        for m in [*self.convs, *self.pools]:
            m.reset_parameters()
        self.lin1.reset_parameters()
        self.lin2.reset_parameters()

    def forward(self, data):
        x, edge_index, batch = data.x, data.edge_index, data.batch
        x = F.relu(self.conv1(x, edge_index))
        reads = [global_mean_pool(x, batch)]
        last = len(self.convs) - 1
        for i, conv in enumerate(self.convs):
            x = F.relu(conv(x, edge_index))
            reads.append(global_mean_pool(x, batch))
            if i % 2 == 0 and i < last:
                x, edge_index, batch = self._coarsen(i // 2, x, edge_index, batch)
        return _head(self, self.jump(reads))

    def __repr__(self):
        return self.__class__.__name__


class TopK(_JKPoolNet):
    """kernel/top_k.py:8-51 (TopKPooling, ratio 0.8)."""

    def __init__(self, dataset, num_layers, hidden, ratio=0.8):
        self.ratio = ratio
        super().__init__(dataset, num_layers, hidden)

    def _make_pool(self, hidden):
        return TopKPooling(hidden, self.ratio)


class SAGPool(TopK):
    """kernel/sag_pool.py:8-51 (SAGPooling with a GraphConv score, ratio 0.8)."""

    def _make_pool(self, hidden):
        return SAGPooling(hidden, self.ratio)


class HardPool(_JKPoolNet):
    """kernel/hard_pool.py:14-57: gcn_meta's HardPooling in SAGPooling's place."""

    def _make_pool(self, hidden):
        return HardPooling(hidden)


class EdgePool(_JKPoolNet):
    """kernel/edge_pool.py:8-51 (EdgePooling; four return values)."""

    def _make_pool(self, hidden):
        return EdgePooling(hidden)

    def _coarsen(self, k, x, edge_index, batch):
        x, edge_index, batch, _ = self.pools[k](x, edge_index, batch=batch)
        return x, edge_index, batch


class Graclus(_JKPoolNet):
    """kernel/graclus.py:9-47: graclus matching + max_pool (no parameters)."""

    def _make_pool(self, hidden):
        return torch.nn.Identity()

    def _coarsen(self, k, x, edge_index, batch):
        cluster = graclus(edge_index, num_nodes=x.size(0))
        data = max_pool(cluster, Batch(x=x, edge_index=edge_index, batch=batch))
        return data.x, data.edge_index, data.batch

    def reset_parameters(self):
        self.conv1.reset_parameters()
        for m in self.convs:
            m.reset_parameters()
        self.jump.reset_parameters()
        self.lin1.reset_parameters()
        self.lin2.reset_parameters()


class TopKNew(torch.nn.Module):
    """kernel/top_k_new.py:8-45: GCNConv layers, a TopKPooling after every
    conv (num_layers pools), one mean read-out at the end."""

    def __init__(self, dataset, num_layers, hidden, ratio=0.8):
        super().__init__()
        self.ratio = ratio
        self.conv1 = GCNConv(dataset.num_features, hidden)
        self.convs = torch.nn.ModuleList([GCNConv(hidden, hidden) for _ in range(num_layers - 1)])
        self.pools = torch.nn.ModuleList([self._make_pool(hidden) for _ in range(num_layers)])
        self.lin1 = Linear(hidden, hidden)
        self.lin2 = Linear(hidden, dataset.num_classes)

    def _make_pool(self, hidden):
        return TopKPooling(hidden, self.ratio)

    def reset_parameters(self):
        for m in [self.conv1, *self.convs, *self.pools, self.lin1, self.lin2]:
            m.reset_parameters()

    def forward(self, data):
        x, edge_index, batch = data.x, data.edge_index, data.batch
        for conv, pool in zip([self.conv1, *self.convs], self.pools):
            x = F.relu(conv(x, edge_index))
            x, edge_index, _, batch, _, _ = pool(x, edge_index, batch=batch)
        return _head(self, global_mean_pool(x, batch))

    def __repr__(self):
        return self.__class__.__name__


class SAGPoolNew(TopKNew):
    """kernel/sag_pool_new.py:9-46 (SAGPooling, default ratio 0.5)."""

    def __init__(self, dataset, num_layers, hidden):
        super().__init__(dataset, num_layers, hidden, ratio=0.5)

    def _make_pool(self, hidden):
        return SAGPooling(hidden)


class _SAGEReadoutNet(torch.nn.Module):
    """SAGEConv stack (ReLU) followed by one graph read-out (``_readout``)."""

    def __init__(self, dataset, num_layers, hidden, readout_width):
        super().__init__()
        self.conv1 = SAGEConv(dataset.num_features, hidden)
        self.convs = torch.nn.ModuleList([SAGEConv(hidden, hidden)
                                          for _ in range(num_layers - 1)])
        self.lin1 = Linear(readout_width, hidden)
        self.lin2 = Linear(hidden, dataset.num_classes)

    def reset_parameters(self):
        for m in [self.conv1, *self.convs, *self._readout_modules(), self.lin1, self.lin2]:
            m.reset_parameters()

    def _readout_modules(self):
        return []

    def forward(self, data):
        x, edge_index, batch = data.x, data.edge_index, data.batch
        for conv in [self.conv1, *self.convs]:
            x = F.relu(conv(x, edge_index))
        return _head(self, self._readout(x, batch))

    def __repr__(self):
        return self.__class__.__name__


class GlobalAttentionNet(_SAGEReadoutNet):
    """kernel/global_attention.py:7-38: gate Linear(hidden, 1)."""

    def __init__(self, dataset, num_layers, hidden):
        super().__init__(dataset, num_layers, hidden, hidden)
        self.att = GlobalAttention(Linear(hidden, 1))

    def _readout_modules(self):
        return [self.att]

    def _readout(self, x, batch):
        return self.att(x, batch)


class Set2SetNet(_SAGEReadoutNet):
    """kernel/set2set.py:7-38: Set2Set(hidden, processing_steps=4)."""

    def __init__(self, dataset, num_layers, hidden):
        super().__init__(dataset, num_layers, hidden, 2 * hidden)
        self.set2set = Set2Set(hidden, processing_steps=4)

    def _readout_modules(self):
        return [self.set2set]

    def _readout(self, x, batch):
        return self.set2set(x, batch)


class SortPool(_SAGEReadoutNet):
    """kernel/sort_pool.py:7-37: global_sort_pool with k = 10."""

    def __init__(self, dataset, num_layers, hidden):
        self.k = 10
        super().__init__(dataset, num_layers, hidden, self.k * hidden)

    def _readout(self, x, batch):
        return global_sort_pool(x, batch, self.k)


class Block(torch.nn.Module):
    """kernel/diff_pool.py:8-29: two DenseSAGEConv (ReLU) + JK + Linear."""

    def __init__(self, in_channels, hidden_channels, out_channels, mode='cat'):
        super().__init__()
        self.conv1 = DenseSAGEConv(in_channels, hidden_channels)
        self.conv2 = DenseSAGEConv(hidden_channels, out_channels)
        self.jump = JumpingKnowledge(mode)
        width = hidden_channels + out_channels if mode == 'cat' else out_channels
        self.lin = Linear(width, out_channels)

    def reset_parameters(self):
        for m in (self.conv1, self.conv2, self.lin):
            m.reset_parameters()

    def forward(self, x, adj, mask=None, add_loop=True):
        x1 = F.relu(self.conv1(x, adj, mask, add_loop))
        x2 = F.relu(self.conv2(x1, adj, mask, add_loop))
        return self.lin(self.jump([x1, x2]))


class DiffPool(torch.nn.Module):
    """kernel/diff_pool.py:33-85 on dense batches (``data.x`` [B, N, F],
    ``data.adj`` [B, N, N], ``data.mask`` [B, N]; get_dataset(sparse=False))."""

    def __init__(self, dataset, num_layers, hidden, ratio=0.25):
        super().__init__()
        num_nodes = ceil(ratio * dataset[0].num_nodes)
        self.embed_block1 = Block(dataset.num_features, hidden, hidden)
        self.pool_block1 = Block(dataset.num_features, hidden, num_nodes)
        self.embed_blocks = torch.nn.ModuleList()
        self.pool_blocks = torch.nn.ModuleList()
        for _ in range((num_layers // 2) - 1):
            num_nodes = ceil(ratio * num_nodes)
            self.embed_blocks.append(Block(hidden, hidden, hidden))
            self.pool_blocks.append(Block(hidden, hidden, num_nodes))
        self.jump = JumpingKnowledge(mode='cat')
        self.lin1 = Linear((len(self.embed_blocks) + 1) * hidden, hidden)
        self.lin2 = Linear(hidden, dataset.num_classes)

    def reset_parameters(self):
        for m in [self.embed_block1, self.pool_block1, *self.embed_blocks, *self.pool_blocks,
                  self.jump, self.lin1, self.lin2]:
            m.reset_parameters()

    def forward(self, data):
        x, adj, mask = data.x, data.adj, data.mask
        s = self.pool_block1(x, adj, mask, add_loop=True)
        x = F.relu(self.embed_block1(x, adj, mask, add_loop=True))
        reads = [x.mean(dim=1)]
        x, adj, _, _ = dense_diff_pool(x, adj, s, mask)
        last = len(self.embed_blocks) - 1
        for i, (embed, pool) in enumerate(zip(self.embed_blocks, self.pool_blocks)):
            s = pool(x, adj)
            x = F.relu(embed(x, adj))
            reads.append(x.mean(dim=1))
            if i < last:
                x, adj, _, _ = dense_diff_pool(x, adj, s)
        return _head(self, self.jump(reads))

    def __repr__(self):
        return self.__class__.__name__


NETS = {n.__name__: n for n in (TopK, SAGPool, EdgePool, Graclus, HardPool, TopKNew, SAGPoolNew,
                                 GlobalAttentionNet, Set2SetNet, SortPool, DiffPool)}

__all__ = list(NETS) + ["Block", "NETS"]
