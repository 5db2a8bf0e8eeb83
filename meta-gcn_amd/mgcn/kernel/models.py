"""The graph-classification models of the reference's kernel/ benchmark
(kernel/gcn.py, kernel/gin.py, kernel/graph_sage.py), on mgcn's PyG-1.x convs.

Each is ``Net(dataset, num_layers, hidden)`` with ``reset_parameters()`` and
``forward(data) -> log_softmax`` over graphs: convs with ReLU, (JumpingKnowledge),
``global_mean_pool`` over ``data.batch``, lin1 + ReLU, dropout 0.5, lin2.
The pooling-operator nets (TopK, SAGPool, EdgePool, Graclus, DiffPool,
Set2Set, SortPool, GlobalAttention, HardPool) live in :mod:`.pool_nets`.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.nn import BatchNorm1d as BN
from torch.nn import ReLU, Sequential

from ..models import Linear
from ..pyg import GCNConv, GINConv, JumpingKnowledge, SAGEConv, global_mean_pool


class _Readout(torch.nn.Module):
    """Shared head: optional JK, mean pool, lin1 + ReLU, dropout, lin2."""

    def _setup_head(self, dataset, num_layers, hidden, mode):
        self.jump = JumpingKnowledge(mode) if mode is not None else None
        width = num_layers * hidden if mode == "cat" else hidden
        self.lin1 = Linear(width, hidden)
        self.lin2 = Linear(hidden, dataset.num_classes)

    def _head(self, xs, batch):
        x = self.jump(xs) if self.jump is not None else xs[-1]
        x = global_mean_pool(x, batch)
        x = F.relu(self.lin1(x))
        x = F.dropout(x, p=0.5, training=self.training)
        return F.log_softmax(self.lin2(x), dim=-1)

    def reset_parameters(self):
        for m in self.convs_all():
            m.reset_parameters()
        if self.jump is not None:
            self.jump.reset_parameters()
        self.lin1.reset_parameters()
        self.lin2.reset_parameters()

    def convs_all(self):
        return [self.conv1, *self.convs]

    def __repr__(self):
        return self.__class__.__name__


class GCN(_Readout):
    """kernel/gcn.py:7-36"""

    def __init__(self, dataset, num_layers, hidden, mode=None):
        super().__init__()
        self.conv1 = GCNConv(dataset.num_features, hidden)
        self.convs = torch.nn.ModuleList([GCNConv(hidden, hidden) for _ in range(num_layers - 1)])
        self._setup_head(dataset, num_layers, hidden, mode)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        x = F.relu(self.conv1(x, edge_index))
        xs = [x]
        for conv in self.convs:
            x = F.relu(conv(x, edge_index))
            xs.append(x)
        return self._head(xs, data.batch)


class GCNWithJK(GCN):
    """kernel/gcn.py:39-76"""

    def __init__(self, dataset, num_layers, hidden, mode="cat"):
        super().__init__(dataset, num_layers, hidden, mode)


class GraphSAGE(_Readout):
    """kernel/graph_sage.py:7-36"""

    def __init__(self, dataset, num_layers, hidden, mode=None):
        super().__init__()
        self.conv1 = SAGEConv(dataset.num_features, hidden)
        self.convs = torch.nn.ModuleList([SAGEConv(hidden, hidden)
                                          for _ in range(num_layers - 1)])
        self._setup_head(dataset, num_layers, hidden, mode)

    forward = GCN.forward


class GraphSAGEWithJK(GraphSAGE):
    """kernel/graph_sage.py:39-76"""

    def __init__(self, dataset, num_layers, hidden, mode="cat"):
        super().__init__(dataset, num_layers, hidden, mode)


def _gin_mlp(fin, hidden):
    return Sequential(Linear(fin, hidden), ReLU(), Linear(hidden, hidden), ReLU(), BN(hidden))


class GIN0(_Readout):
    """kernel/gin.py:7-47 (train_eps=False); the GIN MLP ends in ReLU + BN,
    so the convs are not followed by another activation."""

    train_eps = False

    def __init__(self, dataset, num_layers, hidden, mode=None):
        super().__init__()
        self.conv1 = GINConv(_gin_mlp(dataset.num_features, hidden), train_eps=self.train_eps)
        self.convs = torch.nn.ModuleList([GINConv(_gin_mlp(hidden, hidden),
                                                  train_eps=self.train_eps)
                                          for _ in range(num_layers - 1)])
        self._setup_head(dataset, num_layers, hidden, mode)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        x = self.conv1(x, edge_index)
        xs = [x]
        for conv in self.convs:
            x = conv(x, edge_index)
            xs.append(x)
        return self._head(xs, data.batch)


class GIN0WithJK(GIN0):
    """kernel/gin.py:50-95"""

    def __init__(self, dataset, num_layers, hidden, mode="cat"):
        super().__init__(dataset, num_layers, hidden, mode)


class GIN(GIN0):
    """kernel/gin.py:98-140 (train_eps=True)"""

    train_eps = True


class GINWithJK(GIN):
    """kernel/gin.py:143-190"""

    def __init__(self, dataset, num_layers, hidden, mode="cat"):
        super().__init__(dataset, num_layers, hidden, mode)
