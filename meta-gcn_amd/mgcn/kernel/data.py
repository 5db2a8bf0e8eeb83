"""Config-1 data plumbing of the reference's kernel/ benchmark, offline.

The reference loads TU graph-classification datasets through PyG 1.x
(kernel/datasets.py:34-94 -> torch_geometric.datasets.TUDataset, which
downloads) and batches them with PyG's DataLoader (kernel/train_eval.py:36-43).
Neither PyG nor a network exists here, so this module restates:

* ``read_tu_data`` -- PyG 1.x's reader of the TU text format
  (``{name}_A.txt`` 1-based "i, j" edges, ``_graph_indicator``,
  ``_graph_labels``, optional ``_node_labels`` / ``_node_attributes``):
  edge ids shifted to 0-based, self loops removed, edges coalesced (sorted by
  (row, col), duplicates dropped), node labels one-hot per column after
  subtracting the column minimum, graph labels mapped to 0..C-1 through
  ``unique(sorted=True, return_inverse=True)``, split into per-graph
  ``Data`` with local node ids;
* ``TUDataset`` -- the dataset object the driver indexes (``dataset[idx]``,
  ``dataset.data.y``, ``num_features``, ``num_classes``, ``transform``);
* the transforms ``get_dataset`` installs (kernel/datasets.py:10-31,59-70):
  ``OneHotDegree``, ``NormalizedDegree``, ``NodeFeatureOnes``;
* ``Batch`` / ``DataLoader`` -- PyG-style collation: node features and labels
  concatenated, ``edge_index`` offset by the running node count, a ``batch``
  vector of graph ids;
* ``synthetic_tu`` -- a MUTAG-shaped stand-in (SURVEY.md §8(d) config 1:
  188 graphs, ~18 nodes / ~40 directed edges each, 7 one-hot node labels,
  2 classes) for when the TU files are not supplied.

Host-side data plumbing only (CPU tensors until ``Batch.to(device)``); the
convs that consume the batches run on libmgcn.
"""
from __future__ import annotations

import os
import os.path as osp

import numpy as np
import torch
import torch.nn.functional as F


class Data:
    """One graph (or a collated batch): attributes x, edge_index, y, batch."""

    def __init__(self, x=None, edge_index=None, y=None, batch=None, num_nodes=None):
        self.x = x
        self.edge_index = edge_index
        self.y = y
        self.batch = batch
        self._num_nodes = num_nodes

    @property
    def num_nodes(self) -> int:
        if self._num_nodes is not None:
            return int(self._num_nodes)
        if self.x is not None:
            return int(self.x.size(0))
        return int(self.edge_index.max()) + 1 if self.edge_index.numel() else 0

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.size(1))

    def __contains__(self, key) -> bool:  # `'adj' in data` (kernel/train_eval.py:31)
        return getattr(self, key, None) is not None

    def clone(self) -> "Data":
        c = Data(num_nodes=self._num_nodes)
        for k in ("x", "edge_index", "y", "batch"):
            v = getattr(self, k)
            setattr(c, k, v.clone() if isinstance(v, torch.Tensor) else v)
        return c

    def to(self, device) -> "Data":
        for k in ("x", "edge_index", "y", "batch"):
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self


class Batch(Data):
    """PyG-style mini-batch of graphs (torch_geometric.data.Batch)."""

    @property
    def num_graphs(self) -> int:
        return int(self.y.numel()) if self.y is not None else int(self.batch.max()) + 1

    @staticmethod
    def from_data_list(graphs) -> "Batch":
        xs, eis, ys, bs = [], [], [], []
        off = 0
        for g, d in enumerate(graphs):
            n = d.num_nodes
            if d.x is not None:
                xs.append(d.x)
            eis.append(d.edge_index + off)
            if d.y is not None:
                ys.append(d.y.view(-1))
            bs.append(torch.full((n,), g, dtype=torch.long))
            off += n
        return Batch(x=torch.cat(xs, 0) if xs else None,
                     edge_index=torch.cat(eis, 1) if eis else torch.zeros(2, 0, dtype=torch.long),
                     y=torch.cat(ys, 0) if ys else None,
                     batch=torch.cat(bs, 0) if bs else torch.zeros(0, dtype=torch.long),
                     num_nodes=off)


class DataLoader:
    """Mini-batches of ``batch_size`` graphs; ``shuffle`` draws a fresh
    permutation from torch's global generator every epoch (as torch's
    RandomSampler under PyG's DataLoader does)."""

    def __init__(self, dataset, batch_size=1, shuffle=False, share=None, generator=None):
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.share, self.generator = share, generator  # data-parallel replicas

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def _batches(self):
        """Index lists of the global batches, cut to this rank's share (an
        empty share stays in the sequence: every replica steps together)."""
        n = len(self.dataset)
        order = (torch.randperm(n, generator=self.generator).tolist() if self.shuffle
                 else list(range(n)))
        for i in range(0, n, self.batch_size):
            idx = order[i:i + self.batch_size]
            yield self.share(idx) if self.share is not None else idx

    def __iter__(self):
        for idx in self._batches():
            yield Batch.from_data_list([self.dataset[j] for j in idx]) if idx else None


class DenseData:
    """One graph padded to a fixed node count (torch_geometric ToDense
    output): x [N, F], adj [N, N], mask [N] (bool), y; a DenseDataLoader
    batch stacks them (x [B, N, F], adj [B, N, N], mask [B, N])."""

    def __init__(self, x=None, adj=None, mask=None, y=None):
        self.x, self.adj, self.mask, self.y = x, adj, mask, y
        self.batch = None
        self.edge_index = None

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(-2)) if self.x is not None else int(self.adj.size(-1))

    @property
    def num_graphs(self) -> int:
        return int(self.x.size(0)) if self.x.dim() == 3 else 1

    def __contains__(self, key) -> bool:
        return getattr(self, key, None) is not None

    def to(self, device) -> "DenseData":
        for k in ("x", "adj", "mask", "y"):
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self


class ToDense:
    """torch_geometric.transforms.ToDense(num_nodes) (PyG 1.3): dense
    adjacency (duplicate edges summed), node mask, x zero-padded to
    ``num_nodes`` rows (kernel/datasets.py:91-94)."""

    def __init__(self, num_nodes=None):
        self.num_nodes = num_nodes

    def __call__(self, data):
        n0 = data.num_nodes
        n = n0 if self.num_nodes is None else self.num_nodes
        assert n0 <= n, f"graph of {n0} nodes does not fit ToDense({n})"
        adj = torch.zeros(n, n, dtype=torch.float)
        if data.edge_index.numel():
            adj.index_put_((data.edge_index[0], data.edge_index[1]),
                           torch.ones(data.edge_index.size(1)), accumulate=True)
        mask = torch.zeros(n, dtype=torch.bool)
        mask[:n0] = True
        x = None
        if data.x is not None:
            x = torch.cat([data.x, data.x.new_zeros([n - data.x.size(0)] + list(data.x.size())[1:])],
                          dim=0)
        y = data.y
        if y is not None and y.size(0) == n0 and n0 != 1:
            y = torch.cat([y, y.new_zeros([n - n0] + list(y.size())[1:])], dim=0)
        return DenseData(x=x, adj=adj, mask=mask, y=y)


class DenseDataLoader:
    """torch_geometric.data.DenseDataLoader: stacks every attribute."""

    def __init__(self, dataset, batch_size=1, shuffle=False, share=None, generator=None):
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.share, self.generator = share, generator

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    _batches = DataLoader._batches

    def __iter__(self):
        for idx in self._batches():
            if not idx:
                yield None
                continue
            items = [self.dataset[j] for j in idx]
            yield DenseData(**{k: torch.stack([getattr(d, k) for d in items])
                               for k in ("x", "adj", "mask", "y")})


# ---------------------------------------------------------------- TU format
def _read(folder, prefix, name, dtype):
    path = osp.join(folder, f"{prefix}_{name}.txt")
    with open(path) as f:
        rows = [[float(v) for v in line.replace(",", " ").split()] for line in f if line.strip()]
    t = torch.tensor(rows, dtype=torch.float64)
    t = t.to(dtype)
    return t.squeeze(-1) if t.dim() == 2 and t.size(1) == 1 else t


def _one_hot_columns(labels: torch.Tensor) -> torch.Tensor:
    if labels.dim() == 1:
        labels = labels.unsqueeze(-1)
    labels = labels - labels.min(dim=0)[0]
    cols = [F.one_hot(c, num_classes=int(c.max()) + 1) for c in labels.unbind(dim=-1)]
    return torch.cat(cols, dim=-1).to(torch.float)


def coalesce(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Sort by (row, col) and drop duplicate edges (torch_sparse.coalesce)."""
    if edge_index.numel() == 0:
        return edge_index
    key = edge_index[0] * num_nodes + edge_index[1]
    key = torch.unique(key, sorted=True)
    return torch.stack([key // num_nodes, key % num_nodes], 0)


def read_tu_data(folder: str, prefix: str, use_node_attr: bool = False):
    """Per-graph ``Data`` list and the dataset's label vector, from the TU
    text files in ``folder`` (PyG 1.x torch_geometric.io.read_tu_data)."""
    files = set(os.listdir(folder))
    edge_index = _read(folder, prefix, "A", torch.long).view(-1, 2).t() - 1
    batch = _read(folder, prefix, "graph_indicator", torch.long).view(-1) - 1
    feats = []
    n_attr = 0
    if f"{prefix}_node_attributes.txt" in files and use_node_attr:
        attr = _read(folder, prefix, "node_attributes", torch.float)
        attr = attr.unsqueeze(-1) if attr.dim() == 1 else attr
        feats.append(attr)
        n_attr = attr.size(1)
    if f"{prefix}_node_labels.txt" in files:
        feats.append(_one_hot_columns(_read(folder, prefix, "node_labels", torch.long)))
    x = torch.cat(feats, dim=-1) if feats else None
    y = _read(folder, prefix, "graph_labels", torch.long).view(-1)
    _, y = torch.unique(y, sorted=True, return_inverse=True)
    num_nodes = batch.numel()
    keep = edge_index[0] != edge_index[1]  # remove_self_loops
    edge_index = coalesce(edge_index[:, keep], num_nodes)
    # split into graphs (node ids are contiguous per graph in the TU format)
    n_graphs = int(batch.max()) + 1
    node_count = torch.bincount(batch, minlength=n_graphs)
    node_start = torch.cumsum(node_count, 0) - node_count
    edge_graph = batch[edge_index[0]]
    order = torch.argsort(edge_graph, stable=True)
    edge_index, edge_graph = edge_index[:, order], edge_graph[order]
    edge_count = torch.bincount(edge_graph, minlength=n_graphs)
    graphs = []
    e0 = 0
    for g in range(n_graphs):
        s, n, m = int(node_start[g]), int(node_count[g]), int(edge_count[g])
        ei = edge_index[:, e0:e0 + m] - s
        e0 += m
        graphs.append(Data(x=None if x is None else x[s:s + n], edge_index=ei,
                           y=y[g:g + 1], num_nodes=n))
    return graphs, y, n_attr


class _Store:
    """``dataset.data`` (the reference reads ``dataset.data.y`` for k_fold and
    ``dataset.data.x is None`` in get_dataset)."""

    def __init__(self, graphs):
        self._graphs = graphs

    @property
    def y(self):
        return torch.cat([g.y.view(-1) for g in self._graphs], 0)

    @property
    def x(self):
        if self._graphs and self._graphs[0].x is None:
            return None
        return torch.cat([g.x for g in self._graphs], 0)


class TUDataset:
    """In-memory graph-classification dataset with PyG's indexing surface."""

    def __init__(self, root: str | None = None, name: str | None = None, graphs=None,
                 transform=None, use_node_attr: bool = False):
        if graphs is None:
            folder = None
            for cand in (osp.join(root, name, "raw"), osp.join(root, "raw"), osp.join(root, name),
                         root):
                if cand and osp.exists(osp.join(cand, f"{name}_A.txt")):
                    folder = cand
                    break
            if folder is None:
                raise FileNotFoundError(
                    f"TU files {name}_A.txt etc. not found under {root} (no download here; "
                    "use synthetic_tu() for a MUTAG-shaped stand-in)")
            graphs, _, _ = read_tu_data(folder, name, use_node_attr)
        self.name = name
        self._graphs = list(graphs)
        self.transform = transform
        self.data = _Store(self._graphs)

    def __len__(self):
        return len(self._graphs)

    def _get(self, i):
        d = self._graphs[i]
        return self.transform(d.clone()) if self.transform is not None else d

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return self._get(int(idx))
        if isinstance(idx, torch.Tensor):
            if idx.dtype == torch.bool:
                idx = idx.nonzero().view(-1)
            idx = idx.tolist()
        elif isinstance(idx, slice):
            idx = list(range(len(self)))[idx]
        sub = TUDataset(name=self.name, graphs=[self._graphs[int(i)] for i in idx],
                        transform=self.transform)
        return sub

    def __iter__(self):
        for i in range(len(self)):
            yield self._get(i)

    @property
    def num_features(self) -> int:
        d = self._get(0)
        return 0 if d.x is None else int(d.x.size(1))

    @property
    def num_classes(self) -> int:
        return int(self.data.y.max()) + 1

    def collate(self, data_list):  # kernel/datasets.py:51 (add_sl): keep the list
        self._graphs = list(data_list)
        self.data = _Store(self._graphs)
        return self.data, None

    def __repr__(self):
        return f"{self.name}({len(self)})"


def synthetic_tu(name: str = "MUTAG", n_graphs: int = 188, n_labels: int = 7,
                 n_classes: int = 2, seed: int = 0) -> TUDataset:
    """MUTAG-shaped synthetic dataset: ring-plus-chords molecules of 10-28
    nodes (about 18 nodes, 40 directed edges on average), 7 one-hot node
    labels, class-dependent label frequencies so the task is learnable."""
    rng = np.random.default_rng(seed)
    graphs = []
    for g in range(n_graphs):
        c = g % n_classes
        n = int(rng.integers(10, 29))
        ring = np.arange(n)
        s = np.concatenate([ring, rng.integers(0, n, n // 10 + 1)])
        d = np.concatenate([(ring + 1) % n, rng.integers(0, n, n // 10 + 1)])
        keep = s != d
        s, d = s[keep], d[keep]
        ei = torch.from_numpy(np.stack([np.concatenate([s, d]), np.concatenate([d, s])]))
        ei = coalesce(ei.long(), n)
        p = np.full(n_labels, 1.0)
        p[c % n_labels] += 3.0
        lab = rng.choice(n_labels, size=n, p=p / p.sum())
        x = F.one_hot(torch.from_numpy(lab).long(), n_labels).float()
        graphs.append(Data(x=x, edge_index=ei, y=torch.tensor([c]), num_nodes=n))
    return TUDataset(name=name, graphs=graphs)


# ---------------------------------------------------------------- transforms
def degree(index: torch.Tensor, num_nodes: int | None = None, dtype=None) -> torch.Tensor:
    n = num_nodes if num_nodes is not None else (int(index.max()) + 1 if index.numel() else 0)
    out = torch.bincount(index, minlength=n)
    return out.to(dtype) if dtype is not None else out


class OneHotDegree:
    """x = one_hot(out-degree) (cat to x if present), torch_geometric.transforms."""

    def __init__(self, max_degree: int, in_degree: bool = False, cat: bool = True):
        self.max_degree, self.in_degree, self.cat = max_degree, in_degree, cat

    def __call__(self, data):
        idx = data.edge_index[1 if self.in_degree else 0]
        deg = degree(idx, data.num_nodes, dtype=torch.long).clamp(max=self.max_degree)
        deg = F.one_hot(deg, num_classes=self.max_degree + 1).to(torch.float)
        data.x = torch.cat([data.x, deg], -1) if (data.x is not None and self.cat) else deg
        return data


class NormalizedDegree:
    """x = (out-degree - mean) / std (kernel/datasets.py:10-19)."""

    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def __call__(self, data):
        deg = degree(data.edge_index[0], data.num_nodes, dtype=torch.float)
        data.x = ((deg - self.mean) / self.std).view(-1, 1)
        return data


class NodeFeatureOnes:
    """x = ones [N, 1] for featureless graphs (kernel/datasets.py:22-31)."""

    def __call__(self, data):
        data.x = torch.ones(data.num_nodes, 1)
        return data


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data


def get_dataset(name: str, root: str | None = None, sparse: bool = True, x_deg: bool = True,
                add_sl: bool = False, cleaned: bool = False, synthetic: bool | None = None):
    """kernel/datasets.py:34-94 ``get_dataset``.  ``root`` holds the TU files
    (default ``<repo>/data/<name>``, the reference's layout); ``synthetic``
    True (or None with the files absent) uses ``synthetic_tu``.  The dense
    DiffPool variant (``sparse=False``) keeps the graphs up to a size limit
    and pads them with ToDense (:func:`_dense_filter`)."""
    if root is None:
        root = osp.join(osp.dirname(osp.dirname(osp.dirname(osp.dirname(
            osp.abspath(__file__))))), "data", name)
    if synthetic or (synthetic is None and not osp.exists(root)):
        dataset = synthetic_tu(name)
    else:
        dataset = TUDataset(root, name)
    if add_sl:
        from ..pyg import add_remaining_self_loops
        data_list = []
        for data in dataset:
            data.edge_index, _ = add_remaining_self_loops(data.edge_index,
                                                          num_nodes=data.num_nodes)
            data_list.append(data)
        dataset.collate(data_list)
    if dataset.data.x is None:
        if x_deg:
            max_degree, degs = 0, []
            for data in dataset:
                degs.append(degree(data.edge_index[0], data.num_nodes, dtype=torch.long))
                max_degree = max(max_degree, int(degs[-1].max()) if degs[-1].numel() else 0)
            if max_degree < 1000:
                dataset.transform = OneHotDegree(max_degree)
            else:
                deg = torch.cat(degs, 0).to(torch.float)
                dataset.transform = NormalizedDegree(deg.mean().item(), deg.std().item())
        else:
            dataset.transform = NodeFeatureOnes()
    if not sparse:
        dataset = _dense_filter(dataset, name)
    return dataset


def _dense_filter(dataset, name):
    """kernel/datasets.py:72-94: drop graphs above 5 x the mean node count
    (1.5 x for REDDIT-BINARY), capped at the largest graph, and pad the rest
    to that size with ToDense (after the feature transform)."""
    total = max_n = 0
    for d in dataset._graphs:
        total += d.num_nodes
        max_n = max(max_n, d.num_nodes)
    factor = 1.5 if name == 'REDDIT-BINARY' else 5
    limit = min(int(total / len(dataset) * factor), max_n)
    keep = [i for i, d in enumerate(dataset._graphs) if d.num_nodes <= limit]
    dataset = dataset[torch.tensor(keep)]
    dataset.transform = ToDense(limit) if dataset.transform is None else \
        Compose([dataset.transform, ToDense(limit)])
    return dataset
