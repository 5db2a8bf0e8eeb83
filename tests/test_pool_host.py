"""Host-side pieces of the pooling operators and the dense (DiffPool) data
path: no GPU, no libmgcn compute calls."""
import os

import numpy as np
import torch

from mgcn.kernel.data import DenseDataLoader, ToDense, get_dataset

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _pyg_merge(ei, order, n):
    """PyG 1.3 EdgePooling.__merge_edges__ matching, literally (set-based)."""
    nodes_remaining = set(range(n))
    cluster = [None] * n
    i, chosen = 0, []
    for e in order:
        s, t = int(ei[0, e]), int(ei[1, e])
        if s not in nodes_remaining or t not in nodes_remaining:
            continue
        chosen.append(e)
        cluster[s] = i
        nodes_remaining.remove(s)
        if s != t:
            cluster[t] = i
            nodes_remaining.remove(t)
        i += 1
    for node in nodes_remaining:
        cluster[node] = i
        i += 1
    return np.array(cluster), np.array(chosen, dtype=np.int64), i


def merge_edges_greedy(edge_index_np: np.ndarray, order: np.ndarray, num_nodes: int):
    """Array restatement of the same walk (boolean free mask, the leftover
    free nodes numbered by np.nonzero): the form the device kernel's
    numbering step follows (csrc/pool.hip)."""
    free = np.ones(num_nodes, dtype=bool)
    cluster = np.empty(num_nodes, dtype=np.int64)
    chosen = []
    i = 0
    src, dst = edge_index_np[0], edge_index_np[1]
    for e in order.tolist():
        s, t = int(src[e]), int(dst[e])
        if not free[s] or not free[t]:
            continue
        chosen.append(e)
        cluster[s] = i
        free[s] = False
        if s != t:
            cluster[t] = i
            free[t] = False
        i += 1
    rest = np.nonzero(free)[0]
    cluster[rest] = np.arange(i, i + rest.size)
    return cluster, np.asarray(chosen, dtype=np.int64), i + rest.size


def test_merge_edges_greedy_matches_pyg_loop():
    rng = np.random.default_rng(0)
    for n, E in [(1, 0), (5, 3), (40, 90), (300, 500), (1000, 400)]:
        ei = rng.integers(0, n, (2, E))
        ei[:, ::7] = ei[0, ::7]  # self loops
        order = rng.permutation(E)
        a = merge_edges_greedy(ei, order, n)
        b = _pyg_merge(ei, order, n)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        assert a[2] == b[2]


def test_to_dense_and_dense_loader():
    g = get_dataset("MUTAG", synthetic=True)[0]
    d = ToDense(30)(g)
    n = g.num_nodes
    assert d.x.shape == (30, g.x.size(1)) and d.adj.shape == (30, 30)
    assert d.mask.sum().item() == n and bool(d.mask[:n].all())
    ref = torch.zeros(30, 30)
    for s, t in g.edge_index.t().tolist():
        ref[s, t] += 1
    assert torch.equal(d.adj, ref)
    assert torch.equal(d.x[n:], torch.zeros(30 - n, g.x.size(1)))
    ds = get_dataset("MUTAG", sparse=False, synthetic=True)
    assert 'adj' in ds[0]
    limit = ds[0].x.size(0)
    assert all(ds[i].x.size(0) == limit for i in range(len(ds)))
    b = next(iter(DenseDataLoader(ds, 16)))
    assert b.x.shape == (16, limit, ds.num_features) and b.adj.shape == (16, limit, limit)
    assert b.mask.shape == (16, limit) and b.y.view(-1).shape == (16,)


def test_hardpool_fixtures_are_consistent():
    """The reference's eval-mode HardPooling output: kept nodes are the
    targets of the selected edges, the pooled edge list is the induced
    subgraph relabelled, batch follows perm."""
    for name in ("hardpool_add", "hardpool_add_bias", "hardpool_mean", "hardpool_sunk"):
        d = np.load(os.path.join(GOLDEN, name + ".npz"))
        perm = d["perm"]
        assert np.all(np.diff(perm) > 0)
        np.testing.assert_array_equal(d["out_batch"], d["batch"][perm])
        pos = {int(p): i for i, p in enumerate(perm)}
        kept = [(pos[a], pos[b]) for a, b in d["edge_index"].T.tolist() if a in pos and b in pos]
        np.testing.assert_array_equal(d["out_edge_index"], np.array(kept).T.reshape(2, -1))
        assert d["out"].shape == (perm.size, d["x"].shape[1])
