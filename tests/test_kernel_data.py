"""Config-1 plumbing: TU loader, batching,
k-fold split, early stopping -- host-side, CPU only.

The TU semantics are PyG 1.x's reader (not importable here: parity for the
loader is pinned by hand-derived expectations on a written dataset, the fold
split by sklearn itself, which the reference calls the same way)."""
import numpy as np
import pytest
import torch

from mgcn.kernel import (Batch, DataLoader, EarlyStopping, NormalizedDegree, OneHotDegree,
                         TUDataset, get_dataset, k_fold, read_tu_data, synthetic_tu)


def _write_tu(folder, name="TOY", node_labels=True):
    # graph 1: nodes 1-3, edges 1-2, 2-1, 2-3, 3-2, duplicate 1-2, self loop 3-3
    # graph 2: nodes 4-5, edges 4-5, 5-4
    # graph 3: node 6, no edges
    edges = [(1, 2), (2, 1), (2, 3), (3, 2), (1, 2), (3, 3), (5, 4), (4, 5)]
    (folder / f"{name}_A.txt").write_text("".join(f"{a}, {b}\n" for a, b in edges))
    (folder / f"{name}_graph_indicator.txt").write_text("1\n1\n1\n2\n2\n3\n")
    (folder / f"{name}_graph_labels.txt").write_text("-1\n1\n-1\n")
    if node_labels:
        (folder / f"{name}_node_labels.txt").write_text("2\n3\n2\n4\n2\n3\n")


def test_read_tu_data_semantics(tmp_path):
    _write_tu(tmp_path)
    graphs, y, _ = read_tu_data(str(tmp_path), "TOY")
    assert len(graphs) == 3
    assert y.tolist() == [0, 1, 0]  # unique(sorted, return_inverse)
    g1, g2, g3 = graphs
    # 0-based, local ids, self loop removed, duplicate dropped, sorted by (row, col)
    assert g1.edge_index.tolist() == [[0, 1, 1, 2], [1, 0, 2, 1]]
    assert g2.edge_index.tolist() == [[0, 1], [1, 0]]
    assert g3.edge_index.shape == (2, 0) and g3.num_nodes == 1
    # node labels 2,3,4 -> minus min -> one-hot of width 3
    assert g1.x.tolist() == [[1, 0, 0], [0, 1, 0], [1, 0, 0]]
    assert g2.x.tolist() == [[0, 0, 1], [1, 0, 0]]
    ds = TUDataset(str(tmp_path), "TOY")
    assert ds.num_features == 3 and ds.num_classes == 2 and len(ds) == 3
    assert ds.data.y.tolist() == [0, 1, 0]
    sub = ds[torch.tensor([2, 0])]
    assert [d.num_nodes for d in sub] == [1, 3]


def test_get_dataset_featureless_uses_one_hot_degree(tmp_path):
    root = tmp_path / "TOY"
    root.mkdir()
    _write_tu(root, node_labels=False)
    ds = get_dataset("TOY", root=str(root), synthetic=False)
    assert isinstance(ds.transform, OneHotDegree) and ds.transform.max_degree == 2
    x = ds[0].x  # out-degrees 1, 2, 1 -> one-hot width 3
    assert x.tolist() == [[0, 1, 0], [0, 0, 1], [0, 1, 0]]
    assert ds.num_features == 3
    nd = NormalizedDegree(1.0, 2.0)(ds._graphs[0].clone())
    assert nd.x.view(-1).tolist() == [0.0, 0.5, 0.0]
    dense = get_dataset("TOY", root=str(root), sparse=False)  # DiffPool's ToDense path
    assert 'adj' in dense[0] and dense[0].adj.size(0) == dense[0].x.size(0)


def test_add_sl_adds_remaining_loops(tmp_path):
    root = tmp_path / "TOY"
    root.mkdir()
    _write_tu(root)
    ds = get_dataset("TOY", root=str(root), add_sl=True, synthetic=False)
    g1 = ds[0]
    loops = (g1.edge_index[0] == g1.edge_index[1]).sum().item()
    assert loops == 3 and g1.num_edges == 7


def test_batch_collation_offsets():
    ds = synthetic_tu(n_graphs=10)
    b = Batch.from_data_list([ds[i] for i in (3, 7, 1)])
    sizes = [ds[i].num_nodes for i in (3, 7, 1)]
    assert b.num_nodes == sum(sizes) and b.num_graphs == 3
    assert b.batch.tolist() == sum(([g] * n for g, n in enumerate(sizes)), [])
    e1 = ds[3].num_edges
    assert torch.equal(b.edge_index[:, e1:e1 + ds[7].num_edges], ds[7].edge_index + sizes[0])
    assert torch.equal(b.x, torch.cat([ds[i].x for i in (3, 7, 1)]))
    torch.manual_seed(0)
    seen = torch.cat([bt.y for bt in DataLoader(ds, 4, shuffle=True)])
    assert seen.numel() == 10 and len(DataLoader(ds, 4)) == 3


def test_k_fold_protocol():
    from sklearn.model_selection import StratifiedKFold
    ds = synthetic_tu()
    tr, te, va = k_fold(ds, 10, random_state=12345)
    skf = StratifiedKFold(10, shuffle=True, random_state=12345)
    ref = [idx for _, idx in skf.split(np.zeros(len(ds)), ds.data.y.numpy())]
    for i in range(10):
        assert te[i].tolist() == ref[i].tolist()
        assert va[i].tolist() == ref[i - 1].tolist()  # val = previous fold's test
        parts = torch.cat([tr[i], te[i], va[i]]).sort()[0]
        assert parts.tolist() == list(range(len(ds)))  # a partition
    y = ds.data.y
    for t in te:  # stratified: class balance within one graph of the whole
        assert abs(y[t].float().mean().item() - y.float().mean().item()) < 0.06


def test_early_stopping():
    es = EarlyStopping(patience=2, mode="min", verbose=False)
    for v in (1.0, 0.9, 0.95, 0.96):
        es(v)
    assert es.early_stop and es.best == 0.9
    off = EarlyStopping(patience=-1)
    for v in (1.0, 2.0, 3.0):
        off(v)
    assert not off.early_stop
