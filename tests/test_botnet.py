"""Config-3 harness (mgcn.botnet): the .npz dataset layout round trip, the
PyG-style batching, the optim/metrics.py metrics and optim/focal_loss.py
FocalLoss against hand-computed values (CPU); a short train_botnet.py run on
small synthetic botnet graphs (GPU)."""
import math

import numpy as np
import pytest
import torch

from mgcn import botnet

SMALL = dict(n_nodes=3000, bg_edges=8000, max_deg=300, p2p_nodes=200, p2p_edges=1000)


def test_npz_round_trip_and_batching(tmp_path):
    graphs = botnet.synthetic_botnet(3, seed=5, **SMALL)
    path = str(tmp_path / "g.npz")
    botnet.save_npz(graphs, path)
    for in_memory in (False, True):
        ds = botnet.GraphDataset(path, in_memory=in_memory)
        assert len(ds) == 3
        for g, d in zip(graphs, ds):
            assert d.num_nodes == g["num_nodes"]
            torch.testing.assert_close(d.x, g["x"], rtol=0, atol=0)
            assert torch.equal(d.edge_index, g["edge_index"])
            assert torch.equal(d.y, g["y"]) and torch.equal(d.edge_y, g["edge_y"])
    # x = [1, degree incl. self loop]; edge_y marks bot-bot edges
    g = graphs[0]
    assert torch.all(g["x"][:, 0] == 1)
    assert torch.equal(g["x"][:, 1].long(), torch.bincount(g["edge_index"][0], minlength=3000))
    ei, y = g["edge_index"], g["y"].bool()
    assert torch.equal(g["edge_y"].bool(), y[ei[0]] & y[ei[1]])
    batches = list(botnet.GraphDataLoader(ds, batch_size=2))
    assert len(batches) == 2
    b = batches[0]
    assert b.x.shape[0] == 6000 and b.edge_index.shape[1] == 2 * ei.shape[1]
    assert torch.equal(b.edge_index[:, ei.shape[1]:], graphs[1]["edge_index"] + 3000)


def test_generator_matches_config3_shape():
    ei, n, mask = botnet.make_botnet_graph(seed=0)
    deg = torch.bincount(ei[1], minlength=n)
    assert n == 143_107 and int(mask.sum()) == 10_000
    assert ei.shape[1] == 2 * (350_000 + 49_566) + n
    assert 3000 < int(deg.max()) < 9000  # heavy head near the quoted 5.9k


def test_metrics_known_values():
    pred = torch.tensor([1, 1, 0, 0, 1, 0, 0, 0])
    tgt = torch.tensor([1, 0, 0, 1, 1, 0, 0, 0])
    # tp 2, fp 1, tn 4, fn 1
    assert botnet.accuracy(pred, tgt) == 6 / 8
    assert (botnet.true_positive(pred, tgt), botnet.false_positive(pred, tgt),
            botnet.true_negative(pred, tgt), botnet.false_negative(pred, tgt)) == (2, 1, 4, 1)
    assert botnet.recall(pred, tgt) == 2 / 3 and botnet.precision(pred, tgt) == 2 / 3
    assert math.isclose(botnet.f1_score(pred, tgt), 2 / 3)
    assert botnet.false_positive_rate(pred, tgt) == 1 / 5
    assert botnet.false_negative_rate(pred, tgt) == 1 / 3
    # no positive prediction: precision -1 (metrics.py:35-40), f1 by its formula
    none = torch.zeros(8, dtype=torch.long)
    assert botnet.precision(none, tgt) == -1
    assert botnet.f1_score(none, tgt) == 0.0  # rec 0: 2*(-1*0)/(-1+0)
    # no positive target: the reference divides by zero; nan here
    assert math.isnan(botnet.recall(pred, torch.zeros(8, dtype=torch.long)))


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_focal_loss_formula(reduction):
    torch.manual_seed(0)
    s = torch.randn(50, 2, dtype=torch.float64)
    t = torch.randint(0, 2, (50,))
    fl = botnet.FocalLoss(alpha=1, gamma=2, reduction=reduction)(s, t)
    p = np.exp(s.numpy()) / np.exp(s.numpy()).sum(1, keepdims=True) + 1e-8
    pt = p[np.arange(50), t.numpy()]
    ref = -(1 - pt) ** 2 * np.log(pt)
    ref = {"mean": ref.mean(), "sum": ref.sum(), "none": ref}[reduction]
    np.testing.assert_allclose(fl.numpy(), ref, rtol=1e-12)
    # gamma 0, alpha 1 is cross entropy up to the 1e-8 shift
    ce = torch.nn.functional.cross_entropy(s, t)
    assert abs(float(botnet.FocalLoss(alpha=1, gamma=0)(s, t)) - float(ce)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("aggr,focal", [("add", False), ("max", True)])
def test_train_botnet_small(cuda, tmp_path, aggr, focal):
    torch.manual_seed(0)
    paths = []
    for i, n in enumerate((2, 1, 1)):
        p = str(tmp_path / f"{i}.npz")
        botnet.save_npz(botnet.synthetic_botnet(n, seed=10 * i, **SMALL), p)
        paths.append(p)
    ds = [botnet.GraphDataset(p) for p in paths]
    hist = botnet.train(*ds, enc_sizes=[32] * 4, residual_hop=1, aggr=aggr, focal=focal,
                        lr=0.01, epochs=4, device=cuda, log=lambda s: None,
                        save_path=str(tmp_path / "best.pt"))
    assert len(hist["train_loss"]) == 4 and all(math.isfinite(v) for v in hist["train_loss"])
    assert hist["train_loss"][-1] < hist["train_loss"][0]
    t = hist["test"]
    assert 0.0 <= t["acc"] <= 1.0 and math.isfinite(t["loss"])
    state = torch.load(str(tmp_path / "best.pt"), weights_only=True)
    assert all(v.device.type == "cuda" for v in state.values())


def test_cross_entropy_matches_torch():
    import torch
    from mgcn.botnet import CrossEntropyLoss
    g = torch.Generator().manual_seed(0)
    s = torch.randn(1000, 2, generator=g, requires_grad=True)
    y = torch.randint(0, 2, (1000,), generator=g)
    for red in ("mean", "sum", "none"):
        a = CrossEntropyLoss(red)(s, y)
        b = torch.nn.CrossEntropyLoss(reduction=red)(s, y)
        torch.testing.assert_close(a, b)
    ga, = torch.autograd.grad(CrossEntropyLoss()(s, y), s)
    gb, = torch.autograd.grad(torch.nn.CrossEntropyLoss()(s, y), s)
    torch.testing.assert_close(ga, gb)
