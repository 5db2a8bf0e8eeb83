"""Config-3 harness: botnet node classification (src/run/train_botnet.py,
src/gcn_meta/data/{dataset,data,dataloader}.py, optim/{metrics,focal_loss,
earlystop}.py of the reference), on mgcn's GCNModel.

Data.  The reference reads HDF5 files (h5py / deepdish, gcn_meta/data/
dataset.py:15-48): file attribute ``num_graphs``; group ``str(i)`` per graph
with datasets ``x`` (f4 [N, 2] = [1, degree]), ``y`` (u1 [N], 1 = bot),
``edge_index`` (i8 [2, E]), ``edge_y`` (u1 [E]) and attributes ``num_nodes``,
``num_edges``, ``num_evils`` (data_add_edges_ey.py:119-156).  Neither h5py nor
the data exist here, so :class:`GraphDataset` reads

* ``.npz`` archives with the same content, keys ``"num_graphs"`` and
  ``"<i>/<name>"`` (``scripts/botnet_h5_to_npz.py`` converts an HDF5 file
  where h5py is installed; :func:`save_npz` writes one), and
* the HDF5 files themselves when h5py is importable.

:func:`synthetic_botnet` makes config-3-shaped graphs (heavy-tailed
background, max degree ~5.9k, a 10k-node P2P overlay of bots) when no data
is supplied.  ``GraphData`` drops ``num_edges`` / ``num_evils`` like the
reference (data.py:16-19); graphs are batched PyG-style.

Training (:func:`train`) follows train_botnet.py:190-346: GCNModel(in=1,
enc_sizes, classes=2, residual_hop, deg_norm, aggr, bias, final_type) called
as ``model(x[:, 0:1], edge_index, deg_K=x[:, 1])``; CrossEntropyLoss or
FocalLoss(alpha=1, gamma=2); Adam(lr, weight_decay); ReduceLROnPlateau(min,
factor 0.25, patience 1) and EarlyStopping(patience 5) on the validation
loss; per-graph metrics averaged over the validation / test graphs; the best
model kept (state_dict, not a pickled module) and tested at the end.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from .kernel.data import Batch, Data
from .kernel.train_eval import EarlyStopping

__all__ = ["GraphData", "GraphDataset", "GraphDataLoader", "save_npz", "synthetic_botnet",
           "make_botnet_graph", "FocalLoss", "CrossEntropyLoss",
           "accuracy", "recall", "precision", "f1_score",
           "false_positive_rate", "false_negative_rate", "evaluate", "train"]

_FIELDS = ("x", "y", "edge_index", "edge_y")


# ------------------------------------------------------------------ data
class GraphData(Data):
    """One botnet graph (gcn_meta/data/data.py): arrays -> tensors; the
    ``num_edges`` / ``num_evils`` attributes are dropped as in the reference."""

    def __init__(self, graph: dict):
        super().__init__(x=torch.as_tensor(np.asarray(graph["x"])),
                         edge_index=torch.as_tensor(np.asarray(graph["edge_index"])).long(),
                         y=torch.as_tensor(np.asarray(graph["y"])),
                         num_nodes=int(graph["num_nodes"]) if "num_nodes" in graph else None)
        self.edge_y = (torch.as_tensor(np.asarray(graph["edge_y"]))
                       if graph.get("edge_y") is not None else None)


class GraphDataset:
    """List of static graphs stored in one ``.npz`` (or HDF5, with h5py)."""

    def __init__(self, path: str, in_memory: bool = False):
        self.path = path
        if path.endswith(".npz"):
            self._npz = np.load(path, allow_pickle=False)
            self.num_graphs = int(self._npz["num_graphs"])
            self._h5 = None
            if in_memory:
                self._cache = [self._read_npz(i) for i in range(self.num_graphs)]
        else:
            try:
                import h5py
            except ImportError as e:  # pragma: no cover - h5py absent here
                raise RuntimeError(f"{path}: HDF5 needs h5py (absent); convert with "
                                   "scripts/botnet_h5_to_npz.py where h5py exists") from e
            self._h5 = h5py.File(path, "r")
            self.num_graphs = int(self._h5.attrs["num_graphs"])
            self._npz = None
        self.in_memory = in_memory and self._npz is not None

    def _read_npz(self, i):
        g = {k: self._npz[f"{i}/{k}"] for k in _FIELDS if f"{i}/{k}" in self._npz}
        if f"{i}/num_nodes" in self._npz:
            g["num_nodes"] = int(self._npz[f"{i}/num_nodes"])
        return g

    def __len__(self):
        return self.num_graphs

    def __getitem__(self, i: int) -> GraphData:
        if self.in_memory:
            return GraphData(self._cache[i])
        if self._npz is not None:
            return GraphData(self._read_npz(i))
        grp = self._h5[str(i)]  # h5group_to_dict (data/utils.py)
        g = {k: v[()] for k, v in grp.items()}
        g.update({k: v for k, v in grp.attrs.items()})
        return GraphData(g)


class GraphDataLoader:
    """Batches of graphs collated PyG-style (data/dataloader.py).
    ``share`` (data-parallel replicas, :class:`mgcn.dist.DataParallel`):
    each global batch is cut down to this rank's share of its graphs (None
    where the share is empty); ``generator``: the shuffle's RNG (every
    replica must draw the same order)."""

    def __init__(self, dataset, batch_size=1, shuffle=False, share=None, generator=None):
        self.dataset, self.batch_size, self.shuffle = dataset, int(batch_size), shuffle
        self.share, self.generator = share, generator

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.dataset)
        order = (torch.randperm(n, generator=self.generator).tolist() if self.shuffle
                 else list(range(n)))
        for i in range(0, n, self.batch_size):
            idx = order[i:i + self.batch_size]
            if self.share is not None:
                idx = self.share(idx)
                if not idx:
                    yield None
                    continue
            yield Batch.from_data_list([self.dataset[j] for j in idx])


def save_npz(graphs, path: str) -> None:
    """Write graphs ({x, y, edge_index, edge_y, num_nodes}) in the .npz layout."""
    arrays = {"num_graphs": np.array(len(graphs), dtype=np.int64)}
    for i, g in enumerate(graphs):
        for k in _FIELDS:
            if g.get(k) is not None:
                v = g[k]
                arrays[f"{i}/{k}"] = v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
        arrays[f"{i}/num_nodes"] = np.array(int(g["num_nodes"]), dtype=np.int64)
    np.savez(path, **arrays)


def make_botnet_graph(n_nodes: int = 143_107, bg_edges: int = 350_000, max_deg: int = 5_900,
                      p2p_nodes: int = 10_000, p2p_edges: int = 49_566, seed: int = 0):
    """Config-3 stand-in (the botnet HDF5 data is not in the reference tree):
    one graph of n_nodes with a heavy-tailed (Chung-Lu, power-law exponent
    ~2.1) background whose largest expected degree is max_deg
    (botnet_plot.ipynb:460 shows 5.9k), plus a p2p overlay of p2p_edges
    random edges among p2p_nodes bots (hard_attn_evil_edge.ipynb:203),
    symmetrised, self-loops appended (data_procs/loop.py).  Returns
    (edge_index, n_nodes, bot_mask)."""
    g = torch.Generator().manual_seed(seed)
    rank = torch.arange(1, n_nodes + 1, dtype=torch.float64)
    w = rank.pow(-1.0 / 1.1)
    w = w / w.sum()
    # expected degree of node i ~ 2 * bg_edges * w_i; clamp the head at max_deg
    w = torch.minimum(w, torch.full_like(w, max_deg / (2.0 * bg_edges)))
    perm = torch.randperm(n_nodes, generator=g)
    w = w[perm]
    s = torch.multinomial(w, bg_edges, replacement=True, generator=g)
    d = torch.multinomial(w, bg_edges, replacement=True, generator=g)
    bots = torch.randperm(n_nodes, generator=g)[:p2p_nodes]
    ps = bots[torch.randint(0, p2p_nodes, (p2p_edges,), generator=g)]
    pd = bots[torch.randint(0, p2p_nodes, (p2p_edges,), generator=g)]
    s, d = torch.cat([s, ps]), torch.cat([d, pd])
    loops = torch.arange(n_nodes)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    mask = torch.zeros(n_nodes, dtype=torch.bool)
    mask[bots] = True
    return ei, n_nodes, mask


def synthetic_botnet(n_graphs: int = 2, seed: int = 0, **kw) -> list[dict]:
    """Config-3-shaped graphs in the dataset's field layout: x = [1, degree]
    (f4), y = bot mask (u1), edge_y = 1 on bot-bot edges."""
    graphs = []
    for i in range(n_graphs):
        ei, n, mask = make_botnet_graph(seed=seed + i, **kw)
        deg = torch.bincount(ei[0], minlength=n).to(torch.float32)
        x = torch.stack([torch.ones(n), deg], 1)
        edge_y = (mask[ei[0]] & mask[ei[1]]).to(torch.uint8)
        graphs.append({"x": x, "y": mask.to(torch.uint8), "edge_index": ei, "edge_y": edge_y,
                       "num_nodes": n})
    return graphs


# ------------------------------------------------------------------ metrics
# optim/metrics.py: binary classification, pred / target LongTensors
def accuracy(pred, target):
    return (pred == target).sum().item() / target.numel()


def true_positive(pred, target):
    return (target[pred == 1] == 1).sum().item()


def false_positive(pred, target):
    return (target[pred == 1] == 0).sum().item()


def true_negative(pred, target):
    return (target[pred == 0] == 0).sum().item()


def false_negative(pred, target):
    return (target[pred == 0] == 1).sum().item()


def _div(a, b):
    # metrics.py:32,53,60 divide unguarded (ZeroDivisionError on a graph
    # with no positives / negatives); nan here, so one such graph cannot
    # abort an evaluation.
    return a / b if b != 0 else float("nan")


def recall(pred, target):
    return _div(true_positive(pred, target), (target == 1).sum().item())


def precision(pred, target):
    p = (pred == 1).sum().item()
    return true_positive(pred, target) / p if p != 0 else -1  # the reference's -1


def f1_score(pred, target):
    prec, rec = precision(pred, target), recall(pred, target)
    return 2 * (prec * rec) / (prec + rec) if (prec + rec) != 0 else 0


def false_positive_rate(pred, target):
    return _div(false_positive(pred, target), (target == 0).sum().item())


def false_negative_rate(pred, target):
    return _div(false_negative(pred, target), (target == 1).sum().item())


class FocalLoss(nn.Module):
    """optim/focal_loss.py: -alpha (1 - p_t)^gamma log p_t on softmax + 1e-8."""

    def __init__(self, alpha=0.25, gamma=2.0, reduction="mean"):
        super().__init__()
        assert reduction in ("mean", "sum", "none")
        self.alpha, self.gamma, self.reduction, self.eps = alpha, gamma, reduction, 1e-8

    def forward(self, scores, target):
        probs = F.softmax(scores, dim=1) + self.eps
        probs = probs[torch.arange(len(target), device=target.device), target]
        loss = -self.alpha * torch.pow(1 - probs, self.gamma) * torch.log(probs)
        if self.reduction == "mean":
            return loss.mean()
        if self.reduction == "sum":
            return loss.sum()
        return loss


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss() of train_botnet.py:290 (no class weights) as
    -log_softmax(scores)[i, target_i] reduced with a plain mean/sum.  Same
    value within fp32 rounding; torch's fused nll_loss forward/backward runs
    as a single-workgroup reduction on this device (0.26 + 0.13 ms for the
    286k-node config-3 batch, 7 % of the step) while these are chip-wide."""

    def __init__(self, reduction="mean"):
        super().__init__()
        assert reduction in ("mean", "sum", "none")
        self.reduction = reduction

    def forward(self, scores, target):
        nll = -F.log_softmax(scores, dim=1).gather(1, target.view(-1, 1)).view(-1)
        if self.reduction == "mean":
            return nll.mean()
        if self.reduction == "sum":
            return nll.sum()
        return nll


# ------------------------------------------------------------------ loop
def _forward(model, batch):
    return model(batch.x[:, 0].view(-1, 1), batch.edge_index, deg_K=batch.x[:, 1])


@torch.no_grad()
def evaluate(model, loader, criterion, device, dp=None):
    """train_botnet.py:249-283: loss and metrics per graph, averaged.  With
    ``dp`` (data-parallel replicas) every rank evaluates its share of the
    graphs and the sums are combined (the same averages on every rank)."""
    model.eval()
    keys = ("loss", "acc", "fpr", "fnr", "rec", "prc", "f1")
    tot = dict.fromkeys(keys, 0.0)
    n = 0
    for batch in loader:
        if batch is None:
            continue
        batch.to(device)
        x = _forward(model, batch)
        y = batch.y.long()
        pred = x.argmax(dim=1)
        vals = (float(criterion(x, y)), accuracy(pred, y), false_positive_rate(pred, y),
                false_negative_rate(pred, y), recall(pred, y), precision(pred, y),
                f1_score(pred, y))
        for k, v in zip(keys, vals):
            tot[k] += v
        n += 1
    if dp is not None and dp.world > 1:
        sums = dp.all_sum([tot[k] for k in keys] + [n])
        tot, n = dict(zip(keys, sums[:-1])), int(sums[-1])
    return {k: v / max(n, 1) for k, v in tot.items()}


def _time_since(start):
    s = time.time() - start
    m = math.floor(s / 60)
    return f"{m}m {s - 60 * m:.0f}s"


def train(train_ds, val_ds, test_ds, enc_sizes=(32,) * 8, residual_hop=0, deg_norm="sm",
          aggr="add", bias=False, dropout=0.0, final="proj", act="relu", layer_act="relu",
          lr=1e-3, weight_decay=5e-4, epochs=5, batch_size=1, shuffle=False, focal=False,
          device="cuda:0", save_path=None, log=print, dp=False, group=None, seed=None):
    """The train_botnet.py loop on mgcn.models.GCNModel; returns a history
    dict (per-epoch train loss and validation metrics, final test metrics).

    ``dp=True`` (torch.distributed initialised, one process per GPU): the
    same loop as data-parallel replicas (:class:`mgcn.dist.DataParallel`):
    rank 0's initial parameters are broadcast, every global batch of
    ``batch_size`` graphs is dealt out graph by graph, each rank's summed
    loss is divided by the global node count (so the all-reduced gradient is
    the single-process batch-mean one), every rank steps the same Adam;
    validation / test graphs are split and their metric sums combined.
    ``seed``: torch.manual_seed before the model is built (and the shuffle
    order's generator)."""
    from .models import GCNModel
    if seed is not None:
        torch.manual_seed(seed)
    model = GCNModel(1, list(enc_sizes), 2, non_linear=act, non_linear_layer_wise=layer_act,
                     residual_hop=residual_hop, dropout=dropout, final_type=final,
                     pred_on="node", deg_norm=deg_norm, aggr=aggr, bias=bool(bias)).to(device)
    dpr = None
    if dp:
        from .dist import DataParallel
        dpr = DataParallel(model.parameters(), group)
        dpr.broadcast_params()
    Crit = FocalLoss if focal else CrossEntropyLoss
    kw = {"alpha": 1, "gamma": 2} if focal else {}
    criterion = Crit(**kw)
    crit_sum = Crit(reduction="sum", **kw)
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.25, patience=1)
    stopper = EarlyStopping(patience=5, verbose=True)
    gen = torch.Generator().manual_seed(seed if seed is not None else 0) if dpr else None
    share = dpr.share if dpr is not None and dpr.world > 1 else None
    train_loader = GraphDataLoader(train_ds, batch_size=batch_size, shuffle=shuffle, share=share,
                                   generator=gen)
    val_loader = GraphDataLoader(val_ds, batch_size=1, share=share)
    test_loader = GraphDataLoader(test_ds, batch_size=1, share=share)
    hist = {"train_loss": [], "val": []}
    best_state, best_epoch = None, 0
    start = time.time()
    for ep in range(epochs):
        model.train()
        loss_sum, graphs = 0.0, 0
        for batch in train_loader:
            opt.zero_grad()
            if share is None:
                batch.to(device)
                x = _forward(model, batch)
                loss = criterion(x, batch.y.long())
                loss.backward()
                opt.step()
                loss_sum += loss.item()
            else:
                # this rank's graphs: summed loss / the global batch's node count
                n_loc = 0 if batch is None else int(batch.num_nodes)
                (n_glob,) = dpr.all_sum([n_loc])
                local = 0.0
                if batch is not None:
                    batch.to(device)
                    x = _forward(model, batch)
                    loss = crit_sum(x, batch.y.long()) / n_glob
                    loss.backward()
                    local = loss.item()
                dpr.reduce_grads()
                opt.step()
                loss_sum += dpr.all_sum([local])[0]
            graphs += batch_size
        hist["train_loss"].append(loss_sum / max(graphs, 1))
        m = evaluate(model, val_loader, criterion, device, dpr)
        hist["val"].append(m)
        log(f"epoch {ep + 1}: train loss {hist['train_loss'][-1]:.5f}, val loss "
            f"{m['loss']:.5f}, acc {m['acc']:.5f}, f1 {m['f1']:.5f} ({_time_since(start)})")
        sched.step(m["loss"])
        stopper(m["loss"])
        if stopper.improved:
            best_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
            best_epoch = ep
            # the replicas hold identical states: one writer (rank 0), so
            # ranks on a shared filesystem never write the file concurrently
            if save_path and (dpr is None or dpr.rank == 0):
                torch.save(best_state, save_path)
        elif stopper.early_stop:
            log("Early stopping here.")
            break
    if best_state is not None:
        model.load_state_dict(best_state)
    hist["best_epoch"] = best_epoch
    hist["test"] = evaluate(model, test_loader, criterion, device, dpr)
    log(f"test (best epoch {best_epoch + 1}): " +
        ", ".join(f"{k} {v:.5f}" for k, v in hist["test"].items()))
    return hist
