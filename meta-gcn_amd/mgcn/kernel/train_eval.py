"""Config-1 driver: 10-fold cross-validation of a graph-classification model
(kernel/train_eval.py:17-188, kernel/main.py:76-116 of the reference).

Same protocol as the reference:
* ``k_fold`` -- sklearn ``StratifiedKFold(folds, shuffle=True,
  random_state=12345)`` on the graph labels; fold i tests on split i,
  validates on split i - 1 and trains on the rest (train_eval.py:120-135);
* per fold: ``model.reset_parameters()``, Adam(lr, weight_decay), one train
  pass + val/test evaluation per epoch, lr *= ``lr_decay_factor`` every
  ``lr_decay_step_size`` epochs, optional early stopping on the val loss
  (``EarlyStopping``, src/gcn_meta/optim/earlystop.py);
* loss ``nll_loss`` on the model's log-softmax output; per fold the epoch of
  best val accuracy selects val/test loss and test accuracy; the means and
  standard deviations over folds are returned.

``cross_validation_with_val_set`` returns the SIX values train_eval.py:106
returns; the reference's main.py:93 unpacks three and crashes after the
first sweep -- ``run_sweep`` here unpacks six.
"""
from __future__ import annotations

import time

import torch
import torch.nn.functional as F
from torch import tensor

from .data import DataLoader, DenseDataLoader


class EarlyStopping:
    """Stop when the monitored metric has not improved for ``patience``
    calls; ``patience < 0`` disables (src/gcn_meta/optim/earlystop.py)."""

    def __init__(self, patience=7, mode="min", verbose=False, logger=None):
        assert mode in ("min", "max")
        self.patience, self.mode, self.verbose = patience, mode, verbose
        self.logging = logger.info if logger else print
        self.counter = 0
        self.best = None
        self.improved = False
        self.early_stop = False

    def __call__(self, val_metric):
        if self.patience is None or self.patience < 0:
            return
        if self.best is None:
            self.best, self.improved = val_metric, True
        elif (self.mode == "min" and val_metric < self.best) or \
                (self.mode == "max" and val_metric > self.best):
            self.best, self.improved, self.counter = val_metric, True, 0
        else:
            self.improved = False
            self.counter += 1
            if self.verbose:
                self.logging(f"EarlyStopping counter: {self.counter} out of {self.patience}")
            if self.counter >= self.patience:
                self.early_stop = True


def k_fold(dataset, folds, random_state=12345):
    """(train, test, val) index lists per fold (train_eval.py:120-135)."""
    from sklearn.model_selection import StratifiedKFold
    skf = StratifiedKFold(folds, shuffle=True, random_state=random_state)
    y = dataset.data.y
    test_indices, train_indices = [], []
    for _, idx in skf.split(torch.zeros(len(dataset)), y):
        test_indices.append(torch.from_numpy(idx))
    val_indices = [test_indices[i - 1] for i in range(folds)]
    for i in range(folds):
        train_mask = torch.ones(len(dataset), dtype=torch.bool)
        train_mask[test_indices[i]] = 0
        train_mask[val_indices[i]] = 0
        train_indices.append(train_mask.nonzero().view(-1))
    return train_indices, test_indices, val_indices


def num_graphs(data):
    return data.num_graphs if data.batch is not None else data.x.size(0)


def train(model, optimizer, loader, device, dp=None):
    """One epoch (train_eval.py:134-148).  ``dp`` (:class:`mgcn.dist.
    DataParallel`, the loader built with its ``share``): each rank sums the
    nll of its share of a batch over the batch's GLOBAL graph count, the
    gradients are all-reduced, every rank steps the same optimizer -- the
    single-process step within fp32 summation order."""
    model.train()
    total = 0.0
    if dp is not None and dp.world > 1:
        for data in loader:
            optimizer.zero_grad()
            n_loc = 0 if data is None else num_graphs(data)
            (n_glob,) = dp.all_sum([n_loc])
            local = 0.0
            if data is not None:
                data = data.to(device)
                loss = F.nll_loss(model(data), data.y.view(-1), reduction="sum") / n_glob
                loss.backward()
                local = loss.item() * n_glob
            dp.reduce_grads()
            total += dp.all_sum([local])[0]
            optimizer.step()
        return total / len(loader.dataset)
    for data in loader:
        optimizer.zero_grad()
        data = data.to(device)
        out = model(data)
        loss = F.nll_loss(out, data.y.view(-1))
        loss.backward()
        total += loss.item() * num_graphs(data)
        optimizer.step()
    return total / len(loader.dataset)


def _combine(dp, *vals):
    return tuple(dp.all_sum(vals)) if dp is not None and dp.world > 1 else vals


@torch.no_grad()
def eval_acc(model, loader, device, dp=None):
    model.eval()
    correct = 0
    for data in loader:
        if data is None:
            continue
        data = data.to(device)
        pred = model(data).max(1)[1]
        correct += pred.eq(data.y.view(-1)).sum().item()
    (correct,) = _combine(dp, correct)
    return correct / len(loader.dataset)


@torch.no_grad()
def eval_loss(model, loader, device, dp=None):
    model.eval()
    loss = 0.0
    for data in loader:
        if data is None:
            continue
        data = data.to(device)
        loss += F.nll_loss(model(data), data.y.view(-1), reduction="sum").item()
    (loss,) = _combine(dp, loss)
    return loss / len(loader.dataset)


@torch.no_grad()
def eval_loss_acc(model, loader, device, dp=None):
    model.eval()
    loss, correct = 0.0, 0
    for data in loader:
        if data is None:
            continue
        data = data.to(device)
        out = model(data)
        loss += F.nll_loss(out, data.y.view(-1), reduction="sum").item()
        correct += out.max(1)[1].eq(data.y.view(-1)).sum().item()
    loss, correct = _combine(dp, loss, correct)
    return loss / len(loader.dataset), correct / len(loader.dataset)


def cross_validation_with_val_set(dataset, model, folds, epochs, batch_size, lr,
                                  lr_decay_factor, lr_decay_step_size, weight_decay,
                                  random_state=12345, es_patience=-1, logger=None,
                                  log_details=False, device=None, dp=False, group=None,
                                  seed=0):
    """Returns (val_loss_mean, val_acc_mean, val_acc_std, test_loss_mean,
    test_acc_mean, test_acc_std) -- train_eval.py:17-117.

    ``dp=True`` (torch.distributed initialised, one process per GPU): every
    fold trains as data-parallel replicas (:class:`mgcn.dist.DataParallel`:
    rank 0's reset parameters broadcast, each batch dealt out graph by
    graph, gradients all-reduced, the shuffle drawn from a generator seeded
    with ``seed`` on every rank), evaluation split and combined."""
    logging = logger.info if logger is not None else print
    device = device or torch.device("cuda")
    val_losses, val_accs, test_losses, test_accs, durations = [], [], [], [], []
    for fold, (train_idx, test_idx, val_idx) in enumerate(
            zip(*k_fold(dataset, folds, random_state))):
        Loader = DenseDataLoader if 'adj' in dataset[0] else DataLoader  # train_eval.py:32-39
        model.to(device).reset_parameters()
        dpr = share = gen = None
        if dp:
            from ..dist import DataParallel
            dpr = DataParallel(model.parameters(), group)
            dpr.broadcast_params()
            gen = torch.Generator().manual_seed(seed + fold)  # the same order on every rank
            if dpr.world > 1:
                share = dpr.share
        train_loader = Loader(dataset[train_idx], batch_size, shuffle=True, share=share,
                              generator=gen)
        val_loader = Loader(dataset[val_idx], batch_size, shuffle=False, share=share)
        test_loader = Loader(dataset[test_idx], batch_size, shuffle=False, share=share)
        optimizer = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
        stopper = EarlyStopping(patience=es_patience, mode="min", verbose=True)
        if torch.device(device).type == "cuda":
            torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for epoch in range(1, epochs + 1):
            train_loss = train(model, optimizer, train_loader, device, dpr)
            val_loss, val_acc = eval_loss_acc(model, val_loader, device, dpr)
            val_losses.append(val_loss)
            val_accs.append(val_acc)
            test_loss, test_acc = eval_loss_acc(model, test_loader, device, dpr)
            test_losses.append(test_loss)
            test_accs.append(test_acc)
            if log_details:
                logging(f"Fold {fold + 1:02d} / Epoch {epoch + 1:03d}: Train loss: "
                        f"{train_loss:.4f}, Val loss: {val_loss:.4f}, Val acc: {val_acc:.3f}, "
                        f"Test loss: {test_loss:.4f}, Test acc: {test_acc:.3f}")
            if epoch % lr_decay_step_size == 0:
                for pg in optimizer.param_groups:
                    pg["lr"] = lr_decay_factor * pg["lr"]
            stopper(val_loss)
            if stopper.early_stop:
                break
        if torch.device(device).type == "cuda":
            torch.cuda.synchronize(device)
        durations.append(time.perf_counter() - t0)
    # (the reference views the per-epoch lists as [folds, epochs]: early
    # stopping would break that reshape; here the runs must be complete too)
    val_loss, val_acc = tensor(val_losses).view(folds, epochs), tensor(val_accs).view(folds, epochs)
    test_loss = tensor(test_losses).view(folds, epochs)
    test_acc = tensor(test_accs).view(folds, epochs)
    duration = tensor(durations)
    val_acc, argmin = val_acc.max(dim=1)
    rows = torch.arange(folds, dtype=torch.long)
    val_loss, test_loss, test_acc = val_loss[rows, argmin], test_loss[rows, argmin], \
        test_acc[rows, argmin]
    out = (val_loss.mean().item(), val_acc.mean().item(), val_acc.std().item(),
           test_loss.mean().item(), test_acc.mean().item(), test_acc.std().item())
    logging("Best epoch for each fold: " + " ".join(str(i + 1) for i in argmin.tolist()))
    logging("Val Loss: {:.4f}, Val Accuracy: {:.3f} ± {:.3f}, Test Loss: {:.4f}, "
            "Test Accuracy: {:.3f} ± {:.3f}, Duration: {:.3f}".format(
                *out, duration.mean().item()))
    return out


def run_sweep(datasets, nets, layers, hiddens, folds=10, epochs=100, batch_size=128, lr=0.01,
              lr_decay_factor=0.5, lr_decay_step_size=50, random_state=12345, es_patience=-1,
              add_sl=False, root=None, synthetic=None, device=None):
    """kernel/main.py:76-116: best (val loss) hyper-parameters per
    (dataset, net); returns the result lines."""
    from itertools import product

    from .data import get_dataset
    results = []
    for name, Net in product(datasets, nets):
        best, best_hyper = (float("inf"), 0.0, 0.0), None
        for num_layers, hidden in product(layers, hiddens):
            dataset = get_dataset(name, root=root, sparse=Net.__name__ != "DiffPool",
                                  x_deg=True, add_sl=add_sl, synthetic=synthetic)
            model = Net(dataset, num_layers, hidden)
            val_loss, _, _, _, test_acc, test_std = cross_validation_with_val_set(
                dataset, model, folds=folds, epochs=epochs, batch_size=batch_size, lr=lr,
                lr_decay_factor=lr_decay_factor, lr_decay_step_size=lr_decay_step_size,
                weight_decay=0, random_state=random_state, es_patience=es_patience,
                device=device)
            if val_loss < best[0]:
                best, best_hyper = (val_loss, test_acc, test_std), (num_layers, hidden)
        results.append(f"{name} - {Net.__name__} {best_hyper}: {best[1]:.3f} ± {best[2]:.3f}")
    return results
