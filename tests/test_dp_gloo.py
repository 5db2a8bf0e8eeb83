"""Data-parallel replicas (mgcn.dist.DataParallel) and the sharded module
surface (mgcn.dist.ShardedGCNStack) under gloo on the CPU, world 2 and 4,
against world 1 of the same code.

* the config-1 CV loop (mgcn.kernel.train_eval, kernel/train_eval.py:17-148)
  with ``dp=True``: each batch dealt out graph by graph, summed nll over the
  global graph count, gradients all-reduced, Adam on every rank -- after
  whole epochs the parameters, losses and accuracies equal world 1 within
  fp32 summation order (the model is a small pure-torch graph classifier:
  the replica logic is model-agnostic, and libmgcn needs a GPU);
* ShardedGCNStack wrapping a GCNStack: forward rows and dX rows bit for bit
  world 1's, gradients (after allreduce_grads) within fp32 tolerance, on the
  wrapped module's own parameters (local compute: tests/cpu_backend.py).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _MeanPoolNet(torch.nn.Module):
    """mean pool of x per graph -> Linear -> ReLU -> Linear -> log_softmax."""

    def __init__(self, fin, hid, classes):
        super().__init__()
        self.l1 = torch.nn.Linear(fin, hid)
        self.l2 = torch.nn.Linear(hid, classes)

    def reset_parameters(self):
        g = torch.Generator().manual_seed(7)
        for p in self.parameters():
            with torch.no_grad():
                p.copy_(torch.randn(p.shape, generator=g) * 0.3)

    def forward(self, data):
        G = data.num_graphs
        s = torch.zeros(G, data.x.size(1)).index_add_(0, data.batch, data.x)
        c = torch.bincount(data.batch, minlength=G).clamp(min=1).to(s.dtype)
        h = torch.relu(self.l1(s / c[:, None]))
        return torch.log_softmax(self.l2(h), dim=1)


def _cv_worker(rank, world, port, q):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from mgcn.kernel.data import get_dataset
        from mgcn.kernel.train_eval import cross_validation_with_val_set
        ds = get_dataset("MUTAG", synthetic=True)
        model = _MeanPoolNet(ds.num_features, 16, ds.num_classes)
        out = cross_validation_with_val_set(ds, model, folds=3, epochs=3, batch_size=32, lr=0.01,
                                            lr_decay_factor=0.5, lr_decay_step_size=2,
                                            weight_decay=0, device=torch.device("cpu"),
                                            dp=True, seed=3, logger=_Quiet())
        q.put({"rank": rank, "out": out,
               "params": [p.detach().numpy().copy() for p in model.parameters()]})
    finally:
        dist.destroy_process_group()


class _Quiet:
    def info(self, *a):
        pass


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r["rank"])


@pytest.mark.parametrize("world", [2, 4])
def test_cv_loop_data_parallel_matches_one_process(world):
    one = _spawn(_cv_worker, 1)[0]
    many = _spawn(_cv_worker, world)
    for r in many:
        # every replica ends with the same parameters as one process
        for a, b in zip(r["params"], one["params"]):
            np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(r["out"], one["out"], rtol=1e-4, atol=1e-5)
    for r in many[1:]:  # replicas identical to each other, bit for bit
        for a, b in zip(r["params"], many[0]["params"]):
            np.testing.assert_array_equal(a, b)


def _stack_worker(rank, world, port, q, aggr):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd"),
                    HERE]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from cpu_backend import CpuBackend
        from mgcn.dist import ShardedGCNStack
        from mgcn.models import GCNLayer, GCNStack
        g = torch.Generator().manual_seed(0)
        N, F = 300, 16
        s = torch.randint(0, N, (1500,), generator=g)
        d = torch.randint(0, N, (1500,), generator=g)
        loops = torch.arange(N)
        ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
        X = torch.randn(N, F, generator=g)
        dY = torch.randn(N, F, generator=g)
        torch.manual_seed(1)
        stack = GCNStack([GCNLayer(F, F, deg_norm='sm', aggr=aggr, bias=True,
                                   non_linear='relu' if i < 2 else 'none') for i in range(3)])
        m = ShardedGCNStack(stack, ei, N, backend=CpuBackend(), device=torch.device("cpu"))
        xl = m.local_rows(X).clone().requires_grad_(True)
        y = m(x_local=xl)
        y.backward(m.local_rows(dY))
        m.allreduce_grads()
        q.put({"rank": rank, "lo": m.shard.lo, "hi": m.shard.hi, "fused": m.fused,
               "y": y.detach().numpy(), "dx": xl.grad.numpy(),
               "grads": [p.grad.numpy().copy() for p in stack.parameters()],
               "names": [n for n, _ in stack.named_parameters()]})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,aggr", [(2, "add"), (4, "mean"), (2, "max")])
def test_sharded_gcn_stack_module_matches_one_process(world, aggr):
    one = _spawn(_stack_worker, 1, aggr)[0]
    many = _spawn(_stack_worker, world, aggr)
    assert one["fused"] == (aggr != "max")
    assert one["names"] == ["layers.0.gcn.node_models.0.weight_node",
                            "layers.0.gcn.node_models.0.bias",
                            "layers.1.gcn.node_models.0.weight_node",
                            "layers.1.gcn.node_models.0.bias",
                            "layers.2.gcn.node_models.0.weight_node",
                            "layers.2.gcn.node_models.0.bias"]
    for r in many:
        lo, hi = r["lo"], r["hi"]
        np.testing.assert_array_equal(r["y"], one["y"][lo:hi])
        np.testing.assert_array_equal(r["dx"], one["dx"][lo:hi])
        for a, b in zip(r["grads"], one["grads"]):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5 * max(1, np.abs(b).max()))


def _grad_flag_worker(rank, world, port, q):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mgcn.dist import DataParallel
        a = torch.nn.Parameter(torch.ones(3))      # every rank takes a gradient
        b = torch.nn.Parameter(torch.ones(2))      # only rank 0 does
        c = torch.nn.Parameter(torch.ones(4))      # no rank does
        dp = DataParallel([a, b, c])
        loss = (a * (rank + 1)).sum() + ((b * 2).sum() if rank == 0 else 0.0)
        loss.backward()
        dp.reduce_grads()
        q.put({"rank": rank, "a": a.grad.numpy().copy(), "b": b.grad.numpy().copy(),
               "c": c.grad is None})
    finally:
        dist.destroy_process_group()


def test_data_parallel_keeps_untouched_grads_none():
    """A parameter no rank gave a gradient keeps grad None after reduce_grads
    (as in one process, so Adam skips it); one that only some ranks touched
    gets the sum (no zero grads for untouched parameters)."""
    res = _spawn(_grad_flag_worker, 2)
    for r in res:
        np.testing.assert_array_equal(r["a"], np.full(3, 3.0))
        np.testing.assert_array_equal(r["b"], np.full(2, 2.0))
        assert r["c"]
