"""Data-parallel replicas and the sharded module surface on the GPU with
libmgcn: two ranks sharing cuda:0 (gloo carries HIP tensors; the 8-GPU runs
use RCCL through the same code) against one rank.

* the config-3 botnet loop (mgcn.botnet.train, src/run/train_botnet.py:219-294)
  with ``dp=True``: two epochs of GCNModel + CE + Adam on tiny botnet-shaped
  graphs (batch of 2 graphs: one per rank) -- train losses, validation /
  test metrics and the final parameters equal one process within fp32
  summation order;
* ShardedGCNStack wrapping a GCNStack on libmgcn: forward and dX rows bit
  for bit the single-device GCNStack's, the wrapped parameters' gradients
  (after allreduce_grads) within fp32 tolerance.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # several ranks share cuda:0 at HIP's default hardware queue count (round
    # 6: the round-5 workaround of two queues per rank is gone; the r4g abort
    # it guarded against is re-run at the default).
    # MGCN_TEST_HW_QUEUES=n restores a per-rank queue cap for an A/B.
    if os.environ.get("MGCN_TEST_HW_QUEUES"):
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ["MGCN_TEST_HW_QUEUES"]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)


def _botnet_worker(rank, world, port, q, paths):
    _init(rank, world, port)
    try:
        from mgcn.botnet import GraphDataset, train
        tr, va, te = (GraphDataset(p, in_memory=True) for p in paths)
        hist = train(tr, va, te, enc_sizes=(32,) * 4, residual_hop=1, epochs=2, batch_size=2,
                     shuffle=True, device="cuda:0", dp=True, seed=5, log=lambda *a: None)
        q.put({"rank": rank, "train_loss": hist["train_loss"],
               "val": [v["loss"] for v in hist["val"]], "test": hist["test"]})
    finally:
        dist.destroy_process_group()


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


def test_botnet_training_data_parallel_matches_one_process(cuda, tmp_path):
    from mgcn import botnet
    kw = dict(n_nodes=3000, bg_edges=9000, max_deg=300, p2p_nodes=300, p2p_edges=900)
    paths = []
    for name, n, seed in (("train", 4, 0), ("val", 2, 10), ("test", 2, 20)):
        p = str(tmp_path / f"{name}.npz")
        botnet.save_npz(botnet.synthetic_botnet(n, seed=seed, **kw), p)
        paths.append(p)
    one = _spawn(_botnet_worker, 1, paths)[0]
    two = _spawn(_botnet_worker, 2, paths)
    for r in two:
        np.testing.assert_allclose(r["train_loss"], one["train_loss"], rtol=1e-4)
        np.testing.assert_allclose(r["val"], one["val"], rtol=1e-4)
        for k, v in one["test"].items():
            if np.isfinite(v):
                assert abs(r["test"][k] - v) <= 1e-4 * max(1.0, abs(v)), (k, r["test"][k], v)


def _stack_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from mgcn.dist import ShardedGCNStack
        from mgcn.models import GCNLayer, GCNStack
        g = torch.Generator().manual_seed(0)
        N, F = 4000, 128
        s = torch.randint(0, N, (20000,), generator=g)
        d = torch.randint(0, N, (20000,), generator=g)
        loops = torch.arange(N)
        ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
        X = torch.randn(N, F, generator=g)
        dY = torch.randn(N, F, generator=g)
        torch.manual_seed(1)
        stack = GCNStack([GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                                   non_linear='relu' if i < 2 else 'none')
                          for i in range(3)]).cuda()
        res = {"rank": rank}
        if world == 1:  # the single-device module itself
            x = X.cuda().requires_grad_(True)
            y = stack(x, ei.cuda())
            y.backward(dY.cuda())
            res.update(lo=0, hi=N, y=y.detach().cpu().numpy(), dx=x.grad.cpu().numpy())
        else:
            m = ShardedGCNStack(stack, ei.cuda(), N)
            assert m.fused
            xl = m.local_rows(X.cuda()).clone().requires_grad_(True)
            y = m(x_local=xl)
            y.backward(m.local_rows(dY.cuda()))
            m.allreduce_grads()
            res.update(lo=m.shard.lo, hi=m.shard.hi, y=y.detach().cpu().numpy(),
                       dx=xl.grad.cpu().numpy())
        torch.cuda.synchronize()
        res["grads"] = [p.grad.cpu().numpy() for p in stack.parameters()]
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_sharded_gcn_stack_module_matches_single_device(cuda):
    one = _spawn(_stack_worker, 1)[0]
    two = _spawn(_stack_worker, 2)
    for r in two:
        lo, hi = r["lo"], r["hi"]
        np.testing.assert_array_equal(r["y"], one["y"][lo:hi])
        np.testing.assert_array_equal(r["dx"], one["dx"][lo:hi])
        for a, b in zip(r["grads"], one["grads"]):
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4 * max(1, np.abs(b).max()))
