"""The RCCL branch of mgcn.dist, executed on the one GPU a builder box has.

The 8-GPU node is the driver's; every other multi-rank test runs its
collectives over gloo.  Here a ONE-rank `nccl` (= RCCL on ROCm) process group
with mgcn.dist.set_force_collectives(True) makes the sharded stack issue every
collective a rank of a multi-GPU group issues -- the chunked
all_gather_into_tensor(async_op=True) of each layer's rows (dense), the packed
exchange's size gather and payload gather (packed; later steps at the learnt
speculative capacity, and re-sent when it is too small), the all_gather of the
inverse degrees at setup, the bucketed all_reduce of the gradients, and
DataParallel's all_sum / broadcast / has-grad-flagged all_reduce -- on RCCL's
stream, over HIP tensors.  The results must equal, bit for bit, the same
model in a one-rank gloo group without forced collectives (where world 1
copies instead): an all-gather or all-reduce over one rank is the identity.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem(N=4000, pairs=20000, F=128, L=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    s = torch.randint(0, N, (pairs,), generator=g)
    d = torch.randint(0, N, (pairs,), generator=g)
    loops = torch.arange(N)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    X = torch.randn(N, F, generator=g)
    Ws = [torch.randn(F, F, generator=g) * 0.2 for _ in range(L)]
    bs = [torch.randn(F, generator=g) * 0.1 for _ in range(L)]
    dY = torch.randn(N, F, generator=g)
    return ei, N, X, Ws, bs, dY


def _child(backend, force, port, q):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from mgcn import dist as mdist
        mdist.set_force_collectives(force)
        res = {"backend": dist.get_backend()}
        for F, aggr in ((128, "add"), (128, "mean"), (256, "add")):
            ei, N, X, Ws, bs, dY = _problem(F=F, seed=F)
            # F = 256: chunks packed in one pass (mgcn_pack_rows, below its
            # size threshold here); F = 128: the two passes
            mdist.FUSED_PACK_MIN_BYTES = 0 if F == 256 else 32 << 20
            for pack in (False, True):
                mdist.set_pack_exchange(pack)
                m = mdist.ShardedGCN(ei, N, Ws, bs, device=dev, aggr=aggr, chunks=3)
                assert m.fused
                key = f"{F}-{aggr}-{'packed' if pack else 'dense'}"
                # packed: step 2 sends every chunk at the sizes step 1 learnt
                # (speculative capacity) and learns half of them (slack -50 %),
                # step 3 sends at those (every chunk re-sent at its true
                # size): each step the same bits
                for step, slack in enumerate((0.02, -0.5, -0.5) if pack else (0.02,)):
                    mdist.SPEC_SLACK = slack
                    for p in m.params():
                        p.grad = None
                    Xl = m.local_rows(X).requires_grad_(True)
                    out = m.forward(Xl)
                    out.backward(m.local_rows(dY))
                    mdist.allreduce_grads(m.params())
                    torch.cuda.synchronize()
                    got = [out.detach().cpu().numpy(), Xl.grad.cpu().numpy()] + \
                        [p.grad.cpu().numpy() for p in m.params()]
                    if step == 0:
                        res[key] = got
                    else:
                        res[f"{key}-step{step}-same"] = all(
                            np.array_equal(a, b) for a, b in zip(got, res[key]))
                mdist.SPEC_SLACK = 0.02
        res["packed_words"] = dict(mdist.STATS)
        # DataParallel: all_sum, broadcast, the flagged gradient all-reduce
        lin = torch.nn.Linear(8, 4).to(dev)
        unused = torch.nn.Parameter(torch.ones(3, device=dev))
        dp = mdist.DataParallel(list(lin.parameters()) + [unused])
        dp.broadcast_params()
        lin(torch.ones(2, 8, device=dev)).sum().backward()
        dp.reduce_grads()
        res["dp"] = [lin.weight.grad.cpu().numpy(), unused.grad is None,
                     dp.all_sum([1.5, 2.0])]
        q.put(res)
    finally:
        dist.destroy_process_group()


def _run(backend, force):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(backend, force, _free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    return res


def test_rccl_one_rank_forced_collectives_match_world_one(cuda):
    ref = _run("gloo", False)
    rc = _run("nccl", True)
    assert rc["backend"] == "nccl"
    # the packed exchange really ran (sizes gathered, payload sent packed)
    assert 0 < rc["packed_words"]["sent_words"] < rc["packed_words"]["dense_words"]
    # the speculative-capacity steps: used, the too-small one re-sent, same bits
    assert rc["packed_words"].get("spec_chunks", 0) > 0, rc["packed_words"]
    assert rc["packed_words"].get("spec_resent", 0) > 0, rc["packed_words"]
    assert rc["packed_words"].get("pack_one_pass", 0) > 0, rc["packed_words"]
    for key in ref:
        if key in ("backend", "packed_words", "dp"):
            continue
        if key.endswith("-same"):
            assert rc[key] and ref[key], key
            continue
        for a, b in zip(rc[key], ref[key]):
            np.testing.assert_array_equal(a, b, err_msg=key)
    np.testing.assert_array_equal(rc["dp"][0], ref["dp"][0])
    assert rc["dp"][1] and ref["dp"][1]  # no rank gave a grad: stays None
    assert rc["dp"][2] == [1.5, 2.0]
