"""Destination-range sharding (mgcn.dist) under gloo, world size 2 and 4, on
the CPU: sharded forward outputs must equal the single-process run bit for
bit (every destination row is local, COO order kept) and so must the
per-rank dH; replicated-parameter gradients (all-reduced partial sums) match
within fp32 tolerance.  Local compute is the CPU test double in
tests/cpu_backend.py; the GPU run of the same path uses libmgcn + RCCL."""
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


def _problem(N=300, pairs=1500, F=16, L=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    s = torch.randint(0, N, (pairs,), generator=g)
    d = torch.randint(0, N, (pairs,), generator=g)
    loops = torch.arange(N)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    X = torch.randn(N, F, generator=g)
    Ws = [torch.randn(F, F, generator=g) * 0.3 for _ in range(L)]
    bs = [torch.randn(F, generator=g) * 0.1 for _ in range(L)]
    dY = torch.randn(N, F, generator=g)
    return ei, N, X, Ws, bs, dY


def _run(rank, world, port, aggr, out_q, F=16, fused=True, chunks=4, pack=True, force=False,
         slack=None, one_pass=True):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "meta-gcn_amd"),
                    HERE]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from cpu_backend import CpuBackend
        from mgcn import dist as mdist
        from mgcn.dist import ShardedGCN
        mdist.set_pack_exchange(pack)
        mdist.set_force_collectives(force)
        mdist.set_fused_pack(one_pass)
        mdist.FUSED_PACK_MIN_BYTES = 0  # the tests' chunks are small
        if slack is not None:
            mdist.SPEC_SLACK = slack
        ei, N, X, Ws, bs, dY = _problem(F=F)
        m = ShardedGCN(ei, N, Ws, bs, device=torch.device("cpu"), aggr=aggr,
                       backend=CpuBackend(), fused=fused, chunks=chunks)
        assert m.fused == (fused and aggr != "max")
        Xl = m.local_rows(X).requires_grad_(True)
        out = m.forward(Xl)
        out.backward(m.local_rows(dY))
        from mgcn.dist import allreduce_grads
        allreduce_grads(m.params())
        res = {"rank": rank, "lo": m.shard.lo, "hi": m.shard.hi, "out": out.detach().numpy(),
               "dX": Xl.grad.numpy(), "grads": [p.grad.numpy() for p in m.params()]}
        # the bench's form: replicated input in the exchange layout, no x grad
        for p in m.params():
            p.grad = None
        out2 = m.forward(X_table=m.input_table(X))
        out2.backward(m.local_rows(dY))
        allreduce_grads(m.params())
        res["out_table"] = out2.detach().numpy()
        res["grads_table"] = [p.grad.numpy() for p in m.params()]
        res["stats"] = dict(mdist.STATS)
        out_q.put(res)
    finally:
        dist.destroy_process_group()


def _launch(world, aggr, F=16, fused=True, chunks=4, pack=True, force=False, slack=None,
            one_pass=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, aggr, q, F, fused, chunks, pack,
                                            force, slack, one_pass))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r["rank"])
    return res


@pytest.mark.parametrize("world,aggr,F,fused,chunks", [
    (2, "add", 16, True, 4), (2, "mean", 16, True, 3), (4, "add", 16, True, 4),
    (4, "mean", 16, True, 1), (2, "max", 16, True, 4), (4, "max", 16, True, 4),
    (2, "add", 16, False, 4), (4, "add", 256, True, 4), (4, "mean", 256, False, 2),
    (2, "max", 256, True, 3)])
def test_sharded_matches_single_process(world, aggr, F, fused, chunks):
    """World P against world 1 of the same path: fused stack (sum / mean,
    chunked all-gathers) or per-layer path (max, or fused=False), F = 16 and
    256, local input rows (with dX) and the replicated input table."""
    single = _launch(1, aggr, F, fused, chunks)[0]
    shards = _launch(world, aggr, F, fused, chunks)
    assert shards[0]["lo"] == 0 and shards[-1]["hi"] == single["out"].shape[0]
    for r in shards:
        lo, hi = r["lo"], r["hi"]
        np.testing.assert_array_equal(r["out"], single["out"][lo:hi])   # forward: bitwise
        np.testing.assert_array_equal(r["dX"], single["dX"][lo:hi])     # adjoint rows: bitwise
        np.testing.assert_array_equal(r["out_table"], single["out"][lo:hi])
        for key in ("grads", "grads_table"):                            # all-reduced partials
            for g, g1 in zip(r[key], single[key]):
                np.testing.assert_allclose(g, g1, rtol=1e-5, atol=1e-5 * max(1, np.abs(g1).max()))


@pytest.mark.parametrize("world,aggr,F,chunks,one_pass", [
    (2, "add", 32, 4, True), (4, "mean", 64, 3, True), (2, "add", 128, 3, True),
    (2, "add", 128, 3, False), (2, "mean", 96, 2, True)])
def test_packed_exchange_is_bitwise_the_dense_one(world, aggr, F, chunks, one_pass):
    """The zero-skipping exchange (ReLU'd forward tables, ReLU-masked
    backward tables) against the dense exchange of the same sharded stack:
    every output, dX row and gradient bit for bit, with fewer words sent
    (F = 128: the in-place table in ONE receive buffer, dist._single_recv_words).
    Chunks packed in one pass (mgcn_pack_rows' double) or in two (count,
    scan, values: set_fused_pack(False), and F = 96, which the one pass does
    not take)."""
    packed = _launch(world, aggr, F, True, chunks, pack=True, one_pass=one_pass)
    dense = _launch(world, aggr, F, True, chunks, pack=False)
    for rp, rd in zip(packed, dense):
        for key in ("out", "dX", "out_table"):
            np.testing.assert_array_equal(rp[key], rd[key])
        for key in ("grads", "grads_table"):
            for g, g1 in zip(rp[key], rd[key]):
                np.testing.assert_array_equal(g, g1)
        st = rp["stats"]
        assert 0 < st["sent_words"] < 0.8 * st["dense_words"], st
        # the second pass sent every in-place chunk at the sizes the first learnt
        assert st.get("spec_chunks", 0) > 0 and st.get("spec_resent", 0) == 0, st
        assert (st.get("pack_one_pass", 0) > 0) == (one_pass and F % 32 == 0 and F // 32 in
                                                    (1, 2, 4, 8)), st
        assert rd["stats"]["dense_words"] == 0


@pytest.mark.parametrize("world,F,chunks", [(2, 128, 3), (2, 256, 2)])
def test_speculative_exchange_resends_chunks_that_outgrow_their_capacity(world, F, chunks):
    """The second pass of every worker sends each in-place packed chunk at
    the capacity the first pass learnt (dist.SPEC_EXCHANGE); with the slack
    set to -50 % every such chunk outgrows it, and result() must send it
    again at its true size before the next layer reads it: the same bits as
    the dense exchange, with resends counted."""
    packed = _launch(world, "add", F, True, chunks, pack=True, slack=-0.5)
    dense = _launch(world, "add", F, True, chunks, pack=False)
    for rp, rd in zip(packed, dense):
        for key in ("out", "dX", "out_table"):
            np.testing.assert_array_equal(rp[key], rd[key])
        for key in ("grads", "grads_table"):
            for g, g1 in zip(rp[key], rd[key]):
                np.testing.assert_array_equal(g, g1)
        assert rp["stats"].get("spec_resent", 0) > 0, rp["stats"]


@pytest.mark.parametrize("aggr", ["add", "mean"])
def test_forced_collectives_at_world_one(aggr):
    """set_force_collectives(True) in a one-rank group: every exchange
    (chunked all-gathers, the packed exchange's size gather and payload, the
    gradient all-reduce) goes through torch.distributed -- the path
    tests/test_gpu_rccl.py runs on RCCL -- and the results are bit for bit
    the world-1 copies'."""
    forced = _launch(1, aggr, 32, True, 3, pack=True, force=True)[0]
    plain = _launch(1, aggr, 32, True, 3, pack=True, force=False)[0]
    for key in ("out", "dX", "out_table"):
        np.testing.assert_array_equal(forced[key], plain[key])
    for key in ("grads", "grads_table"):
        for g, g1 in zip(forced[key], plain[key]):
            np.testing.assert_array_equal(g, g1)
    st = forced["stats"]
    assert 0 < st["sent_words"] < st["dense_words"], st
    assert plain["stats"]["dense_words"] == 0


def test_fused_and_per_layer_paths_agree():
    """The fused sharded stack and the per-layer sharded path compute the
    same layers: outputs within fp32 association tolerance ((A x) W against
    A (x W)), dX and gradients within tolerance."""
    a = _launch(2, "add", 16, True)
    b = _launch(2, "add", 16, False)
    for ra, rb in zip(a, b):
        np.testing.assert_allclose(ra["out"], rb["out"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ra["dX"], rb["dX"], rtol=1e-4, atol=1e-5)
        for g, g1 in zip(ra["grads"], rb["grads"]):
            np.testing.assert_allclose(g, g1, rtol=1e-4, atol=1e-4 * max(1, np.abs(g1).max()))


def test_single_process_double_matches_oracle(oracle):
    """The CPU double (world 1) against the C oracle, one layer, W = I."""
    sys.path.insert(0, HERE)
    from cpu_backend import CpuBackend
    from mgcn.dist import build_shard, sharded_aggregate
    ei, N, X, Ws, bs, dY = _problem(L=1)
    be = CpuBackend()
    sh = build_shard(ei, N, "sm", backend=be)
    x = X.clone().requires_grad_(True)
    y = sharded_aggregate(x, sh, "add", bs[0], relu=True, backend=be)
    y.backward(dY)
    wf, wb, rs = oracle.edge_factors(ei.numpy(), N, "sm")
    y_ref, _ = oracle.aggr_fwd(ei.numpy(), X.numpy(), wf, "add", bs[0].numpy(), True)
    np.testing.assert_array_equal(y.detach().numpy(), y_ref)
    dH, _ = oracle.aggr_bwd(ei.numpy(), dY.numpy(), wb, rs, "add", y_ref, True, None)
    np.testing.assert_array_equal(x.grad.numpy(), dH)


def test_table_positions_layout():
    """Row i of rank k sits at c*P*cr + k*cr + (i - c*cr), c = i // cr: each
    chunk's all-gather fills one contiguous block."""
    from mgcn.dist import table_positions
    bounds = [0, 5, 9, 14]
    pos = table_positions(torch.arange(14), bounds, 2).tolist()
    # rank 0 rows 0..4, rank 1 rows 5..8, rank 2 rows 9..13, cr = 2, P = 3
    assert pos[:5] == [0, 1, 6, 7, 12]
    assert pos[5:9] == [2, 3, 8, 9]
    assert pos[9:] == [4, 5, 10, 11, 16]
    assert len(set(pos)) == 14


def test_partition_balances_edges():
    from mgcn.dist import partition_nodes
    rp = torch.tensor([0, 10, 10, 10, 50, 51, 60, 100])
    b = partition_nodes(rp, 3)
    assert b[0] == 0 and b[-1] == 7 and all(x <= y for x, y in zip(b, b[1:]))


def test_build_shard_rejects_differentiable_norm_inputs():
    """The sharded path builds its norms once, outside autograd: an
    edge_weight / deg that requires grad raises instead of silently getting
    no gradient (the single-device modules are the differentiable path)."""
    import pytest
    from mgcn.dist import build_shard
    ei = torch.tensor([[0, 1, 2, 0, 1, 2], [1, 2, 0, 0, 1, 2]])
    ew = torch.ones(6, requires_grad=True)
    with pytest.raises(NotImplementedError):
        build_shard(ei, 3, "sm", edge_weight=ew)
    with pytest.raises(NotImplementedError):
        build_shard(ei, 3, "sm", deg=torch.ones(3, requires_grad=True))


@pytest.mark.parametrize("fused,aggr", [(True, "add"), (False, "add"), (True, "max")])
def test_emulated_rank_runs_the_rank_local_step(fused, aggr):
    """build_shard(emulate=(r, P)): one process stands in for rank r of P
    without torch.distributed (the config-5 rank timing,
    scripts/config5_rank.py).  Its shard equals the real rank's (same rows,
    slots, weights), a one-layer forward over the true input table equals the
    single-process rows bit for bit, and the 3-layer step runs on the
    persistent exchange tables (other ranks' rows left as they are).  The
    per-layer path exchanges x W, which an emulated rank holds only for its
    own rows, so only its running is checked."""
    sys.path.insert(0, HERE)
    from cpu_backend import CpuBackend
    from mgcn.dist import ShardedGCN
    ei, N, X, Ws, bs, dY = _problem(F=16)
    be = CpuBackend()
    cpu = torch.device("cpu")
    one = ShardedGCN(ei, N, Ws[:1], bs[:1], device=cpu, aggr=aggr, backend=be, fused=fused)
    y1 = one.forward(X_table=one.input_table(X)).detach()
    for r in range(3):
        m = ShardedGCN(ei, N, Ws[:1], bs[:1], device=cpu, aggr=aggr, backend=be, fused=fused,
                       emulate=(r, 3))
        sh = m.shard
        assert sh.emulated and sh.world == 3 and sh.rank == r
        y = m.forward(X_table=m.input_table(X)).detach()
        if m.fused:  # reads the input table itself (the per-layer path exchanges x W)
            assert torch.equal(y, y1[sh.lo:sh.hi])
        m3 = ShardedGCN(ei, N, Ws, bs, device=cpu, aggr=aggr, backend=be, fused=fused,
                        emulate=(r, 3))
        step = m3.step_fn(X, dY)
        step()
        step()
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m3.params())
        assert set(m3.shard._tables) and all(t.shape[0] == m3.shard.table_rows
                                             for t in m3.shard._tables.values())
