"""Pooling operators (mgcn.pool) and the pooling nets of kernel/ on the GPU.

HardPooling (the reference's own module) is checked against fixtures made
from the reference code (tests/golden/make_golden.py hardpool).  The PyG 1.3
operators have no reference fixtures (PyG is un-vendored; parity unpinned
beyond the restatements): each is compared with an independent CPU
restatement of PyG 1.3's published algorithm written here (loops / numpy),
on the same inputs.
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _batch_graphs(rng, sizes, deg=3, loops=False):
    eis, batch, off = [], [], 0
    for g, n in enumerate(sizes):
        s = rng.integers(0, n, deg * n)
        d = rng.integers(0, n, deg * n)
        s, d = np.concatenate([s, d]), np.concatenate([d, s])
        if loops:
            s, d = np.concatenate([s, np.arange(n)]), np.concatenate([d, np.arange(n)])
        eis.append(np.stack([s, d]) + off)
        batch.append(np.full(n, g))
        off += n
    return (torch.from_numpy(np.concatenate(eis, 1).astype(np.int64)),
            torch.from_numpy(np.concatenate(batch).astype(np.int64)))


# ------------------------------------------------------------ restatements
def ref_softmax(src, index, n):
    src = src.double()
    mx = torch.full((n,) + tuple(src.shape[1:]), -math.inf, dtype=torch.float64)
    for e in range(src.size(0)):
        mx[index[e]] = torch.maximum(mx[index[e]], src[e])
    out = (src - mx[index]).exp()
    den = torch.zeros_like(mx).index_add_(0, index, out)
    return out / (den[index] + 1e-16)


def ref_scatter_max_arg(src, index, n):
    src = src.numpy()
    out = np.full((n,) + src.shape[1:], -np.inf, dtype=np.float64)
    arg = np.full((n,) + src.shape[1:], -1, dtype=np.int64)
    for e in range(src.shape[0]):  # torch_scatter 1.x CPU: sequential, `>=`
        m = src[e] >= out[index[e]]
        out[index[e]] = np.where(m, src[e], out[index[e]])
        arg[index[e]] = np.where(m, e, arg[index[e]])
    out[arg < 0] = 0
    return out, arg


def ref_topk(score, ratio, batch):
    perm = []
    for g in range(int(batch.max()) + 1):
        idx = np.nonzero(batch.numpy() == g)[0]
        k = int(math.ceil(ratio * idx.size))
        order = idx[np.argsort(-score.numpy()[idx], kind="stable")]
        perm.extend(order[:k].tolist())
    return torch.tensor(perm)


def ref_filter_adj(ei, perm, n):
    pos = {int(p): i for i, p in enumerate(perm.tolist())}
    keep = [(pos[int(a)], pos[int(b)]) for a, b in ei.t().tolist() if a in pos and b in pos]
    return torch.tensor(keep, dtype=torch.long).t().reshape(2, -1)


# ------------------------------------------------------------------ tests
def test_softmax_and_scatter_max_arg(cuda):
    from mgcn.pool import scatter_max_arg, softmax
    rng = np.random.default_rng(0)
    E, N = 3000, 400
    index = torch.from_numpy(rng.integers(0, N - 20, E))  # last rows empty
    src = torch.randn(E, 3)
    src[::97] = src[1]  # ties
    got = softmax(src.to(cuda), index.to(cuda), N).cpu()
    torch.testing.assert_close(got.double(), ref_softmax(src, index, N), rtol=1e-5, atol=1e-7)
    out, arg = scatter_max_arg(src.to(cuda), index.to(cuda), N)
    ro, ra = ref_scatter_max_arg(src, index.numpy(), N)
    np.testing.assert_array_equal(arg.cpu().numpy(), ra)
    np.testing.assert_array_equal(out.cpu().numpy(), ro.astype(np.float32))
    o1, a1 = scatter_max_arg(src[:, 0].to(cuda), index.to(cuda), N)  # 1-D src
    np.testing.assert_array_equal(a1.cpu().numpy(), ra[:, 0])


def test_topk_filter_adj_and_topk_pooling(cuda):
    from mgcn.pool import TopKPooling, filter_adj, topk
    rng = np.random.default_rng(1)
    ei, batch = _batch_graphs(rng, [9, 1, 30, 17])
    n = batch.numel()
    score = torch.randn(n)
    perm = topk(score.to(cuda), 0.8, batch.to(cuda)).cpu()
    assert torch.equal(perm, ref_topk(score, 0.8, batch))
    ei2, _ = filter_adj(ei.to(cuda), None, perm.to(cuda), n)
    assert torch.equal(ei2.cpu(), ref_filter_adj(ei, perm, n))

    torch.manual_seed(0)
    pool = TopKPooling(16, ratio=0.5).to(cuda)
    x = torch.randn(n, 16, requires_grad=True)
    xg = x.detach().to(cuda).requires_grad_(True)
    out, ei3, _, b3, perm3, sc3 = pool(xg, ei.to(cuda), batch=batch.to(cuda))
    w = pool.weight.detach().cpu()
    s = torch.tanh((x * w).sum(-1) / w.norm(p=2, dim=-1))
    rp = ref_topk(s.detach(), 0.5, batch)
    assert torch.equal(perm3.cpu(), rp)
    torch.testing.assert_close(out.cpu(), (x[rp] * s[rp].view(-1, 1)).detach(), rtol=1e-5,
                               atol=1e-6)
    assert torch.equal(ei3.cpu(), ref_filter_adj(ei, rp, n))
    assert torch.equal(b3.cpu(), batch[rp])
    (out.sum() + sc3.sum()).backward()
    assert torch.isfinite(xg.grad).all() and pool.weight.grad is not None


def test_sag_pooling_graphconv_score(cuda):
    from mgcn.pool import SAGPooling
    rng = np.random.default_rng(2)
    ei, batch = _batch_graphs(rng, [15, 22, 8])
    n = batch.numel()
    torch.manual_seed(1)
    pool = SAGPooling(12, ratio=0.5).to(cuda)
    x = torch.randn(n, 12)
    out, ei2, _, b2, perm, sc = pool(x.to(cuda), ei.to(cuda), batch=batch.to(cuda))
    g = pool.gnn
    ref = torch.tanh(_graphconv_add(x, ei, g).view(-1))
    rp = ref_topk(ref.float(), 0.5, batch)
    assert torch.equal(perm.cpu(), rp)
    torch.testing.assert_close(sc.cpu().double(), ref[rp], rtol=1e-5, atol=1e-6)
    assert torch.equal(ei2.cpu(), ref_filter_adj(ei, rp, n))


def _graphconv_add(x, ei, g):
    """PyG 1.3 GraphConv (aggr 'add', SAGPooling's default) restated."""
    h = x.double() @ g.weight.detach().cpu().double()
    agg = torch.zeros_like(h).index_add_(0, ei[1], h[ei[0]])
    return agg + x.double() @ g.lin.weight.detach().cpu().double().t() + \
        g.lin.bias.detach().cpu().double()


def _pyg_merge_edges(ei, score, n):
    """PyG 1.3 EdgePooling.__merge_edges__, literally (set-based)."""
    nodes_remaining = set(range(n))
    cluster = torch.empty(n, dtype=torch.long)
    order = torch.argsort(score, descending=True, stable=True)
    i, chosen = 0, []
    for e in order.tolist():
        s = ei[0, e].item()
        if s not in nodes_remaining:
            continue
        t = ei[1, e].item()
        if t not in nodes_remaining:
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
    return cluster, chosen, i


def test_edge_pooling_matches_pyg_merge(cuda):
    from mgcn.pool import EdgePooling
    rng = np.random.default_rng(3)
    ei, batch = _batch_graphs(rng, [10, 25, 6], deg=2)
    n = batch.numel()
    torch.manual_seed(2)
    pool = EdgePooling(8).to(cuda).eval()
    x = torch.randn(n, 8)
    xg = x.to(cuda).requires_grad_(True)
    new_x, new_ei, new_b, info = pool(xg, ei.to(cuda), batch.to(cuda))
    lin = pool.lin
    raw = (torch.cat([x[ei[0]], x[ei[1]]], -1).double() @ lin.weight.detach().cpu().double().t()
           + lin.bias.detach().cpu().double()).view(-1)
    e = ref_softmax(raw, ei[1], n) + 0.5
    cluster, chosen, C = _pyg_merge_edges(ei, e.float(), n)
    assert torch.equal(info.cluster.cpu(), cluster)
    sc = torch.cat([e[chosen], torch.ones(C - len(chosen), dtype=torch.float64)])
    ref_x = torch.zeros(C, 8, dtype=torch.float64).index_add_(0, cluster, x.double()) * sc.view(-1, 1)
    torch.testing.assert_close(new_x.detach().cpu().double(), ref_x, rtol=1e-5, atol=1e-6)
    key = torch.unique(cluster[ei[0]] * C + cluster[ei[1]])
    assert torch.equal(new_ei.cpu(), torch.stack([key // C, key % C]))
    assert torch.equal(new_b.cpu(), torch.zeros(C, dtype=torch.long).scatter_(0, cluster, batch))
    new_x.sum().backward()
    assert torch.isfinite(xg.grad).all()
    ux, uei, ub = pool.unpool(new_x.detach(), info)
    assert ux.shape == x.shape and torch.equal(ub.cpu(), batch)


@pytest.mark.parametrize("n,E,loops,dups", [
    (1, 0, False, False), (5, 0, False, False), (1, 1, True, False), (12, 30, True, True),
    (700, 2500, True, True), (3000, 1500, False, False), (5000, 40000, True, True),
    (20000, 60000, False, True)])
def test_edge_merge_greedy_device_matches_pyg_walk(cuda, n, E, loops, dups):
    """mgcn_edge_merge_greedy (device, locally-dominant rounds) against PyG
    1.3's sequential set-based walk: the same cluster of every node, the same
    contracted edges in the same order, the same cluster count -- with self
    loops, duplicate / reversed edges, isolated nodes and more nodes and
    edges than one 1024-thread scan block."""
    from mgcn.pool import edge_merge_greedy
    rng = np.random.default_rng(n * 7 + E)
    s = rng.integers(0, n, E)
    d = rng.integers(0, n, E)
    if loops and E:
        k = max(1, E // 10)
        d[:k] = s[:k]
    if dups and E > 4:
        k = E // 5
        s[-k:], d[-k:] = d[:k], s[:k]  # reversed copies of the first edges
    ei = torch.from_numpy(np.stack([s, d]).astype(np.int64))
    order = torch.from_numpy(rng.permutation(E).astype(np.int64))
    nodes_remaining = set(range(n))
    cluster = torch.empty(n, dtype=torch.long)
    i, chosen = 0, []
    for e in order.tolist():
        a, b = int(s[e]), int(d[e])
        if a not in nodes_remaining or b not in nodes_remaining:
            continue
        chosen.append(e)
        cluster[a] = i
        nodes_remaining.remove(a)
        if a != b:
            cluster[b] = i
            nodes_remaining.remove(b)
        i += 1
    for node in sorted(nodes_remaining):
        cluster[node] = i
        i += 1
    c_dev, ch_dev, C = edge_merge_greedy(ei.to(cuda), order.to(cuda), n)
    assert C == i
    assert torch.equal(c_dev.cpu(), cluster)
    assert ch_dev.cpu().tolist() == chosen


def test_edge_merge_greedy_rejects_malformed_input(cuda):
    """Endpoints outside [0, N) and an order that is not a permutation are
    caught on the device before any indexed write (IndexError, as the host
    walk raised)."""
    from mgcn.pool import edge_merge_greedy
    ei = torch.tensor([[0, 1, 2], [1, 2, 0]], dtype=torch.int64, device=cuda)
    order = torch.tensor([2, 0, 1], dtype=torch.int64, device=cuda)
    c, ch, C = edge_merge_greedy(ei, order, 3)
    assert C == 2 and ch.numel() == 1
    for bad_ei, bad_order, n in [
            (torch.tensor([[0, 1, 5], [1, 2, 0]]), order, 3),     # endpoint >= N
            (torch.tensor([[0, -1, 2], [1, 2, 0]]), order, 3),    # negative endpoint
            (ei, torch.tensor([2, 0, 3]), 3),                     # order out of range
            (ei, torch.tensor([2, 0, 0]), 3)]:                    # repeated position
        with pytest.raises(IndexError):
            edge_merge_greedy(bad_ei.to(cuda), bad_order.to(cuda), n)
    torch.cuda.synchronize()


def test_graclus_is_a_maximal_matching_and_max_pool(cuda):
    from mgcn.kernel.data import Batch
    from mgcn.pool import graclus, max_pool
    rng = np.random.default_rng(4)
    ei, batch = _batch_graphs(rng, [12, 40, 3, 25], deg=2)
    n = batch.numel()
    torch.manual_seed(3)
    cl = graclus(ei.to(cuda), num_nodes=n).cpu()
    edges = set(map(tuple, ei.t().tolist()))
    members = {}
    for v, c in enumerate(cl.tolist()):
        members.setdefault(c, []).append(v)
    for c, vs in members.items():
        assert len(vs) <= 2 and c == min(vs)
        if len(vs) == 2:
            assert (vs[0], vs[1]) in edges or (vs[1], vs[0]) in edges
    single = {vs[0] for vs in members.values() if len(vs) == 1}
    assert not any(a in single and b in single and a != b for a, b in edges)  # maximal
    x = torch.randn(n, 5)
    data = max_pool(cl.to(cuda), Batch(x=x.to(cuda), edge_index=ei.to(cuda), batch=batch.to(cuda)))
    uniq, inv = torch.unique(cl, sorted=True, return_inverse=True)
    ref = torch.stack([x[inv == c].max(0)[0] for c in range(uniq.numel())])
    torch.testing.assert_close(data.x.cpu(), ref)
    e2 = inv[ei]
    e2 = e2[:, e2[0] != e2[1]]
    key = torch.unique(e2[0] * uniq.numel() + e2[1])
    assert torch.equal(data.edge_index.cpu(), torch.stack([key // uniq.numel(), key % uniq.numel()]))
    assert torch.equal(data.batch.cpu(), torch.stack([batch[inv == c][0]
                                                      for c in range(uniq.numel())]))


def test_readouts_sort_attention_set2set(cuda):
    from mgcn.models import Linear
    from mgcn.pool import GlobalAttention, Set2Set, global_sort_pool
    rng = np.random.default_rng(5)
    sizes = [7, 15, 3, 12]
    batch = torch.from_numpy(np.concatenate([np.full(n, g) for g, n in enumerate(sizes)]))
    n = batch.numel()
    x = torch.randn(n, 6)
    # global_sort_pool, k = 10: per graph sort by the last channel, pad with 0
    got = global_sort_pool(x.to(cuda), batch.to(cuda), 10).cpu()
    rows = []
    for g in range(len(sizes)):
        xg = x[batch == g]
        xg = xg[torch.argsort(xg[:, -1], descending=True, stable=True)][:10]
        rows.append(torch.cat([xg, torch.zeros(10 - xg.size(0), 6)]).view(-1))
    torch.testing.assert_close(got, torch.stack(rows))
    # GlobalAttention with a Linear gate
    torch.manual_seed(4)
    att = GlobalAttention(Linear(6, 1)).to(cuda)
    got = att(x.to(cuda), batch.to(cuda)).detach().cpu().double()
    gate = x.double() @ att.gate_nn.weight.detach().cpu().double().t() + \
        att.gate_nn.bias.detach().cpu().double()
    a = ref_softmax(gate, batch, len(sizes))
    ref = torch.zeros(len(sizes), 6, dtype=torch.float64).index_add_(0, batch, a * x.double())
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    # Set2Set(6, 4): the same LSTM weights on the CPU
    s2s = Set2Set(6, processing_steps=4).to(cuda)
    got = s2s(x.to(cuda), batch.to(cuda)).detach().cpu()
    lstm = torch.nn.LSTM(12, 6, 1)
    lstm.load_state_dict({k: v.cpu() for k, v in s2s.lstm.state_dict().items()})
    B = len(sizes)
    h = (torch.zeros(1, B, 6), torch.zeros(1, B, 6))
    q_star = torch.zeros(B, 12)
    with torch.no_grad():
        for _ in range(4):
            q, h = lstm(q_star.unsqueeze(0), h)
            q = q.view(B, 6)
            e = (x * q[batch]).sum(-1, keepdim=True)
            a = ref_softmax(e, batch, B).float()
            r = torch.zeros(B, 6).index_add_(0, batch, a * x)
            q_star = torch.cat([q, r], -1)
    torch.testing.assert_close(got, q_star, rtol=1e-4, atol=1e-5)


def test_dense_sage_and_diff_pool(cuda):
    from mgcn.pool import DenseSAGEConv, dense_diff_pool
    torch.manual_seed(5)
    B, N, C = 3, 9, 4
    x = torch.randn(B, N, C)
    adj = (torch.rand(B, N, N) < 0.3).float()
    mask = torch.ones(B, N, dtype=torch.bool)
    mask[1, 6:] = False
    conv = DenseSAGEConv(C, 5).to(cuda)
    got = conv(x.to(cuda), adj.to(cuda), mask.to(cuda)).cpu()
    a = adj.clone()
    a[:, torch.arange(N), torch.arange(N)] = 1
    ref = (a @ x) / a.sum(-1, keepdim=True).clamp(min=1) @ conv.weight.detach().cpu() + \
        conv.bias.detach().cpu()
    ref = ref * mask.unsqueeze(-1)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    s = torch.randn(B, N, 3)
    out, out_adj, link, ent = dense_diff_pool(x.to(cuda), adj.to(cuda), s.to(cuda), mask.to(cuda))
    S = torch.softmax(s, -1) * mask.unsqueeze(-1)
    xm = x * mask.unsqueeze(-1)
    torch.testing.assert_close(out.cpu(), S.transpose(1, 2) @ xm, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out_adj.cpu(), S.transpose(1, 2) @ adj @ S, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(link.cpu(), torch.norm(adj - S @ S.transpose(1, 2), p=2) / adj.numel())
    torch.testing.assert_close(ent.cpu(), (-S * torch.log(S + 1e-15)).sum(-1).mean())


@pytest.mark.parametrize("B,N,C,K", [(3, 9, 4, 3), (5, 37, 20, 7), (1, 1, 1, 1)])
def test_diff_pool_dense_products_on_libmgcn_with_gradients(cuda, B, N, C, K):
    """DenseSAGEConv -> dense_diff_pool on mgcn_gemm_batched (ops.bmm, the
    last vendor GEMM of a module path, round 5): forward values and the
    gradients of x, s and the conv's weight / bias against fp64 torch autograd
    on the CPU (the products are exact fp32 on MFMA; tolerance is fp32
    summation order)."""
    from mgcn import ops
    from mgcn.pool import DenseSAGEConv, dense_diff_pool
    torch.manual_seed(B * 100 + N)
    x = torch.randn(B, N, C)
    adj = (torch.rand(B, N, N) < 0.3).float()
    mask = torch.ones(B, N, dtype=torch.bool)
    if N > 2:
        mask[0, N // 2:] = False
    s0 = torch.randn(B, N, K)
    conv = DenseSAGEConv(C, K).to(cuda)
    ref_conv = DenseSAGEConv(C, K).double()
    ref_conv.load_state_dict({k: v.double().cpu() for k, v in conv.state_dict().items()})
    outs = []
    for dev, m in ((cuda, conv), ("cpu", ref_conv)):
        dt = torch.float32 if dev != "cpu" else torch.float64
        xx = x.to(dev, dt).requires_grad_(True)
        ss = s0.to(dev, dt).requires_grad_(True)
        if dev == "cpu":
            import mgcn.pool as P
            saved = P.bmm
            P.bmm = lambda a, b: torch.matmul(a, b)  # the fp64 reference products
        try:
            h = m(xx, adj.to(dev, dt), mask.to(dev))
            out, out_adj, link, ent = dense_diff_pool(h, adj.to(dev, dt), ss, mask.to(dev))
        finally:
            if dev == "cpu":
                P.bmm = saved
        loss = out.sum() + (out_adj * out_adj).sum() + link + ent
        loss.backward()
        outs.append([out.detach(), out_adj.detach(), xx.grad, ss.grad, m.weight.grad, m.bias.grad])
    for got, ref in zip(*outs):
        torch.testing.assert_close(got.cpu().double(), ref, rtol=1e-4, atol=1e-4)
    assert ops.bmm(torch.randn(2, 3, 4, device=cuda), torch.randn(4, 5, device=cuda)).shape == (2, 3, 5)


@pytest.mark.parametrize("name", ["hardpool_add", "hardpool_add_bias", "hardpool_mean",
                                  "hardpool_sunk"])
def test_hard_pooling_matches_reference(cuda, name):
    """Eval-mode HardPooling == the reference module (fixtures from
    hard_attention_pool.py itself): pooled features and dx bitwise, kept
    nodes / edges / batch exactly -- including the no-out-edge quirk."""
    from mgcn.pool import HardPooling
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    F = d["x"].shape[1]
    pool = HardPooling(F, aggr=str(d["meta"][0]), bias="bias" in d.files).to(cuda).eval()
    with torch.no_grad():
        pool.att_weight.copy_(torch.from_numpy(d["att_weight"]))
        if "bias" in d.files:
            pool.bias.copy_(torch.from_numpy(d["bias"]))
    x = torch.from_numpy(d["x"]).to(cuda).requires_grad_(True)
    out, ei, _, b, perm, score = pool(x, torch.from_numpy(d["edge_index"]).to(cuda),
                                      torch.from_numpy(d["batch"]).to(cuda))
    np.testing.assert_array_equal(perm.cpu().numpy(), d["perm"])
    np.testing.assert_array_equal(ei.cpu().numpy(), d["out_edge_index"])
    np.testing.assert_array_equal(b.cpu().numpy(), d["out_batch"])
    np.testing.assert_array_equal(score.cpu().numpy(), d["score"])
    np.testing.assert_allclose(out.detach().cpu().numpy(), d["out"], rtol=1e-6, atol=1e-6)
    out.backward(torch.from_numpy(d["dY"]).to(cuda))
    np.testing.assert_allclose(x.grad.cpu().numpy(), d["dx"], rtol=1e-6, atol=1e-6)


def test_hard_pooling_training_mode(cuda):
    """Training: Gumbel-softmax weights per source node (each source's
    out-edge weights sum to 1), graph kept unchanged, gradients flow."""
    from mgcn.pool import HardPooling
    rng = np.random.default_rng(6)
    ei, batch = _batch_graphs(rng, [10, 20])
    n = batch.numel()
    pool = HardPooling(8, att_dropout=0.0).to(cuda).train()
    x = torch.randn(n, 8, device=cuda, requires_grad=True)
    store = []
    out, ei2, _, b2, perm, score = pool(x, ei.to(cuda), batch.to(cuda), attn_store=store)
    assert torch.equal(perm.cpu(), torch.arange(n)) and torch.equal(ei2.cpu(), ei)
    alpha = store[0].cpu().double().view(-1)
    sums = torch.zeros(n, dtype=torch.float64).index_add_(0, ei[0], alpha)
    has = torch.bincount(ei[0], minlength=n) > 0
    torch.testing.assert_close(sums[has], torch.ones(int(has.sum()), dtype=torch.float64),
                               rtol=1e-5, atol=1e-5)
    out.sum().backward()
    assert torch.isfinite(x.grad).all() and torch.isfinite(pool.att_weight.grad).all()


# --------------------------------------------------------------- the nets
@pytest.mark.parametrize("net", ["TopK", "SAGPool", "EdgePool", "Graclus", "HardPool", "TopKNew",
                                 "SAGPoolNew", "GlobalAttentionNet", "Set2SetNet", "SortPool",
                                 "DiffPool"])
def test_pool_net_trains(cuda, net):
    """Every pooling net of kernel/main.py: forward (train and eval) and a
    few Adam steps on a synthetic MUTAG-shaped batch; the loss drops."""
    import torch.nn.functional as F
    from mgcn.kernel import NETS, get_dataset
    from mgcn.kernel.data import DataLoader, DenseDataLoader
    torch.manual_seed(7)
    Net = NETS[net]
    ds = get_dataset("MUTAG", sparse=net != "DiffPool", synthetic=True)
    model = Net(ds, 4, 32).to(cuda)
    model.reset_parameters()
    Loader = DenseDataLoader if net == "DiffPool" else DataLoader
    data = next(iter(Loader(ds, 64, shuffle=False))).to(cuda)
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    losses = []
    for _ in range(8):
        opt.zero_grad()
        out = model(data)
        assert out.shape == (64, ds.num_classes) and torch.isfinite(out).all()
        loss = F.nll_loss(out, data.y.view(-1))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses
    model.eval()
    with torch.no_grad():
        out = model(data)
    assert torch.isfinite(out).all()


def test_cross_validation_with_pool_nets(cuda):
    """kernel/train_eval.py driver on a sparse pooling net and on DiffPool's
    dense batches (DenseDataLoader chosen by 'adj' in the data)."""
    from mgcn.kernel import DiffPool, TopK, cross_validation_with_val_set, get_dataset
    for Net, sparse in [(TopK, True), (DiffPool, False)]:
        ds = get_dataset("MUTAG", sparse=sparse, synthetic=True)
        ds = ds[torch.arange(60)]
        res = cross_validation_with_val_set(ds, Net(ds, 2, 16), folds=3, epochs=2, batch_size=16,
                                            lr=0.01, lr_decay_factor=0.5, lr_decay_step_size=50,
                                            weight_decay=0, logger=None, device=torch.device(cuda))
        assert len(res) == 6 and all(math.isfinite(v) for v in res)
