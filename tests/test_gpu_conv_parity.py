"""Module-level parity of the PyG conv surface
that kernel/gcn.py, gin.py, graph_sage.py and the pooling nets (top_k.py:11,
15 ...) build on: mgcn.pyg GCNConv / GINConv / SAGEConv / GraphConv, through
libmgcn on the GPU, against the reference and the oracle.

* GCNConv: the gcnconv_* fixtures were produced by the reference's own
  NodeModelAdditive(deg_norm='sm', aggr='add', bias=True) on the graph after
  PyG 1.3's add_remaining_self_loops (tests/golden/make_golden.py conv; the
  in-repo copy of the normalisation is src/gcn_meta/models/gcn.py:57-86).
* GINConv / SAGEConv / GraphConv: PyG is not vendored, so their composition
  (loop handling, (1 + eps) x, the Linear around the aggregation) follows
  PyG 1.3 and is restated in the test; every aggregation in it is the C
  oracle's (the reference's index_select -> mul -> scatter order).

Bars: W = I (and a zero Linear for GraphConv) makes every dense product exact,
so outputs and dx must match BIT FOR BIT; random weights compare against the
fp64 product of the oracle's aggregate with |err| <= 1e-5 * (|agg| |W| + |b|)
+ 1e-6 (the north star's 1e-5 relative fp32), gradients within fp32
summation-order tolerance as stated per assertion.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    return t.detach().cpu().numpy()


def _graph(rng, N, E, isolated=0, mid_loops=0, tail_loops=False):
    """Random multigraph; ``mid_loops`` self-pairs scattered through the edge
    list, optional one-loop-per-node tail, ``isolated`` nodes without edges."""
    a = N - isolated
    s = rng.integers(0, a, E)
    d = rng.integers(0, a, E)
    if mid_loops:
        v = rng.integers(0, a, mid_loops)
        at = np.sort(rng.integers(0, E, mid_loops))
        s, d = np.insert(s, at, v), np.insert(d, at, v)
    if tail_loops:
        s, d = np.concatenate([s, np.arange(N)]), np.concatenate([d, np.arange(N)])
    return np.stack([s, d]).astype(np.int64)


def _bound_check(y, agg, W, b, slack=0.0):
    """|y - (agg W + b)| <= 1e-5 (|agg| |W| + |b|) + 1e-6 + slack, in fp64."""
    agg = agg.astype(np.float64)
    W = W.astype(np.float64)
    ref = agg @ W + (0 if b is None else b.astype(np.float64))
    bound = np.abs(agg) @ np.abs(W) + (0 if b is None else np.abs(b.astype(np.float64)))
    err = np.abs(y.astype(np.float64) - ref)
    assert (err <= 1e-5 * bound + 1e-6 + slack).all(), float((err / (bound + 1e-30)).max())


# --------------------------------------------------------------- GCNConv
@pytest.mark.parametrize("name", golden_names("gcnconv_"))
def test_gcnconv_matches_reference_fixture(cuda, name):
    """A8: kernel/gcn.py:10,13 GCNConv(F, F[, improved]) on a raw graph with
    mid-list self-pairs (and optional weights): the loops are replaced as
    PyG does, then the reference's 'sm' aggregation.  F = 128 runs the fused
    aggregate-then-transform kernels."""
    from mgcn.pyg import GCNConv
    z = load_golden(name)
    improved, identity, use_ew = (bool(int(v)) for v in z["meta"])
    F = z["x"].shape[1]
    conv = GCNConv(F, F, improved=improved).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(_t(z["W"], cuda))
        conv.bias.copy_(_t(z["b"], cuda))
    x = _t(z["x"], cuda).requires_grad_(True)
    ew = _t(z["edge_weight"], cuda) if use_ew else None
    y = conv(x, _t(z["edge_index"], cuda), ew)
    y.backward(_t(z["dZ"], cuda))
    if identity:
        np.testing.assert_array_equal(_np(y), z["y"])
        np.testing.assert_array_equal(_np(x.grad), z["dx"])
    else:
        np.testing.assert_allclose(_np(y), z["y"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(_np(x.grad), z["dx"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(conv.weight.grad), z["dW"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(_np(conv.bias.grad), z["db"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N,E,F", [(3000, 30000, 128), (2000, 16000, 32)])
def test_gcnconv_random_graph_vs_oracle(cuda, oracle, N, E, F):
    """A8 beyond the fixtures' sizes: W = I bitwise against the oracle's
    GCNConv restatement (loops replaced, unit weights, 'sm'), forward and dx."""
    from mgcn.pyg import GCNConv
    rng = np.random.default_rng(N + F)
    ei = _graph(rng, N, E, isolated=N // 50, mid_loops=N // 20)
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32)
    conv = GCNConv(F, F).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(torch.eye(F))
        conv.bias.copy_(_t(b, cuda))
    xt = _t(x, cuda).requires_grad_(True)
    y = conv(xt, _t(ei, cuda))
    y.backward(_t(dZ, cuda))
    r = oracle.gcnconv_fwd_bwd(x, ei, np.eye(F, dtype=np.float32), b, dZ)
    np.testing.assert_array_equal(_np(y), r["y"])
    np.testing.assert_array_equal(_np(xt.grad), r["dH"])
    np.testing.assert_allclose(_np(conv.bias.grad), r["db"], rtol=1e-4, atol=1e-3)


# --------------------------------------------------------------- GINConv
@pytest.mark.parametrize("F", [16, 128])
@pytest.mark.parametrize("eps,train_eps", [(0.0, False), (0.25, True), (-0.5, False)])
def test_ginconv_vs_oracle(cuda, oracle, F, eps, train_eps):
    """A9: kernel/gin.py:10-28 (GIN0, train_eps=False) and :112-119 (GIN,
    train_eps=True).  PyG 1.3 GINConv removes self-loops, then
    nn((1 + eps) x + sum_j x_j).  With nn = Identity the conv output and dx
    are bitwise (1 + eps) x + oracle_sum and (1 + eps) dZ + oracle adjoint;
    with kernel/gin.py's MLP the output matches that MLP (torch fp32 on the
    CPU) applied to the oracle pre-activation."""
    from mgcn.pyg import GINConv
    rng = np.random.default_rng(int(F + 100 * eps + 107))
    N = 2500
    ei = _graph(rng, N, 20000, isolated=30, mid_loops=80, tail_loops=True)
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    ei_nl = oracle.remove_self_loops(ei)
    agg, _ = oracle.aggr_fwd(ei_nl, x, None, "add")
    dH, _ = oracle.aggr_bwd(ei_nl, dZ, None, None, "add")
    one_eps = np.float32(1) + np.float32(eps)
    pre = one_eps * x + agg

    conv = GINConv(torch.nn.Identity(), eps=eps, train_eps=train_eps).to(cuda)
    xt = _t(x, cuda).requires_grad_(True)
    eit = _t(ei, cuda)
    y = conv(xt, eit)
    np.testing.assert_array_equal(_np(y), pre)
    y.backward(_t(dZ, cuda))
    np.testing.assert_array_equal(_np(xt.grad), one_eps * dZ + dH)
    if train_eps:
        ref = float((x.astype(np.float64) * dZ).sum())
        assert abs(float(conv.eps.grad) - ref) <= 1e-5 * float(np.abs(x * dZ).sum())

    torch.manual_seed(5)
    mlp = torch.nn.Sequential(torch.nn.Linear(F, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64),
                              torch.nn.ReLU())
    conv2 = GINConv(mlp, eps=eps, train_eps=train_eps)
    ref = _np(mlp(torch.from_numpy(pre)))
    conv2 = conv2.to(cuda)
    y2 = conv2(_t(x, cuda), eit)
    np.testing.assert_allclose(_np(y2), ref, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------- SAGEConv
@pytest.mark.parametrize("F_in,F_out,use_ew,identity", [(128, 128, False, True),
                                                        (128, 128, True, True),
                                                        (128, 128, False, False),
                                                        (32, 32, False, True),
                                                        (32, 64, True, False)])
def test_sageconv_vs_oracle(cuda, oracle, F_in, F_out, use_ew, identity):
    """A10: kernel/graph_sage.py:10,13 SAGEConv(in, out) (PyG 1.3: loops
    replaced, mean over w_j x_j, then @ W + b).  128 -> 128 runs the fused
    kernel, the other widths aggregate then transform in two launches."""
    from mgcn.pyg import SAGEConv
    rng = np.random.default_rng(F_in * 3 + F_out + use_ew)
    N = 3000
    ei = _graph(rng, N, 24000, isolated=20, mid_loops=60)
    ew = rng.uniform(0.1, 2.0, ei.shape[1]).astype(np.float32) if use_ew else None
    x = rng.standard_normal((N, F_in)).astype(np.float32)
    dZ = rng.standard_normal((N, F_out)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F_out).astype(np.float32)
    W = np.eye(F_in, dtype=np.float32) if identity else \
        (rng.standard_normal((F_in, F_out)) * 0.1).astype(np.float32)
    ei2, ew2 = oracle.add_remaining_self_loops(ei, ew, 1.0, N)
    agg, _ = oracle.aggr_fwd(ei2, x, ew2, "mean")

    conv = SAGEConv(F_in, F_out).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(_t(W, cuda))
        conv.bias.copy_(_t(b, cuda))
    xt = _t(x, cuda).requires_grad_(True)
    y = conv(xt, _t(ei, cuda), None if ew is None else _t(ew, cuda))
    y.backward(_t(dZ, cuda))
    if identity:
        np.testing.assert_array_equal(_np(y), agg + b)
        dH, _ = oracle.aggr_bwd(ei2, dZ, ew2, None, "mean")
        np.testing.assert_array_equal(_np(xt.grad), dH)
    else:
        _bound_check(_np(y), agg, W, b)
        dH, _ = oracle.aggr_bwd(ei2, dZ.astype(np.float64) @ W.T.astype(np.float64), ew2, None,
                                "mean")
        np.testing.assert_allclose(_np(xt.grad), dH, rtol=1e-4, atol=1e-5)
        # fused: dW = Z^T (dZ / count) with Z the undivided sum; two fp32
        # association orders of the same product (as test_gpu_fused.py)
        dW = agg.astype(np.float64).T @ dZ.astype(np.float64)
        bound = np.abs(agg).astype(np.float64).T @ np.abs(dZ).astype(np.float64)
        assert (np.abs(_np(conv.weight.grad) - dW) <= 4e-5 * bound + 1e-6).all()
    np.testing.assert_allclose(_np(conv.bias.grad), dZ.astype(np.float64).sum(0), rtol=1e-4,
                               atol=1e-3)


# -------------------------------------------------------------- GraphConv
@pytest.mark.parametrize("F", [128, 32])
@pytest.mark.parametrize("aggr", ["add", "mean", "max"])
@pytest.mark.parametrize("use_ew", [False, True])
def test_graphconv_vs_oracle(cuda, oracle, F, aggr, use_ew):
    """A11: kernel/top_k.py:11,15 (and sag_pool, hard_pool, edge_pool,
    graclus) GraphConv(in, out, aggr) = aggr_j (w_j x_j W) + lin(x) (PyG 1.3,
    no self-loops added).  W = I with a zero Linear: output and dx bitwise
    the oracle aggregation and its adjoint; random W and Linear: the
    oracle's aggregation of the kernel's own x W (max does not commute with
    W) plus lin(x), and the fp64 bound for add / mean."""
    from mgcn import ops
    from mgcn.pyg import GraphConv
    rng = np.random.default_rng(F + len(aggr) + 10 * use_ew)
    N = 3000
    ei = _graph(rng, N, 24000, isolated=25, mid_loops=40)
    ew = rng.uniform(0.1, 2.0, ei.shape[1]).astype(np.float32) if use_ew else None
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    eit = _t(ei, cuda)
    ewt = None if ew is None else _t(ew, cuda)

    conv = GraphConv(F, F, aggr=aggr).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(torch.eye(F))
        conv.lin.weight.zero_()
        conv.lin.bias.zero_()
    xt = _t(x, cuda).requires_grad_(True)
    y = conv(xt, eit, ewt)
    y.backward(_t(dZ, cuda))
    ref, am = oracle.aggr_fwd(ei, x, ew, aggr)
    np.testing.assert_array_equal(_np(y), ref)
    dH, _ = oracle.aggr_bwd(ei, dZ, ew, None, aggr, argmax=am)
    np.testing.assert_array_equal(_np(xt.grad), dH)

    torch.manual_seed(9)
    conv = GraphConv(F, F, aggr=aggr).to(cuda)
    W = _np(conv.weight)
    y = _np(conv(_t(x, cuda), eit, ewt))
    lin = _np(conv.lin(_t(x, cuda)))
    if aggr == "max":
        H = _np(ops.linear(_t(x, cuda), conv.weight.detach()))
        mref, _ = oracle.aggr_fwd(ei, H, ew, "max")
        np.testing.assert_allclose(y, mref + lin, rtol=1e-5, atol=1e-5)
    else:
        agg, _ = oracle.aggr_fwd(ei, x, ew, aggr)
        # y - lin re-rounds once: up to 2^-24 |y| on top of the product's error
        _bound_check(y - lin, agg, W, None, slack=2.0 ** -23 * np.abs(y).astype(np.float64))
