"""GPU parity of the fused layer kernels (mgcn_spmm_xw_fwd / mgcn_spmm_xw_bwd).

The forward aggregates X first and multiplies by W in the same launch:
(A X) W instead of the reference's A (X W) (gcn_base_models.py:201, 223-237).
Bars, per test:
  * W = I: every bf16x6 product is exact, so the fused forward equals the
    oracle's aggregation (the reference's index_select * norm -> scatter_add
    order) BIT FOR BIT, masks included;
  * random W: |Y - Y64| <= 1e-5 * (|Z| |W|) + 1e-6, Y64 the fp64 product of
    the (bit-exact) fp32 aggregate Z -- the same bound the GEMM tests use;
  * backward: dX is mgcn_spmm_bwd + mgcn_gemm_bwd's BIT FOR BIT (same dH,
    same products and order), dW within 1e-5 of the |.|-weighted fp64 sum,
    bias column sums within fp32 summation-order tolerance.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _graph(rng, N, E, hub=0):
    s = rng.integers(0, N, E)
    d = rng.integers(0, N, E)
    if hub:  # destination 0 and source 1 get `hub` extra edges (long rows)
        d = np.concatenate([d, np.zeros(hub, np.int64), rng.integers(0, N, hub)])
        s = np.concatenate([s, rng.integers(0, N, hub), np.ones(hub, np.int64)])
    s = np.concatenate([s, np.arange(N)])
    d = np.concatenate([d, np.arange(N)])
    return np.stack([s, d]).astype(np.int64)


GRAPHS = [
    # N, E, hub
    (20000, 200000, 0),
    (4097, 40000, 0),     # last chunk partial
    (33, 100, 0),
    (1, 0, 0),
    (3000, 20000, 700),   # rows far longer than a 32-edge metadata batch
]


def _plan(cuda, ei, N, deg_norm):
    from mgcn.graph import plan_for
    plan = plan_for(_t(ei, cuda), N)
    return plan, plan.norm(deg_norm)


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,aggr,bias,relu", [("sm", "add", True, True),
                                                     ("rw", "mean", False, True),
                                                     (None, "add", True, False),
                                                     ("sm", "mean", True, False)])
def test_fused_forward_identity_weights_bitwise(cuda, oracle, N, E, hub, deg_norm, aggr, bias,
                                                relu):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(N + E + hub)
    ei = _graph(rng, N, E, hub)
    F = 128
    X = rng.standard_normal((N, F)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32) if bias else None
    plan, norm = _plan(cuda, ei, N, deg_norm)
    rm = torch.empty(N, 4, dtype=torch.int32, device=cuda) if relu else None
    Y = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, _t(X, cuda), torch.eye(F, device=cuda),
                        L.REDUCE_CODES[aggr], None if b is None else _t(b, cuda), relu,
                        relu_mask=rm)
    wf, _, _ = oracle.edge_factors(ei, N, deg_norm)
    y_ref, _ = oracle.aggr_fwd(ei, X, wf, aggr, b, relu)
    np.testing.assert_array_equal(Y.cpu().numpy(), y_ref)
    if relu:
        assert torch.equal(rm, ops.make_relu_mask(Y))


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("aggr", ["add", "mean"])
def test_fused_forward_random_weights_vs_fp64(cuda, oracle, N, E, hub, aggr):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(7 * N + E)
    ei = _graph(rng, N, E, hub)
    F = 128
    X = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) * 0.1).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32)
    plan, norm = _plan(cuda, ei, N, "sm")
    Y = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, _t(X, cuda), _t(W, cuda), L.REDUCE_CODES[aggr],
                        _t(b, cuda), False).cpu().numpy().astype(np.float64)
    wf, _, _ = oracle.edge_factors(ei, N, "sm")
    Z, _ = oracle.aggr_fwd(ei, X, wf, aggr)  # the kernel's own aggregate, bit for bit
    ref = Z.astype(np.float64) @ W.astype(np.float64) + b
    bound = np.abs(Z).astype(np.float64) @ np.abs(W).astype(np.float64) + np.abs(b)
    assert (np.abs(Y - ref) <= 1e-5 * bound + 1e-6).all()
    # and against the reference's association A (X W) in fp64
    H = X.astype(np.float64) @ W.astype(np.float64)
    src, dst = ei
    w = wf.astype(np.float64)
    ref2 = np.zeros((N, F))
    np.add.at(ref2, dst, H[src] * w[:, None])
    if aggr == "mean":
        ref2 /= np.maximum(np.bincount(dst, minlength=N), 1)[:, None]
    ref2 += b
    assert (np.abs(Y - ref2) <= 1e-5 * bound + 1e-6).all()


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,epi", [("sm", "relu"), ("rw", "relu_div"), (None, "store"),
                                          ("sm", "dw_only")])
def test_fused_backward_vs_two_launch(cuda, N, E, hub, deg_norm, epi):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(3 * N + E + len(epi))
    ei = _graph(rng, N, E, hub)
    F = 128
    plan, norm = _plan(cuda, ei, N, deg_norm)
    g = torch.Generator(device=cuda).manual_seed(N)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    dY = torch.randn(N, F, device=cuda, generator=g)
    rm = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g))
    rd = plan.in_cnt if epi == "relu_div" else None
    mask = rm if epi in ("relu", "relu_div") else None
    dH = ops.spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, L.REDUCE_SUM)
    want_dx = epi != "dw_only"
    dWa, dXa, csa = ops.gemm_bwd(X, dH, W, want_dx=want_dx, relu_mask=mask, row_div=rd)
    dWb, dXb, csb = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W,
                                    want_dx=want_dx, relu_mask=mask, row_div=rd)
    if want_dx:
        assert torch.equal(dXa, dXb)
    else:
        assert dXb is None
    ref = X.double().t() @ dH.double()
    bound = X.double().abs().t() @ dH.double().abs()
    assert ((dWb.double() - ref).abs() <= 1e-5 * bound + 1e-6).all()
    if mask is not None:
        torch.testing.assert_close(csb, csa, rtol=1e-4, atol=1e-3)
        undiv = dXb if rd is None else dXb * rd[:, None]
        torch.testing.assert_close(csb.double(), undiv.double().sum(0), rtol=1e-4, atol=1e-3)
    # deterministic, and dW alone is the same dW
    dWc = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W, want_dx=False)[0]
    assert torch.equal(dWb, dWc)


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,epi", [(None, "relu"), ("sm", "store"), (None, "dw_only")])
def test_fused_max_backward_vs_two_launch(cuda, N, E, hub, deg_norm, epi):
    """Max adjoint inside the fused backward (winner bits through slot_map):
    dX bitwise equal to mgcn_spmm_bwd(MAX) + mgcn_gemm_bwd, dW within the
    fp64-bounded tolerance of X^T dH."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(7 * N + E + len(epi))
    ei = _graph(rng, N, E, hub)
    F = 128
    plan, norm = _plan(cuda, ei, N, deg_norm)
    g = torch.Generator(device=cuda).manual_seed(N + 1)
    H = torch.randn(N, F, device=cuda, generator=g)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    dY = torch.randn(N, F, device=cuda, generator=g)
    _, win = ops.spmm_fwd(plan.fwd, norm.w_fwd, H, L.REDUCE_MAX, mask_plan=plan)
    sm = plan.slot_map()
    mask = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g)) \
        if epi == "relu" else None
    dH = ops.spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, L.REDUCE_MAX, win_mask=win,
                      slot_map=sm)
    want_dx = epi != "dw_only"
    dWa, dXa, csa = ops.gemm_bwd(X, dH, W, want_dx=want_dx, relu_mask=mask)
    dWb, dXb, csb = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W,
                                    want_dx=want_dx, relu_mask=mask, win_mask=win, slot_map=sm)
    if want_dx:
        assert torch.equal(dXa, dXb)
    ref = X.double().t() @ dH.double()
    bound = X.double().abs().t() @ dH.double().abs()
    assert ((dWb.double() - ref).abs() <= 1e-5 * bound + 1e-6).all()
    if mask is not None:
        torch.testing.assert_close(csb, csa, rtol=1e-4, atol=1e-3)


def test_fused_backward_accumulate_and_empty(cuda):
    """accumulate adds into dW; zero rows give a zero dW / colsum."""
    from mgcn import _lib as L
    from mgcn import ops
    lib = L.load()
    rng = np.random.default_rng(5)
    N, F = 2000, 128
    ei = _graph(rng, N, 20000)
    plan, norm = _plan(cuda, ei, N, "sm")
    X = torch.randn(N, F, device=cuda)
    W = torch.randn(F, F, device=cuda)
    dY = torch.randn(N, F, device=cuda)
    dW = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, want_dx=False)[0]
    acc = torch.ones(F, F, device=cuda)
    ws_bytes = int(lib.mgcn_spmm_xw_bwd_workspace_bytes(N, F, F))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    v = plan.bwd
    rc = lib.mgcn_spmm_xw_bwd(N, N, F, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(norm.w_bwd), None,
                              L.ptr(dY), F, L.ptr(X), F, L.ptr(W), F, L.ptr(acc), F, 1, None, 0,
                              None, None, None, None, None, L.ptr(ws), ws_bytes,
                              L.stream_of(cuda))
    L.check(rc, "mgcn_spmm_xw_bwd")
    assert torch.equal(acc, dW + 1.0)
    dW0 = torch.full((F, F), 5.0, device=cuda)
    cs0 = torch.full((F,), 5.0, device=cuda)
    rc = lib.mgcn_spmm_xw_bwd(0, 1, F, F, L.ptr(v.rowptr), None, None, None, L.ptr(dY), F,
                              L.ptr(X), F, L.ptr(W), F, L.ptr(dW0), F, 0, L.ptr(X), F,
                              L.ptr(torch.zeros(1, 4, dtype=torch.int32, device=cuda)), None,
                              L.ptr(cs0), None, None, L.ptr(ws), ws_bytes, L.stream_of(cuda))
    L.check(rc, "mgcn_spmm_xw_bwd(empty)")
    assert not dW0.any() and not cs0.any()


def test_fused_kernels_reject_unsupported(cuda):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(6)
    N = 500
    plan, norm = _plan(cuda, _graph(rng, N, 4000), N, "sm")
    assert not plan.fwd.n_heavy
    assert ops.spmm_xw_supported(plan.fwd, 128, 128, L.REDUCE_SUM)
    assert not ops.spmm_xw_supported(plan.fwd, 64, 64, L.REDUCE_SUM)
    assert not ops.spmm_xw_supported(plan.fwd, 128, 128, L.REDUCE_MAX)
    with pytest.raises(L.MgcnError, match="unsupported"):
        ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, torch.randn(N, 64, device=cuda),
                        torch.randn(64, 64, device=cuda), L.REDUCE_SUM)
    with pytest.raises(L.MgcnError, match="unsupported"):
        ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, torch.randn(N, 128, device=cuda),
                        torch.randn(128, 128, device=cuda), L.REDUCE_MAX)


def _hub_src_graph(rng, N, E, hub):
    """Uniform in-degrees, but source 1 has `hub` extra out-edges: the fwd
    view has no heavy row, the bwd view (the adjoint's rows) has one."""
    s = np.concatenate([rng.integers(0, N, E), np.ones(hub, np.int64), np.arange(N)])
    d = np.concatenate([rng.integers(0, N, E), rng.integers(0, N, hub), np.arange(N)])
    return np.stack([s, d]).astype(np.int64)


@pytest.mark.parametrize("z_middle", [False, True], ids=["zmid0", "zmid1"])
@pytest.mark.parametrize("graph", ["er", "hub_src"])
@pytest.mark.parametrize("aggr,deg_norm,x_grad", [("add", "sm", True), ("mean", "rw", True),
                                                  ("max", None, True), ("max", "sm", True),
                                                  ("add", "sm", False), ("mean", None, False)])
def test_gcn_stack_fused_vs_two_launch(cuda, aggr, deg_norm, x_grad, graph, z_middle):
    """The stack with the fused kernels against the same stack on the
    GEMM + SpMM launches: outputs within fp32 association tolerance, dx
    bitwise below the top layer's first adjoint (same dH, same products) up
    to the forward's differences, all gradients within tolerance.  'hub_src'
    has a heavy row in the bwd view only: the fused forward applies, the
    dX-only gather must not (it falls back to spmm_bwd + gemm_bwd); z_middle
    sends the middle layer through the Z^T dY form as well."""
    from mgcn import ops
    from mgcn.graph import plan_for
    from mgcn.models import GCNLayer, GCNStack
    torch.manual_seed(0)
    rng = np.random.default_rng(13)
    N, F = 20000, 128
    ei = _t(_graph(rng, N, 200000) if graph == "er" else _hub_src_graph(rng, N, 200000, 3000),
            cuda)
    plan = plan_for(ei, N)
    assert plan.fwd.n_heavy == 0 and (plan.bwd.n_heavy > 0) == (graph == "hub_src")
    layers = [GCNLayer(F, F, deg_norm=deg_norm, aggr=aggr, bias=True,
                       non_linear='relu' if i < 2 else 'none').to(cuda) for i in range(3)]
    for layer in layers:
        with torch.no_grad():
            layer.gcn.node_models[0].bias.uniform_(-0.1, 0.1)
    stack = GCNStack(layers)
    # x_grad False: the bottom layer's backward is the dW pass alone (no gather)
    x = torch.randn(N, F, device=cuda, requires_grad=x_grad)
    dZ = torch.randn(N, F, device=cuda)
    outs = []
    for fused in (True, False):
        ops.set_fused_layers(fused)
        ops.set_z_middle(z_middle)
        try:
            for p in stack.parameters():
                p.grad = None
            x.grad = None
            y = stack(x, ei)
            y.backward(dZ)
            outs.append((y.detach(), x.grad.clone() if x_grad else None,
                         [p.grad.clone() for p in stack.parameters()]))
        finally:
            ops.set_fused_layers(True)
            ops.set_z_middle(False)
    (ya, xa, ga), (yb, xb, gb) = outs
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    if x_grad:
        torch.testing.assert_close(xa, xb, rtol=1e-4, atol=1e-5)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("kind", ["node_model_sm", "node_model_mean_relu", "gcnconv", "sageconv",
                                  "graphconv_mean"])
def test_single_layer_modules_fused_vs_two_launch(cuda, kind):
    """The conv modules route 128 -> 128 sum / mean layers through the fused
    kernels (ops.gcn_layer); against the same modules on the GEMM + SpMM
    launches: outputs within fp32 association tolerance, gradients within
    fp32 tolerance."""
    from mgcn import ops
    from mgcn.models import NodeModelAdditive
    from mgcn.pyg import GCNConv, GraphConv, SAGEConv
    torch.manual_seed(3)
    rng = np.random.default_rng(31)
    N, F = 12000, 128
    ei = _t(_graph(rng, N, 120000), cuda)
    if kind == "node_model_sm":
        m, call = NodeModelAdditive(F, F, deg_norm='sm', aggr='add', bias=True), None
    elif kind == "node_model_mean_relu":
        m = NodeModelAdditive(F, F, deg_norm='rw', aggr='mean', bias=True)
        call = lambda mod, x: mod.forward_fused(x, ei, relu=True)  # noqa: E731
    elif kind == "gcnconv":
        m, call = GCNConv(F, F), None
    elif kind == "sageconv":
        m, call = SAGEConv(F, F), None
    else:
        m, call = GraphConv(F, F, aggr='mean'), None
    m = m.to(cuda)
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() == 1:
                p.uniform_(-0.1, 0.1)
    x = torch.randn(N, F, device=cuda, requires_grad=True)
    dZ = torch.randn(N, F, device=cuda)
    outs = []
    for fused in (True, False):
        ops.set_fused_layers(fused)
        try:
            for p in m.parameters():
                p.grad = None
            x.grad = None
            y = call(m, x) if call is not None else m(x, ei)
            y.backward(dZ)
            outs.append((y.detach(), x.grad.clone(), [p.grad.clone() for p in m.parameters()]))
        finally:
            ops.set_fused_layers(True)
    (ya, xa, ga), (yb, xb, gb) = outs
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xa, xb, rtol=1e-4, atol=1e-5)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,aggr,epi", [("sm", "add", "relu"), ("rw", "mean", "relu_div"),
                                               (None, "add", "store")])
def test_z_dw_and_dx_only_backward(cuda, oracle, N, E, hub, deg_norm, aggr, epi):
    """The reassociated backward of the GCN stack: the forward's Z (the
    aggregate before W; mean: before the division) is bitwise the sum SpMM of
    X; dW = Z^T dY' (mgcn_gemm_bwd, dW only; mean: dY' = dY / count) is within
    the fp64-bounded tolerance of the reference's X^T (A^T dY); the dX-only
    backward (X = NULL, dW = NULL) is bitwise the full fused form's dX and
    column sums."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(11 * N + E + len(epi))
    ei = _graph(rng, N, E, hub)
    F = 128
    plan, norm = _plan(cuda, ei, N, deg_norm)
    reduce = L.REDUCE_CODES[aggr]
    g = torch.Generator(device=cuda).manual_seed(N + 7)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    dY = torch.randn(N, F, device=cuda, generator=g)
    Y0 = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, reduce)
    Y, Z = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, reduce, want_z=True)
    assert torch.equal(Y, Y0)
    Zs = ops.spmm_fwd(plan.fwd, norm.w_fwd, X, L.REDUCE_SUM)
    Zs = Zs[0] if isinstance(Zs, tuple) else Zs
    assert torch.equal(Z, Zs)
    # dW from Z: mean pairs the undivided Z with the pre-divided dY
    dYp = dY / plan.in_cnt[:, None] if aggr == "mean" else dY
    dW = ops.gemm_bwd(Z, dYp, W, want_dx=False)[0]
    dH = ops.spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dYp, L.REDUCE_SUM)
    ref = X.double().t() @ dH.double()
    bound = X.double().abs().t() @ dH.double().abs()
    # two fp32-rounded association orders of the same product
    assert ((dW.double() - ref).abs() <= 4e-5 * bound + 1e-6).all()
    # the dW-only pass with dH's column sums (the top layer's bias gradient)
    dW2, dX2, cs = ops.gemm_bwd(Z, dYp, W, want_dx=False, dh_colsum=True)
    assert dX2 is None and torch.equal(dW2, dW)
    torch.testing.assert_close(cs.double(), dYp.double().sum(0), rtol=1e-5, atol=1e-4)
    rm = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g))
    rd = plan.in_cnt if epi == "relu_div" else None
    mask = rm if epi in ("relu", "relu_div") else None
    _, dXa, csa = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dYp, X, W,
                                  relu_mask=mask, row_div=rd)
    dWb, dXb, csb = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dYp, None, W,
                                    relu_mask=mask, row_div=rd)
    assert dWb is None
    assert torch.equal(dXa, dXb)
    if mask is not None:
        # (the warp-specialised dX-only form folds the column sums in its own
        # order: within fp32 summation-order tolerance of the full form's)
        torch.testing.assert_close(csa, csb, rtol=1e-5, atol=1e-4)
    with pytest.raises(ValueError, match="dX only"):
        ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dYp, None, W, want_dx=False)


@pytest.mark.parametrize("acts", [("none", "none"), ("relu", "none"), ("none", "relu", "none")])
def test_gcn_stack_keeps_z_only_where_the_backward_reads_it(cuda, acts):
    """The forward stores the aggregate Z of a layer only when the backward
    forms that layer's dW as Z^T dY: the bottom layer, or a layer whose lower
    layer ends in a ReLU (its mask feeds the dX-only gather's epilogue) --
    except the top layer when ops._TOP_FULL is set (it then takes the dW + dX
    adjoint with its bias gradient in the same launch and keeps no Z).  A
    layer above a 'none' layer keeps no N x F Z (and its gradients still
    match the two-launch stack)."""
    from mgcn import ops
    from mgcn.models import GCNLayer, GCNStack
    torch.manual_seed(1)
    rng = np.random.default_rng(17)
    N, F = 6000, 128
    ei = _t(_graph(rng, N, 60000), cuda)
    n = len(acts)
    stack = GCNStack([GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                               non_linear=a).to(cuda) for a in acts])
    x = torch.randn(N, F, device=cuda, requires_grad=True)
    dZ = torch.randn(N, F, device=cuda)
    y = stack(x, ei)
    zs = y.grad_fn.saved_tensors[5 * n:6 * n]
    for i in range(n):
        want = i == 0 or (acts[i - 1] == "relu" and i == n - 1 and not ops._TOP_FULL)
        assert (zs[i].numel() > 0) == want, (i, acts)
    y.backward(dZ)
    got = [x.grad.clone()] + [p.grad.clone() for p in stack.parameters()]
    ops.set_fused_layers(False)
    try:
        x.grad = None
        for p in stack.parameters():
            p.grad = None
        stack(x, ei).backward(dZ)
    finally:
        ops.set_fused_layers(True)
    ref = [x.grad] + [p.grad for p in stack.parameters()]
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)


def test_spmm_xw_fwd_validates_relu_mask(cuda):
    """A wrongly shaped / typed mask would be an out-of-bounds device write."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(2)
    N = 300
    plan, norm = _plan(cuda, _graph(rng, N, 2000), N, "sm")
    X = torch.randn(N, 128, device=cuda)
    W = torch.randn(128, 128, device=cuda)
    for bad in (torch.empty(N - 1, 4, dtype=torch.int32, device=cuda),
                torch.empty(N, 4, dtype=torch.int64, device=cuda),
                torch.empty(4, N, dtype=torch.int32, device=cuda).t()):
        with pytest.raises(ValueError, match="relu_mask"):
            ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, relu=True, relu_mask=bad)
    with pytest.raises(ValueError, match="needs relu"):
        ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, relu=False,
                        relu_mask=torch.empty(N, 4, dtype=torch.int32, device=cuda))


def test_fused_gating_beyond_32bit_offsets(cuda):
    """N = 8.5M nodes at F = 128: the gathered tables (X forward, dY
    backward) are 4.35 GB, past the fused kernels' 32-bit offsets
    (mgcn_spmm_xw_fwd / _bwd reject them).  GCNStack and GCNConv must route
    such graphs to the two-launch path (64-bit offsets) instead of raising;
    sampled output rows of a GCNConv layer against fp64 (|err| <= 1e-5 *
    the |.|-weighted sum), and the stack's output and dx equal to the same
    stack with the fused kernels switched off."""
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import plan_for
    from mgcn.models import GCNLayer, GCNStack
    from mgcn.pyg import GCNConv
    N, F, E = 8_500_000, 128, 25_000_000
    g = torch.Generator(device=cuda).manual_seed(0)
    s = torch.randint(0, N, (E,), device=cuda, generator=g)
    d = torch.randint(0, N, (E,), device=cuda, generator=g)
    loops = torch.arange(N, device=cuda)
    ei = torch.stack([torch.cat([s, loops]), torch.cat([d, loops])])
    del s, d
    x = torch.randn(N, F, device=cuda, generator=g)
    plan = plan_for(ei, N)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    assert plan.fwd.n_heavy == 0 and plan.bwd.n_heavy == 0
    assert not ops.spmm_xw_supported(plan.fwd, F, F, L.REDUCE_SUM)
    assert not ops.layer_fusable(plan, x, W, L.REDUCE_SUM)
    from mgcn.graph import CSRView
    edge = CSRView(rowptr=plan.fwd.rowptr, col=plan.fwd.col, eid=plan.fwd.eid, n_rows=N,
                   n_cols=8_388_607)  # the largest table the kernels take at F = 128
    assert ops.spmm_xw_supported(edge, F, F, L.REDUCE_SUM)
    edge.n_cols += 1
    assert not ops.spmm_xw_supported(edge, F, F, L.REDUCE_SUM)

    conv = GCNConv(F, F).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(W)
        conv.bias.uniform_(-0.1, 0.1)
    y = conv(x, ei)
    torch.cuda.synchronize()
    rows = torch.from_numpy(np.random.default_rng(1).choice(N, 512, replace=False)).to(cuda)
    # GCNConv drops the graph's own loops and appends one per node: every
    # random self-pair is dropped, so the edges are the non-loop pairs + loops
    src, dst = ei
    keep = src != dst
    keep[E:] = True
    src, dst = src[keep], dst[keep]
    deg = torch.bincount(src, minlength=N).double()
    dinv = deg.pow(-0.5)
    sel = torch.isin(dst, rows)
    es, ed = src[sel], dst[sel]
    w = dinv[es] * dinv[ed]
    H = x[es].double() @ W.double()
    Hm = x[es].double().abs() @ W.double().abs()
    pos = torch.searchsorted(rows.sort().values, ed)
    ref = torch.zeros(rows.numel(), F, dtype=torch.float64, device=cuda)
    bnd = torch.zeros_like(ref)
    ref.index_add_(0, pos, H * w[:, None])
    bnd.index_add_(0, pos, Hm * w[:, None])
    rs = rows.sort().values
    ref += conv.bias.double()
    bnd += conv.bias.double().abs()
    err = (y[rs].double() - ref).abs()
    assert bool((err <= 1e-5 * bnd + 1e-6).all()), float((err / bnd).max())
    del y, conv

    torch.manual_seed(2)
    stack = GCNStack([GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                               non_linear=a).to(cuda) for a in ("relu", "none")])
    xg = x.requires_grad_(True)
    dZ = torch.randn(N, F, device=cuda, generator=g)
    outs = []
    for fused in (True, False):
        ops.set_fused_layers(fused)
        try:
            xg.grad = None
            yy = stack(xg, ei)
            yy.backward(dZ)
            outs.append((yy.detach()[rs], xg.grad[rs].clone()))
            del yy
        finally:
            ops.set_fused_layers(True)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
