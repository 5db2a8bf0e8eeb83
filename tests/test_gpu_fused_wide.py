"""GPU parity of the 256-wide fused layer kernels (fused_wide.hip: config 5's
F = 256, BASELINE.json configs[4]) -- mgcn_spmm_xw_fwd / the dX-only
mgcn_spmm_xw_bwd at F_in = F_out = 256, and the stacks that run on them.

Reference: NodeModelAdditive's x @ W then gather -> * norm -> scatter_add
(src/gcn_meta/models/gcn_base_models.py:201, 223-241) and its autograd
adjoints.  Bars:
  * W = I: every bf16x6 product is exact, so the forward (Y, Z, the ReLU mask
    words) and the adjoint's dX equal the C oracle BIT FOR BIT;
  * random W: |Y - Y64| <= 1e-5 (|Z| |W| + |b|) + 1e-6 with Y64 the fp64
    product of the bit-exact aggregate Z; dX likewise against the fp64
    dH W^T of the bit-exact adjoint dH;
  * a gathered table past 4 GiB (5M rows x 1 KB) through both kernels;
  * GCNStack 256 -> 256 (3 layers): y and x.grad bit for bit the oracle
    chain at W = I, every dW / db within the |.|-weighted fp64 bound.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F = 256


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _graph(rng, N, E, hub=0):
    s = rng.integers(0, N, E)
    d = rng.integers(0, N, E)
    if hub:
        d = np.concatenate([d, np.zeros(hub, np.int64), rng.integers(0, N, hub)])
        s = np.concatenate([s, rng.integers(0, N, hub), np.ones(hub, np.int64)])
    s = np.concatenate([s, np.arange(N)])
    d = np.concatenate([d, np.arange(N)])
    return np.stack([s, d]).astype(np.int64)


GRAPHS = [(20000, 200000, 0), (4097, 40000, 0), (33, 100, 0), (1, 0, 0), (3000, 20000, 700)]


@pytest.fixture(autouse=True, params=[3, 0], ids=["ws", "legacy"])
def wide_form(request):
    """Every test runs on the warp-specialised kernels (wide_ws = 3, the
    default) and on the 16-row two-workgroup form (wide_ws = 0)."""
    from mgcn import _lib as L
    L.set_option("wide_ws", request.param)
    yield request.param
    L.set_option("wide_ws", 3)


def _plan(cuda, ei, N, deg_norm):
    from mgcn.graph import plan_for
    plan = plan_for(_t(ei, cuda), N)
    return plan, plan.norm(deg_norm)


def _mask_words(Y):
    """[N, 256] -> the 8-word ReLU mask layout (feature f: word 4 (f >> 7) +
    (f & 3), bit (f & 127) >> 2)."""
    pos = (Y > 0)
    N = Y.shape[0]
    out = np.zeros((N, 8), np.uint32)
    for f in range(F):
        out[:, 4 * (f >> 7) + (f & 3)] |= pos[:, f].astype(np.uint32) << np.uint32((f & 127) >> 2)
    return out.view(np.int32)


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,aggr,bias,relu", [("sm", "add", True, True),
                                                     ("rw", "mean", False, True),
                                                     (None, "add", True, False),
                                                     ("sm", "mean", True, False)])
def test_wide_forward_identity_weights_bitwise(cuda, oracle, N, E, hub, deg_norm, aggr, bias,
                                               relu):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(N + E + hub + 1)
    ei = _graph(rng, N, E, hub)
    X = rng.standard_normal((N, F)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32) if bias else None
    plan, norm = _plan(cuda, ei, N, deg_norm)
    rm = torch.empty(N, 8, dtype=torch.int32, device=cuda) if relu else None
    Y, Z = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, _t(X, cuda), torch.eye(F, device=cuda),
                           L.REDUCE_CODES[aggr], None if b is None else _t(b, cuda), relu,
                           relu_mask=rm, want_z=True)
    wf, _, _ = oracle.edge_factors(ei, N, deg_norm)
    y_ref, _ = oracle.aggr_fwd(ei, X, wf, aggr, b, relu)
    np.testing.assert_array_equal(Y.cpu().numpy(), y_ref)
    z_ref, _ = oracle.aggr_fwd(ei, X, wf, "add")  # Z: the undivided aggregate
    np.testing.assert_array_equal(Z.cpu().numpy(), z_ref)
    if relu:
        np.testing.assert_array_equal(rm.cpu().numpy(), _mask_words(y_ref))


@pytest.mark.parametrize("N,E,hub", GRAPHS[:3] + GRAPHS[4:])
@pytest.mark.parametrize("aggr", ["add", "mean"])
def test_wide_forward_random_weights_vs_fp64(cuda, oracle, N, E, hub, aggr):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(7 * N + E + 5)
    ei = _graph(rng, N, E, hub)
    X = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) * 0.1).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32)
    plan, norm = _plan(cuda, ei, N, "sm")
    Y = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, _t(X, cuda), _t(W, cuda), L.REDUCE_CODES[aggr],
                        _t(b, cuda), False).cpu().numpy().astype(np.float64)
    wf, _, _ = oracle.edge_factors(ei, N, "sm")
    Z, _ = oracle.aggr_fwd(ei, X, wf, aggr)
    ref = Z.astype(np.float64) @ W.astype(np.float64) + b
    bound = np.abs(Z).astype(np.float64) @ np.abs(W).astype(np.float64) + np.abs(b)
    err = np.abs(Y - ref)
    assert (err <= 1e-5 * bound + 1e-6).all(), float((err / (bound + 1e-6)).max())


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,epi", [("sm", "relu"), ("rw", "relu_div"), (None, "store")])
def test_wide_backward_dx_identity_bitwise(cuda, oracle, N, E, hub, deg_norm, epi):
    """dX-only adjoint at W = I: dX = relu'(lower) (A^T dY) [/ count] bit for
    bit the oracle adjoint; the column sums within fp32 order tolerance."""
    from mgcn import ops
    rng = np.random.default_rng(3 * N + E + len(epi))
    ei = _graph(rng, N, E, hub)
    plan, norm = _plan(cuda, ei, N, deg_norm)
    dY = rng.standard_normal((N, F)).astype(np.float32)
    lower = rng.standard_normal((N, F)).astype(np.float32)  # the lower layer's output
    rm = rd = None
    if epi != "store":
        rm = _t(_mask_words(lower), cuda)
    if epi == "relu_div":
        rd = plan.in_cnt
    _, dX, cs = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, _t(dY, cuda), None,
                                torch.eye(F, device=cuda), relu_mask=rm, row_div=rd)
    _, wb, rs = oracle.edge_factors(ei, N, deg_norm)
    dH, _ = oracle.aggr_bwd(ei, dY, wb, rs, "add")
    ref = dH
    if epi != "store":
        ref = np.where(lower > 0, dH, 0).astype(np.float32)
        cs_ref = ref.astype(np.float64).sum(0)
        assert np.allclose(cs.cpu().numpy(), cs_ref, rtol=1e-4,
                           atol=1e-4 * max(1.0, float(np.abs(ref).sum(0).max())))
    if epi == "relu_div":
        cnt = np.maximum(np.bincount(ei[1], minlength=N), 1).astype(np.float32)
        ref = (ref / cnt[:, None]).astype(np.float32)
    np.testing.assert_array_equal(dX.cpu().numpy(), ref)


@pytest.mark.parametrize("N,E,hub", GRAPHS[:2] + GRAPHS[4:])
def test_wide_backward_dx_random_weights_vs_fp64(cuda, oracle, N, E, hub):
    from mgcn import ops
    rng = np.random.default_rng(11 * N + E)
    ei = _graph(rng, N, E, hub)
    plan, norm = _plan(cuda, ei, N, "sm")
    dY = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) * 0.1).astype(np.float32)
    lower = rng.standard_normal((N, F)).astype(np.float32)
    _, dX, cs = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, _t(dY, cuda), None, _t(W, cuda),
                                relu_mask=_t(_mask_words(lower), cuda))
    _, wb, rs = oracle.edge_factors(ei, N, "sm")
    dH, _ = oracle.aggr_bwd(ei, dY, wb, rs, "add")  # the kernel's own dH, bit for bit
    m = lower > 0
    ref = np.where(m, dH.astype(np.float64) @ W.T.astype(np.float64), 0)
    bound = np.where(m, np.abs(dH).astype(np.float64) @ np.abs(W).T.astype(np.float64), 0)
    err = np.abs(dX.cpu().numpy().astype(np.float64) - ref)
    assert (err <= 1e-5 * bound + 1e-6).all(), float((err / (bound + 1e-6)).max())


def test_wide_kernels_gather_from_a_table_past_4gib(cuda, oracle):
    """5M source rows x 1 KB = 5.1 GB gathered by 24k destination rows (most
    byte offsets beyond 2^32): the forward and the dX-only adjoint bit for
    bit the oracle at W = I (the F = 128 kernels stop at 4 GiB)."""
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import build_view
    T, R, E = 5_000_000, 24_000, 260_000
    rng = np.random.default_rng(5)
    src = rng.integers(0, T, E)
    dst = rng.integers(0, R, E)
    src[:R], dst[:R] = T - 1 - np.arange(R), np.arange(R)  # the table's last rows too
    g = torch.Generator(device=cuda).manual_seed(1)
    X = torch.randn(T, F, device=cuda, generator=g)
    assert X.numel() * 4 > 2 ** 32
    w = rng.uniform(0.1, 1.0, E).astype(np.float32)
    fwd = build_view(_t(dst, cuda), _t(src, cuda), R, T)
    wf = _t(w, cuda)[fwd.eid.long()]
    eye = torch.eye(F, device=cuda)
    Y = ops.spmm_xw_fwd(fwd, wf, X, eye, L.REDUCE_SUM)
    Xh = X.cpu().numpy()
    ei = np.stack([src, dst])
    y_ref, _ = oracle.aggr_fwd(ei, Xh, w, "add", num_nodes=R)
    np.testing.assert_array_equal(Y.cpu().numpy(), y_ref)
    # the adjoint gathers dY over the transposed slots: here the [T, 256]
    # table is dY of a "layer" whose rows are the R destinations' sources
    bwd = build_view(_t(dst, cuda), _t(src, cuda), R, T)  # rows R, cols T: the same shape
    _, dX, _ = ops.spmm_xw_bwd(bwd, wf, None, X, None, eye)
    np.testing.assert_array_equal(dX.cpu().numpy(), y_ref)


def _stack(cuda, Ws, bs):
    from mgcn.models import GCNLayer, GCNStack
    layers = []
    for i, (W, b) in enumerate(zip(Ws, bs)):
        layer = GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                         non_linear='relu' if i < len(Ws) - 1 else 'none').to(cuda)
        with torch.no_grad():
            layer.gcn.node_models[0].weight_node.copy_(W)
            layer.gcn.node_models[0].bias.copy_(b)
        layers.append(layer)
    return GCNStack(layers)


def test_wide_stack_identity_bitwise_and_on_fused_kernels(cuda, oracle):
    """GCNStack of three 256 -> 256 layers (config 5's model) at W = I: y and
    x.grad bit for bit the oracle chain, on the fused kernels (forward with
    Z, dX-only adjoint, dense Z^T dY dW) -- no two-launch SpMM runs."""
    from mgcn import ops
    rng = np.random.default_rng(21)
    N = 30000
    ei = _graph(rng, N, 300000)
    X = rng.standard_normal((N, F)).astype(np.float32)
    dY = rng.standard_normal((N, F)).astype(np.float32)
    bs = [torch.from_numpy(rng.uniform(-0.1, 0.1, F).astype(np.float32)) for _ in range(3)]
    stack = _stack(cuda, [torch.eye(F)] * 3, bs)
    names = []
    ops.set_kernel_timer(lambda name, start, *a: names.append(name) if start else None)
    try:
        x = _t(X, cuda).requires_grad_(True)
        y = stack(x, _t(ei, cuda))
        y.backward(_t(dY, cuda))
        torch.cuda.synchronize()
    finally:
        ops.set_kernel_timer(None)
    assert "spmm_fwd" not in names and "spmm_bwd" not in names, names
    assert names.count("spmm_xw_fwd_z") == 3 and names.count("spmm_xw_bwd_dx") == 3, names
    wf, wb, rs = oracle.edge_factors(ei, N, "sm")
    h, outs = X, []
    for l in range(3):
        h, _ = oracle.aggr_fwd(ei, h, wf, "add", bs[l].numpy(), relu=l < 2)
        outs.append(h)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), outs[-1])
    g = dY
    for l in range(2, -1, -1):
        g, _ = oracle.aggr_bwd(ei, g, wb, rs, "add", outs[l], l < 2, None)
    np.testing.assert_array_equal(x.grad.cpu().numpy(), g)


def test_wide_stack_random_weights_vs_fp64(cuda, oracle):
    """The same stack with glorot weights: each layer's output at its own
    input, every dW / db and dx within 1e-5 of the |.|-weighted fp64 chain
    (the ReLU decisions from the stack's own activations)."""
    from fp64_ref import A64, within
    from mgcn.models import GCNStack
    rng = np.random.default_rng(22)
    N = 30000
    ei = _graph(rng, N, 300000)
    a = (6.0 / (2 * F)) ** 0.5
    Ws = [torch.from_numpy(rng.uniform(-a, a, (F, F)).astype(np.float32)) for _ in range(3)]
    bs = [torch.from_numpy(rng.uniform(-0.1, 0.1, F).astype(np.float32)) for _ in range(3)]
    X = _t(rng.standard_normal((N, F)).astype(np.float32), cuda)
    dY = _t(rng.standard_normal((N, F)).astype(np.float32), cuda)
    stack = _stack(cuda, Ws, bs)
    eic = _t(ei, cuda)
    x = X.clone().requires_grad_(True)
    y = stack(x, eic)
    y.backward(dY)
    params = list(stack.parameters())
    gW = [p.grad for p in params[0::2]]
    gb = [p.grad for p in params[1::2]]
    with torch.no_grad():
        acts = [X, GCNStack(stack.layers[:1])(X, eic), GCNStack(stack.layers[:2])(X, eic)]
    wf, _, _ = oracle.edge_factors(ei, N, "sm")
    A = A64(torch.from_numpy(ei), wf, N, cuda)
    W64 = [w.to(cuda, torch.float64) for w in Ws]
    b64 = [b.to(cuda, torch.float64) for b in bs]
    outs = acts[1:] + [y.detach()]
    for l in range(3):
        xin = acts[l].double()
        ref = A.apply(xin @ W64[l]) + b64[l]
        if l < 2:
            ref = ref.clamp_min(0)
        bound = A.apply(xin.abs() @ W64[l].abs(), absolute=True) + b64[l].abs()
        ok, worst = within(outs[l].double() - ref, bound, 1e-5)
        assert ok, ("forward", l, worst)
    g, gm = dY.double(), dY.double().abs()
    for l in range(2, -1, -1):
        dH = A.apply(g, transpose=True)
        dHm = A.apply(gm, transpose=True, absolute=True)
        xin = acts[l].double()
        ok, worst = within(gW[l].double() - xin.t() @ dH, xin.abs().t() @ dHm, 1e-5)
        assert ok, ("dW", l, worst)
        ok, worst = within(gb[l].double() - g.sum(0), gm.sum(0), 1e-5)
        assert ok, ("db", l, worst)
        dX, dXm = dH @ W64[l].t(), dHm @ W64[l].abs().t()
        if l == 0:
            ok, worst = within(x.grad.double() - dX, dXm, 1e-5)
            assert ok, ("dx", worst)
        else:
            mask = (acts[l] > 0).double()
            g, gm = dX * mask, dXm * mask


def test_wide_stack_frozen_middle_weight(cuda, oracle):
    """a 256-wide stack whose middle weight needs no gradient (and
    a frozen bottom one).  The middle layer keeps no Z, so its backward runs
    the dX-only adjoint with the 8-word ReLU mask of the layer below (no dW
    product, no 4-word-mask GEMM epilogue); the other gradients equal the
    unfrozen stack's bit for bit, the frozen weights get none."""
    rng = np.random.default_rng(31)
    N = 20000
    ei = _graph(rng, N, 200000)
    a = (6.0 / (2 * F)) ** 0.5
    Ws = [torch.from_numpy(rng.uniform(-a, a, (F, F)).astype(np.float32)) for _ in range(3)]
    bs = [torch.from_numpy(rng.uniform(-0.1, 0.1, F).astype(np.float32)) for _ in range(3)]
    X = _t(rng.standard_normal((N, F)).astype(np.float32), cuda)
    dY = _t(rng.standard_normal((N, F)).astype(np.float32), cuda)
    eic = _t(ei, cuda)
    res = []
    for frozen in ((), (1,), (0, 1)):
        stack = _stack(cuda, Ws, bs)
        params = list(stack.parameters())
        for l in frozen:
            params[2 * l].requires_grad_(False)
        x = X.clone().requires_grad_(True)
        y = stack(x, eic)
        y.backward(dY)
        for l in frozen:
            assert params[2 * l].grad is None
        res.append((y.detach(), x.grad, [p.grad for p in params]))
    base = res[0]
    for y, gx, grads in res[1:]:
        assert torch.equal(y, base[0]) and torch.equal(gx, base[1])
        for g, g0 in zip(grads, base[2]):
            if g is not None:
                assert torch.equal(g, g0)


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("aggr", ["add", "mean"])
def test_wide_forms_agree_bitwise(cuda, wide_form, N, E, hub, aggr):
    """Random W, bias, ReLU: the warp-specialised kernels (W^T image as the A
    operand, the same six products per k-step in the same order) give the
    16-row kernels' Y, Z, mask words and dX bit for bit; column sums agree
    within fp32 reordering."""
    from mgcn import _lib as L
    from mgcn import ops
    if wide_form != 3:
        pytest.skip("one comparison per graph")
    rng = np.random.default_rng(5 * N + E + hub)
    ei = _graph(rng, N, E, hub)
    plan, norm = _plan(cuda, ei, N, "sm")
    X = _t(rng.standard_normal((N, F)).astype(np.float32), cuda)
    W = _t((rng.standard_normal((F, F)) * 0.1).astype(np.float32), cuda)
    b = _t(rng.uniform(-0.5, 0.5, F).astype(np.float32), cuda)
    lower = _t(_mask_words(rng.standard_normal((N, F)).astype(np.float32)), cuda)
    rd = plan.in_cnt if aggr == "mean" else None
    out = {}
    for form in (3, 0):
        L.set_option("wide_ws", form)
        rm = torch.empty(N, 8, dtype=torch.int32, device=cuda)
        Y, Z = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_CODES[aggr], b, True,
                               relu_mask=rm, want_z=True)
        _, dX, cs = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, X, None, W, relu_mask=lower,
                                    row_div=rd)
        out[form] = (Y, Z, rm, dX, cs)
    L.set_option("wide_ws", 3)
    for a, c in zip(out[3][:4], out[0][:4]):
        assert torch.equal(a, c)
    torch.testing.assert_close(out[3][4], out[0][4], rtol=1e-5, atol=1e-4)
