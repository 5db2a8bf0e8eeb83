"""GPU parity of the warp-specialised F = 128 adjoint (fused.hip,
spmm_xw_bwd_ws_kernel, DWS): mgcn_spmm_xw_bwd's dW + dX form (mgcn_set_option
"xw_ws_full" 1, the default), its max adjoint and its dY column sums
(mgcn_spmm_xw_bwd_hcs), against the two-phase kernel and the oracle; the
dense dW passes (mgcn_gemm_bwd dW-only, mgcn_gemm_bwd_dw_cs).

Reference: the adjoints of NodeModelAdditive's x @ W then gather -> * norm ->
scatter_add (src/gcn_meta/models/gcn_base_models.py:201, 223-241).
Bars:
  * dX bit for bit the two-phase kernel's and, at W = I, the oracle adjoint's;
  * dW within the |.|-weighted fp64 bound of X^T dH (two fp32 association
    orders of one product); column sums within fp32 summation-order tolerance;
  * empty / 1-row / ragged chunks, guard bands around every output;
  * the GCN stack on DWS against the two-phase stack.
(The dX-only warp-specialised form and DWL -- the lower layer's dW fused into
the dX-only adjoint -- and the LDS-free / warp-specialised dW passes were
measured slower and removed in round 6; their tests went with them.)
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F = 128


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


def _plan(cuda, ei, N, deg_norm):
    from mgcn.graph import plan_for
    plan = plan_for(_t(ei, cuda), N)
    return plan, plan.norm(deg_norm)


SENT = 0x7FBADBAD
BAND = 4096


def _guarded(shape, dev, dtype=torch.float32):
    n = int(np.prod(shape))
    base = torch.full((BAND + n + BAND,), SENT, dtype=torch.int32, device=dev)
    mid = base[BAND:BAND + n]
    if dtype == torch.float32:
        mid = mid.view(torch.float32)
    return base, mid.view(*shape)


def _intact(base):
    torch.cuda.synchronize()
    return bool((base[:BAND] == SENT).all()) and bool((base[base.numel() - BAND:] == SENT).all())


@pytest.fixture
def xw_ws_full():
    from mgcn import _lib as L
    yield lambda v: L.set_option("xw_ws_full", v)
    L.set_option("xw_ws_full", 1)  # the default


@pytest.mark.parametrize("N,E,hub", GRAPHS)
@pytest.mark.parametrize("deg_norm,epi", [("sm", "relu"), ("rw", "relu_div"), (None, "store")])
def test_ws_full_matches_two_phase(cuda, oracle, xw_ws_full, N, E, hub, deg_norm, epi):
    """mgcn_spmm_xw_bwd's dW + dX form on the warp-specialised kernel
    (mgcn_set_option "xw_ws_full" 1, DWS): dX bit for bit the two-phase full
    kernel's (and the oracle adjoint's at W = I), dW = X^T (A^T dY) within the
    fp64 |.|-bound and the two-phase dW within twice it (split-K order)."""
    from mgcn import ops
    rng = np.random.default_rng(7 * N + E + len(epi))
    ei = _graph(rng, N, E, hub)
    plan, norm = _plan(cuda, ei, N, deg_norm)
    g = torch.Generator(device=cuda).manual_seed(N + 29)
    dY = torch.randn(N, F, device=cuda, generator=g)
    X = torch.randn(N, F, device=cuda, generator=g)
    lower = torch.randn(N, F, device=cuda, generator=g)
    rm = ops.make_relu_mask(lower) if epi != "store" else None
    rd = plan.in_cnt if epi == "relu_div" else None
    Wr = torch.randn(F, F, device=cuda, generator=g) * 0.1
    out = {}
    for form in (1, 0):
        xw_ws_full(form)
        for name, W in (("eye", torch.eye(F, device=cuda)), ("rand", Wr)):
            out[form, name] = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W,
                                              relu_mask=rm, row_div=rd)
    # the adjoint dH = A^T dY in fp64 (the kernels' dH is the SpMM's, bit for bit)
    _, wb, rs = oracle.edge_factors(ei, N, deg_norm)
    dH, _ = oracle.aggr_bwd(ei, dY.cpu().numpy(), wb, rs, "add")
    dH = torch.from_numpy(np.asarray(dH)).to(cuda).double()
    ref = X.double().t() @ dH
    bound = X.double().abs().t() @ dH.abs()
    for name in ("eye", "rand"):
        dW1, dX1, cs1 = out[1, name]
        dW0, dX0, cs0 = out[0, name]
        assert torch.equal(dX1, dX0)
        if rm is not None:
            torch.testing.assert_close(cs1, cs0, rtol=1e-5, atol=1e-4)
        assert ((dW1.double() - ref).abs() <= 4e-5 * bound + 1e-6).all()
        assert ((dW1.double() - dW0.double()).abs() <= 8e-5 * bound + 1e-6).all()
    refx = dH.float().cpu().numpy()
    if epi != "store":
        refx = np.where(lower.cpu().numpy() > 0, refx, 0).astype(np.float32)
    if epi == "relu_div":
        cnt = np.maximum(np.bincount(ei[1], minlength=N), 1).astype(np.float32)
        refx = (refx / cnt[:, None]).astype(np.float32)
    np.testing.assert_array_equal(out[1, "eye"][1].cpu().numpy(), refx)


def test_ws_full_guard_bands_on_row_chunks(cuda, xw_ws_full):
    """The DWS form on row-range views at 1, 15, 17, 31, 33, 190 rows and
    empty: dX / colsum / dW / workspace bands untouched, dX rows bit for bit
    the whole view's, dW the chunk's own X^T dH within the fp64 bound."""
    from mgcn import _lib as L
    from mgcn import ops
    N = 600
    rng = np.random.default_rng(19)
    ei = _graph(rng, N, 5000)
    plan, norm = _plan(cuda, ei, N, "sm")
    lib = L.load()
    g = torch.Generator(device=cuda).manual_seed(6)
    dY = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    X = torch.randn(N, F, device=cuda, generator=g)
    rm = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g))
    xw_ws_full(1)
    _, dXf, _ = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, relu_mask=rm)
    dHf = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, torch.eye(F, device=cuda))[1]
    for a in (0, 5, 211):
        for n in (1, 15, 17, 31, 33, 190, 0):
            if a + n > N:
                continue
            v = plan.bwd.rows(a, a + n)
            bx, dX = _guarded((max(n, 1), F), cuda)
            bc, cs = _guarded((F,), cuda)
            bw, dW = _guarded((F, F), cuda)
            wsb = int(lib.mgcn_spmm_xw_bwd_workspace_bytes(n, F, F))
            bws, ws = _guarded((max(wsb // 4, 1),), cuda)
            with L.device_guard(cuda):
                rc = lib.mgcn_spmm_xw_bwd(
                    n, v.n_cols, F, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(norm.w_bwd), None,
                    L.ptr(dY), F, L.ptr(X[a:]), F, L.ptr(W), F, L.ptr(dW), F, 0, L.ptr(dX), F,
                    L.ptr(rm[a:]), None, L.ptr(cs), None, None, L.ptr(ws), wsb, L.stream_of(cuda))
            L.check(rc, "mgcn_spmm_xw_bwd")
            for b in (bx, bc, bw, bws):
                assert _intact(b), (a, n)
            if n:
                assert torch.equal(dX, dXf[a:a + n])
                dH = dHf[a:a + n].double()
                ref = X[a:a + n].double().t() @ dH
                bound = X[a:a + n].double().abs().t() @ dH.abs()
                assert ((dW.double() - ref).abs() <= 4e-5 * bound + 1e-6).all()
            else:
                assert (dW == 0).all()


@pytest.mark.parametrize("aggr,deg_norm", [("add", "sm"), ("mean", "rw")])
def test_stack_ws_full_vs_two_phase(cuda, xw_ws_full, aggr, deg_norm):
    """A 4-layer 128-wide stack whose middle layers take the full adjoint: the
    DWS form against the two-phase kernel -- y and x.grad bitwise, every
    dW / db within tolerance."""
    from mgcn.models import GCNLayer, GCNStack
    torch.manual_seed(4)
    rng = np.random.default_rng(29)
    N = 8000
    ei = _t(_graph(rng, N, 80000), cuda)
    stack = GCNStack([GCNLayer(F, F, deg_norm=deg_norm, aggr=aggr, bias=True,
                               non_linear="relu" if i < 3 else "none").to(cuda) for i in range(4)])
    x = torch.randn(N, F, device=cuda, requires_grad=True)
    dZ = torch.randn(N, F, device=cuda)
    res = []
    for form in (1, 0):
        xw_ws_full(form)
        x.grad = None
        for p in stack.parameters():
            p.grad = None
        y = stack(x, ei)
        y.backward(dZ)
        res.append((y.detach(), x.grad.clone(), [p.grad.clone() for p in stack.parameters()]))
    (ya, xa, ga), (yb, xb, gb) = res
    assert torch.equal(ya, yb) and torch.equal(xa, xb)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("N,E", [(20000, 200000), (33, 100), (1, 0), (4097, 40000)])
def test_ws_full_hcs_column_sums(cuda, N, E):
    """mgcn_spmm_xw_bwd_hcs: the DWS adjoint plus the column sums of dY (the
    layer's own bias gradient) from the same launch -- dW / dX / colsum bit for
    bit the plain DWS call's, dy_colsum within the fp64 |.|-bound of dY.sum(0);
    a non-square view is refused."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(N + 3)
    ei = _graph(rng, N, E)
    plan, norm = _plan(cuda, ei, N, "sm")
    g = torch.Generator(device=cuda).manual_seed(N + 31)
    dY = torch.randn(N, F, device=cuda, generator=g)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    rm = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g))
    hc = torch.full((F,), float("nan"), device=cuda)
    a = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, relu_mask=rm, dy_colsum_out=hc)
    L.set_option("xw_ws_full", 1)
    b = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, relu_mask=rm)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    ref = dY.double().sum(0)
    bound = dY.double().abs().sum(0)
    assert ((hc.double() - ref).abs() <= 1e-5 * bound + 1e-6).all()
    if N > 40:
        v = plan.bwd.rows(0, N // 2)
        with pytest.raises(ValueError):
            ops.spmm_xw_bwd(v, norm.w_bwd, None, dY, X[:N // 2], W, dy_colsum_out=hc)


@pytest.mark.parametrize("aggr,deg_norm", [("add", "sm"), ("mean", "rw")])
@pytest.mark.parametrize("hcs,defer", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("layers", [2, 3])
def test_stack_top_full_vs_z_form(cuda, monkeypatch, layers, hcs, defer, aggr, deg_norm):
    """The stack's top layer on the dW + dX adjoint (ops._TOP_FULL, the
    default), its bias gradient from a column-sum pass or (hcs) from the same
    launch (ops._TOP_HCS), against the Z form (Z kept,
    dX-only adjoint + dense Z^T dY pass): y and x.grad bit for bit, every
    dW / db within tolerance."""
    from mgcn import ops
    from mgcn.models import GCNLayer, GCNStack
    torch.manual_seed(5)
    rng = np.random.default_rng(31)
    N = 8000
    ei = _t(_graph(rng, N, 80000), cuda)
    stack = GCNStack([GCNLayer(F, F, deg_norm=deg_norm, aggr=aggr, bias=True,
                               non_linear="relu" if i < layers - 1 else "none").to(cuda)
                      for i in range(layers)])
    x = torch.randn(N, F, device=cuda, requires_grad=True)
    dZ = torch.randn(N, F, device=cuda)
    res = []
    monkeypatch.setattr(ops, "_TOP_HCS", hcs)
    monkeypatch.setattr(ops, "_TOP_CS_DEFER", defer)
    for top_full in (True, False):
        monkeypatch.setattr(ops, "_TOP_FULL", top_full)
        x.grad = None
        for p in stack.parameters():
            p.grad = None
        y = stack(x, ei)
        y.backward(dZ)
        res.append((y.detach(), x.grad.clone(), [p.grad.clone() for p in stack.parameters()]))
    (ya, xa, ga), (yb, xb, gb) = res
    assert torch.equal(ya, yb) and torch.equal(xa, xb)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("N,E,hub", [(20000, 200000, 0), (3000, 20000, 700), (33, 100, 0)])
def test_gather_unroll_forms_bitwise(cuda, N, E, hub):
    """The gathers in flight per row (forward spmm_xw_unroll 4 / 5 / 6, DWS
    xw_ws_full_unroll 4 / 5 / 6) change only the load schedule: every row is
    still folded in edge order, so Y, Z, the masks, dX, dW and the column
    sums are bit for bit the same."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(N + 41)
    ei = _graph(rng, N, E, hub)
    plan, norm = _plan(cuda, ei, N, "sm")
    g = torch.Generator(device=cuda).manual_seed(N + 43)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    b = torch.randn(F, device=cuda, generator=g) * 0.1
    dY = torch.randn(N, F, device=cuda, generator=g)
    rm = ops.make_relu_mask(torch.randn(N, F, device=cuda, generator=g))
    fwd, bwd = {}, {}
    try:
        for u in (4, 5, 6):
            L.set_option("spmm_xw_unroll", u)
            rmo = torch.empty_like(rm)
            y, z = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, b, True,
                                   relu_mask=rmo, want_z=True)
            fwd[u] = (y, z, rmo)
            L.set_option("xw_ws_full_unroll", u)
            bwd[u] = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, relu_mask=rm)
    finally:  # the defaults
        L.set_option("spmm_xw_unroll", 5)
        L.set_option("xw_ws_full_unroll", 5)
    for u in (5, 6):
        for a, c in zip(fwd[u], fwd[4]):
            assert torch.equal(a, c)
        for a, c in zip(bwd[u], bwd[4]):
            assert torch.equal(a, c)


@pytest.mark.parametrize("M", [1, 31, 33, 4097, 300000])
@pytest.mark.parametrize("hcs", [False, True])
def test_dw_pass_with_third_stream_colsum(cuda, M, hcs):
    """mgcn_gemm_bwd_dw_cs: dW (and dH's column sums) bit for bit mgcn_gemm_bwd's
    dW-only pass (the same kernel, chunk map and fold), plus the column sums of
    a third matrix S streamed in the same pass, within fp32 summation
    tolerance of the fp64 sums; an empty M zeroes every output."""
    from mgcn import _lib as L
    from mgcn import ops
    lib = L.load()
    g = torch.Generator(device=cuda).manual_seed(M + 3)
    Z = torch.randn(M, F, device=cuda, generator=g)
    dY = torch.randn(M, F, device=cuda, generator=g)
    S = torch.randn(M, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g)
    ref_dw, _, ref_cs = ops.gemm_bwd(Z, dY, W, want_dx=False, dh_colsum=hcs)
    dW = torch.empty(F, F, device=cuda)
    cs = torch.empty(F, device=cuda) if hcs else None
    scs = torch.empty(F, device=cuda)
    wsb = int(lib.mgcn_gemm_bwd_dw_cs_workspace_bytes(M))
    ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    with L.device_guard(cuda):
        rc = lib.mgcn_gemm_bwd_dw_cs(M, L.ptr(Z), F, L.ptr(dY), F, L.ptr(dW), F, 0, L.ptr(cs),
                                     L.ptr(S), F, L.ptr(scs), L.ptr(ws), wsb, L.stream_of(cuda))
    L.check(rc, "mgcn_gemm_bwd_dw_cs")
    assert torch.equal(dW, ref_dw)
    if hcs:
        assert torch.equal(cs, ref_cs)
    bound = S.double().abs().sum(0)
    assert ((scs.double() - S.double().sum(0)).abs() <= 1e-5 * bound + 1e-6).all()
    dW2, scs2 = ops.dw_pass_cs(Z, dY, S)
    assert torch.equal(dW2, dW) and torch.equal(scs2, scs)
    z = torch.full((F,), float("nan"), device=cuda)
    with L.device_guard(cuda):
        rc = lib.mgcn_gemm_bwd_dw_cs(0, L.ptr(Z), F, L.ptr(dY), F, L.ptr(dW), F, 0, None,
                                     L.ptr(S), F, L.ptr(z), L.ptr(ws), wsb, L.stream_of(cuda))
    L.check(rc, "mgcn_gemm_bwd_dw_cs")
    assert (z == 0).all() and (dW == 0).all()
