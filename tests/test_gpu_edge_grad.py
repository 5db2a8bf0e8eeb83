"""GPU parity of the edge-weight / degree gradients (degnorm_const is
differentiable in edge_weight and deg, gcn_base_models.py:102-140):
libmgcn mgcn_edge_weight_grad (the SDDMM adjoint of the per-slot weights)
behind graph._grad_norm's differentiable weights and ops._AggregateW.

Bars: the forward output and dx stay BIT FOR BIT the reference's (the same
kernels run; with W = I every product is exact); the weight gradients sum
F products per edge in a different order than the reference's CPU sum, so
they compare within fp32 tolerance (rtol 1e-4 of the per-edge magnitude
sum_f |dY||H|, checked explicitly at the kernel level); NaN where the
reference's own autograd gives NaN (its 0 * inf at zero degrees).
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


@pytest.mark.parametrize("name", golden_names("ewgrad_") + golden_names("degrad_"))
def test_node_model_weight_gradients_match_reference(cuda, name):
    from mgcn.models import NodeModelAdditive
    z = load_golden(name)
    deg_norm, aggr, given, identity = (str(v) for v in z["meta"])
    F = z["x"].shape[1]
    m = NodeModelAdditive(F, F, deg_norm=deg_norm, aggr=aggr, bias=True).to(cuda)
    with torch.no_grad():
        m.weight_node.copy_(_t(z["W"], cuda))
        m.bias.copy_(_t(z["b"], cuda))
    x = _t(z["x"], cuda).requires_grad_(True)
    ew = _t(z["edge_weight"], cuda).requires_grad_(True) if given == "ew" else None
    deg = _t(z["deg"], cuda).requires_grad_(True) if given == "deg" else None
    y = m(x, _t(z["edge_index"], cuda), deg=deg, edge_weight=ew)
    if identity == "1":
        np.testing.assert_array_equal(_np(y), z["y"])
    else:
        np.testing.assert_allclose(_np(y), z["y"], rtol=1e-5, atol=1e-5)
    y.backward(_t(z["dZ"], cuda))
    if identity == "1":
        np.testing.assert_array_equal(_np(x.grad), z["dx"])
    else:
        np.testing.assert_allclose(_np(x.grad), z["dx"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(m.bias.grad), z["db"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(_np(m.weight_node.grad), z["dW"], rtol=1e-4, atol=1e-3)
    got, want = (_np(ew.grad), z["dew"]) if given == "ew" else (_np(deg.grad), z["ddeg"])
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    np.testing.assert_allclose(got[ok], want[ok], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("F", [1, 7, 64, 128, 300])
@pytest.mark.parametrize("aggr", ["add", "max"])
def test_edge_weight_grad_kernel_vs_fp64(cuda, F, aggr):
    """mgcn_edge_weight_grad against an fp64 dot product per slot (max: over
    the features the slot won, from the forward's winner bits), on a ragged
    graph with empty rows, a hub row and multi-edges."""
    import mgcn  # noqa: F401
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import plan_for
    g = torch.Generator().manual_seed(F)
    N, E = 700, 6000
    src = torch.randint(0, N, (E,), generator=g)
    dst = torch.randint(0, N - 50, (E,), generator=g)  # rows N-50.. stay empty
    dst[:600] = 3  # a hub row past the heavy thresholds
    ei = torch.stack([src, dst]).to(cuda)
    plan = plan_for(ei, N)
    H = torch.randn(N, F, generator=g).to(cuda)
    dY = torch.randn(N, F, generator=g).to(cuda)
    win = None
    if aggr == "max":
        norm = plan.norm(None)
        _, win = ops.spmm_fwd(plan.fwd, norm.w_fwd, H, L.REDUCE_MAX, None, False, mask_plan=plan)
    dw = _np(ops.edge_weight_grad(plan.fwd, H, dY, win_mask=win)).astype(np.float64)
    col = plan.fwd.col.long().cpu().numpy()
    rp = plan.fwd.rowptr.cpu().numpy()
    rows = np.repeat(np.arange(N), np.diff(rp))
    Hn, dYn = H.cpu().numpy().astype(np.float64), dY.cpu().numpy().astype(np.float64)
    prod = dYn[rows] * Hn[col]
    if win is not None:
        words = win.cpu().numpy().view(np.uint32).reshape(len(col), -1)
        f = np.arange(F)
        mask = (words[:, f >> 5] >> (f & 31)) & 1
        prod = prod * mask
    want = prod.sum(1)
    scale = np.abs(prod).sum(1) + 1e-30
    assert np.all(np.abs(dw - want) <= 1e-5 * scale), np.max(np.abs(dw - want) / scale)


def test_gcn_layer_edge_weight_grad_vs_oracle_f128(cuda):
    """A 128-wide GCN layer on a 20k-node graph, edge_weight requiring grad:
    y, dx, dW, db and d(edge_weight) against the reference's op sequence in
    torch CPU ops (oracle.torch_layer_reference, pinned to the ewgrad
    fixtures in tests/test_oracle.py)."""
    from oracle import oracle as orc
    from mgcn.models import NodeModelAdditive
    g = torch.Generator().manual_seed(3)
    N, E, F = 20000, 200000, 128
    ei = torch.randint(0, N, (2, E), generator=g)
    ei = torch.cat([ei, torch.arange(N).repeat(2, 1)], 1)
    ew = torch.rand(ei.size(1), generator=g) + 0.1
    x = torch.randn(N, F, generator=g)
    dZ = torch.randn(N, F, generator=g)
    m = NodeModelAdditive(F, F, deg_norm='sm', aggr='add', bias=True).to(cuda)
    with torch.no_grad():
        m.bias.uniform_(-0.1, 0.1)
    W, b = m.weight_node.detach().cpu(), m.bias.detach().cpu()
    xc = x.clone().requires_grad_(True)
    ewc = ew.clone().requires_grad_(True)
    Wc = W.clone().requires_grad_(True)
    yc = orc.torch_layer_reference(xc, ei, Wc, b, deg_norm="sm", edge_weight=ewc)
    yc.backward(dZ)
    xg = x.to(cuda).requires_grad_(True)
    ewg = ew.to(cuda).requires_grad_(True)
    y = m(xg, ei.to(cuda), edge_weight=ewg)
    y.backward(dZ.to(cuda))
    np.testing.assert_allclose(_np(y), yc.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(_np(xg.grad), xc.grad.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(m.weight_node.grad), Wc.grad.numpy(), rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(_np(ewg.grad), ewc.grad.numpy(), rtol=1e-3, atol=1e-4)


def test_degnorm_const_differentiable(cuda):
    """NodeModelBase.degnorm_const returns the reference's weights (bitwise,
    as the degnorm_* fixtures pin them) with their autograd history."""
    from mgcn.models import NodeModelBase
    z = load_golden("degnorm_sm_computed_ew1")
    ei = _t(z["edge_index"], cuda)
    ew = _t(z["edge_weight"], cuda).requires_grad_(True)
    norm = NodeModelBase.degnorm_const(ei, 300, None, ew, 'sm')
    np.testing.assert_array_equal(_np(norm), z["norm"])
    g = torch.randn(norm.numel(), device=cuda)
    (norm * g).sum().backward()
    ewc = torch.from_numpy(z["edge_weight"]).requires_grad_(True)
    src, dst = torch.from_numpy(z["edge_index"])
    deg = torch.zeros(300).scatter_add(0, src, ewc)
    a = deg.pow(-0.5)
    a = a.masked_fill(a == float("inf"), 0)
    ((a[src] * ewc * a[dst]) * g.cpu()).sum().backward()
    np.testing.assert_allclose(_np(ew.grad), ewc.grad.numpy(), rtol=1e-5, atol=1e-6)


def test_stacks_with_edge_weight_grad_run_layer_by_layer(cuda):
    """GCNStack and GCNConv with edge weights requiring grad take the
    differentiable path (no fused kernel drops the weights' gradient): the
    stack's edge_weight.grad equals the sum of its layers' run one by one."""
    from mgcn.models import GCNLayer, GCNStack
    from mgcn.pyg import GCNConv
    g = torch.Generator().manual_seed(11)
    N, E, F = 3000, 30000, 128
    ei = torch.randint(0, N, (2, E), generator=g).to(cuda)
    ew = (torch.rand(E, generator=g) + 0.1).to(cuda)
    x = torch.randn(N, F, generator=g).to(cuda)
    torch.manual_seed(0)
    layers = [GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                       non_linear='relu' if i < 2 else 'none').to(cuda) for i in range(3)]
    stack = GCNStack(layers)
    e1 = ew.clone().requires_grad_(True)
    stack(x, ei, edge_weight=e1).sum().backward()
    e2 = ew.clone().requires_grad_(True)
    h = x
    for layer in layers:
        h = layer(h, ei, None, None, e2)
    h.sum().backward()
    # the stack shares one weight graph (its three layers' slot gradients are
    # summed before the chain to edge_weight), the layers build one each: the
    # same sums in a different order
    torch.testing.assert_close(e1.grad, e2.grad, rtol=1e-4, atol=1e-5 * e2.grad.abs().max().item())
    conv = GCNConv(F, F).to(cuda)
    e3 = ew.clone().requires_grad_(True)
    conv(x, ei, e3).sum().backward()
    assert e3.grad is not None and torch.isfinite(e3.grad).all() and e3.grad.abs().sum() > 0


def test_unnormalised_layer_ignores_deg_requiring_grad(cuda, oracle):
    """deg_norm=None never reads deg (gcn_base_models.py:209-211): a deg that
    requires grad is ignored (no gradient, no error) and the layer is the
    plain sum bit for bit (W = I)."""
    from mgcn.models import NodeModelAdditive
    rng = np.random.default_rng(5)
    N, F = 300, 16
    s, d = rng.integers(0, N, 2000), rng.integers(0, N, 2000)
    ei = np.stack([np.concatenate([s, np.arange(N)]), np.concatenate([d, np.arange(N)])])
    x = rng.standard_normal((N, F)).astype(np.float32)
    m = NodeModelAdditive(F, F, deg_norm=None, aggr='add', bias=False).to(cuda)
    with torch.no_grad():
        m.weight_node.copy_(torch.eye(F))
    deg = torch.rand(N, device=cuda).add_(1.0).requires_grad_(True)
    y = m(_t(x, cuda), _t(ei, cuda), deg=deg)
    y.sum().backward()
    assert deg.grad is None
    ref, _ = oracle.aggr_fwd(ei, x, None, "add")
    np.testing.assert_array_equal(_np(y), ref)
