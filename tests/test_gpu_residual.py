"""The fused residual-layer kernels (libmgcn mgcn_residual_layer_fwd / _bwd,
residual.hip): one GCNModel layer with its residual Linear at F = 32 (the
botnet stack of config 3, gcn_model.py:89-105 with residual_hop = 1), on
skewed graphs whose rows take every path (light rows in the fused kernel,
heavy and giant rows through the SpMM's workgroup kernels then the fused
epilogue).

Bars:
  * W = I, Wr = 0, no biases: every product is exact, so Z = relu(A x) equals
    the oracle's aggregation BIT FOR BIT, and the masks are its ReLU bits;
  * backward with W = I, Wr = 0: dX = dH = A^T (relu' dZ) bit for bit the
    oracle adjoint; with W = 0, Wr = I: dX = dS = relu2' dZ exactly;
  * random weights: forward, dx and all four parameter gradients against the
    two-launch layer (ops._ResidualGCNLayer: x @ [W | Wr^T], SpMM, join) within
    fp32 tolerance (the fused layer associates (A x) W).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _skewed(rng, N, E, hubs=((0, 2000), (1, 300), (2, 700))):
    """Random graph + hub nodes (in- and out-edges) + self-loops: heavy rows
    above 128 edges, giant ones above 512, in both views."""
    s, d = [rng.integers(0, N, E)], [rng.integers(0, N, E)]
    for h, k in hubs:
        s += [rng.integers(0, N, k), np.full(k, h)]
        d += [np.full(k, h), rng.integers(0, N, k)]
    s.append(np.arange(N))
    d.append(np.arange(N))
    return np.stack([np.concatenate(s), np.concatenate(d)]).astype(np.int64)


def _plan(cuda, ei, N, deg_norm):
    from mgcn.graph import plan_for
    plan = plan_for(_t(ei, cuda), N)
    return plan, plan.norm(deg_norm)


@pytest.mark.parametrize("deg_norm,aggr", [("sm", "add"), ("rw", "mean"), (None, "add")])
@pytest.mark.parametrize("relu1,relu2", [(True, True), (True, False), (False, True)])
def test_residual_layer_identity_bitwise(cuda, oracle, deg_norm, aggr, relu1, relu2):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(7 + relu1 + 2 * relu2 + len(aggr))
    N, F = 6000, 32
    ei = _skewed(rng, N, 40000)
    plan, norm = _plan(cuda, ei, N, deg_norm)
    assert plan.fwd.n_heavy > 0 and plan.fwd.n_giant > 0 and plan.bwd.n_giant > 0
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    reduce = L.REDUCE_CODES[aggr]
    xt = _t(x, cuda).requires_grad_(True)
    eye, zero = torch.eye(F, device=cuda), torch.zeros(F, F, device=cuda)
    Wt, Wrt = eye.clone().requires_grad_(True), zero.clone().requires_grad_(True)
    assert ops.residual_layer_supported(plan, xt, Wt, Wrt, reduce)
    Z = ops._ResidualLayerFused.apply(xt, plan, norm, reduce, relu1, relu2, Wt, None, Wrt, None)
    wf, wb, rs = oracle.edge_factors(ei, N, deg_norm)
    agg, _ = oracle.aggr_fwd(ei, x, wf, aggr, None, relu1)
    ref = np.maximum(agg, 0) if relu2 else agg
    np.testing.assert_array_equal(Z.detach().cpu().numpy(), ref)
    Z.backward(_t(dZ, cuda))
    # Wr = 0: dX = dH = A^T (relu1' relu2' dZ) [/ count], the oracle adjoint
    g = np.where(ref > 0, dZ, 0) if relu2 else dZ
    dH, _ = oracle.aggr_bwd(ei, g, wb, rs, aggr, agg, relu1, None)
    np.testing.assert_array_equal(xt.grad.cpu().numpy(), dH)
    # W = 0, Wr = I: dX = dS exactly
    xt.grad = None
    Z = ops._ResidualLayerFused.apply(xt, plan, norm, reduce, relu1, relu2, zero, None, eye, None)
    Z.backward(_t(dZ, cuda))
    z = x.copy()
    zz = np.maximum(np.maximum(0, 0) + z, 0) if relu2 else z  # relu1(0) + x
    np.testing.assert_array_equal(Z.detach().cpu().numpy(), zz)
    np.testing.assert_array_equal(xt.grad.cpu().numpy(), np.where(zz > 0, dZ, 0) if relu2 else dZ)


@pytest.mark.parametrize("deg_norm,aggr,bias", [("sm", "add", False), ("sm", "add", True),
                                                ("rw", "mean", True), (None, "mean", False)])
@pytest.mark.parametrize("relu2", [True, False])
def test_residual_layer_vs_two_launch(cuda, deg_norm, aggr, bias, relu2):
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(11 + bias + 2 * relu2)
    N, F = 8000, 32
    ei = _skewed(rng, N, 60000)
    plan, norm = _plan(cuda, ei, N, deg_norm)
    reduce = L.REDUCE_CODES[aggr]
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(N, F, device=cuda, generator=g)
    dZ = torch.randn(N, F, device=cuda, generator=g)
    params = [torch.randn(F, F, device=cuda, generator=g) * 0.2,
              torch.randn(F, device=cuda, generator=g) * 0.1 if bias else None,
              torch.randn(F, F, device=cuda, generator=g) * 0.2,
              torch.randn(F, device=cuda, generator=g) * 0.1]
    outs = []
    for fn in (ops._ResidualLayerFused, ops._ResidualGCNLayer):
        xi = x.clone().requires_grad_(True)
        ps = [None if p is None else p.clone().requires_grad_(True) for p in params]
        Z = fn.apply(xi, plan, norm, reduce, True, relu2, *ps)
        Z.backward(dZ)
        outs.append([Z.detach(), xi.grad] + [None if p is None else p.grad for p in ps])
    for a, b in zip(*outs):
        if b is None:
            assert a is None
            continue
        scale = float(b.abs().max())
        torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-5 * max(1.0, scale))


def test_residual_layer_deterministic_and_first_layer_fallback(cuda):
    """Repeated runs are bitwise identical (fixed summation orders, no
    atomics); a 1 -> 32 first layer (F_in != 32) keeps the two-launch path."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(3)
    N, F = 5000, 32
    plan, norm = _plan(cuda, _skewed(rng, N, 30000), N, "sm")
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(N, F, device=cuda, generator=g)
    W, Wr = torch.randn(F, F, device=cuda, generator=g), torch.randn(F, F, device=cuda, generator=g)
    b = torch.randn(F, device=cuda, generator=g)
    dZ = torch.randn(N, F, device=cuda, generator=g)
    res = []
    for _ in range(2):
        xi = x.clone().requires_grad_(True)
        ps = [p.clone().requires_grad_(True) for p in (W, b, Wr, b)]
        Z = ops._ResidualLayerFused.apply(xi, plan, norm, L.REDUCE_SUM, True, True, *ps)
        Z.backward(dZ)
        res.append([Z.detach(), xi.grad] + [p.grad for p in ps])
    for a, c in zip(*res):
        assert torch.equal(a, c)
    x1 = torch.randn(N, 1, device=cuda)
    assert not ops.residual_layer_supported(plan, x1, torch.randn(1, F, device=cuda),
                                            torch.randn(F, 1, device=cuda), L.REDUCE_SUM)


@pytest.mark.parametrize("aggr,deg_norm,bias", [("add", "sm", False), ("mean", "rw", True)])
def test_residual_stack_matches_layer_by_layer(cuda, aggr, deg_norm, bias):
    """mgcn_residual_stack_fwd / _bwd (one host call per direction for a run
    of 32 -> 32 layers) against the same layers as separate fused nodes:
    outputs, dx and the weight gradients bit for bit (same kernels, same
    order), on a skewed graph.  The bias gradients of the layers below the
    top come from the mask pass fused into the layer above's dX store in the
    stack (the same dS / dA values, column-summed per block of that kernel
    instead of the mask kernel's rows): equal to fp32 rounding."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(17 + bias)
    N, F, nl = 5000, 32, 4
    plan, norm = _plan(cuda, _skewed(rng, N, 30000), N, deg_norm)
    reduce = L.REDUCE_CODES[aggr]
    g = torch.Generator(device=cuda).manual_seed(9)
    x = torch.randn(N, F, device=cuda, generator=g)
    dZ = torch.randn(N, F, device=cuda, generator=g)
    params = [(torch.randn(F, F, device=cuda, generator=g) * 0.3,
               torch.randn(F, device=cuda, generator=g) * 0.1 if bias else None,
               torch.randn(F, F, device=cuda, generator=g) * 0.3,
               torch.randn(F, device=cuda, generator=g) * 0.1) for _ in range(nl)]
    relu1s = [True] * nl
    relu2s = [True] * (nl - 1) + [False]
    outs = []
    for stacked in (True, False):
        xi = x.clone().requires_grad_(True)
        ps = [tuple(None if p is None else p.clone().requires_grad_(True) for p in q)
              for q in params]
        if stacked:
            y = ops.residual_stack(xi, plan, norm, aggr, relu1s, relu2s, ps)
        else:
            y = xi
            for q, r1, r2 in zip(ps, relu1s, relu2s):
                y = ops._ResidualLayerFused.apply(y, plan, norm, reduce, r1, r2, *q)
        y.backward(dZ)
        outs.append([y.detach(), xi.grad] + [p.grad for q in ps for p in q if p is not None])
    for a, b in zip(*outs):
        if a.dim() == 1:  # a bias gradient
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * max(1.0, b.abs().max().item()))
        else:
            assert torch.equal(a, b)



@pytest.mark.parametrize("deg_norm,aggr,bias", [("sm", "add", False), ("sm", "add", True),
                                                ("rw", "mean", True)])
@pytest.mark.parametrize("relu1,relu2", [(True, True), (True, False)])
@pytest.mark.parametrize("need_x", [False, True])
def test_input_layer_vs_two_launch_and_fp64(cuda, deg_norm, aggr, bias, relu1, relu2, need_x):
    """The in_channels = 1 input layer as (A x) W (ops._InputLayer: a 1-wide
    SpMM + mgcn_input_layer_fwd / _bwd) against the two-launch layer
    (_ResidualGCNLayer: x @ [W | Wr^T], 32-wide SpMM, join -- the reference's
    A (x W)) on a skewed graph with heavy and giant rows: Z, the four
    parameter gradients and dx within fp32 tolerance, and Z within 1e-5 of an
    fp64 restatement relative to its |.| bound."""
    from fp64_ref import A64, within
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(41 + bias + 2 * relu2 + 4 * need_x)
    N, F = 7000, 32
    ei = _skewed(rng, N, 50000)
    plan, norm = _plan(cuda, ei, N, deg_norm)
    assert plan.fwd.n_giant > 0
    reduce = L.REDUCE_CODES[aggr]
    g = torch.Generator(device=cuda).manual_seed(13)
    x = torch.randn(N, 1, device=cuda, generator=g)
    dZ = torch.randn(N, F, device=cuda, generator=g)
    params = [torch.randn(1, F, device=cuda, generator=g),
              torch.randn(F, device=cuda, generator=g) * 0.3 if bias else None,
              torch.randn(F, 1, device=cuda, generator=g),
              torch.randn(F, device=cuda, generator=g) * 0.3]
    assert ops.input_layer_supported(plan, x, params[0], params[2], reduce)
    outs = []
    for fn in (ops._InputLayer, ops._ResidualGCNLayer):
        xi = x.clone().requires_grad_(need_x)
        ps = [None if p is None else p.clone().requires_grad_(True) for p in params]
        Z = fn.apply(xi, plan, norm, reduce, relu1, relu2, *ps)
        Z.backward(dZ)
        outs.append([Z.detach(), xi.grad] + [None if p is None else p.grad for p in ps])
    for a, b in zip(*outs):
        if b is None:
            assert a is None
            continue
        scale = float(b.abs().max())
        torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-5 * max(1.0, scale))
    # Z against fp64 (the relu decisions from the fp32 result where it is not
    # within rounding of zero)
    from oracle import oracle as orc
    wf, _, _ = orc.edge_factors(ei, N, deg_norm)
    A = A64(torch.from_numpy(ei), wf, N, cuda, mean=aggr == "mean")
    a64 = A.apply(x.double())
    am = A.apply(x.double().abs(), absolute=True)
    W64, Wr64 = params[0].double(), params[2].double()
    b64 = params[1].double() if bias else torch.zeros(F, dtype=torch.float64, device=cuda)
    br64 = params[3].double()
    z1 = a64 @ W64 + b64
    if relu1:
        z1 = z1.clamp_min(0)
    z = z1 + x.double() @ Wr64.t() + br64
    if relu2:
        z = z.clamp_min(0)
    bound = am @ W64.abs() + b64.abs() + x.double().abs() @ Wr64.abs().t() + br64.abs()
    ok, worst = within(outs[0][0].double() - z, bound, 1e-5)
    assert ok, worst
