"""The headline workload itself, checked at its own size: BASELINE config 2
(N = 1M, E = 10M + 1M self-loops, F = 128, three GCN layers 'sm' / 'add' +
bias, ReLU between), built by bench.make_stack exactly as bench.py times it,
so the kernels checked here are the timed ones: the Z-writing fused forward
(mgcn_spmm_xw_fwd), the middle layer's dW + dX gather kernel, the dX-only
gather (mgcn_spmm_xw_bwd, X = NULL), the dW-only dense pass (mgcn_gemm_bwd)
and the bottom layer without any gather.  Reference: the reference's
NodeModelAdditive forward and autograd adjoints, gcn_base_models.py:199-243.

(a) W = I: every bf16x6 product is exact, so the output and x.grad must equal
    the C oracle's layer-by-layer chain BIT FOR BIT.
(b) bench.py's seeded random W (glorot) and b: per layer, the stack's output
    against the fp64 A (X_l W_l) + b_l at the stack's own input X_l, within
    1e-5 * (|A| |X_l| |W_l| + |b_l|) + 1e-6; all dW, all db and dx on 4096
    sampled rows against the fp64 adjoints at the stack's activations, within
    1e-5 of the |.|-weighted chain (the same products with |A|, |W|, |dY|).
The fp64 references run on the GPU in torch (index_add_ over edge chunks),
the per-edge weights are the oracle's.
"""
import numpy as np
import pytest
import torch
from fp64_ref import A64 as _A64

pytestmark = pytest.mark.gpu

N_SAMPLE = 4096


@pytest.fixture(scope="module")
def config2(cuda):
    from bench import make_er_graph, make_inputs
    ei, N = make_er_graph(1_000_000, 5_000_000)
    X, Ws, bs, dY = make_inputs(N, 128, 3)
    return ei, N, X, Ws, bs, dY


def _np(t):
    return t.detach().cpu().numpy()


def test_config2_stack_identity_weights_bitwise(cuda, oracle, config2):
    """(a) W = I through the bench's stack (x.requires_grad, so the bottom
    layer's dX-only gather runs too): y and x.grad bit for bit the oracle's
    chain -- forward relu(A h + b) twice then A h + b, adjoint A^T with the
    ReLU masks of the stack's own outputs."""
    from bench import make_stack
    ei, N, X, _, bs, dY = config2
    F = X.shape[1]
    eye = torch.eye(F)
    stack = make_stack(cuda, [eye] * 3, bs)
    x = X.to(cuda).requires_grad_(True)
    y = stack(x, ei.to(cuda))
    y.backward(dY.to(cuda))
    ein = ei.numpy()
    wf, wb, rs = oracle.edge_factors(ein, N, "sm")
    h, outs = X.numpy(), []
    for l in range(3):
        h, _ = oracle.aggr_fwd(ein, h, wf, "add", bs[l].numpy(), relu=l < 2)
        outs.append(h)
    np.testing.assert_array_equal(_np(y), outs[-1])
    g = dY.numpy()
    for l in range(2, -1, -1):
        g, _ = oracle.aggr_bwd(ein, g, wb, rs, "add", outs[l], l < 2, None)
    np.testing.assert_array_equal(_np(x.grad), g)


def test_config2_stack_random_weights_vs_fp64(cuda, oracle, config2):
    """(b) bench.py's weights: forward per layer, every dW / db, and dx on
    sampled rows within the |.|-weighted 1e-5 bound of fp64."""
    from bench import make_stack
    from mgcn.models import GCNStack
    ei, N, X, Ws, bs, dY = config2
    eic = ei.to(cuda)
    Xd, dYd = X.to(cuda), dY.to(cuda)
    stack = make_stack(cuda, Ws, bs)
    params = list(stack.parameters())
    # exactly the bench step: x without grad (the bottom layer runs no gather)
    y = stack(Xd, eic)
    y.backward(dYd)
    gW = [p.grad.clone() for p in params[0::2]]
    gb = [p.grad.clone() for p in params[1::2]]
    # the stack's intermediate activations: the forward of its first l
    # layers (the same kernels, bit for bit)
    with torch.no_grad():
        acts = [Xd, GCNStack(stack.layers[:1])(Xd, eic), GCNStack(stack.layers[:2])(Xd, eic)]
        assert torch.equal(GCNStack(stack.layers)(Xd, eic), y.detach())
    # dx: the same stack with x requiring grad (bottom layer: dX-only gather)
    for p in params:
        p.grad = None
    xg = Xd.clone().requires_grad_(True)
    stack(xg, eic).backward(dYd)
    gx = xg.grad

    wf, _, _ = oracle.edge_factors(ei.numpy(), N, "sm")
    A = _A64(ei, wf, N, cuda)
    W64 = [w.to(cuda, torch.float64) for w in Ws]
    b64 = [b.to(cuda, torch.float64) for b in bs]
    outs = acts[1:] + [y.detach()]
    for l in range(3):
        xin = acts[l].double()
        ref = A.apply(xin @ W64[l]) + b64[l]
        if l < 2:
            ref = ref.clamp_min(0)
        bound = A.apply(xin.abs() @ W64[l].abs(), absolute=True) + b64[l].abs()
        err = (outs[l].double() - ref).abs()
        assert bool((err <= 1e-5 * bound + 1e-6).all()), (l, float((err / bound).max()))
    g = dY.to(cuda, torch.float64)
    gm = g.abs()
    rows = torch.from_numpy(np.random.default_rng(0).choice(N, N_SAMPLE, replace=False)).to(cuda)
    for l in range(2, -1, -1):
        dH = A.apply(g, transpose=True)
        dHm = A.apply(gm, transpose=True, absolute=True)
        xin = acts[l].double()
        dW_ref = xin.t() @ dH
        dW_bound = xin.abs().t() @ dHm
        err = (gW[l].double() - dW_ref).abs()
        assert bool((err <= 1e-5 * dW_bound + 1e-6).all()), (l, float((err / dW_bound).max()))
        db_ref = g.sum(0)
        err = (gb[l].double() - db_ref).abs()
        assert bool((err <= 1e-5 * gm.sum(0) + 1e-6).all()), (l, float(err.max()))
        dX = dH @ W64[l].t()
        dXm = dHm @ W64[l].abs().t()
        if l == 0:
            err = (gx[rows].double() - dX[rows]).abs()
            assert bool((err <= 1e-5 * dXm[rows] + 1e-6).all()), float((err / dXm[rows]).max())
        else:
            mask = (acts[l] > 0).double()  # the stack's own ReLU masks
            g, gm = dX * mask, dXm * mask
