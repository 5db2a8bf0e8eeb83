"""Property-based parity (hypothesis): random ragged graphs -- empty rows,
isolated nodes, self-loops, multi-edges, hub rows past the heavy-row
thresholds, odd feature widths, exact-tie values for max -- through the
libmgcn aggregation, forward and adjoint bit for bit against the oracle
(the reference's scatter_add / scatter_mean / scatter_max arithmetic)."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu


@st.composite
def graphs(draw):
    N = draw(st.integers(1, 400))
    E = draw(st.integers(0, 3000))
    seed = draw(st.integers(0, 2**31 - 1))
    rng = np.random.default_rng(seed)
    s = rng.integers(0, N, E)
    d = rng.integers(0, N, E)
    if draw(st.booleans()) and E:  # a hub destination / source past the heavy thresholds
        k = draw(st.sampled_from([129, 300, 600, 1500]))
        d = np.concatenate([d, np.full(k, rng.integers(0, N))])
        s = np.concatenate([s, rng.integers(0, N, k)])
    if draw(st.booleans()) and s.size:  # duplicates (multi-edges)
        pick = rng.integers(0, s.size, max(1, s.size // 10))
        s, d = np.concatenate([s, s[pick]]), np.concatenate([d, d[pick]])
    if draw(st.booleans()):  # self-loops for every node, appended (loop.py order)
        s, d = np.concatenate([s, np.arange(N)]), np.concatenate([d, np.arange(N)])
    F = draw(st.sampled_from([1, 3, 4, 8, 31, 32, 64, 100, 128, 130]))
    ties = draw(st.booleans())
    return np.stack([s, d]).astype(np.int64), N, F, seed, ties


@settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
@given(g=graphs(), deg_norm=st.sampled_from([None, "sm", "rw"]),
       aggr=st.sampled_from(["add", "mean", "max"]), relu=st.booleans(), bias=st.booleans())
def test_aggregate_property_bitwise(cuda, oracle, g, deg_norm, aggr, relu, bias):
    import mgcn
    ei, N, F, seed, ties = g
    rng = np.random.default_rng(seed + 1)
    H = rng.standard_normal((N, F)).astype(np.float32)
    if ties:  # exact ties decide max's winner (torch_scatter 1.x: the later edge)
        H = np.round(H * 2).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32) if bias else None
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    wf, wb, rs = oracle.edge_factors(ei, N, deg_norm)
    y_ref, am = oracle.aggr_fwd(ei, H, wf, aggr, b, relu)
    dH_ref, _ = oracle.aggr_bwd(ei, dZ, wb, rs, aggr, y_ref, relu, am)
    Ht = torch.from_numpy(H).to(cuda).requires_grad_(True)
    bt = torch.from_numpy(b).to(cuda) if bias else None
    y = mgcn.aggregate(Ht, torch.from_numpy(ei).to(cuda), aggr=aggr, deg_norm=deg_norm, bias=bt,
                       relu=relu)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), y_ref)
    y.backward(torch.from_numpy(dZ).to(cuda))
    np.testing.assert_array_equal(Ht.grad.cpu().numpy(), dH_ref)
