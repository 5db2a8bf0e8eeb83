"""Device-side failure reporting of the warp-specialised kernels (round 6,
ABI 21: mgcn_check_device / MGCN_EDEVICE).

The 128-wide adjoint (fused.hip, spmm_xw_bwd_ws_kernel) and the 256-wide layer
kernels (fused_wide.hip, spmm_xw_wide_ws_kernel) hand chunks between their
gather and MFMA waves through LDS counters with bounded spins.  A spin past
its bound makes every wave leave, and the kernel's outputs are then
incomplete: the kernel must say so.  The experiment build (libmgcn_exp.so,
`make -C meta-gcn_amd/csrc exp`, built by __graft_entry__.build()) lets the
bound be set to 1 poll ("ws_spin_limit"), which forces the abort path on any
non-trivial graph; these tests check that the failure surfaces

  * through mgcn_check_device(stream, sync=1) (mgcn.check_device), and
  * through the next mgcn_spmm_xw_* call without an explicit check,

and that the same experiment build at the default bound computes exactly the
product library's results.  No reference counterpart (SURVEY.md §8(b)
conventions: 0 / MGCN_E* return codes + mgcn_last_error).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP_LIB = os.path.join(ROOT, "meta-gcn_amd", "mgcn", "libmgcn_exp.so")


def _graph(rng, N, E):
    s = rng.integers(0, N, E)
    d = rng.integers(0, N, E)
    s = np.concatenate([s, d, np.arange(N)])
    d2 = np.concatenate([d, s[:E], np.arange(N)])
    return torch.from_numpy(np.stack([s, d2]).astype(np.int64))


@pytest.fixture
def exp_lib(cuda):
    """libmgcn_exp.so swapped in as mgcn's library for the test (spin bound
    restored, the product library put back afterwards)."""
    from mgcn import _lib as L
    assert os.path.exists(EXP_LIB), (
        f"{EXP_LIB} missing: build it with `make -C meta-gcn_amd/csrc exp` "
        "(__graft_entry__.build() does)")
    prod = L.load()
    exp = L.load(EXP_LIB)
    L._lib = exp
    try:
        yield exp
    finally:
        exp.mgcn_set_option(b"ws_spin_limit", 1 << 25)
        torch.cuda.synchronize()
        exp.mgcn_check_device(None, 1)  # leave no pending word behind
        L._lib = prod


def _spin(lib, n):
    from mgcn import _lib as L
    L.check(lib.mgcn_set_option(b"ws_spin_limit", int(n)), "ws_spin_limit")


def test_product_library_rejects_experiment_switches(cuda):
    from mgcn import _lib as L
    lib = L.load()
    for name in (b"ws_spin_limit", b"wide_dbg", b"xw_ws_dbg"):
        assert lib.mgcn_set_option(name, 1) == L.EINVAL
        assert b"experiment builds only" in lib.mgcn_last_error()


@pytest.mark.parametrize("F", [128, 256])
def test_abort_surfaces_through_check_device(cuda, exp_lib, F):
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import plan_for
    N = 40000
    ei = _graph(np.random.default_rng(F), N, 8 * N).to(cuda)
    plan = plan_for(ei, N)
    norm = plan.norm("sm")
    g = torch.Generator(device=cuda).manual_seed(F)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    dY = torch.randn(N, F, device=cuda, generator=g)

    def run():
        if F == 128:  # the DWS adjoint: dW + dX in one launch
            return ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W)
        return ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM)  # the wide WS forward

    good = run()
    L.check_device(sync=True)  # default bound: nothing to report
    _spin(exp_lib, 1)
    run()  # the launch itself returns OK: the failure is only known on the device
    with pytest.raises(L.MgcnError, match="spin bound") as ei_:
        L.check_device(sync=True)
    assert "code 5" in str(ei_.value)
    L.check_device(sync=True)  # reading the word cleared it
    # the default bound again: the experiment build computes the product's bits
    _spin(exp_lib, 1 << 25)
    again = run()
    L.check_device(sync=True)
    good = good if isinstance(good, tuple) else (good,)
    again = again if isinstance(again, tuple) else (again,)
    for a, b in zip(good, again):
        if a is not None:
            assert torch.equal(a, b)


def test_abort_fails_the_next_call(cuda, exp_lib):
    """Without an explicit check the next mgcn_spmm_xw_* call reports it."""
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import plan_for
    N, F = 30000, 256
    ei = _graph(np.random.default_rng(7), N, 8 * N).to(cuda)
    plan = plan_for(ei, N)
    norm = plan.norm("sm")
    g = torch.Generator(device=cuda).manual_seed(7)
    dY = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    _spin(exp_lib, 1)
    ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)  # wide dX-only
    torch.cuda.synchronize()
    _spin(exp_lib, 1 << 25)
    with pytest.raises(L.MgcnError, match="spmm_xw_wide_ws_kernel"):
        ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)
    # reported once: the call after that runs normally
    ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)
    L.check_device(sync=True)
