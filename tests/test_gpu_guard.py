"""Guard bands around every buffer libmgcn writes (round-5 audit of the r4g
abort: HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION in torch's reduce kernel right
after the sharded backward's chunked dX-only adjoints, world 4, ~190-row
chunks -- gpurun_out/r4g/gpu_tests.log:47-75).

Every output, mask, column-sum vector and workspace of the entries the
sharded stack calls -- mgcn_spmm_xw_fwd, the dX-only and full
mgcn_spmm_xw_bwd, mgcn_gemm_bwd (dW-only with the bias column sums),
mgcn_gemm_nn's ReLU epilogue, mgcn_spmm_fwd / _bwd, relu_bwd_colsum and the
pack / unpack of the zero-skipping exchange -- is placed inside a larger
allocation whose bands before and after it hold a sentinel bit pattern.
Each entry runs on row-range views of a CSR (the dist path's `rows(a, e)`
chunks: absolute slot offsets, a nonzero first row) at 1, 15, 17, 31, 33 and
190 rows, and at empty chunks; afterwards every band must be untouched, and
the rows written must equal the same rows of a whole-view run bit for bit.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SENT = 0x7FBADBAD  # a NaN bit pattern no kernel writes
BAND = 4096        # 16 KB of sentinel words on each side


class Guarded:
    """A [*shape] tensor (16-byte aligned, contiguous) between two sentinel bands."""

    def __init__(self, shape, dtype, dev, fill=None):
        n = int(np.prod(shape)) if len(shape) else 1
        words = (n + 3) // 4 if dtype == torch.uint8 else n
        self.base = torch.full((BAND + words + BAND,), SENT, dtype=torch.int32, device=dev)
        mid = self.base[BAND:BAND + words]
        if dtype == torch.float32:
            mid = mid.view(torch.float32)
        elif dtype == torch.uint8:
            mid = mid.view(torch.uint8)[:n]
        self.t = mid.view(*shape) if len(shape) else mid
        if fill is not None:
            self.t.copy_(fill)
        assert self.t.data_ptr() % 16 == 0

    def intact(self):
        torch.cuda.synchronize()
        b = self.base
        return bool((b[:BAND] == SENT).all()) and bool((b[b.numel() - BAND:] == SENT).all())


def _graph(N=600, pairs=5000, seed=0):
    g = torch.Generator().manual_seed(seed)
    s = torch.randint(0, N, (pairs,), generator=g)
    d = torch.randint(0, N, (pairs,), generator=g)
    loops = torch.arange(N)
    return torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])


SIZES = [1, 15, 17, 31, 33, 190, 0]
STARTS = [0, 5, 211]


@pytest.fixture(scope="module")
def setup(cuda):
    from mgcn.graph import plan_for
    N = 600
    ei = _graph(N).to(cuda)
    plan = plan_for(ei, N)
    norm = plan.norm("sm")
    assert plan.fwd.n_heavy == 0
    return N, plan, norm


def _ws(lib, name, *args):
    return int(getattr(lib, name)(*args))


@pytest.mark.parametrize("F", [128, 256])
def test_fused_forward_bands(cuda, setup, F):
    from mgcn import _lib as L
    from mgcn import ops
    N, plan, norm = setup
    lib = L.load()
    g = torch.Generator(device=cuda).manual_seed(F)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    b = torch.randn(F, device=cuda, generator=g) * 0.1
    mw = ops.mask_words(F)
    Yf, Zf = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, b, True,
                             relu_mask=(mf := torch.empty(N, mw, dtype=torch.int32, device=cuda)),
                             want_z=True)
    wsb = _ws(lib, "mgcn_spmm_xw_fwd_workspace_bytes", F, F)
    for a in STARTS:
        for n in SIZES:
            if a + n > N:
                continue
            v = plan.fwd.rows(a, a + n)
            Y = Guarded((n, F), torch.float32, cuda)
            Z = Guarded((n, F), torch.float32, cuda)
            M = Guarded((n, mw), torch.int32, cuda)
            ws = Guarded((max(wsb, 16),), torch.uint8, cuda)
            with L.device_guard(cuda):
                rc = lib.mgcn_spmm_xw_fwd(n, v.n_cols, F, F, L.ptr(v.rowptr), L.ptr(v.col),
                                          L.ptr(norm.w_fwd), L.ptr(X), F, L.ptr(W), F, L.ptr(b),
                                          L.ptr(Y.t), F, L.REDUCE_SUM, 1, L.ptr(M.t), L.ptr(Z.t), F,
                                          L.ptr(ws.t) if wsb else None, wsb, L.stream_of(cuda))
            L.check(rc, "mgcn_spmm_xw_fwd")
            for gd in (Y, Z, M, ws):
                assert gd.intact(), (F, a, n)
            assert torch.equal(Y.t, Yf[a:a + n]) and torch.equal(Z.t, Zf[a:a + n])
            assert torch.equal(M.t, mf[a:a + n])


@pytest.mark.parametrize("F", [128, 256])
@pytest.mark.parametrize("mean", [False, True])
def test_dx_only_adjoint_bands(cuda, setup, F, mean):
    from mgcn import _lib as L
    from mgcn import ops
    N, plan, norm = setup
    lib = L.load()
    g = torch.Generator(device=cuda).manual_seed(2 * F + mean)
    dY = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    mw = ops.mask_words(F)
    rm = torch.randint(-2 ** 31, 2 ** 31 - 1, (N, mw), dtype=torch.int32, device=cuda,
                       generator=g)
    rd = plan.in_cnt if mean else None
    _, dXf, csf = ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, None, W, relu_mask=rm,
                                  row_div=rd)
    wsb = _ws(lib, "mgcn_spmm_xw_bwd_workspace_bytes", N, F, F)
    for a in STARTS:
        for n in SIZES:
            if a + n > N:
                continue
            v = plan.bwd.rows(a, a + n)
            dX = Guarded((n, F), torch.float32, cuda)
            cs = Guarded((F,), torch.float32, cuda, fill=torch.zeros(F))
            ws = Guarded((wsb,), torch.uint8, cuda)
            for acc in (0, 1):
                with L.device_guard(cuda):
                    rc = lib.mgcn_spmm_xw_bwd(
                        n, v.n_cols, F, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(norm.w_bwd), None,
                        L.ptr(dY), F, None, 0, L.ptr(W), F, None, 0, acc, L.ptr(dX.t), F,
                        L.ptr(rm[a:]), L.ptr(rd[a:] if rd is not None else None), L.ptr(cs.t),
                        None, None, L.ptr(ws.t), wsb, L.stream_of(cuda))
                L.check(rc, "mgcn_spmm_xw_bwd")
            for gd in (dX, cs, ws):
                assert gd.intact(), (F, a, n)
            assert torch.equal(dX.t, dXf[a:a + n])


def test_full_adjoint_and_dw_pass_bands(cuda, setup):
    from mgcn import _lib as L
    N, plan, norm = setup
    lib = L.load()
    F = 128
    g = torch.Generator(device=cuda).manual_seed(3)
    dY = torch.randn(N, F, device=cuda, generator=g)
    X = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    rm = torch.randint(-2 ** 31, 2 ** 31 - 1, (N, 4), dtype=torch.int32, device=cuda, generator=g)
    wsb = _ws(lib, "mgcn_spmm_xw_bwd_workspace_bytes", N, F, F)
    wsg = _ws(lib, "mgcn_gemm_bwd_workspace_bytes", N, F, F)
    for a in STARTS:
        for n in SIZES:
            if a + n > N:
                continue
            v = plan.bwd.rows(a, a + n)
            dW = Guarded((F, F), torch.float32, cuda)
            dX = Guarded((n, F), torch.float32, cuda)
            cs = Guarded((F,), torch.float32, cuda)
            ws = Guarded((wsb,), torch.uint8, cuda)
            with L.device_guard(cuda):
                rc = lib.mgcn_spmm_xw_bwd(
                    n, v.n_cols, F, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(norm.w_bwd), None,
                    L.ptr(dY), F, L.ptr(X[a:]), F, L.ptr(W), F, L.ptr(dW.t), F, 0, L.ptr(dX.t), F,
                    L.ptr(rm[a:]), None, L.ptr(cs.t), None, None, L.ptr(ws.t), wsb,
                    L.stream_of(cuda))
            L.check(rc, "mgcn_spmm_xw_bwd (full)")
            for gd in (dW, dX, cs, ws):
                assert gd.intact(), (a, n)
            # the dense dW-only pass with the dH column sums (mgcn_gemm_bwd)
            dW2 = Guarded((F, F), torch.float32, cuda)
            cs2 = Guarded((F,), torch.float32, cuda)
            ws2 = Guarded((wsg,), torch.uint8, cuda)
            with L.device_guard(cuda):
                rc = lib.mgcn_gemm_bwd(n, F, F, L.ptr(X[a:]), F, L.ptr(dY[a:]), F, L.ptr(W), F,
                                       L.ptr(dW2.t), F, 0, None, F, None, None, L.ptr(cs2.t),
                                       L.ptr(ws2.t), wsg, L.stream_of(cuda))
            L.check(rc, "mgcn_gemm_bwd")
            for gd in (dW2, cs2, ws2):
                assert gd.intact(), (a, n)
            ref = (X[a:a + n].double().t() @ dY[a:a + n].double()).float()
            torch.testing.assert_close(dW2.t, ref, rtol=1e-4, atol=1e-4)


def test_spmm_gemm_elementwise_bands(cuda, setup):
    from mgcn import _lib as L
    from mgcn import ops
    N, plan, norm = setup
    lib = L.load()
    F = 128
    g = torch.Generator(device=cuda).manual_seed(4)
    H = torch.randn(N, F, device=cuda, generator=g)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    Yf, _ = ops.spmm_fwd(plan.fwd, norm.w_fwd, H, L.REDUCE_SUM)
    dHf = ops.spmm_bwd(plan.bwd, norm.w_bwd, None, H, L.REDUCE_SUM)
    for a in STARTS:
        for n in SIZES:
            if a + n > N:
                continue
            Y = Guarded((n, F), torch.float32, cuda)
            ops.spmm_fwd(plan.fwd.rows(a, a + n), norm.w_fwd, H, L.REDUCE_SUM, out=Y.t)
            dH = Guarded((n, F), torch.float32, cuda)
            ops.spmm_bwd(plan.bwd.rows(a, a + n), norm.w_bwd, None, H, L.REDUCE_SUM, out=dH.t)
            assert Y.intact() and dH.intact(), (a, n)
            assert torch.equal(Y.t, Yf[a:a + n]) and torch.equal(dH.t, dHf[a:a + n])
            # gemm_nn's ReLU-mask epilogue (the unfused dX) with guarded outputs
            if n:
                rm = ops.make_relu_mask(H[a:a + n])
                wsb = _ws(lib, "mgcn_gemm_nn_workspace_bytes", n, F)
                C = Guarded((n, F), torch.float32, cuda)
                cs = Guarded((F,), torch.float32, cuda)
                ws = Guarded((wsb,), torch.uint8, cuda)
                Wt = W.t()
                with L.device_guard(cuda):
                    rc = lib.mgcn_gemm_nn(n, F, F, L.ptr(H[a:]), F, L.ptr(W), Wt.stride(0),
                                          Wt.stride(1), L.ptr(C.t), F, L.ptr(rm), None,
                                          L.ptr(cs.t), L.ptr(ws.t), wsb, L.stream_of(cuda))
                L.check(rc, "mgcn_gemm_nn")
                assert C.intact() and cs.intact() and ws.intact(), (a, n)
                # relu_bwd_colsum with a guarded column-sum workspace
                wsc = _ws(lib, "mgcn_colsum_workspace_bytes", n, F)
                dYo = Guarded((n, F), torch.float32, cuda)
                db = Guarded((F,), torch.float32, cuda)
                ws3 = Guarded((max(wsc, 16),), torch.uint8, cuda)
                with L.device_guard(cuda):
                    rc = lib.mgcn_relu_bwd_colsum(n, F, L.ptr(H[a:]), L.ptr(Y.t), 1, None,
                                                  L.ptr(dYo.t), L.ptr(db.t), L.ptr(ws3.t), wsc,
                                                  L.stream_of(cuda))
                L.check(rc, "mgcn_relu_bwd_colsum")
                assert dYo.intact() and db.intact() and ws3.intact(), (a, n)


@pytest.mark.parametrize("F", [128, 256])
def test_pack_unpack_bands(cuda, F):
    from mgcn import ops
    g = torch.Generator(device=cuda).manual_seed(F)
    for n in [1, 15, 17, 31, 33, 190]:
        rows = torch.relu(torch.randn(n, F, device=cuda, generator=g))
        words = F // 32
        counts = Guarded((n,), torch.int32, cuda)
        # the count pass writes only the header's mask words: its guard bands
        # and the interleaved position words must stay as they are
        hdr = Guarded((n, 2 * words), torch.int32, cuda)
        hdr.t.fill_(-1)
        ops.pack_rows_count(rows, hdr.t, counts.t)
        assert (hdr.t[:, 1::2] == -1).all()
        total = int(counts.t.sum())
        offs = torch.cumsum(counts.t, 0, dtype=torch.int32) - counts.t
        seg = 2 * n * words + total
        send = Guarded((seg,), torch.int32, cuda)
        send.t[:2 * n * words] = hdr.t.view(-1)
        ops.pack_rows_values(rows, offs, send.t[:2 * n * words].view(n, 2 * words),
                             send.t[2 * n * words:])
        masks = hdr
        P = 3
        recv = torch.cat([send.t] * P)
        out = Guarded((P * n, F), torch.float32, cuda)
        ops.unpack_rows(recv, P, n, seg, out.t)
        for gd in (masks, counts, send, out):
            assert gd.intact(), (F, n)
        assert torch.equal(out.t, rows.repeat(P, 1))


@pytest.mark.parametrize("F", [32, 128, 256])
def test_single_pass_pack_bands(cuda, F):
    """mgcn_pack_rows: header, values (sized to exactly the nonzero words),
    the device total and the look-back workspace between sentinel bands,
    at row counts inside one tile and across tiles; the packed buffer is the
    two-pass one."""
    from mgcn import _lib as L
    from mgcn import ops
    lib = L.load()
    g = torch.Generator(device=cuda).manual_seed(F + 1)
    for n in [1, 15, 17, 31, 33, 190, 1000, 4099]:
        rows = torch.relu(torch.randn(n, F, device=cuda, generator=g))
        words = F // 32
        nv = int((rows.view(torch.int32) != 0).sum())
        hdr = Guarded((n, 2 * words), torch.int32, cuda)
        vals = Guarded((nv,), torch.int32, cuda)
        tot = Guarded((2,), torch.int32, cuda)
        wsb = _ws(lib, "mgcn_pack_rows_workspace_bytes", n, F)
        ws = Guarded((wsb,), torch.uint8, cuda)
        rc = lib.mgcn_pack_rows(n, F, L.ptr(rows), F, L.ptr(hdr.t), L.ptr(vals.t), L.ptr(tot.t),
                                L.ptr(ws.t), wsb, L.stream_of(cuda))
        L.check(rc, "mgcn_pack_rows")
        for gd in (hdr, vals, tot, ws):
            assert gd.intact(), (F, n)
        assert int(tot.t.view(torch.int64)[0]) == nv
        counts = torch.empty(n, dtype=torch.int32, device=cuda)
        h2 = torch.empty(n, 2 * words, dtype=torch.int32, device=cuda)
        ops.pack_rows_count(rows, h2, counts)
        v2 = torch.empty(nv, dtype=torch.int32, device=cuda)
        ops.pack_rows_values(rows, torch.cumsum(counts, 0, dtype=torch.int32) - counts, h2, v2)
        assert torch.equal(hdr.t, h2) and torch.equal(vals.t, v2)
