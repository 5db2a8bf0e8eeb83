"""libmgcn's zero-skipping row packing (mgcn_pack_rows_count / _values,
mgcn_unpack_rows; mgcn.dist's packed table exchange) on the GPU: the packed
buffer is word for word the layout the CPU double (tests/cpu_backend.py)
writes, and unpacking restores every row bit for bit -- -0.0, NaN, denormals,
all-zero and all-dense rows included -- across several segments."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _rows(n, F, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, F, generator=g)
    x = torch.where(torch.rand(n, F, generator=g) < 0.5, torch.zeros(()), x)
    if n >= 8:
        x[0] = 0.0                       # all zero
        x[1] = torch.randn(F, generator=g)  # dense
        x[2, ::3] = -0.0                 # negative zeros are values
        x[3, 1] = float("nan")
        x[3, 2] = float("inf")
        x[4, :5] = 1e-42                 # denormals
    return x


def _pack_gpu(x, cuda):
    from mgcn import ops
    n, F = x.shape
    w = F // 32
    xs = x.to(cuda)
    head = 2 * n * w
    send = torch.empty(head + n * F, dtype=torch.int32, device=cuda)
    counts = torch.empty(n, dtype=torch.int32, device=cuda)
    hdr = send[:head].view(n, 2 * w)
    ops.pack_rows_count(xs, hdr, counts)
    total = int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts
    ops.pack_rows_values(xs, offs, hdr, send[head:head + total])
    return send[:head + total].cpu(), counts.cpu()


def _pack_cpu(x):
    from cpu_backend import CpuBackend
    be = CpuBackend()
    n, F = x.shape
    w = F // 32
    head = 2 * n * w
    send = torch.empty(head + n * F, dtype=torch.int32)
    counts = torch.empty(n, dtype=torch.int32)
    hdr = send[:head].view(n, 2 * w)
    be.pack_count(x, hdr, counts)
    total = int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts
    be.pack_values(x, offs, hdr, send[head:head + total])
    return send[:head + total], counts


@pytest.mark.parametrize("n,F", [(1, 32), (37, 32), (1000, 128), (4097, 256), (64, 96),
                                 (130, 512),
                                 # past one grid-stride trip of the capped grid (the
                                 # pack kernels take 4 rows per wave and trip)
                                 (300_001, 256), (270_007, 128)])
def test_pack_layout_matches_cpu_double_and_round_trips(cuda, n, F):
    from mgcn import ops
    x = _rows(n, F, seed=n + F)
    got, cnt = _pack_gpu(x, cuda)
    ref, cnt_ref = _pack_cpu(x)
    assert torch.equal(cnt, cnt_ref)
    np.testing.assert_array_equal(got.numpy(), ref.numpy())
    # three segments (three ranks' chunks) expanded at once
    xs = [x, _rows(n, F, seed=7), _rows(n, F, seed=8)]
    packs = [_pack_gpu(t, cuda)[0] for t in xs]
    seg = max(p.numel() for p in packs)
    buf = torch.zeros(3 * seg, dtype=torch.int32)
    for p, t in enumerate(packs):
        buf[p * seg:p * seg + t.numel()] = t
    out = torch.full((3 * n, F), 123.0, device=cuda)
    ops.unpack_rows(buf.to(cuda), 3, n, seg, out)
    back = out.cpu().view(torch.int32).numpy()
    want = torch.cat(xs).view(torch.int32).numpy()
    np.testing.assert_array_equal(back, want)  # bit for bit, -0.0 and NaN payloads included


def test_pack_rows_with_a_leading_dimension(cuda):
    """Rows of a wider buffer (ld > F): only the F columns travel."""
    from mgcn import ops
    n, F = 300, 64
    big = _rows(n, 2 * F, seed=3).to(cuda)
    x = big[:, :F]
    w = F // 32
    counts = torch.empty(n, dtype=torch.int32, device=cuda)
    hdr = torch.empty(n, 2 * w, dtype=torch.int32, device=cuda)
    ops.pack_rows_count(x, hdr, counts)
    ref_h = torch.empty(n, 2 * w, dtype=torch.int32)
    ref_c = torch.empty(n, dtype=torch.int32)
    from cpu_backend import CpuBackend
    CpuBackend().pack_count(x.cpu().contiguous(), ref_h, ref_c)
    assert torch.equal(hdr.cpu()[:, 0::2], ref_h[:, 0::2]) and torch.equal(counts.cpu(), ref_c)


def _pack_gpu_one_pass(xs, cuda):
    from mgcn import ops
    n, F = xs.shape
    head = 2 * n * (F // 32)
    send = torch.full((head + n * F,), -7, dtype=torch.int32, device=cuda)
    total = torch.full((1,), -1, dtype=torch.int64, device=cuda)
    ops.pack_rows(xs, send[:head].view(n, 2 * (F // 32)), send[head:], total)
    t = int(total.item())
    return send[:head + t], t


@pytest.mark.parametrize("n,F", [(1, 32), (37, 32), (515, 64), (1000, 128), (4097, 256),
                                 (300_001, 256), (270_007, 128), (100_003, 32)])
def test_single_pass_pack_is_the_two_pass_pack(cuda, n, F):
    """mgcn_pack_rows (one read, decoupled look-back over tiles) writes the
    buffer mgcn_pack_rows_count + _values write, word for word, and its
    device total is the values' number (thousands of tiles at the larger
    sizes: look-back windows past 64 predecessors)."""
    x = _rows(n, F, seed=n * 3 + F)
    got, t = _pack_gpu_one_pass(x.to(cuda), cuda)
    ref, cnt = _pack_gpu(x, cuda)
    assert t == int(cnt.sum())
    np.testing.assert_array_equal(got.cpu().numpy(), ref.numpy())
    if n <= 5000:
        np.testing.assert_array_equal(got.cpu().numpy(), _pack_cpu(x)[0].numpy())


def test_single_pass_pack_at_a_rank_chunk_with_a_leading_dimension(cuda):
    """A config-5-sized chunk (1.56M rows x 256, ~1.6 GB; ReLU'd, about half
    zeros) taken from a wider buffer (ld > F), against the two-pass pack on
    the device; empty input writes total = 0."""
    from mgcn import ops
    n, F = 1_560_000, 256
    g = torch.Generator(device=cuda).manual_seed(11)
    big = torch.relu(torch.randn(n, F + 32, device=cuda, generator=g))
    x = big[:, :F]
    got, t = _pack_gpu_one_pass(x, cuda)
    head = 2 * n * (F // 32)
    send = torch.empty(head + n * F, dtype=torch.int32, device=cuda)
    counts = torch.empty(n, dtype=torch.int32, device=cuda)
    hdr = send[:head].view(n, 2 * (F // 32))
    ops.pack_rows_count(x, hdr, counts)
    offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts
    ops.pack_rows_values(x, offs, hdr, send[head:])
    assert t == int(counts.sum())
    assert torch.equal(got, send[:head + t])
    del big, send, got
    total = torch.full((1,), -1, dtype=torch.int64, device=cuda)
    e = torch.empty(0, F, device=cuda)
    ops.pack_rows(e, torch.empty(0, 16, dtype=torch.int32, device=cuda),
                  torch.empty(0, dtype=torch.int32, device=cuda), total)
    assert int(total.item()) == 0


# ------------------------------------------------- in-place packed gather
def _packed_table(T, cr, cuda, n_bufs=2):
    """T [S cr, F] (S segments of cr rows) packed segment by segment into
    n_bufs separate device buffers: a PackedTable over them."""
    from mgcn import ops
    S = T.size(0) // cr
    segs = [_pack_gpu(T[s * cr:(s + 1) * cr], cuda)[0] for s in range(S)]
    per = -(-S // n_bufs)
    bufs, seg_buf, seg_off = [], [], []
    for b in range(n_bufs):
        part = segs[b * per:(b + 1) * per]
        if not part:
            break
        off = 0
        words = []
        for p in part:
            seg_buf.append(len(bufs))
            seg_off.append(off)
            words.append(p)
            off += p.numel()
        words.append(torch.zeros(4, dtype=torch.int32))  # the 16-B value reads' slack
        bufs.append(torch.cat(words).to(cuda))
    return ops.PackedTable(bufs, seg_buf, seg_off, cr, ops.packed_row_bits(cr), T.size(1))


def _graph_view(rng, n_rows, T_rows, E, cuda, heavy=0):
    from mgcn.graph import CSRView
    dst = np.concatenate([rng.integers(0, n_rows, E), np.zeros(heavy, np.int64)])
    src = np.concatenate([rng.integers(0, T_rows, E), rng.integers(0, T_rows, heavy)])
    order = np.argsort(dst, kind="stable")
    rowptr = np.zeros(n_rows + 1, np.int64)
    rowptr[1:] = np.cumsum(np.bincount(dst, minlength=n_rows))
    col = src[order].astype(np.int32)
    w = rng.uniform(0.1, 1.0, len(col)).astype(np.float32)
    v = CSRView(rowptr=torch.from_numpy(rowptr).to(cuda), col=torch.from_numpy(col).to(cuda),
                eid=torch.from_numpy(order.astype(np.int32)).to(cuda), n_rows=n_rows,
                n_cols=T_rows)
    return v, torch.from_numpy(w).to(cuda)


def _mask256(Z):
    """[rows, 8] ReLU mask words of a 256-wide layer (fused_wide.hip layout:
    feature f at word 4 (f >> 7) + (f & 3), bit (f & 127) >> 2)."""
    f = torch.arange(256, device=Z.device)
    word = 4 * (f >> 7) + (f & 3)
    bit = (f & 127) >> 2
    m = torch.zeros(Z.size(0), 8, dtype=torch.int64, device=Z.device)
    m.index_add_(1, word, (Z > 0).long() << bit)
    return torch.where(m >= 2 ** 31, m - 2 ** 32, m).to(torch.int32)


def _pk_view(v, cr, rb):
    from mgcn import ops
    from mgcn.graph import CSRView
    return CSRView(rowptr=v.rowptr, col=ops.packed_cols(v.col, cr, rb), eid=v.eid,
                   n_rows=v.n_rows, n_cols=v.n_cols)


def _relu_mask(Z):
    """The lower layer's ReLU mask words of Z (> 0) in the fused kernels'
    layout for Z's width."""
    from mgcn import ops
    return _mask256(Z) if Z.size(1) == 256 else ops.make_relu_mask(Z)


@pytest.mark.parametrize("n_rows,cr,S,E,heavy", [(5000, 700, 6, 60000, 0), (33, 1000, 3, 300, 150),
                                                 (4097, 4097, 2, 50000, 0)])
@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("F", [128, 256])
def test_packed_gather_forward_bitwise_the_dense_table(cuda, n_rows, cr, S, E, heavy, mean, F):
    """mgcn_spmm_xw_fwd_packed == mgcn_spmm_xw_fwd on the unpacked table: Y,
    Z and the ReLU mask words bit for bit (ragged segments, rows past 32 / 64
    slots, empty rows, -0.0 values; at F = 256 two receive buffers, at
    F = 128 one -- its kernels read the table through one 2-GiB range)."""
    from mgcn import _lib as L
    from mgcn import ops
    rng = np.random.default_rng(n_rows + S)
    T = torch.relu(torch.randn(S * cr, F, generator=torch.Generator().manual_seed(S)))
    T[::7, ::5] = -0.0
    tab = _packed_table(T, cr, cuda, n_bufs=2 if F == 256 else 1)
    v, w = _graph_view(rng, n_rows, S * cr, E, cuda, heavy)
    vp = _pk_view(v, cr, tab.row_bits)
    g = torch.Generator(device=cuda).manual_seed(1)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    b = torch.randn(F, device=cuda, generator=g)
    red = L.REDUCE_MEAN if mean else L.REDUCE_SUM
    outs = []
    for view, X in ((v, T.to(cuda)), (vp, tab)):
        rm = torch.empty(n_rows, ops.mask_words(F), dtype=torch.int32, device=cuda)
        y, z = ops.spmm_xw_fwd(view, w, X, W, red, b, True, relu_mask=rm, want_z=True)
        outs.append((y, z, rm))
    for a, b_ in zip(*outs):
        assert torch.equal(a.view(torch.int32), b_.view(torch.int32))


@pytest.mark.parametrize("n_rows,cr,S,E", [(5000, 700, 6, 60000), (33, 1000, 3, 300)])
@pytest.mark.parametrize("epi", ["store", "relu", "relu_div"])
@pytest.mark.parametrize("F", [128, 256])
def test_packed_gather_adjoint_bitwise_the_dense_table(cuda, n_rows, cr, S, E, epi, F):
    """mgcn_spmm_xw_bwd_packed == the dX-only mgcn_spmm_xw_bwd on the unpacked
    table: dX bit for bit, the accumulated column sums too."""
    from mgcn import ops
    rng = np.random.default_rng(7 * n_rows + S)
    T = torch.randn(S * cr, F, generator=torch.Generator().manual_seed(S + 1))
    T = torch.where(torch.rand(S * cr, F, generator=torch.Generator().manual_seed(2)) < 0.5,
                    torch.zeros(()), T)
    tab = _packed_table(T, cr, cuda, n_bufs=3 if F == 256 else 1)
    v, w = _graph_view(rng, n_rows, S * cr, E, cuda)
    vp = _pk_view(v, cr, tab.row_bits)
    g = torch.Generator(device=cuda).manual_seed(3)
    W = torch.randn(F, F, device=cuda, generator=g) * 0.1
    rs = torch.rand(n_rows, device=cuda, generator=g)
    rm = rd = None
    if epi != "store":
        rm = _relu_mask(torch.randn(n_rows, F, device=cuda, generator=g))
    if epi == "relu_div":
        rd = torch.randint(1, 9, (n_rows,), device=cuda, generator=g).float()
    outs = []
    for view, X in ((v, T.to(cuda)), (vp, tab)):
        cs = torch.full((F,), 0.5, device=cuda) if rm is not None else None
        _, dX, c = ops.spmm_xw_bwd(view, w, rs, X, None, W, relu_mask=rm, row_div=rd,
                                   colsum_acc=cs)
        outs.append((dX, c))
    assert torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32))
    if rm is not None:
        assert torch.equal(outs[0][1], outs[1][1])


def test_packed_table_of_f128_must_fit_one_range(cuda):
    """An F = 128 packed table spanning more than 2 GiB (segments in buffers
    far apart) is refused with an error, never read."""
    from mgcn import _lib as L
    from mgcn import ops
    cr, F = 64, 128
    T = torch.relu(torch.randn(2 * cr, F, generator=torch.Generator().manual_seed(5)))
    tab = _packed_table(T, cr, cuda, n_bufs=1)
    W = torch.randn(F, F, device=cuda) * 0.1
    v, w = _graph_view(np.random.default_rng(1), 10, 2 * cr, 50, cuda)
    vp = _pk_view(v, cr, tab.row_bits)
    c = tab.c_struct()
    c.seg_base[1] = (1 << 29) + 8  # a second segment past the 2-GiB range
    c.n_words = (1 << 29) + 16
    lib = L.load()
    Y = torch.empty(10, F, device=cuda)
    rc = lib.mgcn_spmm_xw_fwd_packed(10, F, F, L.ptr(vp.rowptr), L.ptr(vp.col), L.ptr(w),
                                     L.byref(c), L.ptr(W), F, None, L.ptr(Y), F, L.REDUCE_SUM, 0,
                                     None, None, 0, None, 0, L.stream_of(cuda))
    assert rc == L.EINVAL and b"2 GiB" in lib.mgcn_last_error()
