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
    head = n * (1 + w)
    send = torch.empty(head + n * F, dtype=torch.int32, device=cuda)
    counts = torch.empty(n, dtype=torch.int32, device=cuda)
    ops.pack_rows_count(xs, send[n:head].view(n, w), counts)
    total = int(counts.sum())
    offs = send[:n]
    torch.cumsum(counts, 0, dtype=torch.int32, out=offs)
    offs.sub_(counts)
    ops.pack_rows_values(xs, send[n:head].view(n, w), offs, send[head:head + total])
    return send[:head + total].cpu(), counts.cpu()


def _pack_cpu(x):
    from cpu_backend import CpuBackend
    be = CpuBackend()
    n, F = x.shape
    w = F // 32
    head = n * (1 + w)
    send = torch.empty(head + n * F, dtype=torch.int32)
    counts = torch.empty(n, dtype=torch.int32)
    be.pack_count(x, send[n:head].view(n, w), counts)
    total = int(counts.sum())
    send[:n] = torch.cumsum(counts, 0, dtype=torch.int32) - counts
    be.pack_values(x, send[n:head].view(n, w), send[:n], send[head:head + total])
    return send[:head + total], counts


@pytest.mark.parametrize("n,F", [(1, 32), (37, 32), (1000, 128), (4097, 256), (64, 96)])
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
    masks = torch.empty(n, w, dtype=torch.int32, device=cuda)
    ops.pack_rows_count(x, masks, counts)
    ref_m = torch.empty(n, w, dtype=torch.int32)
    ref_c = torch.empty(n, dtype=torch.int32)
    from cpu_backend import CpuBackend
    CpuBackend().pack_count(x.cpu().contiguous(), ref_m, ref_c)
    assert torch.equal(masks.cpu(), ref_m) and torch.equal(counts.cpu(), ref_c)
