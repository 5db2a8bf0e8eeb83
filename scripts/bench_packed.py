"""The fused layer kernels gathering a dense table vs the same table packed
(mgcn_spmm_xw_fwd / _bwd vs mgcn_spmm_xw_fwd_packed / _bwd_packed).  Default:
a config-5 rank's shape, 6.24M destination rows of ~11 slots over a table of
C * P segments of cr rows (4 x 8 x 1.56M = 50M rows, F = 256); `--config2`:
config 2's shape at F = 128 (1M rows of 11 slots over a 1M-row table in 8
segments, one receive buffer).  Half the table's words are +0.0 (a ReLU'd
layer).  `--alias` points that many consecutive segments at one physical
segment (the emulated rank's stand-in).  Prints one JSON line of per-launch
times (HIP events, median of --reps).

    python scripts/bench_packed.py [--rows 6240000 --cr 1561000 --segs 32 --reps 5]
    python scripts/bench_packed.py --config2
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_240_000)
    ap.add_argument("--cr", type=int, default=1_561_000)
    ap.add_argument("--segs", type=int, default=32)
    ap.add_argument("--deg", type=int, default=11)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--alias", type=int, default=8, help="segments sharing one physical segment")
    ap.add_argument("--config2", action="store_true", help="config 2's shape at F = 128")
    args = ap.parse_args()
    F = 256
    if args.config2:
        F = 128
        args.rows, args.cr, args.segs, args.alias = 1_000_000, 125_000, 8, 1
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import CSRView
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    T_rows = args.segs * args.cr
    n = args.rows
    nnz = n * args.deg
    rowptr = torch.arange(0, nnz + 1, args.deg, dtype=torch.int64, device=dev)
    col = torch.randint(0, T_rows, (nnz,), device=dev, generator=g, dtype=torch.int64)
    col = col.to(torch.int32)
    w = torch.rand(nnz, device=dev, generator=g)
    view = CSRView(rowptr=rowptr, col=col, eid=torch.zeros(1, dtype=torch.int32, device=dev),
                   n_rows=n, n_cols=T_rows)
    rb = ops.packed_row_bits(args.cr)
    pview = CSRView(rowptr=rowptr, col=ops.packed_cols(col, args.cr, rb), eid=view.eid,
                    n_rows=n, n_cols=T_rows)
    W = torch.randn(F, F, device=dev, generator=g) * 0.06
    b = torch.randn(F, device=dev, generator=g) * 0.1
    res = {"rows": n, "slots": nnz, "table_rows": T_rows, "segments": args.segs,
           "seg_rows": args.cr, "alias": args.alias}

    def timeit(fn):
        ts = []
        for _ in range(args.reps + 1):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts[1:])

    # the table, ReLU'd, built and packed one physical segment at a time
    n_phys = args.segs // args.alias
    bufs, seg_buf, seg_off = [], [], []
    W32 = F // 32
    packed_words = 0
    dense = torch.empty(T_rows, F, device=dev)
    for p in range(n_phys):
        x = torch.relu(torch.randn(args.cr, F, device=dev, generator=g))
        for k in range(args.alias):
            s = p * args.alias + k
            dense[s * args.cr:(s + 1) * args.cr] = x
        head = 2 * args.cr * W32
        send = torch.empty(head + args.cr * F + 4, dtype=torch.int32, device=dev)
        counts = torch.empty(args.cr, dtype=torch.int32, device=dev)
        hdr = send[:head].view(args.cr, 2 * W32)
        ops.pack_rows_count(x, hdr, counts)
        offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts
        cap = int(counts.sum())
        ops.pack_rows_values(x, offs, hdr, send[head:head + cap])
        packed_words += head + cap
        buf = send[:head + cap + 4].clone()
        del send
        bufs.append(buf)
        for k in range(args.alias):
            seg_buf.append(p)
            seg_off.append(0)
    if F == 128:  # one receive buffer (the F = 128 kernels' single range)
        offs_ = [0]
        for b_ in bufs:
            offs_.append(offs_[-1] + b_.numel())
        one = torch.cat(bufs)
        seg_off = [offs_[p] for p in seg_buf]
        seg_buf = [0] * len(seg_buf)
        bufs = [one]
    tab = ops.PackedTable(bufs, seg_buf, seg_off, args.cr, rb, F)
    res["packed_over_dense"] = packed_words / (n_phys * args.cr * F)
    rm = torch.empty(n, ops.mask_words(F), dtype=torch.int32, device=dev)
    Y = torch.empty(n, F, device=dev)
    Z = torch.empty(n, F, device=dev)
    res["fwd_dense_ms"] = timeit(lambda: ops.spmm_xw_fwd(view, w, dense, W, L.REDUCE_SUM, b, True,
                                                         relu_mask=rm, want_z=True, out=Y, z_out=Z))
    y_d = Y.clone()
    res["fwd_packed_ms"] = timeit(lambda: ops.spmm_xw_fwd(pview, w, tab, W, L.REDUCE_SUM, b, True,
                                                          relu_mask=rm, want_z=True, out=Y, z_out=Z))
    res["fwd_bitwise"] = bool(torch.equal(y_d, Y))
    dX = torch.empty(n, F, device=dev)
    cs = torch.zeros(F, device=dev)
    res["bwd_dense_ms"] = timeit(lambda: ops.spmm_xw_bwd(view, w, None, dense, None, W, relu_mask=rm,
                                                         dx_out=dX, colsum_acc=cs))
    x_d = dX.clone()
    res["bwd_packed_ms"] = timeit(lambda: ops.spmm_xw_bwd(pview, w, None, tab, None, W, relu_mask=rm,
                                                          dx_out=dX, colsum_acc=cs))
    res["bwd_bitwise"] = bool(torch.equal(x_d, dX))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
