"""Gather rate against the size of the gathered table (config 5's question:
its rank-local kernels gather 1-KB rows from a 51-GB table).

R destination rows of `deg` uniformly random in-edges each, sources drawn
from the first T rows of one resident [T_max, F] table; for each T the fused
forward (mgcn_spmm_xw_fwd, Z written) and the plain SpMM are timed with HIP
events and reported as algorithmic GB/s.  A rate that falls with T while the
bytes per launch stay fixed is address translation, not HBM.

    python scripts/bench_table_size.py [--rows 1560000 --deg 11 --feat 256]
Prints one JSON line per (F, T).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_560_000)
    ap.add_argument("--deg", type=int, default=11)
    ap.add_argument("--feat", type=int, nargs="+", default=[256, 128])
    ap.add_argument("--tables", type=int, nargs="+",
                    default=[1_560_000, 6_250_000, 25_000_000, 50_000_000])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import build_view
    R, D = args.rows, args.deg
    g = torch.Generator(device=dev).manual_seed(0)
    dst = torch.arange(R, device=dev).repeat_interleave(D)
    u = torch.rand(R * D, device=dev, generator=g)
    for F in args.feat:
        Tmax = max(args.tables)
        X = torch.empty(Tmax, F, device=dev)
        X.normal_(generator=g)
        W = torch.randn(F, F, device=dev, generator=g) / F ** 0.5
        for T in args.tables:
            src = (u * T).long().clamp_(max=T - 1)
            view = build_view(dst, src, R, T, schedule=False)
            Xt = X[:T]
            nnz = R * D
            b_spmm = 8 * (R + 1) + nnz * (4 + 4 * F) + 4 * R * F
            rec = {"F": F, "table_rows": T, "table_gb": T * F * 4 / 1e9, "rows": R, "nnz": nnz}
            if ops.spmm_xw_supported(view, F, F, L.REDUCE_SUM):
                Y = torch.empty(R, F, device=dev)
                Z = torch.empty(R, F, device=dev)
                ms = timed(lambda: ops.spmm_xw_fwd(view, None, Xt, W, L.REDUCE_SUM, want_z=True,
                                                   out=Y, z_out=Z))
                byts = b_spmm + 4 * R * F
                rec.update(xw_fwd_ms=ms, xw_fwd_gbs=byts / ms / 1e6)
            ms = timed(lambda: ops.spmm_fwd(view, None, Xt, L.REDUCE_SUM))
            rec.update(spmm_ms=ms, spmm_gbs=b_spmm / ms / 1e6)
            print(json.dumps(rec), flush=True)
            del view
        del X


if __name__ == "__main__":
    main()
