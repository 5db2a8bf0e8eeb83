"""Config 5 at full size on ONE MI355X: N = 50M nodes, 250M pairs symmetrised
to E = 500M edges + 50M self-loops (550M slots), F = 256 (BASELINE.json
configs[4]).  The 8-GPU run shards destination rows; every rank still
gathers from the whole [N, F] feature matrix (51 GB) through int64 offsets
(N F = 12.8e9 > 2^31), which is what this checks:

* the sm-normalised forward SpMM and its adjoint over the whole graph, and
* bitwise equality, for a random sample of destination (source) rows, with a
  sequential fp32 restatement in COO order on the host (the oracle's
  arithmetic: products rounded, then added in edge order), and of the
  per-slot weights with dinv[src] * dinv[dst], dinv = 1 / sqrt(out-degree);
* the SpMM rate at this size (algorithmic bytes / HIP-event time).

    python scripts/config5_check.py [--nodes 50000000 --pairs 250000000 --feat 256]
Prints one JSON line.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

import mgcn  # noqa: E402
from mgcn import _lib as L  # noqa: E402
from mgcn.graph import schedule_rows  # noqa: E402
from mgcn.ops import spmm_bwd, spmm_fwd  # noqa: E402


def check_rows(view, w, X, Y, rows, dinv, src_is_col):
    """Sequential fp32 recomputation of Y[rows] from the view's slots."""
    bad = wbad = 0
    for r in rows.tolist():
        b, e = int(view.rowptr[r]), int(view.rowptr[r + 1])
        col = view.col[b:e].long()
        ww = w[b:e].cpu().numpy()
        # per-slot weight = dinv[src] * dinv[dst]
        other = col.cpu().numpy()
        ds, dd = (dinv[other], dinv[r]) if src_is_col else (dinv[r], dinv[other])
        wref = (ds * np.float32(dd)).astype(np.float32)
        wbad += int((wref != ww).sum())
        xs = X[col].cpu().numpy()
        acc = np.zeros(X.size(1), dtype=np.float32)
        for k in range(e - b):
            acc = (acc + (xs[k] * ww[k]).astype(np.float32)).astype(np.float32)
        bad += int((acc != Y[r].cpu().numpy()).sum())
    return bad, wbad


def time_it(fn, reps=3):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000_000)
    ap.add_argument("--pairs", type=int, default=250_000_000)
    ap.add_argument("--feat", type=int, default=256)
    ap.add_argument("--sample", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N, P, F = args.nodes, args.pairs, args.feat
    g = torch.Generator(device=dev).manual_seed(0)
    s = torch.randint(0, N, (P,), device=dev, generator=g)
    d = torch.randint(0, N, (P,), device=dev, generator=g)
    loops = torch.arange(N, device=dev)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    del s, d, loops
    nnz = ei.size(1)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    plan = mgcn.build_plan(ei, N)
    schedule_rows(plan.fwd)
    schedule_rows(plan.bwd)
    norm = plan.norm("sm")
    t1.record()
    torch.cuda.synchronize()
    prep_ms = t0.elapsed_time(t1)
    deg = torch.bincount(ei[0], minlength=N).cpu().numpy().astype(np.float32)
    dinv = (np.float32(1.0) / np.sqrt(deg)).astype(np.float32)
    dinv[np.isinf(dinv)] = 0
    del ei
    torch.cuda.empty_cache()
    X = torch.randn(N, F, device=dev, generator=g)
    Y, _ = spmm_fwd(plan.fwd, norm.w_fwd, X, L.REDUCE_SUM)
    torch.cuda.synchronize()
    byts = 8 * (N + 1) + nnz * (8 + 4 * F) + 4 * N * F
    ms_f = time_it(lambda: spmm_fwd(plan.fwd, norm.w_fwd, X, L.REDUCE_SUM, out=Y))
    rng = np.random.default_rng(1)
    rows = torch.from_numpy(rng.integers(0, N, args.sample))
    bad_f, wbad_f = check_rows(plan.fwd, norm.w_fwd, X, Y, rows, dinv, src_is_col=True)
    del Y
    torch.cuda.empty_cache()
    dH = spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, X, L.REDUCE_SUM)
    torch.cuda.synchronize()
    ms_b = time_it(lambda: spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, X, L.REDUCE_SUM,
                                    out=dH))
    bad_b, wbad_b = check_rows(plan.bwd, norm.w_bwd, X, dH, rows, dinv, src_is_col=False)
    out = {"workload": "config5 single-GPU full graph: N=%d, E=%d (+%d loops), F=%d" %
           (N, 2 * P, N, F), "nnz": nnz, "graph_prep_ms": prep_ms,
           "spmm_fwd_ms": ms_f, "spmm_bwd_ms": ms_b, "bytes_per_launch": byts,
           "fwd_gbs": byts / ms_f / 1e6, "bwd_gbs": byts / ms_b / 1e6,
           "edges_per_s_fwd": 2 * P / (ms_f * 1e-3),
           "sampled_rows": args.sample, "mismatched_values_fwd": bad_f,
           "mismatched_values_bwd": bad_b, "mismatched_weights": wbad_f + wbad_b,
           "max_in_degree": int((plan.fwd.rowptr[1:] - plan.fwd.rowptr[:-1]).max()),
           "peak_mem_gb": torch.cuda.max_memory_allocated() / 1e9}
    print(json.dumps(out), flush=True)
    if bad_f or bad_b or wbad_f or wbad_b:
        sys.exit(1)


if __name__ == "__main__":
    main()
