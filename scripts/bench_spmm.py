"""Microbenchmark of the SpMM kernels on the config-2 graph (tuning aid).

    python scripts/bench_spmm.py [--reps 20] [--variants]

Times mgcn_spmm_fwd / mgcn_spmm_bwd with HIP events (interleaved variants in
one process, cdna_hip_programming.md §5.4 rule 24) and prints JSON lines with
the algorithmic GB/s of each.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]

import torch  # noqa: E402

import mgcn  # noqa: E402
from mgcn import ops  # noqa: E402
from mgcn.graph import plan_for  # noqa: E402
from bench import make_er_graph, spmm_bytes  # noqa: E402


def time_it(fn, reps):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    fn()
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    return ms[len(ms) // 2], ms[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--variants", action="store_true")
    ap.add_argument("--max", action="store_true",
                    help="the max aggregation (winner bits forward, MAXM adjoint) at every unroll")
    ap.add_argument("--once", action="store_true", help="one fwd + one bwd launch (for PMC runs)")
    ap.add_argument("--calibrate", action="store_true",
                    help="known-byte launches for PMC calibration: a 2 GiB copy, and the SpMM "
                         "on a 4M-node permutation graph (every 512-B row gathered exactly once)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.calibrate:
        src = torch.randn(512 * 1024 * 1024 // 1, device=dev)  # 2 GiB
        dst = torch.empty_like(src)
        dst.copy_(src)
        del src, dst
        Np = 4_000_000
        perm = torch.randperm(Np, device=dev)
        ei = torch.stack([perm, torch.arange(Np, device=dev)])
        Hp = torch.randn(Np, 128, device=dev)
        plan = plan_for(ei, Np)
        ops.spmm_fwd(plan.fwd, None, Hp, 0)
        torch.cuda.synchronize()
        print(json.dumps({"copy_read_bytes": 2**31, "copy_write_bytes": 2**31,
                          "perm_spmm_read_bytes": spmm_bytes(Np, Np, 128) - 4 * Np - 4 * Np * 128,
                          "perm_spmm_write_bytes": 4 * Np * 128}))
        return
    ei, N = make_er_graph()
    ei = ei.to(dev)
    F = args.feat
    H = torch.randn(N, F, device=dev)
    plan = plan_for(ei, N)
    norm = plan.norm("sm")
    nnz = plan.nnz
    if args.once:
        ops.spmm_fwd(plan.fwd, norm.w_fwd, H, 0)
        ops.spmm_bwd(plan.bwd, norm.w_bwd, None, H, 0)
        torch.cuda.synchronize()
        return
    B = spmm_bytes(N, nnz, F)
    if args.max:
        from mgcn import _lib as L
        sm = plan.slot_map()
        _, win = ops.spmm_fwd(plan.fwd, None, H, L.REDUCE_MAX, mask_plan=plan)
        Bm = B + 16 * nnz  # + the winner record of every edge (written / read)
        for u in (4, 6, 8):
            mgcn.set_option("spmm_unroll", u)
            f_med, f_min = time_it(lambda: ops.spmm_fwd(plan.fwd, None, H, L.REDUCE_MAX,
                                                        mask_plan=plan), args.reps)
            b_med, b_min = time_it(lambda: ops.spmm_bwd(plan.bwd, None, None, H, L.REDUCE_MAX,
                                                        win_mask=win, slot_map=sm), args.reps)
            s_med, _ = time_it(lambda: ops.spmm_fwd(plan.fwd, None, H, 0), args.reps)
            print(json.dumps({"variant": f"max_u{u}", "fwd_ms": f_med, "fwd_gbs": Bm / f_med / 1e6,
                              "bwd_ms": b_med, "bwd_gbs": Bm / b_med / 1e6, "sum_fwd_ms": s_med}),
                  flush=True)
        mgcn.set_option("spmm_unroll", 8)
        return
    variants = [("default", {})]
    if args.variants:
        variants += [(f"vec{v}_u{u}", {"spmm_vec": v, "spmm_unroll": u})
                     for v in (2, 4) for u in (4, 8, 16)]
    for name, opts in variants:
        mgcn.set_option("spmm_vec", opts.get("spmm_vec", 0))
        mgcn.set_option("spmm_unroll", opts.get("spmm_unroll", 8))
        f_med, f_min = time_it(lambda: ops.spmm_fwd(plan.fwd, norm.w_fwd, H, 0), args.reps)
        b_med, b_min = time_it(lambda: ops.spmm_bwd(plan.bwd, norm.w_bwd, None, H, 0), args.reps)
        print(json.dumps({"variant": name, "fwd_ms": f_med, "fwd_min_ms": f_min,
                          "fwd_gbs": B / f_med / 1e6, "bwd_ms": b_med,
                          "bwd_gbs": B / b_med / 1e6, "bytes": B}), flush=True)
    mgcn.set_option("spmm_vec", 0)
    mgcn.set_option("spmm_unroll", 8)


if __name__ == "__main__":
    main()
