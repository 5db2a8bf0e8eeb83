"""Fused layer forward (mgcn_spmm_xw_fwd) vs gemm_nn + spmm_fwd on config 2.

    python scripts/bench_fused.py [--reps 20] [--unroll 4 8]

Times both forms with HIP events, interleaved in one process, checks the
fused output against the two-launch output (fp32 tolerance) and, with W = I,
bit for bit against the SpMM.  Prints one JSON line per form.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]

import torch  # noqa: E402

import mgcn  # noqa: E402
from mgcn import _lib as L  # noqa: E402
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
    ap.add_argument("--unroll", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--reduce", default="add")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ei, n = make_er_graph()
    ei = ei.to(dev)
    plan = plan_for(ei, n)
    norm = plan.norm("sm")
    red = L.REDUCE_CODES[args.reduce]
    F = 128
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(n, F, device=dev, generator=g)
    W = (torch.rand(F, F, device=dev, generator=g) * 2 - 1) * (6 / (2 * F)) ** 0.5
    b = (torch.rand(F, device=dev, generator=g) * 0.2 - 0.1)
    rm_a = torch.empty(n, 4, dtype=torch.int32, device=dev)
    rm_b = torch.empty(n, 4, dtype=torch.int32, device=dev)

    def two_launch():
        H, _ = ops.gemm_nn(X, W)
        return ops.spmm_fwd(plan.fwd, norm.w_fwd, H, red, b, True, relu_mask=rm_a)[0]

    def fused():
        return ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, red, b, True, relu_mask=rm_b)

    # numerics
    ya = two_launch()
    yb = fused()
    torch.cuda.synchronize()
    err = ((ya - yb).abs() / (ya.abs() + 1e-3)).max().item()
    mask_eq = bool(torch.equal(ops.make_relu_mask(yb), rm_b))
    eye = torch.eye(F, device=dev)
    zi = ops.spmm_fwd(plan.fwd, norm.w_fwd, X, red, b, True)[0]
    zf = ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, eye, red, b, True)
    bitwise_eye = bool(torch.equal(zi, zf))
    nnz = plan.fwd.nnz
    byt_f = spmm_bytes(n, nnz, F) + 16 * n
    out = {"two_launch_vs_fused_max_rel": err, "mask_matches_Y": mask_eq,
           "W_eye_bitwise": bitwise_eye}
    print(json.dumps(out), flush=True)
    # backward: spmm_bwd + gemm_bwd vs spmm_xw_bwd (mask of the layer below = rm_b)
    dY = torch.randn(n, F, device=dev, generator=g)
    rd = plan.in_cnt if red == L.REDUCE_MEAN else None

    def two_launch_bwd():
        dH = ops.spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, L.REDUCE_SUM)
        return ops.gemm_bwd(X, dH, W, relu_mask=rm_b, row_div=rd)

    def fused_bwd():
        return ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W,
                               relu_mask=rm_b, row_div=rd)

    def fused_bwd_dw():
        return ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, X, W, want_dx=False)

    def two_launch_bwd_dw():
        dH = ops.spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, L.REDUCE_SUM)
        return ops.gemm_bwd(X, dH, W, want_dx=False)

    dWa, dXa, csa = two_launch_bwd()
    dWb, dXb, csb = fused_bwd()
    dWc = fused_bwd_dw()[0]
    torch.cuda.synchronize()
    out = {"bwd_dX_bitwise": bool(torch.equal(dXa, dXb)),
           "bwd_dW_max_rel": ((dWa - dWb).abs().max() / dWa.abs().max()).item(),
           "bwd_dW_only_vs_full_bitwise": bool(torch.equal(dWb, dWc)),
           "bwd_colsum_max_rel": ((csa - csb).abs().max() / csa.abs().max()).item()}
    print(json.dumps(out), flush=True)
    res = {}
    for rep in range(2):
        res.setdefault("two_launch", []).append(time_it(two_launch, args.reps)[0])
        res.setdefault("two_launch_bwd", []).append(time_it(two_launch_bwd, args.reps)[0])
        res.setdefault("two_launch_bwd_dw", []).append(time_it(two_launch_bwd_dw, args.reps)[0])
        for u in args.unroll:
            L.set_option("spmm_xw_unroll", u)
            res.setdefault(f"fused_u{u}", []).append(time_it(fused, args.reps)[0])
            res.setdefault(f"fused_bwd_u{u}", []).append(time_it(fused_bwd, args.reps)[0])
            res.setdefault(f"fused_bwd_dw_u{u}", []).append(time_it(fused_bwd_dw, args.reps)[0])
    for k, v in res.items():
        ms = min(v)
        print(json.dumps({"form": k, "ms": ms, "gbs_fused_bytes": byt_f / ms / 1e6}), flush=True)


if __name__ == "__main__":
    main()
