"""The F = 256 fused layer kernels (fused_wide.hip) at config 5's rank-local
shape, A/B over their options in one process.

R destination rows with `deg` uniformly random in-edges each from a resident
[T, 256] table (default: one config-5 launch -- 1.56M rows x 11 edges from the
50M-row, 51-GB table), timed with HIP events:
  * spmm_fwd  -- the plain SpMM (the gather ceiling at this table size),
  * xw_fwd_z  -- mgcn_spmm_xw_fwd with Z, bias, ReLU and the 8-word masks,
  * xw_bwd_dx -- the dX-only mgcn_spmm_xw_bwd with the lower layer's mask and
                 column sums (the same view read as the adjoint's),
for every `--opts` setting (mgcn_set_option name=value[,name=value]); each
setting's outputs must equal the first's bit for bit.  Algorithmic bytes as
bench.launch_bytes.  Prints one JSON line.

    python scripts/bench_wide.py [--opts wide_pair=0 wide_pair=3 ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402


def timed(fn, reps):
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
    ap.add_argument("--table", type=int, default=50_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--opts", nargs="+", default=["wide_pair=0", "wide_pair=3"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import build_view
    R, D, T, F = args.rows, args.deg, args.table, 256
    g = torch.Generator(device=dev).manual_seed(0)
    dst = torch.arange(R, device=dev).repeat_interleave(D)
    src = torch.randint(0, T, (R * D,), device=dev, generator=g)
    view = build_view(dst, src, R, T, schedule=False)
    del dst, src
    w = torch.rand(R * D, device=dev, generator=g) * 0.2
    X = torch.empty(T, F, device=dev)
    X.normal_(generator=g)
    W = torch.randn(F, F, device=dev, generator=g) / F ** 0.5
    b = torch.randn(F, device=dev, generator=g) * 0.1
    mask_in = torch.randint(-2 ** 31, 2 ** 31 - 1, (R, 8), dtype=torch.int32, device=dev,
                            generator=g)
    nnz = R * D
    # algorithmic bytes: rowptr + per slot (col, w, gathered row) + outputs
    b_spmm = 8 * (R + 1) + nnz * (8 + 4 * F) + 4 * R * F
    b_fwd_z = b_spmm + 4 * R * F + 32 * R          # + Z, + masks
    b_dx = b_spmm + 32 * R                          # + the lower layer's masks
    Y = torch.empty(R, F, device=dev)
    Z = torch.empty(R, F, device=dev)
    m = torch.empty(R, 8, dtype=torch.int32, device=dev)
    dX = torch.empty(R, F, device=dev)
    cs = torch.zeros(F, device=dev)
    out = {"workload": f"{R} rows x {D} random in-edges from a [{T}, {F}] table "
                       f"({T * F * 4 / 1e9:.1f} GB)", "runs": []}
    t = timed(lambda: ops.spmm_fwd(view, w, X, L.REDUCE_SUM, out=Y), args.reps)
    out["spmm_fwd"] = {"ms": t, "tbs": b_spmm / t / 1e9}
    ref = None
    for opt in args.opts:
        for kv in opt.split(","):
            k, v = kv.split("=")
            L.set_option(k, int(v))

        def fwd():
            ops.spmm_xw_fwd(view, w, X, W, L.REDUCE_SUM, b, True, relu_mask=m, want_z=True,
                            out=Y, z_out=Z)

        def bwd():
            ops.spmm_xw_bwd(view, w, None, X, None, W, relu_mask=mask_in, dx_out=dX,
                            colsum_acc=cs)
        tf = timed(fwd, args.reps)
        tb = timed(bwd, args.reps)
        cs.zero_()
        fwd()
        bwd()
        torch.cuda.synchronize()
        res = [Y.clone(), Z.clone(), m.clone(), dX.clone(), cs.clone()]
        same = cs_rel = None
        if ref is None:
            ref = res
        else:
            # Y, Z, masks, dX bit for bit; the column sums' fold order is
            # the form's own
            same = all(torch.equal(a, c) for a, c in zip(res[:4], ref[:4]))
            cs_rel = float(((res[4] - ref[4]).abs().max() / ref[4].abs().max().clamp_min(1e-30)))
        out["runs"].append({"opts": opt, "xw_fwd_z_ms": tf, "xw_fwd_z_tbs": b_fwd_z / tf / 1e9,
                            "xw_bwd_dx_ms": tb, "xw_bwd_dx_tbs": b_dx / tb / 1e9,
                            "bitwise_same_as_first": same, "colsum_rel_diff": cs_rel})
        print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
