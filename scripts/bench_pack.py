"""The packed exchange's pack of one row chunk: two passes (mgcn_pack_rows_count,
the scan of the counts, mgcn_pack_rows_values) vs the single pass
(mgcn_pack_rows).  Default: a config-5 rank's chunk (1.56M rows x 256,
ReLU'd: about half +0.0); `--config2`: a config-2 chunk at P = 8 (125k x 128).
Prints one JSON line of per-call times (HIP events, median of --reps) and the
rate against the single pass's algorithmic bytes (the rows read once, the
header and values written).

    python scripts/bench_pack.py [--rows 1561000 --F 256 --reps 20]
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
    ap.add_argument("--rows", type=int, default=1_561_000)
    ap.add_argument("--F", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--config2", action="store_true")
    args = ap.parse_args()
    if args.config2:
        args.rows, args.F = 125_000, 128
    from mgcn import ops
    dev = torch.device("cuda:0")
    n, F = args.rows, args.F
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.relu(torch.randn(n, F, device=dev, generator=g))
    head = 2 * n * (F // 32)
    send = torch.empty(head + n * F + 4, dtype=torch.int32, device=dev)
    hdr = send[:head].view(n, 2 * (F // 32))
    vals = send[head:head + n * F]
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)

    def two_pass():
        ops.pack_rows_count(x, hdr, counts)
        t = counts.sum(dtype=torch.int64).view(1)
        offs = torch.cumsum(counts, 0, dtype=torch.int32)
        offs.sub_(counts)
        ops.pack_rows_values(x, offs, hdr, vals)
        return t

    def one_pass():
        ops.pack_rows(x, hdr, vals, total)

    def timeit(fn):
        ts = []
        for _ in range(args.reps + 2):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts[2:])

    res = {"rows": n, "F": F}
    res["two_pass_ms"] = timeit(two_pass)
    ref = send.clone()
    res["one_pass_ms"] = timeit(one_pass)
    res["bitwise"] = bool(torch.equal(ref, send))
    nv = int(total.item())
    res["values_over_dense"] = nv / (n * F)
    alg = 4 * n * F + 4 * head + 4 * nv  # rows read once, header + values written
    res["one_pass_gbs"] = alg / res["one_pass_ms"] / 1e6
    res["two_pass_gbs_same_bytes"] = alg / res["two_pass_ms"] / 1e6
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
