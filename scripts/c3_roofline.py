"""Config-3 roofline: per kernel (name x grid, so the light-row and the
heavy-row launches of the residual kernel stay apart) the average duration
from a rocprofv3 kernel trace, and from separate --pmc passes the L2 hit rate
(TCC_HIT / (TCC_HIT + TCC_MISS)) and the bytes beyond L2 (FETCH_SIZE, x2 for
16-B-per-lane loads on gfx950, MI355X_MICROARCH.md HBM section; WRITE_SIZE).
Every table of config 3 fits the 256-MB Infinity Cache (the [286k, 32]
activations are 37 MB), so the bytes beyond L2 are served by it, and the bound
to compare with is the guide's Infinity-Cache gather rate (8.6 TB/s for
uniformly random rows of a 38-MB table), not HBM.

    python scripts/c3_roofline.py <trace dir> <pmc dir: hit/miss> <pmc dir: FETCH_SIZE> \\
        <pmc dir: WRITE_SIZE> <out.json>
"""
import csv
import glob
import json
import os
import sys

MALL_GATHER_TBS = 8.6   # MI355X_MICROARCH.md: random rows of a 38-MB table, gathered
HBM_TBS = 8.0
FETCH_FACTOR = 2.0      # FETCH_SIZE reports half the bytes of 16-B-per-lane reads


def short(name):
    n = name
    for pre in ("void ", "mgcn::(anonymous namespace)::", "at::native::", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n.split("(")[0]


def csv_rows(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def durations(d):
    out = {}
    for r in csv_rows(d, "*kernel_trace.csv"):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
        out.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


def counters(d, names):
    per = {}
    for r in csv_rows(d, "*counter_collection.csv"):
        if r["Counter_Name"] not in names:
            continue
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        key = (short(r["Kernel_Name"]), grid, r["Dispatch_Id"])
        per.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for (name, grid, _), v in per.items():
        out.setdefault((name, grid), []).append(v)
    return out


def main():
    trace, hit_d, fetch_d, write_d, dst = sys.argv[1:6]
    dur = durations(trace)
    hits = counters(hit_d, {"TCC_HIT_sum", "TCC_MISS_sum"})
    fetch = counters(fetch_d, {"FETCH_SIZE"})
    write = counters(write_d, {"WRITE_SIZE"})
    # the grid of a launch differs between the trace and the pmc runs only
    # where the launch depends on timing; match on (name, grid), else on name
    res = {}
    for key, ts in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        name, grid = key
        if not any(s in name for s in ("residual", "spmm_heavy", "gemm", "fold", "spmm_kernel")):
            continue
        rec = {"kernel": name, "grid": grid, "dispatches": len(ts),
               "avg_us": sum(ts) / len(ts), "total_us": sum(ts)}
        h = hits.get(key)
        if h:
            hs = sum(x.get("TCC_HIT_sum", 0.0) for x in h)
            ms = sum(x.get("TCC_MISS_sum", 0.0) for x in h)
            rec["l2_hit_rate"] = hs / (hs + ms) if hs + ms else None
        fb = fetch.get(key)
        wb = write.get(key)
        if fb and wb:
            rd = FETCH_FACTOR * 1024.0 * sum(x["FETCH_SIZE"] for x in fb) / len(fb)
            wr = 1024.0 * sum(x["WRITE_SIZE"] for x in wb) / len(wb)
            rec["beyond_l2_read_bytes"] = rd
            rec["write_bytes"] = wr
            gbs = (rd + wr) / (rec["avg_us"] * 1e-6) / 1e9
            rec["beyond_l2_GBs"] = gbs
            rec["frac_of_mall_gather_rate"] = gbs / (MALL_GATHER_TBS * 1e3)
        res["%s|%d" % key] = rec
    out = {"method": __doc__.strip().splitlines()[0], "mall_gather_TBs": MALL_GATHER_TBS,
           "hbm_TBs": HBM_TBS, "fetch_factor": FETCH_FACTOR, "kernels": res}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for k, r in list(res.items())[:14]:
        print(f"{r['kernel'][:44]:44s} grid {r['grid']:7d} n {r['dispatches']:4d} "
              f"{r['avg_us']:7.1f} us  L2 hit {r.get('l2_hit_rate', float('nan')):.2f}  "
              f"beyond-L2 {r.get('beyond_l2_GBs', float('nan')):7.0f} GB/s")


if __name__ == "__main__":
    main()
