"""HBM traffic of the pack kernels from scripts/prof_pack_pmc.sh's two passes:
per dispatch, FETCH_SIZE (x2: gfx950 tallies a 128-B streamed request at 64 B,
MI355X_MICROARCH.md HBM section) and WRITE_SIZE against the single pass's
algorithmic bytes at bench_pack.py's default chunk (1,561,000 x 256, the
values counted from its JSON line).

    python scripts/pack_pmc_summary.py gpurun_out/pkpmc profiles/r06/pack_pmc.json
"""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != counter:
            continue
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"]) * 1024.0
    out = {}
    for (name, _), v in acc.items():
        out.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(src, "pmc1"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "pmc2"), "WRITE_SIZE")
    line = [l for l in open(os.path.join(src, "pmc1.log")) if l.startswith("{")][-1]
    b = json.loads(line)
    n, F = b["rows"], b["F"]
    nv = b["values_over_dense"] * n * F
    rows_b = 4.0 * n * F
    out_b = 4.0 * (2 * n * F // 32) + 4.0 * nv
    res = {"method": __doc__.strip().splitlines()[0], "bench": b, "kernels": {}}
    for short in ("pack_rows_kernel", "pack_count_kernel", "pack_values_kernel"):
        fk = next((v for k, v in fetch.items() if short in k), None)
        wk = next((v for k, v in write.items() if short in k), None)
        if fk is None or wk is None:
            continue
        alg_r = rows_b
        alg_w = {"pack_rows_kernel": out_b, "pack_count_kernel": 4.0 * n * F // 32 + 4.0 * n,
                 "pack_values_kernel": out_b - 4.0 * n * F // 32}[short]
        res["kernels"][short] = {"fetch_bytes_x2": 2 * fk, "write_bytes": wk,
                                 "alg_read_bytes": alg_r, "alg_write_bytes": alg_w,
                                 "read_over_alg": 2 * fk / alg_r, "write_over_alg": wk / alg_w}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main()
