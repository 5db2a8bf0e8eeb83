"""Timeline of one config-3 training step from a rocprofv3 kernel trace
(scripts/prof_config3.sh / kstats_c3.sh write one): the last full step's
dispatches in start order with their queue, duration and the idle gap before
each, then the step's span, the time some kernel was running (union of the
dispatch intervals), and the per-kernel-name totals on the critical queue.

    python scripts/c3_timeline.py <dir with *kernel_trace.csv>
"""
import argparse
import csv
import glob
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for r in csv.DictReader(open(f[0])):
        rows.append({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]),
                     "end": int(r["End_Timestamp"]),
                     "queue": r.get("Queue_Id") or r.get("Stream_Id") or "?"})
    rows.sort(key=lambda x: x["start"])
    return rows


def short(name):
    n = name
    for pre in ("void ", "mgcn::(anonymous namespace)::", "at::native::", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    args = ap.parse_args()
    rows = load(args.dir)
    # the steady-state step: the shortest period L with which the dispatch
    # names repeat at the end of the trace
    # (trailing kernels after the last step -- the script's own bookkeeping --
    # are skipped: the window may end up to 64 dispatches before the trace)
    names = [r["name"] for r in rows]
    found = None
    for tail in range(0, 64):
        e = len(names) - tail
        L = next((n for n in range(5, e // 3 + 1)
                  if names[e - n:e] == names[e - 2 * n:e - n] == names[e - 3 * n:e - 2 * n]), None)
        if L is not None:
            found = (e - L, e)
            break
    if found is None:
        sys.exit("no repeating step found")
    a, b = found
    step = rows[a:b]
    t0 = step[0]["start"]
    span = step[-1]["end"] - t0
    busy, cur_s, cur_e = 0, None, None
    for r in sorted(step, key=lambda x: x["start"]):
        if cur_e is None or r["start"] > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = r["start"], r["end"]
        else:
            cur_e = max(cur_e, r["end"])
    busy += cur_e - cur_s
    print(f"step: {len(step)} dispatches, span {span / 1e3:.1f} us, some kernel running "
          f"{busy / 1e3:.1f} us ({100.0 * busy / span:.0f} %)")
    last_end = {}
    tot = {}
    for r in step:
        q = r["queue"]
        gap = r["start"] - last_end.get(q, r["start"])
        last_end[q] = r["end"]
        d = r["end"] - r["start"]
        tot.setdefault(short(r["name"]), [0, 0])
        tot[short(r["name"])][0] += 1
        tot[short(r["name"])][1] += d
        print(f"{(r['start'] - t0) / 1e3:9.1f} q{q:>3} {d / 1e3:7.1f} us  gap {gap / 1e3:6.1f}  "
              f"{short(r['name'])}")
    print("\nper kernel: calls, total us")
    for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:4d} {d / 1e3:9.1f}  {k}")


if __name__ == "__main__":
    main()
