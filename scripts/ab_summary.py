"""One line per A/B run (scripts/gpu_ab.sh): ms/step and per-kernel averages
of the JSON a workload printed (its last JSON line)."""
import json
import sys


def main():
    path, label = sys.argv[1], sys.argv[2]
    lines = [ln for ln in open(path) if ln.lstrip().startswith("{")]
    if not lines:
        print(label, "no JSON")
        return
    d = json.loads(lines[-1])
    items = [("", d)] if "ms_per_step" in d else [(k, v) for k, v in d.items()
                                                   if isinstance(v, dict) and "ms_per_step" in v]
    for k, v in items:
        kern = {n: round(x["avg_ms"], 4) for n, x in (v.get("kernels") or {}).items()
                if isinstance(x, dict) and "avg_ms" in x}
        print(label, k, round(v["ms_per_step"], 4), kern)


if __name__ == "__main__":
    main()
