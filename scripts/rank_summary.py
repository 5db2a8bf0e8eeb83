"""One line per config5_rank.py log: ms/step packed and dense, and the
per-kernel averages (used by the A/B calls of DESIGN §7).
    python scripts/rank_summary.py <tag> <log> ..."""
import json
import sys

tag = sys.argv[1]
for f in sys.argv[2:]:
    s = open(f).read()
    d = json.loads(s[s.index('{"workload"'):].strip().splitlines()[0])
    print(tag, f, round(d["ms_per_step"], 3), round(d["ms_per_step_dense_exchange"], 3),
          {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()}, flush=True)
