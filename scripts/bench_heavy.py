"""Heavy-row SpMM microbenchmark: star graphs (destination 0 with D in-edges
from random sources over N nodes), forward SpMM time vs D and F, heavy path
vs the lane-group path (threshold raised so the row stays there)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from mgcn import ops  # noqa: E402
from mgcn.graph import build_plan, find_heavy  # noqa: E402
from mgcn._lib import set_option  # noqa: E402
from bench_spmm import time_it  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N = 300_000
    g = torch.Generator().manual_seed(0)
    for F in (32, 128):
        H = torch.randn(N, F, device=dev)
        for D in (512, 2048, 6400):
            src = torch.randint(0, N, (D,), generator=g)
            ei = torch.stack([src, torch.zeros(D, dtype=torch.long)]).to(dev)
            plan = build_plan(ei, N)
            res = {"F": F, "D": D, "n_heavy": plan.fwd.n_heavy}
            set_option("heavy_side_stream", 0)
            for hb in (256, 512, 1024):
                set_option("heavy_block", hb)
                for kb in (64, 160):
                    set_option("heavy_lds_kb", kb)
                    res[f"b{hb}_{kb}k_us"] = round(time_it(
                        lambda: ops.spmm_fwd(plan.fwd, None, H, 0), 20)[0] * 1e3, 1)
            set_option("heavy_side_stream", 1)
            set_option("heavy_lds_kb", 160)
            set_option("heavy_block", 1024)
            find_heavy(plan.fwd, thr=1 << 40)  # lane-group path only
            res["lanegroup_us"] = time_it(lambda: ops.spmm_fwd(plan.fwd, None, H, 0), 20)[0] * 1e3
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
