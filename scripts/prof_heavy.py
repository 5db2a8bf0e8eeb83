"""Phase timing of the heavy-row SpMM kernel (workgroup 0) from a library built
with -DMGCN_HEAVY_PROFILE (`make -C meta-gcn_amd/csrc prof`, a separate
libmgcn_prof.so loaded through MGCN_LIB): per batch, the
clock64 span of the fold wave's and the producer waves' work and the barrier
wait, on star graphs (one destination, D sources)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
os.environ.setdefault("MGCN_LIB", os.path.join(ROOT, "meta-gcn_amd", "mgcn", "libmgcn_prof.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mgcn import _lib, ops  # noqa: E402
from mgcn.graph import build_plan  # noqa: E402


def main():
    lib = _lib.load()
    fn = lib.mgcn_debug_heavy_prof
    fn.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    N = 300_000
    g = torch.Generator().manual_seed(0)
    for F, D in ((32, 6400), (128, 6400)):
        H = torch.randn(N, F, device=dev)
        src = torch.randint(0, N, (D,), generator=g)
        ei = torch.stack([src, torch.zeros(D, dtype=torch.long)]).to(dev)
        plan = build_plan(ei, N)
        for _ in range(3):
            ops.spmm_fwd(plan.fwd, None, H, 0)
        torch.cuda.synchronize()
        buf = np.zeros((3, 256, 2), dtype=np.uint64)
        _lib.check(fn(buf.ctypes.data), "prof")
        ts = buf.astype(np.int64)
        nb = int((ts[0, :, 1] > 0).sum())
        t0 = ts[0, 0, 0]
        rows = []
        for b in range(nb):
            rows.append({
                "b": b,
                "fold": int(ts[0, b, 1] - ts[0, b, 0]),
                "prod_first": int(ts[1, b, 1] - ts[1, b, 0]),
                "prod_last": int(ts[2, b, 1] - ts[2, b, 0]),
                "phase": int((ts[0, b + 1, 0] if b + 1 < nb else ts[0, b, 1]) - ts[0, b, 0]),
            })
        tot = int(ts[0, nb - 1, 1] - t0)
        med = {k: int(np.median([r[k] for r in rows])) for k in ("fold", "prod_first", "prod_last", "phase")}
        print(json.dumps({"F": F, "D": D, "batches": nb, "cycles_total": tot, "median": med}), flush=True)


if __name__ == "__main__":
    main()
