"""Phase timing of the fused layer backward (workgroup 0, waves 0 and 7) from
the profiling build (`make -C meta-gcn_amd/csrc xprof`, loaded through
MGCN_LIB): per chunk the cycles of the gather phase, the first barrier, the
dW MFMAs, the dX MFMAs + epilogue, and the second barrier."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
os.environ.setdefault("MGCN_LIB", os.path.join(ROOT, "meta-gcn_amd", "mgcn", "libmgcn_xprof.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mgcn import _lib as L  # noqa: E402
from mgcn import ops  # noqa: E402
from mgcn.graph import plan_for  # noqa: E402
from bench import make_er_graph  # noqa: E402


def main():
    lib = L.load()
    fn = lib.mgcn_debug_xw_prof
    fn.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    ei, n = make_er_graph()
    plan = plan_for(ei.to(dev), n)
    norm = plan.norm("sm")
    F = 128
    X = torch.randn(n, F, device=dev)
    W = torch.randn(F, F, device=dev) * 0.1
    dY = torch.randn(n, F, device=dev)
    rm = ops.make_relu_mask(torch.randn(n, F, device=dev))
    for kind in ("bwd", "bwd_dw"):
        for _ in range(3):
            ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, want_dx=kind == "bwd",
                            relu_mask=rm if kind == "bwd" else None)
        torch.cuda.synchronize()
        buf = np.zeros((2, 64, 6), dtype=np.uint64)
        L.check(fn(buf.ctypes.data), "prof")
        ts = buf.astype(np.int64)
        names = ["gather", "to_barrier1", "dW", "dX+epi", "barrier2"]
        for w in range(2):
            valid = [i for i in range(1, 64) if ts[w, i, 0] > 0 and ts[w, i, 5] > 0]
            d = np.array([[ts[w, i, k + 1] - ts[w, i, k] for k in range(5)] for i in valid])
            tot = np.array([ts[w, i, 5] - ts[w, i, 0] for i in valid])
            print(json.dumps({"kind": kind, "wave": [0, 7][w], "chunks": len(valid),
                              "mean_cycles": dict(zip(names, d.mean(0).round().tolist())),
                              "chunk_cycles": float(tot.mean())}), flush=True)


if __name__ == "__main__":
    main()
