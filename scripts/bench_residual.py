"""Microbenchmark of one config-3 residual layer (tuning aid): the fused
residual-layer kernels (mgcn_residual_layer_fwd / _bwd) against the
two-launch layer (x @ [W | Wr^T], SpMM, join) on the botnet-shaped batch.

    python scripts/bench_residual.py [--reps 20]      (MGCN_LIB selects a build)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from bench import batch_graphs, make_botnet_graph  # noqa: E402


def time_it(fn, reps):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    fn()
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from mgcn import _lib as L
    from mgcn import ops
    from mgcn.graph import plan_for
    dev = torch.device("cuda:0")
    g1, n1, _ = make_botnet_graph(seed=0)
    g2, n2, _ = make_botnet_graph(seed=1)
    ei, N = batch_graphs([(g1, n1), (g2, n2)])
    ei = ei.to(dev)
    plan = plan_for(ei, N)
    deg = torch.bincount(ei[0], minlength=N).float()
    norm = plan.norm("sm", deg=deg)
    F = 32
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, F, device=dev, generator=g).requires_grad_(True)
    ps = [(torch.randn(F, F, device=dev, generator=g) * 0.2).requires_grad_(True), None,
          (torch.randn(F, F, device=dev, generator=g) * 0.2).requires_grad_(True),
          (torch.randn(F, device=dev, generator=g) * 0.1).requires_grad_(True)]
    dZ = torch.randn(N, F, device=dev, generator=g)
    out = {"lib": os.environ.get("MGCN_LIB", "default"), "nodes": N, "nnz": plan.nnz,
           "heavy_fwd": plan.fwd.n_heavy, "giant_fwd": plan.fwd.n_giant}
    for name, fn in (("fused", ops._ResidualLayerFused), ("two_launch", ops._ResidualGCNLayer)):
        def fwd(fn=fn):
            with torch.no_grad():
                fn.apply(x, plan, norm, L.REDUCE_SUM, True, True, *ps)
        Z = fn.apply(x, plan, norm, L.REDUCE_SUM, True, True, *ps)

        def bwd(Z=Z):
            torch.autograd.grad(Z, [x, ps[0], ps[2], ps[3]], dZ, retain_graph=True)
        out[name + "_fwd_ms"] = time_it(fwd, args.reps)
        out[name + "_bwd_ms"] = time_it(bwd, args.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
