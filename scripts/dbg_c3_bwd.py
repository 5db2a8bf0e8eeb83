"""Debug: config-3 residual stack backward at full size vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import numpy as np
import torch
from bench import batch_graphs, make_botnet_graph
from oracle import oracle as orc
from mgcn import ops
from mgcn import _lib as L
from mgcn.graph import plan_for

dev = torch.device("cuda:0")
g1, n1, _ = make_botnet_graph(seed=0)
g2, n2, _ = make_botnet_graph(seed=1)
ei, N = batch_graphs([(g1, n1), (g2, n2)])
deg = torch.bincount(ei[0], minlength=N).float()
ein = ei.numpy()
outdeg = np.bincount(ein[0], minlength=N)
indeg = np.bincount(ein[1], minlength=N)
wf, wb, rs = orc.edge_factors(ein, N, "sm", deg=deg.numpy())
rng = np.random.default_rng(32)
F = 32
x = rng.standard_normal((N, F)).astype(np.float32)
dZ = rng.standard_normal((N, F)).astype(np.float32)
eid = ei.to(dev)
plan = plan_for(eid, N)
norm = plan.norm("sm", deg=deg.to(dev))
print("heavy fwd", plan.fwd.n_heavy, plan.fwd.n_giant, "bwd", plan.bwd.n_heavy, plan.bwd.n_giant)
eye, zero = torch.eye(F, device=dev), torch.zeros(F, F, device=dev)
agg, _ = orc.aggr_fwd(ein, x, wf, "add", None, True)
for relu2 in (True, False):
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    Z = ops._ResidualLayerFused.apply(xt, plan, norm, L.REDUCE_SUM, True, relu2, eye, None, zero, None)
    Z.backward(torch.from_numpy(dZ).to(dev))
    torch.cuda.synchronize()
    print("layer fwd equal:", np.array_equal(Z.detach().cpu().numpy(), agg))
    g = np.where(agg > 0, dZ, 0) if relu2 else dZ
    dH, _ = orc.aggr_bwd(ein, g, wb, rs, "add", agg, True, None)
    got = xt.grad.cpu().numpy()
    bad = np.any(got != dH, axis=1)
    print("relu2", relu2, "single layer dX mismatching rows:", int(bad.sum()), "of", N,
          "max abs", float(np.abs(got - dH).max()))
    if bad.any():
        idx = np.nonzero(bad)[0]
        print("  outdeg of bad rows: min", outdeg[idx].min(), "max", outdeg[idx].max(),
              "median", np.median(outdeg[idx]), "; rows with outdeg>128:", int((outdeg > 128).sum()),
              "bad among them", int(bad[outdeg > 128].sum()))
        print("  first bad", idx[:10], outdeg[idx[:10]])
# two-layer stack vs layer by layer
for nl in (2, 3):
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    params = [(eye.clone(), None, zero.clone(), None) for _ in range(nl)]
    y = ops.residual_stack(xt, plan, norm, "add", [True] * nl, [True] * (nl - 1) + [False], params)
    y.backward(torch.from_numpy(dZ).to(dev))
    torch.cuda.synchronize()
    h, outs = x, []
    for _ in range(nl):
        h, _ = orc.aggr_fwd(ein, h, wf, "add", None, True)
        outs.append(h)
    print("stack", nl, "fwd equal", np.array_equal(y.detach().cpu().numpy(), outs[-1]))
    gg = dZ
    for l in range(nl - 1, -1, -1):
        gg, _ = orc.aggr_bwd(ein, gg, wb, rs, "add", outs[l], True, None)
    got = xt.grad.cpu().numpy()
    bad = np.any(got != gg, axis=1)
    print("stack", nl, "dX mismatching rows", int(bad.sum()), "max abs", float(np.abs(got - gg).max()))
