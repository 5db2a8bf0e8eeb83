"""Debug: config-3 residual stack backward at full size vs the oracle, under
libmgcn option variants (side stream, fused mask pass, fences)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import numpy as np
import torch
import mgcn
from bench import batch_graphs, make_botnet_graph
from oracle import oracle as orc
from mgcn import ops
from mgcn.graph import plan_for

dev = torch.device("cuda:0")
g1, n1, _ = make_botnet_graph(seed=0)
g2, n2, _ = make_botnet_graph(seed=1)
ei, N = batch_graphs([(g1, n1), (g2, n2)])
deg = torch.bincount(ei[0], minlength=N).float()
ein = ei.numpy()
wf, wb, rs = orc.edge_factors(ein, N, "sm", deg=deg.numpy())
rng = np.random.default_rng(32)
F = 32
x = rng.standard_normal((N, F)).astype(np.float32)
dZ = rng.standard_normal((N, F)).astype(np.float32)
plan = plan_for(ei.to(dev), N)
norm = plan.norm("sm", deg=deg.to(dev))
eye, zero = torch.eye(F, device=dev), torch.zeros(F, F, device=dev)
nl = 3
h, outs = x, []
for _ in range(nl):
    h, _ = orc.aggr_fwd(ein, h, wf, "add", None, True)
    outs.append(h)
gg = dZ
grads = []
for l in range(nl - 1, -1, -1):
    gg, _ = orc.aggr_bwd(ein, gg, wb, rs, "add", outs[l], True, None)
    grads.append(gg)


def run(tag):
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    params = [(eye.clone(), None, zero.clone(), None) for _ in range(nl)]
    y = ops.residual_stack(xt, plan, norm, "add", [True] * nl, [True] * (nl - 1) + [False], params)
    y.backward(torch.from_numpy(dZ).to(dev))
    torch.cuda.synchronize()
    got = xt.grad.cpu().numpy()
    bad = np.any(got != gg, axis=1)
    print(tag, "fwd equal", np.array_equal(y.detach().cpu().numpy(), outs[-1]),
          "dX bad rows", int(bad.sum()), "max abs", float(np.abs(got - gg).max()), flush=True)


run("default")
run("default again")
mgcn.set_option("heavy_side_fence", 1); run("fence"); mgcn.set_option("heavy_side_fence", 0)
mgcn.set_option("residual_fused_mask", 0); run("unfused mask"); mgcn.set_option("residual_fused_mask", 1)
mgcn.set_option("heavy_side_stream", 0); run("no side stream"); mgcn.set_option("heavy_side_stream", 1)

