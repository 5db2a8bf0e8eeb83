"""Stage-by-stage GPU vs oracle diagnostic (dinv, edge weights, spmm, gemm)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import numpy as np, torch, mgcn
from mgcn import ops
from mgcn.graph import plan_for
from oracle import oracle as orc
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
N, E, F = 2000, 16000, 128
s = rng.integers(0, N, E); d = rng.integers(0, N, E)
ei = np.stack([np.concatenate([s, d, np.arange(N)]), np.concatenate([d, s, np.arange(N)])])
x = rng.standard_normal((N, F)).astype(np.float32)
eit = torch.from_numpy(ei).to(dev)
plan = plan_for(eit, N)
norm = plan.norm('sm')
deg_o, dinv_o, norm_o = orc.degnorm(ei, N, method='sm')
print("deg equal:", np.array_equal(norm.deg.cpu().numpy(), deg_o))
dv = norm.dinv.cpu().numpy()
print("dinv equal:", np.array_equal(dv, dinv_o), "ndiff", int((dv != dinv_o).sum()))
i = np.nonzero(dv != dinv_o)[0][:5]
print(" examples deg", deg_o[i], "gpu", dv[i], "cpu", dinv_o[i])
# per-edge weights in COO order
w = torch.empty_like(norm.w_fwd); w[plan.fwd.eid.long()] = norm.w_fwd
wn = w.cpu().numpy()
print("w_fwd (COO) equal:", np.array_equal(wn, norm_o), "ndiff", int((wn != norm_o).sum()))
# spmm with oracle weights injected
wo = torch.from_numpy(norm_o).to(dev)[plan.fwd.eid.long()].contiguous()
Y, _ = ops.spmm_fwd(plan.fwd, wo, torch.from_numpy(x).to(dev), 0)
y_ref, _ = orc.aggr_fwd(ei, x, norm_o, "add")
yn = Y.cpu().numpy()
print("spmm (same weights) equal:", np.array_equal(yn, y_ref), "ndiff", int((yn != y_ref).sum()))
# unweighted spmm
Y2, _ = ops.spmm_fwd(plan.fwd, None, torch.from_numpy(x).to(dev), 0)
y2, _ = orc.aggr_fwd(ei, x, None, "add")
print("spmm unweighted equal:", np.array_equal(Y2.cpu().numpy(), y2))
# gemm with identity
xt = torch.from_numpy(x).to(dev)
h = xt @ torch.eye(F, device=dev)
print("x @ I == x:", torch.equal(h, xt))
# torch GPU sqrt/div vs CPU
dg = torch.from_numpy(deg_o).to(dev)
r = (1.0 / torch.sqrt(dg)).cpu().numpy()
print("torch gpu 1/sqrt == cpu:", np.array_equal(r, dinv_o))
