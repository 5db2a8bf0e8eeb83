"""Run one fused layer kernel a few times on the config-2 graph for
rocprofv3 PMC passes:
    python scripts/prof_fused_once.py {fwd,fwd_z,bwd,bwd_dw,bwd_dx,gemm_dw,gemm_dw_cs,spmm} [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from mgcn import _lib as L  # noqa: E402
from mgcn import ops  # noqa: E402
from mgcn.graph import plan_for  # noqa: E402
from bench import make_er_graph  # noqa: E402

kind = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
ei, n = make_er_graph()
plan = plan_for(ei.to(dev), n)
norm = plan.norm("sm")
F = 128
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(n, F, device=dev, generator=g)
W = torch.randn(F, F, device=dev, generator=g) * 0.1
b = torch.randn(F, device=dev, generator=g) * 0.1
dY = torch.randn(n, F, device=dev, generator=g)
rm = ops.make_relu_mask(torch.randn(n, F, device=dev, generator=g))
rmS = torch.randn(n, F, device=dev, generator=g)
fn = {"fwd": lambda: ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, b, True,
                                     relu_mask=rm),
      "bwd": lambda: ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, relu_mask=rm),
      "bwd_dw": lambda: ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, X, W, want_dx=False),
      "fwd_z": lambda: ops.spmm_xw_fwd(plan.fwd, norm.w_fwd, X, W, L.REDUCE_SUM, b, True,
                                       relu_mask=rm, want_z=True),
      "bwd_dx": lambda: ops.spmm_xw_bwd(plan.bwd, norm.w_bwd, None, dY, None, W, relu_mask=rm),
      "gemm_dw": lambda: ops.gemm_bwd(X, dY, W, want_dx=False, dh_colsum=True),
      # the bottom layer's dW = Z^T dY + the top layer's bias gradient (column
      # sums of a third stream, mgcn_gemm_bwd_dw_cs) -- the bench step's form
      "gemm_dw_cs": lambda: ops.dw_pass_cs(X, dY, rmS),
      "spmm": lambda: ops.spmm_bwd(plan.bwd, norm.w_bwd, None, dY, L.REDUCE_SUM)}[kind]
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", kind)
