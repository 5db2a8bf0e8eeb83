"""Run one dense-GEMM kind a few times at config-2 shape for rocprofv3 PMC
passes: python scripts/prof_gemm_once.py {bwd_relu,bwd_dw,tn,nn_relu,nn} [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from mgcn.ops import gemm_bwd, gemm_nn, gemm_tn, make_relu_mask  # noqa: E402

kind = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
M, F = 1_000_000, 128
X = torch.randn(M, F, device=dev)
dH = torch.randn(M, F, device=dev)
W = torch.randn(F, F, device=dev)
RM = make_relu_mask(torch.randn(M, F, device=dev))
fn = {"bwd_relu": lambda: gemm_bwd(X, dH, W, relu_mask=RM),
      "bwd_dw": lambda: gemm_bwd(X, dH, W, want_dx=False),
      "tn": lambda: gemm_tn(X, dH),
      "nn_relu": lambda: gemm_nn(dH, W, transpose_w=True, relu_mask=RM),
      "nn": lambda: gemm_nn(X, W)}[kind]
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", kind)
