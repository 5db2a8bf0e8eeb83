"""Time mgcn_gemm_bwd (config-2 shape) under the experiment builds listed in
argv (each a libmgcn.so path; MGCN_LIB selects it in a child process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd"), os.path.join(ROOT, "scripts")]
import torch
from mgcn.ops import gemm_bwd, make_relu_mask, gemm_tn, gemm_nn
from bench_spmm import time_it
dev = torch.device("cuda:0")
M, F = 1_000_000, 128
X = torch.randn(M, F, device=dev); dH = torch.randn(M, F, device=dev)
W = torch.randn(F, F, device=dev); RM = make_relu_mask(torch.randn(M, F, device=dev))
out = {"lib": os.environ["MGCN_LIB"], "opts": os.environ.get("MGCN_OPTIONS", "")}
for name, fn in [("relu", lambda: gemm_bwd(X, dH, W, relu_mask=RM)),
                 ("dw_only", lambda: gemm_bwd(X, dH, W, want_dx=False)),
                 ("tn", lambda: gemm_tn(X, dH)),
                 ("nn_relu", lambda: gemm_nn(dH, W, transpose_w=True, relu_mask=RM))]:
    med, mn = time_it(fn, 20)
    out[name] = round(med, 4); out[name + "_min"] = round(mn, 4)
print(json.dumps(out), flush=True)
'''.replace("ROOT", repr(ROOT))

for spec in sys.argv[1:]:
    lib, _, opts = spec.partition(":")
    env = dict(os.environ, MGCN_LIB=os.path.abspath(lib), MGCN_OPTIONS=opts)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=300)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
    if r.returncode:
        sys.exit(r.returncode)
