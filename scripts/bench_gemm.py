"""Microbenchmark of the feature-transform GEMMs at config-2 shape (M = 1M, F = 128)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from mgcn._lib import set_option  # noqa: E402
from mgcn.ops import gemm_nn, gemm_tn  # noqa: E402
from bench_spmm import time_it  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, F = 1_000_000, 128
    X = torch.randn(M, F, device=dev)
    dH = torch.randn(M, F, device=dev)
    Z = torch.randn(M, F, device=dev)
    W = torch.randn(F, F, device=dev)
    fl = 2.0 * M * F * F
    for name, fn in [("gemm_nn", lambda: gemm_nn(X, W)),
                     ("gemm_nn_t_relu", lambda: gemm_nn(dH, W, transpose_w=True, Z=Z)),
                     ("gemm_tn", lambda: gemm_tn(X, dH)),
                     ("gemm_tn_v1", lambda: gemm_tn(X, dH)),
                     ("gemm_tn_v2", lambda: gemm_tn(X, dH)),
                     ("torch_mm", lambda: torch.matmul(X, W)),
                     ("torch_tn", lambda: torch.matmul(X.t(), dH))]:
        set_option("gemm_tn_variant", int(name[-1]) if name.startswith("gemm_tn_v") else 0)
        med, mn = time_it(fn, 20)
        print(json.dumps({"kernel": name, "ms": med, "min_ms": mn, "tflops": fl / med / 1e9}),
              flush=True)


if __name__ == "__main__":
    main()
