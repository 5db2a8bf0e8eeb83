"""Microbenchmark of the feature-transform GEMMs at config-2 shape (M = 1M,
F = 128), per product arithmetic (gemm_precision 0 = f32 MFMA, 1 = bf16x6),
with the error against an fp64 product normalised by |A| |B| (the scale of
an fp32 rounding bound)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from mgcn._lib import set_option  # noqa: E402
from mgcn.ops import gemm_bwd, gemm_nn, gemm_tn, make_relu_mask  # noqa: E402
from bench_spmm import time_it  # noqa: E402


def norm_err(C, A, B):
    """max |C - A B| / (|A| |B|) elementwise, products in fp64."""
    ref = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs()
    return float(((C.double() - ref).abs() / scale.clamp_min(1e-300)).max())


def main():
    dev = torch.device("cuda:0")
    M, F = 1_000_000, 128
    X = torch.randn(M, F, device=dev)
    dH = torch.randn(M, F, device=dev)
    Z = torch.randn(M, F, device=dev)
    W = torch.randn(F, F, device=dev)
    RM = make_relu_mask(Z)
    fl = 2.0 * M * F * F
    s = 65536
    for prec in (0, 1):
        set_option("gemm_precision", prec)
        errs = {"nn": norm_err(gemm_nn(X[:s], W)[0], X[:s], W),
                "tn": norm_err(gemm_tn(X[:s], dH[:s]), X[:s].t(), dH[:s])}
        for name, fn in [("gemm_nn", lambda: gemm_nn(X, W)),
                         ("gemm_nn_t_relu", lambda: gemm_nn(dH, W, transpose_w=True, relu_mask=RM)),
                         ("gemm_tn", lambda: gemm_tn(X, dH))]:
            med, mn = time_it(fn, 20)
            print(json.dumps({"kernel": name, "precision": ["f32", "bf16x6"][prec], "ms": med,
                              "min_ms": mn, "tflops": fl / med / 1e9,
                              "norm_err": errs["tn" if name == "gemm_tn" else "nn"]}), flush=True)
    set_option("gemm_precision", 1)
    # fused adjoints: dW + dX (+ ReLU / bias colsum) from one pass; dW alone
    for name, fn in [("gemm_bwd_relu", lambda: gemm_bwd(X, dH, W, relu_mask=RM)),
                     ("gemm_bwd_dw_only", lambda: gemm_bwd(X, dH, W, want_dx=False))]:
        med, mn = time_it(fn, 20)
        by = (12 * F + 16) * M if "relu" in name else 8 * F * M
        print(json.dumps({"kernel": name, "precision": "bf16x6", "ms": med, "min_ms": mn,
                          "gbs": by / med / 1e6}), flush=True)
    errs = {"nn": norm_err(torch.matmul(X[:s], W), X[:s], W),
            "tn": norm_err(torch.matmul(X[:s].t(), dH[:s]), X[:s].t(), dH[:s])}
    for name, fn in [("torch_mm", lambda: torch.matmul(X, W)),
                     ("torch_tn", lambda: torch.matmul(X.t(), dH))]:
        med, mn = time_it(fn, 20)
        print(json.dumps({"kernel": name, "ms": med, "min_ms": mn, "tflops": fl / med / 1e9,
                          "norm_err": errs["tn" if name == "torch_tn" else "nn"]}), flush=True)


if __name__ == "__main__":
    main()
