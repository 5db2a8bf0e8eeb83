"""The dense products of a config-5 rank at F = 256 (6.24M local rows):
dW = Z^T dY (mgcn_gemm_tn, bf16x6), H = X W and dX = dH W^T (mgcn_gemm_nn),
timed with HIP events, with algorithmic GB/s and the error against fp64
normalised by |A| |B|.

    python scripts/bench_wide_gemm.py [--rows 6243575 --feat 256]
Prints one JSON line per product.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def norm_err(C, A, B):
    ref = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs()
    return float(((C.double() - ref).abs() / scale.clamp_min(1e-300)).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_243_575)
    ap.add_argument("--feat", type=int, default=256)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="mgcn_set_option before the run (A/B)")
    ap.add_argument("--tn-only", action="store_true", help="time only mgcn_gemm_tn")
    args = ap.parse_args()
    from mgcn import ops
    from mgcn import _lib as L
    for kv in args.opt:
        k, v = kv.split("=")
        L.set_option(k, int(v))
    dev = torch.device("cuda:0")
    M, F = args.rows, args.feat
    g = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(M, F, device=dev, generator=g)
    dY = torch.randn(M, F, device=dev, generator=g)
    W = torch.randn(F, F, device=dev, generator=g) / F ** 0.5
    ops.VENDOR_GEMMS.clear()
    ms = timed(lambda: ops.gemm_tn(Z, dY))
    C = ops.gemm_tn(Z, dY)
    print(json.dumps({"op": "gemm_tn Z^T dY", "K": M, "M": F, "N": F, "ms": ms,
                      "gbs": 8.0 * M * F / ms / 1e6,
                      "tflops_equiv": 2.0 * M * F * F / ms / 1e9,
                      "err": norm_err(C, Z.t(), dY),
                      # bit digest of C: A/B builds of one product compare bit for bit
                      "digest": int(C.view(torch.int32).to(torch.int64).mul_(
                          torch.arange(1, C.numel() + 1, device=dev).view_as(C)).sum())}),
          flush=True)
    if args.tn_only:
        return
    s = 200_000
    for name, fn, chk in [
            ("gemm_nn X W", lambda: ops.gemm_nn(Z, W),
             lambda: norm_err(ops.gemm_nn(Z[:s], W)[0], Z[:s], W)),
            ("gemm_nn dH W^T", lambda: ops.gemm_nn(dY, W, transpose_w=True),
             lambda: norm_err(ops.gemm_nn(dY[:s], W, transpose_w=True)[0], dY[:s], W.t()))]:
        ms = timed(fn)
        print(json.dumps({"op": name, "M": M, "K": F, "N": F, "ms": ms,
                          "gbs": 8.0 * M * F / ms / 1e6,
                          "tflops_equiv": 2.0 * M * F * F / ms / 1e9, "err": chk()}), flush=True)
    print(json.dumps({"vendor_gemms": {str(k): v for k, v in ops.VENDOR_GEMMS.items()}}))


if __name__ == "__main__":
    main()
