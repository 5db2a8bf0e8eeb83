"""fp64 references for the GPU tests at the timed workloads' own sizes
(test infrastructure: torch on the GPU in float64).

``A64`` is the aggregation A x (its transpose, and |A|) with per-edge weights
from the C oracle, summed in fp64 with ``index_add_`` over edge chunks; the
|.|-weighted forms give the error bounds the fp32 results are held to
(|y - y64| <= tol * (|A| |x| |W| + ...), the same products with absolute
values).
"""
import torch


class A64:
    """x -> A x (and A^T, |A|) in fp64 on the GPU with the oracle's weights
    (``w`` None: unit weights; ``mean``: divided by max(in-degree, 1))."""

    def __init__(self, ei, w, N, dev, chunk=1 << 21, mean=False):
        self.src = ei[0].to(dev)
        self.dst = ei[1].to(dev)
        if w is None:
            self.w = torch.ones(self.src.numel(), dtype=torch.float64, device=dev)
        else:
            self.w = torch.as_tensor(w).to(dev, torch.float64)
        self.N, self.chunk = N, chunk
        self.inv_cnt = None
        if mean:
            cnt = torch.bincount(self.dst, minlength=N).clamp_(min=1).to(torch.float64)
            self.inv_cnt = 1.0 / cnt

    def apply(self, H, transpose=False, absolute=False):
        if transpose and self.inv_cnt is not None:
            H = H * self.inv_cnt[:, None]
        out = torch.zeros(self.N, H.size(1), dtype=torch.float64, device=H.device)
        for a in range(0, self.src.numel(), self.chunk):
            s, d = self.src[a:a + self.chunk], self.dst[a:a + self.chunk]
            w = self.w[a:a + self.chunk]
            if absolute:
                w = w.abs()
            fr, to = (d, s) if transpose else (s, d)
            out.index_add_(0, to, H[fr] * w[:, None])
        if not transpose and self.inv_cnt is not None:
            out = out * self.inv_cnt[:, None]
        return out


def within(err, bound, tol, atol=1e-6):
    """(ok, worst err / (tol bound + atol)) for |err| <= tol * bound + atol
    elementwise; ``tol`` a number or a tensor broadcast against ``bound``
    (e.g. a per-row rounding bound)."""
    err = err.abs()
    lim = tol * bound + atol
    ok = bool((err <= lim).all())
    worst = float((err / lim).max()) if err.numel() else 0.0
    return ok, worst
