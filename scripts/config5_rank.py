"""Config 5's sharded step, one rank's share timed on ONE MI355X
(BASELINE.json configs[4]: N = 50M nodes, 250M pairs symmetrised to
E = 500M edges + 50M self-loops, F = 256, 8 GPUs, destination-range shards).

The rank-local compute of the P-way sharded step is what one GPU of the
8-GPU run executes between its exchanges: rank r of P builds its shard
(mgcn.dist.build_shard(emulate=(r, P)): the edges into and out of its
destination range, columns remapped to the exchange table, the same norms),
and runs the product step -- ShardedGCN: 3 GCN layers 256 -> 256 ('sm',
'add', bias, ReLU between), forward + backward to every weight and bias --
with the exchange tables resident (the replicated input in the exchange
layout; the layer tables written only at this rank's rows; no RCCL).  So
the measured time is the step minus its all-gathers; the script also
reports per-kernel HIP-event times and algorithmic GB/s (bench.KernelTimer
accounting), and the predicted P = 1 / 2 / 4 / 8 curve from the measured
rank-local time (which scales with rows / P) and the all-gathers' bytes at
the xGMI link rate.

    python scripts/config5_rank.py [--world 8 --rank 0 --steps 3 --warmup 1]
Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from bench import KernelTimer, launch_bytes  # noqa: E402

XGMI_LINK_GBS = 153.0  # per link and direction
HBM_WRITE_TBS = 5.0    # streaming write rate charged for the received words (upper-bound term)


def _global_ids(t, sh):
    """exchange-table positions -> global node ids (mgcn.dist.table_positions
    inverted): t = c P cr + k cr + (i - c cr)."""
    P, cr = sh.world, sh.chunk_rows
    c = torch.div(t, P * cr, rounding_mode="floor")
    k = torch.div(t - c * P * cr, cr, rounding_mode="floor")
    i = c * cr + (t - c * P * cr - k * cr)
    b = torch.tensor(sh.bounds, dtype=torch.int64, device=t.device)
    return b[k] + i


def receive_load(step, args, N, F, L, fused, packed, ratio, dev):
    """The packed step timed beside a stand-in for the writes a real rank's
    RCCL receive makes into its HBM while it computes: per step, the received
    (P - 1) / P of every exchanged table (packed ones at `ratio`) written by
    `--recv-load-wgs` workgroups on a side stream (libmgcn_exp.so's
    mgcn_exp_hbm_write_load; a collective runs in a few dozen workgroups).
    Returns the main stream's ms per step under that load, the side stream's,
    and the load's time alone."""
    from mgcn import _lib as L_
    from mgcn import dist as mdist
    lib = L_.load()
    fn = getattr(lib, "mgcn_exp_hbm_%s_load" % args.recv_load_kind, None)
    if fn is None:
        sys.exit("--recv-load-wgs needs MGCN_LIB=<libmgcn_exp.so> (make -C meta-gcn_amd/csrc exp)")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                   ctypes.c_void_p]
    fn.restype = ctypes.c_int
    P = args.world
    tables = (2 * (L - 1)) if fused else (2 * L)
    packed_tables = (2 * L - 3) if packed else 0
    eff = tables - packed_tables + packed_tables * ratio
    per_step = int(eff * 4.0 * N * F * (P - 1) / P) // 16 * 16
    buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(device=dev)
    mdist.set_pack_exchange(True)

    def load(n_steps):
        with torch.cuda.stream(side):
            L_.check(fn(buf.data_ptr(), buf.numel(), per_step * n_steps, args.recv_load_wgs,
                        side.cuda_stream), "mgcn_exp_hbm_write_load")

    # the load alone
    torch.cuda.synchronize()
    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a0.record(side)
    load(args.steps)
    a1.record(side)
    torch.cuda.synchronize()
    alone = a0.elapsed_time(a1) / args.steps
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    side.wait_stream(main)
    e0.record(main)
    s0.record(side)
    load(args.steps)  # the whole timed region's receive writes, from its start
    s1.record(side)
    for _ in range(args.steps):
        step()
    e1.record(main)
    torch.cuda.synchronize()
    # per-kernel times of one more step beside the load (HIP events)
    from mgcn import ops
    timer = KernelTimer()
    side.wait_stream(main)
    load(2)  # (twice the step's bytes: the load surely spans the whole step)
    ops.set_kernel_timer(timer)
    step()
    torch.cuda.synchronize()
    ops.set_kernel_timer(None)
    kern = {}
    for name, k in timer.summary().items():
        k.pop("sizes")
        kern[name] = {kk: round(v, 4) if isinstance(v, float) else v for kk, v in k.items()}
    del buf
    return {"workgroups": args.recv_load_wgs, "kind": args.recv_load_kind,
            "bytes_per_step": per_step,
            "kernels_under_load": kern,
            "alone_ms_per_step": alone, "alone_TBs": per_step / (alone * 1e-3) / 1e12,
            "ms_per_step_under_load": e0.elapsed_time(e1) / args.steps,
            "side_ms_per_step_under_load": s0.elapsed_time(s1) / args.steps,
            "note": "main stream: the packed rank step (P segments aliased, as in ms_per_step); "
                    "side stream: the step's received bytes written by a workgroup-limited "
                    "kernel (16-B nt stores), a stand-in for RCCL's receive into HBM; the "
                    "xGMI transfer itself is not modelled here"}


def sample_check(model, Xt, odeg, n_rows, F, tol=1e-5):
    """Config-5 parity at its own size (gcn_base_models.py:201, 223-241):
    windows of ``n_rows`` destination rows of the rank's forward layer
    (mgcn_spmm_xw_fwd on the fused wide kernel: Y = relu((A X) W + b)) and of
    its dX-only adjoint (dX = (A^T dY) W^T) against a host-independent fp64
    restatement -- the symmetric norm rebuilt from the global out-degrees in
    fp64, the table positions mapped back to global ids, the sums in fp64 --
    within tol x the |.| bound (|A| |X| |W| + |b|)."""
    from mgcn import _lib as L
    from mgcn import ops
    sh = model.shard
    W0, b0, W1 = model.W[0].detach(), model.b[0].detach(), model.W[1].detach()
    dinv = odeg.to(torch.float64).pow(-0.5)
    dinv[torch.isinf(dinv)] = 0.0
    res = {"rows_per_window": n_rows, "windows": [], "tol": tol}
    worst = 0.0
    for a in (0, sh.rows // 2, max(sh.rows - n_rows, 0)):
        e = min(a + n_rows, sh.rows)
        for kind, view, w in (("fwd", sh.fwd, sh.w_fwd), ("dx", sh.bwd, sh.w_bwd)):
            v = view.rows(a, e)
            rp = v.rowptr.to(torch.int64)
            s0, s1 = int(rp[0]), int(rp[-1])
            cols = v.col[s0:s1].to(torch.int64)
            deg = (rp[1:] - rp[:-1])
            row_of = torch.repeat_interleave(torch.arange(e - a, device=cols.device), deg)
            me = sh.lo + a + row_of            # this rank's node of each slot
            other = _global_ids(cols, sh)      # the gathered node
            w64 = dinv[me] * dinv[other]
            g = Xt[cols].to(torch.float64)
            agg = torch.zeros(e - a, F, dtype=torch.float64, device=g.device)
            agg.index_add_(0, row_of, g * w64[:, None])
            absg = torch.zeros_like(agg).index_add_(0, row_of, g.abs() * w64.abs()[:, None])
            if kind == "fwd":
                y = ops.spmm_xw_fwd(v, w, Xt, W0, L.REDUCE_SUM, b0, True)
                ref = torch.relu(agg @ W0.double() + b0.double())
                bound = absg @ W0.double().abs() + b0.double().abs()
            else:
                y = ops.spmm_xw_bwd(v, w, None, Xt, None, W1)[1]
                ref = agg @ W1.double().t()
                bound = absg @ W1.double().abs().t()
            err = (y.double() - ref).abs()
            ratio = float((err / (tol * bound + 1e-30)).max())
            worst = max(worst, ratio)
            res["windows"].append({"kind": kind, "rows": [sh.lo + a, sh.lo + e],
                                   "slots": s1 - s0, "max_err_over_bound": ratio,
                                   "max_abs_err": float(err.max())})
    res["worst"] = worst
    res["ok"] = worst <= 1.0
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000_000)
    ap.add_argument("--pairs", type=int, default=250_000_000)
    ap.add_argument("--feat", type=int, default=256)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-fused", action="store_true")
    ap.add_argument("--dense-exchange", action="store_true",
                    help="no zero-skipping: the ReLU'd tables travel dense")
    ap.add_argument("--check-rows", type=int, default=1024,
                    help="rows per window of the sampled fp64 check (0: no check)")
    ap.add_argument("--recv-load-kind", choices=["write", "copy"], default="write",
                    help="the stand-in writes the received bytes (write) or also reads as many "
                         "(copy: a rank's all-gather reads its own segment for every peer)")
    ap.add_argument("--recv-load-wgs", type=int, default=0,
                    help="also time the packed step beside a stand-in for a real rank's RCCL "
                         "receive: this many workgroups writing the step's received bytes into "
                         "HBM on a side stream (needs MGCN_LIB=<libmgcn_exp.so>: "
                         "mgcn_exp_hbm_write_load)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from mgcn import ops
    from mgcn import dist as mdist
    from mgcn.dist import ShardedGCN
    N, P, F, L = args.nodes, args.pairs, args.feat, args.layers
    t0 = time.perf_counter()
    g = torch.Generator(device=dev).manual_seed(0)
    s = torch.randint(0, N, (P,), device=dev, generator=g)
    d = torch.randint(0, N, (P,), device=dev, generator=g)
    loops = torch.arange(N, device=dev)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    del s, d, loops
    gw = torch.Generator().manual_seed(2)
    gb = torch.Generator().manual_seed(3)
    a = (6.0 / (F + F)) ** 0.5
    Ws = [torch.rand(F, F, generator=gw) * (2 * a) - a for _ in range(L)]
    bs = [torch.rand(F, generator=gb) * 0.2 - 0.1 for _ in range(L)]
    model = ShardedGCN(ei, N, Ws, bs, device=dev, chunks=args.chunks, fused=not args.no_fused,
                       emulate=(args.rank, args.world))
    sh = model.shard
    nnz = int(ei.size(1))
    # out-degrees for the fp64 restatement of the norms (sampled check)
    odeg = torch.bincount(ei[0], minlength=N) if args.check_rows else None
    del ei
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    prep_s = time.perf_counter() - t0
    # the replicated input in the exchange layout and this rank's upstream gradient
    Xt = torch.randn(sh.table_rows, F, device=dev, generator=g)
    dYl = torch.randn(sh.rows, F, device=dev, generator=g)
    step = model.step_fn(None, None, X_table=Xt, dY_local=dYl)

    def run(packed):
        sh._tables = None  # the other run's persistent dense tables
        torch.cuda.empty_cache()
        mdist.set_pack_exchange(packed)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        mdist.STATS.update(dense_words=0, sent_words=0)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        st = dict(mdist.STATS)
        return ms, (st["sent_words"] / st["dense_words"] if st["dense_words"] else 1.0)

    # the step with every table kept dense (the rank-local compute alone), then
    # with the zero-skipping exchange: the pack of every ReLU'd table, the
    # receive-side write of all P segments of it (a real rank's RCCL receive),
    # and the next layer gathering the packed segments in place (round 6; no
    # unpack pass -- MGCN_PACK_INPLACE=0 restores the round-5 unpack)
    ms_dense, _ = run(False)
    packed = model.fused and not args.dense_exchange
    ms, ratio = run(True) if packed else (ms_dense, 1.0)
    recv_load = None
    if args.recv_load_wgs > 0:
        recv_load = receive_load(step, args, N, F, L, model.fused, packed, ratio, dev)
    timer = KernelTimer()
    ops.set_kernel_timer(timer)
    step()
    torch.cuda.synchronize()
    ops.set_kernel_timer(None)
    kern = {}
    for name, k in timer.summary().items():
        byts = 0.0
        for r, e in k.pop("sizes"):
            b, _ = launch_bytes(name, r or 0, e or 0, F)
            byts += b or 0.0
        t = k["total_ms"] * 1e-3
        kern[name] = dict(k, bytes=byts / k["launches"], gbs=byts / t / 1e9 if t else None)
    kernel_ms = sum(k["total_ms"] for k in kern.values())
    check = sample_check(model, Xt, odeg, args.check_rows, F) if args.check_rows else None
    del odeg
    # predicted curve.  Local work of a rank at P: the measured step (its
    # compute, the pack, the in-place packed gathers) scales with its rows
    # (8 / P of rank 0's here).  Each exchanged table is an all-gather of
    # [N, F] fp32, a rank receiving (P - 1) / P of it over P - 1 xGMI links;
    # packed tables at `ratio` of their words.  The received words are written
    # into the rank's HBM by the exchange; the emulated rank aliases its own
    # segment instead, so `local_ms_recv` adds that write at HBM_WRITE_TBS as
    # if it did not overlap the compute (an upper bound).
    tables = (2 * (L - 1)) if model.fused else (2 * L)
    # the fused stack packs the ReLU'd forward tables (L - 1) and the
    # ReLU-masked backward ones (L - 2); the top layer's dY travels dense
    packed_tables = (2 * L - 3) if packed else 0
    eff_tables = tables - packed_tables + packed_tables * ratio
    curve = {}
    for p in (1, 2, 4, 8):
        compute = ms_dense * args.world / p
        local = (ms if packed_tables else ms_dense) * args.world / p if p > 1 else compute
        recv = 0.0 if p == 1 else eff_tables * 4.0 * N * F * (p - 1) / p / (HBM_WRITE_TBS * 1e12) * 1e3
        xch = 0.0 if p == 1 else eff_tables * (4.0 * N * F * (p - 1) / p) / (
            (p - 1) * XGMI_LINK_GBS * 1e9) * 1e3
        xch_dense = 0.0 if p == 1 else tables * (4.0 * N * F * (p - 1) / p) / (
            (p - 1) * XGMI_LINK_GBS * 1e9) * 1e3
        step_ms = max(local, xch)
        curve[str(p)] = {"compute_ms": compute, "local_ms": local, "exchange_ms": xch,
                         "local_ms_recv": local + recv,
                         "step_ms_overlapped_recv": max(local + recv, xch),
                         "exchange_ms_dense": xch_dense,
                         "step_ms_overlapped": step_ms,
                         "step_ms_overlapped_dense": max(compute, xch_dense),
                         "step_ms_serial": local + xch,
                         "edges_per_s_overlapped": 2 * P * L / (step_ms * 1e-3)}
    out = {"workload": f"config5 rank {args.rank} of {args.world}: N={N}, E={2 * P} (+{N} loops), "
                       f"F={F}, {L}-layer GCN (sm, add, bias, ReLU) fwd+bwd, exchange tables "
                       "resident (no RCCL; ms_per_step includes the zero-skipping exchange's "
                       "pack and the receive-side write of all P segments of every packed "
                       "table, gathered in place by the next layer)",
           "path": ("fused layer kernels (_ShardedStack)" if model.fused else
                    "per layer: x @ W (mgcn_gemm_nn) + SpMM; adjoint SpMM + dW (mgcn_gemm_tn) + "
                    "dX (mgcn_gemm_nn)"),
           "rows": sh.rows, "fwd_slots": int(sh.fwd.nnz), "bwd_slots": int(sh.bwd.nnz),
           "nnz_global": nnz, "table_rows": sh.table_rows, "prep_s": prep_s,
           "ms_per_step": ms, "ms_per_step_dense_exchange": ms_dense,
           "kernel_ms_per_step": kernel_ms,
           "rank_edges_per_s": (sh.fwd.nnz - sh.rows) * L / (ms_dense * 1e-3),
           "kernels": kern, "exchanged_tables_per_step": tables,
           "packed_tables_per_step": packed_tables,
           "packed_exchange_ratio": ratio if packed_tables else None,
           "dense_equivalent_tables_per_step": eff_tables,
           "xgmi_link_gbs": XGMI_LINK_GBS, "predicted_curve": curve,
           "pack_inplace": mdist.PACK_INPLACE,
           "peak_mem_gb": torch.cuda.max_memory_allocated() / 1e9,
           "sampled_check": check}
    if recv_load is not None:
        # P = world with the local step measured beside the receive writes
        p = args.world
        x8 = curve[str(p)]["exchange_ms"]
        recv_load["step_ms_p%d" % p] = max(recv_load["ms_per_step_under_load"], x8)
        recv_load["speedup_1_to_%d" % p] = curve["1"]["compute_ms"] / recv_load["step_ms_p%d" % p]
        out["recv_load"] = recv_load
    print(json.dumps(out), flush=True)
    if check is not None and not check["ok"]:
        sys.exit("config5_rank: sampled rows outside the fp64 bound")


if __name__ == "__main__":
    main()
