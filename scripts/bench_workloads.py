"""Secondary workloads of BASELINE.json (parity/coverage cases, not the
headline bench line):

  config3: botnet-shaped node classification, 2 graphs x 143,107 nodes per
           batch (bsz = 2, run_botnet.sh:14), 12-layer GCNModel F = 32,
           residual_hop = 1, deg_norm 'sm', bias 0, final proj 32 -> 2,
           CrossEntropy + Adam step (train_botnet.py:276-294).
  config4: the config-2 graph with the GIN / SAGE / max aggregators: 3-layer
           stacks of NodeModelAdditive(deg_norm=None, aggr=add|mean|max).

    python scripts/bench_workloads.py --workload config3 [--steps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from bench import batch_graphs, make_botnet_graph, make_er_graph, make_inputs  # noqa: E402


HOST = {}


def timed(step, steps, warmup):
    """Seconds per step; HOST['ms'] = host time to issue one step (the time the
    Python loop takes before the final sync): when it is close to the step
    time, the workload is bound by launch issue, not by the GPU."""
    step()
    torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    HOST["ms"] = t_issue / steps * 1e3
    return t


def kernel_times(step):
    """{kernel: launches, avg_ms, total_ms} of one step (HIP events on the
    launch stream around every libmgcn call)."""
    from bench import KernelTimer
    from mgcn import ops
    timer = KernelTimer()
    ops.set_kernel_timer(timer)
    step()
    torch.cuda.synchronize()
    ops.set_kernel_timer(None)
    out = {}
    for name, k in timer.summary().items():
        k.pop("sizes")
        out[name] = {kk: round(v, 4) if isinstance(v, float) else v for kk, v in k.items()}
    return out


def config3(args, dev):
    from mgcn.models import GCNModel
    g1, n1, m1 = make_botnet_graph(seed=0)
    g2, n2, m2 = make_botnet_graph(seed=1)
    ei, N = batch_graphs([(g1, n1), (g2, n2)])
    n_edges = ei.shape[1] - N
    deg = torch.bincount(ei[0], minlength=N).float()
    x = torch.stack([torch.ones(N), deg], 1).to(dev)
    y = torch.cat([m1, m2]).long().to(dev)
    ei = ei.to(dev)
    torch.manual_seed(0)
    model = GCNModel(1, [32] * 12, 2, non_linear='relu', non_linear_layer_wise='relu',
                     residual_hop=1, dropout=0.0, final_type='proj', pred_on='node',
                     deg_norm='sm', aggr='add', bias=False).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-4,
                           **({"fused": True} if args.adam == "fused" else {}))
    from mgcn.botnet import CrossEntropyLoss
    crit = CrossEntropyLoss()

    def step():
        opt.zero_grad()
        out = model(x[:, 0].view(-1, 1), ei, deg_K=x[:, 1])
        crit(out, y).backward()
        opt.step()
    t = timed(step, args.steps, args.warmup)
    return {"workload": "config3 botnet-shaped 2x143,107 nodes, 12-layer GCNModel F=32 rh=1, "
                        "CE + Adam", "nodes": N, "edges": n_edges, "max_in_degree":
            int(torch.bincount(ei[1], minlength=N).max()), "ms_per_step": t * 1e3,
            "edges_per_s": n_edges * 12 / t, "host_issue_ms_per_step": HOST["ms"]}


def config4(args, dev):
    from mgcn.models import GCNLayer, GCNStack
    ei_cpu, N = make_er_graph()
    ei = ei_cpu.to(dev)
    n_edges = ei.shape[1] - N
    X, Ws, bs, dY = make_inputs(N, 128, 3)
    X, dY = X.to(dev), dY.to(dev)
    res = {"workload": "config4 ER N=1M E=10M F=128, 3-layer stacks deg_norm=None", "edges": n_edges}
    for aggr in args.aggr.split(","):
        layers = []
        for i in range(3):
            layer = GCNLayer(128, 128, deg_norm=None, aggr=aggr, bias=True,
                             non_linear='relu' if i < 2 else 'none').to(dev)
            with torch.no_grad():
                layer.gcn.node_models[0].weight_node.copy_(Ws[i])
                layer.gcn.node_models[0].bias.copy_(bs[i])
            layers.append(layer)
        stack = GCNStack(layers)
        params = list(stack.parameters())

        def step():
            for p in params:
                p.grad = None
            stack(X, ei).backward(dY)
        t = timed(step, args.steps, args.warmup)
        res[aggr] = {"ms_per_step": t * 1e3, "edges_per_s": n_edges * 3 / t}
        if args.timers:
            res[aggr]["kernels"] = kernel_times(step)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["config3", "config4"], required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--aggr", default="add,mean,max", help="config4: aggregators to run")
    ap.add_argument("--adam", choices=["default", "fused"], default="fused",
                    help="config3: torch Adam implementation: fused (one multi-tensor kernel; "
                         "the same update, 0.28 ms/step less host issue) or default (foreach)")
    ap.add_argument("--timers", action="store_true",
                    help="also time one more step with HIP events around every libmgcn launch "
                         "(bench.KernelTimer) and report them per kernel")
    ap.add_argument("--heavy-thr", type=int, default=None,
                    help="rows above this degree take the heavy-row kernels (mgcn.graph.HEAVY_THRESHOLD)")
    ap.add_argument("--opt", action="append", default=[],
                    help="libmgcn option name=value (mgcn_set_option), repeatable")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.heavy_thr is not None:
        import mgcn.graph
        mgcn.graph.HEAVY_THRESHOLD = args.heavy_thr
    if args.opt:
        import mgcn
        lib = mgcn.load()
        for kv in args.opt:
            k, v = kv.split("=")
            mgcn._lib.check(lib.mgcn_set_option(k.encode(), int(v)), "mgcn_set_option")
    fn = {"config3": config3, "config4": config4}[args.workload]
    print(json.dumps(fn(args, dev)), flush=True)


if __name__ == "__main__":
    main()
