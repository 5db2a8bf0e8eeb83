"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE itself.

Run in the build container (needs /root/reference, read-only):

    python tests/golden/make_golden.py            # gcn_meta cases
    python tests/golden/make_golden.py hardpool   # HardPooling cases
    python tests/golden/make_golden.py conv       # GCNConv cases
    python tests/golden/make_golden.py ewgrad     # edge_weight / deg gradients

It imports the reference's own gcn_meta modules
(/root/reference/src/gcn_meta/models/{gcn_base_models,common,gcn_multi_kernel,
gcn_model}.py) and runs them on seeded small graphs, recording inputs,
outputs and gradients.  Their third-party imports are not vendored and not
installed here, so this script registers:

* ``torch_scatter`` -- a restatement of torch_scatter 1.x's published
  algorithm (positional signature ``(src, index, dim, out, dim_size,
  fill_value)``, as called at common.py:59):
    scatter_add  = out.scatter_add_(dim, index.expand_as(src), src)
    scatter_mean = scatter_add(...) / scatter_add(ones).clamp(min=1)
    scatter_max  = sequential in-order scan with `src >= out` (CPU kernel),
                   returning (out, argmax); its backward routes grad_out to
                   the saved argmax only (scatter_(arg + 1) then narrow).
* ``torch_geometric.nn.inits`` -- glorot / zeros (PyG's published formulas);
* ``torch_geometric.utils.scatter_`` -- a placeholder: only imported by the
  attention modules that gcn_multi_kernel.py:5-6 pulls in, never called here.

The fixtures therefore pin "reference code + torch_scatter 1.x restatement"
(the caveat SURVEY.md §8(c) records).  Nothing of the reference is copied
into the fixtures: they hold only arrays (inputs and expected outputs).
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------- stubs
def _install_stubs():
    ts = types.ModuleType("torch_scatter")

    def gen(src, index, dim=-1, out=None, dim_size=None, fill_value=0):
        dim = range(src.dim())[dim]
        if index.dim() == 1:
            index_size = [1] * src.dim()
            index_size[dim] = src.size(dim)
            index = index.view(index_size).expand_as(src)
        if out is None:
            out_size = list(src.size())
            out_size[dim] = dim_size if dim_size is not None else int(index.max().item()) + 1
            out = src.new_full(out_size, fill_value)
        return src, out, index, dim

    def scatter_add(src, index, dim=-1, out=None, dim_size=None, fill_value=0):
        src, out, index, dim = gen(src, index, dim, out, dim_size, fill_value)
        return out.scatter_add_(dim, index, src)

    def scatter_mean(src, index, dim=-1, out=None, dim_size=None, fill_value=0):
        out = scatter_add(src, index, dim, out, dim_size, fill_value)
        count = scatter_add(torch.ones_like(src), index, dim, None, out.size(dim))
        return out / count.clamp(min=1)

    class ScatterMax(torch.autograd.Function):
        @staticmethod
        def forward(ctx, out, src, index, dim):
            assert dim == 0
            o = out.detach().numpy().copy()
            s = src.detach().numpy()
            ix = index.numpy()[:, 0] if index.dim() > 1 else index.numpy()
            arg = np.full(o.shape, -1, dtype=np.int64)
            for e in range(s.shape[0]):  # sequential, in edge order, `>=`
                d = ix[e]
                m = s[e] >= o[d]
                o[d][m] = s[e][m]
                arg[d][m] = e
            arg_t = torch.from_numpy(arg)
            ctx.save_for_backward(index, arg_t)
            ctx.dim = dim
            return torch.from_numpy(o), arg_t

        @staticmethod
        def backward(ctx, grad_out, grad_arg):
            index, arg = ctx.saved_tensors
            size = list(index.size())
            size[ctx.dim] += 1
            grad_src = grad_out.new_zeros(size)
            grad_src.scatter_(ctx.dim, arg.detach() + 1, grad_out)
            grad_src = grad_src.narrow(ctx.dim, 1, index.size(ctx.dim))
            return None, grad_src, None, None

    def scatter_max(src, index, dim=-1, out=None, dim_size=None, fill_value=None):
        if fill_value is None:
            fill_value = torch.finfo(src.dtype).min
        src, out, index, dim = gen(src, index, dim, out, dim_size, fill_value)
        return ScatterMax.apply(out, src, index, dim)

    ts.scatter_add, ts.scatter_mean, ts.scatter_max = scatter_add, scatter_mean, scatter_max

    tg = types.ModuleType("torch_geometric")
    tgn = types.ModuleType("torch_geometric.nn")
    tgi = types.ModuleType("torch_geometric.nn.inits")
    tgu = types.ModuleType("torch_geometric.utils")

    def glorot(t):
        if t is not None:
            stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
            t.data.uniform_(-stdv, stdv)

    def zeros(t):
        if t is not None:
            t.data.fill_(0)

    def pyg_scatter_(name, src, index, dim_size=None):
        # PyG 1.3 torch_geometric/utils/scatter.py (used by HardPooling)
        assert name in ["add", "mean", "max"]
        op = getattr(ts, "scatter_{}".format(name))
        fill_value = -1e38 if name == "max" else 0
        out = op(src, index, 0, None, dim_size, fill_value)
        if isinstance(out, tuple):
            out = out[0]
        if name == "max":
            out[out == fill_value] = 0
        return out

    def filter_adj(edge_index, edge_attr, perm, num_nodes=None):
        # PyG 1.3 torch_geometric/nn/pool/topk_pool.py filter_adj
        mask = perm.new_full((num_nodes,), -1)
        mask[perm] = torch.arange(perm.size(0), dtype=torch.long)
        row, col = mask[edge_index[0]], mask[edge_index[1]]
        keep = (row >= 0) & (col >= 0)
        row, col = row[keep], col[keep]
        if edge_attr is not None:
            edge_attr = edge_attr[keep]
        return torch.stack([row, col], dim=0), edge_attr

    tgi.glorot, tgi.zeros, tgu.scatter_ = glorot, zeros, pyg_scatter_
    tgp = types.ModuleType("torch_geometric.nn.pool")
    tgpt = types.ModuleType("torch_geometric.nn.pool.topk_pool")
    tgpt.filter_adj = filter_adj
    sys.modules.update({"torch_scatter": ts, "torch_geometric": tg, "torch_geometric.nn": tgn,
                        "torch_geometric.nn.inits": tgi, "torch_geometric.utils": tgu,
                        "torch_geometric.nn.pool": tgp,
                        "torch_geometric.nn.pool.topk_pool": tgpt})


def _import_reference():
    _install_stubs()
    sys.path.insert(0, REF_SRC)
    from gcn_meta.models import common, gcn_base_models, gcn_model  # noqa: E402
    return common, gcn_base_models, gcn_model


# -------------------------------------------------------------- graphs
def make_graph(rng, N, E, self_loops=True, isolated=0, symmetric=False):
    """Random directed multigraph; optional isolated nodes (no edges at all),
    self-loops appended at the end as data_procs/loop.py:13-17 does."""
    active = N - isolated
    s = rng.integers(0, active, E)
    d = rng.integers(0, active, E)
    if symmetric:
        s, d = np.concatenate([s, d]), np.concatenate([d, s])
    # a few explicit duplicates (multi-edges are legal, src/gcn_meta/README.md:20-22)
    k = max(1, E // 50)
    pick = rng.integers(0, s.size, k)
    s, d = np.concatenate([s, s[pick]]), np.concatenate([d, d[pick]])
    if self_loops:
        loops = np.arange(N)
        s, d = np.concatenate([s, loops]), np.concatenate([d, loops])
    return np.stack([s, d]).astype(np.int64)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def save(name, **arrays):
    path = os.path.join(OUT_DIR, name + ".npz")
    clean = {}
    for k, v in arrays.items():
        if v is None:
            continue
        if isinstance(v, torch.Tensor):
            v = v.detach().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(path, **clean)
    return path


# --------------------------------------------------------------- cases
def node_model_case(gbm, name, rng, N, E, F, deg_norm, aggr, bias, deg_mode, use_ew, identity,
                    self_loops=True, isolated=0, relu_layer=None, gm=None):
    ei = make_graph(rng, N, E, self_loops=self_loops, isolated=isolated)
    nnz = ei.shape[1]
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    ew = rng.uniform(0.1, 2.0, nnz).astype(np.float32) if use_ew else None
    deg = None
    if deg_mode == "true":
        deg = np.bincount(ei[0], minlength=N).astype(np.float32)
    elif deg_mode == "random":
        deg = rng.uniform(0.0, 5.0, N).astype(np.float32)
        deg[rng.integers(0, N, max(1, N // 20))] = 0.0  # inf -> 0 path
    torch.manual_seed(int(rng.integers(0, 2**31)))
    if relu_layer is not None:
        layer = gm.GCNLayer(F, F, deg_norm=deg_norm, aggr=aggr, bias=bias, non_linear='relu')
        nm = layer.gcn.node_models[0]
    else:
        layer = nm = gbm.NodeModelAdditive(F, F, deg_norm=deg_norm, aggr=aggr, bias=bias)
    with torch.no_grad():
        if identity:
            nm.weight_node.copy_(torch.eye(F))
        if bias:
            nm.bias.uniform_(-0.5, 0.5)
    xt = _t(x).requires_grad_(True)
    kwargs = dict(deg=None if deg is None else _t(deg),
                  edge_weight=None if ew is None else _t(ew))
    if relu_layer is not None:
        y = layer(xt, _t(ei), None, kwargs["deg"], kwargs["edge_weight"])
    else:
        y = layer(xt, _t(ei), **kwargs)
    y.backward(_t(dZ))
    save(name, edge_index=ei, x=x, W=nm.weight_node.detach(),
         b=None if nm.bias is None else nm.bias.detach(), deg=deg, edge_weight=ew, dZ=dZ, y=y,
         dx=xt.grad, dW=nm.weight_node.grad, db=None if nm.bias is None else nm.bias.grad,
         meta=np.array([deg_norm or "none", aggr, int(bias), int(identity),
                        int(relu_layer is not None)]))


def scatter_case(common, name, rng, E, N, F, op, empty_rows=True):
    hi = N - (N // 10 if empty_rows else 0)
    index = rng.integers(0, hi, E).astype(np.int64)
    if op == "max":
        # duplicates inside one segment exercise the tie rule
        src = rng.integers(-4, 5, (E, F)).astype(np.float32)
    else:
        src = rng.standard_normal((E, F)).astype(np.float32)
    dY = rng.standard_normal((N, F)).astype(np.float32)
    st = _t(src).requires_grad_(True)
    out = common.scatter_(op, st, _t(index), dim_size=N)
    out.backward(_t(dY))
    save(name, src=src, index=index, dY=dY, out=out, dsrc=st.grad, meta=np.array([op]))


def degnorm_case(gbm, name, rng, N, E, method, deg_mode, use_ew):
    ei = make_graph(rng, N, E, self_loops=(deg_mode != "none_loops"), isolated=N // 10)
    nnz = ei.shape[1]
    ew = rng.uniform(0.1, 2.0, nnz).astype(np.float32) if use_ew else None
    deg = rng.uniform(0.0, 4.0, N).astype(np.float32) if deg_mode == "given" else None
    norm = gbm.NodeModelBase.degnorm_const(_t(ei), N, None if deg is None else _t(deg),
                                           None if ew is None else _t(ew), method)
    save(name, edge_index=ei, deg=deg, edge_weight=ew, norm=norm,
         meta=np.array([method, deg_mode, int(use_ew)]))


def model12_case(gm, name, rng, N, E, L=12, F=32):
    """Botnet configuration (src/run/run_botnet.sh:14, train_botnet.py:190-212):
    GCNModel(in=1, enc=[32]*12, residual_hop=1, deg_norm='sm', bias=False,
    final='proj' -> 2 classes), deg passed from x[:, 1].  dropout=0 here so
    the pass is deterministic."""
    ei = make_graph(rng, N, E, self_loops=True, symmetric=True)
    deg = np.bincount(ei[0], minlength=N).astype(np.float32)
    x = np.stack([np.ones(N, np.float32), deg], 1)
    torch.manual_seed(1234)
    model = gm.GCNModel(1, [F] * L, 2, non_linear='relu', non_linear_layer_wise='relu',
                        residual_hop=1, dropout=0.0, final_type='proj', pred_on='node',
                        deg_norm='sm', aggr='add', bias=False)
    xt = _t(x)
    out = model(xt[:, 0:1], _t(ei), deg_K=xt[:, 1])
    g = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(_t(g))
    params = {("p_" + k): v.detach() for k, v in model.state_dict().items()}
    grads = {("g_" + k): p.grad for k, p in model.named_parameters()}
    save(name, edge_index=ei, x=x, dout=g, out=out, **params, **grads)


def hardpool_case(hap, name, rng, sizes, F, aggr, bias, lonely=True, sunk=0):
    """HardPooling (hard_attention_pool.py:23-131) in eval mode on a batch of
    graphs; ``lonely`` gives one node no out-edge (argmax -1 in torch_scatter
    1.x, which the reference turns into marking the last edge).  ``sunk``
    nodes get features -sign(att_weight[:F]) * 1e17, so every out-edge score
    of theirs is far below scatter_max's fill_value -1e16 (:76): no winner,
    argmax -1, as for a node without out-edges."""
    eis, batch, off = [], [], 0
    for g, n in enumerate(sizes):
        E = 3 * n
        s = rng.integers(0, n, E)
        d = rng.integers(0, n, E)
        if lonely and g == 0:
            keep = s != n - 1  # node n - 1 of graph 0 has no out-edge
            s, d = s[keep], d[keep]
        eis.append(np.stack([s, d]) + off)
        batch.append(np.full(n, g))
        off += n
    ei = np.concatenate(eis, 1).astype(np.int64)
    batch = np.concatenate(batch).astype(np.int64)
    x = rng.standard_normal((off, F)).astype(np.float32)
    torch.manual_seed(int(rng.integers(0, 2**31)))
    pool = hap.HardPooling(F, aggr=aggr, bias=bias)
    if bias:
        with torch.no_grad():
            pool.bias.uniform_(-0.5, 0.5)
    pool.eval()
    if sunk:
        a_src = pool.att_weight.detach().numpy()[0, :F]
        for v in rng.choice(off, sunk, replace=False):
            x[v] = -np.sign(a_src).astype(np.float32) * np.float32(1e17)
    xt = _t(x).requires_grad_(True)
    out, ei2, _, b2, perm, score = pool(xt, _t(ei), _t(batch))
    dY = rng.standard_normal(tuple(out.shape)).astype(np.float32)
    out.backward(_t(dY))
    save(name, x=x, edge_index=ei, batch=batch, att_weight=pool.att_weight.detach(),
         bias=None if pool.bias is None else pool.bias.detach(), out=out, out_edge_index=ei2,
         out_batch=b2, perm=perm, score=score, dY=dY, dx=xt.grad,
         meta=np.array([aggr]))


def main_hardpool():
    """Only the HardPooling fixtures (``python make_golden.py hardpool``)."""
    _install_stubs()
    sys.path.insert(0, REF_SRC)
    from gcn_meta.models import hard_attention_pool as hap  # noqa: E402
    rng = np.random.default_rng(20261016)
    hardpool_case(hap, "hardpool_add", rng, [12, 30, 7], 16, "add", False)
    hardpool_case(hap, "hardpool_add_bias", rng, [25, 9, 40, 16], 16, "add", True)
    hardpool_case(hap, "hardpool_mean", rng, [20, 33], 8, "mean", False, lonely=False)
    hardpool_case(hap, "hardpool_sunk", rng, [18, 26], 8, "add", False, lonely=False, sunk=6)
    print("wrote 4 hardpool fixtures to", OUT_DIR)


def add_remaining_self_loops(ei, ew, fill, N):
    """PyG 1.3 torch_geometric.utils.add_remaining_self_loops (published
    algorithm; PyG is not vendored in the reference): drop every existing
    self-loop, append one loop per node at the end; a node that had a loop
    keeps that loop's weight (the last one in COO order), the others get
    ``fill``."""
    mask = ei[0] != ei[1]
    loops = np.arange(N, dtype=np.int64)
    ei2 = np.concatenate([ei[:, mask], np.stack([loops, loops])], 1)
    lw = np.full(N, fill, np.float32)
    inv = ~mask
    lw[ei[0][inv]] = ew[inv]  # numpy fancy assignment: the last write wins
    ew2 = np.concatenate([ew[mask], lw]).astype(np.float32)
    return ei2, ew2


def gcnconv_case(gbm, name, rng, N, E, F, use_ew, improved, identity, isolated=0):
    """PyG GCNConv(F, F, improved) as kernel/gcn.py uses it, pinned through the
    reference's own NodeModelAdditive(deg_norm='sm', aggr='add', bias=True):
    GCNConv.norm + propagate('add') is gcn_base_models.py:199-243 with
    edge_weight = the unit (or given) weights after add_remaining_self_loops
    -- the same formula the in-repo copy src/gcn_meta/models/gcn.py:57-86
    writes (deg over row, dinv[row] * w * dinv[col], message norm * x_j,
    scatter_add over col, + bias).  The raw graph keeps random self-pairs in
    the middle of the edge list (the loop handling is part of what is
    pinned)."""
    ei = make_graph(rng, N, E, self_loops=False, isolated=isolated)
    # a few explicit self-pairs mid-list (dropped and re-added as tail loops)
    k = max(1, N // 25)
    v = rng.integers(0, N - isolated, k)
    at = np.sort(rng.integers(0, ei.shape[1], k))
    ei = np.insert(ei, at, np.stack([v, v]), axis=1).astype(np.int64)
    ew = rng.uniform(0.1, 2.0, ei.shape[1]).astype(np.float32) if use_ew else None
    # GCNConv.norm: unit weights first when none are given, THEN the loops
    # (an existing loop keeps its weight 1, new loops get the fill value)
    ew_in = ew if ew is not None else np.ones(ei.shape[1], np.float32)
    ei2, ew2 = add_remaining_self_loops(ei, ew_in, 2.0 if improved else 1.0, N)
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    torch.manual_seed(int(rng.integers(0, 2**31)))
    nm = gbm.NodeModelAdditive(F, F, deg_norm='sm', aggr='add', bias=True)
    with torch.no_grad():
        if identity:
            nm.weight_node.copy_(torch.eye(F))
        nm.bias.uniform_(-0.5, 0.5)
    xt = _t(x).requires_grad_(True)
    y = nm(xt, _t(ei2), edge_weight=_t(ew2))
    y.backward(_t(dZ))
    save(name, edge_index=ei, edge_weight=ew, x=x, W=nm.weight_node.detach(), b=nm.bias.detach(),
         dZ=dZ, y=y, dx=xt.grad, dW=nm.weight_node.grad, db=nm.bias.grad,
         meta=np.array([int(improved), int(identity), int(use_ew)]))


def ewgrad_case(gbm, name, rng, N, E, F, deg_norm, aggr, identity, given="ew", isolated=10):
    """NodeModelAdditive with edge_weight (or deg) requiring grad: records the
    gradient degnorm_const passes back to it (gcn_base_models.py:102-140)."""
    ei = make_graph(rng, N, E, self_loops=True, isolated=isolated)
    nnz = ei.shape[1]
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    ew = rng.uniform(0.1, 2.0, nnz).astype(np.float32)
    deg = rng.uniform(0.5, 5.0, N).astype(np.float32)
    deg[rng.integers(0, N, max(1, N // 20))] = 0.0  # the inf -> 0 entries
    torch.manual_seed(int(rng.integers(0, 2**31)))
    nm = gbm.NodeModelAdditive(F, F, deg_norm=deg_norm, aggr=aggr, bias=True)
    with torch.no_grad():
        if identity:
            nm.weight_node.copy_(torch.eye(F))
        nm.bias.uniform_(-0.5, 0.5)
    xt = _t(x).requires_grad_(True)
    ewt = _t(ew).requires_grad_(True) if given == "ew" else None
    degt = _t(deg).requires_grad_(True) if given == "deg" else None
    y = nm(xt, _t(ei), deg=degt, edge_weight=ewt)
    y.backward(_t(dZ))
    save(name, edge_index=ei, x=x, W=nm.weight_node.detach(), b=nm.bias.detach(),
         edge_weight=ew if given == "ew" else None, deg=deg if given == "deg" else None, dZ=dZ,
         y=y, dx=xt.grad, dW=nm.weight_node.grad, db=nm.bias.grad,
         dew=None if ewt is None else ewt.grad, ddeg=None if degt is None else degt.grad,
         meta=np.array([deg_norm, aggr, given, int(identity)]))


def main_ewgrad():
    """Only the edge_weight / deg gradient fixtures (``python make_golden.py ewgrad``)."""
    _, gbm, _ = _import_reference()
    rng = np.random.default_rng(20261018)
    n = 0
    for deg_norm in ["sm", "rw"]:
        for aggr in ["add", "mean", "max"]:
            ewgrad_case(gbm, f"ewgrad_{deg_norm}_{aggr}", rng, 400, 3000, 16, deg_norm, aggr,
                        True)
            n += 1
        ewgrad_case(gbm, f"degrad_{deg_norm}_add", rng, 400, 3000, 16, deg_norm, "add", True,
                    given="deg")
        n += 1
    ewgrad_case(gbm, "ewgrad_sm_add_f128", rng, 500, 5000, 128, "sm", "add", False)
    n += 1
    print(f"wrote {n} edge-weight gradient fixtures to", OUT_DIR)


def main_conv():
    """Only the GCNConv fixtures (``python make_golden.py conv``)."""
    _, gbm, _ = _import_reference()
    rng = np.random.default_rng(20261017)
    gcnconv_case(gbm, "gcnconv_id", rng, 500, 4000, 16, False, False, True, isolated=20)
    gcnconv_case(gbm, "gcnconv_ew_id", rng, 400, 3000, 32, True, False, True)
    gcnconv_case(gbm, "gcnconv_improved_id", rng, 400, 3000, 16, False, True, True, isolated=10)
    gcnconv_case(gbm, "gcnconv_f128_id", rng, 600, 6000, 128, False, False, True)
    gcnconv_case(gbm, "gcnconv_f128", rng, 600, 6000, 128, False, False, False)
    gcnconv_case(gbm, "gcnconv_ew_f128", rng, 500, 5000, 128, True, True, False)
    print("wrote 6 gcnconv fixtures to", OUT_DIR)


def main():
    common, gbm, gm = _import_reference()
    rng = np.random.default_rng(20250824)
    n = 0
    # A. aggregation bit-exact cases: W = I so H = x and dx = dH
    for deg_norm in ["sm", "rw", None]:
        for aggr in ["add", "mean", "max"]:
            for bias in [True, False]:
                F = {"add": 16, "mean": 32, "max": 16}[aggr]
                node_model_case(gbm, f"aggr_{deg_norm or 'none'}_{aggr}_b{int(bias)}", rng, 500,
                                4000, F, deg_norm, aggr, bias, "none", False, True,
                                isolated=20)
                n += 1
    for deg_norm in ["sm", "rw"]:
        for aggr in ["add", "max"]:
            node_model_case(gbm, f"aggr_{deg_norm}_{aggr}_deg", rng, 400, 3000, 16, deg_norm,
                            aggr, True, "random", False, True)
            node_model_case(gbm, f"aggr_{deg_norm}_{aggr}_ew", rng, 400, 3000, 16, deg_norm, aggr,
                            True, "none", True, True)
            n += 2
    node_model_case(gbm, "aggr_sm_add_noloops", rng, 400, 3000, 16, "sm", "add", True, "none",
                    False, True, self_loops=False, isolated=40)
    node_model_case(gbm, "aggr_sm_add_f128", rng, 300, 3000, 128, "sm", "add", True, "true",
                    False, True)
    node_model_case(gbm, "aggr_sm_add_relu", rng, 400, 3000, 32, "sm", "add", True, "none", False,
                    True, relu_layer=True, gm=gm)
    node_model_case(gbm, "aggr_rw_mean_relu", rng, 400, 3000, 32, "rw", "mean", True, "none",
                    False, True, relu_layer=True, gm=gm)
    n += 4
    # B. full layer with a random weight (tolerance comparisons)
    for deg_norm, aggr in [("sm", "add"), ("rw", "mean"), (None, "max"), ("sm", "max")]:
        node_model_case(gbm, f"layer_{deg_norm or 'none'}_{aggr}", rng, 400, 3000, 32, deg_norm,
                        aggr, True, "none", False, False)
        n += 1
    # C. common.scatter_ on explicit [E, F] sources
    for op in ["add", "mean", "max"]:
        scatter_case(common, f"scatter_{op}", rng, 5000, 300, 8, op)
        n += 1
    # D. degnorm_const
    for method in ["sm", "rw"]:
        for deg_mode, use_ew in [("computed", False), ("given", False), ("computed", True),
                                 ("none_loops", False)]:
            degnorm_case(gbm, f"degnorm_{method}_{deg_mode}_ew{int(use_ew)}", rng, 300, 2000,
                         method, deg_mode, use_ew)
            n += 1
    # E. 12-layer botnet-shaped GCNModel
    model12_case(gm, "model12_botnet", rng, 600, 1500)
    n += 1
    print(f"wrote {n} fixtures to {OUT_DIR}")


if __name__ == "__main__":
    if sys.argv[1:] == ["hardpool"]:
        main_hardpool()
    elif sys.argv[1:] == ["conv"]:
        main_conv()
    elif sys.argv[1:] == ["ewgrad"]:
        main_ewgrad()
    else:
        main()
