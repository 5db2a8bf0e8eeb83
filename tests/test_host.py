"""CPU-only checks of the host layer and the C ABI boundary (no GPU compute)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden

HEADER = os.path.join(ROOT, "include", "mgcn.h")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mgcn_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    """libmgcn.so loads (no compute) and exports exactly what include/mgcn.h declares."""
    from mgcn import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 13
    for n in names:
        assert hasattr(lib, n), f"libmgcn.so does not export {n}"
    # the Python binding declares a signature for every C entry point
    assert sorted(_lib.SIGNATURES) == names


def test_abi_version_and_option_errors():
    import mgcn
    lib = mgcn.load()
    assert lib.mgcn_abi_version() == mgcn._lib.ABI_VERSION == 22
    assert lib.mgcn_set_option(b"no_such_option", 1) == 1
    assert b"unknown option" in lib.mgcn_last_error()
    # the switches that change results (timing experiments) and the spin bound
    # of the warp-specialised kernels exist only in libmgcn_exp.so
    for name in (b"ws_spin_limit", b"wide_dbg", b"xw_ws_dbg"):
        assert lib.mgcn_set_option(name, 1) == 1
        assert b"experiment builds only" in lib.mgcn_last_error()
    with pytest.raises(mgcn.MgcnError):
        mgcn.set_option("spmm_unroll", 3)
    mgcn.set_option("spmm_unroll", 8)


def test_c_abi_rejects_bad_arguments_without_touching_memory():
    """Argument validation happens on the host before any launch."""
    import mgcn
    lib = mgcn.load()
    assert lib.mgcn_spmm_fwd(-1, 4, None, None, None, None, None, 4, None, 4, 0, None, 0, None,
                             None, None, None, 0, 0, None) == 1
    assert lib.mgcn_spmm_fwd(4, 4, None, None, None, None, None, 4, None, 4, 7, None, 0, None,
                             None, None, None, 0, 0, None) == 1
    assert b"bad reduce" in lib.mgcn_last_error()
    assert lib.mgcn_degree_norm(4, None, None, None, None, 9, None, None, None) == 1
    assert lib.mgcn_csr_build(None, None, -1, 0, 0, None, None, None, None, 0, None) == 1
    # zero-sized work is a successful no-op
    assert lib.mgcn_spmm_fwd(0, 4, None, None, None, None, None, 4, None, 4, 0, None, 0, None,
                             None, None, None, 0, 0, None) == 0
    assert lib.mgcn_csr_workspace_bytes(1000, 100) > 0
    assert lib.mgcn_gemm_tn_workspace_bytes(1 << 20, 128, 128) >= 128 * 128 * 4
    # the ReLU mask needs relu and F <= 128
    assert lib.mgcn_spmm_fwd(4, 256, None, None, None, None, None, 256, None, 256, 0, None, 1,
                             None, None, 1, None, 0, 0, None) == 1
    assert lib.mgcn_relu_mask(4, 129, None, 129, None, None) == 1
    assert lib.mgcn_set_option(b"gemm_precision", 2) == 1


def test_no_cpu_fallback():
    """The product path refuses CPU tensors loudly (never a silent CPU path)."""
    import mgcn
    from mgcn.models import NodeModelAdditive
    x = torch.randn(5, 4)
    ei = torch.tensor([[0, 1, 2], [1, 2, 3]])
    with pytest.raises(mgcn.MgcnError, match="HIP device"):
        mgcn.aggregate(x, ei)
    with pytest.raises(mgcn.MgcnError, match="HIP device"):
        NodeModelAdditive(4, 4)(x, ei)
    with pytest.raises(mgcn.MgcnError, match="HIP device"):
        mgcn.scatter_("add", x, torch.tensor([0, 0, 1, 1, 2]))


def test_module_surface_matches_reference_state_dicts():
    """Parameter names/shapes equal the reference's, so checkpoints interchange:
    the reference's own 12-layer botnet GCNModel state_dict (golden fixture)
    loads strictly into mgcn's GCNModel."""
    from mgcn.models import GCNModel, GCNLayer, NodeModelAdditive
    z = load_golden("model12_botnet")
    sd = {k[2:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("p_")}
    m = GCNModel(1, [32] * 12, 2, residual_hop=1, dropout=0.0, final_type='proj',
                 deg_norm='sm', aggr='add', bias=False)
    m.load_state_dict(sd, strict=True)
    assert list(NodeModelAdditive(3, 5).state_dict()) == ["weight_node", "bias"]
    assert NodeModelAdditive(3, 5).weight_node.shape == (3, 5)
    assert "gcn.node_models.0.weight_node" in GCNLayer(3, 5).state_dict()
    with pytest.raises(AssertionError):
        NodeModelAdditive(3, 5, deg_norm="bad")
    with pytest.raises(NotImplementedError):
        NodeModelAdditive(3, 5, edge_gate="proj")


def test_pyg_surface_parameter_names():
    from torch.nn import Linear, ReLU, Sequential
    from mgcn.pyg import GCNConv, GINConv, GraphConv, JumpingKnowledge, SAGEConv
    assert sorted(GCNConv(7, 16).state_dict()) == ["bias", "weight"]
    assert sorted(SAGEConv(7, 16).state_dict()) == ["bias", "weight"]
    assert sorted(GraphConv(7, 16, aggr='mean').state_dict()) == ["lin.bias", "lin.weight",
                                                                    "weight"]
    gin = GINConv(Sequential(Linear(7, 16), ReLU()), train_eps=True)
    assert "eps" in dict(gin.named_parameters())
    assert "eps" in GINConv(Sequential(Linear(7, 16)), train_eps=False).state_dict()
    xs = [torch.randn(4, 3), torch.randn(4, 3)]
    assert JumpingKnowledge('cat')(xs).shape == (4, 6)
    assert JumpingKnowledge('max')(xs).shape == (4, 3)
    assert JumpingKnowledge('lstm', channels=3, num_layers=2)(xs).shape == (4, 3)


def test_self_loop_utilities_follow_pyg13():
    from mgcn.pyg import add_remaining_self_loops, remove_self_loops
    ei = torch.tensor([[0, 1, 1, 2], [1, 1, 2, 0]])
    w = torch.tensor([1.0, 5.0, 2.0, 3.0])
    ei2, w2 = add_remaining_self_loops(ei, w, 7.0, 3)
    assert ei2.tolist() == [[0, 1, 2, 0, 1, 2], [1, 2, 0, 0, 1, 2]]
    assert w2.tolist() == [1.0, 2.0, 3.0, 7.0, 5.0, 7.0]  # old loop weight kept
    ei3, _ = remove_self_loops(ei)
    assert ei3.tolist() == [[0, 1, 2], [1, 2, 0]]


def test_graph_cache_key_tracks_version_and_identity():
    from mgcn.graph import cache_key
    ei = torch.tensor([[0, 1], [1, 0]])
    k1 = cache_key(ei, 2)
    ei.add_(0)  # in-place op bumps the version counter
    assert cache_key(ei, 2) != k1
    assert cache_key(ei, 3) != cache_key(ei, 2)


def test_bench_workload_shape():
    """config 2 generator: 2*pairs symmetric edges + N loops at the end."""
    from bench import make_er_graph, spmm_bytes
    ei, n = make_er_graph(1000, 5000)
    assert ei.shape == (2, 11000) and n == 1000
    assert torch.equal(ei[:, -1000:], torch.arange(1000).repeat(2, 1))
    assert torch.equal(ei[0, :5000], ei[1, 5000:10000])
    assert spmm_bytes(1_000_000, 11_000_000, 128) == 6_240_000_008


def test_oracle_is_not_imported_by_product():
    """The product package never references the oracle (checker only)."""
    pkg = os.path.join(ROOT, "meta-gcn_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
                assert "liboracle" not in text, f


@pytest.mark.parametrize("method,given", [("sm", "ew"), ("rw", "ew"), ("sm", "deg"),
                                          ("rw", "deg"), (None, "ew")])
def test_grad_norm_chain_matches_reference_autograd(monkeypatch, method, given):
    """graph._grad_norm (edge_weight / deg requiring grad) against autograd of
    the reference's own expression (gcn_base_models.py:117-142: scatter_add
    of the weights over edge_index[0], pow(-1/2 | -1), inf -> 0 in place,
    dinv[row] * w * dinv[col]).  Host logic only: the degree kernel is the
    CPU double's (tests/cpu_backend.py); the SDDMM is a GPU test."""
    import mgcn.graph as G
    from cpu_backend import CpuBackend
    be = CpuBackend()
    monkeypatch.setattr(G, "degree_norm", be.degree_norm)
    g = torch.Generator().manual_seed(7)
    N, E = 40, 160
    ei = torch.randint(0, N, (2, E), generator=g)
    ei[:, :5] = torch.tensor([[3, 3, 3, 9, 9], [1, 2, 3, 9, 0]])
    plan = be.build_plan(ei, N)
    ew = (torch.rand(E, generator=g) + 0.1).requires_grad_(given == "ew")
    deg = (torch.rand(N, generator=g) * 4).requires_grad_(given == "deg")
    with torch.no_grad():
        deg[[5, 11]] = 0.0  # the inf -> 0 entries (gradient masked there)
    ew_r = ew.detach().clone().requires_grad_(given == "ew")
    deg_r = deg.detach().clone().requires_grad_(given == "deg")
    src, dst = ei
    if given == "ew":
        d = torch.zeros(N).scatter_add(0, src, ew_r)
    else:
        d = deg_r
    if method is None:
        w_ref = ew_r
    else:
        a = d.pow(-0.5) if method == "sm" else d.pow(-1)
        a = a.clone()
        a[a == float("inf")] = 0
        if method == "rw" and given == "deg":
            w_ref = a[src]  # per-slot dinv[src]: x * dinv before the gather
        elif method == "sm":
            w_ref = a[src] * ew_r * a[dst] if given == "ew" else a[src] * a[dst]
        else:
            w_ref = a[src] * ew_r
    nm = plan.norm(method, deg=None if given == "ew" else deg,
                   edge_weight=ew if given == "ew" else None)
    assert nm.grad and nm.w_fwd.requires_grad
    eid = plan.fwd.eid.long()
    w = torch.zeros(E).index_put((eid,), nm.w_fwd)
    torch.testing.assert_close(w.detach(), w_ref.detach(), rtol=1e-6, atol=0)
    gout = torch.randn(E, generator=g)
    (w * gout).sum().backward()
    (w_ref * gout).sum().backward()
    got, want = (ew.grad, ew_r.grad) if given == "ew" else (deg.grad, deg_r.grad)
    finite = torch.isfinite(want)
    assert torch.equal(finite, torch.isfinite(got))
    torch.testing.assert_close(got[finite], want[finite], rtol=1e-5, atol=1e-6)
    if nm.w_bwd is not None:
        assert not nm.w_bwd.requires_grad
        torch.testing.assert_close(nm.w_bwd, w.detach()[plan.bwd.eid.long()], rtol=0, atol=0)


def test_pyg_loop_helpers_match_oracle_restatement(oracle):
    """mgcn.pyg.add_remaining_self_loops / remove_self_loops (PyG 1.3, torch
    index bookkeeping) against the oracle's numpy restatement, including
    several loops on one node (the last one's weight is carried)."""
    import numpy as np
    import torch
    from mgcn.pyg import add_remaining_self_loops, remove_self_loops
    rng = np.random.default_rng(4)
    N = 60
    ei = rng.integers(0, N, (2, 400))
    ei[1, ::7] = ei[0, ::7]  # many self-pairs, several per node
    ew = rng.uniform(0.1, 2.0, 400).astype(np.float32)
    for w in (ew, None):
        a, aw = add_remaining_self_loops(torch.from_numpy(ei),
                                         None if w is None else torch.from_numpy(w), 2.0, N)
        b, bw = oracle.add_remaining_self_loops(ei, w, 2.0, N)
        np.testing.assert_array_equal(a.numpy(), b)
        if w is None:
            assert aw is None and bw is None
        else:
            np.testing.assert_array_equal(aw.numpy(), bw)
    np.testing.assert_array_equal(remove_self_loops(torch.from_numpy(ei))[0].numpy(),
                                  oracle.remove_self_loops(ei))


def test_dense_products_never_route_to_a_vendor_gemm():
    """Every 2-D fp32 product of the module surface routes to a libmgcn
    kernel (mm_route): configs 2-5 (128 -> 128, the botnet stack's 1 -> 32,
    32 -> 32 and 32 -> 2 heads with their transposes, 256 -> 256) and the
    kernel/ nets' widths (TU inputs 3 / 7 / 21 / 89, hidden 16-128, 2-6
    classes); torch.matmul is left only for non-2-D / non-fp32 operands."""
    import torch
    from mgcn.ops import mm_route
    shapes = [(128, 128), (1, 32), (32, 1), (32, 32), (32, 2), (2, 32), (64, 64), (256, 256),
              (128, 256), (256, 128)]
    for fin in (3, 7, 21, 89):
        for hid in (16, 32, 64, 128):
            shapes += [(fin, hid), (hid, fin)]
    for hid in (16, 32, 64, 128):
        for c in (2, 6):
            shapes += [(hid, c), (c, hid), (hid, hid), (2 * hid, hid), (hid, 2 * hid)]
    for K, N in shapes:
        assert mm_route(K, N) in ("nn", "small_k"), (K, N)
    assert mm_route(32, 128) == "nn" and mm_route(1, 32) == "small_k"
    assert mm_route(128, 128, dim=3) == "vendor"
    assert mm_route(128, 128, dtype=torch.float16) == "vendor"
