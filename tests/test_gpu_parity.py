"""GPU parity: libmgcn kernels (through the C ABI via mgcn) against the golden
fixtures of the reference and against the C oracle.

Bar (north_star): the aggregation is integer-indexed fp32 work done in the
reference's exact operation order, so given the same H it must match BIT FOR
BIT (np.testing.assert_array_equal).  Whole layers include a GEMM whose
rounding differs between BLAS libraries: those compare with
rtol = 1e-5 (forward) / 1e-4 (gradients) as stated per test.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu


def _t(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def _meta(z):
    m = [str(v) for v in z["meta"]]
    return (None if m[0] == "none" else m[0]), m[1], bool(int(m[2])), bool(int(m[3])), \
        bool(int(m[4]))


def _np(t):
    return t.detach().cpu().numpy()


# ------------------------------------------------------------ fixtures
@pytest.mark.parametrize("name", golden_names("aggr_"))
def test_aggregate_matches_reference_bitwise(cuda, name):
    import mgcn
    z = load_golden(name)
    deg_norm, aggr, bias, identity, relu = _meta(z)
    x = _t(z["x"], cuda).requires_grad_(True)
    ei = _t(z["edge_index"], cuda)
    b = _t(z["b"], cuda).requires_grad_(True) if bias else None
    deg = _t(z["deg"], cuda) if "deg" in z else None
    ew = _t(z["edge_weight"], cuda) if "edge_weight" in z else None
    y = mgcn.aggregate(x, ei, aggr=aggr, deg_norm=deg_norm, deg=deg, edge_weight=ew, bias=b,
                       relu=relu)
    np.testing.assert_array_equal(_np(y), z["y"])
    y.backward(_t(z["dZ"], cuda))
    np.testing.assert_array_equal(_np(x.grad), z["dx"])
    if bias:
        np.testing.assert_allclose(_np(b.grad), z["db"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("name", golden_names("layer_"))
def test_node_model_additive_matches_reference(cuda, name):
    from mgcn.models import NodeModelAdditive
    z = load_golden(name)
    deg_norm, aggr, bias, _, _ = _meta(z)
    F = z["x"].shape[1]
    m = NodeModelAdditive(F, F, deg_norm=deg_norm, aggr=aggr, bias=bias).to(cuda)
    with torch.no_grad():
        m.weight_node.copy_(_t(z["W"], cuda))
        if bias:
            m.bias.copy_(_t(z["b"], cuda))
    x = _t(z["x"], cuda).requires_grad_(True)
    y = m(x, _t(z["edge_index"], cuda))
    np.testing.assert_allclose(_np(y), z["y"], rtol=1e-5, atol=1e-5)
    y.backward(_t(z["dZ"], cuda))
    np.testing.assert_allclose(_np(x.grad), z["dx"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(m.weight_node.grad), z["dW"], rtol=1e-4, atol=1e-3)
    if bias:
        np.testing.assert_allclose(_np(m.bias.grad), z["db"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("name", golden_names("scatter_"))
def test_scatter_matches_reference_bitwise(cuda, name):
    import mgcn
    z = load_golden(name)
    op = str(z["meta"][0])
    src = _t(z["src"], cuda).requires_grad_(True)
    out = mgcn.scatter_(op, src, _t(z["index"], cuda), dim_size=z["out"].shape[0])
    np.testing.assert_array_equal(_np(out), z["out"])
    out.backward(_t(z["dY"], cuda))
    np.testing.assert_array_equal(_np(src.grad), z["dsrc"])


@pytest.mark.parametrize("name", golden_names("degnorm_"))
def test_degnorm_const_matches_reference_bitwise(cuda, name):
    from mgcn.models import NodeModelBase
    z = load_golden(name)
    method = str(z["meta"][0])
    ei = _t(z["edge_index"], cuda)
    deg = _t(z["deg"], cuda) if "deg" in z else None
    ew = _t(z["edge_weight"], cuda) if "edge_weight" in z else None
    norm = NodeModelBase.degnorm_const(ei, 300, deg, ew, method)
    np.testing.assert_array_equal(_np(norm), z["norm"])


def test_gcn_model_12_layer_botnet_matches_reference(cuda):
    """Config 3 shape (run_botnet.sh:14): 12 layers F=32, residual_hop=1."""
    from mgcn.models import GCNModel
    z = load_golden("model12_botnet")
    model = GCNModel(1, [32] * 12, 2, non_linear='relu', non_linear_layer_wise='relu',
                     residual_hop=1, dropout=0.0, final_type='proj', pred_on='node',
                     deg_norm='sm', aggr='add', bias=False).to(cuda)
    sd = {k[2:]: _t(v, cuda) for k, v in z.items() if k.startswith("p_")}
    model.load_state_dict(sd)
    x = _t(z["x"], cuda)
    out = model(x[:, 0:1], _t(z["edge_index"], cuda), deg_K=x[:, 1])
    np.testing.assert_allclose(_np(out), z["out"], rtol=1e-4, atol=1e-4)
    out.backward(_t(z["dout"], cuda))
    for k, p in model.named_parameters():
        ref = z["g_" + k]
        scale = max(1.0, float(np.abs(ref).max()))
        np.testing.assert_allclose(_np(p.grad), ref, rtol=1e-3, atol=1e-4 * scale, err_msg=k)


# ------------------------------------------------- random graphs vs oracle
def _graph(rng, N, E, loops=True, heavy=0, heavy_src=0):
    s = rng.integers(0, N, E)
    d = rng.integers(0, N, E)
    if heavy:  # destinations 0..3 get `heavy` extra in-edges between them
        d = np.concatenate([d, rng.integers(0, 4, heavy)])
        s = np.concatenate([s, rng.integers(0, N, heavy)])
    if heavy_src:  # source 1 gets `heavy_src` extra out-edges
        s = np.concatenate([s, np.ones(heavy_src, np.int64)])
        d = np.concatenate([d, rng.integers(0, N, heavy_src)])
    if loops:
        s = np.concatenate([s, np.arange(N)])
        d = np.concatenate([d, np.arange(N)])
    return np.stack([s, d]).astype(np.int64)


CASES = [
    # N, E, F, deg_norm, aggr, relu, heavy (extra in-edges on rows 0..3)
    (20000, 200000, 128, "sm", "add", True, 0),
    (20000, 200000, 64, "rw", "mean", False, 0),
    (20000, 200000, 32, None, "max", False, 0),
    (5000, 60000, 7, "sm", "max", True, 0),
    (5000, 60000, 2, "rw", "add", False, 0),
    (3000, 30000, 300, "sm", "mean", True, 0),
    (3000, 30000, 128, "sm", "add", False, 12000),  # one destination of degree 12k
    (3000, 30000, 1, "sm", "add", False, 0),
    (3000, 30000, 32, "sm", "max", True, 9000),
    (3000, 30000, 32, "rw", "mean", False, 7000),
    (3000, 30000, 300, None, "max", False, 2000),
    (3000, 30000, 7, "sm", "add", True, 1000),
    (5000, 20000, 32, "sm", "add", False, 300),  # skewed, no heavy row: degree order only
    (5000, 20000, 16, None, "max", False, 300),
    (4000, 40000, 256, "sm", "max", True, 0),     # two 128-feature chunks of winner records
    (2000, 80000, 128, None, "max", False, 0),    # light rows of degree 20..65: several
                                                  # 32-edge winner windows per row
]


@pytest.mark.parametrize("N,E,F,deg_norm,aggr,relu,heavy", CASES)
def test_random_graph_vs_oracle_bitwise(cuda, oracle, N, E, F, deg_norm, aggr, relu, heavy):
    import mgcn
    rng = np.random.default_rng(N + E + F)
    ei = _graph(rng, N, E, heavy=heavy, heavy_src=heavy // 2)
    H = rng.standard_normal((N, F)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, F).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    wf, wb, rs = oracle.edge_factors(ei, N, deg_norm)
    y_ref, am = oracle.aggr_fwd(ei, H, wf, aggr, b, relu)
    dH_ref, db_ref = oracle.aggr_bwd(ei, dZ, wb, rs, aggr, y_ref, relu, am, want_db=True)
    Ht = _t(H, cuda).requires_grad_(True)
    bt = _t(b, cuda).requires_grad_(True)
    y = mgcn.aggregate(Ht, _t(ei, cuda), aggr=aggr, deg_norm=deg_norm, bias=bt, relu=relu)
    np.testing.assert_array_equal(_np(y), y_ref)
    y.backward(_t(dZ, cuda))
    np.testing.assert_array_equal(_np(Ht.grad), dH_ref)
    np.testing.assert_allclose(_np(bt.grad), db_ref, rtol=1e-4, atol=1e-3)


def test_noncontiguous_and_strided_inputs(cuda, oracle):
    import mgcn
    rng = np.random.default_rng(7)
    N, F = 2000, 64
    ei = _graph(rng, N, 20000)
    big = rng.standard_normal((N, 2 * F)).astype(np.float32)
    H = big[:, ::2]
    wf, _, _ = oracle.edge_factors(ei, N, "sm")
    y_ref, _ = oracle.aggr_fwd(ei, H, wf, "add")
    Ht = _t(big, cuda)[:, ::2]
    y = mgcn.aggregate(Ht, _t(ei, cuda), aggr="add", deg_norm="sm")
    np.testing.assert_array_equal(_np(y), y_ref)


def test_empty_graph_and_isolated_nodes(cuda):
    import mgcn
    N, F = 17, 8
    H = torch.randn(N, F, device=cuda)
    ei = torch.zeros(2, 0, dtype=torch.long, device=cuda)
    for aggr in ["add", "mean", "max"]:
        y = mgcn.aggregate(H, ei, aggr=aggr, deg_norm="sm")
        assert torch.equal(y, torch.zeros_like(y))


def test_out_of_range_index_raises(cuda):
    import mgcn
    H = torch.randn(4, 8, device=cuda)
    ei = torch.tensor([[0, 1], [2, 4]], device=cuda)
    mgcn.clear_cache()
    with pytest.raises(IndexError):
        mgcn.aggregate(H, ei)


def test_deterministic_repeat(cuda):
    import mgcn
    rng = np.random.default_rng(3)
    ei = _t(_graph(rng, 10000, 100000), cuda)
    H = torch.randn(10000, 128, device=cuda)
    y1 = mgcn.aggregate(H, ei, deg_norm="sm")
    y2 = mgcn.aggregate(H, ei, deg_norm="sm")
    assert torch.equal(y1, y2)


# --------------------------------------------- full size (config 2) properties
@pytest.mark.slow
def test_config2_full_size_forward_backward_bitwise(cuda, oracle):
    """BASELINE config 2 (N = 1M, 10M symmetrised edges + 1M loops, F = 128):
    the headline workload itself, forward and adjoint, bit for bit against
    the C oracle (a few seconds of single-threaded CPU)."""
    import mgcn
    from bench import make_er_graph
    ei, N = make_er_graph(1_000_000, 5_000_000)
    eic = ei.to(cuda)
    g = torch.Generator().manual_seed(1)
    H = torch.randn(N, 128, generator=g)
    dZ = torch.randn(N, 128, generator=g)
    Ht = H.to(cuda).requires_grad_(True)
    y = mgcn.aggregate(Ht, eic, deg_norm="sm", relu=True)
    y.backward(dZ.to(cuda))
    ein = ei.numpy()
    wf, wb, rs = oracle.edge_factors(ein, N, "sm")
    y_ref, _ = oracle.aggr_fwd(ein, H.numpy(), wf, "add", None, True)
    np.testing.assert_array_equal(_np(y), y_ref)
    dH_ref, _ = oracle.aggr_bwd(ein, dZ.numpy(), wb, rs, "add", y_ref, True, None)
    np.testing.assert_array_equal(_np(Ht.grad), dH_ref)


# ----------------------------------------------------------------- dense
@pytest.fixture(params=[1, 0], ids=["bf16x6", "f32"])
def gemm_precision(request):
    """Both product arithmetics of the dense GEMMs (bf16x6 is the default)."""
    import mgcn
    mgcn.set_option("gemm_precision", request.param)
    yield request.param
    mgcn.set_option("gemm_precision", 1)


@pytest.mark.parametrize("K,M,N", [(1_000_000, 128, 128), (4097, 128, 128), (3000, 7, 130),
                                   (50, 32, 2), (0, 4, 4), (286_214, 32, 32), (286_214, 2, 32),
                                   (1001, 17, 5), (77, 128, 256), (1_000_003, 128, 128),
                                   # M = 32, N = 32 / 64: the staged kernel (config 3's
                                   # [dW | dWr^T]), whole and ragged 64-row chunks
                                   (286_214, 32, 64), (100, 32, 64), (64, 32, 32), (65, 32, 64),
                                   # 256 x 256 (config 5's dW): one workgroup per split
                                   # owns the whole C; whole, ragged and tiny splits
                                   (2_000_003, 256, 256), (4097, 256, 256), (17, 256, 256),
                                   (1, 256, 256)])
def test_gemm_tn_matches_fp64(cuda, K, M, N, gemm_precision):
    """dW = A^T B (f32 MFMA: exact f32 products; bf16x6: the exact three-term
    bf16 split, six products on bf16 MFMA; f32 accumulation in a different
    order than any BLAS): |err| <= 1e-5 * sum_k |a_k b_k| + 1e-6."""
    from mgcn.ops import gemm_tn
    g = torch.Generator(device=cuda).manual_seed(K + M)
    A = torch.randn(K, M, device=cuda, generator=g)
    B = torch.randn(K, N, device=cuda, generator=g)
    C = gemm_tn(A, B)
    ref = A.double().t() @ B.double()
    bound = A.double().abs().t() @ B.double().abs()
    assert ((C.double() - ref).abs() <= 1e-5 * bound + 1e-6).all()
    C2 = gemm_tn(A, B)
    assert torch.equal(C, C2)  # deterministic


@pytest.mark.parametrize("K,M,N,n1", [(286_214, 32, 64, 32), (4097, 128, 256, 128),
                                      (4097, 256, 256, 128),
                                      (3000, 7, 130, 5), (1001, 17, 5, 0), (1001, 17, 5, 5),
                                      (0, 4, 6, 2)])
def test_gemm_tn_split_equals_gemm_tn(cuda, K, M, N, n1):
    """mgcn_gemm_tn_split (the residual layer's [dW | dWr^T] in one pass):
    the same products and fold as mgcn_gemm_tn, columns [n1, N) written
    transposed -- bitwise equal to slicing the plain product."""
    from mgcn.ops import gemm_tn, gemm_tn_split
    g = torch.Generator(device=cuda).manual_seed(K + N)
    A = torch.randn(K, M, device=cuda, generator=g)
    B = torch.randn(K, N, device=cuda, generator=g)
    C = gemm_tn(A, B)
    C1, C2t = gemm_tn_split(A, B, n1)
    assert C1.shape == (M, n1) and C2t.shape == (N - n1, M)
    assert C1.is_contiguous() and C2t.is_contiguous()
    assert torch.equal(C1, C[:, :n1]) and torch.equal(C2t, C[:, n1:].t())


def test_gemm_bf16x6_error_at_fp32_level(cuda):
    """The bf16x6 products are no less accurate than exact-f32 MFMA: max
    error / (|A| |B|) against fp64 within 2x of the f32 form's (measured:
    3e-7 vs 5e-7 for X W at K = 128), on operands spanning 2^-40..2^40."""
    import mgcn
    from mgcn.ops import gemm_nn, gemm_tn
    g = torch.Generator(device=cuda).manual_seed(5)
    A = torch.randn(65536, 128, device=cuda, generator=g)
    A = A * torch.exp2(torch.randint(-40, 40, A.shape, device=cuda, generator=g).float())
    W = torch.randn(128, 128, device=cuda, generator=g)
    B = torch.randn(65536, 128, device=cuda, generator=g)
    errs = {}
    for prec in (0, 1):
        mgcn.set_option("gemm_precision", prec)
        C = gemm_nn(A, W)[0].double()
        D = gemm_tn(A, B).double()
        e_nn = ((C - A.double() @ W.double()).abs() / (A.double().abs() @ W.double().abs())).max()
        e_tn = ((D - A.double().t() @ B.double()).abs() /
                (A.double().abs().t() @ B.double().abs())).max()
        errs[prec] = (float(e_nn), float(e_tn))
    mgcn.set_option("gemm_precision", 1)
    assert errs[1][0] <= 2 * errs[0][0] + 1e-7, errs
    assert errs[1][1] <= 2 * errs[0][1] + 1e-7, errs


def test_gemm_nonfinite_and_range_edge_operands(cuda, gemm_precision):
    """+-inf and |x| near FLT_MAX (where bf16 RNE overflows, 3.3962e38 ..
    3.4028e38) in either operand: the products are +-inf where fp32 matmul
    gives +-inf and finite (within the usual bound) where it is finite --
    never the NaN of inf - inf inside the bf16 split."""
    from mgcn.ops import gemm_nn, gemm_tn
    g = torch.Generator(device=cuda).manual_seed(17)
    M, K = 4097, 128
    A = torch.randn(M, K, device=cuda, generator=g) * 1e-3
    W = torch.rand(K, K, device=cuda, generator=g) * 0.1 + 0.1  # positive: signs predictable
    A[0, 0] = float("inf")
    A[1, 3] = float("-inf")
    A[2, 5] = 3.4e38
    A[3, 7] = -3.39e38
    A[4, 9] = 3.3961514e38
    A[5, 11] = torch.finfo(torch.float32).max
    B = torch.rand(M, K, device=cuda, generator=g) * 0.1 + 0.1
    for C, ref, bound in (
            (gemm_nn(A, W)[0], A.double() @ W.double(), A.double().abs() @ W.double().abs()),
            (gemm_tn(A, B), A.double().t() @ B.double(), A.double().abs().t() @ B.double().abs())):
        C = C.double()
        inf = torch.isinf(ref)
        assert inf.any() and not torch.isnan(C).any()
        assert torch.equal(C[inf], ref[inf])  # same signed infinities
        fin = ~inf
        assert torch.isfinite(C[fin]).all()
        assert ((C[fin] - ref[fin]).abs() <= 1e-5 * bound[fin] + 1e-6).all()
    # the other operand: W with an inf column entry and a near-FLT_MAX one
    A2 = torch.rand(M, K, device=cuda, generator=g) * 0.1 + 0.1
    W2 = W.clone()
    W2[4, 2] = float("inf")
    W2[6, 9] = 3.4e38
    C = gemm_nn(A2, W2)[0].double()
    ref = A2.double() @ W2.double()
    assert torch.equal(torch.isinf(C), torch.isinf(ref)) and not torch.isnan(C).any()
    fin = torch.isfinite(ref)
    assert ((C[fin] - ref[fin]).abs() <= 1e-5 * (A2.double() @ W2.double().abs())[fin]).all()


def test_relu_mask_layout(cuda, oracle):
    """mgcn_relu_mask / the SpMM's fused mask: bit b of word v <=> Z[i, 4b+v] > 0,
    for the fused F = 128 rows, heavy rows and other F."""
    from mgcn.ops import make_relu_mask
    import mgcn
    g = torch.Generator().manual_seed(3)
    for F in (128, 100, 64, 32, 7):
        Z = torch.randn(1000, F, generator=g)
        Z[::7] = 0.0
        m = make_relu_mask(Z.to(cuda)).cpu().numpy().view(np.uint32)
        ref = np.zeros((1000, 4), np.uint32)
        pos = (Z.numpy() > 0)
        for f in range(F):
            ref[:, f & 3] |= pos[:, f].astype(np.uint32) << np.uint32(f >> 2)
        np.testing.assert_array_equal(m, ref)
    # fused in the forward SpMM, including heavy rows (star centres)
    N = 3000
    s = torch.randint(0, N, (20000,), generator=g)
    d = torch.randint(0, N, (20000,), generator=g)
    hub = torch.arange(0, 900)
    ei = torch.stack([torch.cat([s, hub]), torch.cat([d, torch.zeros_like(hub)])])
    for F in (128, 64):
        H = torch.randn(N, F, generator=g).to(cuda)
        plan = mgcn.build_plan(ei.to(cuda), N)
        assert plan.fwd.n_heavy > 0
        norm = plan.norm("sm")
        rm = torch.empty(N, 4, dtype=torch.int32, device=cuda)
        Y, _ = mgcn.ops.spmm_fwd(plan.fwd, norm.w_fwd, H, 0, None, True, relu_mask=rm)
        assert torch.equal(rm, make_relu_mask(Y))


@pytest.mark.parametrize("M,K,N,trans", [(1_000_000, 128, 128, False), (1_000_000, 128, 128, True),
                                         (1000, 64, 100, False), (777, 32, 7, True), (1, 128, 128, False),
                                         (286_214, 32, 32, False), (286_214, 32, 32, True),
                                         (5000, 32, 2, False), (3000, 64, 40, True)])
def test_gemm_nn_matches_fp64(cuda, M, K, N, trans, gemm_precision):
    from mgcn.ops import gemm_nn
    g = torch.Generator(device=cuda).manual_seed(M + K + N)
    A = torch.randn(M, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g) if trans else \
        torch.randn(K, N, device=cuda, generator=g)
    Wm = W.t() if trans else W
    C, cs = gemm_nn(A, W, transpose_w=trans)
    ref = A.double() @ Wm.double()
    bound = A.double().abs() @ Wm.double().abs()
    assert ((C.double() - ref).abs() <= 1e-5 * bound + 1e-6).all()
    assert cs is None
    # fused ReLU-backward epilogue: C = Z > 0 ? A W : 0, colsum = sum_m C
    Z = torch.randn(M, N, device=cuda, generator=g)
    C2, cs2 = gemm_nn(A, W, transpose_w=trans, Z=Z)
    assert torch.equal(C2, torch.where(Z > 0, C, torch.zeros_like(C)))
    ref_cs = C2.double().sum(0)
    assert torch.allclose(cs2.double(), ref_cs, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,K,N,trans", [
    # K = 256 (config 5's x @ W and dH W^T): 64-column groups on one XCD each
    (1_000_003, 256, 256, False), (100_000, 256, 256, True), (70_001, 256, 100, False),
    (5000, 256, 32, True), (33, 256, 256, False),
    # K <= 128 with N > 128: 128-column groups
    (300_000, 128, 256, False), (1000, 128, 300, True), (3000, 64, 200, False),
    # the generic tiled kernel: K outside {32, 64, 128, 256} (TU inputs, hidden 16)
    (10_000, 16, 16, False), (10_000, 89, 64, True), (3000, 21, 130, False),
    (777, 300, 5, True), (65, 12, 33, False), (50_000, 130, 128, False), (1, 9, 1, True)])
def test_gemm_nn_wide_and_generic_matches_fp64(cuda, M, K, N, trans, gemm_precision):
    """mgcn_gemm_nn on every shape (ABI v15): the tuned kernel's column
    groups (K = 256, N > 128) and the generic tiled kernel, both precisions,
    against fp64 within 1e-5 of sum_k |a_k b_k|; deterministic; the fused
    ReLU-mask epilogue where it applies (tuned kernel, N <= 128)."""
    from mgcn import ops
    g = torch.Generator(device=cuda).manual_seed(M + 3 * K + N)
    A = torch.randn(M, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g) if trans else \
        torch.randn(K, N, device=cuda, generator=g)
    Wm = W.t() if trans else W
    C, _ = ops.gemm_nn(A, W, transpose_w=trans)
    ref = A.double() @ Wm.double()
    bound = A.double().abs() @ Wm.double().abs()
    err = (C.double() - ref).abs()
    assert bool((err <= 1e-5 * bound + 1e-6).all()), float((err / (bound + 1e-6)).max())
    assert torch.equal(C, ops.gemm_nn(A, W, transpose_w=trans)[0])
    if ops.gemm_nn_epi_supported(K, N):
        Z = torch.randn(M, N, device=cuda, generator=g)
        C2, cs2 = ops.gemm_nn(A, W, transpose_w=trans, Z=Z)
        assert torch.equal(C2, torch.where(Z > 0, C, torch.zeros_like(C)))
        assert torch.allclose(cs2.double(), C2.double().sum(0), rtol=1e-4, atol=1e-3)


def test_linear_layers_of_odd_widths_stay_on_libmgcn(cuda):
    """x @ W and F.linear of the module surface at widths the tuned kernels
    do not take run on libmgcn (no torch.matmul), forward and backward."""
    from mgcn import ops
    from mgcn.models import Linear
    ops.VENDOR_GEMMS.clear()
    g = torch.Generator(device=cuda).manual_seed(3)
    for fin, fout in [(89, 16), (16, 6), (21, 64), (7, 130), (300, 2)]:
        x = torch.randn(5000, fin, device=cuda, generator=g).requires_grad_(True)
        lin = Linear(fin, fout).to(cuda)
        W = torch.randn(fin, fout, device=cuda, generator=g).requires_grad_(True)
        y = lin(x) + ops.linear(x, W)
        y.backward(torch.ones_like(y))
        ref = x.detach().double() @ lin.weight.detach().double().t() + lin.bias.detach().double() \
            + x.detach().double() @ W.detach().double()
        assert torch.allclose(y.detach().double(), ref, rtol=1e-5, atol=1e-4)
        dx = torch.ones(5000, fout, device=cuda, dtype=torch.float64) @ \
            (lin.weight.detach().double() + W.detach().double().t())
        assert torch.allclose(x.grad.double(), dx, rtol=1e-5, atol=1e-4)
    assert not ops.VENDOR_GEMMS, dict(ops.VENDOR_GEMMS)


@pytest.mark.parametrize("M", [1_000_000, 1_000_003, 4097, 31, 1, 0])
def test_gemm_bwd_matches_fp64(cuda, M):
    """Fused adjoints (mgcn_gemm_bwd): dW = X^T dH and dX = dH W^T within
    1e-5 of the |.|-weighted fp64 sums; the ReLU / row-divisor epilogue
    equals masking and dividing the plain dX; dW matches mgcn_gemm_tn's
    bound, is deterministic and accumulates."""
    from mgcn.ops import gemm_bwd, make_relu_mask
    g = torch.Generator(device=cuda).manual_seed(M + 1)
    X = torch.randn(M, 128, device=cuda, generator=g)
    dH = torch.randn(M, 128, device=cuda, generator=g)
    W = torch.randn(128, 128, device=cuda, generator=g)
    dW, dX, cs = gemm_bwd(X, dH, W)
    assert cs is None
    ref_w = X.double().t() @ dH.double()
    bound_w = X.double().abs().t() @ dH.double().abs()
    assert ((dW.double() - ref_w).abs() <= 1e-5 * bound_w + 1e-6).all()
    ref_x = dH.double() @ W.double().t()
    bound_x = dH.double().abs() @ W.double().abs().t()
    assert ((dX.double() - ref_x).abs() <= 1e-5 * bound_x + 1e-6).all()
    # dW alone, repeat (deterministic), accumulate
    dW2, none, _ = gemm_bwd(X, dH, W, want_dx=False)
    assert none is None and torch.equal(dW, dW2)
    acc = torch.ones(128, 128, device=cuda)
    gemm_bwd(X, dH, W, want_dx=False, dW_out=acc, accumulate=True)
    assert torch.equal(acc, dW + 1.0)
    # fused ReLU backward (+ mean's row divisor) and bias-gradient column sums
    Z = torch.randn(M, 128, device=cuda, generator=g)
    rm = make_relu_mask(Z)
    dW3, dX3, cs3 = gemm_bwd(X, dH, W, relu_mask=rm)
    masked = torch.where(Z > 0, dX, torch.zeros_like(dX))
    assert torch.equal(dW3, dW) and torch.equal(dX3, masked)
    torch.testing.assert_close(cs3.double(), masked.double().sum(0), rtol=1e-4, atol=1e-3)
    div = torch.randint(1, 20, (M,), device=cuda, generator=g).float()
    _, dX4, cs4 = gemm_bwd(X, dH, W, relu_mask=rm, row_div=div)
    assert torch.equal(dX4, masked / div[:, None]) and torch.equal(cs4, cs3)


def test_gemm_bwd_strided_inputs(cuda):
    """Row strides > F (views into wider buffers) give the contiguous result."""
    from mgcn.ops import gemm_bwd
    g = torch.Generator(device=cuda).manual_seed(9)
    Xw = torch.randn(5000, 136, device=cuda, generator=g)
    Hw = torch.randn(5000, 132, device=cuda, generator=g)
    W = torch.randn(128, 128, device=cuda, generator=g)
    a = gemm_bwd(Xw[:, :128], Hw[:, 4:], W)
    b = gemm_bwd(Xw[:, :128].contiguous(), Hw[:, 4:].contiguous(), W)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_gcn_stack_identity_weights_bitwise_vs_oracle(cuda, oracle):
    """3 fused layers with W = I: every layer's aggregation and the whole
    adjoint chain (dx) are bit-exact against the oracle layer by layer."""
    from mgcn.models import GCNLayer, GCNStack
    rng = np.random.default_rng(11)
    N, F = 6000, 128
    ei = _graph(rng, N, 60000)
    x = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    layers = [GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                       non_linear='relu' if i < 2 else 'none').to(cuda) for i in range(3)]
    bs = []
    for layer in layers:
        nm = layer.gcn.node_models[0]
        with torch.no_grad():
            nm.weight_node.copy_(torch.eye(F))
            nm.bias.uniform_(-0.2, 0.2)
        bs.append(nm.bias.detach().cpu().numpy())
    stack = GCNStack(layers)
    xt = _t(x, cuda).requires_grad_(True)
    y = stack(xt, _t(ei, cuda))
    y.backward(_t(dZ, cuda))
    wf, wb, rs = oracle.edge_factors(ei, N, "sm")
    hs = [x]
    for i in range(3):
        h, _ = oracle.aggr_fwd(ei, hs[-1], wf, "add", bs[i], relu=i < 2)
        hs.append(h)
    np.testing.assert_array_equal(_np(y), hs[-1])
    g = dZ
    dbs = []
    for i in range(2, -1, -1):
        g, db = oracle.aggr_bwd(ei, g, wb, rs, "add", hs[i + 1], relu=i < 2, want_db=True)
        dbs.append(db)
    np.testing.assert_array_equal(_np(xt.grad), g)
    for layer, db in zip(layers[::-1], dbs):
        np.testing.assert_allclose(_np(layer.gcn.node_models[0].bias.grad), db, rtol=1e-4,
                                   atol=1e-3)


def test_gcn_stack_matches_layer_by_layer(cuda):
    """Stack on the GEMM + SpMM launches == the same GCNLayers run one by one
    (forward and dW bitwise: same kernels; db within fp32 summation-order
    tolerance).  The fused aggregate+transform kernels are compared with
    this path in tests/test_gpu_fused.py."""
    from mgcn import ops
    ops.set_fused_layers(False)
    try:
        _stack_vs_layers(cuda)
    finally:
        ops.set_fused_layers(True)


def _stack_vs_layers(cuda):
    from mgcn.models import GCNLayer, GCNStack
    torch.manual_seed(0)
    rng = np.random.default_rng(12)
    N, F = 20000, 128
    ei = _t(_graph(rng, N, 200000), cuda)
    layers = [GCNLayer(F, F, deg_norm='sm', aggr='add', bias=True,
                       non_linear='relu' if i < 2 else 'none').to(cuda) for i in range(3)]
    for layer in layers:
        with torch.no_grad():
            layer.gcn.node_models[0].bias.uniform_(-0.1, 0.1)
    x = torch.randn(N, F, device=cuda)
    dZ = torch.randn(N, F, device=cuda)
    stack = GCNStack(layers)
    y1 = stack(x, ei)
    y1.backward(dZ)
    g1 = [p.grad.clone() for p in stack.parameters()]
    for p in stack.parameters():
        p.grad = None
    h = x
    for layer in layers:
        h = layer(h, ei)
    assert torch.equal(h, y1)
    h.backward(dZ)
    for (name, p), a in zip(stack.named_parameters(), g1):
        if name.endswith("weight_node"):
            assert torch.equal(p.grad, a), name
        else:
            torch.testing.assert_close(p.grad, a, rtol=1e-4, atol=1e-3)


def test_heavy_rows_are_listed(cuda):
    """Rows above the threshold get the workgroup path in both views."""
    from mgcn.graph import HEAVY_THRESHOLD, plan_for
    rng = np.random.default_rng(5)
    ei = _t(_graph(rng, 2000, 10000, heavy=12 * HEAVY_THRESHOLD, heavy_src=2 * HEAVY_THRESHOLD),
            cuda)
    plan = plan_for(ei, 2000)
    deg_in = (plan.fwd.rowptr[1:] - plan.fwd.rowptr[:-1])
    deg_out = (plan.bwd.rowptr[1:] - plan.bwd.rowptr[:-1])
    assert set(plan.fwd.heavy.tolist()) == set(torch.nonzero(deg_in > HEAVY_THRESHOLD)[:, 0].tolist())
    assert set(plan.bwd.heavy.tolist()) == set(torch.nonzero(deg_out > HEAVY_THRESHOLD)[:, 0].tolist())
    assert plan.bwd.n_heavy >= 1


@pytest.mark.parametrize("F", [128, 7, 300])
def test_max_adjoint_mask_equals_argmax_routing(cuda, oracle, F):
    """mgcn_max_mask + win_mask adjoint == the argmax-routed adjoint, bit for
    bit (light and heavy rows, ragged words), and == the oracle."""
    from mgcn import ops
    from mgcn.graph import plan_for
    rng = np.random.default_rng(F)
    N = 3000
    ei = _graph(rng, N, 30000, heavy=3000, heavy_src=2000)
    H = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    wf, wb, rs = oracle.edge_factors(ei, N, None)
    y_ref, am_ref = oracle.aggr_fwd(ei, H, wf, "max")
    dH_ref, _ = oracle.aggr_bwd(ei, dZ, wb, rs, "max", y_ref, False, am_ref)
    plan = plan_for(_t(ei, cuda), N)
    Y, argmax = ops.spmm_fwd(plan.fwd, None, _t(H, cuda), 2)
    mask = ops.max_mask(plan, argmax)
    d_arg = ops.spmm_bwd(plan.bwd, None, None, _t(dZ, cuda), 2, argmax=argmax)
    d_mask = ops.spmm_bwd(plan.bwd, None, None, _t(dZ, cuda), 2, win_mask=mask,
                          slot_map=plan.slot_map())
    assert torch.equal(d_arg, d_mask)
    np.testing.assert_array_equal(_np(d_mask), dH_ref)
    # the forward kernels (lane-group and heavy rows) write the same bits directly
    Y2, fused = ops.spmm_fwd(plan.fwd, None, _t(H, cuda), 2, mask_plan=plan)
    assert torch.equal(Y2, Y)
    assert torch.equal(fused, mask)


HEAVY_CONFIGS = [
    # libmgcn options for the heavy-row launches (read at plan time / launch)
    {"heavy_giant_thr": 0},                      # every heavy row giant, 1024 threads
    {"heavy_giant_thr": 1 << 40},                # none giant: 256-thread launch only
    {"heavy_giant_thr": 0, "heavy_block": 256, "heavy_lds_kb": 16},  # many small batches
    {"heavy_giant_thr": 0, "heavy_block": 512, "heavy_lds_kb": 24},
    {"heavy_giant_thr": 600, "heavy_mid_lds_kb": 16, "heavy_side_stream": 0},
]
HEAVY_DEFAULTS = {"heavy_giant_thr": 512, "heavy_block": 1024, "heavy_lds_kb": 160,
                  "heavy_mid_lds_kb": 40, "heavy_side_stream": 1}


@pytest.mark.parametrize("cfg", HEAVY_CONFIGS)
@pytest.mark.parametrize("F,aggr", [(32, "add"), (128, "mean"), (7, "max"), (64, "max")])
def test_heavy_path_configurations_bitwise(cuda, oracle, cfg, F, aggr):
    """Giant / mid heavy-row launches, block sizes and batch sizes all give
    the reference's bits (fwd and adjoint, incl. ragged last batches)."""
    import mgcn
    rng = np.random.default_rng(F + len(aggr))
    N = 3000
    ei = _graph(rng, N, 30000, heavy=6000, heavy_src=2500)
    H = rng.standard_normal((N, F)).astype(np.float32)
    dZ = rng.standard_normal((N, F)).astype(np.float32)
    wf, wb, rs = oracle.edge_factors(ei, N, "sm")
    y_ref, am = oracle.aggr_fwd(ei, H, wf, aggr)
    dH_ref, _ = oracle.aggr_bwd(ei, dZ, wb, rs, aggr, y_ref, False, am)
    try:
        for k, v in cfg.items():
            mgcn.set_option(k, v)
        mgcn.clear_cache()
        Ht = _t(H, cuda).requires_grad_(True)
        y = mgcn.aggregate(Ht, _t(ei, cuda), aggr=aggr, deg_norm="sm")
        np.testing.assert_array_equal(_np(y), y_ref)
        y.backward(_t(dZ, cuda))
        np.testing.assert_array_equal(_np(Ht.grad), dH_ref)
    finally:
        for k, v in HEAVY_DEFAULTS.items():
            mgcn.set_option(k, v)
        mgcn.clear_cache()


@pytest.mark.parametrize("M,fin,fout", [(286_214, 32, 32), (286_214, 32, 2), (5000, 7, 16)])
def test_linear_matches_torch(cuda, M, fin, fout):
    """mgcn.models.Linear (libmgcn GEMMs) == torch.nn.Linear within fp32 tolerance."""
    from mgcn.models import Linear
    torch.manual_seed(M + fin)
    ref = torch.nn.Linear(fin, fout).to(cuda)
    lin = Linear(fin, fout).to(cuda)
    lin.load_state_dict(ref.state_dict())
    x = torch.randn(M, fin, device=cuda)
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    dy = torch.randn(M, fout, device=cuda)
    y1, y2 = lin(x1), ref(x2)
    torch.testing.assert_close(y1, y2, rtol=1e-5, atol=1e-5)
    y1.backward(dy)
    y2.backward(dy)
    torch.testing.assert_close(x1.grad, x2.grad, rtol=1e-5, atol=1e-5)
    # dW, db sum over M = 286k rows: check against fp64 with a summation bound
    ref_dw = dy.double().t() @ x.double()
    bound = dy.double().abs().t() @ x.double().abs()
    assert ((lin.weight.grad.double() - ref_dw).abs() <= 1e-5 * bound + 1e-6).all()
    ref_db = dy.double().sum(0)
    assert ((lin.bias.grad.double() - ref_db).abs() <= 1e-5 * dy.double().abs().sum(0) + 1e-6).all()


@pytest.mark.parametrize("aggr,deg_norm,bias", [("add", "sm", False), ("mean", "rw", True),
                                                ("max", None, True)])
def test_gcn_model_residual_fused_matches_step_by_step(cuda, aggr, deg_norm, bias):
    """GCNModel(residual_hop=1) through the fused residual layer nodes equals
    the step-for-step path (gcn_model.py:86-125): forward bitwise where the
    layer keeps the reference's association (max, and the first 1 -> 32
    layer), within fp32 tolerance where the 32 -> 32 layers run
    (A x) W on the fused residual-layer kernels (add, mean); gradients within
    fp32 GEMM tolerance; includes a skewed (heavy-row) graph."""
    from mgcn.models import GCNModel
    rng = np.random.default_rng(21)
    N = 4000
    ei = _t(_graph(rng, N, 30000, heavy=3000), cuda)
    deg = torch.bincount(ei[0], minlength=N).float()
    x = torch.randn(N, 1, device=cuda)
    torch.manual_seed(3)
    model = GCNModel(1, [32] * 5, 2, non_linear='relu', non_linear_layer_wise='relu',
                     residual_hop=1, dropout=0.0, final_type='proj', pred_on='node',
                     deg_norm=deg_norm, aggr=aggr, bias=bias).to(cuda)
    dout = torch.randn(N, 2, device=cuda)
    res = {}
    for fused in (True, False):
        GCNModel.fuse_residual = fused
        try:
            for p in model.parameters():
                p.grad = None
            out = model(x, ei, deg_K=deg)
            out.backward(dout)
            res[fused] = (out.detach().clone(),
                          {k: p.grad.clone() for k, p in model.named_parameters()})
        finally:
            GCNModel.fuse_residual = True
    if aggr == "max":
        assert torch.equal(res[True][0], res[False][0])
    else:
        torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-4,
                                   atol=1e-5 * max(1.0, float(res[False][0].abs().max())))
    for k, g in res[False][1].items():
        scale = max(1.0, float(g.abs().max()))
        torch.testing.assert_close(res[True][1][k], g, rtol=1e-4, atol=1e-5 * scale, msg=k)


def test_residual_act_kernels(cuda):
    """mgcn_residual_act / _bwd against torch on strided operands."""
    from mgcn.ops import residual_act, residual_act_bwd
    g = torch.Generator(device=cuda).manual_seed(2)
    n, F = 3001, 32
    Z1 = torch.relu(torch.randn(n, F, device=cuda, generator=g))
    HR = torch.randn(n, 2 * F, device=cuda, generator=g)
    rb = torch.randn(F, device=cuda, generator=g)
    for relu in (True, False):
        Z = residual_act(Z1, HR[:, F:], rb, relu)
        ref = Z1 + (HR[:, F:] + rb)
        assert torch.equal(Z, torch.relu(ref) if relu else ref)
        dZ = torch.randn(n, F, device=cuda, generator=g)
        DH = torch.zeros(n, 2 * F, device=cuda)
        dA = torch.empty(n, F, device=cuda)
        div = torch.randint(1, 9, (n,), device=cuda, generator=g).float()
        sums = residual_act_bwd(dZ, Z, relu, Z1, True, dA, DH[:, F:], row_div=div)
        dS = torch.where(Z > 0, dZ, torch.zeros_like(dZ)) if relu else dZ
        a = torch.where(Z1 > 0, dS, torch.zeros_like(dS))
        assert torch.equal(DH[:, F:], dS) and torch.equal(dA, a / div[:, None])
        torch.testing.assert_close(sums[:F].double(), a.double().sum(0), rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(sums[F:].double(), dS.double().sum(0), rtol=1e-5, atol=1e-4)


def test_int64_offsets_beyond_2_31_elements(cuda):
    """N F > 2^31 (config 5 gathers from a 51 GB [50M, 256] matrix): forward
    and adjoint SpMM rows sampled across the whole range equal a sequential
    fp32 restatement in COO order bit for bit (scripts/config5_check.py runs
    the full config-5 size: profiles/r01/config5_check.json)."""
    from mgcn import _lib as L
    from mgcn.ops import spmm_bwd, spmm_fwd
    import mgcn
    N, P, F = 20_000_000, 20_000_000, 128  # N F = 2.56e9
    g = torch.Generator(device=cuda).manual_seed(5)
    s = torch.randint(0, N, (P,), device=cuda, generator=g)
    d = torch.randint(0, N, (P,), device=cuda, generator=g)
    ar = torch.arange(N, device=cuda)
    ei = torch.stack([torch.cat([s, d, ar]), torch.cat([d, s, ar])])
    del s, d, ar
    plan = mgcn.build_plan(ei, N)
    norm = plan.norm("sm")
    del ei
    X = torch.randn(N, F, device=cuda, generator=g)
    Y, _ = spmm_fwd(plan.fwd, norm.w_fwd, X, L.REDUCE_SUM)
    dH = spmm_bwd(plan.bwd, norm.w_bwd, None, X, L.REDUCE_SUM)
    rows = torch.cat([torch.tensor([N - 1, N - 2]),
                      torch.from_numpy(np.random.default_rng(0).integers(N // 2, N, 14))])
    for view, w, out in ((plan.fwd, norm.w_fwd, Y), (plan.bwd, norm.w_bwd, dH)):
        for r in rows.tolist():
            b, e = int(view.rowptr[r]), int(view.rowptr[r + 1])
            xs = X[view.col[b:e].long()].cpu().numpy()
            ww = w[b:e].cpu().numpy()
            acc = np.zeros(F, dtype=np.float32)
            for k in range(e - b):
                acc = (acc + (xs[k] * ww[k]).astype(np.float32)).astype(np.float32)
            np.testing.assert_array_equal(out[r].cpu().numpy(), acc)


@pytest.mark.parametrize("M,K,N,tw", [(286_214, 1, 64, False), (286_214, 2, 32, True),
                                      (1000, 8, 7, False), (3, 5, 128, True), (7, 3, 5, True),
                                      (0, 2, 4, False)])
def test_gemm_small_k_matches_fp64(cuda, M, K, N, tw):
    """mgcn_gemm_small_k (the 1 -> F input layer, the F -> 2 projection's dX):
    within fp32 rounding of fp64 (k-ordered fma); K = 1 is the single product
    bit for bit."""
    from mgcn.ops import gemm_small_k
    g = torch.Generator(device=cuda).manual_seed(M + K + N)
    A = torch.randn(M, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g) if tw else \
        torch.randn(K, N, device=cuda, generator=g)
    C = gemm_small_k(A, W, transpose_w=tw)
    Wm = W.t() if tw else W
    ref = A.double() @ Wm.double()
    bound = A.double().abs() @ Wm.double().abs()
    assert C.shape == (M, N)
    assert ((C.double() - ref).abs() <= 2e-7 * K * bound + 1e-30).all()
    if K == 1:
        assert torch.equal(C, A * Wm)
