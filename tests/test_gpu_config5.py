"""Config 5 at its own size under ``pytest -m gpu`` (BASELINE.json configs[4]:
N = 50M nodes, 250M random pairs symmetrised to E = 500M edges + 50M
self-loops, F = 256, 3 GCN layers 256 -> 256 ('sm', 'add', bias, ReLU between),
destination-range sharded over 8 ranks).

The 8-GPU run is the driver's, not ours; what one GPU can check is a rank's
whole share: ``build_shard(emulate=(r, 8))`` builds rank r's shard of the full
graph in this process (its destination rows' in-edges and its source rows'
out-edges, columns remapped to the exchange table, the norms from the global
out-degrees), and the product step (:class:`mgcn.dist.ShardedGCN`, the fused
256-wide kernels) runs forward + backward to every weight and bias with the
exchange tables resident (no RCCL: the emulated exchange writes the rank's own
rows, dense, or packs and unpacks them at all 8 positions, packed).  Ranks 0
and 7 (7: the ragged last row chunk), dense and packed exchange.

Every local kernel call of the step goes through a checking backend that
compares it, at the tables it actually read, with a host-independent fp64
restatement of the reference layer (gcn_base_models.py:65-146 for the norm,
:201 and :223-241 for the layer, its autograd adjoints):

  * forward Y = relu((A X) W + b): one window of 1,024 destination rows per
    row chunk and layer (12 windows = 12,288 rows per run), the norm rebuilt
    from the global out-degrees in fp64, table positions mapped back to global
    node ids, within 1e-5 x the |.| bound (|A| |X| |W| + |b|) -- north_star's
    1e-5 relative fp32 bar;
  * adjoint dX = relu'(lower) ((A^T dY) W^T): one window of 1,024 source
    rows per chunk and layer (8 windows), same bound;
  * dW = Z^T dY over ALL of the rank's 6.2M rows (the forward's own Z and the
    step's dY) against fp64, within 1e-5 x |Z|^T |dY| (bf16x6 products, fp32
    split-K accumulation over 6.2M rows; measured worst 0.09 of that bound);
  * db: the top layer's (column sums of dY) and the lower layers' (column sums
    of the masked dX, accumulated over the chunks on the device) against fp64
    sums of the same rows, within 1e-5 x the sums of |.|.

The reference itself is single-device (src/run/train_botnet.py:219); the
sharded layout is SURVEY.md §8(e).  Needs ~210 GB of HBM (one MI355X: 288 GB).
"""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N_NODES, N_PAIRS, FEAT, LAYERS, WORLD = 50_000_000, 250_000_000, 256, 3, 8
WIN = 1024
TOL = 1e-5
TOL_DW = 1e-5


def _global_ids(t, sh):
    """exchange-table positions -> global node ids (mgcn.dist.table_positions
    inverted): t = c P cr + k cr + (i - c cr)."""
    P, cr = sh.world, sh.chunk_rows
    c = torch.div(t, P * cr, rounding_mode="floor")
    k = torch.div(t - c * P * cr, cr, rounding_mode="floor")
    i = c * cr + (t - c * P * cr - k * cr)
    b = torch.tensor(sh.bounds, dtype=torch.int64, device=t.device)
    return b[k] + i


def _mask_bits(rm, F):
    """[rows, F/32] int32 ReLU mask words (fused_wide.hip layout: feature f
    at word 4 (f >> 7) + (f & 3), bit (f & 127) >> 2) -> bool [rows, F]."""
    f = torch.arange(F, device=rm.device)
    word = 4 * (f >> 7) + (f & 3)
    bit = (f & 127) >> 2
    return ((rm.long()[:, word] >> bit) & 1).bool()


def _packed_rows(tab, s_, i_):
    """Rows i_ of segments s_ of a PackedTable, decoded from the buffers in
    torch (pack.hip layout: row i's header pairs (mask_w, pos_w) at words
    2 W i .. of its segment, its values at head + pos_0 ..)."""
    F, W = tab.F, tab.F // 32
    head = 2 * W * tab.seg_rows
    out = torch.zeros(s_.numel(), F, dtype=torch.int32, device=s_.device)
    seg_buf = torch.tensor(tab.seg_buf, device=s_.device)
    seg_off = torch.tensor(tab.seg_off, dtype=torch.int64, device=s_.device)
    for bi, buf in enumerate(tab.bufs):
        sel = torch.nonzero(seg_buf[s_] == bi).view(-1)
        if sel.numel() == 0:
            continue
        base = seg_off[s_[sel]]
        h = base.view(-1, 1) + 2 * W * i_[sel].view(-1, 1) + torch.arange(2 * W, device=s_.device)
        hdr = buf[h].to(torch.int64) & 0xFFFFFFFF
        bits = ((hdr[:, 0::2].unsqueeze(-1) >> torch.arange(32, device=s_.device)) & 1).bool()
        bits = bits.view(-1, F)
        rank = torch.cumsum(bits.long(), 1) - 1
        idx = base.view(-1, 1) + head + hdr[:, 1:2] + rank
        vals = buf[torch.where(bits, idx, torch.zeros_like(idx))]
        out[sel] = torch.where(bits, vals, torch.zeros_like(vals))
    return out.view(torch.float32)


class _Checks:
    def __init__(self):
        self.worst = {}
        self.rows = {}

    def add(self, kind, ratio, rows=0):
        self.worst[kind] = max(self.worst.get(kind, 0.0), float(ratio))
        self.rows[kind] = self.rows.get(kind, 0) + rows


def _checking_backend(dinv, rng):
    from mgcn.dist import HipBackend

    class CheckingBackend(HipBackend):
        """HipBackend whose every local call is checked against fp64."""
        sh = None
        checks = _Checks()
        colsum64 = None

        def _window(self, view, w_parent_rowptr):
            a = (view.rowptr.data_ptr() - w_parent_rowptr.data_ptr()) // 8  # chunk's first row
            n = view.n_rows
            o = int(rng.integers(0, max(n - WIN, 0) + 1))
            return a, o, min(o + WIN, n)

        def _agg64(self, view, tab, a, o, e):
            """fp64 (A tab) for rows [o, e) of the chunk view and its |A| |tab|."""
            sh = self.sh
            rp = view.rowptr[o:e + 1].to(torch.int64)
            s0, s1 = int(rp[0]), int(rp[-1])
            cols = view.col[s0:s1].to(torch.int64)
            deg = rp[1:] - rp[:-1]
            row_of = torch.repeat_interleave(torch.arange(e - o, device=cols.device), deg)
            me = sh.lo + a + o + row_of
            if isinstance(tab, torch.Tensor):
                other = _global_ids(cols, sh)
                g = tab[cols].to(torch.float64)
            else:  # a packed table gathered in place: rows decoded from the segments
                s_ = cols >> tab.row_bits
                i_ = cols & ((1 << tab.row_bits) - 1)
                other = _global_ids(s_ * tab.seg_rows + i_, sh)
                g = _packed_rows(tab, s_, i_).to(torch.float64)
            w64 = dinv[me] * dinv[other]
            agg = torch.zeros(e - o, g.size(1), dtype=torch.float64, device=g.device)
            agg.index_add_(0, row_of, g * w64[:, None])
            absg = torch.zeros_like(agg).index_add_(0, row_of, g.abs() * w64.abs()[:, None])
            return agg, absg

        def spmm_xw_fwd(self, view, w, tab, W, reduce, b, relu, relu_mask=None, want_z=False,
                        out=None, z_out=None):
            res = super().spmm_xw_fwd(view, w, tab, W, reduce, b, relu, relu_mask=relu_mask,
                                      want_z=want_z, out=out, z_out=z_out)
            Y = res[0] if want_z else res
            a, o, e = self._window(view, self.sh.fwd.rowptr)
            agg, absg = self._agg64(view, tab, a, o, e)
            W64 = W.detach().double()
            ref = agg @ W64 + b.detach().double()
            bound = absg @ W64.abs() + b.detach().double().abs()
            if relu:
                ref = torch.relu(ref)
            err = (Y[o:e].double() - ref).abs()
            self.checks.add("fwd", (err / (TOL * bound + 1e-30)).max(), e - o)
            if want_z:  # Z = A X of the same rows, the dW pass's operand
                zerr = (z_out[o:e].double() - agg).abs()
                self.checks.add("z", (zerr / (TOL * absg + 1e-30)).max())
            return res

        def spmm_xw_bwd_dx(self, view_t, w_t, row_scale, dY, W, relu_mask=None, row_div=None,
                           out=None, colsum=None):
            res = super().spmm_xw_bwd_dx(view_t, w_t, row_scale, dY, W, relu_mask=relu_mask,
                                         row_div=row_div, out=out, colsum=colsum)
            a, o, e = self._window(view_t, self.sh.bwd.rowptr)
            agg, absg = self._agg64(view_t, dY, a, o, e)
            W64 = W.detach().double()
            ref = agg @ W64.t()
            bound = absg @ W64.abs().t()
            if relu_mask is not None:
                keep = _mask_bits(relu_mask[o:e], W.size(0))
                ref = torch.where(keep, ref, torch.zeros_like(ref))
            err = (out[o:e].double() - ref).abs()
            self.checks.add("dx", (err / (TOL * bound + 1e-30)).max(), e - o)
            if colsum is not None:  # fp64 column sums of the device's dX rows, all chunks
                d = out.double()
                s, sa = d.sum(0), d.abs().sum(0)
                if self.colsum64 is None:
                    self.colsum64 = [s, sa, colsum]
                else:
                    self.colsum64[0] += s
                    self.colsum64[1] += sa
            return res

        def gemm_bwd_dw(self, Z, dY, W, dh_colsum=False):
            if self.colsum64 is not None:  # the lower layer's db, complete now
                s, sa, dev = self.colsum64
                self.checks.add("db", ((dev.double() - s).abs() / (TOL * sa + 1e-30)).max())
                self.colsum64 = None
            dW, cs = super().gemm_bwd_dw(Z, dY, W, dh_colsum=dh_colsum)
            ref = torch.zeros(Z.size(1), dY.size(1), dtype=torch.float64, device=Z.device)
            bound = torch.zeros_like(ref)
            for r0 in range(0, Z.size(0), 1 << 20):
                z = Z[r0:r0 + (1 << 20)].double()
                y = dY[r0:r0 + (1 << 20)].double()
                ref += z.t() @ y
                bound += z.abs().t() @ y.abs()
                del z, y
            self.checks.add("dw", ((dW.double() - ref).abs() / (TOL_DW * bound + 1e-30)).max(),
                            Z.size(0))
            if dh_colsum:
                d = dY.double()
                self.checks.add("db", ((cs.double() - d.sum(0)).abs() /
                                       (TOL * d.abs().sum(0) + 1e-30)).max())
            return dW, cs

    return CheckingBackend()


@pytest.fixture(scope="module")
def config5(cuda):
    props = torch.cuda.get_device_properties(cuda)
    if props.total_memory < 250e9:
        pytest.skip(f"config 5's rank needs ~210 GB of HBM ({props.total_memory / 1e9:.0f} GB here)")
    g = torch.Generator(device=cuda).manual_seed(0)
    s = torch.randint(0, N_NODES, (N_PAIRS,), device=cuda, generator=g)
    d = torch.randint(0, N_NODES, (N_PAIRS,), device=cuda, generator=g)
    loops = torch.arange(N_NODES, device=cuda)
    ei = torch.stack([torch.cat([s, d, loops]), torch.cat([d, s, loops])])
    del s, d, loops
    odeg = torch.bincount(ei[0], minlength=N_NODES).to(torch.float64)
    dinv = odeg.pow(-0.5)
    dinv[torch.isinf(dinv)] = 0.0
    del odeg
    gw = torch.Generator().manual_seed(2)
    gb = torch.Generator().manual_seed(3)
    a = (6.0 / (2 * FEAT)) ** 0.5
    Ws = [torch.rand(FEAT, FEAT, generator=gw) * (2 * a) - a for _ in range(LAYERS)]
    bs = [torch.rand(FEAT, generator=gb) * 0.2 - 0.1 for _ in range(LAYERS)]
    yield ei, dinv, Ws, bs
    del ei, dinv
    torch.cuda.empty_cache()


@pytest.mark.parametrize("rank", [0, 7])
def test_config5_rank_fp64(cuda, config5, rank):
    from mgcn import dist as mdist
    from mgcn.dist import ShardedGCN
    ei, dinv, Ws, bs = config5
    be = _checking_backend(dinv, np.random.default_rng(100 + rank))
    model = ShardedGCN(ei, N_NODES, Ws, bs, device=cuda, chunks=4, backend=be,
                       emulate=(rank, WORLD))
    sh = model.shard
    be.sh = sh
    assert model.fused, "config 5's 256-wide layers must run on the fused kernels"
    assert sh.rows > 6_000_000 and sh.world == WORLD
    if rank == WORLD - 1:  # the ragged last chunk
        assert sh.rows < sh.pad_rows
    g = torch.Generator(device=cuda).manual_seed(rank)
    Xt = torch.randn(sh.table_rows, FEAT, device=cuda, generator=g)
    dYl = torch.randn(sh.rows, FEAT, device=cuda, generator=g)
    step = model.step_fn(None, None, X_table=Xt, dY_local=dYl)
    try:
        for packed in (False, True):
            sh._tables = None  # (the dense run's persistent tables: freed before the packed run)
            torch.cuda.empty_cache()
            mdist.set_pack_exchange(packed)
            be.checks = _Checks()
            mdist.STATS.update(dense_words=0, sent_words=0)
            step()
            torch.cuda.synchronize()
            ck = be.checks
            print(f"rank {rank} packed={packed}: worst err/bound "
                  f"{ {k: round(v, 4) for k, v in ck.worst.items()} }, rows {ck.rows}, "
                  f"packed ratio {mdist.STATS['sent_words'] / max(mdist.STATS['dense_words'], 1):.3f}")
            assert ck.rows["fwd"] >= 3 * WIN and ck.rows["dx"] >= 3 * WIN
            assert ck.rows["dw"] == LAYERS * sh.rows
            for kind in ("fwd", "z", "dx", "dw", "db"):
                assert ck.worst[kind] <= 1.0, (kind, ck.worst[kind])
            if packed:  # ReLU'd tables really travelled packed
                assert 0 < mdist.STATS["sent_words"] < 0.75 * mdist.STATS["dense_words"]
            for p in model.params():
                assert p.grad is not None and torch.isfinite(p.grad).all()
    finally:
        mdist.set_pack_exchange("auto")
        be.sh = None
        del step, Xt, dYl, model, sh
        torch.cuda.empty_cache()
