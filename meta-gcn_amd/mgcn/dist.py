"""Destination-range sharding of the GCN aggregation over torch.distributed.

The reference is single-device; north_star asks for the
edge list to be sharded by destination-node range across the GPUs of a node
with an RCCL exchange of node embeddings over xGMI.  Design (SURVEY.md §8(e),
DESIGN.md §7):

* nodes are split into P contiguous ranges balanced on (in-edges + rows),
  from a global in-degree count (no sort of the global graph); rank k owns
  rows [lo_k, hi_k) of X, of every layer's output and of dX;
* every rank filters the COO list once for the edges INTO its rows (the fwd
  view, rows = its destinations) and OUT OF its rows (the bwd view, rows = its
  sources) and sorts only those (stable, so each row keeps COO order and the
  sums stay bit-identical to one device); degrees of its sources are summed
  locally and the inverse degrees all-gathered once;
* exchange layout: row i of rank k lives at ``c*P*cr + k*cr + (i - c*cr)``
  of a [C*P*cr, F] table, c = i // cr (C row chunks of cr rows).  A layer's
  output is produced chunk by chunk and each chunk's all-gather
  (``all_gather_into_tensor`` of cr rows, RCCL over xGMI) is issued as soon as
  the chunk is written, so it runs while the next chunk is computed; the
  column indices of both views are remapped once to table positions, so the
  kernels read the gathered table in place;
* forward, per layer: the fused aggregate-then-transform kernel
  (mgcn_spmm_xw_fwd) over the rank's destinations reads the table of the
  layer's input (layer 0: the replicated input features, no exchange);
* backward, per layer: the upstream dY rows are all-gathered (chunked, as
  they are produced by the layer above) while dW = Z_k^T dY_k runs on local
  data (the forward kept Z_k = the rank's aggregate); then the dX-only gather
  kernel (mgcn_spmm_xw_bwd, X = NULL) over the rank's sources, with the lower
  layer's ReLU mask / mean divisor / bias column sums in its epilogue;
* replicated parameters: one bucketed all_reduce of every weight / bias
  gradient per step;
* zero-skipping exchange: the tables exchanged between layers are ReLU
  outputs (forward) or gradients masked by the same ReLU (backward), about
  half +0.0 words.  Such a chunk travels packed (libmgcn mgcn_pack_rows_*:
  per-row offsets, nonzero bit masks, the nonzero words) and is expanded in
  place on arrival (mgcn_unpack_rows), bit for bit; the ranks first
  all-gather their packed sizes so every rank sends the same buffer length,
  and a chunk whose largest packed form is no smaller than the dense one goes
  dense (:class:`_ChunkExchange`).

Layers the fused kernels do not take (max, F not 128 / 256, heavy rows,
128-wide tables past 4 GiB) run per layer: H_k = X_k W, all-gather H, the aggregation SpMM over the
rank's destinations; adjoint: all-gather dY (and argmax for max), the adjoint
SpMM over the rank's sources.

Forward rows and dX rows are bitwise equal to one device; parameter
gradients are all-reduced partial sums (fp32 tolerance).  The local compute
goes through a backend object (default :class:`HipBackend`, libmgcn); tests
substitute a CPU double (tests/cpu_backend.py) under gloo.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _lib as L
from .graph import CSRView


class HipBackend:
    """Local compute on libmgcn (the only production backend)."""

    def build_view(self, key, other, n_key, n_other):
        from .graph import build_view
        return build_view(key, other, n_key, n_other, schedule=False)

    def degree_norm(self, n, bwd, deg, ew, code):
        from .graph import degree_norm
        return degree_norm(n, bwd, deg, ew, code)

    def edge_norm(self, view, rows_are_dst, dinv, ew, code):
        from .graph import edge_norm
        return edge_norm(view, rows_are_dst, dinv, ew, code)

    def finalize_view(self, view):
        from .graph import schedule_rows
        return schedule_rows(view)

    def fused_ok(self, shard, F_in, F_out, reduce):
        from .ops import dw_pass_supported, spmm_xw_supported
        return (spmm_xw_supported(shard.fwd, F_in, F_out, reduce) and
                spmm_xw_supported(shard.bwd, F_out, F_in, L.REDUCE_SUM) and
                dw_pass_supported(F_in, F_out))

    def spmm_xw_fwd(self, *a, **k):
        from .ops import spmm_xw_fwd
        return spmm_xw_fwd(*a, **k)

    def spmm_xw_bwd_dx(self, view_t, w_t, row_scale, dY, W, relu_mask=None, row_div=None,
                       out=None, colsum=None):
        """dX only (X = NULL): returns the lower layer's bias column sums or
        None; with ``colsum`` (and relu_mask) they are added into it on the
        device instead."""
        from .ops import spmm_xw_bwd
        return spmm_xw_bwd(view_t, w_t, row_scale, dY, None, W, relu_mask=relu_mask,
                           row_div=row_div, dx_out=out, colsum_acc=colsum)[2]

    def gemm_bwd_dw(self, Z, dY, W, dh_colsum=False):
        from .ops import dw_pass
        return dw_pass(Z, dY, W, dh_colsum=dh_colsum)

    def mask_words(self, F):
        from .ops import mask_words
        return mask_words(F)

    def pack_count(self, rows, hdr, counts):
        from .ops import pack_rows_count
        pack_rows_count(rows, hdr, counts)

    def pack_values(self, rows, offs, hdr, vals):
        from .ops import pack_rows_values
        pack_rows_values(rows, offs, hdr, vals)

    def pack_rows(self, rows, hdr, vals, total):
        from .ops import pack_rows
        pack_rows(rows, hdr, vals, total)

    def pack_rows_ok(self, F):
        from .ops import PACK_ROWS_WIDTHS
        return F in PACK_ROWS_WIDTHS

    def packed_gather_ok(self, F):
        """The fused layer kernels of width F gather packed tables in place
        (mgcn_spmm_xw_fwd_packed / _bwd_packed: F = 128 and 256)."""
        return F in (128, 256)

    def unpack(self, buf, n_seg, n, seg_words, out):
        from .ops import unpack_rows
        unpack_rows(buf, n_seg, n, seg_words, out)

    def spmm_fwd(self, *a, **k):
        from .ops import spmm_fwd
        return spmm_fwd(*a, **k)

    def spmm_bwd(self, *a, **k):
        from .ops import spmm_bwd
        return spmm_bwd(*a, **k)

    def relu_bwd_colsum(self, *a, **k):
        from .ops import relu_bwd_colsum
        return relu_bwd_colsum(*a, **k)

    def linear(self, x, W):
        from .ops import linear
        return linear(x, W)


def partition_nodes(rowptr: torch.Tensor, parts: int) -> list[int]:
    """Contiguous node ranges with ~equal (in-edges + rows) per part;
    ``rowptr`` is the cumulative in-degree ([N + 1], rowptr[0] = 0)."""
    rp = rowptr.to("cpu", torch.int64)
    n = rp.numel() - 1
    cost = rp + torch.arange(n + 1, dtype=torch.int64)  # cumulative cost up to row i
    total = int(cost[-1])
    bounds = [0]
    for k in range(1, parts):
        target = total * k // parts
        b = int(torch.searchsorted(cost, torch.tensor(target), right=False))
        bounds.append(max(bounds[-1], min(b, n)))
    bounds.append(n)
    return bounds


def table_positions(ids: torch.Tensor, bounds, chunk_rows: int) -> torch.Tensor:
    """Global node id -> row of the exchange table (module docstring)."""
    world = len(bounds) - 1
    b = torch.tensor(bounds, dtype=torch.int64, device=ids.device)
    g = ids.to(torch.int64)
    owner = torch.bucketize(g, b[1:], right=True)
    i = g - b[owner]
    c = torch.div(i, chunk_rows, rounding_mode="floor")
    return c * (world * chunk_rows) + owner * chunk_rows + (i - c * chunk_rows)


@dataclass
class Shard:
    rank: int
    world: int
    bounds: list
    lo: int
    hi: int
    max_rows: int
    chunks: int          # C
    chunk_rows: int      # cr
    fwd: CSRView         # rows = my destinations, col = table positions of the sources
    bwd: CSRView         # rows = my sources, col = table positions of the destinations
    w_fwd: torch.Tensor | None
    w_bwd: torch.Tensor | None
    row_scale: torch.Tensor | None   # RW without edge weights: dinv of my sources
    in_cnt: torch.Tensor             # max(in-degree, 1) of my rows (MEAN)
    cnt_table: torch.Tensor          # the same for every node, table layout (MEAN adjoint)
    chunk_edges_fwd: list            # edges of each row chunk (host ints, byte accounting)
    chunk_edges_bwd: list
    # emulated rank (one process standing in for rank `rank` of `world`, no
    # collectives): the exchange tables are persistent buffers whose other
    # ranks' rows are left as they are -- the rank-local compute of the
    # sharded step timed on one GPU (scripts/config5_rank.py)
    emulated: bool = False
    _tables: dict = None
    _pk_views: tuple = None
    # packed exchange: the largest packed value count over the ranks of each
    # (exchange, row chunk) at its last exchange (identical on every rank:
    # it comes from the all-gathered sizes) -- the next exchange's capacity
    cap_hint: dict = None

    def packed_views(self):
        """(fwd, bwd, row_bits): the two views with their columns as packed
        positions (segment << row_bits) | row -- the addresses of the
        in-place gather from a :class:`mgcn.ops.PackedTable` (built once)."""
        if self._pk_views is None:
            from .ops import packed_cols, packed_row_bits
            rb = packed_row_bits(self.chunk_rows)
            views = []
            for v in (self.fwd, self.bwd):
                views.append(CSRView(rowptr=v.rowptr, col=packed_cols(v.col, self.chunk_rows, rb),
                                     eid=v.eid, n_rows=v.n_rows, n_cols=v.n_cols,
                                     n_edges=v.n_edges))
            self._pk_views = (views[0], views[1], rb)
        return self._pk_views

    def view_for(self, table, which: str, a: int, e: int, n_edges: int):
        """Rows [a, e) of the fwd / bwd view addressing `table` (dense or packed)."""
        if isinstance(table, torch.Tensor):
            v = self.fwd if which == "fwd" else self.bwd
        else:
            f, b, _ = self.packed_views()
            v = f if which == "fwd" else b
        return v.rows(a, e, n_edges)

    @property
    def rows(self) -> int:
        return self.hi - self.lo

    @property
    def table_rows(self) -> int:
        return self.chunks * self.world * self.chunk_rows

    @property
    def pad_rows(self) -> int:
        return self.chunks * self.chunk_rows

    def chunk(self, c: int):
        a = c * self.chunk_rows
        return a, max(a, min(a + self.chunk_rows, self.rows))

    def to_table(self, full: torch.Tensor) -> torch.Tensor:
        """A replicated [N, ...] tensor in the exchange layout (setup only)."""
        n = self.bounds[-1]
        pos = table_positions(torch.arange(n, device=full.device), self.bounds, self.chunk_rows)
        out = torch.zeros((self.table_rows,) + tuple(full.shape[1:]), dtype=full.dtype,
                          device=full.device)
        out[pos] = full
        return out

    def local_rows(self, full: torch.Tensor) -> torch.Tensor:
        return full[self.lo:self.hi]


# Run every collective of the sharded path even in a one-rank group
# (set_force_collectives / env MGCN_FORCE_COLLECTIVES=1): the RCCL calls --
# the chunked all_gather_into_tensor(async_op=True), the packed exchange's
# size gather and payload, the bucketed all_reduce -- then execute on one GPU
# exactly as a rank of a multi-GPU group issues them
# (tests/test_gpu_rccl.py); by default world 1 copies instead.
FORCE_COLLECTIVES = os.environ.get("MGCN_FORCE_COLLECTIVES", "0") != "0"


def set_force_collectives(enabled: bool) -> None:
    global FORCE_COLLECTIVES
    FORCE_COLLECTIVES = bool(enabled)


def _collective(world: int) -> bool:
    """True when a group of ``world`` ranks exchanges through torch.distributed."""
    return world > 1 or (FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized())


def _all_gather_flat(local: torch.Tensor, n_pad: int, world: int, group=None) -> torch.Tensor:
    """[n, ...] per rank (n <= n_pad) -> [world * n_pad, ...] rank-major."""
    buf = torch.zeros((n_pad,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[:local.size(0)] = local
    if not _collective(world):
        return buf
    out = torch.empty((world * n_pad,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    _gather_into(out, buf, world, group, False)
    return out


def _gather_into(out, inp, world, group, async_op):
    if not _collective(world):
        out.copy_(inp)
        return None
    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    return dist.all_gather(list(out.chunk(world)), inp, group=group, async_op=async_op)


def _gather_chunk(shard: Shard, c: int, local_pad: torch.Tensor, table: torch.Tensor, group):
    """Issue the all-gather of row chunk c (async); returns the work or None.
    Emulated rank: only this rank's slice of the chunk is written."""
    cr, P = shard.chunk_rows, shard.world
    if shard.emulated:
        a = c * P * cr + shard.rank * cr
        table[a:a + cr].copy_(local_pad[c * cr:(c + 1) * cr])
        return None
    return _gather_into(table[c * P * cr:(c + 1) * P * cr], local_pad[c * cr:(c + 1) * cr], P,
                        group, True)


def new_table(shard: Shard, F: int, dtype, device, slot: str) -> torch.Tensor:
    """An exchange table [C*P*cr, F]: a fresh buffer, or (emulated rank) the
    shard's persistent one for ``slot`` -- a rank-local timing of the
    sharded step must not allocate 51 GB per layer where the real step
    receives it from its peers.  The stack's forward and backward share the
    two slots "t0" / "t1" (a forward table is dead once the next layer has
    read it), so an emulated config-5 rank holds the input and two tables."""
    if not shard.emulated:
        return torch.empty(shard.table_rows, F, dtype=dtype, device=device)
    if shard._tables is None:
        shard._tables = {}
    key = (slot, F, dtype, str(device))
    t = shard._tables.get(key)
    if t is None:
        t = torch.zeros(shard.table_rows, F, dtype=dtype, device=device)
        shard._tables[key] = t
    return t


_SIZE_STREAMS = {}


def _size_stream(dev):
    """Side stream (per device) of the packed exchange's size read-back."""
    st = _SIZE_STREAMS.get(dev.index)
    if st is None:
        st = torch.cuda.Stream(device=dev)
        _SIZE_STREAMS[dev.index] = st
    return st


def _wait(works):
    for w in works or ():
        if w is not None:
            w.wait()


PACK_EXCHANGE = "auto"  # mgcn.dist.set_pack_exchange
PACK_AUTO_MAX_WORLD = 4
# words a dense exchange would have received vs words sent, over every packed
# exchange of this process (bench / scripts/config5_rank.py report the ratio)
STATS = {"dense_words": 0, "sent_words": 0}


def set_pack_exchange(enabled) -> None:
    """Zero-skipping (packed) exchange of the ReLU'd tables of the sharded
    stack: True / False, or "auto" (the default).  Packing about halves the
    words on xGMI.  Where the next layer's fused kernel gathers packed tables
    in place (F = 128 / 256, round 6: no unpack pass) "auto" packs row chunks
    of at least PACK_AUTO_MIN_CHUNK_BYTES (smaller ones cost more in launches
    than they save on the links); elsewhere the received segments are
    expanded into the dense table first (mgcn_unpack_rows), a pass that
    writes the received (P - 1)/P of every table, and "auto" packs only up to
    PACK_AUTO_MAX_WORLD ranks (the link time a table saves shrinks as 1/P
    while that pass grows)."""
    global PACK_EXCHANGE
    PACK_EXCHANGE = enabled if enabled == "auto" else bool(enabled)


# mgcn.dist.set_pack_inplace: gather packed tables in place where the kernels
# can (True, the default) or always expand them (False: the round-5 path, A/B)
PACK_INPLACE = os.environ.get("MGCN_PACK_INPLACE", "1") != "0"


def set_pack_inplace(enabled: bool) -> None:
    global PACK_INPLACE
    PACK_INPLACE = bool(enabled)


# Speculative capacity (round 6).  An all-gather moves equal sizes, so a
# packed chunk is sent at the largest packed size over the ranks; the first
# exchange of a table learns that size on the host (one event wait per chunk,
# one chunk behind).  Every later exchange of the same (layer, direction,
# chunk) sends at the size the last one saw plus SPEC_SLACK, issuing the
# payload right behind the pack with no host wait; the all-gathered sizes are
# checked once per table, when the next layer asks for it (one host sync per
# table instead of one per chunk), and a chunk whose size outgrew its
# capacity on some rank is all-gathered again at its true size before anything
# reads it -- the same bits either way.  set_spec_exchange(False): round 5's
# per-chunk form always.
SPEC_EXCHANGE = os.environ.get("MGCN_SPEC_EXCHANGE", "1") != "0"
SPEC_SLACK = 0.02  # capacity = last size x (1 + SLACK) + 64 words (tests set it below 0)


def set_spec_exchange(enabled: bool) -> None:
    global SPEC_EXCHANGE
    SPEC_EXCHANGE = bool(enabled)


# Single-pass pack (round 6): where the backend has it (mgcn_pack_rows, F in
# 32 / 64 / 128 / 256) a chunk is packed in one read of its rows, its value
# count left on the device -- no count pass, no scan of the counts, the pack
# done before the sizes are exchanged.  set_fused_pack(False): the two passes.
FUSED_PACK = os.environ.get("MGCN_FUSED_PACK", "1") != "0"
# ... for chunks of at least this many bytes: a small chunk has fewer tiles
# than the GPU has CUs and its look-back costs more than the second read
# (config 2 at P = 8, 31k x 128 rows: 27 vs 22 us; 125k x 128: 57 vs 74 us)
FUSED_PACK_MIN_BYTES = 32 << 20


def set_fused_pack(enabled: bool) -> None:
    global FUSED_PACK
    FUSED_PACK = bool(enabled)


def _spec_cap(true_words: int, limit: int) -> int:
    c = int(true_words * (1.0 + SPEC_SLACK)) + (64 if SPEC_SLACK >= 0 else 0)
    return max(0, min(c, limit))


def _single_recv_words(shard: Shard, F: int) -> int:
    """Words of the one receive buffer an F = 128 in-place table lives in:
    every row chunk's P segments at dense capacity (header + cr F words)."""
    cr = shard.chunk_rows
    return shard.chunks * shard.world * (2 * cr * (F // 32) + cr * F) + 4


def _inplace_ok(shard: Shard, backend, F: int) -> bool:
    """In place: at most 64 segments; at F = 128 (whose kernels address the
    whole table through one 32-bit range) a table whose single receive buffer
    spans at most 2 GiB - 16 B."""
    return PACK_INPLACE and getattr(backend, "packed_gather_ok", lambda f: False)(F) and \
        shard.chunks * shard.world <= 64 and \
        (F != 128 or _single_recv_words(shard, F) * 4 <= 0x7ffffff0)


# "auto" packs an in-place table only when its row chunks are at least this
# big: a packed chunk costs a fixed ~70 us of launches and host work (pack,
# sizes, payload), which small chunks do not earn back on the links (round 6,
# scripts/config5_rank.py at config 2's shape, one rank of P = 8, 16-MB
# chunks: 1.96 ms/step packed vs 1.14 dense, against 1.16 vs 1.67 ms of
# exchange; config 5's 1.6-GB chunks: 120 vs 108 ms against 110 vs 167)
PACK_AUTO_MIN_CHUNK_BYTES = 32 << 20


def _pack_on(shard: Shard, backend=None, F: int = 0) -> bool:
    if PACK_EXCHANGE == "auto":
        if backend is not None and _inplace_ok(shard, backend, F):
            return shard.chunk_rows * F * 4 >= PACK_AUTO_MIN_CHUNK_BYTES
        return shard.world <= PACK_AUTO_MAX_WORLD
    return bool(PACK_EXCHANGE)


class _ChunkExchange:
    """All-gathers the row chunks of one [rows, F] fp32 tensor into an
    exchange table, chunk by chunk as the caller produces them.  ``packed``:
    each chunk is packed (pack.hip's layout: per-row header pairs (mask_w,
    pos_w), then the nonzero words; libmgcn mgcn_pack_rows_*), the ranks
    all-gather their packed sizes, then send buffers of the largest size.
    The received segments are then either gathered IN PLACE by the next
    kernel (``inplace``: the result is a :class:`mgcn.ops.PackedTable` over
    the chunks' receive buffers, no dense table is ever written) or expanded
    into the dense table (mgcn_unpack_rows; a chunk whose largest packed form
    is not smaller than the dense chunk then goes dense) -- bit for bit the
    dense exchange either way.  The packed path needs each chunk's sizes on
    the host: :meth:`start` issues a chunk's pack and size exchange,
    :meth:`finish` (called one chunk later, so the GPU has the next chunk's
    compute queued while the host waits on an event) its payload.  Emulated
    rank: the rank's own segment stands in for all P (copied into the P
    positions of the receive buffer, or packed and unpacked at all P
    positions: the receive-side work of a real rank, with its own data; no
    collective runs)."""

    def __init__(self, shard: Shard, local_pad: torch.Tensor, table, group, backend,
                 packed: bool, inplace: bool = False, key=None):
        """``table``: the dense table, or a callable that allocates it (only
        called when some chunk goes dense).  ``key``: this exchange's place in
        the step (layer, direction), under which the shard keeps each chunk's
        packed size for the next step's speculative capacity (None: never
        speculate)."""
        self.sh, self.local, self.group, self.be = shard, local_pad, group, backend
        self._table = table
        F = local_pad.size(1)
        # (the packed form's value positions are int32, pack.hip: a chunk of
        # 2^31 words or more goes dense)
        self.packed = bool(packed) and local_pad.dtype == torch.float32 and F % 32 == 0 and \
            hasattr(backend, "pack_count") and (_collective(shard.world) or shard.emulated) and \
            shard.chunk_rows * F < 2 ** 31
        self.inplace = self.packed and bool(inplace)
        self.words = F // 32
        self.pending = []
        self.works = []
        self.stats = STATS
        self.recv = []      # inplace: the chunks' receive buffers
        self.seg = []       # inplace: words per segment of each chunk
        # inplace at F = 128: ONE receive buffer for every chunk (the kernels
        # address the table through one range), chunk c's segments from word
        # c P (header + cr F) on; self.base[c] = that word
        self.single = self.inplace and F == 128
        self.big = None
        self.base = []
        self.key = key
        self.spec = []      # speculative chunks: (c, rows, send, counts, totals, work, cap)
        self.spec_ev = []   # ... and (GPU) where each one's sizes are done
        if shard.cap_hint is None:
            shard.cap_hint = {}

    @property
    def table(self):
        if callable(self._table):
            self._table = self._table()
        return self._table

    def start(self, c: int) -> None:
        sh = self.sh
        if not self.packed:
            self.works.append(_gather_chunk(sh, c, self.local, self.table, self.group))
            return
        cr = sh.chunk_rows
        rows = self.local[c * cr:(c + 1) * cr]
        dev = rows.device
        head = 2 * cr * self.words
        # (+4 words: a lane's 16-B value read may run 3 words past the values)
        send = torch.empty(head + cr * rows.size(1) + 4, dtype=torch.int32, device=dev)
        F = rows.size(1)
        if FUSED_PACK and hasattr(self.be, "pack_rows") and self.be.pack_rows_ok(F) and \
                cr * F * 4 >= FUSED_PACK_MIN_BYTES:
            # packed here, once: counts None tells _payload the values are in
            counts = None
            self.stats["pack_one_pass"] = self.stats.get("pack_one_pass", 0) + 1
            total = torch.empty(1, dtype=torch.int64, device=dev)
            self.be.pack_rows(rows, send[:head].view(cr, 2 * self.words),
                              send[head:head + cr * F], total)
        else:
            counts = torch.empty(cr, dtype=torch.int32, device=dev)
            self.be.pack_count(rows, send[:head].view(cr, 2 * self.words), counts)
            total = counts.sum(dtype=torch.int64).view(1)
        P = sh.world
        if sh.emulated or not _collective(P):
            totals, work = total, None
        else:
            totals = torch.empty(P, dtype=torch.int64, device=dev)
            work = _gather_into(totals, total, P, self.group, True)
        # (in place only: a truncated segment is then read by nothing before
        # result() has re-sent it; the expanding path would unpack it at once.
        # An emulated rank takes it too: it times a real rank's later steps)
        hint = sh.cap_hint.get((self.key, c)) if (
            SPEC_EXCHANGE and self.inplace and self.key is not None) else None
        if hint is not None:
            # speculative: the payload goes right behind the pack at the
            # capacity the last exchange saw; result() checks the sizes.  (An
            # event marks where this chunk's sizes are done on the compute
            # stream: result() waits for those, not for the payloads queued
            # behind them.)
            if dev.type == "cuda":
                ev_sz = torch.cuda.Event()
                ev_sz.record()
                self.spec_ev.append(ev_sz)
            self._payload(c, rows, send, counts, hint)
            self.spec.append((c, rows, send, counts, totals, work, hint))
            self.stats["spec_chunks"] = self.stats.get("spec_chunks", 0) + 1
            return
        # the sizes reach the host through a side stream that waits only for
        # the size exchange: finish() then waits for THAT (an event), not for
        # everything queued on the compute stream after it (`.item()` on the
        # compute stream would drain the next chunk's kernels first, leaving
        # the GPU idle until the host queued more)
        host = ev = None
        if dev.type == "cuda":
            side = _size_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                if work is not None:
                    work.wait()
                host = torch.empty(totals.numel(), dtype=torch.int64, pin_memory=True)
                host.copy_(totals, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            totals.record_stream(side)
            work = None
        self.pending.append((c, rows, send, counts, totals, work, host, ev))

    def finish(self, keep: int = 0) -> None:
        """Issue the payloads of all started chunks but the last ``keep``."""
        while len(self.pending) > keep:
            self._finish_one(*self.pending.pop(0))

    def _finish_one(self, c, rows, send, counts, totals, work, host, ev):
        if ev is not None:
            ev.synchronize()  # the size exchange (and its copy) only
            cap = int(host.max())
        else:
            if work is not None:
                work.wait()
            cap = int(totals.max())
        if self.key is not None:
            self.sh.cap_hint[(self.key, c)] = _spec_cap(cap, self.sh.chunk_rows * rows.size(1))
        self._payload(c, rows, send, counts, cap)

    def _payload(self, c, rows, send, counts, cap, again=False):
        """Pack chunk c's values and issue its payload at ``cap`` value words
        per rank (``again``: a speculative chunk re-sent at its true size;
        its values are packed already)."""
        sh = self.sh
        cr, P, F = sh.chunk_rows, sh.world, rows.size(1)
        head = 2 * cr * self.words
        seg = head + cap
        if not again:
            self.stats["dense_words"] += cr * F * P
        if seg >= cr * F and not self.inplace:  # nothing to gain: dense
            self.stats["sent_words"] += cr * F * P
            self.works.append(_gather_chunk(sh, c, self.local, self.table, self.group))
            return
        self.stats["sent_words"] += seg * P
        if not again and counts is not None:
            offs = torch.cumsum(counts, 0, dtype=torch.int32)
            offs.sub_(counts)
            # every value (the send buffer holds a dense chunk's worth); the
            # first `cap` words travel
            self.be.pack_values(rows, offs, send[:head].view(cr, 2 * self.words),
                                send[head:head + cr * F])
        if self.single:
            dcap = head + cr * F
            if self.big is None:
                self.big = torch.empty(_single_recv_words(sh, F), dtype=torch.int32,
                                       device=rows.device)
                self.big[-4:].zero_()
            base = c * P * dcap
            if sh.emulated:  # the rank's own segment at chunk c's place, aliased P times
                self.big[base:base + seg].copy_(send[:seg])
                self._put(c, again, seg=0, base=base)
            else:
                _gather_into(self.big[base:base + P * seg], send[:seg], P, self.group, False)
                self._put(c, again, seg=seg, base=base)
            return
        if self.inplace:
            if sh.emulated:
                # the rank's own segment stands in for all P (its P positions
                # alias it): no collective and no copy -- the receive-side
                # write of a real rank is the exchange's, which
                # scripts/config5_rank.py accounts for separately
                self._put(c, again, seg=0, recv=send)
                return
            # P segments back to back (+4 words: a lane's 16-B value read may
            # run 3 words past the last segment's values)
            recv = torch.empty(P * seg + 4, dtype=torch.int32, device=rows.device)
            recv[P * seg:].zero_()
            _gather_into(recv[:P * seg], send[:seg], P, self.group, False)
            self._put(c, again, seg=seg, recv=recv)
            return
        blk = self.table[c * P * cr:(c + 1) * P * cr]
        if sh.emulated:  # a real rank's receive-side work: P segments unpacked
            for p in range(P):
                self.be.unpack(send[:seg], 1, cr, seg, blk[p * cr:(p + 1) * cr])
            return
        recv = torch.empty(P * seg, dtype=torch.int32, device=rows.device)
        _gather_into(recv, send[:seg], P, self.group, False)
        self.be.unpack(recv, P, cr, seg, blk)

    def _put(self, c, again, seg, base=None, recv=None):
        """Record chunk c's in-place segments (chunks are started in order;
        ``again`` replaces chunk c's record)."""
        if again:
            self.seg[c] = seg
            if recv is not None:
                self.recv[c] = recv
            return
        assert len(self.seg) == c, "chunks are exchanged in order"
        self.seg.append(seg)
        if base is not None:
            self.base.append(base)
        if recv is not None:
            self.recv.append(recv)

    def _check_spec(self) -> None:
        """One host sync for every speculative chunk of this exchange: their
        all-gathered sizes; a chunk that outgrew its capacity on some rank is
        sent again at its true size (every rank decides alike: the sizes are
        all-gathered); the hints follow the sizes."""
        if not self.spec:
            return
        tots = [t for *_, t, _w, _cap in self.spec]
        if self.spec_ev:
            # the sizes reach the host through the side stream, which waits
            # for them alone: the compute stream keeps running the payloads
            # (and whatever else is queued) while the host waits
            dev = tots[0].device
            side = _size_stream(dev)
            with torch.cuda.stream(side):
                for ev_sz in self.spec_ev:
                    side.wait_event(ev_sz)
                for *_, work, _cap in self.spec:
                    if work is not None:
                        work.wait()
                dsz = torch.stack([t.view(-1).max() for t in tots])
                host = torch.empty(dsz.numel(), dtype=dsz.dtype, pin_memory=True)
                host.copy_(dsz, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            for t in tots:
                t.record_stream(side)
            ev.synchronize()
            sizes = host
        else:
            for *_, work, _cap in self.spec:
                if work is not None:
                    work.wait()
            sizes = torch.stack([t.view(-1).max() for t in tots]).cpu()
        lim = self.sh.chunk_rows * self.local.size(1)
        for (c, rows, send, counts, totals, work, cap), true in zip(self.spec, sizes.tolist()):
            self.sh.cap_hint[(self.key, c)] = _spec_cap(int(true), lim)
            if true > cap:
                self.stats["spec_resent"] = self.stats.get("spec_resent", 0) + 1
                self._payload(c, rows, send, counts, int(true), again=True)
        self.spec = []
        self.spec_ev = []

    def wait(self) -> None:
        self.finish()
        self._check_spec()
        _wait(self.works)
        self.works = []

    def result(self):
        """The exchanged table: the dense table, or (inplace) the
        PackedTable over the chunks' receive buffers (segment c P + k = rank
        k's part of row chunk c, the exchange layout's order)."""
        self.wait()
        if not self.inplace:
            return self.table
        from .ops import PackedTable
        from .ops import packed_row_bits
        P = self.sh.world
        seg_buf, seg_off = [], []
        for c, sg in enumerate(self.seg):
            for k in range(P):
                # (emulated rank: sg = 0, all P alias its own)
                seg_buf.append(0 if self.single else c)
                seg_off.append((self.base[c] if self.single else 0) + k * sg)
        return PackedTable([self.big] if self.single else self.recv, seg_buf, seg_off,
                           self.sh.chunk_rows,
                           packed_row_bits(self.sh.chunk_rows), self.local.size(1))


def gather_table(shard: Shard, local: torch.Tensor, group=None, slot: str = "g") -> torch.Tensor:
    """My rows [rows, F] -> the exchange table [C*P*cr, F] on every rank."""
    pad = torch.empty((shard.pad_rows,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    pad[:shard.rows] = local
    if shard.pad_rows > shard.rows:
        pad[shard.rows:].zero_()
    if local.dim() == 2:
        table = new_table(shard, local.size(1), local.dtype, local.device, slot)
    else:
        table = torch.empty((shard.table_rows,) + tuple(local.shape[1:]), dtype=local.dtype,
                            device=local.device)
    _wait([_gather_chunk(shard, c, pad, table, group) for c in range(shard.chunks)])
    return table


def _local_view(backend, key, other, sel, lo, hi, n_other, bounds, cr, T):
    """CSR of the selected edges over global rows [0, hi) (rows < lo empty),
    eid = global COO ids; returned with the global columns (for the norms) and
    the finishing step that slices rows [lo, hi) and remaps the columns."""
    v = backend.build_view(key[sel], other[sel], hi, n_other)
    v.eid = sel[v.eid.long()].to(torch.int32)

    def finish():
        col = table_positions(v.col, bounds, cr).to(torch.int32)
        return CSRView(rowptr=v.rowptr[lo:].contiguous(), col=col, eid=v.eid, n_rows=hi - lo,
                       n_cols=T)
    return v, finish


def build_shard(edge_index: torch.Tensor, num_nodes: int, deg_norm="sm", deg=None,
                edge_weight=None, group=None, backend=None, device=None, chunks: int = 4,
                emulate=None) -> Shard:
    """One-time setup of this rank's part of the graph (module docstring).
    ``edge_index`` (and ``deg`` / ``edge_weight``) is the full graph on every
    rank; only the rank's own edges are sorted.  ``emulate=(rank, world)``:
    build rank ``rank`` of ``world`` in this one process without
    torch.distributed (the degrees that the real ranks all-gather are
    counted here over the whole graph; no exchange ever runs)."""
    backend = backend or HipBackend()
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                       for t in (edge_weight, deg)):
        # the shard's norms are built outside autograd (once per graph); the
        # single-device path (GraphPlan.norm) is the differentiable one
        raise NotImplementedError("build_shard: edge_weight / deg requiring grad is not supported "
                                  "on the sharded path (detach them, or use the single-device "
                                  "modules)")
    if emulate is not None:
        rank, world = (int(v) for v in emulate)
        if not 0 <= rank < world:
            raise ValueError(f"build_shard: emulate={emulate}")
    else:
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    if device is not None:
        edge_index = edge_index.to(device)
        deg = None if deg is None else deg.to(device)
        edge_weight = None if edge_weight is None else edge_weight.to(device)
    N = int(num_nodes)
    src, dst = edge_index[0].to(torch.int64), edge_index[1].to(torch.int64)
    dev = src.device
    in_deg = torch.bincount(dst, minlength=N)
    rowptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(in_deg, 0)
    bounds = partition_nodes(rowptr, world)
    lo, hi = bounds[rank], bounds[rank + 1]
    max_rows = max(max(bounds[k + 1] - bounds[k] for k in range(world)), 1)
    C = max(1, min(int(chunks), max_rows))
    cr = -(-max_rows // C)
    T = C * world * cr
    code = L.NORM_CODES[deg_norm]
    ew = None if edge_weight is None else edge_weight.reshape(-1).to(torch.float32).contiguous()
    if code == L.NORM_NONE or ew is not None:
        deg = None
    sel_f = torch.nonzero((dst >= lo) & (dst < hi)).view(-1)
    sel_b = torch.nonzero((src >= lo) & (src < hi)).view(-1)
    fwd_g, fwd_finish = _local_view(backend, dst, src, sel_f, lo, hi, N, bounds, cr, T)
    bwd_g, bwd_finish = _local_view(backend, src, dst, sel_b, lo, hi, N, bounds, cr, T)
    dinv = None
    if code != L.NORM_NONE:
        if deg is not None:  # given degrees (gcn_base_models.py:119-121): no exchange
            _, dinv = backend.degree_norm(N, None, deg.reshape(-1).to(torch.float32).contiguous(),
                                          None, code)
        elif emulate is not None:  # every rank's out-degrees, counted here
            if ew is not None:
                raise NotImplementedError("build_shard(emulate=...): edge weights")
            odeg = torch.bincount(src, minlength=N).to(torch.float32).contiguous()
            _, dinv = backend.degree_norm(N, None, odeg, None, code)
        else:  # out-degree of my sources over their complete rows, then all-gathered
            _, dl = backend.degree_norm(hi, bwd_g, None, ew, code)
            mine = _all_gather_flat(dl[lo:hi], max_rows, world, group)
            dinv = torch.cat([mine[k * max_rows:k * max_rows + bounds[k + 1] - bounds[k]]
                              for k in range(world)])
    row_scale = w_bwd = None
    if code == L.NORM_NONE and ew is None:
        w_fwd = None
    elif code == L.NORM_RW and ew is None:
        # x * dinv before the gather (gcn_base_models.py:217-220); the adjoint
        # post-scales by dinv of the source
        w_fwd = backend.edge_norm(fwd_g, True, dinv, None, code)
        row_scale = dinv[lo:hi].contiguous()
    else:
        w_fwd = backend.edge_norm(fwd_g, True, dinv, ew, code)
        w_bwd = backend.edge_norm(bwd_g, False, dinv, ew, code)
    fwd = backend.finalize_view(fwd_finish())
    bwd = backend.finalize_view(bwd_finish())
    cnt = in_deg.clamp(min=1).to(torch.float32)
    rp_f = fwd.rowptr.to("cpu")
    rp_b = bwd.rowptr.to("cpu")
    ce_f, ce_b = [], []
    for c in range(C):
        a = c * cr
        b = max(a, min(a + cr, hi - lo))
        ce_f.append(int(rp_f[b] - rp_f[a]) if b > a else 0)
        ce_b.append(int(rp_b[b] - rp_b[a]) if b > a else 0)
    sh = Shard(rank, world, bounds, lo, hi, max_rows, C, cr, fwd, bwd, w_fwd, w_bwd, row_scale,
               cnt[lo:hi].contiguous(), None, ce_f, ce_b, emulated=emulate is not None)
    sh.cnt_table = sh.to_table(cnt)
    return sh


# ------------------------------------------------------------ per-layer path
class _ShardedAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H_local, bias, shard: Shard, reduce: int, relu: bool, backend, group):
        Htab = gather_table(shard, H_local.contiguous(), group, slot="fwd")
        Y, argmax = backend.spmm_fwd(shard.fwd, shard.w_fwd, Htab, reduce, bias, relu)
        ctx.shard, ctx.reduce, ctx.relu, ctx.backend, ctx.group = shard, reduce, relu, backend, group
        ctx.has_bias = bias is not None
        ctx.save_for_backward(Y if relu else None, argmax)
        return Y

    @staticmethod
    def backward(ctx, dZ):
        Y, argmax = ctx.saved_tensors
        sh, be = ctx.shard, ctx.backend
        need_b = ctx.has_bias and ctx.needs_input_grad[1]
        dY, db = be.relu_bwd_colsum(dZ.contiguous(), Y, ctx.relu, need_b)
        dYtab = gather_table(sh, dY, ctx.group, slot="bwd")
        argtab = None
        if ctx.reduce == L.REDUCE_MAX:
            argtab = gather_table(sh, argmax, ctx.group, slot="arg")
        dH = be.spmm_bwd(sh.bwd, sh.w_bwd, sh.row_scale, dYtab, ctx.reduce,
                         cnt=sh.cnt_table if ctx.reduce == L.REDUCE_MEAN else None, argmax=argtab)
        return dH, db, None, None, None, None, None


def sharded_aggregate(H_local, shard: Shard, aggr="add", bias=None, relu=False, backend=None,
                      group=None):
    """Aggregation of the rank's destination rows; H_local = this rank's rows."""
    return _ShardedAggregate.apply(H_local, bias, shard, L.REDUCE_CODES[aggr], bool(relu),
                                   backend or HipBackend(), group)


# --------------------------------------------------------- fused stack path
class _ShardedStack(torch.autograd.Function):
    """Sum / mean 128 -> 128 layers with ReLU between them, on the fused
    kernels, with chunked all-gathers overlapping the compute (module
    docstring).  ``x`` is the input either as the exchange table (replicated
    input features, ``x_is_table``) or as this rank's rows."""

    @staticmethod
    def forward(ctx, x, shard: Shard, reduce, relus, backend, group, x_is_table, *params):
        Ws, bs = params[0::2], params[1::2]
        if not all(relus[:-1]):
            raise ValueError("_ShardedStack: every layer below the top needs its ReLU (its mask "
                             "feeds the adjoint's epilogue)")
        sh, be = shard, backend
        rows, C = sh.rows, sh.chunks
        dev = x.device
        tab = x if x_is_table else gather_table(sh, x, group, slot="t1")
        zs, rms, outs = [], [], []
        n = len(Ws)
        for i, (W, b) in enumerate(zip(Ws, bs)):
            F_in, F_out = W.shape
            last = i == n - 1
            out = torch.empty(sh.pad_rows, F_out, dtype=torch.float32, device=dev)
            if sh.pad_rows > rows:
                out[rows:].zero_()  # padding rows travel too (packed: as zeros)
            want_z = bool(ctx.needs_input_grad[7 + 2 * i])
            z = torch.empty(sh.pad_rows, F_in, dtype=torch.float32, device=dev) if want_z else None
            rm = None
            if relus[i] and not last:
                rm = torch.empty(sh.pad_rows, 4 * ((F_out + 127) // 128), dtype=torch.int32,
                                 device=dev)
            # the layer's output rows (ReLU'd below the top) travel packed;
            # the next layer gathers them in place where its kernel can
            xch = None
            if not last:
                pk = relus[i] and _pack_on(sh, be, F_out)
                slot = "t%d" % (i & 1)
                xch = _ChunkExchange(sh, out, lambda F=F_out, s_=slot: new_table(
                    sh, F, torch.float32, dev, s_), group, be, pk,
                    inplace=pk and _inplace_ok(sh, be, F_out), key=("fwd", i, F_out))
            for c in range(C):
                a, e = sh.chunk(c)
                if e > a:
                    be.spmm_xw_fwd(sh.view_for(tab, "fwd", a, e, sh.chunk_edges_fwd[c]), sh.w_fwd,
                                   tab, W, reduce, b, relus[i],
                                   relu_mask=None if rm is None else rm[a:e], want_z=want_z,
                                   out=out[a:e], z_out=None if z is None else z[a:e])
                if xch is not None:
                    xch.start(c)
                    xch.finish(keep=1)
            outs.append(out)
            zs.append(z)
            rms.append(rm)
            tab = None if xch is None else xch.result()
        ctx.shard, ctx.reduce, ctx.relus, ctx.backend, ctx.group = sh, reduce, relus, be, group
        ctx.n = n
        ctx.x_is_table = x_is_table
        ctx.has_bias = [b is not None for b in bs]
        ctx.save_for_backward(*Ws, outs[-1], *[t if t is not None else torch.empty(0)
                                               for t in zs + rms])
        return outs[-1][:rows]

    @staticmethod
    def backward(ctx, dZ):
        sh, be, group, n = ctx.shard, ctx.backend, ctx.group, ctx.n
        saved = ctx.saved_tensors
        Ws, top_out = saved[:n], saved[n]
        zs, rms = saved[n + 1:2 * n + 1], saved[2 * n + 1:3 * n + 1]
        relus = ctx.relus
        rows, C = sh.rows, sh.chunks
        dev = dZ.device
        mean = ctx.reduce == L.REDUCE_MEAN
        rd = sh.in_cnt if mean else None
        gW, gb = [None] * n, [None] * n
        top = n - 1
        dY = torch.empty(sh.pad_rows, Ws[top].size(1), dtype=torch.float32, device=dev)
        # the top bias gradient from the dW pass over dY (no separate read)
        top_cs = not relus[top] and rd is None and ctx.has_bias[top] and zs[top].numel() > 0
        if relus[top] or rd is not None or (ctx.has_bias[top] and not top_cs):
            d, gb[top] = be.relu_bwd_colsum(dZ.contiguous(), top_out[:rows], relus[top],
                                            ctx.has_bias[top], row_div=rd)
            dY[:rows] = d
        else:
            dY[:rows] = dZ
        need_x = ctx.needs_input_grad[0] and not ctx.x_is_table

        def wants_dx(l):  # layer l's adjoint gather runs (and its dY is exchanged)
            return l > 0 or need_x

        # top layer's dY: all of it is local already; gather it in chunks
        tab = works = None
        if wants_dx(top):
            tab = new_table(sh, dY.size(1), torch.float32, dev, "t%d" % (top & 1))
            works = [_gather_chunk(sh, c, dY, tab, group) for c in range(C)]
        dx = None
        for l in range(top, -1, -1):
            W = Ws[l]
            # dW = Z^T dY on local rows, while the dY chunks travel
            if zs[l].numel():
                gW[l], cs = be.gemm_bwd_dw(zs[l][:rows], dY[:rows], W,
                                           dh_colsum=bool(top_cs and l == top))
                if top_cs and l == top:
                    gb[top] = cs
            if not wants_dx(l):
                break
            if isinstance(works, _ChunkExchange):
                tab = works.result()  # (dense, or the packed table gathered in place)
            else:
                _wait(works)
            dX = torch.empty(sh.pad_rows, W.size(0), dtype=torch.float32, device=dev)
            xch = None
            if l > 0 and wants_dx(l - 1):
                if sh.pad_rows > rows:
                    dX[rows:].zero_()  # padding rows travel too (packed: as zeros)
                # masked by the lower layer's ReLU: travels packed
                Fx = W.size(0)
                pk = relus[l - 1] and _pack_on(sh, be, Fx)
                slot = "t%d" % ((l - 1) & 1)
                xch = _ChunkExchange(sh, dX, lambda F=Fx, s_=slot: new_table(
                    sh, F, torch.float32, dev, s_), group, be, pk,
                    inplace=pk and _inplace_ok(sh, be, Fx), key=("bwd", l, Fx))
            works = []
            # the lower layer's bias gradient: every chunk's column sums are
            # added into one device vector by the adjoint launches themselves
            # (mgcn_spmm_xw_bwd accumulate, in chunk order; no host reduction)
            csum = None
            if l > 0 and ctx.has_bias[l - 1]:
                csum = torch.zeros(W.size(0), dtype=torch.float32, device=dev)
            for c in range(C):
                a, e = sh.chunk(c)
                if e > a:
                    be.spmm_xw_bwd_dx(
                        sh.view_for(tab, "bwd", a, e, sh.chunk_edges_bwd[c]), sh.w_bwd,
                        None if sh.row_scale is None else sh.row_scale[a:e], tab, W,
                        relu_mask=rms[l - 1][a:e] if l > 0 else None,
                        row_div=rd[a:e] if (l > 0 and rd is not None) else None, out=dX[a:e],
                        colsum=csum)
                if xch is not None:
                    xch.start(c)
                    xch.finish(keep=1)
            # (the exchange's last chunk is finished at the next layer's
            # result(), after its dW)
            works = xch
            if l > 0:
                if ctx.has_bias[l - 1]:
                    gb[l - 1] = csum
                dY, tab = dX, None
            else:
                dx = dX[:rows]
        grads = []
        for w, b in zip(gW, gb):
            grads += [w, b]
        return (dx, None, None, None, None, None, None, *grads)


class ShardedGCN:
    """Stack of GCN layers (NodeModelAdditive deg_norm / aggr + bias, ReLU
    between layers) over a destination-range sharded graph: the bench's N > 1
    model.  Sum / mean 128-wide stacks run on :class:`_ShardedStack`; other
    stacks layer by layer (:func:`sharded_aggregate`)."""

    def __init__(self, edge_index, num_nodes, Ws, bs, device, deg_norm="sm", aggr="add",
                 group=None, backend=None, chunks: int = 4, fused: bool = True, emulate=None):
        self.backend = backend or HipBackend()
        self.group = group
        self.device = device
        self.shard = build_shard(edge_index, num_nodes, deg_norm, group=group,
                                 backend=self.backend, device=device, chunks=chunks,
                                 emulate=emulate)
        self.aggr = aggr
        self.reduce = L.REDUCE_CODES[aggr]
        self.W = [w.to(device).clone().requires_grad_(True) for w in Ws]
        self.b = [b.to(device).clone().requires_grad_(True) for b in bs]
        self.fused = bool(fused) and self.reduce != L.REDUCE_MAX and all(
            self.backend.fused_ok(self.shard, w.size(0), w.size(1), self.reduce) for w in self.W)

    def params(self):
        return self.W + self.b

    def local_rows(self, full: torch.Tensor) -> torch.Tensor:
        return full[self.shard.lo:self.shard.hi].to(self.device)

    def input_table(self, full: torch.Tensor) -> torch.Tensor:
        """Replicated input features in the exchange layout (setup, untimed):
        the first layer then reads them in place, with no exchange."""
        return self.shard.to_table(full.to(self.device))

    def _relus(self):
        return tuple(i < len(self.W) - 1 for i in range(len(self.W)))

    def forward(self, X_local=None, X_table=None):
        if self.fused:
            params = []
            for w, b in zip(self.W, self.b):
                params += [w, b]
            x, is_tab = (X_table, True) if X_table is not None else (X_local, False)
            return _ShardedStack.apply(x, self.shard, self.reduce, self._relus(), self.backend,
                                       self.group, is_tab, *params)
        h = X_local if X_local is not None else X_table[
            table_positions(torch.arange(self.shard.lo, self.shard.hi, device=X_table.device),
                            self.shard.bounds, self.shard.chunk_rows)]
        L_ = len(self.W)
        for i in range(L_):
            H = self.backend.linear(h, self.W[i])
            h = sharded_aggregate(H, self.shard, self.aggr, self.b[i], relu=i < L_ - 1,
                                  backend=self.backend, group=self.group)
        return h

    def step_fn(self, X, dY, X_table=None, dY_local=None):
        """fwd + bwd to every weight and bias + the gradient all-reduce, with
        the replicated input features resident in the exchange layout (given
        as the full [N, F] X, or directly as the table; dY as the full [N, F]
        upstream gradient or this rank's rows)."""
        Xt = X_table if X_table is not None else self.input_table(X)
        dYl = dY_local if dY_local is not None else self.local_rows(dY)
        params = self.params()

        def step():
            for p in params:
                p.grad = None
            out = self.forward(X_table=Xt)
            out.backward(dYl)
            allreduce_grads(params, self.group)
        return step


class ShardedGCNStack(torch.nn.Module):
    """The module surface of the sharded path: a :class:`mgcn.models.GCNStack`
    (its GCNLayers and their reference-compatible parameters) run over a
    destination-range sharded graph -- ``forward`` takes this rank's input
    rows (or the replicated input in the exchange layout) and returns this
    rank's output rows; gradients land on the wrapped stack's parameters,
    partial per rank until :meth:`allreduce_grads` (one bucketed all_reduce)
    makes them the single-device gradients.  Sum / mean stacks whose layers
    below the top use ReLU run on :class:`_ShardedStack` (fused kernels,
    chunked all-gathers overlapped with the compute); others layer by layer.

    Equivalence with the single-device module (tests/test_dist_gloo.py,
    tests/test_gpu_dist.py): forward rows and dX rows bit for bit, parameter
    gradients within fp32 summation order.
    """

    def __init__(self, stack, edge_index, num_nodes, group=None, backend=None, chunks: int = 4,
                 device=None, fused: bool = True, deg=None, emulate=None):
        super().__init__()
        self.stack = stack
        layers = list(stack.layers)
        nms = [layer.gcn.node_models[0] for layer in layers]
        if any(len(layer.gcn.node_models) != 1 for layer in layers) or \
                len({(nm.deg_norm, nm.aggr) for nm in nms}) != 1:
            raise NotImplementedError("ShardedGCNStack: single-kernel layers with one deg_norm / "
                                      "aggr")
        acts = [layer.non_linear_name for layer in layers]
        if any(a not in ("relu", "none") for a in acts):
            raise NotImplementedError("ShardedGCNStack: 'relu' / 'none' layer activations")
        self.group = group
        self.backend = backend or HipBackend()
        self.relus = tuple(a == "relu" for a in acts)
        self.aggr = nms[0].aggr
        self.reduce = L.REDUCE_CODES[self.aggr]
        dev = device if device is not None else nms[0].weight_node.device
        self.shard = build_shard(edge_index, num_nodes, nms[0].deg_norm, deg=deg, group=group,
                                 backend=self.backend, device=dev, chunks=chunks, emulate=emulate)
        self._nms = nms
        self.fused = bool(fused) and self.reduce != L.REDUCE_MAX and all(self.relus[:-1]) and all(
            self.backend.fused_ok(self.shard, nm.weight_node.size(0), nm.weight_node.size(1),
                                  self.reduce) for nm in nms)

    def local_rows(self, full: torch.Tensor) -> torch.Tensor:
        return full[self.shard.lo:self.shard.hi]

    def input_table(self, full: torch.Tensor) -> torch.Tensor:
        return self.shard.to_table(full)

    def forward(self, x_local=None, x_table=None):
        if (x_local is None) == (x_table is None):
            raise ValueError("ShardedGCNStack: give x_local (this rank's rows) or x_table")
        if self.fused:
            params = []
            for nm in self._nms:
                params += [nm.weight_node, nm.bias]
            x, is_tab = (x_table, True) if x_table is not None else (x_local, False)
            return _ShardedStack.apply(x, self.shard, self.reduce, self.relus, self.backend,
                                       self.group, is_tab, *params)
        h = x_local if x_local is not None else x_table[
            table_positions(torch.arange(self.shard.lo, self.shard.hi, device=x_table.device),
                            self.shard.bounds, self.shard.chunk_rows)]
        for nm, relu in zip(self._nms, self.relus):
            H = self.backend.linear(h, nm.weight_node)
            h = sharded_aggregate(H, self.shard, self.aggr, nm.bias, relu=relu,
                                  backend=self.backend, group=self.group)
        return h

    def allreduce_grads(self) -> None:
        allreduce_grads(list(self.parameters()), self.group)


class DataParallel:
    """Data-parallel replicas over torch.distributed (one process per GPU,
    the whole model on every rank): the north star's "natural DP cases"
     -- the config-3 botnet loop and the config-1 CV loop,
    whose graphs are independent.  A step's global batch (the items one
    process would take) is dealt out item by item (rank r takes items r, r +
    P, ...); each rank sums its items' losses and divides by the GLOBAL
    count, so after :meth:`reduce_grads` (one bucketed all_reduce SUM) every
    rank holds the gradient of the single-process mean loss and takes the
    same optimizer step.  Equal to one process within fp32 summation order
    (tests/test_dist_gloo.py).  World 1 (or torch.distributed not
    initialised): a pass-through."""

    def __init__(self, params, group=None):
        self.params = [p for p in params]
        self.group = group
        on = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1

    def share(self, items):
        return list(items)[self.rank::self.world]

    def broadcast_params(self) -> None:
        """Rank 0's parameters to every rank (identical replicas)."""
        if not _collective(self.world):
            return
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(p.data, src=dist.get_global_rank(self.group, 0)
                               if self.group is not None else 0, group=self.group)

    def all_sum(self, values, device=None):
        """Sum a few numbers over the ranks (one all_reduce); returns floats."""
        if not _collective(self.world):
            return [float(v) for v in values]
        dev = device if device is not None else (self.params[0].device if self.params else "cpu")
        if dist.get_backend(self.group) == "nccl" and torch.device(dev).type != "cuda":
            dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
        dist.all_reduce(t, group=self.group)
        return [float(v) for v in t.tolist()]

    def reduce_grads(self) -> None:
        """All-reduce (sum) every parameter's gradient; a rank whose share
        was empty (or whose parameters took no gradient) contributes zeros.
        A parameter that NO rank gave a gradient keeps ``grad = None`` -- as
        in one process, where the optimizer then skips it (no weight decay,
        no moment decay): a per-parameter "has grad" flag travels in the same
        bucketed all_reduce."""
        if not _collective(self.world):
            return
        params = [p for p in self.params if p.requires_grad]
        if not params:
            return
        dev = params[0].device
        has = torch.tensor([float(p.grad is not None) for p in params], dtype=torch.float32,
                           device=dev)
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        _allreduce_flat([p.grad for p in params] + [has], self.group)
        for p, h in zip(params, has.tolist()):
            if h == 0.0:
                p.grad = None


def _allreduce_flat(tensors, group=None) -> None:
    """Sum the tensors over the ranks in place with ONE all_reduce of their
    concatenation (a bucket: one RCCL call per step, not one per tensor)."""
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, group=group)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


def allreduce_grads(params, group=None) -> None:
    """One bucketed all_reduce (sum) of the replicated parameters' gradients."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads or not dist.is_initialized() or not _collective(dist.get_world_size(group)):
        return
    _allreduce_flat(grads, group)
