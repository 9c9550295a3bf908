"""Multi-GPU merges of the aggregation path.

One process per GPU.  Two transports carry the exchanges:

  * torch.distributed (default): on an "nccl" group its collectives are RCCL over xGMI on
    MI355X; on "gloo" (the CPU tests, and the ranks that share one GPU in the world-size-2
    GPU test) device tensors are staged through the host.
  * RCCL through libigx.so's igx_dist_* C ABI (the same entry points a cgo caller binds),
    with IGX_DIST=igx on an "nccl" group; torch.distributed only hands rank 0's ncclUniqueId
    to the other ranks.

Only data movement and bookkeeping live here; every aggregation and merge runs in libigx.so:

  log2 histograms (C3)      dense u32[keys][27] per rank -> all-reduce(sum)            exact
  group-by / distinct (C4)  local partial groups -> all-to-all by hash(key) -> the owner
                            merges them (igx_groupby_update_ex: SUM of partials, MIN of
                            first index) -> each key lives on exactly one rank         exact
  top-K (C2, C5)            per-rank K candidates -> all-gather -> one more top-K with
                            the global first index as the position                     exact
                            (keys are rank-disjoint after the exchange or by ingest)

The reference merges nodes by concatenating per-node arrays (snapshotcombiner.go:79-106);
an exact global merge is stricter and equal to the single-device result on the union.
"""
from __future__ import annotations

import ctypes as C
import os

from .runtime import torch_mod, context, ptr

_comm = None


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def world():
    """(rank, world_size); (0, 1) without an initialised process group."""
    d = _dist()
    return (d.get_rank(), d.get_world_size()) if d else (0, 1)


class TorchComm:
    """torch.distributed transport (gloo, or any backend torch supports for these calls).
    Device tensors go through the host when the backend is gloo."""

    name = "torch"

    def __init__(self, d):
        self.d = d
        self.stage = d.get_backend() == "gloo"

    def _out(self, t):
        return t.cpu() if self.stage and t.is_cuda else t

    def allreduce_u32(self, hist):
        torch = torch_mod()
        h = self._out(hist)
        self.d.all_reduce(h.view(torch.int32), op=self.d.ReduceOp.SUM)   # same bits mod 2^32
        if h is not hist:
            hist.copy_(h)
        return hist

    def allgather_rows(self, rows):
        torch = torch_mod()
        d, ws = self.d, self.d.get_world_size()
        r = self._out(rows)
        n = torch.tensor([r.shape[0]], dtype=torch.int64, device=r.device)
        ns = [torch.empty_like(n) for _ in range(ws)]
        d.all_gather(ns, n)
        counts = [int(x.item()) for x in ns]
        m = max(counts)
        pad = torch.zeros((max(1, m), r.shape[1]), dtype=r.dtype, device=r.device)
        if r.shape[0]:
            pad[: r.shape[0]] = r
        outs = [torch.empty_like(pad) for _ in range(ws)]
        d.all_gather(outs, pad)
        return torch.cat([o[:c] for o, c in zip(outs, counts)]).to(rows.device)

    def alltoallv_rows(self, rows, counts):
        torch = torch_mod()
        d = self.d
        r = self._out(rows)
        send_counts = torch.tensor(counts, dtype=torch.int64, device=r.device)
        recv_counts = torch.empty_like(send_counts)
        d.all_to_all_single(recv_counts, send_counts)
        rc = recv_counts.tolist()
        out = torch.empty((sum(rc), r.shape[1]), dtype=r.dtype, device=r.device)
        d.all_to_all_single(out, r.contiguous(), rc, list(counts))
        return out.to(rows.device)


class IgxComm:
    """RCCL transport through libigx.so (igx_dist_*).  Rank 0's ncclUniqueId reaches the
    other ranks over the torch process group; everything after that is the C ABI."""

    name = "igx"

    def __init__(self, d, timeout_ms=None):
        torch = torch_mod()
        from . import _abi
        rank, ws = d.get_rank(), d.get_world_size()
        self.h, self.ws = None, ws
        uid = (C.c_uint8 * _abi.DIST_ID_BYTES)()
        ok, err = 1, None
        try:
            self.ctx = context()
            if rank == 0:
                ok = int(self.ctx.L.igx_dist_get_unique_id(uid) == 0)
            dev = torch.device("cuda", self.ctx.device)
        except Exception as e:   # noqa: BLE001 -- still join the broadcast below, flagged
            ok, err, dev = 0, e, torch.device("cuda", torch.cuda.current_device())
        # every rank joins the broadcast whatever happened above (the last byte carries rank
        # 0's status), so no rank is left waiting in it while the others move on
        t = torch.tensor(list(uid) + [ok], dtype=torch.uint8, device=dev)
        d.broadcast(t, 0)
        v = t.cpu().tolist()
        # every rank's status, before any rank enters igx_dist_init: a rank that cannot open the
        # transport would otherwise leave its peers inside ncclCommInitRank until the deadline
        # (IGX_DIST_TIMEOUT_MS) -- now all of them raise here and select_transport falls back
        st = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=dev)
        d.all_reduce(st, op=d.ReduceOp.MIN)
        if err is not None:
            raise RuntimeError(f"IgxComm on rank {rank}: {err}")
        if not v[-1]:
            raise RuntimeError("igx_dist_get_unique_id failed on rank 0")
        if int(st.item()) == 0:
            raise RuntimeError(f"IgxComm on rank {rank}: a peer could not open the transport")
        uid = (C.c_uint8 * _abi.DIST_ID_BYTES)(*v[:-1])
        h = C.c_void_p()
        self.ctx.check(self.ctx.L.igx_dist_init(self.ctx.h, uid, ws, rank, C.byref(h)))
        self.h = h
        if timeout_ms is not None:
            self.ctx.check(self.ctx.L.igx_dist_set_timeout(self.h, int(timeout_ms)))

    def wait(self):
        """igx_dist_wait: the stream drained, bounded by the communicator's deadline (EIO and
        an aborted communicator when a peer stops answering)."""
        self.ctx.check(self.ctx.L.igx_dist_wait(self.h))

    def _bind(self):
        self.ctx.bind_stream()
        return self.ctx.L

    def allreduce_u32(self, hist):
        L = self._bind()
        self.ctx.check(L.igx_dist_allreduce_u32(self.h, ptr(hist), hist.numel()))
        self.wait()
        return hist

    def allgather_rows(self, rows):
        torch = torch_mod()
        L = self._bind()
        rows = rows.contiguous()
        n, rb = rows.shape
        counts = (C.c_uint64 * self.ws)()
        self.ctx.check(L.igx_dist_allgather_rows(self.h, ptr(rows), n, rb, None, 0, counts))   # size query
        tot = sum(counts)
        out = torch.empty((max(1, tot), rb), dtype=rows.dtype, device=rows.device)
        self.ctx.check(L.igx_dist_allgather_rows(self.h, ptr(rows), n, rb, ptr(out), tot, counts))
        self.wait()
        return out[:tot]

    def alltoallv_rows(self, rows, counts):
        torch = torch_mod()
        L = self._bind()
        rows = rows.contiguous()
        rb = rows.shape[1]
        sc = (C.c_uint64 * self.ws)(*counts)
        rc = (C.c_uint64 * self.ws)()
        self.ctx.check(L.igx_dist_alltoallv_rows(self.h, ptr(rows), sc, rb, None, 0, rc))   # size query
        tot = sum(rc)
        out = torch.empty((max(1, tot), rb), dtype=rows.dtype, device=rows.device)
        self.ctx.check(L.igx_dist_alltoallv_rows(self.h, ptr(rows), sc, rb, ptr(out), tot, rc))
        self.wait()
        return out[:tot]

    def barrier(self):
        self.ctx.check(self._bind().igx_dist_barrier(self.h))

    def close(self):
        if self.h:
            self.ctx.L.igx_dist_destroy(self.h)
            self.h = None


def comm():
    """The transport for the current process group (None without one): the one
    select_transport() agreed on, else torch's own collectives (on an "nccl" group these are
    RCCL over xGMI too), or the igx_dist_* C ABI when IGX_DIST=igx on an nccl group.
    bench.py selects the C ABI at N > 1 (select_transport("igx")); the library's default stays
    torch's collectives until a world >= 2 run on GPUs has checked the C ABI's send/recv loops
    (their planning, igx_dist_plan_*, is tested for 2..8 ranks against gloo)."""
    global _comm
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return None
    if _comm is None:
        use_igx = d.get_backend() == "nccl" and os.environ.get("IGX_DIST", "torch") == "igx"
        _comm = IgxComm(d) if use_igx else TorchComm(d)
    return _comm


def select_transport(prefer="igx"):
    """Pick the transport every rank will use, agreed over the process group: prefer="igx"
    tries the igx_dist_* C ABI (RCCL) on an "nccl" group; if any rank's igx_dist_init fails,
    every rank falls back to torch's collectives.  Returns the transport's name ("igx" or
    "torch"), or None without a multi-rank group."""
    global _comm
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return None
    shutdown()
    c, ok = None, 1
    if prefer == "igx" and d.get_backend() == "nccl":
        try:
            c = IgxComm(d)
        except Exception:   # noqa: BLE001 -- any local failure: agree on the fallback below
            c, ok = None, 0
        torch = torch_mod()
        flag = torch.tensor([ok], dtype=torch.int32,
                            device=torch.device("cuda", torch.cuda.current_device()))
        d.all_reduce(flag, op=d.ReduceOp.MIN)
        if int(flag.item()) == 0 and c is not None:
            c.close()
            c = None
    _comm = c if c is not None else TorchComm(d)
    return _comm.name


def shutdown():
    """Release the RCCL communicator (before destroy_process_group)."""
    global _comm
    if _comm is not None and hasattr(_comm, "close"):
        _comm.close()
    _comm = None


def allreduce_hist(hist, c=None):
    """C3: in-place sum of a u32 histogram over ranks (c: a transport; default comm())."""
    c = c or comm()
    return hist if c is None else c.allreduce_u32(hist)


def allgather_rows(rows, c=None):
    """Concatenate every rank's (n_r, row_bytes) uint8 rows in rank order (n_r may differ)."""
    c = c or comm()
    return rows if c is None else c.allgather_rows(rows)


def partition_by_owner(rows, key_bytes, ws):
    """Group packed rows by the rank that owns their key (igx_partition_rows on the device:
    FNV-1a over the key's u32 words mod ws, stable).  Returns (rows, counts per rank)."""
    from . import engine
    return engine.partition_rows(rows, key_bytes, ws)


def exchange_partitioned(rows, counts, c=None):
    """All-to-all of rows already grouped by destination rank (counts[r] rows for rank r,
    in rank order; rows past their sum are ignored).  Returns the rows this rank owns, in
    source-rank order."""
    c = c or comm()
    rows = rows[:sum(counts)]
    return rows if c is None else c.alltoallv_rows(rows, counts)


def owner_capacity(capacity, ws, slack=1.25):
    """Groups an owner table must hold when `capacity` bounds the distinct keys of the whole
    (global) interval: keys reach their owner by a hash of the key, so an owner holds about
    1/ws of them; slack covers the hash's imbalance (at 1M keys per owner its spread is
    ~0.1 %)."""
    return min(capacity, int(capacity * slack / ws) + 4096)


def exchange_rows(rows, key_bytes):
    """C4 group-by exchange: every partial-group row goes to the rank owning its key."""
    r, ws = world()
    if ws == 1:
        return rows
    part, counts = partition_by_owner(rows, key_bytes, ws)
    return exchange_partitioned(part, counts)


def unpack_rows(rows, key_widths, naggs):
    """Packed group rows (key padded to 4-byte columns | naggs x u64 | first u64) -> SoA
    tensors: key columns (u8 (n, w) for byte keys, typed for 1/2/4/8), aggregates, first."""
    from . import engine
    torch = torch_mod()
    typed = {1: torch.uint8, 2: torch.uint16, 4: torch.uint32, 8: torch.uint64}
    fields, o = [], 0
    for i, w in enumerate(key_widths):
        fields.append((i, o, w, typed.get(w)))
        o += (w + 3) // 4 * 4
    nk = len(key_widths)
    fields += [(nk + x, o + 8 * x, 8, torch.uint64) for x in range(naggs + 1)]
    # the rows cut into columns in one pass on the device (igx_ingest_aos, the wire-format
    # ingest's kernel), not one strided torch copy per field, each re-reading every row
    r8 = rows.contiguous().view(torch.uint8)   # (n, row bytes)
    cols = {}
    for f0 in range(0, len(fields), 16):   # igx_ingest_aos takes up to 16 fields a call
        cols.update(engine.ingest_aos(r8, r8.shape[0], r8.shape[1], fields[f0:f0 + 16]))
    outs = [cols[i] for i in range(len(fields))]
    return outs[:nk], outs[nk:nk + naggs], outs[nk + naggs]


def owner_table(key_widths, out_widths, capacity):
    """The owner's merge table: SUM of the partials per aggregate, first = MIN, in the cached
    form.  A merge's rows are nearly all LDS misses (each key arrives once per rank that saw it),
    which would send AUTO to the partitioned form; but the cached form keeps the owner's keys
    across intervals and finds them, and measures faster (profiles/r06/emulated_rank8_*.json,
    rank 0 of 8: C4 0.98 -> 0.62 ms, C5 1.67 -> 1.53 ms)."""
    from . import _abi, engine
    nk = len(key_widths)
    spec = [_abi.Agg(_abi.AGG_SUM, nk + x, _abi.NO_COL, ow, 0) for x, ow in enumerate(out_widths)]
    t = engine.Table(key_widths, spec, max(1, capacity))
    t.set_mode(_abi.GB_CACHED)
    return t


def merge_partials(rows, key_widths, out_widths, capacity, table=None, sync=True):
    """Owner-side merge of exchanged partial groups on the device: one igx table whose
    aggregates SUM the partials and whose first index is the MIN of the partials' (the
    rows' u64 first column drives igx_groupby_update_ex's index column).  Returns the
    engine.Table, finalized (`table`, when given, is reset and reused; sync=False leaves the
    group count on the device, igx_groupby_finalize_async)."""
    from . import _abi, engine
    kcols, aggs, first = unpack_rows(rows, key_widths, len(out_widths))
    nk = len(kcols)
    if table is None:
        spec = [_abi.Agg(_abi.AGG_SUM, nk + x, _abi.NO_COL, ow, 0) for x, ow in enumerate(out_widths)]
        table = engine.Table(key_widths, spec, max(1, capacity))
        table.set_mode(_abi.GB_CACHED)   # see owner_table()
    else:
        table.reset()
    n = rows.shape[0]
    if n:
        table.update(kcols + aggs + [first], list(range(nk)), n, 0, idx_col=nk + len(aggs))
    table.finalize(sync=sync)
    return table


def merge_topk(cand, key_bytes, naggs, sort_keys, k, c=None):
    """Exact global top-K from all ranks' candidate rows (key | aggs | first): all-gather,
    then igx_topk with the global first index as the position.  sort_keys:
    [(agg_index, desc)] in sortBy order."""
    from . import engine
    torch = torch_mod()
    allc = allgather_rows(cand, c)
    if allc.shape[0] == 0:
        return allc
    o = key_bytes
    keys = [(allc[:, o + 8 * x:o + 8 * x + 8].contiguous().view(torch.uint64).flatten(), desc)
            for x, desc in sort_keys]
    first = allc[:, o + 8 * naggs:o + 8 * naggs + 8].contiguous().view(torch.uint64).flatten()
    idx = engine.sort_perm(keys, allc.shape[0], pos=first, k=k)
    return engine.take([allc], idx)[0]
