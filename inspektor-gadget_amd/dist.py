"""Multi-GPU merges of the aggregation path.

One process per GPU; `torch.distributed` carries the exchanges (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" in the CPU tests).  Only data movement and bookkeeping live here;
every aggregation runs in libigx.so:

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

from .runtime import torch_mod


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def world():
    """(rank, world_size); (0, 1) without an initialised process group."""
    d = _dist()
    return (d.get_rank(), d.get_world_size()) if d else (0, 1)


def allreduce_hist(hist):
    """C3: in-place sum of a u32 histogram over ranks.  u32 addition mod 2^32 equals the
    int32 two's-complement sum, so the buffer is reduced as int32 (RCCL and gloo)."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return hist
    torch = torch_mod()
    d.all_reduce(hist.view(torch.int32), op=d.ReduceOp.SUM)
    return hist


def allgather_rows(rows):
    """Concatenate every rank's (n_r, row_bytes) uint8 rows in rank order (n_r may differ)."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return rows
    torch = torch_mod()
    ws = d.get_world_size()
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    ns = [torch.empty_like(n) for _ in range(ws)]
    d.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    m = max(counts)
    pad = torch.zeros((max(1, m), rows.shape[1]), dtype=rows.dtype, device=rows.device)
    if rows.shape[0]:
        pad[: rows.shape[0]] = rows
    outs = [torch.empty_like(pad) for _ in range(ws)]
    d.all_gather(outs, pad)
    return torch.cat([o[:c] for o, c in zip(outs, counts)])


def partition_by_owner(rows, key_bytes, ws):
    """Group packed rows by the rank that owns their key (igx_partition_rows on the device:
    FNV-1a over the key's u32 words mod ws, stable).  Returns (rows, counts per rank)."""
    from . import engine
    return engine.partition_rows(rows, key_bytes, ws)


def exchange_partitioned(rows, counts):
    """All-to-all of rows already grouped by destination rank (counts[r] rows for rank r,
    in rank order).  Returns the rows this rank owns, in source-rank order."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return rows
    torch = torch_mod()
    send_counts = torch.tensor(counts, dtype=torch.int64, device=rows.device)
    recv_counts = torch.empty_like(send_counts)
    d.all_to_all_single(recv_counts, send_counts)
    rc = recv_counts.tolist()
    out = torch.empty((sum(rc), rows.shape[1]), dtype=rows.dtype, device=rows.device)
    d.all_to_all_single(out, rows.contiguous(), rc, list(counts))
    return out


def exchange_rows(rows, key_bytes):
    """C4 group-by exchange: every partial-group row goes to the rank owning its key."""
    d = _dist()
    ws = 1 if d is None else d.get_world_size()
    if ws == 1:
        return rows
    part, counts = partition_by_owner(rows, key_bytes, ws)
    return exchange_partitioned(part, counts)


def unpack_rows(rows, key_widths, naggs):
    """Packed group rows (key padded to 4-byte columns | naggs x u64 | first u64) -> SoA
    tensors: key columns (u8 (n, w) for byte keys, typed for 1/2/4/8), aggregates, first."""
    torch = torch_mod()
    typed = {1: torch.uint8, 2: torch.uint16, 4: torch.uint32, 8: torch.uint64}
    cols, o = [], 0
    for w in key_widths:
        c = rows[:, o:o + w].contiguous()
        cols.append(c.view(typed[w]).flatten() if w in typed else c)
        o += (w + 3) // 4 * 4
    aggs = [rows[:, o + 8 * x:o + 8 * x + 8].contiguous().view(torch.uint64).flatten()
            for x in range(naggs)]
    first = rows[:, o + 8 * naggs:o + 8 * naggs + 8].contiguous().view(torch.uint64).flatten()
    return cols, aggs, first


def merge_partials(rows, key_widths, out_widths, capacity):
    """Owner-side merge of exchanged partial groups on the device: one igx table whose
    aggregates SUM the partials and whose first index is the MIN of the partials' (the
    rows' u64 first column drives igx_groupby_update_ex's index column).  Returns the
    engine.Table, finalized."""
    from . import _abi, engine
    kcols, aggs, first = unpack_rows(rows, key_widths, len(out_widths))
    nk = len(kcols)
    spec = [_abi.Agg(_abi.AGG_SUM, nk + x, _abi.NO_COL, ow, 0) for x, ow in enumerate(out_widths)]
    tab = engine.Table(key_widths, spec, max(1, capacity))
    n = rows.shape[0]
    if n:
        tab.update(kcols + aggs + [first], list(range(nk)), n, 0, idx_col=nk + len(aggs))
    tab.finalize()
    return tab


def merge_topk(cand, key_bytes, naggs, sort_keys, k):
    """Exact global top-K from all ranks' candidate rows (key | aggs | first): all-gather,
    then igx_topk with the global first index as the position.  sort_keys:
    [(agg_index, desc)] in sortBy order."""
    from . import engine
    torch = torch_mod()
    allc = allgather_rows(cand)
    if allc.shape[0] == 0:
        return allc
    o = key_bytes
    keys = [(allc[:, o + 8 * x:o + 8 * x + 8].contiguous().view(torch.uint64).flatten(), desc)
            for x, desc in sort_keys]
    first = allc[:, o + 8 * naggs:o + 8 * naggs + 8].contiguous().view(torch.uint64).flatten()
    idx = engine.sort_perm(keys, allc.shape[0], pos=first, k=k)
    return engine.take([allc], idx)[0]
