"""pkg/columns/group on the GPU.

GroupEntries (pkg/columns/group/group.go:51-121): for each groupBy name in turn, rows with
equal values of that ONE column form a group (successive, not composite --
group_test.go:101-129); each output row is a copy of the group's first row with every
`group:sum` column summed and wrapped to its width (flattenValues :123-165); the result is
sorted ascending by the group column (:115).  "" groups everything into one row and stops.

Device path: igx_groupby (exact keys, first-occurrence index) -> gather first rows ->
overwrite sums -> igx_sort_perm.  Float `group:sum` columns keep the reference's sequential
addition order (float64 adds, a float32 field rounding after each): a stable sort of the rows
by the group key makes each group one run in input order, and igx_segment_fsum walks the
runs.  Groups are keyed by the column's bytes; the reference keys by the value's string form
(getStringFromValue, :27-47), which differs only for floats whose distinct bit patterns print
alike (NaN payloads).
"""
from __future__ import annotations

from . import _abi
from ._abi import IgxError
from .columns import Columns, EventBatch, GroupTypeSum, KINDS
from .runtime import torch_mod
from . import engine


class GroupError(ValueError):
    pass


def _wrap_sum(col, s64):
    """u64 sum -> column dtype, wrapping to the column width (SetInt/SetUint)."""
    torch = torch_mod()
    from .columns import torch_dtype
    dt = torch_dtype(col.kind)
    if col.width == 8:
        return s64.view(dt)
    # truncate: reinterpret the little-endian low bytes
    b = s64.view(torch.uint8).view(-1, 8)[:, : col.width].contiguous()
    return b.view(dt).flatten()


def _group_one(cols: Columns, batch: EventBatch, col, all_rows: bool):
    torch = torch_mod()
    dev = batch.device()
    n = batch.n
    every = [c for c in cols.GetOrderedColumns() if c.GroupType == GroupTypeSum and not c.virtual]
    sums = [c for c in every if KINDS[c.kind][0] != _abi.KIND_FLOAT]
    fsums = [c for c in every if KINDS[c.kind][0] == _abi.KIND_FLOAT]
    tensors = batch.tensors_in_schema_order()
    if all_rows:
        keycol = torch.zeros(max(1, n), dtype=torch.uint32, device=dev)
        tensors = tensors + [keycol]
        key_idx = len(tensors) - 1
        kw = 4
    else:
        key_idx = cols.index(col.Name)
        t = tensors[key_idx]
        kw = t.shape[1] if t.dim() == 2 else t.element_size()
    valid = batch.valid
    aggs = []
    for c in sums:
        aggs.append(_abi.Agg(_abi.AGG_SUM, cols.index(c.Name), _abi.NO_COL, c.width, 0))
    if valid is not None:
        tensors = tensors + [valid]
        vidx = len(tensors) - 1
    tab = engine.Table([kw], aggs, capacity=max(16, n))
    try:
        preds = []
        if valid is not None:
            p = _abi.Pred()
            p.col, p.cmp, p.negate, p.ref_len = vidx, _abi.CMP_EQ, 1, 1
            p.ref[0] = 0
            preds.append(p)            # valid != 0  (nil entries skipped)
        tab.update(tensors, [key_idx], n, 0, preds)
        fin = tab.finalize()
        _, agg_t, first = engine.table_tensors(tab, fin)
    finally:
        tab.destroy()
    G = fin["n_groups"]
    first64 = first.view(torch.int64)
    out = batch.take(first64)
    for c, s in zip(sums, agg_t):
        out.data[c.Name.lower()] = _wrap_sum(c, s)
    if fsums and G:
        kt = tensors[key_idx]
        kb = kt if kt.dim() == 2 else kt.view(torch.uint8).view(-1, kt.element_size())
        perm = engine.sort_perm([(kb[:n], False, _abi.KIND_BYTES)], n, valid=valid)
        ctx = engine.context()
        from .columns import torch_dtype
        for c in fsums:
            v = batch[c.Name]
            acc = torch.empty(max(1, n), dtype=torch.float64, device=dev)
            ctx.check(ctx.L.igx_segment_fsum(ctx.h, engine.ptr(kb), kb.stride(0), kb.shape[1], engine.ptr(perm), n,
                                             engine.ptr(valid), engine.ptr(v), v.element_size(), engine.ptr(acc)))
            out.data[c.Name.lower()] = acc[first64].to(torch_dtype(c.kind))
    out.valid = None
    return out, first


def GroupEntries(cols: Columns, batch, group_by):
    if batch is None:
        return None
    new = batch
    for name in group_by:
        name = name.lower()
        if name == "":
            out, _ = _group_one(cols, batch, None, True)
            return out
        col, ok = cols.GetColumn(name)
        if not ok:
            raise GroupError(f'could not group by "{name}": column not found')
        grouped, first = _group_one(cols, new, col, False)
        # sort.SortEntries(columns, outEntries, []string{groupName}) -- group.go:115
        from . import sort as _sort
        new = _sort.SortEntries(cols, grouped, [name], pos=first)
    return new
