"""pkg/columns/group on the GPU.

GroupEntries (pkg/columns/group/group.go:51-121): for each groupBy name in turn, rows with
equal values of that ONE column form a group (successive, not composite --
group_test.go:101-129); each output row is a copy of the group's first row with every
`group:sum` column summed and wrapped to its width (flattenValues :123-165); the result is
sorted ascending by the group column (:115).  "" groups everything into one row and stops.

Device path: igx_groupby (exact keys, first-occurrence index) -> gather first rows ->
overwrite sums -> igx_sort_perm.  Float `group:sum` columns would need the reference's
sequential float64 addition order and are rejected (IGX_ENOTSUP).
"""
from __future__ import annotations

from . import _abi
from ._abi import IgxError
from .columns import Columns, EventBatch, GroupTypeSum, KINDS, gather
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
    sums = [c for c in cols.GetOrderedColumns() if c.GroupType == GroupTypeSum and not c.virtual]
    for c in sums:
        if KINDS[c.kind][0] == _abi.KIND_FLOAT:
            raise IgxError(_abi.IGX_ENOTSUP, f"float group:sum column {c.Name!r} on the GPU path")
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
    if kw == 3 or (kw > 4 and kw % 4):
        raise IgxError(_abi.IGX_ENOTSUP, f"group key width {kw}")
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
    out = batch.take(first.view(torch.int64))
    for c, s in zip(sums, agg_t):
        out.data[c.Name.lower()] = _wrap_sum(c, s)
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
