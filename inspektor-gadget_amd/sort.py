"""pkg/columns/sort on the GPU.

Entry points of pkg/columns/sort/sort.go: Prepare (:87-111), ColumnSorterCollection.Sort
(:35-83), SortEntries (:116-123), CanSortBy (:139-144), FilterSortableColumns (:147-178).
The order produced is exactly Go 1.19 sort.SliceStable's under getLessFunc (:125-135),
DESC tie reversal included, via one stable LSD radix sort on the device.
"""
from __future__ import annotations

import ctypes as C

from . import _abi
from .columns import Columns, EventBatch
from .runtime import torch_mod
from . import engine


def _prepare_raw(cols: Columns, sort_by):
    arr, n = cols.schema()
    enc = [s.encode() for s in sort_by]
    argv = (C.c_char_p * max(1, len(enc)))(*enc)
    out = (_abi.SortKey * max(1, len(enc)))()
    nout, nbad = C.c_uint32(), C.c_uint32()
    rc = _abi.lib().igx_sort_prepare(arr, n, argv, len(enc), out, C.byref(nout), C.byref(nbad))
    if rc:
        raise _abi.IgxError(rc, "igx_sort_prepare failed")
    return [out[i] for i in range(nout.value)]


def FilterSortableColumns(cols: Columns, sort_by):
    valid, invalid = [], []
    for s in sort_by:
        (valid if _prepare_raw(cols, [s]) else invalid).append(s)
    return valid, invalid


def CanSortBy(cols: Columns, sort_by) -> bool:
    valid, _ = FilterSortableColumns(cols, sort_by)
    return len(valid) == len(sort_by)


class ColumnSorterCollection:
    def __init__(self, cols: Columns, keys):
        self.cols = cols
        self.keys = keys          # igx SortKey (schema index, desc, kind) in sortBy order

    def Perm(self, batch: EventBatch, pos=None, k=None):
        """Sorted row order of `batch` (u32 device tensor).  pos: pre-sort position per row
        (default: row index) -- the canonical order ties fall back to."""
        torch = torch_mod()
        if batch is None or batch.n == 0:
            return torch.empty(0, dtype=torch.uint32)
        ordered = self.cols.GetOrderedColumns()
        keys = []
        for sk in self.keys:
            c = ordered[sk.col]
            keys.append((batch[c.Name], bool(sk.desc), sk.kind))
        return engine.sort_perm_kinds(keys, batch.n, pos=pos, valid=batch.valid, k=k)

    def Sort(self, batch: EventBatch, pos=None):
        """Returns the batch in sorted order (the reference sorts []*T in place).  A view (a
        filtered slice of pointers) is sorted through its selection vector: the result is the
        same entries' row ids in sorted order, no column read beyond the sort keys."""
        if batch is None:
            return batch
        pend = batch.pending() if pos is None else None
        if pend is not None:   # a selection whose length is on the device: sorted there, no round trip
            sel, cnt = pend
            base, base_valid = batch._base, batch._base_valid
            ordered = self.cols.GetOrderedColumns()
            keys = [(base[ordered[sk.col].Name.lower()], bool(sk.desc), sk.kind) for sk in self.keys]
            if keys and self._device_countable(keys):
                if sel.shape[0] == 0:
                    return batch
                out = engine.sort_perm_kinds(keys, int(sel.shape[0]), valid=base_valid, rowmap=sel.contiguous(),
                                             d_count=cnt)
                return EventBatch(batch.cols, base, base_valid, sel=out, sel_count=cnt)
            # otherwise the synchronous path below (n read on the host)
        if batch.n == 0:
            return batch
        base, base_valid, sel = batch.base()
        if sel is None or pos is not None:
            return batch.take(self.Perm(batch, pos))
        ordered = self.cols.GetOrderedColumns()
        keys = [(base[ordered[sk.col].Name.lower()], bool(sk.desc), sk.kind) for sk in self.keys]
        if sel.dtype != torch_mod().int32 and sel.dtype != torch_mod().uint32:
            sel = sel.to(torch_mod().int32)
        out = engine.sort_perm_kinds(keys, batch.n, valid=base_valid, rowmap=sel.contiguous())
        return EventBatch(batch.cols, base, base_valid, sel=out)


    @staticmethod
    def _device_countable(keys):
        """igx_sort_perm_dn's shape: no float key (a NaN takes the exact Go path, which needs the
        length on the host)."""
        return all(kind != _abi.KIND_FLOAT for _, _, kind in keys)


def Prepare(cols: Columns, sort_by) -> ColumnSorterCollection:
    return ColumnSorterCollection(cols, _prepare_raw(cols, list(sort_by)))


def SortEntries(cols: Columns, batch, sort_by, pos=None):
    if batch is None:
        return None
    return Prepare(cols, sort_by).Sort(batch, pos)
