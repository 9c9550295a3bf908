"""pkg/columns/filter on the GPU.

Same entry points and error texts as pkg/columns/filter/filter.go:
  GetFilterFromString (:91-172)    -> host parser in libigx.so (igx_filter_parse)
  GetFiltersFromStrings (:175-185) -> "invalid filter %q: %w"
  FilterSpecs.MatchAll / MatchAny / FilterSpec.Match (:266-291) -> device scan
  FilterEntries (:294-325)         -> sequential filters, nil rows skipped, order kept
Regex rules (`~`) parse exactly as in the reference but the device scan rejects them
with IGX_ENOTSUP (RE2 on the GPU is a SURVEY.md §8(f) "next" item).
"""
from __future__ import annotations

import ctypes as C

from . import _abi
from ._abi import IgxError
from .columns import Columns, EventBatch
from .runtime import context, ptr, torch_mod
from . import engine


class FilterError(ValueError):
    pass


def _go_q(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


class FilterSpec:
    def __init__(self, cols: Columns, pred: _abi.Pred, text: str):
        self.cols = cols
        self.pred = pred
        self.text = text
        self.column = cols.GetOrderedColumns()[pred.col]
        self.negate = bool(pred.negate)

    def Match(self, batch: EventBatch):
        """Row ids of `batch` this filter matches (nil rows excluded)."""
        return _scan(batch, [self])


class FilterSpecs(list):
    def MatchAll(self, batch: EventBatch):
        return _scan(batch, list(self))

    def MatchAny(self, batch: EventBatch):
        torch = torch_mod()
        if not self:
            return torch.empty(0, dtype=torch.uint32, device=batch.device())
        return engine.filter_rows(batch.tensors_in_schema_order(), [s.pred for s in self],
                                  batch.n, batch.valid, any=True)


def GetFilterFromString(cols: Columns, filt: str) -> FilterSpec:
    arr, n = cols.schema()
    pred = _abi.Pred()
    err = C.create_string_buffer(512)
    rc = _abi.lib().igx_filter_parse(arr, n, filt.encode(), C.byref(pred), err, 512)
    if rc == _abi.IGX_ENOTSUP:
        raise IgxError(rc, err.value.decode())
    if rc:
        raise FilterError(err.value.decode())
    return FilterSpec(cols, pred, filt)


def GetFiltersFromStrings(cols: Columns, filters) -> FilterSpecs:
    out = FilterSpecs()
    for f in filters:
        try:
            out.append(GetFilterFromString(cols, f))
        except FilterError as e:
            raise FilterError(f"invalid filter {_go_q(f)}: {e}") from None
    return out


def _scan(batch: EventBatch, specs):
    """AND of specs over the batch on the device (igx_filter: 4 predicates per mark launch,
    later launches AND into the same bitmask); returns selected row ids (u32)."""
    return engine.filter_rows(batch.tensors_in_schema_order(), [s.pred for s in specs],
                              batch.n, batch.valid)


def FilterEntries(cols: Columns, batch, filters):
    """filter.go:294-325.  Returns the matching rows as a new batch (None for None)."""
    if batch is None:
        return None
    out = batch
    for f in filters:
        try:
            fs = GetFilterFromString(cols, f)
        except FilterError as e:
            raise FilterError(f"could not apply filter {_go_q(f)}: {e}") from None
        idx = _scan(out, [fs])
        out = out.take(idx)
    if not filters:
        # no filters: the reference returns its (nil) outEntries slice
        return batch.take(_scan(batch, [])) if batch.valid is not None else batch   # drops nil rows
    return out
