"""pkg/columns/filter on the GPU.

Same entry points and error texts as pkg/columns/filter/filter.go:
  GetFilterFromString (:91-172)    -> host parser in libigx.so (igx_filter_parse)
  GetFiltersFromStrings (:175-185) -> "invalid filter %q: %w"
  FilterSpecs.MatchAll / MatchAny / FilterSpec.Match (:266-291) -> device scan, a nil row
                                      giving Match(nil) == negate (:286-291)
  FilterEntries (:294-325)         -> sequential filters, nil rows skipped, order kept; no
                                      filters -> the never-assigned (nil) outEntries
Regex rules (`~`) run on the device too: igx_filter compiles them on the host into a DFA
over rune classes (igx_regex.cpp) that k_filter walks per row.
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
        """Row ids of `batch` this filter matches; a nil row matches iff the filter is
        negated (filter.go:286-291)."""
        return _scan(batch, [self], nil_match=True)


class FilterSpecs(list):
    def MatchAll(self, batch: EventBatch):
        """filter.go:266-273 per row: a nil row is kept iff every spec is negated (or
        there are none)."""
        return _scan(batch, list(self), nil_match=True)

    def MatchAny(self, batch: EventBatch):
        """filter.go:276-283 per row: no specs select nothing; a nil row is kept iff some
        spec is negated."""
        torch = torch_mod()
        if not self:
            return torch.empty(0, dtype=torch.uint32, device=batch.device())
        return engine.filter_rows(batch.tensors_in_schema_order(), [s.pred for s in self],
                                  batch.n, batch.valid, any=True, nil_match=True)


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


def _scan(batch: EventBatch, specs, nil_match=False):
    """AND of specs over the batch on the device (igx_filter_ex: 4 predicates per mark
    launch, later launches AND into the same bitmask); returns selected row ids (u32).
    nil_match=False skips nil rows (FilterEntries); True applies Match(nil) == negate."""
    return engine.filter_rows(batch.tensors_in_schema_order(), [s.pred for s in specs],
                              batch.n, batch.valid, nil_match=nil_match)


def FilterEntries(cols: Columns, batch, filters):
    """filter.go:294-325.  Returns the matching rows as a new batch, None for None (:295-297)
    and None when there are no filters: the reference returns `outEntries`, which only the
    filter loop assigns, so it is still the nil slice (:299,321-324)."""
    if batch is None:
        return None
    specs = []
    for f in filters:
        try:
            specs.append(GetFilterFromString(cols, f))
        except FilterError as e:
            raise FilterError(f"could not apply filter {_go_q(f)}: {e}") from None
    if not specs:
        return None
    # The reference narrows `entries` filter by filter (:301-322); the rows left at the end
    # are the non-nil rows every filter matches, in input order -- one AND scan and one
    # compaction here.  (A parse error returns before any result either way.)  Over a plain
    # batch the result is a view whose length stays on the device until asked for (len(),
    # .n): SortEntries of it then runs without a host round trip.
    if batch.sel is None:
        idx, cnt = engine.filter_rows(batch.tensors_in_schema_order(), [s.pred for s in specs], batch.n,
                                      batch.valid, device_count=True)
        return EventBatch(batch.cols, batch._base, batch._base_valid, sel=idx, sel_count=cnt)
    return batch.take(_scan(batch, specs))
