"""pkg/gadgets/top shared helpers (pkg/gadgets/top/top.go)."""
from __future__ import annotations

from .sort import SortEntries

MaxRowsDefault = 20          # top.go:26
IntervalDefault = 1          # top.go:27
IntervalParam, MaxRowsParam, SortByParam = "interval", "max_rows", "sort_by"


def SortStats(stats, sort_by, col_map, pos=None):
    """top.go:39-41: columnssort.SortEntries(*colMap, stats, sortBy)."""
    return SortEntries(col_map, stats, sort_by, pos=pos)


def ComputeIterations(interval: float, timeout: float) -> int:
    """top.go:45-56."""
    if timeout <= 0:
        return 0
    if timeout < interval:
        raise ValueError("timeout must be greater than interval")
    if (timeout / interval) != int(timeout / interval):
        raise ValueError("timeout must be a multiple of interval")
    return int(timeout / interval)
