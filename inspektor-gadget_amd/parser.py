"""pkg/parser on the GPU path: the filter -> sort -> callback pipeline every gadget's
events pass through on their way to the frontends.

Reference: pkg/parser/parser.go -- NewParser (:112-117), SetSorting (:362-370),
SetFilters (:372-384), SetEventCallback (:155-176), eventHandler (:184-197),
eventHandlerArray (:199-224), JSONHandlerFuncArray (:263-288), EnableSnapshots (:119-137),
EnableCombiner / Flush (:139-150); VerifyColumnNames is pkg/columns/columns.go:137-152;
the snapshot combiner is pkg/snapshotcombiner/snapshotcombiner.go:56-106.

Events arrive as EventBatch objects (SoA device columns, optional nil mask) instead of
[]*T.  A batch stands for the reference's array callback argument; the per-event handler
takes a batch too and delivers the events that pass the filters in their original order,
which is what calling the reference's per-event handler on each of them does.  MatchAll
runs as one order-preserving device compaction (igx_filter), Sort as one device radix
sort with Go's SliceStable tie order (igx_sort_perm).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from .columns import Columns, EventBatch
from . import filter as _filter
from . import sort as _sort
from .runtime import torch_mod


class ParserError(ValueError):
    pass


def VerifyColumnNames(cols: Columns, names):
    """columns.go:139-152: lower-case, strip one '-' prefix, split known / unknown."""
    valid, invalid = [], []
    for n in names:
        n = n.lower()
        if n.startswith("-"):
            n = n[1:]
        (valid if cols.GetColumn(n)[1] else invalid).append(n)
    return valid, invalid


def _go_list(xs):
    return "[" + " ".join(xs) + "]"


def concat(batches: List[EventBatch]) -> Optional[EventBatch]:
    """Concatenate batches of one schema (device), keeping order."""
    batches = [b for b in batches if b is not None]
    if not batches:
        return None
    if len(batches) == 1:
        return batches[0]
    torch = torch_mod()
    cols = batches[0].cols
    data = {k: torch.cat([b.data[k] for b in batches]) for k in batches[0].data}
    valid = None
    if any(b.valid is not None for b in batches):
        valid = torch.cat([b.valid if b.valid is not None else
                           torch.ones(b.n, dtype=torch.uint8, device=b.device()) for b in batches])
    return EventBatch(cols, data, valid)


@dataclass
class CombinerStats:
    """snapshotcombiner.Stats (snapshotcombiner.go:23-28)."""
    Epochs: int = 0
    CurrentSnapshots: int = 0
    ExpiredSnapshots: int = 0
    TotalSnapshots: int = 0


class SnapshotCombiner:
    """snapshotcombiner.go:56-106: per-key latest snapshot with a TTL counted in
    GetSnapshots calls.  Concatenation follows key insertion order (the reference
    iterates a Go map: unordered)."""

    def __init__(self, ttl: int):
        self.defaultTTL = ttl
        self.snaps: Dict[str, list] = {}     # key -> [snapshot, ttl, count]
        self.epoch = 0

    def AddSnapshot(self, key: str, snapshot: EventBatch):
        if key in self.snaps:
            e = self.snaps[key]
            e[0], e[1], e[2] = snapshot, self.defaultTTL, e[2] + 1
        else:
            self.snaps[key] = [snapshot, self.defaultTTL, 1]

    def GetSnapshots(self):
        self.epoch += 1
        st = CombinerStats(Epochs=self.epoch)
        out = []
        for e in self.snaps.values():
            if e[1] == self.defaultTTL:
                st.CurrentSnapshots += 1
            if e[1] > 0:
                out.append(e[0])
                e[1] -= 1
            else:
                st.ExpiredSnapshots += 1
        st.TotalSnapshots = len(self.snaps)
        return concat(out), st


class Parser:
    """parser[T] for one Columns schema."""

    def __init__(self, cols: Columns):
        self.columns = cols
        self.sortBy: List[str] = []
        self.sortSpec: Optional[_sort.ColumnSorterCollection] = None
        self.filters: List[str] = []
        self.filterSpecs: Optional[_filter.FilterSpecs] = None
        self.eventCallback: Optional[Callable] = None
        self.eventCallbackArray: Optional[Callable] = None
        self.snapshotCombiner: Optional[SnapshotCombiner] = None
        self.eventCombinerEnabled = False
        self.combinedEvents: List[EventBatch] = []

    # -- configuration -----------------------------------------------------------------
    def GetColumns(self):
        return self.columns.GetColumnMap()

    def VerifyColumnNames(self, names):
        return VerifyColumnNames(self.columns, names)

    def SetSorting(self, sortBy):
        _, invalid = self.VerifyColumnNames(sortBy)
        if invalid:
            raise ParserError(f"invalid columns to sort by: {_go_list(invalid)}")
        self.sortSpec = _sort.Prepare(self.columns, sortBy)
        self.sortBy = list(sortBy)

    def SetFilters(self, filters):
        if not filters:
            return
        self.filterSpecs = _filter.GetFiltersFromStrings(self.columns, filters)
        self.filters = list(filters)

    def SetEventCallback(self, cb: Callable, array: bool = True):
        """The reference switches on the callback's Go type; here `array` says whether it
        takes a whole batch (func([]*T)) or the events one by one (func(*T))."""
        if array:
            self.eventCallbackArray = cb
        else:
            self.eventCallback = cb

    def EnableSnapshots(self, ttl: int):
        """parser.go:119-137 without the ticker goroutine: call Tick() per interval."""
        if self.eventCallbackArray is None:
            raise RuntimeError("EnableSnapshots needs EventCallbackArray set")
        self.snapshotCombiner = SnapshotCombiner(ttl)

    def Tick(self):
        out, _ = self.snapshotCombiner.GetSnapshots()
        self.eventCallbackArray(out)

    def EnableCombiner(self):
        if self.eventCallbackArray is None:
            raise RuntimeError("eventCallbackArray has to be set before using EnableCombiner()")
        self.eventCombinerEnabled = True
        self.combinedEvents = []

    def Flush(self):
        self.eventCallbackArray(concat(self.combinedEvents))

    # -- handlers ----------------------------------------------------------------------
    def _match(self, batch: EventBatch) -> EventBatch:
        if batch is None or self.filterSpecs is None:
            return batch
        return batch.take(self.filterSpecs.MatchAll(batch))

    def eventHandler(self, cb, enrichers=()):
        if cb is None:
            raise RuntimeError("cb can't be nil in eventHandler from parser")

        def handle(batch: EventBatch):
            for e in enrichers:
                e(batch)
            out = self._match(batch)
            if out is not None and out.n:
                cb(out)
        return handle

    def eventHandlerArray(self, cb, enrichers=()):
        if cb is None:
            raise RuntimeError("cb can't be nil in eventHandlerArray from parser")

        def handle(batch: EventBatch):
            for e in enrichers:
                e(batch)
            out = self._match(batch)
            if self.sortSpec is not None and out is not None:
                out = self.sortSpec.Sort(out)
            cb(out)
        return handle

    def EventHandlerFunc(self, *enrichers):
        return self.eventHandler(self.eventCallback, enrichers)

    def EventHandlerFuncArray(self, *enrichers):
        return self.eventHandlerArray(self.eventCallbackArray, enrichers)

    def BatchHandlerFuncArray(self, key: str, *enrichers):
        """JSONHandlerFuncArray (parser.go:263-288) minus the JSON decoding: batches from
        source `key` go to the combiner or snapshot combiner when enabled."""
        cb = self.eventCallbackArray
        if self.eventCombinerEnabled:
            cb = self.combinedEvents.append
        elif self.snapshotCombiner is not None:
            sc = self.snapshotCombiner
            cb = lambda b: sc.AddSnapshot(key, b)   # noqa: E731
        return self.eventHandlerArray(cb, enrichers)


def NewParser(cols: Columns) -> Parser:
    return Parser(cols)
