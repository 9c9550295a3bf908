"""Column schema + SoA event batches (the pkg/columns analogue).

Reference: pkg/columns/columns.go (NewColumns :51, GetColumn lower-cases :83-86,
AddColumn virtual columns :282-309, SetExtractor :320-332) and columninfo.go (Column
:43-66, `group:sum` tag :159-171).  The reference reads fields of []*T through reflection
offsets (GetField, columns.go:343-347); here every column is a device array (SoA) of a
fixed width, which is what the gfx950 kernels stream.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from . import _abi
from .runtime import torch_mod

# Go reflect kind -> (igx kind class, width in bytes; strings take their declared width)
KINDS = {
    "int": (_abi.KIND_INT, 8), "int8": (_abi.KIND_INT, 1), "int16": (_abi.KIND_INT, 2),
    "int32": (_abi.KIND_INT, 4), "int64": (_abi.KIND_INT, 8),
    "uint": (_abi.KIND_UINT, 8), "uint8": (_abi.KIND_UINT, 1), "uint16": (_abi.KIND_UINT, 2),
    "uint32": (_abi.KIND_UINT, 4), "uint64": (_abi.KIND_UINT, 8),
    "float32": (_abi.KIND_FLOAT, 4), "float64": (_abi.KIND_FLOAT, 8),
    "string": (_abi.KIND_BYTES, None), "bool": (_abi.KIND_BOOL, 1),
    "struct": (_abi.KIND_OTHER, 0),
}

GroupTypeNone, GroupTypeSum = 0, 1          # types.go:26-31
OrderAsc, OrderDesc = True, False           # types.go:37-38


def torch_dtype(kind: str):
    torch = torch_mod()
    return {"int": torch.int64, "int8": torch.int8, "int16": torch.int16, "int32": torch.int32,
            "int64": torch.int64, "uint": torch.uint64, "uint8": torch.uint8,
            "uint16": torch.uint16, "uint32": torch.uint32, "uint64": torch.uint64,
            "float32": torch.float32, "float64": torch.float64, "bool": torch.bool}[kind]


@dataclass
class Column:
    Name: str
    kind: str                        # Go reflect kind name
    width: int = 0                   # bytes per row (strings: fixed width)
    GroupType: int = GroupTypeNone
    virtual: bool = False
    extractor: Optional[Callable] = None

    def Kind(self):
        return self.kind

    def IsVirtual(self):
        return self.virtual

    def HasCustomExtractor(self):
        return self.extractor is not None

    @property
    def igx_kind(self):
        return KINDS[self.kind][0]


class Columns:
    """NewColumns[T] for a flat SoA schema.  fields: (name, kind[, width][, "group:sum"])."""

    def __init__(self, fields=()):
        self._cols: Dict[str, Column] = {}
        self._order: List[str] = []
        for f in fields:
            name, kind = f[0], f[1]
            width = None
            group = GroupTypeNone
            for extra in f[2:]:
                if isinstance(extra, int):
                    width = extra
                elif extra == "group:sum":
                    group = GroupTypeSum
            kc, w = KINDS[kind]
            if w is None:
                if width is None:
                    raise ValueError(f"string column {name!r} needs a fixed width")
                w = width
            self._add(Column(name, kind, w, group))

    def _add(self, col: Column):
        key = col.Name.lower()
        if key in self._cols:
            raise ValueError(f"duplicate column name {col.Name!r}")
        self._cols[key] = col
        self._order.append(key)
        self._schema = None

    # -- reference API -------------------------------------------------------------
    def GetColumn(self, name: str):
        c = self._cols.get(name.lower())
        return c, c is not None

    def GetColumnMap(self):
        return self

    def GetOrderedColumns(self):
        return [self._cols[k] for k in self._order]

    def AddColumn(self, name: str, extractor: Callable):
        """Virtual column (columns.go:282-309): kind String, no backing field."""
        self._add(Column(name, "string", 0, virtual=True, extractor=extractor))

    def SetExtractor(self, name: str, fn: Callable):
        """columns.go:320-332; sorting still uses the raw field kind (sort.go:46-48)."""
        c, ok = self.GetColumn(name)
        if not ok:
            raise KeyError(name)
        c.extractor = fn
        self._schema = None

    MustAddColumn = AddColumn
    MustSetExtractor = SetExtractor

    # -- igx plumbing ----------------------------------------------------------------
    def index(self, name: str) -> int:
        return self._order.index(name.lower())

    def names(self):
        return [self._cols[k].Name for k in self._order]

    def schema(self):
        """ctypes igx_schema_col array (cached; names kept alive on self)."""
        if self._schema is None:
            cols = self.GetOrderedColumns()
            self._names = [c.Name.lower().encode() for c in cols]
            arr = (_abi.SchemaCol * max(1, len(cols)))()
            for i, c in enumerate(cols):
                flags = (_abi.COL_VIRTUAL if c.virtual else 0) | \
                        (_abi.COL_EXTRACTOR if (c.extractor and not c.virtual) else 0)
                kind = _abi.KIND_BYTES if (c.extractor is not None) else c.igx_kind
                arr[i] = _abi.SchemaCol(self._names[i], kind, c.width, flags, c.igx_kind)
            self._schema = (arr, len(cols))
        return self._schema


class EventBatch:
    """SoA batch on the device: name -> tensor ((n,) scalars or (n, W) uint8 strings),
    plus an optional `valid` uint8 mask (0 = nil entry, as a nil *T in the reference).

    A batch may be a *view*: a selection vector `sel` (u32 device tensor of row ids into the
    base columns) over another batch's columns -- what the reference's FilterEntries and
    SortEntries return: a fresh slice of pointers to the same entries (filter.go:294-325,
    sort.go:116-123), no entry copied.  Taking rows of a view composes the selection; a
    column of a view is gathered on first access (`batch[name]`, `data`, `valid`)."""

    def __init__(self, cols: Columns, data: dict, valid=None, sel=None, sel_count=None):
        self.cols = cols
        self._base = {k.lower(): v for k, v in data.items()}
        self._base_valid = valid
        any_t = next(iter(self._base.values())) if self._base else valid
        self.base_n = 0 if any_t is None else int(any_t.shape[0])
        self.sel = sel
        # a selection whose length is still on the device (u64 tensor): `sel` then has the
        # capacity of its upper bound and `n` synchronises on first use (FilterEntries ->
        # SortEntries runs without a host round trip: filter.FilterEntries, sort.Sort)
        self.sel_count = sel_count if sel is not None else None
        self._mat = {}
        self._valid_mat = None
        self._n = None if self.sel_count is not None else (self.base_n if sel is None else int(sel.shape[0]))

    @property
    def n(self):
        if self._n is None:
            k = int(self.sel_count.item())
            self.sel = self.sel[:k]
            self.sel_count = None
            self._n = k
        return self._n

    @n.setter
    def n(self, v):
        self._n = v

    def pending(self):
        """(selection of capacity n_max, device count) while the length is on the device, else None."""
        return (self.sel, self.sel_count) if self.sel_count is not None else None

    def __len__(self):
        return self.n

    def _gather(self, t):
        from . import engine                 # igx_take on the device
        self.n                               # a device-side length is read (and sel trimmed) first
        return engine.take([t], self.sel, self.base_n)[0]

    def __getitem__(self, name):
        name = name.lower()
        if self.sel is None:
            return self._base[name]
        if name not in self._mat:
            self._mat[name] = self._gather(self._base[name])
        return self._mat[name]

    def _own(self):
        """Turn a view into a plain batch of its rows (every column gathered once)."""
        if self.sel is None:
            return
        cols = {k: self[k] for k in self._base}
        valid = self.valid
        self._base, self._base_valid, self.sel = cols, valid, None
        self._mat, self._valid_mat = {}, None
        self.base_n = self.n

    @property
    def data(self):
        """Every column (a view becomes a plain batch of its rows first: the dict may be
        written to)."""
        self._own()
        return self._base

    @property
    def valid(self):
        if self.sel is None or self._base_valid is None:
            return self._base_valid
        if self._valid_mat is None:
            self._valid_mat = self._gather(self._base_valid)
        return self._valid_mat

    @valid.setter
    def valid(self, v):
        self._own()
        self._base_valid = v

    def base(self):
        """(base columns, base valid mask, selection or None) -- for passes that read a view
        through its selection vector instead of gathering it."""
        self.n
        return self._base, self._base_valid, self.sel

    def device(self):
        t = next(iter(self._base.values()))
        return t.device

    def tensors_in_schema_order(self):
        """One tensor per schema column (virtual columns get a 1-byte placeholder)."""
        torch = torch_mod()
        out = []
        for c in self.cols.GetOrderedColumns():
            t = self.data.get(c.Name.lower())
            if t is None:
                t = torch.zeros(max(1, self.n), dtype=torch.uint8, device=self.device())
            out.append(t)
        return out

    def take(self, idx):
        """Rows idx (device ids into this batch) as a view: the selection vector composed,
        no column copied (gather a column with batch[name], or all with materialize())."""
        if self.sel is None:
            sel = idx
        else:
            from . import engine
            n = self.n    # read first: reading n trims a pending (device-count) selection
            sel = engine.take([self.sel], idx, n)[0]
        return EventBatch(self.cols, self._base, self._base_valid, sel=sel)

    def materialize(self):
        """This batch as a plain batch of its rows (every column gathered)."""
        self._own()
        return self

    def to_host(self):
        return {k: host(v) for k, v in self.data.items()}


def host(t):
    """Device tensor -> numpy (unsigned shell dtypes through a signed view)."""
    import numpy as np
    torch = torch_mod()
    m = {torch.uint16: (torch.int16, np.uint16), torch.uint32: (torch.int32, np.uint32),
         torch.uint64: (torch.int64, np.uint64)}
    if t.dtype in m:
        alt, npd = m[t.dtype]
        return t.view(alt).cpu().numpy().view(npd)
    return t.cpu().numpy()


def to_device(a, device="cuda"):
    """numpy -> device tensor keeping unsigned widths."""
    import numpy as np
    torch = torch_mod()
    m = {np.dtype(np.uint16): (np.int16, torch.uint16), np.dtype(np.uint32): (np.int32, torch.uint32),
         np.dtype(np.uint64): (np.int64, torch.uint64)}
    a = np.ascontiguousarray(a)
    if a.dtype in m:
        sd, td = m[a.dtype]
        return torch.from_numpy(a.view(sd)).to(device).view(td)
    return torch.from_numpy(a).to(device)
