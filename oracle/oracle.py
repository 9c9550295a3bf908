"""CPU oracle for the igx event-aggregation path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product package (``inspektor-gadget_amd``) never imports it.

Two halves:

* ctypes bindings to ``liboracle.so`` (``igx_oracle.c``): bulk integer work -- filter
  evaluation, Go ``sort.SliceStable`` restatement, keyed aggregation, log2 histograms,
  synthetic generators -- fast enough for parity at 1M-10M rows.
* pure-Python restatements of the small, string-heavy reference logic:
  ``GetFilterFromString`` parsing (pkg/columns/filter/filter.go:53-172),
  ``GroupEntries`` (pkg/columns/group/group.go:27-165), the Go stable sort on tiny inputs
   and the closed-form tie order, ``getReport``
  (pkg/gadgets/profile/block-io/tracer/tracer.go:56-90) and the network-policy advisor
  (pkg/gadgets/advise/networkpolicy/advisor/advisor.go:100-387).

Pinning: every restatement here is checked against the reference's own table tests and
golden files re-encoded under ``tests/golden`` (tests/test_oracle_golden.py).  The DESC
tie order of the Go stdlib sort is pinned only by the transliteration itself ("parity
unpinned" at the Go-stdlib boundary).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import re
import subprocess
import struct
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else C.c_void_p(0)


def _declare(L):
    u64, vp = C.c_uint64, C.c_void_p
    L.or_gen_tcp.argtypes = [u64] * 5 + [vp, u64, u64] + [vp] * 10
    L.or_gen_open.argtypes = [u64, vp, u64, u64] + [vp] * 8
    L.or_gen_bio.argtypes = [u64, vp, u64, u64, u64, vp, vp, vp]
    L.or_gen_np.argtypes = [u64, u64, u64, u64, u64] + [vp] * 8
    L.or_gen_file.argtypes = [u64] * 5 + [vp, u64, u64] + [vp] * 6
    L.or_filter.argtypes = [vp, C.c_uint32, vp, u64, vp]
    L.or_filter.restype = u64
    L.or_sort_entries.argtypes = [vp, u64, vp, vp, C.c_uint32]
    L.or_groupby.argtypes = [vp, C.c_uint32, u64, vp, vp, C.c_uint32, u64, u64, vp, vp, vp]
    L.or_groupby.restype = u64
    L.or_log2l.argtypes = [u64]
    L.or_log2l.restype = u64
    L.or_hist_log2.argtypes = [vp, vp, vp, u64, vp, C.c_uint32, C.c_uint32, u64,
                               C.c_uint32, vp]
    L.or_top_tcp.argtypes = [vp] * 10 + [u64, u64, u64, C.c_uint32, vp, vp, vp, vp]
    L.or_top_tcp.restype = u64
    L.or_top_tcp_mt.argtypes = [vp] * 10 + [u64, u64, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
    L.or_top_tcp_mt.restype = u64
    L.or_groupby_topk_mt.argtypes = [vp, C.c_uint32, u64, vp, vp, C.c_uint32, u64, C.c_uint32, vp, vp,
                                     C.c_uint32, C.c_uint32, vp, vp, vp]
    L.or_groupby_topk_mt.restype = u64
    L.or_hist_log2_mt.argtypes = [vp, vp, vp, u64, vp, C.c_uint32, C.c_uint32, u64, C.c_uint32, vp,
                                  C.c_uint32]
    L.or_np_advise_strings.argtypes = [vp] * 7 + [u64]
    L.or_np_advise_strings.restype = u64


# ------------------------------------------------------------------------------------
# column vocabulary (Go reflect kinds -> width/class)
# ------------------------------------------------------------------------------------
KIND_CLASS = {
    "int": ("int", 8), "int8": ("int", 1), "int16": ("int", 2), "int32": ("int", 4),
    "int64": ("int", 8), "uint": ("uint", 8), "uint8": ("uint", 1), "uint16": ("uint", 2),
    "uint32": ("uint", 4), "uint64": ("uint", 8), "float32": ("float", 4),
    "float64": ("float", 8), "string": ("string", None), "bool": ("bool", 1),
    "struct": ("struct", 0),
}
CLASS_CODE = {"int": 0, "uint": 1, "float": 2, "string": 3}
OPS = {"eq": 0, "lt": 2, "le": 3, "gt": 4, "ge": 5}


@dataclass
class OCol:
    name: str
    kind: str            # reflect kind name, e.g. "int8", "string"
    width: int = 0       # bytes per row in the SoA batch (strings: fixed width)
    virtual: bool = False
    extractor: bool = False


class FilterError(Exception):
    pass


@dataclass
class OPred:
    col: OCol
    op: str
    negate: bool
    ref: bytes = b""
    regex: object = None


def _parse_int(s: str, bits=64):
    # strconv.ParseInt(s, 10, 64): optional sign, decimal digits only, range-checked
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        raise ValueError(s)
    v = int(s, 10)
    if not (-(1 << 63) <= v < (1 << 63)):
        raise ValueError(s)
    return v


def _parse_uint(s: str):
    # strconv.ParseUint(s, 10, 64): no sign, decimal digits only
    if not re.fullmatch(r"[0-9]+", s):
        raise ValueError(s)
    v = int(s, 10)
    if v >= (1 << 64):
        raise ValueError(s)
    return v


def _parse_float(s: str):
    # strconv.ParseFloat(s, 64) (decimal / exponent / inf / nan forms)
    t = s.lower()
    if t in ("inf", "+inf", "infinity", "+infinity"):
        return math.inf
    if t in ("-inf", "-infinity"):
        return -math.inf
    if t == "nan":
        return math.nan
    if not re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)(e[+-]?\d+)?", t):
        raise ValueError(s)
    return float(t)


def parse_filter(cols: dict, filt: str) -> OPred:
    """GetFilterFromString (filter.go:91-172) + getValueFromFilterSpec (:53-87)."""
    info = filt.split(":", 1)
    if len(info) == 1:
        info.append("")                                   # :93-96
    col = cols.get(info[0].lower())                       # columns.go:84 lower-cases
    if col is None:
        raise FilterError(f'could not apply filter: column "{info[0]}" not found')
    rule = info[1]
    negate = False
    if rule.startswith("!"):                              # :113-117
        negate = True
        rule = rule[1:]
    op = "eq"
    regex = None
    if rule.startswith("~"):                              # :119-127
        op = "regex"
        rule = rule[1:]
        try:
            regex = re.compile(rule)
        except re.error as e:
            raise FilterError(f"could not compile regular expression {rule!r}: {e}")
    elif rule.startswith(">="):
        op, rule = "ge", rule[2:]
    elif rule.startswith(">"):
        op, rule = "gt", rule[1:]
    elif rule.startswith("<="):
        op, rule = "le", rule[2:]
    elif rule.startswith("<"):
        op, rule = "lt", rule[1:]
    cls, w = KIND_CLASS[col.kind]
    if op == "regex":
        if cls != "string":                               # :146-148
            raise FilterError(f'tried to apply regular expression on non-string column "{col.name}"')
        return OPred(col, op, negate, regex=regex)
    if cls == "int":
        try:
            v = _parse_int(rule)
        except ValueError:
            raise FilterError(f'tried to compare "{rule}" to int column "{col.name}"')
        ref = (v & ((1 << (8 * w)) - 1)).to_bytes(w, "little")   # Convert() truncates
    elif cls == "uint":
        try:
            v = _parse_uint(rule)
        except ValueError:
            raise FilterError(f'tried to compare "{rule}" to uint column "{col.name}"')
        ref = (v & ((1 << (8 * w)) - 1)).to_bytes(w, "little")
    elif cls == "float":
        try:
            v = _parse_float(rule)
        except ValueError:
            raise FilterError(f'tried to compare "{rule}" to float column "{col.name}"')
        ref = struct.pack("<f" if w == 4 else "<d", v)
    elif cls == "string":
        b = rule.encode()
        ref = b[: col.width].ljust(col.width, b"\0")
        if len(b) > col.width:
            # a reference longer than the fixed-width column: equality can never hold
            ref = b
    else:
        raise FilterError(f'tried to match "{rule}" on unsupported column "{col.name}"')
    return OPred(col, op, negate, ref=ref)


class _CPred(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("width", C.c_uint32), ("kind", C.c_uint32),
                ("op", C.c_uint32), ("negate", C.c_uint32), ("ref", C.c_void_p)]


def match_rows(preds, batch: dict, valid=None):
    """MatchAll over SoA rows (filter.go:266-273); FilterEntries order (:294-325).
    Returns the selected row indices (np.uint32)."""
    n = len(valid) if valid is not None else len(next(iter(batch.values())))
    keep = np.ones(n, dtype=bool) if valid is None else valid.astype(bool).copy()
    cpreds = []
    refbufs = []
    for p in preds:
        col = batch[p.col.name]
        if p.op == "regex":
            sel = np.zeros(n, dtype=bool)
            for i in range(n):
                if keep[i]:
                    s = bytes(col[i]).rstrip(b"\0").decode(errors="replace")
                    sel[i] = (p.regex.search(s) is not None) != p.negate
            keep &= sel
            continue
        cls, w = KIND_CLASS[p.col.kind]
        if cls == "string" and len(p.ref) > p.col.width:
            # longer reference than the column: compare as Go strings in Python
            sel = np.zeros(n, dtype=bool)
            for i in range(n):
                s = bytes(col[i]).rstrip(b"\0")
                c = (s > p.ref) - (s < p.ref)
                r = {"eq": c == 0, "lt": c < 0, "le": c <= 0, "gt": c > 0, "ge": c >= 0}[p.op]
                sel[i] = r != p.negate
            keep &= sel
            continue
        rb = np.frombuffer(p.ref, dtype=np.uint8).copy()
        refbufs.append(rb)
        colc = np.ascontiguousarray(col)
        refbufs.append(colc)
        cpreds.append(_CPred(colc.ctypes.data, p.col.width if cls == "string" else w,
                             CLASS_CODE[cls], OPS[p.op], int(p.negate), rb.ctypes.data))
    arr = (_CPred * max(1, len(cpreds)))(*cpreds)
    valid8 = keep.astype(np.uint8)
    out = np.empty(n, dtype=np.uint32)
    k = lib().or_filter(C.cast(arr, C.c_void_p), len(cpreds), _p(valid8), n, _p(out))
    return out[:k]


def match_all(preds, batch: dict, valid=None):
    """FilterSpecs.MatchAll applied to every entry (filter.go:266-273), nil entries included:
    FilterSpec.Match(nil) returns its negate flag (:286-291), so a nil entry is kept iff every
    spec is negated (vacuously with no specs).  Returns the kept row indices (np.uint32)."""
    sel = match_rows(preds, batch, valid)
    if valid is None or not all(p.negate for p in preds):
        return sel
    nil = np.nonzero(~np.asarray(valid).astype(bool))[0].astype(np.uint32)
    return np.union1d(sel, nil).astype(np.uint32)


def match_any(preds, batch: dict, valid=None):
    """FilterSpecs.MatchAny per entry (filter.go:276-283): no specs keep nothing; a nil entry
    is kept iff some spec is negated (Match(nil) == negate, :286-291)."""
    if not preds:
        return np.zeros(0, np.uint32)
    sel = np.zeros(0, np.uint32)
    for p in preds:
        sel = np.union1d(sel, match_rows([p], batch, valid))
    if valid is not None and any(p.negate for p in preds):
        nil = np.nonzero(~np.asarray(valid).astype(bool))[0]
        sel = np.union1d(sel, nil)
    return sel.astype(np.uint32)


def filter_entries(cols: dict, batch: dict, valid, filters):
    """FilterEntries (filter.go:294-325) over SoA rows: returns the kept row ids in order, or
    None where the reference returns a nil slice (nil input; no filters, since only the
    filter loop assigns outEntries)."""
    if batch is None:
        return None
    out = None
    ids = np.arange(len(next(iter(batch.values()))), dtype=np.uint32)
    v = None if valid is None else np.asarray(valid).astype(bool)
    for f in filters:
        p = parse_filter(cols, f)
        sub = {k: np.asarray(a)[ids] for k, a in batch.items()}
        keep = match_rows([p], sub, None if v is None else v[ids])
        ids = ids[keep]
        out = ids
    return out


# ------------------------------------------------------------------------------------
# sort
# ------------------------------------------------------------------------------------
class _CSortKey(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("width", C.c_uint32), ("kind", C.c_uint32),
                ("desc", C.c_uint32)]


def go_sort_entries(keys, n, valid=None, perm=None):
    """SortEntries via the Go 1.19 SliceStable restatement (C).  keys = list of
    (np column indexed by row id, kind, desc) in sortBy order.  Returns the permutation
    (row ids in output order) starting from `perm` (default identity)."""
    perm = np.arange(n, dtype=np.uint32) if perm is None else np.array(perm, dtype=np.uint32)
    ks, hold = [], []
    for colarr, kind, desc in keys:
        cls, w = KIND_CLASS[kind]
        a = np.ascontiguousarray(colarr)
        hold.append(a)
        width = a.shape[1] if cls == "string" else w
        ks.append(_CSortKey(a.ctypes.data, width, CLASS_CODE[cls], int(desc)))
    arr = (_CSortKey * max(1, len(ks)))(*ks)
    v8 = None if valid is None else np.ascontiguousarray(valid.astype(np.uint8))
    lib().or_sort_entries(_p(perm), len(perm), _p(v8), C.cast(arr, C.c_void_p), len(ks))
    return perm


def go_slice_stable_py(data: list, less):
    """Pure-Python transliteration of Go 1.19 sort.SliceStable;
    `less(i, j)` reads the live list.  For small inputs only."""
    n = len(data)

    def swap(i, j):
        data[i], data[j] = data[j], data[i]

    def insertion(a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and less(j, j - 1):
                swap(j, j - 1)
                j -= 1

    def swap_range(a, b, m):
        for t in range(m):
            swap(a + t, b + t)

    def rotate(a, m, b):
        i, j = m - a, b - m
        while i != j:
            if i > j:
                swap_range(m - i, m, j)
                i -= j
            else:
                swap_range(m - i, m + j - i, i)
                j -= i
        swap_range(m - i, m, i)

    def sym_merge(a, m, b):
        if m - a == 1:
            i, j = m, b
            while i < j:
                h = (i + j) >> 1
                if less(h, a):
                    i = h + 1
                else:
                    j = h
            for k in range(a, i - 1):
                swap(k, k + 1)
            return
        if b - m == 1:
            i, j = a, m
            while i < j:
                h = (i + j) >> 1
                if not less(m, h):
                    i = h + 1
                else:
                    j = h
            for k in range(m, i, -1):
                swap(k, k - 1)
            return
        mid = (a + b) >> 1
        nn = mid + m
        if m > mid:
            start, r = nn - b, mid
        else:
            start, r = a, m
        p = nn - 1
        while start < r:
            c = (start + r) >> 1
            if not less(p - c, c):
                start = c + 1
            else:
                r = c
        end = nn - start
        if start < m < end:
            rotate(start, m, end)
        if a < start < mid:
            sym_merge(a, start, mid)
        if mid < end < b:
            sym_merge(mid, end, b)

    bs, a, b = 20, 0, 20
    while b <= n:
        insertion(a, b)
        a, b = b, b + bs
    insertion(a, n)
    while bs < n:
        a, b = 0, 2 * bs
        while b <= n:
            sym_merge(a, a + bs, b)
            a, b = b, b + 2 * bs
        if a + bs < n:
            sym_merge(a, a + bs, n)
        bs *= 2
    return data


def go_sort_entries_py(rows: list, keys):
    """SortEntries on a list of row values (None = nil entry) using the pure-Python Go
    stable sort; keys = [(getter, desc)] in sortBy order (sort.go:35-135)."""
    data = list(rows)
    for getter, desc in reversed(keys):
        def less(i, j, getter=getter, desc=desc):
            if data[i] is None:
                return False
            if data[j] is None:
                return True
            return (not (getter(data[i]) < getter(data[j]))) != (not desc)
        go_slice_stable_py(data, less)
    return data


def closed_form_perm(key_values, descs, n):
    """SURVEY.md §0.3 closed form: effective direction of key i is desc_i XOR
    (desc_1 ^ ... ^ desc_{i-1}); final tie-break is the pre-sort position, ascending
    iff sum(desc) is even.  key_values: list of sequences of comparable python values."""
    eff, par = [], 0
    for d in descs:
        eff.append(bool(d) ^ bool(par))
        par ^= int(bool(d))

    class K:
        __slots__ = ("i",)

        def __init__(self, i):
            self.i = i

        def __lt__(self, o):
            for vals, e in zip(key_values, eff):
                a, b = vals[self.i], vals[o.i]
                if a != b:
                    return (a > b) if e else (a < b)
            return (self.i > o.i) if par else (self.i < o.i)

    return sorted(range(n), key=K)


# ------------------------------------------------------------------------------------
# keyed aggregation / histograms
# ------------------------------------------------------------------------------------
class _CAgg(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("val_width", C.c_uint32), ("val", C.c_void_p),
                ("cond_width", C.c_uint32), ("cond", C.c_void_p), ("cond_val", C.c_uint64),
                ("out_width", C.c_uint32), ("val_signed", C.c_uint32), ("div", C.c_uint64)]


def groupby(keys_packed: np.ndarray, aggs, valid=None, base_idx=0, max_groups=None):
    """Generic keyed aggregation in first-occurrence order.  keys_packed: (n, kb) uint8.
    aggs: list of dicts {kind: 'count'|'sum', val: array|None, cond: array|None,
    cond_val: int, out_width: int, div: int (sum of val // div per event)}.  Returns (keys (G,kb), aggs (naggs,G) u64, first)."""
    keys_packed = np.ascontiguousarray(keys_packed, dtype=np.uint8)
    n, kb = keys_packed.shape
    maxG = max_groups or max(1, n)
    cag, hold = [], []
    for a in aggs:
        val = a.get("val")
        cond = a.get("cond")
        if val is not None:
            val = np.ascontiguousarray(val)
            hold.append(val)
        if cond is not None:
            cond = np.ascontiguousarray(cond)
            hold.append(cond)
        cag.append(_CAgg(0 if a["kind"] == "count" else 1,
                         0 if val is None else val.dtype.itemsize,
                         0 if val is None else val.ctypes.data,
                         0 if cond is None else cond.dtype.itemsize,
                         0 if cond is None else cond.ctypes.data,
                         int(a.get("cond_val", 0)), int(a.get("out_width", 8)),
                         int(val is not None and val.dtype.kind == "i"), int(a.get("div", 0))))
    arr = (_CAgg * max(1, len(cag)))(*cag)
    out_keys = np.empty((maxG, kb), dtype=np.uint8)
    out_aggs = np.zeros((max(1, len(aggs)), maxG), dtype=np.uint64)
    out_first = np.empty(maxG, dtype=np.uint64)
    v8 = None if valid is None else np.ascontiguousarray(valid.astype(np.uint8))
    G = lib().or_groupby(_p(keys_packed), kb, n, _p(v8), C.cast(arr, C.c_void_p), len(cag),
                         base_idx, maxG, _p(out_keys), _p(out_aggs), _p(out_first))
    if G == (1 << 64) - 1:
        raise RuntimeError("oracle groupby: too many groups")
    return out_keys[:G], out_aggs[: len(aggs), :G], out_first[:G]


def log2l(v: int) -> int:
    return int(lib().or_log2l(v))


def hist_log2(dev, cont, delta, devs, ncont, divisor=1000, nslots=27):
    devs = np.ascontiguousarray(devs, dtype=np.uint32)
    hist = np.zeros((max(1, len(devs)) * ncont, nslots), dtype=np.uint32)
    delta = np.ascontiguousarray(delta).view(np.int64)
    dev = np.ascontiguousarray(np.zeros(len(delta), np.uint32) if dev is None else dev, dtype=np.uint32)
    cont = np.ascontiguousarray(np.zeros(len(delta), np.uint32) if cont is None else cont, dtype=np.uint32)
    delta = np.ascontiguousarray(delta).view(np.int64)
    lib().or_hist_log2(_p(dev), _p(cont), _p(delta), len(dev), _p(devs), len(devs), ncont,
                       divisor, nslots, _p(hist))
    return hist


def get_report(slots):
    """getReport (profile/block-io/tracer/tracer.go:56-90): Data[i] = {Count, 1<<i,
    (1<<(i+1))-1}, truncated to data[:indexMax] (drops the last non-zero slot)."""
    data, index_max = [], 0
    for i, v in enumerate(slots):
        if v > 0:
            index_max = i
        data.append({"count": int(v), "intervalStart": ((1 << (i + 1)) >> 1),
                     "intervalEnd": (1 << (i + 1)) - 1})
    return data[:index_max]


# ------------------------------------------------------------------------------------
# synthetic generators (bit-identical with csrc/k_gen.hip)
# ------------------------------------------------------------------------------------
def zipf_cdf(G: int, s: float) -> np.ndarray:
    """u63 fixed-point CDF thresholds of Zipf(s) over ranks 1..G; last == 1<<63."""
    k = np.arange(1, G + 1, dtype=np.float64)
    w = k ** (-s)
    c = np.cumsum(w)
    c /= c[-1]
    t = np.minimum(np.floor(c * float(1 << 63)), float(1 << 63)).astype(np.float64)
    out = np.empty(G, dtype=np.uint64)
    out[:] = t.astype(np.uint64)
    out[-1] = np.uint64(1 << 63)
    return out


def lognormal_quantiles(mu: float, sigma: float, nq: int = 4096, cap: int = 1 << 40):
    """nq+1 monotone quantile boundaries (u64 ns) of lognormal(mu, sigma), capped."""
    from scipy.stats import norm
    p = (np.arange(nq + 1, dtype=np.float64) + 0.5) / (nq + 1)
    q = np.exp(mu + sigma * norm.ppf(p))
    q = np.minimum(q, float(cap))
    q = np.maximum.accumulate(np.floor(q)).astype(np.uint64)
    return q


def perm_params(G: int):
    """Affine bijection r -> (r*A + B) mod G used to scramble key ranks."""
    A = 999983
    while math.gcd(A, G) != 1:
        A += 2
    return A % G if G > 1 else 1, 12345 % G if G > 1 else 0


_PAR_MIN = 4_000_000


def _par_gen(fn, head, base, n, outs, threads=None):
    """Run a counter-based generator (event i depends only on seed and base + i) on slices of
    [0, n) in threads; ctypes releases the GIL during each call.  Bit-identical to one call."""
    T = threads or cpu_threads()
    if n < _PAR_MIN or T == 1:
        fn(*head, base, n, *[_p(o) for o in outs])
        return
    from concurrent.futures import ThreadPoolExecutor
    cuts = [n * t // T for t in range(T + 1)]
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda t: fn(*head, base + cuts[t], cuts[t + 1] - cuts[t],
                                 *[_p(o[cuts[t]:cuts[t + 1]]) for o in outs]), range(T)))


def gen_tcp(seed, rank, G, cdf, base, n):
    A, B = perm_params(G)
    o = {
        "saddr": np.empty((n, 16), np.uint8), "daddr": np.empty((n, 16), np.uint8),
        "mntns": np.empty(n, np.uint64), "pid": np.empty(n, np.uint32),
        "comm": np.empty((n, 16), np.uint8), "lport": np.empty(n, np.uint16),
        "dport": np.empty(n, np.uint16), "family": np.empty(n, np.uint16),
        "size": np.empty(n, np.uint32), "dir": np.empty(n, np.uint8),
    }
    _par_gen(lib().or_gen_tcp, (seed, rank, G, A, B, _p(cdf)), base, n,
             [o[k] for k in ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")])
    return o


def gen_open(seed, comm_cdf, base, n):
    o = {"pid": np.empty(n, np.uint32), "uid": np.empty(n, np.uint32),
         "mntns": np.empty(n, np.uint64), "comm": np.empty((n, 16), np.uint8),
         "ret": np.empty(n, np.int64), "fd": np.empty(n, np.int64),
         "err": np.empty(n, np.int64), "path": np.empty(n, np.uint32)}
    lib().or_gen_open(seed, _p(comm_cdf), base, n,
                      *[_p(o[k]) for k in ("pid", "uid", "mntns", "comm", "ret", "fd", "err",
                                           "path")])
    return o


def gen_bio(seed, q, base, n):
    o = {"dev": np.empty(n, np.uint32), "cont": np.empty(n, np.uint32),
         "delta": np.empty(n, np.uint64)}
    _par_gen(lib().or_gen_bio, (seed, _p(q), len(q) - 1), base, n, [o["dev"], o["cont"], o["delta"]])
    return o


def gen_np(seed, nsrc, npeer, base, n):
    o = {"src": np.empty(n, np.uint32), "peer": np.empty(n, np.uint32),
         "port": np.empty(n, np.uint16), "pkt": np.empty(n, np.uint8),
         "type": np.empty(n, np.uint8), "proto": np.empty(n, np.uint8),
         "hostip": np.empty(n, np.uint32), "raddr": np.empty(n, np.uint32)}
    _par_gen(lib().or_gen_np, (seed, nsrc, npeer), base, n,
             [o[k] for k in ("src", "peer", "port", "pkt", "type", "proto", "hostip", "raddr")])
    return o


def gen_file(seed, rank, G, cdf, base, n):
    A, B = perm_params(G)
    o = {"inode": np.empty(n, np.uint64), "dev": np.empty(n, np.uint32),
         "pid": np.empty(n, np.uint32), "tid": np.empty(n, np.uint32),
         "op": np.empty(n, np.uint8), "count": np.empty(n, np.uint32)}
    _par_gen(lib().or_gen_file, (seed, rank, G, A, B, _p(cdf)), base, n,
             [o[k] for k in ("inode", "dev", "pid", "tid", "op", "count")])
    return o


def np_mark(ev):
    """advisor.go:279-292 on the encoded C4 stream: type normal (0), pkt HOST (0) or
    OUTGOING (4), and not (HOST and PodHostIP == RemoteAddr)."""
    t, p = ev["type"], ev["pkt"]
    return (t == 0) & ((p == 0) | (p == 4)) & ~((p == 0) & (ev["hostip"] == ev["raddr"]))


def np_advise_strings(ev):
    """or_np_advise_strings: GeneratePolicies' dedup on the reference's own string keys
    (advisor.go:130-159 key building, :279-320 maps) over an or_gen_np batch; returns the number
    of (source, direction, peer) entries = the distinct tuples of the device table."""
    cols = [np.ascontiguousarray(ev[k]) for k in ("src", "peer", "port", "pkt", "type", "hostip", "raddr")]
    return int(lib().or_np_advise_strings(*[_p(c) for c in cols], len(cols[0])))


def pad_keys(batch, names):
    """pack_cols with every column padded to 4 bytes (the device's packed key layout)."""
    parts = []
    for nm in names:
        a = np.ascontiguousarray(batch[nm])
        n = a.shape[0]
        b = a.view(np.uint8).reshape(n, -1)
        w = b.shape[1]
        if w % 4:
            b = np.concatenate([b, np.zeros((n, 4 - w % 4), np.uint8)], axis=1)
        parts.append(b)
    return np.concatenate(parts, axis=1)


TCP_KEY_COLS = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")


def pack_cols(batch, names):
    """Concatenate SoA columns row-wise into a (n, kb) uint8 key matrix."""
    parts = []
    for nm in names:
        a = np.ascontiguousarray(batch[nm])
        n = a.shape[0]
        parts.append(a.view(np.uint8).reshape(n, -1))
    return np.concatenate(parts, axis=1)


def top_tcp(ev, k=20, base_idx=0, max_groups=None):
    """Reference-shaped CPU path (igx_oracle.c §6).  Returns (G, rows) where rows are
    dicts for the first k sorted stats."""
    n = len(ev["pid"])
    maxG = max_groups or n
    keys = np.empty((k, 72), np.uint8)
    sent, recv, first = (np.empty(k, np.uint64) for _ in range(3))
    cols = [np.ascontiguousarray(ev[c]) for c in ("saddr", "daddr", "mntns", "pid", "comm",
                                                  "lport", "dport", "family", "size", "dir")]
    G = lib().or_top_tcp(*[_p(c) for c in cols], n, base_idx, maxG, k, _p(keys), _p(sent),
                         _p(recv), _p(first))
    m = min(k, G)
    return G, keys[:m], sent[:m], recv[:m], first[:m]


def from_cstring_rows(a, width):
    """gadgets.FromCString per row (bytes before the first NUL), zero-padded to width."""
    n, w = a.shape
    out = np.zeros((n, width), np.uint8)
    nul = (a == 0)
    first = np.where(nul.any(axis=1), nul.argmax(axis=1), w)
    keep = np.arange(w)[None, :] < first[:, None]
    out[:, :w] = np.where(keep, a, 0)
    return out


def decode_open_events(samples, boot_to_wall_ns=0):
    """trace/open/tracer/tracer.go:182-208 over raw perf samples (n, >=304) of struct event
    (opensnoop.h:14-24; bpf2go opensnoopEvent offsets ts 0, pid 8, uid 12, mntns 16, ret 24,
    flags 28, comm 32, fname 48..302)."""
    s = np.ascontiguousarray(samples)
    n = s.shape[0]
    u64 = lambda off: s[:, off:off + 8].copy().view(np.uint64).ravel()   # noqa: E731
    u32 = lambda off: s[:, off:off + 4].copy().view(np.uint32).ravel()   # noqa: E731
    ret = s[:, 24:28].copy().view(np.int32).ravel().astype(np.int64)
    return {"timestamp": (u64(0) + np.uint64(boot_to_wall_ns & 0xFFFFFFFFFFFFFFFF)).view(np.int64),
            "pid": u32(8), "uid": u32(12), "mntns": u64(16), "ret": ret,
            "fd": np.where(ret >= 0, ret, 0), "err": np.where(ret < 0, -ret, 0),
            "comm": from_cstring_rows(s[:, 32:48], 16), "path": from_cstring_rows(s[:, 48:303], 256)}


def ip_string(b16, family: int) -> str:
    """gadgets.IPStringFromBytes (pkg/gadgets/helpers.go:111-120) with ipType chosen as the
    tcp tracer does (top/tcp/tracer/tracer.go:199-206: 6 iff family == AF_INET6), restating
    Go's net/netip Addr.String: string4 dotted decimal; Is4In6 -> "::ffff:" + string4 of the
    last four bytes; else appendTo6 -- lowercase hex groups without leading zeros, the first
    longest run of >= 2 zero groups replaced by "::"."""
    b = bytes(b16)
    if family != 10:
        return ".".join(str(x) for x in b[:4])
    if b[:10] == bytes(10) and b[10:12] == b"\xff\xff":
        return "::ffff:" + ".".join(str(x) for x in b[12:16])
    g = [(b[2 * i] << 8) | b[2 * i + 1] for i in range(8)]
    zs, ze = 255, 255
    for i in range(8):
        j = i
        while j < 8 and g[j] == 0:
            j += 1
        if j - i >= 2 and j - i > ze - zs:
            zs, ze = i, j
    out = []
    i = 0
    while i < 8:
        if i == zs:
            out.append("::")
            i = ze
            if i >= 8:
                break
        elif i > 0:
            out.append(":")
        out.append("%x" % g[i])
        i += 1
    return "".join(out)


def ip_text_rows(addr, family, width=40):
    """(n, width) zero-padded ip_string texts (the device layout of igx_ip_text)."""
    n = addr.shape[0]
    out = np.zeros((n, width), np.uint8)
    memo = {}
    for i in range(n):
        key = (addr[i].tobytes(), int(family[i]))
        t = memo.get(key)
        if t is None:
            t = memo[key] = ip_string(key[0], key[1]).encode()
        out[i, :len(t)] = np.frombuffer(t, np.uint8)
    return out


# ------------------------------------------------------------------------------------
# GroupEntries (pkg/columns/group/group.go:27-165) on Python row objects
# ------------------------------------------------------------------------------------
def _go_string_from_value(v, kind):
    # getStringFromValue (group.go:27-47)
    cls = KIND_CLASS[kind][0]
    if cls in ("int", "uint"):
        return str(int(v))
    if cls == "float":
        return _go_format_float_E(float(v))
    return str(v)


def _go_format_float_E(f):
    """strconv.FormatFloat(f, 'E', -1, 64): shortest round-trip digits, d.dddE+dd."""
    if f != f:
        return "NaN"
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    if f == 0:
        return ("-" if math.copysign(1, f) < 0 else "") + "0E+00"
    s = repr(abs(f))
    mant, ex = (s.split("e")[0], int(s.split("e")[1])) if "e" in s else (s, 0)
    ip, fp = mant.split(".") if "." in mant else (mant, "")
    digits = ip + fp
    point = len(ip) + ex
    stripped = digits.lstrip("0")
    lead = len(digits) - len(stripped)
    stripped = stripped.rstrip("0")
    e10 = point - lead - 1
    m = stripped[0] + ("." + stripped[1:] if len(stripped) > 1 else "")
    return ("-" if f < 0 else "") + m + "E" + ("+" if e10 >= 0 else "-") + "%02d" % abs(e10)


def group_entries(cols: dict, entries: list, group_by: list, sum_cols: dict):
    """GroupEntries.  entries: list of dicts (None = nil).  cols: lower-name -> OCol.
    sum_cols: name -> kind for `group:sum` columns.  Map order is replaced by the
    canonical first-occurrence order; the result of each pass is then
    sorted ascending by the group column exactly as group.go:115 does."""
    if entries is None:
        return None, None
    new = entries
    for gname in group_by:
        gname = gname.lower()
        if gname == "":
            vals = [e for e in entries if e is not None]
            return [_flatten(vals, sum_cols)] if vals else [], None
        col = cols.get(gname)
        if col is None:
            return None, FilterError(f'could not group by "{gname}": column not found')
        groups = {}
        for e in new:
            if e is None:
                continue
            groups.setdefault(_go_string_from_value(e[col.name], col.kind), []).append(e)
        out = [_flatten(v, sum_cols) for v in groups.values()]
        out = go_sort_entries_py(out, [(lambda r, n=col.name: r[n], False)])
        new = out
    return new, None


def _flatten(vals, sum_cols):
    base = dict(vals[0])
    for v in vals[1:]:
        for name, kind in sum_cols.items():
            cls, w = KIND_CLASS[kind]
            if cls == "float":
                # field.SetFloat(field.Float() + cur.Float()): a float32 field rounds every add
                s = float(base[name]) + float(v[name])
                base[name] = float(np.float32(s)) if w == 4 else s
            else:
                s = int(base[name]) + int(v[name])
                s &= (1 << (8 * w)) - 1
                if cls == "int" and s >= 1 << (8 * w - 1):
                    s -= 1 << (8 * w)
                base[name] = s
    return base


# ------------------------------------------------------------------------------------------
# advise network-policy (pkg/gadgets/advise/networkpolicy/advisor/advisor.go) -- a direct
# restatement over parsed JSON events, event by event, with Python dicts in place of Go maps.
# ------------------------------------------------------------------------------------------
ADVISOR_IGNORE = {"controller-revision-hash", "pod-template-generation", "pod-template-hash"}


def _adv_keys(labels):                                   # labelFilteredKeyList :104-116
    return sorted(k for k in (labels or {}) if k not in ADVISOR_IGNORE)


def _adv_filter(labels):                                 # labelFilter :118-127
    return {k: v for k, v in (labels or {}).items() if k not in ADVISOR_IGNORE}


def _adv_keystr(labels):                                 # labelKeyString :132-141
    return ",".join("%s=%s" % (k, labels[k]) for k in _adv_keys(labels))


def _adv_peer_key(e):                                    # networkPeerKey :150-160
    k = e.get("remoteKind", "")
    if k in ("pod", "svc"):
        r = k + ":" + e.get("remoteNamespace", "") + ":" + _adv_keystr(e.get("remoteLabels"))
    elif k == "other":
        r = k + ":" + e.get("remoteAddr", "")
    else:
        r = ""
    return "%s:%d" % (r, int(e.get("port", 0)))


def _adv_rule(e):                                        # eventToRule :162-216
    ports = [{"port": int(e.get("port", 0)), "protocol": e.get("proto", "").upper()}]
    k = e.get("remoteKind", "")
    if k in ("pod", "svc"):
        lab = _adv_filter(e.get("remoteLabels")) if k == "pod" else dict(e.get("remoteLabels") or {})
        peer = {"podSelector": ({"matchLabels": lab} if lab else {})}
        if e.get("namespace", "") != e.get("remoteNamespace", ""):
            peer["namespaceSelector"] = {"matchLabels": {"kubernetes.io/metadata.name":
                                                         e.get("remoteNamespace", "")}}
        return ports, [peer]
    if k == "other":
        a = e.get("remoteAddr", "")
        return ports, ([] if a == "127.0.0.1" else [{"ipBlock": {"cidr": a + "/32"}}])
    raise ValueError("unknown event")


def _yaml_scalar(v):
    import re as _re
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    s = str(v)
    if s == "":
        return '""'
    if _re.fullmatch(r"[-+]?\d+(\.\d*)?([eE][-+]?\d+)?|true|false|null|~|yes|no|on|off|y|n", s, _re.I):
        return '"%s"' % s
    if _re.fullmatch(r"[A-Za-z0-9_./][A-Za-z0-9_./ -]*", s) and not s.endswith(" "):
        return s
    return "'" + s.replace("'", "''") + "'"


def yaml_text(v, ind=0):
    """go-yaml v2 block style as sigs.k8s.io/yaml emits it: sorted keys, sequences at
    their key's indentation, {} / [] for empty collections."""
    lines = []
    p = " " * ind

    def leaf(x):
        return "{}" if isinstance(x, dict) else ("[]" if isinstance(x, list) else _yaml_scalar(x))
    if isinstance(v, dict):
        for k in sorted(v):
            x = v[k]
            if isinstance(x, dict) and x:
                lines.append("%s%s:" % (p, k))
                lines.append(yaml_text(x, ind + 2).rstrip("\n"))
            elif isinstance(x, list) and x:
                lines.append("%s%s:" % (p, k))
                lines.append(yaml_text(x, ind).rstrip("\n"))
            else:
                lines.append("%s%s: %s" % (p, k, leaf(x)))
    else:
        for x in v:
            if isinstance(x, (dict, list)) and x:
                body = yaml_text(x, ind + 2).rstrip("\n")
                lines.append(p + "- " + body[ind + 2:])
            else:
                lines.append("%s- %s" % (p, leaf(x)))
    return "\n".join(lines) + "\n"


def advisor_policies(events):
    """GeneratePolicies (:277-372).  Sources are visited in first-occurrence order and the
    final name sort is stable (Go's map order + sort.Slice leave equal names unordered)."""
    by_src = {}
    for e in events:                                     # :279-300
        if e.get("type") != "normal":
            continue
        pk = e.get("pktType", "")
        if pk not in ("HOST", "OUTGOING"):
            continue
        if pk == "HOST" and e.get("podHostIP", "") == e.get("remoteAddr", ""):
            continue
        key = e.get("namespace", "") + ":" + _adv_keystr(e.get("podLabels"))
        by_src.setdefault(key, []).append(e)
    out = []
    for evs in by_src.values():
        egress, ingress = {}, {}
        for e in evs:                                    # :302-320 first event wins
            k = _adv_peer_key(e)
            d = egress if e.get("pktType") == "OUTGOING" else ingress
            if k not in d:
                d[k] = e
        def rules(d, field):
            r = []
            for e in d.values():
                ports, peers = _adv_rule(e)
                if peers:
                    r.append({"ports": ports, field: peers})
            return sorted(r, key=lambda x: (x["ports"][0]["protocol"], x["ports"][0]["port"], yaml_text(x)))
        e0 = evs[0]
        name = (e0.get("podOwner") or e0.get("pod", "")) + "-network"
        lab = _adv_filter(e0.get("podLabels"))
        spec = {"podSelector": ({"matchLabels": lab} if lab else {}), "policyTypes": ["Ingress", "Egress"]}
        ing, egr = rules(ingress, "from"), rules(egress, "to")
        if ing:
            spec["ingress"] = ing
        if egr:
            spec["egress"] = egr
        out.append({"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
                    "metadata": {"creationTimestamp": None, "name": name,
                                 "namespace": e0.get("namespace", "")},
                    "spec": spec, "status": {}})
    out.sort(key=lambda p: p["metadata"]["name"])
    return out


# ------------------------------------------------------------------------------------
# multi-GPU exchange reference (dist.py / k_partition.hip)
# ------------------------------------------------------------------------------------
def key_owner(keys, ws):
    """Owner rank of each packed key row ((n, kb) uint8, kb % 4 == 0): FNV-1a(32) over the
    key's little-endian u32 words, mod ws -- igx_partition_rows' function."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, kb = keys.shape
    w = keys.view(np.uint32).reshape(n, kb // 4).astype(np.uint64)
    h = np.full(n, 0x811C9DC5, dtype=np.uint64)
    for j in range(kb // 4):
        h = ((h ^ w[:, j]) * np.uint64(16777619)) & np.uint64(0xFFFFFFFF)
    return (h % np.uint64(ws)).astype(np.int64)


def partition_rows(rows, key_bytes, ws):
    """Stable grouping of rows by key_owner; returns (rows, counts)."""
    owner = key_owner(np.ascontiguousarray(rows[:, :key_bytes]), ws)
    order = np.argsort(owner, kind="stable")
    return np.ascontiguousarray(rows[order]), np.bincount(owner, minlength=ws).tolist()


# ------------------------------------------------------------------------------------
# all-cores CPU baselines (igx_oracle.c §7): same results as the single-thread paths
# ------------------------------------------------------------------------------------
def cpu_threads():
    """Host threads a baseline may use: the process's CPU affinity, capped by
    OMP_NUM_THREADS when set (the GPU box's per-GPU CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def top_tcp_mt(ev, k=20, base_idx=0, threads=None, checksum=False):
    """or_top_tcp on `threads` threads (hash-partitioned by key).  Returns (G, sent, recv,
    first) of the first k sorted rows, plus the full-table checksum (tcp_group_checksum
    summed over every group) when `checksum`."""
    T = threads or cpu_threads()
    n = len(ev["pid"])
    sent, recv, first = (np.empty(k, np.uint64) for _ in range(3))
    cs = np.zeros(1, np.uint64)
    cols = [np.ascontiguousarray(ev[c]) for c in ("saddr", "daddr", "mntns", "pid", "comm",
                                                  "lport", "dport", "family", "size", "dir")]
    G = lib().or_top_tcp_mt(*[_p(c) for c in cols], n, base_idx, T, k, _p(sent), _p(recv), _p(first),
                            _p(cs) if checksum else None)
    m = min(k, G)
    out = (G, sent[:m], recv[:m], first[:m])
    return out + (int(cs[0]),) if checksum else out


def tcp_group_checksum(fields66, sent, recv, first):
    """numpy twin of igx_oracle.c group_csum summed over groups: fields66 (G, 66) uint8 are
    the key fields in ip_key_t order without padding."""
    with np.errstate(over="ignore"):
        h = np.full(len(sent), 14695981039346656037, np.uint64)
        for i in range(66):
            h ^= fields66[:, i].astype(np.uint64)
            h *= np.uint64(1099511628211)
        z = h ^ (sent * np.uint64(0x9E3779B97F4A7C15)) ^ (recv * np.uint64(0xC2B2AE3D27D4EB4F)) ^ \
            (first * np.uint64(0x165667B19E3779F9))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        z = z ^ (z >> np.uint64(31))
        return int(z.sum(dtype=np.uint64))


def groupby_topk_mt(keys_packed, aggs, valid=None, base_idx=0, sort=(), k=0, threads=None, checksum=False):
    """or_groupby_topk_mt: keyed aggregation (aggs as for groupby) + the first k groups
    sorted by [(agg index, desc)] on `threads` threads.  Returns (G, first (k,), aggs (k, naggs)),
    plus the whole-table checksum (group_checksum over every group) when `checksum`."""
    T = threads or cpu_threads()
    keys_packed = np.ascontiguousarray(keys_packed, dtype=np.uint8)
    n, kb = keys_packed.shape
    cag, hold = [], []
    for a in aggs:
        val, cond = a.get("val"), a.get("cond")
        if val is not None:
            val = np.ascontiguousarray(val)
            hold.append(val)
        if cond is not None:
            cond = np.ascontiguousarray(cond)
            hold.append(cond)
        cag.append(_CAgg(0 if a["kind"] == "count" else 1, 0 if val is None else val.dtype.itemsize,
                         0 if val is None else val.ctypes.data, 0 if cond is None else cond.dtype.itemsize,
                         0 if cond is None else cond.ctypes.data, int(a.get("cond_val", 0)),
                         int(a.get("out_width", 8)), int(val is not None and val.dtype.kind == "i"),
                         int(a.get("div", 0))))
    arr = (_CAgg * max(1, len(cag)))(*cag)
    sa = np.array([x for x, _ in sort] or [0], np.uint32)
    sd = np.array([int(d) for _, d in sort] or [0], np.uint32)
    first = np.zeros(max(1, k), np.uint64)
    out = np.zeros((max(1, k), max(1, len(aggs))), np.uint64)
    v8 = None if valid is None else np.ascontiguousarray(valid.astype(np.uint8))
    cs = np.zeros(1, np.uint64)
    G = lib().or_groupby_topk_mt(_p(keys_packed), kb, n, _p(v8), C.cast(arr, C.c_void_p), len(cag), base_idx,
                                 T, _p(sa), _p(sd), len(sort), k, _p(first), _p(out), _p(cs) if checksum else None)
    if G == (1 << 64) - 1:
        raise MemoryError("or_groupby_topk_mt")
    m = min(k, G)
    res = (G, first[:m], out[:m, :len(aggs)])
    return res + (int(cs[0]),) if checksum else res


def group_checksum(keys, aggs, first):
    """numpy twin of igx_oracle.c group_csum_generic summed over groups: keys (G, kb) uint8
    in the packed layout (pad_keys), aggs a list of (G,) uint64 columns, first (G,) uint64."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    mix = lambda z: _mix64(z)   # noqa: E731
    with np.errstate(over="ignore"):
        h = np.full(keys.shape[0], 14695981039346656037, np.uint64)
        for i in range(keys.shape[1]):
            h ^= keys[:, i].astype(np.uint64)
            h *= np.uint64(1099511628211)
        z = h ^ (np.asarray(first, np.uint64) * np.uint64(0x165667B19E3779F9))
        for a in aggs:
            z = mix(z ^ (np.asarray(a, np.uint64) * np.uint64(0x9E3779B97F4A7C15)))
        return int(mix(z).sum(dtype=np.uint64))


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))


def hist_log2_mt(dev, cont, delta, devs, ncont, divisor=1000, nslots=27, threads=None):
    T = threads or cpu_threads()
    devs = np.ascontiguousarray(devs, dtype=np.uint32)
    hist = np.zeros((max(1, len(devs)) * ncont, nslots), dtype=np.uint32)
    delta = np.ascontiguousarray(delta).view(np.int64)
    dev = np.ascontiguousarray(np.zeros(len(delta), np.uint32) if dev is None else dev, dtype=np.uint32)
    cont = np.ascontiguousarray(np.zeros(len(delta), np.uint32) if cont is None else cont, dtype=np.uint32)
    lib().or_hist_log2_mt(_p(dev), _p(cont), _p(delta), len(dev), _p(devs), len(devs), ncont, divisor, nslots,
                          _p(hist), T)
    return hist
