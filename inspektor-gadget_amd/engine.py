"""Thin tensor-level wrappers over the igx C ABI (device tensors in, device tensors out).

The reference-shaped API (columns / filter / sort / group / top / gadgets) is built on
these.  Everything here enqueues libigx.so kernels on torch's current stream.
"""
import ctypes as C
import os
import math

from . import _abi
from ._abi import Agg, Col, Pred, SortKey, TableView, IgxError
from .runtime import context, ptr, col_of, dtype_kind, torch_mod

# ------------------------------------------------------------------------------------
# synthetic streams; bit-identical with the CPU oracle
# ------------------------------------------------------------------------------------
TCP_FIELDS = (("saddr", "u8x16"), ("daddr", "u8x16"), ("mntns", "u64"), ("pid", "u32"),
              ("comm", "u8x16"), ("lport", "u16"), ("dport", "u16"), ("family", "u16"),
              ("size", "u32"), ("dir", "u8"))
OPEN_FIELDS = (("pid", "u32"), ("uid", "u32"), ("mntns", "u64"), ("comm", "u8x16"),
               ("ret", "i64"), ("fd", "i64"), ("err", "i64"), ("path", "u32"))
BIO_FIELDS = (("dev", "u32"), ("cont", "u32"), ("delta", "i64"))
NP_FIELDS = (("src", "u32"), ("peer", "u32"), ("port", "u16"), ("pkt", "u8"), ("type", "u8"),
             ("proto", "u8"), ("hostip", "u32"), ("raddr", "u32"))
FILE_FIELDS = (("inode", "u64"), ("dev", "u32"), ("pid", "u32"), ("tid", "u32"), ("op", "u8"),
               ("count", "u32"))


def zipf_cdf(G: int, s: float):
    """Host table for the generators: u63 fixed-point CDF thresholds of Zipf(s) over ranks
    1..G (last == 1 << 63); k_gen.hip draws a rank by binary search of a u63 uniform."""
    import numpy as np
    k = np.arange(1, G + 1, dtype=np.float64)
    c = np.cumsum(k ** (-s))
    c /= c[-1]
    out = np.minimum(np.floor(c * float(1 << 63)), float(1 << 63)).astype(np.uint64)
    out[-1] = np.uint64(1 << 63)
    return out


def lognormal_quantiles(mu: float, sigma: float, nq: int = 4096, cap: int = 1 << 40):
    """Host table for igx_gen_bio: nq+1 monotone quantile boundaries (u64 ns) of
    lognormal(mu, sigma), capped (SURVEY.md §8(d) C3 latencies)."""
    import numpy as np
    from scipy.stats import norm
    p = (np.arange(nq + 1, dtype=np.float64) + 0.5) / (nq + 1)
    q = np.minimum(np.exp(mu + sigma * norm.ppf(p)), float(cap))
    return np.maximum.accumulate(np.floor(q)).astype(np.uint64)


def _alloc(fields, n, device):
    torch = torch_mod()
    dt = {"u8": torch.uint8, "u16": torch.uint16, "u32": torch.uint32, "u64": torch.uint64,
          "i64": torch.int64}
    out = {}
    for name, f in fields:
        if f == "u8x16":
            out[name] = torch.empty((n, 16), dtype=torch.uint8, device=device)
        else:
            out[name] = torch.empty(n, dtype=dt[f], device=device)
    return out


def perm_params(G):
    A = 999983
    while math.gcd(A, G) != 1:
        A += 2
    return (A % G, 12345 % G) if G > 1 else (1, 0)


def gen_tcp(seed, rank, G, cdf, base, n, out=None):
    ctx = context()
    ev = out or _alloc(TCP_FIELDS, n, cdf.device)
    A, B = perm_params(G)
    ctx.check(ctx.L.igx_gen_tcp(ctx.h, seed, rank, G, A, B, ptr(cdf), base, n,
                                *[ptr(ev[k]) for k, _ in TCP_FIELDS]))
    return ev


def gen_open(seed, comm_cdf, base, n):
    ctx = context()
    ev = _alloc(OPEN_FIELDS, n, comm_cdf.device)
    ctx.check(ctx.L.igx_gen_open(ctx.h, seed, ptr(comm_cdf), base, n,
                                 *[ptr(ev[k]) for k, _ in OPEN_FIELDS]))
    return ev


def gen_bio(seed, q, base, n):
    ctx = context()
    ev = _alloc(BIO_FIELDS, n, q.device)
    ctx.check(ctx.L.igx_gen_bio(ctx.h, seed, ptr(q), q.numel() - 1, base, n,
                                *[ptr(ev[k]) for k, _ in BIO_FIELDS]))
    return ev


def gen_np(seed, nsrc, npeer, base, n, device="cuda"):
    ctx = context()
    ev = _alloc(NP_FIELDS, n, device)
    ctx.check(ctx.L.igx_gen_np(ctx.h, seed, nsrc, npeer, base, n,
                               *[ptr(ev[k]) for k, _ in NP_FIELDS]))
    return ev


def gen_file(seed, rank, G, cdf, base, n):
    ctx = context()
    ev = _alloc(FILE_FIELDS, n, cdf.device)
    A, B = perm_params(G)
    ctx.check(ctx.L.igx_gen_file(ctx.h, seed, rank, G, A, B, ptr(cdf), base, n,
                                 *[ptr(ev[k]) for k, _ in FILE_FIELDS]))
    return ev


# ------------------------------------------------------------------------------------
# filter
# ------------------------------------------------------------------------------------
def filter_rows(cols, preds, n, valid=None, any=False, nil_match=False, device_count=False):
    """cols: list of device tensors (indexed by Pred.col); preds: list of Pred.
    any=False: AND (MatchAll); any=True: OR (MatchAny); any number of preds.
    nil_match=False: nil rows (valid == 0) are skipped (FilterEntries, filter.go:310-314);
    True: a nil row evaluates Match(nil) == negate per pred (filter.go:286-291).
    Returns (idx u32 tensor of length n_selected); with device_count=True, (idx of capacity n,
    count u64 device tensor) and no host synchronisation."""
    torch = torch_mod()
    ctx = context()
    dev = cols[0].device if cols else (valid.device if valid is not None else "cuda")
    ccols = (Col * max(1, len(cols)))(*[col_of(t, dtype_kind(t)) for t in cols])
    cpreds = (Pred * max(1, len(preds)))(*preds)
    out = torch.empty(max(1, n), dtype=torch.uint32, device=dev)
    cnt = torch.zeros(1, dtype=torch.uint64, device=dev)
    flags = (_abi.FILTER_ANY if any else 0) | (_abi.FILTER_NIL_MATCH if nil_match else 0)
    ctx.check(ctx.L.igx_filter_ex(ctx.h, ccols, len(cols), cpreds, len(preds), ptr(valid), n, flags,
                                  ptr(out), ptr(cnt)))
    if device_count:
        return out, cnt
    k = int(cnt.item())
    return out[:k]


def take(tensors, idx, nrows=None, pad=False):
    """igx_take: rows idx (device u32/int32/int64) of every tensor ((n,) or (n, W)) gathered
    on the device into fresh tensors of the same dtypes -- the compacted batch FilterEntries
    returns (filter.go:294-325).  Ids >= nrows yield zero rows; pad=True marks the callers
    that rely on it (the padded top-K merge), and IGX_DEBUG_TAKE=1 makes every other call
    raise IndexError on such an id."""
    torch = torch_mod()
    ctx = context()
    if idx.dtype not in (torch.int32, torch.uint32):
        idx = idx.to(torch.int32)
    idx = idx.contiguous()
    k = int(idx.numel())
    tensors = [t.contiguous() for t in tensors]
    outs = [torch.empty((k,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) for t in tensors]
    if k and tensors:
        n = int(tensors[0].shape[0]) if nrows is None else nrows
        if not pad and os.environ.get("IGX_DEBUG_TAKE"):
            # debug assert (one host sync): igx_take zero-fills ids >= nrows, which only the
            # padded top-K merge relies on; the torch index_select it replaced raised here
            hi = int(idx.to(torch.int64).max())
            if hi >= n or int(idx.to(torch.int64).min()) < 0:
                raise IndexError(f"take: row id {hi} out of range for {n} rows")
        ccols = (Col * len(tensors))(*[col_of(t, dtype_kind(t), t[0].numel() * t.element_size() if t.dim() > 1 else None)
                                         for t in tensors])
        dst = (C.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
        ctx.check(ctx.L.igx_take(ctx.h, ccols, len(tensors), n, ptr(idx), k, dst))
    return outs


# ------------------------------------------------------------------------------------
# sort
# ------------------------------------------------------------------------------------
def sort_perm(keys, n, pos=None, valid=None, k=None, rowmap=None, d_count=None):
    """keys: list of (tensor, desc) in sortBy order.  Returns u32 permutation (first k).
    rowmap (u32, n rows): sort the selection vector -- row i is row rowmap[i] of the key
    columns, valid and pos (igx_sort_perm_ex); the result is then rowmap values in order.
    d_count (u64 device tensor, with rowmap): the slice is rowmap[:d_count], n its upper bound
    (igx_sort_perm_dn: no host round trip); the result has capacity n, its first d_count
    entries sorted."""
    torch = torch_mod()
    ctx = context()
    dev = keys[0][0].device if keys else (pos.device if pos is not None else "cuda")
    sk = []
    for key in keys:
        t, desc = key[0], key[1]
        kind = key[2] if len(key) > 2 else dtype_kind(t)
        width = t.shape[1] if t.dim() == 2 else t.element_size()
        sk.append(SortKey(C.c_void_p(t.data_ptr()), width, kind, 1 if desc else 0, 0))
    arr = (SortKey * max(1, len(sk)))(*sk)
    m = n if k is None else min(k, n)
    out = torch.empty(max(1, m), dtype=torch.uint32, device=dev)
    if n == 0:
        return out[:0]
    if rowmap is not None:
        if k is not None:
            raise ValueError("a top-K over a selection vector: sort the view first")
        if d_count is not None:
            ctx.check(ctx.L.igx_sort_perm_dn(ctx.h, arr, len(sk), n, ptr(d_count), ptr(pos), ptr(valid),
                                             ptr(rowmap), ptr(out)))
        else:
            ctx.check(ctx.L.igx_sort_perm_ex(ctx.h, arr, len(sk), n, ptr(pos), ptr(valid), ptr(rowmap), ptr(out)))
    elif k is None:
        ctx.check(ctx.L.igx_sort_perm(ctx.h, arr, len(sk), n, ptr(pos), ptr(valid), ptr(out)))
    else:
        if valid is not None:
            raise ValueError("topk does not take a nil mask")
        ctx.check(ctx.L.igx_topk(ctx.h, arr, len(sk), n, ptr(pos), m, ptr(out)))
    return out[:m]


sort_perm_kinds = sort_perm


# ------------------------------------------------------------------------------------
# group-by table
# ------------------------------------------------------------------------------------
class Table:
    """igx_table: keyed aggregation with first-occurrence tracking."""

    def __init__(self, key_widths, aggs, capacity, ctx=None):
        self.ctx = context() if ctx is None else ctx
        kw = (C.c_uint32 * len(key_widths))(*key_widths)
        ca = (Agg * max(1, len(aggs)))(*aggs)
        h = C.c_void_p()
        self.ctx.check(self.ctx.L.igx_groupby_create(self.ctx.h, kw, len(key_widths), ca,
                                                     len(aggs), capacity, C.byref(h)))
        self.h = h
        self.key_widths = list(key_widths)
        self.naggs = len(aggs)
        self.out_widths = [int(a.out_width) or 8 for a in aggs]
        self.capacity = capacity

    def update(self, cols, key_cols, n, base_idx=0, preds=(), valid=None, idx_col=None):
        """igx_groupby_update_ex: rows [0,n) of cols; valid (u8) masks rows out; idx_col is
        the index of a u64 column of global event indices (merging partial groups)."""
        ctx = self.ctx
        ctx.bind_stream()
        ccols = (Col * len(cols))(*[col_of(t, dtype_kind(t)) for t in cols])
        kc = (C.c_uint32 * len(key_cols))(*key_cols)
        cp = (Pred * max(1, len(preds)))(*preds)
        ctx.check(ctx.L.igx_groupby_update_ex(self.h, ccols, len(cols), kc, cp, len(preds),
                                              ptr(valid), _abi.NO_COL if idx_col is None else idx_col,
                                              n, base_idx))

    def wait(self):
        """igx_groupby_wait: the group count of the last finalize(sync=False), with its status
        (IGX_ENOSPC raises as finalize would have)."""
        n = C.c_uint64()
        self.ctx.check(self.ctx.L.igx_groupby_wait(self.h, C.byref(n)))
        if getattr(self, "fin", None) is not None:
            self.fin["n_groups"] = n.value
        return n.value

    def info(self):
        """igx_groupby_info: the current interval's form and AUTO's plan, as a dict."""
        from ._abi import GroupbyInfo
        v = GroupbyInfo()
        self.ctx.check(self.ctx.L.igx_groupby_info(self.h, C.byref(v)))
        return {f: getattr(v, f) for f, _ in GroupbyInfo._fields_ if f != "pad"}

    def reset(self):
        self.ctx.check(self.ctx.L.igx_groupby_reset(self.h))

    def set_mode(self, mode):
        """igx_groupby_set_mode: _abi.GB_AUTO (default), GB_CACHED, GB_DIRECT or GB_PART."""
        self.ctx.check(self.ctx.L.igx_groupby_set_mode(self.h, mode))

    def finalize(self, sync=True):
        """Returns the table view (raw device pointers, slot-indexed) as a dict; `groups_ptr`
        lists the n_groups occupied slots.  sync=True synchronises (igx_groupby_finalize);
        sync=False leaves the group count on the device (igx_groupby_finalize_async:
        n_groups is None until wait(), and a top-K sort reads the count on the device)."""
        v = TableView()
        if sync:
            self.ctx.check(self.ctx.L.igx_groupby_finalize(self.h, C.byref(v)))
        else:
            self.ctx.check(self.ctx.L.igx_groupby_finalize_async(self.h, C.byref(v)))
        self._view = v
        self.fin = {"n_groups": v.n_groups if sync else None, "n_slots": v.n_slots, "key_bytes": v.key_bytes,
                    "key_stride": v.key_stride, "val_stride": v.val_stride, "keys_ptr": v.keys,
                    "aggs_ptr": [v.aggs[i] for i in range(v.naggs)], "first_ptr": v.first_idx,
                    "groups_ptr": v.groups, "d_n_groups": v.d_n_groups}
        return self.fin

    def sort(self, keys, k=0):
        """igx_groupby_sort: keys = [(src, index_or_(offset,width,kind), desc)].  Returns the
        first k (0 = all) group slots in SortStats order (device u32)."""
        torch = torch_mod()
        ts = []
        for src, what, desc in keys:
            if src == _abi.TSRC_KEY:
                off, w, kind = what
                ts.append(_abi.TSortKey(src, 0, off, w, kind, int(desc)))
            elif src == _abi.TSRC_IPTEXT:
                addr_off, fam_off = what
                ts.append(_abi.TSortKey(src, fam_off, addr_off, 16, _abi.KIND_BYTES, int(desc)))
            else:
                ts.append(_abi.TSortKey(src, int(what or 0), 0, 0, 0, int(desc)))
        arr = (_abi.TSortKey * max(1, len(ts)))(*ts)
        G = self.fin["n_groups"]
        if G is None:   # finalize(sync=False): a top-K over integer keys reads the count on the device
            dev_ok = 0 < k <= 4096 and 2 * k < self.capacity and all(t.src != _abi.TSRC_IPTEXT and not (t.src == _abi.TSRC_KEY and
                                                                             t.kind == _abi.KIND_FLOAT) for t in ts)
            if not dev_ok:
                G = self.wait()
        # without the count, k slots come back; those past the group count are 0xFFFFFFFF
        # (gather() turns them into zero rows)
        m = k if G is None else (G if k == 0 else min(k, G))
        out = torch.empty(max(1, m), dtype=torch.int32, device=torch.device("cuda", torch.cuda.current_device()))
        if m:
            self.ctx.check(self.ctx.L.igx_groupby_sort(self.h, arr, len(ts), m, ptr(out)))
        return out[:m]

    def topk_counts(self):
        """igx_groupby_topk_counts (synchronous): (top-Ks answered by the hinted path, by the full
        selection) so far."""
        out = (C.c_uint64 * 2)()
        self.ctx.check(self.ctx.L.igx_groupby_topk_counts(self.h, out))
        return int(out[0]), int(out[1])

    def gather(self, slots):
        """Packed rows (len(slots), key_bytes + 8*naggs + 8) for the given slots."""
        torch = torch_mod()
        row = self.fin["key_bytes"] + 8 * self.naggs + 8
        k = slots.numel()
        out = torch.empty((max(1, k), row), dtype=torch.uint8, device=slots.device)
        if k:
            self.ctx.check(self.ctx.L.igx_groupby_gather(self.h, ptr(slots), k, ptr(out)))
        return out[:k]

    def partition(self, nparts, out_widths=None):
        """igx_partition_groups: the finalized table's groups as packed rows (key | aggregates
        wrapped to out_widths | first index), grouped by owner part (FNV-1a over the key words
        mod nparts, as igx_partition_rows), stable in slot order within a part -- the sender
        side of the owner exchange, with the group count read on the device (works after
        finalize(sync=False)).  Returns (rows (capacity, row_bytes) u8, counts (nparts,) i64),
        both on the device; rows past the counts' sum are unused."""
        torch = torch_mod()
        ctx = self.ctx
        ctx.bind_stream()
        fin = self.fin
        rb = fin["key_bytes"] + 8 * self.naggs + 8
        dev = torch.device("cuda", torch.cuda.current_device())
        buf = getattr(self, "_part_buf", None)
        if buf is None or buf.shape != (self.capacity, rb):
            buf = self._part_buf = torch.empty((max(1, self.capacity), rb), dtype=torch.uint8, device=dev)
        cnt = torch.empty(nparts, dtype=torch.int64, device=dev)
        ow = (C.c_uint32 * max(1, self.naggs))(*(out_widths or self.out_widths))
        ctx.check(ctx.L.igx_partition_groups(ctx.h, C.byref(self._view), ow, nparts, ptr(buf), self.capacity,
                                             ptr(cnt)))
        return buf, cnt

    def destroy(self):
        if self.h:
            self.ctx.L.igx_groupby_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def table_tensors(tab, fin):
    """Dense copies of the finalized groups (occupied-slot order) as torch tensors:
    keys (G, key_bytes) u8, aggs [ (G,) u64 ], first (G,) u64."""
    torch = torch_mod()
    ctx = tab.ctx
    dev = torch.device("cuda", torch.cuda.current_device())
    G = fin["n_groups"]
    slots = torch.empty(max(1, G), dtype=torch.int32, device=dev)[:G]
    if G:
        ctx.check(ctx.L.igx_memcpy_d2d(ctx.h, ptr(slots), C.c_void_p(fin["groups_ptr"]), G * 4))
    rows = tab.gather(slots)
    kb = fin["key_bytes"]
    keys = rows[:, :kb].contiguous()
    # flat copies: a one-row slice counts as contiguous and keeps its byte offset and row
    # stride, which a u64 view rejects
    aggs = [rows[:, kb + 8 * i: kb + 8 * i + 8].reshape(-1).clone().view(torch.uint64)
            for i in range(tab.naggs)]
    first = rows[:, kb + 8 * tab.naggs:].reshape(-1).clone().view(torch.uint64)
    return keys, aggs, first


# ------------------------------------------------------------------------------------
# advise network-policy
# ------------------------------------------------------------------------------------
def np_mark(typ, pkt, hostip, raddr):
    """igx_np_mark: u8 keep mask of the advisor's event filter (advisor.go:279-292)."""
    torch = torch_mod()
    ctx = context()
    n = typ.numel()
    keep = torch.empty(max(4, (n + 3) // 4 * 4), dtype=torch.uint8, device=typ.device)
    ctx.check(ctx.L.igx_np_mark(ctx.h, ptr(typ), ptr(pkt), ptr(hostip), ptr(raddr), n, ptr(keep)))
    return keep[:n]


# ------------------------------------------------------------------------------------
# log2 histograms
# ------------------------------------------------------------------------------------
def hist_log2(dev, cont, delta, devs, ncont, divisor=1000, nslots=27, hist=None):
    torch = torch_mod()
    ctx = context()
    n = delta.numel()
    if hist is None:
        hist = torch.zeros((max(1, len(devs)) * ncont, nslots), dtype=torch.uint32, device=delta.device)
    hd = (C.c_uint32 * max(1, len(devs)))(*devs)
    ctx.check(ctx.L.igx_hist_log2(ctx.h, ptr(dev), ptr(cont), ptr(delta), n, hd, len(devs),
                                  ncont, divisor, nslots, ptr(hist)))
    return hist


def hist_log2_keyed(delta, cmd_flags=None, dev=None, divisor=1000, nslots=27, capacity=1 << 16):
    """biolatency with targ_per_flag / targ_per_disk (biolatency.bpf.c:116-150): one log2
    histogram per distinct raw hist_key{cmd_flags, dev}, any values (a column left None is the
    key field the BPF program leaves 0).  igx_log2_slots gives each event its slot, then a
    group-by on (cmd_flags, dev, slot) counts them (u32 slots, wrapping like the BPF map's).
    Returns [(cmd_flags, dev, u32 slots (nslots,))] in the order of each key's first event (the
    BPF map's own order is its hash order)."""
    import numpy as np
    from .columns import host
    torch = torch_mod()
    ctx = context()
    n = delta.numel()
    slot = torch.empty(max(4, (n + 3) // 4 * 4), dtype=torch.uint8, device=delta.device)[:n]
    keep = torch.empty(max(4, (n + 3) // 4 * 4), dtype=torch.uint8, device=delta.device)[:n]
    if n:
        ctx.check(ctx.L.igx_log2_slots(ctx.h, ptr(delta), n, divisor, nslots, ptr(slot), ptr(keep)))
    cols, widths = [], []
    for c in (cmd_flags, dev):
        if c is not None:
            cols.append(c)
            widths.append(4)
    cols.append(slot)
    widths.append(1)
    tab = Table(widths, [Agg(_abi.AGG_COUNT, 0, _abi.NO_COL, 4, 0)], capacity)
    try:
        if n:
            tab.update(cols, list(range(len(cols))), n, valid=keep)
        fin = tab.finalize()
        keys, aggs, first = table_tensors(tab, fin)
    finally:
        tab.destroy()
    k, cnt, f = host(keys), host(aggs[0]), host(first)
    nk = len(widths) - 1
    w = k[:, :4 * nk].copy().view(np.uint32).reshape(len(k), nk) if nk else np.zeros((len(k), 0), np.uint32)
    sl = k[:, 4 * nk]
    out = {}
    for i in range(len(k)):
        vals = [int(x) for x in w[i]]
        cf = vals.pop(0) if cmd_flags is not None else 0
        dv = vals.pop(0) if dev is not None else 0
        e = out.setdefault((cf, dv), [np.zeros(nslots, np.uint32), int(f[i])])
        e[0][sl[i]] = np.uint32(int(cnt[i]) & 0xFFFFFFFF)
        e[1] = min(e[1], int(f[i]))
    return [(cf, dv, h) for (cf, dv), (h, _) in sorted(out.items(), key=lambda kv: kv[1][1])]


# ------------------------------------------------------------------------------------
# data movement either side of the path
# ------------------------------------------------------------------------------------
def partition_rows(rows, key_bytes, nparts):
    """igx_partition_rows: (n, row_bytes) uint8 device rows grouped by owner part
    (FNV-1a over the key words mod nparts), stable within a part.  Returns (rows, counts)
    with counts a host list."""
    torch = torch_mod()
    ctx = context()
    n, rb = rows.shape
    rows = rows.contiguous()
    out = torch.empty_like(rows)
    cnt = torch.zeros(nparts, dtype=torch.int64, device=rows.device)
    ctx.check(ctx.L.igx_partition_rows(ctx.h, ptr(rows), n, rb, key_bytes, nparts, ptr(out), ptr(cnt)))
    return out, cnt.cpu().tolist()


def ip_text(addr, family, n=None, rowmap=None):
    """igx_ip_text: IPStringFromBytes (helpers.go:111-120) of n rows on the device.
    addr: uint8 (n, 16) or a byte view with a row stride; family: u16 column (or a byte view
    whose first two bytes per row are the family).  Returns uint8 (n, IPTEXT_WIDTH),
    zero-padded texts."""
    torch = torch_mod()
    ctx = context()
    n = addr.shape[0] if n is None else n
    astride = addr.stride(0) * addr.element_size()
    fstride = family.stride(0) * family.element_size()
    out = torch.empty((max(1, n), _abi.IPTEXT_WIDTH), dtype=torch.uint8, device=addr.device)
    if n:
        ctx.check(ctx.L.igx_ip_text(ctx.h, ptr(addr), astride, ptr(family), fstride,
                                    None if rowmap is None else ptr(rowmap), n, ptr(out)))
    return out[:n]


def ingest_open_events(samples, n=None, sample_bytes=_abi.OPEN_SAMPLE_BYTES, boot_to_wall_ns=0):
    """igx_ingest_open_events: trace open perf samples (device uint8, n x sample_bytes) ->
    the Event columns of trace/open/tracer/tracer.go:182-208 (timestamp, pid, uid, mntns, ret,
    fd, err as int64 / u32 / u64 tensors; comm (n, 16) and path (n, 256) uint8)."""
    torch = torch_mod()
    ctx = context()
    n = samples.numel() // sample_bytes if n is None else n
    dev = samples.device
    m = max(1, n)
    cols = {"timestamp": torch.empty(m, dtype=torch.int64, device=dev),
            "pid": torch.empty(m, dtype=torch.uint32, device=dev),
            "uid": torch.empty(m, dtype=torch.uint32, device=dev),
            "mntns": torch.empty(m, dtype=torch.uint64, device=dev),
            "ret": torch.empty(m, dtype=torch.int64, device=dev),
            "fd": torch.empty(m, dtype=torch.int64, device=dev),
            "err": torch.empty(m, dtype=torch.int64, device=dev),
            "comm": torch.empty((m, 16), dtype=torch.uint8, device=dev),
            "path": torch.empty((m, 256), dtype=torch.uint8, device=dev)}
    oc = _abi.OpenCols(*[cols[f].data_ptr() for f, _ in _abi.OpenCols._fields_])
    ctx.check(ctx.L.igx_ingest_open_events(ctx.h, ptr(samples), n, sample_bytes, boot_to_wall_ns, C.byref(oc)))
    return {k: v[:n] for k, v in cols.items()}


def ingest_aos(records, n, rec_bytes, fields, device=None):
    """igx_ingest_aos: records (device uint8, n x rec_bytes) -> {name: SoA column}.
    fields: [(name, offset, width, dtype)] with dtype a torch dtype (width 1/2/4/8) or
    None for a byte column (n, width)."""
    torch = torch_mod()
    ctx = context()
    dev = records.device if device is None else device
    cols = {}
    for name, off, width, dt in fields:
        cols[name] = (torch.empty((n, width), dtype=torch.uint8, device=dev) if dt is None
                      else torch.empty(n, dtype=dt, device=dev))
    offs = (C.c_uint32 * len(fields))(*[f[1] for f in fields])
    wids = (C.c_uint32 * len(fields))(*[f[2] for f in fields])
    outs = (C.c_void_p * len(fields))(*[cols[f[0]].data_ptr() for f in fields])
    ctx.check(ctx.L.igx_ingest_aos(ctx.h, ptr(records), n, rec_bytes, offs, wids, len(fields), outs))
    return cols
