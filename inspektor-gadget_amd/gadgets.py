"""The aggregation gadgets as their tracers expose them: top tcp / file / block-io and
profile block-io, on top of libigx.so.

Each `Top*` class is the user-space half of a reference tracer plus the BPF map update it
drains, re-cut for batches of events resident in HBM:

  feed(events)   the BPF probe for every event of a batch: the probe's filters (fused
                 group-by predicates), the map key, lookup-or-insert and the `+=` updates
                 (igx_groupby_update_ex on the device)
  nextStats()    tracer.nextStats: one Stats row per map entry, top.SortStats(SortBy),
                 then the map is emptied for the next interval (the deferred Delete loop)
  NextEvent()    one tick of tracer.run: nextStats() truncated to MaxRows, wrapped in
                 top.Event (the eventCallback payload)

References (paths under the reference root):
  top tcp       pkg/gadgets/top/tcp/tracer/tracer.go:147-265, bpf/tcptop.bpf.c:33-110,
                types/types.go:27-101
  top file      pkg/gadgets/top/file/tracer/tracer.go:148-247, bpf/filetop.bpf.c:39-94,
                types/types.go:30-62
  top block-io  pkg/gadgets/top/block-io/tracer/tracer.go:211-310, bpf/biotop.bpf.c:85-130,
                types/types.go:31-65
  profile block-io  pkg/gadgets/profile/block-io/tracer/tracer.go:56-90 (getReport),
                tracer/gadget.go:85-143 (reportToString), bpf/biolatency.bpf.c:100-154

The reference's pre-sort order (BPF hash iteration) is replaced by each group's first
event index; everything else -- keys, wrap widths, sort order including
the DESC tie reversal, truncation -- is the reference's.  Sorting runs on the device over
the whole table; only the rows that are returned are copied to the host.
"""
from __future__ import annotations

import bisect
import ipaddress
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import _abi, engine
from .columns import Columns, host
from .runtime import torch_mod
from . import sort as _sort
from . import top as _top

AF_INET, AF_INET6 = 2, 10                 # syscall.AF_INET / AF_INET6
REQ_OP_WRITE = 1                          # biotop.bpf.c:106 (REQ_OP_MASK = 0xff)

# ------------------------------------------------------------------------------------
# pkg/gadgets/helpers.go
# ------------------------------------------------------------------------------------


def FromCString(b) -> str:
    """helpers.go:76-83: bytes up to the first NUL."""
    b = bytes(b)
    i = b.find(b"\0")
    return (b if i < 0 else b[:i]).decode("utf-8", "replace")


def IPStringFromBytes(b, ipType: int) -> str:
    """helpers.go:111-120: netip.AddrFrom4 / AddrFrom16 .String()."""
    b = bytes(b)
    if ipType == 4:
        return ".".join(str(x) for x in b[:4])
    if ipType == 6:
        if b[:10] == b"\0" * 10 and b[10:12] == b"\xff\xff":   # netip prints 4in6 dotted
            return "::ffff:" + ".".join(str(x) for x in b[12:16])
        return str(ipaddress.IPv6Address(b))
    return ""


# ------------------------------------------------------------------------------------
# table-backed top gadget
# ------------------------------------------------------------------------------------
@dataclass
class Event:
    """top.Event[T] (pkg/gadgets/top/top.go:30-34)."""
    Error: str = ""
    Stats: list = field(default_factory=list)


def _pred(col, cmp, ref_bytes, negate=0, guard=None):
    """igx_pred; guard = (column, value bytes): the test applies only where that column
    holds that value (a check one probe makes and another does not)."""
    p = _abi.Pred()
    p.col, p.cmp, p.negate, p.ref_len = col, cmp, negate, len(ref_bytes)
    for i, x in enumerate(ref_bytes):
        p.ref[i] = x
    if guard is not None:
        p.guard_col, gref = guard
        p.guard_len = len(gref)
        for i, x in enumerate(gref):
            p.guard_ref[i] = x
    return p


class _TopTracer:
    """Shared machinery.  Subclasses define:
      EVENT      [(name, kind, width)] event columns the probe reads (SoA, device)
      KEY        names of the map key's fields, in key-struct order
      AGGS       [(kind, value column | None, cond column | None, cond value, out width, divisor)]
      STATS_COLS Columns of the Stats struct (what sortBy names refer to)
      SORT_SRC   Stats column -> ("agg", i) | ("key", field) | ("const",)
      ALIASES    [(name, event column, torch dtype)]: the column's memory read as another type
                 (appended after EVENT, e.g. an argument the probe declares signed)
      SortByDefault
    and _preds() (the probe's filters) and _stats(rows) (Stats objects)."""

    EVENT: list = []
    KEY: list = []
    AGGS: list = []
    SORT_SRC: Dict[str, tuple] = {}
    SortByDefault: list = []
    ALIASES: list = []

    def __init__(self, MaxRows=_top.MaxRowsDefault, SortBy=None, capacity=1 << 20, Interval=1, ctx=None):
        self.MaxRows = MaxRows
        self.SortBy = list(self.SortByDefault if SortBy is None else SortBy)
        self.Interval = Interval
        self.ev_index = {name: i for i, (name, _, _) in enumerate(self.EVENT)}
        for j, (name, _, _) in enumerate(self.ALIASES):
            self.ev_index[name] = len(self.EVENT) + j
        self.ev_width = {name: w for name, _, w in self.EVENT}
        widths = [self.ev_width[k] for k in self.KEY]
        aggs = []
        for kind, vcol, ccol, cval, ow, div in self.AGGS:
            aggs.append(_abi.Agg(kind, 0 if vcol is None else self.ev_index[vcol],
                                 _abi.NO_COL if ccol is None else self.ev_index[ccol], ow, cval, div))
        self.table = engine.Table(widths, aggs, capacity, ctx=ctx)
        self.key_off = {}
        o = 0
        for k in self.KEY:
            self.key_off[k] = o
            o += (self.ev_width[k] + 3) // 4 * 4
        self.key_bytes = o
        self.batches = []          # (base_idx, n, events) fed this interval
        self.next_idx = 0

    # -- the probe --------------------------------------------------------------------
    def _preds(self):
        return []

    def feed(self, events: dict, n: Optional[int] = None, base_idx: Optional[int] = None):
        """Run the BPF probe over a batch: events maps EVENT names to device tensors."""
        torch = torch_mod()
        n = int(events[self.KEY[0]].shape[0]) if n is None else n
        base = self.next_idx if base_idx is None else base_idx
        cols = []
        for name, kind, w in self.EVENT:
            t = events.get(name)
            if t is None:
                # columns the probe does not need for this config (e.g. a condition column
                # that no aggregate uses) still need a readable pointer
                t = torch.zeros(max(1, n), dtype=torch.uint8, device=events[self.KEY[0]].device)
            cols.append(t)
        for _, src, dtype in self.ALIASES:
            cols.append(cols[self.ev_index[src]].view(getattr(torch, dtype)))
        self.table.update(cols, [self.ev_index[k] for k in self.KEY], n, base, self._preds())
        self.batches.append((base, n, events))
        self.next_idx = base + n

    # -- nextStats ----------------------------------------------------------------------
    def _sort_keys(self, sort_by):
        """top.SortStats(stats, sortBy, colMap) as table sort keys (sort.Prepare rules:
        unknown / virtual columns dropped; bool columns skipped at sort time)."""
        keys = []
        for sk in _sort._prepare_raw(self.STATS_COLS, sort_by):
            if sk.kind in (_abi.KIND_BOOL, _abi.KIND_OTHER):
                continue
            name = self.STATS_COLS.GetOrderedColumns()[sk.col].Name.lower()
            src = self.SORT_SRC.get(name)
            if src is None:
                raise _abi.IgxError(_abi.IGX_ENOTSUP, f"sorting by {name!r} needs the host")
            desc = bool(sk.desc)
            if src[0] == "agg":
                keys.append((_abi.TSRC_AGG, src[1], desc))
            elif src[0] == "iptext":      # Saddr / Daddr: IPStringFromBytes text order
                keys.append((_abi.TSRC_IPTEXT, (self.key_off[src[1]], self.key_off[src[2]]), desc))
            elif src[0] == "key":
                f = src[1]
                kind = src[2] if len(src) > 2 else sk.kind
                keys.append((_abi.TSRC_KEY, (self.key_off[f], self.ev_width[f], kind), desc))
            else:
                keys.append((_abi.TSRC_CONST, 0, desc))
        return keys

    def _gather_first(self, first, name):
        """Values of event column `name` at global event indices `first` (the BPF first
        insert's attributes: filetop.bpf.c:68-85)."""
        torch = torch_mod()
        out = [None] * len(first)
        bases = [b for b, _, _ in self.batches]
        by_batch = {}
        for i, f in enumerate(first):
            j = bisect.bisect_right(bases, int(f)) - 1
            by_batch.setdefault(j, []).append((i, int(f) - bases[j]))
        for j, lst in by_batch.items():
            t = self.batches[j][2].get(name)
            if t is None:
                continue
            li = torch.tensor([r for _, r in lst], dtype=torch.int32, device=t.device)
            vals = host(_take(t, li))
            for (i, _), v in zip(lst, vals):
                out[i] = v
        return out

    def nextStats(self, limit: Optional[int] = None):
        """All Stats of the interval in SortStats order (limit: only the first `limit`
        rows are materialised -- the order is the same); empties the map."""
        fin = self.table.finalize()
        G = fin["n_groups"]
        k = G if limit is None else min(limit, G)
        stats = []
        if k:
            slots = self.table.sort(self._sort_keys(self.SortBy), k)
            rows = host(self.table.gather(slots))
            stats = self._stats(rows)
        self.table.reset()
        self.batches = []
        return stats

    def NextEvent(self):
        """One tick of tracer.run: stats[:MaxRows] in a top.Event."""
        return Event(Stats=self.nextStats(limit=self.MaxRows))

    def _unpack(self, rows):
        """Packed table rows -> (dict of key fields as numpy, aggregates list, first)."""
        import numpy as np
        kf = {}
        np_t = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}
        for f in self.KEY:
            o, w = self.key_off[f], self.ev_width[f]
            seg = np.ascontiguousarray(rows[:, o:o + w])
            kf[f] = seg if w not in np_t else seg.view(np_t[w]).ravel()
        kb = self.key_bytes
        aggs = [np.ascontiguousarray(rows[:, kb + 8 * i:kb + 8 * i + 8]).view(np.uint64).ravel()
                for i in range(len(self.AGGS))]
        first = np.ascontiguousarray(rows[:, kb + 8 * len(self.AGGS):]).view(np.uint64).ravel()
        return kf, aggs, first

    def destroy(self):
        self.table.destroy()


def _take(t, li):
    from . import engine                     # igx_take on the device
    return engine.take([t], li)[0]


def _stats_columns(fields, extractors=(), virtual=()):
    cols = Columns([("node", "string", 64), ("namespace", "string", 64), ("pod", "string", 64),
                    ("container", "string", 64), ("mntns", "uint64")] + list(fields))
    for name in extractors:
        cols.SetExtractor(name, lambda s: "")
    for name in virtual:
        cols.AddColumn(name, lambda s: "")
    return cols


_ENRICH = {"node": ("const",), "namespace": ("const",), "pod": ("const",), "container": ("const",)}

# ------------------------------------------------------------------------------------
# top tcp
# ------------------------------------------------------------------------------------


@dataclass
class TcpStats:
    """pkg/gadgets/top/tcp/types/types.go:46-58."""
    Node: str = ""           # eventtypes.CommonData (pkg/types/types.go:73-87), filled by enrichers
    Namespace: str = ""
    Pod: str = ""
    Container: str = ""
    MountNsID: int = 0
    Pid: int = 0
    Comm: str = ""
    Family: int = 0
    Saddr: str = ""
    Daddr: str = ""
    Sport: int = 0
    Dport: int = 0
    Sent: int = 0
    Received: int = 0
    FirstIndex: int = 0      # canonical pre-sort position (not in the reference struct)


def copied_pred(copied_col, dir_col):
    """ig_toptcp_clean's `if (copied <= 0) return 0;` (tcptop.bpf.c:124-130) as a group-by
    predicate: `copied > 0` (int32) on the rows with dir == 1 (tcp_cleanup_rbuf); sends pass."""
    return _pred(copied_col, _abi.CMP_GT, (0).to_bytes(4, "little"), guard=(dir_col, b"\x01"))


class TopTcpTracer(_TopTracer):
    """top tcp: probe_ip keyed by ip_key_t, sent/received += size."""
    EVENT = [("saddr", "bytes", 16), ("daddr", "bytes", 16), ("mntns", "uint", 8), ("pid", "uint", 4),
             ("comm", "bytes", 16), ("lport", "uint", 2), ("dport", "uint", 2), ("family", "uint", 2),
             ("size", "uint", 4), ("dir", "uint", 1)]
    KEY = ["saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family"]
    # dir 0 = tcp_sendmsg (sent), 1 = tcp_cleanup_rbuf (received)
    AGGS = [(_abi.AGG_SUM, "size", "dir", 0, 8, 0), (_abi.AGG_SUM, "size", "dir", 1, 8, 0)]
    # the receive probe's argument is `int copied` (tcptop.bpf.c:125)
    ALIASES = [("copied", "size", "int32")]
    STATS_COLS = _stats_columns([("pid", "int32"), ("comm", "string", 16), ("ip", "uint16"),
                                 ("saddr", "string", 46), ("daddr", "string", 46), ("sport", "uint16"),
                                 ("dport", "uint16"), ("sent", "uint64"), ("recv", "uint64")],
                                extractors=("ip", "sent", "recv"), virtual=("local", "remote"))
    SORT_SRC = dict(_ENRICH, mntns=("key", "mntns"), pid=("key", "pid", _abi.KIND_INT),
                    comm=("key", "comm"), ip=("key", "family"), sport=("key", "lport"),
                    dport=("key", "dport"), sent=("agg", 0), recv=("agg", 1),
                    saddr=("iptext", "saddr", "family"), daddr=("iptext", "daddr", "family"))
    SortByDefault = ["-sent", "-recv"]      # types.go:27

    def __init__(self, TargetPid=0, TargetFamily=-1, **kw):
        super().__init__(**kw)
        self.TargetPid = TargetPid
        self.TargetFamily = TargetFamily

    def _preds(self):
        """tcptop.bpf.c:42-55: target_pid (0 = all), target_family (-1 = all), then the
        probe drops every family but AF_INET / AF_INET6; before any of it the receive probe
        returns when `copied <= 0` (tcptop.bpf.c:124-130; sends have no such check)."""
        fam, pid = self.ev_index["family"], self.ev_index["pid"]
        recv_pos = copied_pred(self.ev_index["copied"], self.ev_index["dir"])
        inet = _pred(fam, _abi.CMP_IN, AF_INET.to_bytes(2, "little") + AF_INET6.to_bytes(2, "little"))
        if self.TargetFamily not in (-1, AF_INET, AF_INET6):
            # an impossible family: the two tests contradict, no event is kept
            return [_pred(fam, _abi.CMP_EQ, (self.TargetFamily & 0xFFFF).to_bytes(2, "little")), inet]
        preds = [inet if self.TargetFamily == -1 else
                 _pred(fam, _abi.CMP_EQ, self.TargetFamily.to_bytes(2, "little")), recv_pos]
        if self.TargetPid:
            preds.append(_pred(pid, _abi.CMP_EQ, (self.TargetPid & 0xFFFFFFFF).to_bytes(4, "little")))
        return preds

    def _stats(self, rows):
        kf, (sent, recv), first = self._unpack(rows)
        out = []
        for i in range(rows.shape[0]):
            fam = int(kf["family"][i])
            ipt = 6 if fam == AF_INET6 else 4           # tracer.go:199-203
            pid = int(kf["pid"][i])
            out.append(TcpStats(MountNsID=int(kf["mntns"][i]), Pid=pid - (1 << 32) if pid >= 1 << 31 else pid,
                                Comm=FromCString(kf["comm"][i]), Family=fam,
                                Saddr=IPStringFromBytes(kf["saddr"][i], ipt),
                                Daddr=IPStringFromBytes(kf["daddr"][i], ipt),
                                Sport=int(kf["lport"][i]), Dport=int(kf["dport"][i]),
                                Sent=int(sent[i]), Received=int(recv[i]), FirstIndex=int(first[i])))
        return out


# ------------------------------------------------------------------------------------
# top file
# ------------------------------------------------------------------------------------
@dataclass
class FileStats:
    """pkg/gadgets/top/file/types/types.go:37-51."""
    Node: str = ""           # eventtypes.CommonData (pkg/types/types.go:73-87), filled by enrichers
    Namespace: str = ""
    Pod: str = ""
    Container: str = ""
    MountNsID: int = 0
    Pid: int = 0
    Tid: int = 0
    Comm: str = ""
    Reads: int = 0
    Writes: int = 0
    ReadBytes: int = 0
    WriteBytes: int = 0
    FileType: int = 0
    Filename: str = ""
    FirstIndex: int = 0


READ, WRITE = 0, 1                       # filetop.h enum op


class TopFileTracer(_TopTracer):
    """top file: probe_entry keyed by file_id{inode, dev, pid, tid}; reads/writes++ and
    read/write_bytes += count; the first insert records mntns / comm / filename / type,
    which here are the attributes of the group's first event."""
    EVENT = [("inode", "uint", 8), ("dev", "uint", 4), ("pid", "uint", 4), ("tid", "uint", 4),
             ("op", "uint", 1), ("count", "uint", 4), ("ftype", "uint", 1)]
    KEY = ["inode", "dev", "pid", "tid"]
    AGGS = [(_abi.AGG_COUNT, None, "op", READ, 8, 0), (_abi.AGG_SUM, "count", "op", READ, 8, 0),
            (_abi.AGG_COUNT, None, "op", WRITE, 8, 0), (_abi.AGG_SUM, "count", "op", WRITE, 8, 0)]
    STATS_COLS = _stats_columns([("pid", "uint32"), ("tid", "uint32"), ("comm", "string", 16),
                                 ("reads", "uint64"), ("writes", "uint64"), ("rbytes", "uint64"),
                                 ("wbytes", "uint64"), ("t", "uint8"), ("file", "string", 64)],
                                extractors=("rbytes", "wbytes"))
    SORT_SRC = dict(_ENRICH, pid=("key", "pid"), tid=("key", "tid"), reads=("agg", 0),
                    rbytes=("agg", 1), writes=("agg", 2), wbytes=("agg", 3))
    SortByDefault = ["-reads", "-writes", "-rbytes", "-wbytes"]   # types.go:30

    def __init__(self, TargetPid=0, AllFiles=False, **kw):
        super().__init__(**kw)
        self.TargetPid = TargetPid
        self.AllFiles = AllFiles

    def _preds(self):
        """filetop.bpf.c:49-60: target_pid; regular_file_only && !S_ISREG -> drop (the
        event's ftype is the BPF type_ letter: 'R' regular, 'S' socket, 'O' other)."""
        preds = []
        if self.TargetPid:
            preds.append(_pred(self.ev_index["pid"], _abi.CMP_EQ, (self.TargetPid & 0xFFFFFFFF).to_bytes(4, "little")))
        if not self.AllFiles:
            preds.append(_pred(self.ev_index["ftype"], _abi.CMP_EQ, b"R"))
        return preds

    def _stats(self, rows):
        kf, (reads, rbytes, writes, wbytes), first = self._unpack(rows)
        mntns = self._gather_first(first, "mntns")
        comm = self._gather_first(first, "comm")
        fname = self._gather_first(first, "filename")
        ftype = self._gather_first(first, "ftype")
        out = []
        for i in range(rows.shape[0]):
            out.append(FileStats(MountNsID=int(mntns[i]) if mntns[i] is not None else 0,
                                 Pid=int(kf["pid"][i]), Tid=int(kf["tid"][i]),
                                 Comm=FromCString(comm[i].tobytes()) if comm[i] is not None else "",
                                 Reads=int(reads[i]), Writes=int(writes[i]), ReadBytes=int(rbytes[i]),
                                 WriteBytes=int(wbytes[i]),
                                 FileType=int(ftype[i]) if ftype[i] is not None else 0,
                                 Filename=FromCString(fname[i].tobytes()) if fname[i] is not None else "",
                                 FirstIndex=int(first[i])))
        return out


# ------------------------------------------------------------------------------------
# top block-io
# ------------------------------------------------------------------------------------
@dataclass
class BlockIOStats:
    """pkg/gadgets/top/block-io/types/types.go:35-48."""
    Node: str = ""           # eventtypes.CommonData (pkg/types/types.go:73-87), filled by enrichers
    Namespace: str = ""
    Pod: str = ""
    Container: str = ""
    MountNsID: int = 0
    Pid: int = 0
    Comm: str = ""
    Write: bool = False
    Major: int = 0
    Minor: int = 0
    Bytes: int = 0
    MicroSecs: int = 0
    Operations: int = 0
    FirstIndex: int = 0


class TopBlockIOTracer(_TopTracer):
    """top block-io: ig_topio_done keyed by info_t{mntnsid, pid, rwflag, major, minor,
    name}; us += (now - start)/1000, bytes += data_len, io++ (u32)."""
    EVENT = [("mntns", "uint", 8), ("pid", "uint", 4), ("rwflag", "int", 4), ("major", "int", 4),
             ("minor", "int", 4), ("comm", "bytes", 16), ("data_len", "uint", 8), ("delta_ns", "uint", 8)]
    KEY = ["mntns", "pid", "rwflag", "major", "minor", "comm"]
    AGGS = [(_abi.AGG_SUM, "data_len", None, 0, 8, 0), (_abi.AGG_SUM, "delta_ns", None, 0, 8, 1000),
            (_abi.AGG_COUNT, None, None, 0, 4, 0)]
    STATS_COLS = _stats_columns([("pid", "int32"), ("comm", "string", 16), ("r/w", "bool"),
                                 ("major", "int"), ("minor", "int"), ("bytes", "uint64"),
                                 ("time", "uint64"), ("ops", "uint32")], extractors=("r/w",))
    SORT_SRC = dict(_ENRICH, mntns=("key", "mntns"), pid=("key", "pid", _abi.KIND_INT),
                    comm=("key", "comm"), major=("key", "major", _abi.KIND_INT),
                    minor=("key", "minor", _abi.KIND_INT), bytes=("agg", 0), time=("agg", 1),
                    ops=("agg", 2))
    SortByDefault = ["-ops", "-bytes", "-time"]    # types.go:31

    def _stats(self, rows):
        import numpy as np
        kf, (nbytes, us, io), first = self._unpack(rows)
        out = []
        for i in range(rows.shape[0]):
            pid = int(kf["pid"][i])
            out.append(BlockIOStats(MountNsID=int(kf["mntns"][i]), Pid=pid - (1 << 32) if pid >= 1 << 31 else pid,
                                    Comm=FromCString(kf["comm"][i]), Write=int(kf["rwflag"][i]) != 0,
                                    Major=int(np.int32(np.uint32(kf["major"][i]))),
                                    Minor=int(np.int32(np.uint32(kf["minor"][i]))),
                                    Bytes=int(nbytes[i]), MicroSecs=int(us[i]),
                                    Operations=int(io[i]) & 0xFFFFFFFF, FirstIndex=int(first[i])))
        return out


# ------------------------------------------------------------------------------------
# output side: the Stats types' column tags and JSON fields
# ------------------------------------------------------------------------------------
# eventtypes.CommonData + WithMountNsID (pkg/types/types.go:73-87,217-219)
_COMMON_COLS = [("Node", "string", "node,template:node", ["kubernetes"]),
                ("Namespace", "string", "namespace,template:namespace", ["kubernetes"]),
                ("Pod", "string", "pod,template:pod", ["kubernetes"]),
                ("Container", "string", "container,template:container", ["kubernetes", "runtime"]),
                ("MountNsID", "uint64", "mntns,template:ns", [])]
_COMMON_JSON = [("Node", "node", True), ("Namespace", "namespace", True), ("Pod", "pod", True),
                ("Container", "container", True), ("MountNsID", "mountnsid", True)]

STATS_OUTPUT = {
    # pkg/gadgets/top/tcp/types/types.go:46-101
    "tcp": {
        "fields": _COMMON_COLS + [("Pid", "int32", "pid,template:pid", []), ("Comm", "string", "comm,template:comm", []),
                                  ("Family", "uint16", "ip,maxWidth:2", []),
                                  ("Saddr", "string", "saddr,template:ipaddr,hide", []),
                                  ("Daddr", "string", "daddr,template:ipaddr,hide", []),
                                  ("Sport", "uint16", "sport,template:ipport,hide", []),
                                  ("Dport", "uint16", "dport,template:ipport,hide", []),
                                  ("Sent", "uint64", "sent,order:1002", []),
                                  ("Received", "uint64", "recv,order:1003", [])],
        "json": _COMMON_JSON + [("Pid", "pid", True), ("Comm", "comm", True), ("Family", "family", True),
                                ("Saddr", "saddr", True), ("Daddr", "daddr", True), ("Sport", "sport", True),
                                ("Dport", "dport", True), ("Sent", "sent", True), ("Received", "received", True)],
    },
    # pkg/gadgets/top/file/types/types.go:37-66
    "file": {
        "fields": _COMMON_COLS + [("Pid", "uint32", "pid,template:pid", []), ("Tid", "uint32", "tid,template:pid,hide", []),
                                  ("Comm", "string", "comm,template:comm", []), ("Reads", "uint64", "reads", []),
                                  ("Writes", "uint64", "writes", []), ("ReadBytes", "uint64", "rbytes", []),
                                  ("WriteBytes", "uint64", "wbytes", []), ("FileType", "uint8", "T,maxWidth:1", []),
                                  ("Filename", "string", "file", [])],
        "json": _COMMON_JSON + [("Pid", "pid", True), ("Tid", "tid", True), ("Comm", "comm", True),
                                ("Reads", "reads", True), ("Writes", "writes", True), ("ReadBytes", "rbytes", True),
                                ("WriteBytes", "wbytes", True), ("FileType", "fileType", True),
                                ("Filename", "filename", True)],
    },
    # pkg/gadgets/top/block-io/types/types.go:34-61
    "block-io": {
        "fields": _COMMON_COLS + [("Pid", "int32", "pid", []), ("Comm", "string", "comm", []),
                                  ("Write", "bool", "r/w,maxWidth:3", []), ("Major", "int", "major", []),
                                  ("Minor", "int", "minor", []), ("Bytes", "uint64", "bytes", []),
                                  ("MicroSecs", "uint64", "time", []), ("Operations", "uint32", "ops", [])],
        "json": _COMMON_JSON + [("Pid", "pid", True), ("Comm", "comm", True), ("Write", "write", True),
                                ("Major", "major", True), ("Minor", "minor", True), ("Bytes", "bytes", True),
                                ("MicroSecs", "us", True), ("Operations", "ops", True)],
    },
}


def StatsColumns(gadget: str):
    """types.GetColumns() of a top gadget's Stats: the tagged fields plus its extractors and
    virtual columns, as a textcolumns.ColumnMap (every column; see OutputColumns for the
    frontends' tag filter)."""
    from . import textcolumns as T
    spec = STATS_OUTPUT[gadget]
    cm = T.ColumnMap([(attr, kind, tag) for attr, kind, tag, _ in spec["fields"]])
    for attr, kind, tag, tags in spec["fields"]:
        cm.cols[tag.split(",")[0].lower()].Tags = list(tags)
    if gadget == "tcp":
        cm.SetExtractor("ip", lambda st: "4" if st.Family == AF_INET else "6")
        cm.SetExtractor("sent", lambda st: T.BytesSize(float(st.Sent)))
        cm.SetExtractor("recv", lambda st: T.BytesSize(float(st.Received)))
        cm.AddColumn("local", lambda st: f"{st.Saddr}:{st.Sport}", MinWidth=21, MaxWidth=51, Order=1000)
        cm.AddColumn("remote", lambda st: f"{st.Daddr}:{st.Dport}", MinWidth=21, MaxWidth=51, Order=1000)
    elif gadget == "file":
        cm.SetExtractor("rbytes", lambda st: T.BytesSize(float(st.ReadBytes)))
        cm.SetExtractor("wbytes", lambda st: T.BytesSize(float(st.WriteBytes)))
        cm.SetExtractor("T", lambda st: chr(st.FileType))
    else:
        cm.SetExtractor("r/w", lambda st: "W" if st.Write else "R")
    return cm


def OutputColumns(gadget: str, metadata_tag: str = ""):
    """The column map a frontend formats with (parser-tableformatter.go:60-65): columns
    without tags, plus those carrying metadata_tag ("kubernetes" for kubectl-gadget, "runtime"
    for ig with a container runtime; "" = untagged only)."""
    cm = StatsColumns(gadget)
    cm.cols = {k: c for k, c in cm.cols.items() if not c.Tags or (metadata_tag and metadata_tag in c.Tags)}
    return cm


def render_table(gadget: str, stats, metadata_tag: str = "", terminal_width: int = 0, columns=None) -> str:
    """The columns output of one interval (GadgetParser.TransformIntoTable over the interval's
    []*Stats, cmd/common/utils/parser-tableformatter.go:106-111)."""
    from . import textcolumns as T
    f = T.TextColumnsFormatter(OutputColumns(gadget, metadata_tag), DefaultColumns=columns)
    return T.TransformIntoTable(f, stats, terminal_width)


def render_json(gadget: str, stats) -> str:
    """-o json: json.Marshal of the interval's []*Stats (cmd/common/registry.go:511-520)."""
    from . import textcolumns as T
    return T.marshal_array(stats, STATS_OUTPUT[gadget]["json"])


def rwflag_of(cmd_flags):
    """biotop.bpf.c:106: !!((cmd_flags & REQ_OP_MASK) == REQ_OP_WRITE) (host helper)."""
    return int((int(cmd_flags) & 0xFF) == REQ_OP_WRITE)


# ------------------------------------------------------------------------------------
# streaming interval mode
# ------------------------------------------------------------------------------------
class StreamingTopTracer:
    """The top tracers' run loop (e.g. pkg/gadgets/top/tcp/tracer/tracer.go:228-265: a
    ticker calls nextStats, emits stats[:MaxRows], counts Iterations down) over two device
    tables.  A tick swaps the tables before draining, so the next interval's events are
    aggregated into the other table -- on a HIP stream of its own -- while the host sorts,
    gathers and builds the Stats of the interval that just closed (the BPF map keeps taking
    events while nextStats walks and deletes it).

    cls: a _TopTracer subclass; kw: its constructor arguments (MaxRows, SortBy, capacity,
    filter options).  Events get global indices continuing across intervals."""

    def __init__(self, cls, Iterations=0, device=None, **kw):
        torch = torch_mod()
        from .runtime import Context
        dev = torch.cuda.current_device() if device is None else device
        self.Iterations = Iterations
        self.count = Iterations
        self.streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        self.ctxs = [Context(dev, stream=s) for s in self.streams]
        self.tracers = []
        for s, c in zip(self.streams, self.ctxs):
            with torch.cuda.stream(s):
                self.tracers.append(cls(ctx=c, **kw))
        self.cur = 0
        self.next_idx = 0
        self.done = False

    def feed(self, events: dict, n: Optional[int] = None):
        """Events of the current interval (device tensors made on torch's current stream)."""
        torch = torch_mod()
        tr, s = self.tracers[self.cur], self.streams[self.cur]
        s.wait_stream(torch.cuda.current_stream())
        n = int(events[tr.KEY[0]].shape[0]) if n is None else n
        with torch.cuda.stream(s):
            tr.feed(events, n, base_idx=self.next_idx)
        for t in events.values():
            t.record_stream(s)           # the caller's tensors stay alive for the update
        self.next_idx += n

    def tick(self):
        """ticker.C: the interval ends -> top.Event with stats[:MaxRows]; None after the
        last iteration."""
        if self.done:
            return None
        torch = torch_mod()
        closed = self.cur
        self.cur ^= 1                    # later feeds go to the other table
        with torch.cuda.stream(self.streams[closed]):
            ev = self.tracers[closed].NextEvent()
        if self.Iterations > 0:
            self.count -= 1
            self.done = self.count == 0
        return ev

    def run(self, intervals):
        """Generator over intervals (each an iterable of event batches): interval k+1's
        updates are enqueued before the host blocks on interval k's drain."""
        pending = False
        for batches in intervals:
            if pending:
                # enqueue this interval's batches into the fresh table, then drain the old one
                closed = self.cur ^ 1
                for b in batches:
                    self.feed(b)
                torch = torch_mod()
                with torch.cuda.stream(self.streams[closed]):
                    ev = self.tracers[closed].NextEvent()
                yield ev
                if self.Iterations > 0:
                    self.count -= 1
                    if self.count == 0:
                        return
            else:
                for b in batches:
                    self.feed(b)
            self.cur ^= 1
            pending = True
        if pending:
            yield self.tick_closed()

    def tick_closed(self):
        torch = torch_mod()
        closed = self.cur ^ 1
        with torch.cuda.stream(self.streams[closed]):
            return self.tracers[closed].NextEvent()

    def destroy(self):
        for t in self.tracers:
            t.destroy()
        for c in self.ctxs:
            c.close()



# ------------------------------------------------------------------------------------
# profile block-io
# ------------------------------------------------------------------------------------
MAX_SLOTS = 27          # biolatency.h:6


@dataclass
class Data:
    """profile/block-io/types/types.go:17-21."""
    count: int
    intervalStart: int
    intervalEnd: int


@dataclass
class Report:
    """profile/block-io/types/types.go:23-27."""
    ValType: str = ""
    Data: List[Data] = field(default_factory=list)
    Time: str = ""

    def to_json(self) -> str:
        """json.Marshal(report) with the reference's omitempty tags."""
        d = {}
        if self.ValType:
            d["valType"] = self.ValType
        if self.Data:
            d["data"] = [{k: v for k, v in (("count", x.count), ("intervalStart", x.intervalStart),
                                             ("intervalEnd", x.intervalEnd)) if k != "intervalEnd" or v}
                         for x in self.Data]
        if self.Time:
            d["ts"] = self.Time
        return json.dumps(d, separators=(",", ":"))


def getReport(slots, val_type="usecs") -> Report:
    """tracer.go:56-90: Data[i] = {Count, 1<<i, (1<<(i+1))-1}, truncated to
    data[:indexMax] -- the highest non-zero slot is dropped (reference behaviour)."""
    data, index_max = [], 0
    for i, v in enumerate(slots):
        v = int(v)
        if v > 0:
            index_max = i
        data.append(Data(v, (1 << (i + 1)) >> 1, (1 << (i + 1)) - 1))
    return Report(ValType=val_type, Data=data[:index_max])


def starsToString(val: int, valMax: int, width: int) -> str:
    """gadget.go:88-110 (bcc print_stars)."""
    if valMax == 0:
        return " " * width
    stars = min(val, valMax) * width // valMax
    s = "*" * stars + " " * (width - stars)
    if val > valMax:
        s += "+"
    return s


def reportToString(report: Report) -> str:
    """gadget.go:112-143 (bcc print_log2_hist)."""
    if not report.Data:
        return ""
    val_max = max(d.count for d in report.Data)
    out = ["%5s%-19s : count    distribution\n" % ("", report.ValType)]
    for d in report.Data:
        out.append("%10d -> %-10d : %-8d |%s|\n" % (d.intervalStart, d.intervalEnd, d.count,
                                                   starsToString(d.count, val_max, 40)))
    return "".join(out)


class ProfileBlockIOTracer:
    """profile block-io: ig_profio_done's log2 histogram on the device.

    devs=None is the shipped gadget (no targ_per_disk / targ_per_flag: one key {0,0} for
    every I/O); devs=[MKDEV(major, minor), ...] (and ncont > 1 with a container column)
    keys per device (and per container), the C3 extension.  ms=True is targ_ms."""

    def __init__(self, devs=None, ncont=1, ms=False, per_disk=False, per_flag=False):
        self.devs = list(devs or [])
        self.ncont = ncont
        self.divisor = 1000000 if ms else 1000
        self.val_type = "msecs" if ms else "usecs"
        self.hist = None
        # targ_per_disk / targ_per_flag (biolatency.bpf.c:116-131): histograms keyed by the raw
        # hist_key{cmd_flags, dev} values instead of the dense dev x container index
        self.per_disk, self.per_flag = per_disk, per_flag
        self.keyed = {}   # (cmd_flags, dev) -> u32 slots, in first-event order

    def feed(self, delta_ns, dev=None, cont=None, cmd_flags=None):
        if self.per_disk or self.per_flag:
            import numpy as np
            for cf, dv, h in engine.hist_log2_keyed(delta_ns, cmd_flags if self.per_flag else None,
                                                    dev if self.per_disk else None, self.divisor, MAX_SLOTS):
                cur = self.keyed.setdefault((cf, dv), np.zeros(MAX_SLOTS, np.uint32))
                cur += h   # u32 wrap, like __sync_fetch_and_add on the map's u32 slots
            return
        self.hist = engine.hist_log2(dev, cont, delta_ns, self.devs, self.ncont, self.divisor,
                                     MAX_SLOTS, hist=self.hist)

    def slots(self):
        """u32 slots per key, host numpy (nkeys, 27); keyed mode: in first-event order."""
        import numpy as np
        if self.per_disk or self.per_flag:
            if not self.keyed:
                return np.zeros((0, MAX_SLOTS), np.uint32)
            return np.stack(list(self.keyed.values()))
        if self.hist is None:
            return np.zeros((max(1, len(self.devs)) * self.ncont, MAX_SLOTS), np.uint32)
        return host(self.hist)

    def keys(self):
        """keyed mode: the hist_key{cmd_flags, dev} of each row of slots()."""
        return list(self.keyed.keys())

    def getReport(self, key: int = 0) -> Report:
        """The reference reads the first key only (NextKey(nil), the BPF map's hash order); key
        picks one here (first-event order in keyed mode)."""
        return getReport(self.slots()[key], self.val_type)

    def Stop(self) -> str:
        """tracer.go:92-113: json.Marshal(getReport(...))."""
        return self.getReport().to_json()
