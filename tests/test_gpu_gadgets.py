"""GPU parity of the gadget mirrors (inspektor-gadget_amd/gadgets.py) and the parser
pipeline (parser.py) against the oracle: the BPF probe semantics (oracle.groupby, with the
probe filters as a row mask), nextStats -> top.SortStats in first-occurrence order
(oracle.go_sort_entries, the Go 1.19 SliceStable restatement), MaxRows truncation, and
profile block-io's histogram + getReport.  All bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as T
    return T


@pytest.fixture(scope="module")
def G(igx):
    import importlib
    return importlib.import_module("inspektor-gadget_amd.gadgets")


def _dev(H, ev):
    return {k: H.to_device(v) for k, v in ev.items()}


def _ref_top(oracle, key_arrays, aggs, valid, sort_spec, k, base_idx=0):
    """Reference nextStats + SortStats + truncation: groups in first-occurrence order,
    SliceStable per sortBy key.  sort_spec: [(fn(groups)->column, kind, desc)]."""
    keys = oracle.pad_keys(key_arrays, list(key_arrays))
    okeys, oaggs, ofirst = oracle.groupby(keys, aggs, valid=valid, base_idx=base_idx)
    grp = {"keys": okeys, "aggs": oaggs, "first": ofirst}
    perm = oracle.go_sort_entries([(fn(grp), kind, desc) for fn, kind, desc in sort_spec], len(ofirst))
    sel = perm[:k].astype(np.int64)
    return len(ofirst), okeys[sel], oaggs[:, sel], ofirst[sel]


def _agg_col(i):
    return lambda g: g["aggs"][i]


@pytest.mark.parametrize("target_pid,target_family", [(0, -1), (0, 10), (4242, -1), (0, 7)])
def test_top_tcp_tracer(oracle, igx, torch, G, target_pid, target_family):
    H = igx.columns
    Gk, n = 5000, 300_000
    cdf = oracle.zipf_cdf(Gk, 1.1)
    ev_h = oracle.gen_tcp(0xC2, 0, Gk, cdf, 0, n)
    ev_h["family"][::7] = 1          # AF_UNIX: the probe drops it
    if target_pid:
        ev_h["pid"][::3] = target_pid
    ev = _dev(H, ev_h)
    tr = G.TopTcpTracer(TargetPid=target_pid, TargetFamily=target_family, MaxRows=20, capacity=2 * Gk)
    half = n // 2
    tr.feed({k: v[:half] for k, v in ev.items()})
    tr.feed({k: v[half:] for k, v in ev.items()})
    evt = tr.NextEvent()
    fam, pid = ev_h["family"], ev_h["pid"]
    keep = ((fam == 2) | (fam == 10)) & ~((ev_h["dir"] == 1) & (ev_h["size"].view(np.int32) <= 0))
    if target_family != -1:
        keep &= fam == target_family
    if target_pid:
        keep &= pid == target_pid
    names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")
    Gn, keys, aggs, first = _ref_top(
        oracle, {k: ev_h[k] for k in names},
        [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
         {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}], keep,
        [(_agg_col(0), "uint64", True), (_agg_col(1), "uint64", True)], 20)
    assert len(evt.Stats) == min(20, Gn)
    assert [s.FirstIndex for s in evt.Stats] == [int(x) for x in first]
    assert [(s.Sent, s.Received) for s in evt.Stats] == list(zip(aggs[0].tolist(), aggs[1].tolist()))
    for s, kb in zip(evt.Stats, keys):
        assert s.Pid == int(kb[40:44].view(np.int32)[0])
        assert s.Comm == G.FromCString(kb[44:60].tobytes())
        assert s.Sport == int(kb[60:62].view(np.uint16)[0]) and s.Family in (2, 10)
        ipt = 6 if s.Family == 10 else 4
        assert s.Saddr == G.IPStringFromBytes(kb[0:16].tobytes(), ipt)
    # the interval is drained: the next tick is empty
    assert tr.NextEvent().Stats == []
    tr.destroy()


@pytest.mark.parametrize("target_pid", [0, 4242])
def test_top_tcp_receive_copied_drop(oracle, igx, torch, G, target_pid):
    """ig_toptcp_clean returns before probe_ip when `int copied <= 0` (tcptop.bpf.c:124-130);
    the send probe has no such check (:112-116), so a zero-size send still creates its group.
    The stream holds zero and negative (int32) receives, zero-size sends, and keys whose only
    events are dropped receives (those groups must not exist).  Through TopTcpTracer (the
    guarded predicate fused into the cached kernel, and with target_pid a third predicate,
    so one of them runs as a row mask) and every group-by form, against the oracle's
    or_top_tcp / or_top_tcp_mt, which restate the drop."""
    H = igx.columns
    Gk, n = 4000, 400_000
    ev_h = oracle.gen_tcp(0xC2, 3, Gk, oracle.zipf_cdf(Gk, 1.1), 0, n)
    rng = np.random.default_rng(11)
    size = ev_h["size"]
    r = rng.integers(0, 8, n)
    size[r == 0] = 0                                                    # copied == 0 / size 0
    size[r == 1] = np.uint32(0x80000000) | size[r == 1]                 # negative as int32
    size[r == 2] = np.uint32(0xFFFFFFFF)                                # -1
    size[r == 3] = np.uint32(0x7FFFFFFF)                                # INT_MAX: kept
    # keys seen only through dropped receives: rows of a fresh pid, all dir 1 with copied <= 0
    lone = rng.choice(n, 300, replace=False)
    ev_h["pid"][lone] = np.uint32(7_000_000) + np.arange(300, dtype=np.uint32)
    ev_h["dir"][lone] = 1
    size[lone] = 0
    if target_pid:
        ev_h["pid"][::3] = target_pid
    ev = _dev(H, ev_h)
    dir_, s32 = ev_h["dir"], size.view(np.int32)
    assert ((dir_ == 1) & (s32 <= 0)).sum() > 1000 and ((dir_ == 0) & (size == 0)).sum() > 1000
    keep = ~((dir_ == 1) & (s32 <= 0))
    if target_pid:
        keep &= ev_h["pid"] == target_pid
    names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")
    Gn, keys, aggs, first = _ref_top(
        oracle, {k: ev_h[k] for k in names},
        [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
         {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}],
        keep & ((ev_h["family"] == 2) | (ev_h["family"] == 10)),
        [(_agg_col(0), "uint64", True), (_agg_col(1), "uint64", True)], 20)
    if not target_pid:   # the C restatements carry the drop themselves
        Gc, _, csent, crecv, cfirst = oracle.top_tcp(ev_h, 20)
        Gm, msent, mrecv, mfirst = oracle.top_tcp_mt(ev_h, 20, threads=4)
        assert Gc == Gm == Gn
        assert list(cfirst) == list(mfirst) == [int(x) for x in first]
        assert list(csent) == list(msent) == aggs[0].tolist() and list(crecv) == aggs[1].tolist()
    A = igx._abi
    for mode in (A.GB_AUTO, A.GB_CACHED, A.GB_DIRECT, A.GB_PART):
        tr = G.TopTcpTracer(TargetPid=target_pid, MaxRows=20, capacity=2 * Gk)
        tr.table.set_mode(mode)
        tr.feed(ev)
        evt = tr.NextEvent()
        assert tr.table.fin["n_groups"] == Gn, mode
        assert [s.FirstIndex for s in evt.Stats] == [int(x) for x in first], mode
        assert [(s.Sent, s.Received) for s in evt.Stats] == list(zip(aggs[0].tolist(), aggs[1].tolist())), mode
        tr.destroy()


def test_top_tcp_sort_by_key_columns(oracle, igx, torch, G):
    """SortBy over key columns (pid is int32: signed order; comm bytes) and a constant
    enrichment column whose '-' only flips the tie parity."""
    H = igx.columns
    Gk, n = 3000, 100_000
    ev_h = oracle.gen_tcp(0xC2, 1, Gk, oracle.zipf_cdf(Gk, 1.1), 0, n)
    ev_h["pid"][::5] |= np.uint32(0x80000000)          # negative pids as int32
    ev = _dev(H, ev_h)
    names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")
    for sort_by in (["comm", "-pid"], ["-namespace", "pid"], ["-ip", "-sport", "recv"], ["bogus", "-recv"]):
        tr = G.TopTcpTracer(SortBy=sort_by, capacity=2 * Gk)
        tr.feed(ev)
        stats = tr.nextStats()
        spec = []
        for s in sort_by:
            d, c = s.startswith("-"), s.lstrip("-")
            if c == "comm":
                spec.append((lambda g: g["keys"][:, 44:60], "string", d))
            elif c == "pid":
                spec.append((lambda g: g["keys"][:, 40:44].copy().view(np.int32).ravel(), "int32", d))
            elif c == "namespace":
                spec.append((lambda g: np.zeros((len(g["first"]), 1), np.uint8), "string", d))
            elif c == "ip":
                spec.append((lambda g: g["keys"][:, 68:70].copy().view(np.uint16).ravel(), "uint16", d))
            elif c == "sport":
                spec.append((lambda g: g["keys"][:, 60:62].copy().view(np.uint16).ravel(), "uint16", d))
            elif c == "recv":
                spec.append((_agg_col(1), "uint64", d))
        Gn, _, _, first = _ref_top(
            oracle, {k: ev_h[k] for k in names},
            [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
             {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}],
            (ev_h["family"] == 2) | (ev_h["family"] == 10), spec, n)
        assert [s.FirstIndex for s in stats] == [int(x) for x in first], sort_by
        tr.destroy()


def _ip_cases():
    """Edge cases of netip's text form: all-zero, loopback, leading / trailing / tied zero
    runs, a single zero group (never "::"), IPv4-mapped, and family != AF_INET6."""
    v6 = ["::", "::1", "1::", "1:0:1::1:0:0", "2001:db8::1", "2001:db8:0:1:0:0:0:1", "fe80::1:2:3:4",
          "ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff", "0:1:0:1:0:1:0:1", "1:2:3:4:5:6:7:0", "::ffff:10.0.0.1",
          "::ffff:0:0", "::fffe:1.2.3.4", "abcd:ef01::"]
    import ipaddress
    rows = [(ipaddress.IPv6Address(a).packed, 10) for a in v6]
    rows += [(bytes([10, 0, 255, 7]) + bytes(12), 2), (bytes([0, 0, 0, 0]) + bytes(range(12)), 2),
             (bytes([192, 168, 1, 100]) + bytes(12), 0), (bytes(range(16)), 7)]
    return rows


def test_ip_text_matches_netip(oracle, igx, torch):
    """igx_ip_text == IPStringFromBytes (helpers.go:111-120) on edge cases and random
    addresses, through a row map."""
    H = igx.columns
    rng = np.random.default_rng(11)
    rows = _ip_cases()
    for _ in range(5000):
        g = rng.integers(0, 3, 8)
        v = rng.integers(0, 65536, 8) * (g > 0)
        rows.append((b"".join(int(x).to_bytes(2, "big") for x in v), int(rng.choice([2, 10, 10]))))
    n = len(rows)
    addr = np.frombuffer(b"".join(r[0] for r in rows), np.uint8).reshape(n, 16).copy()
    fam = np.array([r[1] for r in rows], np.uint16)
    want = oracle.ip_text_rows(addr, fam)
    got = H.host(igx.engine.ip_text(H.to_device(addr), H.to_device(fam)))
    assert np.array_equal(got, want)
    for i in range(len(_ip_cases())):
        assert bytes(got[i]).rstrip(b"\0").decode() == G_ipstr(igx, rows[i])
    rowmap = rng.permutation(n).astype(np.int32)
    got2 = H.host(igx.engine.ip_text(H.to_device(addr), H.to_device(fam), rowmap=H.to_device(rowmap)))
    assert np.array_equal(got2, want[rowmap])


def G_ipstr(igx, row):
    return igx.gadgets.IPStringFromBytes(row[0], 6 if row[1] == 10 else 4)


def test_top_tcp_sort_by_addresses(oracle, igx, torch, G):
    """SortBy saddr / daddr: the Stats strings (tracer.go:199-206) in Go string order."""
    H = igx.columns
    Gk, n = 3000, 100_000
    ev_h = oracle.gen_tcp(0xC2, 2, Gk, oracle.zipf_cdf(Gk, 1.1), 0, n)
    rng = np.random.default_rng(3)
    pool = np.frombuffer(b"".join(a for a, _ in _ip_cases()[:14]), np.uint8).reshape(14, 16)
    sel = rng.random(n) < 0.3
    ev_h["family"][sel] = 10
    ev_h["saddr"][sel] = pool[rng.integers(0, 14, int(sel.sum()))]
    ev_h["daddr"][sel] = pool[rng.integers(0, 14, int(sel.sum()))]
    ev = _dev(H, ev_h)
    names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")

    def text(off):
        return lambda g: oracle.ip_text_rows(g["keys"][:, off:off + 16],
                                             g["keys"][:, 68:70].copy().view(np.uint16).ravel())
    for sort_by in (["saddr"], ["-daddr", "recv"], ["-saddr", "-daddr"], ["daddr", "-sent"]):
        tr = G.TopTcpTracer(SortBy=sort_by, capacity=1 << 17)
        tr.feed(ev)
        stats = tr.nextStats()
        spec = []
        for s_ in sort_by:
            d, c = s_.startswith("-"), s_.lstrip("-")
            spec.append({"saddr": (text(0), "string", d), "daddr": (text(16), "string", d),
                         "recv": (_agg_col(1), "uint64", d), "sent": (_agg_col(0), "uint64", d)}[c])
        Gn, _, _, first = _ref_top(
            oracle, {k: ev_h[k] for k in names},
            [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
             {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}],
            (ev_h["family"] == 2) | (ev_h["family"] == 10), spec, n)
        assert [s.FirstIndex for s in stats] == [int(x) for x in first], sort_by
        # and the strings the rows carry are in that order
        key = [s.Saddr if sort_by[0].lstrip("-") == "saddr" else s.Daddr for s in stats]
        assert key == sorted(key, key=lambda x: x.encode(), reverse=sort_by[0].startswith("-"))
        tr.destroy()


def _file_events(n, G_keys, seed=5):
    rng = np.random.default_rng(seed)
    kid = rng.zipf(1.3, n) % G_keys
    ev = {"inode": (kid.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)),
          "dev": (kid % 7).astype(np.uint32), "pid": (1000 + kid % 97).astype(np.uint32),
          "tid": (1000 + kid % 97 + (kid % 3)).astype(np.uint32),
          "op": rng.integers(0, 2, n).astype(np.uint8),
          "count": rng.integers(1, 1 << 20, n).astype(np.uint32),
          "ftype": np.array([ord("R"), ord("S"), ord("O")], np.uint8)[
              np.where(kid % 5 == 0, 1, np.where(kid % 11 == 0, 2, 0))],
          "mntns": rng.integers(1, 1 << 40, n).astype(np.uint64),
          "comm": np.frombuffer(b"".join(b"proc%-12d" % (i % 50) for i in range(n)), np.uint8).reshape(n, 16).copy(),
          "filename": np.frombuffer(b"".join(b"/var/f%-26d" % (i % 77) for i in range(n)), np.uint8).reshape(n, 32).copy()}
    return ev


@pytest.mark.parametrize("all_files", [False, True])
def test_top_file_tracer(oracle, igx, torch, G, all_files):
    H = igx.columns
    n = 200_000
    ev_h = _file_events(n, 20_000)
    ev = _dev(H, ev_h)
    tr = G.TopFileTracer(AllFiles=all_files, MaxRows=50, capacity=1 << 16)
    tr.feed(ev, base_idx=777)
    stats = tr.NextEvent().Stats
    keep = np.ones(n, bool) if all_files else ev_h["ftype"] == ord("R")
    op = ev_h["op"]
    Gn, keys, aggs, first = _ref_top(
        oracle, {k: ev_h[k] for k in ("inode", "dev", "pid", "tid")},
        [{"kind": "count", "cond": op, "cond_val": 0}, {"kind": "sum", "val": ev_h["count"], "cond": op, "cond_val": 0},
         {"kind": "count", "cond": op, "cond_val": 1}, {"kind": "sum", "val": ev_h["count"], "cond": op, "cond_val": 1}],
        keep, [(_agg_col(0), "uint64", True), (_agg_col(2), "uint64", True), (_agg_col(1), "uint64", True),
               (_agg_col(3), "uint64", True)], 50, base_idx=777)
    assert [s.FirstIndex for s in stats] == [int(x) for x in first]
    assert [(s.Reads, s.ReadBytes, s.Writes, s.WriteBytes) for s in stats] == \
        list(zip(*(a.tolist() for a in aggs)))
    for s, f in zip(stats, first):          # first-insert attributes (filetop.bpf.c:68-85)
        r = int(f) - 777
        assert s.MountNsID == int(ev_h["mntns"][r]) and s.FileType == int(ev_h["ftype"][r])
        assert s.Comm == G.FromCString(ev_h["comm"][r].tobytes())
        assert s.Filename == G.FromCString(ev_h["filename"][r].tobytes())
    tr.destroy()


def test_top_block_io_tracer(oracle, igx, torch, G):
    """biotop: key info_t, bytes += data_len, us += delta_ns / 1000 per event, io++ (u32);
    default sort ["-ops","-bytes","-time"] = ops DESC, bytes ASC, time DESC, position DESC."""
    H = igx.columns
    n = 250_000
    rng = np.random.default_rng(11)
    kid = rng.zipf(1.2, n) % 4000
    ev_h = {"mntns": (4026531840 + kid % 13).astype(np.uint64), "pid": (100 + kid % 400).astype(np.uint32),
            "rwflag": (kid % 2).astype(np.int32), "major": np.full(n, 8, np.int32),
            "minor": (16 * (kid % 5)).astype(np.int32),
            "comm": np.frombuffer(b"".join(b"kworker/%-8d" % (k % 400) for k in kid), np.uint8).reshape(n, 16).copy(),
            "data_len": (4096 * rng.integers(1, 64, n)).astype(np.uint64),
            "delta_ns": rng.integers(0, 5_000_000, n).astype(np.uint64)}
    ev_h["data_len"][::97] = np.uint64(4096)       # ties on bytes
    ev = _dev(H, ev_h)
    tr = G.TopBlockIOTracer(MaxRows=30, capacity=1 << 14)
    tr.feed(ev)
    stats = tr.NextEvent().Stats
    Gn, keys, aggs, first = _ref_top(
        oracle, {k: ev_h[k] for k in ("mntns", "pid", "rwflag", "major", "minor", "comm")},
        [{"kind": "sum", "val": ev_h["data_len"]}, {"kind": "sum", "val": ev_h["delta_ns"], "div": 1000},
         {"kind": "count", "out_width": 4}], None,
        [(lambda g: (g["aggs"][2] & 0xFFFFFFFF).astype(np.uint32), "uint32", True),
         (_agg_col(0), "uint64", True), (_agg_col(1), "uint64", True)], 30)
    assert [s.FirstIndex for s in stats] == [int(x) for x in first]
    assert [(s.Bytes, s.MicroSecs, s.Operations) for s in stats] == list(zip(*(a.tolist() for a in aggs)))
    assert all(s.Major == 8 for s in stats)
    tr.destroy()


def test_profile_block_io_single_key(oracle, igx, torch, G):
    """The shipped gadget: one key for every I/O (no per-disk / per-flag constants)."""
    H = igx.columns
    n = 1_500_000
    q = oracle.lognormal_quantiles(np.log(2e5), 1.5)
    ev_h = oracle.gen_bio(0xC3, q, 0, n)
    ev_h["delta"].view(np.int64)[::101] = -5          # negative deltas are skipped
    tr = G.ProfileBlockIOTracer()
    d = H.to_device(ev_h["delta"]).view(torch.int64)
    tr.feed(d[: n // 3])
    tr.feed(d[n // 3:])
    ref = oracle.hist_log2(None, None, ev_h["delta"], [], 1)
    assert np.array_equal(tr.slots(), ref)
    rep = tr.getReport()
    assert [x.count for x in rep.Data] == [x["count"] for x in oracle.get_report(ref[0])]
    assert tr.Stop() == rep.to_json()


def test_hist_u16_counter_carry(oracle, igx, torch):
    """Every event in one bin: each workgroup's 16-bit LDS counter crosses 0x8000 several
    times and moves it to HBM; the total must be exact."""
    E, H = igx.engine, igx.columns
    n = 40_000_000
    delta = torch.full((n,), 5000, dtype=torch.int64, device="cuda")
    h = H.host(E.hist_log2(None, None, delta, [], 1))
    assert int(h[0, 2]) == n and int(h.sum()) == n
    dev = torch.full((n,), 7, dtype=torch.uint32, device="cuda")
    cont = (torch.arange(n, device="cuda") % 3).to(torch.int32).view(torch.uint32)
    h2 = H.host(E.hist_log2(dev, cont, delta, [5, 7], 3))
    assert h2.shape == (6, 27) and h2[:3].sum() == 0
    assert [int(h2[3 + c, 2]) for c in range(3)] == [(n + 2 - c) // 3 for c in range(3)]


def test_parser_pipeline_c1(oracle, igx, torch):
    """parser.eventHandlerArray: MatchAll compaction -> sortSpec.Sort -> callback."""
    import importlib
    P = importlib.import_module("inspektor-gadget_amd.parser")
    E, H = igx.engine, igx.columns
    n = 200_000
    ccdf = H.to_device(oracle.zipf_cdf(64, 1.0))
    ev = E.gen_open(0xC1, ccdf, 0, n)
    cols = H.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"), ("comm", "string", 16),
                      ("ret", "int64"), ("fd", "int64"), ("err", "int64"), ("path", "uint32")])
    batch = H.EventBatch(cols, ev)
    p = P.NewParser(cols)
    p.SetFilters(["err:0", "pid:>=1000"])
    p.SetSorting(["comm", "-pid"])
    got = []
    p.SetEventCallback(got.append)
    p.EventHandlerFuncArray()(batch)
    out = got[0]
    ev_h = {k: H.host(v) for k, v in ev.items()}
    sel = np.nonzero((ev_h["err"] == 0) & (ev_h["pid"] >= 1000))[0]
    perm = oracle.go_sort_entries([(ev_h["comm"][sel], "string", False), (ev_h["pid"][sel], "uint32", True)], len(sel))
    assert out.n == len(sel)
    assert np.array_equal(H.host(out["pid"]), ev_h["pid"][sel][perm])
    assert np.array_equal(H.host(out["comm"]), ev_h["comm"][sel][perm])
    # per-event handler: filtered, original order
    got1 = []
    p.SetEventCallback(got1.append, array=False)
    p.EventHandlerFunc()(batch)
    assert np.array_equal(H.host(got1[0]["pid"]), ev_h["pid"][sel])
    # combiner: two sources, flushed in arrival order
    p.EnableCombiner()
    h = p.BatchHandlerFuncArray("node1")
    h(batch)
    h(batch)
    got.clear()
    p.Flush()
    assert got[0].n == 2 * len(sel)


def _open_samples(n, seed=21):
    """Raw opensnoop perf samples: random garbage after each C string's NUL, names with no
    NUL at all (255 bytes), comm with no NUL (16 bytes), negative rets, random padding."""
    rng = np.random.default_rng(seed)
    s = rng.integers(0, 256, (n, 304), dtype=np.uint8)
    s[:, 8:12] = rng.integers(0, 40000, n).astype(np.uint32).view(np.uint8).reshape(n, 4)
    s[:, 24:28] = np.where(rng.random(n) < 0.1, rng.integers(-13, 0, n), rng.integers(3, 1024, n)).astype(
        np.int32).view(np.uint8).reshape(n, 4)
    names = [b"bash", b"sshd", b"containerd", b"kubelet", b"node_exporter", b"x" * 16]
    for i in range(n):
        nm = names[i % len(names)]
        s[i, 32:32 + len(nm)] = np.frombuffer(nm, np.uint8)
        if len(nm) < 16:
            s[i, 32 + len(nm)] = 0
        k = int(rng.integers(0, 256))
        if k < 255:
            s[i, 48 + k] = 0          # else: no NUL in the 255 name bytes
        s[i, 48:48 + min(k, 3)] = np.frombuffer(b"/et"[:min(k, 3)], np.uint8)
    return s


def test_trace_open_samples_decode(oracle, igx, torch):
    """igx_ingest_open_events == tracer.go:182-208 over raw struct event samples."""
    H = igx.columns
    n = 20_001
    s = _open_samples(n)
    boot = 1_700_000_000_123_456_789
    got = igx.engine.ingest_open_events(H.to_device(s), boot_to_wall_ns=boot)
    want = oracle.decode_open_events(s, boot)
    for k, v in want.items():
        g = H.host(got[k])
        assert np.array_equal(g.view(v.dtype) if g.dtype != v.dtype else g, v), k
    # a stride larger than the struct (samples with trailing bytes)
    s2 = np.concatenate([s[:777], np.zeros((777, 16), np.uint8)], axis=1)
    got2 = igx.engine.ingest_open_events(H.to_device(s2), sample_bytes=320)
    assert np.array_equal(H.host(got2["path"]), want["path"][:777])


def test_trace_open_pipeline_from_samples(oracle, igx, torch):
    """C1 from the wire: perf samples -> Event columns -> filters ["err:0","pid:>=1000"] ->
    sort ["comm","-pid"] (parser.go:199-224), against the oracle's decode + Go sort."""
    import importlib
    P = importlib.import_module("inspektor-gadget_amd.parser")
    H = igx.columns
    n = 30_000
    s = _open_samples(n, seed=5)
    batch = igx.wire.trace_open_batch(H.to_device(s))
    p = P.NewParser(batch.cols)
    p.SetFilters(["err:0", "pid:>=1000", "path:~^/et"])
    p.SetSorting(["comm", "-pid"])
    got = []
    p.SetEventCallback(got.append)
    p.EventHandlerFuncArray()(batch)
    ev = oracle.decode_open_events(s)
    sel = np.nonzero((ev["err"] == 0) & (ev["pid"] >= 1000) &
                     (ev["path"][:, 0] == ord("/")) & (ev["path"][:, 1] == ord("e")) & (ev["path"][:, 2] == ord("t")))[0]
    perm = oracle.go_sort_entries([(ev["comm"][sel], "string", False), (ev["pid"][sel], "uint32", True)], len(sel))
    out = got[0]
    assert out.n == len(sel) > 0
    assert np.array_equal(H.host(out["pid"]), ev["pid"][sel][perm])
    assert np.array_equal(H.host(out["path"]), ev["path"][sel][perm])


def test_streaming_intervals_double_buffered(oracle, igx, torch, G):
    """StreamingTopTracer (tracer.go:228-265 over two device tables on two HIP streams):
    each interval's Event equals a one-shot tracer over that interval's events; global
    event indices continue across intervals; Iterations stops the loop."""
    H = igx.columns
    Gk = 4000
    cdf = oracle.zipf_cdf(Gk, 1.1)
    intervals, bases = [], []
    base = 0
    for k in range(4):
        n1, n2 = 60_000 + 1000 * k, 40_000
        e1 = _dev(H, oracle.gen_tcp(0xC2, k, Gk, cdf, base, n1))
        e2 = _dev(H, oracle.gen_tcp(0xC2, k, Gk, cdf, base + n1, n2))
        intervals.append([e1, e2])
        bases.append(base)
        base += n1 + n2
    st = G.StreamingTopTracer(G.TopTcpTracer, MaxRows=25, SortBy=["-sent", "-recv"], capacity=2 * Gk)
    got = list(st.run(intervals))
    st.destroy()
    assert len(got) == 4
    for k, ev in enumerate(got):
        one = G.TopTcpTracer(MaxRows=25, SortBy=["-sent", "-recv"], capacity=2 * Gk)
        for b in intervals[k]:
            one.feed(b)
        want = one.NextEvent()
        one.destroy()
        assert len(ev.Stats) == len(want.Stats) == 25
        for a, b in zip(ev.Stats, want.Stats):
            assert a.FirstIndex == b.FirstIndex + bases[k]
            a.FirstIndex = b.FirstIndex
            assert a == b
    st2 = G.StreamingTopTracer(G.TopTcpTracer, Iterations=2, MaxRows=5, capacity=2 * Gk)
    assert len(list(st2.run(intervals))) == 2
    st2.destroy()


def test_profile_block_io_raw_keys(oracle, igx, torch):
    """targ_per_disk / targ_per_flag (biolatency.bpf.c:116-131): one histogram per raw
    hist_key{cmd_flags, dev} (any values, including 0 and 0xffffffff), counts equal to the
    oracle's per-key log2 histograms; negative deltas skipped (:113-114); two feeds accumulate;
    keys in first-event order."""
    E, H, G = igx.engine, igx.columns, igx.gadgets
    rng = np.random.default_rng(5)
    n = 400_000
    q = E.lognormal_quantiles(np.log(2e5), 1.5)
    ev = E.gen_bio(0xC3, H.to_device(q), 0, 2 * n)
    delta = H.host(ev["delta"].view(torch.int64)).copy()
    delta[rng.integers(0, 2 * n, 1000)] = -5
    flags_pool = np.array([0, 1, 0x801, 0x4001, 0xFFFFFFFF], np.uint32)
    devs_pool = np.array([(8 << 20) | 0, (8 << 20) | 16, (259 << 20) | 1, 0], np.uint32)
    cf = flags_pool[rng.integers(0, len(flags_pool), 2 * n)]
    dv = devs_pool[rng.integers(0, len(devs_pool), 2 * n)]
    for per_disk, per_flag in ((True, False), (False, True), (True, True)):
        tr = G.ProfileBlockIOTracer(per_disk=per_disk, per_flag=per_flag)
        for b in range(2):
            sl = slice(b * n, (b + 1) * n)
            tr.feed(H.to_device(delta[sl]), dev=H.to_device(dv[sl]), cmd_flags=H.to_device(cf[sl]))
        kf = cf if per_flag else np.zeros(2 * n, np.uint32)
        kd = dv if per_disk else np.zeros(2 * n, np.uint32)
        order = []   # keys by their first kept event (a negative delta never creates a key)
        for a, b, d in zip(kf.tolist(), kd.tolist(), delta.tolist()):
            if d >= 0 and (a, b) not in order:
                order.append((a, b))
        got_keys = tr.keys()
        assert got_keys == order
        for key, h in zip(got_keys, tr.slots()):
            m = (kf == key[0]) & (kd == key[1])
            ref = oracle.hist_log2(None, None, delta[m], [], 1)[0]
            assert np.array_equal(h, ref), key
