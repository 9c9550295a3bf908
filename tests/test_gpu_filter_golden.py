"""The reference's filter table (pkg/columns/filter/filter_test.go:50-298, re-encoded in
tests/golden/filter_table.json) run through the device scan: every row's filter is parsed
by igx_filter_parse and evaluated by igx_filter (k_filter.hip) over the 5 records + nil held
as device columns; the selected count must equal the table's.  Regex rows take the device
DFA, float rows the IEEE compares, the int8:300 row the Convert truncation."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
NP = {"int": np.int64, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
      "uint": np.uint64, "uint8": np.uint8, "uint16": np.uint16, "uint32": np.uint32, "uint64": np.uint64,
      "float32": np.float32, "float64": np.float64}


def _device_fixture(igx):
    H = igx.columns
    d = json.load(open(os.path.join(GOLDEN, "filter_table.json")))
    recs = d["records"]
    n = len(recs)
    schema, data = [], {}
    for name, kind in d["columns"]:
        if kind == "string":
            schema.append((name, "string", 16))
            a = np.zeros((n, 16), np.uint8)
            for i, r in enumerate(recs):
                if r is not None:
                    b = r["string"].encode()
                    a[i, :len(b)] = np.frombuffer(b, np.uint8)
        elif kind in NP:
            schema.append((name, kind))
            a = np.zeros(n, NP[kind])
            for i, r in enumerate(recs):
                if r is not None and name != "time":
                    a[i] = r["v"]
        else:
            schema.append((name, kind))
            a = np.zeros(n, np.uint8)
        data[name] = H.to_device(a)
    valid = H.to_device(np.array([r is not None for r in recs], np.uint8))
    cols = H.Columns(schema)
    return d, cols, H.EventBatch(cols, data, valid=valid)


def test_filter_table_on_device(igx):
    """Every non-error row through the reference's own route, FilterEntries (filter.go:294-325,
    nil entry skipped), and through FilterSpecs.MatchAll, where the nil entry is kept iff the
    filter is negated (Match(nil) == negate, :286-291)."""
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    nil = [i for i, r in enumerate(d["records"]) if r is None][0]
    assert len(d["rows"]) == 111
    ran = 0
    for row in d["rows"]:
        try:
            spec = F.GetFilterFromString(cols, row["filter"])
        except F.FilterError:
            assert row["error"], row
            continue
        assert not row["error"], row
        out = F.FilterEntries(cols, batch, [row["filter"]])
        assert out.n == row["count"], row
        got = H.host(F.FilterSpecs([spec]).MatchAll(batch)).tolist()
        assert len(got) == row["count"] + (1 if spec.negate else 0), row
        assert (nil in got) == spec.negate, row
        ran += 1
    assert ran == sum(not r["error"] for r in d["rows"]) == 84


def test_filter_table_multi_on_device(igx):
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    sel = H.host(F.GetFiltersFromStrings(cols, d["multi"]["filters"]).MatchAll(batch))
    assert len(sel) == 1
    out = F.FilterEntries(cols, batch, d["multi"]["filters"])
    assert out.n == 1 and int(H.host(out["int"])[0]) == d["multi"]["int"]


def test_filter_entries_nil_rows_and_chaining(igx):
    """FilterEntries (filter.go:294-325) over the golden records + nil: nil input and no
    filters both return nil (outEntries is only assigned inside the filter loop); each
    filter compacts the batch (igx_take) before the next one; more than 4 predicates in one
    MatchAll AND into one bitmask over several mark launches."""
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    assert F.FilterEntries(cols, None, [""]) is None
    assert F.FilterEntries(cols, batch, []) is None
    rows = [r for r in d["rows"] if not r["error"] and r["count"] > 0 and "!" not in r["filter"]]
    # the same filter five times: 4 predicates per mark launch, the fifth ANDs into the mask
    f = rows[0]["filter"]
    sel = H.host(F.GetFiltersFromStrings(cols, [f] * 5).MatchAll(batch))
    assert len(sel) == rows[0]["count"]
    assert np.array_equal(sel, H.host(F.GetFiltersFromStrings(cols, [f]).MatchAll(batch)))
    chained = F.FilterEntries(cols, batch, [f, f])
    assert chained.n == rows[0]["count"]
    assert np.array_equal(H.host(chained.valid), np.ones(chained.n, np.uint8))


def test_match_any_on_device(igx):
    """FilterSpecs.MatchAny (filter.go:276-283) through igx_filter_any and MatchAll
    (:266-273) through igx_filter_ex: the union / intersection of the single-filter
    selections of the golden table, for 1, 4 and 9 specs (more than one predicate chunk);
    since a single negated spec keeps the nil entry, the nil entry is in the union iff some
    spec is negated and in the intersection iff all are; no specs select nothing (any) or
    everything (all)."""
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    good = [r["filter"] for r in d["rows"] if not r["error"]]
    rng = np.random.default_rng(3)
    for m in (1, 4, 9, 9, 9):
        pick = [good[i] for i in rng.choice(len(good), size=m, replace=False)]
        union = set()
        for f in pick:
            union |= set(H.host(F.GetFiltersFromStrings(cols, [f]).MatchAll(batch)).tolist())
        got = H.host(F.GetFiltersFromStrings(cols, pick).MatchAny(batch))
        assert got.tolist() == sorted(union), pick
        inter = set(range(len(d["records"])))
        for f in pick:
            inter &= set(H.host(F.GetFiltersFromStrings(cols, [f]).MatchAll(batch)).tolist())
        got = H.host(F.GetFiltersFromStrings(cols, pick).MatchAll(batch))
        assert got.tolist() == sorted(inter), pick
    assert F.FilterSpecs().MatchAny(batch).numel() == 0
    assert H.host(F.FilterSpecs().MatchAll(batch)).tolist() == list(range(len(d["records"])))


@pytest.mark.parametrize("filters", [["pid:!7", "comm:!bash"],           # all negated
                                     ["pid:!7", "pid:>=1000"],           # mixed
                                     ["comm:~^(bash|sshd)$"],            # none negated
                                     [],                                 # no filters
                                     ["pid:!1", "pid:!2", "pid:!3", "pid:!4", "uid:!0", "comm:!x"]])
def test_parser_array_handler_nil_rows(oracle, igx, torch, filters):
    """parser.eventHandlerArray (parser.go:199-224) over a batch holding nil entries: MatchAll
    keeps a nil entry iff every filter is negated (the Match(nil) == negate of filter.go:286-291);
    the kept rows then sort with nils last (sort.go:127-132).  Checked against the oracle's
    MatchAll and Go SliceStable restatement.  SetFilters([]) leaves filterSpecs nil, so every
    entry passes (parser.go:340-343)."""
    import importlib
    P = importlib.import_module("inspektor-gadget_amd.parser")
    H = igx.columns
    rng = np.random.default_rng(5)
    n = 50_000
    names = [b"bash", b"sshd", b"x", b"kubelet"]
    comm = np.zeros((n, 16), np.uint8)
    pick = rng.integers(0, len(names), n)
    for i, nm in enumerate(names):
        comm[pick == i, :len(nm)] = np.frombuffer(nm, np.uint8)
    pid = rng.integers(0, 2000, n).astype(np.uint32)
    uid = rng.integers(0, 3, n).astype(np.uint32)
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    cols = H.Columns([("pid", "uint32"), ("uid", "uint32"), ("comm", "string", 16)])
    batch = H.EventBatch(cols, {"pid": H.to_device(pid), "uid": H.to_device(uid), "comm": H.to_device(comm)},
                         valid=H.to_device(valid))
    p = P.NewParser(cols)
    p.SetFilters(filters)
    p.SetSorting(["-pid"])
    got = []
    p.SetEventCallback(got.append)
    p.EventHandlerFuncArray()(batch)
    out = got[0]
    ocols = {"pid": oracle.OCol("pid", "uint32", 4), "uid": oracle.OCol("uid", "uint32", 4),
             "comm": oracle.OCol("comm", "string", 16)}
    hb = {"pid": pid, "uid": uid, "comm": comm}
    if filters:
        sel = oracle.match_all([oracle.parse_filter(ocols, f) for f in filters], hb, valid)
    else:
        sel = np.arange(n, dtype=np.uint32)
    nil_kept = int((valid[sel] == 0).sum())
    assert nil_kept == (int((valid == 0).sum()) if all("!" in f for f in filters) else 0)
    perm = oracle.go_sort_entries([(pid[sel], "uint32", True)], len(sel), valid=valid[sel])
    assert out.n == len(sel)
    assert np.array_equal(H.host(out.valid), valid[sel][perm])
    live = valid[sel][perm] == 1
    assert np.array_equal(H.host(out["pid"])[live], pid[sel][perm][live])
    assert np.array_equal(H.host(out["comm"])[live], comm[sel][perm][live])
    # the per-event handler: MatchAll per event, original order, nils included the same way
    got1 = []
    p.SetEventCallback(got1.append, array=False)
    p.EventHandlerFunc()(batch)
    assert np.array_equal(H.host(got1[0].valid), valid[sel])
