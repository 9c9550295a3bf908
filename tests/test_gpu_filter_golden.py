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
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    assert len(d["rows"]) == 111
    ran = 0
    for row in d["rows"]:
        try:
            spec = F.GetFilterFromString(cols, row["filter"])
        except F.FilterError:
            assert row["error"], row
            continue
        assert not row["error"], row
        got = H.host(F.FilterSpecs([spec]).MatchAll(batch)) if hasattr(F, "FilterSpecs") else \
            H.host(F.GetFiltersFromStrings(cols, [row["filter"]]).MatchAll(batch))
        assert len(got) == row["count"], row
        ran += 1
    assert ran == sum(not r["error"] for r in d["rows"]) == 84


def test_filter_table_multi_on_device(igx):
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    sel = H.host(F.GetFiltersFromStrings(cols, d["multi"]["filters"]).MatchAll(batch))
    assert len(sel) == 1


def test_filter_entries_nil_rows_and_chaining(igx):
    """FilterEntries (filter.go:294-325) over the golden records + nil: no filters keeps the
    non-nil rows in order; each filter compacts the batch (igx_take) before the next one;
    more than 4 predicates in one MatchAll AND into one bitmask over several mark launches."""
    F, H = igx.filter, igx.columns
    d, cols, batch = _device_fixture(igx)
    recs = d["records"]
    live = [i for i, r in enumerate(recs) if r is not None]
    out = F.FilterEntries(cols, batch, [])
    assert out.n == len(live)
    assert np.array_equal(H.host(out.valid), np.ones(len(live), np.uint8))
    name = next(n for n, k in d["columns"] if k == "string")
    assert np.array_equal(H.host(out[name]), H.host(batch[name])[live])
    rows = [r for r in d["rows"] if not r["error"] and r["count"] > 0]
    # the same filter five times: 4 predicates per mark launch, the fifth ANDs into the mask
    f = rows[0]["filter"]
    sel = H.host(F.GetFiltersFromStrings(cols, [f] * 5).MatchAll(batch))
    assert len(sel) == rows[0]["count"]
    assert np.array_equal(sel, H.host(F.GetFiltersFromStrings(cols, [f]).MatchAll(batch)))
    chained = F.FilterEntries(cols, batch, [f, f])
    assert chained.n == rows[0]["count"]


def test_match_any_on_device(igx):
    """FilterSpecs.MatchAny (filter.go:276-283) through igx_filter_any and MatchAll
    (:266-273) through igx_filter: the union / intersection of the single-filter selections
    of the golden table, for 1, 4 and 9 specs (more than one predicate chunk), nil never
    matching; no specs select nothing."""
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
