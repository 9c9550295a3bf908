"""Pin the CPU oracle against the reference's own table tests and golden vectors.

Sources (relative to the reference repo root):
  pkg/columns/filter/filter_test.go:23-298  (table re-encoded in golden/filter_table.json)
  pkg/columns/filter/examples_test.go:24-89 (// Output: goldens)
  pkg/columns/group/group_test.go:24-171    (expected structs, re-encoded below)
  pkg/columns/sort/sort_test.go:59-231      (first-element checks, CanSortBy tables)
  SURVEY.md §8c log2 known answers (bits.bpf.h:8-29)
"""
import json
import os
import random

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _filter_fixture(O):
    d = json.load(open(os.path.join(GOLDEN, "filter_table.json")))
    cols = {}
    batch = {}
    recs = d["records"]
    n = len(recs)
    valid = np.array([r is not None for r in recs], dtype=bool)
    for name, kind in d["columns"]:
        cls, w = O.KIND_CLASS[kind]
        width = 16 if cls == "string" else w
        cols[name] = O.OCol(name, kind, width)
        if cls == "string":
            a = np.zeros((n, 16), np.uint8)
            for i, r in enumerate(recs):
                if r is not None and name == "string":
                    b = r["string"].encode()
                    a[i, : len(b)] = np.frombuffer(b, np.uint8)
        elif cls in ("int", "uint", "float"):
            dt = {"int": {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64},
                  "uint": {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64},
                  "float": {4: np.float32, 8: np.float64}}[cls][w]
            a = np.zeros(n, dt)
            for i, r in enumerate(recs):
                if r is not None and name != "time":
                    a[i] = r["v"]
        else:
            a = np.zeros(n, np.uint8)
        batch[name] = a
    return d, cols, batch, valid


def test_filter_table(oracle):
    O = oracle
    d, cols, batch, valid = _filter_fixture(O)
    assert len(d["rows"]) == 111
    for row in d["rows"]:
        try:
            p = O.parse_filter(cols, row["filter"])
            got = len(O.match_rows([p], batch, valid))
            err = False
        except O.FilterError:
            got, err = 0, True
        assert err == row["error"], row
        assert got == row["count"], row


def test_filter_multi_and_nil(oracle):
    O = oracle
    d, cols, batch, valid = _filter_fixture(O)
    preds = [O.parse_filter(cols, f) for f in d["multi"]["filters"]]
    sel = O.match_rows(preds, batch, valid)
    assert len(sel) == 1 and batch["int"][sel[0]] == 1
    # Match(nil) returns negate (filter.go:287-289): non-negated -> False
    p = O.parse_filter(cols, "int8:1")
    assert p.negate is False


def test_filter_entries_and_match_nil_semantics(oracle):
    """FilterEntries (filter.go:294-325): nil input -> nil (filter_test.go:257-262), no
    filters -> nil (outEntries is only assigned in the loop), table counts through the
    reference's own route; MatchAll / MatchAny over a batch with a nil entry: the nil entry
    is kept iff Match(nil) == negate holds for all / any specs (:266-291)."""
    O = oracle
    d, cols, batch, valid = _filter_fixture(O)
    nil = int(np.nonzero(~valid)[0][0])
    assert O.filter_entries(cols, None, None, [""]) is None
    assert O.filter_entries(cols, batch, valid, []) is None
    for row in d["rows"]:
        if row["error"]:
            continue
        out = O.filter_entries(cols, batch, valid, [row["filter"]])
        assert len(out) == row["count"] and nil not in out.tolist(), row
        p = O.parse_filter(cols, row["filter"])
        ma = O.match_all([p], batch, valid).tolist()
        assert len(ma) == row["count"] + (1 if p.negate else 0), row
        assert (nil in ma) == p.negate
    # chained: the multi-filter case of filter_test.go:287-298
    out = O.filter_entries(cols, batch, valid, d["multi"]["filters"])
    assert len(out) == 1 and batch["int"][out[0]] == 1
    neg = [O.parse_filter(cols, f) for f in ("int:!1", "int8:!2")]
    pos = O.parse_filter(cols, "int:1")
    assert nil in O.match_all(neg, batch, valid).tolist()
    assert nil not in O.match_all(neg + [pos], batch, valid).tolist()
    assert nil in O.match_all([], batch, valid).tolist()
    assert len(O.match_all([], batch, valid)) == len(valid)
    assert nil in O.match_any([pos, neg[0]], batch, valid).tolist()
    assert nil not in O.match_any([pos], batch, valid).tolist()
    assert len(O.match_any([], batch, valid)) == 0


def test_filter_examples(oracle):
    """examples_test.go:24-89."""
    O = oracle
    names = ["Alice", "Bob", "Eve"]
    ages = np.array([32, 26, 99], np.int64)
    dept = ["Security", "Security", "Security also"]
    def fixed(vals):
        a = np.zeros((3, 16), np.uint8)
        for i, v in enumerate(vals):
            a[i, : len(v)] = np.frombuffer(v.encode(), np.uint8)
        return a
    cols = {"name": O.OCol("name", "string", 16), "age": O.OCol("age", "int", 8),
            "department": O.OCol("department", "string", 16)}
    batch = {"name": fixed(names), "age": ages, "department": fixed(dept)}
    sel = O.match_rows([O.parse_filter(cols, "age:<50"), O.parse_filter(cols, "name:~(?i)e")],
                       batch)
    assert [names[i] for i in sel] == ["Alice"]
    sel = O.match_rows([O.parse_filter(cols, "department:Security")], batch)
    assert [names[i] for i in sel] == ["Alice", "Bob"]


def test_convert_truncation(oracle):
    """getValueFromFilterSpec Convert() wraps to the column width (filter.go:60-74)."""
    O = oracle
    cols = {"x": O.OCol("x", "int8", 1), "u": O.OCol("u", "uint8", 1)}
    assert O.parse_filter(cols, "x:300").ref == bytes([300 & 0xFF])
    assert O.parse_filter(cols, "x:-1").ref == b"\xff"
    assert O.parse_filter(cols, "u:257").ref == b"\x01"
    with pytest.raises(O.FilterError):
        O.parse_filter(cols, "u:-1")


def test_group_entries_golden(oracle):
    """group_test.go:24-171 expected results."""
    O = oracle
    cols = {c: O.OCol(c, k) for c, k in [("name", "string"), ("int", "int64"),
                                          ("uint", "uint64"), ("float", "float64"),
                                          ("secondary", "int"), ("embeddedint", "int64"),
                                          ("embeddedfloat", "float64")]}
    cols["name"].width = 16
    sums = {"int": "int64", "uint": "uint64", "float": "float64", "embeddedint": "int64",
            "embeddedfloat": "float64"}
    def e(name, v, sec):
        return {"name": name, "int": v, "uint": v, "float": float(v), "secondary": sec,
                "embeddedint": v, "embeddedfloat": float(v)}
    entries = [e("a", 1, 1), e("a", 1, 2), e("b", 2, 2), e("b", 2, 3), None]
    res, err = O.group_entries(cols, entries, [""], sums)
    assert err is None and res == [dict(e("a", 6, 1))]
    res, err = O.group_entries(cols, entries, ["name"], sums)
    assert res == [e("a", 2, 1), e("b", 4, 2)]
    res, err = O.group_entries(cols, entries, ["secondary", "name"], sums)
    assert res == [e("a", 4, 1), e("b", 2, 3)]
    res, err = O.group_entries(cols, entries, ["foobar"], sums)
    assert res is None and err is not None
    res, err = O.group_entries(cols, None, ["name"], sums)
    assert res is None and err is None


def test_sort_first_elements(oracle):
    """sort_test.go:59-174: shuffle then SortEntries; only entries[0] is checked there."""
    O = oracle
    recs = [None, dict(int=1, uint=2, string="c", f32=3.0, f64=4.0, group="b", emb=7, ext=1),
            None, dict(int=2, uint=3, string="d", f32=4.0, f64=5.0, group="b", emb=6, ext=2),
            None, dict(int=3, uint=4, string="e", f32=5.0, f64=1.0, group="a", emb=5, ext=3),
            None, dict(int=4, uint=5, string="a", f32=1.0, f64=2.0, group="a", emb=4, ext=4),
            None, dict(int=5, uint=1, string="b", f32=2.0, f64=3.0, group="c", emb=3, ext=5),
            None]
    rng = random.Random(0)
    cases = [(["uint"], "uint", 1), (["-uint"], "uint", 5), (["int"], "int", 1),
             (["-int"], "int", 5), (["float32"], "f32", 1), (["-float32"], "f32", 5),
             (["float64"], "f64", 1), (["-float64"], "f64", 5), (["embeddedInt"], "emb", 3),
             (["-extractor"], "ext", 5), (["string"], "string", "a")]
    names = {"uint": "uint", "int": "int", "float32": "f32", "float64": "f64",
             "embeddedint": "emb", "extractor": "ext", "string": "string", "group": "group"}
    for sort_by, field, want in cases:
        rng.shuffle(recs)
        keys = []
        for s in sort_by:
            desc = s.startswith("-")
            nm = names[s.lstrip("-").lower()]
            keys.append((lambda r, nm=nm: r[nm], desc))
        out = O.go_sort_entries_py(recs, keys)
        assert out[0][field] == want
        assert all(r is None for r in out[5:])          # nil entries sort last
    rng.shuffle(recs)
    out = O.go_sort_entries_py(recs, [(lambda r: r["group"], False), (lambda r: r["string"], False)])
    assert out[0]["group"] == "a" and out[0]["string"] == "a"


@pytest.mark.parametrize("trial", range(6))
def test_closed_form_matches_go_stable(oracle, trial):
    """closed form == Go 1.19 SliceStable restatement (py and C)."""
    O = oracle
    rng = random.Random(1000 + trial)
    for _ in range(60):
        n = rng.randint(0, 260)
        nk = rng.randint(1, 4)
        vals = [[rng.randint(0, 3) for _ in range(n)] for _ in range(nk)]
        descs = [rng.random() < 0.6 for _ in range(nk)]
        rows = list(range(n))
        py = O.go_sort_entries_py(rows, [(lambda r, v=v: v[r], d) for v, d in zip(vals, descs)])
        cf = O.closed_form_perm(vals, descs, n)
        assert py == cf
        cperm = O.go_sort_entries([(np.array(v, np.int64), "int64", d) for v, d in
                                   zip(vals, descs)], n)
        assert list(cperm) == cf


def test_log2_known_answers(oracle):
    """SURVEY.md §8c; log2l (bits.bpf.h:22-29) before the MAX_SLOTS clamp."""
    O = oracle
    want = {0: 0, 1: 0, 2: 1, 3: 1, 1023: 9, 1024: 10, 2 ** 26: 26, 2 ** 40: 40,
            2 ** 64 - 1: 63}
    for v, s in want.items():
        assert O.log2l(v) == s
    # with the clamp as applied in biolatency.bpf.c:146-148
    h = O.hist_log2(np.array([1, 1, 1, 1], np.uint32), np.zeros(4, np.uint32),
                    np.array([0, 999, 1024 * 1000, (2 ** 40) * 1000], np.int64),
                    np.array([1], np.uint32), 1)
    assert h[0, 0] == 2 and h[0, 10] == 1 and h[0, 26] == 1


def test_get_report_quirk(oracle):
    """getReport drops the last non-zero slot (tracer.go:87)."""
    O = oracle
    slots = [0] * 27
    slots[3] = 5
    slots[7] = 2
    rep = O.get_report(slots)
    assert len(rep) == 7 and rep[3]["count"] == 5 and rep[3]["intervalStart"] == 8
    assert O.get_report([4] + [0] * 26) == []


@pytest.mark.parametrize("trial", range(3))
def test_go_stable_with_nan_c_matches_py(oracle, trial):
    """NaN float keys (getLessFunc's `<` unordered, sort.go:125-135): the order is whatever
    Go 1.19's SliceStable does; the C restatement (the GPU NaN path's checker) equals the
    pure-Python transliteration of stable_func on random inputs with NaNs, nil rows, several
    keys and both directions (n up to 300: insertion blocks and several merge levels)."""
    O = oracle
    rng = random.Random(77 + trial)
    for _ in range(40):
        n = rng.randint(0, 300)
        nk = rng.randint(1, 3)
        vals = [[rng.choice([float("nan"), -1.0, 0.0, 2.5, 3.0, float("inf")]) for _ in range(n)] for _ in range(nk)]
        descs = [rng.random() < 0.5 for _ in range(nk)]
        valid = [rng.random() > 0.1 for _ in range(n)]
        rows = [r if valid[r] else None for r in range(n)]
        py = O.go_sort_entries_py(rows, [(lambda r, v=v: v[r], d) for v, d in zip(vals, descs)])
        py = [r if r is not None else None for r in py]
        cperm = O.go_sort_entries([(np.array(v, np.float64), "float64", d) for v, d in zip(vals, descs)], n,
                                  valid=np.array(valid, np.uint8))
        # nil rows come back as None from the py version, in order of their row ids
        nil_rows = iter([r for r in cperm if not valid[r]])
        assert [r if r is not None else next(nil_rows) for r in py] == list(cperm)


# Hand-derived Go 1.19 SliceStable orders with NaN keys (the NaN path was pinned
# only C-vs-Python).  n < 20, so SliceStable is one insertionSort pass per key
# (sort/zsortfunc.go insertionSort_func); less = !(a < b) != asc (sort.go:125-135), i.e.
# a < b for ASC and !(a < b) for DESC, which is true whenever a NaN is involved.  Each
# expectation below was stepped through by hand; nil rows sort last (less(nil, x) = false,
# less(x, nil) = true).  Entries: (keys in sortBy order as (values, desc), valid, expected).
NAN = float("nan")
NAN_VECTORS = [
    ([([3.0, NAN, 1.0, 2.0], False)], None, [0, 1, 2, 3]),     # no adjacent pair is `<`-ordered
    ([([NAN, 2.0, 1.0], False)], None, [0, 2, 1]),
    ([([2.0, 1.0, NAN, 0.0], False)], None, [1, 0, 2, 3]),      # the NaN walls 0.0 off
    ([([1.0, NAN, 2.0], True)], None, [2, 1, 0]),
    ([([NAN, NAN, 5.0], True)], None, [2, 1, 0]),
    ([([0.0, NAN, 0.0, 1.0], True)], None, [3, 2, 1, 0]),       # DESC swaps every tie and NaN
    ([([NAN, 7.0, 1.0], False)], [1, 0, 1], [0, 2, 1]),         # nil row 1 sinks, NaN stays first
    # two keys: the last key's pass runs first ([2, 1, 0]), then k0's pass meets [1, NaN, 0]
    # and moves nothing: row 0 (k0 = 0) stays behind row 2 (k0 = 1)
    ([([0.0, NAN, 1.0], False), ([2.0, 1.0, 0.0], False)], None, [2, 1, 0]),
]


@pytest.mark.parametrize("case", range(len(NAN_VECTORS)))
def test_go_stable_nan_hand_derived(oracle, case):
    O = oracle
    keys, valid, want = NAN_VECTORS[case]
    n = len(want)
    v8 = None if valid is None else np.array(valid, np.uint8)
    got = O.go_sort_entries([(np.array(v, np.float64), "float64", d) for v, d in keys], n, valid=v8)
    assert list(got) == want
    got32 = O.go_sort_entries([(np.array(v, np.float32), "float32", d) for v, d in keys], n, valid=v8)
    assert list(got32) == want
    rows = [r if valid is None or valid[r] else None for r in range(n)]
    py = O.go_sort_entries_py(rows, [(lambda r, v=v: v[r], d) for v, d in keys])
    nil_rows = iter([r for r in want if valid is not None and not valid[r]])
    assert [r if r is not None else next(nil_rows) for r in py] == want
