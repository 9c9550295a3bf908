"""group.GroupEntries on the device (group.go:51-165) against group_test.go's expected
results and against the oracle restatement on random batches, including float group:sum
columns whose sum depends on the input order (float32 rounds after every add)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCHEMA = [("name", "string", 16), ("int", "int64", "group:sum"), ("uint", "uint64", "group:sum"),
          ("float", "float64", "group:sum"), ("secondary", "int64"), ("embeddedint", "int64", "group:sum"),
          ("embeddedfloat", "float64", "group:sum")]


def _batch(igx, entries):
    H = igx.columns
    n = len(entries)
    cols = H.Columns(SCHEMA)
    data = {}
    for name, kind, *rest in SCHEMA:
        if kind == "string":
            a = np.zeros((n, 16), np.uint8)
            for i, e in enumerate(entries):
                if e is not None:
                    b = e[name].encode()
                    a[i, :len(b)] = np.frombuffer(b, np.uint8)
        else:
            a = np.zeros(n, {"int64": np.int64, "uint64": np.uint64, "float64": np.float64}[kind])
            for i, e in enumerate(entries):
                if e is not None:
                    a[i] = e[name]
        data[name] = H.to_device(a)
    valid = H.to_device(np.array([e is not None for e in entries], np.uint8))
    return cols, H.EventBatch(cols, data, valid=valid)


def _rows(igx, out):
    H = igx.columns
    res = []
    for i in range(out.n):
        r = {}
        for name, kind, *rest in SCHEMA:
            v = H.host(out[name])[i]
            r[name] = bytes(v).rstrip(b"\0").decode() if kind == "string" else (
                float(v) if kind == "float64" else int(v))
        res.append(r)
    return res


def _e(name, v, sec):
    return {"name": name, "int": v, "uint": v, "float": float(v), "secondary": sec,
            "embeddedint": v, "embeddedfloat": float(v)}


def test_group_test_go_expectations(igx):
    """group_test.go:24-171."""
    G = igx.group
    entries = [_e("a", 1, 1), _e("a", 1, 2), _e("b", 2, 2), _e("b", 2, 3), None]
    cols, batch = _batch(igx, entries)
    assert _rows(igx, G.GroupEntries(cols, batch, [""])) == [_e("a", 6, 1)]
    assert _rows(igx, G.GroupEntries(cols, batch, ["name"])) == [_e("a", 2, 1), _e("b", 4, 2)]
    assert _rows(igx, G.GroupEntries(cols, batch, ["secondary", "name"])) == [_e("a", 4, 1), _e("b", 2, 3)]
    with pytest.raises(G.GroupError):
        G.GroupEntries(cols, batch, ["foobar"])
    assert G.GroupEntries(cols, None, ["name"]) is None


@pytest.mark.parametrize("f32", [False, True])
def test_float_sums_keep_input_order(oracle, igx, f32):
    """Random values spanning 40 binary orders of magnitude: any other addition order would
    change the low bits of most sums."""
    H = igx.columns
    rng = np.random.default_rng(8 + f32)
    n, ng = 20_000, 300
    fk = "float32" if f32 else "float64"
    schema = [("name", "string", 16), ("cnt", "uint32", "group:sum"), ("x", fk, "group:sum"),
              ("y", fk, "group:sum")]
    names = np.array([f"g{int(k)}".encode() for k in rng.integers(0, ng, n)])
    keys = np.zeros((n, 16), np.uint8)
    for i, b in enumerate(names):
        keys[i, :len(b)] = np.frombuffer(b, np.uint8)
    dt = np.float32 if f32 else np.float64
    x = (rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))).astype(dt)
    y = rng.random(n).astype(dt)
    cnt = np.ones(n, np.uint32)
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    cols = H.Columns(schema)
    batch = H.EventBatch(cols, {"name": H.to_device(keys), "cnt": H.to_device(cnt), "x": H.to_device(x),
                                "y": H.to_device(y)}, valid=H.to_device(valid))
    ocols = {"name": oracle.OCol("name", "string", 16), "cnt": oracle.OCol("cnt", "uint32"),
             "x": oracle.OCol("x", fk), "y": oracle.OCol("y", fk)}
    sums = {"cnt": "uint32", "x": fk, "y": fk}
    ents = [None if not valid[i] else {"name": names[i].decode(), "cnt": 1, "x": float(x[i]), "y": float(y[i])}
            for i in range(n)]
    for group_by in (["name"], [""]):
        want, err = oracle.group_entries(ocols, ents, group_by, sums)
        assert err is None
        out = igx.group.GroupEntries(cols, batch, group_by)
        assert out.n == len(want)
        gx, gy, gc = H.host(out["x"]), H.host(out["y"]), H.host(out["cnt"])
        gn = [bytes(r).rstrip(b"\0").decode() for r in H.host(out["name"])]
        for i, w in enumerate(want):
            assert gn[i] == w["name"] and int(gc[i]) == w["cnt"]
            assert float(gx[i]) == w["x"] and float(gy[i]) == w["y"], (group_by, i)
