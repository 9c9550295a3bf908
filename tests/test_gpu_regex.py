"""`~` filters on the device (filter.go:119-127,212-216): igx_filter with a regex rule on
a string column, against the compiled automaton stepped on the host (tests/test_regex_host.py
pins that automaton to regular-expression search) and, for ASCII data, Python's `re`."""
import importlib
import re

import numpy as np
import pytest

from test_regex_host import compile_blob, run_blob

pytestmark = pytest.mark.gpu


def _strings(n, seed=4):
    rng = np.random.default_rng(seed)
    words = [b"kworker/0:1", b"bash", b"sshd", b"containerd", b"Demo 123", b"demo", b"K8s-agent",
             "café".encode(), b"\xff\xfebad", b"node_exporter", b"", b"x" * 16, b"a\nb",
             "αβγ-api".encode(), "日本語ok".encode(), "µs".encode()]
    out = np.zeros((n, 16), np.uint8)
    pick = rng.integers(0, len(words), n)
    for i, k in enumerate(pick):
        w = words[k][:16]
        out[i, :len(w)] = np.frombuffer(w, np.uint8)
    return out


@pytest.mark.parametrize("rule", ["~^k", "~(?i)demo", "!~(?i)demo", "~er$", "~[0-9]", "~^.{4}$",
                                  "~caf.", "~\\d+:\\d", "~^$", "~x{16}", "~(?s)a.b",
                                  # RE2 assertions, (?m), Unicode classes and folding
                                  "~\\bdemo\\b", "~\\Bsh", "~(?m)^b$", "~(?i)CAFÉ", "~\\p{Ll}{4}$",
                                  "!~[[:upper:]]", "~\\pL\\PL",
                                  # Unicode 13.0.0 scripts (and FoldScript under (?i))
                                  "~^\\p{Greek}", "~\\p{Han}{2}", "!~\\p{Latin}", "~(?i)^\\p{Greek}s$"])
def test_regex_filter_on_device(oracle, igx, rule):
    H = igx.columns
    n = 100_003
    s = _strings(n)
    cols = H.Columns([("comm", "string", 16), ("pid", "uint32")])
    batch = H.EventBatch(cols, {"comm": H.to_device(s), "pid": H.to_device(np.arange(n, dtype=np.uint32))})
    got = H.host(igx.filter.GetFiltersFromStrings(cols, ["comm:" + rule]).MatchAll(batch)).astype(np.int64)
    neg = rule.startswith("!")
    pat = rule.lstrip("!")[1:]
    blob = compile_blob(igx, pat.encode())[1]
    uniq = {}
    want = []
    for i in range(n):
        t = s[i].tobytes()
        if t not in uniq:
            uniq[t] = run_blob(blob, t) != neg
        if uniq[t]:
            want.append(i)
    assert np.array_equal(got, np.array(want, np.int64))


def test_filter_entries_regex_and_range(oracle, igx):
    """FilterEntries applies the filters one after another (filter.go:294-325)."""
    H = igx.columns
    n = 50_000
    s = _strings(n, 9)
    pid = np.arange(n, dtype=np.uint32)
    cols = H.Columns([("comm", "string", 16), ("pid", "uint32")])
    batch = H.EventBatch(cols, {"comm": H.to_device(s), "pid": H.to_device(pid)})
    out = igx.filter.FilterEntries(cols, batch, ["comm:~^(bash|sshd)$", "pid:>=1000"])
    keep = [i for i in range(n) if re.search(r"^(bash|sshd)\Z", s[i].tobytes().split(b"\0")[0].decode("latin-1"))
            and i >= 1000]
    assert np.array_equal(H.host(out["pid"]).astype(np.int64), np.array(keep, np.int64))
