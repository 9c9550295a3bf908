"""The output side against the reference's own tests:
pkg/columns/ellipsis/ellipsis_test.go (table re-encoded in golden/ellipsis_table.json) and
examples_test.go, pkg/columns/formatter/textcolumns/textcolumns_test.go (expected strings
below, each with its test name), plus the top gadgets' Stats rendering (column tags of
pkg/gadgets/top/*/types/types.go) and Go json.Marshal output.  Host only."""
import importlib
import json
import os
from dataclasses import dataclass

import pytest

T = importlib.import_module("inspektor-gadget_amd.textcolumns")
G = importlib.import_module("inspektor-gadget_amd.gadgets")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_ellipsis_table():
    d = json.load(open(os.path.join(GOLDEN, "ellipsis_table.json"), encoding="utf-8"))
    kinds = {"None": T.NONE, "End": T.END, "Start": T.START, "Middle": T.MIDDLE}
    assert len(d["rows"]) == 23
    for r in d["rows"]:
        assert T.ShortenString(r["input"], r["max"], kinds[r["type"]]) == r["result"], r


def test_ellipsis_example():
    """examples_test.go:24-33."""
    assert [T.ShortenString("Foobar123", 8, e) for e in (T.NONE, T.START, T.END, T.MIDDLE)] == \
        ["Foobar12", "…obar123", "Foobar1…", "Foob…123"]


@dataclass
class TS:                       # textcolumns_test.go:28-34 testStruct
    Name: str
    Age: int
    Size: float
    Balance: int
    CanDance: bool


FIELDS = [("Name", "string", "name,width:10"), ("Age", "uint", "age,width:4,align:right,fixed"),
          ("Size", "float32", "size,width:6,precision:2,align:right"), ("Balance", "int", "balance,width:8,align:right"),
          ("CanDance", "bool", "canDance,width:8")]
import numpy as np  # noqa: E402
ENTRIES = [TS("Alice", 32, float(np.float32(1.74)), 1000, True), TS("Bob", 26, float(np.float32(1.73)), -200, True),
           TS("Eve", 99, float(np.float32(5.12)), 1000000, False), None]


def cols():
    return T.ColumnMap(FIELDS)


def test_format_entry_and_table():
    """TestTextColumnsFormatter_FormatEntryAndTable."""
    expected = ["Alice        32   1.74     1000 true    ", "Bob          26   1.73     -200 true    ",
                "Eve          99   5.12  1000000 false   ", ""]
    f = T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH)
    assert [f.FormatEntry(e) for e in ENTRIES] == expected
    assert f.FormatTable(ENTRIES) == "\n".join(["NAME        AGE   SIZE  BALANCE CANDANCE",
                                                "————————————————————————————————————————"] + expected)


def test_format_header_and_divider():
    """TestTextColumnsFormatter_FormatHeader / _FormatRowDivider."""
    f = T.TextColumnsFormatter(cols())
    assert f.FormatHeader() == "NAME        AGE   SIZE  BALANCE CANDANCE"
    f.HeaderStyle = T.HEADER_LOWER
    assert f.FormatHeader() == "name        age   size  balance candance"
    f.HeaderStyle = T.HEADER_NORMAL
    assert f.FormatHeader() == "name        age   size  balance canDance"
    assert T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH).FormatRowDivider() == "—" * 40


def test_recalculate_widths():
    """TestTextColumnsFormatter_RecalculateWidths."""
    f = T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH)
    f.RecalculateWidths(100, True)
    assert len(f.FormatHeader()) == 100 and len(f.FormatRowDivider()) == 100
    for e in ENTRIES[:3]:
        assert len(f.FormatEntry(e)) == 100


def test_adjust_widths_to_content():
    """TestTextColumnsFormatter_AdjustWidthsToContent / ...NoHeaders / ...MaxWidth."""
    f = T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH)
    f.AdjustWidthsToContent(ENTRIES, True, 0, False)
    assert f.FormatHeader() == "NAME   AGE SIZE BALANCE CANDANCE"
    assert f.FormatRowDivider() == "—" * 32
    assert f.FormatEntry(ENTRIES[0]) == "Alice   32 1.74    1000 true    "
    f = T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH)
    f.AdjustWidthsToContent(ENTRIES, False, 0, False)
    assert f.FormatHeader() == "NAME   AGE SIZE BALANCE CAND…"
    assert f.FormatRowDivider() == "—" * 29
    assert f.FormatEntry(ENTRIES[0]) == "Alice   32 1.74    1000 true "
    f = T.TextColumnsFormatter(cols(), RowDivider=T.DIVIDER_DASH)
    f.AdjustWidthsToContent(ENTRIES, False, 9, True)
    assert f.FormatHeader() == "N… …  … …"
    assert f.FormatRowDivider() == "—" * 9
    assert f.FormatEntry(ENTRIES[0]) == "A… …  … …"


def test_width_restrictions():
    """TestWidthRestrictions."""
    @dataclass
    class W:
        Name: str
        SecondField: str
    cm = T.ColumnMap([("Name", "string", "name,width:5,minWidth:2,maxWidth:10"), ("SecondField", "string", "second")])
    f = T.TextColumnsFormatter(cm, RowDivider=T.DIVIDER_DASH, AutoScale=True)
    e = W("123456789012", "123456789012")
    f.RecalculateWidths(40, False)
    assert f.FormatEntry(e).strip() == "123456789… 123456789012"
    f.RecalculateWidths(1, False)
    assert f.FormatEntry(e).strip() == "1… …"


def test_set_shown_columns():
    """TestTextColumnsFormatter_SetShownColumns."""
    for shown, expected in [(None, ["name", "age", "size", "balance", "canDance"]), ([], []), (["name"], ["name"]),
                            (["name", "canDance"], ["name", "canDance"])]:
        f = T.TextColumnsFormatter(cols())
        f.SetShowColumns(shown)
        assert [c.col.Name for c in f.showColumns] == expected
    with pytest.raises(T.ColumnError):
        T.TextColumnsFormatter(cols()).SetShowColumns(["foo"])


def test_tag_errors_and_templates():
    """columninfo.go:119-245 rejections; templates re-apply the field's own settings."""
    for tag in ["x,align", "x,align:middle", "x,ellipsis:bogus", "x,fixed:1", "x,hide:1", "x,order",
                "x,width:abc", "x,template", "x,template:nope", "x,bogus", "x,width:4,minWidth:8",
                "x,width:8,maxWidth:4"]:
        with pytest.raises(T.ColumnError):
            T.ColumnMap([("X", "string", tag)])
    with pytest.raises(T.ColumnError):
        T.ColumnMap([("X", "int", "x,precision:2")])
    c = T.ColumnMap([("P", "int32", "pid,template:pid"), ("S", "uint16", "sport,template:ipport")]).cols
    assert (c["pid"].MinWidth, c["pid"].Width, c["pid"].MaxWidth) == (7, 16, 11)
    assert (c["sport"].MinWidth, c["sport"].Width) == (5, 16)
    assert T.ColumnMap([("N", "string", "node,template:node,width:12")]).cols["node"].Width == 12


def test_bytes_size():
    """go-units BytesSize ("%.4g%s", base 1024)."""
    assert [T.BytesSize(x) for x in (0, 100, 1023, 1024, 1536, 12345, 1048576, 5.5 * 2 ** 30)] == \
        ["0B", "100B", "1023B", "1KiB", "1.5KiB", "12.06KiB", "1MiB", "5.5GiB"]


def test_top_tcp_output():
    """top tcp Stats through the frontends' table (untagged columns: no CommonData) and JSON."""
    rows = [G.TcpStats(MountNsID=4026531840, Pid=1234, Comm="curl", Family=2, Saddr="10.0.0.1", Daddr="10.0.3.7",
                       Sport=40000, Dport=443, Sent=123456, Received=99),
            G.TcpStats(Pid=7, Comm="a-very-long-command-name", Family=10, Saddr="::1", Daddr="fe80::1", Sport=1, Dport=2,
                       Sent=0, Received=5 << 30)]
    out = G.render_table("tcp", rows)
    lines = out.split("\n")
    assert lines[0].split() == ["PID", "COMM", "IP", "LOCAL", "REMOTE", "SENT", "RECV"]
    assert lines[1].split() == ["1234", "curl", "4", "10.0.0.1:40000", "10.0.3.7:443", "120.6KiB", "99B"]
    # widths follow the content (AdjustWidthsToContent, no terminal): the long comm is whole
    assert lines[2].split()[:3] == ["7", "a-very-long-command-name", "6"]
    assert len({len(l) for l in lines}) == 1
    narrow = G.render_table("tcp", rows, terminal_width=60).split("\n")
    assert {len(l) for l in narrow} == {60}
    js = json.loads(G.render_json("tcp", rows))
    assert js[0] == {"mountnsid": 4026531840, "pid": 1234, "comm": "curl", "family": 2, "saddr": "10.0.0.1",
                     "daddr": "10.0.3.7", "sport": 40000, "dport": 443, "sent": 123456, "received": 99}
    assert "sent" not in js[1] and "mountnsid" not in js[1]          # omitempty
    k8s = G.render_table("tcp", rows, metadata_tag="kubernetes").split("\n")[0].split()
    assert k8s[:4] == ["NODE", "NAMESPACE", "POD", "CONTAINER"]
    assert G.render_json("tcp", []) == "[]" and G.render_json("tcp", None) == "null"
    assert T.go_json_string("<a&b> ") == '"\\u003ca\\u0026b\\u003e\\u2028"'


def test_top_file_and_block_io_output():
    f = [G.FileStats(Pid=1, Tid=1, Comm="dd", Reads=0, Writes=3, ReadBytes=0, WriteBytes=3 << 20, FileType=ord("R"),
                     Filename="/tmp/x")]
    lines = G.render_table("file", f).split("\n")
    assert lines[0].split() == ["PID", "COMM", "READS", "WRITES", "RBYTES", "WBYTES", "T", "FILE"]
    assert lines[1].split() == ["1", "dd", "0", "3", "0B", "3MiB", "R", "/tmp/x"]
    b = [G.BlockIOStats(Pid=-1, Comm="kworker", Write=True, Major=8, Minor=16, Bytes=4096, MicroSecs=12, Operations=1)]
    lines = G.render_table("block-io", b).split("\n")
    assert lines[0].split() == ["PID", "COMM", "R/W", "MAJOR", "MINOR", "BYTES", "TIME", "OPS"]
    assert lines[1].split() == ["-1", "kworker", "W", "8", "16", "4096", "12", "1"]
    assert json.loads(G.render_json("block-io", b))[0] == {"pid": -1, "comm": "kworker", "write": True, "major": 8,
                                                           "minor": 16, "bytes": 4096, "us": 12, "ops": 1}
