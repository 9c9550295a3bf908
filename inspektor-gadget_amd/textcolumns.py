"""The output side of the path: the Stats rows the device path
returns, rendered as the reference's frontends render them.

  ellipsis.Shorten / ShortenString         pkg/columns/ellipsis/ellipsis.go:44-79
  column tags, templates and defaults      pkg/columns/columninfo.go:119-245,
                                           pkg/columns/columns.go:155-310, templates.go,
                                           pkg/types/types.go:29-51 (registered templates)
  TextColumnsFormatter                     pkg/columns/formatter/textcolumns/{textcolumns,
                                           output,scaler,helpers,options}.go
  GadgetParser.TransformIntoTable          cmd/common/utils/parser-tableformatter.go:106-111
  JSON (printEventAsJSONFn, json.Marshal)  cmd/common/registry.go:511-520
  units.BytesSize (sent / recv extractors) github.com/docker/go-units v0.5.0 size.go (restated:
                                           "%.4g%s" over 1024-based B..YiB units)

Rendering runs on the host after the device has reduced an interval to its top-K rows
(at most max-rows entries), so none of it is on the hot path.  The per-gadget column sets
restate the reference's `column:"..."` struct tags (top tcp / file / block-io Stats types).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field, fields as dc_fields, is_dataclass
from typing import Callable, Dict, List, Optional

# ---- ellipsis ---------------------------------------------------------------------------
NONE, END, START, MIDDLE = range(4)           # ellipsis.go:19-24
ELLIPSIS = "…"


def Shorten(rs: str, maxLength: int, ellipsisType: int) -> str:
    """ellipsis.Shorten over the string's runes (Python str = code points = Go runes)."""
    if maxLength <= 0:
        return ""
    slen = len(rs)
    if slen <= maxLength:
        return rs
    if maxLength <= 1 and ellipsisType != NONE:
        return ELLIPSIS
    if ellipsisType == START:
        return ELLIPSIS + rs[slen - maxLength + 1:]
    if ellipsisType == END:
        return rs[:maxLength - 1] + ELLIPSIS
    if ellipsisType == MIDDLE:
        mid = maxLength // 2
        end = mid - 1 if maxLength % 2 == 0 else mid
        return rs[:mid] + ELLIPSIS + rs[slen - end:]
    return rs[:maxLength]


ShortenString = Shorten

# ---- columns ------------------------------------------------------------------------------
ALIGN_LEFT, ALIGN_RIGHT = 0, 1                # types.go:20-23
GROUP_NONE, GROUP_SUM = 0, 1
MAX_CHARS = {"uint8": 3, "int8": 4, "uint16": 5, "int16": 6, "uint32": 10, "int32": 11,
             "uint64": 20, "uint": 20, "int64": 20, "int": 20, "bool": 5}      # columninfo.go:26-36
INT_KINDS = ("int", "int8", "int16", "int32", "int64")
UINT_KINDS = ("uint", "uint8", "uint16", "uint32", "uint64")
FLOAT_KINDS = ("float32", "float64")

# pkg/types/types.go:31-50
TEMPLATES: Dict[str, str] = {
    "timestamp": "width:35,maxWidth:35,hide", "node": "width:30,ellipsis:middle", "namespace": "width:30",
    "pod": "width:30,ellipsis:middle", "container": "width:30", "comm": "maxWidth:16", "pid": "minWidth:7",
    "ns": "width:12,hide", "ipaddr": "minWidth:15,maxWidth:45", "ipport": "minWidth:type",
    "syscall": "width:18,maxWidth:28",
}


class ColumnError(ValueError):
    pass


@dataclass
class Column:
    """columns.Column[T] (columninfo.go:43-66): display attributes of one column."""
    Name: str
    kind: str                                    # Go reflect kind ("string" for extractors)
    attr: Optional[str] = None                   # field of the entry object
    Width: int = 0
    MinWidth: int = 0
    MaxWidth: int = 0
    Alignment: int = ALIGN_LEFT
    Visible: bool = True
    GroupType: int = GROUP_NONE
    EllipsisType: int = END
    FixedWidth: bool = False
    Precision: int = 2
    Order: int = 0
    Tags: List[str] = field(default_factory=list)
    Extractor: Optional[Callable] = None
    template: str = ""

    def Kind(self):
        return self.kind

    def value(self, entry):
        """GetRef: the extractor's string, or the raw field."""
        if self.Extractor is not None:
            return self.Extractor(entry)
        return getattr(entry, self.attr)

    def _width(self, params):
        if len(params) == 1:
            raise ColumnError(f'missing "{params[0]}" value for field "{self.Name}"')
        if params[1] == "type":
            w = MAX_CHARS.get(self.kind, 0)
            if w > 0:
                return w
            raise ColumnError(f'special value "type" used for field "{self.Name}" is only available for '
                              "integer and bool types")
        try:
            return int(params[1])
        except ValueError:
            raise ColumnError(f'invalid width "{params[1]}" for field "{self.Name}"') from None

    def parse_tag_info(self, info):
        """columninfo.go:125-245 (noembed and stringer do not apply to flat rows)."""
        for sub in info:
            params = sub.split(":", 1)
            p = params[0]
            if p == "align":
                if len(params) == 1:
                    raise ColumnError(f'missing alignment value for field "{self.Name}"')
                if params[1] not in ("left", "right"):
                    raise ColumnError(f'invalid alignment "{params[1]}" for field "{self.Name}"')
                self.Alignment = ALIGN_LEFT if params[1] == "left" else ALIGN_RIGHT
            elif p == "ellipsis":
                v = params[1] if len(params) > 1 else ""
                m = {"end": END, "": END, "middle": MIDDLE, "none": NONE, "start": START}
                if v not in m:
                    raise ColumnError(f'invalid ellipsis value "{v}" for field "{self.Name}"')
                self.EllipsisType = m[v]
            elif p == "fixed":
                if len(params) != 1:
                    raise ColumnError(f'parameter fixed on field "{self.Name}" must not have a value')
                self.FixedWidth = True
            elif p == "group":
                if len(params) == 1 or params[1] != "sum":
                    raise ColumnError(f'invalid group value for field "{self.Name}"')
                if self.kind not in INT_KINDS + UINT_KINDS + FLOAT_KINDS:
                    raise ColumnError(f'cannot use sum on field "{self.Name}" of kind "{self.kind}"')
                self.GroupType = GROUP_SUM
            elif p == "hide":
                if len(params) != 1:
                    raise ColumnError(f'parameter hide on field "{self.Name}" must not have a value')
                self.Visible = False
            elif p == "order":
                if len(params) == 1:
                    raise ColumnError(f'missing width value for field "{self.Name}"')
                try:
                    self.Order = int(params[1])
                except ValueError:
                    raise ColumnError(f'invalid order value "{params[1]}" for field "{self.Name}"') from None
            elif p == "precision":
                if self.kind not in FLOAT_KINDS:
                    raise ColumnError(f'field "{self.Name}" is not a float field and thereby cannot have '
                                      "precision defined")
                if len(params) == 1:
                    raise ColumnError(f'missing precision value for field "{self.Name}"')
                w = int(params[1])
                if w < -1:
                    raise ColumnError(f'negative precision value "{params[1]}" for field "{self.Name}"')
                self.Precision = w
            elif p == "width":
                self.Width = self._width(params)
            elif p == "maxWidth":
                self.MaxWidth = self._width(params)
            elif p == "minWidth":
                self.MinWidth = self._width(params)
            elif p == "template":
                if len(params) < 2 or params[1] == "":
                    raise ColumnError(f'no template specified for field "{self.Name}"')
                self.template = params[1]
            else:
                raise ColumnError(f'invalid column parameter "{p}" for field "{self.Name}"')


class ColumnMap:
    """columns.NewColumns[T] over a flat field list (columns.go:155-310): fields are
    (attr, go_kind, tag); an empty tag names the column after the field."""

    DefaultWidth = 16                              # options.go:32

    def __init__(self, fields_):
        self.cols: Dict[str, Column] = {}
        for attr, kind, tag in fields_:
            self._add_field(attr, kind, tag)

    def _add_field(self, attr, kind, tag):
        tag = tag or attr
        c = Column(Name="", kind=kind, attr=attr, Order=len(self.cols) * 10)
        info = tag.split(",")
        c.Name = info[0]
        c.parse_tag_info(info[1:])
        if c.template:
            if c.template not in TEMPLATES:
                raise ColumnError(f'error applying template "{c.template}" on field "{attr}": template not found')
            c.parse_tag_info(TEMPLATES[c.template].split(","))
            c.Name = info[0]
            c.parse_tag_info(info[1:])           # the field's own settings win
        if c.Name == "":
            c.Name = attr
        if c.Width > 0 and c.MinWidth > c.Width:
            raise ColumnError(f'minWidth should not be greater than width on field "{attr}"')
        if c.MaxWidth > 0:
            if c.MaxWidth < c.Width:
                raise ColumnError(f'maxWidth should not be less than width on field "{attr}"')
            if c.MaxWidth < c.MinWidth:
                raise ColumnError(f'maxWidth must be greater than minWidth "{attr}"')
        if c.MaxWidth == 0:
            c.MaxWidth = MAX_CHARS.get(c.kind, 0)
        if c.Width == 0:
            c.Width = self.DefaultWidth
        if c.MinWidth > c.Width:
            c.Width = c.MinWidth
        key = c.Name.lower()
        if key in self.cols:
            raise ColumnError(f'duplicate column "{key}"')
        self.cols[key] = c

    def SetExtractor(self, name, fn):
        """columns.go:320-332: the column now reads as a string."""
        c = self.cols.get(name.lower())
        if c is None:
            raise ColumnError(f'could not set extractor for unknown field "{name}"')
        c.kind = "string"
        c.Extractor = fn

    def AddColumn(self, name, fn, Width=0, MinWidth=0, MaxWidth=0, Visible=True, Order=0, **kw):
        """columns.go:282-309: a virtual column (string kind, extractor only)."""
        key = name.lower()
        if key in self.cols:
            raise ColumnError(f'column already exists: "{key}"')
        c = Column(Name=name, kind="string", Width=Width or self.DefaultWidth, MinWidth=MinWidth,
                   MaxWidth=MaxWidth, Visible=Visible, Order=Order, Extractor=fn, **kw)
        self.cols[key] = c

    def GetColumnMap(self):
        return self.cols


# ---- formatter ------------------------------------------------------------------------------
HEADER_NORMAL, HEADER_UPPER, HEADER_LOWER = range(3)
DIVIDER_SPACE, DIVIDER_TAB, DIVIDER_DASH, DIVIDER_NONE = " ", "\t", "—", ""


def go_format_float(v: float, prec: int) -> str:
    """strconv.FormatFloat(v, 'f', prec, 64)."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if prec < 0:
        import numpy as np
        s = np.format_float_positional(np.float64(v), unique=True, trim="-")
        return s
    return f"{v:.{prec}f}"


def format_value(col: Column, v) -> str:
    """setFormatter (output.go:30-62): the string a value of the column's kind prints as."""
    k = col.kind
    if k in INT_KINDS or k in UINT_KINDS:
        return str(int(v))
    if k in FLOAT_KINDS:
        return go_format_float(float(v), col.Precision)
    if k == "string":
        return str(v)
    if k == "bool":
        return "true" if v else "false"
    return str(v)


class _FCol:
    def __init__(self, col: Column):
        self.col = col
        self.calculatedWidth = col.Width
        self.treatAsFixed = False


class TextColumnsFormatter:
    """textcolumns.NewFormatter (textcolumns.go:42-137) and its output / scaler methods.
    terminal_width stands in for GetTerminalWidth (0 = stdout is not a terminal)."""

    def __init__(self, columns, AutoScale=True, ColumnDivider=DIVIDER_SPACE, DefaultColumns=None,
                 HeaderStyle=HEADER_UPPER, RowDivider=DIVIDER_NONE, terminal_width=0):
        cmap = columns.GetColumnMap() if hasattr(columns, "GetColumnMap") else columns
        self.AutoScale, self.ColumnDivider, self.DefaultColumns = AutoScale, ColumnDivider, DefaultColumns
        self.HeaderStyle, self.RowDivider, self.terminal_width = HeaderStyle, RowDivider, terminal_width
        self.columns = {name: _FCol(c) for name, c in cmap.items()}
        self.currentMaxWidth = -1
        self.showColumns: List[_FCol] = []
        self.fillString = ""
        self.SetShowColumns(DefaultColumns)

    # -- column selection --------------------------------------------------------------
    def SetShowDefaultColumns(self):
        if self.DefaultColumns is not None:
            self.SetShowColumns(self.DefaultColumns)
            return
        # visible columns by Order (sort.Slice; equal Orders keep map order -- random in Go,
        # insertion order here)
        self.showColumns = sorted([c for c in self.columns.values() if c.col.Visible], key=lambda c: c.col.Order)
        self._rebuild()

    def SetShowColumns(self, names):
        if names is None:
            self.SetShowDefaultColumns()
            return
        cols = []
        for n in names:
            c = self.columns.get(n.lower())
            if c is None:
                raise ColumnError(f'column "{n.lower()}" is invalid')
            cols.append(c)
        self.showColumns = cols
        self._rebuild()

    def SetAutoScale(self, enable: bool):
        self.AutoScale = enable
        if enable:
            self._rebuild()
        else:
            for c in self.columns.values():
                c.calculatedWidth = c.col.Width
                c.treatAsFixed = False
            self._build_fill()

    def _rebuild(self):
        self._build_fill()
        self.currentMaxWidth = -1
        self.AdjustWidthsToScreen()

    def _build_fill(self):
        self.fillString = " " * max([c.calculatedWidth for c in self.showColumns] or [0])

    # -- output ----------------------------------------------------------------------------
    def buildFixedString(self, s: str, length: int, ellipsisType: int, alignment: int) -> str:
        if length <= 0:
            return ""
        sh = Shorten(s, length, ellipsisType)
        if len(sh) == length:
            return sh
        pad = self.fillString[0:length - len(sh)]
        return sh + pad if alignment == ALIGN_LEFT else pad + sh

    def FormatEntry(self, entry) -> str:
        if entry is None:
            return ""
        parts = []
        for c in self.showColumns:
            parts.append(self.buildFixedString(format_value(c.col, c.col.value(entry)), c.calculatedWidth,
                                               c.col.EllipsisType, c.col.Alignment))
        return self.ColumnDivider.join(parts)

    def FormatHeader(self) -> str:
        self.AdjustWidthsToScreen()
        parts = []
        for c in self.showColumns:
            name = c.col.Name
            if self.HeaderStyle == HEADER_UPPER:
                name = name.upper()
            elif self.HeaderStyle == HEADER_LOWER:
                name = name.lower()
            parts.append(self.buildFixedString(name, c.calculatedWidth, END, c.col.Alignment))
        return self.ColumnDivider.join(parts)

    def FormatRowDivider(self) -> str:
        if self.RowDivider == DIVIDER_NONE:
            return ""
        n = sum(c.calculatedWidth for c in self.showColumns) + \
            len(self.ColumnDivider) * max(0, len(self.showColumns) - 1)
        reps = -(-n // len(self.RowDivider)) if n else 0
        return (self.RowDivider * reps)[:n]

    def WriteTable(self, entries) -> str:
        out = self.FormatHeader() + "\n"
        if self.RowDivider != DIVIDER_NONE:
            out += self.FormatRowDivider() + "\n"
        for e in entries:
            out += self.FormatEntry(e) + "\n"
        return out

    def FormatTable(self, entries) -> str:
        return self.WriteTable(entries)[:-1]

    # -- scaler ------------------------------------------------------------------------------
    def AdjustWidthsToScreen(self):
        if not self.AutoScale or self.terminal_width == 0:
            return
        self.RecalculateWidths(self.terminal_width, False)

    def RecalculateWidths(self, maxWidth: int, force: bool):
        """scaler.go:27-180."""
        if self.currentMaxWidth == maxWidth:
            return
        self.currentMaxWidth = maxWidth
        if not self.showColumns:
            return
        occ: Dict[str, int] = {}
        divider = (len(self.showColumns) - 1) * len(self.ColumnDivider)
        required = divider
        notFixed = 0
        fixed = divider
        for c in self.showColumns:
            c.treatAsFixed = False
            occ[c.col.Name] = occ.get(c.col.Name, 0) + 1
            if c.col.FixedWidth and not force:
                required += c.col.Width
                fixed += c.col.Width
                continue
            notFixed += c.col.Width
            if c.col.MinWidth > 0 and not force:
                required += c.col.MinWidth
                continue
            required += 1
        if force:
            required = divider + len(self.showColumns)
        if required > maxWidth:
            maxWidth = required
        adjusted = 0
        while True:
            satisfied = True
            addToFixed = removeFromNotFixed = 0
            adjusted = 0
            for c in self.showColumns:
                if (c.col.FixedWidth or c.treatAsFixed) and not force:
                    if c.col.FixedWidth:
                        c.calculatedWidth = c.col.Width
                    continue
                c.calculatedWidth = int(math.floor(c.col.Width / notFixed * (maxWidth - fixed))) if notFixed else 0
                if not force:
                    if c.col.MaxWidth > 0 and c.calculatedWidth > c.col.MaxWidth:
                        c.calculatedWidth = c.col.MaxWidth
                        c.treatAsFixed = True
                        satisfied = False
                        addToFixed += c.calculatedWidth
                        removeFromNotFixed += c.col.Width
                        continue
                    if c.col.MinWidth > 0 and c.calculatedWidth < c.col.MinWidth:
                        c.calculatedWidth = c.col.MinWidth
                        c.treatAsFixed = True
                        satisfied = False
                        addToFixed += c.calculatedWidth
                        removeFromNotFixed += c.col.Width
                        continue
                adjusted += c.calculatedWidth
            if satisfied:
                break
            fixed += addToFixed
            notFixed -= removeFromNotFixed
        leftover = maxWidth - (adjusted + fixed)
        while leftover > 0:
            spent = False
            already = set()
            done = False
            for c in self.showColumns:
                if (c.col.FixedWidth or c.treatAsFixed) and not force:
                    continue
                o = occ[c.col.Name]
                if o > 1:
                    if c.col.Name in already:
                        continue
                    if o <= leftover:
                        c.calculatedWidth += 1
                        leftover -= o
                        spent = True
                        if leftover == 0:
                            done = True
                            break
                        already.add(c.col.Name)
                    continue
                c.calculatedWidth += 1
                leftover -= 1
                spent = True
                if leftover == 0:
                    done = True
                    break
            if done or not spent:
                break
        self._build_fill()

    def AdjustWidthsToContent(self, entries, considerHeaders: bool, maxWidth: int, force: bool):
        """scaler.go:226-315."""
        widths = [c.calculatedWidth if c.col.FixedWidth else 0 for c in self.showColumns]
        for e in entries:
            if e is None:
                continue
            for i, c in enumerate(self.showColumns):
                if c.col.FixedWidth:
                    continue
                widths[i] = max(widths[i], len(format_value(c.col, c.col.value(e))))
        if considerHeaders:
            for i, c in enumerate(self.showColumns):
                if not c.col.FixedWidth:
                    widths[i] = max(widths[i], len(c.col.Name))
        total = 0
        for i, c in enumerate(self.showColumns):
            c.calculatedWidth = widths[i]
            total += widths[i]
        self._build_fill()
        total += len(self.ColumnDivider) * (len(self.showColumns) - 1)
        if maxWidth == 0 or total <= maxWidth:
            return
        self.currentMaxWidth = -1
        self.RecalculateWidths(maxWidth, force)


def TransformIntoTable(formatter: TextColumnsFormatter, entries, terminal_width: int = 0) -> str:
    """GadgetParser.TransformIntoTable (parser-tableformatter.go:106-111)."""
    formatter.SetAutoScale(False)
    formatter.AdjustWidthsToContent(entries, True, terminal_width, True)
    return formatter.FormatTable(entries)


# ---- go-units BytesSize -----------------------------------------------------------------------
_BINARY = ["B", "KiB", "MiB", "GiB", "TiB", "PiB", "EiB", "ZiB", "YiB"]


def BytesSize(size: float) -> str:
    """units.BytesSize: CustomSize("%.4g%s", size, 1024.0, binaryAbbrs)."""
    i = 0
    while size >= 1024.0 and i < len(_BINARY) - 1:
        size /= 1024.0
        i += 1
    return "%.4g%s" % (size, _BINARY[i])


# ---- JSON as encoding/json marshals it -------------------------------------------------------------
def go_json_string(s: str) -> str:
    """encoding/json string encoding: HTML-safe (<, >, & escaped), U+2028/2029 escaped."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_json_value(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return json.dumps(v)
    if isinstance(v, str):
        return go_json_string(v)
    if v is None:
        return "null"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(go_json_value(x) for x in v) + "]"
    raise TypeError(type(v))


def marshal(obj, json_fields) -> str:
    """json.Marshal of one struct: json_fields = [(attr, json name, omitempty)] in struct order
    (embedded structs' fields inline, as encoding/json flattens them)."""
    if obj is None:
        return "null"
    parts = []
    for attr, name, omitempty in json_fields:
        v = getattr(obj, attr)
        if omitempty and (v == 0 or v == "" or v is False or v is None):
            continue
        parts.append(go_json_string(name) + ":" + go_json_value(v))
    return "{" + ",".join(parts) + "}"


def marshal_array(objs, json_fields) -> str:
    """json.Marshal([]*T): what printEventAsJSONFn prints per interval (registry.go:511-520)."""
    if objs is None:
        return "null"
    return "[" + ",".join(marshal(o, json_fields) for o in objs) + "]"
