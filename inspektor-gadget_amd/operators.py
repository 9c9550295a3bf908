"""The drop-in surface above the path: gadget registry, gadget descriptors, operators and the
local runtime, so the GPU gadgets are registered and run the way the reference's are.

  gadgetregistry.Register / Get / GetAll      pkg/gadget-registry/gadget-registry.go:26-49
  GadgetType, GadgetDesc, GadgetInstantiate,  pkg/gadgets/interface.go:23-166
  EventHandlerArraySetter, Run / RunWithResult
  Operator / OperatorInstance, Register,      pkg/operators/operators.go:40-348
  GetOperatorsForGadget, SortOperators,
  Instantiate, PreGadgetRun, Enrich
  gadgetcontext.New                           pkg/gadget-context/gadget-context.go:52-141
  local.Runtime.RunGadget                     pkg/runtime/local/local.go:69-152
  sortable gadget params (max-rows 50,        pkg/gadgets/params.go:24-96
  sort, interval 1)

The registered gadgets are the top tracers of gadgets.py (tcp, file, block-io: interval
gadgets whose maps live in device tables) and profile block-io (a result gadget).  A gadget
instance reads its events from a source callable (`events(interval) -> list of batches`,
the stand-in for the kernel probes); each interval runs the device group-by, SortStats and
truncation, then hands the []*Stats to the parser chain: operator enrichment, MatchAll and
Sort on the device (the Stats rows become a small SoA batch), then the callback.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

from . import gadgets as _g

# ---- gadget types (interface.go:23-38) ------------------------------------------------------
TypeTrace, TypeTraceIntervals, TypeOneShot, TypeProfile = "trace", "traceIntervals", "oneShot", "profile"


def CanSort(t: str) -> bool:
    return t in (TypeOneShot, TypeTraceIntervals)


def IsPeriodic(t: str) -> bool:
    return t == TypeTraceIntervals


class OperatorError(RuntimeError):
    pass


# ---- gadget registry (gadget-registry.go) -------------------------------------------------------
_gadget_registry: Dict[str, "GadgetDesc"] = {}


def Register(desc: "GadgetDesc"):
    key = desc.Category() + "/" + desc.Name()
    if key in _gadget_registry:
        raise OperatorError(f'Gadget "{key}" already registered')
    _gadget_registry[key] = desc


def Get(category: str, name: str) -> Optional["GadgetDesc"]:
    return _gadget_registry.get(category + "/" + name)


def GetAll() -> List["GadgetDesc"]:
    return sorted(_gadget_registry.values(), key=lambda g: f"{g.Category()}-{g.Name()}")


# ---- operators (operators.go) ----------------------------------------------------------------------
class Operator:
    """Base class mirroring the Operator interface; subclasses override what they need."""

    def Name(self) -> str:
        raise NotImplementedError

    def Description(self) -> str:
        return ""

    def GlobalParamDescs(self) -> dict:
        return {}

    def ParamDescs(self) -> dict:
        return {}

    def Dependencies(self) -> List[str]:
        return []

    def CanOperateOn(self, gadget: "GadgetDesc") -> bool:
        return True

    def Init(self, params: dict):
        return None

    def Close(self):
        return None

    def Instantiate(self, gadgetCtx, gadgetInstance, params: dict) -> "OperatorInstance":
        raise NotImplementedError


class OperatorInstance:
    def Name(self) -> str:
        raise NotImplementedError

    def PreGadgetRun(self):
        return None

    def PostGadgetRun(self):
        return None

    def EnrichEvent(self, ev):
        return None


class _Wrapped:
    """operatorWrapper: Init runs once."""

    def __init__(self, op: Operator):
        self.op = op
        self.initialized = False

    def __getattr__(self, name):
        return getattr(self.op, name)

    def Init(self, params):
        if not self.initialized:
            self.initialized = True
            return self.op.Init(params)
        return None


_all_operators: Dict[str, _Wrapped] = {}


def RegisterOperator(op: Operator):
    if op.Name() in _all_operators:
        raise OperatorError(f'operator already registered: "{op.Name()}"')
    _all_operators[op.Name()] = _Wrapped(op)


def GetRaw(name: str) -> Optional[Operator]:
    w = _all_operators.get(name)
    return w.op if w else None


class Operators(list):
    def Init(self, pc: Dict[str, dict]):
        for op in self:
            try:
                op.Init(pc.get(op.Name(), {}))
            except Exception as e:
                raise OperatorError(f'initializing operator "{op.Name()}": {e}') from e

    def Close(self):
        for op in self:
            try:
                op.Close()
            except Exception:   # the reference logs and continues
                pass

    def ParamCollection(self):
        return {op.Name(): dict(op.ParamDescs()) for op in self}

    def Instantiate(self, gadgetCtx, trace, pc: Dict[str, dict]) -> "OperatorInstances":
        out = OperatorInstances()
        for op in self:
            try:
                out.append(op.Instantiate(gadgetCtx, trace, pc.get(op.Name(), {})))
            except Exception as e:
                raise OperatorError(f'start trace on operator "{op.Name()}": {e}') from e
        return out


class OperatorInstances(list):
    def PreGadgetRun(self):
        loaded = OperatorInstances()
        for inst in self:
            try:
                inst.PreGadgetRun()
            except Exception as e:
                loaded.PostGadgetRun()
                raise OperatorError(f'pre gadget run on operator "{inst.Name()}": {e}') from e
            loaded.append(inst)

    def PostGadgetRun(self):
        for inst in self:
            inst.PostGadgetRun()

    def Enrich(self, ev):
        for inst in self:
            try:
                inst.EnrichEvent(ev)
            except Exception as e:
                raise OperatorError(f'operator "{inst.Name()}" failed to enrich event {ev!r}') from e


def GetAllOperators() -> Operators:
    return Operators(_all_operators.values())


def SortOperators(operators) -> Operators:
    """operators.go:269-348: Kahn's algorithm over Dependencies, each popped operator
    prepended, so dependencies come first; missing dependencies and cycles are errors."""
    incoming: Dict[str, int] = {e.Name(): 0 for e in operators}
    for e in operators:
        for d in e.Dependencies():
            incoming[d] = incoming.get(d, 0) + 1
    names = {e.Name() for e in operators}
    for n in incoming:
        if n not in names:
            raise OperatorError(f'dependency "{n}" is not available in operators')
    queue = [e.Name() for e in operators if incoming[e.Name()] == 0]
    result: List = []
    visited = set()
    while queue:
        n = queue.pop(0)
        visited.add(n)
        for s in operators:
            if s.Name() == n:
                result.insert(0, s)
                break
        for d in result[0].Dependencies():
            incoming[d] -= 1
            if incoming[d] == 0:
                queue.append(d)
            if d in visited:
                raise OperatorError("dependency cycle detected")
    for e in operators:
        if e.Name() not in visited:
            raise OperatorError("dependency cycle detected")
    return Operators(result)


def GetOperatorsForGadget(gadget: "GadgetDesc") -> Operators:
    return SortOperators([op for op in _all_operators.values() if op.CanOperateOn(gadget)])


# ---- gadget context + local runtime ---------------------------------------------------------------
class GadgetContext:
    """gadgetcontext.New (gadget-context.go:52-80) without the Go context: a run ends when
    the gadget's event source is exhausted (or after `Iterations` intervals)."""

    def __init__(self, id: str, gadget: "GadgetDesc", gadgetParams: Optional[dict] = None,
                 operatorsParamCollection: Optional[Dict[str, dict]] = None, parser=None, logger=None,
                 timeout: float = 0.0):
        self.id = id
        self.gadget = gadget
        self.gadgetParams = dict(gadget.ParamDescs())
        self.gadgetParams.update(gadgetParams or {})
        self.operatorsParamCollection = operatorsParamCollection or {}
        self.parser = parser
        self.logger = logger
        self.timeout = timeout
        self.operators = GetOperatorsForGadget(gadget)

    def ID(self):
        return self.id

    def GadgetDesc(self):
        return self.gadget

    def Parser(self):
        return self.parser

    def Operators(self):
        return self.operators

    def GadgetParams(self):
        return self.gadgetParams

    def OperatorsParamCollection(self):
        return self.operatorsParamCollection

    def Logger(self):
        return self.logger

    def Timeout(self):
        return self.timeout


class LocalRuntime:
    """runtime/local (local.go:69-152)."""

    def RunGadget(self, ctx: GadgetContext):
        gadget = ctx.GadgetDesc()
        if not hasattr(gadget, "NewInstance"):
            raise OperatorError("gadget not instantiable")
        inst = gadget.NewInstance(ctx.GadgetParams())
        if hasattr(inst, "Init"):
            inst.Init(ctx)
        try:
            ois = ctx.Operators().Instantiate(ctx, inst, ctx.OperatorsParamCollection())
            if hasattr(inst, "SetEventHandlerArray") and ctx.Parser() is not None:
                inst.SetEventHandlerArray(ctx.Parser().EventHandlerFuncArray(ois.Enrich))
            ois.PreGadgetRun()
            try:
                if hasattr(inst, "Run"):
                    inst.Run(ctx)
                    return None
                if hasattr(inst, "RunWithResult"):
                    return {"": inst.RunWithResult(ctx)}
                raise OperatorError("gadget not runnable")
            finally:
                ois.PostGadgetRun()
        finally:
            if hasattr(inst, "Close"):
                inst.Close()


# ---- the Stats parser: enrichment + MatchAll + Sort of []*Stats on the device -----------------------
class StatsParser:
    """parser.Parser for a top gadget's Stats (parser.go:199-224 eventHandlerArray): the
    enrichers run on the host Stats objects, MatchAll and Sort on the device over the rows as a
    SoA batch (gadgets.STATS_OUTPUT names every column's field)."""

    def __init__(self, gadget: str, cols):
        from . import parser as _p
        self.gadget = gadget
        self.cols = cols
        self.p = _p.NewParser(cols)
        self.attr = {tag.split(",")[0].lower(): attr for attr, _, tag, _ in _g.STATS_OUTPUT[gadget]["fields"]}
        self.eventCallbackArray = None

    def SetFilters(self, filters):
        self.p.SetFilters(filters)

    def SetSorting(self, sortBy):
        self.p.SetSorting(sortBy)

    def SetEventCallback(self, cb):
        self.eventCallbackArray = cb

    def _parser_for(self, stats):
        """The parser for this batch: the configured one, or -- when a string value is longer
        than its column's declared width -- one over a copy of the schema whose string columns
        are as wide as the batch's longest value (Go compares whole strings, parser.go:209-221:
        a path or pod name must not be cut to the column width before MatchAll / Sort)."""
        from . import columns as _c
        from . import parser as _p
        wide = {}
        for c in self.cols.GetOrderedColumns():
            attr = self.attr.get(c.Name.lower())
            if c.kind == "string" and not c.virtual and attr:
                m = max((len(str(getattr(s, attr)).encode()) for s in stats), default=0)
                if m > c.width:
                    wide[c.Name.lower()] = (m + 7) // 8 * 8
        if not wide:
            return self.cols, self.p
        key = tuple(sorted(wide.items()))
        cache = self.__dict__.setdefault("_wide", {})
        if key not in cache:
            cols = _c.Columns()
            for c in self.cols.GetOrderedColumns():
                cols._add(_c.Column(c.Name, c.kind, wide.get(c.Name.lower(), c.width), c.GroupType, c.virtual,
                                    c.extractor))
            p = _p.NewParser(cols)
            if self.p.filters:
                p.SetFilters(self.p.filters)
            if self.p.sortSpec is not None:
                p.SetSorting(self.p.sortBy)
            cache[key] = (cols, p)
        return cache[key]

    def _batch(self, stats, cols=None):
        import numpy as np
        from . import columns as H
        cols = self.cols if cols is None else cols
        data = {}
        for c in cols.GetOrderedColumns():
            if c.virtual:
                continue
            name = c.Name.lower()
            attr = self.attr.get(name)
            n = len(stats)
            if c.kind == "string":
                a = np.zeros((n, c.width), np.uint8)
                for i, s in enumerate(stats):
                    b = (getattr(s, attr) if attr else "").encode()[:c.width]
                    a[i, :len(b)] = np.frombuffer(b, np.uint8)
            elif c.kind == "bool":
                a = np.array([bool(getattr(s, attr)) for s in stats], np.bool_)
            else:
                dt = {"int": np.int64, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
                      "uint": np.uint64, "uint8": np.uint8, "uint16": np.uint16, "uint32": np.uint32,
                      "uint64": np.uint64, "float32": np.float32, "float64": np.float64}[c.kind]
                a = np.array([getattr(s, attr) if attr else 0 for s in stats], dt)
            data[name] = H.to_device(a)
        data["__row"] = H.to_device(np.arange(len(stats), dtype=np.int32))
        return H.EventBatch(cols, data)

    def EventHandlerFuncArray(self, *enrichers):
        from . import columns as H

        def handle(stats):
            for e in enrichers:
                for s in stats:
                    e(s)
            out = stats
            if stats and (self.p.filterSpecs is not None or self.p.sortSpec is not None):
                cols, p = self._parser_for(stats)
                b = self._batch(stats, cols)
                if p.filterSpecs is not None:
                    b = b.take(p.filterSpecs.MatchAll(b))
                if p.sortSpec is not None and b.n:
                    b = p.sortSpec.Sort(b)
                out = [stats[int(i)] for i in H.host(b["__row"])] if b.n else []
            if self.eventCallbackArray is not None:
                self.eventCallbackArray(out)
        return handle


# ---- the GPU gadgets ------------------------------------------------------------------------------------
def _sortable_params(sort_default):
    """gadgets/params.go:70-96: max-rows (50), sort (the gadget's default), interval (1 s)."""
    return {"max-rows": 50, "sort": list(sort_default), "interval": 1}


class GadgetDesc:
    """A registered GPU gadget (GadgetDesc + GadgetInstantiate)."""

    def __init__(self, name, category, typ, description, tracer_cls=None, output=None):
        self._name, self._category, self._type, self._description = name, category, typ, description
        self.tracer_cls, self.output = tracer_cls, output

    def Name(self):
        return self._name

    def Category(self):
        return self._category

    def Type(self):
        return self._type

    def Description(self):
        return self._description

    def ParamDescs(self):
        if self.tracer_cls is not None:
            return _sortable_params(self.tracer_cls.SortByDefault)
        return {}

    def Parser(self):
        if self.output is None:
            return None
        return StatsParser(self.output, self.tracer_cls.STATS_COLS)

    def EventPrototype(self):
        return {"tcp": _g.TcpStats, "file": _g.FileStats, "block-io": _g.BlockIOStats}.get(self.output, dict)()

    def NewInstance(self, params: dict):
        if self.tracer_cls is not None:
            return TopGadgetInstance(self, params)
        return ProfileBlockIOInstance(params)


class TopGadgetInstance:
    """A top tracer as a RunGadget: per interval, its event source's batches go through the
    device probe (feed), then nextStats -> stats[:MaxRows] -> the event handler (the ticker loop
    of top/*/tracer/tracer.go run, Iterations counted down by ComputeIterations)."""

    def __init__(self, desc: GadgetDesc, params: dict):
        self.desc = desc
        self.params = params
        self.handler: Optional[Callable] = None
        kw = {k: v for k, v in params.items() if k in ("TargetPid", "TargetFamily", "AllFiles")}
        self.tracer = desc.tracer_cls(MaxRows=int(params.get("max-rows", 50)), SortBy=params.get("sort"),
                                      capacity=int(params.get("capacity", 1 << 20)), **kw)

    def SetEventHandlerArray(self, handler):
        self.handler = handler

    def Run(self, ctx: GadgetContext):
        source = self.params.get("events")
        if source is None:
            raise OperatorError("gadget has no event source (params['events'])")
        iterations = int(self.params.get("iterations", 0))
        i = 0
        while iterations == 0 or i < iterations:
            batches = source(i)
            if batches is None:
                break
            for b in batches:
                self.tracer.feed(b)
            ev = self.tracer.NextEvent()
            if self.handler is not None:
                self.handler(ev.Stats)
            i += 1

    def Close(self):
        self.tracer.destroy()


class ProfileBlockIOInstance:
    """profile block-io as a RunWithResultGadget: every batch of the source feeds the device
    log2 histogram; the result is the JSON report of the first key (tracer.go:171-180)."""

    def __init__(self, params: dict):
        self.params = params

    def RunWithResult(self, ctx: GadgetContext) -> bytes:
        tr = _g.ProfileBlockIOTracer(ms=bool(self.params.get("milliseconds", False)))
        source = self.params.get("events")
        i = 0
        while source is not None:
            batches = source(i)
            if batches is None:
                break
            for b in batches:
                tr.feed(b["delta_ns"], b.get("dev"), b.get("cont"))
            i += 1
        return tr.getReport().to_json().encode()


def _register_builtin():
    Register(GadgetDesc("tcp", "top", TypeTraceIntervals, "Periodically report TCP activity",
                        _g.TopTcpTracer, "tcp"))
    Register(GadgetDesc("file", "top", TypeTraceIntervals, "Periodically report read/write activity by file",
                        _g.TopFileTracer, "file"))
    Register(GadgetDesc("block-io", "top", TypeTraceIntervals, "Periodically report block device I/O activity",
                        _g.TopBlockIOTracer, "block-io"))
    Register(GadgetDesc("block-io", "profile", TypeProfile, "Analyze block I/O performance through a latency "
                        "distribution"))


_register_builtin()


class MountNsEnricher(Operator):
    """A ContainerInfoFromMountNSID enricher (the role of pkg/operators/localmanager and
    kubemanager, operators.go:87-103): sets Node / Namespace / Pod / Container of events from
    their MountNsID through a table given as the per-gadget param "containers"
    ({mntns: (node, namespace, pod, container)})."""

    def Name(self):
        return "MountNsEnricher"

    def Description(self):
        return "adds container metadata from the mount namespace id"

    def ParamDescs(self):
        return {"containers": {}}

    def CanOperateOn(self, gadget):
        return hasattr(gadget.EventPrototype(), "MountNsID")

    def Instantiate(self, gadgetCtx, gadgetInstance, params):
        table = dict(params.get("containers", {}))

        class Inst(OperatorInstance):
            def Name(self_):
                return "MountNsEnricher"

            def EnrichEvent(self_, ev):
                info = table.get(getattr(ev, "MountNsID", None))
                if info:
                    ev.Node, ev.Namespace, ev.Pod, ev.Container = info
        return Inst()


RegisterOperator(MountNsEnricher())
