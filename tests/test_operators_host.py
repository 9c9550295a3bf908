"""Gadget registry, operators and the local runtime (host logic): the SortOperators table of
pkg/operators/operators_test.go:93-195, registry order and errors
(pkg/gadget-registry/gadget-registry.go), operator instantiation / enrichment chains
(operators.go:222-265)."""
import importlib

import pytest

OPS = importlib.import_module("inspektor-gadget_amd.operators")


class TOp(OPS.Operator):
    def __init__(self, name, deps):
        self.n, self.d = name, deps

    def Name(self):
        return self.n

    def Dependencies(self):
        return list(self.d)


def _check(ops, sorted_ops):
    """checkDependencies (operators_test.go:64-84): every operator comes after its deps."""
    assert len(ops) == len(sorted_ops)
    pos = {o.Name(): i for i, o in enumerate(sorted_ops)}
    for o in ops:
        for d in o.Dependencies():
            assert pos[d] < pos[o.Name()], (d, o.Name())


@pytest.mark.parametrize("spec", [
    [("b", ["a"]), ("a", [])],
    [("b", ["a"]), ("c", ["a"]), ("a", [])],
    [("b", ["a"]), ("c", ["a", "b"]), ("a", [])],
    [("c", ["a", "b"]), ("b", ["a"]), ("a", [])],
    [("a", []), ("b", ["a"]), ("c", ["a", "h"]), ("d", ["a"]), ("e", ["d", "b"]), ("f", ["h"]), ("g", ["e"]),
     ("h", ["d"]), ("i", ["g", "f"])],
])
def test_sort_operators(spec):
    ops = [TOp(n, d) for n, d in spec]
    _check(ops, OPS.SortOperators(ops))


def test_sort_operators_errors():
    with pytest.raises(OPS.OperatorError, match='dependency "b" is not available in operators'):
        OPS.SortOperators([TOp("a", ["b"])])
    with pytest.raises(OPS.OperatorError, match="dependency cycle detected"):
        OPS.SortOperators([TOp("a", ["b"]), TOp("b", ["a"]), TOp("c", ["a"])])
    with pytest.raises(OPS.OperatorError, match="dependency cycle detected"):
        OPS.SortOperators([TOp(x, [y]) for x, y in zip("abcdef", "bcdefa")])


def test_registry():
    names = [(g.Category(), g.Name()) for g in OPS.GetAll()]
    assert names == sorted(names, key=lambda cn: f"{cn[0]}-{cn[1]}")
    assert ("top", "tcp") in names and ("profile", "block-io") in names
    g = OPS.Get("top", "tcp")
    assert g.Type() == OPS.TypeTraceIntervals and OPS.IsPeriodic(g.Type()) and OPS.CanSort(g.Type())
    assert g.ParamDescs() == {"max-rows": 50, "sort": ["-sent", "-recv"], "interval": 1}
    assert OPS.Get("top", "nope") is None
    with pytest.raises(OPS.OperatorError, match='Gadget "top/tcp" already registered'):
        OPS.Register(g)


def test_instances_enrich_and_pre_post():
    log = []

    class Op(OPS.Operator):
        def __init__(self, n, fail=None):
            self.n, self.fail = n, fail

        def Name(self):
            return self.n

        def Instantiate(self, ctx, inst, params):
            n, fail = self.n, self.fail

            class I(OPS.OperatorInstance):
                def Name(self_):
                    return n

                def PreGadgetRun(self_):
                    if fail == "pre":
                        raise RuntimeError("boom")
                    log.append(("pre", n))

                def PostGadgetRun(self_):
                    log.append(("post", n))

                def EnrichEvent(self_, ev):
                    ev.append(n)
            return I()
    ois = OPS.Operators([Op("x"), Op("y")]).Instantiate(None, None, {})
    ev = []
    ois.Enrich(ev)
    assert ev == ["x", "y"]
    ois.PreGadgetRun()
    assert log == [("pre", "x"), ("pre", "y")]
    log.clear()
    bad = OPS.Operators([Op("x"), Op("z", fail="pre")]).Instantiate(None, None, {})
    with pytest.raises(OPS.OperatorError, match='pre gadget run on operator "z"'):
        bad.PreGadgetRun()
    assert log == [("pre", "x"), ("post", "x")]        # the loaded ones are rolled back
