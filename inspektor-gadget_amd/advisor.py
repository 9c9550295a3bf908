"""advise network-policy: NetworkPolicyAdvisor with its dedup on the GPU.

Reference: pkg/gadgets/advise/networkpolicy/advisor/advisor.go.
  LoadBuffer (:64-100)        JSON array, else one JSON event per line
  GeneratePolicies (:277-372) filter events (:279-292), group by the local pod key
                              (:294-300), keep the FIRST event per (direction, peer key)
                              (:302-320), one rule per kept event (:321-342), one policy
                              per source named after its first event (:344-366),
                              policies sorted by name (:369-371)
  FormatPolicies (:374-387)   k8s YAML documents joined by "---"

The per-event work -- the filter and the first-event-wins dedup over every event -- runs
in libigx.so: events are dictionary-encoded into SoA columns (source key id, PACKET_*
code, peer key id, port, type, PodHostIP / RemoteAddr ids), igx_np_mark evaluates the
filter and a (src, pkt, peer, port) distinct table keeps each tuple's first event index.
Only the distinct tuples (≈10M for 1B events) come back to the host
to become rules.  sort.Slice on equal policy names is unstable in Go (App. B); here the
sort is stable over sources in first-occurrence order.
"""
from __future__ import annotations

import json
import re

from . import _abi, engine
from .runtime import torch_mod

DEFAULT_LABELS_TO_IGNORE = frozenset({"controller-revision-hash", "pod-template-generation",
                                      "pod-template-hash"})
PKT_CODE = {"HOST": 0, "OUTGOING": 4}     # Linux PACKET_* values; anything else -> 1


class NetworkPolicyAdvisor:
    def __init__(self):
        self.Events = []
        self.LabelsToIgnore = set(DEFAULT_LABELS_TO_IGNORE)
        self.Policies = []

    # ---- input (advisor.go:56-100) ------------------------------------------------------
    def LoadFile(self, filename):
        with open(filename, "rb") as f:
            self.LoadBuffer(f.read())

    def LoadBuffer(self, buf):
        text = buf.decode() if isinstance(buf, (bytes, bytearray)) else buf
        try:
            ev = json.loads(text)
            if isinstance(ev, list):
                self.Events = ev
                return
        except ValueError:
            pass
        events, line = [], 0
        for raw in text.splitlines():
            t = raw.strip()
            if not t:
                continue
            line += 1
            try:
                events.append(json.loads(t))
            except ValueError as e:
                raise ValueError(f"cannot parse line {line}: {e}") from None
        self.Events = events

    # ---- keys (advisor.go:104-160) ------------------------------------------------------
    def labelFilteredKeyList(self, labels):
        return sorted(k for k in (labels or {}) if k not in self.LabelsToIgnore)

    def labelFilter(self, labels):
        return {k: v for k, v in (labels or {}).items() if k not in self.LabelsToIgnore}

    def labelKeyString(self, labels):
        return ",".join(f"{k}={labels[k]}" for k in self.labelFilteredKeyList(labels))

    def localPodKey(self, e):
        return e.get("namespace", "") + ":" + self.labelKeyString(e.get("podLabels"))

    def networkPeerKey(self, e):
        kind = e.get("remoteKind", "")
        if kind in ("pod", "svc"):
            ret = kind + ":" + e.get("remoteNamespace", "") + ":" + self.labelKeyString(e.get("remoteLabels"))
        elif kind == "other":
            ret = kind + ":" + e.get("remoteAddr", "")
        else:
            ret = ""
        return f"{ret}:{int(e.get('port', 0))}"

    # ---- device stage ---------------------------------------------------------------------
    def encode(self):
        """Dictionary-encode the events into the SoA columns the kernels read (numpy)."""
        import numpy as np
        n = len(self.Events)
        cols = {"src": np.zeros(n, np.uint32), "pkt": np.zeros(n, np.uint8),
                "peer": np.zeros(n, np.uint32), "port": np.zeros(n, np.uint16),
                "type": np.zeros(n, np.uint8), "hostip": np.zeros(n, np.uint32),
                "raddr": np.zeros(n, np.uint32)}
        src_ids, peer_ids, addr_ids = {}, {}, {}
        for i, e in enumerate(self.Events):
            cols["type"][i] = 0 if e.get("type") == "normal" else 1
            cols["pkt"][i] = PKT_CODE.get(e.get("pktType", ""), 1)
            cols["hostip"][i] = addr_ids.setdefault(e.get("podHostIP", ""), len(addr_ids))
            cols["raddr"][i] = addr_ids.setdefault(e.get("remoteAddr", ""), len(addr_ids))
            cols["src"][i] = src_ids.setdefault(self.localPodKey(e), len(src_ids))
            cols["peer"][i] = peer_ids.setdefault(self.networkPeerKey(e), len(peer_ids))
            cols["port"][i] = int(e.get("port", 0)) & 0xFFFF
        return cols

    def distinct_tuples(self):
        """(src, pkt, first event index) of every distinct kept (src, pkt, peer, port),
        computed by igx_np_mark + an igx distinct table.  Sorted by first index."""
        import numpy as np
        from . import columns as H
        n = len(self.Events)
        if n == 0:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint8), np.zeros(0, np.uint64)
        enc = self.encode()
        ev = {k: H.to_device(v) for k, v in enc.items()}
        keep = engine.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
        # distinct only: graph.c:102-114 inserts with BPF_NOEXIST and the advisor keeps the first
        # event per tuple (advisor.go:307-319); nothing is counted
        tab = engine.Table([4, 1, 4, 2], [], n)
        try:
            tab.update([ev["src"], ev["pkt"], ev["peer"], ev["port"]], [0, 1, 2, 3], n, 0, valid=keep)
            fin = tab.finalize()
            keys, _, first = engine.table_tensors(tab, fin)
        finally:
            tab.destroy()
        k = H.host(keys)
        f = H.host(first)
        order = np.argsort(f, kind="stable")
        src = k[:, 0:4].copy().view(np.uint32).ravel()[order]
        pkt = k[:, 4].copy()[order]
        return src, pkt, f[order]

    # ---- policies (advisor.go:162-372) ----------------------------------------------------
    def eventToRule(self, e):
        port = int(e.get("port", 0))
        ports = [{"port": port, "protocol": e.get("proto", "").upper()}]
        kind = e.get("remoteKind", "")
        rns = e.get("remoteNamespace", "")
        if kind in ("pod", "svc"):
            labels = self.labelFilter(e.get("remoteLabels")) if kind == "pod" else (e.get("remoteLabels") or {})
            peer = {"podSelector": _selector(labels)}
            if e.get("namespace", "") != rns:
                peer["namespaceSelector"] = {"matchLabels": {"kubernetes.io/metadata.name": rns}}
            peers = [peer]
        elif kind == "other":
            ra = e.get("remoteAddr", "")
            peers = [] if ra == "127.0.0.1" else [{"ipBlock": {"cidr": ra + "/32"}}]
        else:
            raise ValueError("unknown event")
        return ports, peers

    def GeneratePolicies(self):
        self.BuildPolicies(*self.distinct_tuples())

    def BuildPolicies(self, src, pkt, first):
        """Host half of GeneratePolicies from the distinct kept tuples (sorted by first)."""
        per_src = {}                     # src id -> [first event index of each kept tuple]
        for s, p, f in zip(src.tolist(), pkt.tolist(), first.tolist()):
            per_src.setdefault(s, []).append((p, f))
        policies = []
        for s, tuples in per_src.items():            # sources in first-occurrence order
            e0 = self.Events[tuples[0][1]]           # events[0] of the source
            egress, ingress = [], []
            for p, f in tuples:
                ports, peers = self.eventToRule(self.Events[f])
                if not peers:
                    continue
                if p == PKT_CODE["OUTGOING"]:
                    egress.append({"ports": ports, "to": peers})
                else:
                    ingress.append({"ports": ports, "from": peers})
            name = (e0.get("podOwner") or e0.get("pod", "")) + "-network"
            spec = {"podSelector": _selector(self.labelFilter(e0.get("podLabels"))),
                    "policyTypes": ["Ingress", "Egress"]}
            if ingress:
                spec["ingress"] = _sort_rules(ingress)
            if egress:
                spec["egress"] = _sort_rules(egress)
            policies.append({"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
                             "metadata": {"creationTimestamp": None, "name": name,
                                          "namespace": e0.get("namespace", "")},
                             "spec": spec, "status": {}})
        policies.sort(key=lambda p: p["metadata"]["name"])
        self.Policies = policies

    def FormatPolicies(self):
        return "---\n".join(to_yaml(p) for p in self.Policies)


def _selector(labels):
    return {"matchLabels": dict(labels)} if labels else {}


def _sort_rules(rules):
    """sortIngressRules / sortEgressRules (advisor.go:218-275): protocol, port, YAML text."""
    return sorted(rules, key=lambda r: (r["ports"][0]["protocol"], r["ports"][0]["port"], to_yaml(r)))


# ---- sigs.k8s.io/yaml (JSON -> go-yaml v2) emission for the values built above -----------
_PLAIN_OK = re.compile(r"^[A-Za-z0-9_./][A-Za-z0-9_./ -]*$")
_RESOLVES = re.compile(r"^(?:[-+]?(?:\d[\d_]*(?:\.\d*)?|\.\d+)(?:[eE][-+]?\d+)?|0x[0-9a-fA-F_]+|0o?[0-7_]+|"
                       r"0b[01_]+|[-+]?\.(?:inf|Inf|INF)|\.(?:nan|NaN|NAN)|~|null|Null|NULL|"
                       r"y|Y|yes|Yes|YES|n|N|no|No|NO|true|True|TRUE|false|False|FALSE|on|On|ON|"
                       r"off|Off|OFF)$")


def _scalar(v):
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    s = str(v)
    if s == "":
        return '""'
    if _RESOLVES.match(s):
        return '"' + s + '"'
    if _PLAIN_OK.match(s) and not s.endswith(" ") and ": " not in s and " #" not in s:
        return s
    return "'" + s.replace("'", "''") + "'"


def _emit(v, indent, out):
    pad = " " * indent
    if isinstance(v, dict):
        for k in sorted(v):
            x = v[k]
            if isinstance(x, dict) and x:
                out.append(f"{pad}{_scalar(k)}:")
                _emit(x, indent + 2, out)
            elif isinstance(x, list) and x:
                out.append(f"{pad}{_scalar(k)}:")
                _emit(x, indent, out)
            else:
                out.append(f"{pad}{_scalar(k)}: {_leaf(x)}")
    elif isinstance(v, list):
        for x in v:
            if isinstance(x, (dict, list)) and x:
                sub = []
                _emit(x, indent + 2, sub)
                sub[0] = pad + "- " + sub[0][indent + 2:]
                out.extend(sub)
            else:
                out.append(f"{pad}- {_leaf(x)}")


def _leaf(x):
    if isinstance(x, dict):
        return "{}"
    if isinstance(x, list):
        return "[]"
    return _scalar(x)


def to_yaml(v):
    out = []
    _emit(v, 0, out)
    return "\n".join(out) + "\n"
