"""advise network-policy: the reference's golden YAML (advisor_test.go TestLoad over
testdata/*.input|golden, copied as data into tests/golden/advisor/) and synthetic streams.

CPU tests pin the oracle restatement (oracle.advisor_policies) and the product's host stage
(encode -> BuildPolicies -> FormatPolicies) with the oracle standing in for the device
dedup; the GPU test runs the product end to end (igx_np_mark + igx distinct table).
"""
import glob
import json
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "advisor", "*.input")))


def _golden(path):
    return open(path[: -len(".input")] + ".golden").read()


def _oracle_tuples(oracle, adv):
    """oracle stand-in for the device stage: distinct kept (src, pkt, peer, port), first idx."""
    enc = adv.encode()
    if len(adv.Events) == 0:
        return np.zeros(0, np.uint32), np.zeros(0, np.uint8), np.zeros(0, np.uint64)
    names = ("src", "pkt", "peer", "port")
    keys, _, first = oracle.groupby(oracle.pack_cols(enc, names), [{"kind": "count"}],
                                    valid=oracle.np_mark(enc))
    return keys[:, 0:4].copy().view(np.uint32).ravel(), keys[:, 4].copy(), first


def synthetic_events(seed, n):
    r = random.Random(seed)
    nss = ["default", "shop", "kube-system"]
    labels = [{"app": "web", "pod-template-hash": "abc"}, {"app": "db", "tier": "backend"},
              {"app": "cache"}, {}, {"k8s-app": "kube-dns", "controller-revision-hash": "1"}]
    ev = []
    for _ in range(n):
        kind = r.choice(["pod", "svc", "other", "other"])
        e = {"type": r.choice(["normal"] * 20 + ["debug"]), "node": "n1",
             "namespace": r.choice(nss), "pod": "p%d" % r.randrange(6),
             "pktType": r.choice(["HOST", "OUTGOING", "OUTGOING", "MULTICAST"]),
             "proto": r.choice(["tcp", "udp"]), "port": r.choice([53, 80, 443, 8080, 5432]),
             "remoteKind": kind, "podHostIP": "192.168.0.%d" % r.randrange(3)}
        if r.random() < 0.5:
            e["podLabels"] = dict(r.choice(labels))
        if r.random() < 0.3:
            e["podOwner"] = "owner%d" % r.randrange(3)
        if kind in ("pod", "svc"):
            e["remoteNamespace"] = r.choice(nss)
            e["remoteName"] = "r%d" % r.randrange(4)
            if r.random() < 0.7:
                e["remoteLabels"] = dict(r.choice(labels))
            e["remoteAddr"] = "10.0.0.%d" % r.randrange(8)
        else:
            e["remoteAddr"] = r.choice(["127.0.0.1", "192.168.0.1", "8.8.8.8", "1.1.1.%d" % r.randrange(5)])
        ev.append(e)
    return ev


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_oracle_matches_reference_golden(oracle, path):
    a = json.loads(open(path).read()) if open(path).read().strip().startswith("[") else \
        [json.loads(l) for l in open(path) if l.strip()]
    out = "---\n".join(oracle.yaml_text(p) for p in oracle.advisor_policies(a))
    assert out == _golden(path)


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_host_stage_matches_reference_golden(igx, oracle, path):
    adv = igx.advisor.NetworkPolicyAdvisor()
    adv.LoadFile(path)
    adv.BuildPolicies(*_oracle_tuples(oracle, adv))
    assert adv.FormatPolicies() == _golden(path)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_stage_synthetic(igx, oracle, seed):
    ev = synthetic_events(seed, 400)
    adv = igx.advisor.NetworkPolicyAdvisor()
    adv.LoadBuffer("\n".join(json.dumps(e) for e in ev))
    adv.BuildPolicies(*_oracle_tuples(oracle, adv))
    ref = oracle.advisor_policies(ev)
    assert adv.Policies == ref
    assert adv.FormatPolicies() == "---\n".join(oracle.yaml_text(p) for p in ref)


def test_load_errors(igx):
    adv = igx.advisor.NetworkPolicyAdvisor()
    with pytest.raises(ValueError, match="cannot parse line 2"):
        adv.LoadBuffer('{"type":"normal"}\n{bad\n')


@pytest.mark.gpu
def test_device_dedup_end_to_end(igx, oracle):
    for path in GOLDEN:
        adv = igx.advisor.NetworkPolicyAdvisor()
        adv.LoadFile(path)
        adv.GeneratePolicies()
        assert adv.FormatPolicies() == _golden(path), path
    ev = synthetic_events(7, 5000)
    adv = igx.advisor.NetworkPolicyAdvisor()
    adv.LoadBuffer(json.dumps(ev))
    adv.GeneratePolicies()
    assert adv.Policies == oracle.advisor_policies(ev)


def test_string_keyed_generate_policies_counts_the_device_tuples(oracle):
    """C4's CPU baseline (or_np_advise_strings: GeneratePolicies on localPodKey / networkPeerKey
    strings, advisor.go:130-159, 279-320) keeps exactly the (source, direction, peer, port)
    tuples the device's distinct table counts on the same stream."""
    h = oracle.gen_np(0xC4, 10_000, 100_000, 0, 300_000)
    keys = oracle.pad_keys(h, ("src", "pkt", "peer", "port"))
    k, _, _ = oracle.groupby(keys, [], valid=oracle.np_mark(h))
    assert oracle.np_advise_strings(h) == k.shape[0] > 250_000
