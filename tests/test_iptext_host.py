"""The oracle's restatement of netip Addr.String (oracle.ip_string), used to check
igx_ip_text: cross-checked against Python's ipaddress (same RFC 5952 rules for plain IPv6),
plus Go's known answers where Python differs (IPv4-mapped addresses print dotted in Go)."""
import ipaddress

import numpy as np


def test_ip_string_known_answers(oracle):
    s = oracle.ip_string
    assert s(bytes([10, 1, 2, 3]) + bytes(12), 2) == "10.1.2.3"
    assert s(bytes([10, 1, 2, 3]) + bytes(12), 0) == "10.1.2.3"        # ipType 4 unless AF_INET6
    assert s(bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 1]), 10) == "::ffff:10.0.0.1"
    assert s(bytes(16), 10) == "::"
    assert s(bytes(15) + b"\x01", 10) == "::1"
    assert s(ipaddress.IPv6Address("1:0:1::1:0:0").packed, 10) == "1:0:1::1:0:0"   # first longest run
    assert s(ipaddress.IPv6Address("2001:db8:0:1:1:1:1:1").packed, 10) == "2001:db8:0:1:1:1:1:1"


def test_ip_string_matches_rfc5952(oracle):
    rng = np.random.default_rng(2)
    for _ in range(20000):
        g = rng.integers(0, 3, 8)
        v = rng.integers(0, 65536, 8) * (g > 0)
        b = b"".join(int(x).to_bytes(2, "big") for x in v)
        if b[:10] == bytes(10) and b[10:12] == b"\xff\xff":
            continue
        assert oracle.ip_string(b, 10) == str(ipaddress.IPv6Address(b))
