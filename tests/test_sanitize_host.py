"""The host parsers of libigx under AddressSanitizer + UndefinedBehaviorSanitizer (a separate
host build, tests/sanitize/Makefile): igx_filter_parse over every filter_test.go row
(tests/golden/filter_table.json), igx_regex_compile_blob over the regex tests' patterns,
igx_sort_prepare over sort_test.go-style sortBy lists, then seeded random patterns and filter
strings.  Any sanitizer report fails the run (-fno-sanitize-recover, non-zero exit)."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


def _corpus(path):
    g = json.load(open(os.path.join(HERE, "golden", "filter_table.json")))
    from test_regex_host import ASSERT_PATTERNS, FOLD_PATTERNS, PATTERNS
    lines = [f"F\t{r['filter']}" for r in g["rows"]]
    lines += [f"R\t{p}" for p in PATTERNS + ASSERT_PATTERNS + FOLD_PATTERNS]
    lines += ["R\t\\p{Greek}", "R\t[[:alpha:][:^digit:]]{2,5}", "R\t\\Qa.b\\E\\101", "R\t(?m)^$|\\b\\B"]
    lines += ["S\tint,-uint8,nope,virt,ext", "S\t,-,--int", "S\tstring,-string,float64,bool"]
    with open(path, "w", encoding="utf-8") as fh:
        fh.write("\n".join(x.replace("\n", " ") for x in lines) + "\n")


@pytest.mark.timeout(600)
def test_host_parsers_under_asan_ubsan(tmp_path):
    b = subprocess.run(["make", "-s", "-C", SAN], capture_output=True, text=True, timeout=540)
    assert b.returncode == 0, b.stderr[-3000:]
    corpus = str(tmp_path / "corpus.txt")
    _corpus(corpus)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(SAN, "build", "san_main"), corpus], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and "SAN_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
