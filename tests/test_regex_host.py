"""The `~` filter's regex compiler (igx_regex.cpp) on the host: the compiled automaton
(igx_regex_compile_blob), stepped here exactly as the device steps it (k_common.h
regex_match), must agree with a regular-expression search on every string.  The reference
is Go's regexp (RE2); the cross-check uses Python's `re` on patterns and texts where the two
agree (ASCII classes, `$` written as `\\Z` for Python, valid UTF-8 texts), plus known answers
for Go-specific behaviour: invalid UTF-8 bytes are one U+FFFD rune each, (?i)k matches the
Kelvin sign, `$` does not match before a final newline."""
import ctypes as C
import re
import struct

import numpy as np
import pytest


def compile_blob(igx, pattern: bytes):
    L = igx.lib()
    n = C.c_size_t()
    err = C.create_string_buffer(256)
    rc = L.igx_regex_compile_blob(pattern, len(pattern), None, 0, C.byref(n), err, 256)
    if rc:
        return rc, err.value.decode()
    buf = (C.c_uint8 * n.value)()
    rc = L.igx_regex_compile_blob(pattern, len(pattern), buf, n.value, C.byref(n), err, 256)
    assert rc == 0
    return 0, bytes(buf)


def decode_rune(s, i):
    """utf8.DecodeRune: (rune, width); invalid -> (0xFFFD, 1)."""
    c0 = s[i]
    rem = len(s) - i
    if c0 < 0x80:
        return c0, 1
    if 0xC2 <= c0 <= 0xDF and rem >= 2 and (s[i + 1] & 0xC0) == 0x80:
        return ((c0 & 0x1F) << 6) | (s[i + 1] & 0x3F), 2
    if 0xE0 <= c0 <= 0xEF and rem >= 3:
        lo, hi = (0xA0 if c0 == 0xE0 else 0x80), (0x9F if c0 == 0xED else 0xBF)
        if lo <= s[i + 1] <= hi and (s[i + 2] & 0xC0) == 0x80:
            return ((c0 & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F), 3
    if 0xF0 <= c0 <= 0xF4 and rem >= 4:
        lo, hi = (0x90 if c0 == 0xF0 else 0x80), (0x8F if c0 == 0xF4 else 0xBF)
        if lo <= s[i + 1] <= hi and (s[i + 2] & 0xC0) == 0x80 and (s[i + 3] & 0xC0) == 0x80:
            return (((c0 & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6)
                    | (s[i + 3] & 0x3F)), 4
    return 0xFFFD, 1


def run_blob(blob, text: bytes, width=None):
    nstates, ncls, start, nbytes, ob, of, ot, _ = struct.unpack_from("<8I", blob, 0)
    ascii = blob[32:160]
    bounds = struct.unpack_from(f"<{ncls}I", blob, ob)
    flags = blob[of:of + nstates]
    trans = struct.unpack_from(f"<{nstates * ncls}H", blob, ot)
    s = text if width is None else text[:width]
    if b"\0" in s:
        s = s[:s.index(b"\0")]
    st = start
    if not s:
        return (flags[st] & 5) != 0
    if flags[st] & 1:
        return True
    i = 0
    while i < len(s):
        r, w = decode_rune(s, i)
        i += w
        if r < 128:
            cls = ascii[r]
        else:
            cls = max(k for k in range(ncls) if bounds[k] <= r)
        st = trans[st * ncls + cls]
        if flags[st] & 1:
            return True
    return (flags[st] & 2) != 0


PATTERNS = ["Demo", "demo", "(?i)demo", "^de", "mo$", "^$", "a*", "x+y", "colou?r", "gr[ae]y", "[^a-z]",
            r"\d{2,3}", r"^\w+@\w+\.com$", "a|b|cd", "(ab)+c", "(?:foo|bar)baz", "a.c", "a{3}", "a{2,}b",
            r"\s", r"[\d_-]+$", "(?i)k", "(?s)a.b", "x{0}y", "(a|)b", "[a-c]{1,2}x", r"\.", "é", "^.{2}$",
            "(?i)[a-f]+z", "(?i:ab)C", "(a*)*b", "^(?:ab|a)(?:bc|c)$", "z?$", "[]a]", "[^]a]"]
TEXTS = [b"", b"Demo", b"demo", b"a Demo b", b"DEMO", b"dem", b"aaa", b"xxyy", b"color", b"colour",
         b"grey", b"gray", b"ABC", b"12", b"1234", b"joe@x.com", b"joe@x.comz", b"cd", b"ababc",
         b"foobaz", b"barbaz", b"abc", b"aXc", b"a\nc", b"aaab", b"a b", b"_-9", b"K", b"k",
         "é".encode(), "aé".encode(), "éé".encode(), b"y", b"b", b"bx", b"abcx", b".", b"]", b"a",
         b"abc\n", b"\n"]


def py_re(p):
    """Python rendering of a Go pattern for this test's patterns ($ -> \\Z)."""
    return re.compile(p.replace("$", r"\Z"))


@pytest.mark.parametrize("pattern", PATTERNS)
def test_regex_dfa_matches_search(igx, pattern):
    rc, blob = compile_blob(igx, pattern.encode())
    assert rc == 0, blob
    pr = py_re(pattern)
    for t in TEXTS:
        want = pr.search(t.decode("utf-8")) is not None
        assert run_blob(blob, t) == want, (pattern, t)


def test_go_specific_known_answers(igx):
    ok = lambda p, t: run_blob(compile_blob(igx, p)[1], t)   # noqa: E731
    assert ok(b"(?i)k", "K".encode())            # Kelvin sign folds to k in Go
    assert ok(b"(?i)s", "ſ".encode())            # long s folds to s
    assert not ok(b"a$", b"a\n")                      # $ is end of text, not before a final \n
    assert ok(b"^.$", b"\xff")                        # an invalid byte is one rune
    assert not ok(b"^..$", b"\xc3")                   # a truncated sequence is one rune
    assert ok(b"^..$", b"\xc3(")                      # invalid lead byte + '(' = two runes
    assert ok(b"^.$", "é".encode())                   # one valid 2-byte rune
    assert ok(b"\xef\xbf\xbd", b"\xfe")               # U+FFFD literal matches an invalid byte
    assert ok(b"demo", b"demo\0junk")                 # the value ends at the first NUL
    assert not ok(b"junk", b"demo\0junk")


def test_regex_errors_and_unsupported(igx):
    assert compile_blob(igx, b"(?i)??//{demo")[0] == igx._abi.IGX_EINVAL
    assert compile_blob(igx, b"a(b")[0] == igx._abi.IGX_EINVAL
    assert compile_blob(igx, b"[a")[0] == igx._abi.IGX_EINVAL
    assert compile_blob(igx, b"*a")[0] == igx._abi.IGX_EINVAL
    assert compile_blob(igx, rb"[\b]")[0] == igx._abi.IGX_EINVAL      # no \b inside a class in RE2
    assert compile_blob(igx, rb"\1")[0] == igx._abi.IGX_EINVAL        # backreferences do not exist
    assert compile_blob(igx, rb"[[:nope:]]")[0] == igx._abi.IGX_EINVAL
    # neither a category nor a Unicode 13.0.0 script (names are case-sensitive in Go)
    for bad in (rb"\p{Klingon}", rb"\p{greek}", rb"\p{Vithkuqi}", rb"\pQ", rb"[\p{Nope}a]"):
        rc, msg = compile_blob(igx, bad)
        assert rc == igx._abi.IGX_EINVAL and "invalid character class range" in msg, (bad, msg)


# Unicode scripts (Go 1.19 unicode.Scripts, Unicode 13.0.0): cross-checked with the `regex`
# module's \p{Script=..} on texts of runes that 13.0.0 assigns.  Under (?i) Go also adds
# FoldScript (runes of other scripts whose fold orbit meets the script), which `regex` does
# not: those are known answers below.
SCRIPT_PATTERNS = [r"\p{Greek}", r"^\p{Greek}+$", r"\p{Han}", r"^\P{Latin}+$", r"\p{^Cyrillic}", r"^\p{Common}$",
                   r"\p{Arabic}[0-9]", r"[\p{Hiragana}\p{Katakana}]+", r"^\p{Inherited}$", r"[^\p{Hangul}\s]",
                   r"^[\p{Greek}\p{Latin}]+$"]
SCRIPT_TEXTS = ["α", "Ω", "abc", "漢字", "ひらがなカタカナ", "Привет", "µ", "\u0345", "K", "\u212a", "ſ", "ﬀ",
                "٣٤", "ب3", "한국어 ", "ǅ", "1", "", "αβγ1", "\u0300", "\u1f80", "ᾈ", "𐌰", "\U0001F600"]


def _py_script(p):
    import regex
    return regex.compile(p.replace(r"\p{", r"\p{Script=").replace(r"\P{", r"\P{Script=")
                         .replace(r"\p{Script=^", r"\P{Script=").replace("$", r"\Z"))


@pytest.mark.parametrize("pattern", SCRIPT_PATTERNS)
def test_regex_unicode_scripts(igx, pattern):
    rc, blob = compile_blob(igx, pattern.encode())
    assert rc == 0, blob
    pr = _py_script(pattern)
    for t in SCRIPT_TEXTS:
        t = t.encode().decode("unicode_escape") if "\\" in t else t
        assert run_blob(blob, t.encode()) == (pr.search(t) is not None), (pattern, t)


def test_regex_script_fold_known_answers(igx):
    r"""FoldScript: (?i)\p{Greek} takes the micro sign (Common) and U+0345 (Inherited), whose
    orbits meet Greek; (?i)\p{Latin} takes the Kelvin sign's K (already Latin) and not Greek."""
    ok = lambda p, t: run_blob(compile_blob(igx, p.encode())[1], t.encode())   # noqa: E731
    assert ok(r"(?i)^\p{Greek}$", "\u00b5") and not ok(r"^\p{Greek}$", "\u00b5")
    assert ok(r"(?i)^\p{Greek}$", "\u0345") and not ok(r"^\p{Greek}$", "\u0345")
    assert not ok(r"(?i)^\p{Latin}$", "α") and ok(r"(?i)^\P{Greek}$", "a")
    assert ok(r"(?i)^\p{Latin}$", "\u212a") and ok(r"(?i)^\p{Latin}+$", "ſK")      # both Latin already
    assert ok(r"(?i)^\p{Greek}+$", "ΑΩω") and ok(r"(?i)^\p{Cyrillic}$", "\u1c80")  # ᲀ (Cyrillic) folds to в


# Assertions and (?m): Python's re with re.ASCII has RE2's ASCII \b / \w and the same (?m)
# ^ / $ (line starts after '\n', line ends before '\n'); \z is Python's \Z.
ASSERT_PATTERNS = [r"\bfoo\b", r"\Bo\B", r"\bo", r"o\b", r"(?m)^a", r"(?m)b$", r"(?m)^$", r"\Afoo",
                   r"foo\z", r"(?m)^\w+$", r"x\b|\by", r"\b", r"\B", r"^\b$", r"(?m:^b)c", r"a\b\s",
                   r"(?m)a$\n^b", r"\d\b", r"(?m)\Ab"]
ASSERT_TEXTS = [b"", b"foo", b"a foo b", b"food", b"xfoo", b"foo_", b"o", b"ooo", b"a\nb", b"b\na", b"\n",
                b"\n\n", b"ab\ncd", b"x y", b"xy", b"a b", b"12 3", b"a\n", b"\nb", b"foo\n", b"bc", b"b\nbc",
                b" ", b"-", b"_x_"]


@pytest.mark.parametrize("pattern", ASSERT_PATTERNS)
def test_regex_assertions_match_search(igx, pattern):
    rc, blob = compile_blob(igx, pattern.encode())
    assert rc == 0, blob
    pr = re.compile(pattern.replace(r"\z", r"\Z"), re.ASCII)
    for t in ASSERT_TEXTS:
        want = pr.search(t.decode()) is not None
        if pattern == r"\B" and t == b"":
            want = True   # RE2: no word boundary between two non-word sides; Python's \B never matches ""
        assert run_blob(blob, t) == want, (pattern, t)


# Unicode case folding under (?i): Python's re in str mode folds with Unicode simple case
# folding too (same Unicode version, 13.0.0, as Go 1.19).
FOLD_PATTERNS = ["(?i)é", "(?i)straße", "(?i)[à-ö]+", "(?i)σ", "(?i)ǆ", "(?i)[a-z]", "(?i)ω", "(?i)k",
                 "(?i)i", "(?i)[^a-z]", "(?i)θ", "(?i)ꙋ"]
FOLD_TEXTS = ["É", "é", "e", "STRASSE", "STRAẞE", "straße", "ÀÖ", "àö", "×", "Σ", "ς", "σ", "ǅ", "Ǆ", "K",
              "Ω", "Ω", "ω", "I", "i", "ſ", "1", "", "ϑ", "ϴ", "Θ", "ᲈ", "Ꙋ"]


@pytest.mark.parametrize("pattern", FOLD_PATTERNS)
def test_regex_unicode_folding(igx, pattern):
    rc, blob = compile_blob(igx, pattern.encode())
    assert rc == 0, blob
    pr = re.compile(pattern)
    for t in FOLD_TEXTS:
        assert run_blob(blob, t.encode()) == (pr.search(t) is not None), (pattern, t)


def test_regex_dotted_i_known_answers(igx):
    """U+0130 and U+0131 have no simple case folding (CaseFolding.txt has only T / F entries),
    so Go's (?i)i matches neither -- Python's re, which lower-cases, differs here."""
    ok = lambda p, t: run_blob(compile_blob(igx, p.encode())[1], t.encode())   # noqa: E731
    assert not ok("(?i)i", "İ") and not ok("(?i)i", "ı") and not ok("(?i)[a-z]", "İ")
    assert ok("(?i)ı", "ı") and not ok("(?i)ı", "I") and ok("(?i)İ", "İ") and not ok("(?i)İ", "i")


def test_regex_classes_known_answers(igx):
    r"""\p{..} general categories, POSIX classes, \Q..\E and octal escapes (Go regexp
    semantics; parity unpinned by reference vectors -- Go is not in this image)."""
    ok = lambda p, t: run_blob(compile_blob(igx, p.encode())[1], t.encode())   # noqa: E731
    assert ok(r"^\pL+$", "héllo") and not ok(r"^\pL+$", "h3llo")
    assert ok(r"^\p{Lu}", "Émile") and not ok(r"^\p{Lu}", "émile")
    assert ok(r"^\p{^Lu}", "émile") and ok(r"^\PL", "3a") and not ok(r"^\PL", "a3")
    assert ok(r"\p{Nd}", "٣") and not ok(r"\pN", "abc") and ok(r"\pN", "½")
    assert ok(r"^\p{Any}$", "€") and ok(r"\p{Zs}", "a\u00a0b") and ok(r"^\p{Sc}$", "€")
    assert ok(r"(?i)\p{Lu}", "é")                    # Go folds \p classes under (?i)
    assert ok(r"^[[:alpha:]]+$", "abcXYZ") and not ok(r"^[[:alpha:]]+$", "abc1")
    assert ok(r"^[[:^digit:]]+$", "abc") and not ok(r"[[:^digit:]]", "123")
    assert ok(r"^[[:xdigit:][:space:]]+$", "dead beef") and not ok(r"[[:upper:]]", "abc")
    assert ok(r"(?i)[[:upper:]]", "abc")              # folded, like Go
    assert ok(r"(?i)\w", "\u212a") and not ok(r"\w", "\u212a")   # K folds to k, \w is ASCII
    assert ok(r"\Qa.b*\E", "xa.b*y") and not ok(r"\Qa.b*\E", "aab")
    assert ok(r"^\101\060$", "A0") and ok(r"^\x{20ac}$", "€")   # octal escapes; values end at NUL


def test_filter_table_regex_rows_on_the_automaton(igx):
    """filter_test.go:139-143 over the reference table's 5 string values
    (tests/golden/filter_table.json)."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "filter_table.json")))
    strings = [r["string"] for r in g["records"] if r is not None]
    for row in g["rows"]:
        f = row["filter"]
        if not f.startswith("string:") or "~" not in f or row["error"]:
            continue
        rule = f[len("string:"):]
        neg = rule.startswith("!")
        pat = rule.lstrip("!")[1:]
        rc, blob = compile_blob(igx, pat.encode())
        assert rc == 0
        cnt = sum(run_blob(blob, s.encode()) != neg for s in strings)
        assert cnt == row["count"], f


def test_regex_script_table_boundaries(igx):
    r"""Fixed boundary runes of the generated script tables (tools/gen_unicode.py, Unicode
    13.0.0 = Go 1.19's unicode.Version; Python 3.10's unicodedata is also 13.0.0, which names
    the assigned runes used here).  Han ends at U+9FFC in 13.0 (U+9FFD is 14.0); Inherited
    runs U+0300-U+036F and U+0370 is Greek; '@' is Common and 'A' Latin; U+1F978 (13.0) is
    Common while U+1FAE0 (14.0) is unassigned, so neither Common nor any other script."""
    ok = lambda p, r: run_blob(compile_blob(igx, p.encode())[1], chr(r).encode())   # noqa: E731
    assert ok(r"^\p{Han}$", 0x9FFC) and not ok(r"^\p{Han}$", 0x9FFD) and ok(r"^\p{Han}$", 0x4E00)
    assert ok(r"^\p{Han}$", 0x3400) and not ok(r"^\p{Han}$", 0x33FF)
    assert ok(r"^\p{Inherited}$", 0x0300) and ok(r"^\p{Inherited}$", 0x036F)
    assert not ok(r"^\p{Inherited}$", 0x0370) and ok(r"^\p{Greek}$", 0x0370)
    assert not ok(r"^\p{Inherited}$", 0x02FF) and ok(r"^\p{Common}$", 0x02FF)
    assert ok(r"^\p{Common}$", 0x40) and not ok(r"^\p{Common}$", 0x41) and ok(r"^\p{Latin}$", 0x41)
    assert ok(r"^\p{Common}$", 0x1F978) and not ok(r"^\p{Common}$", 0x1FAE0)
    assert ok(r"^\P{Common}$", 0x1FAE0) and not ok(r"^\p{Han}$", 0x1FAE0)
