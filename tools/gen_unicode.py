"""Generates inspektor-gadget_amd/csrc/igx_unicode.h: the Unicode tables the regex compiler
(igx_regex.cpp) needs for Go regexp parity -- general-category ranges (\\p{L}, \\pN, ...) and
simple case-fold orbits ((?i) on non-ASCII runes) and the Unicode 13.0.0 scripts (\\p{Greek}).

Go 1.19's regexp uses package unicode at Unicode 13.0.0; this script requires the same
version from Python's unicodedata.  Fold orbits follow Go's unicode.SimpleFold: runes whose
simple case folding (CaseFolding.txt status C + S) is equal.  unicodedata has no simple
folding, so it is recovered as str.casefold() when that is one rune (status C), else
str.lower() when that is one rune (the status-S entries: U+1E9E -> U+00DF, the Greek
iota-subscript capitals), else the rune itself (no simple folding: U+0130, U+0131 keep their
own one-rune orbits, as in Go's caseOrbit table).
Scripts: Go 1.19's unicode.Scripts holds the 156 scripts of Unicode 13.0.0 (SCRIPTS below).
unicodedata has no script property, so each rune's script comes from the `regex` module's
\\p{Script=...} (a newer Unicode), kept only for runes that 13.0.0 assigns (category not Cn):
every such rune is in exactly one of the 156 (asserted).  Runes whose script changed after
13.0.0 would follow the newer data ("parity unpinned" for those).

    python3 tools/gen_unicode.py > inspektor-gadget_amd/csrc/igx_unicode.h
"""
import sys
import unicodedata
from collections import defaultdict

import regex   # script property data (newer Unicode; restricted below to what 13.0.0 assigns)

assert unicodedata.unidata_version == "13.0.0", unicodedata.unidata_version

CATS = ["Cc", "Cf", "Co", "Cs", "Ll", "Lm", "Lo", "Lt", "Lu", "Mc", "Me", "Mn", "Nd", "Nl", "No",
        "Pc", "Pd", "Pe", "Pf", "Pi", "Po", "Ps", "Sc", "Sk", "Sm", "So", "Zl", "Zp", "Zs"]
MAXRUNE = 0x10FFFF


def simple_fold(r):
    c = chr(r)
    f = c.casefold()
    if len(f) == 1:
        return ord(f)
    lo = c.lower()
    return ord(lo) if len(lo) == 1 else r


SCRIPTS = """Adlam Ahom Anatolian_Hieroglyphs Arabic Armenian Avestan Balinese Bamum Bassa_Vah Batak Bengali
Bhaiksuki Bopomofo Brahmi Braille Buginese Buhid Canadian_Aboriginal Carian Caucasian_Albanian Chakma Cham Cherokee
Chorasmian Common Coptic Cuneiform Cypriot Cyrillic Deseret Devanagari Dives_Akuru Dogra Duployan Egyptian_Hieroglyphs
Elbasan Elymaic Ethiopic Georgian Glagolitic Gothic Grantha Greek Gujarati Gunjala_Gondi Gurmukhi Han Hangul
Hanifi_Rohingya Hanunoo Hatran Hebrew Hiragana Imperial_Aramaic Inherited Inscriptional_Pahlavi Inscriptional_Parthian
Javanese Kaithi Kannada Katakana Kayah_Li Kharoshthi Khitan_Small_Script Khmer Khojki Khudawadi Lao Latin Lepcha Limbu
Linear_A Linear_B Lisu Lycian Lydian Mahajani Makasar Malayalam Mandaic Manichaean Marchen Masaram_Gondi Medefaidrin
Meetei_Mayek Mende_Kikakui Meroitic_Cursive Meroitic_Hieroglyphs Miao Modi Mongolian Mro Multani Myanmar Nabataean
Nandinagari New_Tai_Lue Newa Nko Nushu Nyiakeng_Puachue_Hmong Ogham Ol_Chiki Old_Hungarian Old_Italic Old_North_Arabian
Old_Permic Old_Persian Old_Sogdian Old_South_Arabian Old_Turkic Oriya Osage Osmanya Pahawh_Hmong Palmyrene Pau_Cin_Hau
Phags_Pa Phoenician Psalter_Pahlavi Rejang Runic Samaritan Saurashtra Sharada Shavian Siddham SignWriting Sinhala
Sogdian Sora_Sompeng Soyombo Sundanese Syloti_Nagri Syriac Tagalog Tagbanwa Tai_Le Tai_Tham Tai_Viet Takri Tamil Tangut
Telugu Thaana Thai Tibetan Tifinagh Tirhuta Ugaritic Vai Wancho Warang_Citi Yezidi Yi Zanabazar_Square""".split()


def script_ranges():
    """[(lo, hi, script index)] of every rune Unicode 13.0.0 assigns, in rune order."""
    assert len(SCRIPTS) == len(set(SCRIPTS)) == 156
    s = "".join(chr(c) for c in range(MAXRUNE + 1))
    owner = {}
    for k, name in enumerate(SCRIPTS):
        for m in regex.finditer(r"\p{Script=" + name + r"}+", s):
            for c in range(m.start(), m.end()):
                if unicodedata.category(chr(c)) != "Cn":
                    assert c not in owner, (name, hex(c))
                    owner[c] = k
    for c in range(MAXRUNE + 1):   # every assigned rune but private use / surrogates has a script
        assert (c in owner) == (unicodedata.category(chr(c)) not in ("Cn", "Co", "Cs")), hex(c)
    out, cur = [], None
    for c in sorted(owner):
        if cur and cur[1] == c - 1 and cur[2] == owner[c]:
            cur[1] = c
        else:
            if cur:
                out.append(tuple(cur))
            cur = [c, c, owner[c]]
    out.append(tuple(cur))
    return out


def main():
    # general-category ranges (unassigned Cn is not a class in Go's unicode.Categories)
    ranges = []
    cur = None
    for r in range(MAXRUNE + 1):
        cat = unicodedata.category(chr(r))
        k = CATS.index(cat) if cat in CATS else -1
        if cur and cur[2] == k and cur[1] == r - 1:
            cur[1] = r
        else:
            if cur and cur[2] >= 0:
                ranges.append(tuple(cur))
            cur = [r, r, k]
    if cur and cur[2] >= 0:
        ranges.append(tuple(cur))
    # fold orbits
    orbit = defaultdict(list)
    for r in range(MAXRUNE + 1):
        if 0xD800 <= r <= 0xDFFF:
            continue
        orbit[simple_fold(r)].append(r)
    folds = sorted((r, key) for key, rs in orbit.items() if len(rs) > 1 for r in rs)
    out = sys.stdout
    out.write("// igx_unicode.h -- GENERATED by tools/gen_unicode.py from Python's unicodedata (Unicode 13.0.0,\n"
              "// the version of Go 1.19's package unicode).  Do not edit.\n#pragma once\n#include <cstdint>\n\n")
    out.write("namespace igx_unicode {\n\n")
    out.write("// two-letter general categories, indexed by UCatRange::cat\n")
    out.write("static const char *const kCats[] = {" + ", ".join(f'"{c}"' for c in CATS) + "};\n")
    out.write(f"static constexpr int kNumCats = {len(CATS)};\n\n")
    out.write("struct UCatRange { uint32_t lo, hi; uint8_t cat; };\n")
    out.write(f"// every assigned rune, in rune order ({len(ranges)} ranges)\n")
    out.write("static const UCatRange kCatRanges[] = {\n")
    for i in range(0, len(ranges), 4):
        out.write("    " + " ".join(f"{{0x{a:X}, 0x{b:X}, {k}}}," for a, b, k in ranges[i:i + 4]) + "\n")
    out.write("};\n\n")
    out.write("struct UFold { uint32_t r, key; };\n")
    out.write(f"// runes with a non-trivial simple-fold orbit, by rune; equal keys = one orbit ({len(folds)})\n")
    out.write("static const UFold kFolds[] = {\n")
    for i in range(0, len(folds), 6):
        out.write("    " + " ".join(f"{{0x{r:X}, 0x{k:X}}}," for r, k in folds[i:i + 6]) + "\n")
    out.write("};\n\n")
    scr = script_ranges()
    out.write("// Unicode 13.0.0 scripts (Go 1.19 unicode.Scripts), indexed by UScriptRange::script\n")
    out.write("static const char *const kScripts[] = {\n")
    for i in range(0, len(SCRIPTS), 6):
        out.write("    " + " ".join(f'"{n}",' for n in SCRIPTS[i:i + 6]) + "\n")
    out.write("};\n")
    out.write(f"static constexpr int kNumScripts = {len(SCRIPTS)};\n")
    out.write("struct UScriptRange { uint32_t lo, hi; uint8_t script; };\n")
    out.write(f"// every rune with a script, in rune order ({len(scr)} ranges)\n")
    out.write("static const UScriptRange kScriptRanges[] = {\n")
    for i in range(0, len(scr), 4):
        out.write("    " + " ".join(f"{{0x{a:X}, 0x{b:X}, {k}}}," for a, b, k in scr[i:i + 4]) + "\n")
    out.write("};\n\n}  // namespace igx_unicode\n")


if __name__ == "__main__":
    main()
