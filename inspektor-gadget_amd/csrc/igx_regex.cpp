// igx_regex.cpp -- RE2-syntax regular expressions compiled to a rune-class DFA for the
// device filter scan (the `~` rule of pkg/columns/filter/filter.go:119-127,212-216:
// regexp.Compile + MatchString(field) != negate).
//
// Semantics follow Go's regexp on a string: the text is a sequence of runes decoded with
// utf8.DecodeRune (an invalid byte is one U+FFFD rune), MatchString is an unanchored search,
// `.` is any rune but '\n' (any rune with (?s)), `^`/`$` are the text's ends, or line ends
// under (?m); \A \z \b \B are RE2's empty-width assertions (\b on ASCII word runes), \d \s
// \w and the [[:name:]] classes are ASCII as in RE2, \pN / \p{Name} are Unicode general
// categories or, after them, scripts (\p{Greek}; igx_unicode.h, Unicode 13.0.0 like Go 1.19),
// and (?i) folds every rune with its simple-fold orbit (k ↔ K ↔ U+212A, s ↔ S ↔ U+017F, ...)
// -- classes too, as Go's parser folds them (FoldCategory / FoldScript).  Syntax errors
// surface at igx_filter_parse.
//
// Pipeline: recursive-descent parse -> Thompson NFA over rune sets and empty-width
// assertions -> alphabet split into the elementary rune intervals the sets use (word runes
// and '\n' always get intervals of their own) -> subset construction.  A DFA state is a set
// of NFA states plus the context of the previous rune (start of text / '\n' / word rune /
// other): on the next rune the assertions that hold between the two are known, the set is
// closed over them and, if a match is complete there, the transition goes to the absorbing
// accept state; otherwise the search start is re-added.  Per state, bit1 of the flags says
// whether a match completes at the end of the text (`$`, `\z`, `\b` before the end).
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "igx_internal.h"
#include "igx_regex.h"
#include "igx_unicode.h"

namespace {

typedef std::vector<std::pair<uint32_t, uint32_t>> Ranges;   // [lo, hi] rune intervals, sorted

constexpr uint32_t MAXRUNE = 0x10FFFF;

Ranges normalize(Ranges r) {
    std::sort(r.begin(), r.end());
    Ranges o;
    for (auto &p : r) {
        if (!o.empty() && p.first <= o.back().second + 1) o.back().second = std::max(o.back().second, p.second);
        else o.push_back(p);
    }
    return o;
}

Ranges negate(const Ranges &r) {
    Ranges o;
    uint32_t next = 0;
    for (auto &p : r) {
        if (p.first > next) o.push_back({next, p.first - 1});
        next = p.second + 1;
    }
    if (next <= MAXRUNE) o.push_back({next, MAXRUNE});
    return o;
}

// simple-fold orbits (unicode.SimpleFold): rune -> orbit members, from igx_unicode.h
const std::map<uint32_t, std::vector<uint32_t>> &fold_orbits() {
    static const std::map<uint32_t, std::vector<uint32_t>> m = [] {
        std::map<uint32_t, std::vector<uint32_t>> by_key, by_rune;
        for (const auto &f : igx_unicode::kFolds) by_key[f.key].push_back(f.r);
        for (const auto &f : igx_unicode::kFolds) by_rune[f.r] = by_key[f.key];
        return by_rune;
    }();
    return m;
}

void add_fold(Ranges &r, uint32_t c) {
    r.push_back({c, c});
    const auto &m = fold_orbits();
    auto it = m.find(c);
    if (it != m.end())
        for (uint32_t o : it->second) r.push_back({o, o});
}

// a class under (?i): every rune's orbit (appendFoldedClass in Go's regexp/syntax)
Ranges fold_ranges(const Ranges &in) {
    Ranges r = in;
    const auto &m = fold_orbits();
    for (const auto &p : in)
        for (auto it = m.lower_bound(p.first); it != m.end() && it->first <= p.second; ++it)
            for (uint32_t o : it->second) r.push_back({o, o});
    return normalize(r);
}

// Go's regexp/syntax EmptyOp bits
enum : uint8_t { E_BEGIN_LINE = 1, E_END_LINE = 2, E_BEGIN_TEXT = 4, E_END_TEXT = 8, E_WORD = 16, E_NOWORD = 32 };

enum NType : uint8_t { N_SET, N_SPLIT, N_EPS, N_ASSERT, N_MATCH };
struct NState {
    NType t;
    int set = -1;        // rune-set id (N_SET); the EmptyOp (N_ASSERT)
    int out = -1, out2 = -1;
};

bool word_rune(uint32_t c) {
    return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
}

// \p{Name}: a general category (two letters, or one letter for the major class), or Any
bool unicode_class(const std::string &name, Ranges *out) {
    Ranges r;
    if (name == "Any") {
        *out = {{0, MAXRUNE}};
        return true;
    }
    bool any = false;
    for (int k = 0; k < igx_unicode::kNumCats; ++k) {
        const char *c = igx_unicode::kCats[k];
        if (name == c || (name.size() == 1 && name[0] == c[0])) {
            any = true;
            for (const auto &x : igx_unicode::kCatRanges)
                if (x.cat == k) r.push_back({x.lo, x.hi});
        }
    }
    // unicode.Scripts, looked up after the categories and case-sensitively, as Go 1.19's
    // regexp/syntax unicodeTable does; under (?i) group() adds the fold orbits (FoldScript)
    for (int k = 0; !any && k < igx_unicode::kNumScripts; ++k) {
        if (name != igx_unicode::kScripts[k]) continue;
        any = true;
        for (const auto &x : igx_unicode::kScriptRanges)
            if (x.script == k) r.push_back({x.lo, x.hi});
    }
    if (!any) return false;
    *out = normalize(r);
    return true;
}

// [[:name:]] (RE2's ASCII POSIX classes)
bool posix_class(const std::string &name, Ranges *out) {
    static const std::map<std::string, Ranges> t = {
        {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}}, {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
        {"ascii", {{0, 0x7F}}}, {"blank", {{'\t', '\t'}, {' ', ' '}}}, {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
        {"digit", {{'0', '9'}}}, {"graph", {{'!', '~'}}}, {"lower", {{'a', 'z'}}}, {"print", {{' ', '~'}}},
        {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}}, {"space", {{'\t', '\r'}, {' ', ' '}}},
        {"upper", {{'A', 'Z'}}}, {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
        {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}}};
    auto it = t.find(name);
    if (it == t.end()) return false;
    *out = normalize(it->second);
    return true;
}

struct Compiler {
    std::string re;
    size_t i = 0;
    bool icase = false, dotnl = false, multiline = false;
    std::string err;       // syntax error (parse) -> EINVAL
    bool unsup = false;    // valid RE2 we do not compile -> ENOTSUP
    std::vector<NState> st;
    std::vector<Ranges> sets;
    // dangling outs are kept as (state, which) pairs to survive vector growth
    struct Hole { int s; int which; };
    struct F { int start; std::vector<Hole> outs; };

    int add(NType t, int set = -1) {
        st.push_back(NState{t, set, -1, -1});
        return (int)st.size() - 1;
    }
    void patch(const std::vector<Hole> &h, int to) {
        for (auto &x : h) (x.which ? st[x.s].out2 : st[x.s].out) = to;
    }
    F single(NType t, int set = -1) {
        const int s = add(t, set);
        return F{s, {{s, 0}}};
    }
    F set_frag(Ranges r) {
        sets.push_back(normalize(std::move(r)));
        return single(N_SET, (int)sets.size() - 1);
    }
    F empty() { return single(N_EPS); }
    F assertion(uint8_t op) { return single(N_ASSERT, op); }
    F cat(F a, F b) {
        patch(a.outs, b.start);
        return F{a.start, b.outs};
    }
    F alt(F a, F b) {
        const int s = add(N_SPLIT);
        st[s].out = a.start;
        st[s].out2 = b.start;
        F f{s, a.outs};
        f.outs.insert(f.outs.end(), b.outs.begin(), b.outs.end());
        return f;
    }
    F star(F a) {
        const int s = add(N_SPLIT);
        st[s].out = a.start;
        patch(a.outs, s);
        return F{s, {{s, 1}}};
    }
    F plus(F a) {
        const int s = add(N_SPLIT);
        st[s].out = a.start;
        patch(a.outs, s);
        return F{a.start, {{s, 1}}};
    }
    F quest(F a) {
        const int s = add(N_SPLIT);
        st[s].out = a.start;
        F f{s, a.outs};
        f.outs.push_back({s, 1});
        return f;
    }

    bool eof() const { return i >= re.size(); }
    char peek() const { return re[i]; }

    // decode one UTF-8 rune of the pattern (Go: invalid pattern UTF-8 is an error)
    bool pat_rune(uint32_t *r) {
        const unsigned char c = (unsigned char)re[i];
        if (c < 0x80) { *r = c; ++i; return true; }
        int n = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
        if (!n || i + n > re.size()) { err = "invalid UTF-8"; return false; }
        uint32_t v = c & (0x7F >> n);
        for (int k = 1; k < n; ++k) v = (v << 6) | ((unsigned char)re[i + k] & 0x3F);
        i += n;
        *r = v;
        return true;
    }

    Ranges literal_set(uint32_t c) {
        Ranges r;
        if (icase) add_fold(r, c);
        else r.push_back({c, c});
        return r;
    }

    // a class escape or [:name:] group under the current flags (Go's appendGroup: folded
    // first, then negated)
    Ranges group(const Ranges &cls, bool neg) {
        const Ranges c = icase ? fold_ranges(cls) : normalize(cls);
        return neg ? negate(c) : c;
    }

    // \pN, \p{Name}, \p{^Name}, \PN (after the 'p' / 'P'); false with err / unsup set
    bool unicode_escape(bool neg, Ranges *out) {
        if (eof()) { err = "invalid character class range"; return false; }
        std::string name;
        if (peek() == '{') {
            const size_t e = re.find('}', i);
            if (e == std::string::npos) { err = "invalid character class range"; return false; }
            name = re.substr(i + 1, e - i - 1);
            i = e + 1;
        } else {
            uint32_t c;
            if (!pat_rune(&c)) return false;
            name = std::string(1, (char)c);
        }
        if (!name.empty() && name[0] == '^') {
            neg = !neg;
            name = name.substr(1);
        }
        Ranges r;
        if (!unicode_class(name, &r)) {   // neither a category nor a script: Go's ErrInvalidCharRange
            err = "invalid character class range";
            return false;
        }
        *out = group(r, neg);
        return true;
    }

    // escapes usable inside and outside classes; returns false with err/unsup set
    bool escape(Ranges *out, bool *is_class) {
        if (eof()) { err = "trailing backslash at end of expression"; return false; }
        const char c = re[i++];
        *is_class = true;
        const Ranges digit = {{'0', '9'}}, space = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}},
                     word = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
        switch (c) {
        case 'd': *out = group(digit, false); return true;
        case 'D': *out = group(digit, true); return true;
        case 's': *out = group(space, false); return true;
        case 'S': *out = group(space, true); return true;
        case 'w': *out = group(word, false); return true;
        case 'W': *out = group(word, true); return true;
        case 'p': return unicode_escape(false, out);
        case 'P': return unicode_escape(true, out);
        default: break;
        }
        *is_class = false;
        uint32_t v;
        switch (c) {
        case 't': v = '\t'; break;
        case 'n': v = '\n'; break;
        case 'r': v = '\r'; break;
        case 'f': v = '\f'; break;
        case 'v': v = '\v'; break;
        case 'a': v = 7; break;
        case '1': case '2': case '3': case '4': case '5': case '6': case '7':
            // a lone non-zero digit would be a backreference (not RE2); with more octal
            // digits it is an octal escape
            if (eof() || peek() < '0' || peek() > '7') { err = "invalid escape sequence"; return false; }
            [[fallthrough]];
        case '0': {
            v = (uint32_t)(c - '0');
            for (int k = 0; k < 2 && !eof() && peek() >= '0' && peek() <= '7'; ++k) v = v * 8 + (uint32_t)(re[i++] - '0');
            break;
        }
        case 'x': {
            auto hex = [](char h) { return h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 :
                                           h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1; };
            if (!eof() && peek() == '{') {
                ++i;
                v = 0;
                int nd = 0;
                while (!eof() && peek() != '}') {
                    const int d = hex(re[i++]);
                    if (d < 0) { err = "invalid escape sequence"; return false; }
                    v = v * 16 + d;
                    if (++nd > 8 || v > MAXRUNE) { err = "invalid escape sequence"; return false; }
                }
                if (eof() || !nd) { err = "invalid escape sequence"; return false; }
                ++i;
            } else {
                if (i + 2 > re.size() || hex(re[i]) < 0 || hex(re[i + 1]) < 0) { err = "invalid escape sequence"; return false; }
                v = hex(re[i]) * 16 + hex(re[i + 1]);
                i += 2;
            }
            break;
        }
        default:
            if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) {
                err = "invalid escape sequence";   // \b \B \A \z \Q are handled before this
                return false;
            }
            v = (unsigned char)c;   // escaped punctuation
        }
        *out = literal_set(v);
        return true;
    }

    bool cls(Ranges *out) {   // after '['
        bool neg = false;
        if (!eof() && peek() == '^') { neg = true; ++i; }
        Ranges r;
        bool first = true;
        while (!eof() && (peek() != ']' || first)) {
            first = false;
            if (peek() == '[' && i + 1 < re.size() && re[i + 1] == ':') {   // [:alpha:], [:^alpha:]
                const size_t e = re.find(":]", i + 2);
                if (e != std::string::npos) {
                    std::string name = re.substr(i + 2, e - i - 2);
                    bool pneg = false;
                    if (!name.empty() && name[0] == '^') { pneg = true; name = name.substr(1); }
                    Ranges g;
                    if (!posix_class(name, &g)) { err = "invalid character class range"; return false; }
                    const Ranges x = group(g, pneg);
                    r.insert(r.end(), x.begin(), x.end());
                    i = e + 2;
                    continue;
                }
            }
            uint32_t lo;
            if (peek() == '\\') {
                ++i;
                Ranges e;
                bool is_class;
                if (!escape(&e, &is_class)) return false;
                if (is_class) { r.insert(r.end(), e.begin(), e.end()); continue; }
                lo = e[0].first;
            } else if (!pat_rune(&lo)) {
                return false;
            }
            uint32_t hi = lo;
            if (i + 1 < re.size() && peek() == '-' && re[i + 1] != ']') {
                ++i;
                if (peek() == '\\') {
                    ++i;
                    Ranges e;
                    bool is_class;
                    if (!escape(&e, &is_class)) return false;
                    if (is_class) { err = "invalid character class range"; return false; }
                    hi = e[0].first;
                } else if (!pat_rune(&hi)) {
                    return false;
                }
                if (hi < lo) { err = "invalid character class range"; return false; }
            }
            if (icase) {
                const Ranges x = fold_ranges({{lo, hi}});
                r.insert(r.end(), x.begin(), x.end());
            } else {
                r.push_back({lo, hi});
            }
        }
        if (eof()) { err = "missing closing ]"; return false; }
        ++i;   // ']'
        r = normalize(r);
        *out = neg ? negate(r) : r;
        return true;
    }

    bool atom(F *f) {
        const char c = peek();
        if (c == '(') {
            ++i;
            bool save_i = icase, save_s = dotnl, save_m = multiline;
            if (!eof() && peek() == '?') {
                ++i;
                if (!eof() && (peek() == 'P' || peek() == '<')) {   // named group
                    while (!eof() && peek() != '>') ++i;
                    if (eof()) { err = "invalid named capture"; return false; }
                    ++i;
                } else {
                    bool on = true, any = false;
                    while (!eof() && peek() != ':' && peek() != ')') {
                        const char fc = re[i++];
                        any = true;
                        if (fc == '-') on = false;
                        else if (fc == 'i') icase = on;
                        else if (fc == 's') dotnl = on;
                        else if (fc == 'U') { /* ungreedy: no effect on match/no match */ }
                        else if (fc == 'm') multiline = on;
                        else { err = "invalid or unsupported Perl syntax"; return false; }
                    }
                    if (eof()) { err = "missing closing )"; return false; }
                    if (!any && peek() == ')') { err = "invalid or unsupported Perl syntax"; return false; }
                    if (peek() == ')') {   // flags for the rest of the enclosing group
                        ++i;
                        *f = empty();
                        return true;
                    }
                    ++i;   // ':'
                }
            }
            F inner;
            if (!alternation(&inner)) return false;
            if (eof() || peek() != ')') { err = "missing closing )"; return false; }
            ++i;
            icase = save_i;
            dotnl = save_s;
            multiline = save_m;
            *f = inner;
            return true;
        }
        if (c == '[') {
            ++i;
            Ranges r;
            if (!cls(&r)) return false;
            *f = set_frag(r);
            return true;
        }
        if (c == '.') {
            ++i;
            *f = set_frag(dotnl ? Ranges{{0, MAXRUNE}} : negate({{'\n', '\n'}}));
            return true;
        }
        if (c == '^') { ++i; *f = assertion(multiline ? E_BEGIN_LINE : E_BEGIN_TEXT); return true; }
        if (c == '$') { ++i; *f = assertion(multiline ? E_END_LINE : E_END_TEXT); return true; }
        if (c == '\\' && i + 1 < re.size()) {
            const char e = re[i + 1];
            if (e == 'A') { i += 2; *f = assertion(E_BEGIN_TEXT); return true; }
            if (e == 'z') { i += 2; *f = assertion(E_END_TEXT); return true; }
            if (e == 'b') { i += 2; *f = assertion(E_WORD); return true; }
            if (e == 'B') { i += 2; *f = assertion(E_NOWORD); return true; }
            if (e == 'Q') {   // literal text up to \E (or the end of the pattern)
                i += 2;
                const size_t q = re.find("\\E", i);
                const size_t end = q == std::string::npos ? re.size() : q;
                F acc = empty();
                while (i < end) {
                    uint32_t rn;
                    if (!pat_rune(&rn)) return false;
                    acc = cat(acc, set_frag(literal_set(rn)));
                }
                if (q != std::string::npos) i = q + 2;
                *f = acc;
                return true;
            }
        }
        if (c == '\\') {
            ++i;
            Ranges r;
            bool is_class;
            if (!escape(&r, &is_class)) return false;
            *f = set_frag(r);
            return true;
        }
        uint32_t rn;
        if (!pat_rune(&rn)) return false;
        *f = set_frag(literal_set(rn));
        return true;
    }

    // copy of a fragment's states (for {n,m} expansion)
    F clone(const F &a, int lo_state, int hi_state) {
        std::map<int, int> m;
        for (int s = lo_state; s < hi_state; ++s) m[s] = add(st[s].t, st[s].set);
        for (int s = lo_state; s < hi_state; ++s) {
            const int d = m[s];
            st[d].out = st[s].out >= 0 && m.count(st[s].out) ? m[st[s].out] : st[s].out;
            st[d].out2 = st[s].out2 >= 0 && m.count(st[s].out2) ? m[st[s].out2] : st[s].out2;
        }
        F f{m[a.start], {}};
        for (auto &h : a.outs) f.outs.push_back({m[h.s], h.which});
        return f;
    }

    bool repeat(F *f) {
        const int lo_state = (int)st.size();
        if (!eof() && (peek() == '*' || peek() == '+' || peek() == '?')) {
            err = std::string("missing argument to repetition operator: `") + peek() + "`";
            return false;
        }
        const size_t at = i;
        if (!atom(f)) return false;
        const bool flag_group = re.compare(at, 2, "(?") == 0 && re[i - 1] == ')' && st.size() == (size_t)lo_state + 1 &&
                                st.back().t == N_EPS && re.find(':', at) > i;
        if (flag_group && !eof() && (peek() == '*' || peek() == '+' || peek() == '?')) {
            err = std::string("missing argument to repetition operator: `") + peek() + "`";
            return false;
        }
        bool had_op = false;
        while (!eof()) {
            const char c = peek();
            int mn = -1, mx = -1;
            if (c == '*') { ++i; mn = 0; mx = -1; }
            else if (c == '+') { ++i; mn = 1; mx = -1; }
            else if (c == '?') { ++i; mn = 0; mx = 1; }
            else if (c == '{') {
                size_t j = i + 1;
                int a = 0, b = -1, nd = 0;
                while (j < re.size() && re[j] >= '0' && re[j] <= '9') { a = a * 10 + (re[j] - '0'); ++j; ++nd; if (a > 1000) break; }
                if (!nd) break;   // literal '{'
                if (j < re.size() && re[j] == ',') {
                    ++j;
                    int nd2 = 0;
                    b = 0;
                    while (j < re.size() && re[j] >= '0' && re[j] <= '9') { b = b * 10 + (re[j] - '0'); ++j; ++nd2; if (b > 1000) break; }
                    if (!nd2) b = -1;
                } else {
                    b = a;
                }
                if (j >= re.size() || re[j] != '}') break;   // literal '{'
                if (a > 1000 || b > 1000 || (b >= 0 && b < a)) { err = "invalid repeat count"; return false; }
                i = j + 1;
                mn = a;
                mx = b;
            } else {
                break;
            }
            if (had_op) { err = "invalid nested repetition operator"; return false; }
            had_op = true;
            if (!eof() && peek() == '?') ++i;   // non-greedy: same match/no match
            const int hi_state = (int)st.size();
            if (mn == 0 && mx == -1) *f = star(*f);
            else if (mn == 1 && mx == -1) *f = plus(*f);
            else if (mn == 0 && mx == 1) *f = quest(*f);
            else {
                if ((mx < 0 ? mn + 1 : mx) * (hi_state - lo_state) > 4000) { unsup = true; return false; }
                // every copy is cloned from the unpatched original before any is linked
                const int ncopies = mx < 0 ? mn + 1 : mx;
                std::vector<F> cp;
                cp.push_back(*f);
                for (int k = 1; k < ncopies; ++k) cp.push_back(clone(*f, lo_state, hi_state));
                F acc;
                bool have = false;
                for (int k = 0; k < ncopies; ++k) {
                    F x = k < mn ? cp[k] : (mx < 0 ? star(cp[k]) : quest(cp[k]));
                    acc = have ? cat(acc, x) : x;
                    have = true;
                }
                *f = have ? acc : empty();
            }
            if (st.size() > 20000) { unsup = true; return false; }
        }
        return true;
    }

    bool concat(F *f) {
        bool have = false;
        F acc;
        while (!eof() && peek() != '|' && peek() != ')') {
            F x;
            if (!repeat(&x)) return false;
            acc = have ? cat(acc, x) : x;
            have = true;
        }
        *f = have ? acc : empty();
        return true;
    }

    bool alternation(F *f) {
        if (!concat(f)) return false;
        while (!eof() && peek() == '|') {
            ++i;
            F g;
            if (!concat(&g)) return false;
            *f = alt(*f, g);
        }
        return true;
    }
};

// epsilon closure over splits and the assertions that hold (`ops`); keeps rune sets and
// the match state
void closure(const std::vector<NState> &st, std::vector<int> &set, uint8_t ops) {
    std::vector<char> seen(st.size(), 0);
    std::vector<int> stack(set.begin(), set.end());
    std::vector<int> out;
    while (!stack.empty()) {
        const int s = stack.back();
        stack.pop_back();
        if (s < 0 || seen[s]) continue;
        seen[s] = 1;
        const NState &x = st[s];
        switch (x.t) {
        case N_SPLIT: stack.push_back(x.out); stack.push_back(x.out2); break;
        case N_EPS: stack.push_back(x.out); break;
        case N_ASSERT: if (((uint8_t)x.set & ~ops) == 0) stack.push_back(x.out); break;
        default: out.push_back(s); break;   // N_SET, N_MATCH
        }
    }
    std::sort(out.begin(), out.end());
    set.swap(out);
}

// context of the previous rune: the start of the text, '\n', a word rune, anything else
enum Ctx : uint8_t { C_BEGIN = 0, C_NL = 1, C_WORD = 2, C_OTHER = 3 };

// the assertions that hold between a previous rune of context `c` and the next rune (or the
// end of the text): emptyOpContext in Go's regexp/syntax
uint8_t ops_between(uint8_t c, bool end, bool next_nl, bool next_word) {
    uint8_t op = 0;
    if (c == C_BEGIN) op |= E_BEGIN_TEXT | E_BEGIN_LINE;
    if (c == C_NL) op |= E_BEGIN_LINE;
    if (end) op |= E_END_TEXT | E_END_LINE;
    if (next_nl) op |= E_END_LINE;
    op |= ((c == C_WORD) != (!end && next_word)) ? E_WORD : E_NOWORD;
    return op;
}

}  // namespace

int igx_regex_compile(const char *pattern, size_t len, RegexDfa *dfa, std::string *why) {
    Compiler c;
    c.re.assign(pattern, len);
    Compiler::F f;
    if (!c.alternation(&f) || (!c.eof() && c.err.empty() && !c.unsup)) {
        if (c.unsup) { *why = "unsupported regular-expression syntax for the device scan"; return IGX_ENOTSUP; }
        *why = c.err.empty() ? "unexpected )" : c.err;
        return IGX_EINVAL;
    }
    if (c.unsup) { *why = "unsupported regular-expression syntax for the device scan"; return IGX_ENOTSUP; }
    const int match = c.add(N_MATCH);
    c.patch(f.outs, match);
    const int start = f.start;
    const auto &st = c.st;
    // which parts of the previous rune's context any assertion reads
    uint8_t used = 0;
    for (const auto &x : st)
        if (x.t == N_ASSERT) used |= (uint8_t)x.set;
    const bool need_nl = used & (E_BEGIN_LINE | E_END_LINE), need_word = used & (E_WORD | E_NOWORD);
    auto ctx_of = [&](bool nl, bool word) -> uint8_t {   // contexts that no assertion tells apart merge
        if (nl && need_nl) return C_NL;
        if (word && need_word) return C_WORD;
        return C_OTHER;
    };
    // alphabet: elementary intervals of all sets; '\n' and the word runes always apart
    std::set<uint32_t> cuts = {0, MAXRUNE + 1, '\n', '\n' + 1, '0', '9' + 1, 'A', 'Z' + 1, '_', '_' + 1, 'a', 'z' + 1};
    for (auto &r : c.sets)
        for (auto &p : r) { cuts.insert(p.first); cuts.insert(p.second + 1); }
    std::vector<uint32_t> bounds(cuts.begin(), cuts.end());   // class k = [bounds[k], bounds[k+1])
    const uint32_t ncls = (uint32_t)bounds.size() - 1;
    if (ncls > RegexDfa::MAXCLS) { *why = "regular expression uses too many character classes"; return IGX_ENOTSUP; }
    // set membership per class
    std::vector<std::vector<char>> in(c.sets.size(), std::vector<char>(ncls, 0));
    for (size_t s = 0; s < c.sets.size(); ++s)
        for (auto &p : c.sets[s]) {
            const uint32_t a = (uint32_t)(std::lower_bound(bounds.begin(), bounds.end(), p.first) - bounds.begin());
            const uint32_t b = (uint32_t)(std::lower_bound(bounds.begin(), bounds.end(), p.second + 1) - bounds.begin());
            for (uint32_t k = a; k < b; ++k) in[s][k] = 1;
        }
    // DFA states: (NFA states before closure, previous-rune context); state 0 accepts
    std::map<std::pair<std::vector<int>, uint8_t>, int> ids;
    std::vector<std::pair<std::vector<int>, uint8_t>> states = {{{}, C_OTHER}};
    auto intern = [&](std::vector<int> v, uint8_t cx) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        auto key = std::make_pair(std::move(v), cx);
        auto it = ids.find(key);
        if (it != ids.end()) return it->second;
        const int id = (int)states.size();
        ids.emplace(key, id);
        states.push_back(std::move(key));
        return id;
    };
    const int d0 = intern({start}, C_BEGIN);
    std::vector<uint16_t> trans;
    std::vector<uint8_t> flags;
    for (size_t d = 0; d < states.size(); ++d) {
        if (states.size() > RegexDfa::MAXSTATES) { *why = "regular expression needs too many automaton states"; return IGX_ENOTSUP; }
        if (d == 0) {   // accept: absorbing
            flags.push_back(1 | 2 | 4);
            for (uint32_t k = 0; k < ncls; ++k) trans.push_back(0);
            continue;
        }
        const std::vector<int> cur = states[d].first;
        const uint8_t cx = states[d].second;
        uint8_t fl = 0;
        std::vector<int> e = cur;
        closure(st, e, ops_between(cx, true, false, false));   // the text ends here
        if (std::binary_search(e.begin(), e.end(), match)) fl |= 2;
        if (d == (size_t)d0 && (fl & 2)) fl |= 4;               // the empty text matches
        flags.push_back(fl);
        for (uint32_t k = 0; k < ncls; ++k) {
            const bool nl = bounds[k] == '\n', word = word_rune(bounds[k]);
            std::vector<int> x = cur;
            closure(st, x, ops_between(cx, false, nl, word));
            if (std::binary_search(x.begin(), x.end(), match)) {   // a match is complete before this rune
                trans.push_back(0);
                continue;
            }
            std::vector<int> nx;
            for (int s : x)
                if (st[s].t == N_SET && in[st[s].set][k]) nx.push_back(st[s].out);
            nx.push_back(start);   // unanchored search: a match may start at every rune
            trans.push_back((uint16_t)intern(std::move(nx), ctx_of(nl, word)));
        }
    }
    dfa->nstates = (uint32_t)states.size();
    dfa->ncls = ncls;
    dfa->start = (uint32_t)d0;
    dfa->trans = std::move(trans);
    dfa->flags = std::move(flags);
    dfa->bounds.assign(bounds.begin(), bounds.end() - 1);
    for (uint32_t r = 0; r < 128; ++r)
        dfa->ascii[r] = (uint8_t)(std::upper_bound(bounds.begin(), bounds.end(), r) - bounds.begin() - 1);
    return IGX_OK;
}

std::vector<uint8_t> igx_regex_blob(const RegexDfa &d) {
    RegexBlobHeader h{};
    h.nstates = d.nstates;
    h.ncls = d.ncls;
    h.start = d.start;
    size_t off = sizeof(RegexBlobHeader) + 128;
    h.off_bounds = (uint32_t)off;
    off += 4 * d.ncls;
    h.off_flags = (uint32_t)off;
    off += (d.nstates + 3) / 4 * 4;
    h.off_trans = (uint32_t)off;
    off += 2 * (size_t)d.nstates * d.ncls;
    h.bytes = (uint32_t)((off + 15) / 16 * 16);
    std::vector<uint8_t> b(h.bytes, 0);
    std::memcpy(b.data(), &h, sizeof h);
    std::memcpy(b.data() + sizeof h, d.ascii, 128);
    std::memcpy(b.data() + h.off_bounds, d.bounds.data(), 4 * d.ncls);
    std::memcpy(b.data() + h.off_flags, d.flags.data(), d.nstates);
    std::memcpy(b.data() + h.off_trans, d.trans.data(), 2 * (size_t)d.nstates * d.ncls);
    return b;
}
