// igx_host.cpp -- host side of libigx.so: contexts, the filter-string parser, sort
// planning and the C-ABI entry points that dispatch to the gfx950 kernels.
//
// The parser and planner restate the reference's Go host logic so the device kernels
// receive exactly the predicates / key orders the reference would evaluate:
//   GetFilterFromString + getValueFromFilterSpec  pkg/columns/filter/filter.go:53-172
//   Prepare + FilterSortableColumns              pkg/columns/sort/sort.go:87-111,147-178
//   Sort's per-kind dispatch (bool/struct skipped) pkg/columns/sort/sort.go:35-83
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "igx_internal.h"
#include "igx_regex.h"

int igx_fail(igx_ctx *ctx, int code, const char *fmt, ...) {
    if (ctx) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

int igx_scratch(igx_ctx *ctx, size_t bytes, void **out) {
    if (bytes > ctx->scratch_bytes) {
        IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->scratch) (void)hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        size_t want = std::max(bytes, ctx->scratch_bytes * 3 / 2);
        want = igx_align(want, 1 << 20);
        hipError_t e = hipMalloc(&ctx->scratch, want);
        if (e != hipSuccess) {
            ctx->scratch_bytes = 0;
            return igx_fail(ctx, IGX_ENOMEM, "scratch: cannot allocate %zu bytes", want);
        }
        ctx->scratch_bytes = want;
    }
    *out = ctx->scratch;
    return IGX_OK;
}

int igx_pinned(igx_ctx *ctx, size_t bytes, void **out) {
    if (bytes > ctx->pinned_bytes) {
        IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        size_t want = igx_align(std::max<size_t>(bytes, 4096), 4096);
        IGX_HIP(ctx, hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault));
        ctx->pinned_bytes = want;
    }
    *out = ctx->pinned;
    return IGX_OK;
}

// ---------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------
extern "C" int igx_version(void) { return IGX_VERSION; }

extern "C" int igx_open(int device, uint32_t flags, igx_ctx **out) {
    (void)flags;
    if (!out) return IGX_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return IGX_ENOENT;
    if (device < 0 || device >= n) return IGX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return IGX_EIO;
    auto *ctx = new igx_ctx();
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        ctx->num_cus = prop.multiProcessorCount;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            delete ctx;
            return IGX_ENOTSUP;   // built for gfx950 (MI355X) only
        }
    }
    if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return IGX_EIO;
    }
    ctx->stream = ctx->own;
    *out = ctx;
    return IGX_OK;
}

extern "C" int igx_close(igx_ctx *ctx) {
    if (!ctx) return IGX_OK;
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    for (auto &r : ctx->regex) (void)hipFree(r.second);
    if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
    if (ctx->nan_word) (void)hipFree(ctx->nan_word);
    if (ctx->lsd_status) (void)hipFree(ctx->lsd_status);
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    delete ctx;
    return IGX_OK;
}

extern "C" const char *igx_last_error(igx_ctx *ctx) { return ctx ? ctx->err.c_str() : "no context"; }

extern "C" int igx_set_stream(igx_ctx *ctx, void *s) {
    if (!ctx) return IGX_EINVAL;
    hipStream_t ns = static_cast<hipStream_t>(s);
    if (ns != ctx->stream && ctx->scratch) {
        // the scratch arena (and the pinned staging) belong to the context, not to a stream: work
        // enqueued next on the new stream waits for what the old stream still has in flight, so
        // two calls on different streams never share the arena concurrently
        if (!ctx->handoff) IGX_HIP(ctx, hipEventCreateWithFlags(&ctx->handoff, hipEventDisableTiming));
        IGX_HIP(ctx, hipEventRecord(ctx->handoff, ctx->stream));
        IGX_HIP(ctx, hipStreamWaitEvent(ns, ctx->handoff, 0));
    }
    ctx->stream = ns;
    return IGX_OK;
}

extern "C" void *igx_get_stream(igx_ctx *ctx) { return ctx ? ctx->stream : nullptr; }

extern "C" int igx_sync(igx_ctx *ctx) {
    if (!ctx) return IGX_EINVAL;
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return IGX_OK;
}

extern "C" int igx_malloc(igx_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out) return IGX_EINVAL;
    if (hipMalloc(out, bytes ? bytes : 1) != hipSuccess)
        return igx_fail(ctx, IGX_ENOMEM, "igx_malloc(%zu) failed", bytes);
    return IGX_OK;
}

extern "C" int igx_free(igx_ctx *ctx, void *p) {
    if (!ctx) return IGX_EINVAL;
    IGX_HIP(ctx, hipFree(p));
    return IGX_OK;
}

extern "C" int igx_memcpy_h2d(igx_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return IGX_EINVAL;
    IGX_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return IGX_OK;
}

extern "C" int igx_memcpy_d2h(igx_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return IGX_EINVAL;
    IGX_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return IGX_OK;
}

extern "C" int igx_memcpy_d2d(igx_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return IGX_EINVAL;
    if (bytes) IGX_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return IGX_OK;
}

// ---------------------------------------------------------------------------------------
// filter-string parser (host only)
// ---------------------------------------------------------------------------------------
namespace {

std::string lower(const std::string &s) {
    std::string r = s;
    for (auto &c : r) c = (char)std::tolower((unsigned char)c);
    return r;
}

// Go's %q for the plain ASCII names/values seen here
std::string q(const std::string &s) {
    std::string r = "\"";
    for (unsigned char c : s) {
        if (c == '"' || c == '\\') { r += '\\'; r += (char)c; }
        else if (c < 0x20 || c == 0x7f) { char b[8]; snprintf(b, sizeof b, "\\x%02x", c); r += b; }
        else r += (char)c;
    }
    return r + "\"";
}

int put_err(char *errbuf, size_t errlen, int code, const std::string &msg) {
    if (errbuf && errlen) {
        size_t n = std::min(errlen - 1, msg.size());
        std::memcpy(errbuf, msg.data(), n);
        errbuf[n] = 0;
    }
    return code;
}

int find_col(const igx_schema_col *cols, uint32_t ncols, const std::string &name) {
    const std::string l = lower(name);
    for (uint32_t i = 0; i < ncols; ++i)
        if (cols[i].name && lower(cols[i].name) == l) return (int)i;
    return -1;
}

// strconv.ParseInt(s, 10, 64)
bool parse_int64(const std::string &s, int64_t *out) {
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i >= s.size()) return false;
    unsigned __int128 v = 0;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (unsigned)(s[i] - '0');
        if (v > ((unsigned __int128)1 << 63)) return false;
    }
    if (!neg && v > (((unsigned __int128)1 << 63) - 1)) return false;
    *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
    return true;
}

// strconv.ParseUint(s, 10, 64)
bool parse_uint64(const std::string &s, uint64_t *out) {
    if (s.empty()) return false;
    unsigned __int128 v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return false;
        v = v * 10 + (unsigned)(c - '0');
        if (v > (unsigned __int128)UINT64_MAX) return false;
    }
    *out = (uint64_t)v;
    return true;
}

// strconv.ParseFloat(s, 64): decimal/exponent, hex float, inf/infinity/nan (any case)
bool parse_float64(const std::string &s, double *out) {
    if (s.empty()) return false;
    std::string l = lower(s);
    std::string body = (l[0] == '+' || l[0] == '-') ? l.substr(1) : l;
    if (body == "inf" || body == "infinity") { *out = l[0] == '-' ? -INFINITY : INFINITY; return true; }
    if (body == "nan") { *out = NAN; return true; }
    for (char c : l)
        if (!(std::isdigit((unsigned char)c) || c == '.' || c == 'e' || c == '+' || c == '-' || c == 'x' ||
              c == 'p' || (c >= 'a' && c <= 'f')))
            return false;
    if (body.empty() || body.find("nan") != std::string::npos || body.find("inf") != std::string::npos) return false;
    errno = 0;
    char *end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    if (end != s.c_str() + s.size()) return false;
    if (errno == ERANGE && std::isinf(v)) return false;   // Go: ErrRange
    *out = v;
    return true;
}

// Light RE2 syntax check (the device scan does not evaluate regexes, but parse errors
// must surface at GetFilterFromString time like regexp.Compile's, filter.go:123-126):
// unbalanced parentheses/brackets, repetition operators without an operand, bad (?flags).
bool regex_syntax_ok(const std::string &re, std::string *why) {
    int depth = 0;
    bool have_atom = false;   // something a repetition operator can apply to
    bool last_rep = false;
    for (size_t i = 0; i < re.size(); ++i) {
        char c = re[i];
        if (c == '\\') {
            if (i + 1 >= re.size()) { *why = "trailing backslash at end of expression"; return false; }
            ++i;
            have_atom = true;
            last_rep = false;
        } else if (c == '[') {
            size_t j = i + 1;
            if (j < re.size() && re[j] == '^') ++j;
            if (j < re.size() && re[j] == ']') ++j;
            while (j < re.size() && re[j] != ']') { if (re[j] == '\\') ++j; ++j; }
            if (j >= re.size()) { *why = "missing closing ]"; return false; }
            i = j;
            have_atom = true;
            last_rep = false;
        } else if (c == '(') {
            if (i + 1 < re.size() && re[i + 1] == '?') {
                size_t j = i + 2;
                if (j < re.size() && (re[j] == 'P' || re[j] == '<')) {   // named group
                    ++depth;
                    have_atom = false;
                    last_rep = false;
                    i = j;
                    continue;
                }
                while (j < re.size() && (std::strchr("imsU-", re[j]) != nullptr)) ++j;
                if (j >= re.size()) { *why = "missing closing )"; return false; }
                if (re[j] == ')') {             // flag group: no atom produced
                    i = j;
                    last_rep = false;
                    continue;
                }
                if (re[j] != ':') { *why = "invalid or unsupported Perl syntax"; return false; }
                i = j;
            }
            ++depth;
            have_atom = false;
            last_rep = false;
        } else if (c == ')') {
            if (depth == 0) { *why = "unexpected )"; return false; }
            --depth;
            have_atom = true;
            last_rep = false;
        } else if (c == '|') {
            have_atom = false;
            last_rep = false;
        } else if (c == '*' || c == '+' || c == '?') {
            if (last_rep && c == '?') { last_rep = false; continue; }   // lazy modifier
            if (!have_atom || last_rep) { *why = std::string("missing argument to repetition operator: `") + c + "`"; return false; }
            last_rep = true;
        } else if (c == '{') {
            size_t j = i + 1;
            bool digits = false;
            while (j < re.size() && (std::isdigit((unsigned char)re[j]) || re[j] == ',')) { digits = true; ++j; }
            if (digits && j < re.size() && re[j] == '}') {
                if (!have_atom || last_rep) { *why = "missing argument to repetition operator"; return false; }
                i = j;
                last_rep = true;
            } else {
                have_atom = true;   // literal '{'
                last_rep = false;
            }
        } else {
            have_atom = true;
            last_rep = false;
        }
    }
    if (depth) { *why = "missing closing )"; return false; }
    return true;
}

}  // namespace

extern "C" int igx_filter_parse(const igx_schema_col *cols, uint32_t ncols, const char *filter,
                                igx_pred *out, char *errbuf, size_t errlen) {
    if (!cols || !filter || !out) return put_err(errbuf, errlen, IGX_EINVAL, "invalid arguments");
    std::memset(out, 0, sizeof *out);
    std::string f(filter);
    std::string name, rule;
    size_t colon = f.find(':');
    if (colon == std::string::npos) { name = f; rule = ""; }       // filter.go:93-96
    else { name = f.substr(0, colon); rule = f.substr(colon + 1); }
    int ci = find_col(cols, ncols, name);
    if (ci < 0) return put_err(errbuf, errlen, IGX_ENOENT, "could not apply filter: column " + q(name) + " not found");
    const igx_schema_col &col = cols[ci];
    out->col = (uint32_t)ci;
    if (!rule.empty() && rule[0] == '!') { out->negate = 1; rule = rule.substr(1); }   // :113-117
    uint32_t cmp = IGX_CMP_EQ;
    if (!rule.empty() && rule[0] == '~') {                                             // :119-127
        cmp = IGX_CMP_REGEX;
        rule = rule.substr(1);
        std::string why;
        if (!regex_syntax_ok(rule, &why))
            return put_err(errbuf, errlen, IGX_EINVAL,
                           "could not compile regular expression " + q(rule) + ": error parsing regexp: " + why);
    } else if (rule.rfind(">=", 0) == 0) { cmp = IGX_CMP_GE; rule = rule.substr(2); }
    else if (rule.rfind(">", 0) == 0) { cmp = IGX_CMP_GT; rule = rule.substr(1); }
    else if (rule.rfind("<=", 0) == 0) { cmp = IGX_CMP_LE; rule = rule.substr(2); }
    else if (rule.rfind("<", 0) == 0) { cmp = IGX_CMP_LT; rule = rule.substr(1); }
    out->cmp = cmp;
    const bool virt = (col.flags & (IGX_COL_VIRTUAL | IGX_COL_EXTRACTOR)) != 0;
    if (cmp == IGX_CMP_REGEX && col.kind != IGX_KIND_BYTES)
        return put_err(errbuf, errlen, IGX_EINVAL, "tried to apply regular expression on non-string column " + q(col.name));
    if (cmp == IGX_CMP_REGEX) {
        if (rule.size() > IGX_MAX_REF) return put_err(errbuf, errlen, IGX_ENOTSUP, "regular expression too long");
        std::memcpy(out->ref, rule.data(), rule.size());
        out->ref_len = (uint32_t)rule.size();
        return virt ? put_err(errbuf, errlen, IGX_ENOTSUP, "filter on virtual/extractor column " + q(col.name))
                    : IGX_OK;
    }
    switch (col.kind) {                                                                // :54-85
    case IGX_KIND_INT: {
        int64_t v;
        if (!parse_int64(rule, &v))
            return put_err(errbuf, errlen, IGX_EINVAL, "tried to compare " + q(rule) + " to int column " + q(col.name));
        uint64_t u = (uint64_t)v;   // reflect Convert: truncate to the column width
        for (uint32_t b = 0; b < col.width && b < 8; ++b) out->ref[b] = (uint8_t)(u >> (8 * b));
        out->ref_len = col.width;
        break;
    }
    case IGX_KIND_UINT: {
        uint64_t v;
        if (!parse_uint64(rule, &v))
            return put_err(errbuf, errlen, IGX_EINVAL, "tried to compare " + q(rule) + " to uint column " + q(col.name));
        for (uint32_t b = 0; b < col.width && b < 8; ++b) out->ref[b] = (uint8_t)(v >> (8 * b));
        out->ref_len = col.width;
        break;
    }
    case IGX_KIND_FLOAT: {
        double v;
        if (!parse_float64(rule, &v))
            return put_err(errbuf, errlen, IGX_EINVAL, "tried to compare " + q(rule) + " to float column " + q(col.name));
        if (col.width == 4) {
            float f32 = (float)v;
            std::memcpy(out->ref, &f32, 4);
        } else {
            std::memcpy(out->ref, &v, 8);
        }
        out->ref_len = col.width;
        break;
    }
    case IGX_KIND_BYTES:
        if (rule.size() > IGX_MAX_REF) return put_err(errbuf, errlen, IGX_ENOTSUP, "filter value longer than 256 bytes");
        std::memcpy(out->ref, rule.data(), rule.size());
        out->ref_len = (uint32_t)rule.size();
        break;
    default:
        return put_err(errbuf, errlen, IGX_EINVAL, "tried to match " + q(rule) + " on unsupported column " + q(col.name));
    }
    if (virt)   // the reference reinterprets memory here; reject instead
        return put_err(errbuf, errlen, IGX_ENOTSUP, "filter on virtual/extractor column " + q(col.name));
    return IGX_OK;
}

// compile (once per pattern and context) and upload a regex automaton
static int regex_device(igx_ctx *ctx, const char *pat, size_t len, const uint8_t **out) {
    const std::string key(pat, len);
    auto it = ctx->regex.find(key);
    if (it == ctx->regex.end()) {
        RegexDfa dfa;
        std::string why;
        const int rc = igx_regex_compile(pat, len, &dfa, &why);
        if (rc) return igx_fail(ctx, rc, "regular expression %s: %s", key.c_str(), why.c_str());
        const std::vector<uint8_t> blob = igx_regex_blob(dfa);
        void *d = nullptr;
        IGX_HIP(ctx, hipMalloc(&d, blob.size()));
        const hipError_t e = hipMemcpy(d, blob.data(), blob.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return igx_fail(ctx, IGX_EIO, "regex upload: %s", hipGetErrorString(e));
        }
        it = ctx->regex.emplace(key, d).first;
    }
    *out = static_cast<const uint8_t *>(it->second);
    return IGX_OK;
}

extern "C" int igx_regex_compile_blob(const char *pattern, size_t len, uint8_t *out, size_t cap,
                                      size_t *out_len, char *errbuf, size_t errlen) {
    if (!pattern || !out_len) return IGX_EINVAL;
    RegexDfa dfa;
    std::string why;
    const int rc = igx_regex_compile(pattern, len, &dfa, &why);
    if (rc) return put_err(errbuf, errlen, rc, why);
    const std::vector<uint8_t> blob = igx_regex_blob(dfa);
    *out_len = blob.size();
    if (out && cap >= blob.size()) std::memcpy(out, blob.data(), blob.size());
    return IGX_OK;
}

int igx_check_guard(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred &p) {
    if (p.guard_col >= ncols) return igx_fail(ctx, IGX_EINVAL, "predicate guard column %u out of range", p.guard_col);
    const igx_col &g = cols[p.guard_col];
    if (g.kind != IGX_KIND_INT && g.kind != IGX_KIND_UINT)
        return igx_fail(ctx, IGX_EINVAL, "predicate guard on a non-integer column");
    if (p.guard_len != g.width || (g.width != 1 && g.width != 2 && g.width != 4 && g.width != 8))
        return igx_fail(ctx, IGX_EINVAL, "predicate guard of %u bytes on a %u-byte column", p.guard_len, g.width);
    return IGX_OK;
}

uint64_t igx_guard_ref(const igx_pred &p) {
    uint64_t r = 0;
    for (uint32_t b = 0; b < p.guard_len && b < 8; ++b) r |= (uint64_t)p.guard_ref[b] << (8 * b);
    return r;
}

int igx_build_preds(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                    uint32_t npreds, DevPreds *out) {
    std::memset(out, 0, sizeof *out);
    if (npreds > IGX_KMAX_PREDS)
        return igx_fail(ctx, IGX_ENOTSUP, "more than %d predicates in one scan", IGX_KMAX_PREDS);
    for (uint32_t i = 0; i < npreds; ++i) {
        const igx_pred &p = preds[i];
        if (p.col >= ncols) return igx_fail(ctx, IGX_EINVAL, "predicate column %u out of range", p.col);
        if (p.cmp > IGX_CMP_GE) return igx_fail(ctx, IGX_EINVAL, "filter: comparison %u is not a FilterSpec", p.cmp);
        const igx_col &c = cols[p.col];
        DevPred &d = out->p[i];
        if (p.cmp == IGX_CMP_REGEX) {   // filter.go:146-148: regex rules need a string column
            if (c.kind != IGX_KIND_BYTES) return igx_fail(ctx, IGX_EINVAL, "regular expression on a non-string column");
            int rc = regex_device(ctx, reinterpret_cast<const char *>(p.ref), std::min<uint32_t>(p.ref_len, IGX_MAX_REF),
                                  &d.dfa);
            if (rc) return rc;
        }
        d.ptr = static_cast<const uint8_t *>(c.ptr);
        d.width = c.width;
        d.kind = c.kind;
        d.cmp = p.cmp;
        d.negate = p.negate;
        d.ref_len = p.ref_len;
        if (c.kind == IGX_KIND_BOOL || c.kind == IGX_KIND_OTHER)
            return igx_fail(ctx, IGX_EINVAL, "predicate on unsupported column kind");
        if (c.kind != IGX_KIND_BYTES && c.width != 1 && c.width != 2 && c.width != 4 && c.width != 8)
            return igx_fail(ctx, IGX_EINVAL, "predicate on a %u-byte scalar", c.width);
        if (c.kind == IGX_KIND_FLOAT && c.width != 4 && c.width != 8)
            return igx_fail(ctx, IGX_EINVAL, "float column width %u", c.width);
        std::memcpy(d.ref, p.ref, IGX_MAX_REF);
        if (p.guard_len) {
            int rc = igx_check_guard(ctx, cols, ncols, p);
            if (rc) return rc;
            d.gptr = static_cast<const uint8_t *>(cols[p.guard_col].ptr);
            d.gwidth = p.guard_len;
            d.gref = igx_guard_ref(p);
        }
    }
    out->n = npreds;
    return IGX_OK;
}

static int filter_chunked(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                          uint32_t npreds, uint32_t flags, const uint8_t *valid, uint64_t nrows,
                          uint32_t *out_idx, uint64_t *out_n) {
    if (!ctx) return IGX_EINVAL;
    if (flags & ~(uint32_t)(IGX_FILTER_ANY | IGX_FILTER_NIL_MATCH))
        return igx_fail(ctx, IGX_EINVAL, "filter: unknown flags 0x%x", flags);
    if (!out_n || (nrows && !out_idx)) return igx_fail(ctx, IGX_EINVAL, "filter: null output");
    if (nrows >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "filter: more than 2^32 rows");
    if (npreds && !preds) return igx_fail(ctx, IGX_EINVAL, "filter: null predicates");
    for (uint32_t i = 0; i < npreds; ++i)
        if (preds[i].guard_len) return igx_fail(ctx, IGX_EINVAL, "filter: guarded predicates are group-by only");
    const uint32_t nchunks = npreds ? (npreds + IGX_KMAX_PREDS - 1) / IGX_KMAX_PREDS : 1;
    std::vector<DevPreds> dps(nchunks);
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t b = c * IGX_KMAX_PREDS;
        const uint32_t m = npreds - b < IGX_KMAX_PREDS ? npreds - b : IGX_KMAX_PREDS;
        int rc = igx_build_preds(ctx, cols, ncols, npreds ? preds + b : nullptr, npreds ? m : 0, &dps[c]);
        if (rc) return rc;
    }
    return launch_filter_chunks(ctx, dps.data(), nchunks, (flags & IGX_FILTER_ANY) ? 1u : 0u,
                                (flags & IGX_FILTER_NIL_MATCH) ? 1u : 0u, valid, nrows, out_idx, out_n);
}

extern "C" int igx_filter(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                          uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
                          uint64_t *out_n) {
    return filter_chunked(ctx, cols, ncols, preds, npreds, 0, valid, nrows, out_idx, out_n);
}

extern "C" int igx_filter_any(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                              uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
                              uint64_t *out_n) {
    return filter_chunked(ctx, cols, ncols, preds, npreds, IGX_FILTER_ANY | IGX_FILTER_NIL_MATCH, valid, nrows,
                          out_idx, out_n);
}

extern "C" int igx_filter_ex(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                             uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t flags,
                             uint32_t *out_idx, uint64_t *out_n) {
    return filter_chunked(ctx, cols, ncols, preds, npreds, flags, valid, nrows, out_idx, out_n);
}

// ---------------------------------------------------------------------------------------
// sort
// ---------------------------------------------------------------------------------------
extern "C" int igx_sort_prepare(const igx_schema_col *cols, uint32_t ncols, const char *const *sort_by,
                                uint32_t n, igx_sortkey *out, uint32_t *out_n, uint32_t *out_invalid) {
    if (!cols || (n && !sort_by) || !out_n) return IGX_EINVAL;
    uint32_t k = 0, bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        std::string s = sort_by[i] ? sort_by[i] : "";
        if (s.empty()) { ++bad; continue; }                  // sort.go:152-156
        bool desc = false;
        if (s[0] == '-') { desc = true; s = s.substr(1); }
        int ci = find_col(cols, ncols, s);
        if (ci < 0 || (cols[ci].flags & IGX_COL_VIRTUAL)) { ++bad; continue; }   // :163-172
        if (out) {
            igx_sortkey &o = out[k];
            o.ptr = nullptr;
            o.col = (uint32_t)ci;
            o.desc = desc;
            o.kind = (cols[ci].flags & IGX_COL_EXTRACTOR) ? cols[ci].raw_kind : cols[ci].kind;   // :46-48
            o.width = cols[ci].width;
        }
        ++k;
    }
    *out_n = k;
    if (out_invalid) *out_invalid = bad;
    return IGX_OK;
}

static int sort_common(igx_ctx *ctx, const igx_sortkey *keys, const uint32_t *strides, uint32_t nkeys,
                       uint64_t nrows, const uint64_t *pos, const uint8_t *valid, uint32_t *out, uint32_t limit,
                       const uint32_t *rowmap, uint32_t pos_stride = 8, uint32_t direct_mask = 0,
                       const uint64_t *d_nrows = nullptr, TopkHint *hint = nullptr) {
    if (!ctx) return IGX_EINVAL;
    if (nrows == 0) return IGX_OK;                          // sort.go:36-38
    if (!out) return igx_fail(ctx, IGX_EINVAL, "sort: null output");
    std::vector<SortPlanKey> plan;
    std::vector<GoSortKey> go;   // the same passes as sort.go runs them (the exact NaN path)
    uint32_t parity = 0;
    for (uint32_t i = 0; i < nkeys; ++i) {
        const igx_sortkey &k = keys[i];
        if (k.kind == IGX_KIND_BOOL || k.kind == IGX_KIND_OTHER) continue;   // sort.go:77-78
        if (k.width == 0) {   // constant column: a pass that orders nothing, parity only
            parity ^= k.desc ? 1u : 0u;
            go.push_back(GoSortKey{nullptr, 0, k.kind, 0, k.desc ? 0u : 1u, 1u});
            continue;
        }
        go.push_back(GoSortKey{static_cast<const uint8_t *>(k.ptr), k.width, k.kind, strides ? strides[i] : k.width,
                               k.desc ? 0u : 1u, 0u});
        SortPlanKey p{};
        p.ptr = static_cast<const uint8_t *>(k.ptr);
        p.width = k.width;
        p.kind = k.kind;
        p.stride = strides ? strides[i] : k.width;
        p.direct = (direct_mask >> i) & 1u;
        if (!p.ptr) return igx_fail(ctx, IGX_EINVAL, "sort: key %u has no column", i);
        if (k.kind == IGX_KIND_BYTES) {
            p.words = (k.width + 3) / 4;
        } else {
            if (k.width != 1 && k.width != 2 && k.width != 4 && k.width != 8)
                return igx_fail(ctx, IGX_EINVAL, "sort: %u-byte scalar key", k.width);
            if (k.kind == IGX_KIND_FLOAT && k.width < 4) return igx_fail(ctx, IGX_EINVAL, "sort: bad float width");
            p.words = k.width == 8 ? 2 : 1;
        }
        // closed form: effective direction = desc_i XOR parity of earlier keys
        p.desc_eff = (k.desc ? 1u : 0u) ^ parity;
        parity ^= k.desc ? 1u : 0u;
        plan.push_back(p);
    }
    if (plan.empty()) {
        // nothing sortable: the slice is left as is (SortEntries with only invalid keys is a no-op)
        // (no pass runs, so nil entries stay where they are too): identity permutation
        return launch_sort_perm(ctx, nullptr, 0, nrows, nullptr, false, nullptr, out, limit, rowmap);
    }
    return launch_sort_perm(ctx, plan.data(), (uint32_t)plan.size(), nrows, pos, parity != 0, valid, out, limit,
                            rowmap, pos_stride, go.data(), (uint32_t)go.size(), d_nrows, hint);
}

int sort_common_rows(igx_ctx *ctx, const igx_sortkey *keys, const uint32_t *strides, uint32_t nkeys,
                     uint64_t nrows, const uint32_t *rowmap, const uint64_t *pos, uint32_t pos_stride,
                     uint32_t limit, uint32_t *out, uint32_t direct_mask, const uint64_t *d_nrows,
                     TopkHint *hint) {
    return sort_common(ctx, keys, strides, nkeys, nrows, pos, nullptr, out, limit, rowmap, pos_stride, direct_mask,
                       d_nrows, hint);
}

extern "C" int igx_ip_text(igx_ctx *ctx, const uint8_t *addr, uint32_t addr_stride, const uint8_t *family,
                           uint32_t family_stride, const uint32_t *rowmap, uint64_t n, uint8_t *out) {
    if (!ctx) return IGX_EINVAL;
    if (n && (!addr || !family || !out)) return igx_fail(ctx, IGX_EINVAL, "ip_text: null argument");
    if (n && (addr_stride < 16 || family_stride < 2))
        return igx_fail(ctx, IGX_EINVAL, "ip_text: strides must cover 16-byte addresses and 2-byte families");
    if (reinterpret_cast<uintptr_t>(out) % 8) return igx_fail(ctx, IGX_EINVAL, "ip_text: output not 8-byte aligned");
    return launch_ip_text(ctx, addr, addr_stride, family, family_stride, rowmap, n, out);
}

extern "C" int igx_sort_perm(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
                             const uint64_t *pos, const uint8_t *valid, uint32_t *out_perm) {
    return sort_common(ctx, keys, nullptr, nkeys, nrows, pos, valid, out_perm, 0, nullptr);
}

extern "C" int igx_sort_perm_ex(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
                                const uint64_t *pos, const uint8_t *valid, const uint32_t *rowmap, uint32_t *out_perm) {
    return sort_common(ctx, keys, nullptr, nkeys, nrows, pos, valid, out_perm, 0, rowmap);
}

extern "C" int igx_sort_perm_dn(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows_max,
                                const uint64_t *d_nrows, const uint64_t *pos, const uint8_t *valid,
                                const uint32_t *rowmap, uint32_t *out_perm) {
    if (ctx && !d_nrows) return igx_fail(ctx, IGX_EINVAL, "sort_perm_dn: null device row count");
    return sort_common(ctx, keys, nullptr, nkeys, nrows_max, pos, valid, out_perm, 0, rowmap, 8, 0, d_nrows);
}

extern "C" int igx_topk(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
                        const uint64_t *pos, uint32_t k, uint32_t *out_idx) {
    if (k == 0) return IGX_OK;
    return sort_common(ctx, keys, nullptr, nkeys, nrows, pos, nullptr, out_idx, k, nullptr);
}

extern "C" int igx_log2_slots(igx_ctx *ctx, const int64_t *delta, uint64_t nrows, uint64_t divisor, uint32_t nslots,
                              uint8_t *slot, uint8_t *keep) {
    if (!ctx) return IGX_EINVAL;
    return launch_log2_slots(ctx, delta, nrows, divisor, nslots, slot, keep);
}

extern "C" int igx_hist_log2(igx_ctx *ctx, const uint32_t *dev, const uint32_t *cont, const int64_t *delta,
                             uint64_t nrows, const uint32_t *devs, uint32_t ndev, uint32_t ncont,
                             uint64_t divisor, uint32_t nslots, uint32_t *hist) {
    if (!ctx) return IGX_EINVAL;
    if (nrows && (!delta || !hist || (ndev && (!dev || !devs)))) return igx_fail(ctx, IGX_EINVAL, "hist: null argument");
    return launch_hist_log2(ctx, dev, cont, delta, nrows, devs, ndev, ncont, divisor, nslots, hist);
}
