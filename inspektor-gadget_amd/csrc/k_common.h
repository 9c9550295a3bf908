// k_common.h -- device helpers shared by the gfx950 kernels.
#pragma once

#include "igx_internal.h"

#define IGX_WAVE 64

__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Load a little-endian scalar of `width` bytes (1,2,4,8) as u64, optionally sign-extended.
__device__ __forceinline__ uint64_t ld_scalar(const uint8_t *p, uint32_t width, uint64_t row,
                                              bool sign) {
    switch (width) {
    case 1: {
        uint8_t v = p[row];
        return sign ? (uint64_t)(int64_t)(int8_t)v : v;
    }
    case 2: {
        uint16_t v = reinterpret_cast<const uint16_t *>(p)[row];
        return sign ? (uint64_t)(int64_t)(int16_t)v : v;
    }
    case 4: {
        uint32_t v = reinterpret_cast<const uint32_t *>(p)[row];
        return sign ? (uint64_t)(int64_t)(int32_t)v : v;
    }
    default:
        return reinterpret_cast<const uint64_t *>(p)[row];
    }
}

__device__ __forceinline__ uint64_t ref_scalar(const DevPred &d, bool sign) {
    uint64_t v = 0;
    for (uint32_t b = 0; b < d.width && b < 8; ++b) v |= (uint64_t)d.ref[b] << (8 * b);
    if (sign && d.width < 8) {
        uint64_t m = 1ull << (8 * d.width - 1);
        v = (v ^ m) - m;
    }
    return v;
}

// three-way compare of row vs reference; returns 2 for unordered (NaN).
__device__ __forceinline__ int pred_cmp(const DevPred &d, uint64_t row) {
    if (d.kind == IGX_KIND_BYTES) {
        const uint8_t *f = d.ptr + row * d.width;
        // d.ref_len > width cannot be equal; compare the common prefix then lengths
        uint32_t n = d.width;
        if ((n & 3) == 0 && (((uintptr_t)f) & 3) == 0) {
            for (uint32_t w = 0; w < n / 4; ++w) {
                uint32_t a = __builtin_bswap32(*reinterpret_cast<const uint32_t *>(f + 4 * w));
                uint32_t b = ((uint32_t)d.ref[4 * w] << 24) | ((uint32_t)d.ref[4 * w + 1] << 16) |
                             ((uint32_t)d.ref[4 * w + 2] << 8) | d.ref[4 * w + 3];
                if (a != b) return a < b ? -1 : 1;
            }
        } else {
            for (uint32_t i = 0; i < n; ++i) {
                uint8_t a = f[i], b = d.ref[i];
                if (a != b) return a < b ? -1 : 1;
            }
        }
        // equal over the column width: a longer reference is greater
        return d.ref_len > n ? -1 : 0;
    }
    if (d.kind == IGX_KIND_FLOAT) {
        double a, b;
        if (d.width == 4) {
            float x = reinterpret_cast<const float *>(d.ptr)[row];
            float y;
            __builtin_memcpy(&y, d.ref, 4);
            a = x;
            b = y;
        } else {
            a = reinterpret_cast<const double *>(d.ptr)[row];
            __builtin_memcpy(&b, d.ref, 8);
        }
        if (a != a || b != b) return 2;
        return a < b ? -1 : (a > b ? 1 : 0);
    }
    bool sign = d.kind == IGX_KIND_INT;
    uint64_t a = ld_scalar(d.ptr, d.width, row, sign), b = ref_scalar(d, sign);
    if (sign) {
        int64_t x = (int64_t)a, y = (int64_t)b;
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    return a < b ? -1 : (a > b ? 1 : 0);
}

// regexp.MatchString over a fixed-width string column (filter.go:212-216): the value is
// the bytes up to the first NUL (gadgets.FromCString), decoded rune by rune like
// utf8.DecodeRune (an invalid or truncated sequence is one U+FFFD rune of one byte), and
// run through the host-compiled DFA (igx_regex.cpp) over rune classes.
struct RegexBlobHdr {
    uint32_t nstates, ncls, start, bytes, off_bounds, off_flags, off_trans, pad;
};

__device__ __forceinline__ uint32_t decode_rune(const uint8_t *s, uint32_t n, uint32_t i, uint32_t *len) {
    const uint32_t c0 = s[i];
    *len = 1;
    if (c0 < 0x80) return c0;
    const uint32_t rem = n - i;
    if (c0 >= 0xC2 && c0 <= 0xDF && rem >= 2) {
        const uint32_t c1 = s[i + 1];
        if ((c1 & 0xC0) == 0x80) { *len = 2; return ((c0 & 0x1F) << 6) | (c1 & 0x3F); }
    } else if (c0 >= 0xE0 && c0 <= 0xEF && rem >= 3) {
        const uint32_t c1 = s[i + 1], c2 = s[i + 2];
        const uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;   // no overlong, no surrogates
        if (c1 >= lo && c1 <= hi && (c2 & 0xC0) == 0x80) {
            *len = 3;
            return ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (c2 & 0x3F);
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4 && rem >= 4) {
        const uint32_t c1 = s[i + 1], c2 = s[i + 2], c3 = s[i + 3];
        const uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
        if (c1 >= lo && c1 <= hi && (c2 & 0xC0) == 0x80 && (c3 & 0xC0) == 0x80) {
            *len = 4;
            return ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((c2 & 0x3F) << 6) | (c3 & 0x3F);
        }
    }
    return 0xFFFD;
}

__device__ __forceinline__ bool regex_match(const uint8_t *blob, const uint8_t *s, uint32_t width) {
    const RegexBlobHdr *h = reinterpret_cast<const RegexBlobHdr *>(blob);
    const uint8_t *ascii = blob + sizeof(RegexBlobHdr);
    const uint32_t *bounds = reinterpret_cast<const uint32_t *>(blob + h->off_bounds);
    const uint8_t *flags = blob + h->off_flags;
    const uint16_t *trans = reinterpret_cast<const uint16_t *>(blob + h->off_trans);
    uint32_t n = 0;
    while (n < width && s[n]) ++n;
    uint32_t st = h->start;
    if (n == 0) return (flags[st] & 5u) != 0;
    if (flags[st] & 1u) return true;
    for (uint32_t i = 0; i < n;) {
        uint32_t len;
        const uint32_t r = decode_rune(s, n, i, &len);
        i += len;
        uint32_t cls;
        if (r < 128) {
            cls = ascii[r];
        } else {   // last class whose first rune <= r
            uint32_t lo = 0, hi = h->ncls;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (bounds[mid] <= r) lo = mid; else hi = mid;
            }
            cls = lo;
        }
        st = trans[st * h->ncls + cls];
        if (flags[st] & 1u) return true;
    }
    return (flags[st] & 2u) != 0;
}

// getComparisonFuncForComparisonType (filter.go:236-263): (field OP ref) != negate
__device__ __forceinline__ bool pred_match(const DevPred &d, uint64_t row) {
    if (d.gwidth) {   // guarded (group-by only): rows of another kind pass
        uint64_t g = 0;
        for (uint32_t b = 0; b < d.gwidth; ++b) g |= (uint64_t)d.gptr[row * d.gwidth + b] << (8 * b);
        if (g != d.gref) return true;
    }
    if (d.cmp == IGX_CMP_REGEX) return regex_match(d.dfa, d.ptr + row * d.width, d.width) != (d.negate != 0);
    int c = pred_cmp(d, row);
    bool r;
    if (c == 2) r = false;
    else switch (d.cmp) {
        case IGX_CMP_EQ: r = c == 0; break;
        case IGX_CMP_LT: r = c < 0; break;
        case IGX_CMP_LE: r = c <= 0; break;
        case IGX_CMP_GT: r = c > 0; break;
        case IGX_CMP_GE: r = c >= 0; break;
        default: r = false;
        }
    return r != (d.negate != 0);
}

__device__ __forceinline__ bool preds_match_all(const DevPreds &dp, uint64_t row) {
    bool ok = true;
    for (uint32_t p = 0; p < dp.n; ++p) ok = ok && pred_match(dp.p[p], row);
    return ok;
}

// FilterSpecs.MatchAny (filter.go:276-283): true on the first matching spec
__device__ __forceinline__ bool preds_match_any(const DevPreds &dp, uint64_t row) {
    bool ok = false;
    for (uint32_t p = 0; p < dp.n; ++p) ok = ok || pred_match(dp.p[p], row);
    return ok;
}

// agent-scope relaxed loads/stores: `global_load/store ... sc1` on gfx950 -- the
// write-through / L1-bypass forms MI355X_MICROARCH.md §Workgroup dispatch validates
// for cross-workgroup hand-offs.
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
