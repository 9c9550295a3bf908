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

// getComparisonFuncForComparisonType (filter.go:236-263): (field OP ref) != negate
__device__ __forceinline__ bool pred_match(const DevPred &d, uint64_t row) {
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
