// k_sort.hip -- stable LSD radix sort reproducing the reference's tie order (kernel (3)).
//
// Reference: ColumnSorterCollection.Sort (pkg/columns/sort/sort.go:35-83) runs one Go
// 1.19 sort.SliceStable pass per key, last key first, with getLessFunc (:125-135)
// `!(a<b) != order`.  For DESC that comparator is `a >= b`; SliceStable always asks
// less(later, earlier), so every DESC pass reverses ties.  The composite order is
// therefore a single lexicographic order (verified by
// tests/test_oracle_golden.py::test_closed_form_matches_go_stable):
//   key i compares in direction desc_i XOR desc_1 ^ ... ^ desc_{i-1}, and the final
//   tie-break is the pre-sort position, ascending iff sum(desc) is even.
// nil entries (valid==0) sort last (sort.go:127-132), in input order.
//
// Implementation: compose every row into big-endian u32 words (SoA, most significant
// word first), one word group per key; DESC keys are bit-NOT-ed, signed ints get their
// sign bit flipped, floats the IEEE total-order flip, strings stay big-endian bytes; the
// position goes last (NOT-ed when the parity is odd).  One AND/OR reduction finds the
// byte digits that are constant over all rows; only the others get a pass.  Each pass is
// histogram -> scan -> stable scatter (wave64 ballot multi-split ranks, tile order kept
// by per-digit running counters in LDS).  Words below the current digit are no longer
// carried (LSD never reads them again).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "k_common.h"

namespace {

constexpr int TB = 256;
constexpr int IPT = 16;
constexpr int TILE = TB * IPT;   // 4096 rows per tile
// The radix passes' histogram and scatter kernels run a tile with 1024 threads (4 rows each):
// at ~1M rows a pass has about one tile per CU, and a 256-thread block working through 16
// rows per thread one barrier step at a time left the pass latency-bound (~30 us).
#ifndef IGX_RADIX_STB
#define IGX_RADIX_STB 1024
#endif
constexpr int STB = IGX_RADIX_STB;
constexpr int SIPT = 4;
constexpr int RTILE = STB * SIPT;   // rows per radix-pass tile
constexpr int MAXW = 80;          // composed words (keys + pos + nil; wider keys: ENOTSUP)
constexpr int NSK = 32;           // sort keys

__device__ __forceinline__ uint32_t be_word(const uint8_t *p, uint32_t width, uint32_t j) {
    if (4 * j + 4 <= width && (reinterpret_cast<uintptr_t>(p) & 3) == 0)   // a whole aligned dword
        return __builtin_bswap32(*reinterpret_cast<const uint32_t *>(p + 4 * j));
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        uint32_t o = 4 * j + b;
        v = (v << 8) | (o < width ? p[o] : 0u);
    }
    return v;
}

// ---- string dictionaries -------------------------------------------------------------
// A multi-word string key costs one radix pass per live byte (C1's 16-byte `comm`: 12 of its
// 16 passes).  When the key has few distinct values, the sort replaces it by its rank among
// them: equal strings get equal ranks and the ranks keep the strings' byte order, so the
// stable LSD passes over the rank produce exactly the order of the passes over the bytes --
// with one or two live digits instead of a dozen.  k_dict_build collects the distinct values:
// each workgroup first in an LDS table over its own rows, then only those into the global
// table (an open-addressed table of {tag, index} slots, the values in claim order -- a few
// values over a million rows would otherwise send every row's L1-bypassing probe to the same
// few L2 lines: 0.91 ms for C1 measured); k_dict_rank sorts the distinct values in one
// workgroup's LDS (bitonic, over indices) and writes each one's rank next to it; k_compose
// looks every row's rank up.  More distinct values than the dictionary holds void it (ctl[1]);
// the host then composes the raw bytes (one more read-back, launch_sort_perm).
constexpr int DICT_W = 8;                // key words a dictionary takes (strings of <= 32 bytes)
constexpr uint32_t DICT_MAXD = 4096;     // distinct values (power of two)
constexpr uint32_t DICT_LDS_WORDS = 16384;   // k_dict_rank: distinct values x words in LDS
constexpr int DICT_MAXK = 4;             // dictionary keys per sort
constexpr uint64_t DICT_MIN_ROWS = 1u << 16;
constexpr uint32_t DENT = 16;            // words per dictionary entry (value, rank, padding)

struct DictRef {
    uint32_t *slot;     // 2 x (mask + 1): {tag (0 empty, 1 being written, else hash | 2), index}
    uint32_t *keys;     // cap x DENT: the distinct values in claim order, one 64-B line each:
                        // the value's words, then (k_dict_rank) its rank at word DICT_W
    uint32_t *ctl;      // [0] distinct values claimed, [1] void (over capacity)
    uint32_t *rowidx;   // per slice row (k_dict_build): its value's index (k_compose reads the rank there)
    uint32_t mask, cap, nw;
};

struct DictBuildArgs {
    DictRef d;
    const uint8_t *ptr;
    uint32_t width, rstride;
    const uint32_t *rowmap;
    const uint8_t *valid;
    const uint64_t *d_n;
    uint64_t n;
};

__device__ __forceinline__ uint32_t dict_hash(const uint32_t (&k)[DICT_W], uint32_t nw) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int j = 0; j < DICT_W; ++j)
        if ((uint32_t)j < nw) h = (h ^ k[j]) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 29;
    return (uint32_t)h;
}

__device__ __forceinline__ bool dict_eq(const uint32_t *v, const uint32_t (&k)[DICT_W], uint32_t nw) {
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < DICT_W; ++j)
        if ((uint32_t)j < nw) diff |= v[j] ^ k[j];
    return diff == 0;
}

// Insert a value into the global table (the value's hash h); returns its index (DL_NONE: the
// dictionary is void).  One probe per iteration: a lane that finds its slot being written
// looks again next iteration, so a claimer of the same wave (which publishes within its own
// iteration) is never waited for inside a branch.
constexpr uint32_t DL_NONE = 0xFFFFFFFFu;
__device__ uint32_t dict_insert(const DictRef &d, const uint32_t (&k)[DICT_W], uint32_t h) {
    const uint32_t tg = h | 2u;
    uint32_t s = h & d.mask;
    for (uint32_t probes = 0, spins = 0; probes <= d.mask;) {
        const uint32_t t = __hip_atomic_load(&d.slot[2 * s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0u) {
            if (atomicCAS(&d.slot[2 * s], 0u, 1u) == 0u) {
                const uint32_t idx = atomicAdd(&d.ctl[0], 1u);
                if (idx >= d.cap) {   // over capacity: the dictionary is void (the slot stays busy)
                    atomicOr(&d.ctl[1], 1u);
                    return DL_NONE;
                }
#pragma unroll
                for (int j = 0; j < DICT_W; ++j)
                    if ((uint32_t)j < d.nw) d.keys[(uint64_t)idx * DENT + j] = k[j];
                d.slot[2 * s + 1] = idx;
                __hip_atomic_store(&d.slot[2 * s], tg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                return idx;
            }
            continue;   // lost the claim: read the slot again
        }
        if (t == 1u) {   // being written
            if (__hip_atomic_load(&d.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return DL_NONE;
            if (++spins > (1u << 20)) { atomicOr(&d.ctl[1], 2u); return DL_NONE; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (t == tg) {
            const uint32_t idx = d.slot[2 * s + 1];
            if (dict_eq(d.keys + (uint64_t)idx * DENT, k, d.nw)) return idx;
        }
        s = (s + 1) & d.mask;
        ++probes;
    }
    atomicOr(&d.ctl[1], 2u);   // no free slot (cannot happen: at most half the slots are claimed)
    return DL_NONE;
}

// The collection: DB_RPT rows per thread (their loads in flight together; one workgroup per
// DB_ROWS rows); a workgroup with more than DL_CAP distinct values (or a full LDS table)
// sends the rest straight to the global table.  Every row's value index goes to rowidx.
constexpr uint32_t DB_T = 1024, DB_RPT = 8, DB_ROWS = DB_T * DB_RPT;
constexpr uint32_t DL_SLOTS = 2048, DL_CAP = 1024, DL_GLOBAL = 0x80000000u;

__global__ __launch_bounds__(DB_T) void k_dict_build(DictBuildArgs a) {
    __shared__ uint32_t ltag[DL_SLOTS];   // 0 empty, 1 being written, else hash | 2
    __shared__ uint32_t lidx[DL_SLOTS];   // the value's local index, DL_NONE: it went global
    __shared__ uint32_t lval[DL_CAP * DICT_W];
    __shared__ uint32_t lhash[DL_CAP];
    __shared__ uint32_t lglob[DL_CAP];    // local value -> its global index
    __shared__ uint32_t lcount;
    const DictRef &d = a.d;
    for (uint32_t t = threadIdx.x; t < DL_SLOTS; t += DB_T) ltag[t] = 0;
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    const uint64_t n = a.d_n ? min(a.n, *a.d_n) : a.n;
    const uint64_t base = (uint64_t)blockIdx.x * DB_ROWS + threadIdx.x;
    // every row's words first (all loads in flight together), then the inserts
    uint32_t k[DB_RPT][DICT_W];
    bool live[DB_RPT];
#pragma unroll
    for (int r = 0; r < (int)DB_RPT; ++r) {
        const uint64_t i = base + (uint64_t)r * DB_T;
        live[r] = i < n;
        const uint64_t src = live[r] ? (a.rowmap ? a.rowmap[i] : i) : 0;
        if (live[r] && a.valid) live[r] = a.valid[src] != 0;   // nil rows compose zeros, not a rank
        const uint8_t *p = a.ptr + src * a.rstride;
#pragma unroll
        for (int j = 0; j < DICT_W; ++j) k[r][j] = live[r] && (uint32_t)j < d.nw ? be_word(p, a.width, j) : 0u;
    }
    uint32_t lr[DB_RPT];   // the row's local index, or DL_GLOBAL | its global index
#pragma unroll
    for (int r = 0; r < (int)DB_RPT; ++r) {
        lr[r] = DL_NONE;
        if (!live[r]) continue;
        const uint32_t h = dict_hash(k[r], d.nw), tg = h | 2u;
        uint32_t s = h & (DL_SLOTS - 1);
        // global unless the value is (now) in this workgroup's list: a full list (DL_NONE) or a
        // full table sends it to the global table directly
        bool global = true;
        for (uint32_t probes = 0, spins = 0; probes < DL_SLOTS;) {
            const uint32_t t = __hip_atomic_load(&ltag[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == 0u) {
                if (atomicCAS(&ltag[s], 0u, 1u) == 0u) {
                    const uint32_t li = atomicAdd(&lcount, 1u);
                    if (li < DL_CAP) {
#pragma unroll
                        for (int j = 0; j < DICT_W; ++j)
                            if ((uint32_t)j < d.nw) lval[li * d.nw + j] = k[r][j];
                        lhash[li] = h;
                        lidx[s] = li;
                        lr[r] = li;
                        global = false;
                    } else {
                        lidx[s] = DL_NONE;   // this value (and any sharing its hash) goes global
                    }
                    __hip_atomic_store(&ltag[s], tg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                continue;
            }
            if (t == 1u) {
                if (++spins > (1u << 22)) { atomicOr(&d.ctl[1], 2u); break; }
                continue;
            }
            if (t == tg) {
                const uint32_t li = lidx[s];
                if (li == DL_NONE) break;
                if (dict_eq(lval + li * d.nw, k[r], d.nw)) {
                    lr[r] = li;
                    global = false;
                    break;
                }
            }
            s = (s + 1) & (DL_SLOTS - 1);
            ++probes;
        }
        if (global) lr[r] = DL_GLOBAL | dict_insert(d, k[r], h);
    }
    __syncthreads();
    const uint32_t nloc = min(lcount, DL_CAP);
    for (uint32_t li = threadIdx.x; li < nloc; li += DB_T) {
        uint32_t v[DICT_W];
#pragma unroll
        for (int j = 0; j < DICT_W; ++j) v[j] = (uint32_t)j < d.nw ? lval[li * d.nw + j] : 0u;
        lglob[li] = dict_insert(d, v, lhash[li]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < (int)DB_RPT; ++r) {
        if (!live[r]) continue;
        const uint32_t x = lr[r];
        d.rowidx[base + (uint64_t)r * DB_T] = (x & DL_GLOBAL) ? (x == DL_NONE ? DL_NONE : x & ~DL_GLOBAL) : lglob[x];
    }
}

// k_dict_rank (one workgroup): the distinct values into LDS, a bitonic sort of their indices
// (the values are distinct, so no tie order to keep), the rank of value i next to its words.
// (Run by k_dict_build's last workgroup instead: 39 vs 23 + 13 us on C1 -- the collection's
// workgroups then hold the ranking's 80 KB of LDS.)
__global__ __launch_bounds__(1024) void k_dict_rank(DictRef d) {
    extern __shared__ uint32_t dl[];
    if (d.ctl[1]) return;   // void: the host composes the raw bytes
    const uint32_t D = min(d.ctl[0], d.cap), nw = d.nw;
    if (D == 0) return;   // no live row (an empty slice, every row nil): nothing to rank
    uint32_t N = 2;
    while (N < D) N <<= 1;
    uint32_t *kv = dl, *ix = dl + (size_t)d.cap * nw;
    for (uint32_t t = threadIdx.x; t < D * nw; t += 1024) kv[t] = d.keys[(t / nw) * DENT + t % nw];
    for (uint32_t t = threadIdx.x; t < N; t += 1024) ix[t] = t;
    __syncthreads();
    if (D <= 256) {
        // few values: P threads per value each count the values below it among every P-th one
        // (at most D^2 / 1024 compares in a row), then add up in LDS -- the bitonic network's
        // 21 barrier-separated stages cost more at C1's 64 names
        __shared__ uint32_t rk[256];
        if (threadIdx.x < 256) rk[threadIdx.x] = 0;
        __syncthreads();
        uint32_t P = 4;   // D >= 1: P <= 512
        while (P < 512 && P * 2 * D <= 1024) P *= 2;
        const uint32_t v = threadIdx.x / P, part = threadIdx.x % P;
        if (v < D) {
            uint32_t y[DICT_W];
#pragma unroll
            for (int j = 0; j < DICT_W; ++j) y[j] = (uint32_t)j < nw ? kv[v * nw + j] : 0u;
            uint32_t cnt = 0;
            for (uint32_t u = part; u < D; u += P) {
                uint32_t x[DICT_W];
#pragma unroll
                for (int j = 0; j < DICT_W; ++j) x[j] = (uint32_t)j < nw ? kv[u * nw + j] : 0u;
                // x < y lexicographically, without branches: the first differing word decides
                bool lt = false, eq = true;
#pragma unroll
                for (int j = 0; j < DICT_W; ++j) {
                    lt = lt || (eq && x[j] < y[j]);
                    eq = eq && x[j] == y[j];
                }
                cnt += lt ? 1u : 0u;
            }
            atomicAdd(&rk[v], cnt);
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < D; t += 1024) d.keys[(uint64_t)t * DENT + DICT_W] = rk[t];
        return;
    }
    // greater(a, b): pad indices (>= D) sort last
    auto greater = [&](uint32_t a, uint32_t b) -> bool {
        if (a >= D || b >= D) return a >= D && (b < D || a > b);
        const uint32_t *x = kv + (size_t)a * nw, *y = kv + (size_t)b * nw;
        for (uint32_t j = 0; j < nw; ++j)
            if (x[j] != y[j]) return x[j] > y[j];
        return false;
    };
    for (uint32_t k = 2; k <= N; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < N; t += 1024) {
                const uint32_t u = t ^ j;
                if (u > t) {
                    const uint32_t a = ix[t], b = ix[u];
                    if (greater(a, b) == ((t & k) == 0)) {
                        ix[t] = b;
                        ix[u] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t t = threadIdx.x; t < D; t += 1024) d.keys[(uint64_t)ix[t] * DENT + DICT_W] = t;
}

// the rank of slice row r's value (k_compose; garbage only when the dictionary is void, and
// the host then discards this compose)
__device__ __forceinline__ uint32_t dict_rank(const DictRef &d, uint64_t r) {
    const uint32_t idx = d.rowidx[r];
    return idx < d.cap ? d.keys[(uint64_t)idx * DENT + DICT_W] : 0u;
}

struct ComposeArgs {
    const uint8_t *ptr[NSK];
    uint32_t width[NSK], kind[NSK], desc[NSK], words[NSK], rstride[NSK], direct[NSK];   // direct: read at i, not rowmap[i]
    uint32_t dict[NSK];                  // 0, or 1 + the key's dictionary (words[k] is then 1: the rank)
    DictRef dref[DICT_MAXK];
    uint32_t nkeys, has_nil, pos_words, pos_not, pos_stride;   // pos_stride in bytes
    uint32_t reverse;     // pos_words == 0: slot i holds row n-1-i (the position order is descending)
    const uint64_t *pos;
    const uint8_t *valid;
    const uint32_t *rowmap;
    const uint64_t *d_n;  // nullable: the row count on the device (n is then its upper bound)
    uint64_t n, stride;   // stride = words array pitch (elements)
    uint32_t *nan_seen;   // set to 1 when a float key of a non-nil row is NaN (k_andor_final
                          // moves it into res and clears it: the word is the context's, zero
                          // between sorts)
    const uint32_t *skip; // nullable: nonzero on the device when a hinted top-K already answered
};

__global__ __launch_bounds__(TB) void k_compose(ComposeArgs a, uint32_t *__restrict__ words,
                                                uint32_t *__restrict__ payload) {
    const uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
    const uint64_t n = a.d_n ? min(a.n, *a.d_n) : a.n;
    if (i >= n) return;
    const uint64_t r = a.reverse ? n - 1 - i : i;       // the row composed into slot i
    const uint64_t src = a.rowmap ? a.rowmap[r] : r;   // where its values live
    bool nil = a.valid && a.valid[src] == 0;
    uint32_t w = 0;
    if (a.has_nil) words[(w++) * a.stride + i] = nil ? 1u : 0u;
    for (uint32_t k = 0; k < a.nkeys; ++k) {
        const uint32_t nw = a.words[k];
        if (nil) {
            for (uint32_t j = 0; j < nw; ++j) words[(w + j) * a.stride + i] = 0;
            w += nw;
            continue;
        }
        const uint32_t inv = a.desc[k] ? 0xFFFFFFFFu : 0u;
        const uint8_t *p = a.ptr[k] + (a.direct[k] ? r : src) * a.rstride[k];
        if (a.dict[k]) {
            words[w * a.stride + i] = dict_rank(a.dref[a.dict[k] - 1], r) ^ inv;
        } else if (a.kind[k] == IGX_KIND_BYTES) {
            for (uint32_t j = 0; j < nw; ++j) words[(w + j) * a.stride + i] = be_word(p, a.width[k], j) ^ inv;
        } else if (a.kind[k] == IGX_KIND_FLOAT) {
            if (a.width[k] == 4) {
                uint32_t b = *reinterpret_cast<const uint32_t *>(p);
                if ((b & 0x7FFFFFFFu) > 0x7F800000u) *a.nan_seen = 1u;   // unordered: see launch_sort_perm
                if (b == 0x80000000u) b = 0;                       // -0 == +0 in Go
                b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
                words[w * a.stride + i] = b ^ inv;
            } else {
                uint64_t b = *reinterpret_cast<const uint64_t *>(p);
                if ((b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) *a.nan_seen = 1u;
                if (b == 0x8000000000000000ull) b = 0;
                b = (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
                words[w * a.stride + i] = (uint32_t)(b >> 32) ^ inv;
                words[(w + 1) * a.stride + i] = (uint32_t)b ^ inv;
            }
        } else {
            const bool sgn = a.kind[k] == IGX_KIND_INT;
            uint64_t v = ld_scalar(p, a.width[k], 0, false);
            if (sgn) v ^= 1ull << (8 * a.width[k] - 1);
            if (nw == 1) {
                words[w * a.stride + i] = (uint32_t)v ^ inv;
            } else {
                words[w * a.stride + i] = (uint32_t)(v >> 32) ^ inv;
                words[(w + 1) * a.stride + i] = (uint32_t)v ^ inv;
            }
        }
        w += nw;
    }
    uint64_t p = a.pos ? *reinterpret_cast<const uint64_t *>(reinterpret_cast<const uint8_t *>(a.pos) +
                                                             src * a.pos_stride)
                       : i;
    if (a.pos_not && !nil) p = ~p;
    if (a.pos_words == 2) {
        words[w * a.stride + i] = (uint32_t)(p >> 32);
        words[(w + 1) * a.stride + i] = (uint32_t)p;
    } else if (a.pos_words == 1) {
        words[w * a.stride + i] = (uint32_t)p;
    }
    payload[i] = (uint32_t)src;
}

// The tables' SortStats shape: NK 8-byte integer keys (aggregates or the first index) read
// through the slot list, the first index as the position, no nil mask.  Every load of a row
// issues before any is used (the generic kernel's runtime key loop waits once per key).
template <int NK>
__global__ __launch_bounds__(TB) void k_compose_u64(ComposeArgs a, uint32_t *__restrict__ words,
                                                    uint32_t *__restrict__ payload) {
    const uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= a.n || (a.d_n && i >= *a.d_n)) return;
    const uint64_t src = a.rowmap[i];
    uint64_t v[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) v[k] = *reinterpret_cast<const uint64_t *>(a.ptr[k] + src * a.rstride[k]);
    uint64_t ps = *reinterpret_cast<const uint64_t *>(reinterpret_cast<const uint8_t *>(a.pos) + src * a.pos_stride);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const uint64_t inv = a.desc[k] ? ~0ull : 0ull;
        const uint64_t x = (a.kind[k] == IGX_KIND_INT ? v[k] ^ (1ull << 63) : v[k]) ^ inv;
        words[(uint64_t)(2 * k) * a.stride + i] = (uint32_t)(x >> 32);
        words[(uint64_t)(2 * k + 1) * a.stride + i] = (uint32_t)x;
    }
    if (a.pos_not) ps = ~ps;
    words[(uint64_t)(2 * NK) * a.stride + i] = (uint32_t)(ps >> 32);
    words[(uint64_t)(2 * NK + 1) * a.stride + i] = (uint32_t)ps;
    payload[i] = (uint32_t)src;
}

// k_compose_u64 with k_andor folded in (the tables' top-K): a fixed grid
// sweeps the rows, CU rows in flight per thread (their slot and value-record loads issued
// before any is used), composes their words and keeps every word's AND / OR in registers; each
// block leaves its partials where k_andor would have, so k_andor_final follows unchanged and
// the composed words are never read back for the reduction.
constexpr uint32_t CAO_BLOCKS = 2048;   // partials per word (k_andor_final: 32 per lane)
template <int NK>
__global__ __launch_bounds__(TB) void k_compose_u64_ao(ComposeArgs a, uint32_t *__restrict__ words,
                                                       uint32_t *__restrict__ payload, uint32_t *__restrict__ part) {
    constexpr int KW = 2 * NK + 2;
    constexpr int CU = 4;
    __shared__ uint32_t red[2][KW][TB / 64];
    if (a.skip && *a.skip) return;
    const uint64_t n = a.d_n ? min(a.n, *a.d_n) : a.n;
    uint32_t va[KW], vo[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) {
        va[w] = 0xFFFFFFFFu;
        vo[w] = 0;
    }
    const uint64_t step = (uint64_t)gridDim.x * TB;
    for (uint64_t i0 = (uint64_t)blockIdx.x * TB + threadIdx.x; i0 < n; i0 += CU * step) {
        uint64_t src[CU], v[CU][NK], ps[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint64_t i = i0 + u * step;
            src[u] = i < n ? a.rowmap[i] : a.rowmap[i0];
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
#pragma unroll
            for (int k = 0; k < NK; ++k) v[u][k] = *reinterpret_cast<const uint64_t *>(a.ptr[k] + src[u] * a.rstride[k]);
            ps[u] = *reinterpret_cast<const uint64_t *>(reinterpret_cast<const uint8_t *>(a.pos) + src[u] * a.pos_stride);
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint64_t i = i0 + u * step;
            if (i >= n) break;
            uint32_t wv[KW];
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const uint64_t inv = a.desc[k] ? ~0ull : 0ull;
                const uint64_t x = (a.kind[k] == IGX_KIND_INT ? v[u][k] ^ (1ull << 63) : v[u][k]) ^ inv;
                wv[2 * k] = (uint32_t)(x >> 32);
                wv[2 * k + 1] = (uint32_t)x;
            }
            const uint64_t p = a.pos_not ? ~ps[u] : ps[u];
            wv[2 * NK] = (uint32_t)(p >> 32);
            wv[2 * NK + 1] = (uint32_t)p;
#pragma unroll
            for (int w = 0; w < KW; ++w) {
                words[(uint64_t)w * a.stride + i] = wv[w];
                va[w] &= wv[w];
                vo[w] |= wv[w];
            }
            payload[i] = (uint32_t)src[u];
        }
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int w = 0; w < KW; ++w) {
        for (int o = 32; o > 0; o >>= 1) {
            va[w] &= __shfl_xor(va[w], o);
            vo[w] |= __shfl_xor(vo[w], o);
        }
        if (lane == 0) {
            red[0][w][wave] = va[w];
            red[1][w][wave] = vo[w];
        }
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)KW) {
        const uint32_t w = threadIdx.x;
        uint32_t x = 0xFFFFFFFFu, y = 0;
        for (int j = 0; j < TB / 64; ++j) {
            x &= red[0][w][j];
            y |= red[1][w][j];
        }
        part[2 * ((uint64_t)w * gridDim.x + blockIdx.x)] = x;
        part[2 * ((uint64_t)w * gridDim.x + blockIdx.x) + 1] = y;
    }
}

// per-word AND / OR over all rows -> part[(w * gridDim.x + block) * 2 + {0: and, 1: or}].
// 16-byte loads, four in flight per lane; partials, not atomics: the words' results share
// one line, and same-line atomics from every workgroup serialise at the memory side.
__global__ __launch_bounds__(TB) void k_andor(const uint32_t *__restrict__ words, uint64_t n,
                                              uint64_t stride, uint32_t *__restrict__ part,
                                              const uint64_t *__restrict__ d_n) {
    __shared__ uint32_t red[2][TB / 64];
    if (d_n) n = min(n, *d_n);
    const uint32_t w = blockIdx.y;
    const uint32_t *col = words + (uint64_t)w * stride;   // stride is a multiple of 64 rows
    const uint4 *v4 = reinterpret_cast<const uint4 *>(col);
    const uint64_t n4 = n / 4;
    uint32_t va = 0xFFFFFFFFu, vo = 0;
    const uint64_t step = (uint64_t)gridDim.x * TB;
    uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
    for (; i + 3 * step < n4; i += 4 * step) {
        uint4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = v4[i + j * step];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            va &= q[j].x & q[j].y & q[j].z & q[j].w;
            vo |= q[j].x | q[j].y | q[j].z | q[j].w;
        }
    }
    for (; i < n4; i += step) {
        const uint4 q = v4[i];
        va &= q.x & q.y & q.z & q.w;
        vo |= q.x | q.y | q.z | q.w;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {   // rows past the last whole quad
        const uint32_t x = col[n4 * 4 + threadIdx.x];
        va &= x;
        vo |= x;
    }
    for (int o = 32; o > 0; o >>= 1) {
        va &= __shfl_xor(va, o);
        vo |= __shfl_xor(vo, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = va;
        red[1][threadIdx.x >> 6] = vo;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 1; j < TB / 64; ++j) {
            va &= red[0][j];
            vo |= red[1][j];
        }
        part[2 * ((uint64_t)w * gridDim.x + blockIdx.x)] = va;
        part[2 * ((uint64_t)w * gridDim.x + blockIdx.x) + 1] = vo;
    }
}

struct SelState;
__device__ void sel_state_init(const uint32_t *res, uint32_t nw, uint64_t n, uint32_t k, SelState *st,
                               const uint64_t *d_n);
__device__ void sel_state_skip(SelState *st, uint32_t k);

// res[2w], res[2w + 1] = AND / OR of word w over k_andor's nb partials (one wave per word),
// res[2 kw] = the NaN flag, which is cleared for the next sort, res[2 kw + 1] = a void string
// dictionary, res[2 kw + 2..3] = the device row count (d_n).  With st (the device top-K)
// the selection state is initialised from them too and its histogram cleared.
__global__ __launch_bounds__(1024) void k_andor_final(const uint32_t *__restrict__ part, uint32_t nb, uint32_t KW,
                                                      uint32_t *__restrict__ res, uint32_t *__restrict__ nan_seen,
                                                      SelState *st, uint64_t n, uint32_t k,
                                                      const uint64_t *__restrict__ d_n, uint32_t *__restrict__ hist,
                                                      const uint32_t *__restrict__ dctl = nullptr, uint32_t ndict = 0,
                                                      const uint32_t *skip = nullptr) {
    __shared__ uint32_t r[2 * MAXW];
    if (skip && *skip) {   // a hinted top-K answered: the selection passes find nothing to do
        if (st && threadIdx.x == 0) sel_state_skip(st, k);
        return;
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t w = wave; w < KW; w += 1024 / 64) {
        uint32_t va = 0xFFFFFFFFu, vo = 0;
        for (uint32_t b = lane; b < nb; b += 64) {
            va &= part[2 * ((uint64_t)w * nb + b)];
            vo |= part[2 * ((uint64_t)w * nb + b) + 1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            va &= __shfl_xor(va, o);
            vo |= __shfl_xor(vo, o);
        }
        if (lane == 0) {
            res[2 * w] = r[2 * w] = va;
            res[2 * w + 1] = r[2 * w + 1] = vo;
        }
    }
    if (threadIdx.x == 0) {
        res[2 * KW] = *nan_seen;
        *nan_seen = 0;
        // the read-back's other words: a void dictionary, the device row count
        uint32_t dv = 0;
        for (uint32_t j = 0; j < ndict; ++j) dv |= dctl[4 * j + 1];
        res[2 * KW + 1] = dv;
        const uint64_t dn = d_n ? *d_n : 0;
        res[2 * KW + 2] = (uint32_t)dn;
        res[2 * KW + 3] = (uint32_t)(dn >> 32);
    }
    if (!st) return;
    for (uint32_t b = threadIdx.x; b < (1u << 12); b += 1024) hist[b] = 0;
    __syncthreads();
    if (threadIdx.x == 0) sel_state_init(r, KW, n, k, st, d_n);
}

__global__ __launch_bounds__(STB) void k_radix_hist(const uint32_t *__restrict__ dw, uint32_t shift,
                                                    uint64_t n, uint32_t nblocks,
                                                    uint32_t *__restrict__ hist, uint32_t tile_major) {
    // one histogram per wave (a skewed digit's same-bin adds spread over 16 copies), summed
    __shared__ uint32_t h[STB / 64][256];
    const uint32_t t = threadIdx.x, wave = t >> 6;
    for (uint32_t i = t; i < (STB / 64) * 256; i += STB) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RTILE;
    uint32_t d[SIPT];
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = base + (uint64_t)j * STB + t;
        d[j] = i < n ? dw[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = base + (uint64_t)j * STB + t;
        if (i < n) atomicAdd(&h[wave][(d[j] >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (t < 256) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < STB / 64; ++w) c += h[w][t];
        if (tile_major) hist[(uint64_t)blockIdx.x * 256 + t] = c;
        else hist[(uint64_t)t * nblocks + blockIdx.x] = c;
    }
}

// Three-phase exclusive scan over m u32 values (the [digit][tile] histogram): per-chunk
// sums, one block scanning the chunk sums, per-chunk scans with their carry.
constexpr uint32_t SCAN_CHUNK = 4096;   // 1024 threads x 4

__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t *tmp, uint32_t &total) {
    // tmp: 16 words of LDS; wave-level inclusive scan then wave totals
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    uint32_t wpre = 0;
    total = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        const uint32_t t = tmp[w];
        if (w < wave) wpre += t;
        total += t;
    }
    __syncthreads();
    return wpre + x - v;
}

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint32_t *__restrict__ v, uint64_t m,
                                                      uint32_t *__restrict__ part) {
    __shared__ uint32_t tmp[16];
    const uint64_t b = (uint64_t)blockIdx.x * SCAN_CHUNK + 4 * threadIdx.x;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (b + j < m) ? v[b + j] : 0u;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; ++w) t += tmp[w];
        part[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void k_scan_parts(uint32_t *__restrict__ part, uint32_t np) {
    __shared__ uint32_t tmp[16];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < np; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < np ? part[i] : 0u;
        uint32_t total;
        const uint32_t e = block_excl_scan_1024(v, tmp, total);
        if (i < np) part[i] = carry + e;
        carry += total;
    }
}

__global__ __launch_bounds__(1024) void k_scan_apply(uint32_t *__restrict__ v, uint64_t m,
                                                     const uint32_t *__restrict__ part) {
    __shared__ uint32_t tmp[16];
    const uint64_t b = (uint64_t)blockIdx.x * SCAN_CHUNK + 4 * threadIdx.x;
    uint32_t x[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        x[j] = (b + j < m) ? v[b + j] : 0u;
        s += x[j];
    }
    uint32_t total;
    uint32_t run = part[blockIdx.x] + block_excl_scan_1024(s, tmp, total);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (b + j < m) v[b + j] = run;
        run += x[j];
    }
}

static void launch_scan(hipStream_t st, uint32_t *v, uint64_t m, uint32_t *part) {
    const uint32_t np = (uint32_t)((m + SCAN_CHUNK - 1) / SCAN_CHUNK);
    hipLaunchKernelGGL(k_scan_reduce, dim3(np), dim3(1024), 0, st, v, m, part);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, part, np);
    hipLaunchKernelGGL(k_scan_apply, dim3(np), dim3(1024), 0, st, v, m, part);
}

struct ScatterArgs {
    const uint32_t *in[MAXW];
    uint32_t *out[MAXW];
    uint32_t nlive;
    uint32_t dword;      // index into in[] of the digit word
    uint32_t shift;
    uint32_t nblocks;
    uint64_t n;
    const uint32_t *pin;
    uint32_t *pout;
    const uint32_t *off;  // scanned hist [256][nblocks], or null: the prefetching kernel
                          // scans the raw counts cnt ([nblocks][256]) itself (nblocks <= SCAN_FREE_TILES)
    const uint32_t *cnt;
};

constexpr uint32_t SCAN_FREE_TILES = 512;

// this tile's base of every digit from the raw counts, stored tile-major ([tile][digit]: a
// wave reads 64 digits of one tile in one request): the block's four 256-thread quarters each
// sum digit t's counts over a quarter of the tiles (before this one, and all), TDB_U loads in
// flight per thread; the quarters' sums meet in LDS and the digit totals are scanned across
// the first 256 threads -- the three scan kernels a pass would otherwise need.  Called by the
// whole block; threads 0..255 get digit t's base, the others 0.  tmp: 4 + 2 x 1024 words.
constexpr uint32_t NPART = STB / 256;   // 256-thread parts of a radix block
constexpr int TDB_U = 16;               // count loads in flight per thread (32: no faster on C1)
__device__ __forceinline__ uint32_t tile_digit_base(const uint32_t *__restrict__ cnt, uint32_t nb, uint32_t *tmp) {
    const uint32_t t = threadIdx.x & 255u, part = threadIdx.x >> 8, lane = t & 63, wave = t >> 6;
    const uint32_t me = blockIdx.x;
    const uint32_t q0 = (uint32_t)((uint64_t)nb * part / NPART), q1 = (uint32_t)((uint64_t)nb * (part + 1) / NPART);
    uint32_t pre = 0, tot = 0;
    uint32_t q = q0;
    for (; q + TDB_U <= q1; q += TDB_U) {
        uint32_t v[TDB_U];
#pragma unroll
        for (int u = 0; u < TDB_U; ++u) v[u] = cnt[(uint64_t)(q + u) * 256 + t];
#pragma unroll
        for (int u = 0; u < TDB_U; ++u) {
            tot += v[u];
            if (q + u < me) pre += v[u];
        }
    }
    for (; q < q1; ++q) {
        const uint32_t v = cnt[(uint64_t)q * 256 + t];
        tot += v;
        if (q < me) pre += v;
    }
    uint32_t *spre = tmp + 4, *stot = tmp + 4 + STB;
    spre[threadIdx.x] = pre;
    stot[threadIdx.x] = tot;
    __syncthreads();
    const bool mine = threadIdx.x < 256;
    if (mine) {
        pre = 0;
        tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < NPART; ++q) {
            pre += spre[256 * q + t];
            tot += stot[256 * q + t];
        }
    }
    uint32_t inc = mine ? tot : 0u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d);
        if ((int)lane >= d) inc += y;
    }
    if (mine && lane == 63) tmp[wave] = inc;
    __syncthreads();
    uint32_t ex = inc - (mine ? tot : 0u);
    for (uint32_t w = 0; w < wave; ++w) ex += tmp[w];
    return mine ? ex + pre : 0u;
}

__global__ __launch_bounds__(STB) void k_radix_scatter(ScatterArgs a) {
    __shared__ uint32_t base[256], running[256];
    __shared__ uint32_t wcnt[STB / 64][256], wpre[STB / 64][256];
    const uint32_t t = threadIdx.x, wave = t >> 6;
    if (t < 256) {
        base[t] = a.off[(uint64_t)t * a.nblocks + blockIdx.x];
        running[t] = 0;
    }
    for (uint32_t i = t; i < (STB / 64) * 256; i += STB) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tbase = (uint64_t)blockIdx.x * RTILE;
    const uint32_t *dw = a.in[a.dword];
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = tbase + (uint64_t)j * STB + t;
        const bool valid = i < a.n;
        const uint32_t d = valid ? (dw[i] >> a.shift) & 255u : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t rank = __popcll(peers & lanemask_lt());
        if (valid && rank == 0) wcnt[wave][d] = __popcll(peers);
        __syncthreads();
        if (t < 256) {
            uint32_t r = running[t];
#pragma unroll
            for (int w = 0; w < STB / 64; ++w) {
                wpre[w][t] = r;
                r += wcnt[w][t];
                wcnt[w][t] = 0;
            }
            running[t] = r;
        }
        __syncthreads();
        if (valid) {
            const uint64_t pos = (uint64_t)base[d] + wpre[wave][d] + rank;
            for (uint32_t w = 0; w < a.nlive; ++w) a.out[w][pos] = a.in[w][i];
            a.pout[pos] = a.pin[i];
        }
    }
}

// The same pass for at most NLMAX live words: every row of the tile (SIPT per thread) is
// loaded up front, so their round trips overlap each other and the ballots and barriers (the
// generic kernel loads them only at the write, after both barriers).
template <int NLMAX>
__global__ __launch_bounds__(STB) void k_radix_scatter_pf(ScatterArgs a) {
    __shared__ uint32_t base[256], running[256], stmp[4 + 2 * STB];
    __shared__ uint32_t wcnt[STB / 64][256], wpre[STB / 64][256];
    const uint32_t t = threadIdx.x, wave = t >> 6;
    const uint32_t b0 = a.off ? (t < 256 ? a.off[(uint64_t)t * a.nblocks + blockIdx.x] : 0u)
                              : tile_digit_base(a.cnt, a.nblocks, stmp);
    if (t < 256) {
        base[t] = b0;
        running[t] = 0;
    }
    for (uint32_t i = t; i < (STB / 64) * 256; i += STB) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tbase = (uint64_t)blockIdx.x * RTILE;
    uint32_t cw[SIPT][NLMAX], cp[SIPT];
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = tbase + (uint64_t)j * STB + t;
        if (i < a.n) {
#pragma unroll
            for (int w = 0; w < NLMAX; ++w)
                if ((uint32_t)w < a.nlive) cw[j][w] = a.in[w][i];
            cp[j] = a.pin[i];
        }
    }
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = tbase + (uint64_t)j * STB + t;
        const bool valid = i < a.n;
        uint32_t dv = 0;
#pragma unroll
        for (int w = 0; w < NLMAX; ++w)
            if ((uint32_t)w == a.dword) dv = cw[j][w];
        const uint32_t d = valid ? (dv >> a.shift) & 255u : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t rank = __popcll(peers & lanemask_lt());
        if (valid && rank == 0) wcnt[wave][d] = __popcll(peers);
        __syncthreads();
        if (t < 256) {
            uint32_t r = running[t];
#pragma unroll
            for (int w = 0; w < STB / 64; ++w) {
                wpre[w][t] = r;
                r += wcnt[w][t];
                wcnt[w][t] = 0;
            }
            running[t] = r;
        }
        __syncthreads();
        if (valid) {
            const uint64_t pos = (uint64_t)base[d] + wpre[wave][d] + rank;
#pragma unroll
            for (int w = 0; w < NLMAX; ++w)
                if ((uint32_t)w < a.nlive) a.out[w][pos] = cw[j][w];
            a.pout[pos] = cp[j];
        }
    }
}

// ---- device-planned LSD passes (full sorts without float keys, composed keys <= 8 words) ----
// The same stable LSD order as the host-planned passes above, with no host round trip and one
// launch per possible byte digit (least significant first).  Each pass kernel decides on the
// device whether its digit varies -- its global histogram, added up by the pass before it, has
// no bin holding all n rows -- and, if not, only histograms the next digit and exits (the buffers
// stay as they are).  An active pass:
//   - takes a ticket (tile order = dispatch order), loads its tile's rows (the words up to its
//     own, the payload), ranks every row among its wave's equal digits (multi-split ballots);
//   - publishes its 256 digit counts as tagged 64-bit words (sc1 stores) and sums the counts of
//     the tiles before it (sc1 polls of the tags: those tiles hold earlier tickets, so they are
//     running or done) -- the stable base of each digit in this tile;
//   - adds the NEXT digit's counts of its rows to that digit's global histogram (rows are only
//     permuted by a pass, so any tiling gives the same totals; 8 replicas against same-address
//     serialisation);
//   - writes its rows through LDS in tile-sorted order, so consecutive lanes store consecutive
//     addresses of a digit's run instead of scattering one 4-byte store per lane;
//   - the last tile to finish flips the current-buffer word for the next pass.
// The first digit's histogram comes from k_lsd_h0; k_lsd_out copies the final payload.  The row
// count may live on the device (d_n): grids are sized for the upper bound, extra tiles exit.
// Tags carry (call epoch, pass), so the status words are never cleared.
constexpr int LSD_MAXW = 8;
constexpr int LSD_MAXD = 4 * LSD_MAXW;
constexpr int LSD_REP = 8;   // global histogram replicas per digit

struct LsdCtl {
    uint32_t cur, err, pad0, pad1;
    uint32_t ticket[LSD_MAXD];
    uint32_t done[LSD_MAXD];
    uint32_t hist[LSD_MAXD][LSD_REP][256];   // per digit, replicated; zeroed per call
};

// wave64 multi-split: the lanes (of `act`) whose 8-bit digit equals this lane's
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, uint64_t act) {
    uint64_t peers = act;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

__device__ __forceinline__ uint32_t lsd_n(uint64_t nmax, const uint64_t *d_n) {
    return (uint32_t)(d_n ? min(nmax, *d_n) : nmax);
}

// add the digit counts of this block's rows (LDS h[256], already summed) to replica blockIdx % 8
__device__ __forceinline__ void lsd_hist_flush(uint32_t *h, LsdCtl *ctl, uint32_t q) {
    __syncthreads();
    if (threadIdx.x < 256 && h[threadIdx.x])
        atomicAdd(&ctl->hist[q][blockIdx.x % LSD_REP][threadIdx.x], h[threadIdx.x]);
}

// per-row digit -> LDS counts: one add per distinct digit of a wave
__device__ __forceinline__ void lsd_count(uint32_t *h, uint32_t d, bool ok) {
    const uint64_t peers = digit_peers(d, __ballot(ok));
    if (ok && (peers & lanemask_lt()) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
}

// the first digit's histogram: byte 0 of the last (least significant) word
__global__ __launch_bounds__(STB) void k_lsd_h0(const uint32_t *__restrict__ W, uint32_t KW, uint64_t stride,
                                                uint64_t nmax, const uint64_t *__restrict__ d_n, LsdCtl *ctl) {
    __shared__ uint32_t h[256];
    const uint32_t n = lsd_n(nmax, d_n);
    const uint64_t base = (uint64_t)blockIdx.x * RTILE;
    if (base >= n) return;
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t *col = W + (uint64_t)(KW - 1) * stride;
    uint32_t v[SIPT];
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = base + (uint64_t)j * STB + threadIdx.x;
        v[j] = i < n ? col[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < SIPT; ++j) lsd_count(h, v[j] & 255u, base + (uint64_t)j * STB + threadIdx.x < n);
    lsd_hist_flush(h, ctl, 0);
}

struct LsdArgs {
    uint32_t *W[2];
    uint32_t *P[2];
    uint64_t stride, nmax;
    const uint64_t *d_n;
    uint64_t *status;     // [tile][256] tagged counts (the context's own array)
    LsdCtl *ctl;
    uint32_t KW, pass, tag, pad;
};

template <int NLMAX>
__global__ __launch_bounds__(STB) void k_lsd_pass(LsdArgs a) {
    __shared__ uint32_t wc[SIPT][STB / 64][256];   // counts, then exclusive offsets inside each digit
    __shared__ uint32_t gb[256], toff[256], base[256], qsum[NPART < 4 ? 4 : NPART][256], hn[256];
    __shared__ uint32_t stage[RTILE];
    __shared__ uint8_t sdig[RTILE];
    __shared__ uint32_t tile_s, flags;
    const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t n = lsd_n(a.nmax, a.d_n);
    const uint32_t p = a.pass, ND = 4 * a.KW;
    const uint32_t w = a.KW - 1 - p / 4, shift = 8 * (p % 4);
    const bool has_next = p + 1 < ND;
    const uint32_t wn = a.KW - 1 - (p + 1) / 4, shn = 8 * ((p + 1) % 4);   // the next digit
    // this digit's global histogram (summed replicas): constant iff one bin holds all n rows
    if (t == 0) flags = 0;
    if (t < 256) hn[t] = 0;
    __syncthreads();
    if (t < 256) {
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < LSD_REP; ++r) c += a.ctl->hist[p][r][t];
        gb[t] = c;
        if (c == n) flags = 1;
    }
    __syncthreads();
    const uint32_t cur = a.ctl->cur;
    if (flags || n < 2) {
        // inactive: only the next digit's histogram (over this block's rows of the unchanged buffer)
        const uint64_t tb = (uint64_t)blockIdx.x * RTILE;
        if (!has_next || tb >= n || n < 2) return;
        const uint32_t *col = a.W[cur] + (uint64_t)wn * a.stride;
#pragma unroll
        for (int j = 0; j < SIPT; ++j) {
            const uint64_t i = tb + (uint64_t)j * STB + t;
            lsd_count(hn, i < n ? (col[i] >> shn) & 255u : 0u, i < n);
        }
        lsd_hist_flush(hn, a.ctl, p + 1);
        return;
    }
    // global exclusive base of each digit value (256-thread scan of gb)
    if (t < 256) {
        const uint32_t c = gb[t];
        uint32_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if ((int)lane >= d) inc += y;
        }
        if (lane == 63) qsum[0][wave] = inc;
        base[t] = inc - c;
    }
    if (t == 0) tile_s = atomicAdd(&a.ctl->ticket[p], 1u);
    for (uint32_t i = t; i < SIPT * (STB / 64) * 256; i += STB) (&wc[0][0][0])[i] = 0;
    __syncthreads();
    if (t < 256) {
        for (uint32_t q = 0; q < wave; ++q) base[t] += qsum[0][q];
        gb[t] = base[t];   // keep: the global base of digit t
    }
    __syncthreads();   // qsum is rewritten by the predecessor sums below
    const uint32_t tile = tile_s;
    const uint32_t ntiles = (n + RTILE - 1) / RTILE;
    if (tile >= ntiles) return;
    const uint32_t nl = w + 1;   // every word up to this one is carried
    const uint64_t tbase = (uint64_t)tile * RTILE;
    uint32_t cw[SIPT][NLMAX], cp[SIPT], dg[SIPT], rk[SIPT];
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const uint64_t i = tbase + (uint64_t)j * STB + t;
        if (i < n) {
#pragma unroll
            for (int l = 0; l < NLMAX; ++l)
                if ((uint32_t)l < nl) cw[j][l] = a.W[cur][(uint64_t)l * a.stride + i];
            cp[j] = a.P[cur][i];
        }
    }
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        const bool valid = tbase + (uint64_t)j * STB + t < n;
        uint32_t dv = 0, dvn = 0;
#pragma unroll
        for (int l = 0; l < NLMAX; ++l) {
            if ((uint32_t)l == w) dv = cw[j][l];
            if ((uint32_t)l == wn) dvn = cw[j][l];
        }
        dg[j] = valid ? (dv >> shift) & 255u : 0u;
        const uint64_t peers = digit_peers(dg[j], __ballot(valid));
        rk[j] = (uint32_t)__popcll(peers & lt);
        if (valid && rk[j] == 0) wc[j][wave][dg[j]] = (uint32_t)__popcll(peers);
        if (has_next) lsd_count(hn, valid ? (dvn >> shn) & 255u : 0u, valid);
    }
    __syncthreads();
    if (t < 256) {   // (sub-row, wave) order is the tile's row order: the stable offsets
        uint32_t r = 0;
#pragma unroll
        for (int j = 0; j < SIPT; ++j) {
#pragma unroll
            for (int v = 0; v < STB / 64; ++v) {
                const uint32_t x = wc[j][v][t];
                wc[j][v][t] = r;
                r += x;
            }
        }
        __hip_atomic_store(&a.status[(uint64_t)tile * 256 + t], ((uint64_t)a.tag << 32) | r, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        toff[t] = r;   // the tile's count of digit t (scanned below)
        if (has_next && hn[t]) atomicAdd(&a.ctl->hist[p + 1][tile % LSD_REP][t], hn[t]);
    }
    // the counts of the tiles before this one: four quarters of 256 threads, one digit each
    {
        const uint32_t d = t & 255u, q = t >> 8;
        const uint32_t q0 = tile * q / NPART, q1 = tile * (q + 1) / NPART;
        uint32_t sum = 0;
        for (uint32_t j = q0; j < q1; j += 8) {   // 8 polls in flight per thread
            uint64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                v[u] = j + u < q1 ? __hip_atomic_load(&a.status[(uint64_t)(j + u) * 256 + d], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : (uint64_t)a.tag << 32;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                uint32_t spins = 0;
                while ((uint32_t)(v[u] >> 32) != a.tag) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 22)) {   // never expected: a tile before this one holds an earlier ticket
                        atomicOr(&a.ctl->err, 1u);
                        break;
                    }
                    v[u] = __hip_atomic_load(&a.status[(uint64_t)(j + u) * 256 + d], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                }
                sum += (uint32_t)v[u];
            }
        }
        qsum[q][d] = sum;
    }
    __syncthreads();
    if (t < 256) {
        // where digit t's run starts in this tile's LDS order (exclusive scan of the tile counts),
        // and where it goes: the digit's global base + the tiles before this one
        const uint32_t c = toff[t];
        uint32_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if ((int)lane >= d) inc += y;
        }
        uint32_t pre = 0;
#pragma unroll
        for (uint32_t q = 0; q < NPART; ++q) pre += qsum[q][t];
        base[t] = gb[t] + pre;
        gb[t] = inc - c;   // wave-local exclusive start (gb is free now)
        if (lane == 63) hn[wave] = inc;   // wave totals (hn is free now)
    }
    __syncthreads();
    if (t < 256) {
        uint32_t add = 0;
        for (uint32_t q = 0; q < wave; ++q) add += hn[q];
        toff[t] = gb[t] + add;
    }
    __syncthreads();
    // tile-sorted LDS position of each row, then every carried word and the payload staged
    uint32_t lp[SIPT];
#pragma unroll
    for (int j = 0; j < SIPT; ++j) {
        lp[j] = toff[dg[j]] + wc[j][wave][dg[j]] + rk[j];
        if (tbase + (uint64_t)j * STB + t < n) sdig[lp[j]] = (uint8_t)dg[j];
    }
    const uint32_t tn = min<uint32_t>(RTILE, n - (uint32_t)tbase);
    for (uint32_t l = 0; l <= nl; ++l) {   // l == nl: the payload
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SIPT; ++j) {
            if (tbase + (uint64_t)j * STB + t < n) {
                uint32_t x = cp[j];
#pragma unroll
                for (int m = 0; m < NLMAX; ++m)
                    if ((uint32_t)m == l && l < nl) x = cw[j][m];   // l == nl: the payload
                stage[lp[j]] = x;
            }
        }
        __syncthreads();
        uint32_t *out = l < nl ? a.W[cur ^ 1] + (uint64_t)l * a.stride : a.P[cur ^ 1];
        for (uint32_t i = t; i < tn; i += STB) {
            const uint32_t d = sdig[i];
            out[base[d] + i - toff[d]] = stage[i];
        }
    }
    __syncthreads();
    if (t == 0) {
        __threadfence();
        if (atomicAdd(&a.ctl->done[p], 1u) == ntiles - 1) a.ctl->cur = cur ^ 1;   // the next pass reads what this wrote
    }
}

__global__ __launch_bounds__(256) void k_lsd_out(uint32_t *const P0, uint32_t *const P1, const LsdCtl *__restrict__ ctl,
                                                 uint64_t nmax, const uint64_t *__restrict__ d_n, uint32_t limit,
                                                 uint32_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t n = min<uint64_t>(lsd_n(nmax, d_n), limit ? limit : nmax);
    if (i >= n) return;
    out[i] = ctl->err ? 0xFFFFFFFFu : (ctl->cur ? P1 : P0)[i];   // a failed wait poisons the result
}

// ---- top-K by radix select (k <= SEL_SMALL_K) -----------------------------------------
// The composed keys are unique (the position word is part of them), so the k smallest
// rows form an exact set.  Each pass histograms a 12-bit digit of the candidates
// (MSB first, starting at the first bit that varies), keeps every row whose digit is below
// the bin holding the k-th row and carries the rows of that bin to the next pass.  The
// accepted k rows are then ranked against each other (one workgroup per row).
constexpr int SEL_BITS = 12;
constexpr uint32_t SEL_BINS = 1u << SEL_BITS;
constexpr uint32_t SEL_SMALL_K = 4096;

__device__ __forceinline__ uint32_t sel_digit(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                              uint64_t i, uint32_t bitpos, uint32_t nbits) {
    const uint32_t w = bitpos >> 5, o = bitpos & 31;
    const uint64_t hi = W[(uint64_t)w * stride + i];
    const uint64_t lo = (w + 1 < nw) ? W[(uint64_t)(w + 1) * stride + i] : 0ull;
    const uint64_t x = (hi << 32) | lo;
    return (uint32_t)((x << o) >> (64 - nbits));
}

__global__ __launch_bounds__(TB) void k_sel_hist(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                 const uint32_t *__restrict__ cand, uint64_t n, uint32_t bitpos,
                                                 uint32_t nbits, uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[SEL_BINS];
    for (uint32_t b = threadIdx.x; b < SEL_BINS; b += TB) h[b] = 0;
    __syncthreads();
    for (uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x; j < n; j += (uint64_t)gridDim.x * TB) {
        const uint64_t i = cand ? cand[j] : j;
        atomicAdd(&h[sel_digit(W, stride, nw, i, bitpos, nbits)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < SEL_BINS; b += TB)
        if (h[b]) atomicAdd(&hist[b], h[b]);
}

// rows with digit < b -> acc (appended), digit == b -> out (next candidates).  One global
// reservation per workgroup and list (a single returning atomic word saturates quickly).
__global__ __launch_bounds__(TB) void k_sel_split(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                  const uint32_t *__restrict__ cand, uint64_t n, uint32_t bitpos,
                                                  uint32_t nbits, uint32_t b, uint32_t *__restrict__ acc,
                                                  uint32_t *__restrict__ acc_cnt, uint32_t *__restrict__ out,
                                                  uint32_t *__restrict__ out_cnt) {
    __shared__ uint32_t lcnt[2], gbase[2];
    if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t row[IPT], pos[IPT];
    uint32_t kind[IPT];   // 0 drop, 1 accept, 2 carry
    const uint64_t tbase = (uint64_t)blockIdx.x * TILE;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t q = tbase + (uint64_t)j * TB + threadIdx.x;
        kind[j] = 0;
        row[j] = 0;
        if (q < n) {
            row[j] = cand ? cand[q] : (uint32_t)q;
            const uint32_t d = sel_digit(W, stride, nw, row[j], bitpos, nbits);
            kind[j] = d < b ? 1u : (d == b ? 2u : 0u);
        }
        const uint64_t m1 = __ballot(kind[j] == 1), m2 = __ballot(kind[j] == 2);
        uint32_t b1 = 0, b2 = 0;
        if (lane == 0) {
            if (m1) b1 = atomicAdd(&lcnt[0], (uint32_t)__popcll(m1));
            if (m2) b2 = atomicAdd(&lcnt[1], (uint32_t)__popcll(m2));
        }
        b1 = __shfl(b1, 0);
        b2 = __shfl(b2, 0);
        pos[j] = kind[j] == 1 ? b1 + __popcll(m1 & lanemask_lt()) : b2 + __popcll(m2 & lanemask_lt());
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        gbase[0] = lcnt[0] ? atomicAdd(acc_cnt, lcnt[0]) : 0;
        gbase[1] = lcnt[1] ? atomicAdd(out_cnt, lcnt[1]) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (kind[j] == 1) acc[gbase[0] + pos[j]] = row[j];
        else if (kind[j] == 2) out[gbase[1] + pos[j]] = row[j];
    }
}

// ---- the same selection without host round trips ------------------------------------------
// (top-K of keys without floats, where no NaN check is needed: the tables' SortStats).  The
// first pass runs grid-wide with its bin picked on the device; the few candidates it leaves
// (the rows of one 12-bit bin) are finished by one workgroup.
struct SelState {
    uint32_t bitpos, nbits, b, krem, n, acc_cnt, out_cnt, err;
};

__device__ void sel_state_init(const uint32_t *res, uint32_t nw, uint64_t n, uint32_t k, SelState *st,
                               const uint64_t *d_n) {
    if (d_n) n = min(n, *d_n);
    uint32_t bitpos = nw * 32;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint32_t diff = res[2 * w] ^ res[2 * w + 1];
        if (diff) {
            bitpos = 32 * w + (uint32_t)__clz(diff);
            break;
        }
    }
    st->bitpos = bitpos;
    st->nbits = min((uint32_t)SEL_BITS, nw * 32 - min(bitpos, nw * 32));
    st->b = 0;
    st->krem = k;
    st->n = (uint32_t)n;
    st->acc_cnt = 0;
    st->out_cnt = 0;
    st->err = 0;
}

// no rows: the selection passes return at once
__device__ void sel_state_skip(SelState *st, uint32_t k) {
    st->n = 0;
    st->krem = k;
    st->nbits = 0;
    st->b = 0;
    st->acc_cnt = st->out_cnt = st->err = 0;
}

__global__ __launch_bounds__(TB) void k_sel_hist_d(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                   const SelState *__restrict__ st, uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[SEL_BINS];
    const uint32_t n = st->n, bitpos = st->bitpos, nbits = st->nbits;
    if (n <= st->krem || nbits == 0) return;
    for (uint32_t b = threadIdx.x; b < SEL_BINS; b += TB) h[b] = 0;
    __syncthreads();
    // A table's sums are skewed: most groups share the lowest bins, and same-address LDS
    // atomics serialise, so the lanes on the wave's first lane's bin add as one
    for (uint64_t j0 = (uint64_t)blockIdx.x * TB; j0 < n; j0 += (uint64_t)gridDim.x * TB) {
        const uint64_t j = j0 + threadIdx.x;
        const bool live = j < n;
        const uint32_t d = live ? sel_digit(W, stride, nw, j, bitpos, nbits) : 0xFFFFFFFFu;
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
        const uint64_t same = __ballot(d == d0);
        if (d == d0) {
            if ((threadIdx.x & 63) == (uint32_t)__ffsll((long long)same) - 1 && d0 != 0xFFFFFFFFu)
                atomicAdd(&h[d0], (uint32_t)__popcll(same));
        } else if (live) {
            atomicAdd(&h[d], 1u);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < SEL_BINS; b += TB)
        if (h[b]) atomicAdd(&hist[b], h[b]);
}

// the bin holding the krem-th row: b, and the rows below it (accepted)
__device__ __forceinline__ void sel_pick_block(const uint32_t *hist, uint32_t krem, uint32_t *tmp, uint32_t &b,
                                               uint32_t &below, uint32_t &inb) {
    // 1024 threads x 4 bins, inclusive prefix per thread, then across the block
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = hist[threadIdx.x * 4 + j];
        s += v[j];
    }
    uint32_t total;
    const uint32_t ex = block_excl_scan_1024(s, tmp, total);
    uint32_t run = ex;
    if (threadIdx.x == 0) tmp[16] = SEL_BINS;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (run < krem && run + v[j] >= krem) {   // exactly one bin crosses
            tmp[16] = threadIdx.x * 4 + j;
            tmp[17] = run;
            tmp[18] = v[j];
        }
        run += v[j];
    }
    __syncthreads();
    b = tmp[16];
    below = tmp[17];
    inb = tmp[18];
    __syncthreads();
}

// the bin holding the krem-th row, found by each split workgroup itself (TB threads x 16 bins;
// the histogram is 16 KB in L2): no pick kernel between the histogram and the split
__device__ __forceinline__ uint32_t sel_pick_tb(const uint32_t *__restrict__ hist, uint32_t krem, uint32_t *tmp) {
    constexpr uint32_t PER = SEL_BINS / TB;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4 *h4 = reinterpret_cast<const uint4 *>(hist + threadIdx.x * PER);
    uint32_t v[PER], s = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER / 4; ++q) {
        const uint4 x = h4[q];
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) s += v[j];
    uint32_t inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d);
        if ((int)lane >= d) inc += y;
    }
    if (lane == 63) tmp[wave] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (uint32_t q = 0; q < wave; ++q) run += tmp[q];
    if (run < krem && run + s >= krem) {   // exactly one thread's bins cross krem
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            if (run < krem && run + v[j] >= krem) tmp[TB / 64] = threadIdx.x * PER + j;
            run += v[j];
        }
    }
    __syncthreads();
    return tmp[TB / 64];
}

// grid-wide split of pass 1 (rows are 0..n-1): digit < b -> acc, digit == b -> out
__global__ __launch_bounds__(TB) void k_sel_split_d(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                    SelState *st, const uint32_t *__restrict__ hist,
                                                    uint32_t *__restrict__ acc, uint32_t *__restrict__ out) {
    const uint32_t n = st->n;
    if (n <= st->krem || st->nbits == 0) return;
    __shared__ uint32_t ptmp[TB / 64 + 1];
    const uint32_t bitpos = st->bitpos, nbits = st->nbits, b = sel_pick_tb(hist, st->krem, ptmp);
    __shared__ uint32_t lcnt[2], gbase[2];
    if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t row[IPT], pos[IPT], kind[IPT];
    const uint64_t tbase = (uint64_t)blockIdx.x * TILE;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t q = tbase + (uint64_t)j * TB + threadIdx.x;
        kind[j] = 0;
        row[j] = (uint32_t)q;
        if (q < n) {
            const uint32_t d = sel_digit(W, stride, nw, q, bitpos, nbits);
            kind[j] = d < b ? 1u : (d == b ? 2u : 0u);
        }
        const uint64_t m1 = __ballot(kind[j] == 1), m2 = __ballot(kind[j] == 2);
        uint32_t b1 = 0, b2 = 0;
        if (lane == 0) {
            if (m1) b1 = atomicAdd(&lcnt[0], (uint32_t)__popcll(m1));
            if (m2) b2 = atomicAdd(&lcnt[1], (uint32_t)__popcll(m2));
        }
        b1 = __shfl(b1, 0);
        b2 = __shfl(b2, 0);
        pos[j] = kind[j] == 1 ? b1 + __popcll(m1 & lanemask_lt()) : b2 + __popcll(m2 & lanemask_lt());
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        gbase[0] = lcnt[0] ? atomicAdd(&st->acc_cnt, lcnt[0]) : 0;
        gbase[1] = lcnt[1] ? atomicAdd(&st->out_cnt, lcnt[1]) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (kind[j] == 1) acc[gbase[0] + pos[j]] = row[j];
        else if (kind[j] == 2) out[gbase[1] + pos[j]] = row[j];
    }
}

// one workgroup: the remaining passes over the candidates of pass 1 (or all rows when n <= k),
// then acc holds exactly k rows
__global__ __launch_bounds__(1024) void k_sel_finish(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                     SelState *st, uint32_t *__restrict__ acc, uint32_t *cnd0,
                                                     uint32_t *cnd1, uint32_t k, const uint32_t *__restrict__ payload,
                                                     uint32_t *__restrict__ out, const uint32_t *skip = nullptr) {
    __shared__ uint32_t h[SEL_BINS];
    __shared__ uint32_t tmp[20], cnt[2];
    if (skip && *skip) return;
    uint32_t n = st->n, krem = st->krem, bitpos = st->bitpos, nbits = st->nbits, nacc = 0;
    const uint32_t *cand = nullptr;   // nullptr: rows 0..n-1
    uint32_t *nxt = cnd0;
    if (n > krem && nbits) {   // pass 1 ran grid-wide
        nacc = st->acc_cnt;
        krem -= nacc;
        n = st->out_cnt;
        cand = cnd0;
        nxt = cnd1;
        bitpos += nbits;
    }
    while (n > krem) {
        if (bitpos >= nw * 32) {   // composed keys equal: cannot happen (the position is in them)
            if (threadIdx.x == 0) st->err = 1;
            return;
        }
        nbits = min((uint32_t)SEL_BITS, nw * 32 - bitpos);
        for (uint32_t b = threadIdx.x; b < SEL_BINS; b += 1024) h[b] = 0;
        if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < n; j += 1024)
            atomicAdd(&h[sel_digit(W, stride, nw, cand ? cand[j] : j, bitpos, nbits)], 1u);
        __syncthreads();
        uint32_t b, below, inb;
        sel_pick_block(h, krem, tmp, b, below, inb);
        for (uint32_t j = threadIdx.x; j < n; j += 1024) {
            const uint32_t i = cand ? cand[j] : j;
            const uint32_t d = sel_digit(W, stride, nw, i, bitpos, nbits);
            if (d < b) acc[nacc + atomicAdd(&cnt[0], 1u)] = i;
            else if (d == b) nxt[atomicAdd(&cnt[1], 1u)] = i;
        }
        __syncthreads();
        nacc += below;
        krem -= below;
        n = inb;
        cand = nxt;
        nxt = nxt == cnd0 ? cnd1 : cnd0;
        bitpos += nbits;
        __syncthreads();
    }
    for (uint32_t j = threadIdx.x; j < n; j += 1024) acc[nacc + j] = cand ? cand[j] : j;   // n == krem
    if (!out) return;   // k x words > SEL_BINS: k_sel_rank ranks them
    // rank of each accepted row among the others (full composed-key compare, as k_sel_rank)
    // on an LDS copy of their words; output positions past the rows that exist read 0xFFFFFFFF
    __syncthreads();
    const uint32_t kk = min(k, st->n);
    uint32_t *kw = h;   // the histogram is done with: kk x nw words
    for (uint32_t q = threadIdx.x; q < kk * nw; q += 1024) {
        const uint32_t r = q / nw, w = q % nw;
        kw[q] = W[(uint64_t)w * stride + acc[r]];
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < k; r += 1024) {
        if (r >= kk) {
            out[r] = 0xFFFFFFFFu;
            continue;
        }
        uint32_t less = 0;
        for (uint32_t j = 0; j < kk; ++j) {
            int c = 0;
            for (uint32_t w = 0; w < nw && c == 0; ++w) {
                const uint32_t x = kw[j * nw + w], y = kw[r * nw + w];
                c = x < y ? -1 : (x > y ? 1 : 0);
            }
            less += c < 0;
        }
        out[less] = payload[acc[r]];
    }
}

// rank of acc[r] among the k accepted rows (full composed-key compare) -> out_perm
__global__ __launch_bounds__(TB) void k_sel_rank(const uint32_t *__restrict__ W, uint64_t stride, uint32_t nw,
                                                 const uint32_t *__restrict__ acc, uint32_t k,
                                                 const uint32_t *__restrict__ payload, uint32_t *__restrict__ out,
                                                 const SelState *__restrict__ st, const uint32_t *skip = nullptr) {
    __shared__ uint32_t red[TB / 64];
    if (skip && *skip) return;
    const uint32_t r = blockIdx.x;
    if (st) {   // the row count was on the device: fewer rows than k leave the tail unset
        k = min(k, st->n);
        if (r >= k) {
            if (threadIdx.x == 0) out[r] = 0xFFFFFFFFu;
            return;
        }
    }
    const uint32_t me = acc[r];
    uint32_t less = 0;
    for (uint32_t j = threadIdx.x; j < k; j += TB) {
        const uint32_t o = acc[j];
        int c = 0;
        for (uint32_t w = 0; w < nw && c == 0; ++w) {
            const uint32_t x = W[(uint64_t)w * stride + o], y = W[(uint64_t)w * stride + me];
            c = x < y ? -1 : (x > y ? 1 : 0);
        }
        less += c < 0;
    }
    for (int o = 32; o > 0; o >>= 1) less += __shfl_xor(less, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = less;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < TB / 64; ++w) t += red[w];
        out[t] = payload[me];
    }
}

// ---- the tables' repeated top-K, bounded by a hint ------------------------------------------
// A table's top-K is asked for again every interval, and the groups it returned last time are
// mostly near the top again.  Their keys this interval bound the k-th key (TopkHint,
// igx_internal.h): k_tk_bound finds the k-th smallest composed key among the hinted slots that
// are groups of this interval, k_tk_filter reads one key word per group and keeps the groups at
// or below it (usually a few dozen), k_tk_rank ranks them in one workgroup.  No composed word
// arrays and no selection passes: the tail reads each group's sort key once.  When the bound
// leaves more candidates than one workgroup ranks (or fewer than k hints are groups), `done`
// stays 0 and the full selection runs after it as before; its kernels read `done` and return
// at once when the hinted path answered.
// state: words [0] candidates, [1] done, [2] no bound; the bound (NK + 1 u64) from byte 16;
// [14] / [15] the top-Ks the hinted / the full path answered (igx_groupby_topk_counts); the
// candidates from word 16.
template <int NK>
constexpr uint32_t tk_cc() { return NK <= 2 ? 2048u : 1024u; }   // candidates k_tk_rank holds in LDS
static_assert(64 + 2048 * 4 <= TK_STATE_BYTES, "state holds the candidates");

template <int NK>
__device__ __forceinline__ void tk_tuple(const ComposeArgs &a, uint64_t src, uint64_t (&t)[NK + 1]) {
#pragma unroll
    for (int k = 0; k < NK; ++k) t[k] = *reinterpret_cast<const uint64_t *>(a.ptr[k] + src * a.rstride[k]);
    const uint64_t p = *reinterpret_cast<const uint64_t *>(reinterpret_cast<const uint8_t *>(a.pos) + src * a.pos_stride);
#pragma unroll
    for (int k = 0; k < NK; ++k)
        t[k] = (a.kind[k] == IGX_KIND_INT ? t[k] ^ (1ull << 63) : t[k]) ^ (a.desc[k] ? ~0ull : 0ull);
    t[NK] = a.pos_not ? ~p : p;
}

// -1 / 0 / 1: x before / equal to / after y in the composed order
template <int NK>
__device__ __forceinline__ int tk_cmp(const uint64_t *x, const uint64_t *y) {
#pragma unroll
    for (int k = 0; k <= NK; ++k)
        if (x[k] != y[k]) return x[k] < y[k] ? -1 : 1;
    return 0;
}

template <int NK>
__global__ __launch_bounds__(1024) void k_tk_bound(ComposeArgs a, const uint32_t *__restrict__ hints, uint32_t nh,
                                                   const uint32_t *__restrict__ occ, uint64_t nslots, uint32_t k,
                                                   uint32_t *__restrict__ st) {
    __shared__ uint64_t tup[TK_MAXK][NK + 1];
    __shared__ uint32_t ok[TK_MAXK];
    const uint32_t h = threadIdx.x;
    bool v = false;
    if (h < nh) {
        const uint32_t s = hints[h];
        v = s < nslots && ((occ[s >> 5] >> (s & 31)) & 1u);
        if (v) {
            uint64_t t[NK + 1];
            tk_tuple<NK>(a, s, t);
#pragma unroll
            for (int w = 0; w <= NK; ++w) tup[h][w] = t[w];
        }
    }
    ok[h] = v ? 1u : 0u;
    const uint32_t nvalid = (uint32_t)__syncthreads_count(v);
    if (nvalid < k) {   // no bound: the full selection answers
        if (h == 0) {
            st[0] = 0;
            st[1] = 0;
            st[2] = 1;
        }
        return;
    }
    if (v) {
        uint32_t less = 0, eq = 0;
        for (uint32_t j = 0; j < nh; ++j) {
            if (!ok[j]) continue;
            const int c = tk_cmp<NK>(tup[j], tup[h]);
            less += c < 0;
            eq += c == 0;
        }
        if (less <= k - 1 && less + eq > k - 1) {   // the k-th smallest (equal hints write the same)
            uint64_t *b = reinterpret_cast<uint64_t *>(st + 4);
#pragma unroll
            for (int w = 0; w <= NK; ++w) b[w] = tup[h][w];
        }
    }
    if (h == 0) {
        st[0] = 0;
        st[1] = 0;
        st[2] = 0;
    }
}

// the groups whose composed key is at or below the bound -> candidates (slots); past tk_cc they
// are only counted.  One key word per group decides unless it equals the bound's.
template <int NK>
__global__ __launch_bounds__(TB) void k_tk_filter(ComposeArgs a, uint32_t *__restrict__ st) {
    constexpr int CU = 4;
    if (st[2]) return;
    const uint64_t *bp = reinterpret_cast<const uint64_t *>(st + 4);
    const uint64_t b0 = bp[0];
    uint32_t *cand = st + 16;
    const uint64_t n = a.d_n ? min(a.n, *a.d_n) : a.n;
    const uint64_t inv0 = a.desc[0] ? ~0ull : 0ull;
    const uint64_t sg0 = a.kind[0] == IGX_KIND_INT ? 1ull << 63 : 0ull;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t step = (uint64_t)gridDim.x * TB;
    for (uint64_t i0 = (uint64_t)blockIdx.x * TB + threadIdx.x; i0 - lane < n; i0 += CU * step) {
        uint64_t src[CU], x[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint64_t i = i0 + u * step;
            src[u] = a.rowmap[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) x[u] = *reinterpret_cast<const uint64_t *>(a.ptr[0] + src[u] * a.rstride[0]);
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint64_t i = i0 + u * step;
            const uint64_t c0 = (x[u] ^ sg0) ^ inv0;
            bool take = false;
            if (i < n) {
                if (c0 < b0) {
                    take = true;
                } else if (c0 == b0) {
                    uint64_t t[NK + 1];
                    tk_tuple<NK>(a, src[u], t);
                    take = tk_cmp<NK>(t, bp) <= 0;
                }
            }
            const uint64_t m = __ballot(take);
            if (m) {
                uint32_t base = 0;
                if (lane == (uint32_t)__ffsll((long long)m) - 1) base = atomicAdd(&st[0], (uint32_t)__popcll(m));
                base = __shfl(base, __ffsll((long long)m) - 1);
                const uint32_t r = base + (uint32_t)__popcll(m & lanemask_lt());
                if (take && r < tk_cc<NK>()) cand[r] = (uint32_t)src[u];
            }
        }
    }
}

// rank the candidates (full composed keys, in LDS) -> out[0 .. k) and the next call's hints;
// done = 1.  More candidates than fit, or none bound: done stays 0.
template <int NK>
__global__ __launch_bounds__(1024) void k_tk_rank(ComposeArgs a, uint32_t *__restrict__ st, uint32_t k,
                                                  uint32_t *__restrict__ out, uint32_t *__restrict__ hints) {
    constexpr uint32_t CC = tk_cc<NK>();
    __shared__ uint64_t tup[CC][NK + 1];
    __shared__ uint32_t slot[CC];
    const uint32_t m = st[0];
    if (st[2] || m > CC || m < k) return;
    const uint32_t *cand = st + 16;
    for (uint32_t j = threadIdx.x; j < m; j += 1024) {
        const uint32_t s = cand[j];
        slot[j] = s;
        uint64_t t[NK + 1];
        tk_tuple<NK>(a, s, t);
#pragma unroll
        for (int w = 0; w <= NK; ++w) tup[j][w] = t[w];
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < m; r += 1024) {
        uint32_t less = 0;
        for (uint32_t j = 0; j < m; ++j) less += tk_cmp<NK>(tup[j], tup[r]) < 0;
        if (less < k) {
            out[less] = slot[r];
            hints[less] = slot[r];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st[1] = 1;
        st[14] += 1;
    }
}

// the full selection answered (done == 0, or no hinted path ran: done null): its top-K become
// the next call's hints
__global__ __launch_bounds__(1024) void k_tk_save(const uint32_t *__restrict__ out, uint32_t k,
                                                  uint32_t *__restrict__ hints, const uint32_t *done,
                                                  uint32_t *__restrict__ st) {
    if (done && *done) return;
    for (uint32_t r = threadIdx.x; r < k; r += 1024) hints[r] = out[r];
    if (threadIdx.x == 0) st[15] += 1;
}

// ---- IP address text (gadgets.IPStringFromBytes, pkg/gadgets/helpers.go:111-120) ----------
// netip.AddrFrom4(b[0:4]).String() when family != AF_INET6, else netip.AddrFrom16(b).String():
// dotted decimal; IPv4-mapped as "::ffff:a.b.c.d"; otherwise RFC 5952 hex groups without
// leading zeros, the first longest run of >= 2 zero groups written "::" (Go netip appendTo6).
// Rows are rendered zero-padded to IGX_IPTEXT_WIDTH bytes, so a byte compare of two rows is
// Go's string compare of the two texts.
constexpr int IPW = IGX_IPTEXT_WIDTH;
static_assert(IPW % 8 == 0, "rows are written as 8-byte words");

__device__ __forceinline__ int ip_put_dec(uint8_t *o, int p, uint32_t v) {
    if (v >= 100) o[p++] = (uint8_t)('0' + v / 100);
    if (v >= 10) o[p++] = (uint8_t)('0' + (v / 10) % 10);
    o[p++] = (uint8_t)('0' + v % 10);
    return p;
}

__device__ __forceinline__ int ip_put_hex(uint8_t *o, int p, uint32_t v) {
    bool started = false;
    for (int sh = 12; sh >= 0; sh -= 4) {
        const uint32_t d = (v >> sh) & 15u;
        if (d || started || sh == 0) {
            o[p++] = (uint8_t)(d < 10 ? '0' + d : 'a' + d - 10);
            started = true;
        }
    }
    return p;
}

__device__ __forceinline__ int ip_put4(uint8_t *o, int p, const uint8_t *b) {
    for (int j = 0; j < 4; ++j) {
        if (j) o[p++] = '.';
        p = ip_put_dec(o, p, b[j]);
    }
    return p;
}

__global__ __launch_bounds__(TB) void k_ip_text(const uint8_t *__restrict__ addr, uint32_t astride,
                                                const uint8_t *__restrict__ fam, uint32_t fstride,
                                                const uint32_t *__restrict__ rowmap, uint64_t n,
                                                uint8_t *__restrict__ out) {
    __shared__ uint2 buf[TB][IPW / 8];   // one text per thread
    const uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
    uint8_t *o = reinterpret_cast<uint8_t *>(buf[threadIdx.x]);
    for (int j = 0; j < IPW / 8; ++j) buf[threadIdx.x][j] = make_uint2(0, 0);
    if (i < n) {
        const uint64_t src = rowmap ? rowmap[i] : i;
        uint8_t b[16];
        for (int j = 0; j < 16; ++j) b[j] = addr[src * astride + j];
        const uint32_t f = (uint32_t)fam[src * fstride] | ((uint32_t)fam[src * fstride + 1] << 8);
        int p = 0;
        if (f != 10) {                                   // ipType 4 (tracer.go:199-203)
            p = ip_put4(o, p, b);
        } else {
            bool mapped = b[10] == 0xFF && b[11] == 0xFF;
            for (int j = 0; j < 10; ++j) mapped = mapped && b[j] == 0;
            if (mapped) {
                const char pre[7] = {':', ':', 'f', 'f', 'f', 'f', ':'};
                for (int j = 0; j < 7; ++j) o[p++] = (uint8_t)pre[j];
                p = ip_put4(o, p, b + 12);
            } else {
                uint32_t g[8];
                for (int j = 0; j < 8; ++j) g[j] = ((uint32_t)b[2 * j] << 8) | b[2 * j + 1];
                int zs = 255, ze = 255;   // the first longest run of >= 2 zero groups
                for (int s = 0; s < 8; ++s) {
                    int e = s;
                    while (e < 8 && g[e] == 0) ++e;
                    if (e - s >= 2 && e - s > ze - zs) { zs = s; ze = e; }
                }
                for (int s = 0; s < 8; ++s) {
                    if (s == zs) {
                        o[p++] = ':';
                        o[p++] = ':';
                        s = ze;
                        if (s >= 8) break;
                    } else if (s > 0) {
                        o[p++] = ':';
                    }
                    p = ip_put_hex(o, p, g[s]);
                }
            }
        }
    }
    __syncthreads();
    // write the block's rows x IPW bytes out as 8-B stores
    const uint64_t row0 = (uint64_t)blockIdx.x * TB;
    const uint64_t rows = n - row0 < (uint64_t)TB ? n - row0 : (uint64_t)TB;
    uint2 *dst = reinterpret_cast<uint2 *>(out + row0 * IPW);
    for (uint32_t q = threadIdx.x; q < rows * (IPW / 8); q += TB) dst[q] = buf[q / (IPW / 8)][q % (IPW / 8)];
}

// ---- GroupEntries' float group:sum (pkg/columns/group/group.go:133-156) ---------------------
// flattenValues starts from the group's first entry and, for every later entry in input
// order, does field = SetFloat(field.Float() + cur.Float()): float64 addition, then the
// field's own rounding (a float32 column rounds after every add).  That order is kept: perm is
// a stable sort of the rows by the group key, so each group is one contiguous run in input
// order; the thread at a run's first row walks the run.
__global__ __launch_bounds__(TB) void k_segment_fsum(const uint8_t *__restrict__ keys, uint32_t kstride,
                                                     uint32_t kbytes, const uint32_t *__restrict__ perm,
                                                     uint64_t n, const uint8_t *__restrict__ valid,
                                                     const uint8_t *__restrict__ vals, uint32_t vwidth,
                                                     double *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = perm[i];
    if (valid && !valid[r]) return;
    auto same = [&](uint32_t a, uint32_t b) {
        const uint8_t *p = keys + (uint64_t)a * kstride, *q = keys + (uint64_t)b * kstride;
        for (uint32_t j = 0; j < kbytes; ++j)
            if (p[j] != q[j]) return false;
        return true;
    };
    if (i > 0) {
        const uint32_t pr = perm[i - 1];
        if ((!valid || valid[pr]) && same(pr, r)) return;   // not the first row of its run
    }
    auto val = [&](uint32_t row) -> double {
        return vwidth == 4 ? (double)reinterpret_cast<const float *>(vals)[row]
                           : reinterpret_cast<const double *>(vals)[row];
    };
    double s = val(r);
    for (uint64_t j = i + 1; j < n; ++j) {
        const uint32_t q = perm[j];
        if ((valid && !valid[q]) || !same(q, r)) break;
        s = s + val(q);
        if (vwidth == 4) s = (double)(float)s;   // SetFloat on a float32 field
    }
    out[r] = s;
}

}  // namespace

extern "C" int igx_segment_fsum(igx_ctx *ctx, const uint8_t *keys, uint32_t key_stride, uint32_t key_bytes,
                                const uint32_t *perm, uint64_t n, const uint8_t *valid, const void *vals,
                                uint32_t val_width, double *out) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (!keys || !perm || !vals || !out) return igx_fail(ctx, IGX_EINVAL, "segment_fsum: null argument");
    if (val_width != 4 && val_width != 8) return igx_fail(ctx, IGX_EINVAL, "segment_fsum: float width %u", val_width);
    if (n >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "segment_fsum: too many rows");
    hipLaunchKernelGGL(k_segment_fsum, dim3((unsigned)((n + TB - 1) / TB)), dim3(TB), 0, ctx->stream, keys,
                       key_stride, key_bytes, perm, n, valid, static_cast<const uint8_t *>(vals), val_width, out);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

int launch_ip_text(igx_ctx *ctx, const uint8_t *addr, uint32_t astride, const uint8_t *fam, uint32_t fstride,
                   const uint32_t *rowmap, uint64_t n, uint8_t *out) {
    if (n == 0) return IGX_OK;
    hipLaunchKernelGGL(k_ip_text, dim3((unsigned)((n + TB - 1) / TB)), dim3(TB), 0, ctx->stream, addr, astride, fam,
                       fstride, rowmap, n, out);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

// The pre-sort order when there is no position column: row r (or rowmap[r])
__global__ void k_iota_map(uint32_t *out, const uint32_t *rowmap, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = rowmap ? rowmap[i] : (uint32_t)i;
}

// A NaN in a float key: run SliceStable itself (k_gostable.hip) from the pre-sort order.
static int sort_exact_go(igx_ctx *ctx, const SortPlanKey *keys, uint32_t nkeys, uint64_t nrows, const uint64_t *pos,
                         const uint8_t *valid, uint32_t *out_perm, uint32_t limit, const uint32_t *rowmap,
                         uint32_t pos_stride, const GoSortKey *gokeys, uint32_t ngokeys) {
    for (uint32_t k = 0; k < nkeys; ++k)
        if (keys[k].direct)   // per-row rendered text (IP addresses) is indexed by sorted row, not by source row
            return igx_fail(ctx, IGX_ENOTSUP, "sort: NaN float key together with an IP-text key");
    uint32_t *data = nullptr;
    IGX_HIP(ctx, hipMalloc(&data, nrows * 4));
    int rc = IGX_OK;
    if (pos)   // rows in position order (a sort on the position alone)
        rc = launch_sort_perm(ctx, nullptr, 0, nrows, pos, false, nullptr, data, 0, rowmap, pos_stride);
    else
        hipLaunchKernelGGL(k_iota_map, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, ctx->stream, data, rowmap,
                           nrows);
    if (!rc) rc = launch_go_stable(ctx, gokeys, ngokeys, nrows, valid, data);
    const uint64_t m = limit ? std::min<uint64_t>(limit, nrows) : nrows;
    if (!rc && hipMemcpyAsync(out_perm, data, m * 4, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess) rc = IGX_EIO;
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(data);
    if (rc) return rc == IGX_EIO ? igx_fail(ctx, rc, "sort: exact path copy failed") : rc;
    return IGX_OK;
}

int launch_sort_perm(igx_ctx *ctx, const SortPlanKey *keys, uint32_t nkeys, uint64_t nrows,
                     const uint64_t *pos, bool pos_not, const uint8_t *valid,
                     uint32_t *out_perm, uint32_t limit, const uint32_t *rowmap, uint32_t pos_stride,
                     const GoSortKey *gokeys, uint32_t ngokeys, const uint64_t *d_nrows, TopkHint *hint) {
    if (nrows == 0) return IGX_OK;
    if (nrows >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "sort: too many rows");
    if (nkeys > NSK) return igx_fail(ctx, IGX_ENOTSUP, "sort: more than %d keys", NSK);
    ComposeArgs ca{};
    uint32_t KW = valid ? 1 : 0;
    for (uint32_t k = 0; k < nkeys; ++k) {
        ca.ptr[k] = keys[k].ptr;
        ca.width[k] = keys[k].width;
        ca.kind[k] = keys[k].kind;
        ca.desc[k] = keys[k].desc_eff;
        ca.words[k] = keys[k].words;
        ca.rstride[k] = keys[k].stride ? keys[k].stride : keys[k].width;
        ca.direct[k] = keys[k].direct;
        KW += keys[k].words;
    }
    ca.rowmap = rowmap;
    ca.d_n = d_nrows;
    bool any_float = false;
    for (uint32_t k = 0; k < nkeys; ++k) any_float = any_float || keys[k].kind == IGX_KIND_FLOAT;
    // A full sort by row order (no position column, no nil mask) needs no position words: the
    // LSD passes are stable, so composing the rows in the tie order -- ascending, or reversed
    // when the parity makes it descending -- orders the ties without passes of their own.  (A
    // top-K keeps them: the selection needs unique keys.)
    const bool sel_shape = limit && limit <= SEL_SMALL_K && nrows > 2ull * limit;
    const bool drop_pos = pos == nullptr && valid == nullptr && !sel_shape && !std::getenv("IGX_SORT_POSWORDS");
    const uint32_t pos_words = drop_pos ? 0 : (pos == nullptr ? 1 : 2);
    ca.reverse = drop_pos && pos_not ? 1u : 0u;
    KW += pos_words;
    if (KW > MAXW) return igx_fail(ctx, IGX_ENOTSUP, "sort: composed key too wide");
    ca.nkeys = nkeys;
    ca.has_nil = valid ? 1 : 0;
    ca.pos_words = pos_words;
    ca.pos_not = pos_not ? 1 : 0;
    ca.pos = pos;
    ca.pos_stride = pos_stride ? pos_stride : 8;
    ca.valid = valid;
    ca.n = nrows;
    const uint64_t stride = igx_align(nrows, 64);
    ca.stride = stride;

    const uint32_t nblocks = (uint32_t)((nrows + RTILE - 1) / RTILE);
    const size_t words_b = igx_align((size_t)KW * stride * 4, 256);
    const size_t pay_b = igx_align(stride * 4, 256);
    const size_t hist_b = igx_align((size_t)256 * nblocks * 4, 256) +
                          igx_align(((size_t)256 * nblocks + SCAN_CHUNK - 1) / SCAN_CHUNK * 4, 256);
    constexpr uint32_t ANDOR_BLOCKS = 256;
    const size_t res_b = igx_align((size_t)KW * 8 + 16, 256) +
                         igx_align((size_t)KW * std::max<uint32_t>(ANDOR_BLOCKS, CAO_BLOCKS) * 8, 256);
    const bool use_sel = limit && limit <= SEL_SMALL_K && nrows > 2ull * limit;
    // Full sorts without float keys may plan their passes on the device (k_lsd_*: no host read at
    // all) with IGX_SORT_DEVPLAN=1.  Measured on C1 (1M rows, 16 live digits) they are slower
    // than the host-planned passes (0.55-0.61 vs 0.46 ms), so the default is the
    // host plan: one read-back of the AND/OR words -- and of a device row count, when there is
    // one -- per sort.
    const bool use_lsd = !use_sel && !any_float && KW > 0 && KW <= (uint32_t)LSD_MAXW &&
                         std::getenv("IGX_SORT_DEVPLAN") != nullptr;
    if (d_nrows && (any_float || (use_sel && !(rowmap && !valid))))
        return igx_fail(ctx, IGX_EINVAL, "sort: a device row count needs integer or string keys (and, for a top-K, "
                                         "a slot list and no nil mask)");
    // String dictionaries (k_dict_*): host-planned full sorts of many rows, multi-word string
    // keys of at most DICT_W words.  IGX_SORT_DICT=0 turns them off.
    uint32_t ndict = 0, dict_of[NSK] = {};
    const char *dict_env = std::getenv("IGX_SORT_DICT");
    if (!use_sel && !use_lsd && nrows >= DICT_MIN_ROWS && !(dict_env && std::strcmp(dict_env, "0") == 0))
        for (uint32_t k = 0; k < nkeys && ndict < (uint32_t)DICT_MAXK; ++k)
            if (keys[k].kind == IGX_KIND_BYTES && keys[k].words >= 2 && keys[k].words <= (uint32_t)DICT_W &&
                !keys[k].direct)
                dict_of[k] = ++ndict;
    // dictionaries: ctl (16 B each) | slots (each) | values + ranks (each); one memset clears
    // the ctl words and the slots
    constexpr uint32_t DSLOTS = 2 * DICT_MAXD;
    const size_t dict_ctl_b = igx_align((size_t)DICT_MAXK * 16, 256), dict_slot_b = (size_t)DSLOTS * 8;
    const size_t dict_val_b = (size_t)DICT_MAXD * DENT * 4 + igx_align((size_t)nrows * 4, 256);   // + rowidx
    const size_t dict_clear_b = ndict ? dict_ctl_b + ndict * dict_slot_b : 0;
    const size_t dict_b = ndict ? dict_clear_b + ndict * dict_val_b : 0;
    const size_t sel_b = use_sel ? igx_align((igx_align(limit, 64) + 2 * stride + 64 + SEL_BINS) * 4, 256) : 0;
    static_assert(sizeof(SelState) <= 64 * 4, "SelState fits the 64 words before the selection histogram");
    if (!ctx->nan_word) {
        IGX_HIP(ctx, hipMalloc(&ctx->nan_word, 64));
        IGX_HIP(ctx, hipMemsetAsync(ctx->nan_word, 0, 64, ctx->stream));
    }
    const size_t lsd_b = use_lsd ? igx_align(sizeof(LsdCtl), 256) : 0;
    if (use_lsd) {
        // the tagged per-tile counts: the context's own array, zeroed when it grows and when the
        // epoch wraps, so a word of an earlier call never carries a live tag
        const size_t need = (size_t)nblocks * 256;
        if (need > ctx->lsd_status_words) {
            IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->lsd_status) (void)hipFree(ctx->lsd_status);
            ctx->lsd_status = nullptr;
            ctx->lsd_status_words = 0;
            const size_t want = std::max(need, (size_t)256 * 256);
            IGX_HIP(ctx, hipMalloc(&ctx->lsd_status, want * 8));
            IGX_HIP(ctx, hipMemsetAsync(ctx->lsd_status, 0, want * 8, ctx->stream));
            ctx->lsd_status_words = want;
            ctx->lsd_epoch = 0;
        }
        if (++ctx->lsd_epoch >= (1u << 26)) {
            IGX_HIP(ctx, hipMemsetAsync(ctx->lsd_status, 0, ctx->lsd_status_words * 8, ctx->stream));
            ctx->lsd_epoch = 1;
        }
    }
    void *s;
    int rc = igx_scratch(ctx, 2 * words_b + 2 * pay_b + hist_b + res_b + sel_b + lsd_b + dict_b, &s);
    if (rc) return rc;
    char *c = reinterpret_cast<char *>(s);
    uint32_t *W[2] = {reinterpret_cast<uint32_t *>(c), reinterpret_cast<uint32_t *>(c + words_b)};
    uint32_t *P[2] = {reinterpret_cast<uint32_t *>(c + 2 * words_b),
                      reinterpret_cast<uint32_t *>(c + 2 * words_b + pay_b)};
    uint32_t *hist = reinterpret_cast<uint32_t *>(c + 2 * words_b + 2 * pay_b);
    uint32_t *scan_part = hist + igx_align((size_t)256 * nblocks, 64);
    uint32_t *res = reinterpret_cast<uint32_t *>(c + 2 * words_b + 2 * pay_b + hist_b);
    char *dict_base = c + 2 * words_b + 2 * pay_b + hist_b + res_b + sel_b + lsd_b;
    uint32_t *dctl = reinterpret_cast<uint32_t *>(dict_base);
    for (uint32_t k = 0, j = 0; k < nkeys; ++k) {
        if (!dict_of[k]) continue;
        char *q = dict_base + dict_clear_b + j * dict_val_b;
        DictRef &d = ca.dref[j];
        d.ctl = dctl + 4 * j;
        d.slot = reinterpret_cast<uint32_t *>(dict_base + dict_ctl_b + j * dict_slot_b);
        d.keys = reinterpret_cast<uint32_t *>(q);
        d.rowidx = reinterpret_cast<uint32_t *>(q + (size_t)DICT_MAXD * DENT * 4);
        ++j;
        d.nw = keys[k].words;
        d.cap = std::min<uint32_t>(DICT_MAXD, DICT_LDS_WORDS / d.nw);
        d.mask = DSLOTS - 1;
    }
    const uint32_t KW_raw = KW;
    uint32_t KW_dict = KW_raw;
    for (uint32_t k = 0; k < nkeys; ++k)
        if (dict_of[k]) KW_dict -= keys[k].words - 1;

    const uint32_t cblocks = (uint32_t)((nrows + TB - 1) / TB);
    ca.nan_seen = ctx->nan_word;
    bool u64_shape = rowmap && pos && !valid && pos_words == 2 && nkeys >= 1 && nkeys <= 4;
    for (uint32_t k = 0; k < nkeys && u64_shape; ++k)
        u64_shape = (keys[k].kind == IGX_KIND_UINT || keys[k].kind == IGX_KIND_INT) && keys[k].width == 8 &&
                    keys[k].words == 2 && !keys[k].direct;
    uint32_t *hres = nullptr;
    uint32_t ablocks = 0;
    // A table's top-K with a hint (k_tk_*): the hinted path runs first and the full selection
    // after it only does work when the hinted path could not answer.
    const char *tk_e = std::getenv("IGX_TOPK_HINT");   // A/B knob: 0 = always the full selection
    const bool tk_env = !(tk_e && std::strcmp(tk_e, "0") == 0);
    const char *tk_m = std::getenv("IGX_TOPK_HINT_MIN");   // rows below which the full selection is cheap anyway
    const uint64_t tk_min = tk_m ? std::strtoull(tk_m, nullptr, 0) : 65536ull;
    const bool tk_on = hint && tk_env && u64_shape && use_sel && !use_lsd && !any_float && rowmap && !valid &&
                       ndict == 0 && limit <= TK_MAXK && nrows >= tk_min;
    const uint32_t *tk_done = nullptr;
    if (tk_on && hint->nh) {
        uint32_t *st = hint->state;
        const uint32_t nh = std::min<uint32_t>(hint->nh, TK_MAXK);
        const uint32_t fb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(CAO_BLOCKS, (nrows + 4 * TB - 1) / (4 * TB)));
        switch (nkeys) {
#define IGX_TK_LAUNCH(NK)                                                                                              \
    case NK:                                                                                                           \
        hipLaunchKernelGGL(k_tk_bound<NK>, dim3(1), dim3(TK_MAXK), 0, ctx->stream, ca, hint->slots, nh, hint->occ,     \
                           hint->nslots, limit, st);                                                                   \
        hipLaunchKernelGGL(k_tk_filter<NK>, dim3(fb), dim3(TB), 0, ctx->stream, ca, st);                               \
        hipLaunchKernelGGL(k_tk_rank<NK>, dim3(1), dim3(1024), 0, ctx->stream, ca, st, limit, out_perm, hint->slots);  \
        break;
            IGX_TK_LAUNCH(1)
            IGX_TK_LAUNCH(2)
            IGX_TK_LAUNCH(3)
            IGX_TK_LAUNCH(4)
#undef IGX_TK_LAUNCH
        }
        IGX_HIP(ctx, hipGetLastError());
        tk_done = st + 1;
    }
    ca.skip = tk_done;
    // Compose, reduce, read back.  With dictionaries the first attempt composes the ranks; a
    // void dictionary (more distinct values than it holds) is seen in the read-back, and the
    // second attempt composes the raw bytes.
    for (int attempt = 0;; ++attempt) {
        const bool with_dict = ndict && attempt == 0;
        KW = with_dict ? KW_dict : KW_raw;
        for (uint32_t k = 0; k < nkeys; ++k) {
            ca.dict[k] = with_dict ? dict_of[k] : 0u;
            ca.words[k] = with_dict && dict_of[k] ? 1u : keys[k].words;
        }
        if (with_dict) {
            IGX_HIP(ctx, hipMemsetAsync(dict_base, 0, dict_clear_b, ctx->stream));
            for (uint32_t k = 0; k < nkeys; ++k) {
                if (!dict_of[k]) continue;
                DictBuildArgs da{};
                da.d = ca.dref[dict_of[k] - 1];
                da.ptr = keys[k].ptr;
                da.width = keys[k].width;
                da.rstride = ca.rstride[k];
                da.rowmap = rowmap;
                da.valid = valid;
                da.d_n = d_nrows;
                da.n = nrows;
                hipLaunchKernelGGL(k_dict_build, dim3((unsigned)((nrows + DB_ROWS - 1) / DB_ROWS)), dim3(DB_T), 0,
                                   ctx->stream, da);
                const size_t lds = ((size_t)da.d.cap * da.d.nw + DICT_MAXD) * 4;
                static bool attr = false;
                if (!attr) {
                    // up to 80 KB of dynamic LDS (gfx950's 160 KB per CU holds it); a refused
                    // attribute fails the sort here rather than letting k_compose read stale ranks
                    const hipError_t ae = hipFuncSetAttribute(reinterpret_cast<const void *>(k_dict_rank),
                                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                                              (int)((DICT_LDS_WORDS + DICT_MAXD) * 4));
                    if (ae != hipSuccess) return igx_fail(ctx, IGX_EIO, "sort: k_dict_rank LDS: %s", hipGetErrorString(ae));
                    attr = true;
                }
                hipLaunchKernelGGL(k_dict_rank, dim3(1), dim3(1024), lds, ctx->stream, da.d);
                // a launch that did not start leaves the ranks unwritten: fail instead of composing them
                if (const hipError_t le = hipGetLastError(); le != hipSuccess)
                    return igx_fail(ctx, IGX_EIO, "sort: k_dict_rank launch: %s", hipGetErrorString(le));
            }
        }
        uint32_t *apart = res + igx_align((size_t)KW * 2 + 4, 64);
        uint32_t fused_ao = 0;   // k_compose_u64_ao's grid: it left the AND / OR partials
        if (u64_shape && !use_lsd) {
            fused_ao = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(CAO_BLOCKS, (nrows + 4 * TB - 1) / (4 * TB)));
            switch (nkeys) {
            case 1: hipLaunchKernelGGL(k_compose_u64_ao<1>, dim3(fused_ao), dim3(TB), 0, ctx->stream, ca, W[0], P[0], apart); break;
            case 2: hipLaunchKernelGGL(k_compose_u64_ao<2>, dim3(fused_ao), dim3(TB), 0, ctx->stream, ca, W[0], P[0], apart); break;
            case 3: hipLaunchKernelGGL(k_compose_u64_ao<3>, dim3(fused_ao), dim3(TB), 0, ctx->stream, ca, W[0], P[0], apart); break;
            default: hipLaunchKernelGGL(k_compose_u64_ao<4>, dim3(fused_ao), dim3(TB), 0, ctx->stream, ca, W[0], P[0], apart); break;
            }
        } else if (u64_shape) {
            switch (nkeys) {
            case 1: hipLaunchKernelGGL(k_compose_u64<1>, dim3(cblocks), dim3(TB), 0, ctx->stream, ca, W[0], P[0]); break;
            case 2: hipLaunchKernelGGL(k_compose_u64<2>, dim3(cblocks), dim3(TB), 0, ctx->stream, ca, W[0], P[0]); break;
            case 3: hipLaunchKernelGGL(k_compose_u64<3>, dim3(cblocks), dim3(TB), 0, ctx->stream, ca, W[0], P[0]); break;
            default: hipLaunchKernelGGL(k_compose_u64<4>, dim3(cblocks), dim3(TB), 0, ctx->stream, ca, W[0], P[0]); break;
            }
        } else {
            hipLaunchKernelGGL(k_compose, dim3(cblocks), dim3(TB), 0, ctx->stream, ca, W[0], P[0]);
        }
        if (KW == 0) {   // no key and no position words: the (possibly reversed) row order itself
            const uint64_t m = limit ? std::min<uint64_t>(limit, nrows) : nrows;
            IGX_HIP(ctx, hipMemcpyAsync(out_perm, P[0], m * 4, hipMemcpyDeviceToDevice, ctx->stream));
            IGX_HIP(ctx, hipGetLastError());
            return IGX_OK;
        }
        if (use_lsd) {
            LsdCtl *ctl = reinterpret_cast<LsdCtl *>(c + 2 * words_b + 2 * pay_b + hist_b + res_b + sel_b);
            IGX_HIP(ctx, hipMemsetAsync(ctl, 0, sizeof(LsdCtl), ctx->stream));
            hipLaunchKernelGGL(k_lsd_h0, dim3(nblocks), dim3(STB), 0, ctx->stream, W[0], KW, stride, nrows, d_nrows, ctl);
            LsdArgs la{};
            la.W[0] = W[0];
            la.W[1] = W[1];
            la.P[0] = P[0];
            la.P[1] = P[1];
            la.stride = stride;
            la.nmax = nrows;
            la.d_n = d_nrows;
            la.status = ctx->lsd_status;
            la.ctl = ctl;
            la.KW = KW;
            for (uint32_t p = 0; p < KW * 4; ++p) {
                la.pass = p;
                la.tag = (ctx->lsd_epoch << 5) | p;
                // pass p works on word KW-1-p/4 and carries the words up to it
                if (KW - p / 4 <= 4)
                    hipLaunchKernelGGL(k_lsd_pass<4>, dim3(nblocks), dim3(STB), 0, ctx->stream, la);
                else
                    hipLaunchKernelGGL(k_lsd_pass<8>, dim3(nblocks), dim3(STB), 0, ctx->stream, la);
            }
            const uint64_t m = limit ? std::min<uint64_t>(limit, nrows) : nrows;
            hipLaunchKernelGGL(k_lsd_out, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, P[0], P[1], ctl,
                               nrows, d_nrows, limit, out_perm);
            IGX_HIP(ctx, hipGetLastError());
            return IGX_OK;
        }
        if (fused_ao) {
            ablocks = fused_ao;
        } else {
            ablocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ANDOR_BLOCKS, nrows / (4 * TB)));
            hipLaunchKernelGGL(k_andor, dim3(ablocks, KW), dim3(TB), 0, ctx->stream, W[0], nrows, stride, apart, d_nrows);
        }
        if (use_sel && !any_float && rowmap) {
            // top-K of a table's groups without host round trips (SelState on the device): no float
            // key, so no NaN check; the first differing bit is found on the device; the position
            // (first index) makes every composed key unique.  After the compose and AND/OR passes:
            // the final AND/OR (which also initialises the selection), the first histogram, the
            // split (each workgroup picks the bin itself) and the one-workgroup finish, which
            // ranks the k rows itself when their words fit its LDS.
            uint32_t *acc = reinterpret_cast<uint32_t *>(c + 2 * words_b + 2 * pay_b + hist_b + res_b);
            uint32_t *cnd[2] = {acc + igx_align(limit, 64), acc + igx_align(limit, 64) + stride};
            SelState *stp = reinterpret_cast<SelState *>(cnd[1] + stride);
            uint32_t *dh = reinterpret_cast<uint32_t *>(stp) + 64;   // SEL_BINS
            hipLaunchKernelGGL(k_andor_final, dim3(1), dim3(1024), 0, ctx->stream, apart, ablocks, KW, res,
                               ctx->nan_word, stp, nrows, limit, d_nrows, dh, nullptr, 0u, tk_done);
            // about 16 rows per thread: each workgroup adds its nonzero bins to the global
            // histogram, and a skewed table's low bins take one same-address atomic per workgroup
            const uint32_t hb = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(64, nrows / (16 * TB)));
            hipLaunchKernelGGL(k_sel_hist_d, dim3(hb), dim3(TB), 0, ctx->stream, W[0], stride, KW, stp, dh);
            hipLaunchKernelGGL(k_sel_split_d, dim3((uint32_t)((nrows + TILE - 1) / TILE)), dim3(TB), 0, ctx->stream,
                               W[0], stride, KW, stp, dh, acc, cnd[0]);
            const bool fused = limit <= 1024 && (uint64_t)limit * KW <= SEL_BINS;   // the k rows' words fit its LDS
            hipLaunchKernelGGL(k_sel_finish, dim3(1), dim3(1024), 0, ctx->stream, W[0], stride, KW, stp, acc, cnd[0],
                               cnd[1], limit, P[0], fused ? out_perm : nullptr, tk_done);
            if (!fused)
                hipLaunchKernelGGL(k_sel_rank, dim3(limit), dim3(TB), 0, ctx->stream, W[0], stride, KW, acc, limit, P[0],
                                   out_perm, stp, tk_done);
            if (tk_on) {   // the full selection's answer (if it ran) becomes the next call's hints
                hipLaunchKernelGGL(k_tk_save, dim3(1), dim3(1024), 0, ctx->stream, out_perm, limit, hint->slots, tk_done,
                                   hint->state);
                hint->nh = limit;
            }
            IGX_HIP(ctx, hipGetLastError());
            return IGX_OK;
        }
        hipLaunchKernelGGL(k_andor_final, dim3(1), dim3(1024), 0, ctx->stream, apart, ablocks, KW, res, ctx->nan_word,
                           nullptr, nrows, limit, d_nrows, nullptr, with_dict ? dctl : nullptr, with_dict ? ndict : 0u);
        // one read-back: the AND/OR words, the NaN flag, a void dictionary, the device row count
        rc = igx_pinned(ctx, KW_raw * 8 + 16, reinterpret_cast<void **>(&hres));
        if (rc) return rc;
        IGX_HIP(ctx, hipMemcpyAsync(hres, res, KW * 8 + 16, hipMemcpyDeviceToHost, ctx->stream));
        IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (with_dict && hres[2 * KW + 1]) {
            if (hres[2 * KW + 1] & 2u) return igx_fail(ctx, IGX_EIO, "sort: string dictionary build failed");
            continue;   // over capacity: compose the raw bytes
        }
        break;
    }
    // Go's `<` is unordered on NaN, so getLessFunc (sort.go:125-135) is no strict weak order
    // once a NaN is present and SliceStable's result depends on its insertion-sort blocks and
    // symMerge steps, not on the values alone: no radix order reproduces it, so the passes run
    // as SliceStable itself (k_gostable.hip).
    if (hres[2 * KW]) {
        if (!gokeys) return igx_fail(ctx, IGX_ENOTSUP, "sort: NaN in a float sort key");
        return sort_exact_go(ctx, keys, nkeys, nrows, pos, valid, out_perm, limit, rowmap, pos_stride, gokeys, ngokeys);
    }

    if (use_sel) {
        // top-K: radix select on the composed keys, then rank the k survivors
        uint32_t bitpos = KW * 32;
        for (uint32_t w = 0; w < KW; ++w) {
            const uint32_t diff = hres[2 * w] ^ hres[2 * w + 1];
            if (diff) {
                bitpos = 32 * w + (uint32_t)__builtin_clz(diff);
                break;
            }
        }
        // selection scratch: acc | cand A | cand B | counters | hist
        uint32_t *acc = reinterpret_cast<uint32_t *>(c + 2 * words_b + 2 * pay_b + hist_b + res_b);
        uint32_t *cnd[2] = {acc + igx_align(limit, 64), acc + igx_align(limit, 64) + stride};
        uint32_t *cnt = cnd[1] + stride;            // [0] acc count, [1] next-candidate count
        uint32_t *dh = cnt + 64;                    // SEL_BINS
        uint32_t *hh;
        rc = igx_pinned(ctx, SEL_BINS * 4 + 64, reinterpret_cast<void **>(&hh));
        if (rc) return rc;
        IGX_HIP(ctx, hipMemsetAsync(cnt, 0, 8, ctx->stream));
        const uint32_t *cand = nullptr;
        uint64_t n = nrows;
        uint32_t krem = limit, cur_c = 0;
        while (n > krem) {
            if (bitpos >= KW * 32) return igx_fail(ctx, IGX_EIO, "topk: composed keys not unique");
            const uint32_t nbits = std::min<uint32_t>(SEL_BITS, KW * 32 - bitpos);
            IGX_HIP(ctx, hipMemsetAsync(dh, 0, SEL_BINS * 4, ctx->stream));
            const uint32_t hb = (uint32_t)std::min<uint64_t>(1024, (n + TB - 1) / TB);
            hipLaunchKernelGGL(k_sel_hist, dim3(hb), dim3(TB), 0, ctx->stream, W[0], stride, KW, cand, n, bitpos,
                               nbits, dh);
            IGX_HIP(ctx, hipMemcpyAsync(hh, dh, SEL_BINS * 4, hipMemcpyDeviceToHost, ctx->stream));
            IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
            uint32_t b = 0;
            uint64_t below = 0;
            for (; b < (1u << nbits); ++b) {
                if (below + hh[b] >= krem) break;
                below += hh[b];
            }
            uint32_t *nxt = cnd[cur_c];
            IGX_HIP(ctx, hipMemsetAsync(cnt + 1, 0, 4, ctx->stream));
            const uint32_t sb = (uint32_t)((n + TILE - 1) / TILE);
            hipLaunchKernelGGL(k_sel_split, dim3(sb), dim3(TB), 0, ctx->stream, W[0], stride, KW, cand, n, bitpos,
                               nbits, b, acc, cnt, nxt, cnt + 1);
            krem -= (uint32_t)below;
            n = hh[b];
            cand = nxt;
            cur_c ^= 1;
            bitpos += nbits;
        }
        if (krem)   // every remaining candidate is in (n == krem); limit - krem were accepted
            IGX_HIP(ctx, hipMemcpyAsync(acc + (limit - krem), cand, (size_t)krem * 4, hipMemcpyDeviceToDevice,
                                        ctx->stream));
        hipLaunchKernelGGL(k_sel_rank, dim3(limit), dim3(TB), 0, ctx->stream, W[0], stride, KW, acc, limit, P[0],
                           out_perm, nullptr);
        IGX_HIP(ctx, hipGetLastError());
        return IGX_OK;
    }

    if (d_nrows) {   // the slice's length, read back with the AND/OR words
        uint64_t dn;
        std::memcpy(&dn, hres + 2 * KW + 2, 8);   // (k_andor_final copies it into res)
        nrows = std::min<uint64_t>(nrows, dn);
        if (nrows == 0) return IGX_OK;
    }
    const uint32_t pblocks = (uint32_t)((nrows + RTILE - 1) / RTILE);
    // digit plan: word w (0 = most significant), byte b (0 = least significant in word)
    std::vector<int> live_word(KW, 0);
    for (uint32_t w = 0; w < KW; ++w) live_word[w] = (hres[2 * w] ^ hres[2 * w + 1]) != 0;
    int cur = 0;
    for (int w = (int)KW - 1; w >= 0; --w) {
        uint32_t diff = hres[2 * w] ^ hres[2 * w + 1];
        if (!diff) continue;
        // live words for passes on word w: all w' <= w with any variation
        ScatterArgs sa{};
        uint32_t nl = 0;
        uint32_t dslot = 0;
        for (int v = 0; v <= w; ++v) {
            if (!live_word[v]) continue;
            if (v == w) dslot = nl;
            sa.in[nl] = W[cur] + (uint64_t)v * stride;
            sa.out[nl] = W[cur ^ 1] + (uint64_t)v * stride;
            ++nl;
        }
        sa.nlive = nl;
        sa.dword = dslot;
        sa.nblocks = pblocks;
        sa.n = nrows;
        sa.off = hist;
        for (int b = 0; b < 4; ++b) {
            if (((diff >> (8 * b)) & 255u) == 0) continue;
            sa.shift = 8 * b;
            sa.pin = P[cur];
            sa.pout = P[cur ^ 1];
            const bool scan_free = nl <= 8 && pblocks <= SCAN_FREE_TILES;
            hipLaunchKernelGGL(k_radix_hist, dim3(pblocks), dim3(STB), 0, ctx->stream,
                               sa.in[dslot], sa.shift, nrows, pblocks, hist, scan_free ? 1u : 0u);
            sa.off = scan_free ? nullptr : hist;
            sa.cnt = hist;
            if (!scan_free) launch_scan(ctx->stream, hist, (uint64_t)256 * pblocks, scan_part);
            if (nl <= 4)
                hipLaunchKernelGGL(k_radix_scatter_pf<4>, dim3(pblocks), dim3(STB), 0, ctx->stream, sa);
            else if (nl <= 8)
                hipLaunchKernelGGL(k_radix_scatter_pf<8>, dim3(pblocks), dim3(STB), 0, ctx->stream, sa);
            else
                hipLaunchKernelGGL(k_radix_scatter, dim3(pblocks), dim3(STB), 0, ctx->stream, sa);
            // swap buffers: the next pass reads what this one wrote
            cur ^= 1;
            for (uint32_t l = 0; l < nl; ++l) {
                const uint32_t *tmp = sa.in[l];
                sa.in[l] = sa.out[l];
                sa.out[l] = const_cast<uint32_t *>(tmp);
            }
        }
        live_word[w] = 0;   // never read again below this point
    }
    const uint64_t m = limit ? std::min<uint64_t>(limit, nrows) : nrows;
    IGX_HIP(ctx, hipMemcpyAsync(out_perm, P[cur], m * 4, hipMemcpyDeviceToDevice, ctx->stream));
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
