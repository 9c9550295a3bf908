// k_groupby.hip -- keyed per-interval aggregation (kernel (2)).
//
// Reference semantics: the top gadgets' BPF hash maps, e.g. probe_ip
// (pkg/gadgets/top/tcp/tracer/bpf/tcptop.bpf.c:33-110): build a fixed key struct,
// lookup-or-insert, `+=` into the value; nextStats (tracer.go:147-226) drains one Stats
// row per key.  Keys are compared in full (exact, like the BPF map's memcmp), values
// wrap at their declared width, and each group remembers the global index of its first
// event -- the canonical pre-sort order that replaces BPF map order.
//
// HBM table: S = 2^k slots (S >= 2 x capacity), open addressing with linear probing.
// Each slot has a key record (KR = 32..256 B, one cache line for every built-in layout):
//     [0, KOFF)            key words (KW x u32, packed; each key column padded to 4 B)
//     KOFF                 u64 tag   (hash bits 16..63 | generation; another generation = empty)
//     KOFF + 8             u64 ready (epoch << 48 | first_ins + 1.  An epoch before the
//                          generation's = key not yet published; the interval's own epoch =
//                          first_ins is this interval's: an upper bound of the group's first,
//                          whose value record holds first <= first_ins (or will, once the
//                          interval's atomics land); an earlier epoch of the generation = a
//                          key kept from an earlier interval, not yet seen in this one)
// and a value record (VR = 8 x 2^m B):  u64 first (first-occurrence event index), then
// u64 aggregate a at 8 + 8a.  The two are kept apart because 64-bit atomics execute at
// the memory side and drop their line from L2 (MI355X_MICROARCH.md, store flavours and
// global atomics): key records are written once per interval and stay L2-resident for
// the probes, value records only ever receive fire-and-forget atomics.
// The slot index IS the group id; igx_groupby_finalize lists the occupied slots from a
// bitmap (one bit per slot, so the list costs S/8 bytes, not a walk of every key record):
// the partitioned form's claimers set it, the cached form's mark a byte map with plain byte
// stores that finalize folds into it, the direct form's are read off the tags.  A reset bumps the epoch instead of rewriting the table: records of an
// older epoch read as empty and the claimer initialises its value record (first =
// first_ins, aggregates 0) before it publishes `ready`.
// Keys outlive their interval (a *generation* spans intervals): the reference drains its BPF
// map every interval (tcp/tracer/tracer.go:154-171) and re-inserts every recurring key, here a
// reset that continues the generation only returns the previous interval's groups' value
// records to (first = UINT64_MAX, sums 0), from finalize's slot list.  The first miss of a kept
// key in an interval finds it (no CAS, no key or value-record stores): it re-stamps `ready`
// with the interval's epoch and first_ins = its index + 1 (so its own first-index minimum is
// pushed like any earlier event's) and marks the occupancy byte.  So the interval's output is
// still exactly its own groups, sums and first indices.  A generation ends (the next interval
// starts an empty one: tag bits = that interval's epoch) when the keys it holds plus a full
// interval's capacity would pass 4/5 of the slots, after a failed interval, when the
// interval runs the direct or partitioned form, or at the epoch counter's wrap.
// A new key claims a record with a 64-bit CAS on the tag, writes its key with write-through
// (sc1) stores and publishes `ready` with an sc1 store after `s_waitcnt vmcnt(0)`; readers
// load the key record with 16-byte sc1 buffer loads (one round trip) and compare the key
// in registers (MI355X_MICROARCH.md §Workgroup dispatch, hand-off table row 1).
//
// Each workgroup (1024 threads, one per CU) keeps an LDS key cache: 8-way set associative
// on the key hash, entries hold the full key, its slot and the workgroup's partial aggregates;
// first come, never evicted, so the Zipf-hot keys settle in LDS and their events cost only
// their own input bytes plus LDS atomics.  A miss is resolved at once, while its row is in
// registers: HBM probe, adoption of a free LDS entry when its set has one, and otherwise
// its HBM updates go to the server wave through an LDS ring (see "HBM atomics through an
// LDS ring").  Eight waves stream rows, seven resolve misses, the sixteenth issues the atomics.  The
// cache is committed with HBM atomics at the end.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <string>
#include <utility>
#include <vector>

#include <thread>

#include "k_common.h"

// event-stream loads of the group-by kernels: non-temporal (read once; IGX_GB_STREAM_NT=0
// builds a plain-load variant for cache-residency experiments)
#ifndef IGX_GB_STREAM_NT
#define IGX_GB_STREAM_NT 1
#endif
#if IGX_GB_STREAM_NT
#define IGX_STREAM_LOAD(p) __builtin_nontemporal_load(p)
#else
#define IGX_STREAM_LOAD(p) (*(p))
#endif
// a stream load, non-temporal (IGX_STREAM_LOAD) unless the caller asks for a plain one
template <bool NT, class T>
__device__ __forceinline__ T stream_ld(const T *p) {
    if constexpr (NT) return IGX_STREAM_LOAD(p);
    else return *p;
}

namespace {

#ifndef IGX_GB_DIRECT_U
#define IGX_GB_DIRECT_U 2
#endif
constexpr uint32_t SLOT_OVF = 0xFFFFFFFFu;
constexpr int KWMAX = 32;
constexpr int AMAX = 4;   // top file needs 4 (reads, rbytes, writes, wbytes)
constexpr int PMAX = 2;   // more predicates: run igx_filter first
constexpr int GTB = 1024;
constexpr uint32_t ST_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t ST_BUSY = 0xFFFFFFFEu;
constexpr uint32_t GHOST = 1024;                 // admission filter entries (LDS)
constexpr uint64_t EP_MAX = 0xFFFF;              // epoch bits in a tag / in `ready`
constexpr uint64_t READY_IDX = (1ull << 48) - 1;  // `ready` = epoch << 48 | (first_ins + 1)

__device__ __forceinline__ bool ready_ok(uint64_t ready, uint64_t ep) { return (ready >> 48) == ep; }
// published in the generation that started at epoch gep (the interval's epoch is ep >= gep;
// epochs only grow within a generation: the counter's wrap clears the table)
__device__ __forceinline__ bool ready_pub(uint64_t ready, uint32_t gep, uint64_t ep) {
    const uint64_t r = ready >> 48;
    return r >= gep && r <= ep;
}
// the device generation block behind the error block (u64 words of igx_table::err):
// [3] the generation's first epoch (tag bits), [4] keys claimed in the generation before this
// interval (~0: end it), [5] keys claimed in this interval
constexpr int GEN_WORD = 3;

__host__ __device__ constexpr uint32_t koff_of(int kw) { return (uint32_t)((4 * kw + 7) & ~7); }
__host__ __device__ constexpr uint32_t pow2_at_least(uint32_t b) {
    uint32_t r = 8;
    while (r < b) r <<= 1;
    return r;
}
__host__ __device__ constexpr uint32_t krec_bytes(int kw) { return pow2_at_least(koff_of(kw) + 16); }
__host__ __device__ constexpr uint32_t vrec_bytes(uint32_t naggs) { return pow2_at_least(8 + 8 * naggs); }

// Every input byte is fetched with an unconditional load (no load sits behind a runtime
// branch), so all of a row's loads issue back to back and retire under one wait.
struct GbArgs {
    // static layouts: one base pointer per key column
    const uint8_t *kcol[16];
    // generic layout: word w = (dword at kptr[w] + row*kwidth[w] + koff[w]) & kmask[w], or,
    // for a column whose width is neither 1, 2 nor a multiple of 4, its kbytes[w] bytes
    // loaded one by one (such a column is not dword aligned)
    const uint8_t *kptr[KWMAX];
    uint32_t kwidth[KWMAX];
    uint32_t koff[KWMAX];
    uint32_t kmask[KWMAX];
    uint32_t kbytes[KWMAX];
    // aggregates: value = SUM column (vwidth bytes) or 1 (COUNT), if cond column == cval
    const uint8_t *vptr[AMAX];
    const uint8_t *cptr[AMAX];
    uint64_t cval[AMAX];
    uint64_t vdiv[AMAX];    // 0: plain value, else value / vdiv (unsigned)
    uint32_t vwidth[AMAX], vsign[AMAX], vcount[AMAX], cwidth[AMAX], hascond[AMAX];
    // per aggregate: load its value / condition column (1), or reuse aggregate vshare /
    // cshare's dwords (same column; AMAX = not shared)
    uint32_t vload[AMAX], cload[AMAX], vshare[AMAX], cshare[AMAX];
    // load geometry: row stride (0 = nothing to load: dword 0 of the pointer) and the
    // offset of the high dword (4 for 8-byte columns, else 0)
    uint32_t vldw[AMAX], cldw[AMAX], vhioff[AMAX], chioff[AMAX], phioff[PMAX], validw;
    uint32_t naggs;
    // scalar predicates (FilterSpec on a <= 8-byte column), AND-ed.  pldw: load stride (0 when
    // pshare < AMAX: the column is aggregate pshare's value column, whose raw value is reused).
    // A guarded predicate applies to the rows whose guard column equals gref; the fused
    // kernels read the guard as aggregate pguard's condition value (a guard on any other
    // column goes to the row mask), the mask kernel loads it from gptr (gwidth bytes).
    const uint8_t *pptr[PMAX];
    const uint8_t *gptr[PMAX];
    uint64_t pref[PMAX], gref[PMAX];
    uint32_t pwidth[PMAX], pkind[PMAX], pcmp[PMAX], pneg[PMAX], pcnt[PMAX];
    uint32_t pldw[PMAX], pshare[PMAX], pguard[PMAX], gwidth[PMAX];
    uint32_t npred;
    uint32_t lds_entries;   // E (8 x sets)
    uint32_t direct;        // 1: probers issue their HBM atomics; the server wave probes too
    uint32_t sm;            // 1: state-machine probers (IGX_GB_PROBER=0: batch probers)
    uint32_t admit_mask;    // LDS admission on a key's (admit_mask + 1)-th miss (ghost_admit), 0: on the first
    uint32_t nl;            // loader waves (1..14)
    // input
    const uint8_t *valid;   // nullable: rows with 0 are skipped (nil / filtered entries)
    const uint8_t *validp;  // valid, or the dummy column when there is none (always loaded)
    const uint64_t *fidx;   // nullable: per-row global event index (merging partial groups)
    uint64_t n, base_idx;
    // table
    uint8_t *krec;          // key records
    uint64_t *vrec;         // value records
    uint32_t krec_len;      // KR
    uint32_t krec_total;    // S x KR (< 2^32)
    uint32_t vrec_words;    // VR / 8
    uint32_t vrec_total;    // S x VR when below 4 GiB (16-B buffer stores of a claim), else 0
    uint32_t *err;
    uint32_t *occ;          // occupancy bitmap, one bit per slot (set by the partitioned form's claimers)
    uint8_t *occb;          // occupancy byte map, one byte per slot: the cached form's claimers store
                            // 1 with a plain byte store (no atomic: one claimer per slot), finalize
                            // folds it into the bitmap (k_slots_count)
    uint64_t ep;            // the interval's epoch (1..EP_MAX): tags and `ready` of older
                            // epochs read as empty (the direct and partitioned forms, which
                            // always start a generation: their generation is ep)
    uint64_t *gen;          // the device generation block (GEN_WORD): the cached form reads its
                            // generation there and counts its claims into it
    uint64_t rmask;         // probe region slots - 1 (probing wraps inside a region)
    uint32_t sshift;        // home slot = h >> sshift (the hash's top bits)
    uint32_t max_probe;
    // diagnostics (IGX_GB_DEBUG; compiled into the top-tcp key's debug kernel only):
    // bit0 stop after load+hash, bit1 drop LDS misses, bit10 probers drop the cells they take, bit2 drop HBM atomics, bit3 count
    // hits/misses, bit8 no HBM probe (a hash-derived slot), bit9 no LDS accumulate on hits
    uint32_t dbg;
    unsigned long long *dbg_cnt;
    // sample-seeded LDS cache (cached form, kept keys): nseeds records of seed_words u32 each
    // (key words padded to quads | HBM slot | pad | hash) that every workgroup adopts into its
    // cache before the stream starts, when they belong to the current generation (*seed_gep)
    const uint32_t *seeds;
    const uint64_t *seed_gep;
    uint32_t nseeds;
};

// Key hash: NH (the UMAC inner hash) over the key's word pairs -- one 32x32->64 multiply
// per 8 key bytes, sum(( k[2i] + K[2i]) * (k[2i+1] + K[2i+1])) mod 2^64 -- then the murmur3
// 64-bit finaliser.  Exactness never depends on it (keys are compared in full); it only
// spreads slots, LDS sets and tags.
__device__ __forceinline__ uint32_t nh_const(int i) {
    return 0x9E3779B9u * (uint32_t)(2 * i + 1) + 0x7F4A7C15u;   // odd, distinct per word
}

template <int KW>
__device__ __forceinline__ uint64_t hash_key(const uint32_t (&k)[KW]) {
    uint64_t h = 0x243F6A8885A308D3ull ^ (uint64_t)KW;
#pragma unroll
    for (int w = 0; w < KW; w += 2) {
        const uint32_t a = k[w] + nh_const(w);
        const uint32_t b = ((w + 1 < KW) ? k[w + 1] : 0u) + nh_const(w + 1);
        h += (uint64_t)a * (uint64_t)b;
    }
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}

// aligned dword containing byte `off`, shifted so that byte lands in bits 0..7; the
// dword containing a column's last byte never crosses its last 4-byte block (no overrun)
__device__ __forceinline__ uint32_t ldw(const uint8_t *base, uint64_t off) {
    const uint32_t d = *reinterpret_cast<const uint32_t *>(base + (off & ~3ull));
    return d >> ((uint32_t)(off & 3u) * 8u);
}

// zero-extended little-endian value of `width` (1, 2, 4 or 8) bytes at row; branch-free
[[maybe_unused]] __device__ __forceinline__ uint64_t ld_val(const uint8_t *base, uint64_t row, uint32_t width) {
    const uint64_t b = row * width;
    const uint32_t lomask = width >= 4 ? 0xFFFFFFFFu : ((1u << (8 * width)) - 1u);
    const uint32_t lo = ldw(base, b) & lomask;
    const uint32_t hi = ldw(base, b + (width == 8 ? 4u : 0u));
    return (uint64_t)lo | ((uint64_t)(width == 8 ? hi : 0u) << 32);
}

__device__ __forceinline__ uint64_t sext(uint64_t v, uint32_t width) {
    const uint32_t sh = 64u - 8u * width;
    return sh ? (uint64_t)(((int64_t)(v << sh)) >> sh) : v;
}

// Key layouts.  StaticLayout<W...> fixes the key column widths at compile time (the
// reference's BPF key structs: ip_key_t, file_id, the advisor tuple, single columns), so
// every key load is one typed load (dwordx4 for a 16-byte column) with no descriptors in
// registers.  GenericLayout<KW> handles any other layout from per-word descriptors.
template <int... W>
struct StaticLayout {
    static constexpr int NC = sizeof...(W);
    static constexpr int Ws[NC] = {W...};
    static constexpr int words(int c) { return (Ws[c] + 3) / 4; }
    static constexpr int off(int c) {
        int o = 0;
        for (int i = 0; i < c; ++i) o += words(i);
        return o;
    }
    static constexpr int KW = off(NC);
    static constexpr bool is_static = true;

    template <int c, bool NT>
    __device__ __forceinline__ static void load_col(const GbArgs &a, uint64_t row, uint32_t *k) {
        constexpr int w = Ws[c];
        constexpr int o = off(c);
        const uint8_t *p = a.kcol[c];
        // the event stream is read once: non-temporal loads, so it does not push the
        // table's key records out of the caches
        if constexpr (w == 16) {
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            const v4u q = stream_ld<NT>(reinterpret_cast<const v4u *>(p) + row);
            k[o] = q.x; k[o + 1] = q.y; k[o + 2] = q.z; k[o + 3] = q.w;
        } else if constexpr (w == 8) {
            typedef unsigned int v2u __attribute__((ext_vector_type(2)));
            const v2u q = stream_ld<NT>(reinterpret_cast<const v2u *>(p) + row);
            k[o] = q.x; k[o + 1] = q.y;
        } else if constexpr (w == 4) {
            k[o] = stream_ld<NT>(reinterpret_cast<const uint32_t *>(p) + row);
        } else if constexpr (w == 2) {
            k[o] = stream_ld<NT>(reinterpret_cast<const uint16_t *>(p) + row);
        } else if constexpr (w == 1) {
            k[o] = stream_ld<NT>(p + row);
        } else {
            static_assert(w % 4 == 0, "key widths other than 1/2 must be multiples of 4");
#pragma unroll
            for (int j = 0; j < w / 4; ++j) k[o + j] = reinterpret_cast<const uint32_t *>(p + row * w)[j];
        }
    }
    template <bool NT, size_t... I>
    __device__ __forceinline__ static void load_all(const GbArgs &a, uint64_t row, uint32_t *k,
                                                    std::index_sequence<I...>) {
        (load_col<(int)I, NT>(a, row, k), ...);
    }
    template <bool NT = true>
    __device__ __forceinline__ static void load(const GbArgs &a, uint64_t row, uint32_t (&k)[KW]) {
        load_all<NT>(a, row, k, std::make_index_sequence<NC>{});
    }
};

template <int KWG>
struct GenericLayout {
    static constexpr int KW = KWG;
    static constexpr bool is_static = false;
    template <bool NT = true>
    __device__ __forceinline__ static void load(const GbArgs &a, uint64_t row, uint32_t (&k)[KW]) {
#pragma unroll
        for (int w = 0; w < KW; ++w) {
            const uint64_t off = row * a.kwidth[w] + a.koff[w];
            if (a.kbytes[w]) {   // an unaligned column: byte loads (uniform branch)
                uint32_t v = 0;
                for (uint32_t b = 0; b < a.kbytes[w]; ++b) v |= (uint32_t)a.kptr[w][off + b] << (8 * b);
                k[w] = v;
            } else {
                k[w] = ldw(a.kptr[w], off) & a.kmask[w];
            }
        }
    }
};

// FilterSpec on a scalar column, evaluated on an already loaded value
// (getComparisonFuncForComparisonType, filter.go:236-263: (field OP ref) != negate).
__device__ __forceinline__ bool pred_scalar(uint64_t v, uint64_t ref, uint32_t width, uint32_t kind,
                                            uint32_t cmp, uint32_t neg, uint32_t cnt) {
    if (cmp == IGX_CMP_IN) {   // set membership: cnt values of `width` bytes packed in ref
        const uint64_t m = width >= 8 ? ~0ull : ((1ull << (8 * width)) - 1);
        bool in = false;
        for (uint32_t i = 0; i < cnt; ++i) in = in || v == ((ref >> (8 * width * i)) & m);
        return in != (neg != 0);
    }
    int c;
    if (kind == IGX_KIND_FLOAT) {
        double x, y;
        if (width == 4) {
            x = __uint_as_float((uint32_t)v);
            y = __uint_as_float((uint32_t)ref);
        } else {
            x = __longlong_as_double((long long)v);
            y = __longlong_as_double((long long)ref);
        }
        c = (x != x || y != y) ? 2 : (x < y ? -1 : (x > y ? 1 : 0));
    } else if (kind == IGX_KIND_INT) {
        const int64_t x = (int64_t)sext(v, width), y = (int64_t)sext(ref, width);
        c = x < y ? -1 : (x > y ? 1 : 0);
    } else {
        c = v < ref ? -1 : (v > ref ? 1 : 0);
    }
    bool r = c != 2 && ((cmp == IGX_CMP_EQ && c == 0) || (cmp == IGX_CMP_LT && c < 0) ||
                        (cmp == IGX_CMP_LE && c <= 0) || (cmp == IGX_CMP_GT && c > 0) ||
                        (cmp == IGX_CMP_GE && c >= 0));
    return r != (neg != 0);
}

// A key's home slot is the hash's top bits and linear probing wraps inside the slot's
// region (table.rbits): a bucket of the partitioned form (also the hash's top bits) then owns
// whole regions of the table, in every form alike.
__device__ __forceinline__ uint64_t home_slot(const GbArgs &a, uint64_t h) { return h >> a.sshift; }
__device__ __forceinline__ uint64_t next_slot(const GbArgs &a, uint64_t s) {
    return (s & ~a.rmask) | ((s + 1) & a.rmask);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(const GbArgs &a) {
    return __builtin_amdgcn_make_buffer_rsrc(a.krec, (short)0, (int)a.krec_total, 0x00020000);
}

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// the first 16*NQ bytes of a key record (key, tag, ready) as sc1 loads (L2-served)
template <int NQ>
__device__ __forceinline__ void load_rec(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t (&d)[NQ * 4]) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * i, 0, 16 /* sc1 */);
        d[4 * i] = q.x; d[4 * i + 1] = q.y; d[4 * i + 2] = q.z; d[4 * i + 3] = q.w;
    }
}

// lookup-or-insert in the HBM table; returns the slot (SLOT_OVF: table full) and the
// slot's first_ins (claiming event index).  An event with a larger index never needs the
// atomicMin on the value record's first: the group's first is min(first_ins, that field).
template <int KW>
constexpr int probe_quads() { return (int)((koff_of(KW) + 16 + 15) / 16); }   // key, tag, ready

// the home slot's record, issued early so its round trip overlaps other work
template <int KW>
__device__ __forceinline__ void probe_issue(const GbArgs &a, uint64_t h, uint32_t (&d)[probe_quads<KW>() * 4]) {
    load_rec<probe_quads<KW>()>(rec_rsrc(a), (uint32_t)(home_slot(a, h) * a.krec_len), d);
}

// A claimer's value record: first = its event index, aggregate x = vinit[x] (the claiming
// event's own values, so they need no atomic; null: 0), written through (sc1) as 16-B stores
// where the record array allows buffer addressing -- a claim's stores are memory-side write
// requests each, and they are the largest share of a high-cardinality interval's requests.
// The padding words of the record are never read and not written.
// (All indices are compile-time: a register array indexed at run time would live in scratch.)
template <int NV>
__device__ __forceinline__ void vrec_init(const GbArgs &a, uint64_t s, uint64_t gidx, const uint64_t (&v)[NV]) {
    uint64_t w[NV + 2];
    w[0] = gidx;
#pragma unroll
    for (int x = 0; x < NV; ++x) w[1 + x] = v[x];
    w[NV + 1] = 0;
    uint64_t *vr = a.vrec + s * a.vrec_words;
    const uint32_t nw = 1 + a.naggs;   // <= 1 + NV
    if (a.vrec_total) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.vrec, (short)0, (int)a.vrec_total, 0x00020000);
        const uint32_t off = (uint32_t)(s * a.vrec_words * 8);
#pragma unroll
        for (int j = 0; j < NV + 1; j += 2) {
            if ((uint32_t)j >= nw) break;
            if ((uint32_t)j + 1 < nw) {
                const u4v q = {(uint32_t)w[j], (uint32_t)(w[j] >> 32), (uint32_t)w[j + 1], (uint32_t)(w[j + 1] >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(q, rs, off + 8 * j, 0, 16 /* sc1 */);
            } else {
                st_agent(vr + j, w[j]);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NV + 1; ++j)
            if ((uint32_t)j < nw) st_agent(vr + j, w[j]);
    }
}

// d holds the home slot's record (probe_issue).  vinit: the event's aggregate values, written
// into the value record when this call claims the slot (claimed = true; the caller then adds
// them nowhere else).
template <int KW, bool SET_OCC, int NV>
__device__ __forceinline__ uint32_t find_or_insert(const GbArgs &a, const uint32_t (&k)[KW], uint64_t h,
                                                   uint64_t gidx, uint64_t &first_ins,
                                                   uint32_t (&d)[probe_quads<KW>() * 4],
                                                   const uint64_t (&vinit)[NV], bool &claimed) {
    constexpr uint32_t KOFF = koff_of(KW);
    constexpr int NQ = probe_quads<KW>();
    const uint64_t tag = (h & ~EP_MAX) | a.ep;
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(a);
    uint64_t s = home_slot(a, h);
    for (uint32_t probe = 0; probe < a.max_probe; ++probe) {
        const uint32_t off = (uint32_t)(s * a.krec_len);
        if (probe) load_rec<NQ>(rs, off, d);
        uint8_t *r = a.krec + off;
        uint64_t t = (uint64_t)d[KOFF / 4] | ((uint64_t)d[KOFF / 4 + 1] << 32);
        uint64_t ready = (uint64_t)d[KOFF / 4 + 2] | ((uint64_t)d[KOFF / 4 + 3] << 32);
        if ((t & EP_MAX) != a.ep) {   // empty in this interval (never claimed, or an older epoch's)
            if (gidx >= READY_IDX) {   // an index column value that `ready` cannot carry
                atomicOr(a.err, 8u);
                return SLOT_OVF;
            }
            const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long *>(r + KOFF),
                                           (unsigned long long)t, (unsigned long long)tag);
            if (old == t) {
                // key words as 16-byte write-through stores (each store is one memory-side write)
#pragma unroll
                for (int w = 0; w < KW; w += 4) {
                    if (w + 3 < KW) {
                        const u4v q = {k[w], k[w + 1], k[w + 2], k[w + 3]};
                        __builtin_amdgcn_raw_buffer_store_b128(q, rs, off + 4 * w, 0, 16 /* sc1 */);
                    } else if (w + 1 < KW) {
                        st_agent(reinterpret_cast<uint64_t *>(r + 4 * w), (uint64_t)k[w] | ((uint64_t)k[w + 1] << 32));
                        if (w + 2 < KW) st_agent(reinterpret_cast<uint32_t *>(r + 4 * w + 8), k[w + 2]);
                    } else {
                        st_agent(reinterpret_cast<uint32_t *>(r + 4 * w), k[w]);
                    }
                }
                // the value record starts at first = first_ins and the claimer's own values
                // (no reset pass)
                vrec_init<NV>(a, s, gidx, vinit);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_agent(reinterpret_cast<uint64_t *>(r + KOFF + 8), (a.ep << 48) | (gidx + 1));
                if (SET_OCC) atomicOr(a.occ + (s >> 5), 1u << (s & 31));
                first_ins = gidx;
                claimed = true;
                return (uint32_t)s;
            }
            t = old;
            ready = 0;   // the claimer may still be writing the key
        }
        if (t == tag) {
            if (!ready_ok(ready, a.ep)) {
                uint32_t spins = 0;
                while (!ready_ok(ld_agent(reinterpret_cast<const uint64_t *>(r + KOFF + 8)), a.ep)) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 22)) {
                        atomicOr(a.err, 2u);
                        return SLOT_OVF;
                    }
                }
                load_rec<NQ>(rs, off, d);
            }
            bool eq = true;
#pragma unroll
            for (int w = 0; w < KW; ++w) eq = eq && (d[w] == k[w]);
            if (!eq) {
                // The quads of one snapshot are separate loads: `ready` may have been sampled
                // after the key quads, so a tag hit with a key mismatch is re-read once, now
                // ordered after the ready observation (genuine 64-bit tag collisions are rare).
                load_rec<NQ>(rs, off, d);
                eq = true;
#pragma unroll
                for (int w = 0; w < KW; ++w) eq = eq && (d[w] == k[w]);
            }
            if (eq) {
                first_ins = (((uint64_t)d[KOFF / 4 + 2] | ((uint64_t)d[KOFF / 4 + 3] << 32)) & READY_IDX) - 1;
                return (uint32_t)s;
            }
        }
        s = next_slot(a, s);
    }
    atomicOr(a.err, 4u);
    return SLOT_OVF;
}

template <int KW>
struct LdsCache {
    static constexpr int KP = (KW + 3) & ~3;   // key words padded to 16 B
    uint32_t *tag;     // E: 0 = empty, else the low hash word | 1 (set once, by the claimer)
    uint32_t *st;      // E: ST_EMPTY until published, then the HBM slot
    uint32_t *key;     // E x KP
    uint64_t *agg;     // naggs x E
    uint64_t *first;   // E
    uint32_t *ghost;   // GHOST recent miss tags (admission filter)
    uint32_t E;        // 8 x nsets
    uint32_t nsets;
};

// full key compare: every quad is loaded before any is compared (a short-circuit compare
// becomes one LDS round trip per quad)
template <int KW>
__device__ __forceinline__ bool lds_key_eq(const LdsCache<KW> &c, uint32_t e, const uint32_t (&k)[KW]) {
    constexpr int NQ = LdsCache<KW>::KP / 4;
    const uint4 *p = reinterpret_cast<const uint4 *>(c.key) + (uint64_t)e * (LdsCache<KW>::KP / 4);
    uint4 q[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) q[i] = p[i];
    // the padding words are compared too (lds_adopt zeroes them): the loads stay whole
    // 16-byte reads instead of being narrowed to the key's words and split
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        diff |= q[i].x ^ (4 * i + 0 < KW ? k[4 * i + 0] : 0u);
        diff |= q[i].y ^ (4 * i + 1 < KW ? k[4 * i + 1] : 0u);
        diff |= q[i].z ^ (4 * i + 2 < KW ? k[4 * i + 2] : 0u);
        diff |= q[i].w ^ (4 * i + 3 < KW ? k[4 * i + 3] : 0u);
    }
    asm volatile("" : "+v"(diff));   // keep the OR of XORs: LLVM splits `== 0` into per-word compares
    return diff == 0;
}

// ---- per-row pieces ------------------------------------------------------------------
// Every input dword of the row is loaded unconditionally first (unused predicate and
// aggregate slots point at a readable dummy column, set up by the host), and only then
// combined.  A load whose value is used inside a branch forces the wait into that branch,
// so each guarded column used to cost a memory round trip of its own; issued together
// they retire under one wait.
template <bool NT = true>
__device__ __forceinline__ uint32_t ldd(const uint8_t *base, uint64_t off) {
    return stream_ld<NT>(reinterpret_cast<const uint32_t *>(base + (off & ~3ull)));
}

// zero-extended value of `width` bytes from the aligned dwords lo (holding its first byte)
// and hi (the next dword; used for width 8 only)
__device__ __forceinline__ uint64_t assemble(uint32_t lo, uint32_t hi, uint64_t off, uint32_t width) {
    const uint32_t lomask = width >= 4 ? 0xFFFFFFFFu : ((1u << (8 * width)) - 1u);
    const uint32_t l = (lo >> ((uint32_t)(off & 3u) * 8u)) & lomask;
    return (uint64_t)l | ((uint64_t)(width == 8 ? hi : 0u) << 32);
}

// The raw dwords of one row: issued by issue_row, combined by decode_row.  The main loop
// issues row i+1 before it waits for row i's HBM probe, so the two round trips overlap.
// NA is the number of aggregate slots the kernel carries (2 or 4).
template <class L, int NA>
struct RowRaw {
    uint32_t k[L::KW];
    uint32_t vraw, plo[PMAX], phi[PMAX], vlo[NA], vhi[NA], clo[NA], chi[NA];
};

template <class L, int NA, bool NT = true>
__device__ __forceinline__ void issue_row(const GbArgs &a, uint64_t row, RowRaw<L, NA> &R) {
    // unconditional loads; slots with nothing to load read dword 0 of the dummy column
    // (width 0: one cached line for the whole wave)
    R.vraw = ldd<NT>(a.validp, row * a.validw);
#pragma unroll
    for (int p = 0; p < PMAX; ++p) {
        const uint64_t b = row * a.pldw[p];
        R.plo[p] = ldd<NT>(a.pptr[p], b);
        R.phi[p] = ldd<NT>(a.pptr[p], b + a.phioff[p]);
    }
    L::template load<NT>(a, row, R.k);
#pragma unroll
    for (int x = 0; x < NA; ++x) {
        const uint64_t bv = row * a.vldw[x], bc = row * a.cldw[x];
        R.vlo[x] = ldd<NT>(a.vptr[x], bv);
        R.vhi[x] = ldd<NT>(a.vptr[x], bv + a.vhioff[x]);
        R.clo[x] = ldd<NT>(a.cptr[x], bc);
        R.chi[x] = ldd<NT>(a.cptr[x], bc + a.chioff[x]);
    }
}

// The cached kernel's stream loads: non-temporal, so the event stream does not push the
// table's key records out of the caches -- except for the top-file key, whose kernel is faster
// with plain loads (C5 5.94-5.98 -> 5.84 ms with a plain-load build, C2 3.7 -> 4.0).
template <class L>
constexpr bool cached_stream_nt() { return !std::is_same<L, StaticLayout<8, 4, 4, 4>>::value; }

// aggregates reading a column an earlier one already loaded reuse its value
template <int NA>
__device__ __forceinline__ void share_raw(const GbArgs &a, uint64_t (&rv)[NA], uint64_t (&rc)[NA]) {
#pragma unroll
    for (int x = 1; x < NA; ++x) {
#pragma unroll
        for (int y = 0; y < x; ++y) {
            if (a.vshare[x] == (uint32_t)y) rv[x] = rv[y];
            if (a.cshare[x] == (uint32_t)y) rc[x] = rc[y];
        }
    }
}

// the value each aggregate adds: 1 (COUNT) or the column's value (sign-extended, divided),
// 0 when its condition column does not hold cval
template <int NA>
__device__ __forceinline__ void vals_from_raw(const GbArgs &a, const uint64_t (&rv)[NA], const uint64_t (&rc)[NA],
                                              uint64_t (&v)[NA]) {
#pragma unroll
    for (int x = 0; x < NA; ++x) {
        uint64_t val = 0;
        if (x < (int)a.naggs) {
            val = a.vcount[x] ? 1ull : (a.vsign[x] ? sext(rv[x], a.vwidth[x]) : rv[x]);
            if (a.vdiv[x]) val /= a.vdiv[x];
            if (a.hascond[x] && rc[x] != a.cval[x]) val = 0;
        }
        v[x] = val;
    }
}

// A row's key words, whether it is kept (valid and predicates), and the zero-extended raw
// value / condition column values of its aggregates (an aggregate that shares another's
// column takes that one's value).  vals_from_raw turns them into the added values; the
// partitioned form stores the raw values of the loaded columns in its records.
template <class L, int NA>
__device__ __forceinline__ bool row_raw(const GbArgs &a, uint64_t row, const RowRaw<L, NA> &R,
                                        uint32_t (&k)[L::KW], uint64_t (&rv)[NA], uint64_t (&rc)[NA]) {
#pragma unroll
    for (int w = 0; w < L::KW; ++w) k[w] = R.k[w];
#pragma unroll
    for (int x = 0; x < NA; ++x) {
        rv[x] = assemble(R.vlo[x], R.vhi[x], row * a.vwidth[x], a.vwidth[x]);
        rc[x] = assemble(R.clo[x], R.chi[x], row * a.cwidth[x], a.cwidth[x]);
    }
    share_raw<NA>(a, rv, rc);
    bool ok = !a.valid || ((R.vraw >> ((uint32_t)(row & 3u) * 8u)) & 0xFFu) != 0;
#pragma unroll
    for (int p = 0; p < PMAX; ++p) {
        if (p < (int)a.npred) {
            uint64_t pv = assemble(R.plo[p], R.phi[p], row * a.pwidth[p], a.pwidth[p]);
#pragma unroll
            for (int x = 0; x < NA; ++x)
                if (a.pshare[p] == (uint32_t)x) pv = rv[x];
            bool r = pred_scalar(pv, a.pref[p], a.pwidth[p], a.pkind[p], a.pcmp[p], a.pneg[p], a.pcnt[p]);
#pragma unroll
            for (int x = 0; x < NA; ++x)
                if (a.pguard[p] == (uint32_t)x) r = r || rc[x] != a.gref[p];
            ok = ok && r;
        }
    }
    return ok;
}

template <class L, int NA>
__device__ __forceinline__ bool decode_row(const GbArgs &a, uint64_t row, const RowRaw<L, NA> &R,
                                           uint32_t (&k)[L::KW], uint64_t (&v)[NA]) {
    uint64_t rv[NA], rc[NA];
    const bool ok = row_raw<L, NA>(a, row, R, k, rv, rc);
    vals_from_raw<NA>(a, rv, rc, v);
    return ok;
}

// The LDS cache is 8-way set associative: the key hash's high word picks a set of 8
// consecutive entries, its low word (| 1) is the entry's tag.  A lookup reads the set's 8
// tags with two 16-byte LDS loads and compares full keys only on a tag match, so a miss
// costs two LDS reads, not a walk.  Entries are first come, never evicted: the claimer
// CASes the tag from 0, writes the key, then publishes the HBM slot in `st` (release); a
// reader that matches a tag but still sees ST_EMPTY treats it as a miss (its event takes
// the HBM path, which is only slower).
__device__ __forceinline__ uint32_t lds_tag(uint64_t h) { return (uint32_t)h | 1u; }

template <int KW>
__device__ __forceinline__ uint32_t lds_set(const LdsCache<KW> &c, uint64_t h) {
    return (uint32_t)(((h >> 32) * (uint64_t)c.nsets) >> 32) * 8u;
}

template <int KW>
__device__ __forceinline__ void lds_tags(const LdsCache<KW> &c, uint32_t base, uint32_t (&tg)[8]) {
    const uint4 t0 = *reinterpret_cast<const uint4 *>(c.tag + base);
    const uint4 t1 = *reinterpret_cast<const uint4 *>(c.tag + base + 4);
    tg[0] = t0.x; tg[1] = t0.y; tg[2] = t0.z; tg[3] = t0.w;
    tg[4] = t1.x; tg[5] = t1.y; tg[6] = t1.z; tg[7] = t1.w;
}

template <int KW>
__device__ __forceinline__ int lds_lookup(const LdsCache<KW> &c, const uint32_t (&k)[KW], uint64_t h, uint32_t &gs) {
    const uint32_t base = lds_set(c, h), t = lds_tag(h);
    uint32_t tg[8];
    lds_tags(c, base, tg);
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) m |= (tg[j] == t ? 1u : 0u) << j;
    while (m) {   // usually zero or one candidate
        const uint32_t e = base + (uint32_t)(__builtin_ffs((int)m) - 1);
        m &= m - 1;
        const uint32_t s = __hip_atomic_load(&c.st[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (s < ST_BUSY && lds_key_eq<KW>(c, e, k)) {
            gs = s;
            return (int)e;
        }
    }
    return -1;
}

// adopt a free entry of the key's set for a key just resolved in HBM
// Admission filter of the LDS cache.  Entries are never evicted, so admitting every missing
// key fills the cache with whichever keys come first, and the Zipf tail -- rare keys, but
// most of the misses together -- takes most entries.  A key is admitted on its second miss
// seen through a direct-mapped table of recent miss tags (GHOST entries): a tail key is
// overwritten before it misses again, a mid-frequency key is not.  (Simulated on the C2
// stream: 60 % -> 67 % LDS hits per CU at 1 088 entries; ideal LFU per set is 69 %.)
template <int KW>
__device__ __forceinline__ bool ghost_admit(const GbArgs &a, const LdsCache<KW> &c, uint64_t h) {
    if (!a.admit_mask) return true;
    // entry = tag (low 2 bits cleared) | misses seen before this one (0..3)
    const uint32_t g = (uint32_t)(h >> 20) & (GHOST - 1), t = lds_tag(h) & ~3u;
    const uint32_t cur = c.ghost[g];
    if ((cur & ~3u) == t) {
        const uint32_t seen = (cur & 3u) + 1u;
        if (seen >= a.admit_mask) return true;
        c.ghost[g] = t | seen;
        return false;
    }
    c.ghost[g] = t;   // racing writers: either tag wins, both outcomes are valid
    return false;
}

template <int KW>
__device__ __forceinline__ int lds_adopt(const LdsCache<KW> &c, const uint32_t (&k)[KW], uint64_t h, uint32_t gs) {
    const uint32_t base = lds_set(c, h);
    uint32_t tg[8];
    lds_tags(c, base, tg);
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) m |= (tg[j] == 0 ? 1u : 0u) << j;
    if (!m) return -1;   // set full
    const uint32_t e = base + (uint32_t)(__builtin_ffs((int)m) - 1);
    if (atomicCAS(&c.tag[e], 0u, lds_tag(h)) != 0u) return -1;   // lost the race: HBM path
    uint4 *kp = reinterpret_cast<uint4 *>(c.key) + (uint64_t)e * (LdsCache<KW>::KP / 4);
#pragma unroll
    for (int i = 0; i < LdsCache<KW>::KP / 4; ++i)
        kp[i] = make_uint4(4 * i + 0 < KW ? k[4 * i + 0] : 0u, 4 * i + 1 < KW ? k[4 * i + 1] : 0u,
                           4 * i + 2 < KW ? k[4 * i + 2] : 0u, 4 * i + 3 < KW ? k[4 * i + 3] : 0u);
    __hip_atomic_store(&c.st[e], gs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (int)e;
}

__device__ __forceinline__ uint64_t row_gidx(const GbArgs &a, uint64_t row) {
    return a.fidx ? a.fidx[row] : a.base_idx + row;
}

// value-record words as global (address space 1) pointers, so their atomics are global_*
// instructions: a flat atomic also counts in lgkmcnt and stalls the next LDS wait
__device__ __forceinline__ unsigned long long *rec_first(const GbArgs &a, uint32_t gs) {
    return reinterpret_cast<unsigned long long *>(a.vrec + (uint64_t)gs * a.vrec_words);
}
__device__ __forceinline__ unsigned long long *rec_agg(const GbArgs &a, uint32_t gs, int x) {
    return reinterpret_cast<unsigned long long *>(a.vrec + (uint64_t)gs * a.vrec_words + 1 + x);
}
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ void gadd(unsigned long long *p, unsigned long long v) {
    __hip_atomic_fetch_add((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gmin(unsigned long long *p, unsigned long long v) {
    __hip_atomic_fetch_min((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#else
__device__ inline void gadd(unsigned long long *, unsigned long long) {}   // host pass: never called
__device__ inline void gmin(unsigned long long *, unsigned long long) {}
#endif

template <int KW, int NA>
__device__ __forceinline__ void lds_accumulate(const GbArgs &a, const LdsCache<KW> &c, int slot,
                                               const uint64_t (&v)[NA], uint64_t gidx) {
#pragma unroll
    for (int x = 0; x < NA; ++x)
        if (x < (int)a.naggs && v[x])
            atomicAdd(reinterpret_cast<unsigned long long *>(&c.agg[x * c.E + slot]), (unsigned long long)v[x]);
    // rows arrive nearly in index order: a plain read skips most of the minima
    if (gidx < c.first[slot]) atomicMin(reinterpret_cast<unsigned long long *>(&c.first[slot]), (unsigned long long)gidx);
}

// ---- HBM atomics through an LDS ring ---------------------------------------------------
// A wave's vmcnt counts its stores and atomics with its loads, in issue order, so a miss's
// memory-side atomics delayed that wave's next load wait by their whole acknowledgement
// latency (longer than a load's).  Producer waves therefore push each HBM update as a
// 16-byte ring entry {slot, lap|what, value} into LDS, and one server wave per workgroup
// issues them; it loads nothing, so nothing ever waits on their acknowledgement.
constexpr uint32_t ARING = 512;             // HBM-update ring entries (16 B each)
// Every wait on another wave is bounded: a wait that never ends sets err bit 4
// (igx_groupby_finalize then fails with IGX_ENOSPC) instead of hanging the GPU.
constexpr uint32_t SPIN_LIMIT = 1u << 24;
constexpr uint32_t WHAT_MIN = 15;           // entry kind: atomicMin on `first`
// (Round 6 tried padding each lane's run of entries so that no miss's updates straddle an 8-lane
// group of the server's instruction: the memory-side atomic requests fell by 1M of the 7M that
// grouping predicted, and the kernels did not get faster -- DESIGN.md §4, "Round 6: the
// memory-side atomics".  Not kept.)
// wave roles in a workgroup: a.nl loaders stream rows, the next 15 - a.nl waves (probers)
// resolve LDS misses against HBM, and the last wave serves the HBM-update ring
constexpr uint32_t NWAVES = GTB / 64;
constexpr uint32_t NL_DEFAULT = 8;    // loader waves (7 probers + 1 server); IGX_GB_LOADERS sweeps

struct Ring {
    uint2 *lo;            // {slot, (lap << 4) | what}
    uint64_t *hi;         // value
    uint32_t *ctl;        // [0] tail (reserved), [1] head (consumed), [2] producer waves done
};

__device__ __forceinline__ uint32_t ring_lap(uint32_t p) { return (p / ARING + 1u) << 4; }

// Push this lane's HBM updates (the aggregates it adds, and a first-index minimum when
// gidx < first_ins) for slot gs.  Called by the active (missing) lanes of a producer wave.
template <int NA>
__device__ __forceinline__ void ring_push(const GbArgs &a, const Ring &r, uint32_t gs, const uint64_t (&v)[NA],
                                          uint64_t gidx, uint64_t first_ins) {
    if (a.direct) {   // the prober issues its own atomics (no server wave)
#pragma unroll
        for (int x = 0; x < NA; ++x)
            if (x < (int)a.naggs && v[x]) gadd(rec_agg(a, gs, x), (unsigned long long)v[x]);
        if (gidx < first_ins) gmin(rec_first(a, gs), (unsigned long long)gidx);
        return;
    }
    // A lane's entries are consecutive in the ring, so the server issues one slot's updates
    // from adjacent lanes of one instruction: they fall in the slot's value record, one 64-B
    // line, and leave the CU as one memory-side atomic request instead of one per update
    // (top file: count and bytes of the same op, two updates per miss).
    bool has[NA + 1];
    uint32_t c = 0;
#pragma unroll
    for (int x = 0; x <= NA; ++x) {
        has[x] = x < NA ? (x < (int)a.naggs && v[x] != 0) : gidx < first_ins;
#ifdef IGX_DIAG_HALF_ATOMICS   // diagnostic build only (wrong sums): the bound of one atomic per miss
        if (NA == 4 && (x == 1 || x == 3)) has[x] = false;
#endif
        c += has[x] ? 1u : 0u;
    }
    const uint64_t lt = lanemask_lt();
    uint32_t pre = 0, total = 0;   // wave prefix / total of c (c <= NA + 1 <= 5: three bits)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint64_t m = __ballot((c >> b) & 1u);
        pre += (uint32_t)__popcll(m & lt) << b;
        total += (uint32_t)__popcll(m) << b;
    }
    if (!total) return;
    const uint64_t active = __ballot(true);
    const uint32_t leader = (uint32_t)__ffsll((long long)active) - 1;
    uint32_t base = 0;
    if ((threadIdx.x & 63) == leader) base = atomicAdd(&r.ctl[0], total);
    base = __shfl(base, (int)leader);
    // wait for room: the server frees entries as it issues them
    uint32_t spins = 0;
    for (; base + total - __hip_atomic_load(&r.ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > ARING;) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_LIMIT) { atomicOr(a.err, 16u); return; }   // never expected: fail, do not hang
    }
    if ((a.dbg & 65536u) && spins && (threadIdx.x & 63) == leader)
        atomicAdd(a.dbg_cnt + 6, 1ull * spins);   // prober: update ring full
    uint32_t p = base + pre;
#pragma unroll
    for (int x = 0; x <= NA; ++x) {
        if (has[x]) {
            r.hi[p % ARING] = x < NA ? v[x] : gidx;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            r.lo[p % ARING] = make_uint2(gs, ring_lap(p) | (x < NA ? (uint32_t)x : WHAT_MIN));
            ++p;
        }
    }
}

// Diagnostics (IGX_GB_DEBUG bit 18, the debug kernels only): what one wave-wide atomic
// instruction becomes at the memory side, counted into dbg_cnt[base ..]: +0 lanes, +1 of them
// minima, +2 distinct (value record, opcode) pairs -- the L2 sends a record's same-opcode lanes
// of one instruction as one request --, +3 distinct (128-B line, opcode) pairs,
// +4 instructions whose first record continues the previous instruction's last (a miss's
// updates split over two instructions).  Kept per wave in registers, added at the end.
__device__ __forceinline__ void atomics_account(const GbArgs &a, bool live, uint32_t slot, bool is_min, uint32_t lane,
                                                uint32_t base) {
    uint64_t todo = __ballot(live);
    if (!todo) return;
    const uint64_t nmin = (uint64_t)__popcll(__ballot(live && is_min));
    uint64_t recs = 0, lines = 0;
    const uint32_t per_line = max(1u, 128u / (a.vrec_words * 8));
    while (todo) {
        const uint32_t l = (uint32_t)__ffsll((long long)todo) - 1;
        const uint32_t s0 = __shfl(slot, (int)l), k0 = __shfl((uint32_t)is_min, (int)l);
        todo &= ~__ballot(live && slot == s0 && (uint32_t)is_min == k0);
        ++recs;
    }
    todo = __ballot(live);
    while (todo) {
        const uint32_t l = (uint32_t)__ffsll((long long)todo) - 1;
        const uint32_t s0 = __shfl(slot, (int)l) / per_line, k0 = __shfl((uint32_t)is_min, (int)l);
        todo &= ~__ballot(live && slot / per_line == s0 && (uint32_t)is_min == k0);
        ++lines;
    }
    const uint64_t nlive = (uint64_t)__popcll(__ballot(live));
    if (lane == 0) {
        atomicAdd(a.dbg_cnt + base, (unsigned long long)nlive);
        atomicAdd(a.dbg_cnt + base + 1, (unsigned long long)nmin);
        atomicAdd(a.dbg_cnt + base + 2, (unsigned long long)recs);
        atomicAdd(a.dbg_cnt + base + 3, (unsigned long long)lines);
    }
}

// the server wave: issue ring entries in order until every producer is done and the ring
// is empty
template <bool DBG>
__device__ __forceinline__ void ring_serve(const GbArgs &a, const Ring &r, uint32_t lane) {
    uint32_t head = 0;
    [[maybe_unused]] uint32_t prev_last = 0xFFFFFFFFu;   // diagnostics: the last record of the previous instruction
    for (;;) {
        const uint32_t t = __hip_atomic_load(&r.ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (t == head) {
            if (__hip_atomic_load(&r.ctl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == NWAVES - 1 - a.nl &&
                __hip_atomic_load(&r.ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == head)
                break;
            __builtin_amdgcn_s_sleep(2);   // idle until the probers push or finish (no limit:
            if (DBG && (a.dbg & 65536u) && lane == 0) atomicAdd(a.dbg_cnt + 7, 1ull);   // server idle
            continue;                      // they bound their own waits)
        }
        const uint32_t n = min(t - head, 64u);
        uint32_t slot = 0xFFFFFFFFu, what = 0;
        if (lane < n) {
            const uint32_t p = head + lane;
            uint64_t w;
            uint32_t spins = 0;
            while (((uint32_t)((w = __hip_atomic_load(reinterpret_cast<uint64_t *>(&r.lo[p % ARING]),
                                                      __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 32) &
                    ~15u) != ring_lap(p)) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > SPIN_LIMIT) { atomicOr(a.err, 16u); break; }
            }
            const uint64_t val = r.hi[p % ARING];
            slot = (uint32_t)w;
            what = (uint32_t)(w >> 32) & 15u;
            if (DBG && (a.dbg & 131072u)) {   // diagnostics: plain stores instead of the atomics
                if (what == WHAT_MIN) *rec_first(a, slot) = val;
                else *rec_agg(a, slot, (int)what) = val;
            } else if (!(DBG && (a.dbg & 4u))) {
                if (what == WHAT_MIN) gmin(rec_first(a, slot), val);
                else gadd(rec_agg(a, slot, (int)what), val);
            }
        }
        if (DBG && (a.dbg & 262144u)) {
            const bool live = lane < n;
            atomics_account(a, live, slot, what == WHAT_MIN, lane, 8);
            // the same pairs split at 32-, 16- and 8-lane boundaries: which grouping of the
            // instruction's lanes the memory-side request count follows
            for (uint32_t g = 0; g < 3; ++g) {
                const uint32_t sh = 5 - g;
                uint64_t todo = __ballot(live);
                uint64_t cnt = 0;
                while (todo) {
                    const uint32_t l = (uint32_t)__ffsll((long long)todo) - 1;
                    const uint32_t s0 = __shfl(slot, (int)l), k0 = __shfl(what == WHAT_MIN ? 1u : 0u, (int)l);
                    todo &= ~__ballot(live && slot == s0 && (what == WHAT_MIN ? 1u : 0u) == k0 && (lane >> sh) == (l >> sh));
                    ++cnt;
                }
                if (lane == 0) atomicAdd(a.dbg_cnt + 13 + g, (unsigned long long)cnt);
            }
            const uint32_t first_slot = __shfl(slot, 0), last_slot = __shfl(slot, (int)(n - 1));
            if (lane == 0 && first_slot == prev_last) atomicAdd(a.dbg_cnt + 12, 1ull);
            prev_last = last_slot;
        }
        head += n;
        if (lane == 0) __hip_atomic_store(&r.ctl[1], head, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// ---- loader -> prober hand-off: the miss ring -----------------------------------------
// A loader that misses the LDS cache does not probe HBM itself (its next row would wait
// for the probe's round trip): it writes the row's key, hash, index and aggregate values
// into a ring cell and moves on.  Prober waves take 64 cells at a time and resolve them.
// Cells follow the bounded MPMC sequence protocol: cell i starts with seq = i; the
// producer of position p waits for seq == p, fills the cell and sets seq = p + 1; the
// consumer of p waits for seq == p + 1, reads the cell and sets seq = p + MRING.
constexpr uint32_t MRING = 256;

template <int KW, int NA>
struct MissRing {
    static constexpr int KQ = LdsCache<KW>::KP / 4;          // key quads
    static constexpr int EQ = KQ + 1 + (NA + 1) / 2;         // + {hash, index} + values
    uint4 *cell;      // MRING x EQ
    uint32_t *seq;    // MRING
    uint32_t *ctl;    // [0] tail (reservations), [1] head (claims), [2] loader waves done
    uint32_t *err;
    unsigned long long *waits;   // diagnostics (IGX_GB_DEBUG bit 16): sleep counts, else null
};

template <int KW, int NA>
__device__ __forceinline__ void miss_push(const MissRing<KW, NA> &m, const uint32_t (&k)[KW], uint64_t h,
                                          uint64_t gidx, const uint64_t (&v)[NA]) {
    const uint64_t active = __ballot(true);
    const uint32_t leader = (uint32_t)__ffsll((long long)active) - 1;
    uint32_t base = 0;
    if ((threadIdx.x & 63) == leader) base = atomicAdd(&m.ctl[0], (uint32_t)__popcll(active));
    base = __shfl(base, (int)leader);
    const uint32_t p = base + (uint32_t)__popcll(active & lanemask_lt());
    uint32_t *sq = &m.seq[p % MRING];
    uint32_t spins = 0;
    for (; __hip_atomic_load(sq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != p;) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_LIMIT) { atomicOr(m.err, 16u); return; }
    }
    if (m.waits && spins) atomicAdd(m.waits + 4, (unsigned long long)spins);   // loader: ring full
    uint4 *cl = m.cell + (uint64_t)(p % MRING) * MissRing<KW, NA>::EQ;
#pragma unroll
    for (int q = 0; q < MissRing<KW, NA>::KQ; ++q)
        cl[q] = make_uint4(4 * q + 0 < KW ? k[4 * q + 0] : 0u, 4 * q + 1 < KW ? k[4 * q + 1] : 0u,
                           4 * q + 2 < KW ? k[4 * q + 2] : 0u, 4 * q + 3 < KW ? k[4 * q + 3] : 0u);
    cl[MissRing<KW, NA>::KQ] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)gidx, (uint32_t)(gidx >> 32));
#pragma unroll
    for (int x = 0; x < NA; x += 2) {
        const uint64_t v1 = x + 1 < NA ? v[x + 1] : 0ull;
        cl[MissRing<KW, NA>::KQ + 1 + x / 2] = make_uint4((uint32_t)v[x], (uint32_t)(v[x] >> 32), (uint32_t)v1,
                                                          (uint32_t)(v1 >> 32));
    }
    __hip_atomic_store(sq, p + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Probers resolve PB misses per lane at a time (PB = 1: two per lane measured slower -- C5
// 6.41 -> 6.72-6.80 ms, C2 unchanged, and for the 72-B key they spill): the LDS cache again (a prober may have adopted the key since), then
// the HBM table, then adoption of a free LDS entry or the HBM-update ring.

template <int KW, int NA>
struct MissRow {
    uint32_t k[KW];
    uint64_t h, gidx;
    uint64_t v[NA];
};

template <int KW, int NA>
__device__ __forceinline__ void read_cell(const MissRing<KW, NA> &m, uint32_t p, MissRow<KW, NA> &x) {
    const uint4 *cl = m.cell + (uint64_t)(p % MRING) * MissRing<KW, NA>::EQ;
#pragma unroll
    for (int q = 0; q < MissRing<KW, NA>::KQ; ++q) {
        const uint4 t = cl[q];
        if (4 * q + 0 < KW) x.k[4 * q + 0] = t.x;
        if (4 * q + 1 < KW) x.k[4 * q + 1] = t.y;
        if (4 * q + 2 < KW) x.k[4 * q + 2] = t.z;
        if (4 * q + 3 < KW) x.k[4 * q + 3] = t.w;
    }
    const uint4 hq = cl[MissRing<KW, NA>::KQ];
    x.h = (uint64_t)hq.x | ((uint64_t)hq.y << 32);
    x.gidx = (uint64_t)hq.z | ((uint64_t)hq.w << 32);
#pragma unroll
    for (int i = 0; i < NA; i += 2) {
        const uint4 t = cl[MissRing<KW, NA>::KQ + 1 + i / 2];
        x.v[i] = (uint64_t)t.x | ((uint64_t)t.y << 32);
        if (i + 1 < NA) x.v[i + 1] = (uint64_t)t.z | ((uint64_t)t.w << 32);
    }
}

// The state-machine prober: every lane owns one miss and advances it by one step per round
// trip, so a lane that has to claim a record (CAS, then key / value stores, then `ready`)
// does not hold the other 63 lanes for the extra round trips.  Per iteration: free lanes
// take cells from the miss ring; lanes in PROBE load their slot's record, lanes in CASQ
// issue their claim; one wait covers all of it (and the previous iteration's stores); then
// PUB lanes publish, CAS lanes act on the result, PROBE lanes read their record.
// States: FREE -> PROBE -> (found: FREE) | (empty: CASQ -> CAS -> (won: PUB -> FREE) |
// (lost: PROBE)).
template <int KW, int NA, bool DBG>
__device__ __forceinline__ void finish_miss(const GbArgs &a, const LdsCache<KW> &c, const Ring &r,
                                            const MissRow<KW, NA> &x, uint32_t gs, uint64_t first_ins,
                                            bool claimed = false) {
    const int ad = ghost_admit<KW>(a, c, x.h) ? lds_adopt<KW>(c, x.k, x.h, gs) : -1;
    if (claimed) return;   // the claim wrote this event's values into the new record
    if (ad >= 0) lds_accumulate<KW, NA>(a, c, ad, x.v, x.gidx);
    else ring_push<NA>(a, r, gs, x.v, x.gidx, first_ins);
}

// A kept key's first miss of the interval (its `ready` carries an earlier epoch of the
// generation): `ready` takes the interval's epoch and first_ins = gidx + 1 -- an upper bound the
// value record will meet, because this event's own minimum is pushed (gidx < first_ins) -- and
// the slot is marked occupied.  Racing re-stamps of one key each push their own minimum, so
// whichever `ready` lands, every later reader's first_ins is met.  Returns the first_ins to use.
template <int KW>
__device__ __forceinline__ uint64_t restamp(const GbArgs &a, uint64_t s, uint64_t gidx) {
    if (gidx + 1 >= READY_IDX) {   // an index column value that `ready` cannot carry
        atomicOr(a.err, 8u);
        return READY_IDX;          // still correct: every event pushes its minimum
    }
    st_agent(reinterpret_cast<uint64_t *>(a.krec + s * a.krec_len + koff_of(KW) + 8), (a.ep << 48) | (gidx + 2));
    __builtin_nontemporal_store((uint8_t)1, a.occb + s);
    return gidx + 1;
}

template <int KW, int NA, bool DBG>
__device__ __forceinline__ void prober_sm(const GbArgs &a, const LdsCache<KW> &c, const Ring &r,
                                          const MissRing<KW, NA> &m, uint32_t lane, uint32_t gep,
                                          uint32_t *nclaim) {
    constexpr uint32_t KOFF = koff_of(KW);
    constexpr int NQ = probe_quads<KW>();
    constexpr uint32_t FREE = 0, PROBE = 1, CASQ = 2, PUB = 3;
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(a);
    MissRow<KW, NA> x;
    uint32_t st = FREE, s = 0, probes = 0, tries = 0, reread = 0;
    uint64_t expect = 0;
    for (uint32_t idle = 0;;) {
        // 1. refill the free lanes with cells the loaders have reserved
        const uint64_t fm = __ballot(st == FREE);
        bool drained = false;
        if (fm) {
            const uint32_t tail = __hip_atomic_load(&m.ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const bool done = __hip_atomic_load(&m.ctl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == a.nl;
            const uint32_t head = __hip_atomic_load(&m.ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t avail = (int32_t)(tail - head) > 0 ? tail - head : 0u;
            const uint32_t want = min((uint32_t)__popcll(fm), avail);
            drained = done && avail == 0;
            if (want) {
                const uint32_t leader = (uint32_t)__ffsll((long long)fm) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&m.ctl[1], want);
                base = __shfl(base, (int)leader);
                const uint32_t rank = (uint32_t)__popcll(fm & lanemask_lt());
                if (st == FREE && rank < want) {
                    const uint32_t p = base + rank;
                    uint32_t *sq = &m.seq[p % MRING];
                    bool have = true;
                    for (uint32_t spins = 0;
                         __hip_atomic_load(sq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != p + 1;) {
                        if (__hip_atomic_load(&m.ctl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == a.nl &&
                            p >= __hip_atomic_load(&m.ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                            have = false;   // over-claimed past the end of a finished stream
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > SPIN_LIMIT) { atomicOr(a.err, 16u); have = false; break; }
                    }
                    if (have) {
                        read_cell<KW, NA>(m, p, x);
                        __hip_atomic_store(sq, p + MRING, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        uint32_t gs = SLOT_OVF;
                        const int slot = lds_lookup<KW>(c, x.k, x.h, gs);   // adopted meanwhile?
                        if (slot >= 0) {
                            lds_accumulate<KW, NA>(a, c, slot, x.v, x.gidx);
                        } else {
                            st = PROBE;
                            s = (uint32_t)home_slot(a, x.h);
                            probes = 0;
                            tries = 0;
                            reread = 0;
                        }
                    }
                }
            }
        }
        const uint64_t busy = __ballot(st != FREE);
        if (!busy) {
            if (drained) break;
            __builtin_amdgcn_s_sleep(1);   // waiting for misses: as long as the stream lasts
            if (++idle > SPIN_LIMIT) { atomicOr(a.err, 16u); break; }
            continue;
        }
        idle = 0;
        // 2. issue this round trip's loads and claims
        const uint64_t tag = (x.h & ~EP_MAX) | gep;
        uint8_t *rec = a.krec + (uint64_t)s * a.krec_len;
        uint32_t d[NQ * 4];
        uint64_t cas_old = 0;
        const bool probed = st == PROBE;   // only these lanes have a record in d this round
        if (probed) load_rec<NQ>(rs, s * a.krec_len, d);
        if (st == CASQ)
            cas_old = atomicCAS(reinterpret_cast<unsigned long long *>(rec + KOFF), (unsigned long long)expect,
                                (unsigned long long)tag);
        // 3. one wait: probe data, claims, and the previous iteration's stores
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // 4. publish the records claimed last iteration (their stores are now complete)
        if (st == PUB) {
            st_agent(reinterpret_cast<uint64_t *>(rec + KOFF + 8), (a.ep << 48) | (x.gidx + 1));
            __builtin_nontemporal_store((uint8_t)1, a.occb + s);
            finish_miss<KW, NA, DBG>(a, c, r, x, s, x.gidx, true);
            st = FREE;
        }
        // 5. claims: won -> write key and value record now, publish next iteration
        if (st == CASQ) {
            if (cas_old == expect) {
#pragma unroll
                for (int w = 0; w < KW; w += 2) {
                    if (w + 1 < KW)
                        st_agent(reinterpret_cast<uint64_t *>(rec + 4 * w), (uint64_t)x.k[w] | ((uint64_t)x.k[w + 1] << 32));
                    else
                        st_agent(reinterpret_cast<uint32_t *>(rec + 4 * w), x.k[w]);
                }
                vrec_init<NA>(a, s, x.gidx, x.v);   // with this event's own values (finish_miss skips them)
                st = PUB;
            } else if (cas_old == tag) {
                st = PROBE;   // lost to a claim of the same hash: read its key once `ready` is set
                if (++tries > (1u << 18)) { atomicOr(a.err, 2u); st = FREE; }
            } else {
                st = PROBE;   // lost to another key (the CAS saw the current tag): next slot
                reread = 0;
                s = (uint32_t)next_slot(a, s);
                if (++probes >= a.max_probe) { atomicOr(a.err, 4u); st = FREE; }
            }
        }
        {   // this round's claims (every earlier PUB lane published in step 4)
            const uint64_t pub = __ballot(st == PUB);
            if (pub && lane == 0) atomicAdd(nclaim, (uint32_t)__popcll(pub));
        }
        // 6. probe results (lanes that lost a claim in step 5 read their record next round)
        if (probed && st == PROBE) {
            const uint64_t t = (uint64_t)d[KOFF / 4] | ((uint64_t)d[KOFF / 4 + 1] << 32);
            const uint64_t ready = (uint64_t)d[KOFF / 4 + 2] | ((uint64_t)d[KOFF / 4 + 3] << 32);
            if ((t & EP_MAX) != gep) {
                expect = t;          // empty in this generation: claim it next round trip
                st = CASQ;
                if (++tries > (1u << 18)) { atomicOr(a.err, 2u); st = FREE; }
            } else if (t == tag) {
                if (!ready_pub(ready, gep, a.ep)) {
                    if (++tries > (1u << 18)) { atomicOr(a.err, 2u); st = FREE; }   // the claimer is still writing
                } else {
                    bool eq = true;
#pragma unroll
                    for (int w = 0; w < KW; ++w) eq = eq && (d[w] == x.k[w]);
                    if (eq) {
                        const uint64_t fi = (ready >> 48) == a.ep ? (ready & READY_IDX) - 1 : restamp<KW>(a, s, x.gidx);
                        finish_miss<KW, NA, DBG>(a, c, r, x, s, fi);
                        st = FREE;
                    } else if (!reread) {
                        reread = 1;  // the key quads may predate `ready`: read once more
                        ++tries;
                    } else {
                        reread = 0;
                        s = (uint32_t)next_slot(a, s);
                        if (++probes >= a.max_probe) { atomicOr(a.err, 4u); st = FREE; }
                    }
                }
            } else {
                reread = 0;
                s = (uint32_t)next_slot(a, s);
                if (++probes >= a.max_probe) { atomicOr(a.err, 4u); st = FREE; }
            }
        }
    }
}

// Cooperative claim stores (the whole wave calls it; `claim` marks the lanes that won a
// slot's tag this round).  A claimer's key record (key words, padding, tag) and value record
// (first = its event index, its own values) are spread over the wave -- lane l writes quad
// l % CQ of the (l / CQ)-th claim of the round -- so each record leaves as one store
// instruction's adjacent 16-B pieces: one write-through request per 64 B, instead of a request
// per 16-B store of a lane writing its record alone (C5: 5 of a claim's 8 requests, C2: 7 of 10).
// Ends with s_waitcnt vmcnt(0): the records are visible before the claimers publish `ready`.
template <int KW, int NA, bool WAIT = true>
__device__ __forceinline__ void claim_store_coop(const GbArgs &a, bool claim, uint32_t s, const uint32_t (&k)[KW],
                                                 uint64_t tag, uint64_t gidx, const uint64_t (&v)[NA]) {
    constexpr uint32_t KOFF = koff_of(KW);
    constexpr int KQ = (int)((KOFF + 8) / 16);   // key quads, through the tag word when it ends one
    constexpr int VQ = (NA + 2) / 2;             // first + NA aggregates
    constexpr int CQ = KQ + VQ;
    constexpr uint32_t RPI = 64 / CQ;            // claims per store instruction
    const uint32_t lane = threadIdx.x & 63;
    uint32_t w[CQ * 4];
#pragma unroll
    for (int i = 0; i < KQ * 4; ++i) {
        const uint32_t b = 4u * (uint32_t)i;
        w[i] = b < 4u * KW ? k[i] : (b < KOFF ? 0u : (b == KOFF ? (uint32_t)tag : (uint32_t)(tag >> 32)));
    }
#pragma unroll
    for (int i = 0; i < VQ * 2; ++i) {
        const uint64_t x = i == 0 ? gidx : (i - 1 < NA && (uint32_t)(i - 1) < a.naggs ? v[i - 1 < NA ? i - 1 : 0] : 0ull);
        w[KQ * 4 + 2 * i] = (uint32_t)x;
        w[KQ * 4 + 2 * i + 1] = (uint32_t)(x >> 32);
    }
    const uint32_t r = lane / CQ, q = lane % CQ;
    const __amdgpu_buffer_rsrc_t rk = rec_rsrc(a);
    for (uint64_t todo = __ballot(claim); todo;) {
        uint64_t m = todo;
        for (uint32_t i = 0; i < r && m; ++i) m &= m - 1;   // the r-th claimer of the round
        const bool mine = r < RPI && m != 0;
        const uint32_t src = mine ? (uint32_t)__ffsll((long long)m) - 1 : lane;
        const uint32_t slot = __shfl(s, (int)src);
        uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int qq = 0; qq < CQ; ++qq) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t y = __shfl(w[4 * qq + j], (int)src);
                if (q == (uint32_t)qq) o[j] = y;
            }
        }
        if (mine) {
            const u4v val = {o[0], o[1], o[2], o[3]};
            if (q < (uint32_t)KQ) {
                __builtin_amdgcn_raw_buffer_store_b128(val, rk, slot * a.krec_len + 16 * q, 0, 16 /* sc1 */);
            } else {
                const uint32_t off = 16 * (q - KQ), vlen = a.vrec_words * 8;
                uint64_t *vr = a.vrec + (uint64_t)slot * a.vrec_words;
                if (off + 16 <= vlen) {
                    if (a.vrec_total) {
                        const __amdgpu_buffer_rsrc_t rv =
                            __builtin_amdgcn_make_buffer_rsrc(a.vrec, (short)0, (int)a.vrec_total, 0x00020000);
                        __builtin_amdgcn_raw_buffer_store_b128(val, rv, slot * a.vrec_words * 8 + off, 0, 16 /* sc1 */);
                    } else {
                        st_agent(vr + off / 8, (uint64_t)o[0] | ((uint64_t)o[1] << 32));
                        st_agent(vr + off / 8 + 1, (uint64_t)o[2] | ((uint64_t)o[3] << 32));
                    }
                } else if (off < vlen) {
                    st_agent(vr + off / 8, (uint64_t)o[0] | ((uint64_t)o[1] << 32));
                }
            }
        }
        for (uint32_t i = 0; i < RPI && todo; ++i) todo &= todo - 1;
    }
    if constexpr (WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The batch prober: a wave takes 64 cells of the miss ring and resolves them together, one
// round trip per round: every unresolved lane reads its current slot's record; a lane that
// finds it empty claims it (CAS), and the round's claims are written cooperatively
// (claim_store_coop) and published (`ready`, then the occupancy byte) at the top of the next
// round -- which waits for its probe loads anyway -- or, when the batch is resolved, before the
// wave takes its next cells, so the stores overlap the LDS adoption and ring pushes instead of
// a wait of their own.  A lane that meets its own tag
// not yet published -- possibly claimed by a lane of this very wave -- reads it again next
// round instead of spinning.  Resolved misses then adopt a free LDS entry or go to the
// HBM-update ring.
template <int KW, int NA, bool DBG, int PB>
__device__ __forceinline__ void prober(const GbArgs &a, const LdsCache<KW> &c, const Ring &r,
                                       const MissRing<KW, NA> &m, uint32_t lane, uint32_t gep,
                                       uint32_t *nclaim) {
    constexpr uint32_t KOFF = koff_of(KW);
    constexpr int NQ = probe_quads<KW>();
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(a);
    // a claim written but not yet published: its slot (SLOT_OVF: none) and event index
    uint32_t pend_s[PB];
    uint64_t pend_g[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) pend_s[j] = SLOT_OVF;
    auto publish = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the claims' key / value stores
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            if (pend_s[j] != SLOT_OVF) {
                st_agent(reinterpret_cast<uint64_t *>(a.krec + (uint64_t)pend_s[j] * a.krec_len + KOFF + 8),
                         (a.ep << 48) | (pend_g[j] + 1));
                __builtin_nontemporal_store((uint8_t)1, a.occb + pend_s[j]);
                pend_s[j] = SLOT_OVF;
            }
        }
    };
    for (;;) {
        publish();   // the previous batch's last claims (their stores overlapped its LDS work)
        uint32_t claim = 0;
        if (lane == 0) claim = atomicAdd(&m.ctl[1], 64u * PB);
        claim = __shfl(claim, 0);
        MissRow<KW, NA> x[PB];
        bool have[PB], act[PB];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const uint32_t p = claim + lane + 64u * j;
            uint32_t *sq = &m.seq[p % MRING];
            uint32_t spins = 0;
            have[j] = true;
            while (__hip_atomic_load(sq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != p + 1) {
                if (__hip_atomic_load(&m.ctl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == a.nl) {
                    if (p >= __hip_atomic_load(&m.ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        have[j] = false;   // past the last miss of a finished stream
                        break;
                    }
                    // the loaders are done, so the cell is being written right now: bounded
                    if (++spins > SPIN_LIMIT) { atomicOr(a.err, 16u); have[j] = false; break; }
                }
                __builtin_amdgcn_s_sleep(1);   // waiting for misses: as long as the stream lasts
                if (DBG && m.waits) atomicAdd(m.waits + 5, 1ull);              // prober: ring empty
            }
            if (have[j]) {
                read_cell<KW, NA>(m, p, x[j]);
                __hip_atomic_store(sq, p + MRING, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);   // free
            }
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < PB; ++j) any = any || have[j];
        if (__ballot(any) == 0) break;
        uint32_t gs[PB];
        uint64_t first_ins[PB], s[PB];
        bool claimed[PB], reread[PB];
        uint32_t probes[PB], tries[PB];
        uint32_t d[PB][NQ * 4];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            act[j] = false;
            gs[j] = SLOT_OVF;
            first_ins[j] = 0;
            claimed[j] = reread[j] = false;
            probes[j] = tries[j] = 0;
            if (have[j]) {
                uint32_t g = SLOT_OVF;
                const int slot = lds_lookup<KW>(c, x[j].k, x[j].h, g);
                if (slot >= 0) lds_accumulate<KW, NA>(a, c, slot, x[j].v, x[j].gidx);
                else act[j] = true;
            }
            if (DBG && (a.dbg & 256u) && act[j]) {   // diagnostics: no probe (the home slot, unverified)
                gs[j] = (uint32_t)home_slot(a, x[j].h);
                act[j] = false;
            }
            s[j] = home_slot(a, x[j].h);
            if (act[j]) load_rec<NQ>(rs, (uint32_t)(s[j] * a.krec_len), d[j]);
        }
        for (;;) {
            bool more = false;
#pragma unroll
            for (int j = 0; j < PB; ++j) more = more || act[j];
            if (!__ballot(more)) break;
            publish();   // waits for this round's probe loads, which it needs anyway
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                const uint64_t tag = (x[j].h & ~EP_MAX) | gep;
                bool won = false;
                if (act[j]) {
                    uint8_t *rec = a.krec + s[j] * a.krec_len;
                    uint64_t t = (uint64_t)d[j][KOFF / 4] | ((uint64_t)d[j][KOFF / 4 + 1] << 32);
                    uint64_t ready = (uint64_t)d[j][KOFF / 4 + 2] | ((uint64_t)d[j][KOFF / 4 + 3] << 32);
                    bool next = false;
                    if ((t & EP_MAX) != gep) {   // empty in this generation: claim it
                        if (x[j].gidx >= READY_IDX) {   // an index column value that `ready` cannot carry
                            atomicOr(a.err, 8u);
                            act[j] = false;
                        } else {
                            const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long *>(rec + KOFF),
                                                           (unsigned long long)t, (unsigned long long)tag);
                            if (old == t) {
                                won = true;
                                act[j] = false;
                                gs[j] = (uint32_t)s[j];
                            } else {
                                t = old;     // a claim raced ours: its key may still be in flight
                                ready = 0;
                            }
                        }
                    }
                    if (act[j]) {
                        if (t == tag) {
                            if (!ready_pub(ready, gep, a.ep)) {
                                if (++tries[j] > (1u << 22)) { atomicOr(a.err, 2u); act[j] = false; }   // read again
                            } else {
                                bool eq = true;
#pragma unroll
                                for (int w = 0; w < KW; ++w) eq = eq && (d[j][w] == x[j].k[w]);
                                if (eq) {
                                    gs[j] = (uint32_t)s[j];
                                    first_ins[j] = (ready >> 48) == a.ep ? (ready & READY_IDX) - 1
                                                                         : restamp<KW>(a, s[j], x[j].gidx);
                                    act[j] = false;
                                } else if (!reread[j]) {
                                    // the quads of one snapshot are separate loads: `ready` may have
                                    // been sampled after the key quads, so read the record once more
                                    reread[j] = true;
                                } else {
                                    next = true;
                                }
                            }
                        } else {
                            next = true;
                        }
                    }
                    if (next) {
                        reread[j] = false;
                        s[j] = next_slot(a, s[j]);
                        if (++probes[j] >= a.max_probe) { atomicOr(a.err, 4u); act[j] = false; }
                    }
                }
                if (const uint64_t wm = __ballot(won)) {
                    if (lane == 0) atomicAdd(nclaim, (uint32_t)__popcll(wm));
                    claim_store_coop<KW, NA, false>(a, won, (uint32_t)s[j], x[j].k, tag, x[j].gidx, x[j].v);
                    if (won) {   // published by the next publish() (next round or next batch)
                        pend_s[j] = (uint32_t)s[j];
                        pend_g[j] = x[j].gidx;
                        first_ins[j] = x[j].gidx;
                        claimed[j] = true;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < PB; ++j)
                if (act[j]) load_rec<NQ>(rs, (uint32_t)(s[j] * a.krec_len), d[j]);
        }
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            if (gs[j] == SLOT_OVF) continue;
            const int ad = ghost_admit<KW>(a, c, x[j].h) ? lds_adopt<KW>(c, x[j].k, x[j].h, gs[j]) : -1;
            if (claimed[j]) continue;   // a claim's values are in its new record already
            if (ad >= 0) lds_accumulate<KW, NA>(a, c, ad, x[j].v, x[j].gidx);
            else ring_push<NA>(a, r, gs[j], x[j].v, x[j].gidx, first_ins[j]);
        }
    }
}

// SAMPLE: the same kernel counting the seed sample (seeds_compute), a template instance of its
// own so that traces and profiles keep its launches apart from the interval's
template <class L, bool DBG, int NA, bool SAMPLE = false>
__global__ __launch_bounds__(GTB) void k_groupby(GbArgs a) {
    constexpr int KW = L::KW;
    extern __shared__ uint64_t lds[];
    __shared__ uint32_t ring_ctl[8];
    LdsCache<KW> c;
    c.E = a.lds_entries;
    c.nsets = a.lds_entries / 8;
    const uint32_t E = c.E;
    c.first = lds;
    c.agg = lds + E;
    c.key = reinterpret_cast<uint32_t *>(lds + (1 + a.naggs) * E);
    c.st = c.key + (uint64_t)E * LdsCache<KW>::KP;
    c.tag = c.st + E;
    Ring r;
    r.hi = reinterpret_cast<uint64_t *>(c.tag + E);   // E is a multiple of 8: 8-B aligned
    r.lo = reinterpret_cast<uint2 *>(r.hi + ARING);
    r.ctl = ring_ctl;
    MissRing<KW, NA> m;
    m.cell = reinterpret_cast<uint4 *>(r.lo + ARING);   // 16-B aligned (see launch)
    m.seq = reinterpret_cast<uint32_t *>(m.cell + MRING * MissRing<KW, NA>::EQ);
    m.ctl = ring_ctl + 4;
    m.err = a.err;
    m.waits = (DBG && (a.dbg & 65536u)) ? a.dbg_cnt : nullptr;
    c.ghost = m.seq + MRING;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t e = threadIdx.x; e < E; e += GTB) {
        c.st[e] = ST_EMPTY;
        c.tag[e] = 0;
        c.first[e] = ~0ull;
        for (uint32_t x = 0; x < a.naggs; ++x) c.agg[x * E + e] = 0;
    }
    for (uint32_t e = threadIdx.x; e < ARING; e += GTB) r.lo[e] = make_uint2(0, 0);
    for (uint32_t e = threadIdx.x; e < MRING; e += GTB) m.seq[e] = e;
    for (uint32_t e = threadIdx.x; e < GHOST; e += GTB) c.ghost[e] = 0;
    if (threadIdx.x < 8) ring_ctl[threadIdx.x] = 0;
    __syncthreads();
    if (a.nseeds && *a.seed_gep == *a.gen) {
        // the keys a row sample counted most often, adopted by every workgroup up front (their
        // slots are the generation's: the seeds were looked up in it)
        constexpr uint32_t SW = LdsCache<KW>::KP + 4;
        for (uint32_t i = threadIdx.x; i < a.nseeds; i += GTB) {
            const uint32_t *sr = a.seeds + (uint64_t)i * SW;
            const uint32_t slot = sr[LdsCache<KW>::KP];
            if (slot == SLOT_OVF) continue;
            uint32_t k[KW];
#pragma unroll
            for (int w = 0; w < KW; ++w) k[w] = sr[w];
            const uint64_t h = (uint64_t)sr[LdsCache<KW>::KP + 2] | ((uint64_t)sr[LdsCache<KW>::KP + 3] << 32);
            (void)lds_adopt<KW>(c, k, h, slot);
        }
        __syncthreads();
    }

    if (wave == NWAVES - 1 && !a.direct) {
        ring_serve<DBG>(a, r, lane);
    } else if (wave >= a.nl) {
        // the generation this interval belongs to (the reset kernel decided it on the device)
        const uint32_t gep = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(uint32_t)__hip_atomic_load(a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (a.sm) prober_sm<KW, NA, DBG>(a, c, r, m, lane, gep, &ring_ctl[3]);
        else prober<KW, NA, DBG, 1>(a, c, r, m, lane, gep, &ring_ctl[3]);
        if (lane == 0) atomicAdd(&r.ctl[2], 1u);
    } else {
        const uint32_t PTB = a.nl * 64;   // rows per workgroup step
        const uint64_t stride = (uint64_t)gridDim.x * PTB;
        uint64_t base = (uint64_t)blockIdx.x * PTB + wave * 64;
        RowRaw<L, NA> R;
        uint32_t nmiss = 0;
        if (base < a.n) issue_row<L, NA, cached_stream_nt<L>()>(a, min(base + lane, a.n - 1), R);
        for (; base < a.n; base += stride) {
            const uint64_t row = base + lane;
            uint32_t k[KW];
            uint64_t v[NA];
            bool ok = decode_row<L, NA>(a, row, R, k, v) && row < a.n;
            if (base + stride < a.n) issue_row<L, NA, cached_stream_nt<L>()>(a, min(base + stride + lane, a.n - 1), R);
            const uint64_t h = hash_key<KW>(k);
            if (DBG && (a.dbg & 1u)) {   // diagnostics: load + hash only
                if (ok && h == 0x1234567ull && v[0] == 7) atomicAdd(a.dbg_cnt + 3, 1ull);   // keep live
                ok = false;
            }
            if (ok) {
                uint32_t gs = SLOT_OVF;
                const int slot = lds_lookup<KW>(c, k, h, gs);
                if (DBG && (a.dbg & 8u)) atomicAdd(a.dbg_cnt + (slot >= 0 ? 0 : 1), 1ull);
                if (slot >= 0) {
                    if (!(DBG && (a.dbg & 512u)))   // diagnostics: bit9 no LDS accumulate
                        lds_accumulate<KW, NA>(a, c, slot, v, row_gidx(a, row));
                } else if (!(DBG && (a.dbg & 2u))) {
                    miss_push<KW, NA>(m, k, h, row_gidx(a, row), v);
                    ++nmiss;
                }
            }
        }
        // LDS misses of this interval (err block + 8): the host picks the prober for the next one
        for (int o = 32; o > 0; o >>= 1) nmiss += __shfl_xor(nmiss, o);
        if (lane == 0 && nmiss) atomicAdd(reinterpret_cast<unsigned long long *>(a.err + 2), (unsigned long long)nmiss);
        if (lane == 0) atomicAdd(&m.ctl[2], 1u);
    }

    __syncthreads();
    // the cache's sums: one lane per (entry, aggregate), so an entry's adds leave from adjacent
    // lanes of one instruction into its value record -- one memory-side request per record (the
    // update ring's shape) instead of one per aggregate from a lane that owns the entry
    const uint32_t na = a.naggs;
    for (uint32_t q0 = threadIdx.x & ~63u; q0 < E * na; q0 += GTB) {   // whole waves (the diagnostics' ballots)
        const uint32_t q = q0 + lane;
        const uint32_t e = q / na, x = q - e * na;
        const uint32_t gs = q < E * na ? c.st[e] : ST_EMPTY;
        const uint64_t s = gs < ST_BUSY ? c.agg[x * E + e] : 0ull;
        if (s) gadd(rec_agg(a, gs, (int)x), (unsigned long long)s);
        if (DBG && (a.dbg & 262144u)) atomics_account(a, s != 0, gs, false, lane, 16);
    }
    for (uint32_t e = threadIdx.x; e < E; e += GTB) {
        const uint32_t gs = c.st[e];
        if (gs >= ST_BUSY) continue;
        const uint64_t f = c.first[e];
        const uint64_t rd = ld_agent(reinterpret_cast<const uint64_t *>(a.krec + (uint64_t)gs * a.krec_len +
                                                                        koff_of(KW) + 8));
        // a `ready` not (yet visibly) of this interval bounds nothing: push the minimum
        const uint64_t fi = (rd >> 48) == a.ep ? (rd & READY_IDX) - 1 : ~0ull;
        if (f < fi) gmin(rec_first(a, gs), (unsigned long long)f);
        // a seeded key may have had only LDS hits (never probed, so nothing marked it): every
        // entry with events marks its group occupied (the adopted ones again, harmlessly)
        if (a.nseeds && f != ~0ull) __builtin_nontemporal_store((uint8_t)1, a.occb + gs);
        if (DBG && (a.dbg & 262144u) && f < fi) atomicAdd(a.dbg_cnt + 20, 1ull);   // flush minima
    }
    if (threadIdx.x == 0 && ring_ctl[3])   // the workgroup's claims: the generation's key count
        atomicAdd(reinterpret_cast<unsigned long long *>(a.gen + 2), (unsigned long long)ring_ctl[3]);
}

// ---- AUTO's re-probe: the cached form's LDS miss share, estimated ---------------------------
// After a run of partitioned intervals AUTO asks whether the stream has turned skewed enough for
// the cached form.  Running a whole interval cached to find out cost C4 7.6 ms against 3.0; the
// probe interval now runs partitioned, and this kernel replays the cache's admission on a sample
// of the rows: the cached kernel's per-workgroup row interleaving, its E-entry 8-way sets and
// its second-miss ghost filter, on the key hash alone (a tag match counts as a hit; no HBM slot,
// no sums).  Its misses go to the error block's miss word, which the cached kernel would have
// written; fin_apply scales them to the interval.
template <class L, int NA>
__global__ __launch_bounds__(GTB) void k_gb_estimate(GbArgs a, uint64_t nsample) {
    constexpr int KW = L::KW;
    extern __shared__ uint64_t lds[];
    LdsCache<KW> c{};
    c.E = a.lds_entries;
    c.nsets = a.lds_entries / 8;
    c.tag = reinterpret_cast<uint32_t *>(lds);
    c.ghost = c.tag + c.E;
    for (uint32_t e = threadIdx.x; e < c.E; e += GTB) c.tag[e] = 0;
    for (uint32_t e = threadIdx.x; e < GHOST; e += GTB) c.ghost[e] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n = min(a.n, nsample);
    const uint64_t stride = (uint64_t)gridDim.x * GTB;
    uint32_t nmiss = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * GTB + wave * 64; base < n; base += stride) {
        const uint64_t row = base + lane;
        RowRaw<L, NA> R;
        issue_row<L, NA>(a, min(row, n - 1), R);
        uint32_t k[KW];
        uint64_t v[NA];
        if (!(decode_row<L, NA>(a, row, R, k, v) && row < n)) continue;
        const uint64_t h = hash_key<KW>(k);
        const uint32_t sb = lds_set(c, h), t = lds_tag(h);
        uint32_t tg[8];
        lds_tags(c, sb, tg);
        bool hit = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) hit = hit || tg[j] == t;
        if (hit) continue;
        ++nmiss;
        if (!ghost_admit<KW>(a, c, h)) continue;
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) m |= (tg[j] == 0 ? 1u : 0u) << j;
        if (m) (void)atomicCAS(&c.tag[sb + (uint32_t)(__builtin_ffs((int)m) - 1)], 0u, t);
    }
    for (int o = 32; o > 0; o >>= 1) nmiss += __shfl_xor(nmiss, o);
    if (lane == 0 && nmiss) atomicAdd(reinterpret_cast<unsigned long long *>(a.err + 2), (unsigned long long)nmiss);
}

// ---- the LDS cache's seeds -----------------------------------------------------------------
// Seed i is the key of sample-table slot sslots[i] (igx_groupby_sort's top-E by count over a row
// sample), looked up in the table's current generation (a key not there is no seed: seeds are
// only ever found keys, never claimed).  Also records the generation they belong to.
template <class L>
__global__ __launch_bounds__(256) void k_gb_seeds(GbArgs a, const uint8_t *__restrict__ skrec, uint32_t skrec_len,
                                                  const uint32_t *__restrict__ sslots, uint32_t nseeds,
                                                  uint32_t *__restrict__ seeds, uint64_t *__restrict__ seed_gep) {
    constexpr int KW = L::KW;
    constexpr uint32_t KP = LdsCache<KW>::KP, KOFF = koff_of(KW);
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t gep = (uint32_t)*a.gen;
    if (i == 0) *seed_gep = gep;
    if (i >= nseeds) return;
    uint32_t *out = seeds + (uint64_t)i * (KP + 4);
    const uint32_t ss = sslots[i];
    if (ss == 0xFFFFFFFFu) {   // fewer sampled keys than seeds
        out[KP] = SLOT_OVF;
        return;
    }
    uint32_t k[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) k[w] = reinterpret_cast<const uint32_t *>(skrec + (uint64_t)ss * skrec_len)[w];
    const uint64_t h = hash_key<KW>(k);
    const uint64_t tag = (h & ~EP_MAX) | gep;
    uint32_t found = SLOT_OVF;
    uint64_t s = home_slot(a, h);
    for (uint32_t probe = 0; probe < a.max_probe; ++probe) {
        const uint8_t *r = a.krec + s * a.krec_len;
        const uint64_t t = *reinterpret_cast<const uint64_t *>(r + KOFF);
        if ((t & EP_MAX) != gep) break;   // an empty slot of the generation: the key is not there
        if (t == tag && ready_pub(*reinterpret_cast<const uint64_t *>(r + KOFF + 8), gep, a.ep)) {
            bool eq = true;
#pragma unroll
            for (int w = 0; w < KW; ++w) eq = eq && reinterpret_cast<const uint32_t *>(r)[w] == k[w];
            if (eq) {
                found = (uint32_t)s;
                break;
            }
        }
        s = next_slot(a, s);
    }
#pragma unroll
    for (uint32_t w = 0; w < KP; ++w) out[w] = (int)w < KW ? k[w] : 0u;
    out[KP] = found;
    out[KP + 1] = 0;
    out[KP + 2] = (uint32_t)h;
    out[KP + 3] = (uint32_t)(h >> 32);
}

// ---- direct form: no LDS cache ---------------------------------------------------------
// For near-uniform, high-cardinality streams (C4's distinct tuples: nearly every row misses
// any per-CU cache) the LDS cache, its rings and its roles only add work: every row goes
// to HBM anyway.  Here each lane takes rows of a grid-stride sweep (so the whole grid
// advances through the stream in index order and first indices arrive nearly in order --
// the atomicMin on `first` is then rare) and resolves each one itself: probe, compare,
// claim, atomics.  The throughput is the chip's random-access rate (~45-50 G probes/s over
// a 1 GiB table, tools/micro/randacc.hip); occupancy, not a pipeline, hides the latency.
template <class L, int NA>
__global__ __launch_bounds__(256) void k_groupby_direct(GbArgs a) {
    constexpr int KW = L::KW;
    constexpr int U = IGX_GB_DIRECT_U;   // rows in flight per lane: all rows' loads, then all probes
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t row0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; row0 < a.n; row0 += U * stride) {
        RowRaw<L, NA> R[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t row = row0 + u * stride;
            issue_row<L, NA>(a, row < a.n ? row : row0, R[u]);
        }
        uint32_t k[U][KW];
        uint64_t v[U][NA], h[U];
        bool ok[U];
        uint32_t d[U][probe_quads<KW>() * 4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t row = row0 + u * stride;
            ok[u] = row < a.n && decode_row<L, NA>(a, row, R[u], k[u], v[u]);
            h[u] = hash_key<KW>(k[u]);
            if (ok[u]) probe_issue<KW>(a, h[u], d[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const uint64_t gidx = row_gidx(a, row0 + u * stride);
            uint64_t first_ins = 0;
            bool claimed = false;
            // no occupancy bit: finalize rebuilds the bitmap from the tags (k_occ_from_tags),
            // one streaming pass instead of a memory-side atomic per claim
            const uint32_t gs = find_or_insert<KW, false, NA>(a, k[u], h[u], gidx, first_ins, d[u], v[u], claimed);
            if (gs == SLOT_OVF || claimed) continue;
#pragma unroll
            for (int x = 0; x < NA; ++x)
                if (x < (int)a.naggs && v[u][x]) gadd(rec_agg(a, gs, x), (unsigned long long)v[u][x]);
            if (gidx < first_ins) gmin(rec_first(a, gs), (unsigned long long)gidx);
        }
    }
}

// Full clear of tags and `ready` (keys and value records are left as is).  Needed only
// when the epoch counter wraps: every other interval starts by bumping the epoch.
__global__ void k_table_clear(uint8_t *krec, uint32_t krec_len, uint32_t koff, uint64_t ns) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride)
        *reinterpret_cast<uint4 *>(krec + i * krec_len + koff) = make_uint4(0, 0, 0, 0);
}

// ---- finalize: list the occupied slots in ascending order, from the occupancy bitmap ----
constexpr int CT = 256 * 32;   // slots per compaction tile (256 threads x one 32-slot word)

// occupancy bitmap of an interval whose claims did not set it (the direct form): slot s is
// occupied iff its tag carries the interval's epoch.  One lane per 32-slot word; the tags
// are 8-byte loads at the record stride.
__global__ __launch_bounds__(256) void k_occ_from_tags(const uint8_t *__restrict__ krec, uint32_t krec_len,
                                                       uint32_t koff, uint64_t ns, uint64_t ep,
                                                       uint32_t *__restrict__ occ) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w * 32 >= ns) return;
    uint32_t m = 0;
#pragma unroll 8
    for (uint32_t b = 0; b < 32; ++b) {
        const uint64_t s = w * 32 + b;
        const uint64_t t = s < ns ? *reinterpret_cast<const uint64_t *>(krec + s * krec_len + koff) : 0;
        m |= ((t & EP_MAX) == ep ? 1u : 0u) << b;
    }
    occ[w] |= m;   // OR: earlier cached updates of the interval may have set bits already
}

// 4 bytes of the byte map (each 0 or 1) -> 4 bits, byte j -> bit j
__device__ __forceinline__ uint32_t byte_bits(uint32_t w) { return (w | (w >> 7) | (w >> 14) | (w >> 21)) & 0xFu; }

// per-tile counts of occupied slots; with occb, first folds the byte map's 32 bytes of each
// bitmap word into it and clears them (the byte map is left zero for the next interval)
__global__ __launch_bounds__(256) void k_slots_count(uint32_t *__restrict__ occ, uint64_t nwords,
                                                     uint32_t *__restrict__ cnt, uint8_t *__restrict__ occb) {
    __shared__ uint32_t wc[4];
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t m = i < nwords ? occ[i] : 0u;
    if (occb && i < nwords) {
        uint4 *b = reinterpret_cast<uint4 *>(occb) + 2 * i;
        const uint4 b0 = b[0], b1 = b[1];
        const uint32_t w[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        uint32_t f = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) f |= byte_bits(w[j]) << (4 * j);
        if (f) {
            m |= f;
            occ[i] = m;
            b[0] = make_uint4(0, 0, 0, 0);
            b[1] = make_uint4(0, 0, 0, 0);
        }
    }
    uint32_t c = (uint32_t)__popc(m);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// finalize's read-back, written by the kernel that knows the group count straight into the
// table's coherent pinned buffer (no copy after it): err block {bits, pad, LDS misses}, count
// (then, released after them, the finalize's sequence number: the host polls it instead of
// recording an event, whose release would flush L2 between finalize and the top-K)
// It also closes the interval's books in the generation block: an interval that started its
// generation holds every group as a claim (the key count is its group count), one that
// continued adds its claims; a failed interval ends the generation.
__device__ __forceinline__ void fin_export(const uint32_t *err, uint64_t total, uint64_t *host, uint64_t seq, uint64_t ep) {
    const uint64_t e0 = *reinterpret_cast<const volatile uint64_t *>(err);
    const uint64_t e1 = *reinterpret_cast<const volatile uint64_t *>(err + 2);
    volatile uint64_t *gen = reinterpret_cast<volatile uint64_t *>(const_cast<uint32_t *>(err)) + GEN_WORD;
    const bool fresh = gen[0] == ep;
    const uint64_t claims = fresh ? total : gen[2];
    const uint64_t keys = (uint32_t)e0 ? ~0ull : (fresh ? total : gen[1] + claims);
    gen[1] = keys;
    gen[2] = 0;
    __hip_atomic_store(host, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host + 1, e1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host + 2, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host + 4, claims, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host + 5, keys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(host + 3, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_slots_scan(uint32_t *__restrict__ v, uint64_t m, uint64_t *__restrict__ total,
                                                     const uint32_t *__restrict__ err, uint64_t *__restrict__ host,
                                                     uint64_t seq, uint64_t ep) {
    __shared__ uint32_t part[1024];
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t b = threadIdx.x * per, e = min(m, b + per);
    uint32_t s = 0;
    for (uint64_t i = b; i < e; ++i) s += v[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        uint32_t x = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint64_t i = b; i < e; ++i) {
        uint32_t c = v[i];
        v[i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) {
        *total = part[1023];
        fin_export(err, part[1023], host, seq, ep);
    }
}

// The tile's slot list, staged in LDS and written out as one contiguous run.  With off null
// the tile's base is the sum of the counts of the tiles before it (read here: no scan kernel,
// for tables of at most SLOTS_INLINE_TILES tiles), and the last tile writes the total.
constexpr uint32_t SLOTS_INLINE_TILES = 4096;
__global__ __launch_bounds__(256) void k_slots_write(const uint32_t *__restrict__ occ, uint64_t nwords,
                                                     const uint32_t *__restrict__ off, const uint32_t *__restrict__ cnt,
                                                     uint32_t *__restrict__ out, uint64_t *__restrict__ total,
                                                     const uint32_t *__restrict__ err, uint64_t *__restrict__ host,
                                                     uint64_t seq, uint64_t ep) {
    __shared__ uint32_t wsum[4], pre[4];
    __shared__ uint32_t buf[256 * 32];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t m = i < nwords ? occ[i] : 0u;
    const uint32_t c = (uint32_t)__popc(m);
    uint32_t inc = c;   // inclusive scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d);
        if ((int)lane >= d) inc += x;
    }
    if (lane == 63) wsum[wave] = inc;
    uint32_t base = 0;
    if (off) {
        base = off[blockIdx.x];
    } else {
        for (uint32_t j = threadIdx.x; j < blockIdx.x; j += 256) base += cnt[j];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) base += __shfl_xor(base, d);
        if (lane == 0) pre[wave] = base;
    }
    __syncthreads();
    if (!off) base = pre[0] + pre[1] + pre[2] + pre[3];
    uint32_t loc = inc - c;
    for (uint32_t w = 0; w < wave; ++w) loc += wsum[w];
    const uint32_t tile_n = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const uint32_t s0 = (uint32_t)(i * 32);
    while (m) {
        const uint32_t bit = (uint32_t)__ffs(m) - 1;
        buf[loc++] = s0 + bit;
        m &= m - 1;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < tile_n; j += 256) out[base + j] = buf[j];
    if (!off && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        *total = (uint64_t)base + tile_n;
        fin_export(err, (uint64_t)base + tile_n, host, seq, ep);
    }
}

// an interval's reset: the occupancy bitmap and the error block in one launch, and the byte
// map when claims since the last finalize left bytes in it (nb16 of its 16-B quads, else 0).
// It also decides the interval's generation: with `may` (the host's part: the last interval
// was finalized and this one is planned in the cached form) and the generation's keys within
// `limit`, the generation goes on and the last interval's groups (groups[0 .. *ng), finalize's
// slot list) get their value records back to first = UINT64_MAX, sums 0 (vq 16-B quads each);
// otherwise this interval starts a generation at its own epoch.  Every thread reads the same
// words (nothing in this launch writes gen[1] or the slot list), so all agree.
struct ResetGen {
    uint64_t *gen;            // the generation block (err words GEN_WORD..)
    uint64_t ep, limit;
    const uint32_t *groups;
    const uint64_t *ng;
    uint64_t *vrec;
    uint32_t vw, may;         // value-record words (1 or an even number), the host's part
};
__global__ __launch_bounds__(256) void k_reset_clear(uint32_t *__restrict__ occ, uint64_t nwords,
                                                     uint32_t *__restrict__ err, uint4 *__restrict__ occb,
                                                     uint64_t nb16, ResetGen rg) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t n4 = nwords / 4;
    for (uint64_t q = i; q < n4; q += stride) reinterpret_cast<uint4 *>(occ)[q] = make_uint4(0, 0, 0, 0);
    for (uint64_t q = i; q < nb16; q += stride) occb[q] = make_uint4(0, 0, 0, 0);
    if (i < (nwords & 3)) occ[n4 * 4 + i] = 0;
    if (i < 4) err[i] = 0;
    const bool cont = rg.may && rg.gen[1] <= rg.limit;
    if (cont) {
        // one lane per 16-B quad of a record, a record's quads in adjacent lanes: each record
        // leaves as one store instruction's contiguous pieces (one write request per record, the
        // claim stores' shape), not one request per quad of a lane writing its record alone.
        // RU slot-list loads are issued before their stores: one at a time, each store waited
        // for its own load's round trip and the pass was latency-bound.
        constexpr int RU = 8;
        const uint64_t ng = *rg.ng;
        const uint32_t qs = rg.vw == 1 ? 0u : (uint32_t)__builtin_ctz(rg.vw / 2);   // log2 quads per record
        const uint64_t total = ng << qs;
        const uint32_t *__restrict__ groups = rg.groups;
        uint64_t *__restrict__ vrec = rg.vrec;
        for (uint64_t j0 = i; j0 < total; j0 += RU * stride) {
            uint32_t slot[RU];
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const uint64_t j = j0 + u * stride;
                slot[u] = j < total ? groups[j >> qs] : 0u;
            }
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const uint64_t j = j0 + u * stride;
                if (j >= total) break;
                const uint32_t q = (uint32_t)(j & ((1ull << qs) - 1));
                uint64_t *v = vrec + (uint64_t)slot[u] * rg.vw;
                if (rg.vw == 1) *v = ~0ull;
                else reinterpret_cast<uint4 *>(v)[q] = q ? make_uint4(0, 0, 0, 0) : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0);
            }
        }
    }
    if (i == 0) {
        if (!cont) rg.gen[0] = rg.ep;
        rg.gen[2] = 0;
    }
}

// the interval's planned generation did not hold (its first update runs the direct or the
// partitioned form, which start their own): it starts a generation at its epoch
__global__ void k_gen_restart(uint64_t *gen, uint64_t ep) {
    gen[0] = ep;
    gen[2] = 0;
}

// materialise selected groups as packed rows key | aggs | first (the Stats rows of
// nextStats, tracer.go:186-219); aggregates wrap to their out_width (the BPF value width)
struct AggMasks {
    uint32_t m[2 * AMAX];   // (lo, hi) word masks per aggregate
};

__global__ void k_gather_rows(const uint8_t *__restrict__ krec, uint32_t krec_len, const uint64_t *__restrict__ vrec,
                              uint32_t vw, uint32_t key_words, uint32_t naggs, AggMasks am,
                              const uint32_t *__restrict__ idx, uint64_t ns, uint64_t k, uint8_t *__restrict__ out) {
    const uint64_t r = blockIdx.x;
    if (r >= k) return;
    const uint32_t row_words = key_words + 2 * naggs + 2;
    uint32_t *o = reinterpret_cast<uint32_t *>(out) + r * row_words;
    const uint32_t g = idx[r];
    const bool ok = g < ns;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(krec + (uint64_t)g * krec_len);
    const uint32_t *val = reinterpret_cast<const uint32_t *>(vrec + (uint64_t)g * vw);
    for (uint32_t w = threadIdx.x; w < row_words; w += blockDim.x) {
        uint32_t v = 0;
        if (ok) {
            if (w < key_words) v = src[w];
            else if (w < key_words + 2 * naggs) v = val[2 + (w - key_words)] & am.m[w - key_words];
            else v = val[w - key_words - 2 * naggs];
        }
        o[w] = v;
    }
}

// rows kept by `in` (nullable: all) and every predicate of dp -> out (u8; in may be out)
__global__ __launch_bounds__(256) void k_pred_mask(DevPreds dp, const uint8_t *in, uint64_t n, uint8_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        out[i] = (uint8_t)((!in || in[i]) && preds_match_all(dp, i));
}

#include "k_groupby_part.h"

}  // namespace

// ---------------------------------------------------------------------------------------
// host side of the table
// ---------------------------------------------------------------------------------------
struct igx_table {
    igx_ctx *ctx = nullptr;
    uint32_t nkeys = 0;
    uint32_t key_widths[32] = {};
    uint32_t key_words = 0;      // packed words (each column padded to 4 B)
    uint32_t kw_rec = 0;         // key words as the kernel lays them out (static KW or generic width)
    uint32_t koff = 0, krec_len = 0, vrec_len = 0;
    bool generic = false;        // no compile-time layout (or IGX_GB_GENERIC at create)
    igx_agg aggs[AMAX] = {};
    uint32_t naggs = 0;
    uint64_t cap = 0;            // distinct keys promised by the caller
    uint64_t nslots = 0;
    uint32_t sbits = 0;          // log2 nslots
    uint32_t rbits = 0;          // log2 probe-region slots (probing wraps inside a region)
    uint8_t *krec = nullptr;
    uint64_t *vrec = nullptr;
    uint32_t *err = nullptr;
    uint32_t *groups = nullptr;  // occupied slots after finalize
    uint32_t *tile_cnt = nullptr;
    uint32_t *occ = nullptr;     // occupancy bitmap (nslots bits)
    uint8_t *occb = nullptr;     // occupancy byte map (32 x occ_words bytes)
    bool occb_dirty = false;     // cached-form claims since the byte map was last folded / cleared
    uint64_t occ_words = 0;
    uint64_t ep = 0;             // current epoch (1..EP_MAX)
    bool persist = true;         // keys outlive their interval (IGX_GB_PERSIST=0: every reset starts a generation)
    bool fin_since_update = false;   // a finalize listed the groups after the last update
    bool gen_planned = false;    // the reset let the interval continue the generation (device decides by key count)
    bool seed_on = true;         // sample-seeded LDS cache for kept keys (IGX_GB_SEED=0: off)
    igx_table *seed_tab = nullptr;   // the row sample's counting table
    uint32_t *seeds = nullptr;   // seed records (device), nseeds of them
    uint32_t *seed_slots = nullptr;  // the sample table's top-E slots (device)
    uint64_t *seed_gep = nullptr;    // device: the generation the seeds were looked up in
    uint32_t nseeds = 0, seeds_cap = 0;
    uint32_t seed_left = 0;      // seeded intervals before the seeds are recomputed
    bool interval_seeded = false;    // this interval's cached updates adopt the seeds
    uint64_t claims_last = 0;    // the last collected finalize: keys its interval claimed
    uint64_t gen_keys = 0;       // ... and the keys its generation held after it (~0: ended)
    uint64_t *n_groups = nullptr;
    uint64_t rows_fed = 0;       // rows given to update since the last reset
    bool prefer_sm = false;      // the last interval missed the LDS cache on most rows
    bool more_probers = false;   // ... on more than MORE_PROBERS_ON_PM / 1000 of its rows (hysteresis below)
    uint32_t miss_pm = 0;        // LDS misses per 1000 rows of the last measured cached interval
    uint32_t mode = IGX_GB_AUTO; // igx_groupby_set_mode
    uint32_t direct_left = 0;    // AUTO: intervals to run in the direct form before re-measuring
    uint32_t region_off = 0;     // AUTO: intervals to partition exactly after a region overflowed
    bool interval_region = false;   // the interval ran the region variant
    bool interval_direct = false;// the current interval's updates run the direct form
    bool interval_part = false;  // ... the partitioned form
    // partitioned form scratch (grow-only)
    uint32_t *p_recs = nullptr;
    size_t p_recs_bytes = 0;
    uint32_t *p_cnt = nullptr;   // counts / offsets, then scan tile sums, then work items
    size_t p_cnt_bytes = 0;
    uint8_t *p_mask = nullptr;   // row mask of the predicates that are not fused (grow-only)
    size_t p_mask_bytes = 0;
    uint64_t host_groups = 0;
    uint64_t *fin_host = nullptr;   // pinned, coherent: error word, LDS misses, group count (finalize read-back)
    uint64_t *fin_dev = nullptr;    // the same buffer as the kernels address it
    uint64_t fin_seq = 0;           // the last finalize's number (fin_host[3] once it has landed)
    bool fin_pending = false;       // igx_groupby_finalize_async not yet collected
    int fin_status = 0;             // status of a collected asynchronous finalize, not yet returned
    uint64_t fin_status_seq = 0;    // ... and the finalize it belongs to
    // the finalized interval's own bookkeeping, taken when its finalize is issued: the read-back
    // may be collected after the next interval's reset and updates changed the live fields
    struct {
        uint64_t rows_fed;
        bool direct, part, region, probe;
        uint64_t sampled;   // probe: rows the estimator replayed
    } fin_snap{};
    bool interval_probe = false;   // AUTO: the last partitioned interval of a run (k_gb_estimate)
    uint64_t probe_rows = 0;       // ... the rows its estimator replayed
    unsigned long long *dbg_cnt = nullptr;
    // the last top-K's slots per sort (keys + k): the next same top-K's hint (TopkHint)
    struct TkHint {
        uint64_t sig = 0, used = 0;
        uint32_t *slots = nullptr;
        uint32_t nh = 0;
    } tk[4];
    uint32_t *tk_state = nullptr;
    uint64_t tk_clock = 0;
    uint8_t *text[32] = {};      // IP text of the groups, per IGX_TSRC_IPTEXT sort key
    uint64_t text_rows[32] = {};
};

// compile-time key layouts: the reference's BPF key structs + single-column keys
using TcpKey = StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>;   // ip_key_t (tcptop.h:8-17)
using FileKey = StaticLayout<8, 4, 4, 4>;                 // file_id (filetop.h:13-18)
using NetPolicyKey = StaticLayout<4, 1, 4, 2>;            // (src, direction, peer, port)
using BioKey = StaticLayout<8, 4, 4, 4, 4, 16>;           // info_t (biotop.h:24-32)

template <class L>
static bool layout_is(const uint32_t *widths, uint32_t nkeys) {
    if constexpr (L::is_static) {
        if (nkeys != (uint32_t)L::NC) return false;
        for (int c = 0; c < L::NC; ++c)
            if ((int)widths[c] != L::Ws[c]) return false;
        return true;
    }
    return false;
}

static const int kInst[] = {2, 4, 6, 8, 12, 18, 24, 32};

// key words the kernel will use for this key description (0 = generic)
static int static_kw(const uint32_t *w, uint32_t n) {
    if (std::getenv("IGX_GB_GENERIC")) return 0;   // diagnostics
    if (layout_is<TcpKey>(w, n)) return TcpKey::KW;
    if (layout_is<FileKey>(w, n)) return FileKey::KW;
    if (layout_is<NetPolicyKey>(w, n)) return NetPolicyKey::KW;
    if (layout_is<BioKey>(w, n)) return BioKey::KW;
    if (n == 1 && (w[0] == 1 || w[0] == 2 || w[0] == 4 || w[0] == 8 || w[0] == 16)) return (int)((w[0] + 3) / 4);
    return 0;
}

extern "C" int igx_groupby_create(igx_ctx *ctx, const uint32_t *key_widths, uint32_t nkeys, const igx_agg *aggs,
                                  uint32_t naggs, uint64_t capacity, igx_table **out) {
    if (!ctx || !out || !key_widths || nkeys == 0 || nkeys > 16)
        return igx_fail(ctx, IGX_EINVAL, "groupby_create: bad key description");
    if (naggs > AMAX) return igx_fail(ctx, IGX_ENOTSUP, "groupby_create: more than %d aggregates", AMAX);
    for (uint32_t x = 0; x < naggs; ++x) {
        const uint32_t ow = aggs[x].out_width;
        if (ow != 0 && ow != 1 && ow != 2 && ow != 4 && ow != 8)
            return igx_fail(ctx, IGX_EINVAL, "groupby_create: aggregate %u out_width %u", x, ow);
        if (aggs[x].kind != IGX_AGG_COUNT && aggs[x].kind != IGX_AGG_SUM)
            return igx_fail(ctx, IGX_EINVAL, "groupby_create: aggregate %u kind %u", x, aggs[x].kind);
    }
    if (capacity == 0 || capacity > (1ull << 28)) return igx_fail(ctx, IGX_EINVAL, "groupby_create: bad capacity");
    uint32_t words = 0;
    for (uint32_t i = 0; i < nkeys; ++i) {
        const uint32_t w = key_widths[i];
        if (w == 0) return igx_fail(ctx, IGX_EINVAL, "groupby: key width 0");
        words += (w + 3) / 4;
    }
    if (words > KWMAX) return igx_fail(ctx, IGX_ENOTSUP, "groupby: key wider than %d bytes", KWMAX * 4);
    auto *t = new igx_table();
    t->ctx = ctx;
    t->nkeys = nkeys;
    for (uint32_t i = 0; i < nkeys; ++i) t->key_widths[i] = key_widths[i];
    t->key_words = words;
    const int skw = static_kw(key_widths, nkeys);
    t->generic = skw == 0;
    if (skw) {
        t->kw_rec = (uint32_t)skw;
    } else {
        for (int k : kInst)
            if ((uint32_t)k >= words) {
                t->kw_rec = (uint32_t)k;
                break;
            }
    }
    t->koff = koff_of((int)t->kw_rec);
    t->krec_len = krec_bytes((int)t->kw_rec);
    if (const char *d = std::getenv("IGX_GB_KR16"))   // tuning knob: 16-B rounded key records
        if (std::strtoul(d, nullptr, 0)) t->krec_len = (uint32_t)igx_align(t->koff + 16, 16);
    t->vrec_len = vrec_bytes(naggs);
    t->naggs = naggs;
    for (uint32_t i = 0; i < naggs; ++i) t->aggs[i] = aggs[i];
    t->cap = capacity;
    // S >= slotf/4 x capacity (default 2x); a smaller table stays resident in the Infinity Cache
    uint64_t slotf = 8;
    if (const char *d = std::getenv("IGX_GB_SLOTF")) slotf = std::max<uint64_t>(5, std::strtoul(d, nullptr, 0));
    uint64_t ns = 1024;
    while (ns * 4 < slotf * capacity) ns <<= 1;
    t->nslots = ns;
    t->sbits = (uint32_t)__builtin_ctzll(ns);
    // probe regions of max(1024, S / 16384) slots: up to 16K regions, so a bucket of the
    // partitioned form can own whole regions
    t->rbits = std::max<uint32_t>(10, t->sbits > 14 ? t->sbits - 14 : 0);
    if (ns * t->krec_len >= (1ull << 32)) {
        const uint32_t r = t->krec_len;
        delete t;
        return igx_fail(ctx, IGX_ENOTSUP, "groupby_create: table of %llu x %u B exceeds 4 GiB",
                        (unsigned long long)ns, r);
    }
    const uint64_t tiles = (ns + CT - 1) / CT;
    hipError_t e = hipMalloc(&t->krec, ns * t->krec_len);
    if (e == hipSuccess) e = hipMemsetAsync(t->krec, 0, ns * t->krec_len, ctx->stream);
    if (e == hipSuccess) e = hipMalloc(&t->vrec, ns * t->vrec_len);
    if (e == hipSuccess) e = hipMalloc(&t->err, 64);
    if (e == hipSuccess) e = hipMemsetAsync(t->err, 0, 64, ctx->stream);
    if (e == hipSuccess) e = hipMalloc(&t->groups, ns * 4);
    if (e == hipSuccess) e = hipMalloc(&t->tile_cnt, tiles * 4);
    t->occ_words = (ns + 31) / 32;
    if (e == hipSuccess) e = hipMalloc(&t->occ, t->occ_words * 4);
    if (e == hipSuccess) e = hipMalloc(&t->occb, t->occ_words * 32);
    if (e == hipSuccess) e = hipMemsetAsync(t->occb, 0, t->occ_words * 32, ctx->stream);
    if (e == hipSuccess) t->n_groups = reinterpret_cast<uint64_t *>(t->err + 4);   // behind the error block
    if (e == hipSuccess) e = hipMalloc(&t->dbg_cnt, 256);
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void **>(&t->fin_host), 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&t->fin_dev), t->fin_host, 0);
    if (e == hipSuccess) std::fill(t->fin_host, t->fin_host + 8, 0ull);
    if (e == hipSuccess) e = hipMemsetAsync(t->dbg_cnt, 0, 256, ctx->stream);
    if (e != hipSuccess) {
        igx_groupby_destroy(t);
        return igx_fail(ctx, IGX_ENOMEM, "groupby_create: %s", hipGetErrorString(e));
    }
    // tuning / A-B knob (tools/gpu/ab_modes.sh): the initial mode, as igx_groupby_set_mode
    if (const char *m = std::getenv("IGX_GB_MODE")) {
        const unsigned long v = std::strtoul(m, nullptr, 0);
        if (v <= IGX_GB_PART) t->mode = (uint32_t)v;
    }
    if (const char *m = std::getenv("IGX_GB_PERSIST")) t->persist = std::strtoul(m, nullptr, 0) != 0;   // A/B knob
    if (const char *m = std::getenv("IGX_GB_SEED")) t->seed_on = std::strtoul(m, nullptr, 0) != 0;       // A/B knob
    *out = t;
    return igx_groupby_reset(t);
}

static int fin_collect(igx_table *t, uint64_t *n_groups);
static bool fin_landed(const igx_table *t) {
    return __atomic_load_n(t->fin_host + 3, __ATOMIC_ACQUIRE) == t->fin_seq;
}

extern "C" int igx_groupby_reset(igx_table *t) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    // an asynchronous finalize whose read-back has landed is collected now (its AUTO
    // bookkeeping then steers this interval); one still in flight is collected by a later
    // call, so a reset never waits for the device.  A collected error is returned after the
    // reset is done.
    if (t->fin_pending && fin_landed(t)) (void)fin_collect(t, nullptr);
    const int pending_rc = t->fin_status;
    t->fin_status = IGX_OK;
    // A new interval is a new epoch: records of older epochs read as empty and a claimer
    // initialises its value record, so only the bitmap and the error word are cleared.
    bool wrapped = false;
    if (++t->ep > EP_MAX) {
        hipLaunchKernelGGL(k_table_clear, dim3(2048), dim3(256), 0, ctx->stream, t->krec, t->krec_len, t->koff,
                           t->nslots);
        IGX_HIP(ctx, hipGetLastError());
        t->ep = 1;
        wrapped = true;
    }
    // The generation goes on (the device checks its key count) when the last interval's groups
    // were listed by a finalize after its last update and this interval is planned in the cached
    // form (the direct and partitioned forms start their own: k_gen_restart if the plan changes).
    ResetGen rg{};
    rg.gen = reinterpret_cast<uint64_t *>(t->err) + GEN_WORD;
    rg.ep = t->ep;
    // the most keys a generation may hold after an interval: 4/5 of the slots (a 1 024-slot probe
    // region then overflows only past 7 standard deviations of its expected fill)
    const uint64_t fill = t->nslots / 5 * 4;
    rg.limit = fill > t->cap ? fill - t->cap : 0;
    rg.groups = t->groups;
    rg.ng = t->n_groups;
    rg.vrec = t->vrec;
    rg.vw = t->vrec_len / 8;
    const bool planned_cached = !(t->mode == IGX_GB_DIRECT || t->mode == IGX_GB_PART ||
                                  (t->mode == IGX_GB_AUTO && t->direct_left > 0));
    rg.may = t->persist && !wrapped && t->fin_since_update && rg.limit > 0 && planned_cached ? 1u : 0u;
    t->gen_planned = rg.may != 0;
    // the bitmap, the error bits and the LDS-miss count (and the byte map if it holds claims)
    const uint64_t nb16 = t->occb_dirty ? t->occ_words * 2 : 0;
    const uint64_t grid = rg.may ? 2048 : std::min<uint64_t>(1024, (std::max(t->occ_words / 4, nb16) + 255) / 256 + 1);
    hipLaunchKernelGGL(k_reset_clear, dim3((unsigned)grid), dim3(256), 0, ctx->stream, t->occ, t->occ_words, t->err,
                       reinterpret_cast<uint4 *>(t->occb), nb16, rg);
    t->occb_dirty = false;
    IGX_HIP(ctx, hipGetLastError());
    t->rows_fed = 0;
    t->host_groups = 0;
    return pending_rc;
}

extern "C" int igx_groupby_destroy(igx_table *t) {
    if (!t) return IGX_OK;
    (void)hipStreamSynchronize(t->ctx->stream);
    (void)hipFree(t->krec);
    (void)hipFree(t->vrec);
    (void)hipFree(t->err);
    (void)hipFree(t->groups);
    (void)hipFree(t->tile_cnt);
    (void)hipFree(t->occ);
    (void)hipFree(t->occb);
    (void)hipFree(t->dbg_cnt);
    (void)hipFree(t->seeds);
    (void)hipFree(t->seed_slots);
    (void)hipFree(t->seed_gep);
    if (t->seed_tab) igx_groupby_destroy(t->seed_tab);
    (void)hipFree(t->p_recs);
    (void)hipFree(t->p_cnt);
    (void)hipFree(t->p_mask);
    for (auto &h : t->tk) (void)hipFree(h.slots);
    (void)hipFree(t->tk_state);
    for (auto *p : t->text) (void)hipFree(p);
    if (t->fin_host) (void)hipHostFree(t->fin_host);
    delete t;
    return IGX_OK;
}

constexpr size_t GB_LDS_TOTAL = 156 * 1024;    // cache + the two rings (dynamic LDS)
constexpr uint64_t DIRECT_MISS_PCT = 90;        // AUTO: LDS-miss share that selects the partitioned form
// LDS-miss share (per mille of rows) above which a loader wave becomes a prober, and below
// which it turns back: a band, so a stream near the threshold does not flip the roles every
// interval.  Measured: C5 (~42 % misses) 6.15 -> 5.95-6.02 ms with 7 loaders,
// C2 (~35 %) 3.69 -> 3.86 ms, so C2 keeps 8 -- the band sits between the two.
constexpr uint64_t MORE_PROBERS_ON_PM = 390;
constexpr uint64_t MORE_PROBERS_OFF_PM = 370;
constexpr uint32_t DIRECT_RUN = 16;             // ... for this many intervals

// the cached kernel's LDS cache entries (E) for naggs aggregates in its NA-slot variant
template <class L, int NA>
static uint32_t gb_entries(uint32_t naggs) {
    const size_t entry = 4 + 4 + 8 + 8 * naggs + 4 * LdsCache<L::KW>::KP;
    const size_t rings = ARING * 16 + MRING * (16 * MissRing<L::KW, NA>::EQ + 4) + GHOST * 4;
    const size_t budget = GB_LDS_TOTAL - rings;
    return 8 * (uint32_t)std::max<size_t>(1, std::min<size_t>(1024, budget / (8 * entry)));
}
template <class L>
static uint32_t gb_entries_for(uint32_t naggs) {
    return naggs <= 2 ? gb_entries<L, 2>(naggs) : gb_entries<L, AMAX>(naggs);
}

template <class L, bool DBG, int NA, bool SAMPLE = false>
static void launch_gb_as(igx_ctx *ctx, GbArgs &a, uint32_t blocks) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_groupby<L, DBG, NA, SAMPLE>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, GB_LDS_TOTAL);
        attr = true;
    }
    const size_t entry = 4 + 4 + 8 + 8 * a.naggs + 4 * LdsCache<L::KW>::KP;
    const size_t rings = ARING * 16 + MRING * (16 * MissRing<L::KW, NA>::EQ + 4) + GHOST * 4;
    const uint32_t E = gb_entries<L, NA>(a.naggs);
    a.lds_entries = E;
    const size_t lds = E * entry + rings;
    hipLaunchKernelGGL((k_groupby<L, DBG, NA, SAMPLE>), dim3(blocks), dim3(GTB), lds, ctx->stream, a);
}

// k_gb_estimate with the cached kernel's geometry (its E and its GHOST filter)
constexpr uint64_t PROBE_ROWS = 16u << 20;   // rows the re-probe replays (C4: 16M of 125M)
template <class L, int NA>
static void launch_estimate_as(igx_ctx *ctx, GbArgs a, uint32_t blocks, uint64_t nsample) {
    const size_t entry = 4 + 4 + 8 + 8 * a.naggs + 4 * LdsCache<L::KW>::KP;
    const size_t rings = ARING * 16 + MRING * (16 * MissRing<L::KW, NA>::EQ + 4) + GHOST * 4;
    const uint32_t nsets = (uint32_t)std::max<size_t>(1, std::min<size_t>(1024, (GB_LDS_TOTAL - rings) / (8 * entry)));
    a.lds_entries = 8 * nsets;
    a.admit_mask = std::max<uint32_t>(a.admit_mask, 1u);
    const size_t lds = ((size_t)a.lds_entries + GHOST) * 4;
    hipLaunchKernelGGL((k_gb_estimate<L, NA>), dim3(blocks), dim3(GTB), lds, ctx->stream, a, nsample);
}
template <class L>
static void launch_estimate(igx_ctx *ctx, const GbArgs &a, uint32_t blocks, uint64_t nsample) {
    if (a.naggs <= 2) launch_estimate_as<L, 2>(ctx, a, blocks, nsample);
    else launch_estimate_as<L, AMAX>(ctx, a, blocks, nsample);
}

// The diagnostic variants (IGX_GB_DEBUG) are compiled for the top-tcp key only, so the
// production kernels carry none of their code.  Tables with at most two aggregates run a
// kernel that carries two aggregate slots (fewer registers, fewer loads).
template <class L>
static void launch_gb(igx_ctx *ctx, GbArgs &a, uint32_t blocks) {
    if constexpr (std::is_same<L, StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>>::value) {
        if (a.dbg) {
            launch_gb_as<L, true, 2>(ctx, a, blocks);
            return;
        }
    }
#ifdef IGX_GB_DEBUG_FILE
    if constexpr (std::is_same<L, StaticLayout<8, 4, 4, 4>>::value) {
        if (a.dbg) {
            launch_gb_as<L, true, AMAX>(ctx, a, blocks);
            return;
        }
    }
#endif
    if (a.naggs <= 2) launch_gb_as<L, false, 2>(ctx, a, blocks);
    else launch_gb_as<L, false, AMAX>(ctx, a, blocks);
}

// The grid is exactly the blocks that are resident at once (the occupancy the kernel's
// registers allow): every block sweeps a fixed share of the rows, so a block that had to wait
// for a free slot would run its whole share after the others -- a tail of up to 1/8 of the time.
template <class L, int NA>
static void launch_direct_as(igx_ctx *ctx, GbArgs &a) {
    static int per_cu = 0;
    if (!per_cu) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void *>(k_groupby_direct<L, NA>),
                                                         256, 0) != hipSuccess || b < 1)
            b = 4;
        per_cu = std::min(b, 8);
    }
    const uint64_t want = (a.n + 255) / 256;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ctx->num_cus * per_cu));
    hipLaunchKernelGGL((k_groupby_direct<L, NA>), dim3(blocks), dim3(256), 0, ctx->stream, a);
}

template <class L>
static void launch_direct(igx_ctx *ctx, GbArgs &a) {
    if (a.naggs <= 2) launch_direct_as<L, 2>(ctx, a);
    else launch_direct_as<L, AMAX>(ctx, a);
}

static int grow(igx_ctx *ctx, void **p, size_t *have, size_t need) {
    if (*have >= need) return IGX_OK;
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));   // the old buffer may still be in use
    (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    IGX_HIP(ctx, hipMalloc(p, need));
    *have = need;
    return IGX_OK;
}

// The partitioned form (k_groupby_part.h): passes K, O, S, A, B, C -- or, in the region
// variant (AUTO's miss-heavy intervals), A, T, B, I, C: no count pass, buckets filled through
// cursors into regions of 1.25x their share of the rows.
template <class L, int NV>
static int launch_part_as(igx_table *t, igx_ctx *ctx, GbArgs &a, PartArgs &p, bool region) {
    constexpr int KW = L::KW;
    constexpr uint32_t TRA = PTA * part_rows<KW, NV>();
    if (4 * p.rq > (uint32_t)part_w<KW, NV>()) return igx_fail(ctx, IGX_EINVAL, "groupby_update: record layout");
    // final buckets: enough that a bucket's share of the capacity fills at most ~60% of the
    // C block's LDS table; each bucket owns whole probe regions of the table
    // pass C's packed entries (c_row_pe): distinct-only, a static key of <= 3 packed words,
    // row-offset indices; IGX_GBP_NOPE=1 keeps the general table (A/B)
    p.pe = pack_words<L>() <= 3 && t->naggs == 0 && p.iw == 1 &&
           !std::getenv("IGX_GBP_COMBINE") && !std::getenv("IGX_GBP_NOPE");
    const size_t entry = p.pe ? 17 : agg_entry_bytes(KW, t->naggs);
    p.uc = p.rq <= 1 ? 2 : 1;
    if (const char *d = std::getenv("IGX_GBP_UC"))   // tuning knob: records per thread and round of pass C
        p.uc = std::max<uint32_t>(1, std::min<uint32_t>(UCMAX, (uint32_t)std::strtoul(d, nullptr, 0)));
    const size_t stage_c = (size_t)p.uc * PTC * p.rq * 16;
    const uint32_t lb_max = std::min<uint32_t>(PART_LB_MAX, t->sbits - t->rbits);
    auto entries = [&](uint32_t lb, size_t esz) {
        const int64_t occw = (int64_t)1 << (t->sbits - lb - 5);
        const int64_t room = (int64_t)PART_AGG_LDS - (int64_t)stage_c - 8 * occw - 16;
        if (room < (int64_t)(8 * esz)) return 0u;
        // whole 8-way sets, E a multiple of 16: the byte tags keep what follows them 16-B aligned
        return (uint32_t)std::min<int64_t>(65520, room / (int64_t)esz) & ~15u;
    };
    // the bucket count follows the general entry size, so packed entries only lower the load
    // factor (IGX_GBP_PE_LB=1: let them halve the bucket count instead)
    const size_t lb_entry = std::getenv("IGX_GBP_PE_LB") ? entry : agg_entry_bytes(KW, t->naggs);
    uint32_t lb = 0;
    while (lb < lb_max && (double)(t->cap >> lb) > 0.9 * entries(lb, lb_entry)) ++lb;
    p.lb = lb;
    p.f1 = (lb + 1) / 2;
    if (const char *d = std::getenv("IGX_GBP_F1"))   // tuning knob: first-level bucket bits
        p.f1 = std::min<uint32_t>(std::min<uint32_t>(lb, 8u), (uint32_t)std::strtoul(d, nullptr, 0));
    p.f1 = std::max<uint32_t>(p.f1, lb > 8 ? lb - 8 : 0u);   // both levels <= 256 buckets
    p.f2 = lb - p.f1;
    p.sb_log = t->sbits - lb;
    p.occw = 1u << (p.sb_log - 5);
    p.E = entries(lb, entry);
    if (p.E < 16) return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: key of %u words too wide for the partitioned form", KW);
    if (const char *d = std::getenv("IGX_GBP_ENTRIES"))   // tests: a small LDS table overflows
        p.E = std::max<uint32_t>(16, std::min<uint32_t>(p.E, (uint32_t)std::strtoul(d, nullptr, 0))) & ~15u;
    p.maxp = std::min<uint32_t>(p.E / 8, 32);   // sets probed before a row takes the HBM path
    p.combine = 0;   // wave pre-combine: measured slower on C4 and C5
    if (const char *d = std::getenv("IGX_GBP_COMBINE")) p.combine = (uint32_t)std::strtoul(d, nullptr, 0);
    if (const char *d = std::getenv("IGX_GBP_DEBUG")) p.dbg = (uint32_t)std::strtoul(d, nullptr, 0);
    const uint32_t F1 = 1u << p.f1, F2 = 1u << p.f2, NB = 1u << lb;
    // B tiles: as many records (a multiple of PTA, at most 4096) as the tile LDS holds
    uint32_t trb = 4096;
    // (sized for the LDS-order path; the register path then stages 17 B per record in
    // ~52 KB, three blocks per CU: 4 096-record tiles measured 1.06 ms against 0.89 on C4)
    while (trb > PTA && (size_t)trb * (16 * p.rq + 6) + 12 * PART_F_MAX + 72 > PART_TILE_LDS) trb -= PTA;
    if (const char *d = std::getenv("IGX_GBP_TRB"))   // tuning knob: records per B tile (a multiple of PTA)
        trb = std::max<uint32_t>(PTA, std::min<uint32_t>(trb, (uint32_t)std::strtoul(d, nullptr, 0) / PTA * PTA));
    p.trb = trb;
    p.ch = (uint32_t)std::max<uint64_t>(8192, 4 * (a.n / NB + 1));
    p.tiles_a = (uint32_t)((a.n + TRA - 1) / TRA);
    p.nchunk = (p.tiles_a + CHT - 1) / CHT;
    const uint32_t S1 = region ? 1u << PART_S1_LOG : 1u, U1 = F1 * S1;   // first-level runs (slices)
    const uint64_t tiles_b = a.n / trb + U1 + 1;
    uint32_t c2pad = 16;   // final-region cursors one 64-B line apart (pass B's atomics)
    if (const char *d = std::getenv("IGX_GBP_C2PAD")) c2pad = std::max<uint32_t>(1, (uint32_t)std::strtoul(d, nullptr, 0));
    const uint64_t items_max = NB + a.n / p.ch + 1;
    uint64_t r1 = a.n * 5 / 4 / U1 + TRA, r2 = a.n * 5 / 4 / NB + 1024;   // region records
    if (const char *d = std::getenv("IGX_GBP_REGSIZE"))   // tests: small regions overflow
        r1 = r2 = std::max<uint64_t>(1, std::strtoull(d, nullptr, 0));
    if (region && (r1 * U1 >= (1ull << 31) || r2 * NB >= (1ull << 31))) region = false;
    if (region) {
        p.reg1 = (uint32_t)r1;
        p.reg2 = (uint32_t)r2;
        p.s1log = PART_S1_LOG;
        p.c2pad = c2pad;
        // scratch: rc1 | rc2 | tstart | bt | istart | itfb | ctl (u32 words)
        const uint64_t words = U1 * RC1_PAD + NB * c2pad + (U1 + 1) + tiles_b + (NB + 1) + items_max + 4;
        int rc = grow(ctx, reinterpret_cast<void **>(&t->p_cnt), &t->p_cnt_bytes, 4 * words);
        if (!rc) rc = grow(ctx, reinterpret_cast<void **>(&t->p_recs), &t->p_recs_bytes,
                           (size_t)16 * p.rq * (r1 * U1 + r2 * NB));
        if (rc) return rc;
        p.rc1 = t->p_cnt;
        p.rc2 = p.rc1 + U1 * RC1_PAD;
        p.tstart = p.rc2 + NB * c2pad;
        p.bt = p.tstart + U1 + 1;
        p.istart = p.bt + tiles_b;
        p.itfb = p.istart + NB + 1;
        p.ctl = p.itfb + items_max;
        p.recs1 = t->p_recs;
        p.recs2 = t->p_recs + r1 * U1 * p.rq * 4;
    }
    // scratch: cnt1 | csum | hist | start2 | cur2 | tstart | bt | istart | itfb | ctl (u32 words)
    const uint64_t w_cnt1 = (uint64_t)p.tiles_a * F1, w_csum = (uint64_t)p.nchunk * F1;
    const uint64_t words = w_cnt1 + w_csum + NB + (NB + 1) + NB + (F1 + 1) + tiles_b + (NB + 1) + items_max + 4;
    int rc = region ? IGX_OK : grow(ctx, reinterpret_cast<void **>(&t->p_cnt), &t->p_cnt_bytes, 4 * words);
    const size_t rec_bytes = (size_t)16 * p.rq;
    if (!rc && !region) rc = grow(ctx, reinterpret_cast<void **>(&t->p_recs), &t->p_recs_bytes, 2 * rec_bytes * a.n);
    if (rc) return rc;
    if (!region) {
    p.cnt1 = t->p_cnt;
    p.csum = p.cnt1 + w_cnt1;
    p.hist = p.csum + w_csum;
    p.start2 = p.hist + NB;
    p.cur2 = p.start2 + NB + 1;
    p.tstart = p.cur2 + NB;
    p.bt = p.tstart + F1 + 1;
    p.istart = p.bt + tiles_b;
    p.itfb = p.istart + NB + 1;
    p.ctl = p.itfb + items_max;
    p.recs1 = t->p_recs;
    p.recs2 = t->p_recs + (uint64_t)a.n * p.rq * 4;
    }
    const size_t lds_k = 4 * ((size_t)NB + F1);
    const size_t lds_a = (size_t)TRA * (16 * p.rq + 1) + 12 * (size_t)F1 + 4 * 17;
    const size_t lds_b = PackKey<L>::known && L::KW <= 8 && gbp_b_regs(p) ? (size_t)trb * (16 * p.rq + 1) + 12 * (size_t)F2 + 4 * 17
                                                            : (size_t)trb * (16 * p.rq + 6) + 12 * (size_t)F2 + 4 * 17;
    const size_t lds_c = (size_t)p.E * entry + 8 * (size_t)p.occw + 16 + stage_c;
    // dynamic LDS granted to each kernel so far; pass C has a distinct-only instantiation
    constexpr bool PEK = pack_words<L>() <= 3;   // a packed-entry pass C exists for this layout
    static size_t lds_set[6] = {0, 0, 0, 0, 0, 0};
    const void *kern[6] = {reinterpret_cast<const void *>(k_gbp_count<L, NV>),
                           reinterpret_cast<const void *>(k_gbp_a<L, NV>),
                           reinterpret_cast<const void *>(k_gbp_b<L, NV>),
                           reinterpret_cast<const void *>(k_gbp_c<L, NV, AMAX>),
                           reinterpret_cast<const void *>(k_gbp_c<L, NV, 0>),
                           reinterpret_cast<const void *>(k_gbp_c<L, NV, 0, PEK>)};
    const bool pe_c = PEK && p.pe;
    const size_t need[6] = {lds_k, lds_a, lds_b, t->naggs ? lds_c : 0, t->naggs || pe_c ? 0 : lds_c, pe_c ? lds_c : 0};
    for (int i = 0; i < 6; ++i) {
        if (need[i] > lds_set[i]) {
            IGX_HIP(ctx, hipFuncSetAttribute(kern[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)need[i]));
            lds_set[i] = need[i];
        }
    }
    const uint32_t cus = (uint32_t)ctx->num_cus;
    if (region) {
        IGX_HIP(ctx, hipMemsetAsync(p.rc1, 0, 4ull * (U1 * RC1_PAD + NB * p.c2pad), ctx->stream));
        hipLaunchKernelGGL((k_gbp_a<L, NV>), dim3(p.tiles_a), dim3(PTA), lds_a, ctx->stream, a, p);
        if (p.dbg & 256u) return IGX_OK;   // diagnostics: stop after pass A (the table is left unset)
        hipLaunchKernelGGL(k_gbr_tiles, dim3(1), dim3(1024), 0, ctx->stream, p);
        hipLaunchKernelGGL((k_gbp_b<L, NV>), dim3((unsigned)tiles_b), dim3(PTA), lds_b, ctx->stream, a, p);
        if (p.dbg & 512u) return IGX_OK;   // ... after pass B
        hipLaunchKernelGGL(k_gbr_items, dim3(1), dim3(1024), 0, ctx->stream, p);
    }
    if (!region) {
    IGX_HIP(ctx, hipMemsetAsync(p.hist, 0, 4ull * NB, ctx->stream));
    hipLaunchKernelGGL((k_gbp_count<L, NV>), dim3(std::min<uint32_t>(p.tiles_a, 2 * cus)), dim3(PTA), lds_k,
                       ctx->stream, a, p);
    hipLaunchKernelGGL(k_gbp_csum, dim3(p.nchunk), dim3(PTA), 0, ctx->stream, p);
    hipLaunchKernelGGL(k_gbp_scan, dim3(1), dim3(1024), 0, ctx->stream, p);
    hipLaunchKernelGGL(k_gbp_offs, dim3(p.nchunk), dim3(PTA), 0, ctx->stream, p);
    if (p.dbg & 1024u) return IGX_OK;   // diagnostics: stop after the count and the scans
    hipLaunchKernelGGL((k_gbp_a<L, NV>), dim3(p.tiles_a), dim3(PTA), lds_a, ctx->stream, a, p);
    if (p.dbg & 256u) return IGX_OK;   // diagnostics: stop after pass A (the table is left unset)
    hipLaunchKernelGGL((k_gbp_b<L, NV>), dim3((unsigned)tiles_b), dim3(PTA), lds_b, ctx->stream, a, p);
    if (p.dbg & 512u) return IGX_OK;   // ... after pass B
    }
    if (t->naggs)
        hipLaunchKernelGGL((k_gbp_c<L, NV, AMAX>), dim3(2 * cus), dim3(PTC), lds_c, ctx->stream, a, p);
    else if (pe_c)   // distinct-only with packed entries (C4)
        hipLaunchKernelGGL((k_gbp_c<L, NV, 0, PEK>), dim3(2 * cus), dim3(PTC), lds_c, ctx->stream, a, p);
    else   // distinct-only: no aggregate decode or accumulate in the per-record path
        hipLaunchKernelGGL((k_gbp_c<L, NV, 0>), dim3(2 * cus), dim3(PTC), lds_c, ctx->stream, a, p);
    return IGX_OK;
}

// record layout and the loaded columns; predicates become a row mask first
template <class L>
static int launch_part(igx_table *t, igx_ctx *ctx, GbArgs &a) {
    PartArgs p{};
    // packed key words: 1- and 2-byte columns share words, other columns keep theirs
    uint32_t wp = 0, used = 4, shared = 0, w = 0;
    for (uint32_t c = 0; c < t->nkeys; ++c) {
        const uint32_t cw = t->key_widths[c];
        if (cw <= 2) {
            if (used + cw > 4) {
                shared = wp++;
                used = 0;
            }
            p.kpw[w] = shared;
            p.ksh[w] = 8 * used;
            p.kmsk[w] = cw == 1 ? 0xFFu : 0xFFFFu;
            used += cw;
            ++w;
        } else {
            for (uint32_t j = 0; j < (cw + 3) / 4; ++j, ++w) {
                p.kpw[w] = wp++;
                p.ksh[w] = 0;
                p.kmsk[w] = 0xFFFFFFFFu;
            }
        }
    }
    if (w != t->key_words) return igx_fail(ctx, IGX_EINVAL, "groupby_update: internal key packing mismatch");
    p.kpn = wp;
    // each distinct value / condition column once
    uint32_t nv = 0;
    auto col_of = [&](const uint8_t *ptr, uint32_t width) {
        for (uint32_t j = 0; j < nv; ++j)
            if (p.vcol[j] == ptr && p.vcw[j] == width) return j;
        p.vcol[nv] = ptr;
        p.vcw[nv] = width;
        p.vchi[nv] = width == 8 ? 4 : 0;
        return nv++;
    };
    for (uint32_t x = 0; x < AMAX; ++x) {
        p.vsrc[x] = p.csrc[x] = PNV;
        if (x >= t->naggs) continue;
        if (!a.vcount[x]) p.vsrc[x] = col_of(a.vptr[x], a.vwidth[x]);
        if (a.hascond[x]) p.csrc[x] = col_of(a.cptr[x], a.cwidth[x]);
    }
    for (uint32_t j = 0; j < nv; ++j) {
        p.rpos[j] = wp;
        p.rw2[j] = p.vcw[j] == 8;
        wp += 1 + p.rw2[j];
    }
    p.nv = nv;
    for (uint32_t x = 0; x < AMAX; ++x) {
        p.avp[x] = p.vsrc[x] < PNV ? p.rpos[p.vsrc[x]] : 0xFFFFu;
        p.av2[x] = p.vsrc[x] < PNV ? p.rw2[p.vsrc[x]] : 0u;
        p.acp[x] = p.csrc[x] < PNV ? p.rpos[p.csrc[x]] : 0xFFFFu;
        p.ac2[x] = p.csrc[x] < PNV ? p.rw2[p.csrc[x]] : 0u;
    }
    for (uint32_t j = nv; j < PNV; ++j) {   // unused: dword 0 of a readable column
        p.vcol[j] = a.kcol[0];
        p.vcw[j] = 0;
        p.vchi[j] = 0;
        p.rpos[j] = 0;
        p.rw2[j] = 0;
    }
    p.iw = a.fidx ? 2 : 1;
    p.ipos = wp;
    wp += p.iw;
    p.rq = (wp + 3) / 4;
    p.rq_magic = p.rq > 1 ? (uint32_t)((0x100000000ull + p.rq - 1) / p.rq) : 0u;
    if (a.npred) {
        int rc = grow(ctx, reinterpret_cast<void **>(&t->p_mask), &t->p_mask_bytes, igx_align(a.n, 256));
        if (rc) return rc;
        hipLaunchKernelGGL(k_gbp_mask, dim3((unsigned)std::min<uint64_t>(4096, (a.n + 255) / 256)), dim3(256), 0,
                           ctx->stream, a, t->p_mask);
        a.valid = a.validp = t->p_mask;
        a.validw = 1;
        a.npred = 0;
    }
    // AUTO's miss-heavy intervals run the region variant (no count pass); IGX_GB_PART keeps
    // exact runs, whose split work items also take heavily skewed streams in stride
    // The region variant sizes each bucket's region at 1.25x its share of the rows; a bucket
    // past it merges its extra records into the table directly (exact; a wave's spilled
    // records are pre-combined per key first, region_spill).  An interval that overflowed a
    // region switches AUTO to the exact variant for the rest of the partitioned run.
    const bool region = (t->mode == IGX_GB_AUTO || std::getenv("IGX_GBP_REGION")) && !std::getenv("IGX_GBP_EXACT") &&
                        t->region_off == 0;
    t->interval_region = t->interval_region || region;
    if (nv == 0) return launch_part_as<L, 0>(t, ctx, a, p, region);
    if (nv <= 2) return launch_part_as<L, 2>(t, ctx, a, p, region);
    return launch_part_as<L, PNV>(t, ctx, a, p, region);
}

// The sample-seeded LDS cache (tools/cache_sim.py: C2 33.7 -> 31.2 % misses, C5 45.4
// -> 42.6 %, against 30.7 / 42.2 % for an ideal top-E cache).  The first SEED_SAMPLE rows of the
// interval's first update are counted by key in a scratch table (the cached kernel with one COUNT
// aggregate, as its SAMPLE instance: profiles keep its launches apart; the direct form took
// 2.7-3.1 ms for these 1.5M rows -- a sample's hot keys queue on one record's atomics), its top-E
// groups by count are selected on the device (igx_groupby_sort),
// and k_gb_seeds looks each of them up in the table's current generation.  Every workgroup of the
// interval's cached updates adopts the found ones before its stream starts.  Hot keys of a
// stream are stable, so the seeds are recomputed every SEED_EVERY seeded intervals (and after a
// generation ended); seeds of another generation are never adopted (the kernel compares).
constexpr uint32_t SEED_EVERY = 16;   // round 6: 8 -> 16 and rows / 64 -> rows / 128 (profiles/r06/seed_period_ab.txt)
constexpr uint64_t SEED_MIN_ROWS = 8u << 20;    // smaller updates: no seeds (IGX_GB_SEED_MIN overrides)
constexpr uint64_t SEED_SAMPLE = 1u << 20;      // sampled rows: max(1M, rows / SEED_DIV)
constexpr uint64_t SEED_DIV = 128;

template <class L>
static int seeds_compute_static(igx_table *t, igx_ctx *ctx, const GbArgs &a) {
    const uint32_t E = gb_entries_for<L>(t->naggs);
    uint64_t div = SEED_DIV;
    if (const char *d = std::getenv("IGX_GB_SEED_DIV")) div = std::max<uint64_t>(1, std::strtoull(d, nullptr, 0));   // A/B knob
    const uint64_t S = std::min<uint64_t>(a.n, std::max<uint64_t>(SEED_SAMPLE, a.n / div));
    if (t->seed_tab && t->seed_tab->cap < S) {
        igx_groupby_destroy(t->seed_tab);
        t->seed_tab = nullptr;
    }
    if (!t->seed_tab) {
        igx_agg cnt{};
        cnt.kind = IGX_AGG_COUNT;
        cnt.col = IGX_NO_COL;
        cnt.cond_col = IGX_NO_COL;
        cnt.out_width = 8;
        igx_table *st = nullptr;
        int rc = igx_groupby_create(ctx, t->key_widths, t->nkeys, &cnt, 1, std::max<uint64_t>(S, 4ull * E), &st);
        if (rc) return rc;
        st->persist = false;
        st->seed_on = false;
        st->mode = IGX_GB_CACHED;
        t->seed_tab = st;
    }
    if (t->seeds_cap < E) {
        (void)hipFree(t->seeds);
        (void)hipFree(t->seed_slots);
        t->seeds = nullptr;
        t->seed_slots = nullptr;
        t->seeds_cap = 0;
        IGX_HIP(ctx, hipMalloc(&t->seeds, (size_t)E * (LdsCache<L::KW>::KP + 4) * 4));
        IGX_HIP(ctx, hipMalloc(&t->seed_slots, (size_t)E * 4));
        if (!t->seed_gep) IGX_HIP(ctx, hipMalloc(&t->seed_gep, 8));
        t->seeds_cap = E;
    }
    igx_table *st = t->seed_tab;
    (void)fin_collect(st, nullptr);   // the last sample's read-back (landed long ago)
    st->fin_status = IGX_OK;
    (void)igx_groupby_reset(st);
    // the same columns and fused predicates, the sample's rows, one COUNT into the sample table
    // (aggregate 0's columns are still loaded: predicates and guards may read their raw values)
    GbArgs b = a;
    b.n = S;
    b.naggs = 1;
    b.vcount[0] = 1;
    b.hascond[0] = 0;
    b.valid = a.valid;
    b.krec = st->krec;
    b.vrec = st->vrec;
    b.krec_len = st->krec_len;
    b.krec_total = (uint32_t)(st->nslots * st->krec_len);
    b.vrec_words = st->vrec_len / 8;
    b.vrec_total = st->nslots * st->vrec_len < (1ull << 32) ? (uint32_t)(st->nslots * st->vrec_len) : 0u;
    b.err = st->err;
    b.occ = st->occ;
    b.occb = st->occb;
    b.ep = st->ep;
    b.gen = reinterpret_cast<uint64_t *>(st->err) + GEN_WORD;
    b.sshift = 64 - st->sbits;
    b.rmask = (1ull << st->rbits) - 1;
    b.max_probe = 1u << st->rbits;
    b.dbg = 0;
    b.sm = 0;
    b.direct = 0;
    b.nl = NL_DEFAULT;
    b.seeds = nullptr;
    b.seed_gep = nullptr;
    b.nseeds = 0;
    b.dbg_cnt = st->dbg_cnt;
    st->rows_fed = S;
    st->fin_since_update = false;
    st->interval_direct = st->interval_part = false;
    st->occb_dirty = true;
    launch_gb_as<L, false, 2, true>(ctx, b, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((S + GTB - 1) / GTB,
                                                                                           (uint64_t)ctx->num_cus)));
    IGX_HIP(ctx, hipGetLastError());
    int rc = igx_groupby_finalize_async(st, nullptr);
    if (rc) return rc;
    igx_tsortkey key{};
    key.src = IGX_TSRC_AGG;
    key.index = 0;
    key.desc = 1;
    rc = igx_groupby_sort(st, &key, 1, E, t->seed_slots);
    if (rc) return rc;
    hipLaunchKernelGGL(k_gb_seeds<L>, dim3((E + 255) / 256), dim3(256), 0, ctx->stream, a, st->krec, st->krec_len,
                       t->seed_slots, E, t->seeds, t->seed_gep);
    IGX_HIP(ctx, hipGetLastError());
    t->nseeds = E;
    return IGX_OK;
}

template <class L>
static int seeds_compute(igx_table *t, igx_ctx *ctx, const GbArgs &a) {
    if constexpr (!L::is_static) {
        return IGX_ENOTSUP;   // static key layouts only (the reference's BPF key structs)
    } else {
        return seeds_compute_static<L>(t, ctx, a);
    }
}

// one update over layout L in the interval's form
template <class L>
static int launch_form(igx_table *t, igx_ctx *ctx, GbArgs &a, uint32_t blocks) {
    if (t->interval_part && t->interval_probe && t->rows_fed == a.n) {
        t->probe_rows = std::min<uint64_t>(a.n, PROBE_ROWS);
        launch_estimate<L>(ctx, a, blocks, t->probe_rows);
    }
    if (t->interval_part) {
        const GbArgs saved = a;   // launch_part turns the fused predicates into a row mask
        const int rc = launch_part<L>(t, ctx, a);
        if (rc != IGX_ENOMEM || t->mode != IGX_GB_AUTO) return rc;
        // AUTO picked the partitioned form on its own and its scratch does not fit: this
        // update runs cached instead (the forms share the table protocol, so they may mix
        // within an interval), and AUTO measures again at the next interval
        (void)hipGetLastError();
        if (t->interval_probe)   // the cached kernel measures this interval itself: drop the estimate
            IGX_HIP(ctx, hipMemsetAsync(t->err + 2, 0, 8, ctx->stream));
        t->interval_part = false;
        t->interval_probe = false;
        t->direct_left = 0;
        a = saved;
    }
    if (t->interval_direct) {
        launch_direct<L>(ctx, a);
    } else {
        t->occb_dirty = true;   // the cached form's claims mark the byte map
        if (t->rows_fed == a.n) {   // the interval's first update decides whether it is seeded
            uint64_t min_rows = SEED_MIN_ROWS;
            if (const char *m = std::getenv("IGX_GB_SEED_MIN")) min_rows = std::strtoull(m, nullptr, 0);
            t->interval_seeded = false;
            if (L::is_static && t->seed_on && t->gen_planned && !a.dbg && a.n >= min_rows) {
                if (t->seed_left == 0 || !t->nseeds) {
                    uint32_t every = SEED_EVERY;
                    if (const char *e = std::getenv("IGX_GB_SEED_EVERY"))   // A/B knob
                        every = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 0));
                    if (seeds_compute<L>(t, ctx, a) == IGX_OK) t->seed_left = every;
                    else t->nseeds = 0;   // no seeds this time (the sample table failed): plain cache
                }
                --t->seed_left;
                t->interval_seeded = t->nseeds > 0;
            }
        }
        if (t->interval_seeded) {
            a.seeds = t->seeds;
            a.seed_gep = t->seed_gep;
            a.nseeds = t->nseeds;
        }
        launch_gb<L>(ctx, a, blocks);
    }
    return IGX_OK;
}

extern "C" int igx_groupby_set_mode(igx_table *t, uint32_t mode) {
    if (!t) return IGX_EINVAL;
    if (mode > IGX_GB_PART) return igx_fail(t->ctx, IGX_EINVAL, "groupby_set_mode: mode %u", mode);
    t->mode = mode;
    t->direct_left = 0;
    return IGX_OK;
}

extern "C" int igx_groupby_update(igx_table *t, const igx_col *cols, uint32_t ncols, const uint32_t *key_cols,
                                  const igx_pred *preds, uint32_t npreds, uint64_t nrows, uint64_t base_idx) {
    return igx_groupby_update_ex(t, cols, ncols, key_cols, preds, npreds, nullptr, IGX_NO_COL, nrows, base_idx);
}

extern "C" int igx_groupby_update_ex(igx_table *t, const igx_col *cols, uint32_t ncols, const uint32_t *key_cols,
                                     const igx_pred *preds, uint32_t npreds, const uint8_t *valid, uint32_t idx_col,
                                     uint64_t nrows, uint64_t base_idx) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    if (nrows == 0) return IGX_OK;
    if (!cols || !key_cols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: null columns");
    if (nrows >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "groupby_update: more than 2^32 rows in one call");
    if (base_idx + nrows >= READY_IDX)   // `ready` carries first_ins + 1 (a kept key's: index + 2) in 48 bits
        return igx_fail(ctx, IGX_EINVAL, "groupby_update: event indices reach 2^48 (rebase the interval's indices)");
    t->rows_fed += nrows;
    t->fin_since_update = false;
    GbArgs a{};
    uint32_t w = 0;
    for (uint32_t k = 0; k < t->nkeys; ++k) {
        const uint32_t ci = key_cols[k];
        if (ci >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: key column %u out of range", ci);
        const igx_col &c = cols[ci];
        if (c.width != t->key_widths[k])
            return igx_fail(ctx, IGX_EINVAL, "groupby_update: key column %u width %u != %u", k, c.width,
                            t->key_widths[k]);
        const uint8_t *p = static_cast<const uint8_t *>(c.ptr);
        const bool odd = c.width > 2 && c.width % 4;   // 3, 5, 6, 7, 9, ... bytes: byte loads
        const uintptr_t need = odd ? 1 : (c.width >= 16 ? 16 : (c.width >= 4 ? 4 : c.width));
        if (reinterpret_cast<uintptr_t>(p) & (need - 1))
            return igx_fail(ctx, IGX_EINVAL, "groupby_update: key column %u misaligned", k);
        a.kcol[k] = p;
        const uint32_t nw = (c.width + 3) / 4;
        for (uint32_t j = 0; j < nw; ++j, ++w) {
            a.kptr[w] = p;
            a.kwidth[w] = c.width;
            a.koff[w] = 4 * j;
            a.kmask[w] = c.width >= 4 ? 0xFFFFFFFFu : ((1u << (8 * c.width)) - 1u);
            a.kbytes[w] = odd ? std::min<uint32_t>(4, c.width - 4 * j) : 0;
        }
    }
    // any readable dword for loads whose result is discarded (padding words, COUNT, no cond)
    const uint8_t *dummy = static_cast<const uint8_t *>(cols[key_cols[0]].ptr);
    for (; w < KWMAX; ++w) {
        a.kptr[w] = dummy;
        a.kwidth[w] = 0;
        a.koff[w] = 0;
        a.kmask[w] = 0;
    }
    a.naggs = t->naggs;
    for (uint32_t x = t->naggs; x < AMAX; ++x) {   // unused slots are still loaded (issue_row)
        a.vptr[x] = a.cptr[x] = dummy;
        a.vwidth[x] = a.cwidth[x] = 1;
    }
    for (uint32_t x = 0; x < t->naggs; ++x) {
        const igx_agg &g = t->aggs[x];
        a.vcount[x] = g.kind == IGX_AGG_COUNT;
        a.vptr[x] = dummy;
        a.vwidth[x] = 1;
        if (!a.vcount[x]) {
            if (g.col >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: agg column out of range");
            a.vptr[x] = static_cast<const uint8_t *>(cols[g.col].ptr);
            a.vwidth[x] = cols[g.col].width;
            a.vsign[x] = cols[g.col].kind == IGX_KIND_INT;
            if (a.vwidth[x] != 1 && a.vwidth[x] != 2 && a.vwidth[x] != 4 && a.vwidth[x] != 8)
                return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: agg width %u", a.vwidth[x]);
            if (cols[g.col].kind == IGX_KIND_FLOAT)
                return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: float sums are not supported");
            if (g.divisor > 1) {
                if (a.vsign[x])
                    return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: divisor on a signed column");
                a.vdiv[x] = g.divisor;
            }
        }
        a.cptr[x] = dummy;
        a.cwidth[x] = 1;
        if (g.cond_col != IGX_NO_COL) {
            if (g.cond_col >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: cond column out of range");
            const uint32_t cw = cols[g.cond_col].width;
            if (cw != 1 && cw != 2 && cw != 4 && cw != 8)
                return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: condition width %u", cw);
            a.cptr[x] = static_cast<const uint8_t *>(cols[g.cond_col].ptr);
            a.cwidth[x] = cw;
            a.cval[x] = cw == 8 ? g.cond_val : (g.cond_val & ((1ull << (8 * cw)) - 1));
            a.hascond[x] = 1;
        }
    }
    for (uint32_t x = 0; x < AMAX; ++x) {
        a.vshare[x] = a.cshare[x] = AMAX;
        a.vload[x] = x < t->naggs && !a.vcount[x];
        a.cload[x] = x < t->naggs && a.hascond[x];
        for (uint32_t y = 0; y < x; ++y) {
            if (a.vload[x] && a.vshare[x] == AMAX && a.vload[y] && a.vptr[y] == a.vptr[x] && a.vwidth[y] == a.vwidth[x]) {
                a.vshare[x] = y;
                a.vload[x] = 0;
            }
            if (a.cload[x] && a.cshare[x] == AMAX && a.cload[y] && a.cptr[y] == a.cptr[x] && a.cwidth[y] == a.cwidth[x]) {
                a.cshare[x] = y;
                a.cload[x] = 0;
            }
        }
    }
    for (uint32_t x = 0; x < AMAX; ++x) {
        a.vldw[x] = a.vload[x] ? a.vwidth[x] : 0;
        a.cldw[x] = a.cload[x] ? a.cwidth[x] : 0;
        a.vhioff[x] = a.vload[x] && a.vwidth[x] == 8 ? 4 : 0;
        a.chioff[x] = a.cload[x] && a.cwidth[x] == 8 ? 4 : 0;
    }
    // Up to PMAX scalar comparisons (and IN sets) are fused into the kernel; any others --
    // more predicates, regex or string rules -- are AND-ed into a row mask first by a scan
    // with the filter's predicate evaluator (k_common.h), which then masks rows like `valid`.
    std::vector<igx_pred> fused, masked;
    // a guard is fused when it is the condition column of an aggregate (whose raw value the
    // kernel holds anyway): that aggregate's index, else AMAX
    auto guard_agg = [&](const igx_pred &q) -> uint32_t {
        const igx_col &g = cols[q.guard_col];
        for (uint32_t x = 0; x < t->naggs; ++x)
            if (a.hascond[x] && a.cptr[x] == static_cast<const uint8_t *>(g.ptr) && a.cwidth[x] == g.width) return x;
        return AMAX;
    };
    auto fusable = [&](const igx_pred &q) {
        const igx_col &c = cols[q.col];
        return !(q.cmp == IGX_CMP_REGEX || c.kind == IGX_KIND_BYTES || c.kind == IGX_KIND_BOOL ||
                 c.kind == IGX_KIND_OTHER || (c.width != 1 && c.width != 2 && c.width != 4 && c.width != 8) ||
                 (c.kind == IGX_KIND_FLOAT && c.width < 4) || (q.guard_len && guard_agg(q) == AMAX));
    };
    for (uint32_t p = 0; p < npreds; ++p) {
        if (preds[p].col >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: predicate column out of range");
        if (preds[p].guard_len) {
            const int rc = igx_check_guard(ctx, cols, ncols, preds[p]);
            if (rc) return rc;
        }
        (fusable(preds[p]) ? fused : masked).push_back(preds[p]);
    }
    while (fused.size() > PMAX) {   // overflow into the mask, set tests (IN) last: the mask scan has none
        auto it = std::find_if(fused.begin(), fused.end(), [](const igx_pred &q) { return q.cmp != IGX_CMP_IN; });
        if (it == fused.end())
            return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: more than %d set-membership predicates", PMAX);
        masked.push_back(*it);
        fused.erase(it);
    }
    if (!masked.empty()) {
        int rc = grow(ctx, reinterpret_cast<void **>(&t->p_mask), &t->p_mask_bytes, igx_align(nrows, 256));
        if (rc) return rc;
        const uint8_t *in = valid;
        for (size_t b = 0; b < masked.size(); b += IGX_KMAX_PREDS) {
            DevPreds dp;
            rc = igx_build_preds(ctx, cols, ncols, masked.data() + b,
                                 (uint32_t)std::min<size_t>(IGX_KMAX_PREDS, masked.size() - b), &dp);
            if (rc) return rc;
            hipLaunchKernelGGL(k_pred_mask, dim3((unsigned)std::min<uint64_t>(4096, (nrows + 255) / 256)), dim3(256), 0,
                               ctx->stream, dp, in, nrows, t->p_mask);
            IGX_HIP(ctx, hipGetLastError());
            in = t->p_mask;
        }
        valid = t->p_mask;
    }
    preds = fused.data();
    npreds = (uint32_t)fused.size();
    for (uint32_t p = 0; p < npreds; ++p) {
        const igx_pred &q = preds[p];
        const igx_col &c = cols[q.col];
        if (q.cmp == IGX_CMP_IN) {
            if (q.ref_len == 0 || q.ref_len % c.width || q.ref_len > 8 || c.kind == IGX_KIND_FLOAT)
                return igx_fail(ctx, IGX_EINVAL, "groupby_update: IN predicate %u needs 1..8/width "
                                                 "integer values", p);
            a.pcnt[p] = q.ref_len / c.width;
        } else if (q.cmp > IGX_CMP_GE) {
            return igx_fail(ctx, IGX_EINVAL, "groupby_update: predicate %u comparison %u", p, q.cmp);
        }
        a.pptr[p] = static_cast<const uint8_t *>(c.ptr);
        a.pwidth[p] = c.width;
        a.pkind[p] = c.kind;
        a.pcmp[p] = q.cmp;
        a.pneg[p] = q.negate;
        uint64_t r = 0;
        const uint32_t nb = q.cmp == IGX_CMP_IN ? q.ref_len : c.width;
        for (uint32_t b = 0; b < nb; ++b) r |= (uint64_t)q.ref[b] << (8 * b);
        a.pref[p] = r;
        a.pldw[p] = c.width;
        a.pshare[p] = a.pguard[p] = AMAX;
        for (uint32_t x = 0; x < t->naggs; ++x)   // the value column of an aggregate: reuse its load
            if (a.pshare[p] == AMAX && !a.vcount[x] && a.vptr[x] == a.pptr[p] && a.vwidth[x] == c.width) {
                a.pshare[p] = x;
                a.pldw[p] = 0;
            }
        a.gptr[p] = dummy;
        if (q.guard_len) {
            a.pguard[p] = guard_agg(q);
            a.gptr[p] = static_cast<const uint8_t *>(cols[q.guard_col].ptr);
            a.gwidth[p] = q.guard_len;
            a.gref[p] = igx_guard_ref(q);
        }
    }
    for (uint32_t p = npreds; p < PMAX; ++p) {
        a.pptr[p] = a.gptr[p] = dummy;
        a.pwidth[p] = a.pldw[p] = 0;
        a.pshare[p] = a.pguard[p] = AMAX;
    }
    for (uint32_t p = 0; p < PMAX; ++p) a.phioff[p] = a.pwidth[p] == 8 ? 4 : 0;
    a.npred = npreds;
    a.valid = valid;
    a.validp = valid ? valid : dummy;
    a.validw = valid ? 1 : 0;
    a.fidx = nullptr;
    if (idx_col != IGX_NO_COL) {
        if (idx_col >= ncols || cols[idx_col].width != 8)
            return igx_fail(ctx, IGX_EINVAL, "groupby_update: index column must be a u64 column");
        a.fidx = static_cast<const uint64_t *>(cols[idx_col].ptr);
    }
    a.n = nrows;
    a.base_idx = base_idx;
    a.krec = t->krec;
    a.vrec = t->vrec;
    a.krec_len = t->krec_len;
    a.krec_total = (uint32_t)(t->nslots * t->krec_len);
    a.vrec_words = t->vrec_len / 8;
    a.vrec_total = t->nslots * t->vrec_len < (1ull << 32) ? (uint32_t)(t->nslots * t->vrec_len) : 0u;
    a.err = t->err;
    a.occ = t->occ;
    a.occb = t->occb;
    a.ep = t->ep;
    a.gen = reinterpret_cast<uint64_t *>(t->err) + GEN_WORD;
    a.sshift = 64 - t->sbits;
    a.rmask = (1ull << t->rbits) - 1;
    a.max_probe = 1u << t->rbits;
    if (const char *d = std::getenv("IGX_GB_DEBUG")) a.dbg = (uint32_t)std::strtoul(d, nullptr, 0);
    // one loader wave fewer (one prober more) after intervals that missed the cache on more
    // than MORE_PROBERS_ON_PM / 1000 of their rows (until one falls below MORE_PROBERS_OFF_PM)
    a.nl = t->more_probers ? NL_DEFAULT - 1 : NL_DEFAULT;
    if (const char *d = std::getenv("IGX_GB_LOADERS")) {   // tuning knob
        const unsigned long v = std::strtoul(d, nullptr, 0);
        if (v >= 1 && v <= NWAVES - 2) a.nl = (uint32_t)v;
    }
    a.admit_mask = 1;
    a.sm = t->prefer_sm ? 1u : 0u;
    a.direct = 0;
    if (const char *d = std::getenv("IGX_GB_DIRECT")) a.direct = std::strtoul(d, nullptr, 0) ? 1u : 0u;   // ablation
    if (const char *d = std::getenv("IGX_GB_PROBER")) a.sm = std::strtoul(d, nullptr, 0) ? 1u : 0u;   // ablation
    if (const char *d = std::getenv("IGX_GB_ADMIT"))   // ablation: 0 first-miss admission, k: on the (k+1)-th
        a.admit_mask = std::min<uint32_t>(3u, (uint32_t)std::strtoul(d, nullptr, 0));
    a.dbg_cnt = t->dbg_cnt;
    const uint64_t want = (nrows + GTB - 1) / GTB;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ctx->num_cus));
    const uint32_t *kw = t->key_widths;
    // the interval's form is fixed by its first update (the LDS-miss count that drives AUTO
    // is only meaningful for a whole interval of the cached form)
    if (t->rows_fed == nrows) {
        t->interval_direct = t->mode == IGX_GB_DIRECT;
        t->interval_part = t->mode == IGX_GB_PART || (t->mode == IGX_GB_AUTO && t->direct_left > 0);
        t->interval_probe = false;
        t->probe_rows = 0;
        if (t->mode == IGX_GB_AUTO && t->direct_left > 0) t->interval_probe = --t->direct_left == 0;
        t->interval_region = false;
        if (t->region_off > 0) --t->region_off;
    }
    if (std::getenv("IGX_GB_DEBUG")) t->interval_direct = t->interval_part = false;   // diagnostics: cached form
    if (t->gen_planned && (t->interval_direct || t->interval_part)) {
        hipLaunchKernelGGL(k_gen_restart, dim3(1), dim3(1), 0, ctx->stream, a.gen, t->ep);
        IGX_HIP(ctx, hipGetLastError());
        t->gen_planned = false;
    }
    int rc = IGX_OK;
#ifdef IGX_DEV_FAST   // development builds: the bench's key layouts only (fast kernel iteration)
    if (layout_is<TcpKey>(kw, t->nkeys)) rc = launch_form<TcpKey>(t, ctx, a, blocks);
    else if (layout_is<FileKey>(kw, t->nkeys)) rc = launch_form<FileKey>(t, ctx, a, blocks);
    else if (layout_is<NetPolicyKey>(kw, t->nkeys)) rc = launch_form<NetPolicyKey>(t, ctx, a, blocks);
    else return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: layout not in this development build");
#else
    if (t->generic) {
        switch (t->kw_rec) {
        case 2: rc = launch_form<GenericLayout<2>>(t, ctx, a, blocks); break;
        case 4: rc = launch_form<GenericLayout<4>>(t, ctx, a, blocks); break;
        case 6: rc = launch_form<GenericLayout<6>>(t, ctx, a, blocks); break;
        case 8: rc = launch_form<GenericLayout<8>>(t, ctx, a, blocks); break;
        case 12: rc = launch_form<GenericLayout<12>>(t, ctx, a, blocks); break;
        case 18: rc = launch_form<GenericLayout<18>>(t, ctx, a, blocks); break;
        case 24: rc = launch_form<GenericLayout<24>>(t, ctx, a, blocks); break;
        case 32: rc = launch_form<GenericLayout<32>>(t, ctx, a, blocks); break;
        default: return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: no kernel for %u key words", t->kw_rec);
        }
    } else if (layout_is<TcpKey>(kw, t->nkeys)) rc = launch_form<TcpKey>(t, ctx, a, blocks);
    else if (layout_is<FileKey>(kw, t->nkeys)) rc = launch_form<FileKey>(t, ctx, a, blocks);
    else if (layout_is<NetPolicyKey>(kw, t->nkeys))
        rc = launch_form<NetPolicyKey>(t, ctx, a, blocks);
    else if (layout_is<BioKey>(kw, t->nkeys)) rc = launch_form<BioKey>(t, ctx, a, blocks);
    else if (t->nkeys == 1 && kw[0] == 1) rc = launch_form<StaticLayout<1>>(t, ctx, a, blocks);
    else if (t->nkeys == 1 && kw[0] == 2) rc = launch_form<StaticLayout<2>>(t, ctx, a, blocks);
    else if (t->nkeys == 1 && kw[0] == 4) rc = launch_form<StaticLayout<4>>(t, ctx, a, blocks);
    else if (t->nkeys == 1 && kw[0] == 8) rc = launch_form<StaticLayout<8>>(t, ctx, a, blocks);
    else if (t->nkeys == 1 && kw[0] == 16) rc = launch_form<StaticLayout<16>>(t, ctx, a, blocks);
    else return igx_fail(ctx, IGX_EINVAL, "groupby_update: internal layout mismatch");
#endif
    if (rc) return rc;
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

// finalize's device part: the occupied-slot list and the group count, then the count, the
// error word and the LDS-miss count copied to the table's pinned read-back buffer
static int fin_launch(igx_table *t) {
    igx_ctx *ctx = t->ctx;
    const uint64_t tiles = (t->nslots + CT - 1) / CT;
    if (t->interval_direct)
        hipLaunchKernelGGL(k_occ_from_tags, dim3((unsigned)((t->occ_words + 255) / 256)), dim3(256), 0, ctx->stream,
                           t->krec, t->krec_len, t->koff, t->nslots, t->ep, t->occ);
    hipLaunchKernelGGL(k_slots_count, dim3((unsigned)tiles), dim3(256), 0, ctx->stream, t->occ, t->occ_words,
                       t->tile_cnt, t->occb_dirty ? t->occb : (uint8_t *)nullptr);
    t->occb_dirty = false;
    t->fin_since_update = true;
    // the kernel that finds the group count also writes the read-back into fin_host
    const uint64_t seq = ++t->fin_seq;
    t->fin_snap.rows_fed = t->rows_fed;
    t->fin_snap.direct = t->interval_direct;
    t->fin_snap.part = t->interval_part;
    t->fin_snap.region = t->interval_region;
    t->fin_snap.probe = t->interval_part && t->interval_probe;
    t->fin_snap.sampled = t->probe_rows;
    if (tiles <= SLOTS_INLINE_TILES) {
        hipLaunchKernelGGL(k_slots_write, dim3((unsigned)tiles), dim3(256), 0, ctx->stream, t->occ, t->occ_words,
                           (const uint32_t *)nullptr, t->tile_cnt, t->groups, t->n_groups, t->err, t->fin_dev, seq, t->ep);
    } else {
        hipLaunchKernelGGL(k_slots_scan, dim3(1), dim3(1024), 0, ctx->stream, t->tile_cnt, tiles, t->n_groups, t->err,
                           t->fin_dev, seq, t->ep);
        hipLaunchKernelGGL(k_slots_write, dim3((unsigned)tiles), dim3(256), 0, ctx->stream, t->occ, t->occ_words,
                           t->tile_cnt, (const uint32_t *)nullptr, t->groups, (uint64_t *)nullptr, t->err, t->fin_dev, seq, t->ep);
    }
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

static void fin_view(igx_table *t, igx_table_view *view, uint64_t ng) {
    if (!view) return;
    view->n_groups = ng;
    view->n_slots = t->nslots;
    view->key_bytes = t->key_words * 4;
    view->key_stride = t->krec_len;
    view->val_stride = t->vrec_len;
    view->naggs = t->naggs;
    view->keys = t->krec;
    for (uint32_t x = 0; x < 16; ++x) view->aggs[x] = x < t->naggs ? t->vrec + 1 + x : nullptr;
    view->first_idx = t->vrec;
    view->groups = t->groups;
    view->d_n_groups = t->n_groups;
}

// finalize's host part, once the read-back has landed: the count, the AUTO bookkeeping and
// the interval's status
static int fin_apply(igx_table *t) {
    igx_ctx *ctx = t->ctx;
    const uint64_t *h = t->fin_host;   // err block {bits, pad, LDS misses} | group count
    const uint32_t err = reinterpret_cast<const uint32_t *>(h)[0];
    const uint64_t misses = h[1];
    const uint64_t ng = h[2];
    const uint32_t spilled = reinterpret_cast<const uint32_t *>(h)[1];   // a region overflowed
    t->claims_last = h[4];
    t->gen_keys = h[5];
    if (h[4] == ng || h[5] == ~0ull) t->seed_left = 0;   // a generation started or ended: fresh seeds
    const auto &f = t->fin_snap;   // the interval this read-back belongs to
    if (spilled && f.region) t->region_off = DIRECT_RUN + 1;
    t->host_groups = ng;
    // Miss-heavy streams (most rows miss the LDS cache: near-uniform, high-cardinality keys)
    // go faster with the state-machine probers; hit-heavy ones with the batch probers.  When
    // nearly every row missed, the cache is pure overhead: AUTO runs the next DIRECT_RUN
    // intervals in the partitioned form (streamed passes instead of a random HBM probe per
    // row; C4: 4.1 vs 4.4 ms direct, 6.4 ms cached); the last of them re-probes the stream with
    // k_gb_estimate on a sample, and only a stream that has stopped missing goes cached again.
    if (f.rows_fed >= 1000000 && !f.direct && !f.part) {
        t->prefer_sm = misses * 10 > f.rows_fed * 7;
        t->miss_pm = (uint32_t)(misses * 1000 / f.rows_fed);
        t->more_probers = t->miss_pm > (t->more_probers ? MORE_PROBERS_OFF_PM : MORE_PROBERS_ON_PM);
        if (t->mode == IGX_GB_AUTO && misses * 100 > f.rows_fed * DIRECT_MISS_PCT) t->direct_left = DIRECT_RUN;
    }
    // the probe interval (partitioned, with k_gb_estimate on a sample): still nearly all misses
    // -> another run of partitioned intervals; otherwise the next interval runs cached and
    // measures the stream itself
    if (f.probe && f.sampled && t->mode == IGX_GB_AUTO && misses * 100 > f.sampled * DIRECT_MISS_PCT)
        t->direct_left = DIRECT_RUN;
    if (err) return igx_fail(ctx, IGX_ENOSPC, "groupby: table full or probe failure (err=%u)", err);
    if (ng > t->cap)
        return igx_fail(ctx, IGX_ENOSPC, "groupby: %llu distinct keys exceed capacity %llu",
                        (unsigned long long)ng, (unsigned long long)t->cap);
    return IGX_OK;
}

// waits for a pending asynchronous finalize and applies it; its status is kept in fin_status
// until a call returns it (igx_groupby_wait, reset, finalize)
static int fin_collect(igx_table *t, uint64_t *n_groups) {
    if (t->fin_pending) {
        t->fin_pending = false;
        // poll the sequence number; once the stream has drained it must be there
        while (!fin_landed(t)) {
            const hipError_t q = hipStreamQuery(t->ctx->stream);
            if (q == hipSuccess) {
                if (fin_landed(t)) break;
                return t->fin_status = igx_fail(t->ctx, IGX_EIO, "groupby: finalize read-back did not land");
            }
            if (q != hipErrorNotReady) IGX_HIP(t->ctx, q);
            std::this_thread::yield();
        }
        const int rc = fin_apply(t);
        if (rc && !t->fin_status) {
            t->fin_status = rc;
            t->fin_status_seq = t->fin_seq;
        }
    }
    if (n_groups) *n_groups = t->host_groups;
    return t->fin_status;
}

extern "C" int igx_groupby_finalize(igx_table *t, igx_table_view *view) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    (void)fin_collect(t, nullptr);   // the read-back buffer is about to be reused
    int rc = fin_launch(t);
    if (rc) return rc;
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    rc = fin_apply(t);
    fin_view(t, view, t->host_groups);
    if (!rc) rc = t->fin_status;     // an earlier asynchronous finalize's error is not lost
    t->fin_status = IGX_OK;
    return rc;
}

extern "C" int igx_groupby_finalize_async(igx_table *t, igx_table_view *view) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    // the previous interval's read-back (it precedes this interval) is collected first.  A
    // failure of that interval is returned by this call WITHOUT issuing this interval (the view
    // is left untouched), once: a non-zero return always means "not finalized", and calling
    // again issues the interval.  igx_groupby_wait reports an interval's own status only.
    (void)fin_collect(t, nullptr);
    if (const int earlier = t->fin_status) {
        const uint64_t earlier_seq = t->fin_status_seq;
        t->fin_status = IGX_OK;
        const std::string why = igx_last_error(ctx);   // the collected interval's message
        return igx_fail(ctx, earlier, "groupby: the previous interval (finalize %llu) failed: %s; this interval "
                                      "was not finalized",
                        (unsigned long long)earlier_seq, why.c_str());
    }
    const int rc = fin_launch(t);
    if (rc) return rc;
    t->fin_pending = true;
    fin_view(t, view, 0);
    return IGX_OK;
}

extern "C" int igx_groupby_wait(igx_table *t, uint64_t *n_groups) {
    if (!t) return IGX_EINVAL;
    int rc = fin_collect(t, n_groups);
    if (rc && t->fin_status_seq != t->fin_seq) rc = IGX_OK;   // an older interval's (never reached here)
    t->fin_status = IGX_OK;
    return rc;
}

extern "C" int igx_groupby_info(igx_table *t, igx_groupby_info_t *out) {
    if (!t || !out) return IGX_EINVAL;
    std::memset(out, 0, sizeof *out);
    if (t->rows_fed)
        out->form = t->interval_part ? IGX_GB_PART : (t->interval_direct ? IGX_GB_DIRECT : IGX_GB_CACHED);
    out->region = t->interval_part && t->interval_region ? 1u : 0u;
    out->part_left = t->direct_left;
    out->exact_left = t->region_off;
    out->sm_probers = t->prefer_sm ? 1u : 0u;
    out->loaders = t->more_probers ? NL_DEFAULT - 1 : NL_DEFAULT;
    out->miss_permille = t->miss_pm;
    out->rows = t->rows_fed;
    out->claims = t->claims_last;
    out->gen_keys = t->gen_keys;
    out->persist = t->persist ? 1u : 0u;
    return IGX_OK;
}

extern "C" int igx_groupby_gather(igx_table *t, const uint32_t *idx, uint64_t k, uint8_t *out_rows) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    if (k == 0) return IGX_OK;
    if (!idx || !out_rows) return igx_fail(ctx, IGX_EINVAL, "groupby_gather: null argument");
    AggMasks am{};
    for (uint32_t x = 0; x < t->naggs; ++x) {
        const uint32_t ow = t->aggs[x].out_width;
        const uint64_t m = (ow == 0 || ow >= 8) ? ~0ull : ((1ull << (8 * ow)) - 1);
        am.m[2 * x] = (uint32_t)m;
        am.m[2 * x + 1] = (uint32_t)(m >> 32);
    }
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)k), dim3(64), 0, ctx->stream, t->krec, t->krec_len, t->vrec,
                       t->vrec_len / 8, t->key_words, t->naggs, am, idx, t->nslots, k, out_rows);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

// Sort / top-K over the table's groups without materialising them (rows are the occupied
// slots; keys read through the slot list at the record stride).
extern "C" int igx_groupby_sort(igx_table *t, const igx_tsortkey *keys, uint32_t nkeys, uint32_t k,
                                uint32_t *out_slots) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    if (nkeys > 32) return igx_fail(ctx, IGX_ENOTSUP, "groupby_sort: more than 32 keys");
    // After an asynchronous finalize the group count is on the device: a top-K whose keys the
    // device selection handles (no float, no IP text) runs over at most min(capacity, slots)
    // rows bounded by that count; anything else waits for the count first.
    const uint64_t *d_count = nullptr;
    uint64_t nrows = t->host_groups;
    if (t->fin_pending) {
        bool dev_ok = k > 0 && k <= 4096 && 2ull * k < std::min<uint64_t>(t->cap, t->nslots);
        for (uint32_t i = 0; i < nkeys && dev_ok; ++i) {
            const igx_tsortkey &q = keys[i];
            if (q.src == IGX_TSRC_IPTEXT || (q.src == IGX_TSRC_KEY && q.kind == IGX_KIND_FLOAT)) dev_ok = false;
        }
        if (dev_ok) {
            d_count = t->n_groups;
            nrows = std::min<uint64_t>(t->cap, t->nslots);
        } else {
            (void)fin_collect(t, nullptr);   // its status stays for igx_groupby_wait / the next reset
            nrows = t->host_groups;
        }
    }
    igx_sortkey sk[32];
    uint32_t strides[32];
    uint32_t direct = 0;
    for (uint32_t i = 0; i < nkeys; ++i) {
        const igx_tsortkey &q = keys[i];
        sk[i] = igx_sortkey{};
        sk[i].desc = q.desc;
        strides[i] = t->vrec_len;
        if (q.src == IGX_TSRC_AGG) {
            if (q.index >= t->naggs) return igx_fail(ctx, IGX_EINVAL, "groupby_sort: aggregate %u", q.index);
            sk[i].ptr = t->vrec + 1 + q.index;   // little endian: the low out_width bytes
            sk[i].width = t->aggs[q.index].out_width ? t->aggs[q.index].out_width : 8;   // are the wrapped value
            sk[i].kind = IGX_KIND_UINT;
        } else if (q.src == IGX_TSRC_FIRST) {
            sk[i].ptr = t->vrec;
            sk[i].width = 8;
            sk[i].kind = IGX_KIND_UINT;
        } else if (q.src == IGX_TSRC_CONST) {
            sk[i].ptr = t->vrec;   // never read: width 0 marks a parity-only pass
            sk[i].width = 0;
            sk[i].kind = IGX_KIND_BYTES;
        } else if (q.src == IGX_TSRC_KEY) {
            if (q.offset + q.width > t->key_words * 4)
                return igx_fail(ctx, IGX_EINVAL, "groupby_sort: key bytes out of range");
            sk[i].ptr = t->krec + q.offset;
            strides[i] = t->krec_len;
            sk[i].width = q.width;
            sk[i].kind = q.kind;
        } else if (q.src == IGX_TSRC_IPTEXT) {
            // a Stats string column made from key bytes: render the groups' texts (in slot-list
            // order) and sort them as strings
            if (q.offset + 16 > t->key_words * 4 || q.index + 2 > t->key_words * 4)
                return igx_fail(ctx, IGX_EINVAL, "groupby_sort: address / family bytes out of range");
            const uint64_t ng = std::max<uint64_t>(t->host_groups, 1);
            if (t->text_rows[i] < ng) {
                (void)hipFree(t->text[i]);
                t->text[i] = nullptr;
                t->text_rows[i] = 0;
                IGX_HIP(ctx, hipMalloc(&t->text[i], ng * IGX_IPTEXT_WIDTH));
                t->text_rows[i] = ng;
            }
            const int rc = launch_ip_text(ctx, t->krec + q.offset, t->krec_len, t->krec + q.index, t->krec_len,
                                          t->groups, t->host_groups, t->text[i]);
            if (rc) return rc;
            sk[i].ptr = t->text[i];
            strides[i] = IGX_IPTEXT_WIDTH;
            sk[i].width = IGX_IPTEXT_WIDTH;
            sk[i].kind = IGX_KIND_BYTES;
            direct |= 1u << i;
        } else {
            return igx_fail(ctx, IGX_EINVAL, "groupby_sort: bad source");
        }
    }
    // the hint of the table's repeated top-K (k_sort.hip k_tk_*): any slots give an exact answer,
    // the last top-K's give a tight bound
    TopkHint hint{};
    igx_table::TkHint *th = nullptr;
    if (k > 0 && k <= TK_MAXK) {
        uint64_t sig = 0xcbf29ce484222325ull;   // FNV-1a over the sort's description
        auto mix = [&sig](uint64_t v) {
            for (int b = 0; b < 8; ++b) sig = (sig ^ ((v >> (8 * b)) & 0xFF)) * 0x100000001b3ull;
        };
        mix(k);
        mix(nkeys);
        for (uint32_t i = 0; i < nkeys; ++i) {
            const igx_tsortkey &q = keys[i];
            mix(q.src);
            mix(q.index);
            mix(q.desc);
            mix(q.offset);
            mix(q.width);
            mix(q.kind);
        }
        sig |= 1;
        for (auto &h : t->tk)
            if (h.sig == sig) th = &h;
        if (!th) {   // a new sort: the least recently used entry
            th = &t->tk[0];
            for (auto &h : t->tk)
                if (h.used < th->used) th = &h;
            th->sig = sig;
            th->nh = 0;
        }
        th->used = ++t->tk_clock;
        if (!th->slots) IGX_HIP(ctx, hipMalloc(&th->slots, TK_MAXK * 4));
        if (!t->tk_state) {
            IGX_HIP(ctx, hipMalloc(&t->tk_state, TK_STATE_BYTES));
            IGX_HIP(ctx, hipMemsetAsync(t->tk_state, 0, TK_STATE_BYTES, ctx->stream));
        }
        hint.slots = th->slots;
        hint.nh = th->nh;
        hint.occ = t->occ;
        hint.nslots = t->nslots;
        hint.state = t->tk_state;
    }
    const int rc = sort_common_rows(ctx, sk, strides, nkeys, nrows, t->groups, t->vrec, t->vrec_len, k, out_slots,
                                    direct, d_count, th ? &hint : nullptr);
    if (th) th->nh = rc == IGX_OK ? hint.nh : 0;
    return rc;
}

// Diagnostics: how the table's top-Ks were answered so far (synchronous).
extern "C" int igx_groupby_topk_counts(igx_table *t, uint64_t *out2) {
    if (!t || !out2) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    out2[0] = out2[1] = 0;
    if (!t->tk_state) return IGX_OK;
    uint32_t w[2];
    IGX_HIP(ctx, hipMemcpyAsync(w, t->tk_state + 14, 8, hipMemcpyDeviceToHost, ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    out2[0] = w[0];
    out2[1] = w[1];
    return IGX_OK;
}

// Diagnostics only: LDS-cache hit / miss counters collected when IGX_GB_DEBUG has bit 3.
extern "C" int igx_groupby_debug_counts(igx_table *t, uint64_t *out16) {   // out16: 32 words
    if (!t || !out16) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    IGX_HIP(ctx, hipMemcpyAsync(out16, t->dbg_cnt, 256, hipMemcpyDeviceToHost, ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    IGX_HIP(ctx, hipMemsetAsync(t->dbg_cnt, 0, 256, ctx->stream));
    return IGX_OK;
}
