// k_groupby_part.h -- the partitioned form of the group-by (kernel (2) for high-cardinality
// streams).  Included by k_groupby.hip inside its anonymous namespace: it uses GbArgs, the
// row decoders, the key hash and the HBM table's claim protocol defined there.
//
// Reference semantics are those of k_groupby (the top gadgets' BPF maps, GeneratePolicies'
// first-event-wins map, advisor.go:279-320): exact keys, wrapped sums, first event index.
//
// Near-uniform streams with millions of distinct keys (C4's network-policy tuples, C5's
// 10M files) miss any per-CU cache, and a form that probes the HBM table per row is bound by
// the chip's small-random-access rate (~50-60 G requests/s whatever the table size,
// tools/micro/randacc.hip).  This form turns every per-row access into a streamed one: the
// rows are radix-partitioned by the key hash into NB = 2^lb final buckets in two scatter
// passes, and each final bucket is then aggregated in LDS by one workgroup.
//   K  count, with pass A's tiling: rows per final bucket (the hash's top lb bits) and per
//      (A tile, first-level bucket) (the top f1 bits);
//   O  chunk sums and exclusive offsets of the per-tile counts: each A tile's exact output
//      position per first-level bucket (no atomics in pass A);
//   S  one block: bucket starts, pass B's cursors and tiles, pass C's work items;
//   A  a tile of rows -> records (packed key words | raw loaded columns | index), ranked in
//      LDS by the top f1 hash bits and staged sorted; each first-level bucket's run is
//      written at its exact position: first-level buckets come out contiguous;
//   B  a tile of one first-level bucket's records, sorted in LDS by the next f2 bits; each
//      final bucket's run is written at a cursor reserved with one atomic per (tile,
//      bucket): final buckets come out contiguous;
//   C  a work item = a final bucket (or a slice of a skewed one): its records are read in
//      order, pre-combined within each wave64 (the leader's key collects its duplicates'
//      values with ballot + shuffle), aggregated in an LDS hash table (full key compare, u64
//      sums, min first index), then written to the HBM table.  A final bucket owns whole
//      probe regions of the table (home slot = the hash's top bits; probing wraps inside a
//      region), so an item that is its bucket's only one writes its groups with plain loads
//      and stores.  Slices of a split bucket, and rows that overflow the LDS table, merge with
//      the table's CAS claims and atomics.
// HBM bytes per kept row: the key columns read twice (K, A), the loaded columns once, and
// one record written and read back twice (A -> B -> C); per group one probe of its region.

constexpr uint32_t PTA = 256;                  // threads per block of passes K, A and B
constexpr uint32_t PTC = 512;                  // ... of the aggregate pass (two blocks per CU)
constexpr size_t PART_TILE_LDS = 72 * 1024;    // a B tile: records + 6 B each
constexpr size_t PART_AGG_LDS = 80 * 1024;     // the C block: LDS table + one round of records
constexpr uint32_t PART_LB_MAX = 15;           // final buckets <= 2^15 (count-pass LDS histogram)
constexpr uint32_t PART_F_MAX = 256;           // buckets per scatter level (one per thread)
constexpr uint32_t PNV = 2 * AMAX;             // distinct value / condition columns a record carries
constexpr uint32_t CHT = 64;                   // A tiles per chunk of the offset scan
constexpr uint32_t RC1_PAD = 16;               // words between two slice cursors of pass A
constexpr uint32_t PART_S1_LOG = 3;            // slices per first-level region (regions)
constexpr uint32_t PART_U1_MAX = PART_F_MAX << PART_S1_LOG;

struct PartArgs {
    uint32_t *recs1, *recs2;   // records after pass A / pass B (rq quads each)
    uint32_t *cnt1;            // tiles_a x F1: an A tile's rows per first-level bucket, then the
                               // exact output position of that run (pass O)
    uint32_t *csum;            // nchunk x F1: the same per chunk of CHT A tiles
    uint32_t *hist;            // NB: rows per final bucket (pass K)
    uint32_t *start2;          // NB + 1: first record of each final bucket (prefix of hist)
    uint32_t *cur2;            // NB: pass B's write cursors (final buckets)
    uint32_t *tstart;          // F1 + 1 (regions: U1 + 1): first B tile of each first-level bucket
                               // (regions: of each slice)
    uint32_t *bt;              // B tile -> first-level bucket
    uint32_t *istart;          // NB + 1: first C work item of each final bucket
    uint32_t *itfb;            // C work item -> final bucket
    uint32_t *ctl;             // [0] C work-item dequeue, [1] B tiles, [2] C work items
    // the row's value / condition columns, each loaded once (aggregates sharing a column
    // share it): pointer, width (0 = unused: dword 0 of a readable column) and high-dword
    // offset (4 for 8-byte columns)
    const uint8_t *vcol[PNV];
    uint32_t vcw[PNV], vchi[PNV];
    uint32_t rpos[PNV], rw2[PNV];      // record word of column j's raw value (+1 when 8 bytes)
    uint32_t nv;                       // loaded columns
    uint32_t vsrc[AMAX], csrc[AMAX];   // column of aggregate x's value / condition (PNV = none)
    uint32_t avp[AMAX], acp[AMAX];     // ... its record word (0xFFFF = none) ...
    uint32_t av2[AMAX], ac2[AMAX];     // ... and 1 when it is 8 bytes wide
    uint32_t tiles_a, nchunk;  // A tiles (PTA x rows-per-thread rows each), chunks of CHT tiles
    uint32_t trb;              // records per B tile
    uint32_t f1, f2, lb;       // bucket bits of the two levels, lb = f1 + f2
    uint32_t sb_log;           // log2 table slots per final bucket
    uint32_t occw;             // occupancy bitmap words per final bucket (slots / 32)
    uint32_t rq, rq_magic;     // record quads (16 B); ceil(2^32 / rq) for quad -> record
    uint32_t kpw[KWMAX];       // key word w lives in record word kpw[w] ...
    uint32_t ksh[KWMAX];       // ... at this bit shift (1- and 2-byte columns share words)
    uint32_t kmsk[KWMAX];      // ... with this mask (0 = a padding word)
    uint32_t kpn;              // packed key words
    uint32_t iw, ipos;         // index words (1 = row offset, 2 = global index column) and their word
    uint32_t ch;               // records per C work item (larger buckets are split)
    uint32_t E;                // LDS table entries
    uint32_t uc;               // records per thread and round of pass C
    uint32_t maxp;             // LDS probes before a row takes the HBM path
    uint32_t combine;          // wave pre-combine rounds per 64 records (0 = off)
    uint32_t dbg;              // diagnostics (IGX_GBP_DEBUG): phases to skip, results invalid
    // region variant (no count pass): bucket b's records fill a fixed region of reg records
    // through a cursor (one atomic per (tile, bucket)); a record past its region merges into
    // the table directly (find-or-insert + atomics: exact on any stream)
    // Pass A's cursors are the most contended words of the form (every A tile adds to each of
    // the F1): a first-level region is cut into 2^s1log slices, A tile t fills slice
    // t mod 2^s1log, and each slice's cursor has a 64-B line of its own (RC1_PAD words)
    uint32_t *rc1, *rc2;       // U1 = F1 << s1log slice cursors (stride RC1_PAD) / NB final-region
                               // cursors (records reserved; may pass the region)
    uint32_t reg1, reg2;       // records per first-level slice / final region (0: exact runs)
    uint32_t s1log;            // log2 slices per first-level region (0 in the exact form)
    uint32_t c2pad;            // words between two final-region cursors (rc2)
    uint32_t pe;               // pass C keeps 16-B packed entries (distinct-only, see c_row_pe)
};

// record words (compile-time bound): packed key words, loaded columns, index
template <int KW, int NV>
constexpr int part_w() { return (KW + 2 * NV + 2 + 3) & ~3; }
// rows per thread of passes K and A (a row's loaded dwords stay in registers)
template <int KW, int NV>
constexpr int part_rows() {
#ifdef IGX_PART_R
    return IGX_PART_R;
#else
    return KW + 1 + 2 * NV <= 8 ? 8 : 4;
#endif
}

// a row's loads: nil mask, key columns, the loaded value / condition columns, index column
template <class L, int NV>
struct PRow {
    uint32_t k[L::KW];
    uint32_t vraw;
    uint32_t lo[NV > 0 ? NV : 1], hi[NV > 0 ? NV : 1];
    uint64_t fi;
};

template <class L, int NV, bool VALS>
__device__ __forceinline__ void prow_issue(const GbArgs &a, const PartArgs &p, uint64_t row, PRow<L, NV> &R) {
    R.vraw = ldd(a.validp, row * a.validw);
    L::load(a, row, R.k);
    if constexpr (VALS) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint64_t b = row * p.vcw[j];
            R.lo[j] = ldd(p.vcol[j], b);
            R.hi[j] = ldd(p.vcol[j], b + p.vchi[j]);
        }
        R.fi = a.fidx ? a.fidx[row] : row;
    }
}

template <class L, int NV>
__device__ __forceinline__ bool prow_ok(const GbArgs &a, uint64_t row, const PRow<L, NV> &R) {
    return !a.valid || ((R.vraw >> ((uint32_t)(row & 3u) * 8u)) & 0xFFu) != 0;
}

// The record's packed key words (launch_part's rule: 1- and 2-byte columns share words, the
// others keep theirs), known at compile time for the static key layouts: the passes then
// decode a record with constant offsets and masks (a record's words come from one or two
// 16-B LDS reads) instead of per-word descriptors held in registers.
struct PackTab {
    uint32_t kpw[KWMAX], ksh[KWMAX], kmsk[KWMAX];
    uint32_t kpn;
};
template <class L>
__host__ __device__ constexpr PackTab pack_static() {
    PackTab t{};
    uint32_t wp = 0, used = 4, shared = 0, w = 0;
    for (int c = 0; c < L::NC; ++c) {
        const uint32_t cw = (uint32_t)L::Ws[c];
        if (cw <= 2) {
            if (used + cw > 4) {
                shared = wp++;
                used = 0;
            }
            t.kpw[w] = shared;
            t.ksh[w] = 8 * used;
            t.kmsk[w] = cw == 1 ? 0xFFu : 0xFFFFu;
            used += cw;
            ++w;
        } else {
            for (uint32_t j = 0; j < (cw + 3) / 4; ++j, ++w) {
                t.kpw[w] = wp++;
                t.ksh[w] = 0;
                t.kmsk[w] = 0xFFFFFFFFu;
            }
        }
    }
    t.kpn = wp;
    return t;
}
template <class L, bool S = L::is_static>
struct PackKey {
    static constexpr bool known = false;
};
template <class L>
struct PackKey<L, true> {
    static constexpr bool known = true;
    static constexpr PackTab T = pack_static<L>();
};
// packed key words of a static layout (a large number for the runtime layouts)
template <class L>
__host__ __device__ constexpr uint32_t pack_words() {
    if constexpr (PackKey<L>::known) return PackKey<L>::T.kpn;
    else return 0xFFu;
}

// A record lives in LDS as rq x 4 words while it is built or read: its fields sit at
// runtime word offsets (host-chosen layout), so LDS addressing does the packing and no
// register array is indexed by a runtime value.
template <class L, int NV>
__device__ __forceinline__ void prow_stage(const PartArgs &p, uint64_t row, const PRow<L, NV> &R, uint32_t *rec) {
    constexpr int KW = L::KW;
    if constexpr (PackKey<L>::known) {
        // static key: packed words built in registers, the record's quads written whole
        constexpr PackTab T = PackKey<L>::T;
        constexpr uint32_t NW = (T.kpn + 3) / 4 * 4;
        uint32_t w[NW] = {};
#pragma unroll
        for (int j = 0; j < KW; ++j)
            if (T.kmsk[j]) w[T.kpw[j]] |= (R.k[j] & T.kmsk[j]) << T.ksh[j];
#pragma unroll
        for (uint32_t q = 0; q < NW / 4; ++q)
            reinterpret_cast<uint4 *>(rec)[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        for (uint32_t q = NW / 4; q < p.rq; ++q) reinterpret_cast<uint4 *>(rec)[q] = make_uint4(0, 0, 0, 0);
    } else {
        for (uint32_t q = 0; q < p.rq; ++q) reinterpret_cast<uint4 *>(rec)[q] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < KW; ++j)
            if (p.kmsk[j]) atomicOr(rec + p.kpw[j], (R.k[j] & p.kmsk[j]) << p.ksh[j]);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        if ((uint32_t)j < p.nv) {
            const uint64_t raw = assemble(R.lo[j], R.hi[j], row * p.vcw[j], p.vcw[j]);
            rec[p.rpos[j]] = (uint32_t)raw;
            if (p.rw2[j]) rec[p.rpos[j] + 1] = (uint32_t)(raw >> 32);
        }
    }
    rec[p.ipos] = (uint32_t)R.fi;
    if (p.iw == 2) rec[p.ipos + 1] = (uint32_t)(R.fi >> 32);
}

// the table's key words back from a record in LDS
template <class L>
__device__ __forceinline__ void lds_key(const PartArgs &p, const uint32_t *rec, uint32_t (&k)[L::KW]) {
    if constexpr (PackKey<L>::known) {
        constexpr PackTab T = PackKey<L>::T;
#pragma unroll
        for (int j = 0; j < L::KW; ++j) k[j] = T.kmsk[j] ? (rec[T.kpw[j]] >> T.ksh[j]) & T.kmsk[j] : 0u;
    } else {
#pragma unroll
        for (int j = 0; j < L::KW; ++j) k[j] = p.kmsk[j] ? (rec[p.kpw[j]] >> p.ksh[j]) & p.kmsk[j] : 0u;
    }
}

__device__ __forceinline__ uint64_t lds_field(const uint32_t *rec, uint32_t pos, uint32_t w2) {
    if (pos == 0xFFFFu) return 0;
    return (uint64_t)rec[pos] | (w2 ? (uint64_t)rec[pos + 1] << 32 : 0ull);
}

// aggregate slots of pass C: AMAX, or 0 for a distinct-only table (no aggregates); arrays
// keep one element so that they stay well-formed
__host__ __device__ constexpr int nax(int na) { return na > 0 ? na : 1; }

// a record in LDS -> key words, the values its aggregates add, its global event index
template <class L, int NA>
__device__ __forceinline__ void lds_decode(const GbArgs &a, const PartArgs &p, const uint32_t *rec, uint32_t (&k)[L::KW],
                                           uint64_t (&v)[nax(NA)], uint64_t &gidx) {
    lds_key<L>(p, rec, k);
    v[0] = 0;
    if constexpr (NA > 0) {
        uint64_t rv[NA], rc[NA];
#pragma unroll
        for (int x = 0; x < NA; ++x) {
            rv[x] = lds_field(rec, p.avp[x], p.av2[x]);
            rc[x] = lds_field(rec, p.acp[x], p.ac2[x]);
        }
        vals_from_raw<NA>(a, rv, rc, v);
    }
    const uint64_t idx = lds_field(rec, p.ipos, p.iw == 2);
    gidx = p.iw == 2 ? idx : a.base_idx + idx;
}

// `bits` bits of the hash after its top `skip` bits
__device__ __forceinline__ uint32_t hash_bits(uint64_t h, uint32_t skip, uint32_t bits) {
    return bits ? (uint32_t)((h << skip) >> (64 - bits)) : 0u;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *wsum, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t i = 0; i < blockDim.x / 64; ++i) {
            const uint32_t t = wsum[i];
            wsum[i] = s;
            s += t;
        }
        wsum[16] = s;
    }
    __syncthreads();
    total = wsum[16];
    const uint32_t r = wsum[wave] + incl - x;
    __syncthreads();
    return r;
}

// Fused predicates of an update in the partitioned form: evaluated once into a row mask
// (AND-ed with the nil mask), which the passes then read like `valid`.
__global__ __launch_bounds__(256) void k_gbp_mask(GbArgs a, uint8_t *out) {
    for (uint64_t row = (uint64_t)blockIdx.x * 256 + threadIdx.x; row < a.n; row += (uint64_t)gridDim.x * 256) {
        bool ok = !a.valid || a.valid[row] != 0;
        for (uint32_t q = 0; q < a.npred && q < PMAX; ++q)
            ok = ok && ((a.gwidth[q] && ld_val(a.gptr[q], row, a.gwidth[q]) != a.gref[q]) ||
                        pred_scalar(ld_val(a.pptr[q], row, a.pwidth[q]), a.pref[q], a.pwidth[q], a.pkind[q],
                                    a.pcmp[q], a.pneg[q], a.pcnt[q]));
        out[row] = ok ? 1 : 0;
    }
}

// ---- K: rows per final bucket, and per (A tile, first-level bucket) -------------------------
// Same tiling as pass A (PTA x R rows per tile), one block per tile.
template <class L, int NV>
__global__ __launch_bounds__(PTA) void k_gbp_count(GbArgs a, PartArgs p) {
    constexpr int KW = L::KW;
    constexpr int R = part_rows<KW, NV>();
    constexpr uint32_t TRA = PTA * R;
    extern __shared__ uint32_t hs[];   // NB final-bucket counts, then F1 tile counts
    const uint32_t NB = 1u << p.lb, F1 = 1u << p.f1;
    uint32_t *h1 = hs + NB;
    for (uint32_t i = threadIdx.x; i < NB; i += PTA) hs[i] = 0;
    for (uint32_t t = blockIdx.x; t < p.tiles_a; t += gridDim.x) {
        if (threadIdx.x < F1) h1[threadIdx.x] = 0;
        __syncthreads();
        const uint64_t r0 = (uint64_t)t * TRA;
        PRow<L, NV> R_[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint64_t row = r0 + u * PTA + threadIdx.x;
            prow_issue<L, NV, false>(a, p, row < a.n ? row : a.n - 1, R_[u]);
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint64_t row = r0 + u * PTA + threadIdx.x;
            if (row < a.n && prow_ok<L, NV>(a, row, R_[u])) {
                const uint64_t h = hash_key<KW>(R_[u].k);
                atomicAdd(&hs[hash_bits(h, 0, p.lb)], 1u);
                atomicAdd(&h1[hash_bits(h, 0, p.f1)], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x < F1) p.cnt1[(uint64_t)t * F1 + threadIdx.x] = h1[threadIdx.x];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NB; i += PTA)
        if (hs[i]) atomicAdd(&p.hist[i], hs[i]);
}

// exclusive prefix (from r) of n values at stride `stride`, in place; loads go out 16 at a
// time (a load-store-load chain on one array is one memory round trip per element)
__device__ __forceinline__ void scan_column(uint32_t *v, uint32_t stride, uint32_t n, uint32_t r) {
    for (uint32_t c0 = 0; c0 < n; c0 += 16) {
        uint32_t x[16];
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) x[i] = c0 + i < n ? v[(uint64_t)(c0 + i) * stride] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) {
            if (c0 + i < n) v[(uint64_t)(c0 + i) * stride] = r;
            r += x[i];
        }
    }
}

// O1: per chunk of CHT A tiles, rows per first-level bucket
__global__ __launch_bounds__(PTA) void k_gbp_csum(PartArgs p) {
    const uint32_t F1 = 1u << p.f1, c = blockIdx.x;
    if (threadIdx.x >= F1) return;
    const uint32_t t0 = c * CHT, t1 = min(p.tiles_a, t0 + CHT);
    uint32_t s = 0;
    for (uint32_t t = t0; t < t1; ++t) s += p.cnt1[(uint64_t)t * F1 + threadIdx.x];
    p.csum[(uint64_t)c * F1 + threadIdx.x] = s;
}

// ---- S: bucket starts, cursors, chunk offsets, B tiles, C work items (one block) -----------
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t *v, uint32_t lo, uint32_t hi, uint32_t x) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (v[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(1024) void k_gbp_scan(PartArgs p) {
    __shared__ uint32_t wsum[17];
    __shared__ uint32_t ts[PART_F_MAX + 1];
    const uint32_t NB = 1u << p.lb, F1 = 1u << p.f1, F2 = 1u << p.f2;
    const uint32_t per = (NB + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t s = 0, si = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        const uint32_t c = b < NB ? p.hist[b] : 0u;
        s += c;
        si += (c + p.ch - 1) / p.ch;
    }
    uint32_t tot, toti;
    uint32_t run = block_excl_scan(s, wsum, tot);
    uint32_t runi = block_excl_scan(si, wsum, toti);
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        if (b >= NB) break;
        const uint32_t c = p.hist[b], ni = (c + p.ch - 1) / p.ch;
        p.start2[b] = run;
        p.cur2[b] = run;
        p.istart[b] = runi;
        for (uint32_t k = 0; k < ni; ++k) p.itfb[runi + k] = b;
        run += c;
        runi += ni;
    }
    // first-level buckets: record counts, starts (= start2 of their first final bucket),
    // chunk offsets and B tiles
    uint32_t c1 = 0;
    if (threadIdx.x < F1)
        for (uint32_t b2 = 0; b2 < F2; ++b2) c1 += p.hist[threadIdx.x * F2 + b2];
    uint32_t tot1, tott;
    const uint32_t st1 = block_excl_scan(c1, wsum, tot1);
    const uint32_t nt = (c1 + p.trb - 1) / p.trb;
    const uint32_t tst = block_excl_scan(nt, wsum, tott);
    if (threadIdx.x < F1) {
        scan_column(p.csum + threadIdx.x, F1, p.nchunk, st1);
        p.tstart[threadIdx.x] = tst;
        ts[threadIdx.x] = tst;
    }
    if (threadIdx.x == 0) {
        p.start2[NB] = tot;
        p.istart[NB] = toti;
        p.tstart[F1] = tott;
        ts[F1] = tott;
        p.ctl[0] = 0;
        p.ctl[1] = tott;
        p.ctl[2] = toti;
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < tott; t += 1024) p.bt[t] = upper_bound_u32(ts, 0, F1 + 1, t) - 1;
}

// O2: each A tile's exact output position per first-level bucket (cnt1 in place)
__global__ __launch_bounds__(PTA) void k_gbp_offs(PartArgs p) {
    const uint32_t F1 = 1u << p.f1, c = blockIdx.x;
    if (threadIdx.x >= F1) return;
    const uint32_t t0 = c * CHT, t1 = min(p.tiles_a, t0 + CHT);
    scan_column(p.cnt1 + (uint64_t)t0 * F1 + threadIdx.x, F1, t1 - t0, p.csum[(uint64_t)c * F1 + threadIdx.x]);
}

template <int KW, int NA>
__device__ __forceinline__ void hbm_merge(const GbArgs &a, const uint32_t (&k)[KW], uint64_t h,
                                          const uint64_t (&v)[NA], uint64_t first);

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(x, o);
        x = y < x ? y : x;
    }
    return x;
}

// Staged records that found their region full are merged into the table directly (exact;
// never on a hashed stream whose buckets stay within 1.25x their share).  The whole wave
// calls it, `spill` marks the lanes holding such a record.  A region overflows when one key
// is hot (its bucket receives its share many times over), so the spilled records of a wave
// are mostly that key's: they are pre-combined across the wave first (wave64 ballot +
// shuffle: every distinct key's sums and minimum first index reduced onto its lowest lane),
// and only the leaders merge -- one record's atomics per key per wave instead of per row.
template <class L>
__device__ __forceinline__ void region_spill(const GbArgs &a, const PartArgs &p, bool spill, const uint32_t *rec) {
    constexpr int KW = L::KW;
    const uint64_t any = __ballot(spill);
    if (!any) return;
    const uint32_t lane = threadIdx.x & 63;
    // err block word 1: a region overflowed this interval (AUTO then partitions exactly)
    if ((int)lane == __ffsll((long long)any) - 1 && !*reinterpret_cast<volatile const uint32_t *>(a.err + 1))
        *reinterpret_cast<volatile uint32_t *>(a.err + 1) = 1u;
    uint32_t k[KW];
    uint64_t v[AMAX], gidx = ~0ull;
#pragma unroll
    for (int w = 0; w < KW; ++w) k[w] = 0;
#pragma unroll
    for (int x = 0; x < AMAX; ++x) v[x] = 0;
    if (spill) lds_decode<L, AMAX>(a, p, rec, k, v, gidx);
    const uint64_t h = hash_key<KW>(k);
    bool lead = spill;
    for (uint64_t todo = any; todo;) {   // one round per distinct key among the spilled lanes
        const int ld = __ffsll((long long)todo) - 1;
        bool same = ((todo >> lane) & 1ull) && h == __shfl((unsigned long long)h, ld);
        if (__ballot(same) != (1ull << ld)) {
#pragma unroll
            for (int w = 0; w < KW; ++w) same = same && k[w] == __shfl(k[w], ld);
        }
        const uint64_t peers = __ballot(same);
        todo &= ~peers;
        if (__popcll(peers) < 2) continue;
#pragma unroll
        for (int x = 0; x < AMAX; ++x) {
            if (x < (int)a.naggs) {
                const unsigned long long t = wave_sum_u64(same ? (unsigned long long)v[x] : 0ull);
                if ((int)lane == ld) v[x] = t;
            }
        }
        const unsigned long long f = wave_min_u64(same ? (unsigned long long)gidx : ~0ull);
        if ((int)lane == ld) gidx = f;
        else if (same) lead = false;
    }
    if (lead) hbm_merge<KW, AMAX>(a, k, h, v, gidx);
}

// a partition pass's record store, written once and read back only by the next pass.  Pass
// B's are non-temporal: its runs (~48 records) fill whole lines, and on C4 pass B took 1 % less
// and pass C, which no longer finds L2 full of B's dirty lines, 6 % less
// (profiles/r06/part_stnt_ab.txt).  Pass A's stay plain: non-temporal, A took 14 % more (its
// runs into the first-level regions leave partial lines that L2 merges).
template <bool NT>
__device__ __forceinline__ void st_rec(uint4 *p, const uint4 q) {
    if constexpr (NT) __builtin_nontemporal_store(u4v{q.x, q.y, q.z, q.w}, reinterpret_cast<u4v *>(p));
    else *p = q;
}

// ---- A: a tile of rows -> records, each first-level bucket's run at its exact position -----
// The tile's rows stay in registers (R per thread, all loads issued at once); a row's rank
// in its bucket comes from an LDS atomic, so the records are staged in LDS already sorted
// and leave as whole runs, 16 B per lane.
template <class L, int NV>
__global__ __launch_bounds__(PTA) void k_gbp_a(GbArgs a, PartArgs p) {
    constexpr int KW = L::KW;
    constexpr int R = part_rows<KW, NV>();
    constexpr uint32_t TRA = PTA * R;
    extern __shared__ uint8_t lds_raw[];
    const uint32_t F = 1u << p.f1, rq = p.rq;
    uint4 *stage = reinterpret_cast<uint4 *>(lds_raw);                   // TRA x rq quads, sorted
    uint8_t *sb = lds_raw + (size_t)TRA * rq * 16;                       // TRA: bucket of each position
    uint32_t *hist = reinterpret_cast<uint32_t *>(sb + TRA);             // F
    uint32_t *off = hist + F, *base = off + F, *wsum = base + F;
    const uint32_t t = blockIdx.x, sl = t & ((1u << p.s1log) - 1u);   // region slice of this tile
    if (threadIdx.x < F) {
        hist[threadIdx.x] = 0;
        if (!p.reg1) base[threadIdx.x] = p.cnt1[(uint64_t)t * F + threadIdx.x];
    }
    __syncthreads();
    const uint64_t r0 = (uint64_t)t * TRA;
    PRow<L, NV> R_[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint64_t row = r0 + u * PTA + threadIdx.x;
        prow_issue<L, NV, true>(a, p, row < a.n ? row : a.n - 1, R_[u]);
    }
    uint32_t bk[R], rk[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint64_t row = r0 + u * PTA + threadIdx.x;
        bk[u] = 0xFFFFFFFFu;
        if (row < a.n && prow_ok<L, NV>(a, row, R_[u])) {
            bk[u] = hash_bits(hash_key<KW>(R_[u].k), 0, p.f1);
            rk[u] = atomicAdd(&hist[bk[u]], 1u);
        }
    }
    __syncthreads();
    uint32_t total;
    const uint32_t o = block_excl_scan(threadIdx.x < F ? hist[threadIdx.x] : 0u, wsum, total);
    if (threadIdx.x < F) {
        off[threadIdx.x] = o;
        const uint32_t hc = hist[threadIdx.x];   // region variant: this tile's run at the bucket's cursor
        if (p.reg1) base[threadIdx.x] = hc ? atomicAdd(p.rc1 + ((threadIdx.x << p.s1log) + sl) * RC1_PAD, hc) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < R; ++u) {
        if (bk[u] == 0xFFFFFFFFu) continue;
        const uint64_t row = r0 + u * PTA + threadIdx.x;
        const uint32_t pos = off[bk[u]] + rk[u];
        prow_stage<L, NV>(p, row, R_[u], reinterpret_cast<uint32_t *>(stage + pos * rq));
        sb[pos] = (uint8_t)bk[u];
    }
    __syncthreads();
    if (p.dbg & 1u) return;
    uint4 *out = reinterpret_cast<uint4 *>(p.recs1);
    const uint32_t nq = total * rq;
    // every lane of a wave runs the same number of iterations (the spill path is wave-wide)
    for (uint32_t q0 = threadIdx.x & ~63u; q0 < nq; q0 += PTA) {
        const uint32_t qi = q0 + (threadIdx.x & 63);
        const bool live = qi < nq;
        const uint32_t j = rq == 1 ? qi : __umulhi(qi, p.rq_magic);   // sorted position
        const uint32_t q = qi - j * rq, b = live ? sb[j] : 0u;
        const uint32_t g = base[b] + j - off[b];
        bool spill = false;
        if (!live) {
        } else if (!p.reg1) st_rec<false>(&out[(uint64_t)g * rq + q], stage[qi]);
        else if (g < p.reg1) st_rec<false>(&out[((uint64_t)((b << p.s1log) + sl) * p.reg1 + g) * rq + q], stage[qi]);
        else spill = q == 0;
        if (p.reg1) region_spill<L>(a, p, spill, reinterpret_cast<const uint32_t *>(stage + (uint64_t)(live ? j : 0u) * rq));
    }
}

// region variant, between A and B: B tiles of each first-level slice (tstart, bt, ctl[1])
__global__ __launch_bounds__(1024) void k_gbr_tiles(PartArgs p) {
    __shared__ uint32_t wsum[17];
    __shared__ uint32_t ts[PART_U1_MAX + 1];
    const uint32_t U1 = 1u << (p.f1 + p.s1log);
    const uint32_t per = (U1 + 1023) / 1024, u0 = threadIdx.x * per;
    uint32_t nt = 0;
    for (uint32_t i = 0; i < per; ++i)
        if (u0 + i < U1) nt += (min(p.rc1[(u0 + i) * RC1_PAD], p.reg1) + p.trb - 1) / p.trb;
    uint32_t tot;
    uint32_t st = block_excl_scan(nt, wsum, tot);
    for (uint32_t i = 0; i < per && u0 + i < U1; ++i) {
        p.tstart[u0 + i] = st;
        ts[u0 + i] = st;
        st += (min(p.rc1[(u0 + i) * RC1_PAD], p.reg1) + p.trb - 1) / p.trb;
    }
    if (threadIdx.x == 0) {
        p.tstart[U1] = tot;
        ts[U1] = tot;
        p.ctl[1] = tot;
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < tot; t += 1024) p.bt[t] = upper_bound_u32(ts, 0, U1 + 1, t) - 1;
}

// region variant, after B: C work items from the final regions' fills (a final bucket larger
// than ch is split)
__global__ __launch_bounds__(1024) void k_gbr_items(PartArgs p) {
    __shared__ uint32_t wsum[17];
    const uint32_t NB = 1u << p.lb;
    const uint32_t per = (NB + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t si = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        const uint32_t c = b < NB ? min(p.rc2[b * p.c2pad], p.reg2) : 0u;
        si += (c + p.ch - 1) / p.ch;
    }
    uint32_t toti;
    uint32_t runi = block_excl_scan(si, wsum, toti);
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        if (b >= NB) break;
        const uint32_t c = min(p.rc2[b * p.c2pad], p.reg2), ni = (c + p.ch - 1) / p.ch;
        p.istart[b] = runi;
        for (uint32_t k = 0; k < ni; ++k) p.itfb[runi + k] = b;
        runi += ni;
    }
    if (threadIdx.x == 0) {
        p.istart[NB] = toti;
        p.ctl[0] = 0;
        p.ctl[2] = toti;
    }
}

// ---- B: a tile of one first-level bucket's records -> its final buckets --------------------
// pass B's register path (static key layouts, one-quad records; the host sizes its LDS;
// the template also takes two-quad records, parity-green but not measured faster on C5's
// partitioned form, so it stays off): each thread holds its records in registers, ranks them there and stages them in
// LDS already sorted, so the output phase reads position -> bucket -> base like pass A (the
// LDS-order path reads position -> input index -> bucket -> base)
__host__ __device__ inline bool gbp_b_regs(const PartArgs &p) {
    return p.rq == 1 && p.trb <= 16 * PTA && !(p.dbg & 6u);
}

template <class L, int RQ, int MB>   // MB records per thread (trb <= MB PTA)
__device__ __forceinline__ void gbp_b_run(const GbArgs &a, const PartArgs &p, uint8_t *lds_raw, const u4v *src,
                                          uint32_t cnt, uint32_t b1) {
    constexpr int KW = L::KW;
    const uint32_t F = 1u << p.f2, trb = p.trb;
    uint4 *stage = reinterpret_cast<uint4 *>(lds_raw);                   // trb x RQ quads, sorted
    uint8_t *sb = lds_raw + (size_t)trb * RQ * 16;                       // final bucket of each position
    uint32_t *hist = reinterpret_cast<uint32_t *>(sb + trb);
    uint32_t *off = hist + F, *base = off + F, *wsum = base + F;
    u4v x[MB][RQ];
#pragma unroll
    for (int m = 0; m < MB; ++m)
        if (m * PTA + threadIdx.x < cnt) {
#pragma unroll
            for (int q = 0; q < RQ; ++q) x[m][q] = __builtin_nontemporal_load(src + (m * PTA + threadIdx.x) * RQ + q);
        }
    if (threadIdx.x < F) hist[threadIdx.x] = 0;
    __syncthreads();
    uint32_t bk[MB], rk[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        bk[m] = 0xFFFFu;
        if (m * PTA + threadIdx.x < cnt) {
            uint32_t w[4 * RQ];
#pragma unroll
            for (int q = 0; q < RQ; ++q) {
                w[4 * q] = x[m][q].x;
                w[4 * q + 1] = x[m][q].y;
                w[4 * q + 2] = x[m][q].z;
                w[4 * q + 3] = x[m][q].w;
            }
            uint32_t k[KW];
            lds_key<L>(p, w, k);
            bk[m] = hash_bits(hash_key<KW>(k), p.f1, p.f2);
            rk[m] = atomicAdd(&hist[bk[m]], 1u);
        }
    }
    __syncthreads();
    const uint32_t c = threadIdx.x < F ? hist[threadIdx.x] : 0u;
    uint32_t total;
    const uint32_t o = block_excl_scan(c, wsum, total);
    if (threadIdx.x < F) {
        off[threadIdx.x] = o;
        const uint32_t fb = (b1 << p.f2) + threadIdx.x;
        base[threadIdx.x] = c ? atomicAdd(p.reg2 ? p.rc2 + fb * p.c2pad : p.cur2 + fb, c) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        if (bk[m] == 0xFFFFu) continue;
        const uint32_t pos = off[bk[m]] + rk[m];
#pragma unroll
        for (int q = 0; q < RQ; ++q) stage[pos * RQ + q] = make_uint4(x[m][q].x, x[m][q].y, x[m][q].z, x[m][q].w);
        sb[pos] = (uint8_t)bk[m];
    }
    __syncthreads();
    uint4 *out = reinterpret_cast<uint4 *>(p.recs2);
    const uint32_t nq = cnt * RQ;
    for (uint32_t q0 = threadIdx.x & ~63u; q0 < nq; q0 += PTA) {   // wave-uniform trip count
        const uint32_t qi = q0 + (threadIdx.x & 63);
        const bool live = qi < nq;
        const uint32_t jj = qi / RQ, q = qi % RQ;
        const uint32_t b = live ? sb[jj] : 0u;
        const uint32_t g = base[b] + jj - off[b];
        bool spill = false;
        if (!live) {
        } else if (!p.reg2) st_rec<true>(&out[(uint64_t)g * RQ + q], stage[qi]);
        else if (g < p.reg2) st_rec<true>(&out[((uint64_t)((b1 << p.f2) + b) * p.reg2 + g) * RQ + q], stage[qi]);
        else spill = q == 0;
        if (p.reg2) region_spill<L>(a, p, spill, reinterpret_cast<const uint32_t *>(stage + (uint64_t)(live ? jj : 0u) * RQ));
    }
}

// B tile `blockIdx.x` = records [j * trb, (j + 1) * trb) of first-level bucket b1 in recs1
// (contiguous): loaded flat into LDS (coalesced), ranked by the next f2 hash bits with LDS
// atomics, and each final bucket's run written at a cursor reserved with one atomic.
template <class L, int NV>
__global__ __launch_bounds__(PTA) void k_gbp_b(GbArgs a, PartArgs p) {
    constexpr int KW = L::KW;
    constexpr int U = 16;              // quads in flight per thread: a whole tile at once
    extern __shared__ uint8_t lds_raw[];
    const uint32_t tile = blockIdx.x;
    if (tile >= p.ctl[1]) return;
    const uint32_t F = 1u << p.f2, rq = p.rq, trb = p.trb;
    uint4 *stage = reinterpret_cast<uint4 *>(lds_raw);                   // trb x rq quads, input order
    uint16_t *bkt = reinterpret_cast<uint16_t *>(lds_raw + (size_t)trb * rq * 16);
    uint16_t *rank = bkt + trb, *perm = rank + trb;
    uint32_t *hist = reinterpret_cast<uint32_t *>(perm + trb);
    uint32_t *off = hist + F, *base = off + F, *wsum = base + F;
    const uint32_t u = p.bt[tile], b1 = u >> p.s1log;   // slice u of first-level bucket b1
    const uint32_t j = tile - p.tstart[u];
    // exact runs: first-level bucket b1 spans final buckets' starts; regions: [u reg1, + fill)
    const uint32_t s = p.reg1 ? u * p.reg1 + j * trb : p.start2[b1 << p.f2] + j * trb;
    const uint32_t e = p.reg1 ? u * p.reg1 + min(min(p.rc1[u * RC1_PAD], p.reg1), (j + 1) * trb)
                              : min(p.start2[(b1 + 1) << p.f2], s + trb);
    const uint32_t cnt = e - s;
    const u4v *src = reinterpret_cast<const u4v *>(p.recs1) + (uint64_t)s * rq;
    if constexpr (PackKey<L>::known && L::KW <= 8) {   // (wider keys never have 1-2 quad records)
        if (gbp_b_regs(p)) {
            gbp_b_run<L, 1, 16>(a, p, lds_raw, src, cnt, b1);
            return;
        }
    }
    if (threadIdx.x < F) hist[threadIdx.x] = 0;
    const uint32_t nq = cnt * rq;
    for (uint32_t q0 = threadIdx.x; q0 < nq && !(p.dbg & 2u); q0 += PTA * U) {
        u4v x[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q0 + u * PTA < nq) x[u] = __builtin_nontemporal_load(src + q0 + u * PTA);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q0 + u * PTA < nq) stage[q0 + u * PTA] = make_uint4(x[u].x, x[u].y, x[u].z, x[u].w);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += PTA) {
        uint32_t k[KW];
        lds_key<L>(p, reinterpret_cast<const uint32_t *>(stage + i * rq), k);
        const uint32_t b2 = hash_bits(hash_key<KW>(k), p.f1, p.f2);
        bkt[i] = (uint16_t)b2;
        rank[i] = (uint16_t)atomicAdd(&hist[b2], 1u);
    }
    __syncthreads();
    const uint32_t c = threadIdx.x < F ? hist[threadIdx.x] : 0u;
    uint32_t total;
    const uint32_t o = block_excl_scan(c, wsum, total);
    if (threadIdx.x < F) {
        off[threadIdx.x] = o;
        const uint32_t fb = (b1 << p.f2) + threadIdx.x;
        base[threadIdx.x] = c ? atomicAdd(p.reg2 ? p.rc2 + fb * p.c2pad : p.cur2 + fb, c) : 0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += PTA) perm[off[bkt[i]] + rank[i]] = (uint16_t)i;
    __syncthreads();
    if (p.dbg & 4u) return;
    uint4 *out = reinterpret_cast<uint4 *>(p.recs2);
    for (uint32_t q0 = threadIdx.x & ~63u; q0 < nq; q0 += PTA) {   // wave-uniform trip count
        const uint32_t qi = q0 + (threadIdx.x & 63);
        const bool live = qi < nq;
        const uint32_t jj = rq == 1 ? qi : __umulhi(qi, p.rq_magic);   // sorted position
        const uint32_t q = qi - jj * rq;
        const uint32_t sidx = live ? perm[jj] : 0u, b = bkt[sidx];
        const uint32_t g = base[b] + jj - off[b];
        bool spill = false;
        if (!live) {
        } else if (!p.reg2) st_rec<true>(&out[(uint64_t)g * rq + q], stage[sidx * rq + q]);
        else if (g < p.reg2) st_rec<true>(&out[((uint64_t)((b1 << p.f2) + b) * p.reg2 + g) * rq + q], stage[sidx * rq + q]);
        else spill = q == 0;
        if (p.reg2) region_spill<L>(a, p, spill, reinterpret_cast<const uint32_t *>(stage + (uint64_t)sidx * rq));
    }
}

// ---- C: an LDS hash table per work item ----------------------------------------------------
template <int KW>
struct AggTab {
    uint64_t *first;     // E: min event index (~0 = none yet)
    uint64_t *agg;       // naggs x E
    uint8_t *tag;        // E: 0 = empty, TAG_BUSY = claimed, key being written, else 0x80 | 7 bits
                         // of the LDS hash (published: the key words are valid)
    uint32_t *key;       // E x KW
    uint32_t *occ_old;   // occw: the bucket's occupancy bitmap words before this flush
    uint32_t *occ_new;   // occw: slots claimed by this flush
    uint32_t *flag;      // [0] some row of the item took the HBM path, [1] the item
    uint32_t E;
};
constexpr uint32_t TAG_BUSY = 1;

__host__ __device__ constexpr size_t agg_entry_bytes(uint32_t kw, uint32_t naggs) { return 9 + 4 * (size_t)kw + 8 * (size_t)naggs; }

// every key word of entry e compared with k: all loads issued before any compare (a
// short-circuit compare is one dependent LDS round trip per word)
template <int KW>
__device__ __forceinline__ bool at_key_eq(const AggTab<KW> &T, uint32_t e, const uint32_t (&k)[KW]) {
    const uint32_t *p = T.key + (uint64_t)e * KW;
    uint32_t d[KW];
    if constexpr (KW % 4 == 0) {
#pragma unroll
        for (int w = 0; w < KW; w += 4) {
            const uint4 q = *reinterpret_cast<const uint4 *>(p + w);
            d[w] = q.x; d[w + 1] = q.y; d[w + 2] = q.z; d[w + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int w = 0; w < KW; ++w) d[w] = p[w];
    }
    uint32_t diff = 0;
#pragma unroll
    for (int w = 0; w < KW; ++w) diff |= d[w] ^ k[w];
    asm volatile("" : "+v"(diff));   // keep the OR of XORs: LLVM splits `== 0` into per-word compares
    return diff == 0;
}

// 0x80 in each byte of x that is zero, 0 elsewhere (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// find or insert the key's entry; -1 when maxp sets were probed without a match or a free
// entry (the row then goes to HBM).  The table is 8-way set associative: a set's 8 one-byte
// tags are one 8-B LDS load, matched against the key's tag with byte-wise zero tests (a few
// VALU operations for the whole set -- per-tag compares were most of the pass's instructions),
// and full keys are compared only on a tag match, so a wave resolves nearly every row in one
// step (a linear probe makes the whole wave iterate as long as its longest chain).  A claimer
// CASes its empty tag byte 0 -> TAG_BUSY in the set's tag word, writes the key, then turns the
// byte into the published tag; a lane that meets TAG_BUSY in its set reads the set again (the
// claimer is between two LDS writes).
template <int KW>
__device__ __forceinline__ int at_find_insert(const AggTab<KW> &T, const uint32_t (&k)[KW], uint64_t h, uint32_t maxp) {
    const uint32_t t8 = 0x80u | ((uint32_t)h & 0x7Fu), t4 = t8 * 0x01010101u, nsets = T.E >> 3;
    uint32_t set = (uint32_t)(((uint64_t)(uint32_t)h * nsets) >> 32);
    uint32_t *tw = reinterpret_cast<uint32_t *>(T.tag);
    for (uint32_t probes = 0, looks = 0;;) {
        const uint32_t base = set * 8;
        asm volatile("" ::: "memory");   // the set is read afresh on every pass
        const uint2 w = *reinterpret_cast<const uint2 *>(T.tag + base);
        uint64_t mt = (uint64_t)zero_bytes(w.x ^ t4) | (uint64_t)zero_bytes(w.y ^ t4) << 32;
        if (mt) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        while (mt) {   // usually one candidate
            const uint32_t e = base + ((uint32_t)__builtin_ctzll(mt) >> 3);
            mt &= mt - 1;
            if (at_key_eq<KW>(T, e, k)) return (int)e;
        }
        // not found (a key's first record, or a tag collision): the busy and empty entries --
        // the masks most records (repeats of a key already in the table) never need
        if (zero_bytes(w.x ^ 0x01010101u) | zero_bytes(w.y ^ 0x01010101u)) {   // a claim in progress
            if (++looks > SPIN_LIMIT) return -1;   // never expected; the HBM path stays exact
            continue;
        }
        const uint64_t me = (uint64_t)zero_bytes(w.x) | (uint64_t)zero_bytes(w.y) << 32;
        if (me) {
            const uint32_t bit = (uint32_t)__builtin_ctzll(me), j = bit >> 3, e = base + j;
            const uint32_t cur = j < 4 ? w.x : w.y, sh = 8 * (j & 3);
            if (atomicCAS(tw + (e >> 2), cur, cur | (TAG_BUSY << sh)) == cur) {
#pragma unroll
                for (int q = 0; q < KW; ++q) T.key[(uint64_t)e * KW + q] = k[q];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                atomicXor(tw + (e >> 2), (TAG_BUSY ^ t8) << sh);   // BUSY -> the published tag
                return (int)e;
            }
            continue;   // the tag word changed under the CAS: read the set again
        }
        if (++probes >= maxp) return -1;   // set full
        set = set + 1 == nsets ? 0 : set + 1;
    }
}

// one row (or one LDS group) merged into the HBM table with CAS claims and atomics
template <int KW, int NA>
__device__ __forceinline__ void hbm_merge(const GbArgs &a, const uint32_t (&k)[KW], uint64_t h,
                                          const uint64_t (&v)[NA], uint64_t first) {
    uint32_t d[probe_quads<KW>() * 4];
    probe_issue<KW>(a, h, d);
    uint64_t first_ins = 0;
    bool claimed = false;
    const uint32_t gs = find_or_insert<KW, true, NA>(a, k, h, first, first_ins, d, v, claimed);
    if (gs == SLOT_OVF || claimed) return;   // a claim wrote the values into the new record
#pragma unroll
    for (int x = 0; x < NA; ++x)
        if (x < (int)a.naggs && v[x]) gadd(rec_agg(a, gs, x), (unsigned long long)v[x]);
    if (first < first_ins) gmin(rec_first(a, gs), (unsigned long long)first);
}

// an LDS group written to a final bucket this item owns alone: plain loads and stores
template <int KW, int NA>
__device__ __forceinline__ void flush_owned(const GbArgs &a, const AggTab<KW> &T, const uint32_t (&k)[KW],
                                            uint64_t h, const uint64_t (&v)[NA], uint64_t f, uint64_t sb,
                                            uint32_t p_sb_log) {
    constexpr uint32_t KOFF = koff_of(KW);
    uint64_t s = home_slot(a, h);
    if ((s >> p_sb_log) != (sb >> p_sb_log)) {   // never expected: a record in the wrong bucket
        atomicOr(a.err, 32u);
        return;
    }
    if (f >= READY_IDX) {   // an index column value that `ready` cannot carry (as find_or_insert)
        atomicOr(a.err, 8u);
        return;
    }
    for (uint32_t probe = 0; probe < a.max_probe; ++probe, s = next_slot(a, s)) {
        const uint32_t l = (uint32_t)(s - sb), wd = l >> 5, bit = 1u << (l & 31);
        if (T.occ_new[wd] & bit) continue;   // claimed by another group of this flush
        uint8_t *r = a.krec + s * a.krec_len;
        uint64_t *vr = a.vrec + s * a.vrec_words;
        if (T.occ_old[wd] & bit) {           // a group of an earlier update this interval
            bool eq = true;
#pragma unroll
            for (int w = 0; w < KW; ++w) eq = eq && reinterpret_cast<const uint32_t *>(r)[w] == k[w];
            if (!eq) continue;
            vr[0] = min(vr[0], f);
#pragma unroll
            for (int x = 0; x < NA; ++x)
                if (x < (int)a.naggs) vr[1 + x] += v[x];
            return;
        }
        if (atomicOr(&T.occ_new[wd], bit) & bit) continue;   // lost the slot to another group
#pragma unroll
        for (int w = 0; w < KW; ++w) reinterpret_cast<uint32_t *>(r)[w] = k[w];
        *reinterpret_cast<uint64_t *>(r + KOFF) = (h & ~EP_MAX) | a.ep;
        *reinterpret_cast<uint64_t *>(r + KOFF + 8) = (a.ep << 48) | (f + 1);
        vr[0] = f;
        for (uint32_t x = 0; x + 1 < a.vrec_words; ++x) vr[1 + x] = x < a.naggs && x < (uint32_t)NA ? v[x] : 0ull;
        return;
    }
    atomicOr(a.err, 4u);
}


// Wave64 pre-combine (a whole wave calls it): the lowest lane still to be merged leads; the
// lanes holding the same key (hash, then every key word, compared with the leader's) hand
// over their values -- sums and the first index reduced across the wave with shuffles -- and
// drop their rows.  A round that finds no duplicate of its leader ends the pre-combine: on a
// near-uniform stream it costs one round of hash shuffles per 64 rows; on a skewed bucket
// the hot key's rows become one LDS update per wave instead of a queue of same-address
// LDS atomics.
template <int KW, int NA>
__device__ __forceinline__ void wave_combine(const GbArgs &a, uint32_t rounds, bool &ok, const uint32_t (&k)[KW],
                                             uint64_t h, uint64_t (&v)[NA], uint64_t &gidx) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t todo = __ballot(ok);
    for (uint32_t r = 0; r < rounds && todo; ++r) {
        const int L = __ffsll((long long)todo) - 1;
        const uint64_t hl = __shfl((unsigned long long)h, L);
        bool same = ((todo >> lane) & 1ull) && h == hl;
        if (__popcll(__ballot(same)) < 2) break;
#pragma unroll
        for (int w = 0; w < KW; ++w) {
            const uint32_t kl = __shfl(k[w], L);
            same = same && k[w] == kl;
        }
        const uint64_t peers = __ballot(same);
        todo &= ~peers;
        if (__popcll(peers) < 2) continue;
#pragma unroll
        for (int x = 0; x < NA; ++x) {
            if (x < (int)a.naggs) {
                const unsigned long long s = wave_sum_u64(same ? (unsigned long long)v[x] : 0ull);
                if ((int)lane == L) v[x] = s;
            }
        }
        const unsigned long long f = wave_min_u64(same ? (unsigned long long)gidx : ~0ull);
        if ((int)lane == L) gidx = f;
        else if (same) ok = false;
    }
}

// C: work items from a dequeue; per item an LDS hash table, then the groups into HBM.
// An item's records are contiguous: they are read in rounds of UC x PTC records as flat
// 16-B quads (the next round's quads in registers while this round is aggregated from LDS).
constexpr uint32_t UCMAX = 2;

// The LDS table's set and tag need no relation to the table's hash (the records of an item
// already share its top bits): a 32-bit multiply-xorshift of the key words, about a third of
// hash_key's quarter-rate multiplies.  hash_key runs only where a group meets HBM.
template <int KW>
__device__ __forceinline__ uint64_t lds_hash(const uint32_t (&k)[KW]) {
    uint32_t x = 0x9E3779B9u * (uint32_t)KW;
#pragma unroll
    for (int w = 0; w < KW; ++w) {
        x = (x ^ k[w]) * 0x85EBCA6Bu;
        x ^= x >> 13;
    }
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

template <class L, int NA>
__device__ __forceinline__ void c_row(const GbArgs &a, const PartArgs &p, const AggTab<L::KW> &T, bool ok,
                                      const uint32_t *rec) {
    constexpr int KW = L::KW;
    uint32_t k[KW];
    uint64_t v[nax(NA)], gidx = 0;
    lds_decode<L, NA>(a, p, rec, k, v, gidx);
    const uint64_t hh = lds_hash<KW>(k);
    if (p.combine) wave_combine<KW, nax(NA)>(a, p.combine, ok, k, hh, v, gidx);   // IGX_GBP_COMBINE
    if (!ok || (p.dbg & 32u)) return;
    const int ei = at_find_insert<KW>(T, k, hh, p.maxp);
    if (p.dbg & 64u) return;   // diagnostics: no accumulation
    if (ei >= 0) {
#pragma unroll
        for (int x = 0; x < NA; ++x)
            if (x < (int)a.naggs && v[x])
                atomicAdd(reinterpret_cast<unsigned long long *>(&T.agg[(uint64_t)x * T.E + ei]), (unsigned long long)v[x]);
        // records arrive nearly in index order: a plain read skips most of the minima (a
        // read of one address from many lanes is a broadcast, an atomic a queue)
        if (gidx < T.first[ei]) atomicMin(reinterpret_cast<unsigned long long *>(&T.first[ei]), (unsigned long long)gidx);
    } else {
        T.flag[0] = 1;
        hbm_merge<KW, nax(NA)>(a, k, hash_key<KW>(k), v, gidx);
    }
}

// Packed entries (distinct-only tables of static layouts whose key packs into at most 3
// words, events indexed by their row offset): an LDS entry is ONE 16-B word {packed key
// words, first row offset}, so a repeat of a known key costs the set's tag load and one
// entry load -- key compare and first index together -- instead of a key load and a
// separate first-index load, and an entry takes 17 B of LDS instead of 25 (more entries per
// bucket).  Same byte tags and claim protocol as at_find_insert.
template <int PW>
__device__ __forceinline__ int pe_find_insert(uint8_t *tg8, uint4 *ent, uint32_t E, const uint32_t (&kp)[PW],
                                              uint32_t h, uint32_t idx, uint32_t maxp, uint32_t &fst) {
    const uint32_t t8 = 0x80u | (h & 0x7Fu), t4 = t8 * 0x01010101u, nsets = E >> 3;
    uint32_t set = (uint32_t)(((uint64_t)h * nsets) >> 32);
    uint32_t *tw = reinterpret_cast<uint32_t *>(tg8);
    for (uint32_t probes = 0, looks = 0;;) {
        const uint32_t base = set * 8;
        asm volatile("" ::: "memory");   // the set is read afresh on every pass
        const uint2 w = *reinterpret_cast<const uint2 *>(tg8 + base);
        uint64_t mt = (uint64_t)zero_bytes(w.x ^ t4) | (uint64_t)zero_bytes(w.y ^ t4) << 32;
        if (mt) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        while (mt) {
            const uint32_t e = base + ((uint32_t)__builtin_ctzll(mt) >> 3);
            mt &= mt - 1;
            const uint4 q = ent[e];
            uint32_t diff = q.x ^ kp[0];
            if constexpr (PW > 1) diff |= q.y ^ kp[1];
            if constexpr (PW > 2) diff |= q.z ^ kp[2];
            asm volatile("" : "+v"(diff));
            if (diff == 0) {
                fst = q.w;
                return (int)e;
            }
        }
        if (zero_bytes(w.x ^ 0x01010101u) | zero_bytes(w.y ^ 0x01010101u)) {   // a claim in progress
            if (++looks > SPIN_LIMIT) return -1;
            continue;
        }
        const uint64_t me = (uint64_t)zero_bytes(w.x) | (uint64_t)zero_bytes(w.y) << 32;
        if (me) {
            const uint32_t j = (uint32_t)__builtin_ctzll(me) >> 3, e = base + j;
            const uint32_t cur = j < 4 ? w.x : w.y, sh = 8 * (j & 3);
            if (atomicCAS(tw + (e >> 2), cur, cur | (TAG_BUSY << sh)) == cur) {
                ent[e] = make_uint4(kp[0], PW > 1 ? kp[PW > 1 ? 1 : 0] : 0u, PW > 2 ? kp[PW > 2 ? 2 : 0] : 0u, idx);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                atomicXor(tw + (e >> 2), (TAG_BUSY ^ t8) << sh);
                fst = idx;
                return (int)e;
            }
            continue;
        }
        if (++probes >= maxp) return -1;
        set = set + 1 == nsets ? 0 : set + 1;
    }
}

template <class L>
__device__ __forceinline__ void c_row_pe(const GbArgs &a, const PartArgs &p, uint8_t *tg8, uint4 *ent, uint32_t E,
                                         uint32_t *flag, bool ok, const uint32_t *rec) {
    constexpr int PW = (int)pack_words<L>();
    constexpr int KW = L::KW;
    uint32_t kp[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) kp[j] = rec[j];
    const uint32_t idx = rec[p.ipos];
    const uint32_t hh = (uint32_t)lds_hash<PW>(kp);
    if (!ok || (p.dbg & 32u)) return;
    uint32_t fst = 0;
    const int ei = pe_find_insert<PW>(tg8, ent, E, kp, hh, idx, p.maxp, fst);
    if (ei >= 0) {
        if (idx < fst) atomicMin(reinterpret_cast<uint32_t *>(ent + ei) + 3, idx);
    } else {
        flag[0] = 1;
        uint32_t k[KW];
        lds_key<L>(p, rec, k);
        const uint64_t v[1] = {0};
        hbm_merge<KW, 1>(a, k, hash_key<KW>(k), v, a.base_idx + idx);
    }
}

// PE: the packed-entry instance (c_row_pe; distinct-only, pack_words <= 3) -- its own kernel,
// so neither instance carries the other's per-record and flush code (registers are allocated
// over the whole kernel: the two paths together spilled 100-300 SGPRs into VGPR lanes).
// Two 80 KB blocks of PTC threads per CU (one 1 024-thread block over the whole 160 KB, half
// the buckets, measured slower: DESIGN.md §4 "Round 6: pass C").
template <class L, int NV, int NA, bool PE = false>
__global__ __launch_bounds__(PTC) void k_gbp_c(GbArgs a, PartArgs p) {
    constexpr uint32_t TPB = PTC;
    constexpr int KW = L::KW;
    constexpr int QM = part_w<KW, NV>() / 4;   // quads per record, compile-time bound
    extern __shared__ uint64_t lds[];
    AggTab<KW> T;
    const uint32_t E = p.E, rq = p.rq, uc = p.uc, RC = uc * TPB;
    T.E = E;
    T.first = lds;
    T.agg = lds + E;
    T.tag = reinterpret_cast<uint8_t *>(lds + (uint64_t)(1 + a.naggs) * E);
    T.key = reinterpret_cast<uint32_t *>(T.tag + E);   // E is a multiple of 8: 8-B aligned
    T.occ_old = T.key + (uint64_t)E * KW;
    T.occ_new = T.occ_old + p.occw;
    T.flag = T.occ_new + p.occw;
    static_assert(!PE || (NA == 0 && pack_words<L>() <= 3), "packed entries: distinct-only, <= 3 words");
    constexpr bool pe = PE;
    uint8_t *tg8 = reinterpret_cast<uint8_t *>(lds);     // packed entries: E tag bytes ...
    uint4 *ent = reinterpret_cast<uint4 *>(tg8 + E);      // ... then E 16-B entries
    if (pe) {
        T.tag = tg8;
        T.occ_old = reinterpret_cast<uint32_t *>(ent + E);
        T.occ_new = T.occ_old + p.occw;
        T.flag = T.occ_new + p.occw;
    }
    uint4 *stage = reinterpret_cast<uint4 *>(T.flag + 4);   // RC x rq quads (16-B aligned: see the launch)
    const u4v *recs = reinterpret_cast<const u4v *>(p.recs2);
    const uint32_t nitems = p.ctl[2];
    for (;;) {
        if (threadIdx.x == 0) T.flag[1] = atomicAdd(&p.ctl[0], 1u);
        if constexpr (PE) {   // only the tags (a claim writes its whole entry): 16 per store
            for (uint32_t q = threadIdx.x; q < E / 16; q += TPB) reinterpret_cast<uint4 *>(tg8)[q] = make_uint4(0, 0, 0, 0);
        } else {
            for (uint32_t x = threadIdx.x; x < E; x += TPB) {
                if ((x & 3) == 0) reinterpret_cast<uint32_t *>(T.tag)[x >> 2] = 0;
                T.first[x] = ~0ull;
                for (uint32_t g = 0; g < a.naggs; ++g) T.agg[(uint64_t)g * E + x] = 0;
            }
        }
        if (threadIdx.x == 0) T.flag[0] = T.flag[2] = 0;
        __syncthreads();
        const uint32_t it = T.flag[1];
        if (it >= nitems) break;
        const uint32_t fb = p.itfb[it];
        const uint32_t i0 = p.istart[fb], nit = p.istart[fb + 1] - i0, kx = it - i0;
        const uint32_t s0 = p.reg2 ? fb * p.reg2 : p.start2[fb];
        const uint32_t len = p.reg2 ? min(p.rc2[fb * p.c2pad], p.reg2) : p.start2[fb + 1] - s0;
        const uint32_t s = s0 + (uint32_t)((uint64_t)len * kx / nit);
        const uint32_t e = s0 + (uint32_t)((uint64_t)len * (kx + 1) / nit);
        const uint64_t qlast = (uint64_t)e * rq - 1;   // the item's last quad (loads clamp to it)

        u4v pf[UCMAX * QM];
        const uint32_t mq = uc * rq;
        auto prefetch = [&](uint32_t r0) {
#pragma unroll
            for (uint32_t m = 0; m < UCMAX * QM; ++m)
                if (m < mq) pf[m] = __builtin_nontemporal_load(recs + min((uint64_t)r0 * rq + m * TPB + threadIdx.x, qlast));
        };
        if (s < e && !(p.dbg & 8u)) prefetch(s);
        for (uint32_t r0 = s; r0 < e && !(p.dbg & 8u); r0 += RC) {
            const uint32_t nq = min(RC, e - r0) * rq;
            __syncthreads();   // the previous round's records are no longer read
#pragma unroll
            for (uint32_t m = 0; m < UCMAX * QM; ++m)
                if (m < mq && m * TPB + threadIdx.x < nq)
                    stage[m * TPB + threadIdx.x] = make_uint4(pf[m].x, pf[m].y, pf[m].z, pf[m].w);
            __syncthreads();
            if (r0 + RC < e) prefetch(r0 + RC);
            for (uint32_t u = 0; u < uc; ++u) {
                const uint32_t i = u * TPB + threadIdx.x;
                const uint32_t *rec = reinterpret_cast<const uint32_t *>(stage + (uint64_t)min(i, RC - 1) * rq);
                if constexpr (PE) c_row_pe<L>(a, p, tg8, ent, E, T.flag, r0 + i < e, rec);
                else c_row<L, NA>(a, p, T, r0 + i < e, rec);
            }
        }
        __syncthreads();

        // the item's groups into the HBM table
        const bool owned = nit == 1 && T.flag[0] == 0;
        const uint64_t sb = (uint64_t)fb << p.sb_log;
        if (owned) {
            for (uint32_t i = threadIdx.x; i < p.occw; i += TPB) {
                T.occ_old[i] = a.occ[(sb >> 5) + i];
                T.occ_new[i] = 0;
            }
            __syncthreads();
        }
        // About a quarter of the entries hold a group, so a loop over the entries ran the flush
        // with a quarter of each wave's lanes busy, once per TPB entries: the live entries are
        // first listed densely (16-bit ids in the stage buffer, free after the last round; one
        // LDS atomic per wave and pass), so every lane flushes a group.  A stage buffer smaller
        // than 2 E bytes (IGX_GBP_UC=1 on one-quad records) keeps the loop over the entries.
        const bool dense = 2u * E <= RC * rq * 16u && !(p.dbg & 2048u);
        uint16_t *live = reinterpret_cast<uint16_t *>(stage);
        if (dense && !(p.dbg & 16u)) {
            const uint32_t lane = threadIdx.x & 63;
            for (uint32_t x0 = 0; x0 < E; x0 += TPB) {
                const uint32_t x = x0 + threadIdx.x;
                const bool lv = x < E && (T.tag[x] & 0x80u);
                const uint64_t b = __ballot(lv);
                uint32_t base = 0;
                if (lane == 0 && b) base = atomicAdd(&T.flag[2], (uint32_t)__popcll(b));
                base = __shfl(base, 0);
                if (lv) live[base + (uint32_t)__popcll(b & ((1ull << lane) - 1))] = (uint16_t)x;
            }
            __syncthreads();
        }
        const uint32_t nflush = dense ? T.flag[2] : E;
        for (uint32_t i = threadIdx.x; i < nflush && !(p.dbg & 16u); i += TPB) {
            const uint32_t x = dense ? live[i] : i;
            if (!dense && !(T.tag[x] & 0x80u)) continue;
            if constexpr (PE) {
                const uint4 q = ent[x];
                const uint32_t w4[4] = {q.x, q.y, q.z, 0u};
                uint32_t k[KW];
                lds_key<L>(p, w4, k);
                const uint64_t v[1] = {0};
                const uint64_t h = hash_key<KW>(k), f = a.base_idx + q.w;
                if (owned) flush_owned<KW, 1>(a, T, k, h, v, f, sb, p.sb_log);
                else hbm_merge<KW, 1>(a, k, h, v, f);
                continue;
            }
            uint32_t k[KW];
#pragma unroll
            for (int q = 0; q < KW; ++q) k[q] = T.key[(uint64_t)x * KW + q];
            uint64_t v[nax(NA)];
            v[0] = 0;
#pragma unroll
            for (int q = 0; q < NA; ++q) v[q] = q < (int)a.naggs ? T.agg[(uint64_t)q * E + x] : 0ull;
            const uint64_t h = hash_key<KW>(k);
            if (owned) flush_owned<KW, nax(NA)>(a, T, k, h, v, T.first[x], sb, p.sb_log);
            else hbm_merge<KW, nax(NA)>(a, k, h, v, T.first[x]);
        }
        __syncthreads();
        if (owned) {
            for (uint32_t i = threadIdx.x; i < p.occw; i += TPB)
                if (T.occ_new[i]) a.occ[(sb >> 5) + i] = T.occ_old[i] | T.occ_new[i];
            __syncthreads();
        }
    }
}
