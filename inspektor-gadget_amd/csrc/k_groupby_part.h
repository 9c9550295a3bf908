// k_groupby_part.h -- the partitioned form of the group-by (kernel (2) for high-cardinality
// streams).  Included by k_groupby.hip inside its anonymous namespace: it uses GbArgs, the
// row decoders, the key hash and the HBM table's claim protocol defined there.
//
// Reference semantics are those of k_groupby (the top gadgets' BPF maps, GeneratePolicies'
// first-event-wins map, advisor.go:279-320): exact keys, wrapped sums, first event index.
//
// Near-uniform streams with millions of distinct keys (C4's network-policy tuples, C5's
// 10M files) miss any per-CU cache, and the cached / direct forms then pay one random HBM
// probe (plus memory-side atomics) per row -- the chip's small-random-access rate (~40 G/s)
// bounds them.  A one-level scatter into thousands of buckets does no better: its record
// writes are just as random.  This form is a two-level radix partition in which every
// per-row HBM access is streamed and coalesced:
//   A  a block reads a tile of rows, packs the kept ones into records (key words | raw value
//      / condition column values | index) in LDS, sorts them there by the hash's top f1
//      bits (counting sort) and writes the sorted tile contiguously with its bucket offsets;
//   S  per first-level bucket b1: a scan of its counts over the A tiles, b1's start in the
//      B output and its first B tile;
//   B  a block gathers tr2 consecutive records of b1 (its segments of the A tiles), sorts
//      them by the next f2 bits and writes them contiguously (b1's records stay together);
//   I  per final bucket (b1, b2): its records over b1's B tiles -> aggregate work items;
//   C  an item builds its final bucket's groups in an LDS hash table (full key compare, u64
//      sums, min first index) from the bucket's segments of the B tiles, then writes them to
//      the HBM table.  A final bucket owns whole probe regions of the table (home slot = the
//      hash's top bits, probing wraps inside a region), so an item that is its bucket's only
//      one writes its groups with plain loads and stores -- no CAS, no atomics, occupancy
//      bits through an LDS copy of the bucket's bitmap words.  Items of a split bucket (skew)
//      and rows that overflow the LDS table merge with the table's CAS claims and atomics.
// HBM bytes per kept row: the input read once, then one record written and read back twice;
// per group one probe of its home region.

constexpr uint32_t PT = 1024;                  // threads per block of the aggregate pass
constexpr uint32_t PTS = 256;                  // ... of passes A and B (several blocks per CU, so one
                                               // block's loads overlap another's sort and writes)
constexpr size_t PART_TILE_LDS = 40 * 1024;    // an A / B tile (records + 4 B each): 4 blocks per CU
constexpr size_t PART_AGG_LDS = 152 * 1024;
constexpr uint32_t PSEG = 1024;                // segments a C block maps (B tiles of its bucket)
constexpr uint32_t PSEGB = 256;                // segments a B block maps at a time (A tiles)

struct PartArgs {
    uint32_t *recs1, *recs2;   // A / B tiles (rq x 16 B per record)
    uint32_t *h1;              // tiles1 x (F1 + 1): bucket offsets inside each A tile
    uint32_t *p1;              // F1 x (tiles1 + 1): prefix of b1's records over the A tiles
    uint32_t *base1;           // F1 + 1: start of b1 in recs2
    uint32_t *t2base;          // F1 + 1: first B tile of b1
    uint32_t *h2;              // tiles2max x (F2 + 1): bucket offsets inside each B tile
    uint32_t *items;           // F1 * F2 + 1: prefix of the aggregate work items per final bucket
    uint32_t *bmap;            // tiles2max x 3: a B tile's b1, first and last A tile (k_gbp_bmap)
    uint32_t *imap;            // aggregate work item -> final bucket (k_gbp_imap)
    uint32_t imax;             // imap entries
    uint32_t tiles1, tiles2max;
    uint32_t tr1, tr2;         // record slots of an A / B tile
    uint32_t f1, f2;           // bucket bits of the two levels
    uint32_t sb_log;           // log2 table slots per final bucket
    uint32_t occw;             // occupancy bitmap words per final bucket (slots / 32)
    uint32_t rq;               // record quads (16 B)
    uint32_t iw;               // index words: 1 = row offset (gidx = base_idx + row), 2 = global index
    uint32_t ipos;             // record word of the index
    uint32_t vpos[AMAX], cpos[AMAX];   // record word of a stored value / condition column (0 = none)
    uint32_t vw2[AMAX], cw2[AMAX];     // 1: that column is 8 bytes wide (two words)
    uint32_t ch;               // records per aggregate work item (larger buckets are split)
    uint32_t E;                // LDS table entries
    uint32_t maxp;             // LDS probes before a row takes the HBM path
    uint32_t dbg;              // diagnostics (IGX_GBP_DEBUG): phases to skip, results invalid
};

// record words: key words, then the stored raw columns and the index at host-chosen words
template <int KW, int NA>
struct PartRec {
    static constexpr int W = (KW + 4 * NA + 2 + 3) & ~3;
    static constexpr int U = W <= 32 ? 2 : 1;   // records in flight per thread
};

template <int KW, int NA>
__device__ __forceinline__ void rec_pack(const PartArgs &p, const uint32_t (&k)[KW], const uint64_t (&rv)[NA],
                                         const uint64_t (&rc)[NA], uint64_t idx, uint32_t (&w)[PartRec<KW, NA>::W]) {
    constexpr int W = PartRec<KW, NA>::W;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        uint32_t x = 0;
        if (i < KW) {
            x = k[i];
        } else {
            const uint32_t u = (uint32_t)i;
#pragma unroll
            for (int c = 0; c < NA; ++c) {
                if (p.vpos[c] == u) x = (uint32_t)rv[c];
                if (p.vw2[c] && p.vpos[c] + 1 == u) x = (uint32_t)(rv[c] >> 32);
                if (p.cpos[c] == u) x = (uint32_t)rc[c];
                if (p.cw2[c] && p.cpos[c] + 1 == u) x = (uint32_t)(rc[c] >> 32);
            }
            if (p.ipos == u) x = (uint32_t)idx;
            if (p.iw == 2 && p.ipos + 1 == u) x = (uint32_t)(idx >> 32);
        }
        w[i] = x;
    }
}

template <int W>
__device__ __forceinline__ void recs_load(const uint32_t *recs, uint64_t pos, uint32_t rq, uint32_t (&w)[W]) {
    const u4v *src = reinterpret_cast<const u4v *>(recs) + pos * rq;
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
        u4v t = {0, 0, 0, 0};
        if ((uint32_t)q < rq) t = __builtin_nontemporal_load(src + q);
        w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
    }
}

template <int KW, int NA>
__device__ __forceinline__ void rec_decode(const GbArgs &a, const PartArgs &p, const uint32_t (&w)[PartRec<KW, NA>::W],
                                           uint32_t (&k)[KW], uint64_t (&v)[NA], uint64_t &gidx) {
    constexpr int W = PartRec<KW, NA>::W;
#pragma unroll
    for (int i = 0; i < KW; ++i) k[i] = w[i];
    uint64_t rv[NA], rc[NA], idx = 0;
#pragma unroll
    for (int c = 0; c < NA; ++c) rv[c] = rc[c] = 0;
#pragma unroll
    for (int i = KW; i < W; ++i) {
        const uint32_t u = (uint32_t)i;
#pragma unroll
        for (int c = 0; c < NA; ++c) {
            if (p.vpos[c] == u) rv[c] |= w[i];
            if (p.vw2[c] && p.vpos[c] + 1 == u) rv[c] |= (uint64_t)w[i] << 32;
            if (p.cpos[c] == u) rc[c] |= w[i];
            if (p.cw2[c] && p.cpos[c] + 1 == u) rc[c] |= (uint64_t)w[i] << 32;
        }
        if (p.ipos == u) idx |= w[i];
        if (p.iw == 2 && p.ipos + 1 == u) idx |= (uint64_t)w[i] << 32;
    }
    share_raw<NA>(a, rv, rc);
    vals_from_raw<NA>(a, rv, rc, v);
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

// ---- passes A and B: a tile sorted in LDS, written in order --------------------------------
struct TileLds {
    uint4 *stage;        // tr x rq quads: records in staging order
    uint16_t *bkt;       // tr: bucket of each staged record
    uint16_t *perm;      // tr: sorted position -> staged record
    uint32_t *hist;      // F + 1
    uint32_t *wsum;      // 17
};

__device__ __forceinline__ TileLds tile_lds(uint8_t *lds, uint32_t tr, uint32_t rq, uint32_t F) {
    TileLds L;
    L.stage = reinterpret_cast<uint4 *>(lds);
    L.bkt = reinterpret_cast<uint16_t *>(lds + (size_t)tr * rq * 16);
    L.perm = L.bkt + tr;
    L.hist = reinterpret_cast<uint32_t *>(L.perm + tr);
    L.wsum = L.hist + F + 1;
    return L;
}

// `cnt` staged records (hist holds their bucket counts) -> dst in bucket order, the tile's
// bucket offsets (F + 1 words) -> hout.  Order inside a bucket is free (sums commute, the
// first index is a minimum), so ranks come from LDS atomics; the permutation is built in
// LDS so that the HBM writes are the tile in order, 16 B per lane.
__device__ __forceinline__ void tile_sort_write(const TileLds &L, uint32_t cnt, uint32_t F, uint32_t rq,
                                                uint4 *dst, uint32_t *hout) {
    const uint32_t bt = blockDim.x;
    const uint32_t per = (F + bt - 1) / bt;
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = threadIdx.x * per + i;
        s += b < F ? L.hist[b] : 0u;
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, L.wsum, total);
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = threadIdx.x * per + i;
        if (b < F) {
            const uint32_t c = L.hist[b];
            L.hist[b] = run;
            hout[b] = run;
            run += c;
        }
    }
    if (threadIdx.x == 0) hout[F] = total;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += bt) L.perm[atomicAdd(&L.hist[L.bkt[i]], 1u)] = (uint16_t)i;
    __syncthreads();
    const uint32_t nq = cnt * rq;
    for (uint32_t qi = threadIdx.x; qi < nq; qi += bt) {
        const uint32_t j = qi / rq, q = qi - j * rq;
        dst[qi] = L.stage[(uint32_t)L.perm[j] * rq + q];
    }
}

// A: rows [tile * tr1, ...) -> records sorted by the hash's top f1 bits.  The tile is read
// in rounds of RA x PTS rows, the next round's loads issued before the current one is packed.
template <class L, int NA>
__global__ __launch_bounds__(PTS) void k_gbp_a(GbArgs a, PartArgs p) {
    constexpr int KW = L::KW;
    constexpr int W = PartRec<KW, NA>::W;
    extern __shared__ uint8_t lds_raw[];
    const uint32_t F = 1u << p.f1;
    const TileLds T = tile_lds(lds_raw, p.tr1, p.rq, F);
    __shared__ uint32_t cnt_s;
    for (uint32_t b = threadIdx.x; b < F; b += PTS) T.hist[b] = 0;
    if (threadIdx.x == 0) cnt_s = 0;
    __syncthreads();
    const uint64_t r0 = (uint64_t)blockIdx.x * p.tr1;
    const uint64_t r1 = min(a.n, r0 + p.tr1);
    constexpr int RA = sizeof(RowRaw<L, NA>) <= 80 ? 4 : 2;
    RowRaw<L, NA> R[RA];
#pragma unroll
    for (int u = 0; u < RA; ++u)
        if (r0 + u * PTS + threadIdx.x < r1) issue_row<L, NA>(a, r0 + u * PTS + threadIdx.x, R[u]);
    for (uint64_t r = r0; r < r1; r += RA * PTS) {
#pragma unroll
        for (int u = 0; u < RA; ++u) {
            const uint64_t row = r + u * PTS + threadIdx.x;
            uint32_t k[KW];
            uint64_t rv[NA], rc[NA];
            const bool ok = row < r1 && row_raw<L, NA>(a, row, R[u], k, rv, rc);
            const uint64_t idx = a.fidx && row < r1 ? a.fidx[row] : row;
            if (row + RA * PTS < r1) issue_row<L, NA>(a, row + RA * PTS, R[u]);
            // this wave's kept rows take consecutive staging slots
            const uint64_t m = __ballot(ok);
            const uint32_t lane = threadIdx.x & 63, lead = m ? (uint32_t)__ffsll((long long)m) - 1 : 0;
            uint32_t base = 0;
            if (m && lane == lead) base = atomicAdd(&cnt_s, (uint32_t)__popcll(m));
            base = __shfl(base, (int)lead);
            if (ok) {
                const uint32_t slot = base + (uint32_t)__popcll(m & lanemask_lt());
                const uint32_t bk = hash_bits(hash_key<KW>(k), 0, p.f1);
                uint32_t w[W];
                rec_pack<KW, NA>(p, k, rv, rc, idx, w);
#pragma unroll
                for (int q = 0; q < W / 4; ++q)
                    if ((uint32_t)q < p.rq)
                        T.stage[slot * p.rq + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
                T.bkt[slot] = (uint16_t)bk;
                atomicAdd(&T.hist[bk], 1u);
            }
        }
    }
    __syncthreads();
    if (p.dbg & 1u) return;
    tile_sort_write(T, cnt_s, F, p.rq, reinterpret_cast<uint4 *>(p.recs1) + (uint64_t)blockIdx.x * p.tr1 * p.rq,
                    p.h1 + (uint64_t)blockIdx.x * (F + 1));
}

// S1: per b1 (one block each), the exclusive prefix of its counts over the A tiles
__global__ __launch_bounds__(1024) void k_gbp_colscan(PartArgs p) {
    __shared__ uint32_t wsum[17];
    const uint32_t b1 = blockIdx.x, F = 1u << p.f1;
    const uint32_t per = (p.tiles1 + 1023) / 1024, t0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t t = t0 + i;
        if (t < p.tiles1) {
            const uint32_t *h = p.h1 + (uint64_t)t * (F + 1);
            s += h[b1 + 1] - h[b1];
        }
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, wsum, total);
    uint32_t *out = p.p1 + (uint64_t)b1 * (p.tiles1 + 1);
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t t = t0 + i;
        if (t < p.tiles1) {
            const uint32_t *h = p.h1 + (uint64_t)t * (F + 1);
            out[t] = run;
            run += h[b1 + 1] - h[b1];
        }
    }
    if (threadIdx.x == 0) out[p.tiles1] = total;
}

// S2: b1's start in recs2 and its first B tile (one block)
__global__ __launch_bounds__(1024) void k_gbp_base(PartArgs p) {
    __shared__ uint32_t wsum[17];
    const uint32_t F = 1u << p.f1;
    const uint32_t per = (F + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t s = 0, s2 = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        if (b < F) {
            const uint32_t c = p.p1[(uint64_t)b * (p.tiles1 + 1) + p.tiles1];
            s += c;
            s2 += (c + p.tr2 - 1) / p.tr2;
        }
    }
    uint32_t total, total2;
    uint32_t run = block_excl_scan(s, wsum, total);
    uint32_t run2 = block_excl_scan(s2, wsum, total2);
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = b0 + i;
        if (b < F) {
            const uint32_t c = p.p1[(uint64_t)b * (p.tiles1 + 1) + p.tiles1];
            p.base1[b] = run;
            p.t2base[b] = run2;
            run += c;
            run2 += (c + p.tr2 - 1) / p.tr2;
        }
    }
    if (threadIdx.x == 0) {
        p.base1[F] = total;
        p.t2base[F] = total2;
    }
}

// the first index i in [lo, hi) with v[i] > x (v non-decreasing), by binary search
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t *v, uint32_t lo, uint32_t hi, uint32_t x) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (v[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Flat positions over a list of segments (seg_pos: nseg + 1 prefix, in LDS).  The segment
// holding the first position of each 64-position chunk of a round is found by binary search
// (one per chunk, into cs[]); a lane then walks forward from its chunk's segment, a step or
// two since segments hold tens of records.
__device__ __forceinline__ void seg_chunk_starts(const uint32_t *seg_pos, uint32_t nseg, uint32_t q0, uint32_t end,
                                                 uint32_t nchunk, uint32_t *cs) {
    for (uint32_t c = threadIdx.x; c < nchunk; c += blockDim.x) {
        const uint32_t q = q0 + 64 * c;
        cs[c] = q < end ? upper_bound_u32(seg_pos, 0, nseg + 1, q) - 1 : 0u;
    }
}
__device__ __forceinline__ uint32_t seg_of(const uint32_t *seg_pos, const uint32_t *cs, uint32_t q0, uint32_t q) {
    uint32_t s = cs[(q - q0) >> 6];
    while (seg_pos[s + 1] <= q) ++s;
    return s;
}

// B tiles' b1 and the range of A tiles holding their records (the binary searches, done here
// by one thread per B tile, would otherwise be dependent HBM round trips at each B block's start)
__global__ __launch_bounds__(256) void k_gbp_bmap(PartArgs p) {
    const uint32_t F1 = 1u << p.f1;
    const uint32_t tile = blockIdx.x * 256 + threadIdx.x;
    if (tile >= p.t2base[F1]) return;
    const uint32_t b1 = upper_bound_u32(p.t2base, 0, F1 + 1, tile) - 1;
    const uint32_t j = tile - p.t2base[b1];
    const uint32_t *pb = p.p1 + (uint64_t)b1 * (p.tiles1 + 1);
    const uint32_t q0 = j * p.tr2, q1 = min(pb[p.tiles1], q0 + p.tr2);
    const uint32_t t0 = upper_bound_u32(pb, 0, p.tiles1 + 1, q0) - 1;
    p.bmap[3 * tile] = b1;
    p.bmap[3 * tile + 1] = t0;
    p.bmap[3 * tile + 2] = upper_bound_u32(pb, t0, p.tiles1 + 1, q1 - 1) - 1;
}

// B: B tile `blockIdx.x` = records [j * tr2, (j + 1) * tr2) of its b1 (in A-tile order),
// gathered from b1's segments of the A tiles, sorted by the next f2 bits
template <int KW, int NA>
__global__ __launch_bounds__(PTS) void k_gbp_b(PartArgs p) {
    constexpr int W = PartRec<KW, NA>::W;
    constexpr int U = 4;
    extern __shared__ uint8_t lds_raw[];
    const uint32_t F1 = 1u << p.f1, F2 = 1u << p.f2;
    const uint32_t tile = blockIdx.x;
    if (tile >= p.t2base[F1]) return;
    const uint32_t b1 = p.bmap[3 * tile];
    const uint32_t j = tile - p.t2base[b1];
    const uint32_t *pb = p.p1 + (uint64_t)b1 * (p.tiles1 + 1);
    const uint32_t q0 = j * p.tr2, q1 = min(pb[p.tiles1], q0 + p.tr2), cnt = q1 - q0;
    const TileLds T = tile_lds(lds_raw, p.tr2, p.rq, F2);
    uint32_t *seg_pos = T.wsum + 17;           // PSEGB + 1: prefix (in b1 order) of each mapped A tile
    uint32_t *seg_src = seg_pos + PSEGB + 1;   // PSEGB: recs1 index of the segment's first record
    uint32_t *cs = seg_src + PSEGB;            // tr2 / 64: segment of each 64-record chunk
    for (uint32_t b = threadIdx.x; b < F2; b += PTS) T.hist[b] = 0;
    uint32_t t = p.bmap[3 * tile + 1];
    const uint32_t tl = p.bmap[3 * tile + 2];
    for (uint32_t done = q0; done < q1;) {
        __syncthreads();
        const uint32_t nt = min(PSEGB, tl + 1 - t);
        for (uint32_t i = threadIdx.x; i < nt; i += PTS) {
            const uint32_t tt = t + i;
            seg_pos[i] = pb[tt];
            seg_src[i] = tt * p.tr1 + p.h1[(uint64_t)tt * (F1 + 1) + b1];
        }
        if (threadIdx.x == 0) seg_pos[nt] = pb[t + nt];
        __syncthreads();
        const uint32_t end = min(q1, seg_pos[nt]);
        seg_chunk_starts(seg_pos, nt, done, end, (end - done + 63) / 64, cs);
        __syncthreads();
        // records [done, end): flat positions, U loads in flight per thread
        for (uint32_t base = done; base < end && !(p.dbg & 2u); base += PTS * U) {
            uint32_t w[U][W];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = base + (uint32_t)u * PTS + threadIdx.x;
                if (q < end) {
                    const uint32_t sg = seg_of(seg_pos, cs, done, q);
                    recs_load<W>(p.recs1, (uint64_t)seg_src[sg] + (q - seg_pos[sg]), p.rq, w[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = base + (uint32_t)u * PTS + threadIdx.x;
                if (q >= end) continue;
                uint32_t k[KW];
#pragma unroll
                for (int i = 0; i < KW; ++i) k[i] = w[u][i];
                const uint32_t b2 = hash_bits(hash_key<KW>(k), p.f1, p.f2);
                const uint32_t slot = q - q0;
#pragma unroll
                for (int x = 0; x < W / 4; ++x)
                    if ((uint32_t)x < p.rq)
                        T.stage[slot * p.rq + x] = make_uint4(w[u][4 * x], w[u][4 * x + 1], w[u][4 * x + 2], w[u][4 * x + 3]);
                T.bkt[slot] = (uint16_t)b2;
                atomicAdd(&T.hist[b2], 1u);
            }
        }
        done = end;
        t += nt;
    }
    __syncthreads();
    if (p.dbg & 4u) return;
    tile_sort_write(T, cnt, F2, p.rq,
                    reinterpret_cast<uint4 *>(p.recs2) + ((uint64_t)p.base1[b1] + q0) * p.rq,
                    p.h2 + (uint64_t)tile * (F2 + 1));
}

// I: aggregate work items per final bucket (a block per b1, a thread per b2), then their
// prefix (one block)
__global__ __launch_bounds__(256) void k_gbp_icount(PartArgs p) {
    const uint32_t F2 = 1u << p.f2;
    const uint32_t b1 = blockIdx.x;
    const uint32_t j0 = p.t2base[b1], j1 = p.t2base[b1 + 1];
    for (uint32_t b2 = threadIdx.x; b2 < F2; b2 += 256) {
        uint32_t n = 0;
        uint32_t j = j0;
        for (; j + 8 <= j1; j += 8) {   // eight independent loads per step
            uint32_t c[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t *h = p.h2 + (uint64_t)(j + u) * (F2 + 1);
                c[u] = h[b2 + 1] - h[b2];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) n += c[u];
        }
        for (; j < j1; ++j) {
            const uint32_t *h = p.h2 + (uint64_t)j * (F2 + 1);
            n += h[b2 + 1] - h[b2];
        }
        // a chunk of at most ch records and at most PSEG B tiles per item
        p.items[(b1 << p.f2) | b2] = n ? max((n + p.ch - 1) / p.ch, (j1 - j0 + PSEG - 1) / PSEG) : 0u;
    }
}

__global__ __launch_bounds__(1024) void k_gbp_iscan(PartArgs p) {
    __shared__ uint32_t wsum[17];
    const uint32_t nb = 1u << (p.f1 + p.f2);
    const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; ++i) s += b0 + i < nb ? p.items[b0 + i] : 0u;
    uint32_t total;
    uint32_t run = block_excl_scan(s, wsum, total);
    for (uint32_t i = 0; i < per; ++i) {
        if (b0 + i < nb) {
            const uint32_t c = p.items[b0 + i];
            p.items[b0 + i] = run;
            run += c;
        }
    }
    if (threadIdx.x == 0) p.items[nb] = total;
}

// aggregate work item -> its final bucket (one thread per item; the C blocks would otherwise
// start every item with a dependent binary search in HBM)
__global__ __launch_bounds__(256) void k_gbp_imap(PartArgs p) {
    const uint32_t nb = 1u << (p.f1 + p.f2);
    const uint32_t n = min(p.items[nb], p.imax);
    for (uint32_t it = blockIdx.x * 256 + threadIdx.x; it < n; it += gridDim.x * 256)
        p.imap[it] = upper_bound_u32(p.items, 0, nb + 1, it) - 1;
}

// ---- C: an LDS hash table per work item ----------------------------------------------------
template <int KW>
struct AggTab {
    uint64_t *first;     // E: min event index (~0 = none yet)
    uint64_t *agg;       // naggs x E
    uint32_t *tag;       // E: 0 = empty, else the hash's low word | 1 (set once, by the claimer)
    uint32_t *st;        // E: 1 once the claimer has written the key
    uint32_t *key;       // E x KW
    uint32_t *occ_old;   // occw: the bucket's occupancy bitmap words before this flush
    uint32_t *occ_new;   // occw: slots claimed by this flush
    uint32_t *seg_pos;   // PSEG + 1: prefix of the item's segments
    uint32_t *seg_src;   // PSEG: recs2 index of each segment's first record
    uint32_t *cs;        // PT / 64: segment of each 64-record chunk of a round
    uint32_t *flag;      // [0] some row of the item took the HBM path
    uint32_t E;
};

// find or insert the key's entry; -1 when maxp entries were probed without a match or a free
// one (the row then goes to HBM).  A lane that finds its key's entry claimed but not yet
// published looks again on the next pass of the loop instead of spinning in place, so a
// claimer in the same wave (whose key stores follow the CAS in program order) always gets
// to publish first.
template <int KW>
__device__ __forceinline__ int at_find_insert(const AggTab<KW> &T, const uint32_t (&k)[KW], uint64_t h, uint32_t maxp) {
    const uint32_t t = (uint32_t)h | 1u;
    uint32_t e = (uint32_t)(((uint64_t)(uint32_t)h * T.E) >> 32);
    for (uint32_t probes = 0, looks = 0;;) {
        uint32_t cur = __hip_atomic_load(&T.tag[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            cur = atomicCAS(&T.tag[e], 0u, t);
            if (cur == 0) {
#pragma unroll
                for (int w = 0; w < KW; ++w) T.key[(uint64_t)e * KW + w] = k[w];
                __hip_atomic_store(&T.st[e], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)e;
            }
        }
        if (cur == t) {
            if (__hip_atomic_load(&T.st[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
                if (++looks > SPIN_LIMIT) return -1;   // never expected; the HBM path stays exact
                continue;
            }
            bool eq = true;
#pragma unroll
            for (int w = 0; w < KW; ++w) eq = eq && T.key[(uint64_t)e * KW + w] == k[w];
            if (eq) return (int)e;
        }
        if (++probes >= maxp) return -1;
        e = e + 1 == T.E ? 0 : e + 1;
    }
}

// one row (or one LDS group) merged into the HBM table with CAS claims and atomics
template <int KW, int NA>
__device__ __forceinline__ void hbm_merge(const GbArgs &a, const uint32_t (&k)[KW], uint64_t h,
                                          const uint64_t (&v)[NA], uint64_t first) {
    uint32_t d[probe_quads<KW>() * 4];
    probe_issue<KW>(a, h, d);
    uint64_t first_ins = 0;
    const uint32_t gs = find_or_insert<KW, true>(a, k, h, first, first_ins, d);
    if (gs == SLOT_OVF) return;
#pragma unroll
    for (int x = 0; x < NA; ++x)
        if (x < (int)a.naggs && v[x]) gadd(rec_agg(a, gs, x), (unsigned long long)v[x]);
    if (first < first_ins) gmin(rec_first(a, gs), (unsigned long long)first);
}

// an LDS group written to a final bucket this item owns alone: plain loads and stores
template <int KW, int NA>
__device__ __forceinline__ void flush_owned(const GbArgs &a, const AggTab<KW> &T, const uint32_t (&k)[KW],
                                            uint64_t h, const uint64_t (&v)[NA], uint64_t f, uint64_t sb) {
    constexpr uint32_t KOFF = koff_of(KW);
    uint64_t s = home_slot(a, h);
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

template <int KW, int NA>
__global__ __launch_bounds__(PT) void k_gbp_c(GbArgs a, PartArgs p) {
    constexpr int W = PartRec<KW, NA>::W;
    extern __shared__ uint64_t lds[];
    AggTab<KW> T;
    const uint32_t E = p.E;
    T.E = E;
    T.first = lds;
    T.agg = lds + E;
    T.tag = reinterpret_cast<uint32_t *>(lds + (uint64_t)(1 + a.naggs) * E);
    T.st = T.tag + E;
    T.key = T.st + E;
    T.occ_old = T.key + (uint64_t)E * KW;
    T.occ_new = T.occ_old + p.occw;
    T.seg_pos = T.occ_new + p.occw;
    T.seg_src = T.seg_pos + PSEG + 1;
    T.cs = T.seg_src + PSEG;
    T.flag = T.cs + PT / 64;
    const uint32_t F2 = 1u << p.f2, nb = 1u << (p.f1 + p.f2);
    const uint32_t nitems = min(p.items[nb], p.imax);
    for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
        const uint32_t fb = p.imap[it];   // items[fb] <= it < items[fb + 1]
        const uint32_t nit = p.items[fb + 1] - p.items[fb], kx = it - p.items[fb];
        const uint32_t b1 = fb >> p.f2, b2 = fb & (F2 - 1);
        const uint32_t J = p.t2base[b1 + 1] - p.t2base[b1];
        const uint32_t j0 = p.t2base[b1] + (uint32_t)((uint64_t)J * kx / nit);
        const uint32_t j1 = p.t2base[b1] + (uint32_t)((uint64_t)J * (kx + 1) / nit);
        const uint32_t nseg = j1 - j0;   // <= PSEG (k_gbp_icount)
        for (uint32_t e = threadIdx.x; e < E; e += PT) {
            T.tag[e] = 0;
            T.st[e] = 0;
            T.first[e] = ~0ull;
            for (uint32_t x = 0; x < a.naggs; ++x) T.agg[(uint64_t)x * E + e] = 0;
        }
        if (threadIdx.x == 0) *T.flag = 0;
        // the item's segments: bucket b2 of each B tile j in [j0, j1)
        __shared__ uint32_t wsum[17];
        uint32_t len = 0, src = 0;
        if (threadIdx.x < nseg) {
            const uint32_t jj = j0 + threadIdx.x;
            const uint32_t *h = p.h2 + (uint64_t)jj * (F2 + 1);
            len = h[b2 + 1] - h[b2];
            src = p.base1[b1] + (jj - p.t2base[b1]) * p.tr2 + h[b2];
        }
        uint32_t total;
        const uint32_t off = block_excl_scan(len, wsum, total);
        if (threadIdx.x < nseg) {
            T.seg_pos[threadIdx.x] = off;
            T.seg_src[threadIdx.x] = src;
        }
        if (threadIdx.x == 0) T.seg_pos[nseg] = total;
        __syncthreads();

        // rounds of PT records; the next round's loads are issued before this one is processed
        uint32_t w[2][W];
        if (!(p.dbg & 8u) && total) {
            seg_chunk_starts(T.seg_pos, nseg, 0, min(total, PT), (min(total, PT) + 63) / 64, T.cs);
            __syncthreads();
            if (threadIdx.x < total) {
                const uint32_t sg = seg_of(T.seg_pos, T.cs, 0, threadIdx.x);
                recs_load<W>(p.recs2, (uint64_t)T.seg_src[sg] + (threadIdx.x - T.seg_pos[sg]), p.rq, w[0]);
            }
        }
        for (uint32_t base = 0; base < total && !(p.dbg & 8u); base += 2 * PT) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t cur = base + h * PT, nxt = cur + PT;
                if (cur >= total) break;
                __syncthreads();   // every lane has read cs for the current round
                if (nxt < total) seg_chunk_starts(T.seg_pos, nseg, nxt, min(total, nxt + PT), (min(total, nxt + PT) - nxt + 63) / 64, T.cs);
                __syncthreads();
                if (nxt + threadIdx.x < total) {
                    const uint32_t q = nxt + threadIdx.x;
                    const uint32_t sg = seg_of(T.seg_pos, T.cs, nxt, q);
                    recs_load<W>(p.recs2, (uint64_t)T.seg_src[sg] + (q - T.seg_pos[sg]), p.rq, w[1 - h]);
                }
                if (cur + threadIdx.x >= total) continue;
                uint32_t k[KW];
                uint64_t v[NA], gidx;
                rec_decode<KW, NA>(a, p, w[h], k, v, gidx);
                const uint64_t hh = hash_key<KW>(k);
                if (p.dbg & 32u) {   // diagnostics: records loaded and hashed only
                    if (hh == 0x1234567ull && gidx == 7) *T.flag = 2;
                    continue;
                }
                const int e = at_find_insert<KW>(T, k, hh, p.maxp);
                if (p.dbg & 64u) continue;   // diagnostics: no accumulation
                if (e >= 0) {
#pragma unroll
                    for (int x = 0; x < NA; ++x)
                        if (x < (int)a.naggs && v[x])
                            atomicAdd(reinterpret_cast<unsigned long long *>(&T.agg[(uint64_t)x * E + e]),
                                      (unsigned long long)v[x]);
                    atomicMin(reinterpret_cast<unsigned long long *>(&T.first[e]), (unsigned long long)gidx);
                } else {
                    *T.flag = 1;
                    hbm_merge<KW, NA>(a, k, hh, v, gidx);
                }
            }
        }
        __syncthreads();

        // the item's groups into the HBM table
        const bool owned = nit == 1 && *T.flag == 0;
        const uint64_t sb = (uint64_t)fb << p.sb_log;
        if (owned) {
            for (uint32_t i = threadIdx.x; i < p.occw; i += PT) {
                T.occ_old[i] = a.occ[(sb >> 5) + i];
                T.occ_new[i] = 0;
            }
            __syncthreads();
        }
        for (uint32_t e = threadIdx.x; e < E && !(p.dbg & 16u); e += PT) {
            if (!T.st[e]) continue;
            uint32_t k[KW];
#pragma unroll
            for (int x = 0; x < KW; ++x) k[x] = T.key[(uint64_t)e * KW + x];
            uint64_t v[NA];
#pragma unroll
            for (int x = 0; x < NA; ++x) v[x] = x < (int)a.naggs ? T.agg[(uint64_t)x * E + e] : 0ull;
            const uint64_t h = hash_key<KW>(k);
            if (owned) flush_owned<KW, NA>(a, T, k, h, v, T.first[e], sb);
            else hbm_merge<KW, NA>(a, k, h, v, T.first[e]);
        }
        __syncthreads();
        if (owned) {
            for (uint32_t i = threadIdx.x; i < p.occw; i += PT)
                if (T.occ_new[i]) a.occ[(sb >> 5) + i] = T.occ_old[i] | T.occ_new[i];
            __syncthreads();
        }
    }
}
