// k_groupby.hip -- keyed per-interval aggregation (kernel (2)).
//
// Reference semantics: the top gadgets' BPF hash maps, e.g. probe_ip
// (pkg/gadgets/top/tcp/tracer/bpf/tcptop.bpf.c:33-110): build a fixed key struct,
// lookup-or-insert, `+=` into the value; nextStats (tracer.go:147-226) drains one Stats
// row per key.  Keys are compared in full (exact, like the BPF map's memcmp), values
// wrap at their declared width, and each group remembers the global index of its first
// event -- the canonical pre-sort order that replaces BPF map order.
//
// Layout in HBM (one igx_table):
//   slots[C]   16 B {u64 tag, u32 id, u32 -}  open addressing, linear probing, C = 2^k
//   keys[G]    key_stride bytes per dense group id (packed key words)
//   aggs[a][G] u64 per aggregate, first[G] u64, counter u32, err u32
// A new key claims a slot with a 64-bit CAS on the tag, takes a dense id from a counter,
// writes its key with write-through (sc1) stores and publishes the id with an sc1 store
// after `s_waitcnt vmcnt(0)`; readers that hit the same tag poll the id and compare the
// key with sc1 loads (MI355X_MICROARCH.md §Workgroup dispatch, hand-off table row 1).
//
// Partial aggregates are staged per workgroup in LDS (direct-mapped on the dense id,
// first come first served) with LDS u64 atomics; ids that miss go straight to HBM
// atomics; the LDS cache is committed with HBM atomics when the workgroup finishes.
#include "k_common.h"

namespace {

constexpr int TB = 256;
constexpr uint32_t ID_NONE = 0xFFFFFFFFu;
constexpr uint32_t ID_OVF = 0xFFFFFFFEu;
constexpr int KWMAX = 32;
constexpr int AMAX = 8;

enum KMode : uint32_t { KM_ZERO = 0, KM_U8 = 1, KM_U16 = 2, KM_U32 = 4, KM_X4 = 16, KM_CONT = 17 };

struct GbArgs {
    // key words
    const uint8_t *kptr[KWMAX];
    uint32_t kwidth[KWMAX];
    uint32_t koff[KWMAX];
    uint32_t kmode[KWMAX];
    // aggregates
    const uint8_t *vptr[AMAX];
    const uint8_t *cptr[AMAX];
    uint64_t cval[AMAX];
    uint32_t vwidth[AMAX], vsign[AMAX], vcount[AMAX], cwidth[AMAX];
    uint32_t naggs;
    uint32_t lds_entries;   // L (power of two)
    // input
    const uint8_t *valid;
    uint64_t n, base_idx;
    // table
    uint64_t *slots;        // 2 x u64 per slot: [tag][id]
    uint32_t *keys;
    uint32_t key_stride_w;
    uint64_t *aggs[AMAX];
    uint64_t *first;
    uint32_t *counter;
    uint32_t *err;
    uint64_t mask;
    uint32_t cap_ids;
    uint32_t max_probe;
};

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

template <int KW>
__device__ __forceinline__ uint64_t hash_key(const uint32_t (&k)[KW]) {
    uint64_t h = 0x243F6A8885A308D3ull ^ (uint64_t)KW;
#pragma unroll
    for (int w = 0; w < KW; w += 2) {
        uint64_t x = (uint64_t)k[w] | ((w + 1 < KW) ? ((uint64_t)k[w + 1] << 32) : 0ull);
        x *= 0x87C37B91114253D5ull;
        x = rotl64(x, 31);
        x *= 0x4CF5AD432745937Full;
        h ^= x;
        h = rotl64(h, 27) * 5 + 0x52DCE729ull;
    }
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}

template <int KW>
__device__ __forceinline__ void load_key(const GbArgs &a, uint64_t row, uint32_t (&k)[KW]) {
#pragma unroll
    for (int w = 0; w < KW; ++w) {
        const uint32_t m = a.kmode[w];
        const uint8_t *p = a.kptr[w];
        if (m == KM_X4) {
            if constexpr (true) {
                if (w + 3 < KW) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(p + row * a.kwidth[w] + a.koff[w]);
                    k[w] = v.x;
                    if (w + 1 < KW) k[w + 1] = v.y;
                    if (w + 2 < KW) k[w + 2] = v.z;
                    if (w + 3 < KW) k[w + 3] = v.w;
                }
            }
        } else if (m == KM_U32) {
            k[w] = *reinterpret_cast<const uint32_t *>(p + row * a.kwidth[w] + a.koff[w]);
        } else if (m == KM_U16) {
            k[w] = reinterpret_cast<const uint16_t *>(p)[row];
        } else if (m == KM_U8) {
            k[w] = p[row];
        } else if (m == KM_ZERO) {
            k[w] = 0;
        }
    }
}

// lookup-or-insert; returns dense id, ID_OVF on overflow
template <int KW>
__device__ uint32_t find_or_insert(const GbArgs &a, const uint32_t (&k)[KW], uint64_t h) {
    const uint64_t tag = h | 1ull;
    uint64_t s = (h >> 17) & a.mask;
    for (uint32_t probe = 0; probe < a.max_probe; ++probe) {
        uint64_t *slot = a.slots + 2 * s;
        uint64_t t = ld_agent(slot);
        if (t == 0) {
            uint64_t old = atomicCAS(reinterpret_cast<unsigned long long *>(slot), 0ull,
                                     (unsigned long long)tag);
            if (old == 0) {
                uint32_t id = atomicAdd(a.counter, 1u);
                if (id >= a.cap_ids) {
                    atomicOr(a.err, 1u);
                    st_agent(slot + 1, (uint64_t)ID_OVF);
                    return ID_OVF;
                }
                uint32_t *dst = a.keys + (uint64_t)id * a.key_stride_w;
#pragma unroll
                for (int w = 0; w < KW; w += 2) {
                    if (w + 1 < KW)
                        st_agent(reinterpret_cast<uint64_t *>(dst + w),
                                 (uint64_t)k[w] | ((uint64_t)k[w + 1] << 32));
                    else
                        st_agent(dst + w, k[w]);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_agent(slot + 1, (uint64_t)id);
                return id;
            }
            t = old;
        }
        if (t == tag) {
            uint64_t idv = ld_agent(slot + 1);
            uint32_t spins = 0;
            while (idv == (uint64_t)ID_NONE) {
                __builtin_amdgcn_s_sleep(1);
                idv = ld_agent(slot + 1);
                if (++spins > (1u << 22)) {
                    atomicOr(a.err, 2u);
                    return ID_OVF;
                }
            }
            const uint32_t id = (uint32_t)idv;
            if (id == ID_OVF) return ID_OVF;
            const uint32_t *src = a.keys + (uint64_t)id * a.key_stride_w;
            bool eq = true;
#pragma unroll
            for (int w = 0; w < KW; w += 2) {
                if (w + 1 < KW) {
                    uint64_t v = ld_agent(reinterpret_cast<const uint64_t *>(src + w));
                    eq = eq && ((uint32_t)v == k[w]) && ((uint32_t)(v >> 32) == k[w + 1]);
                } else {
                    eq = eq && (ld_agent(src + w) == k[w]);
                }
            }
            if (eq) return id;
        }
        s = (s + 1) & a.mask;
    }
    atomicOr(a.err, 4u);
    return ID_OVF;
}

template <int KW>
__global__ __launch_bounds__(TB) void k_groupby(GbArgs a, DevPreds dp) {
    extern __shared__ uint64_t lds[];
    const uint32_t L = a.lds_entries;
    uint64_t *lfirst = lds;                                   // L
    uint64_t *lagg = lds + L;                                 // naggs x L
    uint32_t *ltag = reinterpret_cast<uint32_t *>(lds + L * (1 + a.naggs));   // L
    for (uint32_t e = threadIdx.x; e < L; e += TB) {
        ltag[e] = ID_NONE;
        lfirst[e] = ~0ull;
        for (uint32_t x = 0; x < a.naggs; ++x) lagg[x * L + e] = 0;
    }
    __syncthreads();

    const uint64_t stride = (uint64_t)gridDim.x * TB;
    for (uint64_t row = (uint64_t)blockIdx.x * TB + threadIdx.x; row < a.n; row += stride) {
        bool ok = true;
        if (a.valid) ok = a.valid[row] != 0;
        if (ok && dp.n) ok = preds_match_all(dp, row);
        if (!ok) continue;
        uint32_t k[KW];
        load_key<KW>(a, row, k);
        const uint64_t h = hash_key<KW>(k);
        const uint32_t id = find_or_insert<KW>(a, k, h);
        if (id == ID_OVF) continue;
        const uint64_t gidx = a.base_idx + row;
        uint64_t v[AMAX];
#pragma unroll
        for (int x = 0; x < AMAX; ++x) {
            v[x] = 0;
            if (x < (int)a.naggs) {
                bool c = true;
                if (a.cptr[x]) c = ld_scalar(a.cptr[x], a.cwidth[x], row, false) == a.cval[x];
                if (c) v[x] = a.vcount[x] ? 1ull : ld_scalar(a.vptr[x], a.vwidth[x], row, a.vsign[x] != 0);
            }
        }
        const uint32_t e = id & (L - 1);
        uint32_t cur = ltag[e];
        if (cur == ID_NONE) {
            cur = atomicCAS(&ltag[e], ID_NONE, id);
            if (cur == ID_NONE) cur = id;
        }
        if (cur == id) {
#pragma unroll
            for (int x = 0; x < AMAX; ++x)
                if (x < (int)a.naggs && v[x])
                    atomicAdd(reinterpret_cast<unsigned long long *>(&lagg[x * L + e]),
                              (unsigned long long)v[x]);
            atomicMin(reinterpret_cast<unsigned long long *>(&lfirst[e]), (unsigned long long)gidx);
        } else {
#pragma unroll
            for (int x = 0; x < AMAX; ++x)
                if (x < (int)a.naggs && v[x])
                    atomicAdd(reinterpret_cast<unsigned long long *>(&a.aggs[x][id]),
                              (unsigned long long)v[x]);
            if (ld_agent(&a.first[id]) > gidx)
                atomicMin(reinterpret_cast<unsigned long long *>(&a.first[id]), (unsigned long long)gidx);
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < L; e += TB) {
        const uint32_t id = ltag[e];
        if (id == ID_NONE) continue;
        for (uint32_t x = 0; x < a.naggs; ++x) {
            const uint64_t s = lagg[x * L + e];
            if (s) atomicAdd(reinterpret_cast<unsigned long long *>(&a.aggs[x][id]), (unsigned long long)s);
        }
        const uint64_t f = lfirst[e];
        if (ld_agent(&a.first[id]) > f)
            atomicMin(reinterpret_cast<unsigned long long *>(&a.first[id]), (unsigned long long)f);
    }
}

__global__ void k_table_reset(uint64_t *slots, uint64_t nslots, uint64_t *first, uint64_t nfirst,
                              uint64_t **aggs, uint32_t naggs, uint32_t *counter) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) {
        slots[2 * i] = 0;
        slots[2 * i + 1] = ID_NONE;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nfirst; i += stride) {
        first[i] = ~0ull;
        for (uint32_t x = 0; x < naggs; ++x) aggs[x][i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x < 2) counter[threadIdx.x] = 0;
}

// groups: copy counter -> u64 n_groups (clamped to cap)
__global__ void k_count(const uint32_t *counter, uint32_t cap, uint64_t *n) {
    uint32_t c = counter[0];
    *n = c > cap ? cap : c;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// host side of the table
// ---------------------------------------------------------------------------------------
struct igx_table {
    igx_ctx *ctx = nullptr;
    uint32_t nkeys = 0;
    uint32_t key_widths[32] = {};
    uint32_t key_words = 0;      // packed words (each column padded to 4 B)
    uint32_t kw_inst = 0;        // instantiated KW >= key_words
    uint32_t key_stride_w = 0;
    igx_agg aggs[AMAX] = {};
    uint32_t naggs = 0;
    uint64_t cap = 0;            // dense ids
    uint64_t nslots = 0;
    uint64_t *slots = nullptr;
    uint32_t *keys = nullptr;
    uint64_t *aggv[AMAX] = {};
    uint64_t **d_aggv = nullptr;
    uint64_t *first = nullptr;
    uint32_t *counter = nullptr;  // [0] = ids, [1] = err
    uint64_t *n_groups = nullptr;
};

static const int kInst[] = {2, 4, 6, 8, 12, 18, 24, 32};

extern "C" int igx_groupby_create(igx_ctx *ctx, const uint32_t *key_widths, uint32_t nkeys,
                                  const igx_agg *aggs, uint32_t naggs, uint64_t capacity,
                                  igx_table **out) {
    if (!ctx || !out || !key_widths || nkeys == 0 || nkeys > 32)
        return igx_fail(ctx, IGX_EINVAL, "groupby_create: bad key description");
    if (naggs > AMAX) return igx_fail(ctx, IGX_ENOTSUP, "groupby_create: more than %d aggregates", AMAX);
    if (capacity == 0 || capacity >= 0xFFFFFFF0ull)
        return igx_fail(ctx, IGX_EINVAL, "groupby_create: bad capacity");
    uint32_t words = 0;
    for (uint32_t i = 0; i < nkeys; ++i) {
        uint32_t w = key_widths[i];
        if (w == 0 || w == 3 || (w > 4 && w % 4)) return igx_fail(ctx, IGX_ENOTSUP, "groupby: key width %u", w);
        words += (w + 3) / 4;
    }
    if (words > KWMAX) return igx_fail(ctx, IGX_ENOTSUP, "groupby: key wider than %d bytes", KWMAX * 4);
    auto *t = new igx_table();
    t->ctx = ctx;
    t->nkeys = nkeys;
    for (uint32_t i = 0; i < nkeys; ++i) t->key_widths[i] = key_widths[i];
    t->key_words = words;
    for (int k : kInst)
        if ((uint32_t)k >= words) { t->kw_inst = k; break; }
    t->key_stride_w = (uint32_t)igx_align(t->kw_inst, 4);   // 16-B aligned keys
    t->naggs = naggs;
    for (uint32_t i = 0; i < naggs; ++i) t->aggs[i] = aggs[i];
    t->cap = capacity;
    uint64_t ns = 1024;
    while (ns < 2 * capacity) ns <<= 1;
    t->nslots = ns;
    hipError_t e = hipMalloc(&t->slots, ns * 16);
    if (e == hipSuccess) e = hipMalloc(&t->keys, capacity * t->key_stride_w * 4);
    for (uint32_t i = 0; i < naggs && e == hipSuccess; ++i) e = hipMalloc(&t->aggv[i], capacity * 8);
    if (e == hipSuccess) e = hipMalloc(&t->d_aggv, AMAX * sizeof(uint64_t *));
    if (e == hipSuccess) e = hipMalloc(&t->first, capacity * 8);
    if (e == hipSuccess) e = hipMalloc(&t->counter, 64);
    if (e == hipSuccess) e = hipMalloc(&t->n_groups, 64);
    if (e == hipSuccess)
        e = hipMemcpyAsync(t->d_aggv, t->aggv, AMAX * sizeof(uint64_t *), hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) {
        igx_groupby_destroy(t);
        return igx_fail(ctx, IGX_ENOMEM, "groupby_create: %s", hipGetErrorString(e));
    }
    *out = t;
    return igx_groupby_reset(t);
}

extern "C" int igx_groupby_reset(igx_table *t) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    hipLaunchKernelGGL(k_table_reset, dim3(1024), dim3(256), 0, ctx->stream, t->slots, t->nslots,
                       t->first, t->cap, t->d_aggv, t->naggs, t->counter);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_groupby_destroy(igx_table *t) {
    if (!t) return IGX_OK;
    (void)hipStreamSynchronize(t->ctx->stream);
    (void)hipFree(t->slots);
    (void)hipFree(t->keys);
    for (auto *p : t->aggv) (void)hipFree(p);
    (void)hipFree(t->d_aggv);
    (void)hipFree(t->first);
    (void)hipFree(t->counter);
    (void)hipFree(t->n_groups);
    delete t;
    return IGX_OK;
}

template <int KW>
static void launch_gb(igx_ctx *ctx, const GbArgs &a, const DevPreds &dp, uint32_t blocks, size_t lds) {
    hipLaunchKernelGGL(k_groupby<KW>, dim3(blocks), dim3(TB), lds, ctx->stream, a, dp);
}

extern "C" int igx_groupby_update(igx_table *t, const igx_col *cols, uint32_t ncols,
                                  const uint32_t *key_cols, const igx_pred *preds, uint32_t npreds,
                                  uint64_t nrows, uint64_t base_idx) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    if (nrows == 0) return IGX_OK;
    if (!cols || !key_cols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: null columns");
    GbArgs a{};
    // key words
    uint32_t w = 0;
    for (uint32_t k = 0; k < t->nkeys; ++k) {
        uint32_t ci = key_cols[k];
        if (ci >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: key column %u out of range", ci);
        const igx_col &c = cols[ci];
        if (c.width != t->key_widths[k])
            return igx_fail(ctx, IGX_EINVAL, "groupby_update: key column %u width %u != %u", k, c.width,
                            t->key_widths[k]);
        const uint8_t *p = static_cast<const uint8_t *>(c.ptr);
        const uint32_t nw = (c.width + 3) / 4;
        const bool x4 = (c.width % 16 == 0) && ((reinterpret_cast<uintptr_t>(p) & 15) == 0);
        for (uint32_t j = 0; j < nw; ++j, ++w) {
            a.kptr[w] = p;
            a.kwidth[w] = c.width;
            a.koff[w] = 4 * j;
            if (c.width == 1) a.kmode[w] = KM_U8;
            else if (c.width == 2) a.kmode[w] = KM_U16;
            else if (x4) a.kmode[w] = (j % 4 == 0) ? KM_X4 : KM_CONT;
            else a.kmode[w] = KM_U32;
        }
    }
    for (; w < KWMAX; ++w) a.kmode[w] = KM_ZERO;
    // x4 groups must fit inside the instantiated width
    for (uint32_t q = 0; q < (uint32_t)t->kw_inst; ++q)
        if (a.kmode[q] == KM_X4 && q + 3 >= (uint32_t)t->kw_inst)
            for (uint32_t r = q; r < (uint32_t)t->kw_inst; ++r) a.kmode[r] = KM_U32;
    // aggregates
    a.naggs = t->naggs;
    for (uint32_t x = 0; x < t->naggs; ++x) {
        const igx_agg &g = t->aggs[x];
        a.vcount[x] = g.kind == IGX_AGG_COUNT;
        if (!a.vcount[x]) {
            if (g.col >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: agg column out of range");
            a.vptr[x] = static_cast<const uint8_t *>(cols[g.col].ptr);
            a.vwidth[x] = cols[g.col].width;
            a.vsign[x] = cols[g.col].kind == IGX_KIND_INT;
            if (a.vwidth[x] != 1 && a.vwidth[x] != 2 && a.vwidth[x] != 4 && a.vwidth[x] != 8)
                return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: agg width %u", a.vwidth[x]);
            if (cols[g.col].kind == IGX_KIND_FLOAT)
                return igx_fail(ctx, IGX_ENOTSUP, "groupby_update: float sums are not supported");
        }
        if (g.cond_col != IGX_NO_COL) {
            if (g.cond_col >= ncols) return igx_fail(ctx, IGX_EINVAL, "groupby_update: cond column out of range");
            a.cptr[x] = static_cast<const uint8_t *>(cols[g.cond_col].ptr);
            a.cwidth[x] = cols[g.cond_col].width;
            a.cval[x] = g.cond_val;
        }
        a.aggs[x] = t->aggv[x];
    }
    DevPreds dp{};
    int rc = igx_build_preds(ctx, cols, ncols, preds, npreds, &dp);
    if (rc) return rc;
    a.valid = nullptr;
    a.n = nrows;
    a.base_idx = base_idx;
    a.slots = t->slots;
    a.keys = t->keys;
    a.key_stride_w = t->key_stride_w;
    a.first = t->first;
    a.counter = t->counter;
    a.err = t->counter + 1;
    a.mask = t->nslots - 1;
    a.cap_ids = (uint32_t)t->cap;
    a.max_probe = (uint32_t)std::min<uint64_t>(t->nslots, 1u << 20);
    // LDS staging: L entries x (8 first + 8 naggs + 4 tag) bytes, <= 48 KB
    uint32_t L = 2048;
    while (L > 64 && (size_t)L * (12 + 8 * t->naggs) > 48 * 1024) L >>= 1;
    a.lds_entries = L;
    const size_t lds = (size_t)L * (12 + 8 * t->naggs);
    const uint64_t want = (nrows + TB - 1) / TB;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ctx->num_cus * 3));
    switch (t->kw_inst) {
    case 2: launch_gb<2>(ctx, a, dp, blocks, lds); break;
    case 4: launch_gb<4>(ctx, a, dp, blocks, lds); break;
    case 6: launch_gb<6>(ctx, a, dp, blocks, lds); break;
    case 8: launch_gb<8>(ctx, a, dp, blocks, lds); break;
    case 12: launch_gb<12>(ctx, a, dp, blocks, lds); break;
    case 18: launch_gb<18>(ctx, a, dp, blocks, lds); break;
    case 24: launch_gb<24>(ctx, a, dp, blocks, lds); break;
    default: launch_gb<32>(ctx, a, dp, blocks, lds); break;
    }
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_groupby_finalize(igx_table *t, igx_table_view *view) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    hipLaunchKernelGGL(k_count, dim3(1), dim3(1), 0, ctx->stream, t->counter, (uint32_t)t->cap, t->n_groups);
    uint64_t *h;
    int rc = igx_pinned(ctx, 16, reinterpret_cast<void **>(&h));
    if (rc) return rc;
    IGX_HIP(ctx, hipMemcpyAsync(h, t->n_groups, 8, hipMemcpyDeviceToHost, ctx->stream));
    IGX_HIP(ctx, hipMemcpyAsync(reinterpret_cast<uint32_t *>(h) + 2, t->counter + 1, 4,
                                hipMemcpyDeviceToHost, ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t ng = h[0];
    const uint32_t err = reinterpret_cast<uint32_t *>(h)[2];
    if (view) {
        view->n_groups = ng;
        view->key_bytes = t->key_words * 4;
        view->key_stride = t->key_stride_w * 4;
        view->naggs = t->naggs;
        view->keys = reinterpret_cast<const uint8_t *>(t->keys);
        for (uint32_t x = 0; x < 16; ++x) view->aggs[x] = x < t->naggs ? t->aggv[x] : nullptr;
        view->first_idx = t->first;
        view->d_n_groups = t->n_groups;
    }
    if (err & 1) return igx_fail(ctx, IGX_ENOSPC, "groupby: more than %llu distinct keys", (unsigned long long)t->cap);
    if (err) return igx_fail(ctx, IGX_EIO, "groupby: table probe failure (err=%u)", err);
    return IGX_OK;
}

// ---------------------------------------------------------------------------------------
// materialise selected groups (the Stats rows of nextStats, tracer.go:186-219)
// ---------------------------------------------------------------------------------------
namespace {
__global__ void k_gather_rows(const uint32_t *__restrict__ keys, uint32_t key_stride_w, uint32_t key_words,
                              const uint64_t *const *__restrict__ aggs, uint32_t naggs,
                              const uint64_t *__restrict__ first, const uint32_t *__restrict__ idx,
                              const uint64_t *__restrict__ n_groups, uint64_t k, uint8_t *__restrict__ out) {
    const uint64_t r = blockIdx.x;
    if (r >= k) return;
    const uint32_t row_words = key_words + 2 * naggs + 2;
    uint32_t *o = reinterpret_cast<uint32_t *>(out) + r * row_words;
    const uint32_t g = idx[r];
    const bool ok = g < *n_groups;
    for (uint32_t w = threadIdx.x; w < row_words; w += blockDim.x) {
        uint32_t v = 0;
        if (ok) {
            if (w < key_words) v = keys[(uint64_t)g * key_stride_w + w];
            else if (w < key_words + 2 * naggs) {
                const uint32_t a = (w - key_words) >> 1;
                const uint64_t s = aggs[a][g];
                v = ((w - key_words) & 1) ? (uint32_t)(s >> 32) : (uint32_t)s;
            } else {
                const uint64_t f = first[g];
                v = ((w - key_words - 2 * naggs) & 1) ? (uint32_t)(f >> 32) : (uint32_t)f;
            }
        }
        o[w] = v;
    }
}
}  // namespace

extern "C" int igx_groupby_gather(igx_table *t, const uint32_t *idx, uint64_t k, uint8_t *out_rows) {
    if (!t) return IGX_EINVAL;
    igx_ctx *ctx = t->ctx;
    if (k == 0) return IGX_OK;
    if (!idx || !out_rows) return igx_fail(ctx, IGX_EINVAL, "groupby_gather: null argument");
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)k), dim3(64), 0, ctx->stream, t->keys, t->key_stride_w,
                       t->key_words, (const uint64_t *const *)t->d_aggv, t->naggs, t->first, idx,
                       t->n_groups, k, out_rows);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
