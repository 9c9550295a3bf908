/*
 * igx_oracle.c -- CPU restatement of Inspektor Gadget's event-aggregation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (`inspektor-gadget_amd/`) links or
 * calls this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it (as the checker / CPU baseline), never as the thing measured or shipped.
 *
 * The reference path is Go (+ eBPF C) and cannot be built in this image (no Go
 * toolchain), so this is a restatement, pinned by the reference's own
 * table tests re-encoded under tests/golden/ (see tests/test_oracle_golden.py).
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference repository root).
 *
 * Contents
 *   1. counter-based synthetic event generators (shared bit-exactly with the GPU
 *      generator kernels in csrc/k_gen.hip; not a reference algorithm)
 *   2. filter predicate evaluation        pkg/columns/filter/filter.go:187-325
 *   3. Go 1.19 sort.SliceStable restatement (stable_func / insertionSort_func /
 *      symMerge_func / rotate_func; stdlib, transliterated in SURVEY.md App. C) driven by
 *      getLessFunc                         pkg/columns/sort/sort.go:35-83,125-135
 *   4. keyed aggregation with first-occurrence ("Go map + BPF hash") semantics
 *      pkg/gadgets/top/tcp/tracer/bpf/tcptop.bpf.c:33-110
 *      pkg/gadgets/top/file/tracer/bpf/filetop.bpf.c:39-94
 *      pkg/gadgets/top/block-io/tracer/bpf/biotop.bpf.c:85-130
 *      pkg/gadgets/trace/network/tracer/bpf/graph.c:102-114 (distinct insert)
 *   5. log2 latency histograms           pkg/gadgets/profile/block-io/tracer/bpf/biolatency.bpf.c:100-154
 *                                        pkg/gadgets/profile/block-io/tracer/bpf/bits.bpf.h:8-29
 *   6. the top-tcp CPU path as the reference runs it (map group-by -> SortEntries ->
 *      truncate), used as the CPU baseline ("port") in bench.py
 *      pkg/gadgets/top/tcp/tracer/tracer.go:147-253, pkg/gadgets/top/top.go:39-41
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;
typedef int64_t i64;

/* ------------------------------------------------------------------------------------
 * 1. Synthetic generators (counter-based: event i's fields depend only on (seed, i)).
 * ---------------------------------------------------------------------------------- */
static inline u64 sm64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
/* stream-separated counter RNG; identical formula in csrc/k_gen.hip */
static inline u64 rnd(u64 seed, u64 stream, u64 i) {
    return sm64(sm64(seed ^ (stream * 0xD1B54A32D192ED03ull)) ^ (i * 0x9E3779B97F4A7C15ull));
}
/* lower_bound over u63 CDF thresholds (last threshold == 1<<63) */
static inline u64 cdf_pick(const u64 *cdf, u64 n, u64 r) {
    u64 u = r >> 1, lo = 0, hi = n - 1;
    while (lo < hi) {
        u64 mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* C2 top-tcp stream.  Key universe of G keys per rank (ingest-partitioned), Zipf over
 * key rank via cdf.  Fields mirror ip_key_t (tcptop.h:8-17) in SoA form. */
void or_gen_tcp(u64 seed, u64 rank, u64 G, u64 permA, u64 permB, const u64 *cdf,
                u64 base, u64 n, u8 *saddr, u8 *daddr, u64 *mntns, u32 *pid, u8 *comm,
                u16 *lport, u16 *dport, u16 *family, u32 *size, u8 *dir) {
    static const char *names[8] = {"nginx", "curl", "postgres", "redis-server",
                                   "java", "python3", "envoy", "node"};
    static const u16 ports[8] = {80, 443, 8080, 53, 3306, 6379, 5432, 9092};
    for (u64 j = 0; j < n; j++) {
        u64 i = base + j;
        u64 r = cdf_pick(cdf, G, rnd(seed, 1, i));
        u64 kid = (r * permA + permB) % G;            /* scrambled local key id */
        u64 gk = kid * 64 + rank;                       /* globally unique key id */
        u64 p = 1000 + (gk >> 4);                        /* 16 keys per pid */
        u64 hp = sm64(p ^ 0x5EED);
        u64 hk = sm64(gk ^ 0xFACE);
        u8 *sa = saddr + 16 * j, *da = daddr + 16 * j, *cm = comm + 16 * j;
        memset(sa, 0, 16); memset(da, 0, 16); memset(cm, 0, 16);
        u16 fam = (hk % 10 == 0) ? 10 : 2;
        u8 s4[4] = {10, 0, (u8)(hp >> 8), (u8)hp};
        u8 d4[4] = {10, (u8)(1 + ((hk >> 40) & 7)), (u8)(hk >> 16), (u8)(hk >> 24)};
        if (fam == 2) {
            memcpy(sa, s4, 4); memcpy(da, d4, 4);
        } else {
            sa[10] = sa[11] = 0xff; memcpy(sa + 12, s4, 4);
            da[10] = da[11] = 0xff; memcpy(da + 12, d4, 4);
        }
        mntns[j] = 4026531840ull + ((hp >> 20) & 63);
        pid[j] = (u32)p;
        const char *nm = names[(hp >> 32) & 7];
        size_t L = strlen(nm);
        memcpy(cm, nm, L);
        cm[L] = (u8)('a' + ((hp >> 40) & 31) % 26);   /* 8 names x 26 suffixes */
        lport[j] = (u16)(1024 + (gk & 15) + 16 * ((hk >> 8) % 2048));
        dport[j] = ports[(hk >> 48) & 7];
        family[j] = fam;
        u64 e = rnd(seed, 2, i);
        dir[j] = (u8)(e & 1);
        size[j] = (u32)(1 + (e >> 8) % 65535);
    }
}

/* C1 trace-open stream (pkg/gadgets/trace/open/types/types.go:22-33 fields).  comm is
 * drawn from a 64-name dictionary with Zipf s=1.0 via comm_cdf (64 thresholds). */
void or_gen_open(u64 seed, const u64 *comm_cdf, u64 base, u64 n, u32 *pid, u32 *uid,
                 u64 *mntns, u8 *comm, i64 *ret, i64 *fd, i64 *err, u32 *path_id) {
    for (u64 j = 0; j < n; j++) {
        u64 i = base + j;
        u64 a = rnd(seed, 1, i), b = rnd(seed, 2, i), c = rnd(seed, 3, i);
        pid[j] = (u32)(1 + a % 32767);
        u64 ur = (a >> 32) % 11;
        uid[j] = ur == 0 ? 0 : (u32)(999 + ur);
        mntns[j] = 4026531840ull + ((a >> 40) & 15);
        u64 k = cdf_pick(comm_cdf, 64, b);
        u8 *cm = comm + 16 * j;
        memset(cm, 0, 16);
        /* name = "proc" + 2 hex-ish letters, <= 15 chars, no NUL */
        static const char *stem[8] = {"bash", "sshd", "containerd", "kubelet", "cat",
                                      "systemd-journal", "runc", "ls"};
        const char *s = stem[k & 7];
        size_t L = strlen(s);
        if (L > 13) L = 13;
        memcpy(cm, s, L);
        cm[L] = (u8)('a' + (k >> 3));
        i64 r;
        if (c % 10 == 0) r = -(i64)(1 + (c >> 8) % 13);
        else r = (i64)(3 + (c >> 8) % 1021);
        ret[j] = r;
        fd[j] = r >= 0 ? r : 0;
        err[j] = r < 0 ? -r : 0;
        path_id[j] = (u32)((c >> 32) & 4095);
    }
}

/* C3 block-io completions: dev (MKDEV(8, 16k), biolatency.h:8-11), container dictionary
 * id, delta_ns from a discretised lognormal quantile table q (nq+1 entries). */
void or_gen_bio(u64 seed, const u64 *q, u64 nq, u64 base, u64 n, u32 *dev, u32 *cont,
                u64 *delta) {
    for (u64 j = 0; j < n; j++) {
        u64 i = base + j;
        u64 a = rnd(seed, 1, i), b = rnd(seed, 2, i);
        dev[j] = (8u << 20) | (u32)(16 * (a & 15));
        cont[j] = (u32)((a >> 8) & 255);
        u64 idx = (b >> 32) % nq;
        u64 lo = q[idx], hi = q[idx + 1];
        delta[j] = lo + (b & 0xffffffffull) % (hi - lo + 1);
    }
}

/* C4 network events (advisor.go:277-320 inputs as dictionary ids). */
void or_gen_np(u64 seed, u64 nsrc, u64 npeer_total, u64 base, u64 n, u32 *src, u32 *peer,
               u16 *port, u8 *pkt, u8 *typ, u8 *proto, u32 *hostip, u32 *raddr) {
    static const u16 ports[8] = {80, 443, 53, 8080, 5432, 6379, 9090, 3000};
    for (u64 j = 0; j < n; j++) {
        u64 i = base + j;
        u64 a = rnd(seed, 1, i), b = rnd(seed, 2, i), c = rnd(seed, 3, i);
        u32 s = (u32)(a % nsrc);
        u64 slot = (a >> 32) & 63;                        /* one of 64 peers of src */
        u32 pe = (u32)(sm64((u64)s * 64 + slot) % npeer_total);
        src[j] = s;
        peer[j] = pe;
        port[j] = ports[(b >> 8) & 7];
        u64 pk = b % 100;
        pkt[j] = pk < 60 ? 4 /*OUTGOING*/ : (pk < 95 ? 0 /*HOST*/ : 1 /*BROADCAST*/);
        typ[j] = (c % 100 == 0) ? 1 : 0;                  /* 0 = normal */
        proto[j] = (u8)((c >> 8) % 3 == 0 ? 17 : 6);
        hostip[j] = 0x0a000000u | (u32)(s & 0xffff);
        raddr[j] = ((c >> 16) % 100 == 0) ? hostip[j] : (0x0a600000u | (pe & 0xfffff));
    }
}

/* C5 top-file stream: key file_id{inode,dev,pid,tid} (filetop.h:13-18). */
void or_gen_file(u64 seed, u64 rank, u64 G, u64 permA, u64 permB, const u64 *cdf, u64 base,
                 u64 n, u64 *inode, u32 *dev, u32 *pid, u32 *tid, u8 *op, u32 *count) {
    for (u64 j = 0; j < n; j++) {
        u64 i = base + j;
        u64 r = cdf_pick(cdf, G, rnd(seed, 1, i));
        u64 kid = (r * permA + permB) % G;
        u64 gk = kid * 64 + rank;
        u64 h = sm64(gk ^ 0xF11E);
        inode[j] = sm64(gk ^ 0x9A7B);                     /* hash64(path) stand-in */
        dev[j] = (u32)((8u << 20) | (u32)(h & 15));
        pid[j] = (u32)(100 + (gk >> 3));
        tid[j] = pid[j] + (u32)(gk & 7);
        u64 e = rnd(seed, 2, i);
        op[j] = (u8)(e & 1);                               /* 0 READ, 1 WRITE */
        count[j] = (u32)(1 + (e >> 8) % ((1u << 20) - 1));
    }
}

/* ------------------------------------------------------------------------------------
 * 2. Filter predicates -- getComparisonFuncForComparisonType (filter.go:236-263):
 *    result = (field OP ref) != negate; FilterSpecs.MatchAll (filter.go:266-273).
 * ---------------------------------------------------------------------------------- */
enum { OR_INT = 0, OR_UINT = 1, OR_FLOAT = 2, OR_BYTES = 3 };
enum { OR_EQ = 0, OR_LT = 2, OR_LE = 3, OR_GT = 4, OR_GE = 5 };

typedef struct {
    const void *ptr;  /* column base */
    u32 width;        /* bytes per row */
    u32 kind;         /* OR_INT / OR_UINT / OR_FLOAT / OR_BYTES */
    u32 op;           /* comparison */
    u32 negate;
    const u8 *ref;    /* reference value, `width` bytes (already Convert()-ed) */
} or_pred;

static int cmp_field(const or_pred *p, u64 row) {
    const u8 *f = (const u8 *)p->ptr + (u64)p->width * row;
    if (p->kind == OR_BYTES) {
        int c = memcmp(f, p->ref, p->width);   /* Go string compare == bytewise unsigned */
        return c < 0 ? -1 : (c > 0);
    }
    if (p->kind == OR_FLOAT) {
        double a, b;
        if (p->width == 4) { float x, y; memcpy(&x, f, 4); memcpy(&y, p->ref, 4); a = x; b = y; }
        else { memcpy(&a, f, 8); memcpy(&b, p->ref, 8); }
        if (a != a || b != b) return 2;          /* unordered: every comparison false */
        return a < b ? -1 : (a > b);
    }
    if (p->kind == OR_INT) {
        i64 a = 0, b = 0;
        switch (p->width) {
        case 1: a = *(const int8_t *)f; b = *(const int8_t *)p->ref; break;
        case 2: { int16_t x, y; memcpy(&x, f, 2); memcpy(&y, p->ref, 2); a = x; b = y; } break;
        case 4: { int32_t x, y; memcpy(&x, f, 4); memcpy(&y, p->ref, 4); a = x; b = y; } break;
        default: memcpy(&a, f, 8); memcpy(&b, p->ref, 8);
        }
        return a < b ? -1 : (a > b);
    }
    u64 a = 0, b = 0;
    memcpy(&a, f, p->width); memcpy(&b, p->ref, p->width);
    return a < b ? -1 : (a > b);
}

static int pred_match(const or_pred *p, u64 row) {
    int c = cmp_field(p, row), r;
    if (c == 2) r = 0;
    else switch (p->op) {
        case OR_EQ: r = c == 0; break;
        case OR_LT: r = c < 0; break;
        case OR_LE: r = c <= 0; break;
        case OR_GT: r = c > 0; break;
        case OR_GE: r = c >= 0; break;
        default: r = 0;
    }
    return r != (int)p->negate;
}

/* FilterEntries (filter.go:294-325): order-preserving selection; nil rows (valid[i]==0)
 * are skipped.  Returns count written to out_idx. */
u64 or_filter(const or_pred *preds, u32 npred, const u8 *valid, u64 n, u32 *out_idx) {
    u64 k = 0;
    for (u64 i = 0; i < n; i++) {
        if (valid && !valid[i]) continue;
        int ok = 1;
        for (u32 p = 0; p < npred && ok; p++) ok = pred_match(&preds[p], i);
        if (ok) out_idx[k++] = (u32)i;
    }
    return k;
}

/* ------------------------------------------------------------------------------------
 * 3. Go 1.19 sort.SliceStable restatement.  `less(i,j)` and `swap` act on the live
 *    permutation `perm` (an array of row ids, the analogue of []*T).
 * ---------------------------------------------------------------------------------- */
typedef struct {
    const void *ptr;   /* column base, indexed by row id */
    u32 width, kind, desc;
} or_sortkey;

typedef struct {
    u32 *perm;
    const u8 *valid;     /* nil entries (valid==0) sort last (sort.go:127-132) */
    const or_sortkey *key;
} less_ctx;

static int col_lt(const or_sortkey *k, u32 a, u32 b) {
    const u8 *fa = (const u8 *)k->ptr + (u64)k->width * a;
    const u8 *fb = (const u8 *)k->ptr + (u64)k->width * b;
    if (k->kind == OR_BYTES) return memcmp(fa, fb, k->width) < 0;
    if (k->kind == OR_FLOAT) {
        if (k->width == 4) { float x, y; memcpy(&x, fa, 4); memcpy(&y, fb, 4); return x < y; }
        double x, y; memcpy(&x, fa, 8); memcpy(&y, fb, 8); return x < y;
    }
    if (k->kind == OR_INT) {
        i64 x = 0, y = 0;
        switch (k->width) {
        case 1: x = *(const int8_t *)fa; y = *(const int8_t *)fb; break;
        case 2: { int16_t p, q; memcpy(&p, fa, 2); memcpy(&q, fb, 2); x = p; y = q; } break;
        case 4: { int32_t p, q; memcpy(&p, fa, 4); memcpy(&q, fb, 4); x = p; y = q; } break;
        default: memcpy(&x, fa, 8); memcpy(&y, fb, 8);
        }
        return x < y;
    }
    u64 x = 0, y = 0;
    memcpy(&x, fa, k->width); memcpy(&y, fb, k->width);
    return x < y;
}

/* getLessFunc (sort.go:125-135): !(a<b) != order, OrderAsc=true (types.go:37-38) */
static inline int go_less(const less_ctx *c, u64 i, u64 j) {
    u32 a = c->perm[i], b = c->perm[j];
    if (c->valid && !c->valid[a]) return 0;
    if (c->valid && !c->valid[b]) return 1;
    int lt = col_lt(c->key, a, b);
    int order_asc = !c->key->desc;
    return (!lt) != order_asc;
}
static inline void go_swap(const less_ctx *c, u64 i, u64 j) {
    u32 t = c->perm[i]; c->perm[i] = c->perm[j]; c->perm[j] = t;
}
static void insertion_sort(const less_ctx *c, u64 a, u64 b) {
    for (u64 i = a + 1; i < b; i++)
        for (u64 j = i; j > a && go_less(c, j, j - 1); j--) go_swap(c, j, j - 1);
}
static void swap_range(const less_ctx *c, u64 a, u64 b, u64 n) {
    for (u64 i = 0; i < n; i++) go_swap(c, a + i, b + i);
}
static void rotate(const less_ctx *c, u64 a, u64 m, u64 b) {
    u64 i = m - a, j = b - m;
    while (i != j) {
        if (i > j) { swap_range(c, m - i, m, j); i -= j; }
        else { swap_range(c, m - i, m + j - i, i); j -= i; }
    }
    swap_range(c, m - i, m, i);
}
static void sym_merge(const less_ctx *c, u64 a, u64 m, u64 b) {
    if (m - a == 1) {
        u64 i = m, j = b;
        while (i < j) { u64 h = (i + j) >> 1; if (go_less(c, h, a)) i = h + 1; else j = h; }
        for (u64 k = a; k + 1 < i; k++) go_swap(c, k, k + 1);
        return;
    }
    if (b - m == 1) {
        u64 i = a, j = m;
        while (i < j) { u64 h = (i + j) >> 1; if (!go_less(c, m, h)) i = h + 1; else j = h; }
        for (u64 k = m; k > i; k--) go_swap(c, k, k - 1);
        return;
    }
    u64 mid = (a + b) >> 1, n = mid + m, start, r;
    if (m > mid) { start = n - b; r = mid; } else { start = a; r = m; }
    u64 p = n - 1;
    while (start < r) {
        u64 cc = (start + r) >> 1;
        if (!go_less(c, p - cc, cc)) start = cc + 1; else r = cc;
    }
    u64 end = n - start;
    if (start < m && m < end) rotate(c, start, m, end);
    if (a < start && start < mid) sym_merge(c, a, start, mid);
    if (mid < end && end < b) sym_merge(c, mid, end, b);
}
static void go_stable(const less_ctx *c, u64 n) {
    u64 bs = 20, a = 0, b = bs;
    while (b <= n) { insertion_sort(c, a, b); a = b; b += bs; }
    insertion_sort(c, a, n);
    while (bs < n) {
        a = 0; b = 2 * bs;
        while (b <= n) { sym_merge(c, a, a + bs, b); a = b; b += 2 * bs; }
        if (a + bs < n) sym_merge(c, a, a + bs, n);
        bs *= 2;
    }
}

/* ColumnSorterCollection.Sort (sort.go:35-83): keys given in sortBy order (first =
 * highest priority); one stable pass per key, last key first (Prepare reverses, :91). */
void or_sort_entries(u32 *perm, u64 n, const u8 *valid, const or_sortkey *keys, u32 nkeys) {
    if (n == 0) return;
    for (int k = (int)nkeys - 1; k >= 0; k--) {
        less_ctx c = {perm, valid, &keys[k]};
        go_stable(&c, n);
    }
}

/* ------------------------------------------------------------------------------------
 * 4. Keyed aggregation (Go-map / BPF-hash semantics, canonical first-occurrence order).
 *    Rows are (packed key bytes, aggregate inputs).  Each aggregate is
 *      COUNT  (cond?): += 1
 *      SUM    (cond?): += value
 *    wrapped to out_width bytes (group.go:137-151 SetInt wraps; BPF u32 io++ wraps).
 *    Groups are emitted in first-occurrence order with their first row index.
 * ---------------------------------------------------------------------------------- */
enum { OR_AGG_COUNT = 0, OR_AGG_SUM = 1 };
typedef struct {
    u32 kind;
    u32 val_width;       /* bytes of the value column (SUM) */
    const void *val;     /* value column (SUM) */
    u32 cond_width;      /* 0 = unconditional */
    const void *cond;    /* condition column */
    u64 cond_val;        /* row counts iff cond == cond_val */
    u32 out_width;       /* wrap width in bytes (1,2,4,8) */
    u32 val_signed;      /* SUM over a signed column: values sign-extend (Go int64 math) */
    u64 div;             /* > 1: add val / div per event (biotop.bpf.c:98,119 `us += delta/1000`) */
} or_agg;

static inline u64 ld_u(const void *p, u32 w, u64 row) {
    const u8 *q = (const u8 *)p + (u64)w * row;
    u64 v = 0; memcpy(&v, q, w); return v;
}
static inline u64 fnv(const u8 *k, u32 n) {
    u64 h = 1469598103934665603ull;
    for (u32 i = 0; i < n; i++) { h ^= k[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

typedef struct {
    u64 cap, mask, n;
    u32 kb;
    u32 *slot;          /* group id + 1, 0 = empty */
    u64 *hash;
} or_map;

static int map_init(or_map *m, u64 expect, u32 kb) {
    u64 cap = 16;
    while (cap < expect * 2) cap <<= 1;
    m->cap = cap; m->mask = cap - 1; m->n = 0; m->kb = kb;
    m->slot = (u32 *)calloc(cap, sizeof(u32));
    m->hash = (u64 *)malloc(cap * sizeof(u64));
    return m->slot && m->hash ? 0 : -1;
}
static void map_free(or_map *m) { free(m->slot); free(m->hash); }

/* returns group id; *is_new set when inserted. keys_out grows as groups are added. */
static u64 map_find_or_insert(or_map *m, const u8 *key, u8 *keys_out, int *is_new) {
    u64 h = fnv(key, m->kb), s = h & m->mask;
    for (;;) {
        u32 g = m->slot[s];
        if (!g) {
            u64 id = m->n++;
            m->slot[s] = (u32)(id + 1);
            m->hash[s] = h;
            memcpy(keys_out + (u64)m->kb * id, key, m->kb);
            *is_new = 1;
            return id;
        }
        if (m->hash[s] == h && memcmp(keys_out + (u64)m->kb * (g - 1), key, m->kb) == 0) {
            *is_new = 0;
            return g - 1;
        }
        s = (s + 1) & m->mask;
    }
}

/* Generic group-by over rows [0,n) of a packed key matrix `keys` (n x kb bytes).  Rows
 * with valid==0 are skipped (nil / filtered).  Outputs: out_keys (G x kb), out_aggs
 * (naggs x maxG, u64 each, column-major), out_first (row index).  Returns G, or
 * (u64)-1 if maxG is exceeded. */
u64 or_groupby(const u8 *keys, u32 kb, u64 n, const u8 *valid, const or_agg *aggs,
               u32 naggs, u64 base_idx, u64 maxG, u8 *out_keys, u64 *out_aggs,
               u64 *out_first) {
    or_map m;
    if (map_init(&m, maxG, kb)) return (u64)-1;
    for (u64 i = 0; i < n; i++) {
        if (valid && !valid[i]) continue;
        int is_new;
        if (m.n >= maxG) {
            /* probe only: a new key would overflow */
        }
        u64 g = map_find_or_insert(&m, keys + (u64)kb * i, out_keys, &is_new);
        if (g >= maxG) { map_free(&m); return (u64)-1; }
        if (is_new) {
            out_first[g] = base_idx + i;
            for (u32 a = 0; a < naggs; a++) out_aggs[(u64)a * maxG + g] = 0;
        }
        for (u32 a = 0; a < naggs; a++) {
            const or_agg *A = &aggs[a];
            if (A->cond_width && ld_u(A->cond, A->cond_width, i) != A->cond_val) continue;
            u64 add = A->kind == OR_AGG_COUNT ? 1 : ld_u(A->val, A->val_width, i);
            if (A->kind != OR_AGG_COUNT && A->val_signed && A->val_width < 8) {
                const u32 sh = 64 - 8 * A->val_width;
                add = (u64)(((int64_t)(add << sh)) >> sh);
            }
            if (A->kind != OR_AGG_COUNT && A->div > 1) add /= A->div;
            u64 *dst = &out_aggs[(u64)a * maxG + g];
            u64 v = *dst + add;
            if (A->out_width < 8) v &= (1ull << (8 * A->out_width)) - 1;
            *dst = v;
        }
    }
    u64 G = m.n;
    map_free(&m);
    return G;
}

/* ------------------------------------------------------------------------------------
 * 5. log2 histograms -- bits.bpf.h:8-29 (log2 / log2l), biolatency.bpf.c:114-149:
 *    delta<0 -> skipped; v = delta / divisor (1000 usecs, 1e6 msecs); slot = log2l(v),
 *    clamped to MAX_SLOTS-1 = 26; slots are u32 (__sync_fetch_and_add wraps).
 * ---------------------------------------------------------------------------------- */
static inline u64 bpf_log2(u32 v) {
    u32 shift, r;
    r = (v > 0xFFFF) << 4; v >>= r;
    shift = (v > 0xFF) << 3; v >>= shift; r |= shift;
    shift = (v > 0xF) << 2; v >>= shift; r |= shift;
    shift = (v > 0x3) << 1; v >>= shift; r |= shift;
    r |= (v >> 1);
    return r;
}
u64 or_log2l(u64 v) {
    u32 hi = (u32)(v >> 32);
    if (hi) return bpf_log2(hi) + 32;
    return bpf_log2((u32)v);
}

/* key = dev_index(dev) * ncont + cont; dev_index via the sorted dev table `devs`.
 * hist is nkeys x nslots u32, accumulated (not cleared). delta is s64 (signed). */
void or_hist_log2(const u32 *dev, const u32 *cont, const i64 *delta, u64 n, const u32 *devs,
                  u32 ndev, u32 ncont, u64 divisor, u32 nslots, u32 *hist) {
    for (u64 i = 0; i < n; i++) {
        i64 d = delta[i];
        if (d < 0) continue;
        u32 di = 0;
        if (ndev) {                                  /* ndev == 0: one key (the shipped gadget) */
            while (di < ndev && devs[di] != dev[i]) di++;
            if (di == ndev) continue;                /* unknown device: not counted */
        }
        if (cont && cont[i] >= ncont) continue;      /* unknown container: not counted */
        u64 v = (u64)d / divisor;
        u64 slot = or_log2l(v);
        if (slot >= nslots) slot = nslots - 1;
        u64 key = (u64)di * ncont + (cont ? cont[i] : 0);
        hist[key * nslots + slot] += 1;
    }
}

/* ------------------------------------------------------------------------------------
 * 6. top-tcp CPU path as the reference runs it, for timing (the "port" CPU baseline):
 *    probe_ip per event (tcptop.bpf.c:83-107: build ip_key_t, lookup-or-insert, +=),
 *    nextStats (tracer.go:147-226: one Stats per map entry), top.SortStats ->
 *    SortEntries(["-sent","-recv"]) (top.go:39-41, sort.go:35-83), truncate to
 *    max-rows (tracer.go:249-253).  Canonical pre-sort order = first occurrence.
 *    Returns the number of groups; out_* receive the first `k` sorted rows.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    u8 saddr[16], daddr[16];
    u64 mntns;
    u32 pid;
    u8 name[16];
    u16 lport, dport, family;
    u16 pad;
} ip_key_t;  /* 72 bytes; tcptop.h:8-17 */

u64 or_top_tcp(const u8 *saddr, const u8 *daddr, const u64 *mntns, const u32 *pid,
               const u8 *comm, const u16 *lport, const u16 *dport, const u16 *family,
               const u32 *size, const u8 *dir, u64 n, u64 base_idx, u64 maxG, u32 k,
               u8 *out_keys /* k x 72 */, u64 *out_sent, u64 *out_recv, u64 *out_first) {
    or_map m;
    if (map_init(&m, maxG, sizeof(ip_key_t))) return (u64)-1;
    u8 *keys = (u8 *)malloc(maxG * sizeof(ip_key_t));
    u64 *sent = (u64 *)malloc(maxG * 8), *recv = (u64 *)malloc(maxG * 8);
    u64 *first = (u64 *)malloc(maxG * 8);
    ip_key_t key;
    for (u64 i = 0; i < n; i++) {
        /* ig_toptcp_clean (tcp_cleanup_rbuf, int copied): `if (copied <= 0) return 0;`
         * before probe_ip, tcptop.bpf.c:124-130; sends have no such check (:112-116), so a
         * zero-size send still creates its group */
        if (dir[i] == 1 && (int32_t)size[i] <= 0) continue;
        if (family[i] != 2 && family[i] != 10) continue;   /* tcptop.bpf.c:54-55 */
        memset(&key, 0, sizeof key);
        memcpy(key.saddr, saddr + 16 * i, 16);
        memcpy(key.daddr, daddr + 16 * i, 16);
        key.mntns = mntns[i]; key.pid = pid[i];
        memcpy(key.name, comm + 16 * i, 16);
        key.lport = lport[i]; key.dport = dport[i]; key.family = family[i];
        int is_new;
        u64 g = map_find_or_insert(&m, (const u8 *)&key, keys, &is_new);
        if (g >= maxG) { g = (u64)-1; break; }
        if (is_new) { sent[g] = recv[g] = 0; first[g] = base_idx + i; }
        if (dir[i]) recv[g] += size[i]; else sent[g] += size[i];
    }
    u64 G = m.n;
    map_free(&m);
    /* []*Stats in canonical order, then SortEntries(-sent,-recv) */
    u32 *perm = (u32 *)malloc((G ? G : 1) * sizeof(u32));
    for (u64 g = 0; g < G; g++) perm[g] = (u32)g;
    or_sortkey ks[2] = {{sent, 8, OR_UINT, 1}, {recv, 8, OR_UINT, 1}};
    or_sort_entries(perm, G, NULL, ks, 2);
    for (u32 r = 0; r < k && r < G; r++) {
        u32 g = perm[r];
        memcpy(out_keys + 72ull * r, keys + 72ull * g, 72);
        out_sent[r] = sent[g]; out_recv[r] = recv[g]; out_first[r] = first[g];
    }
    free(perm); free(keys); free(sent); free(recv); free(first);
    return G;
}

/* ------------------------------------------------------------------------------------
 * 7. All-cores CPU baselines (bench.py cpu_baseline, SURVEY.md §8(d) "all host cores with
 *    the C++ restatement, which is fair").  Same results as the single-thread paths above:
 *      phase 1  each thread scans a contiguous slice of the events, builds each key and
 *               appends the event index to bucket[thread][owner], owner = hash(key) mod T
 *      phase 2  thread j aggregates every event of owner j in global index order (so the
 *               first index it sees for a key is the key's first occurrence)
 *      phase 3  thread j sorts its groups (first-occurrence order) with the Go SliceStable
 *               restatement and keeps the first k
 *      merge    the T x k candidates, in first-occurrence order, sorted once more: equal
 *               to sorting every group, since the sort order is a total order on
 *               (keys, position) under the closed form
 * ---------------------------------------------------------------------------------- */
#include <pthread.h>

typedef struct {
    u64 *first;           /* per group */
    u64 *agg;             /* naggs x cap, group-major rows of naggs */
    u8 *keys;
    u64 cap;
} mt_groups;

typedef struct mt_job mt_job;
struct mt_job {
    /* key source: packed keys (kb bytes per row) or the top-tcp columns (ip_key_t) */
    const u8 *keys;
    u32 kb;
    const u8 *saddr, *daddr, *comm;
    const u64 *mntns;
    const u32 *pid;
    const u16 *lport, *dport, *family;
    const u32 *tcp_size;  /* top tcp: the receive probe's `copied <= 0` drop (with tcp_dir) */
    const u8 *tcp_dir;
    const u8 *valid;
    const or_agg *aggs;
    u32 naggs;
    u64 n, base_idx;
    u32 T;
    const u32 *sort_agg, *sort_desc;
    u32 nsort, k;
    pthread_barrier_t bar;
    u32 **bucket;         /* T x T arrays of event indices */
    u64 *bcnt, *bcap;     /* T x T */
    u64 *G;               /* groups per owner */
    u64 *cand_first;      /* T x k */
    u64 *cand_agg;        /* T x k x naggs */
    u64 *cand_n;          /* per owner */
    u64 *csum;            /* per owner: sum of group_csum over its groups (top tcp only) */
    int want_csum;
    int oom;
};

static inline u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* Order-independent fingerprint of one top-tcp group: FNV-1a-64 over the key fields in
 * ip_key_t order without padding (saddr 16, daddr 16, mntns 8, pid 4, comm 16, lport 2,
 * dport 2, family 2 = 66 bytes), xor sent/recv/first times odd constants, splitmix64
 * finalised.  The full-table checksum is the u64 sum over groups (tests/test_gpu_fullsize.py
 * computes the same from the device table). */
static u64 group_csum(const ip_key_t *k, u64 sent, u64 recv, u64 first) {
    u8 b[66];
    memcpy(b, k->saddr, 16); memcpy(b + 16, k->daddr, 16); memcpy(b + 32, &k->mntns, 8);
    memcpy(b + 40, &k->pid, 4); memcpy(b + 44, k->name, 16); memcpy(b + 60, &k->lport, 2);
    memcpy(b + 62, &k->dport, 2); memcpy(b + 64, &k->family, 2);
    u64 h = 14695981039346656037ull;
    for (int i = 0; i < 66; i++) { h ^= b[i]; h *= 1099511628211ull; }
    return mix64(h ^ (sent * 0x9E3779B97F4A7C15ull) ^ (recv * 0xC2B2AE3D27D4EB4Full) ^ (first * 0x165667B19E3779F9ull));
}

/* Order-independent fingerprint of one generic group: FNV-1a-64 over the packed key (kb
 * bytes, the device's layout: every column padded to 4 B), then the first index and each
 * aggregate folded in through splitmix64.  The full-table checksum is the u64 sum over groups
 * (oracle.group_checksum is the numpy twin applied to the device table). */
static u64 group_csum_generic(const u8 *key, u32 kb, const u64 *agg, u32 na, u64 first) {
    u64 h = 14695981039346656037ull;
    for (u32 i = 0; i < kb; i++) { h ^= key[i]; h *= 1099511628211ull; }
    u64 z = h ^ (first * 0x165667B19E3779F9ull);
    for (u32 a = 0; a < na; a++) z = mix64(z ^ (agg[a] * 0x9E3779B97F4A7C15ull));
    return mix64(z);
}

typedef struct { mt_job *job; u32 t; } mt_arg;

static inline void mt_key(const mt_job *J, u64 i, u8 *buf) {
    if (J->keys) { memcpy(buf, J->keys + (u64)J->kb * i, J->kb); return; }
    ip_key_t *k = (ip_key_t *)buf;
    memset(k, 0, sizeof *k);
    memcpy(k->saddr, J->saddr + 16 * i, 16);
    memcpy(k->daddr, J->daddr + 16 * i, 16);
    k->mntns = J->mntns[i]; k->pid = J->pid[i];
    memcpy(k->name, J->comm + 16 * i, 16);
    k->lport = J->lport[i]; k->dport = J->dport[i]; k->family = J->family[i];
}

static inline int mt_keep(const mt_job *J, u64 i) {
    if (J->valid && !J->valid[i]) return 0;
    if (J->tcp_dir && J->tcp_dir[i] == 1 && (int32_t)J->tcp_size[i] <= 0) return 0;   /* tcptop.bpf.c:127-128 */
    if (J->family && J->family[i] != 2 && J->family[i] != 10) return 0;   /* tcptop.bpf.c:54-55 */
    return 1;
}

static int mt_push(mt_job *J, u64 b, u32 v) {
    if (J->bcnt[b] == J->bcap[b]) {
        u64 nc = J->bcap[b] ? 2 * J->bcap[b] : 4096;
        u32 *p = (u32 *)realloc(J->bucket[b], nc * 4);
        if (!p) return -1;
        J->bucket[b] = p;
        J->bcap[b] = nc;
    }
    J->bucket[b][J->bcnt[b]++] = v;
    return 0;
}

/* growing map: slot -> group id + 1, rehash from the stored hash */
static int mt_grow(or_map *m) {
    u64 cap = m->cap * 2;
    u32 *slot = (u32 *)calloc(cap, 4);
    u64 *hash = (u64 *)malloc(cap * 8);
    if (!slot || !hash) { free(slot); free(hash); return -1; }
    for (u64 s = 0; s < m->cap; s++) {
        if (!m->slot[s]) continue;
        u64 d = m->hash[s] & (cap - 1);
        while (slot[d]) d = (d + 1) & (cap - 1);
        slot[d] = m->slot[s];
        hash[d] = m->hash[s];
    }
    free(m->slot); free(m->hash);
    m->slot = slot; m->hash = hash; m->cap = cap; m->mask = cap - 1;
    return 0;
}

static int mt_groups_fit(mt_groups *g, u64 need, u32 kb, u32 naggs) {
    if (need <= g->cap) return 0;
    u64 nc = g->cap ? 2 * g->cap : 1 << 16;
    while (nc < need) nc *= 2;
    u8 *k = (u8 *)realloc(g->keys, nc * kb);
    if (k) g->keys = k;
    u64 *f = (u64 *)realloc(g->first, nc * 8);
    if (f) g->first = f;
    u64 *a = (u64 *)realloc(g->agg, nc * 8 * (naggs ? naggs : 1));
    if (a) g->agg = a;
    if (!k || !f || !a) return -1;
    g->cap = nc;
    return 0;
}

static void *mt_worker(void *p) {
    mt_arg *A = (mt_arg *)p;
    mt_job *J = A->job;
    const u32 T = J->T, t = A->t, kb = J->keys ? J->kb : (u32)sizeof(ip_key_t), na = J->naggs;
    u8 buf[256];
    /* phase 1: partition this thread's slice by owner */
    const u64 lo = J->n * t / T, hi = J->n * (t + 1) / T;
    for (u64 i = lo; i < hi; i++) {
        if (!mt_keep(J, i)) continue;
        mt_key(J, i, buf);
        const u64 h = fnv(buf, kb);
        if (mt_push(J, (u64)t * T + (u32)((h >> 32) % T), (u32)i)) { J->oom = 1; break; }
    }
    pthread_barrier_wait(&J->bar);
    /* phase 2: aggregate owner t's events in global index order */
    or_map m;
    mt_groups g = {0};
    if (J->oom || map_init(&m, 1 << 15, kb)) { J->oom = 1; pthread_barrier_wait(&J->bar); return NULL; }
    for (u32 s = 0; s < T && !J->oom; s++) {
        const u64 b = (u64)s * T + t;
        for (u64 e = 0; e < J->bcnt[b]; e++) {
            const u64 i = J->bucket[b][e];
            mt_key(J, i, buf);
            if (m.n * 2 >= m.cap && mt_grow(&m)) { J->oom = 1; break; }
            if (mt_groups_fit(&g, m.n + 1, kb, na)) { J->oom = 1; break; }
            int is_new;
            const u64 gi = map_find_or_insert(&m, buf, g.keys, &is_new);
            if (is_new) {
                g.first[gi] = J->base_idx + i;
                for (u32 a = 0; a < na; a++) g.agg[gi * na + a] = 0;
            }
            for (u32 a = 0; a < na; a++) {
                const or_agg *G = &J->aggs[a];
                if (G->cond_width && ld_u(G->cond, G->cond_width, i) != G->cond_val) continue;
                u64 add = G->kind == OR_AGG_COUNT ? 1 : ld_u(G->val, G->val_width, i);
                if (G->kind != OR_AGG_COUNT && G->val_signed && G->val_width < 8) {
                    const u32 sh = 64 - 8 * G->val_width;
                    add = (u64)(((int64_t)(add << sh)) >> sh);
                }
                if (G->kind != OR_AGG_COUNT && G->div > 1) add /= G->div;
                u64 v = g.agg[gi * na + a] + add;
                if (G->out_width < 8) v &= (1ull << (8 * G->out_width)) - 1;
                g.agg[gi * na + a] = v;
            }
        }
    }
    const u64 Gt = m.n;
    map_free(&m);
    J->G[t] = Gt;
    if (J->want_csum && !J->oom) {
        u64 cs = 0;
        if (J->keys)
            for (u64 x = 0; x < Gt; x++) cs += group_csum_generic(g.keys + (u64)kb * x, kb, g.agg + x * na, na, g.first[x]);
        else
            for (u64 x = 0; x < Gt; x++)
                cs += group_csum((const ip_key_t *)(g.keys + (u64)kb * x), g.agg[x * 2], g.agg[x * 2 + 1], g.first[x]);
        J->csum[t] = cs;
    }
    /* phase 3: SortStats over this owner's groups (first-occurrence order), keep k */
    if (!J->oom && J->k && Gt) {
        u32 *perm = (u32 *)malloc(Gt * 4);
        u64 *col = (u64 *)malloc(Gt * 8 * (J->nsort ? J->nsort : 1));
        or_sortkey ks[8];
        if (!perm || !col) { J->oom = 1; }
        else {
            for (u64 x = 0; x < Gt; x++) perm[x] = (u32)x;
            for (u32 s = 0; s < J->nsort && s < 8; s++) {
                for (u64 x = 0; x < Gt; x++) col[s * Gt + x] = g.agg[x * na + J->sort_agg[s]];
                ks[s].ptr = col + s * Gt; ks[s].width = 8; ks[s].kind = OR_UINT; ks[s].desc = J->sort_desc[s];
            }
            or_sort_entries(perm, Gt, NULL, ks, J->nsort);
            const u64 m2 = Gt < J->k ? Gt : J->k;
            for (u64 r = 0; r < m2; r++) {
                J->cand_first[(u64)t * J->k + r] = g.first[perm[r]];
                for (u32 a = 0; a < na; a++) J->cand_agg[((u64)t * J->k + r) * na + a] = g.agg[(u64)perm[r] * na + a];
            }
            J->cand_n[t] = m2;
        }
        free(perm); free(col);
    }
    free(g.keys); free(g.first); free(g.agg);
    pthread_barrier_wait(&J->bar);
    return NULL;
}

static int cmp_u64_pair(const void *a, const void *b) {
    const u64 x = ((const u64 *)a)[0], y = ((const u64 *)b)[0];
    return x < y ? -1 : x > y;
}

/* Returns the number of groups ((u64)-1 on allocation failure); out_first / out_agg
 * (k x naggs) receive the first k rows of the sorted groups. */
static u64 mt_run_csum(mt_job *J, u64 *out_first, u64 *out_agg, u64 *out_csum) {
    const u32 T = J->T ? J->T : 1, na = J->naggs;
    J->T = T;
    J->oom = 0;
    J->bucket = (u32 **)calloc((u64)T * T, sizeof(u32 *));
    J->bcnt = (u64 *)calloc((u64)T * T, 8);
    J->bcap = (u64 *)calloc((u64)T * T, 8);
    J->G = (u64 *)calloc(T, 8);
    J->cand_first = (u64 *)calloc((u64)T * (J->k ? J->k : 1), 8);
    J->cand_agg = (u64 *)calloc((u64)T * (J->k ? J->k : 1) * (na ? na : 1), 8);
    J->cand_n = (u64 *)calloc(T, 8);
    J->csum = (u64 *)calloc(T, 8);
    pthread_t *th = (pthread_t *)malloc(T * sizeof(pthread_t));
    mt_arg *args = (mt_arg *)malloc(T * sizeof(mt_arg));
    u64 G = (u64)-1;
    if (J->bucket && J->bcnt && J->bcap && J->G && J->cand_first && J->cand_agg && J->cand_n && th && args) {
        pthread_barrier_init(&J->bar, NULL, T);
        for (u32 t = 0; t < T; t++) { args[t].job = J; args[t].t = t; }
        for (u32 t = 1; t < T; t++) pthread_create(&th[t], NULL, mt_worker, &args[t]);
        mt_worker(&args[0]);
        for (u32 t = 1; t < T; t++) pthread_join(th[t], NULL);
        pthread_barrier_destroy(&J->bar);
        if (!J->oom) {
            G = 0;
            for (u32 t = 0; t < T; t++) G += J->G[t];
            /* merge: candidates in first-occurrence order, then the same sort */
            u64 nc = 0;
            for (u32 t = 0; t < T; t++) nc += J->cand_n[t];
            if (J->k && nc) {
                u64 *rec = (u64 *)malloc(nc * 8 * (1 + na));
                u64 w = 0;
                for (u32 t = 0; t < T; t++)
                    for (u64 r = 0; r < J->cand_n[t]; r++, w++) {
                        rec[w * (1 + na)] = J->cand_first[(u64)t * J->k + r];
                        for (u32 a = 0; a < na; a++) rec[w * (1 + na) + 1 + a] = J->cand_agg[((u64)t * J->k + r) * na + a];
                    }
                qsort(rec, nc, 8 * (1 + na), cmp_u64_pair);
                u32 *perm = (u32 *)malloc(nc * 4);
                u64 *col = (u64 *)malloc(nc * 8 * (J->nsort ? J->nsort : 1));
                or_sortkey ks[8];
                for (u64 x = 0; x < nc; x++) perm[x] = (u32)x;
                for (u32 s = 0; s < J->nsort && s < 8; s++) {
                    for (u64 x = 0; x < nc; x++) col[s * nc + x] = rec[x * (1 + na) + 1 + J->sort_agg[s]];
                    ks[s].ptr = col + s * nc; ks[s].width = 8; ks[s].kind = OR_UINT; ks[s].desc = J->sort_desc[s];
                }
                or_sort_entries(perm, nc, NULL, ks, J->nsort);
                for (u64 r = 0; r < J->k && r < nc; r++) {
                    out_first[r] = rec[(u64)perm[r] * (1 + na)];
                    for (u32 a = 0; a < na; a++) out_agg[r * na + a] = rec[(u64)perm[r] * (1 + na) + 1 + a];
                }
                free(perm); free(col); free(rec);
            }
        }
    }
    if (out_csum && J->csum && G != (u64)-1) {
        *out_csum = 0;
        for (u32 t = 0; t < T; t++) *out_csum += J->csum[t];
    }
    free(J->csum);
    if (J->bucket)
        for (u64 b = 0; b < (u64)T * T; b++) free(J->bucket[b]);
    free(J->bucket); free(J->bcnt); free(J->bcap); free(J->G); free(J->cand_first); free(J->cand_agg);
    free(J->cand_n); free(th); free(args);
    return G;
}

/* top tcp on T threads: out_* as or_top_tcp (keys omitted), same rows. */
u64 or_top_tcp_mt(const u8 *saddr, const u8 *daddr, const u64 *mntns, const u32 *pid,
                  const u8 *comm, const u16 *lport, const u16 *dport, const u16 *family,
                  const u32 *size, const u8 *dir, u64 n, u64 base_idx, u32 nthreads, u32 k,
                  u64 *out_sent, u64 *out_recv, u64 *out_first, u64 *out_csum) {
    or_agg aggs[2] = {{OR_AGG_SUM, 4, size, 1, dir, 0, 8, 0, 0}, {OR_AGG_SUM, 4, size, 1, dir, 1, 8, 0, 0}};
    const u32 sa[2] = {0, 1}, sd[2] = {1, 1};   /* ["-sent", "-recv"] */
    mt_job J;
    memset(&J, 0, sizeof J);
    J.saddr = saddr; J.daddr = daddr; J.mntns = mntns; J.pid = pid; J.comm = comm;
    J.lport = lport; J.dport = dport; J.family = family;
    J.tcp_size = size; J.tcp_dir = dir;
    J.aggs = aggs; J.naggs = 2; J.n = n; J.base_idx = base_idx; J.T = nthreads;
    J.sort_agg = sa; J.sort_desc = sd; J.nsort = 2; J.k = k;
    J.want_csum = out_csum != NULL;
    u64 *agg = (u64 *)malloc((k ? k : 1) * 16);
    const u64 G = mt_run_csum(&J, out_first, agg, out_csum);
    for (u32 r = 0; r < k && G != (u64)-1 && r < G; r++) { out_sent[r] = agg[2 * r]; out_recv[r] = agg[2 * r + 1]; }
    free(agg);
    return G;
}

/* generic keyed aggregation + top-k by aggregates (sort_agg[s], sort_desc[s] in sortBy
 * order; nsort 0 / k 0 = group count only) on T threads; out_csum (optional) receives the
 * whole-table checksum (sum of group_csum_generic). */
u64 or_groupby_topk_mt(const u8 *keys, u32 kb, u64 n, const u8 *valid, const or_agg *aggs, u32 naggs,
                       u64 base_idx, u32 nthreads, const u32 *sort_agg, const u32 *sort_desc, u32 nsort,
                       u32 k, u64 *out_first, u64 *out_agg, u64 *out_csum) {
    mt_job J;
    memset(&J, 0, sizeof J);
    J.keys = keys; J.kb = kb; J.valid = valid; J.aggs = aggs; J.naggs = naggs; J.n = n;
    J.base_idx = base_idx; J.T = nthreads; J.sort_agg = sort_agg; J.sort_desc = sort_desc;
    J.nsort = nsort; J.k = k;
    J.want_csum = out_csum != NULL;
    return mt_run_csum(&J, out_first, out_agg, out_csum);
}

/* log2 histograms on T threads: private histograms per slice, summed (u32 wrap). */
typedef struct {
    const u32 *dev, *cont; const i64 *delta; u64 lo, hi; const u32 *devs; u32 ndev, ncont; u64 divisor;
    u32 nslots; u32 *hist;
} hist_arg;
static void *hist_worker(void *p) {
    hist_arg *h = (hist_arg *)p;
    or_hist_log2(h->dev ? h->dev + h->lo : NULL, h->cont ? h->cont + h->lo : NULL, h->delta + h->lo,
                 h->hi - h->lo, h->devs, h->ndev, h->ncont, h->divisor, h->nslots, h->hist);
    return NULL;
}
void or_hist_log2_mt(const u32 *dev, const u32 *cont, const i64 *delta, u64 n, const u32 *devs,
                     u32 ndev, u32 ncont, u64 divisor, u32 nslots, u32 *hist, u32 nthreads) {
    const u32 T = nthreads ? nthreads : 1;
    const u64 keys = (u64)(ndev ? ndev : 1) * ncont * nslots;
    u32 *priv = (u32 *)calloc((u64)T * keys, 4);
    pthread_t *th = (pthread_t *)malloc(T * sizeof(pthread_t));
    hist_arg *a = (hist_arg *)malloc(T * sizeof(hist_arg));
    for (u32 t = 0; t < T; t++) {
        a[t] = (hist_arg){dev, cont, delta, n * t / T, n * (t + 1) / T, devs, ndev, ncont, divisor, nslots,
                          priv + (u64)t * keys};
        if (t) pthread_create(&th[t], NULL, hist_worker, &a[t]);
    }
    hist_worker(&a[0]);
    for (u32 t = 1; t < T; t++) pthread_join(th[t], NULL);
    for (u32 t = 0; t < T; t++)
        for (u64 x = 0; x < keys; x++) hist[x] += priv[(u64)t * keys + x];
    free(priv); free(th); free(a);
}

/* ---------------------------------------------------------------------------------------
 * §8: advise network-policy's GeneratePolicies on STRING keys, the reference's own shape
 * (pkg/gadgets/advise/networkpolicy/advisor/advisor.go): per event the filter (:282-292),
 * localPodKey = Namespace + ":" + labelKeyString(PodLabels) (:143-145, labelKeyString :132-141
 * sorts the label keys left after LabelsToIgnore :36-40, :104-116), eventsBySource[key] append
 * (:294-299); then per source, networkPeerKey (:147-158, fmt.Sprintf("%s:%d", ..., Port)) and
 * first-event-wins egress / ingress maps (:302-320).  Returns the number of (source, direction,
 * peer key) entries -- the distinct tuples the device table holds.  Timed as C4's faithful CPU
 * baseline (bench.py); single-threaded like GeneratePolicies.
 *
 * The synthetic C4 stream carries integer ids (or_gen_np); the strings a Kubernetes event would
 * carry are derived from them, one-to-one: source s -> Namespace "ns-<s%50>", PodLabels
 * {app: "app-<s>", pod-template-hash: <hash>, tier: "tier-<s%4>"}; peer p -> RemoteKind pod /
 * svc / other by p%3, RemoteNamespace "ns-<p%50>", RemoteLabels {app: "peer-<p>", pod-template-
 * hash: <hash>}, and for "other" the peer's canonical address 10.96.x.y (the stream's RemoteAddr
 * of that peer).  Go also copies each whole Event into eventsBySource; here the event index is
 * appended (cheaper than the reference).
 * --------------------------------------------------------------------------------------- */
typedef struct { const char *k; char v[24]; } np_label;

static int np_label_cmp(const void *a, const void *b) {
    return strcmp(((const np_label *)a)->k, ((const np_label *)b)->k);
}

static int np_ignored(const char *k) {   /* defaultLabelsToIgnore, advisor.go:36-40 */
    return !strcmp(k, "controller-revision-hash") || !strcmp(k, "pod-template-generation") ||
           !strcmp(k, "pod-template-hash");
}

/* labelKeyString: the labels not ignored, keys sorted, "k=v" joined by "," */
static int np_label_key_string(np_label *L, int nl, char *out) {
    np_label keep[4];
    int m = 0;
    for (int i = 0; i < nl; i++)
        if (!np_ignored(L[i].k)) keep[m++] = L[i];
    qsort(keep, m, sizeof(np_label), np_label_cmp);
    int len = 0;
    for (int i = 0; i < m; i++) len += sprintf(out + len, "%s%s=%s", i ? "," : "", keep[i].k, keep[i].v);
    return len;
}

static int np_pod_labels(u32 id, const char *app_prefix, int with_tier, np_label *L) {
    int n = 0;
    L[n].k = "app"; snprintf(L[n].v, sizeof L[n].v, "%s-%u", app_prefix, id); n++;
    L[n].k = "pod-template-hash"; snprintf(L[n].v, sizeof L[n].v, "%08x", (u32)sm64(id ^ 0xABCD)); n++;
    if (with_tier) { L[n].k = "tier"; snprintf(L[n].v, sizeof L[n].v, "tier-%u", id % 4); n++; }
    return n;
}

static int np_local_pod_key(u32 s, char *out) {   /* localPodKey, advisor.go:146-148 */
    np_label L[4];
    const int nl = np_pod_labels(s, "app", 1, L);
    int len = sprintf(out, "ns-%u:", s % 50);
    return len + np_label_key_string(L, nl, out + len);
}

static int np_peer_key(u32 p, u16 port, char *out) {   /* networkPeerKey, advisor.go:150-159 */
    char ret[160];
    int len;
    if (p % 3 == 0 || p % 3 == 1) {   /* RemoteKindPod / RemoteKindService */
        np_label L[4];
        const int nl = np_pod_labels(p, "peer", 0, L);
        len = sprintf(ret, "%s:ns-%u:", p % 3 == 0 ? "pod" : "svc", p % 50);
        len += np_label_key_string(L, nl, ret + len);
    } else {                          /* RemoteKindOther: the peer's address */
        const u32 a = 0x0a600000u | (p & 0xfffff);
        len = sprintf(ret, "other:%u.%u.%u.%u", a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255);
    }
    (void)len;
    return sprintf(out, "%s:%u", ret, (unsigned)port);
}

/* string-keyed open-addressing table: keys in a byte pool, FNV-1a hashes, generation-cleared */
typedef struct {
    u64 cap, n;
    u64 *h; u64 *off; u32 *len; u32 *gen; u32 *val;
    char *pool; u64 pool_len, pool_cap;
    u32 cur_gen;
} np_smap;

static u64 np_fnv(const char *s, u32 len) {
    u64 h = 14695981039346656037ull;
    for (u32 i = 0; i < len; i++) { h ^= (u8)s[i]; h *= 1099511628211ull; }
    return h;
}

static void np_smap_init(np_smap *m, u64 cap) {
    memset(m, 0, sizeof *m);
    m->cap = 1; while (m->cap < cap * 2) m->cap <<= 1;
    m->h = (u64 *)malloc(m->cap * 8); m->off = (u64 *)malloc(m->cap * 8);
    m->len = (u32 *)malloc(m->cap * 4); m->gen = (u32 *)calloc(m->cap, 4); m->val = (u32 *)malloc(m->cap * 4);
    m->pool_cap = 1 << 20; m->pool = (char *)malloc(m->pool_cap);
    m->cur_gen = 1;
}

static void np_smap_free(np_smap *m) {
    free(m->h); free(m->off); free(m->len); free(m->gen); free(m->val); free(m->pool);
}

static void np_smap_clear(np_smap *m) { m->cur_gen++; m->n = 0; m->pool_len = 0; }

/* index of key, inserting it with val when absent (*added = 1) */
static u32 np_smap_get(np_smap *m, const char *k, u32 len, u32 val, int *added) {
    const u64 h = np_fnv(k, len);
    u64 i = h & (m->cap - 1);
    for (;; i = (i + 1) & (m->cap - 1)) {
        if (m->gen[i] != m->cur_gen) break;
        if (m->h[i] == h && m->len[i] == len && !memcmp(m->pool + m->off[i], k, len)) {
            *added = 0;
            return m->val[i];
        }
    }
    if (m->pool_len + len > m->pool_cap) {
        while (m->pool_len + len > m->pool_cap) m->pool_cap *= 2;
        m->pool = (char *)realloc(m->pool, m->pool_cap);
    }
    memcpy(m->pool + m->pool_len, k, len);
    m->gen[i] = m->cur_gen; m->h[i] = h; m->off[i] = m->pool_len; m->len[i] = len; m->val[i] = val;
    m->pool_len += len;
    m->n++;
    *added = 1;
    return val;
}

u64 or_np_advise_strings(const u32 *src, const u32 *peer, const u16 *port, const u8 *pkt, const u8 *typ,
                         const u32 *hostip, const u32 *raddr, u64 n) {
    /* pass 1: eventsBySource (map[string][]Event; here an index list per source) */
    np_smap bysrc;
    np_smap_init(&bysrc, 1 << 16);
    u64 nsrc_cap = 1 << 12, nsrc = 0;
    u64 *cnt = (u64 *)calloc(nsrc_cap, 8);
    u32 *ev_src = (u32 *)malloc((n ? n : 1) * 4);
    char key[256];
    for (u64 i = 0; i < n; i++) {
        ev_src[i] = 0xFFFFFFFFu;
        if (typ[i] != 0) continue;                                  /* :283-285 */
        if (pkt[i] != 0 && pkt[i] != 4) continue;                   /* :286-288 HOST / OUTGOING */
        if (pkt[i] == 0 && hostip[i] == raddr[i]) continue;         /* :290-292 */
        const int len = np_local_pod_key(src[i], key);
        if (bysrc.n * 2 >= bysrc.cap) {   /* grow: rehash into a bigger table */
            np_smap big;
            np_smap_init(&big, bysrc.cap);
            for (u64 j = 0; j < bysrc.cap; j++)
                if (bysrc.gen[j] == bysrc.cur_gen) {
                    int ad;
                    np_smap_get(&big, bysrc.pool + bysrc.off[j], bysrc.len[j], bysrc.val[j], &ad);
                }
            np_smap_free(&bysrc);
            bysrc = big;
        }
        int added;
        const u32 sidx = np_smap_get(&bysrc, key, (u32)len, (u32)nsrc, &added);
        if (added) {
            if (++nsrc > nsrc_cap) { cnt = (u64 *)realloc(cnt, nsrc_cap * 2 * 8); memset(cnt + nsrc_cap, 0, nsrc_cap * 8); nsrc_cap *= 2; }
        }
        ev_src[i] = sidx;
        cnt[sidx]++;
    }
    /* group the event indices by source, in event order (the appended slices) */
    u64 *start = (u64 *)calloc(nsrc + 1, 8);
    for (u64 s = 0; s < nsrc; s++) start[s + 1] = start[s] + cnt[s];
    u64 *fill = (u64 *)malloc((nsrc + 1) * 8);
    memcpy(fill, start, (nsrc + 1) * 8);
    u32 *evs = (u32 *)malloc((start[nsrc] ? start[nsrc] : 1) * 4);
    for (u64 i = 0; i < n; i++)
        if (ev_src[i] != 0xFFFFFFFFu) evs[fill[ev_src[i]]++] = (u32)i;
    /* pass 2: per source, egressNetworkPeer / ingressNetworkPeer (first event wins) */
    np_smap eg, in;
    np_smap_init(&eg, 1 << 10);
    np_smap_init(&in, 1 << 10);
    u64 total = 0;
    for (u64 s = 0; s < nsrc; s++) {
        const u64 m = start[s + 1] - start[s];
        if (eg.cap < m * 2) { np_smap_free(&eg); np_smap_free(&in); np_smap_init(&eg, m); np_smap_init(&in, m); }
        np_smap_clear(&eg);
        np_smap_clear(&in);
        for (u64 x = start[s]; x < start[s + 1]; x++) {
            const u32 i = evs[x];
            const int len = np_peer_key(peer[i], port[i], key);
            int added;
            np_smap_get(pkt[i] == 4 ? &eg : &in, key, (u32)len, i, &added);
        }
        total += eg.n + in.n;
    }
    np_smap_free(&bysrc); np_smap_free(&eg); np_smap_free(&in);
    free(cnt); free(ev_src); free(start); free(fill); free(evs);
    return total;
}
