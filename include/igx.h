/*
 * igx.h -- C ABI of the MI355X-native Inspektor Gadget event-aggregation path.
 *
 * One shared library, libigx.so (HIP kernels for gfx950 + host C++), built in-tree at
 * inspektor-gadget_amd/libigx.so.  Plain pointers and sizes only; nothing here knows
 * about torch or Go types, so the reference's Go packages can bind it with cgo
 * (INTEGRATION.md shows the binding).
 *
 * Reference interfaces replaced (paths relative to the reference repository root):
 *   igx_filter_parse        filter.GetFilterFromString       pkg/columns/filter/filter.go:91-172
 *                           (+ getValueFromFilterSpec :53-87)
 *   igx_filter              filter.FilterEntries / FilterSpecs.MatchAll
 *                                                             pkg/columns/filter/filter.go:266-325
 *   igx_sort_prepare        sort.Prepare / FilterSortableColumns / CanSortBy
 *                                                             pkg/columns/sort/sort.go:87-111,139-178
 *   igx_sort_perm           ColumnSorterCollection.Sort / SortEntries
 *                                                             pkg/columns/sort/sort.go:35-83,116-123
 *   igx_topk                top.SortStats + stats[:MaxRows]  pkg/gadgets/top/top.go:39-41,
 *                                                             pkg/gadgets/top/tcp/tracer/tracer.go:249-253
 *   igx_groupby_*           BPF hash-map keyed aggregation + nextStats drain
 *                                                             pkg/gadgets/top/tcp/tracer/bpf/tcptop.bpf.c:33-110,
 *                                                             pkg/gadgets/top/tcp/tracer/tracer.go:147-226,
 *                                                             pkg/gadgets/top/file/tracer/bpf/filetop.bpf.c:39-94,
 *                                                             pkg/gadgets/top/block-io/tracer/bpf/biotop.bpf.c:85-130,
 *                                                             pkg/gadgets/trace/network/tracer/bpf/graph.c:102-114
 *                           and group.GroupEntries (one column per call)
 *                                                             pkg/columns/group/group.go:51-121
 *   igx_hist_log2           biolatency histogram              pkg/gadgets/profile/block-io/tracer/bpf/biolatency.bpf.c:100-154
 *                                                             pkg/gadgets/profile/block-io/tracer/bpf/bits.bpf.h:8-29
 *
 * Conventions
 *   - Return codes: IGX_OK (0) or a negative errno-style code.  The message of the last
 *     failure on a context is igx_last_error(ctx); host-only parsers write theirs into
 *     a caller buffer (the Go `error` text, e.g. `could not apply filter: column "x" not
 *     found`).
 *   - "device" pointers are HIP device allocations (igx_malloc or any HIP allocator);
 *     "host" pointers are plain memory.  Nothing is retained past the call except by
 *     igx_table objects, which own their device storage (cgo pointer rules).
 *   - Every device operation is enqueued on the context's stream (igx_set_stream to share
 *     a caller's stream) and is asynchronous unless documented as synchronising.
 */
#ifndef IGX_H
#define IGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IGX_OK 0
#define IGX_ENOENT (-2)
#define IGX_EIO (-5)
#define IGX_ENOMEM (-12)
#define IGX_EINVAL (-22)
#define IGX_ENOSPC (-28)
#define IGX_ENOTSUP (-95)

/* Column kind classes (Go reflect kinds collapsed by arithmetic).  Strings are fixed-width
 * zero-padded byte columns: bytewise unsigned compare == Go string compare because
 * gadgets.FromCString never yields NUL (pkg/gadgets/helpers.go:76-83). */
enum igx_kind {
    IGX_KIND_INT = 0,   /* int, int8..int64 (two's complement, little-endian) */
    IGX_KIND_UINT = 1,  /* uint, uint8..uint64 */
    IGX_KIND_FLOAT = 2, /* float32 / float64 */
    IGX_KIND_BYTES = 3, /* string as fixed-width bytes */
    IGX_KIND_BOOL = 4,  /* bool: not filterable (filter.go:54-85), not sortable (sort.go:77-78) */
    IGX_KIND_OTHER = 5  /* struct and everything else */
};

enum igx_cmp { IGX_CMP_EQ = 0, IGX_CMP_REGEX = 1, IGX_CMP_LT = 2, IGX_CMP_LE = 3,
               IGX_CMP_GT = 4, IGX_CMP_GE = 5,
               /* group-by predicates only (a BPF probe's set test, e.g. tcptop.bpf.c:54
                * `family != AF_INET && family != AF_INET6` -> drop): the field equals one
                * of the ref_len / width values packed in ref (at most 8 bytes) */
               IGX_CMP_IN = 6 };

#define IGX_COL_VIRTUAL 1u   /* columns.AddColumn virtual column (columns.go:282-309) */
#define IGX_COL_EXTRACTOR 2u /* column with SetExtractor (columns.go:320-332) */
#define IGX_NO_COL 0xFFFFFFFFu
#define IGX_MAX_REF 256
#define IGX_MAX_KEY_BYTES 128

/* Schema entry: one column of the event struct T, as derived by columns.NewColumns. */
typedef struct {
    const char *name; /* column name; matched case-insensitively (columns.go:83-86) */
    uint32_t kind;    /* enum igx_kind */
    uint32_t width;   /* bytes per row in the SoA batch */
    uint32_t flags;   /* IGX_COL_* */
    uint32_t raw_kind;/* kind used for sorting extractor columns (sort.go:46-48) */
} igx_schema_col;

/* Device column: row i lives at ptr + i*width. */
typedef struct {
    const void *ptr;
    uint32_t width;
    uint32_t kind;
} igx_col;

/* One compiled filter (FilterSpec).  ref holds the reference value already converted to
 * the column type (reflect Convert truncation, filter.go:64,74). */
typedef struct {
    uint32_t col;     /* index into the schema / column array */
    uint32_t cmp;     /* enum igx_cmp */
    uint32_t negate;
    uint32_t ref_len; /* valid bytes in ref */
    uint8_t ref[IGX_MAX_REF];
    /* Group-by predicates only: a guard restricts the test to the rows whose guard column
     * (guard_col, an integer column of guard_len = 1/2/4/8 bytes) equals guard_ref; the other
     * rows pass.  A BPF program with one probe per event kind checks some fields on one kind
     * only, e.g. top tcp's receive probe drops `copied <= 0` (tcptop.bpf.c:124-130) while the
     * send probe has no such check (:112-116): {col = size as int32, GT 0, guard dir == 1}.
     * guard_len 0 = unguarded (what igx_filter_parse emits; igx_filter rejects guards). */
    uint32_t guard_col;
    uint32_t guard_len;
    uint8_t guard_ref[8];
} igx_pred;

/* One sort key as Prepare emits it, in sortBy order (first = highest priority). */
typedef struct {
    const void *ptr;  /* device column (igx_sort_perm) or unused (igx_sort_prepare) */
    uint32_t width;
    uint32_t kind;
    uint32_t desc;    /* 1 when the sortBy entry had the '-' prefix */
    uint32_t col;     /* schema index (igx_sort_prepare output) */
} igx_sortkey;

typedef struct igx_ctx igx_ctx;
typedef struct igx_table igx_table;

/* ---- context ------------------------------------------------------------------------ */
int igx_open(int device, uint32_t flags, igx_ctx **out);
int igx_close(igx_ctx *ctx);
const char *igx_last_error(igx_ctx *ctx);
/* Share a caller's hipStream_t (NULL = HIP's default/null stream, which is what torch's
 * default stream is).  Until the first call the context uses a stream of its own. */
int igx_set_stream(igx_ctx *ctx, void *hip_stream);
void *igx_get_stream(igx_ctx *ctx);
int igx_sync(igx_ctx *ctx);
int igx_malloc(igx_ctx *ctx, size_t bytes, void **out);
int igx_free(igx_ctx *ctx, void *p);
int igx_memcpy_h2d(igx_ctx *ctx, void *dst, const void *src, size_t bytes);   /* sync */
int igx_memcpy_d2h(igx_ctx *ctx, void *dst, const void *src, size_t bytes);   /* sync */
int igx_memcpy_d2d(igx_ctx *ctx, void *dst, const void *src, size_t bytes);   /* async */
int igx_version(void);

/* ---- filter (host parser + device scan) -------------------------------------------- */
/* GetFilterFromString: parses "col[:[!][~|>=|>|<=|<]value]".  Host only, no GPU needed.
 * Regex rules are returned with cmp=IGX_CMP_REGEX and value = the pattern; igx_filter
 * compiles and runs them (below).  errbuf receives the Go error text. */
int igx_filter_parse(const igx_schema_col *cols, uint32_t ncols, const char *filter,
                     igx_pred *out, char *errbuf, size_t errlen);

/* Regex rules (IGX_CMP_REGEX, on string columns) run on the device: the pattern is compiled
 * on the host to a DFA over rune classes with Go regexp semantics (RE2 syntax incl. \b \B
 * \A \z, (?m) (?i) (?s), \p{..} general categories and scripts of Unicode 13.0.0, POSIX
 * classes; UTF-8 decoded like utf8.DecodeRune; unanchored MatchString).  A pattern whose
 * automaton would exceed the device limits (255 rune classes, 2048 states) returns
 * IGX_ENOTSUP.  igx_regex_compile_blob exposes the compiled automaton (for tests and tools). */
int igx_regex_compile_blob(const char *pattern, size_t len, uint8_t *out, size_t cap,
                           size_t *out_len, char *errbuf, size_t errlen);

/* FilterEntries' per-filter pass (filter.go:301-322): AND of preds (any number) over rows
 * [0,nrows), order-preserving.  valid (device, nullable): 0 marks a nil entry, which is
 * skipped (:310-314).  out_idx (device) receives the selected row ids; *out_n (device u64)
 * their count.  Asynchronous. */
int igx_filter(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
               uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
               uint64_t *out_n);
/* FilterSpecs.MatchAny (filter.go:276-283): OR of preds (any number); zero preds select
 * nothing; a nil row matches iff some pred is negated (Match(nil) == negate, :286-291).
 * Outputs as igx_filter.  Asynchronous. */
int igx_filter_any(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                   uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
                   uint64_t *out_n);
/* The general form.  flags:
 *   IGX_FILTER_ANY        OR of preds (MatchAny) instead of AND (MatchAll);
 *   IGX_FILTER_NIL_MATCH  a nil row yields Match(nil) == negate for every pred (filter.go:
 *                         286-291), combined like the other rows: FilterSpecs.MatchAll keeps a
 *                         nil row iff every pred is negated (or there are none), MatchAny iff
 *                         one is -- what parser.eventHandlerArray relies on (parser.go:209-218).
 *                         Without it nil rows are skipped (FilterEntries).
 * igx_filter == flags 0; igx_filter_any == IGX_FILTER_ANY | IGX_FILTER_NIL_MATCH. */
#define IGX_FILTER_ANY 1u
#define IGX_FILTER_NIL_MATCH 2u
int igx_filter_ex(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                  uint32_t npreds, const uint8_t *valid, uint64_t nrows, uint32_t flags,
                  uint32_t *out_idx, uint64_t *out_n);
/* The compacted batch FilterEntries returns (filter.go:294-325 builds a fresh slice of the
 * selected entries): rows idx[0..k) (device u32, e.g. igx_filter's out_idx) of every column
 * gathered into out[c] (device, k * cols[c].width bytes, rows packed).  Indices >= nrows
 * yield zero rows.  Asynchronous. */
int igx_take(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, uint64_t nrows,
             const uint32_t *idx, uint64_t k, void *const *out);

/* ---- sort / top-K -------------------------------------------------------------------- */
/* Prepare + FilterSortableColumns: keeps valid keys in sortBy order (unknown, empty and
 * virtual columns dropped).  *out_n = number of valid keys; *out_invalid = dropped ones.
 * Bool / unsupported kinds stay in the list (the Go code skips them at Sort time,
 * sort.go:77-78) and are skipped by igx_sort_perm.  Host only. */
int igx_sort_prepare(const igx_schema_col *cols, uint32_t ncols, const char *const *sort_by,
                     uint32_t n, igx_sortkey *out, uint32_t *out_n, uint32_t *out_invalid);

/* Sort permutation with the exact tie order of Go 1.19 sort.SliceStable under
 * getLessFunc (SURVEY.md §0.3 closed form).  pos (device u64, nullable): pre-sort position
 * of each row (NULL = row index).  valid (device, nullable): nil rows sort last.
 * Float keys compare as Go's `<` does: -0 == +0, -Inf < finite < +Inf; a NaN in a float key
 * of a non-nil row makes the comparison unordered (no strict weak order, so SliceStable's
 * output depends on its merge steps) and the call returns IGX_ENOTSUP.
 * out_perm (device u32, nrows).  Synchronises once: the digit plan's read-back (which bytes of
 * the composed key vary, the NaN flag, a device row count); IGX_SORT_DEVPLAN=1 plans full sorts
 * of at most 8 composed words without float keys on the device instead (no read-back; slower
 * at 1M rows).  String keys of 5..32 bytes in full sorts of >= 65 536 rows sort
 * by their rank in a dictionary of their distinct values (at most 4 096; 2 048 for 32 bytes),
 * built on the device -- the same order, a few radix passes instead of one per live byte;
 * more distinct values: the raw bytes, after one more read-back.  IGX_SORT_DICT=0 turns the
 * dictionaries off. */
int igx_sort_perm(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
                  const uint64_t *pos, const uint8_t *valid, uint32_t *out_perm);

/* igx_sort_perm over a selection vector: row i of the slice is row rowmap[i] (device u32) of
 * the key columns -- FilterEntries' result is a slice of pointers into the caller's entries
 * (filter.go:294-325), and SortEntries sorts that slice (sort.go:116-123) without moving the
 * entries.  pos (nullable: slice index) and valid (nullable) are read at rowmap[i].  out_perm
 * receives the rowmap values (base rows) in sorted order: the sorted slice.  rowmap NULL ==
 * igx_sort_perm. */
int igx_sort_perm_ex(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
                     const uint64_t *pos, const uint8_t *valid, const uint32_t *rowmap, uint32_t *out_perm);

/* igx_sort_perm_ex when the row count lives on the device: the slice is rows [0, *d_nrows) of
 * the selection vector, nrows_max its upper bound (d_nrows: device u64, e.g. igx_filter's
 * out_n) -- FilterEntries' count feeds SortEntries without a read-back of its own: it rides
 * the digit plan's read-back (none with IGX_SORT_DEVPLAN=1).  No float key (a NaN would need
 * the host's decision before the count is known), and a top-K needs a slot list and no nil
 * mask: otherwise IGX_EINVAL.  out_perm (device u32, nrows_max) holds the sorted rowmap values
 * in its first *d_nrows entries. */
int igx_sort_perm_dn(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows_max,
                     const uint64_t *d_nrows, const uint64_t *pos, const uint8_t *valid, const uint32_t *rowmap,
                     uint32_t *out_perm);

/* First k rows of the igx_sort_perm order (SortStats + truncate to max-rows).
 * out_idx (device u32, k).  Asynchronous. */
int igx_topk(igx_ctx *ctx, const igx_sortkey *keys, uint32_t nkeys, uint64_t nrows,
             const uint64_t *pos, uint32_t k, uint32_t *out_idx);

/* ---- keyed aggregation (group-by) ------------------------------------------------------ */
enum igx_agg_kind { IGX_AGG_COUNT = 0, IGX_AGG_SUM = 1 };

typedef struct {
    uint32_t kind;      /* enum igx_agg_kind */
    uint32_t col;       /* value column index (SUM) */
    uint32_t cond_col;  /* IGX_NO_COL or column whose value must equal cond_val */
    uint32_t out_width; /* result wraps to this many bytes (1,2,4,8) */
    uint64_t cond_val;
    uint64_t divisor;   /* SUM of an unsigned column: add value / divisor per event (0, 1 =
                         * plain sum), e.g. biotop's `us += delta_ns / 1000`
                         * (pkg/gadgets/top/block-io/tracer/bpf/biotop.bpf.c:98,119) */
} igx_agg;

/* The table is an open-addressing array of n_slots slots; a group's id is its slot.
 * Slot s has a key record at keys + s*key_stride (the packed key) and a value record at
 * first_idx + s*val_stride bytes (u64 first-occurrence index, then the u64 aggregates;
 * aggs[a] points at slot 0's aggregate a).  Aggregates are kept as u64 sums; they wrap to
 * their out_width when read (the low out_width bytes, little-endian).  groups[0..n_groups)
 * lists the occupied slots in ascending slot order (the canonical pre-sort order is
 * first_idx, not this). */
typedef struct {
    uint64_t n_groups;        /* host copy, valid after igx_groupby_finalize */
    uint64_t n_slots;
    uint32_t key_bytes;       /* packed key bytes per group (each key column padded to 4) */
    uint32_t key_stride;      /* key record size: bytes between consecutive slots' keys */
    uint32_t val_stride;      /* value record size: bytes between consecutive slots' values */
    uint32_t naggs;
    const uint8_t *keys;      /* device: slot 0's packed key */
    const uint64_t *aggs[16]; /* device: slot 0's aggregate a; stride val_stride */
    const uint64_t *first_idx;/* device: slot 0's first-occurrence index; stride val_stride */
    const uint32_t *groups;   /* device: occupied slots, n_groups entries */
    const uint64_t *d_n_groups;/* device: group count */
} igx_table_view;

/* Sort key over a table's columns (igx_groupby_sort). */
/* IGX_TSRC_CONST: a column that holds the same value for every group (e.g. the
 * CommonData enrichment strings when nothing enriches).  Go still runs a SliceStable pass
 * for it, so it orders nothing but its '-' flips the tie parity. */
/* IGX_TSRC_IPTEXT: the text of a 16-byte address in the key (offset) under the u16 family
 * in the key (index = its byte offset), as IPStringFromBytes renders it (helpers.go:111-120,
 * top/tcp/tracer/tracer.go:199-206): the Saddr / Daddr string columns of the Stats rows. */
enum igx_tsrc { IGX_TSRC_AGG = 0, IGX_TSRC_FIRST = 1, IGX_TSRC_KEY = 2, IGX_TSRC_CONST = 3, IGX_TSRC_IPTEXT = 4 };
typedef struct {
    uint32_t src;    /* enum igx_tsrc */
    uint32_t index;  /* aggregate index (IGX_TSRC_AGG); family byte offset (IGX_TSRC_IPTEXT) */
    uint32_t offset; /* byte offset in the packed key (IGX_TSRC_KEY, IGX_TSRC_IPTEXT) */
    uint32_t width;  /* bytes (IGX_TSRC_KEY) */
    uint32_t kind;   /* enum igx_kind (IGX_TSRC_KEY) */
    uint32_t desc;   /* '-' prefix */
} igx_tsortkey;

/* capacity = maximum number of distinct groups.  key_widths: byte width of each key
 * column, any width (packed, each padded to a multiple of 4; at most IGX_MAX_KEY_BYTES
 * padded bytes in all).  The table's key records must stay below 4 GiB (S >= 2 x capacity
 * slots of 32..256 B: about 16M groups for the 72-B ip_key_t), IGX_ENOTSUP otherwise. */
int igx_groupby_create(igx_ctx *ctx, const uint32_t *key_widths, uint32_t nkeys,
                       const igx_agg *aggs, uint32_t naggs, uint64_t capacity,
                       igx_table **out);
/* Aggregate rows [0,nrows) of cols into the table; key_cols selects the key columns
 * (in the table's key order); preds are AND-ed filters applied first (the BPF probe
 * checks): any number, of any kind igx_filter takes plus IGX_CMP_IN sets (up to two scalar
 * comparisons / sets are fused into the aggregation kernel, the others -- regex, string
 * rules, more comparisons -- first become a device row mask).  base_idx is the global index of row 0 (first-occurrence order); indices must
 * stay below 2^48 - 1 (IGX_EINVAL otherwise; an index column value at or above it fails the
 * interval at finalize): long-running streams rebase their indices per interval.  Async. */
int igx_groupby_update(igx_table *t, const igx_col *cols, uint32_t ncols,
                       const uint32_t *key_cols, const igx_pred *preds, uint32_t npreds,
                       uint64_t nrows, uint64_t base_idx);
/* igx_groupby_update with two more inputs (either may be absent):
 *   valid   (device u8, nullable): rows with 0 are skipped -- nil entries, or a mask from
 *           igx_np_mark;
 *   idx_col (IGX_NO_COL = row index + base_idx): a u64 column giving each row's global
 *           event index.  Used to merge partial groups from other shards: key columns +
 *           one u64 column per partial aggregate (summed by SUM aggregates) + their first
 *           index, so first = min over shards (SURVEY.md §8(e) group-by exchange). */
int igx_groupby_update_ex(igx_table *t, const igx_col *cols, uint32_t ncols,
                          const uint32_t *key_cols, const igx_pred *preds, uint32_t npreds,
                          const uint8_t *valid, uint32_t idx_col, uint64_t nrows,
                          uint64_t base_idx);
/* Synchronises; fills the view; IGX_ENOSPC if capacity was exceeded. */
int igx_groupby_finalize(igx_table *t, igx_table_view *view);
/* Diagnostics: the form the current interval runs in and AUTO's plan for the next ones. */
typedef struct {
    uint32_t form;       /* IGX_GB_CACHED / IGX_GB_DIRECT / IGX_GB_PART (0 before the interval's first update) */
    uint32_t region;     /* 1: the interval's partitioned updates run the region variant */
    uint32_t part_left;  /* AUTO: intervals still planned in the partitioned form */
    uint32_t exact_left; /* AUTO: intervals partitioned exactly after a region overflowed */
    uint32_t sm_probers; /* the cached form's probers: 1 state machine, 0 batch */
    uint32_t loaders;    /* the cached form's loader waves for the next update (8, or 7 after intervals
                            that missed the LDS cache on > 39 % of their rows, until one falls below 37 %) */
    uint64_t rows;       /* rows fed to the interval so far */
    uint32_t miss_permille;  /* LDS misses per 1000 rows of the last measured cached interval */
    uint32_t persist;    /* 1: keys are kept across intervals (a generation; igx_groupby_reset) */
    uint64_t claims;     /* the last collected finalize: keys its interval inserted (the others were kept) */
    uint64_t gen_keys;   /* ... keys the table's generation held after it (UINT64_MAX: it ended) */
} igx_groupby_info_t;
int igx_groupby_info(igx_table *t, igx_groupby_info_t *out);
/* igx_groupby_finalize without its host synchronisation: the occupied-slot list is built on
 * the device and the group count stays there (view->d_n_groups; view->n_groups is 0 until
 * igx_groupby_wait).  igx_groupby_sort's top-K of such a table (0 < k <= 4096, no float or
 * IP-text key) reads the count on the device, so a whole interval -- reset, update,
 * finalize, sort, gather -- is issued without a host round trip (nextStats' drain,
 * tracer.go:177-226, with no wait in it).  The count and the status igx_groupby_finalize
 * would have returned (IGX_ENOSPC) come back from igx_groupby_wait, or from the first
 * igx_groupby_reset / igx_groupby_finalize that finds the read-back landed (a reset never
 * waits for the device), or, when the next interval's igx_groupby_finalize_async collects it,
 * from that call, which then does NOT issue its own interval (the error text names the failed
 * finalize; calling it again finalizes this interval: a non-zero return always means "not
 * finalized") -- igx_groupby_wait only ever reports the last finalize's own status.  The
 * read-back is written by the kernel that counts the groups into
 * the table's coherent pinned buffer, followed by a sequence number the host polls (no copy
 * and no event on the stream); igx_groupby_wait polls it, and fails with IGX_EIO if the
 * stream drains without it.  Asynchronous. */
int igx_groupby_finalize_async(igx_table *t, igx_table_view *view);
/* Waits for the last igx_groupby_finalize_async: *n_groups (nullable) = its group count;
 * returns its status.  IGX_OK (and the last known count) when none is pending. */
int igx_groupby_wait(igx_table *t, uint64_t *n_groups);
/* Materialise groups idx[0..k) (device u32, e.g. igx_topk output) as packed rows of
 * key_bytes | naggs x u64 | first_idx u64 into out_rows (device) -- the Stats rows
 * nextStats builds (pkg/gadgets/top/tcp/tracer/tracer.go:186-219).  Call after
 * igx_groupby_finalize.  Asynchronous. */
int igx_groupby_gather(igx_table *t, const uint32_t *idx, uint64_t k, uint8_t *out_rows);
/* Per-interval reset (nextStats' Delete loop, tracer.go:154-171): the next interval's groups,
 * sums and first indices are its own.  Keys themselves are kept across intervals while the
 * table runs its cached form: a recurring key is found instead of inserted again, and only the
 * last interval's groups' value records are cleared.  The kept keys end (the next interval
 * starts an empty table) when they plus `capacity` new ones would fill more than 4/5 of the
 * slots, after a failed interval, when an interval runs the direct or partitioned form, or
 * with IGX_GB_PERSIST=0.  Asynchronous. */
int igx_groupby_reset(igx_table *t);
/* How updates run (results are identical in every mode):
 *   IGX_GB_CACHED  one workgroup per CU with an LDS cache of hot keys (Zipf-like streams:
 *                  most rows never leave the CU);
 *   IGX_GB_DIRECT  every row probes the HBM table itself (near-uniform, high-cardinality
 *                  streams, where nearly every row would miss the cache);
 *   IGX_GB_PART    rows are radix-partitioned by key hash in two streamed passes and each
 *                  final bucket is aggregated in LDS, then written to the table with plain
 *                  stores (no atomics; DESIGN.md §4 has its measured cost).  Scratch: two
 *                  record buffers of nrows x 16..128 B;
 *   IGX_GB_AUTO    (default) cached; an interval in which more than 90% of the rows missed
 *                  the cache switches the next 16 intervals to partitioned, then measures
 *                  again.
 * The mode of an interval is fixed by its first update. */
enum igx_gb_mode { IGX_GB_AUTO = 0, IGX_GB_CACHED = 1, IGX_GB_DIRECT = 2, IGX_GB_PART = 3 };
int igx_groupby_set_mode(igx_table *t, uint32_t mode);
/* SortStats over the table's groups (same order as igx_sort_perm with pos = first_idx);
 * writes the first k (0 = all) group slots to out_slots (device u32).  Call after
 * igx_groupby_finalize.  Asynchronous. */
int igx_groupby_sort(igx_table *t, const igx_tsortkey *keys, uint32_t nkeys, uint32_t k,
                     uint32_t *out_slots);
/* Diagnostics (synchronous): out2[0] = top-Ks of this table answered by the hinted path (the
 * slots of the same sort's last top-K bound the k-th key; only the groups at or below the bound
 * are ranked), out2[1] = top-Ks answered by the full selection.  Both give the same slots. */
int igx_groupby_topk_counts(igx_table *t, uint64_t *out2);
int igx_groupby_destroy(igx_table *t);
/* Diagnostics only (IGX_GB_DEBUG env), 32 words: out[0..1] LDS-cache hits / misses (bit 3);
 * out[4..7] sleep counts of loaders on a full miss ring, probers on an empty one, probers on a
 * full update ring, the idle server (bit 16); bit 18, the memory-side atomics: out[8..11] the
 * server wave's updates, of them minima, distinct (value record, opcode) pairs per instruction,
 * distinct (128-B line, opcode) pairs; [12] instructions whose first record continues the
 * previous one's last; [13..15] the distinct (record, opcode) pairs within each 32-, 16- and
 * 8-lane group of the instruction; [16..19] the same four as [8..11] for the final LDS flush's
 * aggregate updates, [20] its minima.  Counters since the last call. */
int igx_groupby_debug_counts(igx_table *t, uint64_t *out32);

/* ---- advise network-policy -------------------------------------------------------------- */
/* keep[i] = 1 iff the advisor would consider event i (advisor.go:279-292): type == normal
 * (0), pkt (PACKET_* code) is HOST (0) or OUTGOING (4), and not (HOST and hostip == raddr).
 * typ/pkt/keep 4-byte aligned, hostip/raddr 16-byte aligned (device).  Asynchronous. */
int igx_np_mark(igx_ctx *ctx, const uint8_t *typ, const uint8_t *pkt, const uint32_t *hostip,
                const uint32_t *raddr, uint64_t nrows, uint8_t *keep);

/* ---- log2 latency histograms ---------------------------------------------------------- */
/* hist[(dev_index(dev)*ncont + cont) * nslots + slot] += 1 for every row with delta >= 0
 * (delta is s64 ns), slot = min(log2l(delta/divisor), nslots-1).  devs (host, ndev <= 64)
 * lists the device numbers (dev_index = position); rows with other devs are ignored.
 * ndev == 0 is the shipped gadget's keying (no targ_per_disk / targ_per_flag): every row
 * is device index 0 and dev may be NULL.  cont may be NULL (ncont must then be 1).
 * hist (device u32, max(ndev,1)*ncont*nslots) accumulates.  Async. */
int igx_hist_log2(igx_ctx *ctx, const uint32_t *dev, const uint32_t *cont,
                  const int64_t *delta, uint64_t nrows, const uint32_t *devs, uint32_t ndev,
                  uint32_t ncont, uint64_t divisor, uint32_t nslots, uint32_t *hist);

/* The raw-key form of the same histograms: biolatency keys its map by hist_key{cmd_flags, dev}
 * when targ_per_flag / targ_per_disk are set (biolatency.bpf.c:116-131), with any values.  Per
 * event, slot[i] = min(log2l(delta[i] / divisor), nslots - 1) and keep[i] = delta[i] >= 0;
 * a group-by with key (cmd_flags, dev, slot) and a COUNT of out_width 4 (the u32 slots) then
 * holds every key's histogram (engine.hist_log2_keyed).  Asynchronous. */
int igx_log2_slots(igx_ctx *ctx, const int64_t *delta, uint64_t nrows, uint64_t divisor, uint32_t nslots,
                   uint8_t *slot, uint8_t *keep);

/* ---- group:sum of float columns, IP text --------------------------------------------- */
/* GroupEntries' float group:sum (group.go:133-156, flattenValues): perm (device u32, n) is a
 * stable sort of the rows by the group key (key_bytes at row * key_stride of keys); each run
 * of equal keys is one group in input order.  For each run, out[first row of the run] =
 * v[first] + v[second] + ... in that order, in float64, rounded to float32 after every add
 * when val_width is 4 (SetFloat on a float32 field).  Rows with valid[row] == 0 (nullable)
 * are nil entries and belong to no run.  Other out entries are left untouched.  Async. */
int igx_segment_fsum(igx_ctx *ctx, const uint8_t *keys, uint32_t key_stride, uint32_t key_bytes,
                     const uint32_t *perm, uint64_t n, const uint8_t *valid, const void *vals,
                     uint32_t val_width, double *out);

/* IPStringFromBytes (pkg/gadgets/helpers.go:111-120) for n rows: addr (16 bytes at row *
 * addr_stride) rendered as netip.AddrFrom16(...).String() when the u16 family at row *
 * family_stride is AF_INET6 (10), else netip.AddrFrom4(addr[0:4]).String().  out (device,
 * 8-byte aligned) receives n x IGX_IPTEXT_WIDTH bytes, each text zero-padded, so byte order
 * of two rows is Go's string order.  rowmap (device, nullable): row r reads row rowmap[r].
 * Asynchronous. */
#define IGX_IPTEXT_WIDTH 40
int igx_ip_text(igx_ctx *ctx, const uint8_t *addr, uint32_t addr_stride, const uint8_t *family,
                uint32_t family_stride, const uint32_t *rowmap, uint64_t n, uint8_t *out);

/* ---- data movement either side of the path ---------------------------------------------- */
/* Sender side of the group-by all-to-all: rows (device, nrows x
 * row_bytes, 4-byte aligned) are copied to out (device, same size) grouped by owner part,
 * stable within a part; owner = FNV-1a(32) over the first key_bytes/4 u32 words of the row,
 * mod nparts (1..64).  part_counts (device u64[nparts]) receives the rows per part.  Async. */
int igx_partition_rows(igx_ctx *ctx, const uint8_t *rows, uint64_t nrows, uint32_t row_bytes,
                       uint32_t key_bytes, uint32_t nparts, uint8_t *out, uint64_t *part_counts);
/* The same partition straight from a finalized table (igx_groupby_finalize or _async): its
 * groups as igx_groupby_gather rows (key words | aggregates wrapped to out_widths[x] bytes
 * (nullable: 8) | first index) grouped by owner part, stable in slot order within a part.  The
 * group count is read on the device (view->d_n_groups), so an asynchronously finalized table
 * is partitioned without a host round trip; out holds cap_rows rows (>= the table's capacity).
 * The sender side of the owner exchange (C4 / C5 at N > 1; replaces the reference's per-node
 * fan-out + client merge, grpc-runtime.go:221-237 -> snapshotcombiner.go:79-106).  Async. */
int igx_partition_groups(igx_ctx *ctx, const igx_table_view *view, const uint32_t *out_widths,
                         uint32_t nparts, uint8_t *out, uint64_t cap_rows, uint64_t *part_counts);
/* ---- multi-GPU merges over RCCL ----------------------------------------
 * One process per GPU.  Replaces the reference's node fan-out + client concatenation
 * (pkg/runtime/grpc/grpc-runtime.go:221-237 -> pkg/snapshotcombiner/snapshotcombiner.go:79-106)
 * with exact merges over xGMI.  Setup: rank 0 calls igx_dist_get_unique_id and hands the
 * IGX_DIST_ID_BYTES bytes to every rank by the caller's own channel (ncclUniqueId); every rank
 * then calls igx_dist_init on its context.  Collectives are enqueued on the context's stream
 * and must be called in the same order on every rank.  The row exchanges all-gather their
 * counts, capacities and an argument-error flag first (they synchronise the stream) and plan
 * with igx_dist_plan_* below, so either every rank proceeds or every rank returns the same
 * error (IGX_ENOSPC, or IGX_EINVAL when some rank's arguments are invalid).  With out == NULL
 * on every rank they are a size query: the counts are exchanged and returned, no rows move.
 * Failure detection: the communicator is non-blocking and every wait inside these calls (a call
 * still being issued, the stream draining after the metadata all-gather, igx_dist_wait) polls
 * ncclCommGetAsyncError under a deadline (IGX_DIST_TIMEOUT_MS, default 120000, or
 * igx_dist_set_timeout).  An RCCL error, an asynchronous error or a missed deadline -- a peer
 * that died mid-collective -- returns IGX_EIO, aborts this rank's communicator (ncclCommAbort:
 * its kernels waiting on the peer exit) and marks it broken: every later call returns IGX_EIO
 * at once.  The reference drops a node that stops answering after its TTL instead of waiting on
 * it (pkg/snapshotcombiner/snapshotcombiner.go:91-100). */
#define IGX_DIST_ID_BYTES 128
typedef struct igx_dist igx_dist;
int igx_dist_get_unique_id(uint8_t *out_id);
int igx_dist_init(igx_ctx *ctx, const uint8_t *id, int nranks, int rank, igx_dist **out);
int igx_dist_destroy(igx_dist *d);
int igx_dist_rank(igx_dist *d, int *rank, int *nranks);
int igx_dist_barrier(igx_dist *d);   /* synchronises (bounded) */
/* The deadline of every wait on this communicator, in ms (> 0). */
int igx_dist_set_timeout(igx_dist *d, int timeout_ms);
/* Bounded hipStreamSynchronize of the context's stream for a caller that must wait on an
 * asynchronous collective (igx_dist_allreduce_u32, the row exchanges' data phase): IGX_EIO, and
 * the communicator aborted, on an RCCL error or when the deadline passes. */
int igx_dist_wait(igx_dist *d);
/* Marks the communicator unusable, as a failed group does: every later call returns IGX_EIO
 * without entering a collective.  For a caller that learned of a peer's failure out of band
 * (e.g. a node's gRPC stream ended, grpc-runtime.go:221-237). */
int igx_dist_mark_broken(igx_dist *d);
/* C3: in-place sum of a u32 buffer (log2 histograms) over all ranks (mod 2^32, exact).  Async. */
int igx_dist_allreduce_u32(igx_dist *d, uint32_t *buf, uint64_t n);
/* Top-K candidate merge (C2, C5): every rank's nrows x row_bytes rows (device) concatenated in
 * rank order into out (device, cap_rows rows); counts (host, nranks, nullable) receives each
 * rank's row count.  Feed the result to igx_topk with the rows' global first index as the
 * position for the exact global top-K. */
int igx_dist_allgather_rows(igx_dist *d, const void *rows, uint64_t nrows, uint32_t row_bytes, void *out,
                            uint64_t cap_rows, uint64_t *counts);
/* Group-by / distinct exchange (C4, C5): rows (device) already grouped by destination rank,
 * send_counts[p] (host) rows for rank p in rank order, go to their rank; out (device,
 * cap_rows rows) receives this rank's rows in source-rank order; recv_counts (host, nranks,
 * nullable) their counts. */
int igx_dist_alltoallv_rows(igx_dist *d, const void *rows, const uint64_t *send_counts, uint32_t row_bytes,
                            void *out, uint64_t cap_rows, uint64_t *recv_counts);
/* igx_partition_rows (owner = FNV-1a of the key words mod nranks) + igx_dist_alltoallv_rows:
 * packed partial-group rows (igx_groupby_gather layout) go to the rank owning their key, which
 * merges them with igx_groupby_update_ex (SUM of partials, MIN of first indices).  *out_nrows =
 * rows received. */
int igx_dist_exchange_groups(igx_dist *d, const void *rows, uint64_t nrows, uint32_t row_bytes,
                             uint32_t key_bytes, void *out, uint64_t cap_rows, uint64_t *out_nrows);
/* The planning step of the row exchanges, as a host function (no GPU, no communicator): every
 * rank calls it on the same all-gathered metadata, so every rank reaches the same decision.
 * meta holds nranks rows, rank r's row written by rank r:
 *   igx_dist_plan_alltoallv: nranks + 2 words = send_counts[0..nranks) | cap_rows | flags
 *   igx_dist_plan_allgather: 3 words          = nrows | cap_rows | flags
 * flags: IGX_DIST_F_BADARG (that rank's own arguments are invalid), IGX_DIST_F_QUERY (a size
 * query: out == NULL).  status: IGX_OK (proceed; for a query on every rank, only the counts are
 * meaningful), IGX_EINVAL (a rank flagged BADARG, or ranks disagree on QUERY), IGX_ENOSPC (a
 * rank's capacity is below the rows it would receive); culprit = that rank (lowest), else -1.
 * Row offsets: send_off[p] = first row this rank sends to rank p (alltoallv; 0 for allgather);
 * recv_off[p] / recv_counts[p] = where rank p's rows land in this rank's output and how many. */
#define IGX_DIST_MAX_RANKS 64
#define IGX_DIST_F_BADARG 1u
#define IGX_DIST_F_QUERY 2u
typedef struct {
    int32_t status;
    int32_t culprit;
    uint64_t total_rows;
    uint64_t recv_counts[IGX_DIST_MAX_RANKS];
    uint64_t send_off[IGX_DIST_MAX_RANKS];
    uint64_t recv_off[IGX_DIST_MAX_RANKS];
} igx_dist_plan;
int igx_dist_plan_alltoallv(int nranks, int rank, const uint64_t *meta, igx_dist_plan *out);
int igx_dist_plan_allgather(int nranks, int rank, const uint64_t *meta, igx_dist_plan *out);

/* The step before the path: array-of-structs records on the device (a BPF
 * map dump of {key, value} structs or perf-ring event structs, e.g. tcptopIpKeyT +
 * tcptopTrafficT, pkg/gadgets/top/tcp/tracer/tcptop_bpfel_x86.go:15-30) are cut into SoA
 * columns: field f (byte offset field_off[f], field_width[f] bytes) of record r goes to
 * out_cols[f] + r * field_width[f].  1..16 fields.  Async. */
/* trace open's perf-ring samples (struct event, pkg/gadgets/trace/open/tracer/bpf/opensnoop.h:14-24,
 * bpf2go opensnoopEvent: ts u64 @0, pid u32 @8, uid u32 @12, mntns u64 @16, ret s32 @24,
 * flags s32 @28, comm[16] @32, fname[255] @48; 304 bytes) -> the Event fields the tracer's
 * run loop fills (trace/open/tracer/tracer.go:182-208):
 *   timestamp = WallTimeFromBootTime(ts) = ts + boot_to_wall_ns;  ret = int(Ret) (sign-
 *   extended); fd = ret >= 0 ? ret : 0;  err = ret < 0 ? -ret : 0;  comm / path =
 *   FromCString (the bytes before the first NUL; the rest of the row zeroed; path rows are
 *   256 bytes, the 255-byte name plus a NUL).
 * samples: device, n x sample_bytes (sample_bytes >= 304, a multiple of 8; 8-byte aligned).
 * Null output columns are skipped.  Asynchronous. */
typedef struct {
    int64_t *timestamp;
    uint32_t *pid;
    uint32_t *uid;
    uint64_t *mntns;
    int64_t *ret;
    int64_t *fd;
    int64_t *err;
    uint8_t *comm;   /* n x 16 */
    uint8_t *path;   /* n x 256 */
} igx_open_cols;
int igx_ingest_open_events(igx_ctx *ctx, const uint8_t *samples, uint64_t n, uint32_t sample_bytes,
                           int64_t boot_to_wall_ns, const igx_open_cols *out);
int igx_ingest_aos(igx_ctx *ctx, const void *records, uint64_t nrec, uint32_t rec_bytes,
                   const uint32_t *field_off, const uint32_t *field_width, uint32_t nfields,
                   void *const *out_cols);

/* ---- test hooks (k_debug.hip; not part of the aggregation path) ----
 * igx_debug_hold_stream: one wave on the context's stream that waits on a host-mapped flag
 * (at most ~max_ms), so a test can make a collective queued behind it miss igx_dist's deadline
 * the way a dead peer would.  igx_debug_release sets the flag, waits for the stream, frees the
 * token; *how = 1 if the wave saw the release, 2 if its own budget ran out. */
int igx_debug_hold_stream(igx_ctx *ctx, uint32_t max_ms, void **token);
int igx_debug_release(igx_ctx *ctx, void *token, uint32_t *how);

/* ---- synthetic event generators (device; bit-identical with oracle/igx_oracle.c) ---- */
int igx_gen_tcp(igx_ctx *ctx, uint64_t seed, uint64_t rank, uint64_t G, uint64_t permA,
                uint64_t permB, const uint64_t *cdf, uint64_t base, uint64_t n, uint8_t *saddr,
                uint8_t *daddr, uint64_t *mntns, uint32_t *pid, uint8_t *comm, uint16_t *lport,
                uint16_t *dport, uint16_t *family, uint32_t *size, uint8_t *dir);
int igx_gen_open(igx_ctx *ctx, uint64_t seed, const uint64_t *comm_cdf, uint64_t base,
                 uint64_t n, uint32_t *pid, uint32_t *uid, uint64_t *mntns, uint8_t *comm,
                 int64_t *ret, int64_t *fd, int64_t *err, uint32_t *path_id);
int igx_gen_bio(igx_ctx *ctx, uint64_t seed, const uint64_t *q, uint64_t nq, uint64_t base,
                uint64_t n, uint32_t *dev, uint32_t *cont, uint64_t *delta);
int igx_gen_np(igx_ctx *ctx, uint64_t seed, uint64_t nsrc, uint64_t npeer, uint64_t base,
               uint64_t n, uint32_t *src, uint32_t *peer, uint16_t *port, uint8_t *pkt,
               uint8_t *typ, uint8_t *proto, uint32_t *hostip, uint32_t *raddr);
int igx_gen_file(igx_ctx *ctx, uint64_t seed, uint64_t rank, uint64_t G, uint64_t permA,
                 uint64_t permB, const uint64_t *cdf, uint64_t base, uint64_t n,
                 uint64_t *inode, uint32_t *dev, uint32_t *pid, uint32_t *tid, uint8_t *op,
                 uint32_t *count);

#ifdef __cplusplus
}
#endif
#endif /* IGX_H */
