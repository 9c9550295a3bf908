// igx_dist.cpp -- the multi-GPU merges of the aggregation path over RCCL (xGMI inside one
// node), behind the C ABI so a cgo caller gets the same entry points as the Python host.
//
// The reference merges node shards by concatenating per-node arrays on the client
// (pkg/snapshotcombiner/snapshotcombiner.go:79-106, fed by one gRPC stream per node,
// pkg/runtime/grpc/grpc-runtime.go:221-237).  Here one process drives one GPU and the shards
// are merged exactly:
//   igx_dist_allreduce_u32    dense log2 histograms (C3): ncclAllReduce(ncclUint32, ncclSum)
//   igx_dist_alltoallv_rows   partial groups to the rank owning their key (C4, C5)
//   igx_dist_exchange_groups  igx_partition_rows + igx_dist_alltoallv_rows
//   igx_dist_allgather_rows   per-rank top-K candidates (C2, C5) for the final igx_topk
// Every collective runs on the context's stream.  Calls that must size their output (the
// row exchanges) first all-gather their counts and capacities, so every rank takes the same
// decision (proceed, or IGX_ENOSPC on all ranks) and no rank is left waiting in a send.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "igx_internal.h"

struct igx_dist {
    igx_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    int timeout_ms = 0;           // bound on every wait (IGX_DIST_TIMEOUT_MS / igx_dist_set_timeout)
    bool broken = false;          // a call failed or timed out: the communicator is aborted and unusable
    uint64_t *d_meta = nullptr;   // device: own meta, then all ranks' meta (sized at init)
    uint64_t *h_meta = nullptr;   // pinned host copy of all ranks' meta
    size_t meta_words = 0;        // per-rank words the buffers hold
    uint8_t *part = nullptr;      // exchange_groups: rows grouped by owner
    size_t part_bytes = 0;
    uint64_t *d_cnt = nullptr;    // exchange_groups: rows per owner
    std::thread *aborter = nullptr;                  // runs ncclCommAbort (see dist_abort)
    std::shared_ptr<std::atomic<int>> abort_done;    // set by the aborter when ncclCommAbort returned
};

// ---- failure detection ----------------------------------------------------------------
// The communicator is non-blocking (ncclConfig_t.blocking = 0): no RCCL call waits on a peer
// inside the library.  Every wait -- a call still being issued (ncclInProgress), or the
// stream draining after a collective -- polls ncclCommGetAsyncError under a deadline.  A peer
// that died mid-collective therefore surfaces as IGX_EIO on every survivor within the
// deadline instead of a hang; the survivors' communicators are aborted (ncclCommAbort makes
// their RCCL kernels that wait on the dead peer exit) and marked broken, so every later call
// fails at once.  The reference's counterpart drops a silent node after its TTL instead of
// waiting on it (pkg/snapshotcombiner/snapshotcombiner.go:91-100; grpc-runtime.go:312-315
// ends a node's stream on error).
static constexpr int DEFAULT_TIMEOUT_MS = 120000;

static int env_timeout_ms() {
    const char *e = std::getenv("IGX_DIST_TIMEOUT_MS");
    if (e && *e) {
        const long v = std::strtol(e, nullptr, 10);
        if (v > 0 && v < (1L << 30)) return (int)v;
    }
    return DEFAULT_TIMEOUT_MS;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ncclCommAbort runs on a helper thread: it returns once the communicator's own work has left
// the GPU, and RCCL orders that work after whatever was queued before it on the caller's stream.
// A collective waiting on a dead peer exits at once on the abort; work queued ahead of it in
// the stream (another library's kernel, a stalled copy) may take longer, and this rank's call
// must still fail within the deadline.  igx_dist_destroy reaps the thread.
static void dist_abort(igx_dist *d) {
    d->broken = true;
    if (d->comm && !d->aborter) {
        ncclComm_t c = d->comm;
        d->comm = nullptr;
        auto done = std::make_shared<std::atomic<int>>(0);
        d->abort_done = done;
        d->aborter = new std::thread([c, done] {
            (void)ncclCommAbort(c);
            done->store(1, std::memory_order_release);
        });
    }
}

// waits up to wait_ms for the aborter; true when it finished (joined), false when it is still
// blocked (detached: it owns only the communicator handle and its own flag)
static bool dist_reap(igx_dist *d, int wait_ms) {
    if (!d->aborter) return true;
    const double t0 = now_ms();
    while (!d->abort_done->load(std::memory_order_acquire) && now_ms() - t0 < wait_ms)
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    const bool done = d->abort_done->load(std::memory_order_acquire) != 0;
    if (done) d->aborter->join();
    else d->aborter->detach();
    delete d->aborter;
    d->aborter = nullptr;
    return done;
}

// marks the communicator broken (aborting it) and fails the call with IGX_EIO
static int dist_fail(igx_dist *d, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int dist_fail(igx_dist *d, const char *fmt, ...) {
    char buf[768];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    dist_abort(d);
    return igx_fail(d->ctx, IGX_EIO, "%s (communicator aborted)", buf);
}

// an RCCL call's result on the non-blocking communicator: ncclInProgress is polled until the
// call is issued, under the deadline; any error aborts the communicator
static int nccl_settle(igx_dist *d, ncclResult_t r, const char *what) {
    const double t0 = now_ms();
    while (r == ncclInProgress) {
        if (now_ms() - t0 > d->timeout_ms) return dist_fail(d, "%s: not issued within %d ms", what, d->timeout_ms);
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (ncclCommGetAsyncError(d->comm, &r) != ncclSuccess) r = ncclInternalError;
    }
    if (r != ncclSuccess) return dist_fail(d, "%s: %s", what, ncclGetErrorString(r));
    return IGX_OK;
}

// waits for the context's stream (collectives included) under the deadline, watching the
// communicator's asynchronous error: the bounded replacement of hipStreamSynchronize
static int dist_sync(igx_dist *d, const char *what) {
    igx_ctx *ctx = d->ctx;
    const double t0 = now_ms();
    for (;;) {
        const hipError_t e = hipStreamQuery(ctx->stream);
        if (e == hipSuccess) return IGX_OK;
        if (e != hipErrorNotReady) {
            return dist_fail(d, "%s: %s", what, hipGetErrorString(e));
        }
        ncclResult_t a = ncclSuccess;
        if (d->comm && ncclCommGetAsyncError(d->comm, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress) {
            return dist_fail(d, "%s: asynchronous error %s", what, ncclGetErrorString(a));
        }
        if (now_ms() - t0 > d->timeout_ms) {
            return dist_fail(d, "%s: timed out after %d ms", what, d->timeout_ms);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

#define IGX_DIST_LIVE(d)                                                                  \
    do {                                                                                  \
        if ((d)->broken || !(d)->comm)                                                    \
            return igx_fail((d)->ctx, IGX_EIO, "dist: communicator broken by an earlier failure"); \
    } while (0)
// an RCCL call outside a group
#define IGX_NCCL(d, expr)                                      \
    do {                                                       \
        int rc_ = nccl_settle((d), (expr), #expr);             \
        if (rc_) return rc_;                                   \
    } while (0)
// inside ncclGroupStart/End: a failure aborts the communicator (which ends the group) and
// marks it broken -- the peers' matching sends / receives may never complete
#define IGX_NCCL_G(d, expr)                                                                  \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess && r_ != ncclInProgress) {                                     \
            (void)ncclGroupEnd();   /* the group depth is per thread: close it first */     \
            return dist_fail((d), "%s: %s", #expr, ncclGetErrorString(r_));                 \
        }                                                                                    \
    } while (0)
#define IGX_NCCL_END(d) IGX_NCCL(d, ncclGroupEnd())

// the widest per-rank meta row any call gathers: alltoallv's send counts, capacity, flags
static constexpr size_t META_WORDS = IGX_DIST_MAX_RANKS + 2;

// ---- planning (host only; tests/test_dist_plan.py checks it against gloo's all-to-all) ----
static void plan_reset(igx_dist_plan *p) {
    std::memset(p, 0, sizeof *p);
    p->culprit = -1;
}

extern "C" int igx_dist_plan_alltoallv(int nranks, int rank, const uint64_t *meta, igx_dist_plan *p) {
    if (!p || !meta || nranks < 1 || nranks > IGX_DIST_MAX_RANKS || rank < 0 || rank >= nranks) return IGX_EINVAL;
    plan_reset(p);
    const size_t W = (size_t)nranks + 2;
    auto row = [&](int r) { return meta + (size_t)r * W; };
    const uint64_t q0 = row(0)[nranks + 1] & IGX_DIST_F_QUERY;
    for (int r = 0; r < nranks && p->culprit < 0; ++r)
        if ((row(r)[nranks + 1] & IGX_DIST_F_BADARG) || (row(r)[nranks + 1] & IGX_DIST_F_QUERY) != q0) {
            p->status = IGX_EINVAL;
            p->culprit = r;
        }
    uint64_t soff = 0, roff = 0;
    for (int q = 0; q < nranks; ++q) {
        p->send_off[q] = soff;
        soff += row(rank)[q];
        p->recv_counts[q] = row(q)[rank];
        p->recv_off[q] = roff;
        roff += p->recv_counts[q];
    }
    p->total_rows = roff;
    if (p->status || q0) return IGX_OK;
    for (int dst = 0; dst < nranks; ++dst) {   // every rank sees every capacity: all fail or none does
        uint64_t tot = 0;
        for (int src = 0; src < nranks; ++src) tot += row(src)[dst];
        if (tot > row(dst)[nranks]) {
            p->status = IGX_ENOSPC;
            p->culprit = dst;
            break;
        }
    }
    return IGX_OK;
}

extern "C" int igx_dist_plan_allgather(int nranks, int rank, const uint64_t *meta, igx_dist_plan *p) {
    if (!p || !meta || nranks < 1 || nranks > IGX_DIST_MAX_RANKS || rank < 0 || rank >= nranks) return IGX_EINVAL;
    plan_reset(p);
    const uint64_t q0 = meta[2] & IGX_DIST_F_QUERY;
    for (int r = 0; r < nranks && p->culprit < 0; ++r)
        if ((meta[3 * r + 2] & IGX_DIST_F_BADARG) || (meta[3 * r + 2] & IGX_DIST_F_QUERY) != q0) {
            p->status = IGX_EINVAL;
            p->culprit = r;
        }
    uint64_t off = 0;
    for (int r = 0; r < nranks; ++r) {
        p->recv_counts[r] = meta[3 * r];
        p->recv_off[r] = off;
        off += meta[3 * r];
    }
    p->total_rows = off;
    if (p->status || q0) return IGX_OK;
    for (int r = 0; r < nranks; ++r)
        if (off > meta[3 * r + 1]) {
            p->status = IGX_ENOSPC;
            p->culprit = r;
            break;
        }
    return IGX_OK;
}

extern "C" int igx_dist_get_unique_id(uint8_t *out_id) {
    if (!out_id) return IGX_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return IGX_EIO;
    std::memcpy(out_id, id.internal, IGX_DIST_ID_BYTES);
    return IGX_OK;
}

extern "C" int igx_dist_init(igx_ctx *ctx, const uint8_t *id, int nranks, int rank, igx_dist **out) {
    if (!ctx || !id || !out) return IGX_EINVAL;
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks)   // every rank gets the same nranks: all fail alike
        return igx_fail(ctx, IGX_EINVAL, "dist_init: rank %d of %d", rank, nranks);
    if (nranks > IGX_DIST_MAX_RANKS)
        return igx_fail(ctx, IGX_ENOTSUP, "dist_init: more than %d ranks", IGX_DIST_MAX_RANKS);
    auto *d = new igx_dist();
    d->ctx = ctx;
    d->rank = rank;
    d->nranks = nranks;
    d->timeout_ms = env_timeout_ms();
    // A local failure (device, allocation) must not skip the communicator's creation: the
    // peers' ncclCommInitRank waits for every rank.  Such a rank joins, then aborts its side.
    // The metadata buffers are sized once here, so no collective ever allocates.
    const hipError_t dev_e = hipSetDevice(ctx->device);
    const bool mem_ok =
        dev_e == hipSuccess && hipMalloc(&d->d_meta, META_WORDS * (nranks + 1) * 8) == hipSuccess &&
        hipHostMalloc(reinterpret_cast<void **>(&d->h_meta), META_WORDS * (nranks + 1) * 8, hipHostMallocDefault) ==
            hipSuccess;
    d->meta_words = META_WORDS;
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, IGX_DIST_ID_BYTES);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;   // every wait is ours, under the deadline (nccl_settle / dist_sync)
    int rc = nccl_settle(d, ncclCommInitRankConfig(&d->comm, nranks, uid, rank, &cfg), "ncclCommInitRankConfig");
    if (!rc && !mem_ok) dist_abort(d);
    if (rc || !mem_ok) {
        (void)dist_reap(d, d->timeout_ms);
        (void)hipFree(d->d_meta);
        (void)hipHostFree(d->h_meta);
        delete d;
        if (rc) return rc;   // ctx->err names the RCCL failure or the timeout
        if (dev_e != hipSuccess) return igx_fail(ctx, IGX_EIO, "dist_init: hipSetDevice(%d): %s", ctx->device,
                                                 hipGetErrorString(dev_e));
        return igx_fail(ctx, IGX_ENOMEM, "dist_init: metadata buffers");
    }
    *out = d;
    return IGX_OK;
}

extern "C" int igx_dist_set_timeout(igx_dist *d, int timeout_ms) {
    if (!d || timeout_ms <= 0) return IGX_EINVAL;
    d->timeout_ms = timeout_ms;
    return IGX_OK;
}

extern "C" int igx_dist_wait(igx_dist *d) {
    if (!d) return IGX_EINVAL;
    IGX_DIST_LIVE(d);
    return dist_sync(d, "dist_wait");
}

extern "C" int igx_dist_destroy(igx_dist *d) {
    if (!d) return IGX_OK;
    // a stream that cannot drain within the deadline (a peer died and some kernel still runs)
    // keeps the buffers: freeing memory a running kernel uses is worse than a leak
    bool drained;
    if (d->comm) {
        drained = dist_sync(d, "dist_destroy") == IGX_OK;   // aborts the communicator on failure
    } else {
        const double t0 = now_ms();
        const int bound = d->broken ? std::min(d->timeout_ms, 2000) : d->timeout_ms;   // broken: deadline spent
        hipError_t e;
        while ((e = hipStreamQuery(d->ctx->stream)) == hipErrorNotReady && now_ms() - t0 < bound)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        drained = e == hipSuccess;
    }
    if (d->comm) {
        if (nccl_settle(d, ncclCommFinalize(d->comm), "ncclCommFinalize") == IGX_OK) {
            (void)ncclCommDestroy(d->comm);
            d->comm = nullptr;
        }
    }
    // a broken communicator already spent its deadline in the call that failed (and, above, in
    // the drain): its aborter gets a short bound here, so destroy waits at most one deadline plus
    // that bound.  An aborter still blocked is detached by dist_reap and stays
    // inside ncclCommAbort; its buffers are kept (a process exiting meanwhile ends it with the
    // process: it touches nothing this library frees).
    if (!dist_reap(d, d->broken ? std::min(d->timeout_ms, 2000) : d->timeout_ms)) drained = false;
    if (drained) {
        (void)hipFree(d->d_meta);
        (void)hipHostFree(d->h_meta);
        (void)hipFree(d->part);
        (void)hipFree(d->d_cnt);
    }
    delete d;
    return IGX_OK;
}

extern "C" int igx_dist_mark_broken(igx_dist *d) {
    if (!d) return IGX_EINVAL;
    dist_abort(d);   // this rank's RCCL kernels that wait on the failed peer exit too
    return IGX_OK;
}

extern "C" int igx_dist_rank(igx_dist *d, int *rank, int *nranks) {
    if (!d) return IGX_EINVAL;
    if (rank) *rank = d->rank;
    if (nranks) *nranks = d->nranks;
    return IGX_OK;
}

// All-gather `words` (<= META_WORDS) u64 of host meta from every rank into
// d->h_meta[rank * words + i].  Synchronises the stream.  Allocates nothing.
static int gather_meta(igx_dist *d, const uint64_t *mine, size_t words) {
    igx_ctx *ctx = d->ctx;
    IGX_DIST_LIVE(d);
    if (words > d->meta_words) return igx_fail(ctx, IGX_EINVAL, "dist: %zu meta words", words);
    uint64_t *h_send = d->h_meta + words * d->nranks;   // the spare row of the pinned buffer
    std::memcpy(h_send, mine, words * 8);
    IGX_HIP(ctx, hipMemcpyAsync(d->d_meta, h_send, words * 8, hipMemcpyHostToDevice, ctx->stream));
    IGX_NCCL(d, ncclAllGather(d->d_meta, d->d_meta + words, words, ncclUint64, d->comm, ctx->stream));
    IGX_HIP(ctx, hipMemcpyAsync(d->h_meta, d->d_meta + words, words * d->nranks * 8, hipMemcpyDeviceToHost,
                                ctx->stream));
    return dist_sync(d, "dist: metadata all-gather");
}

static int plan_fail(igx_dist *d, const igx_dist_plan &p, const char *what) {
    if (p.status == IGX_ENOSPC)
        return igx_fail(d->ctx, IGX_ENOSPC, "%s: %llu rows exceed rank %d's capacity", what,
                        (unsigned long long)p.total_rows, p.culprit);
    return igx_fail(d->ctx, p.status, "%s: invalid arguments on rank %d", what, p.culprit);
}

extern "C" int igx_dist_allreduce_u32(igx_dist *d, uint32_t *buf, uint64_t n) {
    if (!d) return IGX_EINVAL;
    IGX_DIST_LIVE(d);
    if (n == 0) return IGX_OK;
    if (!buf) {
        // the peers are already in (or will enter) the all-reduce of n words: take part with
        // zeros so they complete, then fail this rank's call
        void *z = nullptr;
        if (igx_scratch(d->ctx, n * 4, &z) || hipMemsetAsync(z, 0, n * 4, d->ctx->stream) != hipSuccess ||
            nccl_settle(d, ncclAllReduce(z, z, n, ncclUint32, ncclSum, d->comm, d->ctx->stream), "ncclAllReduce"))
            dist_abort(d);
        return igx_fail(d->ctx, IGX_EINVAL, "dist_allreduce: null buffer");
    }
    // u32 addition mod 2^32 is exact and order-independent: the merged histogram equals the
    // histogram of the union of every rank's events
    IGX_NCCL(d, ncclAllReduce(buf, buf, n, ncclUint32, ncclSum, d->comm, d->ctx->stream));
    return IGX_OK;
}

extern "C" int igx_dist_barrier(igx_dist *d) {
    if (!d) return IGX_EINVAL;
    uint64_t zero = 0;
    int rc = gather_meta(d, &zero, 1);
    return rc;
}

extern "C" int igx_dist_allgather_rows(igx_dist *d, const void *rows, uint64_t nrows, uint32_t row_bytes,
                                       void *out, uint64_t cap_rows, uint64_t *counts) {
    if (!d) return IGX_EINVAL;
    igx_ctx *ctx = d->ctx;
    // local argument checks travel with the counts, so a bad call fails on every rank
    const bool bad = row_bytes == 0 || (out && nrows && !rows);
    const uint64_t mine[3] = {nrows, cap_rows, (bad ? IGX_DIST_F_BADARG : 0u) | (out ? 0u : IGX_DIST_F_QUERY)};
    int rc = gather_meta(d, mine, 3);
    if (rc) return rc;
    igx_dist_plan p;
    (void)igx_dist_plan_allgather(d->nranks, d->rank, d->h_meta, &p);
    if (p.status) return plan_fail(d, p, "dist_allgather");
    const int nr = d->nranks;
    if (counts) std::memcpy(counts, p.recv_counts, nr * 8);
    if (!out) return IGX_OK;   // size query (every rank passes a NULL out)
    auto *o = static_cast<uint8_t *>(out);
    if (nrows)
        IGX_HIP(ctx, hipMemcpyAsync(o + p.recv_off[d->rank] * row_bytes, rows, nrows * row_bytes,
                                    hipMemcpyDeviceToDevice, ctx->stream));
    IGX_NCCL(d, ncclGroupStart());
    for (int q = 0; q < nr; ++q) {
        if (q == d->rank) continue;
        if (nrows) IGX_NCCL_G(d, ncclSend(rows, nrows * row_bytes, ncclUint8, q, d->comm, ctx->stream));
        if (p.recv_counts[q])
            IGX_NCCL_G(d, ncclRecv(o + p.recv_off[q] * row_bytes, p.recv_counts[q] * row_bytes, ncclUint8, q, d->comm,
                                   ctx->stream));
    }
    IGX_NCCL_END(d);
    return IGX_OK;
}

extern "C" int igx_dist_alltoallv_rows(igx_dist *d, const void *rows, const uint64_t *send_counts,
                                       uint32_t row_bytes, void *out, uint64_t cap_rows, uint64_t *recv_counts) {
    if (!d) return IGX_EINVAL;
    igx_ctx *ctx = d->ctx;
    const int nr = d->nranks;
    uint64_t mine[META_WORDS] = {};
    uint64_t nsend = 0;
    for (int q = 0; q < nr && send_counts; ++q) nsend += (mine[q] = send_counts[q]);
    mine[nr] = cap_rows;
    const bool bad = row_bytes == 0 || !send_counts || (out && nsend && !rows);
    mine[nr + 1] = (bad ? IGX_DIST_F_BADARG : 0u) | (out ? 0u : IGX_DIST_F_QUERY);
    int rc = gather_meta(d, mine, nr + 2);
    if (rc) return rc;
    igx_dist_plan p;
    (void)igx_dist_plan_alltoallv(nr, d->rank, d->h_meta, &p);
    if (p.status) return plan_fail(d, p, "dist_alltoallv");
    if (recv_counts) std::memcpy(recv_counts, p.recv_counts, nr * 8);
    if (!out) return IGX_OK;   // size query (every rank passes a NULL out)
    const auto *s = static_cast<const uint8_t *>(rows);
    auto *o = static_cast<uint8_t *>(out);
    const uint64_t self = send_counts[d->rank];
    if (self)
        IGX_HIP(ctx, hipMemcpyAsync(o + p.recv_off[d->rank] * row_bytes, s + p.send_off[d->rank] * row_bytes,
                                    self * row_bytes, hipMemcpyDeviceToDevice, ctx->stream));
    IGX_NCCL(d, ncclGroupStart());
    for (int q = 0; q < nr; ++q) {
        if (q == d->rank) continue;
        const uint64_t sc = send_counts[q], rcv = p.recv_counts[q];
        if (sc) IGX_NCCL_G(d, ncclSend(s + p.send_off[q] * row_bytes, sc * row_bytes, ncclUint8, q, d->comm, ctx->stream));
        if (rcv) IGX_NCCL_G(d, ncclRecv(o + p.recv_off[q] * row_bytes, rcv * row_bytes, ncclUint8, q, d->comm, ctx->stream));
    }
    IGX_NCCL_END(d);
    return IGX_OK;
}

extern "C" int igx_dist_exchange_groups(igx_dist *d, const void *rows, uint64_t nrows, uint32_t row_bytes,
                                        uint32_t key_bytes, void *out, uint64_t cap_rows, uint64_t *out_nrows) {
    if (!d) return IGX_EINVAL;
    igx_ctx *ctx = d->ctx;
    const int nr = d->nranks;
    // a local failure (allocation, partition) must not skip the all-to-all's metadata
    // exchange, or the other ranks wait in it forever: it is reported as a bad argument there,
    // so every rank fails together
    int lerr = IGX_OK;
    const size_t need = (size_t)nrows * row_bytes;
    if (need > d->part_bytes) {
        if (dist_sync(d, "dist_exchange_groups")) return IGX_EIO;   // the buffer may still be read
        (void)hipFree(d->part);
        d->part = nullptr;
        d->part_bytes = 0;
        if (hipMalloc(&d->part, igx_align(std::max<size_t>(need, 1), 1 << 20)) == hipSuccess)
            d->part_bytes = igx_align(std::max<size_t>(need, 1), 1 << 20);
        else
            lerr = IGX_ENOMEM;
    }
    if (!lerr && !d->d_cnt && hipMalloc(&d->d_cnt, IGX_DIST_MAX_RANKS * 8) != hipSuccess) lerr = IGX_ENOMEM;
    uint64_t cnt[IGX_DIST_MAX_RANKS] = {};
    if (!lerr && nrows) {
        lerr = igx_partition_rows(ctx, static_cast<const uint8_t *>(rows), nrows, row_bytes, key_bytes, (uint32_t)nr,
                                  d->part, d->d_cnt);
        if (!lerr && hipMemcpyAsync(cnt, d->d_cnt, nr * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
            lerr = IGX_EIO;
        if (!lerr && dist_sync(d, "dist_exchange_groups: partition counts")) return IGX_EIO;   // aborted: no peer waits
    }
    uint64_t rc_[IGX_DIST_MAX_RANKS] = {};
    if (lerr) {
        const uint64_t zero[IGX_DIST_MAX_RANKS] = {};
        (void)igx_dist_alltoallv_rows(d, nullptr, zero, 0 /* flags this rank BADARG */, out, cap_rows, rc_);
        return igx_fail(ctx, lerr, "dist_exchange_groups: local failure on rank %d (%d)", d->rank, lerr);
    }
    int rc = igx_dist_alltoallv_rows(d, d->part, cnt, row_bytes, out, cap_rows, rc_);
    if (rc) return rc;
    uint64_t tot = 0;
    for (int q = 0; q < nr; ++q) tot += rc_[q];
    if (out_nrows) *out_nrows = tot;
    return IGX_OK;
}
