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
#include <cstring>
#include <vector>

#include "igx_internal.h"

struct igx_dist {
    igx_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    uint64_t *d_meta = nullptr;   // device: own meta, then all ranks' meta
    uint64_t *h_meta = nullptr;   // pinned host copy of all ranks' meta
    size_t meta_words = 0;        // per-rank words the buffers hold
    uint8_t *part = nullptr;      // exchange_groups: rows grouped by owner
    size_t part_bytes = 0;
    uint64_t *d_cnt = nullptr;    // exchange_groups: rows per owner
};

#define IGX_NCCL(d, expr)                                                                   \
    do {                                                                                    \
        ncclResult_t r_ = (expr);                                                           \
        if (r_ != ncclSuccess)                                                              \
            return igx_fail((d)->ctx, IGX_EIO, "%s: %s", #expr, ncclGetErrorString(r_));    \
    } while (0)

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
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return igx_fail(ctx, IGX_EINVAL, "dist_init: rank %d of %d", rank, nranks);
    IGX_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, IGX_DIST_ID_BYTES);
    auto *d = new igx_dist();
    d->ctx = ctx;
    d->rank = rank;
    d->nranks = nranks;
    const ncclResult_t r = ncclCommInitRank(&d->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete d;
        return igx_fail(ctx, IGX_EIO, "ncclCommInitRank(%d of %d): %s", rank, nranks, ncclGetErrorString(r));
    }
    *out = d;
    return IGX_OK;
}

extern "C" int igx_dist_destroy(igx_dist *d) {
    if (!d) return IGX_OK;
    (void)hipStreamSynchronize(d->ctx->stream);
    if (d->comm) (void)ncclCommDestroy(d->comm);
    (void)hipFree(d->d_meta);
    (void)hipHostFree(d->h_meta);
    (void)hipFree(d->part);
    (void)hipFree(d->d_cnt);
    delete d;
    return IGX_OK;
}

extern "C" int igx_dist_rank(igx_dist *d, int *rank, int *nranks) {
    if (!d) return IGX_EINVAL;
    if (rank) *rank = d->rank;
    if (nranks) *nranks = d->nranks;
    return IGX_OK;
}

// All-gather `words` u64 of host meta from every rank into d->h_meta[rank * words + i].
// Synchronises the stream.
static int gather_meta(igx_dist *d, const uint64_t *mine, size_t words) {
    igx_ctx *ctx = d->ctx;
    if (words > d->meta_words) {
        (void)hipFree(d->d_meta);
        (void)hipHostFree(d->h_meta);
        d->d_meta = nullptr;
        d->h_meta = nullptr;
        d->meta_words = 0;
        IGX_HIP(ctx, hipMalloc(&d->d_meta, words * (d->nranks + 1) * 8));
        IGX_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&d->h_meta), words * (d->nranks + 1) * 8,
                                   hipHostMallocDefault));
        d->meta_words = words;
    }
    uint64_t *h_send = d->h_meta + words * d->nranks;   // the spare row of the pinned buffer
    std::memcpy(h_send, mine, words * 8);
    IGX_HIP(ctx, hipMemcpyAsync(d->d_meta, h_send, words * 8, hipMemcpyHostToDevice, ctx->stream));
    IGX_NCCL(d, ncclAllGather(d->d_meta, d->d_meta + words, words, ncclUint64, d->comm, ctx->stream));
    IGX_HIP(ctx, hipMemcpyAsync(d->h_meta, d->d_meta + words, words * d->nranks * 8, hipMemcpyDeviceToHost,
                                ctx->stream));
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return IGX_OK;
}

extern "C" int igx_dist_allreduce_u32(igx_dist *d, uint32_t *buf, uint64_t n) {
    if (!d) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (!buf) return igx_fail(d->ctx, IGX_EINVAL, "dist_allreduce: null buffer");
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
    if (row_bytes == 0) return igx_fail(ctx, IGX_EINVAL, "dist_allgather: zero row width");
    const uint64_t mine[2] = {nrows, cap_rows};
    int rc = gather_meta(d, mine, 2);
    if (rc) return rc;
    const int nr = d->nranks;
    std::vector<uint64_t> cnt(nr), off(nr + 1, 0);
    for (int r = 0; r < nr; ++r) {
        cnt[r] = d->h_meta[2 * r];
        off[r + 1] = off[r] + cnt[r];
    }
    if (counts) std::memcpy(counts, cnt.data(), nr * 8);
    if (!out) return IGX_OK;   // size query (every rank passes a NULL out)
    for (int r = 0; r < nr; ++r)   // every rank sees every capacity: all fail or none does
        if (off[nr] > d->h_meta[2 * r + 1])
            return igx_fail(ctx, IGX_ENOSPC, "dist_allgather: %llu rows exceed rank %d's capacity %llu",
                            (unsigned long long)off[nr], r, (unsigned long long)d->h_meta[2 * r + 1]);
    if (nrows && !rows) return igx_fail(ctx, IGX_EINVAL, "dist_allgather: null rows");
    auto *o = static_cast<uint8_t *>(out);
    if (nrows)
        IGX_HIP(ctx, hipMemcpyAsync(o + off[d->rank] * row_bytes, rows, nrows * row_bytes, hipMemcpyDeviceToDevice,
                                    ctx->stream));
    IGX_NCCL(d, ncclGroupStart());
    for (int p = 0; p < nr; ++p) {
        if (p == d->rank) continue;
        if (nrows) IGX_NCCL(d, ncclSend(rows, nrows * row_bytes, ncclUint8, p, d->comm, ctx->stream));
        if (cnt[p]) IGX_NCCL(d, ncclRecv(o + off[p] * row_bytes, cnt[p] * row_bytes, ncclUint8, p, d->comm, ctx->stream));
    }
    IGX_NCCL(d, ncclGroupEnd());
    return IGX_OK;
}

extern "C" int igx_dist_alltoallv_rows(igx_dist *d, const void *rows, const uint64_t *send_counts,
                                       uint32_t row_bytes, void *out, uint64_t cap_rows, uint64_t *recv_counts) {
    if (!d) return IGX_EINVAL;
    igx_ctx *ctx = d->ctx;
    const int nr = d->nranks;
    if (row_bytes == 0 || !send_counts) return igx_fail(ctx, IGX_EINVAL, "dist_alltoallv: bad arguments");
    std::vector<uint64_t> mine(nr + 1);
    for (int p = 0; p < nr; ++p) mine[p] = send_counts[p];
    mine[nr] = cap_rows;
    int rc = gather_meta(d, mine.data(), nr + 1);
    if (rc) return rc;
    const uint64_t *M = d->h_meta;   // M[src * (nr + 1) + dst], caps at column nr
    if (!out) {   // size query (every rank passes a NULL out)
        if (recv_counts)
            for (int p = 0; p < nr; ++p) recv_counts[p] = M[p * (nr + 1) + d->rank];
        return IGX_OK;
    }
    for (int dst = 0; dst < nr; ++dst) {
        uint64_t tot = 0;
        for (int src = 0; src < nr; ++src) tot += M[src * (nr + 1) + dst];
        if (tot > M[dst * (nr + 1) + nr])
            return igx_fail(ctx, IGX_ENOSPC, "dist_alltoallv: %llu rows exceed rank %d's capacity %llu",
                            (unsigned long long)tot, dst, (unsigned long long)M[dst * (nr + 1) + nr]);
    }
    std::vector<uint64_t> soff(nr + 1, 0), roff(nr + 1, 0);
    for (int p = 0; p < nr; ++p) {
        soff[p + 1] = soff[p] + send_counts[p];
        roff[p + 1] = roff[p] + M[p * (nr + 1) + d->rank];
    }
    if (recv_counts)
        for (int p = 0; p < nr; ++p) recv_counts[p] = roff[p + 1] - roff[p];
    if (soff[nr] && !rows) return igx_fail(ctx, IGX_EINVAL, "dist_alltoallv: null rows");
    const auto *s = static_cast<const uint8_t *>(rows);
    auto *o = static_cast<uint8_t *>(out);
    const uint64_t self = send_counts[d->rank];
    if (self)
        IGX_HIP(ctx, hipMemcpyAsync(o + roff[d->rank] * row_bytes, s + soff[d->rank] * row_bytes, self * row_bytes,
                                    hipMemcpyDeviceToDevice, ctx->stream));
    IGX_NCCL(d, ncclGroupStart());
    for (int p = 0; p < nr; ++p) {
        if (p == d->rank) continue;
        const uint64_t sc = send_counts[p], rcv = roff[p + 1] - roff[p];
        if (sc) IGX_NCCL(d, ncclSend(s + soff[p] * row_bytes, sc * row_bytes, ncclUint8, p, d->comm, ctx->stream));
        if (rcv) IGX_NCCL(d, ncclRecv(o + roff[p] * row_bytes, rcv * row_bytes, ncclUint8, p, d->comm, ctx->stream));
    }
    IGX_NCCL(d, ncclGroupEnd());
    return IGX_OK;
}

extern "C" int igx_dist_exchange_groups(igx_dist *d, const void *rows, uint64_t nrows, uint32_t row_bytes,
                                        uint32_t key_bytes, void *out, uint64_t cap_rows, uint64_t *out_nrows) {
    if (!d) return IGX_EINVAL;
    igx_ctx *ctx = d->ctx;
    const int nr = d->nranks;
    if (nr > 64) return igx_fail(ctx, IGX_ENOTSUP, "dist_exchange_groups: more than 64 ranks");
    const size_t need = (size_t)nrows * row_bytes;
    if (need > d->part_bytes) {
        IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
        (void)hipFree(d->part);
        d->part = nullptr;
        d->part_bytes = 0;
        IGX_HIP(ctx, hipMalloc(&d->part, igx_align(std::max<size_t>(need, 1), 1 << 20)));
        d->part_bytes = igx_align(std::max<size_t>(need, 1), 1 << 20);
    }
    if (!d->d_cnt) IGX_HIP(ctx, hipMalloc(&d->d_cnt, 64 * 8));
    uint64_t cnt[64] = {};
    if (nrows) {
        int rc = igx_partition_rows(ctx, static_cast<const uint8_t *>(rows), nrows, row_bytes, key_bytes,
                                    (uint32_t)nr, d->part, d->d_cnt);
        if (rc) return rc;
        IGX_HIP(ctx, hipMemcpyAsync(cnt, d->d_cnt, nr * 8, hipMemcpyDeviceToHost, ctx->stream));
        IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    uint64_t rc_[64] = {};
    int rc = igx_dist_alltoallv_rows(d, d->part, cnt, row_bytes, out, cap_rows, rc_);
    if (rc) return rc;
    uint64_t tot = 0;
    for (int p = 0; p < nr; ++p) tot += rc_[p];
    if (out_nrows) *out_nrows = tot;
    return IGX_OK;
}
