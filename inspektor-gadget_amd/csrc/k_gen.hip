// k_gen.hip -- synthetic event streams on the device (the data loader for the benches).
//
// Counter-based: event i's fields depend only on (seed, i), so any sub-range can be
// generated on any rank and the CPU oracle (oracle/igx_oracle.c) produces the same bytes
// (tests/test_gpu_parity.py checks this bit for bit).  Shapes follow SURVEY.md §8(d).
#include "k_common.h"

namespace {

constexpr int TB = 256;

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t i) {
    return sm64(sm64(seed ^ (stream * 0xD1B54A32D192ED03ull)) ^ (i * 0x9E3779B97F4A7C15ull));
}
__device__ __forceinline__ uint64_t cdf_pick(const uint64_t *cdf, uint64_t n, uint64_t r) {
    uint64_t u = r >> 1, lo = 0, hi = n - 1;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__constant__ char kNames[8][16] = {"nginx", "curl", "postgres", "redis-server",
                                   "java", "python3", "envoy", "node"};
__constant__ uint32_t kNameLen[8] = {5, 4, 8, 12, 4, 7, 5, 4};
__constant__ uint16_t kTcpPorts[8] = {80, 443, 8080, 53, 3306, 6379, 5432, 9092};
__constant__ char kStems[8][16] = {"bash", "sshd", "containerd", "kubelet", "cat",
                                   "systemd-journal", "runc", "ls"};
__constant__ uint32_t kStemLen[8] = {4, 4, 10, 7, 3, 15, 4, 2};
__constant__ uint16_t kNpPorts[8] = {80, 443, 53, 8080, 5432, 6379, 9090, 3000};

struct TcpOut {
    uint8_t *saddr, *daddr;
    uint64_t *mntns;
    uint32_t *pid;
    uint8_t *comm;
    uint16_t *lport, *dport, *family;
    uint32_t *size;
    uint8_t *dir;
};

__global__ __launch_bounds__(TB) void k_gen_tcp(uint64_t seed, uint64_t rank, uint64_t G, uint64_t A,
                                                uint64_t B, const uint64_t *cdf, uint64_t base,
                                                uint64_t n, TcpOut o) {
    uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = base + j;
    const uint64_t r = cdf_pick(cdf, G, rnd(seed, 1, i));
    const uint64_t kid = (r * A + B) % G;
    const uint64_t gk = kid * 64 + rank;
    const uint64_t p = 1000 + (gk >> 4);
    const uint64_t hp = sm64(p ^ 0x5EED);
    const uint64_t hk = sm64(gk ^ 0xFACE);
    const uint16_t fam = (hk % 10 == 0) ? 10 : 2;
    uint8_t sa[16] = {}, da[16] = {}, cm[16] = {};
    const uint8_t s4[4] = {10, 0, (uint8_t)(hp >> 8), (uint8_t)hp};
    const uint8_t d4[4] = {10, (uint8_t)(1 + ((hk >> 40) & 7)), (uint8_t)(hk >> 16), (uint8_t)(hk >> 24)};
    if (fam == 2) {
        for (int b = 0; b < 4; ++b) { sa[b] = s4[b]; da[b] = d4[b]; }
    } else {
        sa[10] = sa[11] = da[10] = da[11] = 0xff;
        for (int b = 0; b < 4; ++b) { sa[12 + b] = s4[b]; da[12 + b] = d4[b]; }
    }
    const uint32_t nm = (hp >> 32) & 7;
    const uint32_t L = kNameLen[nm];
    for (uint32_t b = 0; b < 16; ++b) cm[b] = b < L ? (uint8_t)kNames[nm][b] : 0;
    cm[L] = (uint8_t)('a' + ((hp >> 40) & 31) % 26);
    uint4 *s4p = reinterpret_cast<uint4 *>(o.saddr + 16 * j);
    uint4 *d4p = reinterpret_cast<uint4 *>(o.daddr + 16 * j);
    uint4 *c4p = reinterpret_cast<uint4 *>(o.comm + 16 * j);
    __builtin_memcpy(s4p, sa, 16);
    __builtin_memcpy(d4p, da, 16);
    __builtin_memcpy(c4p, cm, 16);
    o.mntns[j] = 4026531840ull + ((hp >> 20) & 63);
    o.pid[j] = (uint32_t)p;
    o.lport[j] = (uint16_t)(1024 + (gk & 15) + 16 * ((hk >> 8) % 2048));
    o.dport[j] = kTcpPorts[(hk >> 48) & 7];
    o.family[j] = fam;
    const uint64_t e = rnd(seed, 2, i);
    o.dir[j] = (uint8_t)(e & 1);
    o.size[j] = (uint32_t)(1 + (e >> 8) % 65535);
}

struct OpenOut {
    uint32_t *pid, *uid;
    uint64_t *mntns;
    uint8_t *comm;
    int64_t *ret, *fd, *err;
    uint32_t *path;
};

__global__ __launch_bounds__(TB) void k_gen_open(uint64_t seed, const uint64_t *comm_cdf, uint64_t base,
                                                 uint64_t n, OpenOut o) {
    uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = base + j;
    const uint64_t a = rnd(seed, 1, i), b = rnd(seed, 2, i), c = rnd(seed, 3, i);
    o.pid[j] = (uint32_t)(1 + a % 32767);
    const uint64_t ur = (a >> 32) % 11;
    o.uid[j] = ur == 0 ? 0 : (uint32_t)(999 + ur);
    o.mntns[j] = 4026531840ull + ((a >> 40) & 15);
    const uint64_t k = cdf_pick(comm_cdf, 64, b);
    uint8_t cm[16] = {};
    uint32_t L = kStemLen[k & 7];
    if (L > 13) L = 13;
    for (uint32_t q = 0; q < L; ++q) cm[q] = (uint8_t)kStems[k & 7][q];
    cm[L] = (uint8_t)('a' + (k >> 3));
    __builtin_memcpy(o.comm + 16 * j, cm, 16);
    int64_t r;
    if (c % 10 == 0) r = -(int64_t)(1 + (c >> 8) % 13);
    else r = (int64_t)(3 + (c >> 8) % 1021);
    o.ret[j] = r;
    o.fd[j] = r >= 0 ? r : 0;
    o.err[j] = r < 0 ? -r : 0;
    o.path[j] = (uint32_t)((c >> 32) & 4095);
}

__global__ __launch_bounds__(TB) void k_gen_bio(uint64_t seed, const uint64_t *q, uint64_t nq, uint64_t base,
                                                uint64_t n, uint32_t *dev, uint32_t *cont, uint64_t *delta) {
    uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = base + j;
    const uint64_t a = rnd(seed, 1, i), b = rnd(seed, 2, i);
    dev[j] = (8u << 20) | (uint32_t)(16 * (a & 15));
    cont[j] = (uint32_t)((a >> 8) & 255);
    const uint64_t idx = (b >> 32) % nq;
    const uint64_t lo = q[idx], hi = q[idx + 1];
    delta[j] = lo + (b & 0xffffffffull) % (hi - lo + 1);
}

struct NpOut {
    uint32_t *src, *peer;
    uint16_t *port;
    uint8_t *pkt, *typ, *proto;
    uint32_t *hostip, *raddr;
};

__global__ __launch_bounds__(TB) void k_gen_np(uint64_t seed, uint64_t nsrc, uint64_t npeer, uint64_t base,
                                               uint64_t n, NpOut o) {
    uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = base + j;
    const uint64_t a = rnd(seed, 1, i), b = rnd(seed, 2, i), c = rnd(seed, 3, i);
    const uint32_t s = (uint32_t)(a % nsrc);
    const uint64_t slot = (a >> 32) & 63;
    const uint32_t pe = (uint32_t)(sm64((uint64_t)s * 64 + slot) % npeer);
    o.src[j] = s;
    o.peer[j] = pe;
    o.port[j] = kNpPorts[(b >> 8) & 7];
    const uint64_t pk = b % 100;
    o.pkt[j] = pk < 60 ? 4 : (pk < 95 ? 0 : 1);
    o.typ[j] = (c % 100 == 0) ? 1 : 0;
    o.proto[j] = (uint8_t)((c >> 8) % 3 == 0 ? 17 : 6);
    const uint32_t hip = 0x0a000000u | (uint32_t)(s & 0xffff);
    o.hostip[j] = hip;
    o.raddr[j] = ((c >> 16) % 100 == 0) ? hip : (0x0a600000u | (pe & 0xfffff));
}

struct FileOut {
    uint64_t *inode;
    uint32_t *dev, *pid, *tid;
    uint8_t *op;
    uint32_t *count;
};

__global__ __launch_bounds__(TB) void k_gen_file(uint64_t seed, uint64_t rank, uint64_t G, uint64_t A,
                                                 uint64_t B, const uint64_t *cdf, uint64_t base,
                                                 uint64_t n, FileOut o) {
    uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = base + j;
    const uint64_t r = cdf_pick(cdf, G, rnd(seed, 1, i));
    const uint64_t kid = (r * A + B) % G;
    const uint64_t gk = kid * 64 + rank;
    const uint64_t h = sm64(gk ^ 0xF11E);
    o.inode[j] = sm64(gk ^ 0x9A7B);
    o.dev[j] = (uint32_t)((8u << 20) | (uint32_t)(h & 15));
    const uint32_t pid = (uint32_t)(100 + (gk >> 3));
    o.pid[j] = pid;
    o.tid[j] = pid + (uint32_t)(gk & 7);
    const uint64_t e = rnd(seed, 2, i);
    o.op[j] = (uint8_t)(e & 1);
    o.count[j] = (uint32_t)(1 + (e >> 8) % ((1u << 20) - 1));
}

inline dim3 grid_for(uint64_t n) { return dim3((unsigned)((n + TB - 1) / TB)); }

}  // namespace

extern "C" int igx_gen_tcp(igx_ctx *ctx, uint64_t seed, uint64_t rank, uint64_t G, uint64_t permA,
                           uint64_t permB, const uint64_t *cdf, uint64_t base, uint64_t n, uint8_t *saddr,
                           uint8_t *daddr, uint64_t *mntns, uint32_t *pid, uint8_t *comm, uint16_t *lport,
                           uint16_t *dport, uint16_t *family, uint32_t *size, uint8_t *dir) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (G == 0 || !cdf) return igx_fail(ctx, IGX_EINVAL, "gen_tcp: bad key universe");
    TcpOut o{saddr, daddr, mntns, pid, comm, lport, dport, family, size, dir};
    hipLaunchKernelGGL(k_gen_tcp, grid_for(n), dim3(TB), 0, ctx->stream, seed, rank, G, permA, permB, cdf,
                       base, n, o);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_gen_open(igx_ctx *ctx, uint64_t seed, const uint64_t *comm_cdf, uint64_t base,
                            uint64_t n, uint32_t *pid, uint32_t *uid, uint64_t *mntns, uint8_t *comm,
                            int64_t *ret, int64_t *fd, int64_t *err, uint32_t *path_id) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    OpenOut o{pid, uid, mntns, comm, ret, fd, err, path_id};
    hipLaunchKernelGGL(k_gen_open, grid_for(n), dim3(TB), 0, ctx->stream, seed, comm_cdf, base, n, o);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_gen_bio(igx_ctx *ctx, uint64_t seed, const uint64_t *q, uint64_t nq, uint64_t base,
                           uint64_t n, uint32_t *dev, uint32_t *cont, uint64_t *delta) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (nq == 0) return igx_fail(ctx, IGX_EINVAL, "gen_bio: empty quantile table");
    hipLaunchKernelGGL(k_gen_bio, grid_for(n), dim3(TB), 0, ctx->stream, seed, q, nq, base, n, dev, cont, delta);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_gen_np(igx_ctx *ctx, uint64_t seed, uint64_t nsrc, uint64_t npeer, uint64_t base,
                          uint64_t n, uint32_t *src, uint32_t *peer, uint16_t *port, uint8_t *pkt,
                          uint8_t *typ, uint8_t *proto, uint32_t *hostip, uint32_t *raddr) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (!nsrc || !npeer) return igx_fail(ctx, IGX_EINVAL, "gen_np: empty dictionaries");
    NpOut o{src, peer, port, pkt, typ, proto, hostip, raddr};
    hipLaunchKernelGGL(k_gen_np, grid_for(n), dim3(TB), 0, ctx->stream, seed, nsrc, npeer, base, n, o);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_gen_file(igx_ctx *ctx, uint64_t seed, uint64_t rank, uint64_t G, uint64_t permA,
                            uint64_t permB, const uint64_t *cdf, uint64_t base, uint64_t n,
                            uint64_t *inode, uint32_t *dev, uint32_t *pid, uint32_t *tid, uint8_t *op,
                            uint32_t *count) {
    if (!ctx) return IGX_EINVAL;
    if (n == 0) return IGX_OK;
    if (G == 0 || !cdf) return igx_fail(ctx, IGX_EINVAL, "gen_file: bad key universe");
    FileOut o{inode, dev, pid, tid, op, count};
    hipLaunchKernelGGL(k_gen_file, grid_for(n), dim3(TB), 0, ctx->stream, seed, rank, G, permA, permB, cdf,
                       base, n, o);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
