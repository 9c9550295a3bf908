// Microbenchmark (diagnostics only): appending 8-byte records to B buckets from every CU, the
// write pattern of an update log partitioned at write time.  Each workgroup (one per CU, one
// writer wave like the group-by's server wave, or all 16 waves) owns a chunk per bucket (CH
// records) and appends with plain 8-B stores; the chunk's lines fill over time in the XCD's L2.
// Reports the append rate and whether the records arrived (checksum), for B = 64 .. 4096.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

constexpr uint32_t CH = 512;   // records per chunk (4 KiB)

// per workgroup: nrec records; bucket = hash bits; LDS per-bucket {chunk, fill}
__global__ __launch_bounds__(1024) void k_append(uint64_t *pool, uint32_t *pool_ctr, uint32_t *owner, uint32_t pool_cap,
                                                 uint32_t nb_log, uint64_t nrec, uint32_t writers, uint64_t *sum) {
    extern __shared__ uint32_t lds[];
    const uint32_t NB = 1u << nb_log;
    uint32_t *chunk = lds, *fill = lds + 4 * NB;   // chunk ids: 4 generations per bucket
    for (uint32_t i = threadIdx.x; i < NB; i += blockDim.x) {
        for (int g = 0; g < 4; ++g) chunk[4 * i + g] = 0xFFFFFFFFu;
        fill[i] = 0;
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long acc = 0;
    if (wave < writers) {
        for (uint64_t r = (uint64_t)wave * 64 + lane; r < nrec; r += (uint64_t)writers * 64) {
            const uint64_t v = mix(((uint64_t)blockIdx.x << 40) + r);
            const uint32_t b = (uint32_t)(v >> (64 - nb_log));
            // reserve a position: LDS atomic on the bucket's fill; the lane that takes position
            // 0 of a chunk allocates it, the others wait for the id (bounded)
            const uint32_t pos = atomicAdd(&fill[b], 1u);
            const uint32_t k = pos / CH, w = pos % CH;
            if (w == 0) {
                const uint32_t c = atomicAdd(pool_ctr, 1u);
                if (c < pool_cap) owner[c] = b;
                __hip_atomic_store(&chunk[4 * b + (k & 3)], (k << 24) | (c & 0xFFFFFFu), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            uint32_t e, spins = 0;
            while (((e = __hip_atomic_load(&chunk[4 * b + (k & 3)], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 24) !=
                       (k & 0xFF) ||
                   e == 0xFFFFFFFFu) {
                if (++spins > (1u << 20)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t c = e & 0xFFFFFFu;
            if (c < pool_cap) pool[(uint64_t)c * CH + w] = v;
            acc += v;
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0 && acc) atomicAdd(reinterpret_cast<unsigned long long *>(sum), acc);
}

int main() {
    const uint32_t blocks = 256;
    const uint64_t nrec = 400000;                 // per workgroup (C5: 104M updates / 256)
    const uint32_t pool_cap = (uint32_t)(blocks * nrec / CH + blocks * 4096 + 1024);
    uint64_t *pool, *sum;
    uint32_t *ctr, *owner;
    hipMalloc(&pool, (uint64_t)pool_cap * CH * 8);
    hipMalloc(&owner, (uint64_t)pool_cap * 4);
    hipMalloc(&ctr, 64);
    hipMalloc(&sum, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (uint32_t writers : {1u, 4u, 16u}) {
        for (uint32_t nbl : {6u, 8u, 10u, 12u}) {
            const size_t lds = (size_t)(5u << nbl) * 4 + 16;
            hipFuncSetAttribute(reinterpret_cast<const void *>(k_append), hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
            float best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                hipMemset(ctr, 0, 64);
                hipMemset(sum, 0, 8);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_append, dim3(blocks), dim3(1024), lds, 0, pool, ctr, owner, pool_cap, nbl, nrec,
                                   writers, sum);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            uint32_t used = 0;
            hipMemcpy(&used, ctr, 4, hipMemcpyDeviceToHost);
            const double recs = (double)blocks * nrec;
            printf("writers %2u buckets %5u: %.3f ms  %.1f G records/s  %.0f GB/s of records  chunks %u\n", writers,
                   1u << nbl, best, recs / best / 1e6, recs * 8 / best / 1e6, used);
        }
    }
    return 0;
}
