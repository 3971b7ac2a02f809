// gather_bench.hip - random 4-byte / 8-byte gather and scatter rates by load/store flavour
// (diagnostic for the suffix sort's rank and key passes; not part of the library).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_bench tools/gather_bench.hip
//   tools/gather_bench [table_mib] [queries_m]
//   tools/gather_bench calib     (one dispatch per access pattern, for the PMC calibration)
//
// Every kernel: one query per thread, indices from a precomputed random array (read
// coalesced), results written coalesced, so the random side is the only random traffic.
// The "xcd" lines draw each workgroup's indices from the eighth of the table that belongs to
// its XCD (workgroups are dealt to the 8 XCDs round-robin), so a table of up to 32 MiB keeps
// every XCD's part inside its own 4 MB L2.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

__global__ void k_init_idx(uint32_t *idx, size_t m, uint32_t n, uint64_t seed)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    idx[i] = (uint32_t)(z % n);
}

// indices in the XCD's eighth of the table: workgroup b runs on XCD b mod 8
__global__ void k_init_idx_xcd(uint32_t *idx, size_t m, uint32_t n, uint64_t seed)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint32_t part = n / 8u;
    idx[i] = (uint32_t)(blockIdx.x & 7u) * part + (uint32_t)(z % part);
}

// 16-byte records (the candidate array's entries) at 16-byte slots of the table
__global__ void k_scatter16(uint4 *__restrict__ tab, const uint32_t *__restrict__ idx, size_t m)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    const uint32_t v = (uint32_t)i;
    tab[idx[i]] = make_uint4(v, v + 1u, v + 2u, v + 3u);
}

template <int F>
__global__ void k_gather4(const uint32_t *__restrict__ tab, const uint32_t *__restrict__ idx, size_t m,
                          uint32_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    const uint32_t *p = tab + idx[i];
    uint32_t v;
    if (F == 0)
        v = *p;
    else if (F == 1)
        v = __builtin_nontemporal_load(p);
    else
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[i] = v;
}

template <int F>
__global__ void k_scatter4(uint32_t *__restrict__ tab, const uint32_t *__restrict__ idx, size_t m)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    uint32_t *p = tab + idx[i];
    const uint32_t v = (uint32_t)i;
    if (F == 0)
        *p = v;
    else if (F == 1)
        __builtin_nontemporal_store(v, p);
    else
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8 unaligned bytes from a byte table (the suffix sort's text keys): two aligned words
template <int F>
__global__ void k_gather8(const uint8_t *__restrict__ tab, const uint32_t *__restrict__ idx, size_t m,
                          uint64_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    const size_t pos = idx[i];
    const uint64_t *w = reinterpret_cast<const uint64_t *>(tab + (pos & ~(size_t)7));
    uint64_t a, b;
    if (F == 0) {
        a = w[0];
        b = w[1];
    } else {
        a = __builtin_nontemporal_load(w);
        b = __builtin_nontemporal_load(w + 1);
    }
    const unsigned sh = (unsigned)(pos & 7) * 8u;
    out[i] = (a >> sh) | ((b << 1) << (63u - sh));
}

// Plain coalesced copy of 16-byte words (the calibration's streaming reference).
__global__ void k_copy16(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t m)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < m)
        b[i] = a[i];
}

// Calibration of the FETCH_SIZE / WRITE_SIZE counters (tools/pmc_traffic.py --calib): each kernel
// runs exactly once on known byte counts, so that `rocprofv3 --pmc FETCH_SIZE` (then WRITE_SIZE)
// of `gather_bench calib` gives the counter per access pattern:
//   k_copy16               m16 16-byte reads + writes, coalesced (the guide's x2 fetch case)
//   k_gather4<0> big/small m 4-byte random reads from a 1.6 GB table / a 64 MiB (L2 + MALL) table,
//                          + the 4-byte index read and result write, coalesced
//   k_gather8<0>           m unaligned 8-byte reads (two aligned words) from a 400 MB byte table
//   k_scatter4<0>          m 4-byte random writes into 1.6 GB
//   k_scatter16            m 16-byte random writes into 1.6 GB
static int calib()
{
    const size_t m = 64u << 20, big = (size_t)1600 << 20, small = (size_t)64 << 20;
    uint32_t *tab, *idx, *out;
    CK(hipMalloc(&tab, big + 64));
    CK(hipMalloc(&idx, m * 4));
    CK(hipMalloc(&out, m * 16));
    CK(hipMemset(tab, 1, big + 64));
    const dim3 g((unsigned)((m + 255) / 256)), b(256);
    printf("calib m=%zu accesses per kernel; useful bytes: copy16 %zu read + %zu write; gather4 %zu random + "
           "%zu coalesced read, %zu write; gather8 %zu random read; scatter4 %zu random write; scatter16 %zu random "
           "write\n", m, m * 16, m * 16, m * 4, m * 4, m * 4, m * 8, m * 4, m * 16);
    k_copy16<<<g, b>>>(reinterpret_cast<const uint4 *>(tab), reinterpret_cast<uint4 *>(out), m);
    k_init_idx<<<g, b>>>(idx, m, (uint32_t)(big / 4), 11);
    k_gather4<0><<<g, b>>>(tab, idx, m, out);                              // dispatch: big table
    k_init_idx<<<g, b>>>(idx, m, (uint32_t)(small / 4), 12);
    k_gather4<0><<<g, b>>>(tab, idx, m, out);                              // dispatch: small table
    k_init_idx<<<g, b>>>(idx, m, (uint32_t)(400u << 20), 13);
    k_gather8<0><<<g, b>>>(reinterpret_cast<uint8_t *>(tab), idx, m, reinterpret_cast<uint64_t *>(out));
    k_init_idx<<<g, b>>>(idx, m, (uint32_t)(big / 4), 14);
    k_scatter4<0><<<g, b>>>(tab, idx, m);
    k_init_idx<<<g, b>>>(idx, m, (uint32_t)(big / 16), 15);
    k_scatter16<<<g, b>>>(reinterpret_cast<uint4 *>(tab), idx, m);
    CK(hipDeviceSynchronize());
    return 0;
}

int main(int argc, char **argv)
{
    if (argc > 1 && argv[1][0] == 'c')
        return calib();
    const size_t tab_mib = argc > 1 ? atol(argv[1]) : 400;
    const size_t m = (argc > 2 ? atol(argv[2]) : 64) << 20;
    const uint32_t n4 = (uint32_t)((tab_mib << 20) / 4);
    uint32_t *tab, *idx, *out;
    uint64_t *out8;
    CK(hipMalloc(&tab, (size_t)n4 * 4 + 64));
    CK(hipMalloc(&idx, m * 4));
    CK(hipMalloc(&out, m * 4));
    CK(hipMalloc(&out8, m * 8));
    CK(hipMemset(tab, 1, (size_t)n4 * 4 + 64));
    const dim3 g((unsigned)((m + 255) / 256)), b(256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-28s table %4zu MiB  %6.3f ms  %6.1f G/s\n", name, tab_mib, best, m / (best * 1e-3) / 1e9);
    };
    k_init_idx<<<g, b>>>(idx, m, n4, 12345);
    timeit("gather4 plain", [&] { k_gather4<0><<<g, b>>>(tab, idx, m, out); });
    timeit("gather4 nontemporal", [&] { k_gather4<1><<<g, b>>>(tab, idx, m, out); });
    timeit("gather4 relaxed agent", [&] { k_gather4<2><<<g, b>>>(tab, idx, m, out); });
    timeit("scatter4 plain", [&] { k_scatter4<0><<<g, b>>>(tab, idx, m); });
    timeit("scatter4 nontemporal", [&] { k_scatter4<1><<<g, b>>>(tab, idx, m); });
    timeit("scatter4 relaxed agent", [&] { k_scatter4<2><<<g, b>>>(tab, idx, m); });
    // byte table of a quarter the size (the mapped text is n bytes against n words of rank)
    k_init_idx<<<g, b>>>(idx, m, n4, 777);
    timeit("gather8 bytes plain", [&] { k_gather8<0><<<g, b>>>(reinterpret_cast<uint8_t *>(tab), idx, m, out8); });
    timeit("gather8 bytes nontemporal", [&] { k_gather8<1><<<g, b>>>(reinterpret_cast<uint8_t *>(tab), idx, m, out8); });
    k_init_idx_xcd<<<g, b>>>(idx, m, n4, 4242);
    timeit("gather4 plain xcd", [&] { k_gather4<0><<<g, b>>>(tab, idx, m, out); });
    timeit("scatter4 plain xcd", [&] { k_scatter4<0><<<g, b>>>(tab, idx, m); });
    k_init_idx<<<g, b>>>(idx, m, n4 / 4u, 99);
    timeit("scatter16 plain", [&] { k_scatter16<<<g, b>>>(reinterpret_cast<uint4 *>(tab), idx, m); });
    k_init_idx_xcd<<<g, b>>>(idx, m, n4 / 4u, 98);
    timeit("scatter16 plain xcd", [&] { k_scatter16<<<g, b>>>(reinterpret_cast<uint4 *>(tab), idx, m); });
    CK(hipDeviceSynchronize());
    return 0;
}
