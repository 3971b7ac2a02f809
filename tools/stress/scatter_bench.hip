// scatter_bench.hip - cost of random scattered writes/reads on MI355X HBM (design tool).
// For a destination array of `span` bytes and a random permutation-like index stream of
// `count` elements, times: 4-byte scatter, 16-byte scatter, 4-byte gather, and a coalesced
// copy of the same element count, with hipEvents (median of 5).
//   hipcc --offload-arch=gfx950 -O3 -o scatter_bench scatter_bench.hip && ./scatter_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void k_idx(uint32_t *idx, uint32_t count, uint32_t slots, uint32_t seed)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count)
        idx[i] = (uint32_t)(((uint64_t)mix(i * 2654435761u + seed) * slots) >> 32);
}

__global__ void k_scatter4(const uint32_t *idx, uint32_t count, uint32_t *dst)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count)
        dst[idx[i]] = i;
}

__global__ void k_scatter16(const uint32_t *idx, uint32_t count, uint4 *dst)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count)
        dst[idx[i]] = make_uint4(i, i, i, i);
}

__global__ void k_gather4(const uint32_t *idx, uint32_t count, const uint32_t *src, uint32_t *out)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count)
        out[i] = src[idx[i]];
}

// ILP variants: each thread handles U elements (i, i + G, ..., G = grid threads), every index
// and gathered word loaded before any is used, so U random accesses are in flight per lane.
template <int U>
__global__ void k_gather4_ilp(const uint32_t *idx, uint32_t count, const uint32_t *src, uint32_t *out)
{
    const uint32_t G = gridDim.x * 256, i0 = blockIdx.x * 256 + threadIdx.x;
    uint32_t x[U], v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        x[u] = idx[i0 + u * G < count ? i0 + u * G : 0];
#pragma unroll
    for (int u = 0; u < U; u++)
        v[u] = src[x[u]];
#pragma unroll
    for (int u = 0; u < U; u++)
        if (i0 + u * G < count)
            out[i0 + u * G] = v[u];
}

template <int U>
__global__ void k_scatter4_ilp(const uint32_t *idx, uint32_t count, uint32_t *dst)
{
    const uint32_t G = gridDim.x * 256, i0 = blockIdx.x * 256 + threadIdx.x;
    uint32_t x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        x[u] = idx[i0 + u * G < count ? i0 + u * G : 0];
#pragma unroll
    for (int u = 0; u < U; u++)
        if (i0 + u * G < count)
            dst[x[u]] = i0 + u * G;
}

__global__ void k_copy4(const uint32_t *a, uint32_t count, uint32_t *b)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count)
        b[i] = a[i];
}

template <typename F> float timeit(F f)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> v;
    for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[2];
}

int main()
{
    const uint32_t count = 100000000u;
    uint32_t *idx, *out, *big;
    CK(hipMalloc(&idx, 4ull * count));
    CK(hipMalloc(&out, 4ull * count));
    const size_t big_bytes = 1600ull << 20;
    CK(hipMalloc(&big, big_bytes));
    dim3 g((count + 255) / 256);
    printf("count %u elements\n", count);
    printf("%-28s %10s %10s %12s\n", "op", "span MB", "ms", "ns/elem");
    float cp = timeit([&] { hipLaunchKernelGGL(k_copy4, g, dim3(256), 0, 0, idx, count, out); });
    printf("%-28s %10d %10.3f %12.4f\n", "coalesced copy 4B", 400, cp, cp * 1e6 / count);
    for (uint64_t span : {64ull << 20, 128ull << 20, 200ull << 20, 256ull << 20, 400ull << 20, 1600ull << 20}) {
        if (span > big_bytes) {  // never index past the destination buffer
            printf("span %llu exceeds buffer\n", (unsigned long long)span);
            return 1;
        }
        uint32_t slots4 = (uint32_t)(span / 4);
        hipLaunchKernelGGL(k_idx, g, dim3(256), 0, 0, idx, count, slots4, 7u);
        float s4 = timeit([&] { hipLaunchKernelGGL(k_scatter4, g, dim3(256), 0, 0, idx, count, big); });
        float g4 = timeit([&] { hipLaunchKernelGGL(k_gather4, g, dim3(256), 0, 0, idx, count, big, out); });
        printf("%-28s %10llu %10.3f %12.4f\n", "scatter 4B", (unsigned long long)(span >> 20), s4, s4 * 1e6 / count);
        printf("%-28s %10llu %10.3f %12.4f\n", "gather 4B", (unsigned long long)(span >> 20), g4, g4 * 1e6 / count);
        dim3 q2((count + 511) / 512), q4((count + 1023) / 1024), q8((count + 2047) / 2048);
        float a2 = timeit([&] { hipLaunchKernelGGL(k_gather4_ilp<2>, q2, dim3(256), 0, 0, idx, count, big, out); });
        float a4 = timeit([&] { hipLaunchKernelGGL(k_gather4_ilp<4>, q4, dim3(256), 0, 0, idx, count, big, out); });
        float a8 = timeit([&] { hipLaunchKernelGGL(k_gather4_ilp<8>, q8, dim3(256), 0, 0, idx, count, big, out); });
        float b4 = timeit([&] { hipLaunchKernelGGL(k_scatter4_ilp<4>, q4, dim3(256), 0, 0, idx, count, big); });
        printf("%-28s %10llu %10.3f %12.4f\n", "gather 4B x2/thread", (unsigned long long)(span >> 20), a2, a2 * 1e6 / count);
        printf("%-28s %10llu %10.3f %12.4f\n", "gather 4B x4/thread", (unsigned long long)(span >> 20), a4, a4 * 1e6 / count);
        printf("%-28s %10llu %10.3f %12.4f\n", "gather 4B x8/thread", (unsigned long long)(span >> 20), a8, a8 * 1e6 / count);
        printf("%-28s %10llu %10.3f %12.4f\n", "scatter 4B x4/thread", (unsigned long long)(span >> 20), b4, b4 * 1e6 / count);
        uint32_t slots16 = (uint32_t)(span / 16);
        hipLaunchKernelGGL(k_idx, g, dim3(256), 0, 0, idx, count, slots16, 9u);
        float s16 = timeit([&] { hipLaunchKernelGGL(k_scatter16, g, dim3(256), 0, 0, idx, count, (uint4 *)big); });
        printf("%-28s %10llu %10.3f %12.4f\n", "scatter 16B", (unsigned long long)(span >> 20), s16, s16 * 1e6 / count);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
