// load_stress.hip - minimal check of global-load integrity under concurrent streams.
// T threads, each with its own stream and buffers, repeat: fill T with a pattern, run a
// kernel that loads 8 bytes per position (two aligned u64 words, shifted: the suffix
// sorter's k_sa_init pattern) and stores them, then a kernel that recomputes the value with
// byte loads and counts mismatches. Any mismatch means a load returned wrong data.
//   hipcc --offload-arch=gfx950 -O3 -o load_stress load_stress.hip -lpthread
//   ./load_stress THREADS N ITERS
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <thread>
#include <vector>

__global__ void k_fill(uint8_t *T, size_t n, uint32_t seed)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        T[i] = (uint8_t)(((i * 2654435761u) >> 13) ^ seed ^ (i >> 7));
}

__global__ void k_load(const uint8_t *T, uint32_t n, uint64_t *key)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t *w = reinterpret_cast<const uint64_t *>(T + (i & ~(size_t)7));
    unsigned sh = (unsigned)(i & 7) * 8u;
    uint64_t a = w[0];
    uint64_t v = sh ? ((a >> sh) | (w[1] << (64u - sh))) : a;
    key[i] = v;
}

__global__ void k_check(const uint8_t *T, const uint64_t *key, uint32_t n, unsigned *bad)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint64_t w = 0;
    for (int k = 7; k >= 0; k--)
        w = (w << 8) | T[i + k];
    if (w != key[i])
        atomicAdd(bad, 1u);
}

int main(int argc, char **argv)
{
    int threads = argc > 1 ? atoi(argv[1]) : 2;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 24);
    int iters = argc > 3 ? atoi(argv[3]) : 50;
    std::vector<unsigned> bads(threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&, t] {
            hipSetDevice(0);
            uint8_t *T;
            uint64_t *key;
            unsigned *bad;
            hipStream_t st;
            hipMalloc(&T, n + 256);
            hipMalloc(&key, 8ull * n);
            hipMalloc(&bad, 4);
            hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
            hipMemsetAsync(bad, 0, 4, st);
            hipMemsetAsync(T + n, 0, 256, st);
            unsigned g = (n + 255) / 256;
            for (int it = 0; it < iters; it++) {
                hipLaunchKernelGGL(k_fill, dim3(g), dim3(256), 0, st, T, (size_t)n, (uint32_t)(it * 7 + t));
                hipLaunchKernelGGL(k_load, dim3(g), dim3(256), 0, st, T, n, key);
                hipLaunchKernelGGL(k_check, dim3(g), dim3(256), 0, st, T, key, n, bad);
            }
            hipMemcpyAsync(&bads[t], bad, 4, hipMemcpyDeviceToHost, st);
            hipStreamSynchronize(st);
            hipFree(T);
            hipFree(key);
            hipFree(bad);
            hipStreamDestroy(st);
        });
    }
    for (auto &x : th)
        x.join();
    printf("threads=%d n=%u iters=%d mismatches:", threads, n, iters);
    for (int t = 0; t < threads; t++)
        printf(" %u", bads[t]);
    printf("\n");
    return 0;
}
