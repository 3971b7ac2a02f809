// lds_stress.hip - LDS integrity under concurrent streams: every workgroup fills its LDS
// (SHARED_KB KiB) with a block-specific pattern, waits, and verifies it; T host threads each
// launch the kernel repeatedly on their own stream.
//   hipcc --offload-arch=gfx950 -O3 -o lds_stress lds_stress.hip -lpthread
//   ./lds_stress THREADS BLOCKS ITERS
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <thread>
#include <vector>

constexpr int kWords = 48 * 1024 / 4;

__global__ __launch_bounds__(256) void k_lds(uint32_t salt, unsigned *bad)
{
    __shared__ uint32_t s[kWords];
    const uint32_t tag = (blockIdx.x * 2654435761u) ^ salt;
    for (int i = threadIdx.x; i < kWords; i += 256)
        s[i] = tag ^ (uint32_t)i * 0x9E3779B9u;
    __syncthreads();
    for (int spin = 0; spin < 64; spin++)
        __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    unsigned b = 0;
    for (int i = threadIdx.x; i < kWords; i += 256)
        b += s[(i * 7 + 13) % kWords] != (tag ^ (uint32_t)((i * 7 + 13) % kWords) * 0x9E3779B9u);
    if (b)
        atomicAdd(bad, b);
}

int main(int argc, char **argv)
{
    int threads = argc > 1 ? atoi(argv[1]) : 2;
    int blocks = argc > 2 ? atoi(argv[2]) : 4096;
    int iters = argc > 3 ? atoi(argv[3]) : 200;
    std::vector<unsigned> bads(threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&, t] {
            (void)hipSetDevice(0);
            unsigned *bad;
            hipStream_t st;
            (void)hipMalloc(&bad, 4);
            (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
            (void)hipMemsetAsync(bad, 0, 4, st);
            for (int it = 0; it < iters; it++)
                hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), 0, st, (uint32_t)(it * 131 + t * 7919), bad);
            (void)hipMemcpyAsync(&bads[t], bad, 4, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            (void)hipFree(bad);
            (void)hipStreamDestroy(st);
        });
    }
    for (auto &x : th)
        x.join();
    printf("lds: threads=%d blocks=%d iters=%d mismatches:", threads, blocks, iters);
    for (int t = 0; t < threads; t++)
        printf(" %u", bads[t]);
    printf("\n");
    return 0;
}
