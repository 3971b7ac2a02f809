// scatter.hpp - staged 4-byte scatter for permutation-like writes into arrays far larger than
// the 256 MB Infinity Cache (the Phi array of the PLCP stage, the DC3 levels' rank and name
// arrays).
//
// A direct scatter of m random 4-byte writes into a 1-2 GB array pays a full HBM line per
// write. Here k_sc_stage bins the (index, value) pairs by destination window (2^rlog words,
// one LDS count per window and tile, one global atomic per window and tile) into per-window
// runs, and k_sc_apply writes the runs window by window, XCD-aware (workgroup g runs on XCD
// g mod 8, so XCD x takes windows x, x + 8, ...): the writes in flight on one XCD fall in one
// L2-sized window. Every window receives at most 2^rlog pairs (each index at most once), so
// the runs sit at fixed offsets (window << rlog) of the staging buffer.
#pragma once

#include "internal.hpp"

#include <cstdlib>

namespace salz {
namespace {  // kernels instantiated per translation unit

constexpr uint32_t kScTile = 4096;
constexpr uint32_t kScThreads = 256;
constexpr uint32_t kScWindows = 1024;

// Src: __device__ bool operator()(size_t c, uint32_t &index, uint32_t &value) const
template <class Src>
__global__ __launch_bounds__(kScThreads) void k_sc_stage(Src src, uint32_t m, uint32_t rlog,
                                                         uint32_t *__restrict__ rfill, uint2 *__restrict__ stage)
{
    __shared__ uint32_t cnt[kScWindows];
    constexpr uint32_t kItems = kScTile / kScThreads;
    const uint32_t tid = threadIdx.x;
    for (uint32_t r = tid; r < kScWindows; r += kScThreads)
        cnt[r] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kScTile;
    uint32_t iv[kItems], vv[kItems], loc[kItems];
    bool ok[kItems];
#pragma unroll
    for (uint32_t j = 0; j < kItems; j++) {
        const size_t c = base + (size_t)j * kScThreads + tid;
        ok[j] = src(c < m ? c : 0, iv[j], vv[j]) && c < m;  // loads unconditional (clamped)
    }
#pragma unroll
    for (uint32_t j = 0; j < kItems; j++)
        loc[j] = ok[j] ? atomicAdd(&cnt[iv[j] >> rlog], 1u) : 0u;
    __syncthreads();
    for (uint32_t r = tid; r < kScWindows; r += kScThreads)
        if (cnt[r])
            cnt[r] = (r << rlog) + atomicAdd(&rfill[r], cnt[r]);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kItems; j++)
        if (ok[j])
            stage[cnt[iv[j] >> rlog] + loc[j]] = make_uint2(iv[j], vv[j]);
}

// dst[index * stride + field] = value, window by window
__global__ __launch_bounds__(kScThreads) void k_sc_apply(const uint2 *__restrict__ stage,
                                                         const uint32_t *__restrict__ rfill, uint32_t rlog,
                                                         uint32_t nwin, uint32_t *__restrict__ dst,
                                                         uint32_t stride, uint32_t field)
{
    const uint32_t g = blockIdx.x, tiles = 1u << (rlog - 8);
    const uint32_t k = g >> 3, r = (g & 7u) + 8u * (k >> (rlog - 8));
    if (r >= nwin)
        return;
    const uint32_t x = (k & (tiles - 1u)) * kScThreads + threadIdx.x;
    if (x >= rfill[r])
        return;
    const uint2 e = stage[((size_t)r << rlog) + x];
    dst[(size_t)e.x * stride + field] = e.y;
}

// Scatter m pairs from src into dst (indices < nidx, each at most once), staged through `stage`
// (room for nidx pairs) with window counters rfill (one word per window of 2^rlog indices).
template <class Src>
int scatter_staged(Src src, uint32_t m, uint32_t nidx, uint32_t *dst, uint32_t stride, uint32_t field,
                   uint2 *stage, size_t stage_cap, uint32_t *rfill, hipStream_t st)
{
    if (m == 0)
        return 0;
    uint32_t rlog = 18;  // 1 MB windows of destination words
    while ((((uint64_t)nidx - 1) >> rlog) + 1 > kScWindows)
        rlog++;
    const uint32_t nwin = (uint32_t)((((uint64_t)nidx - 1) >> rlog) + 1);
    // window r's run starts at r << rlog and holds its indices (< nidx): every slot is below nidx
    if ((size_t)nidx > stage_cap) {
        set_error("staged scatter: %u windows of 2^%u exceed the staging buffer (%zu)", nwin, rlog, stage_cap);
        return -1;
    }
    SALZ_HIP(fill_async(rfill, 0, nwin * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_sc_stage<Src>, dim3(grid_for(m, kScTile)), dim3(kScThreads), 0, st, src, m, rlog, rfill,
                       stage);
    SALZ_LAUNCH_CHECK();
    const uint32_t agrid = 8u * ((nwin + 7u) / 8u) << (rlog - 8);
    hipLaunchKernelGGL(k_sc_apply, dim3(agrid), dim3(kScThreads), 0, st, stage, rfill, rlog, nwin, dst, stride,
                       field);
    SALZ_LAUNCH_CHECK();
    return 0;
}

// Stage a scatter whose destination spans more than the Infinity Cache (SALZ_SCATTER_STAGE=0:
// always direct, =1: always staged).
inline bool scatter_stage_wanted(size_t dst_bytes)
{
    const long env = env_num("SALZ_SA", "stage", -1);  // tests: stage=1 always, stage=0 never
    return env < 0 ? dst_bytes > (256u << 20) : env != 0;
}

}  // namespace
}  // namespace salz
