// scatter.hpp - staged 4-byte scatter for permutation-like writes into arrays far larger than
// the 256 MB Infinity Cache (the Phi array of the PLCP stage, the DC3 levels' rank and name
// arrays).
//
// A direct scatter of m random 4-byte writes into a 1-2 GB array pays a full HBM line per
// write. Here k_sc_stage bins the (index, value) pairs by destination window (2^rlog words)
// into per-window runs, and k_sc_apply writes the runs window by window, XCD-aware (workgroup g
// runs on XCD g mod 8, so XCD x takes windows x, x + 8, ...): the writes in flight on one XCD
// fall in one L2-sized window. Every window receives at most 2^rlog pairs (each index at most
// once), so the runs sit at fixed offsets (window << rlog) of the staging buffer.
//
// A staging tile is 8192 pairs (1024 threads, 72 KB of LDS: two workgroups per CU), ordered by
// window in LDS before it leaves: its run for a window (8 pairs on average over 1024 windows) is
// written as one contiguous 64-byte piece, and each window's counter takes one atomic per tile.
// 4096-pair tiles written straight from registers took one device atomic per window and tile
// (~66 M for a 2^28-pair scatter) and wrote 32-byte pieces: Phi at 256 MiB 2.69 -> 1.63 ms at
// 16384-pair tiles; C5 3139 / 3112 -> 3298 / 3284 MB/s (16384) and 3312 / 3307 (8192) on one box,
// profiles/r06t_staged_scatter_ab.txt.
#pragma once

#include "internal.hpp"

#include <cstdlib>

namespace salz {
namespace {  // kernels instantiated per translation unit

constexpr uint32_t kScThreads = 256;   // k_sc_apply
constexpr uint32_t kScWindows = 1024;
constexpr uint32_t kStThreads = 1024;  // k_sc_stage: one thread per window
constexpr uint32_t kStItems = 8;
constexpr uint32_t kStTile = kStThreads * kStItems;

// Src: __device__ bool operator()(size_t c, uint32_t &index, uint32_t &value) const
template <class Src>
__global__ __launch_bounds__(kStThreads) void k_sc_stage(Src src, uint32_t m, uint32_t rlog,
                                                         uint32_t *__restrict__ rfill, uint2 *__restrict__ stage)
{
    __shared__ uint2 buf[kStTile];
    __shared__ uint32_t cnt[kScWindows];  // pairs per window, then the window's offset in buf
    __shared__ uint32_t delta[kScWindows];  // stage slot - buf offset (mod 2^32)
    __shared__ uint32_t wsum[kStThreads / 64];
    const uint32_t tid = threadIdx.x;
    cnt[tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kStTile;
    uint32_t iv[kStItems], vv[kStItems], loc[kStItems];
#pragma unroll
    for (uint32_t j = 0; j < kStItems; j++) {
        const size_t c = base + (size_t)j * kStThreads + tid;
        const bool ok = src(c < m ? c : 0, iv[j], vv[j]) && c < m;  // loads unconditional (clamped)
        loc[j] = ok ? atomicAdd(&cnt[iv[j] >> rlog], 1u) : 0xffffffffu;
    }
    __syncthreads();
    // exclusive scan of the window counts (thread = window), then one atomic per used window
    const uint32_t c = cnt[tid], lane = tid & 63u, wv = tid >> 6;
    uint32_t x = c;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = shfl_up_u32(x, d);
        x += lane >= d ? y : 0u;
    }
    if (lane == 63u)
        wsum[wv] = x;
    __syncthreads();
    uint32_t off = x - c, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kStThreads / 64; w++) {
        off += w < wv ? wsum[w] : 0u;
        total += wsum[w];
    }
    cnt[tid] = off;
    delta[tid] = c ? (tid << rlog) + atomicAdd(&rfill[tid], c) - off : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kStItems; j++)
        if (loc[j] != 0xffffffffu)
            buf[cnt[iv[j] >> rlog] + loc[j]] = make_uint2(iv[j], vv[j]);
    __syncthreads();
    for (uint32_t s = tid; s < total; s += kStThreads) {
        const uint2 e = buf[s];
        stage[delta[e.x >> rlog] + s] = e;
    }
}

// dst[index * stride + field] = value, window by window (one pair per thread: with 8 per thread,
// two windows were in flight per XCD and their dirty lines shared its L2, apply 7.7 -> 11.2 ms
// on the 256 MiB halves block)
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
    hipLaunchKernelGGL(k_sc_stage<Src>, dim3(grid_for(m, kStTile)), dim3(kStThreads), 0, st, src, m, rlog, rfill,
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
