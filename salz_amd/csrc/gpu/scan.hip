// scan.hip - device-wide prefix scans (reduce-then-scan, 4096-element tiles).
//
// Used by every stage that compacts or ranks: group-head ranking in the suffix sorter,
// radix digit offsets, PLCP max-propagation, parse exit sets and emission offsets.
#include "internal.hpp"

namespace salz {
namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;
constexpr size_t kInlineTiles = 1024;

template <typename T> struct SumOp {
    __device__ __forceinline__ static T id() { return T(0); }
    __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
template <typename T> struct MaxOp {
    __device__ __forceinline__ static T id() { return T(0); }
    __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
};

__device__ __forceinline__ uint32_t up(uint32_t v, unsigned d) { return shfl_up_u32(v, d); }
__device__ __forceinline__ uint64_t up(uint64_t v, unsigned d) { return shfl_up_u64(v, d); }

// LDS index with one pad word per 16 elements: a thread's 16 consecutive elements start on
// distinct banks.
__device__ __forceinline__ int pidx(int i) { return i + (i >> 4); }

// Exclusive block scan over 256 threads; returns exclusive prefix, writes block total.
template <typename T, typename Op>
__device__ __forceinline__ T block_excl(T v, T *wsum, T &total, Op op)
{
    unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (unsigned d = 1; d < 64; d <<= 1) {
        T y = up(x, d);
        if (lane >= d)
            x = op(y, x);
    }
    if (lane == 63)
        wsum[wave] = x;
    __syncthreads();
    T wpre = Op::id();
    for (unsigned w = 0; w < wave; w++)
        wpre = op(wpre, wsum[w]);
    total = op(op(wsum[0], wsum[1]), op(wsum[2], wsum[3]));
    T ex = up(x, 1);
    if (lane == 0)
        ex = Op::id();
    __syncthreads();
    return op(wpre, ex);
}

template <typename T, typename Op, typename TI = T>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const TI *__restrict__ in, size_t n,
                                                              T *__restrict__ partial)
{
    __shared__ T wsum[4];
    Op op;
    size_t base = (size_t)blockIdx.x * kScanTile;
    T acc = Op::id();
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        size_t i = base + (size_t)j * kScanThreads + threadIdx.x;
        if (i < n)
            acc = op(acc, (T)in[i]);
    }
    T total;
    block_excl<T, Op>(acc, wsum, total, op);
    if (threadIdx.x == 0)
        partial[blockIdx.x] = total;
}

template <typename T, typename Op, typename TI = T>
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(const TI *__restrict__ in, T *out,
                                                             size_t n, const T *__restrict__ carry,
                                                             int inclusive, T *total_out,
                                                             const T *__restrict__ partial)
{
    __shared__ T s[kScanTile + kScanTile / 16];
    __shared__ T wsum[4];
    Op op;
    size_t base = (size_t)blockIdx.x * kScanTile;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        int l = j * kScanThreads + threadIdx.x;
        size_t i = base + l;
        s[pidx(l)] = i < n ? (T)in[i] : Op::id();
    }
    __syncthreads();
    T loc[kScanItems];
    T sum = Op::id();
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        loc[k] = s[pidx(threadIdx.x * kScanItems + k)];
        sum = op(sum, loc[k]);
    }
    T total;
    T run = block_excl<T, Op>(sum, wsum, total, op);
    T c = carry ? carry[blockIdx.x] : Op::id();
    if (partial) {  // (kernel-uniform) the carry reduced here from the tiles' totals before this one
        T a = Op::id();
        for (uint32_t t = threadIdx.x; t < blockIdx.x; t += kScanThreads)
            a = op(a, partial[t]);
        T ca;
        block_excl<T, Op>(a, wsum, ca, op);
        c = ca;
    }
    run = op(c, run);
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        T nxt = op(run, loc[k]);
        s[pidx(threadIdx.x * kScanItems + k)] = inclusive ? nxt : run;
        run = nxt;
    }
    if (total_out && threadIdx.x == kScanThreads - 1 && blockIdx.x == gridDim.x - 1)
        *total_out = run;  // includes the carry of this (last) tile
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        int l = j * kScanThreads + threadIdx.x;
        size_t i = base + l;
        if (i < n)
            out[i] = s[pidx(l)];
    }
}

// Byte flags (u8 -> u32 sums), whole tiles: a thread's 16 consecutive elements are one 16-byte
// load, so the input needs no LDS transpose and a wave reads 1 KB per instruction.
__device__ __forceinline__ uint32_t bsum4(uint32_t w)
{
    const uint32_t x = (w & 0x00ff00ffu) + ((w >> 8) & 0x00ff00ffu);
    return (x & 0xffffu) + (x >> 16);
}

__global__ __launch_bounds__(kScanThreads) void k_flag_reduce(const uint4 *__restrict__ in,
                                                              uint32_t *__restrict__ partial)
{
    __shared__ uint32_t wsum[4];
    const uint4 v = in[(size_t)blockIdx.x * kScanThreads + threadIdx.x];
    uint32_t total;
    block_excl<uint32_t, SumOp<uint32_t>>(bsum4(v.x) + bsum4(v.y) + bsum4(v.z) + bsum4(v.w), wsum,
                                          total, SumOp<uint32_t>());
    if (threadIdx.x == 0)
        partial[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_flag_scan(const uint4 *__restrict__ in,
                                                            uint32_t *__restrict__ out,
                                                            const uint32_t *__restrict__ carry,
                                                            int inclusive, uint32_t ntiles,
                                                            uint32_t *total_out)
{
    __shared__ uint32_t wsum[4];
    const size_t i = (size_t)blockIdx.x * kScanThreads + threadIdx.x;
    const uint4 v = in[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t total;
    uint32_t run = block_excl<uint32_t, SumOp<uint32_t>>(
        bsum4(v.x) + bsum4(v.y) + bsum4(v.z) + bsum4(v.w), wsum, total, SumOp<uint32_t>());
    run += carry ? carry[blockIdx.x] : 0u;
    uint4 *o = reinterpret_cast<uint4 *>(out) + i * 4;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t e = (w[q] >> (8 * k)) & 0xffu;
            r[k] = inclusive ? run + e : run;
            run += e;
        }
        o[q] = make_uint4(r[0], r[1], r[2], r[3]);
    }
    if (total_out && threadIdx.x == kScanThreads - 1 && blockIdx.x == ntiles - 1)
        *total_out = run;
}

template <typename T, typename Op, typename TI = T>
int scan_impl(const TI *in, T *out, size_t n, bool inclusive, T *total_out, T *tmp,
              size_t tmp_elems, hipStream_t st)
{
    if (n == 0)
        return 0;
    size_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles == 1) {
        hipLaunchKernelGGL((k_scan_tiles<T, Op, TI>), dim3(1), dim3(kScanThreads), 0, st, in, out,
                           n, (const T *)nullptr, inclusive ? 1 : 0, total_out, (const T *)nullptr);
        SALZ_LAUNCH_CHECK();
        return 0;
    }
    if (tmp_elems < tiles) {
        set_error("scan: temp too small (%zu < %zu)", tmp_elems, tiles);
        return -1;
    }
    T *partial = tmp;
    hipLaunchKernelGGL((k_scan_reduce<T, Op, TI>), dim3((unsigned)tiles), dim3(kScanThreads), 0,
                       st, in, n, partial);
    SALZ_LAUNCH_CHECK();
    // Up to kInlineTiles tiles each scanning block reduces the totals before it itself (at most
    // 1023 reads, L2-resident): two launches instead of three (round 5: C3 3010 -> 3031 MB/s);
    // more tiles scan their totals in a launch of their own.
    if (tiles <= kInlineTiles) {
        hipLaunchKernelGGL((k_scan_tiles<T, Op, TI>), dim3((unsigned)tiles), dim3(kScanThreads), 0, st,
                           in, out, n, (const T *)nullptr, inclusive ? 1 : 0, total_out, (const T *)partial);
        SALZ_LAUNCH_CHECK();
        return 0;
    }
    if (scan_impl<T, Op>(partial, partial, tiles, false, nullptr, tmp + tiles,
                         tmp_elems - tiles, st) != 0)
        return -1;
    hipLaunchKernelGGL((k_scan_tiles<T, Op, TI>), dim3((unsigned)tiles), dim3(kScanThreads), 0, st,
                       in, out, n, (const T *)partial, inclusive ? 1 : 0, total_out, (const T *)nullptr);
    SALZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace

size_t scan_temp_elems(size_t n)
{
    size_t t = 0;
    while (n > (size_t)kScanTile) {
        n = (n + kScanTile - 1) / kScanTile;
        t += n;
    }
    return t + 16;
}

int scan_sum_u32(const uint32_t *in, uint32_t *out, size_t n, bool inclusive,
                 uint32_t *total_out, Workspace &ws, hipStream_t st)
{
    return scan_impl<uint32_t, SumOp<uint32_t>>(in, out, n, inclusive, total_out,
                                                (uint32_t *)ws.scan_tmp, ws.scan_tmp_bytes / 4, st);
}

int scan_max_u32(const uint32_t *in, uint32_t *out, size_t n, bool inclusive,
                 uint32_t *total_out, Workspace &ws, hipStream_t st)
{
    return scan_impl<uint32_t, MaxOp<uint32_t>>(in, out, n, inclusive, total_out,
                                                (uint32_t *)ws.scan_tmp, ws.scan_tmp_bytes / 4, st);
}

int scan_sum_u8(const uint8_t *in, uint32_t *out, size_t n, bool inclusive, uint32_t *total_out,
                Workspace &ws, hipStream_t st)
{
    const size_t tiles = n / kScanTile;
    if (n % kScanTile == 0 && tiles > 1 && ((uintptr_t)in & 15u) == 0 && ((uintptr_t)out & 15u) == 0 &&
        ws.scan_tmp_bytes / 4 >= tiles) {
        uint32_t *partial = (uint32_t *)ws.scan_tmp;
        hipLaunchKernelGGL(k_flag_reduce, dim3((unsigned)tiles), dim3(kScanThreads), 0, st,
                           reinterpret_cast<const uint4 *>(in), partial);
        SALZ_LAUNCH_CHECK();
        if (scan_impl<uint32_t, SumOp<uint32_t>>(partial, partial, tiles, false, nullptr,
                                                 partial + tiles, ws.scan_tmp_bytes / 4 - tiles,
                                                 st) != 0)
            return -1;
        hipLaunchKernelGGL(k_flag_scan, dim3((unsigned)tiles), dim3(kScanThreads), 0, st,
                           reinterpret_cast<const uint4 *>(in), out, (const uint32_t *)partial,
                           inclusive ? 1 : 0, (uint32_t)tiles, total_out);
        SALZ_LAUNCH_CHECK();
        return 0;
    }
    return scan_impl<uint32_t, SumOp<uint32_t>, uint8_t>(in, out, n, inclusive, total_out,
                                                         (uint32_t *)ws.scan_tmp,
                                                         ws.scan_tmp_bytes / 4, st);
}

// hipMemsetAsync in one launch: the runtime splits a small or unaligned fill into two or three
// kernels, and the per-round / per-pass flag and counter resets of a block added up to about 100
// fill launches per 16 MiB block (profiles/r05fa_*). 16-byte stores, byte stores for an unaligned
// head and the tail.
__global__ __launch_bounds__(256) void k_fill(uint8_t *__restrict__ p, uint32_t v4, size_t bytes, size_t head)
{
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x, nt = (size_t)gridDim.x * 256;
    const uint8_t v = (uint8_t)v4;
    if (t < head)
        p[t] = v;
    uint8_t *q = p + head;
    const size_t body = (bytes - head) / 16, tail = (bytes - head) % 16;
    uint4 *q4 = reinterpret_cast<uint4 *>(q);
    for (size_t i = t; i < body; i += nt)
        q4[i] = make_uint4(v4, v4, v4, v4);
    if (t < tail)
        q[body * 16 + t] = v;
}

hipError_t fill_async(void *ptr, int value, size_t bytes, hipStream_t st)
{
    if (bytes == 0)
        return hipSuccess;
    const uint32_t b = (uint8_t)value, v4 = b * 0x01010101u;
    const size_t mis = (uintptr_t)ptr & 15u, head = mis ? (16 - mis < bytes ? 16 - mis : bytes) : 0;
    const size_t body = (bytes - head) / 16;
    const size_t want = body > 16 ? (body + 255) / 256 : 1;
    const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, st, static_cast<uint8_t *>(ptr), v4, bytes, head);
    return hipGetLastError();
}

int scan_sum_u64(const uint64_t *in, uint64_t *out, size_t n, bool inclusive,
                 uint64_t *total_out, Workspace &ws, hipStream_t st)
{
    return scan_impl<uint64_t, SumOp<uint64_t>>(in, out, n, inclusive, total_out,
                                                (uint64_t *)ws.scan_tmp, ws.scan_tmp_bytes / 8, st);
}

}  // namespace salz
