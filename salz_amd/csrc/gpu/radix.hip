// radix.hip - stable LSD radix sort of (u64 key, u32 value) pairs for gfx950.
//
// One 8-bit digit per pass, 4096-element tiles (256 threads x 16 items), reduce-then-scan:
//   k_radix_hist    per-tile digit counts (LDS atomics into per-wave sub-histograms), from the
//                   keys or, after a pass that wrote them, from a byte array of this pass's digits
//   k_radix_rowscan per-digit prefixes of the counts over the tiles (+ digit totals; the
//                   scatter adds the digit bases)
//   k_radix_scatter stable tile-local ranking with wave ballots (8 ballots build the peer
//                   mask of lanes sharing a digit; mbcnt gives the rank below), then the
//                   tile is staged in LDS in digit order and written out in contiguous runs.
// Used by the prefix-doubling suffix sorter (sa.hip), which passes only the key bits that
// vary in a round.
#include "internal.hpp"

#include <cstdlib>
#include <vector>

namespace salz {
namespace {

constexpr int kThreads = 256;

// Round 0 of the suffix sorter (sa.hip) can start straight from the text: list entry c is
// suffix init_suffix(c) (common.hpp: the suffixes with fewer than 8 bytes left first,
// shortest first, then the rest in text order) with the big-endian key of its first 8 bytes
// (bytes past its block's suffix text zero). The first pass then builds (key, value) itself
// instead of reading an initial key/value array. A batch of several blocks is then ordered by
// block with extra passes whose digit is the block of the value (kMode 2).
struct TextSrc {
    const uint8_t *T;  // padded text
    Blocks g;
    Alpha a;
    const uint64_t *lrec;  // kMode 4: extraction ranges of the large groups (start << 32 | ...)
    const uint32_t *tmap;  // kMode 4: large group of the first index of every 256
    uint32_t GL;
};

// kMode 4: the large group whose extraction range holds index x (the value). A large group
// outlasts 256 indices, so it is the group of x's 256-tile start or the next one.
__device__ __forceinline__ uint32_t group_of(const TextSrc &t, uint32_t x)
{
    const uint32_t g = t.tmap[x >> 8];
    const uint32_t g1 = g + 1u < t.GL ? g + 1u : g;
    return g1 != g && x >= (uint32_t)(t.lrec[g1] >> 32) ? g1 : g;
}

// (alphabet keys: t.T is the text mapped to symbols, round0_key_mapped)
__device__ __forceinline__ uint64_t init_key(const TextSrc &t, uint32_t i, const uint8_t *code)
{
    (void)code;
    return t.a.bits ? round0_key_mapped(t.T, i, t.g.end(i), t.a) : round0_key(t.T, i, t.g.end(i), t.a);
}

// Round-0 key of suffix i from 16 window bytes (w: the 8 at i, w9: the one at i + 8) for the
// key shapes of round0_key / round0_key_mapped that the single-block text pass serves (raw
// bytes, or 9 symbols of 7 bits of a mapped text).
__device__ __forceinline__ uint64_t window_key(uint64_t w, uint32_t w9, uint32_t left, const Alpha &a)
{
    if (left < 8)
        w &= (1ull << (8u * left)) - 1ull;
    uint64_t x = __builtin_bswap64(w);
    if (a.bits == 0)
        return x;
    const uint32_t b = a.bits;  // (round0_key_mapped's packing)
    x = (x & 0x00FF00FF00FF00FFull) | (((x >> 8) & 0x00FF00FF00FF00FFull) << b);
    x = (x & 0x0000FFFF0000FFFFull) | (((x >> 16) & 0x0000FFFF0000FFFFull) << (2 * b));
    x = (x & 0xFFFFFFFFull) | ((x >> 32) << (4 * b));
    if (a.k == 9)
        x = (x << b) | (left > 8 ? w9 : 0u);
    return x;
}

// digit source of a pass: 0 = key bits, 1 / 3 = key bits of text-built pairs, 2 = block of value,
// 4 = large group of value (value digits are 8-bit; the caller masks key digits to its width)
__device__ __forceinline__ unsigned digit_of(int mode, uint64_t k, uint32_t v, int shift, const TextSrc &t)
{
    return mode == 2 ? (t.g.blk(v) >> shift) & 255u
           : mode == 4 ? (group_of(t, v) >> shift) & 255u
                       : (unsigned)(k >> shift);
}
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
static_assert(kTile == kRadixTile, "tile size mismatch");

template <int kMode, int DB>
__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint64_t *__restrict__ keys,
                                                         const uint32_t *__restrict__ vals,
                                                         uint32_t m, int shift,
                                                         uint32_t *__restrict__ counts,
                                                         uint32_t ntiles, TextSrc txt,
                                                         const uint32_t *__restrict__ tcnt)
{
    // (tcnt: a segmented sort's entries per tile, radix_sort_segmented; digit arrays are counted
    // by k_radix_hist_dig)
    // Sub-histograms (8 per wave by lane & 7 for 8-bit digits, 4 per wave by lane & 3 for 9-bit
    // ones), ND + 1 words apart so the copies of one digit sit in different banks: lanes of a wave
    // adding to a hot digit (text keys' leading bytes are skewed) spread over several addresses
    // instead of serialising on one.
    constexpr int ND = 1 << DB, kCopies = DB == 8 ? 32 : 16, kPerWave = kCopies / 4, kStride = ND + 1;
    constexpr uint32_t kMask = ND - 1;
    static_assert(kMode == 0 || kMode == 1 || DB == 8, "value-digit passes are 8-bit");
    __shared__ uint32_t h[kCopies * kStride];
    unsigned tid = threadIdx.x, wave = tid >> 6;
    for (int i = tid; i < kCopies * kStride; i += kThreads)
        h[i] = 0;
    __syncthreads();
    uint32_t *mine = h + (wave * kPerWave + (tid & (kPerWave - 1u))) * kStride;
    // Two keys per 16-byte load: pair j of thread t is keys 2 (j * kThreads + t) and + 1.
    const size_t base = (size_t)blockIdx.x * kTile;
    const uint4 *kp = reinterpret_cast<const uint4 *>(keys + base);
    const size_t left = tcnt ? tcnt[blockIdx.x] : m > base ? m - base : 0;
    if (kMode == 2 || kMode == 4) {
        for (int j = 0; j < kItems; j++) {
            const size_t i = (size_t)j * kThreads + tid;
            if (i < left)
                atomicAdd(&mine[digit_of(kMode, 0, vals[base + i], shift, txt)], 1u);
        }
    } else if (kMode == 1 && shift == 0 &&
               (txt.a.bits == 0 || txt.a.k == 9)) {
        // Round 0's first digit is its key's low 8 or 9 bits: the 8th byte (raw keys; 9-bit digits
        // add the 7th byte's low bit), or the last symbol with the low bits of the one before (9
        // symbols of 7 bits): two byte loads per suffix instead of the whole key. Loads
        // unconditional (the text is padded), past the suffix's end masked to 0 like the key's bytes.
        const uint32_t b = txt.a.bits ? txt.a.bits : 8u, kl = txt.a.bits ? txt.a.k - 1u : 7u;
        const bool prev = txt.a.bits ? true : DB > 8;  // (the digit takes bits of the byte before)
        uint32_t d[kItems];
        if (txt.g.nb == 1 && base >= 7 && left >= (size_t)kTile) {  // (tile-uniform)
            // One block, a whole tile past the short suffixes: entry c is suffix c - 7, so a
            // thread's 16 consecutive entries need the 17 consecutive bytes from their first
            // suffix + kl - 1 on: three loads instead of 32 byte loads.
            const size_t c0 = base + (size_t)tid * kItems;
            const uint32_t i0 = (uint32_t)(c0 - 7), e = txt.g.npos;
            const size_t p0 = (size_t)i0 + kl - 1u;
            const uint64_t w0 = load_u64_any(txt.T, p0), w1 = load_u64_any(txt.T, p0 + 8);
            const uint32_t w2 = txt.T[p0 + 16];
            auto byte_at = [&](uint32_t k) -> uint32_t {  // T[p0 + k], k <= 16
                return k < 8 ? (uint32_t)(w0 >> (8 * k)) & 255u : k < 16 ? (uint32_t)(w1 >> (8 * (k - 8))) & 255u : w2;
            };
#pragma unroll
            for (int j = 0; j < kItems; j++) {
                const uint32_t i = i0 + (uint32_t)j;
                const uint32_t s7 = i + kl < e ? byte_at((uint32_t)j + 1u) : 0u;
                const uint32_t s6 = prev && i + kl - 1u < e ? byte_at((uint32_t)j) : 0u;
                d[j] = (s7 | (s6 << b)) & kMask;
            }
#pragma unroll
            for (int j = 0; j < kItems; j++)
                atomicAdd(&mine[d[j]], 1u);
        } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            const size_t idx = (size_t)j * kThreads + tid;
            const uint32_t i = init_suffix(idx < left ? base + idx : 0, txt.g), e = txt.g.end(i);
            const uint32_t t7 = txt.T[(size_t)i + kl], t6 = txt.T[(size_t)i + kl - 1u];
            const uint32_t s7 = i + kl < e ? t7 : 0u, s6 = prev && i + kl - 1u < e ? t6 : 0u;
            d[j] = (s7 | (s6 << b)) & kMask;
        }
#pragma unroll
        for (int j = 0; j < kItems; j++)
            if ((size_t)j * kThreads + tid < left)
                atomicAdd(&mine[d[j]], 1u);
        }
    } else if (kMode == 1) {
        // text loads unconditional (clamped entry), so none is issued under a narrower mask
        uint64_t kk[kItems];
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            const size_t i = (size_t)j * kThreads + tid;
            kk[j] = init_key(txt, init_suffix(i < left ? base + i : 0, txt.g), nullptr);
        }
#pragma unroll
        for (int j = 0; j < kItems; j++)
            if ((size_t)j * kThreads + tid < left)
                atomicAdd(&mine[(unsigned)(kk[j] >> shift) & kMask], 1u);
    } else if (left >= (size_t)kTile) {
        uint4 x[kItems / 2];
#pragma unroll
        for (int j = 0; j < kItems / 2; j++)
            x[j] = kp[j * kThreads + tid];
#pragma unroll
        for (int j = 0; j < kItems / 2; j++) {
            const uint64_t k0 = (uint64_t)x[j].y << 32 | x[j].x, k1 = (uint64_t)x[j].w << 32 | x[j].z;
            atomicAdd(&mine[(unsigned)(k0 >> shift) & kMask], 1u);
            atomicAdd(&mine[(unsigned)(k1 >> shift) & kMask], 1u);
        }
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            const size_t i = (size_t)j * kThreads + tid;
            if (i < left)
                atomicAdd(&mine[(unsigned)(keys[base + i] >> shift) & kMask], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = tid; d < (uint32_t)ND; d += kThreads) {
        uint32_t sum = 0;
#pragma unroll
        for (int c = 0; c < kCopies; c++)
            sum += h[c * kStride + d];
        counts[(size_t)d * ntiles + blockIdx.x] = sum;
    }
}

// Per-tile digit counts from the digits the previous scatter wrote (16 per thread: one 16-byte
// load of bytes, or two of 16-bit digits). The loads are issued before the counters are cleared,
// and 16 sub-histograms (4 per wave, by lane & 3; ND + 1 words apart so one digit's copies sit in
// different banks) keep the LDS at 16 KB (8-bit digits): 8 workgroups per CU instead of 4 with 32
// copies, and half the clearing and summing per tile (k_radix_hist with 32 copies: 98 us per
// 100 M digits, latency-bound).
template <typename DT, int DB>
__global__ __launch_bounds__(kThreads) void k_radix_hist_dig(const DT *__restrict__ dig, uint32_t m,
                                                             uint32_t *__restrict__ counts, uint32_t ntiles,
                                                             const uint32_t *__restrict__ tcnt)
{
    // (9-bit digits: 8 copies, 2 per wave, so that the LDS stays at 16 KB: 8 workgroups per CU)
    constexpr int ND = 1 << DB, kStride = ND + 1, kDigCopies = DB == 8 ? 16 : 8, kPerWave = kDigCopies / 4;
    constexpr int kPerLoad = 16 / sizeof(DT), kLoads = kItems / kPerLoad, kBits = 8 * sizeof(DT);
    constexpr uint32_t kMask = ND - 1;
    __shared__ uint32_t h[kDigCopies * kStride];
    const unsigned tid = threadIdx.x, wave = tid >> 6;
    const size_t base = (size_t)blockIdx.x * kTile;
    const size_t left = tcnt ? tcnt[blockIdx.x] : m - base;
    // (the digit buffer has room past m: the loads are unconditional)
    const uint4 *src = reinterpret_cast<const uint4 *>(dig + base + (size_t)tid * kItems);
    uint4 x[kLoads];
#pragma unroll
    for (int q = 0; q < kLoads; q++)
        x[q] = src[q];
    for (int i = tid; i < kDigCopies * kStride; i += kThreads)
        h[i] = 0;
    __syncthreads();
    uint32_t *mine = h + (wave * kPerWave + (tid & (kPerWave - 1u))) * kStride;
#pragma unroll
    for (int q = 0; q < kLoads; q++) {
        const uint32_t w[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
        for (int j = 0; j < kPerLoad; j++)
            if ((size_t)tid * kItems + q * kPerLoad + j < left)
                atomicAdd(&mine[(w[j * kBits / 32] >> (kBits * j % 32)) & kMask], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < (uint32_t)ND; d += kThreads) {
        uint32_t sum = 0;
#pragma unroll
        for (int c = 0; c < kDigCopies; c++)
            sum += h[c * kStride + d];
        counts[(size_t)d * ntiles + blockIdx.x] = sum;
    }
}

// Digit-major tile counts -> per-digit exclusive prefixes over the tiles (in place), one
// workgroup per digit, plus the digit totals; k_radix_scatter adds the digit bases (an
// exclusive scan of the 256 totals) itself. One launch instead of a three-kernel device scan.
// A step takes TH * IT counts: coalesced loads into LDS (one pad word per 32, so that a thread's
// IT consecutive words are conflict-free), IT per thread scanned in registers, a block scan of
// the thread sums, and coalesced stores back. radix_rowscan picks the shape by the tile count:
// 256-thread workgroups for the small sorts that run beside other encodes (a 1024-thread
// workgroup waits for a whole free CU), one step for rows of up to 24576 tiles (100 MB).
__device__ __forceinline__ uint32_t rs_pad(uint32_t x) { return x + (x >> 5); }

template <int TH, int IT>
__global__ __launch_bounds__(TH) void k_radix_rowscan(uint32_t *__restrict__ counts, uint32_t ntiles,
                                                      uint32_t *__restrict__ totals)
{
    constexpr uint32_t kStep = TH * IT;
    __shared__ uint32_t buf[kStep + kStep / 32];
    __shared__ uint32_t wsum[TH / 64];
    uint32_t *row = counts + (size_t)blockIdx.x * ntiles;
    const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < ntiles; base += kStep) {
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t i = base + j * TH + tid;
            buf[rs_pad(j * TH + tid)] = i < ntiles ? row[i] : 0u;
        }
        __syncthreads();
        uint32_t v[IT], sum = 0;
#pragma unroll
        for (int j = 0; j < IT; j++) {
            v[j] = buf[rs_pad(tid * IT + j)];
            sum += v[j];
        }
        uint32_t x = sum;
#pragma unroll
        for (unsigned d = 1; d < 64; d <<= 1) {
            const uint32_t y = shfl_up_u32(x, d);
            if (lane >= d)
                x += y;
        }
        if (lane == 63)
            wsum[wave] = x;
        __syncthreads();
        uint32_t pre = carry, all = 0;
#pragma unroll
        for (unsigned w = 0; w < TH / 64; w++) {
            const uint32_t ws = wsum[w];
            pre += w < wave ? ws : 0u;
            all += ws;
        }
        uint32_t run = pre + x - sum;
#pragma unroll
        for (int j = 0; j < IT; j++) {
            buf[rs_pad(tid * IT + j)] = run;
            run += v[j];
        }
        carry += all;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t i = base + j * TH + tid;
            if (i < ntiles)
                row[i] = buf[rs_pad(j * TH + tid)];
        }
        __syncthreads();
    }
    if (tid == 0)
        totals[blockIdx.x] = carry;
}

// Segmented sort (radix_sort_segmented): the row of digit d (blockIdx.x) in LDS at once (at most
// TH * IT tiles), scanned over all tiles as above, then made relative to the first tile of each
// tile's segment; the segment's first tile also writes the segment's total of digit d
// (segtot[seg * nd + d]), whose scan over the digits k_radix_scatter does per tile.
template <int TH, int IT>
__global__ __launch_bounds__(TH) void k_radix_segscan(uint32_t *__restrict__ counts, uint32_t ntiles,
                                                      const uint32_t *__restrict__ tseg,
                                                      const uint32_t *__restrict__ pt0,
                                                      const uint32_t *__restrict__ ptn,
                                                      uint32_t *__restrict__ segtot, uint32_t nd)
{
    constexpr uint32_t kStep = TH * IT;
    __shared__ uint32_t buf[kStep + kStep / 32 + 1];
    __shared__ uint32_t wsum[TH / 64];
    uint32_t *row = counts + (size_t)blockIdx.x * ntiles;
    const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t i = j * TH + tid;
        buf[rs_pad(i)] = i < ntiles ? row[i] : 0u;
    }
    __syncthreads();
    uint32_t v[IT], sum = 0;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        v[j] = buf[rs_pad(tid * IT + j)];
        sum += v[j];
    }
    uint32_t x = sum;
#pragma unroll
    for (unsigned d = 1; d < 64; d <<= 1) {
        const uint32_t y = shfl_up_u32(x, d);
        if (lane >= d)
            x += y;
    }
    if (lane == 63)
        wsum[wave] = x;
    __syncthreads();
    uint32_t pre = 0, all = 0;
#pragma unroll
    for (unsigned w = 0; w < TH / 64; w++) {
        const uint32_t ws = wsum[w];
        pre += w < wave ? ws : 0u;
        all += ws;
    }
    uint32_t run = pre + x - sum;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        buf[rs_pad(tid * IT + j)] = run;
        run += v[j];
    }
    if (tid == 0)
        buf[rs_pad(kStep)] = all;  // (the prefix past the last tile)
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t i = j * TH + tid;
        if (i < ntiles) {
            const uint32_t sg = tseg[i], t0 = pt0[sg], p0 = buf[rs_pad(t0)];
            row[i] = buf[rs_pad(i)] - p0;
            if (i == t0) {
                const uint32_t t1 = t0 + ptn[sg];
                segtot[(size_t)sg * nd + blockIdx.x] = buf[rs_pad(t1 < ntiles ? t1 : kStep)] - p0;
            }
        }
    }
}

void radix_rowscan(uint32_t *counts, uint32_t ntiles, uint32_t *totals, hipStream_t st, uint32_t ndig)
{
    if (ntiles <= 256 * 16)
        hipLaunchKernelGGL((k_radix_rowscan<256, 16>), dim3(ndig), dim3(256), 0, st, counts, ntiles, totals);
    else if (ntiles <= 512 * 16)
        hipLaunchKernelGGL((k_radix_rowscan<512, 16>), dim3(ndig), dim3(512), 0, st, counts, ntiles, totals);
    else if (ndig > 256)  // (512 rows: three 50 KB workgroups per CU hold them all at once)
        hipLaunchKernelGGL((k_radix_rowscan<512, 24>), dim3(ndig), dim3(512), 0, st, counts, ntiles, totals);
    else
        hipLaunchKernelGGL((k_radix_rowscan<1024, 24>), dim3(ndig), dim3(1024), 0, st, counts, ntiles, totals);
}

// Tile of scatter workgroup b: workgroups are dealt round-robin to the 8 XCDs (b mod 8), so XCD x
// takes the x-th eighth of the tiles in order, and consecutive tiles, whose runs of one digit are
// adjacent in the output, write them through the same L2 (a run's partial end lines merge there).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles)
{
    const uint32_t x = b & 7u, i = b >> 3, per = ntiles >> 3, rem = ntiles & 7u;
    return x * per + (x < rem ? x : rem) + i;
}

// TH threads per 4096-element tile (256: 16 items per thread; 512: 8 items, half the registers
// per thread and twice the waves per CU for the same LDS). DB: digit bits (8, or 9 with 512
// threads: thread = digit in the digit scans); DT: type of the next pass's digit array.
template <int kMode, int TH, int DB, typename DT>
__global__ __launch_bounds__(TH) void k_radix_scatter(
    const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
    uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t m, int shift,
    const uint32_t *__restrict__ offs, uint32_t ntiles, const uint32_t *__restrict__ totals,
    TextSrc txt, DT *__restrict__ dout, int nshift, uint32_t nmask, const uint32_t *__restrict__ tcnt,
    const uint32_t *__restrict__ tseg, const uint32_t *__restrict__ pt0)
{
    // Segmented sort (tseg set, radix_sort_segmented): tile `tile` holds tcnt[tile] entries of
    // segment tseg[tile], whose output starts at tile pt0[seg]; offs are offsets inside the
    // segment and totals its digit totals (ND per segment).
    constexpr int IT = kTile / TH, NW = TH / 64, ND = 1 << DB, DW = ND / 64;
    constexpr uint32_t kMask = ND - 1;
    static_assert(ND <= TH, "one thread per digit");
    static_assert(kMode == 0 || kMode == 1 || kMode == 3 || DB == 8, "value-digit passes are 8-bit");
    // Keys and values are staged one after the other in the same 32 KB (3 workgroups per CU
    // with the counters of 512 threads, instead of 2 with a 48 KB key + value stage).
    __shared__ uint64_t skey[kTile];
    uint32_t *sval = reinterpret_cast<uint32_t *>(skey);
    // (16-bit: a tile's counts stay below 2^16, and the 8-bit passes then fit 4 workgroups per CU)
    __shared__ uint16_t cnt[NW][ND];
    __shared__ uint32_t dstart[ND];
    __shared__ uint32_t gbase[ND];
    __shared__ uint32_t wsum[2][DW];

    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
    for (int i = tid; i < NW * ND; i += TH)
        (&cnt[0][0])[i] = 0;
    __syncthreads();
    const size_t lim = tcnt ? (size_t)tile * kTile + tcnt[tile] : (size_t)m;  // entries end
    const uint32_t sg = tseg ? tseg[tile] : 0u;

    // Warp-striped: wave w owns tile elements [w*IT*64, (w+1)*IT*64), item j covers 64 of them.
    const size_t base = (size_t)tile * kTile + (size_t)wave * (IT * 64);
    uint64_t k[IT];
    uint32_t v[IT];
    uint32_t lrank[IT];
    // kMode 3: one block. Entry c is suffix c - 7 (c >= 7; the first seven are the short
    // suffixes n - 1 - c), so a tile's keys come from one text window of kTile + 16 bytes,
    // staged in LDS (the key stage is free until the ranking is done) with coalesced 8-byte
    // loads, instead of three unaligned global loads per entry.
    if (kMode == 3) {
        uint64_t *W = skey;
        constexpr uint32_t kWords = kTile / 8 + 3;
        const size_t tb = (size_t)tile * kTile;
        const size_t w0 = tb ? (tb - 7) >> 3 : 0;
        const size_t wmax = ((size_t)txt.g.npos + 64) >> 3;  // zero padding past the text
        for (uint32_t q = tid; q < kWords; q += TH) {
            const size_t wq = w0 + q;
            const uint64_t x = reinterpret_cast<const uint64_t *>(txt.T)[wq < wmax ? wq : wmax];
            W[q] = wq < wmax ? x : 0ull;
        }
        __syncthreads();
        const uint32_t npos = txt.g.npos;
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const size_t c = base + (size_t)j * 64 + lane;
            const bool shortsfx = c < 7;
            const uint32_t sfx = shortsfx ? npos - 1u - (uint32_t)c : (uint32_t)c - 7u;
            const uint32_t off = shortsfx ? 0u : (uint32_t)((size_t)sfx - (w0 << 3));
            const uint32_t q = off >> 3, sh = (off & 7u) * 8u;
            const uint64_t a0 = W[q], a1 = W[q + 1];
            uint64_t w = (a0 >> sh) | ((a1 << 1) << (63u - sh));
            uint32_t w9 = (uint32_t)(a1 >> sh) & 255u;
            if (base + (size_t)j * 64 < 7) {  // (wave-uniform: the short suffixes, tile 0 only)
                const uint64_t g = load_u64_any(txt.T, shortsfx ? sfx : 0u);
                w = shortsfx ? g : w;
                w9 = shortsfx ? 0u : w9;
            }
            k[j] = c < m ? window_key(w, w9, npos - sfx, txt.a) : 0ull;
            v[j] = sfx;
        }
        __syncthreads();  // (the window's LDS is the key stage below)
    }
#pragma unroll
    for (int j = 0; j < IT; j++) {
        if (kMode == 3)
            break;
        size_t i = base + (size_t)j * 64 + lane;
        bool ok = i < lim;
        if (kMode == 1) {  // unconditional text loads (clamped entry)
            const uint32_t sfx = init_suffix(ok ? i : 0, txt.g);
            const uint64_t kk = init_key(txt, sfx, nullptr);
            k[j] = ok ? kk : 0ull;
            v[j] = sfx;
        } else {
            k[j] = ok ? kin[i] : 0ull;
            v[j] = ok ? vin[i] : 0u;
        }
    }

#pragma unroll
    for (int j = 0; j < IT; j++) {
        size_t i = base + (size_t)j * 64 + lane;
        bool ok = i < lim;
        unsigned d = digit_of(kMode, k[j], v[j], shift, txt) & kMask;
        uint64_t peers = wave_ballot(ok);
#pragma unroll
        for (int b = 0; b < DB; b++) {
            bool bit = (d >> b) & 1u;
            uint64_t bb = wave_ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        if (!ok)
            peers = 0;
        unsigned below = count_below(peers);
        unsigned total = (unsigned)__popcll(peers);
        int leader = peers ? (int)__ffsll((unsigned long long)peers) - 1 : (int)lane;
        uint32_t old = 0;
        if (ok && (int)lane == leader) {
            old = cnt[wave][d];
            cnt[wave][d] = (uint16_t)(old + total);
        }
        old = shfl_u32(old, leader);
        lrank[j] = old + below;
    }
    __syncthreads();

    // Digit bases (exclusive scan of the ND digit totals) and the tile-local digit starts
    // (exclusive scan of the per-digit tile counts), thread = digit; the per-wave counts become
    // per-wave starts.
    const bool dg = tid < ND;
    uint32_t xt = 0, xc = 0, tt = 0, tot = 0;
    if (dg) {
        tt = totals[tseg ? (size_t)sg * ND + tid : tid];
#pragma unroll
        for (int w = 0; w < NW; w++)
            tot += cnt[w][tid];
        xt = tt;
        xc = tot;
#pragma unroll
        for (unsigned dd = 1; dd < 64; dd <<= 1) {
            const uint32_t yt = shfl_up_u32(xt, dd), yc = shfl_up_u32(xc, dd);
            if (lane >= dd) {
                xt += yt;
                xc += yc;
            }
        }
        if (lane == 63) {
            wsum[0][wave] = xt;
            wsum[1][wave] = xc;
        }
    }
    __syncthreads();
    if (dg) {
        uint32_t pt = 0, pc = 0;
        for (unsigned w = 0; w < wave; w++) {
            pt += wsum[0][w];
            pc += wsum[1][w];
        }
        gbase[tid] = pt + xt - tt + offs[(size_t)tid * ntiles + tile] + (tseg ? pt0[sg] * (uint32_t)kTile : 0u);
        const uint32_t ds = pc + xc - tot;
        dstart[tid] = ds;
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint32_t c = cnt[w][tid];
            cnt[w][tid] = (uint16_t)run;
            run += c;
        }
    }
    __syncthreads();

    if (kMode == 2 || kMode == 4) {
        // block / group passes: the digit is a function of the value, so the values are staged
        // first (their digits give each slot's destination), then the keys
        uint32_t pos[IT];
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const size_t i = base + (size_t)j * 64 + lane;
            const unsigned d = digit_of(kMode, 0, v[j], shift, txt);
            pos[j] = dstart[d] + cnt[wave][d] + lrank[j];
            if (i < m)
                sval[pos[j]] = v[j];
        }
        __syncthreads();
        const size_t tbase = (size_t)tile * kTile;
        const uint32_t tcount = (uint32_t)((m - tbase) < (size_t)kTile ? (m - tbase) : (size_t)kTile);
        uint32_t gdst[IT];
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t s = tid + (uint32_t)j * TH;
            if (s < tcount) {
                const uint32_t val = sval[s];
                const unsigned d = digit_of(kMode, 0, val, shift, txt);
                gdst[j] = gbase[d] + (s - dstart[d]);
                vout[gdst[j]] = val;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const size_t i = base + (size_t)j * 64 + lane;
            if (i < m)
                skey[pos[j]] = k[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t s = tid + (uint32_t)j * TH;
            if (s < tcount)
                kout[gdst[j]] = skey[s];
        }
        return;
    }
    uint32_t pos[IT];  // tile-local sorted position of each item
#pragma unroll
    for (int j = 0; j < IT; j++) {
        size_t i = base + (size_t)j * 64 + lane;
        unsigned d = (unsigned)(k[j] >> shift) & kMask;
        pos[j] = dstart[d] + cnt[wave][d] + lrank[j];
        if (i < lim)
            skey[pos[j]] = k[j];
    }
    __syncthreads();

    size_t tbase = (size_t)tile * kTile;
    uint32_t tcount = (uint32_t)((lim - tbase) < (size_t)kTile ? (lim - tbase) : (size_t)kTile);
    uint32_t gdst[IT];  // global destination of staged slot tid + j * TH
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t s = tid + (uint32_t)j * TH;
        if (s < tcount) {
            uint64_t key = skey[s];
            unsigned d = (unsigned)(key >> shift) & kMask;
            gdst[j] = gbase[d] + (s - dstart[d]);
            kout[gdst[j]] = key;
            if (dout)  // the next pass's digit, for its histogram
                dout[gdst[j]] = (DT)((key >> nshift) & nmask);
        }
    }
    __syncthreads();  // keys out of LDS; the same bytes now stage the values
#pragma unroll
    for (int j = 0; j < IT; j++) {
        size_t i = base + (size_t)j * 64 + lane;
        if (i < lim)
            sval[pos[j]] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t s = tid + (uint32_t)j * TH;
        if (s < tcount)
            vout[gdst[j]] = sval[s];
    }
}

}  // namespace

// Digit widths of a sort over `bits` key bits: 8-bit digits, or where the caller prefers them
// 9-bit digits wherever they save a pass (63-bit text keys: 7 passes instead of 8), the 9-bit
// ones first.
// Measured on one box (round 5, tools/ab_env.sh): a 9-bit pass costs 575 us + 120 us of
// histogram + 30 us of row scan on C2 against 515 + 84 + 17 for an 8-bit one, so the pass it
// saves is spent again: C2 SA 19.79 (8-bit) vs 19.95 ms, mixed 100 MB 24.82 vs 24.72 ms.
static int digit_plan(int bits, bool allow9, bool prefer9, int *width)
{
    const bool nine = prefer9;
    const int p8 = (bits + 7) / 8, p9 = (bits + 8) / 9;
    if (!allow9 || !nine || p9 >= p8) {
        for (int p = 0; p < p8; p++)
            width[p] = 8;
        return p8;
    }
    const int n9 = bits - 8 * p9;  // (p9 passes: n9 of 9 bits, the rest of 8; 0 < n9 <= p9)
    for (int p = 0; p < p9; p++)
        width[p] = p < n9 ? 9 : 8;
    return p9;
}

template <int DB, typename DT>
static void launch_key_scatter(int mode, uint32_t ntiles, hipStream_t st, const uint64_t *kin, const uint32_t *vin,
                               uint64_t *kout, uint32_t *vout, uint32_t m, int shift, const uint32_t *counts,
                               const uint32_t *totals, const TextSrc &txt, DT *dout, int nshift, uint32_t nmask,
                               const uint32_t *tcnt = nullptr, const uint32_t *tseg = nullptr,
                               const uint32_t *pt0 = nullptr)
{
    if (mode == 3)
        hipLaunchKernelGGL((k_radix_scatter<3, 512, DB, DT>), dim3(ntiles), dim3(512), 0, st, kin, vin, kout, vout,
                           m, shift, counts, ntiles, totals, txt, dout, nshift, nmask, tcnt, tseg, pt0);
    else
        hipLaunchKernelGGL((k_radix_scatter<0, 512, DB, DT>), dim3(ntiles), dim3(512), 0, st, kin, vin, kout, vout,
                           m, shift, counts, ntiles, totals, txt, dout, nshift, nmask, tcnt, tseg, pt0);
}

int radix_sort_pairs(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt,
                     uint32_t m, int bit_lo, int bit_hi, Workspace &ws, hipStream_t st,
                     const uint8_t *text, const Blocks *blocks, const Alpha *alpha, uint8_t *digits,
                     bool digits_ready, bool prefer9)
{
    if (m <= 1 || bit_hi <= bit_lo)
        return 0;
    uint32_t ntiles = (m + kTile - 1) / kTile;
    const size_t ncounts = (size_t)ntiles * kMaxDigits;
    if (ncounts + kMaxDigits > ws.radix_counts_elems) {  // + the digit totals
        set_error("radix: count buffer too small");
        return -1;
    }
    uint64_t *kin = *keys, *kout = keys_alt;
    uint32_t *vin = *vals, *vout = vals_alt;
    const Blocks g = blocks ? *blocks : Blocks{0xffffffffu, 1u, m};
    // A batch's round 0: after the key passes, passes on the digits of the value's block
    // (stable), so the list is ordered by (block, key).
    const int blk_bits = blocks && g.nb > 1 ? bit_width(g.nb - 1u) : 0;
    // one block with raw-byte or 8/9-symbol keys: the text pass builds keys from an LDS window
    const bool text_win = g.nb == 1 && g.npos >= 7 &&
                          (!alpha || alpha->bits == 0 || alpha->k == 9);
    // 9-bit digits: key passes of 512 threads only (the generic text pass of a batch and the
    // materialised round-0 list's byte digits keep 8 bits)
    int width[64];
    const int passes_key = digit_plan(bit_hi - bit_lo, !(text && !text_win) && !digits_ready, prefer9, width);
    const int passes = passes_key + (blk_bits + 7) / 8;
    bool wide = false;  // a 9-bit pass: every digit array of this sort is 16-bit
    for (int p = 0; p < passes_key; p++)
        wide |= width[p] > 8;
    // key passes with 512-thread workgroups (8 items per thread; 256 threads with 16 items measured
    // ~0.5% slower on C2, profiles/r03h_tm_radix_ab.txt)
    int shift_key = bit_lo;
    for (int pass = 0; pass < passes; pass++) {
        const int mode = pass >= passes_key ? 2 : (text && pass == 0) ? (text_win ? 3 : 1) : 0;
        const int db = mode == 2 ? 8 : width[pass];
        const int shift = mode == 2 ? 8 * (pass - passes_key) : shift_key;
        TextSrc txt{text, g, Alpha{}, nullptr, nullptr, 0u};
        // digits: written by a key pass for the next key pass, read by that pass's histogram
        const uint8_t *dig_in = digits && (pass > 0 || digits_ready) && mode == 0 ? digits : nullptr;
        uint8_t *dig_out = digits && pass + 1 < passes_key ? digits : nullptr;
        const int nshift = shift + db;
        const uint32_t nmask = pass + 1 < passes_key ? (1u << width[pass + 1]) - 1u : 255u;
        if (alpha)
            txt.a = *alpha;
        if (mode == 1 || mode == 3) {
            if (db == 9)
                hipLaunchKernelGGL((k_radix_hist<1, 9>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                                   ws.radix_counts, ntiles, txt, nullptr);
            else
                hipLaunchKernelGGL((k_radix_hist<1, 8>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                                   ws.radix_counts, ntiles, txt, nullptr);
        } else if (mode == 2) {
            hipLaunchKernelGGL((k_radix_hist<2, 8>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                               ws.radix_counts, ntiles, txt, nullptr);
        } else if (dig_in && wide) {
            const uint16_t *d16 = reinterpret_cast<const uint16_t *>(dig_in);
            if (db == 9)
                hipLaunchKernelGGL((k_radix_hist_dig<uint16_t, 9>), dim3(ntiles), dim3(kThreads), 0, st, d16, m,
                                   ws.radix_counts, ntiles, nullptr);
            else
                hipLaunchKernelGGL((k_radix_hist_dig<uint16_t, 8>), dim3(ntiles), dim3(kThreads), 0, st, d16, m,
                                   ws.radix_counts, ntiles, nullptr);
        } else if (dig_in) {
            hipLaunchKernelGGL((k_radix_hist_dig<uint8_t, 8>), dim3(ntiles), dim3(kThreads), 0, st, dig_in, m,
                               ws.radix_counts, ntiles, nullptr);
        } else if (db == 9) {
            hipLaunchKernelGGL((k_radix_hist<0, 9>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                               ws.radix_counts, ntiles, txt, nullptr);
        } else {
            hipLaunchKernelGGL((k_radix_hist<0, 8>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                               ws.radix_counts, ntiles, txt, nullptr);
        }
        SALZ_LAUNCH_CHECK();
        uint32_t *totals = ws.radix_counts + ncounts;
        radix_rowscan(ws.radix_counts, ntiles, totals, st, 1u << db);
        SALZ_LAUNCH_CHECK();
        // bench.py prices the timed launches at 24 B per element (key + value in and out) + the
        // next pass's digit; the text-sourced and block passes are left out of that roofline
        bool timed = ws.timing && mode == 0 && ws.rx_used + 2 <= ws.rx_pool.size();
        if (timed)
            SALZ_HIP(hipEventRecord(ws.rx_pool[ws.rx_used], st));
        if (mode == 1)
            hipLaunchKernelGGL((k_radix_scatter<1, kThreads, 8, uint8_t>), dim3(ntiles), dim3(kThreads), 0, st, kin,
                               vin, kout, vout, m, shift, ws.radix_counts, ntiles, totals, txt, dig_out, nshift, nmask, nullptr,
                               nullptr, nullptr);
        else if (mode == 2)
            hipLaunchKernelGGL((k_radix_scatter<2, kThreads, 8, uint8_t>), dim3(ntiles), dim3(kThreads), 0, st, kin,
                               vin, kout, vout, m, shift, ws.radix_counts, ntiles, totals, txt, nullptr, 0, 0u, nullptr, nullptr, nullptr);
        else if (wide && db == 9)
            launch_key_scatter<9, uint16_t>(mode, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, totals,
                                            txt, reinterpret_cast<uint16_t *>(dig_out), nshift, nmask);
        else if (wide)
            launch_key_scatter<8, uint16_t>(mode, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, totals,
                                            txt, reinterpret_cast<uint16_t *>(dig_out), nshift, nmask);
        else
            launch_key_scatter<8, uint8_t>(mode, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, totals,
                                           txt, dig_out, nshift, nmask);
        SALZ_LAUNCH_CHECK();
        if (timed) {
            SALZ_HIP(hipEventRecord(ws.rx_pool[ws.rx_used + 1], st));
            ws.rx_used += 2;
            ws.stats.radix_scatter_launches++;
            ws.stats.radix_scatter_elems += m;
            ws.stats.radix_scatter_bytes += (uint64_t)m * (dig_out ? (wide ? 26u : 25u) : 24u);
        }
        if (mode != 2)
            shift_key += db;
        uint64_t *tk = kin;
        kin = kout;
        kout = tk;
        uint32_t *tv = vin;
        vin = vout;
        vout = tv;
    }
    *keys = kin;
    *vals = vin;
    return 0;
}

int radix_sort_by_group(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt, uint32_t m,
                        const uint64_t *lrec, const uint32_t *tmap, uint32_t GL, Workspace &ws, hipStream_t st)
{
    if (m <= 1 || GL <= 1)
        return 0;
    const uint32_t ntiles = (m + kTile - 1) / kTile;
    const size_t ncounts = (size_t)ntiles * kMaxDigits;
    if (ncounts + kMaxDigits > ws.radix_counts_elems) {
        set_error("radix: count buffer too small");
        return -1;
    }
    uint64_t *kin = *keys, *kout = keys_alt;
    uint32_t *vin = *vals, *vout = vals_alt;
    TextSrc txt{nullptr, Blocks{0xffffffffu, 1u, m}, Alpha{}, lrec, tmap, GL};
    const int passes = (bit_width(GL - 1u) + 7) / 8;
    uint32_t *totals = ws.radix_counts + ncounts;
    for (int pass = 0; pass < passes; pass++) {
        hipLaunchKernelGGL((k_radix_hist<4, 8>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, 8 * pass,
                           ws.radix_counts, ntiles, txt, nullptr);
        SALZ_LAUNCH_CHECK();
        radix_rowscan(ws.radix_counts, ntiles, totals, st, 256);
        SALZ_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_radix_scatter<4, kThreads, 8, uint8_t>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin,
                           kout, vout, m, 8 * pass, ws.radix_counts, ntiles, totals, txt, nullptr, 0, 0u, nullptr, nullptr, nullptr);
        SALZ_LAUNCH_CHECK();
        uint64_t *tk = kin;
        kin = kout;
        kout = tk;
        uint32_t *tv = vin;
        vin = vout;
        vout = tv;
    }
    *keys = kin;
    *vals = vin;
    return 0;
}

int radix_sort_segmented(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt,
                         const SegTiles &sg, int bits, Workspace &ws, hipStream_t st, uint8_t *digits)
{
    const uint32_t ntiles = sg.ntiles, m = ntiles * (uint32_t)kTile;
    const size_t ncounts = (size_t)ntiles * kMaxDigits;
    if (ntiles > kSegScanMaxTiles || ncounts + kMaxDigits > ws.radix_counts_elems || !digits) {
        set_error("radix: segmented sort too large");
        return -1;
    }
    uint64_t *kin = *keys, *kout = keys_alt;
    uint32_t *vin = *vals, *vout = vals_alt;
    int width[64];
    const int passes = digit_plan(bits, true, true, width);
    bool wide = false;
    for (int p = 0; p < passes; p++)
        wide |= width[p] > 8;
    const TextSrc txt{nullptr, Blocks{0xffffffffu, 1u, m}, Alpha{}, nullptr, nullptr, 0u};
    int shift = 0;
    for (int pass = 0; pass < passes; pass++) {
        const int db = width[pass], nshift = shift + db;
        const uint32_t nmask = pass + 1 < passes ? (1u << width[pass + 1]) - 1u : 255u;
        uint8_t *dig_out = pass + 1 < passes ? digits : nullptr;
        const uint16_t *d16 = reinterpret_cast<const uint16_t *>(digits);
        if (pass == 0 && db == 9)
            hipLaunchKernelGGL((k_radix_hist<0, 9>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                               ws.radix_counts, ntiles, txt, sg.tcnt);
        else if (pass == 0)
            hipLaunchKernelGGL((k_radix_hist<0, 8>), dim3(ntiles), dim3(kThreads), 0, st, kin, vin, m, shift,
                               ws.radix_counts, ntiles, txt, sg.tcnt);
        else if (wide && db == 9)
            hipLaunchKernelGGL((k_radix_hist_dig<uint16_t, 9>), dim3(ntiles), dim3(kThreads), 0, st, d16, m,
                               ws.radix_counts, ntiles, sg.tcnt);
        else if (wide)
            hipLaunchKernelGGL((k_radix_hist_dig<uint16_t, 8>), dim3(ntiles), dim3(kThreads), 0, st, d16, m,
                               ws.radix_counts, ntiles, sg.tcnt);
        else
            hipLaunchKernelGGL((k_radix_hist_dig<uint8_t, 8>), dim3(ntiles), dim3(kThreads), 0, st, digits, m,
                               ws.radix_counts, ntiles, sg.tcnt);
        SALZ_LAUNCH_CHECK();
        // (the row's LDS sized to the tile count: the small sorts run beside other encodes)
        if (ntiles <= 256 * 8)
            hipLaunchKernelGGL((k_radix_segscan<256, 8>), dim3(1u << db), dim3(256), 0, st, ws.radix_counts, ntiles,
                               sg.tseg, sg.pt0, sg.ptn, sg.segtot, 1u << db);
        else if (ntiles <= 256 * 16)
            hipLaunchKernelGGL((k_radix_segscan<256, 16>), dim3(1u << db), dim3(256), 0, st, ws.radix_counts, ntiles,
                               sg.tseg, sg.pt0, sg.ptn, sg.segtot, 1u << db);
        else if (ntiles <= 512 * 16)
            hipLaunchKernelGGL((k_radix_segscan<512, 16>), dim3(1u << db), dim3(512), 0, st, ws.radix_counts, ntiles,
                               sg.tseg, sg.pt0, sg.ptn, sg.segtot, 1u << db);
        else
            hipLaunchKernelGGL((k_radix_segscan<512, 24>), dim3(1u << db), dim3(512), 0, st, ws.radix_counts, ntiles,
                               sg.tseg, sg.pt0, sg.ptn, sg.segtot, 1u << db);
        SALZ_LAUNCH_CHECK();
        const bool timed = ws.timing && ws.rx_used + 2 <= ws.rx_pool.size();
        if (timed)
            SALZ_HIP(hipEventRecord(ws.rx_pool[ws.rx_used], st));
        if (wide && db == 9)
            launch_key_scatter<9, uint16_t>(0, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, sg.segtot,
                                            txt, reinterpret_cast<uint16_t *>(dig_out), nshift, nmask, sg.tcnt,
                                            sg.tseg, sg.pt0);
        else if (wide)
            launch_key_scatter<8, uint16_t>(0, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, sg.segtot,
                                            txt, reinterpret_cast<uint16_t *>(dig_out), nshift, nmask, sg.tcnt,
                                            sg.tseg, sg.pt0);
        else
            launch_key_scatter<8, uint8_t>(0, ntiles, st, kin, vin, kout, vout, m, shift, ws.radix_counts, sg.segtot,
                                           txt, dig_out, nshift, nmask, sg.tcnt, sg.tseg, sg.pt0);
        SALZ_LAUNCH_CHECK();
        if (timed) {
            SALZ_HIP(hipEventRecord(ws.rx_pool[ws.rx_used + 1], st));
            ws.rx_used += 2;
            ws.stats.radix_scatter_launches++;
            ws.stats.radix_scatter_elems += sg.mvalid;
            ws.stats.radix_scatter_bytes += (uint64_t)sg.mvalid * (dig_out ? (wide ? 26u : 25u) : 24u);
        }
        shift += db;
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    *keys = kin;
    *vals = vin;
    return 0;
}

}  // namespace salz

// ---- test-only: device-resident radix sort self-test (no host work between sorts) ---------
namespace salz {
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_selftest_fill(uint64_t *k, uint32_t *v, uint32_t m, uint64_t seed, int bits,
                                unsigned long long *sum)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    uint64_t x = mix64(seed * 0x9E3779B97F4A7C15ull + i);
    if (bits < 64)
        x &= (1ull << bits) - 1;
    // few distinct keys in half the runs: exercises stability
    if (seed & 1)
        x &= 0xF0F0ull;
    k[i] = x;
    v[i] = (uint32_t)i;
    atomicAdd(sum, (unsigned long long)mix64(x ^ ((uint64_t)i << 40)));
}

__global__ void k_selftest_check(const uint64_t *k, const uint32_t *v, uint32_t m,
                                 unsigned long long *sum, unsigned int *bad)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m)
        return;
    atomicAdd(sum, (unsigned long long)mix64(k[i] ^ ((uint64_t)v[i] << 40)));
    if (i > 0 && (k[i - 1] > k[i] || (k[i - 1] == k[i] && v[i - 1] >= v[i])))
        atomicAdd(bad, 1u);
}

}  // namespace
}  // namespace salz

// nine: 9-bit digits wherever they save a pass (the rank rounds' plan), else 8-bit digits
extern "C" long salz_debug_radix_selftest(int device, uint32_t m, int bits, int iters,
                                          uint64_t seed, int nine)
{
    using namespace salz;
    Workspace ws;
    if (workspace_alloc(ws, device, (size_t)m + 8) != 0)
        return -1;
    long failures = 0;
    unsigned long long *dsum = reinterpret_cast<unsigned long long *>(ws.dscal) + 100;
    unsigned int *dbad = reinterpret_cast<unsigned int *>(ws.dscal) + 300;
    for (int it = 0; it < iters; it++) {
        (void)hipMemsetAsync(dsum, 0, 16, ws.stream);
        (void)hipMemsetAsync(dbad, 0, 4, ws.stream);
        hipLaunchKernelGGL(k_selftest_fill, dim3(grid_for(m, 256)), dim3(256), 0, ws.stream,
                           ws.keyA, ws.valA, m, seed + it, bits, dsum);
        uint64_t *K = ws.keyA;
        uint32_t *V = ws.valA;
        if (radix_sort_pairs(&K, &V, ws.keyB, ws.valB, m, 0, bits, ws, ws.stream, nullptr, nullptr, nullptr,
                             nullptr, false, nine != 0) != 0) {
            failures++;
            break;
        }
        hipLaunchKernelGGL(k_selftest_check, dim3(grid_for(m, 256)), dim3(256), 0, ws.stream, K, V,
                           m, dsum + 1, dbad);
        unsigned long long h[2];
        unsigned int b = 0;
        (void)hipMemcpyAsync(h, dsum, 16, hipMemcpyDeviceToHost, ws.stream);
        (void)hipMemcpyAsync(&b, dbad, 4, hipMemcpyDeviceToHost, ws.stream);
        (void)hipStreamSynchronize(ws.stream);
        if (b || h[0] != h[1]) {
            failures++;
            fprintf(stderr, "radix selftest it=%d m=%u bits=%d: %u order/stability errors, multiset %s\n",
                    it, m, bits, b, h[0] == h[1] ? "ok" : "CHANGED");
        }
    }
    workspace_free(ws);
    return failures;
}
