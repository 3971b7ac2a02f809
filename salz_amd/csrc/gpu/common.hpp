// common.hpp - shared CDNA4 (gfx950) device helpers for the SA-LZ pipeline.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

namespace salz {

constexpr int kWave = 64;  // CDNA wavefront width

// ---- error plumbing (host) -------------------------------------------------------------
void set_error(const char *fmt, ...);

#define SALZ_HIP(call)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            ::salz::set_error("%s:%d: %s -> %s", __FILE__, __LINE__, #call,               \
                              hipGetErrorString(e_));                                     \
            return -1;                                                                    \
        }                                                                                 \
    } while (0)

#define SALZ_LAUNCH_CHECK() SALZ_HIP(hipGetLastError())

static inline unsigned grid_for(size_t n, unsigned per_block)
{
    size_t g = (n + per_block - 1) / per_block;
    return g == 0 ? 1u : (unsigned)g;
}

static inline int bit_width(uint64_t v)  // bits needed to represent v (0 -> 0)
{
    int b = 0;
    while (v) {
        b++;
        v >>= 1;
    }
    return b;
}

// ---- wave primitives (device) --------------------------------------------------------------
__device__ __forceinline__ unsigned lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// number of set bits of `mask` in lanes strictly below this lane
__device__ __forceinline__ unsigned count_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src)
{
    return (uint32_t)__shfl((int)v, src, kWave);
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    uint32_t lo = shfl_u32((uint32_t)v, src), hi = shfl_u32((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t shfl_up_u32(uint32_t v, unsigned d)
{
    return (uint32_t)__shfl_up((int)v, d, kWave);
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, unsigned d)
{
    uint32_t lo = shfl_up_u32((uint32_t)v, d), hi = shfl_up_u32((uint32_t)(v >> 32), d);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int m)
{
    return (uint32_t)__shfl_xor((int)v, m, kWave);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        uint32_t o = shfl_xor_u32(v, m);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        uint32_t o = shfl_xor_u32(v, m);
        v = o > v ? o : v;
    }
    return v;
}

// ---- device index checks ---------------------------------------------------------------
// Kernels whose addresses come from data (suffix ranks, group tables) check them and, on a
// violation, set a bit in this device word and skip the access instead of faulting; the
// host reads the word with the stage's scalars and fails the call (salz_gpu_last_error).
constexpr size_t kErrWord = 60;  // u32 index into Workspace::dscal
enum : uint32_t {
    kErrCommit = 1u, kErrKeys = 2u, kErrSeg = 4u, kErrExtract = 8u, kErrPutback = 16u,
    kErrPhi = 32u, kErrAnsv = 64u, kErrParse = 128u, kErrDc3 = 0x100000u
};

__device__ __forceinline__ bool bad_index(bool bad, uint32_t *err, uint32_t code)
{
    if (bad)
        atomicOr(err, code);
    return bad;
}

// ---- chunk-interleaved layout of the per-position parse arrays --------------------------
// The parse walks each chunk of K = 2^klog positions backwards, one lane per chunk, and the
// 64 lanes of a wave own 64 consecutive chunks (a "tile" of 64K positions). Position
// p = (tile t, lane l, row j) with j = p mod K, l = (p / K) mod 64, t = p / 64K is stored at
// t*64K + j*64 + l, so a wave stepping row j in lockstep touches 64 consecutive elements.
// Arrays in this layout: candidates (ansv.hip), choices, costs and parse state (parse.hip).
constexpr uint32_t kTileChunks = 64;
constexpr uint32_t kMaxChunkLog = 9;  // K <= 512
constexpr size_t kLayoutPad = (size_t)kTileChunks << kMaxChunkLog;  // storage granularity

__host__ __device__ __forceinline__ size_t sidx(uint32_t p, uint32_t klog)
{
    const uint32_t j = p & ((1u << klog) - 1u), c = p >> klog;
    return ((size_t)(c >> 6) << (klog + 6)) | ((size_t)j << 6) | (c & 63u);
}

__host__ __device__ __forceinline__ uint64_t spos(size_t s, uint32_t klog)
{
    const size_t t = s >> (klog + 6), j = (s >> 6) & ((1u << klog) - 1u), l = s & 63u;
    return (((uint64_t)t * 64u + l) << klog) | j;
}

// vnibble_size (lib/salz.c:565-588)
__device__ __forceinline__ uint32_t vn_size(uint32_t v)
{
    uint32_t k = 1;
    k += v >= 8u;
    k += v >= 72u;
    k += v >= 584u;
    k += v >= 4680u;
    k += v >= 37448u;
    k += v >= 299592u;
    k += v >= 2396744u;
    k += v >= 19173960u;
    k += v >= 153391688u;
    k += v >= 1227133512u;
    return k;
}

// A parse candidate side packed into one word: len | vn_size((off - 1) >> 8) << 28, the two
// things the cost model needs (parse.hip CandPacked); len < 3 (no factor) is kept alone. Only
// for blocks under 2^28 positions (len <= n).
constexpr uint32_t kPackLen = (1u << 28) - 1u;
__device__ __forceinline__ uint32_t pack_side(uint32_t off, uint32_t len)
{
    return len >= 3u ? (len & kPackLen) | vn_size((off - 1u) >> 8) << 28 : len & kPackLen;
}

// Index of slot s in a set kept as bits in slot order (ExitBits, internal.hpp): the set bits
// before s, from the word prefix counts wpre and s's word.
__device__ __forceinline__ uint32_t bits_index(const uint64_t *mask, const uint32_t *wpre, size_t s)
{
    const uint64_t m = mask[s >> 6];
    return wpre[s >> 6] + (uint32_t)__popcll(m & ((1ull << (s & 63u)) - 1ull));
}

// ---- batch geometry: several independent blocks encoded by one pipeline pass -------------
// The batch is the concatenation of nb blocks; block b occupies text positions
// [b*bs, b*bs + N_b) with N_b = bs for all but the last block. Its suffix text is the first
// n_b = N_b - 8 bytes (lib/salz.c:197); the 8 bytes after it are "dead" positions: no suffix
// starts there (they are the block's 8 trailing literals, :743-749), their rank is 0 (end of
// text) and the parse treats them as cost-0 ends. Suffix order is (block, suffix), so each
// block's range of the suffix array is that block's own suffix array. npos = end of the last
// block's suffix text = the position space; nsa = live suffixes = npos - 8 (nb - 1).
// One block: bs = 0xffffffff, so every position is in block 0 and end() = npos = n.
struct Blocks {
    uint32_t bs;    // block stride (bytes)
    uint32_t nb;    // blocks
    uint32_t npos;  // (nb - 1) * bs + N_last - 8
    __host__ __device__ __forceinline__ uint32_t blk(uint32_t p) const { return nb == 1 ? 0u : p / bs; }
    __host__ __device__ __forceinline__ uint32_t start(uint32_t p) const { return blk(p) * (nb == 1 ? 0u : bs); }
    // end of p's suffix text (exclusive); p >= end(p) means p is dead
    __host__ __device__ __forceinline__ uint32_t end(uint32_t p) const
    {
        const uint32_t b = blk(p);
        return b + 1u < nb ? b * bs + bs - 8u : npos;
    }
    __host__ __device__ __forceinline__ uint32_t nsa() const { return npos - 8u * (nb - 1u); }
    __host__ __device__ __forceinline__ uint32_t n_last() const { return npos - (nb - 1u) * (nb == 1 ? 0u : bs); }
};

// Round 0 of the suffix sorter lists every suffix once, in an order the stable LSD sort turns
// into "shorter suffix before a longer one it prefixes": first the suffixes with fewer than 8
// bytes left (length 1 of every block, then length 2, ... 7), then the rest in text order.
// List entry c -> its suffix. (One block: c < s -> n - 1 - c, else c - s.)
__host__ __device__ __forceinline__ uint32_t init_suffix(size_t c, const Blocks &g)
{
    if (g.nb == 1 && g.npos >= 7)  // (one block: the 7 short suffixes, then text order)
        return c < 7 ? g.npos - 1u - (uint32_t)c : (uint32_t)c - 7u;
    const uint32_t nl = g.n_last();
    const uint32_t full = g.nb - 1u;  // blocks with n_b = bs - 8 >= 7
    uint32_t cc = (uint32_t)c;
    for (uint32_t len = 1; len <= 7; len++) {
        const uint32_t cnt = full + (nl >= len ? 1u : 0u);
        if (cc < cnt)  // block cc's suffix with `len` bytes left
            return (cc < full ? cc * g.bs + g.bs - 8u : g.npos) - len;
        cc -= cnt;
    }
    const uint32_t per = g.nb == 1 ? 0u : g.bs - 15u;  // long suffixes of a full block
    if (g.nb > 1 && cc < full * per)
        return (cc / per) * g.bs + cc % per;
    return full * (g.nb == 1 ? 0u : g.bs) + (cc - full * per);
}

// Round-0 keys of the suffix sorter. Raw (bits == 0): the first 8 bytes, big-endian, bytes past
// the suffix's end zero (short suffixes are ordered by the initial list order). Alphabet
// (bits > 0): every byte mapped to its rank 1..sigma in the block's alphabet (order-preserving;
// 0 = past the end, below every symbol), k symbols of `bits` bits packed big-endian into the low
// k * bits bits: 7-bit text gives 9 symbols in 63 bits, a binary text 32 symbols (round 0 reaches
// depth 32). Symbols >= 1 are what lets round 1 be keyed by the text (sa.hip): a key padded with
// zeros past the end never equals a longer suffix's. Blocks of more than 127 distinct bytes keep
// raw keys.
struct Alpha {
    uint32_t bits;  // 0: raw bytes
    uint32_t k;     // symbols per key (the depth round 0 sorts to)
    uint8_t code[256];
};

// Unaligned little-endian 8-byte load from an 8-byte-aligned, padded byte buffer.
__device__ __forceinline__ uint64_t load_u64_any(const uint8_t *base, size_t pos)
{
    // Both words are loaded unconditionally (the buffer is padded): no exec-masked second
    // load, and the shift pair (b << 1) << (63 - sh) is 0 for sh == 0.
    const uint64_t *w = reinterpret_cast<const uint64_t *>(base + (pos & ~(size_t)7));
    const unsigned sh = (unsigned)(pos & 7) * 8u;
    const uint64_t a = w[0], b = w[1];
    return (a >> sh) | ((b << 1) << (63u - sh));
}

}  // namespace salz

namespace salz {

// Round-0 key of suffix i whose suffix text ends at e (see Alpha); `code` is the symbol table
// (a.code, or a copy in LDS: kernel-argument memory indexed per lane is slow).
__device__ __forceinline__ uint64_t round0_key(const uint8_t *T, uint32_t i, uint32_t e, const Alpha &a,
                                               const uint8_t *code)
{
    const uint32_t left = e - i;
    if (a.bits == 0) {
        uint64_t w = load_u64_any(T, i);
        if (left < 8)
            w &= (1ull << (8u * left)) - 1ull;
        return __builtin_bswap64(w);
    }
    uint64_t key = 0;
    for (uint32_t j0 = 0; j0 < a.k; j0 += 8) {
        const uint64_t w = load_u64_any(T, (size_t)i + j0);
        const uint32_t cnt = a.k - j0 < 8 ? a.k - j0 : 8u;
        for (uint32_t j = 0; j < cnt; j++) {
            const uint32_t c = j0 + j < left ? code[(w >> (8 * j)) & 255u] : 0u;
            key = (key << a.bits) | c;
        }
    }
    return key;
}

__device__ __forceinline__ uint64_t round0_key(const uint8_t *T, uint32_t i, uint32_t e, const Alpha &a)
{
    return round0_key(T, i, e, a, a.code);
}

// The same from the text already mapped to symbols (Tm[i] = a.code[T[i]], zero padded): no
// table lookups, just the packing (the radix passes that build round 0's keys use this).
__device__ __forceinline__ uint64_t round0_key_mapped(const uint8_t *Tm, uint32_t i, uint32_t e, const Alpha &a)
{
    const uint32_t left = e - i;
    uint64_t key = 0;
    if (a.k == 9) {  // the usual text case (7-bit symbols): straight-line, so the loads of a thread's items batch
        // the two aligned words holding Tm[i, i + 8): the second also holds Tm[i + 8]
        const uint64_t *wp = reinterpret_cast<const uint64_t *>(Tm + ((size_t)i & ~(size_t)7));
        const unsigned sh = (unsigned)(i & 7u) * 8u;
        const uint64_t w0 = wp[0], w1 = wp[1];
        uint64_t w = (w0 >> sh) | ((w1 << 1) << (63u - sh));
        if (left < 8)
            w &= (1ull << (8u * left)) - 1ull;
        // 8 symbols of `bits` bits (first symbol most significant), packed pairwise: byte pairs,
        // then 16-bit pairs, then the two halves (three mask-shift-or steps, not eight)
        const uint32_t b = a.bits;
        uint64_t x = __builtin_bswap64(w);
        x = (x & 0x00FF00FF00FF00FFull) | (((x >> 8) & 0x00FF00FF00FF00FFull) << b);
        x = (x & 0x0000FFFF0000FFFFull) | (((x >> 16) & 0x0000FFFF0000FFFFull) << (2 * b));
        x = (x & 0xFFFFFFFFull) | ((x >> 32) << (4 * b));
        const uint32_t s9 = (uint32_t)(w1 >> sh) & 255u;  // the ninth symbol, Tm[i + 8], zero past the end
        return (x << b) | (left > 8 ? s9 : 0u);
    }
    for (uint32_t j0 = 0; j0 < a.k; j0 += 8) {
        uint64_t w = load_u64_any(Tm, (size_t)i + j0);
        if (left < j0 + 8)
            w = left <= j0 ? 0ull : w & ((1ull << (8u * (left - j0))) - 1ull);
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
            if (j0 + j < a.k)
                key = (key << a.bits) | ((w >> (8 * j)) & 255u);
    }
    return key;
}

// Copy of the symbol table in LDS (every thread of the workgroup calls it, then a barrier).
__device__ __forceinline__ void load_codes(uint8_t *lds, const Alpha &a)
{
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x)
        lds[c] = a.code[c];
}

// Leading equal symbols of two round-0 keys (x = key_a ^ key_b, not both equal).
__device__ __forceinline__ uint32_t round0_lcp(uint64_t x, const Alpha &a)
{
    if (a.bits == 0)
        return x ? (uint32_t)__builtin_clzll(x) >> 3 : 8u;
    const uint32_t kb = a.k * a.bits;
    return x ? ((uint32_t)__builtin_clzll(x) - (64u - kb)) / a.bits : a.k;
}

}  // namespace salz
