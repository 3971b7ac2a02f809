// dc3.hip - suffix array by the difference cover modulo 3 (Kärkkäinen-Sanders skew) for
// highly repetitive blocks.
//
// Replaces libsais() at /root/reference/lib/salz.c:463-469 for inputs where prefix doubling
// (sa.hip) keeps almost every suffix unfinished for ~log2(max LCP) rounds: a Fibonacci word
// has only h + 1 distinct substrings of length h, so all 2^28 suffixes of the 256 MiB config
// stay in play for 26 full-width rounds. Here each level sorts the sample suffixes
// (i mod 3 != 0) by their first three symbols, names the triples, recurses on the 2/3-length
// string of names when names repeat, and merges the sorted sample with the mod-0 suffixes:
// the levels shrink by 2/3, so the whole sort costs about three times its first level.
//
// Per level (string t[0, n) of symbols >= 1, zero past the end; tools/dc3_sim.py models every
// step on the CPU):
//   k_dc3_sample_keys  sample j -> position p(j) (j < n1: 3j + 1, else 3(j - n1) + 2) and its
//                      triple key; n = 1 mod 3 adds a dummy sample at p = n (triple 000, the
//                      unique smallest name), so the names of the mod-1 part end in a unique
//                      symbol and comparisons of the name string never run into the mod-2 part
//   radix sort         (radix.hip) on the triple (or on two symbols, then stably on the first,
//                      when three do not fit 64 bits)
//   k_dc3_heads + scan names 1..D; D == n_sample means the sample is sorted already
//   k_dc3_names        the child's string R[j] = name (R = mod-1 names, then mod-2 names)
//   k_dc3_rank         rank[p] = 1 + sorted position of sample p (0 past the end)
//   k_dc3_mod0         mod-0 suffixes i = p - 1 for the mod-1 samples p in sorted order: the
//                      list is ordered by rank[i + 1], so a stable sort by t[i] sorts it
//   k_dc3_partition /  merge path over the two sorted lists: sample p against mod-0 i compares
//   k_dc3_merge        (t[i], rank[i + 1]) when p = 1 mod 3, (t[i], t[i + 1], rank[i + 2]) when
//                      p = 2 mod 3; 2048 outputs per workgroup, merged in LDS
// Symbols and ranks of a level are interleaved (TR[q] = {t[q], rank[q]}), so the merge's
// comparison operands of one suffix are one 24-byte run.
#include "internal.hpp"
#include "scatter.hpp"

#include <cstdlib>
#include <cstring>

namespace salz {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ uint32_t dc3_pos(uint32_t j, uint32_t n1)
{
    return j < n1 ? 3u * j + 1u : 3u * (j - n1) + 2u;
}

// Level 0: the block's bytes as symbols 1..sigma (order-preserving codes) or byte + 1.
__global__ void k_dc3_text(const uint8_t *__restrict__ T, uint32_t n, Alpha a, int raw, uint2 *__restrict__ tr)
{
    __shared__ uint8_t code[256];
    load_codes(code, a);
    __syncthreads();
    for (size_t q = (size_t)blockIdx.x * kT + threadIdx.x; q < (size_t)n + 8; q += (size_t)gridDim.x * kT) {
        const uint32_t c = q < n ? T[q] : 0u;
        tr[q] = make_uint2(q < n ? (raw ? c + 1u : (uint32_t)code[c]) : 0u, 0u);
    }
}

// Sample keys: full (t[p] << 2b | t[p+1] << b | t[p+2]) or, when 3b > 64, the last two symbols.
__global__ void k_dc3_sample_keys(const uint2 *__restrict__ tr, uint32_t ns, uint32_t n1, int b, int full,
                                  uint64_t *__restrict__ key, uint32_t *__restrict__ val)
{
    const size_t j = (size_t)blockIdx.x * kT + threadIdx.x;
    if (j >= ns)
        return;
    const uint32_t p = dc3_pos((uint32_t)j, n1);
    const uint64_t t0 = tr[p].x, t1 = tr[p + 1].x, t2 = tr[p + 2].x;
    key[j] = full ? (t0 << (2 * b)) | (t1 << b) | t2 : (t1 << b) | t2;
    val[j] = (uint32_t)j;
}

// Second phase of a split triple sort: key = first symbol << 32 | the name of the (second, third)
// pair in the sample sorted by those two (pn: 1 + the distinct pairs below, coalesced), so the
// stable sort on the first symbol leaves every triple's full identity in its key and the names
// come from comparing neighbouring keys (before, k_dc3_heads read both neighbours' triples from
// TR: two random 24-byte runs per sample).
__global__ void k_dc3_first_keys(const uint2 *__restrict__ tr, const uint32_t *__restrict__ val,
                                 const uint32_t *__restrict__ pn, uint32_t ns, uint32_t n1, uint64_t *__restrict__ key)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= ns)
        return;
    key[c] = (uint64_t)tr[dc3_pos(val[c], n1)].x << 32 | pn[c];
}

// Levels whose triples fit kLutMaxBits bits (up to 9 bits a symbol: Fibonacci's first seven
// levels, byte texts' first) are named without sorting: the names are the ranks of the distinct
// triples, so a presence bitmap of the triple keys and its prefix counts give every sample its
// name in sample order, written coalesced into the child string (no radix sort of the sample, no
// name scatter). The sample's sorted order then comes from the child's suffix array, as it does
// after a sort whenever names repeat; a level whose names are all distinct (D = ns) takes the
// sorting path for that order. Bitmaps of up to kLutBits bits are built in LDS per workgroup.
constexpr int kLutBits = 18;
constexpr uint32_t kLutWords = 1u << (kLutBits - 5);
constexpr int kLutMaxBits = 27;  // (9-bit symbols: blocks of all 256 byte values)

__device__ __forceinline__ uint32_t triple_key(const uint2 *__restrict__ tr, uint32_t j, uint32_t n1, int b)
{
    const uint32_t p = dc3_pos(j, n1);
    return (tr[p].x << (2 * b)) | (tr[p + 1].x << b) | tr[p + 2].x;
}

// Presence bits of the sample's triple keys: per workgroup in LDS (a bit is read before it is
// set, so a level with few distinct triples sets each one once per workgroup), then OR'd into
// the global bitmap.
__global__ __launch_bounds__(kT) void k_dc3_presence(const uint2 *__restrict__ tr, uint32_t ns, uint32_t n1, int b,
                                                     uint32_t nwords, uint32_t *__restrict__ bits,
                                                     uint32_t *__restrict__ keys)
{
    __shared__ uint32_t sb[kLutWords];
    for (uint32_t i = threadIdx.x; i < nwords; i += kT)
        sb[i] = 0;
    __syncthreads();
    for (size_t j = (size_t)blockIdx.x * kT + threadIdx.x; j < ns; j += (size_t)gridDim.x * kT) {
        const uint32_t key = triple_key(tr, (uint32_t)j, n1, b), w = key >> 5, m = 1u << (key & 31u);
        keys[j] = key;
        if (!(sb[w] & m))
            atomicOr(&sb[w], m);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nwords; i += kT)
        if (sb[i])
            atomicOr(&bits[i], sb[i]);
}

// The same into a global bitmap of up to 2^kLutMaxBits bits (read before set), whose words'
// popcounts then feed the prefix scan. A grid of at most
// kPresenceGrid workgroups loops over the sample, and each workgroup remembers the keys it set in a
// direct-mapped LDS filter: a periodic block has few distinct triples, and every sample testing and
// setting the same global word (one workgroup per 256 samples) serialised on it (zeros at 256 MiB:
// 8.8 ms for one level).
constexpr uint32_t kPresenceGrid = 2048;
constexpr uint32_t kFilter = 2048;
__global__ __launch_bounds__(kT) void k_dc3_presence_global(const uint2 *__restrict__ tr, uint32_t ns, uint32_t n1,
                                                            int b, uint32_t *__restrict__ bits,
                                                            uint32_t *__restrict__ keys)
{
    __shared__ uint32_t filt[kFilter];
    for (uint32_t k = threadIdx.x; k < kFilter; k += kT)
        filt[k] = 0xffffffffu;  // (no triple key: keys have at most kLutMaxBits bits)
    __syncthreads();
    for (size_t j = (size_t)blockIdx.x * kT + threadIdx.x; j < ns; j += (size_t)gridDim.x * kT) {
        const uint32_t key = triple_key(tr, (uint32_t)j, n1, b), w = key >> 5, m = 1u << (key & 31u);
        keys[j] = key;
        const uint32_t h = (key * 0x9E3779B1u) >> 21;  // (kFilter = 2^11 slots)
        bool todo = filt[h] != key;  // (not set by this workgroup yet)
        // Up to four distinct keys of the wave go through one lane each: in the first pass of the
        // grid every workgroup's filter is empty, and all lanes of a periodic block (one key)
        // reached the same global word (2048 x 256 atomics on one address; zeros at 256 MiB:
        // 4.4 ms for one level)
        uint64_t pend = wave_ballot(todo);
        for (int it = 0; it < 4 && pend; it++) {
            const int ld = (int)__ffsll((unsigned long long)pend) - 1;
            const uint32_t k0 = shfl_u32(key, ld);
            const bool same = todo && key == k0;
            pend &= ~wave_ballot(same);
            if (same && (int)lane_id() != ld)
                todo = false;
        }
        if (!todo)
            continue;
        filt[h] = key;  // (racing lanes may both store; either way the bit is set below)
        if (!(bits[w] & m))  // (a stale cached 0 only costs a redundant atomic)
            atomicOr(&bits[w], m);
    }
}

__global__ void k_dc3_popc(const uint32_t *__restrict__ bits, uint32_t nwords, uint32_t *__restrict__ cnt)
{
    const uint32_t w = blockIdx.x * kT + threadIdx.x;
    if (w < nwords)
        cnt[w] = (uint32_t)__popc(bits[w]);
}

// Exclusive prefix popcounts of the bitmap words (one workgroup, 8 words a thread) and D.
__global__ __launch_bounds__(1024) void k_dc3_lut_scan(const uint32_t *__restrict__ bits, uint32_t nwords,
                                                       uint32_t *__restrict__ pre, uint32_t *__restrict__ D)
{
    static_assert(kLutWords == 1024 * 8, "8 words a thread");
    __shared__ uint32_t wsum[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t c[8], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t w = 8 * tid + k;
        c[k] = w < nwords ? (uint32_t)__popc(bits[w]) : 0u;
        sum += c[k];
    }
    uint32_t x = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = shfl_up_u32(x, d);
        if (lane >= d)
            x += y;
    }
    if (lane == 63)
        wsum[wave] = x;
    __syncthreads();
    uint32_t run = x - sum, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
        run += w < wave ? wsum[w] : 0u;
        all += wsum[w];
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t w = 8 * tid + k;
        if (w < nwords)
            pre[w] = run;
        run += c[k];
    }
    if (tid == 0)
        *D = all;
}

// The child's string in sample order: R[j] = 1 + the distinct triples below j's (keys: the triple
// keys the presence pass wrote in sample order, 4 bytes a sample instead of three 8-byte TR reads).
__global__ void k_dc3_names_lut(const uint32_t *__restrict__ keys, uint32_t ns, const uint32_t *__restrict__ bits,
                                const uint32_t *__restrict__ pre, uint2 *__restrict__ child)
{
    const size_t j = (size_t)blockIdx.x * kT + threadIdx.x;
    if (j >= ns)
        return;
    const uint32_t key = keys[j], w = key >> 5;
    child[j] = make_uint2(1u + pre[w] + (uint32_t)__popc(bits[w] & ((1u << (key & 31u)) - 1u)), 0u);
}

// Name boundaries of the sorted sample: a new key (triple, or first symbol and pair name) starts
// a new name.
__global__ void k_dc3_heads(const uint64_t *__restrict__ key, uint32_t ns, uint32_t *__restrict__ flag)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= ns)
        return;
    const size_t cp = c ? c - 1 : 0;  // unconditional loads (clamped)
    flag[c] = c == 0 || key[c] != key[cp] ? 1u : 0u;
}

// The child's string: R[j] = name of sample j (rank part zero).
__global__ void k_dc3_names(const uint32_t *__restrict__ val, const uint32_t *__restrict__ name, uint32_t ns,
                            uint2 *__restrict__ child)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= ns)
        return;
    child[val[c]] = make_uint2(name[c], 0u);
}

// rank[p] = 1 + sorted position of sample p; the dummy (p = n) keeps rank 0.
__global__ void k_dc3_rank(const uint32_t *__restrict__ sar, uint32_t ns, uint32_t n1, uint32_t n,
                           uint2 *__restrict__ tr, uint32_t *err)
{
    const size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r >= ns)
        return;
    const uint32_t j = sar[r];
    if (bad_index(j >= ns, err, kErrDc3))
        return;
    const uint32_t p = dc3_pos(j, n1);
    if (p < n)
        tr[p].y = (uint32_t)r + 1u;
}

// The same two scatters for scatter_staged (scatter.hpp): TR as u32 words, index = position.
struct RankSrc {
    const uint32_t *sar;
    uint32_t ns, n1, n;
    __device__ __forceinline__ bool operator()(size_t r, uint32_t &idx, uint32_t &val) const
    {
        const uint32_t j = sar[r];
        idx = dc3_pos(j, n1);
        val = (uint32_t)r + 1u;
        return j < ns && idx < n;
    }
};

struct NameSrc {
    const uint32_t *v, *name;
    uint32_t ns;
    __device__ __forceinline__ bool operator()(size_t c, uint32_t &idx, uint32_t &val) const
    {
        idx = v[c];
        val = name[c];
        return idx < ns;
    }
};

__global__ void k_dc3_mod0_flags(const uint32_t *__restrict__ sar, uint32_t ns, uint32_t n1,
                                 uint32_t *__restrict__ flag)
{
    const size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r < ns)
        flag[r] = sar[r] < n1 ? 1u : 0u;
}

// Mod-0 suffixes in rank[i + 1] order (the dummy stands for i = n - 1), keyed by t[i]. With a
// packing (symbols of at most 8 bits, and rank and position fields that leave room for t[i + 1])
// the rest of the merge's comparison operands of i ride along, read from the same TR run as t[i],
// so the merge reads no TR for them: key = t[i] | rank[i + 1] << 8 | rank[i + 2] << (8 + R) |
// t[i + 1]'s high bits << (8 + 2R) (the sort's one 8-bit digit is t[i] alone), value = i | t[i + 1]'s
// low bits << P. (Round 6: up to 8-bit symbols with fields sized per level, was 4 bits with 28-bit
// fields: Fibonacci's levels 3-5 pack too.)
struct Pack {
    uint32_t R, P;  // rank bits, position bits; R = 0: not packed
};

__device__ __forceinline__ uint64_t pack_key(uint2 x0, uint2 x1, uint2 x2, Pack k)
{
    const uint32_t hs = 8u + 2u * k.R;
    const uint64_t hi = hs < 64u ? (uint64_t)(x1.x >> (32u - k.P)) << hs : 0ull;
    return x0.x | ((uint64_t)x1.y << 8) | ((uint64_t)x2.y << (8u + k.R)) | hi;
}

__global__ void k_dc3_mod0(const uint32_t *__restrict__ sar, const uint32_t *__restrict__ idx, uint32_t ns,
                           uint32_t n1, uint32_t n0, const uint2 *__restrict__ tr, uint64_t *__restrict__ key,
                           uint32_t *__restrict__ val, uint32_t *err, Pack pk)
{
    const size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r >= ns)
        return;
    const uint32_t j = sar[r];
    if (j >= n1)
        return;
    const uint32_t c = idx[r], i = 3u * j;
    if (bad_index(c >= n0, err, kErrDc3))
        return;
    if (pk.R) {
        const uint2 x0 = tr[i], x1 = tr[i + 1], x2 = tr[i + 2];
        key[c] = pack_key(x0, x1, x2, pk);
        val[c] = i | (x1.x << pk.P);
    } else {
        key[c] = tr[i].x;
        val[c] = i;
    }
}

// ---- merge of the sorted sample (A) and the sorted mod-0 suffixes (B) ----------------------
struct Quad {
    uint32_t t0, t1, r1, r2;  // t[p], t[p + 1], rank[p + 1], rank[p + 2]
};

__device__ __forceinline__ Quad quad_of(const uint2 *__restrict__ tr, uint32_t p)
{
    const uint2 a = tr[p], b = tr[p + 1], c = tr[p + 2];
    return Quad{a.x, b.x, b.y, c.y};
}

// Mod-0 suffix b before sample suffix a (a at a position = am mod 3)? Never equal.
__device__ __forceinline__ bool b_before_a(const Quad &b, const Quad &a, uint32_t am)
{
    if (b.t0 != a.t0)
        return b.t0 < a.t0;
    if (am == 1)
        return b.r1 < a.r1;
    if (b.t1 != a.t1)
        return b.t1 < a.t1;
    return b.r2 < a.r2;
}

constexpr int kMergeItems = 8;
constexpr uint32_t kMergeTile = kT * kMergeItems;

struct MergeIn {
    const uint32_t *sar;  // sorted sample as child indices (A = sar[dummy ..])
    uint32_t na, dummy, n1;
    const uint32_t *posb;  // sorted mod-0 positions (B)
    uint32_t nb;
    const uint2 *tr;
    const uint64_t *keyb;  // B's sorted keys: when packed, their operands (k_dc3_mod0)
    Pack pk;
};

// Position and comparison operands of B element k (sorted mod-0 index)
__device__ __forceinline__ uint32_t b_pos(const MergeIn &m, uint32_t k)
{
    return m.pk.R ? m.posb[k] & ((1u << m.pk.P) - 1u) : m.posb[k];
}

__device__ __forceinline__ Quad b_quad(const MergeIn &m, uint32_t k)
{
    if (!m.pk.R)
        return quad_of(m.tr, m.posb[k]);
    const uint64_t x = m.keyb[k];
    const uint32_t R = m.pk.R, P = m.pk.P, hs = 8u + 2u * R, rmask = (1u << R) - 1u;
    const uint32_t hi = hs < 64u ? (uint32_t)(x >> hs) << (32u - P) : 0u;
    return Quad{(uint32_t)x & 255u, (m.posb[k] >> P) | hi, (uint32_t)(x >> 8) & rmask,
                (uint32_t)(x >> (8u + R)) & rmask};
}

__device__ __forceinline__ uint32_t a_pos(const MergeIn &m, uint32_t r)
{
    return dc3_pos(m.sar[r + m.dummy], m.n1);
}

// A elements among the first `diag` outputs of every tile boundary (merge path, A first on ties
// -- there are none).
__global__ void k_dc3_partition(MergeIn m, uint32_t ntiles, uint32_t *__restrict__ split)
{
    const size_t t = (size_t)blockIdx.x * kT + threadIdx.x;
    if (t > ntiles)
        return;
    const uint64_t tot = (uint64_t)m.na + m.nb;
    const uint32_t diag = (uint32_t)((uint64_t)t * kMergeTile < tot ? (uint64_t)t * kMergeTile : tot);
    uint32_t lo = diag > m.nb ? diag - m.nb : 0u, hi = diag < m.na ? diag : m.na;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t pa = a_pos(m, mid);
        if (b_before_a(b_quad(m, diag - 1u - mid), quad_of(m.tr, pa), pa % 3u))
            hi = mid;
        else
            lo = mid + 1u;
    }
    split[t] = lo;
}

__global__ __launch_bounds__(kT) void k_dc3_merge(MergeIn m, const uint32_t *__restrict__ split,
                                                  uint32_t *__restrict__ out)
{
    __shared__ Quad sq[kMergeTile];
    __shared__ uint32_t sp[kMergeTile];
    const uint32_t tid = threadIdx.x, t = blockIdx.x;
    const uint64_t tot = (uint64_t)m.na + m.nb;
    const uint32_t d0 = t * kMergeTile;
    const uint32_t d1 = (uint32_t)((uint64_t)d0 + kMergeTile < tot ? (uint64_t)d0 + kMergeTile : tot);
    const uint32_t a0 = split[t], a1 = split[t + 1];
    const uint32_t b0 = d0 - a0, b1 = d1 - a1;
    const uint32_t na = a1 - a0, cnt = d1 - d0;
    // A run then B run, each element's position and comparison operands
    for (uint32_t s = tid; s < cnt; s += kT) {
        const uint32_t p = s < na ? a_pos(m, a0 + s) : b_pos(m, b0 + (s - na));
        sp[s] = p;
        sq[s] = s < na ? quad_of(m.tr, p) : b_quad(m, b0 + (s - na));
    }
    __syncthreads();
    const uint32_t nb = b1 - b0;
    const uint32_t diag = tid * kMergeItems < cnt ? tid * kMergeItems : cnt;
    uint32_t lo = diag > nb ? diag - nb : 0u, hi = diag < na ? diag : na;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (b_before_a(sq[na + diag - 1u - mid], sq[mid], sp[mid] % 3u))
            hi = mid;
        else
            lo = mid + 1u;
    }
    uint32_t ia = lo, ib = diag - lo;
    uint32_t res[kMergeItems];
#pragma unroll
    for (int k = 0; k < kMergeItems; k++) {
        bool take_a;
        if (ia >= na)
            take_a = false;
        else if (ib >= nb)
            take_a = true;
        else
            take_a = !b_before_a(sq[na + ib], sq[ia], sp[ia] % 3u);
        const uint32_t s = take_a ? ia : na + ib;
        res[k] = sp[s < cnt ? s : 0];
        ia += take_a ? 1u : 0u;
        ib += take_a ? 0u : 1u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMergeItems; k++)
        if (diag + k < cnt)
            sp[diag + k] = res[k];
    __syncthreads();
    for (uint32_t s = tid; s < cnt; s += kT)
        out[d0 + s] = sp[s];
}

struct Dc3 {
    Workspace &ws;
    hipStream_t st;
    uint8_t *top;  // arena bump pointer
    uint8_t *end;
    uint32_t *derr;
    int levels = 0;
};

template <typename T> static T *arena_take(Dc3 &d, size_t count)
{
    uint8_t *p = d.top;
    const size_t bytes = (count * sizeof(T) + 255) & ~(size_t)255;
    if (p + bytes > d.end)
        return nullptr;
    d.top += bytes;
    return reinterpret_cast<T *>(p);
}

// Suffix array of the level string tr[0, n) (symbols < 2^b, tail zero) into sa_out.
int dc3_level(Dc3 &d, uint2 *tr, uint32_t n, int b, uint32_t *sa_out)
{
    Workspace &ws = d.ws;
    hipStream_t st = d.st;
    d.levels++;
    if (n == 1) {
        SALZ_HIP(fill_async(sa_out, 0, sizeof(uint32_t), st));
        return 0;
    }
    const uint32_t dummy = n % 3u == 1u ? 1u : 0u;
    const uint32_t n1 = (n + 1u) / 3u + dummy, n2 = n / 3u, ns = n1 + n2, n0 = (n + 2u) / 3u;
    uint32_t *d32 = reinterpret_cast<uint32_t *>(ws.dscal) + 300;
    uint64_t *K = ws.keyA;
    uint32_t *V = ws.valA;
    const bool full = 3 * b <= 64;
    uint8_t *mark = d.top;
    uint32_t *sar = nullptr;
    // Naming by the triples' presence bitmap where they fit kLutMaxBits; wider triples (and a
    // level whose names are all distinct) sort below.
    const uint32_t nwords = 3 * b <= kLutMaxBits ? ((1u << (3 * b)) + 31u) / 32u : 0u;
    const size_t lut_room = nwords > kLutWords ? 2 * (size_t)nwords : 2 * (size_t)kLutWords;
    if (nwords && ws.radix_counts_elems >= lut_room) {
        uint32_t *bits = ws.radix_counts, *pre = bits + (lut_room / 2);
        uint32_t *tkeys = reinterpret_cast<uint32_t *>(ws.keyA);  // (free until the mod-0 sort)
        SALZ_HIP(fill_async(bits, 0, sizeof(uint32_t) * nwords, st));
        if (nwords <= kLutWords) {
            const uint32_t g = grid_for(ns, kT) < 2048u ? grid_for(ns, kT) : 2048u;
            hipLaunchKernelGGL(k_dc3_presence, dim3(g), dim3(kT), 0, st, tr, ns, n1, b, nwords, bits, tkeys);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_dc3_lut_scan, dim3(1), dim3(1024), 0, st, bits, nwords, pre, d32);
            SALZ_LAUNCH_CHECK();
        } else {
            hipLaunchKernelGGL(k_dc3_presence_global,
                               dim3(grid_for(ns, kT) < kPresenceGrid ? grid_for(ns, kT) : kPresenceGrid), dim3(kT), 0,
                               st, tr, ns, n1, b, bits, tkeys);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_dc3_popc, dim3(grid_for(nwords, kT)), dim3(kT), 0, st, bits, nwords, pre);
            SALZ_LAUNCH_CHECK();
            if (scan_sum_u32(pre, pre, nwords, false, d32, ws, st) != 0)
                return -1;
        }
        if (read_scalars(ws, 1200, 8, "dc3.D") != 0)
            return -1;
        const uint32_t D = reinterpret_cast<const uint32_t *>(ws.hscal)[300];
        if (D < ns) {
            uint2 *child = arena_take<uint2>(d, (size_t)ns + 8);
            sar = arena_take<uint32_t>(d, ns);
            if (!child || !sar) {
                set_error("dc3: arena exhausted at level %d (n=%u)", d.levels, n);
                return -1;
            }
            SALZ_HIP(fill_async(child + ns, 0, 8 * sizeof(uint2), st));
            hipLaunchKernelGGL(k_dc3_names_lut, dim3(grid_for(ns, kT)), dim3(kT), 0, st, tkeys, ns, bits, pre, child);
            SALZ_LAUNCH_CHECK();
            if (dc3_level(d, child, ns, bit_width(D), sar) != 0)
                return -1;
        }
    }
    uint32_t *flag = ws.u0, *name = ws.u1;
    // the radix passes' digit bytes (u16 for 9-bit digits) in u3, free during DC3: each pass's
    // histogram reads them instead of the 8-byte keys; 9-bit digits wherever they save a pass
    uint8_t *rdig = reinterpret_cast<uint8_t *>(ws.u3);
    if (!sar) {
        hipLaunchKernelGGL(k_dc3_sample_keys, dim3(grid_for(ns, kT)), dim3(kT), 0, st, tr, ns, n1, b, full ? 1 : 0, K,
                           V);
        SALZ_LAUNCH_CHECK();
        if (radix_sort_pairs(&K, &V, K == ws.keyA ? ws.keyB : ws.keyA, V == ws.valA ? ws.valB : ws.valA, ns, 0,
                             full ? 3 * b : 2 * b, ws, st, nullptr, nullptr, nullptr, rdig, false, true) != 0)
            return -1;
        if (!full) {  // names of the (second, third) pairs, then the stable sort on the first symbol
            hipLaunchKernelGGL(k_dc3_heads, dim3(grid_for(ns, kT)), dim3(kT), 0, st, K, ns, flag);
            SALZ_LAUNCH_CHECK();
            if (scan_sum_u32(flag, name, ns, true, nullptr, ws, st) != 0)
                return -1;
            hipLaunchKernelGGL(k_dc3_first_keys, dim3(grid_for(ns, kT)), dim3(kT), 0, st, tr, V, name, ns, n1, K);
            SALZ_LAUNCH_CHECK();
            if (radix_sort_pairs(&K, &V, K == ws.keyA ? ws.keyB : ws.keyA, V == ws.valA ? ws.valB : ws.valA, ns, 32,
                                 32 + b, ws, st, nullptr, nullptr, nullptr, rdig, false, true) != 0)
                return -1;
        }
        hipLaunchKernelGGL(k_dc3_heads, dim3(grid_for(ns, kT)), dim3(kT), 0, st, K, ns, flag);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(flag, name, ns, true, d32, ws, st) != 0)
            return -1;
        if (read_scalars(ws, 1200, 8, "dc3.D") != 0)
            return -1;
        const uint32_t D = reinterpret_cast<const uint32_t *>(ws.hscal)[300];
        if (D < ns) {
            uint2 *child = arena_take<uint2>(d, (size_t)ns + 8);
            sar = arena_take<uint32_t>(d, ns);
            if (!child || !sar) {
                set_error("dc3: arena exhausted at level %d (n=%u)", d.levels, n);
                return -1;
            }
            if (scatter_stage_wanted((size_t)ns * sizeof(uint2))) {  // x = name, y = 0
                SALZ_HIP(fill_async(child, 0, ((size_t)ns + 8) * sizeof(uint2), st));
                if (scatter_staged(NameSrc{V, name, ns}, ns, ns, reinterpret_cast<uint32_t *>(child), 2u, 0u,
                                   reinterpret_cast<uint2 *>(ws.lsc), 2 * ws.cap_s, ws.radix_counts, st) != 0)
                    return -1;
            } else {
                SALZ_HIP(fill_async(child + ns, 0, 8 * sizeof(uint2), st));
                hipLaunchKernelGGL(k_dc3_names, dim3(grid_for(ns, kT)), dim3(kT), 0, st, V, name, ns, child);
                SALZ_LAUNCH_CHECK();
            }
            if (dc3_level(d, child, ns, bit_width(D), sar) != 0)
                return -1;
        } else {
            sar = ws.u2;  // the sorted sample is the order (survives the mod-0 sort below)
            SALZ_HIP(hipMemcpyAsync(sar, V, (size_t)ns * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        }
    }
    if (scatter_stage_wanted((size_t)n * sizeof(uint2))) {
        if (scatter_staged(RankSrc{sar, ns, n1, n}, ns, n, reinterpret_cast<uint32_t *>(tr), 2u, 1u,
                           reinterpret_cast<uint2 *>(ws.lsc), 2 * ws.cap_s, ws.radix_counts, st) != 0)
            return -1;
    } else {
        hipLaunchKernelGGL(k_dc3_rank, dim3(grid_for(ns, kT)), dim3(kT), 0, st, sar, ns, n1, n, tr, d.derr);
        SALZ_LAUNCH_CHECK();
    }
    // mod-0 list, then its stable sort by t[i]
    hipLaunchKernelGGL(k_dc3_mod0_flags, dim3(grid_for(ns, kT)), dim3(kT), 0, st, sar, ns, n1, flag);
    SALZ_LAUNCH_CHECK();
    if (scan_sum_u32(flag, name, ns, false, d32 + 1, ws, st) != 0)
        return -1;
    K = ws.keyA;
    V = ws.valA;
    // (symbols of more than 8 bits, or fields too wide for t[i + 1]: unpacked keys, the merge
    // reading every operand from TR)
    Pack pk{(uint32_t)bit_width(ns), (uint32_t)bit_width(n)};
    if (b > 8 || pk.P > 31 || 8 + 2 * pk.R > 64 || (64 - 8 - 2 * pk.R) + (32 - pk.P) < (uint32_t)b)
        pk = Pack{0u, 0u};
    hipLaunchKernelGGL(k_dc3_mod0, dim3(grid_for(ns, kT)), dim3(kT), 0, st, sar, name, ns, n1, n0, tr, K, V,
                       d.derr, pk);
    SALZ_LAUNCH_CHECK();
    if (radix_sort_pairs(&K, &V, ws.keyB, ws.valB, n0, 0, b, ws, st, nullptr, nullptr, nullptr, rdig, false, true) !=
        0)
        return -1;
    // merge
    MergeIn mi{sar, ns - dummy, dummy, n1, V, n0, tr, K, pk};
    const uint32_t ntiles = grid_for(n, kMergeTile);
    uint32_t *split = ws.offA;
    hipLaunchKernelGGL(k_dc3_partition, dim3(grid_for((size_t)ntiles + 1, kT)), dim3(kT), 0, st, mi, ntiles, split);
    SALZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_dc3_merge, dim3(ntiles), dim3(kT), 0, st, mi, split, sa_out);
    SALZ_LAUNCH_CHECK();
    d.top = mark;  // the child's string and suffix array are consumed
    return 0;
}

}  // namespace

// Arena bytes for a block of n suffixes: level 0's TR plus, for every deeper level, its TR and
// suffix array (the string lengths shrink to ceil(2n / 3) + 1 per level).
static size_t dc3_arena_bytes(uint32_t n)
{
    size_t bytes = (((size_t)n + 8) * 8 + 255) & ~(size_t)255;
    uint64_t m = n;
    while (m > 1) {
        const uint64_t dm = m % 3 == 1 ? 1 : 0;
        m = (m + 1) / 3 + dm + m / 3;
        bytes += (((m + 8) * 8 + 255) & ~(size_t)255) + ((m * 4 + 255) & ~(size_t)255);
    }
    return bytes + 4096;
}

uint8_t *dc3_arena_reserve(Workspace &ws, size_t need)
{
    if (ws.dc3_bytes < need) {
        if (ws.dc3 && hipFree(ws.dc3) != hipSuccess) {
            set_error("dc3: hipFree of the arena failed");
            return nullptr;
        }
        ws.bytes -= ws.dc3_bytes;
        ws.dc3 = nullptr;
        ws.dc3_bytes = 0;
        void *p = nullptr;
        if (hipMalloc(&p, need) != hipSuccess) {
            set_error("dc3: hipMalloc of %zu bytes failed", need);
            return nullptr;
        }
        ws.dc3 = static_cast<uint8_t *>(p);
        ws.dc3_bytes = need;
        ws.bytes += need;
    }
    return ws.dc3;
}

int stage_suffix_array_dc3(Workspace &ws, const Blocks &bl, const Alpha &codes, int raw)
{
    hipStream_t st = ws.stream;
    const uint32_t n = bl.npos;
    if (bl.nb != 1) {
        set_error("dc3: one block per pass only");
        return -1;
    }
    if (!dc3_arena_reserve(ws, dc3_arena_bytes(n)))
        return -1;
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    Dc3 d{ws, st, ws.dc3, ws.dc3 + ws.dc3_bytes, derr};
    uint2 *tr = arena_take<uint2>(d, (size_t)n + 8);
    const unsigned g = grid_for((size_t)n + 8, kT) < 8192u ? grid_for((size_t)n + 8, kT) : 8192u;
    hipLaunchKernelGGL(k_dc3_text, dim3(g), dim3(kT), 0, st, ws.text, n, codes, raw, tr);
    SALZ_LAUNCH_CHECK();
    uint32_t sigma = 0;
    for (int c = 0; c < 256; c++)
        sigma = codes.code[c] > sigma ? codes.code[c] : sigma;
    const int b = raw ? 9 : bit_width(sigma);
    if (dc3_level(d, tr, n, b, ws.sa) != 0)
        return -1;
    if (read_scalars(ws, 0, 256, "dc3.err") != 0)
        return -1;
    if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
        set_error("dc3 suffix sort: device index check failed (code 0x%x)", e);
        return -1;
    }
    ws.stats.sa_dc3_levels = d.levels;
    ws.lcps_ok = false;  // the LCP array comes from the Phi/PLCP stage (lcp.hip)
    return 0;
}

}  // namespace salz
