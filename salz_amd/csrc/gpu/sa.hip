// sa.hip - suffix array of T[0,n) by prefix doubling with finished-group pruning.
//
// Replaces libsais() at /root/reference/lib/salz.c:463-469. The SA of a text is unique,
// so the result is identical to libsais's; ordering follows libsais's convention (no
// sentinel byte: a suffix sorts before every longer suffix it is a prefix of).
//
// Round 0 sorts all suffixes by their first 8 bytes (big-endian packed u64 key). Suffixes
// with fewer than 8 bytes left are fed first, shortest first, so the stable LSD sort puts
// each of them before the longer suffixes it prefixes; they are always singleton groups.
// Round t >= 1 sorts the still-unfinished suffixes by (group, rank[i + h]) with h = 8*2^(t-1);
// the key holds only the bits that can vary (compact group id | rank bits).
//
// rank[i] = 1 + SA position of the head of i's group; rank[n] = 0 (end of text sorts first).
// Per round:
//   sort        round 0: global LSD radix sort of all suffixes. Later rounds: the active
//               list is already grouped, so only each group's members need ordering by
//               rank[i + h]. Small groups (<= kSmall members) are sorted inside LDS, one
//               workgroup per 2048-entry window of the list (k_seg_small, one HBM read and
//               write); large groups are extracted, radix-sorted on (large-group id, rank)
//               and put back (k_extract / k_putback). Ties may land in any order: equal keys
//               stay one group, so the next round re-sorts them.
//   k_heads_lcp group-head flags of the sorted active list (one 64-bit ballot per wave), and
//               the LCP of every new head with its predecessor (see the comment there; k_heads
//               once the LCP is left to the Phi/PLCP stage)
//   scan        of the per-wave head counts; k_headpos -> group ids and head index per group
//   k_surv      groups of size >= 2 survive: per wave of the list, the survivor entries and the
//               survivor heads as bit masks (from the head ballots alone: a head whose successor
//               is a head too is a singleton); their counts are scanned, so an entry's compact
//               index and new group id are prefix + popcount (large groups take their ids and
//               extraction ranges with one atomic per group in k_commit)
//   k_commit    rank update for every active suffix (in large rounds staged by text range
//               and applied window by window: scatter_staged), SA write for
//               singletons, compaction
//   k_keys      next round's keys: gid << kb | rank[i + h]
#include "internal.hpp"
#include "scatter.hpp"

#include <chrono>
#include <cstdlib>
#include <cstring>

namespace salz {
namespace {

constexpr int kT = 256;
__device__ __forceinline__ uint32_t umin_(uint32_t a, uint32_t b) { return a < b ? a : b; }
constexpr uint32_t kSegT = 2048;     // window of the active list per k_seg_small workgroup
constexpr uint32_t kSmall = kSegT;   // largest group sorted in LDS (must be <= kSegT)
constexpr uint32_t kSegCap = 4096;   // LDS slots: a window's groups span < kSegT + kSmall
constexpr int kSegThreads = 256;
static_assert(kSegCap == 4096, "12-bit slot index in the LDS sort key");

// Round 0's (key, value) list in init_suffix order. Tm: the text mapped to symbols (alphabet
// keys), else the raw text is read. dig: the first radix pass's digit of every key (its low
// byte), so that pass's histogram reads bytes (radix.hip).
__global__ void k_sa_init(const uint8_t *__restrict__ T, const uint8_t *__restrict__ Tm, Blocks g, Alpha a,
                          uint64_t *__restrict__ key, uint32_t *__restrict__ val, uint8_t *__restrict__ dig)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= g.nsa())
        return;
    const uint32_t i = init_suffix(c, g);
    const uint64_t k = Tm ? round0_key_mapped(Tm, i, g.end(i), a) : round0_key(T, i, g.end(i), a);
    key[c] = k;
    val[c] = i;
    if (dig)
        dig[c] = (uint8_t)k;
}

// Round-0 pairs of a split block's own suffixes (list order: short ones first, shortest first,
// then text order).
__global__ void k_list_init(const uint8_t *__restrict__ T, const uint32_t *__restrict__ list, uint32_t m,
                            uint32_t n, Alpha a, uint64_t *__restrict__ key, uint32_t *__restrict__ val)
{
    __shared__ uint8_t code[256];
    load_codes(code, a);
    __syncthreads();
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint32_t i = list[c];
    key[c] = round0_key(T, i, n, a, code);
    val[c] = i;
}

// Tm[i] = symbol of T[i] (and 64 zero bytes of padding past P), for round0_key_mapped.
__global__ void k_map_text(const uint8_t *__restrict__ T, size_t P, Alpha a, uint8_t *__restrict__ Tm)
{
    __shared__ uint8_t code[256];
    load_codes(code, a);
    __syncthreads();
    for (size_t i = ((size_t)blockIdx.x * kT + threadIdx.x) * 16; i < P + 64; i += (size_t)gridDim.x * kT * 16) {
        // 16 bytes per thread in one load and one store (the text buffer is padded past P + 64)
        const uint4 x = *reinterpret_cast<const uint4 *>(T + i);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const size_t at = i + 4 * q + b;
                v |= (at < P ? (uint32_t)code[(w[q] >> (8 * b)) & 255u] : 0u) << (8 * b);
            }
            o[q] = v;
        }
        *reinterpret_cast<uint4 *>(Tm + i) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// Byte presence of the text (the alphabet for round 0's keys): 8 words of 32 bits.
__global__ void k_alpha_presence(const uint8_t *__restrict__ T, size_t P, uint32_t *__restrict__ words)
{
    __shared__ uint32_t w[8];
    if (threadIdx.x < 8)
        w[threadIdx.x] = 0;
    __syncthreads();
    // 16 bytes per thread and step (one load); bits already present are not written again
    for (size_t i = ((size_t)blockIdx.x * kT + threadIdx.x) * 16; i < P; i += (size_t)gridDim.x * kT * 16) {
        const uint4 x = *reinterpret_cast<const uint4 *>(T + i);  // (padded buffer)
        const uint32_t v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const uint32_t c = (v[b >> 2] >> (8 * (b & 3))) & 255u;
            if (i + b < P && !(w[c >> 5] & (1u << (c & 31))))
                atomicOr(&w[c >> 5], 1u << (c & 31));
        }
    }
    __syncthreads();
    if (threadIdx.x < 8 && w[threadIdx.x])
        atomicOr(&words[threadIdx.x], w[threadIdx.x]);
}

// Repetition probe. A suffix is still unfinished at depth 32 iff its first 32 bytes occur at
// another position too, so the share of sampled 32-grams that occur twice anywhere in the block
// estimates the share of suffixes that doubling would still carry at depth 32, which is what
// the depth-32 switch to DC3 tests (stage_suffix_array). Two steps:
//   k_repeat_probe (one workgroup) fingerprints 512 evenly spaced sample points, each as the eight
//     32-grams at q, q + 1, .., q + 7, into an open-addressing table (8192 slots: a 30-bit tag << 2
//     per slot, and how many samples share it). Samples that collide with each other (Fibonacci,
//     periodic blocks: every 32-gram repeats within a few samples) decide at once.
//   k_repeat_scan fingerprints the 32-gram at every position p = 0 mod 8 (aligned words: no byte
//     shifts) and counts the table slots it hits; k_repeat_count calls a point repeated when one of
//     its eight grams occurs at an aligned position other than its own. A copy of the point at any
//     distance d puts exactly one of its eight grams (q + i + d = 0 mod 8) on an aligned position,
//     so this finds repeats at any distance: a text repeated once at distance n / 2, or runs of one
//     byte, where the evenly spaced samples never meet (round 4 sent those to DC3 only at depth 32,
//     after three full-width rounds).
// The fingerprint of the 32 bytes from their four little-endian words: an xor of rotated words
// (full-rate operations), then 32-bit multiplies for the table slot, the filter bit and the 30-bit
// tag. A collision only makes a 32-gram look repeated.
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t gram_fp(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3)
{
    const uint64_t f = w0 ^ rotl64(w1, 19) ^ rotl64(w2, 38) ^ rotl64(w3, 57);
    return f ^ (f >> 29);
}
constexpr uint32_t kProbePoints = 512;
constexpr uint32_t kProbe = 8 * kProbePoints;  // sampled grams
constexpr uint32_t kProbeThreads = 1024;
constexpr uint32_t kProbeSlots = 8192;    // open addressing, at most half full
constexpr uint32_t kFilterBits = 65536;  // one bit per 16-bit fingerprint prefix of a sample (6% set)
__device__ __forceinline__ uint32_t gram_mix(uint64_t h) { return (uint32_t)h * 0x9E3779B1u; }
__device__ __forceinline__ uint32_t gram_slot(uint32_t mx) { return mx >> 19; }
__device__ __forceinline__ uint32_t gram_fbit(uint32_t mx) { return mx >> 16; }
__device__ __forceinline__ uint32_t gram_tag(uint64_t h) { return (((uint32_t)(h >> 32) * 0x85EBCA77u) | 4u) & ~3u; }

// ptab: the table's tags (0 = empty), pmul: samples per slot, gcnt: aligned occurrences (zeroed here
// for the scan), pfilt: the samples' filter bits, pslot: every sample's slot (<< 1 | its own position
// is aligned). out[0]: samples that share their fingerprint with another sample.
__global__ __launch_bounds__(kProbeThreads) void k_repeat_probe(const uint8_t *__restrict__ T, uint32_t n,
                                                                uint32_t *__restrict__ out, uint32_t *__restrict__ ptab,
                                                                uint32_t *__restrict__ pmul, uint32_t *__restrict__ gcnt,
                                                                uint32_t *__restrict__ pfilt, uint32_t *__restrict__ pslot,
                                                                uint32_t *__restrict__ hpos)
{
    __shared__ uint32_t key[kProbeSlots];
    __shared__ uint32_t cnt[kProbeSlots];
    __shared__ uint32_t filt[kFilterBits / 32];
    __shared__ uint32_t dups;
    constexpr uint32_t kPerT = kProbe / kProbeThreads;
    const uint32_t tid = threadIdx.x;
    if (tid == 0)
        dups = 0;
    for (uint32_t i = tid; i < kProbeSlots; i += kProbeThreads) {
        key[i] = 0;
        cnt[i] = 0;
    }
    for (uint32_t i = tid; i < kFilterBits / 32; i += kProbeThreads)
        filt[i] = 0;
    uint64_t w[kPerT][4];  // every sample's loads issued first
    size_t pos[kPerT];
#pragma unroll
    for (uint32_t j = 0; j < kPerT; j++) {
        const uint32_t s = tid + j * kProbeThreads;  // sample s: point s / 8, gram s % 8
        pos[j] = (size_t)(s >> 3) * (n - 40u) / kProbePoints + (s & 7u);
#pragma unroll
        for (int q = 0; q < 4; q++)
            w[j][q] = load_u64_any(T, pos[j] + 8u * q);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPerT; j++) {
        const uint64_t h = gram_fp(w[j][0], w[j][1], w[j][2], w[j][3]);
        const uint32_t tag = gram_tag(h), mx = gram_mix(h);
        uint32_t slot = gram_slot(mx);
        atomicOr(&filt[gram_fbit(mx) >> 5], 1u << (gram_fbit(mx) & 31u));
        for (uint32_t probe = 0; probe < kProbeSlots; probe++) {  // (the table never fills)
            const uint32_t old = atomicCAS(&key[slot], 0u, tag);
            if (old == 0u || old == tag) {
                atomicAdd(&cnt[slot], 1u);
                break;
            }
            slot = (slot + 1u) & (kProbeSlots - 1u);
        }
        if (ptab)
            pslot[tid + j * kProbeThreads] = slot << 1 | ((pos[j] & 7u) == 0u ? 1u : 0u);
    }
    __syncthreads();
    uint32_t d = 0;
    for (uint32_t i = tid; i < kProbeSlots; i += kProbeThreads) {
        d += cnt[i] >= 2u ? cnt[i] : 0u;
        if (ptab) {
            ptab[i] = key[i];
            pmul[i] = cnt[i];
            gcnt[i] = 0u;
            hpos[i] = 0xffffffffu;  // lowest and highest aligned hit (k_repeat_scan)
            hpos[kProbeSlots + i] = 0u;
        }
    }
    if (ptab)
        for (uint32_t i = tid; i < kFilterBits / 32; i += kProbeThreads)
            pfilt[i] = filt[i];
    atomicAdd(&dups, d);
    __syncthreads();
    if (tid == 0)
        *out = dups;
}

// The 32-gram at every position p = 0 mod 8 against the sample table (skipped when the samples
// decided already: dups[0] * 2 >= kProbe). A thread takes 8 such positions from 11 aligned text
// words; a gram whose filter bit is clear (94% of text) goes no further. Hits count per workgroup
// in LDS (saturating at 2), then once per slot into gcnt.
constexpr uint32_t kScanThreads = 256;
__global__ __launch_bounds__(kScanThreads) void k_repeat_scan(const uint8_t *__restrict__ T, uint32_t n,
                                                              const uint32_t *__restrict__ dups,
                                                              const uint32_t *__restrict__ ptab,
                                                              const uint32_t *__restrict__ pfilt,
                                                              uint32_t *__restrict__ gcnt, uint32_t *__restrict__ hpos)
{
    __shared__ uint32_t tab[kProbeSlots];  // tag | hits in this workgroup (2 bits, saturating)
    __shared__ uint32_t filt[kFilterBits / 32];
    if (dups[0] * 2u >= kProbe)
        return;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kProbeSlots; i += kScanThreads)
        tab[i] = ptab[i];
    for (uint32_t i = tid; i < kFilterBits / 32; i += kScanThreads)
        filt[i] = pfilt[i];
    __syncthreads();
    const uint32_t lastw = (n - 32u) / 8u;  // aligned grams: word indices 0..lastw
    const uint64_t *W = reinterpret_cast<const uint64_t *>(T);
    for (size_t g = (size_t)blockIdx.x * kScanThreads + tid; g * 8 <= lastw; g += (size_t)gridDim.x * kScanThreads) {
        uint64_t x[11];  // (the text buffer is padded past N + 64)
#pragma unroll
        for (int q = 0; q < 11; q++)
            x[q] = W[g * 8 + q];
        uint32_t cand = 0;  // grams whose filter bit is set
        uint64_t hs[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            hs[j] = gram_fp(x[j], x[j + 1], x[j + 2], x[j + 3]);
            const uint32_t fb = gram_fbit(gram_mix(hs[j]));
            cand |= ((filt[fb >> 5] >> (fb & 31u)) & 1u) << j;
        }
        if (g * 8 + 7 > lastw)
            cand &= (1u << (lastw - g * 8 + 1)) - 1u;
        while (cand) {
            const uint32_t j = __builtin_ctz(cand);
            cand &= cand - 1u;
            const uint64_t h = hs[j];
            const uint32_t tag = gram_tag(h);
            uint32_t slot = gram_slot(gram_mix(h));
            for (;;) {
                const uint32_t e = tab[slot];
                if (e == 0u)
                    break;
                if ((e & ~3u) == tag) {  // bit 0: hit once, bit 1: hit twice (or-ed, so never past 3)
                    // the first two hits per workgroup also leave their positions (lowest and
                    // highest over the grid): a gram with one aligned copy besides its own has
                    // both recorded, for the twin distance (k_repeat_count)
                    bool rec = false;
                    if (!(e & 2u)) {
                        rec = !(atomicOr(&tab[slot], 1u) & 1u);
                        if (!rec)
                            rec = !(atomicOr(&tab[slot], 2u) & 2u);
                    }
                    if (rec) {
                        const uint32_t p = (uint32_t)(g * 8 + j) * 8u;
                        atomicMin(&hpos[slot], p);
                        atomicMax(&hpos[kProbeSlots + slot], p);
                    }
                    break;
                }
                slot = (slot + 1u) & (kProbeSlots - 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < kProbeSlots; i += kScanThreads) {
        const uint32_t c = (tab[i] & 1u) + ((tab[i] >> 1) & 1u);
        if (c)
            atomicAdd(&gcnt[i], c);
    }
}

// out[0]: the sample points (of kProbePoints) one of whose grams occurs at an aligned position
// other than its own, or is shared with another sample. out[1], out[2]: the twin distance d most
// points share and how many do. A point's twin distance is that of its first gram that no other
// sample shares and that has exactly one aligned copy besides its own (a block holding a text
// twice, at distance d: every point but those in the text's own repeats).
__global__ __launch_bounds__(kProbePoints) void k_repeat_count(const uint32_t *__restrict__ dups,
                                                               const uint32_t *__restrict__ pmul,
                                                               const uint32_t *__restrict__ gcnt,
                                                               const uint32_t *__restrict__ pslot,
                                                               const uint32_t *__restrict__ hpos, uint32_t n,
                                                               uint32_t *__restrict__ out)
{
    __shared__ uint32_t tot;
    __shared__ uint32_t dist[kProbePoints];
    __shared__ unsigned long long best;
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        tot = 0;
        best = 0;
    }
    bool rep = false;
    uint32_t dd = 0;
    if (dups[0] * 2u < kProbe)
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t e = pslot[t * 8u + i], sl = e >> 1, own = e & 1u;
            rep = rep || pmul[sl] >= 2u || gcnt[sl] >= 1u + own;
            if (!dd && pmul[sl] == 1u && gcnt[sl] == 1u + own) {
                const uint32_t q = (uint32_t)((size_t)t * (n - 40u) / kProbePoints) + i;
                const uint32_t lo = hpos[sl], hi = hpos[kProbeSlots + sl];
                const uint32_t other = own && lo == q ? hi : lo;
                dd = other > q ? other - q : q - other;
            }
        }
    dist[t] = dd;
    __syncthreads();
    const uint64_t b = wave_ballot(rep);
    if (lane_id() == 0)
        atomicAdd(&tot, (uint32_t)__popcll(b));
    if (dd) {
        uint32_t same = 0;
        for (uint32_t u = 0; u < kProbePoints; u++)
            same += dist[u] == dd ? 1u : 0u;
        atomicMax(&best, (unsigned long long)same << 32 | dd);
    }
    __syncthreads();
    if (t == 0) {
        out[0] = tot;
        out[1] = (uint32_t)best;
        out[2] = (uint32_t)(best >> 32);
    }
}

// Group-head flags travel as one 64-bit ballot per wave of the sorted list (hmask) plus its
// popcount (wcnt): the group ids are then a scan over m / 64 wave counts, not over m flags.
struct HeadBits {
    uint64_t *hmask;  // ceil(m / 64) words
    uint32_t *wcnt;   // ceil(m / 64) per-wave head counts
    uint32_t *wpre;   // their exclusive scan
};

__device__ __forceinline__ void put_heads(HeadBits hb, size_t c, uint32_t m, bool head)
{
    const uint64_t mask = wave_ballot(head);
    if ((c & 63u) == 0 && c < m) {  // waves wholly past the list's end own no word
        hb.hmask[c >> 6] = mask;
        hb.wcnt[c >> 6] = (uint32_t)__popcll(mask);
    }
}

__global__ void k_heads(const uint64_t *__restrict__ key, const uint32_t *__restrict__ val,
                        uint32_t m, Blocks bl, uint32_t h0, int round0, HeadBits hb)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if ((c & ~(size_t)63) >= m)
        return;  // whole wave past the end
    // every load unconditional (clamped indices): no exec-masked load next to another
    const bool in = c < m;
    const size_t cc = in ? c : 0, cp = cc ? cc - 1 : 0;
    const uint64_t k0 = key[cp], k1 = key[cc];
    const uint32_t v0 = val[cp], v1 = val[cc];
    bool h = cc == 0 || k0 != k1;
    if (round0 && !h)  // short suffixes are singletons; a batch's blocks never share a group
        h = (bl.end(v1) - v1) < h0 || (bl.end(v0) - v0) < h0 || bl.blk(v0) != bl.blk(v1);
    put_heads(hb, c, m, in && h);
}

// Group id + 1 of list entry c (the inclusive head count), from the per-wave head ballots
// (one word per 64 entries: every lane of a wave reads the same two).
__device__ __forceinline__ uint32_t gid1(const HeadBits &hb, size_t c, uint32_t &bit)
{
    const uint64_t mask = hb.hmask[c >> 6];
    const uint32_t lane = (uint32_t)(c & 63u);
    bit = (uint32_t)(mask >> lane) & 1u;
    return hb.wpre[c >> 6] + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull)) + bit;
}

// Head position per group (plus the sentinel headpos[G] = m).
// A wave takes kHpWords words of the list (lane l: entry 64 w + l of each), so a quarter of the
// waves per launch; every word's loads are issued before its stores.
constexpr uint32_t kHpWords = 4;
__global__ void k_headpos(HeadBits hb, uint32_t m, uint32_t *__restrict__ headpos)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const size_t w0 = (x >> 6) * kHpWords;
    const uint32_t lane = (uint32_t)(x & 63u);
    const size_t nw = ((size_t)m + 63) / 64;
    uint64_t mk[kHpWords];
    uint32_t pre[kHpWords];
#pragma unroll
    for (uint32_t k = 0; k < kHpWords; k++) {  // unconditional loads (clamped word)
        const size_t w = w0 + k < nw ? w0 + k : nw - 1;
        mk[k] = hb.hmask[w];
        pre[k] = hb.wpre[w];
    }
#pragma unroll
    for (uint32_t k = 0; k < kHpWords; k++) {
        const size_t c = (w0 + k) * 64 + lane;
        if (c >= m)
            break;
        const uint32_t bit = (uint32_t)(mk[k] >> lane) & 1u;
        const uint32_t g = pre[k] + (uint32_t)__popcll(mk[k] & ((1ull << lane) - 1ull)) + bit;
        if (bit)
            headpos[g - 1u] = (uint32_t)c;
        if (c == m - 1)
            headpos[g] = m;
    }
}

// Survivor masks of wave word w of the list (entries 64w .. 64w + 63): entry c is in a
// singleton group iff it is a head and so is c + 1 (or c is the last entry). se: entries of
// groups of size >= 2; sh: heads of those groups. All loads unconditional (clamped word).
__device__ __forceinline__ void surv_masks(const HeadBits &hb, size_t w, uint32_t m, uint64_t &se, uint64_t &sh)
{
    const size_t nw = ((size_t)m + 63) / 64;
    const bool more = w + 1 < nw;
    const uint64_t h = hb.hmask[w], hn = hb.hmask[more ? w + 1 : w];
    uint64_t nh = (h >> 1) | (more ? (hn & 1ull) << 63 : 0ull);
    const uint64_t left = (uint64_t)m - (uint64_t)w * 64;  // >= 1
    const uint64_t valid = left >= 64 ? ~0ull : (1ull << left) - 1ull;
    if (left <= 64)
        nh |= 1ull << (left - 1);  // the last entry's successor is past the list
    se = valid & ~(h & nh);
    sh = valid & h & ~nh;
}

// Per wave word: (survivor entries << 32 | survivor heads); k_commit reads their exclusive scan.
__global__ __launch_bounds__(kT) void k_surv(HeadBits hb, uint32_t m, uint64_t *__restrict__ P,
                                             uint64_t *__restrict__ lcount)
{
    const size_t w = (size_t)blockIdx.x * kT + threadIdx.x;
    if (w < 2)  // k_commit's large-group counters (lcount[0..1]), zeroed for its atomics
        lcount[w] = 0;
    if (w >= ((size_t)m + 63) / 64)
        return;
    uint64_t se, sh;
    surv_masks(hb, w, m, se, sh);
    P[w] = ((uint64_t)__popcll(se) << 32) | (uint64_t)__popcll(sh);
}

// Next round's group table (ginfo: size << 32 | compact start) is written by each surviving
// group's head; large groups also get their extraction record.
struct GroupTab {
    uint64_t *ginfo;
    uint64_t *lrec;
    uint32_t *lg2g;
};

// Round 0 before a text round: the survivors' text-round keys are written with their compacted
// entries (the symbols at i + h0, k_keys_text's gather done here), when `key` is set.
struct TextNext {
    const uint8_t *Tm;
    uint64_t *key;
    Blocks bl;
    Alpha a;
    uint32_t h0;
};

// gin: the text round (round 1 keyed by text, below): entry c's group id, which its key no
// longer holds; every rank is written there (no entry keeps one: round 0 wrote no survivor's).
// surv_rank = 0: round 0 before a text round writes only the ranks of the suffixes it finishes.
__global__ void k_commit(const uint64_t *__restrict__ key, const uint32_t *__restrict__ val,
                         HeadBits hb, const uint32_t *__restrict__ headpos,
                         const uint64_t *__restrict__ P, unsigned long long *__restrict__ lcount,
                         const uint32_t *__restrict__ off_old, uint32_t *__restrict__ off_new,
                         uint32_t *__restrict__ nval, uint32_t *__restrict__ ngid,
                         uint32_t *__restrict__ rank, uint32_t *__restrict__ sa, GroupTab tab,
                         uint32_t m, uint32_t n, uint32_t nsa, int kb_old, int round0, uint32_t *err,
                         uint32_t ihi, uint32_t *__restrict__ later, uint32_t gbase,
                         const uint32_t *__restrict__ gin, int surv_rank, TextNext tn)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    uint32_t bit;
    const uint32_t g = gid1(hb, c, bit) - 1u;
    uint32_t hp = headpos[g];
    uint32_t size = headpos[g + 1] - hp;
    uint32_t o = round0 ? 0u : off_old[gin ? gin[c] : (uint32_t)(key[c] >> kb_old)];
    uint32_t i = val[c];
    if (bad_index(i >= n || c + o >= nsa || hp > c || size > m, err, kErrCommit))
        return;
    // The first subgroup of an old group keeps the old group's head, so its members' ranks
    // are unchanged; every other rank (and all of round 0 and the text round) is written.
    const bool same = !round0 && !gin && (hp == 0 || (key[hp - 1] >> kb_old) != (key[hp] >> kb_old));
    const uint32_t slot = c + o, rpos = hp + o;  // SA slot (singletons); rank = group head's + 1
    // rank[i] is a random 4-byte scatter (a read-modify-write of a whole HBM burst). Large
    // rounds write only the ranks of i < ihi here and leave every update in list order in
    // `later` for the split passes (k_rank_upper) or the staged scatter (scatter_staged); small
    // ones write rank directly (ihi = ~0, no `later`). The entry that keeps its old head's
    // place keeps its rank.
    const bool keep = (same && rpos == hp + o) || (!surv_rank && size > 1);
    const uint32_t rv = keep ? 0xffffffffu : gbase + rpos + 1u;  // (gbase: a split block's bucket)
    if (!keep && i < ihi)
        rank[i] = rv;
    if (later)
        later[c] = rv;
    if (size == 1) {
        sa[slot] = i;
    } else {
        // compact index = survivor entries before c, new group id = survivor heads up to c - 1
        uint64_t se, sh;
        surv_masks(hb, c >> 6, m, se, sh);
        const uint64_t pw = P[c >> 6], below = (1ull << (c & 63u)) - 1ull;
        const uint32_t idx = (uint32_t)(pw >> 32) + (uint32_t)__popcll(se & below);
        const uint32_t ng = (uint32_t)pw + (uint32_t)__popcll(sh & (below | (below + 1ull))) - 1u;
        nval[idx] = i;
        ngid[idx] = ng;
        if (tn.key)
            tn.key[idx] = round0_key_mapped(tn.Tm, i + tn.h0, tn.bl.end(i), tn.a);
        if ((uint32_t)c == hp) {  // (idx is the group's compact start)
            off_new[ng] = hp + o - idx;
            tab.ginfo[ng] = ((uint64_t)size << 32) | idx;
            if (size > kSmall) {  // large-group id and extraction range (any order serves)
                const uint64_t l = atomicAdd(lcount, ((unsigned long long)size << 32) | 1ull);
                const uint32_t lg = (uint32_t)l;
                tab.lrec[lg] = (l & 0xffffffff00000000ull) | idx;
                tab.lg2g[lg] = ng;
                atomicAdd(lcount + 1, (unsigned long long)((size + kRadixTile - 1) / kRadixTile));  // its radix tiles
            }
        }
    }
}

// LCP as a by-product of the sort. Every SA position r >= 1 becomes a group head exactly once,
// in the round whose keys first tell SA[r-1] and SA[r] apart; all members of the two groups
// then share the same LCP, so the pair at the boundary gives LCP[r] for good:
//   round 0 (8-byte keys):   LCP = leading equal bytes of the two keys, capped by both lengths;
//   round t (keys compare rank[i + hk] within groups sharing hk bytes): LCP = hk + the equal
//   bytes of T[i + hk ..] and T[j + hk ..], fewer than hk. Up to kLcpLane bytes one lane
//   compares; longer compares take 8 lanes each, 128 bytes per step, 8 heads at a time.
// The host stops (and the PLCP stage takes over, lcp.hip) once hk exceeds kLcpMaxHk.
constexpr uint32_t kLcpLane = 32;
constexpr uint32_t kLcpMaxHk = 4096;

// k_heads with the LCP of every new head (writes the head ballots like k_heads).
// Twin mode (tw, twd: k_twin_pairs): a twin pair {x, x + d} that splits on the ranks of a twin pair
// resolved earlier shares far more than 2 hk symbols; its LCP is read from the twin table.
__global__ __launch_bounds__(kT) void k_heads_lcp(
    const uint64_t *__restrict__ K, const uint32_t *__restrict__ V, HeadBits hb,
    const uint32_t *__restrict__ off_old, uint32_t m, Blocks bl, Alpha a, int kb_old, uint32_t hk, int round0,
    const uint8_t *__restrict__ T, uint32_t *__restrict__ lcps, uint32_t *err, const uint32_t *__restrict__ tw,
    uint32_t twd)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    const bool in = c < m;
    // every load unconditional (clamped indices): no exec-masked load next to another
    const size_t cc = in ? c : 0, cp = cc ? cc - 1 : 0;
    const uint64_t k0 = K[cp], k1 = K[cc];
    const uint32_t v0 = V[cp], v1 = V[cc];
    bool head = c == 0 || k0 != k1;
    const uint32_t e1 = bl.end(v1);  // end of v1's suffix text (its block's)
    const bool other_block = bl.blk(v0) != bl.blk(v1);
    const uint32_t h0 = a.bits ? a.k : 8u;  // round 0's depth
    if (round0 && !head)
        head = (e1 - v1) < h0 || (bl.end(v0) - v0) < h0 || other_block;
    put_heads(hb, c, m, in && head);
    const uint32_t g1 = round0 ? 0u : (uint32_t)(k1 >> kb_old);
    const uint32_t o = round0 ? 0u : off_old[g1];
    const uint32_t i = v1, j = v0, mx = i > j ? i : j;
    bool need = false;
    uint32_t pos = 0, lim = 0;
    if (in && head) {
        if (round0) {
            uint32_t l = 0;
            if (c > 0 && !other_block) {  // a block's first suffix: LCP 0
                l = round0_lcp(k0 ^ k1, a);
                l = umin_(l, e1 - i);
                l = umin_(l, e1 - j);
            }
            lcps[c] = l;
        } else if (c > 0 && (uint32_t)(k0 >> kb_old) == g1) {
            pos = (uint32_t)c + o;
            // (same group, so the same block: e1 bounds both suffixes)
            if (!bad_index(i >= e1 || j >= e1 || pos >= bl.nsa() || e1 - mx < hk, err, kErrCommit)) {
                // (the keys differ, so the suffixes differ within hk bytes; lim bounds the
                // compare by the end of the text)
                lim = e1 - mx - hk;
                if (tw && mx - (i < j ? i : j) == twd) {
                    const uint32_t x = i < j ? i : j;
                    lcps[pos] = (tw[x] >> 1) - x;
                } else if (hk <= kLcpLane) {
                    uint32_t l = lim;
                    for (uint32_t off = 0; off < lim; off += 8) {
                        const uint64_t x = load_u64_any(T, (size_t)i + hk + off) ^
                                           load_u64_any(T, (size_t)j + hk + off);
                        if (x) {
                            l = umin_(lim, off + ((uint32_t)__builtin_ctzll(x) >> 3));
                            break;
                        }
                    }
                    lcps[pos] = hk + l;
                } else {
                    need = true;
                }
            }
        }
    }
    // Long compares: eight heads at a time, one per 8-lane group of the wave, 16 bytes per lane
    // and 128 per group and step (a head's compare is bounded by the LCP, so most end in the
    // first steps: the serial memory latencies per wave drop from one per head to about one per
    // eight). Loads past a head's limit read its first bytes again (every load unconditional).
    uint64_t pend = wave_ballot(need);
    const uint32_t lane = lane_id(), sub = lane >> 3, sl8 = lane & 7u;
    while (pend) {
        uint64_t pk = pend;  // group `sub` takes the sub-th pending head in lane order
        for (uint32_t u = 0; u < sub; u++)
            pk &= pk - 1;
        const bool have = pk != 0;
        const int src = have ? (int)__ffsll((unsigned long long)pk) - 1 : 0;
        for (uint32_t u = 0; u < 8; u++)
            pend &= pend - 1;
        const uint32_t si = shfl_u32(i, src) + hk, sj = shfl_u32(j, src) + hk;
        const uint32_t slv = shfl_u32(lim, src), sp = shfl_u32(pos, src);
        const uint32_t sl = have ? slv : 0u;
        uint32_t mis = 0xffffffffu;  // the group's first mismatch offset
        for (uint32_t base = 0;; base += 8 * 16) {
            const uint32_t off = base + sl8 * 16, offc = off < sl ? off : 0u;
            const uint64_t x0 = load_u64_any(T, (size_t)si + offc) ^ load_u64_any(T, (size_t)sj + offc);
            const uint64_t x1 = load_u64_any(T, (size_t)si + offc + 8) ^ load_u64_any(T, (size_t)sj + offc + 8);
            uint32_t mm = 0xffffffffu;
            if (off < sl && (x0 | x1))
                mm = x0 ? off + ((uint32_t)__builtin_ctzll(x0) >> 3) : off + 8u + ((uint32_t)__builtin_ctzll(x1) >> 3);
            mm = umin_(mm, shfl_xor_u32(mm, 1));
            mm = umin_(mm, shfl_xor_u32(mm, 2));
            mm = umin_(mm, shfl_xor_u32(mm, 4));
            if (mis == 0xffffffffu)
                mis = mm;
            const bool done = mis != 0xffffffffu || base + 8 * 16 >= sl;
            if (!wave_ballot(!done))
                break;
        }
        if (have && sl8 == 0)
            lcps[sp] = hk + umin_(mis, sl);
    }
}

// Twin pairs. A block that holds a text twice at distance d (the probe's twin distance) keeps
// every suffix x and its twin x + d in one group for ~log2(n / 2) rounds: their order and LCP are
// decided only by the first mismatch on diagonal d, j = min{j >= x : T[j] != T[j + d] or j + d = n},
// and the twin ends first when j + d = n (it is then a prefix of x's suffix). TW[x] = j << 1 | (x
// first) for x <= L = n - d, a suffix minimum of g[j] = that value at the mismatches and ~0
// elsewhere: per tile of kTwTile positions (k_twin_tiles), across tiles (k_twin_carry), then per
// position (k_twin_fill). Every round then splits the two-member groups {x, x + d} at once
// (k_twin_pairs), so the rounds carry what a text without its copy would.
constexpr uint32_t kTwItems = 16;
constexpr uint32_t kTwTile = kT * kTwItems;

__device__ __forceinline__ uint32_t twin_g(const uint8_t *__restrict__ T, uint32_t j, uint32_t d, uint32_t L)
{
    if (j > L)
        return 0xffffffffu;
    if (j == L)
        return j << 1;  // the twin ends: it sorts first
    const uint8_t a = T[j], b = T[j + d];
    return a != b ? (j << 1) | (a < b ? 1u : 0u) : 0xffffffffu;
}

// per thread: the suffix minimum over its kTwItems positions (written back into v)
__device__ __forceinline__ uint32_t twin_thread(const uint8_t *__restrict__ T, uint32_t x0, uint32_t d, uint32_t L,
                                                uint32_t *v)
{
    uint32_t mn = 0xffffffffu;
#pragma unroll
    for (int k = (int)kTwItems - 1; k >= 0; k--) {
        mn = umin_(mn, twin_g(T, x0 + (uint32_t)k, d, L));
        v[k] = mn;
    }
    return mn;
}

__global__ __launch_bounds__(kT) void k_twin_tiles(const uint8_t *__restrict__ T, uint32_t d, uint32_t L,
                                                   uint32_t *__restrict__ tmin)
{
    __shared__ uint32_t wm[kT / 64];
    uint32_t v[kTwItems];
    const uint32_t x0 = blockIdx.x * kTwTile + threadIdx.x * kTwItems;
    const uint32_t mn = wave_min_u32(twin_thread(T, x0, d, L, v));
    if (lane_id() == 0)
        wm[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0)
        tmin[blockIdx.x] = umin_(umin_(wm[0], wm[1]), umin_(wm[2], wm[3]));
}

// tmin[t] := the minimum over the tiles after t (one workgroup: a segment of tiles per thread)
constexpr uint32_t kTwCarryT = 1024;
__global__ __launch_bounds__(kTwCarryT) void k_twin_carry(uint32_t *__restrict__ tmin, uint32_t ntiles)
{
    __shared__ uint32_t seg[kTwCarryT];
    const uint32_t t = threadIdx.x, per = (ntiles + kTwCarryT - 1) / kTwCarryT;
    const uint32_t lo = t * per, hi = umin_(lo + per, ntiles);
    uint32_t mn = 0xffffffffu;
    for (uint32_t k = lo; k < hi; k++)
        mn = umin_(mn, tmin[k]);
    seg[t] = mn;
    __syncthreads();
    for (uint32_t s = 1; s < kTwCarryT; s <<= 1) {  // suffix minima of the segments
        const uint32_t o = t + s < kTwCarryT ? seg[t + s] : 0xffffffffu;
        __syncthreads();
        seg[t] = umin_(seg[t], o);
        __syncthreads();
    }
    uint32_t after = t + 1 < kTwCarryT ? seg[t + 1] : 0xffffffffu;
    for (uint32_t k = hi; k > lo; k--) {
        const uint32_t x = tmin[k - 1];
        tmin[k - 1] = after;
        after = umin_(after, x);
    }
}

__global__ __launch_bounds__(kT) void k_twin_fill(const uint8_t *__restrict__ T, uint32_t d, uint32_t L,
                                                  const uint32_t *__restrict__ tafter, uint32_t *__restrict__ tw)
{
    __shared__ uint32_t sm[kT];
    uint32_t v[kTwItems];
    const uint32_t tid = threadIdx.x, x0 = blockIdx.x * kTwTile + tid * kTwItems;
    sm[tid] = twin_thread(T, x0, d, L, v);
    __syncthreads();
    for (uint32_t s = 1; s < kT; s <<= 1) {  // suffix minima of the threads' minima
        const uint32_t o = tid + s < kT ? sm[tid + s] : 0xffffffffu;
        __syncthreads();
        sm[tid] = umin_(sm[tid], o);
        __syncthreads();
    }
    const uint32_t after = umin_(tid + 1 < kT ? sm[tid + 1] : 0xffffffffu, tafter[blockIdx.x]);
#pragma unroll
    for (uint32_t k = 0; k < kTwItems; k++)
        if (x0 + k <= L)
            tw[x0 + k] = umin_(v[k], after);
}

// Two-member groups {x, x + d} of the sorted list in order, split into singletons: a wave per
// 64-entry word of the head ballots (the heads of the word and the two after it are read before
// any is set; a pair's second entry, the new head, is followed by a head, so no other wave's pair
// test depends on it). With the sort's LCPs, the new head's LCP is j - x.
__global__ __launch_bounds__(kT) void k_twin_pairs(uint32_t *__restrict__ V, const uint64_t *__restrict__ K,
                                                   const uint32_t *__restrict__ gin, const uint32_t *__restrict__ off_old,
                                                   int kb_old, int round0, HeadBits hb, uint32_t m, uint32_t d,
                                                   const uint32_t *__restrict__ tw, uint32_t *__restrict__ lcps)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    const size_t w = c >> 6, nw = ((size_t)m + 63) / 64;
    if (w >= nw)
        return;  // whole wave
    const uint32_t lane = (uint32_t)(c & 63u);
    const uint64_t h = hb.hmask[w], hn = w + 1 < nw ? hb.hmask[w + 1] : 0ull;
    auto head = [&](size_t e) {
        if (e >= m)
            return true;
        const uint64_t wd = (e >> 6) == w ? h : hn;
        return ((wd >> (e & 63u)) & 1ull) != 0;
    };
    bool done = false;
    uint32_t lcp = 0;
    if (c + 1 < m && head(c) && !head(c + 1) && head(c + 2)) {
        const uint32_t a = V[c], b = V[c + 1];
        if ((a > b ? a - b : b - a) == d) {
            const uint32_t x = a < b ? a : b, v = tw[x];
            const uint32_t first = (v & 1u) ? x : x + d;
            if (a != first) {
                V[c] = first;
                V[c + 1] = a;
            }
            lcp = (v >> 1) - x;
            done = true;
        }
    }
    const uint64_t nb = wave_ballot(done);
    if (lane == 0 && nb) {
        const uint64_t in = nb << 1;  // the new heads at c + 1
        if (in) {
            atomicOr(reinterpret_cast<unsigned long long *>(&hb.hmask[w]), (unsigned long long)in);
            atomicAdd(&hb.wcnt[w], (uint32_t)__popcll(in));
        }
        if (nb >> 63) {
            atomicOr(reinterpret_cast<unsigned long long *>(&hb.hmask[w + 1]), 1ull);
            atomicAdd(&hb.wcnt[w + 1], 1u);
        }
    }
    if (lcps && done) {
        const uint32_t o = round0 ? 0u : off_old[gin ? gin[c] : (uint32_t)(K[c] >> kb_old)];
        lcps[(uint32_t)c + o + 1u] = lcp;
    }
}

// rank 0 (end of text) at a batch's dead positions: the 8 bytes after every block's suffix
// text but the last (the last block's end npos gets rank 0 from the host)
__global__ void k_dead_ranks(Blocks bl, uint32_t *__restrict__ rank)
{
    const uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= 8u * (bl.nb - 1u))
        return;
    const uint32_t b = x >> 3;
    rank[b * bl.bs + bl.bs - 8u + (x & 7u)] = 0u;
}

// Staged rank scatter (scatter.hpp): k_commit leaves the new ranks in list order (later[c],
// 0xffffffff when unchanged); scatter_staged bins them by text window and applies them window by
// window, XCD-aware.
struct LaterSrc {
    const uint32_t *val, *later;
    __device__ __forceinline__ bool operator()(size_t c, uint32_t &idx, uint32_t &v) const
    {
        idx = val[c];
        v = later[c];
        return v != 0xffffffffu;
    }
};

// Later passes of a split rank scatter: ranks of suffixes in [ilo, ihi), from k_commit's list.
__global__ void k_rank_upper(const uint32_t *__restrict__ val, const uint32_t *__restrict__ later,
                             uint32_t m, uint32_t ilo, uint32_t ihi, uint32_t *__restrict__ rank)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint32_t i = val[c], rv = later[c];
    if (i >= ilo && i < ihi && rv != 0xffffffffu)
        rank[i] = rv;
}

// Window plan of the LDS sort, one thread per surviving group (groups are in list order, so
// the groups that start in one window are consecutive ids): the first group starting in a
// window writes the window's lo and first group id, the last one its hi and last small group
// id. A large group can only be the last to start in its window (it runs past the window's
// end), so the owned small groups are [lo, hi) with hi = the large group's start in that case.
struct SegPlan {
    uint32_t *lo, *hi, *g0, *g1;
};

__global__ void k_seg_plan(const uint64_t *__restrict__ ginfo, uint32_t G, SegPlan plan)
{
    size_t g = (size_t)blockIdx.x * kT + threadIdx.x;
    if (g >= G)
        return;
    // unconditional loads (clamped neighbours)
    const uint64_t gi = ginfo[g], gp = ginfo[g ? g - 1 : 0], gn = ginfo[g + 1 < G ? g + 1 : g];
    const uint32_t size = (uint32_t)(gi >> 32), cs = (uint32_t)gi;
    const uint32_t w = cs / kSegT;
    if ((g == 0 || (uint32_t)gp / kSegT != w) && size <= kSmall) {
        plan.lo[w] = cs;
        plan.g0[w] = (uint32_t)g;
    }
    if (g + 1 == G || (uint32_t)gn / kSegT != w) {
        plan.hi[w] = size <= kSmall ? cs + size : cs;
        plan.g1[w] = size <= kSmall ? (uint32_t)g : (uint32_t)g - 1u;
    }
}

// Stable 8-bit LSD passes over bits [12, 12 + nbits) of ITEMS * 256 LDS keys; wave-striped:
// wave w owns slots [w * ITEMS * 64, (w + 1) * ITEMS * 64), item j covers 64 of them.
template <int ITEMS>
__device__ __forceinline__ void seg_lsd(uint64_t *sk, uint32_t (*cnt)[256], uint32_t *wsum, int nbits)
{
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    __syncthreads();
    for (int shift = 12; shift < 12 + nbits; shift += 8) {
        for (int i = tid; i < 4 * 256; i += kSegThreads)
            (&cnt[0][0])[i] = 0;
        __syncthreads();
        uint64_t k[ITEMS];
        uint32_t lrank[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            k[j] = sk[wave * (ITEMS * 64) + j * 64 + lane];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const unsigned d = (unsigned)(k[j] >> shift) & 255u;
            uint64_t peers = ~0ull;
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bb = wave_ballot(bit);
                peers &= bit ? bb : ~bb;
            }
            const unsigned below = count_below(peers);
            const int leader = (int)__ffsll((unsigned long long)peers) - 1;
            uint32_t old = 0;
            if ((int)lane == leader) {
                old = cnt[wave][d];
                cnt[wave][d] = old + (unsigned)__popcll(peers);
            }
            lrank[j] = shfl_u32(old, leader) + below;
        }
        __syncthreads();
        {
            const uint32_t c0 = cnt[0][tid], c1 = cnt[1][tid], c2 = cnt[2][tid], c3 = cnt[3][tid];
            const uint32_t tot = c0 + c1 + c2 + c3;
            uint32_t x = tot;
#pragma unroll
            for (unsigned dd = 1; dd < 64; dd <<= 1) {
                const uint32_t y = shfl_up_u32(x, dd);
                if (lane >= dd)
                    x += y;
            }
            if (lane == 63)
                wsum[wave] = x;
            __syncthreads();
            uint32_t pre = 0;
            for (unsigned w = 0; w < wave; w++)
                pre += wsum[w];
            const uint32_t ds = pre + x - tot;  // the digit's start; the waves' starts follow
            cnt[0][tid] = ds;
            cnt[1][tid] = ds + c0;
            cnt[2][tid] = ds + c0 + c1;
            cnt[3][tid] = ds + c0 + c1 + c2;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const unsigned d = (unsigned)(k[j] >> shift) & 255u;
            sk[cnt[wave][d] + lrank[j]] = k[j];
        }
        __syncthreads();
    }
}

// Groups of one window of the active list, sorted in LDS. The window owns every small group that
// starts in it (a group of <= kSmall members ends before the window's end + kSmall, and no large
// group can sit between two of them), so the owned range [lo, hi) has < kSegCap entries.
//   - A group of at most `tiny` members is ordered by counting: each entry's place is its group's
//     start plus the members with a smaller (key, window index).
//   - The members of the larger groups are gathered at the front of the LDS array and sorted by
//     (local group, key bits, window index) with stable 8-bit LSD passes; an entry's place is then
//     its group's start plus its sorted position minus the group's first sorted position (a
//     binary search: the groups stay contiguous in the sorted array).
// Rank rounds (TEXT = 0): key = group << kb | rank; the LSD passes take the kb rank bits. The
// text round (TEXT = 1, keys = kb text bits, groups in gin): the LSD passes take the top bits of
// the key that keep the sort at 48 bits (6 passes); the runs of equal (group, top bits) they leave
// are marked (rb, need) and ordered by the whole key in k_seg_text_fix.
constexpr uint32_t kPer = kSegCap / kSegThreads;

template <bool TEXT>
__global__ __launch_bounds__(kSegThreads) void k_seg_sort(uint64_t *__restrict__ K, uint32_t *__restrict__ V,
                                                          const uint32_t *__restrict__ gin, SegPlan plan,
                                                          const uint64_t *__restrict__ ginfo, uint32_t m, int kb,
                                                          uint32_t tiny, uint64_t *__restrict__ rb,
                                                          uint32_t *__restrict__ need, uint32_t *err, int lsd_bits)
{
    __shared__ uint64_t sk[kSegCap];  // the window's keys, then the larger groups' LSD keys
    __shared__ uint32_t sv[kSegCap];  // the window's values (by window index)
    __shared__ uint32_t cnt[4][256];  // LSD counters; after the LSD, runb
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t nbig;
    uint64_t *runb = reinterpret_cast<uint64_t *>(&cnt[0][0]);  // TEXT: run starts by window index
    static_assert(sizeof(cnt) >= kSegCap / 8, "LDS alias");

    const unsigned tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = blockIdx.x;
    const uint32_t lo = plan.lo[w];
    if (lo == 0xffffffffu)
        return;  // uniform: no small group starts in this window
    const uint32_t hi = plan.hi[w], g0 = plan.g0[w], g1 = plan.g1[w];
    if (bad_index(hi > m || hi <= lo || hi - lo >= kSegCap || g1 < g0, err, kErrSeg))
        return;
    const uint32_t count = hi - lo;
    const uint64_t mask = kb >= 64 ? ~0ull : (1ull << kb) - 1ull;
    const int gbits = 32 - __builtin_clz((g1 - g0) | 1u);
    const int kr = TEXT ? (kb < lsd_bits - gbits ? kb : lsd_bits - gbits) : kb;  // key bits in the LSD key
    if (tid == 0)
        nbig = 0;
    // the window into LDS: every load issued before the first is used (clamped, unconditional),
    // one memory latency instead of one per 256 entries
    {
        uint64_t wk[kPer];
        uint32_t wv[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t i = tid + j * kSegThreads, ii = i < count ? i : 0u;
            wk[j] = K[lo + ii];
            wv[j] = V[lo + ii];
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t i = tid + j * kSegThreads;
            if (i < count) {
                sk[i] = wk[j];
                sv[i] = wv[j];
            }
        }
    }
    __syncthreads();
    // counted groups: placed now; the larger groups' members: their LSD keys, collected
    uint64_t lk[kPer];
    bool big[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = tid + j * kSegThreads, ii = i < count ? i : 0u;
        const uint64_t ki = sk[ii];
        const uint32_t lg = (TEXT ? gin[lo + ii] : (uint32_t)(ki >> kb)) - g0;  // (unconditional loads)
        const uint64_t gi = ginfo[g0 + lg];
        uint32_t gs = (uint32_t)gi - lo, sz = (uint32_t)(gi >> 32);
        big[j] = false;
        if (i >= count)
            continue;
        if (bad_index(gs > i || gs + sz > count || sz > kSmall, err, kErrSeg)) {
            gs = i;  // (the error ends the sort)
            sz = 0;
        }
        if (sz <= tiny) {
            uint32_t r = 0;
            for (uint32_t x = gs; x < gs + sz; x++) {
                const uint64_t kx = sk[x];
                r += (kx < ki || (kx == ki && x < i)) ? 1u : 0u;
            }
            K[lo + gs + r] = ki;
            V[lo + gs + r] = sv[i];
        } else {
            big[j] = true;
            const uint64_t kbits = TEXT ? ki >> (kb - kr) : ki & mask;
            lk[j] = ((uint64_t)lg << (kr + 12)) | (kbits << 12) | i;
        }
    }
    __syncthreads();  // (the window's keys are no longer read from sk)
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint64_t bm = wave_ballot(big[j]);
        uint32_t base = 0;
        if (lane == 0 && bm)
            base = atomicAdd(&nbig, (uint32_t)__popcll(bm));
        base = shfl_u32(base, 0);
        if (big[j])
            sk[base + count_below(bm)] = lk[j];
    }
    __syncthreads();
    const uint32_t nb = nbig;
    if (nb == 0)
        return;
    const int items = (int)((nb + 255u) / 256u);
    for (uint32_t i = nb + tid; i < (uint32_t)items * kSegThreads; i += kSegThreads)
        sk[i] = ~0ull;  // padding sorts last in every digit
    const int nbits = gbits + kr;
    switch (items) {
    case 1: seg_lsd<1>(sk, cnt, wsum, nbits); break;
    case 2: seg_lsd<2>(sk, cnt, wsum, nbits); break;
    case 3: seg_lsd<3>(sk, cnt, wsum, nbits); break;
    case 4: seg_lsd<4>(sk, cnt, wsum, nbits); break;
    case 5: seg_lsd<5>(sk, cnt, wsum, nbits); break;
    case 6: seg_lsd<6>(sk, cnt, wsum, nbits); break;
    case 7: seg_lsd<7>(sk, cnt, wsum, nbits); break;
    case 8: seg_lsd<8>(sk, cnt, wsum, nbits); break;
    case 9: seg_lsd<9>(sk, cnt, wsum, nbits); break;
    case 10: seg_lsd<10>(sk, cnt, wsum, nbits); break;
    case 11: seg_lsd<11>(sk, cnt, wsum, nbits); break;
    case 12: seg_lsd<12>(sk, cnt, wsum, nbits); break;
    case 13: seg_lsd<13>(sk, cnt, wsum, nbits); break;
    case 14: seg_lsd<14>(sk, cnt, wsum, nbits); break;
    case 15: seg_lsd<15>(sk, cnt, wsum, nbits); break;
    default: seg_lsd<16>(sk, cnt, wsum, nbits); break;
    }
    if (TEXT) {  // (cnt is free again)
        for (uint32_t q = tid; q < kSegCap / 64; q += kSegThreads)
            runb[q] = ~0ull;
        __syncthreads();
    }
    uint64_t outk[kPer];
    uint32_t dst[kPer], vv[kPer];
    bool tie = false;
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t t = tid + j * kSegThreads;
        if (t >= nb)
            continue;
        const uint64_t key = sk[t];
        const uint32_t lg = (uint32_t)(key >> (kr + 12)), i = (uint32_t)key & 0xfffu;
        // the group's first sorted position: the first t' with local group lg
        uint32_t a = 0, z = t;
        while (a < z) {
            const uint32_t mid = (a + z) >> 1;
            if ((uint32_t)(sk[mid] >> (kr + 12)) < lg)
                a = mid + 1;
            else
                z = mid;
        }
        dst[j] = (uint32_t)ginfo[g0 + lg] - lo + (t - a);
        if (TEXT) {
            outk[j] = K[lo + i];  // the whole key (this range of K is written only below)
            if (t > a && (sk[t - 1] >> 12) == (key >> 12)) {  // not a run start
                tie = true;
                atomicAnd(reinterpret_cast<unsigned long long *>(&runb[dst[j] >> 6]), ~(1ull << (dst[j] & 63u)));
            }
        } else {
            outk[j] = ((uint64_t)(g0 + lg) << kb) | ((key >> 12) & mask);
        }
        vv[j] = sv[i];
    }
    __syncthreads();  // (every whole key read from K before any entry is written)
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t t = tid + j * kSegThreads;
        if (t < nb) {
            K[lo + dst[j]] = outk[j];
            V[lo + dst[j]] = vv[j];
        }
    }
    if (TEXT) {
        if (__syncthreads_or(tie)) {
            for (uint32_t q = tid; q < kSegCap / 64; q += kSegThreads)
                rb[(size_t)w * (kSegCap / 64) + q] = runb[q];
            if (tid == 0)
                need[w] = 1u;
        }
    }
}

// SALZ_CHECK=sa: every position must appear exactly once in the suffix array.
__global__ void k_sa_check(const uint32_t *__restrict__ sa, uint32_t nsa, uint32_t n, uint32_t *seen,
                           uint32_t *err)
{
    size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r >= nsa)
        return;
    const uint32_t i = sa[r];
    if (i >= n || atomicAdd(&seen[i], 1u) != 0)
        atomicOr(err, 0x100u);
}

// SALZ_CHECK_ROUNDS=1 (diagnostics): per-round invariants of the suffix sorter.
__global__ void k_dbg_sorted(const uint64_t *__restrict__ K, uint32_t m, uint32_t *err, uint32_t code)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c == 0 || c >= m)
        return;
    if (K[c - 1] > K[c])
        atomicOr(err, code);
}

__global__ void k_dbg_pairs(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V,
                            const uint32_t *__restrict__ rank, const uint8_t *__restrict__ T,
                            uint32_t m, Blocks bl, Alpha a, uint32_t h, int kb, int round0, uint32_t *err)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint32_t i = V[c];
    if (i >= bl.npos) {
        atomicOr(err, 0x10000u);
        return;
    }
    uint64_t want;
    if (round0) {
        want = round0_key(T, i, bl.end(i), a);
        const uint64_t got = K[c];
        if (got != want) {
            atomicOr(err, 0x20000u);
            if (atomicCAS(err + 2, 0u, 1u) == 0u) {
                err[4] = (uint32_t)c;
                err[5] = i;
                err[6] = (uint32_t)(got >> 32);
                err[7] = (uint32_t)got;
                err[8] = (uint32_t)(want >> 32);
                err[9] = (uint32_t)want;
                err[10] = atomicAdd(err + 3, 0u);
            }
            atomicAdd(err + 3, 1u);
        }
    } else if ((K[c] & ((1ull << kb) - 1ull)) != rank[i + h]) {
        atomicOr(err, 0x40000u);
    }
}

// The text round's list (SALZ_CHECK=rounds): every key is the round-0 key at i + h0 of its suffix,
// and the list is sorted by (group, key).
__global__ void k_dbg_text(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V,
                           const uint32_t *__restrict__ gin, const uint8_t *__restrict__ Tm, uint32_t m, Blocks bl,
                           Alpha a, uint32_t h0, uint32_t *err)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint32_t i = V[c];
    if (i >= bl.npos || bl.end(i) - i < h0 || K[c] != round0_key_mapped(Tm, i + h0, bl.end(i), a))
        atomicOr(err, 0x80000u);
    else if (c > 0 && (gin[c - 1] > gin[c] || (gin[c - 1] == gin[c] && K[c - 1] > K[c])))
        atomicOr(err, 0x100000u);
}

__global__ void k_dbg_heads(HeadBits hb, const uint32_t *__restrict__ headpos, uint32_t m,
                            uint32_t *err)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    // unconditional loads (see load_u64_any): no exec-masked load next to another one
    uint32_t bit, pbit;
    const uint32_t g = gid1(hb, c, bit);
    const uint32_t pv = gid1(hb, c ? c - 1 : 0, pbit);
    const uint32_t prev = c ? pv : 0u;
    const uint32_t hfc = (uint32_t)(hb.hmask[c >> 6] >> (c & 63u)) & 1u;
    if (g - prev != hfc || g == 0)
        atomicOr(err, 0x2000u);
    else if (headpos[g - 1] > c || headpos[g] <= c)
        atomicOr(err, 0x4000u);
}

// Members of large groups -> contiguous extracted array, key (large-group id, rank). Large
// group lg owns extracted range [lrec[lg] >> 32, + size) (the ranges follow lg: one atomic
// handed out both); k_tile_lg finds the group holding each 256-entry tile's first entry (a
// binary search over GL ranges), and since a large group outlasts a tile, an entry of the tile
// belongs to that group or the next. So only the mL extracted entries are visited.
__global__ void k_tile_lg(const uint64_t *__restrict__ lrec, uint32_t GL, uint32_t mL, uint32_t *__restrict__ tmap)
{
    const size_t t = (size_t)blockIdx.x * kT + threadIdx.x;
    if (t * kT >= mL)
        return;
    const uint64_t x0 = t * kT;
    uint32_t lo = 0, hi = GL - 1u;  // the last group whose range starts at or before x0
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if ((lrec[mid] >> 32) <= x0)
            lo = mid;
        else
            hi = mid - 1u;
    }
    tmap[t] = lo;
}

__global__ void k_extract(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V,
                          const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ tmap,
                          uint32_t GL, uint32_t m, uint32_t mL, int kb, uint64_t *__restrict__ KC,
                          uint32_t *__restrict__ VC, uint32_t *err)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    if (x >= mL)
        return;
    const uint32_t lg0 = tmap[blockIdx.x];
    const uint64_t r0 = lrec[lg0], r1 = lrec[lg0 + 1u < GL ? lg0 + 1u : lg0];  // unconditional loads
    const bool next = lg0 + 1u < GL && x >= (r1 >> 32);
    const uint32_t lg = next ? lg0 + 1u : lg0;
    const uint64_t r = next ? r1 : r0;
    const uint32_t orig = (uint32_t)r + (uint32_t)(x - (r >> 32));
    if (bad_index(orig >= m, err, kErrExtract))
        return;
    KC[x] = ((uint64_t)lg << kb) | (K[orig] & ((1ull << kb) - 1ull));
    VC[x] = V[orig];
}

// Segmented large-group sort (the rank rounds' default, radix_sort_segmented): every large group
// takes whole radix tiles, so its entries are sorted on the rank bits alone (kb bits: 3 passes of
// 9 for 100 MB blocks) instead of on (large group, rank) (kb + 9..11 bits: 4-5 passes). Tiles of
// each group (ptn), scanned to its first tile (pt0), then the group and entry count of every tile.
__global__ void k_lg_tiles(const uint64_t *__restrict__ lrec, uint32_t GL, uint32_t mL, uint32_t *__restrict__ ptn)
{
    const uint32_t lg = blockIdx.x * kT + threadIdx.x;
    if (lg >= GL)
        return;
    const uint32_t s0 = (uint32_t)(lrec[lg] >> 32), s1 = lg + 1u < GL ? (uint32_t)(lrec[lg + 1u] >> 32) : mL;
    ptn[lg] = (s1 - s0 + kRadixTile - 1u) / kRadixTile;
}

__global__ void k_lg_tilemap(const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ pt0, uint32_t GL,
                             uint32_t mL, uint32_t ntiles, uint32_t *__restrict__ tseg, uint32_t *__restrict__ tcnt)
{
    const uint32_t t = blockIdx.x * kT + threadIdx.x;
    if (t >= ntiles)
        return;
    uint32_t lo = 0, hi = GL - 1u;  // the last group whose first tile is at or before t
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (pt0[mid] <= t)
            lo = mid;
        else
            hi = mid - 1u;
    }
    const uint32_t s0 = (uint32_t)(lrec[lo] >> 32), s1 = lo + 1u < GL ? (uint32_t)(lrec[lo + 1u] >> 32) : mL;
    const uint32_t off = (t - pt0[lo]) * kRadixTile, left = s1 - s0 - off;
    tseg[t] = lo;
    tcnt[t] = left < kRadixTile ? left : kRadixTile;
}

// Entry x of the tiled list: tile x / 4096 of its group, slot x % 4096 (past the tile's count:
// padding). The key keeps its group id in the upper bits (the same for the whole group), so the
// sorted entries go back unchanged.
__global__ void k_extract_seg(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V,
                              const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ pt0,
                              const uint32_t *__restrict__ tseg, const uint32_t *__restrict__ tcnt, uint32_t m,
                              uint32_t ntiles, uint64_t *__restrict__ KC, uint32_t *__restrict__ VC, uint32_t *err)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t t = (uint32_t)(x / kRadixTile), j = (uint32_t)(x % kRadixTile);
    if (t >= ntiles || j >= tcnt[t])
        return;
    const uint32_t lg = tseg[t];
    const uint32_t orig = (uint32_t)lrec[lg] + (t - pt0[lg]) * kRadixTile + j;
    if (bad_index(orig >= m, err, kErrExtract))
        return;
    KC[x] = K[orig];
    VC[x] = V[orig];
}

__global__ void k_putback_seg(const uint64_t *__restrict__ KS, const uint32_t *__restrict__ VS,
                              const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ pt0,
                              const uint32_t *__restrict__ tseg, const uint32_t *__restrict__ tcnt, uint32_t m,
                              uint32_t ntiles, uint64_t *__restrict__ K, uint32_t *__restrict__ V, uint32_t *err)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t t = (uint32_t)(x / kRadixTile), j = (uint32_t)(x % kRadixTile);
    if (t >= ntiles || j >= tcnt[t])
        return;
    const uint32_t lg = tseg[t];
    const uint32_t orig = (uint32_t)lrec[lg] + (t - pt0[lg]) * kRadixTile + j;
    if (bad_index(orig >= m, err, kErrPutback))
        return;
    K[orig] = KS[x];
    V[orig] = VS[x];
}

// Sorted large groups back to their places in the active list, original key format.
__global__ void k_putback(const uint64_t *__restrict__ KS, const uint32_t *__restrict__ VS,
                          const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ lg2g,
                          uint32_t mL, uint32_t GL, uint32_t m, int kb, uint64_t *__restrict__ K,
                          uint32_t *__restrict__ V, uint32_t *err)
{
    size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    if (x >= mL)
        return;
    const uint64_t key = KS[x];
    const uint32_t lg = (uint32_t)(key >> kb);
    if (bad_index(lg >= GL, err, kErrPutback))
        return;
    const uint64_t r = lrec[lg];
    const uint32_t orig = (uint32_t)r + ((uint32_t)x - (uint32_t)(r >> 32));
    if (bad_index(orig >= m, err, kErrPutback))
        return;
    K[orig] = ((uint64_t)lg2g[lg] << kb) | (key & ((1ull << kb) - 1ull));
    V[orig] = VS[x];
}

__global__ void k_keys(const uint32_t *__restrict__ nval, const uint32_t *__restrict__ ngid,
                       const uint32_t *__restrict__ rank, uint32_t m, uint32_t n, uint32_t h, int kb,
                       uint64_t *__restrict__ key, uint32_t *err)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    uint32_t i = nval[c];
    if (bad_index((uint64_t)i + h > n, err, kErrKeys)) {
        key[c] = 0;
        return;
    }
    key[c] = ((uint64_t)ngid[c] << kb) | (uint64_t)rank[i + h];
}

// ---- round 1 keyed by text ------------------------------------------------------------------
// Round 1 orders each depth-h0 group by rank[i + h0], the depth-h0 rank of suffix i + h0. That
// rank is an order-preserving name of the h0 symbols at i + h0, so the round can compare those
// symbols themselves (the round-0 key at i + h0) instead. Then round 0 writes only the ranks of
// the suffixes it finishes (16% of a text block) instead of all n, and the LCP of round 1's new
// heads comes from the two keys instead of a random text read per head; round 1 writes every
// rank of its list. The keys are h0 symbols of >= 1 (an alphabet of at most 127 bytes, Alpha):
// a key padded with zeros past the end of the text is then never equal to a longer suffix's.
// The group of an entry is no longer in its key: `gin` holds it.

// Round 1's key of survivor nval[c]: the round-0 key at i + h0 (a survivor has h0 symbols left),
// from the text mapped to symbols (Tm).
__global__ void k_keys_text(const uint32_t *__restrict__ nval, uint32_t m, Blocks bl, Alpha a, uint32_t h0,
                            const uint8_t *__restrict__ Tm, uint64_t *__restrict__ key)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint32_t i = nval[c];
    key[c] = round0_key_mapped(Tm, i + h0, bl.end(i), a);
}

// Group heads of the text round's sorted list, and the LCP of each new head (two suffixes of one
// depth-h0 group: h0 + the equal leading symbols of their keys; a key padded past the end of the
// text stops at its first zero symbol, so the LCP is exact).
__global__ __launch_bounds__(kT) void k_heads_text(const uint64_t *__restrict__ K, const uint32_t *__restrict__ gin,
                                                   HeadBits hb, const uint32_t *__restrict__ off_old, uint32_t m,
                                                   Alpha a, uint32_t h0, uint32_t *__restrict__ lcps)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    const bool in = c < m;
    const size_t cc = in ? c : 0, cp = cc ? cc - 1 : 0;  // (unconditional loads)
    const uint64_t k0 = K[cp], k1 = K[cc];
    const uint32_t g0 = gin[cp], g1 = gin[cc];
    const bool head = cc == 0 || g0 != g1 || k0 != k1;
    put_heads(hb, c, m, in && head);
    if (lcps && in && head && cc > 0 && g0 == g1)
        lcps[(uint32_t)cc + off_old[g1]] = h0 + round0_lcp(k0 ^ k1, a);
}

// The runs of equal (group, top key bits) that k_seg_sort<1> left (windows flagged in need),
// each ordered by the whole key: runs of up to kRunCount entries by counting (each entry's place
// is the run start + the entries with a smaller (key, index): at depth 13-14 of text a run holds
// 14-20 entries on average), longer ones (a window may hold one of 2000) by a bitonic sort of the
// run in LDS, the whole workgroup on one run at a time.
constexpr uint32_t kRunCount = 64;
constexpr uint32_t kMaxLongRuns = 64;
__global__ __launch_bounds__(kSegThreads) void k_seg_text_fix(uint64_t *__restrict__ K, uint32_t *__restrict__ V,
                                                              SegPlan plan, const uint64_t *__restrict__ rb,
                                                              const uint32_t *__restrict__ need)
{
    __shared__ uint64_t sk[kSegCap];
    __shared__ uint32_t sv[kSegCap];
    __shared__ uint64_t runb[kSegCap / 64];
    __shared__ uint32_t longs[kMaxLongRuns];  // (start << 16 | end) of the long runs
    __shared__ uint32_t nlong;
    const unsigned tid = threadIdx.x;
    const uint32_t w = blockIdx.x;
    if (!need[w])
        return;
    const uint32_t lo = plan.lo[w], count = plan.hi[w] - lo;  // (checked by k_seg_sort)
    const uint32_t nwords = (count + 63u) >> 6;
    if (tid == 0)
        nlong = 0;
    {  // (every load issued before the first is used, as in k_seg_sort)
        uint64_t wk[kPer];
        uint32_t wv[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t i = tid + j * kSegThreads, ii = i < count ? i : 0u;
            wk[j] = K[lo + ii];
            wv[j] = V[lo + ii];
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t i = tid + j * kSegThreads;
            if (i < count) {
                sk[i] = wk[j];
                sv[i] = wv[j];
            }
        }
    }
    for (uint32_t q = tid; q < nwords; q += kSegThreads)
        runb[q] = rb[(size_t)w * (kSegCap / 64) + q];
    __syncthreads();
    // run [rs, re) of entry i: the last start at or below i, the next start above it
    auto run_of = [&](uint32_t i, uint32_t &rs, uint32_t &re) {
        uint32_t wi = i >> 6;
        uint64_t x = runb[wi] & (~0ull >> (63u - (i & 63u)));
        while (!x)
            x = runb[--wi];
        rs = wi * 64u + 63u - (uint32_t)__builtin_clzll(x);
        wi = i >> 6;
        x = (i & 63u) == 63u ? 0ull : runb[wi] & (~0ull << ((i & 63u) + 1u));
        while (!x && ++wi < nwords)
            x = runb[wi];
        re = x ? wi * 64u + (uint32_t)__builtin_ctzll(x) : count;
    };
    // the long runs, listed by their first entries
    for (uint32_t i = tid; i < count; i += kSegThreads)
        if ((runb[i >> 6] >> (i & 63u)) & 1ull) {
            uint32_t rs, re;
            run_of(i, rs, re);
            if (re - rs > kRunCount) {
                const uint32_t k = atomicAdd(&nlong, 1u);
                if (k < kMaxLongRuns)
                    longs[k] = (rs << 16) | re;
            }
        }
    __syncthreads();
    const uint32_t nl = nlong < kMaxLongRuns ? nlong : kMaxLongRuns;  // (a window holds < 64 runs of > 64)
    for (uint32_t r = 0; r < nl; r++) {
        const uint32_t rs = longs[r] >> 16, len = (longs[r] & 0xffffu) - rs;
        uint32_t P = 1;
        while (P < len)
            P <<= 1;
        // ascending-only bitonic network (first step of each merge pairs i with its mirror), so
        // the entries past len act as +inf and are never touched
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = tid; t < P / 2; t += kSegThreads) {
                    const uint32_t i = 2 * t - (t & (j - 1));
                    const uint32_t p = j == (k >> 1) ? (i | (k - 1)) - (i & (k - 1)) : i + j;
                    if (p < len) {
                        const uint64_t a = sk[rs + i], b = sk[rs + p];
                        if (b < a) {
                            const uint32_t va = sv[rs + i], vb = sv[rs + p];
                            sk[rs + i] = b;
                            sk[rs + p] = a;
                            sv[rs + i] = vb;
                            sv[rs + p] = va;
                        }
                    }
                }
                __syncthreads();
            }
    }
    for (uint32_t i = tid; i < count; i += kSegThreads) {
        uint32_t rs, re;
        run_of(i, rs, re);
        if (re - rs < 2)
            continue;
        uint32_t dst = i;
        const uint64_t ki = sk[i];
        if (re - rs <= kRunCount) {
            uint32_t r = 0;
#pragma unroll 8
            for (uint32_t y = rs; y < re; y++) {
                const uint64_t ky = sk[y];
                r += (ky < ki || (ky == ki && y < i)) ? 1u : 0u;
            }
            dst = rs + r;
        }
        K[lo + dst] = ki;
        V[lo + dst] = sv[i];
    }
}

// The text round's large groups: extracted with their keys, their extraction index as the value
// (so a radix sort on the keys followed by one on the large group of the value orders them by
// (group, key)) and their suffixes aside in PC.
__global__ void k_extract_text(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V,
                               const uint64_t *__restrict__ lrec, const uint32_t *__restrict__ tmap, uint32_t GL,
                               uint32_t m, uint32_t mL, uint64_t *__restrict__ KC, uint32_t *__restrict__ VC,
                               uint32_t *__restrict__ PC, uint32_t *err)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    if (x >= mL)
        return;
    const uint32_t lg0 = tmap[blockIdx.x];
    const uint64_t r0 = lrec[lg0], r1 = lrec[lg0 + 1u < GL ? lg0 + 1u : lg0];  // unconditional loads
    const bool next = lg0 + 1u < GL && x >= (r1 >> 32);
    const uint64_t r = next ? r1 : r0;
    const uint32_t orig = (uint32_t)r + (uint32_t)(x - (r >> 32));
    if (bad_index(orig >= m, err, kErrExtract))
        return;
    KC[x] = K[orig];
    VC[x] = (uint32_t)x;
    PC[x] = V[orig];
}

// Sorted position y of the extracted array (now in (large group, key) order, so y lies in its
// group's extraction range) back to its place in the list.
__global__ void k_putback_text(const uint64_t *__restrict__ KS, const uint32_t *__restrict__ VS,
                               const uint32_t *__restrict__ PC, const uint64_t *__restrict__ lrec,
                               const uint32_t *__restrict__ tmap, uint32_t GL, uint32_t m, uint32_t mL,
                               uint64_t *__restrict__ K, uint32_t *__restrict__ V, uint32_t *err)
{
    const size_t y = (size_t)blockIdx.x * kT + threadIdx.x;
    if (y >= mL)
        return;
    const uint32_t lg0 = tmap[blockIdx.x];
    const uint64_t r0 = lrec[lg0], r1 = lrec[lg0 + 1u < GL ? lg0 + 1u : lg0];
    const bool next = lg0 + 1u < GL && y >= (r1 >> 32);
    const uint64_t r = next ? r1 : r0;
    const uint32_t orig = (uint32_t)r + (uint32_t)(y - (r >> 32));
    const uint32_t x = VS[y];
    if (bad_index(orig >= m || x >= mL, err, kErrPutback))
        return;
    K[orig] = KS[y];
    V[orig] = PC[x];
}

}  // namespace

// The repetition probe's three launches (k_repeat_probe, k_repeat_scan, k_repeat_count) over the
// block's n suffixes (n >= 64): results in the u32 words 248 (samples sharing a fingerprint), 249
// (repeated points), 250 (twin distance) and 251 (its points) of dscal, read back by the caller;
// scratch in u1.
static void launch_repeat_probe(Workspace &ws, uint32_t n)
{
    hipStream_t st = ws.stream;
    uint32_t *words = reinterpret_cast<uint32_t *>(ws.dscal) + 240;
    uint32_t *ptab = ws.u1, *pmul = ws.u1 + kProbeSlots, *gcnt = ws.u1 + 2 * kProbeSlots;
    uint32_t *pfilt = ws.u1 + 3 * kProbeSlots, *pslot = pfilt + kFilterBits / 32, *hpos = pslot + kProbe;
    hipLaunchKernelGGL(k_repeat_probe, dim3(1), dim3(kProbeThreads), 0, st, ws.text, n, words + 8, ptab, pmul, gcnt,
                       pfilt, pslot, hpos);
    const uint32_t groups = (n - 32u) / 64u + 1u;  // 8 aligned grams per thread
    const uint32_t grid = grid_for(groups, kScanThreads) < 1024 ? grid_for(groups, kScanThreads) : 1024;
    hipLaunchKernelGGL(k_repeat_scan, dim3(grid), dim3(kScanThreads), 0, st, ws.text, n, words + 8, ptab, pfilt,
                       gcnt, hpos);
    hipLaunchKernelGGL(k_repeat_count, dim3(1), dim3(kProbePoints), 0, st, words + 8, pmul, gcnt, pslot, hpos, n,
                       words + 9);
}

// The probe's verdict from the words read back (hs: ws.hscal as u32): half the samples repeated
// among themselves (long repeats everywhere), or three quarters of them anywhere in the block
// (what the depth-32 switch of the doubling rounds tests).
static bool probe_repetitive(const uint32_t *hs)
{
    return hs[248] * 2 >= kProbe || (uint64_t)hs[249] * 4 >= 3ull * kProbePoints;
}

int block_repetitive(Workspace &ws, uint32_t n)
{
    if (n < (1u << 20))  // (the size from which single blocks take DC3, stage_suffix_array)
        return 0;
    launch_repeat_probe(ws, n);
    SALZ_LAUNCH_CHECK();
    if (read_scalars(ws, 960, 48, "sa.probe") != 0)
        return -1;
    return probe_repetitive(reinterpret_cast<const uint32_t *>(ws.hscal)) ? 1 : 0;
}

int block_alpha_bits(Workspace &ws, uint32_t n)
{
    if (n < 64)
        return 0;
    hipStream_t st = ws.stream;
    uint32_t *words = reinterpret_cast<uint32_t *>(ws.dscal) + 240;
    SALZ_HIP(fill_async(words, 0, 8 * sizeof(uint32_t), st));
    const size_t P = (size_t)n + 8;
    hipLaunchKernelGGL(k_alpha_presence, dim3(grid_for(P, kT * 16) < 2048 ? grid_for(P, kT * 16) : 2048), dim3(kT), 0,
                       st, ws.text, P, words);
    SALZ_LAUNCH_CHECK();
    if (read_scalars(ws, 960, 32, "sa.alpha_bits") != 0)
        return -1;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(ws.hscal) + 240;
    uint32_t sigma = 0;
    for (int w = 0; w < 8; w++)
        sigma += (uint32_t)__builtin_popcount(pw[w]);
    const int bits = bit_width(sigma);
    return bits <= 7 ? bits : 0;
}

int stage_suffix_array(Workspace &ws, const Blocks &bl, const DistSa *dist)
{
    hipStream_t st = ws.stream;
    // position space, live suffixes (a split block: this rank's bucket)
    const uint32_t n = bl.npos, nsa = dist ? dist->m0 : bl.nsa();
    if (nsa == 0)
        return 0;
    uint64_t *K = ws.keyA;
    uint32_t *V = ws.valA;
    uint32_t *offo = ws.offA, *offn = ws.offB;
    uint32_t *headpos = ws.u2, *ngid = ws.u3;
    const size_t nw_max = ((size_t)n + 63) / 64;  // head ballots of up to n list entries, in u0
    HeadBits hb{reinterpret_cast<uint64_t *>(ws.u0), ws.u0 + 2 * nw_max, ws.u0 + 3 * nw_max};
    uint32_t *d32 = reinterpret_cast<uint32_t *>(ws.dscal);
    uint64_t *d64 = ws.dscal + 8;
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    SALZ_HIP(fill_async(derr, 0, sizeof(uint32_t) * 12, st));
    ws.stats.sa_rounds = 0;
    ws.stats.sa_sorted_elems = 0;
    ws.stats.sa_dc3_levels = 0;
    // Scratch borrowed from later stages (free while the suffix array is built): the
    // extracted large groups live in pst (keys) and cand (values), the group table in cand.
    uint8_t *cb = reinterpret_cast<uint8_t *>(ws.cand);
    uint32_t *VC = reinterpret_cast<uint32_t *>(cb);
    GroupTab tab{reinterpret_cast<uint64_t *>(cb + 4 * ws.cap_s), ws.lrec, ws.lg2g};
    uint64_t *KC = ws.pst;

    // Test switches (SALZ_SA, a comma-separated list): plcp, dc3, doubling, global, segmented;
    // SALZ_CHECK=rounds,sa and SALZ_DEBUG=sa.
    static const bool dbg_rounds = env_flag("SALZ_CHECK", "rounds");
    ws.lcps_ok = !env_flag("SALZ_SA", "plcp");  // plcp: the LCP from the Phi/PLCP stage instead
    // Round 0's alphabet: texts of at most 127 distinct bytes get compacted keys (Alpha,
    // common.hpp); others keep raw 8-byte keys.
    Alpha alpha{};
    // DC3 (dc3.hip) instead of doubling for repetitive single blocks: SALZ_SA=dc3 forces it,
    // =doubling never. By default a block of >= 1 MiB starts with DC3 when the repetition probe
    // finds half of its sampled 32-grams repeated, and otherwise switches once the sort has reached depth 32
    // with more than 3/4 of its suffixes still unfinished (long repeats: the following rounds stay
    // that wide; text keeps ~17% at depth 32, Fibonacci and periodic blocks all of them).
    const bool dc3_force = env_flag("SALZ_SA", "dc3") && bl.nb == 1 && n >= 2 && !dist;
    const bool dc3_auto = !env_flag("SALZ_SA", "doubling") && bl.nb == 1 && n >= (1u << 20) && !dist;
    bool dc3_now = false;
    uint32_t twin_d = 0;  // twin distance (k_twin_pairs), 0: none
    Alpha codes{};  // the block's byte codes 1..sigma for DC3 (raw bytes + 1 when not known)
    int codes_raw = 1;
    if (n >= 64) {
        uint32_t *words = reinterpret_cast<uint32_t *>(ws.dscal) + 240;
        SALZ_HIP(fill_async(words, 0, 8 * sizeof(uint32_t), st));
        const size_t P = (size_t)n + 8;
        hipLaunchKernelGGL(k_alpha_presence, dim3(grid_for(P, kT * 16) < 2048 ? grid_for(P, kT * 16) : 2048),
                           dim3(kT), 0, st, ws.text, P, words);
        SALZ_LAUNCH_CHECK();
        if (dc3_auto) {  // (sample table, scan and count in u1: free until round 0's survivor counts)
            launch_repeat_probe(ws, n);
            SALZ_LAUNCH_CHECK();
        }
        if (read_scalars(ws, 960, 48, "sa.alpha") != 0)
            return -1;
        // the probe's verdict: DC3 from the start, or doubling with twin pairs when three quarters
        // of the sample points have one copy at the same distance
        const uint32_t *hs = reinterpret_cast<const uint32_t *>(ws.hscal);
        dc3_now = dc3_auto && probe_repetitive(hs);
        if (dc3_now && (uint64_t)hs[251] * 4 >= 3ull * kProbePoints && hs[250] > 0 && hs[250] < n) {
            twin_d = hs[250];
            dc3_now = false;
        }
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(ws.hscal) + 240;
        uint32_t sigma = 0;
        for (int c = 0; c < 256; c++)
            if (pw[c >> 5] & (1u << (c & 31)))
                alpha.code[c] = (uint8_t)++sigma;
        ws.sigma = sigma;  // (the parse's chunk length on large blocks follows it, pipeline.hip)
        const uint32_t bits = (uint32_t)bit_width(sigma);  // codes 1..sigma, 0 = past the end
        if (sigma <= 255) {
            codes = alpha;
            codes_raw = 0;
        }
        if (bits <= 7) {
            // As many symbols as fit 64 bits: 7-bit alphabets (text) sort round 0 to depth 9 in
            // 8 passes rather than depth 8 in 7; the deeper start leaves fewer suffixes to the
            // doubling rounds (text surrogate: 12% fewer after round 0, 14% after round 1; C2 SA
            // 22.2 -> 21.6 ms against 8 symbols, profiles/r03g_alpha9_ab.txt). Re-measured with
            // the text round (round 5, one box): 8 symbols 20.6 ms against 19.9, enwik9-sized
            // blocks 12.3 against 11.9.
            alpha.bits = bits;
            alpha.k = 64u / bits;
        }
    }
    if (dc3_force || dc3_now)
        return stage_suffix_array_dc3(ws, bl, codes, codes_raw);
    // the twin table (L + 1 entries) and its tile carries, in the DC3 arena
    uint32_t *twin = nullptr;
    if (twin_d) {
        const uint32_t L = n - twin_d, ntw = (L + kTwTile) / kTwTile;  // tiles over [0, L]
        uint8_t *ar = dc3_arena_reserve(ws, ((size_t)L + 1 + ntw) * sizeof(uint32_t) + 256);
        if (!ar)
            return -1;
        twin = reinterpret_cast<uint32_t *>(ar);
        uint32_t *tmin = twin + L + 1;
        hipLaunchKernelGGL(k_twin_tiles, dim3(ntw), dim3(kT), 0, st, ws.text, twin_d, L, tmin);
        SALZ_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_twin_carry, dim3(1), dim3(kTwCarryT), 0, st, tmin, ntw);
        SALZ_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_twin_fill, dim3(ntw), dim3(kT), 0, st, ws.text, twin_d, L, tmin, twin);
        SALZ_LAUNCH_CHECK();
        if (env_flag("SALZ_DEBUG", "sa"))
            fprintf(stderr, "sa twin pairs at distance %u (%u of %u probe points)\n", twin_d,
                    reinterpret_cast<const uint32_t *>(ws.hscal)[251], kProbePoints);
    }
    const uint32_t h0 = alpha.bits ? alpha.k : 8u;
    // The text mapped to symbols for the text-sourced radix pass and the text round's keys (u3
    // is free until round 0's commit writes the group ids, which go to `gin` before a text
    // round): one byte per position, zero padded. (A split block's bucket list lives in u3 and
    // its round 0 reads the raw text: no mapped copy there.)
    uint8_t *tmapped = nullptr;
    if (alpha.bits && !dist) {
        tmapped = reinterpret_cast<uint8_t *>(ws.u3);
        const size_t P = (size_t)n + 8;
        hipLaunchKernelGGL(k_map_text, dim3(grid_for(P + 64, kT * 16)), dim3(kT), 0, st, ws.text, P, alpha,
                           tmapped);
        SALZ_LAUNCH_CHECK();
    }
    SALZ_HIP(fill_async(ws.rank + n, 0, sizeof(uint32_t), st));  // rank[n] = 0
    if (bl.nb > 1) {
        hipLaunchKernelGGL(k_dead_ranks, dim3(grid_for(8u * (bl.nb - 1u), kT)), dim3(kT), 0, st, bl, ws.rank);
        SALZ_LAUNCH_CHECK();
    }
    // Round 0's first radix pass reads the text itself (radix.hip, TextSrc); the initial
    // key/value arrays are only materialised for the per-round checks, and for n = 1 (the
    // sort has nothing to do and would leave them unwritten; the materialised list measured
    // 0.1-0.2 ms slower).
    const bool text_first = !dbg_rounds && nsa > 1 && !dist;
    // Digit bytes of the radix passes (radix.hip) in u2, free during every sort (the head
    // positions are written after it)
    uint8_t *rdig = reinterpret_cast<uint8_t *>(ws.u2);
    if (dist) {
        hipLaunchKernelGGL(k_list_init, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, ws.text, dist->list, nsa, n, alpha,
                           K, V);
        SALZ_LAUNCH_CHECK();
        if (dist->text1 && alpha.bits) {  // (the list in u3 is consumed: the mapped text takes its place)
            tmapped = reinterpret_cast<uint8_t *>(ws.u3);
            const size_t P = (size_t)n + 8;
            hipLaunchKernelGGL(k_map_text, dim3(grid_for(P + 64, kT * 16)), dim3(kT), 0, st, ws.text, P, alpha,
                               tmapped);
            SALZ_LAUNCH_CHECK();
        }
    } else if (!text_first) {
        hipLaunchKernelGGL(k_sa_init, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, ws.text, tmapped, bl, alpha, K, V,
                           rdig);
        SALZ_LAUNCH_CHECK();
    }
    if (dbg_rounds && bl.nb == 1 && !dist) {
        hipLaunchKernelGGL(k_dbg_pairs, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, K, V, ws.rank, ws.text, nsa, bl,
                           alpha, 0u, 0, 1, derr);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 512, "sa.init") != 0)
            return -1;
        if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
            const uint32_t *d = reinterpret_cast<uint32_t *>(ws.hscal) + kErrWord;
            set_error("suffix sort: init pairs check failed (code 0x%x): %u bad; first c=%u i=%u key "
                      "%08x%08x want %08x%08x", e, d[3], d[4], d[5], d[6], d[7], d[8], d[9]);
            return -1;
        }
    }

    uint32_t m = nsa, h = h0, G_act = 0, GL = 0, mL = 0, lgtiles = 0;
    int kb_old = 0, round0 = 1;
    const int kb = bit_width(n);
    static const bool verbose = env_flag("SALZ_DEBUG", "sa");
    const bool mode_global = env_flag("SALZ_SA", "global"), mode_seg = env_flag("SALZ_SA", "segmented");
    // groups of at most seg_tiny members are ordered by counting in k_seg_sort, larger ones by LSD
    // passes in LDS. C2 SA 21.9 / 21.0 / 20.9 / 20.8 / 20.6 / 20.5 / 20.4 / 22.7 ms at 0 / 8 / 16 /
    // 32 / 64 / 128 / 256 / 2048; mixed 100 MB 27.2 (0) -> 25.7 ms (64-256)
    // (profiles/r04n_tiny_sweep.txt)
    constexpr uint32_t seg_tiny = 128;
    // the text round counts groups of up to 256 (C2 SA 20.02 -> 19.89 ms, enwik9-sized blocks
    // 12.2 -> 12.0 ms; the rank rounds of mixed data are faster at 128: profiles/r04w_c3_ab.txt)
    constexpr uint32_t seg_tiny_text = 256;
    // The text round's LDS passes sort (group, top key bits) to 48 bits (6 passes) and leave the
    // rarer ties to k_seg_text_fix: C2 SA 20.29 -> 20.18 ms against 40 bits (5 passes), 52 bits
    // (7 passes) 20.28 (profiles/r04w_c3_ab.txt).
    constexpr int lsd_bits = 48;
    // Round 1 keyed by text (see k_keys_text): one block or a batch, the block's own sort (not a
    // split block's bucket), an alphabet of at most 127 bytes (symbols >= 1, so zero padding
    // is unambiguous); blocks of more than 127 distinct bytes keep round 1 on ranks.
    // (a split block: the decision every rank made in dist_suffix_array, from the same alphabet)
    const bool text1 = dist ? dist->text1 : alpha.bits > 0;
    if (text1 && (!alpha.bits || !tmapped)) {
        set_error("suffix sort: text round without a compacted alphabet");
        return -1;
    }
    const int tbits = (int)(alpha.k * alpha.bits);
    // group ids of the text round's list (its keys are the text): the upper half of lsc, free
    // during every round (the window plan and tile map take its first entries)
    uint32_t *gin = reinterpret_cast<uint32_t *>(ws.lsc) + 2 * ws.cap_s;
    auto t_round = std::chrono::steady_clock::now();
    // The current round's large groups, each in whole radix tiles and sorted on its key bits
    // [0, bits) alone (k_lg_tiles: tiles per group, scanned to first tiles; k_lg_tilemap; extract;
    // radix_sort_segmented; put back): the tile tables in u1, free until k_surv.
    auto sort_large_segmented = [&](int bits) -> int {
        SegTiles sgt{ws.u1, ws.u1 + lgtiles, ws.u1 + 2 * lgtiles, ws.u1 + 2 * lgtiles + GL,
                     ws.u1 + 2 * lgtiles + 2 * GL, lgtiles, mL};
        uint32_t *ptn = const_cast<uint32_t *>(sgt.ptn), *pt0 = const_cast<uint32_t *>(sgt.pt0);
        hipLaunchKernelGGL(k_lg_tiles, dim3(grid_for(GL, kT)), dim3(kT), 0, st, tab.lrec, GL, mL, ptn);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(ptn, pt0, GL, false, nullptr, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_lg_tilemap, dim3(grid_for(lgtiles, kT)), dim3(kT), 0, st, tab.lrec, pt0, GL, mL, lgtiles,
                           const_cast<uint32_t *>(sgt.tseg), const_cast<uint32_t *>(sgt.tcnt));
        SALZ_LAUNCH_CHECK();
        uint64_t *Kx = (K == ws.keyA) ? ws.keyB : ws.keyA;
        uint32_t *Vx = (V == ws.valA) ? ws.valB : ws.valA;
        const uint32_t ngrid = lgtiles * (uint32_t)(kRadixTile / kT);
        hipLaunchKernelGGL(k_extract_seg, dim3(ngrid), dim3(kT), 0, st, K, V, tab.lrec, pt0, sgt.tseg, sgt.tcnt, m,
                           lgtiles, KC, VC, derr);
        SALZ_LAUNCH_CHECK();
        uint64_t *KS = KC;
        uint32_t *VS = VC;
        if (radix_sort_segmented(&KS, &VS, Kx, Vx, sgt, bits, ws, st, rdig) != 0)
            return -1;
        hipLaunchKernelGGL(k_putback_seg, dim3(ngrid), dim3(kT), 0, st, KS, VS, tab.lrec, pt0, sgt.tseg, sgt.tcnt, m,
                           lgtiles, K, V, derr);
        SALZ_LAUNCH_CHECK();
        return 0;
    };
    for (;;) {
        ws.stats.sa_rounds++;
        ws.stats.sa_sorted_elems += m;
        uint64_t *Kx = (K == ws.keyA) ? ws.keyB : ws.keyA;
        uint32_t *Vx = (V == ws.valA) ? ws.valB : ws.valA;
        const char *how = "global";
        bool seg_round = false;
        const bool textr = text1 && ws.stats.sa_rounds == 2;  // this round is keyed by text
        if (textr) {
            // small groups in LDS by (group, key); large ones extracted, radix-sorted on the key
            // and then on their large group (values = extraction index), put back
            how = "text";
            seg_round = true;
            const uint32_t nwin = grid_for(m, kSegT);
            uint32_t *pw = reinterpret_cast<uint32_t *>(ws.lsc);
            SegPlan plan{pw, pw + nwin, pw + 2 * nwin, pw + 3 * nwin};
            SALZ_HIP(fill_async(plan.lo, 0xff, sizeof(uint32_t) * nwin, st));
            hipLaunchKernelGGL(k_seg_plan, dim3(grid_for(G_act, kT)), dim3(kT), 0, st, tab.ginfo, G_act, plan);
            SALZ_LAUNCH_CHECK();
            // run-start bits per window (64 words each) and fix flags, in pst (free until the large
            // groups' extraction)
            uint64_t *rb = ws.pst;
            uint32_t *need = reinterpret_cast<uint32_t *>(ws.pst + (size_t)nwin * (kSegCap / 64));
            SALZ_HIP(fill_async(need, 0, sizeof(uint32_t) * nwin, st));
            hipLaunchKernelGGL(k_seg_sort<true>, dim3(nwin), dim3(kSegThreads), 0, st, K, V, gin, plan, tab.ginfo,
                               m, tbits, seg_tiny_text, rb, need, derr, lsd_bits);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_seg_text_fix, dim3(nwin), dim3(kSegThreads), 0, st, K, V, plan, rb, need);
            SALZ_LAUNCH_CHECK();
            // the large groups: each in whole radix tiles on its 63 key bits (7 passes of 9), or
            // (one large group, or too many tiles for the segmented scan) radix-sorted on the key
            // and then on their large group
            const size_t tseg_words = 2 * (size_t)lgtiles + 2 * (size_t)GL + (size_t)kMaxDigits * GL;
            const bool tlg_seg = mL && GL > 1 && lgtiles <= kSegScanMaxTiles &&
                                 (size_t)lgtiles * kRadixTile <= ws.cap_s && tseg_words <= ws.cap_s;
            if (tlg_seg) {
                if (sort_large_segmented(tbits) != 0)
                    return -1;
            } else if (mL) {
                uint32_t *tmap = pw + 4 * nwin;
                const uint32_t ntile = grid_for(mL, kT);
                // the extracted suffixes beside the group table in cand (16 B per slot: VC 4,
                // ginfo 8, PC 4)
                uint32_t *PC = reinterpret_cast<uint32_t *>(cb + 12 * ws.cap_s);
                hipLaunchKernelGGL(k_tile_lg, dim3(grid_for(ntile, kT)), dim3(kT), 0, st, tab.lrec, GL, mL, tmap);
                SALZ_LAUNCH_CHECK();
                hipLaunchKernelGGL(k_extract_text, dim3(ntile), dim3(kT), 0, st, K, V, tab.lrec, tmap, GL, m, mL, KC,
                                   VC, PC, derr);
                SALZ_LAUNCH_CHECK();
                uint64_t *KS = KC;
                uint32_t *VS = VC;
                if (radix_sort_pairs(&KS, &VS, Kx, Vx, mL, 0, tbits, ws, st, nullptr, nullptr, nullptr, rdig) != 0 ||
                    radix_sort_by_group(&KS, &VS, KS == KC ? Kx : KC, VS == VC ? Vx : VC, mL, tab.lrec, tmap, GL, ws,
                                        st) != 0)
                    return -1;
                hipLaunchKernelGGL(k_putback_text, dim3(ntile), dim3(kT), 0, st, KS, VS, PC, tab.lrec, tmap, GL, m,
                                   mL, K, V, derr);
                SALZ_LAUNCH_CHECK();
            }
        } else if (round0) {
            if (!text_first && bl.nb > 1) {
                set_error("suffix sort: a batch of blocks needs the text-built first pass");
                return -1;
            }
            const int key_bits = alpha.bits ? (int)(alpha.k * alpha.bits) : 64;
            const uint8_t *src_text = !text_first ? nullptr : tmapped ? tmapped : ws.text;
            // (materialised list: k_sa_init wrote the first pass's digits too)
            if (radix_sort_pairs(&K, &V, Kx, Vx, m, 0, key_bits, ws, st, src_text, &bl, &alpha, rdig,
                                 !text_first && !dist && rdig) != 0)
                return -1;
        } else {
            // Global sort of every active suffix on (group, rank) vs. LDS sort of the small
            // groups + global sort of the large ones on (large group, rank): pick the one
            // with less HBM traffic (32 B per element and 8-bit pass; 24 B per LDS-sorted or
            // extracted/put-back element).
            // the large groups in whole tiles, sorted each on its own (one large group, or too many
            // tiles: on (large group, rank) in one list); tile tables in u1 (free until k_surv).
            // Round 5: mixed 100 MB SA 24.76 -> 24.24 ms against the one list.
            const size_t seg_words = 2 * (size_t)lgtiles + 2 * (size_t)GL + (size_t)kMaxDigits * GL;
            const bool lg_seg = mL && GL > 1 && lgtiles <= kSegScanMaxTiles &&
                                (size_t)lgtiles * kRadixTile <= ws.cap_s && seg_words <= ws.cap_s;
            const int bits_all = kb + bit_width(G_act - 1),
                      bits_large = lg_seg ? kb : kb + bit_width(GL ? GL - 1 : 0);
            const double c_all = (double)m * ((bits_all + 7) / 8) * 32.0;
            const double c_seg = (double)(m - mL) * 24.0 + m * 8.0 +
                                 (double)mL * (((bits_large + 7) / 8) * 32.0 + 48.0);
            bool seg = c_seg < c_all;
            if (mode_global || mode_seg)
                seg = mode_seg;
            if (!seg) {
                if (radix_sort_pairs(&K, &V, Kx, Vx, m, 0, bits_all, ws, st, nullptr, nullptr, nullptr, rdig, false,
                                     true) != 0)
                    return -1;
            } else {
                how = "segmented";
                seg_round = true;
                const uint32_t nwin = grid_for(m, kSegT);
                uint32_t *pw = reinterpret_cast<uint32_t *>(ws.lsc);  // free during the sort
                SegPlan plan{pw, pw + nwin, pw + 2 * nwin, pw + 3 * nwin};
                SALZ_HIP(fill_async(plan.lo, 0xff, sizeof(uint32_t) * nwin, st));
                hipLaunchKernelGGL(k_seg_plan, dim3(grid_for(G_act, kT)), dim3(kT), 0, st, tab.ginfo,
                                   G_act, plan);
                SALZ_LAUNCH_CHECK();
                hipLaunchKernelGGL(k_seg_sort<false>, dim3(nwin), dim3(kSegThreads), 0, st, K, V, nullptr, plan,
                                   tab.ginfo, m, kb, seg_tiny, nullptr, nullptr, derr, 0);
                SALZ_LAUNCH_CHECK();
                if (lg_seg) {
                    if (sort_large_segmented(kb) != 0)
                        return -1;
                } else if (mL) {
                    uint32_t *tmap = pw + 4 * nwin;  // (lsc, after the window plan)
                    const uint32_t ntile = grid_for(mL, kT);
                    hipLaunchKernelGGL(k_tile_lg, dim3(grid_for(ntile, kT)), dim3(kT), 0, st, tab.lrec, GL, mL, tmap);
                    SALZ_LAUNCH_CHECK();
                    hipLaunchKernelGGL(k_extract, dim3(ntile), dim3(kT), 0, st, K, V, tab.lrec, tmap, GL, m, mL, kb,
                                       KC, VC, derr);
                    SALZ_LAUNCH_CHECK();
                    uint64_t *KS = KC;
                    uint32_t *VS = VC;
                    if (radix_sort_pairs(&KS, &VS, Kx, Vx, mL, 0, bits_large, ws, st, nullptr, nullptr, nullptr, rdig,
                                         false, true) != 0)
                        return -1;
                    hipLaunchKernelGGL(k_putback, dim3(grid_for(mL, kT)), dim3(kT), 0, st, KS, VS,
                                       tab.lrec, tab.lg2g, mL, GL, m, kb, K, V, derr);
                    SALZ_LAUNCH_CHECK();
                }
            }
        }
        Kx = (K == ws.keyA) ? ws.keyB : ws.keyA;
        Vx = (V == ws.valA) ? ws.valB : ws.valA;

        if (dbg_rounds && textr) {
            hipLaunchKernelGGL(k_dbg_text, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, gin, tmapped, m, bl, alpha,
                               h / 2, derr);
            SALZ_LAUNCH_CHECK();
        }
        if (dbg_rounds && !seg_round && bl.nb == 1) {
            hipLaunchKernelGGL(k_dbg_sorted, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, m, derr, 0x1000u);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_dbg_pairs, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, ws.rank, ws.text, m,
                               bl, alpha, h / 2, kb, round0, derr);
            SALZ_LAUNCH_CHECK();
        }
        if (ws.lcps_ok && !round0 && h / 2 > kLcpMaxHk)
            ws.lcps_ok = false;  // long repeats: the PLCP stage is cheaper than these compares
        if (textr)
            hipLaunchKernelGGL(k_heads_text, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, gin, hb, offo, m, alpha,
                               h / 2, ws.lcps_ok ? ws.lcps : nullptr);
        else if (ws.lcps_ok)
            hipLaunchKernelGGL(k_heads_lcp, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, hb, offo, m, bl,
                               alpha, kb_old, round0 ? 0u : h / 2, round0, ws.text, ws.lcps, derr, twin, twin_d);
        else
            hipLaunchKernelGGL(k_heads, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, m, bl, h0, round0,
                               hb);
        SALZ_LAUNCH_CHECK();
        if (twin) {
            hipLaunchKernelGGL(k_twin_pairs, dim3(grid_for(((size_t)m + 63) / 64 * 64, kT)), dim3(kT), 0, st, V, K,
                               textr ? gin : nullptr, offo, kb_old, round0, hb, m, twin_d, twin,
                               ws.lcps_ok ? ws.lcps : nullptr);
            SALZ_LAUNCH_CHECK();
        }
        if (scan_sum_u32(hb.wcnt, hb.wpre, ((size_t)m + 63) / 64, false, d32 + 0, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_headpos, dim3(grid_for(((size_t)m + 64 * kHpWords - 1) / (64 * kHpWords) * 64, kT)),
                           dim3(kT), 0, st, hb, m, headpos);
        SALZ_LAUNCH_CHECK();
        // The host needs G only for the debug checks; no round waits for it.
        const bool need_G = dbg_rounds || verbose;
        uint32_t G = 0;
        if (need_G) {
            if (read_scalars(ws, 0, 64, "sa.G") != 0)
                return -1;
            G = reinterpret_cast<uint32_t *>(ws.hscal)[0];
        }
        if (dbg_rounds) {
            hipLaunchKernelGGL(k_dbg_heads, dim3(grid_for(m, kT)), dim3(kT), 0, st, hb, headpos, m, derr);
            SALZ_LAUNCH_CHECK();
        }

        // Survivor counts per wave of the list (u1: free once round 0's text pass is done; u0
        // holds the head ballots until k_commit), scanned: d64[0] = survivors << 32 | groups.
        // d64[1] counts the large groups (size << 32 | 1 per group, k_commit's atomics).
        uint64_t *P = reinterpret_cast<uint64_t *>(ws.u1);
        {
            const size_t nw = ((size_t)m + 63) / 64;
            hipLaunchKernelGGL(k_surv, dim3(grid_for(nw, kT)), dim3(kT), 0, st, hb, m, P, d64 + 1);
            SALZ_LAUNCH_CHECK();
            if (scan_sum_u64(P, P, nw, false, d64, ws, st) != 0)
                return -1;
        }
        // Rank updates:
        //   direct  k_commit writes rank[i] (small rounds);
        //   split   k_commit writes the lower text part, k_rank_upper passes the rest, parts of
        //           at most ~200 MB of rank array each (Infinity-Cache-sized windows);
        //   stage   every update binned by text window and applied window by window
        //           (scatter_staged, XCD-aware), for rank arrays far past the cache.
        // Default: up to 512 MB of ranks split from 32M updates, above it stage from 4M, 1 MB
        // windows (Fibonacci 256 MiB: SA 554 -> 505 ms; text 100 MB: SA 24.8 ms split, 25.3
        // staged; profiles/r02l_*). With round 6's LDS-ordered staging tiles C2's rounds after
        // the text round staged come out even with the split (3765 / 3765 against 3785 / 3752 MB/s
        // on one box, profiles/r06t_staged_scatter_ab.txt).
        int mode = (uint64_t)n * 4 <= (512ull << 20) ? (m >= (32u << 20) ? 1 : 0) : (m >= (4u << 20) ? 2 : 0);
        // round 0 before the text round writes only the ranks of the suffixes it finishes
        const bool textnext = round0 && text1;
        if (textnext && mode == 1)
            mode = 0;
        const uint32_t parts_all = (uint32_t)(((uint64_t)n * 4 + (200u << 20) - 1) / (200u << 20));
        const uint32_t parts = mode == 1 ? (parts_all > 1 ? parts_all : 2) : 1;
        const uint32_t span = (uint32_t)(((uint64_t)n + parts - 1) / parts);
        uint32_t *later = reinterpret_cast<uint32_t *>(Kx);  // free until k_keys
        const uint32_t ihi = mode == 0 ? 0xffffffffu : mode == 1 ? span : 0u;
        // (the text round's keys with the survivors' entries, where Kx is not the rank list: round
        // 5, C2 SA -0.35 ms against the separate gather, which staged blocks keep)
        const bool fuse_keys = textnext && mode == 0;
        const TextNext tn{tmapped, fuse_keys ? Kx : nullptr, bl, alpha, h};
        hipLaunchKernelGGL(k_commit, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, hb, headpos,
                           P, reinterpret_cast<unsigned long long *>(d64 + 1), offo, offn, Vx, textnext ? gin : ngid,
                           ws.rank, ws.sa, tab, m, n, nsa, kb_old, round0, derr, ihi, mode ? later : nullptr,
                           dist ? dist->gbase : 0u, textr ? gin : nullptr, textnext ? 0 : 1, tn);
        SALZ_LAUNCH_CHECK();
        for (uint32_t q = 1; q < parts; q++) {
            hipLaunchKernelGGL(k_rank_upper, dim3(grid_for(m, kT)), dim3(kT), 0, st, V, later, m,
                               q * span, q + 1 == parts ? 0xffffffffu : (q + 1) * span, ws.rank);
            SALZ_LAUNCH_CHECK();
        }
        if (mode == 2) {  // (pst is free after this round's sort)
            if (scatter_staged(LaterSrc{V, later}, m, n, ws.rank, 1u, 0u, reinterpret_cast<uint2 *>(ws.pst),
                               ws.cap_s, ws.radix_counts, st) != 0)
                return -1;
        }
        // A split block's ranks leave together: a local failure is folded into the round's
        // allreduce (bit 48 and up count failed ranks) instead of leaving the others blocked.
        bool failed = read_scalars(ws, 0, 256, "sa.m") != 0;
        if (!failed) {
            if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
                set_error("suffix sort: device index check failed (code 0x%x, round %d)", e,
                          ws.stats.sa_rounds);
                failed = true;
            }
        }
        if (failed && !dist)
            return -1;
        const uint64_t tot = failed ? 0 : ws.hscal[8], ltot = failed ? 0 : ws.hscal[9];
        const uint32_t Gnew = (uint32_t)tot, mnew = (uint32_t)(tot >> 32);
        if (!failed && mnew && (h >= n || Gnew == 0)) {
            set_error("suffix sort did not converge (h=%u n=%u m=%u)", h, n, mnew);
            if (!dist)
                return -1;
            failed = true;
        }
        if (verbose) {  // the round's wall time (this round synchronised with the host twice)
            const auto now = std::chrono::steady_clock::now();
            fprintf(stderr, "sa round %d (%s) h=%u m=%u (large %u in %u groups) groups=%u -> "
                    "survivors %u in %u groups  %.3f ms\n", ws.stats.sa_rounds, how, h, m, mL, GL, G,
                    mnew, Gnew, std::chrono::duration<double, std::milli>(now - t_round).count());
            t_round = now;
        }
        if (dist) {  // a split block ends when every rank's bucket is sorted
            constexpr uint64_t kFailedRank = 1ull << 48;
            uint64_t g = failed ? kFailedRank : mnew;
            if (!dist->local && dist->x->allreduce_sum(&g) != 0) {
                set_error("split suffix sort: allreduce failed");
                return -1;
            }
            if (failed)
                return -1;
            if (g >= kFailedRank) {
                set_error("split suffix sort: %llu other rank(s) failed in round %d",
                          (unsigned long long)(g >> 48), ws.stats.sa_rounds);
                return -1;
            }
            if (g == 0)
                break;
            if (mnew == 0) {  // sorted here: keep answering the other ranks' rank requests
                if (dist_idle_rounds(ws, *dist, ws.stats.sa_rounds - 1) != 0)
                    return -1;
                break;
            }
        } else if (mnew == 0) {
            break;
        }
        if (dc3_auto && h >= 32 && (uint64_t)mnew * 4 > (uint64_t)n * 3)
            return stage_suffix_array_dc3(ws, bl, codes, codes_raw);
        if (textnext && fuse_keys) {
            // (written by k_commit)
        } else if (textnext) {  // the text round's keys: the h0 symbols at i + h0 (every rank holds the text)
            hipLaunchKernelGGL(k_keys_text, dim3(grid_for(mnew, kT)), dim3(kT), 0, st, Vx, mnew, bl, alpha, h,
                               tmapped, Kx);
            SALZ_LAUNCH_CHECK();
        } else if (dist && !dist->local) {  // rank[i + h] lives with the rank that owns suffix i + h
            if (dist_keys(ws, *dist, Vx, ngid, mnew, h, kb, Kx) != 0)
                return -1;
        } else {
            hipLaunchKernelGGL(k_keys, dim3(grid_for(mnew, kT)), dim3(kT), 0, st, Vx, ngid, ws.rank,
                               mnew, n, h, kb, Kx, derr);
            SALZ_LAUNCH_CHECK();
        }
        K = Kx;
        V = Vx;
        m = mnew;
        G_act = Gnew;
        GL = (uint32_t)ltot;
        mL = (uint32_t)(ltot >> 32);
        lgtiles = failed ? 0u : (uint32_t)ws.hscal[10];
        kb_old = kb;
        round0 = 0;
        h = (h > 0x7fffffffu) ? 0xffffffffu : 2 * h;
        uint32_t *t = offo;
        offo = offn;
        offn = t;
    }
    static const bool check = env_flag("SALZ_CHECK", "sa");
    if (check && !dist) {
        SALZ_HIP(fill_async(ws.u0, 0, sizeof(uint32_t) * n, st));
        hipLaunchKernelGGL(k_sa_check, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, ws.sa, nsa, n, ws.u0, derr);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 256, "sa.check") != 0)
            return -1;
        if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
            set_error("suffix sort: result is not a permutation (code 0x%x, %d rounds)", e,
                      ws.stats.sa_rounds);
            return -1;
        }
    }
    return 0;
}

}  // namespace salz
