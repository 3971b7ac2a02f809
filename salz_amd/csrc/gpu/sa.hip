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
//   k_heads     group-head flags of the sorted active list
//   scan        -> group ids; k_headpos -> head index per group
//   k_grpkeep   groups of size >= 2 survive; u64 scan packs (new gid, compact start)
//   k_commit    rank update for every active suffix, SA write for singletons, compaction
//   k_keys      next round's keys: gid << kb | rank[i + h]
#include "internal.hpp"

#include <cstdlib>

namespace salz {
namespace {

constexpr int kT = 256;

__global__ void k_sa_init(const uint8_t *__restrict__ T, uint32_t n, uint64_t *__restrict__ key,
                          uint32_t *__restrict__ val)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= n)
        return;
    uint32_t s = n < 7 ? n : 7;
    uint32_t i = c < s ? (n - 1u - (uint32_t)c) : ((uint32_t)c - s);
    uint64_t w = load_u64_any(T, i);
    uint32_t left = n - i;
    if (left < 8)
        w &= (1ull << (8u * left)) - 1ull;
    key[c] = __builtin_bswap64(w);
    val[c] = i;
}

__global__ void k_heads(const uint64_t *__restrict__ key, const uint32_t *__restrict__ val,
                        uint32_t m, uint32_t n, int round0, uint32_t *__restrict__ hf)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    bool h = c == 0 || key[c] != key[c - 1];
    if (round0 && !h)
        h = (n - val[c]) < 8u || (n - val[c - 1]) < 8u;
    hf[c] = h ? 1u : 0u;
}

__global__ void k_headpos(const uint32_t *__restrict__ hf, const uint32_t *__restrict__ gall,
                          uint32_t m, uint32_t *__restrict__ headpos)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    if (hf[c])
        headpos[gall[c] - 1u] = (uint32_t)c;
    if (c == m - 1)
        headpos[gall[c]] = m;
}

__global__ void k_grpkeep(const uint32_t *__restrict__ headpos, uint32_t G,
                          uint64_t *__restrict__ gsc)
{
    size_t g = (size_t)blockIdx.x * kT + threadIdx.x;
    if (g >= G)
        return;
    uint32_t size = headpos[g + 1] - headpos[g];
    gsc[g] = size >= 2 ? (((uint64_t)size << 32) | 1ull) : 0ull;
}

__global__ void k_commit(const uint64_t *__restrict__ key, const uint32_t *__restrict__ val,
                         const uint32_t *__restrict__ gall, const uint32_t *__restrict__ headpos,
                         const uint64_t *__restrict__ gsc, const uint32_t *__restrict__ off_old,
                         uint32_t *__restrict__ off_new, uint32_t *__restrict__ nval,
                         uint32_t *__restrict__ ngid, uint32_t *__restrict__ rank,
                         uint32_t *__restrict__ sa, uint32_t m, int kb_old, int round0)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    uint32_t g = gall[c] - 1u;
    uint32_t hp = headpos[g];
    uint32_t size = headpos[g + 1] - hp;
    uint32_t o = round0 ? 0u : off_old[(uint32_t)(key[c] >> kb_old)];
    uint32_t i = val[c];
    // The first subgroup of an old group keeps the old group's head, so its members' ranks
    // are unchanged; every other rank (and all of round 0) is written.
    const bool same = !round0 && (hp == 0 || (key[hp - 1] >> kb_old) != (key[hp] >> kb_old));
    if (!same)
        rank[i] = hp + o + 1u;
    if (size == 1) {
        sa[c + o] = i;
    } else {
        uint64_t p = gsc[g];
        uint32_t ng = (uint32_t)p, cs = (uint32_t)(p >> 32);
        uint32_t idx = cs + ((uint32_t)c - hp);
        nval[idx] = i;
        ngid[idx] = ng;
        if ((uint32_t)c == hp)
            off_new[ng] = hp + o - cs;
    }
}

__global__ void k_keys(const uint32_t *__restrict__ nval, const uint32_t *__restrict__ ngid,
                       const uint32_t *__restrict__ rank, uint32_t m, uint32_t h, int kb,
                       uint64_t *__restrict__ key)
{
    size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    uint32_t i = nval[c];
    key[c] = ((uint64_t)ngid[c] << kb) | (uint64_t)rank[i + h];
}

}  // namespace

int stage_suffix_array(Workspace &ws, uint32_t n)
{
    hipStream_t st = ws.stream;
    if (n == 0)
        return 0;
    uint64_t *K = ws.keyA;
    uint32_t *V = ws.valA;
    uint32_t *offo = ws.offA, *offn = ws.offB;
    uint32_t *hf = ws.u0, *gall = ws.u1, *headpos = ws.u2, *ngid = ws.u3;
    uint64_t *gsc = ws.g64;
    uint32_t *d32 = reinterpret_cast<uint32_t *>(ws.dscal);
    uint64_t *d64 = ws.dscal + 8;

    SALZ_HIP(hipMemsetAsync(ws.rank + n, 0, sizeof(uint32_t), st));  // rank[n] = 0
    hipLaunchKernelGGL(k_sa_init, dim3(grid_for(n, kT)), dim3(kT), 0, st, ws.text, n, K, V);
    SALZ_LAUNCH_CHECK();

    uint32_t m = n, h = 8;
    int bits = 64, kb_old = 0, round0 = 1;
    const int kb = bit_width(n);
    ws.stats.sa_rounds = 0;
    static const bool verbose = getenv("SALZ_DEBUG_SA") != nullptr;
    ws.stats.sa_sorted_elems = 0;
    for (;;) {
        ws.stats.sa_rounds++;
        ws.stats.sa_sorted_elems += m;
        uint64_t *Kx = (K == ws.keyA) ? ws.keyB : ws.keyA;
        uint32_t *Vx = (V == ws.valA) ? ws.valB : ws.valA;
        if (radix_sort_pairs(&K, &V, Kx, Vx, m, 0, bits, ws, st) != 0)
            return -1;
        Kx = (K == ws.keyA) ? ws.keyB : ws.keyA;
        Vx = (V == ws.valA) ? ws.valB : ws.valA;

        hipLaunchKernelGGL(k_heads, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, m, n, round0,
                           hf);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(hf, gall, m, true, d32 + 0, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_headpos, dim3(grid_for(m, kT)), dim3(kT), 0, st, hf, gall, m,
                           headpos);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 64, "sa.G") != 0)
            return -1;
        uint32_t G = reinterpret_cast<uint32_t *>(ws.hscal)[0];

        hipLaunchKernelGGL(k_grpkeep, dim3(grid_for(G, kT)), dim3(kT), 0, st, headpos, G, gsc);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u64(gsc, gsc, G, false, d64, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_commit, dim3(grid_for(m, kT)), dim3(kT), 0, st, K, V, gall,
                           headpos, gsc, offo, offn, Vx, ngid, ws.rank, ws.sa, m, kb_old, round0);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 128, "sa.m") != 0)
            return -1;
        uint64_t tot = ws.hscal[8];
        uint32_t Gnew = (uint32_t)tot, mnew = (uint32_t)(tot >> 32);
        if (verbose)
            fprintf(stderr, "sa round %d h=%u m=%u bits=%d groups=%u -> survivors %u in %u groups\n",
                    ws.stats.sa_rounds, h, m, bits, G, mnew, Gnew);
        if (mnew == 0)
            break;
        if (h >= n || Gnew == 0) {
            set_error("suffix sort did not converge (h=%u n=%u m=%u)", h, n, mnew);
            return -1;
        }
        hipLaunchKernelGGL(k_keys, dim3(grid_for(mnew, kT)), dim3(kT), 0, st, Vx, ngid, ws.rank,
                           mnew, h, kb, Kx);
        SALZ_LAUNCH_CHECK();
        K = Kx;
        V = Vx;
        m = mnew;
        bits = kb + bit_width(Gnew - 1);
        kb_old = kb;
        round0 = 0;
        h = (h > 0x7fffffffu) ? 0xffffffffu : 2 * h;
        uint32_t *t = offo;
        offo = offn;
        offn = t;
    }
    return 0;
}

}  // namespace salz
