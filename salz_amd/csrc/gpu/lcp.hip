// lcp.hip - LCP array of the suffix array via Phi / irreducible PLCP.
//
// The reference has no LCP pass: it extends each candidate match with 8-byte compares
// seeded by the previous position's length (lib/salz.c:492-538). Its lengths equal the
// exact LCP of the suffix pair in T[0,n), so the GPU path computes the
// exact LCP array once and derives every candidate length from range minima (ansv.hip).
//
//   Phi[SA[r]] = SA[r-1]; PLCP[i] = lcp(i, Phi[i]).
//   i is reducible iff i > 0, Phi[i] > 0 and T[i-1] == T[Phi[i]-1]; then
//   PLCP[i] = PLCP[i-1] - 1. PLCP[i] + i is non-decreasing, so an inclusive max-scan over
//   (irreducible ? PLCP[i] + i : 0) recovers every PLCP value exactly.
// Irreducible values are summed O(n log n) (Kärkkäinen-Manzini-Puglisi); each thread
// compares the first 32 bytes, longer ones go to a work list resolved in doubling windows
// split into 512-byte wave tasks (64 lanes x 8 bytes), so a single 10^8-byte match is
// spread over the whole chip instead of serialising one lane.
#include "internal.hpp"
#include "scatter.hpp"

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kShortBytes = 32;
constexpr uint32_t kTaskBytes = 512;

// A block's first suffix in the suffix array (r = 0, or the previous entry in another block
// of a batch) has no predecessor: PLCP = 0.
__global__ void k_phi(const uint32_t *__restrict__ sa, Blocks bl, uint32_t *__restrict__ phi,
                      uint32_t *err)
{
    size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r >= bl.nsa())
        return;
    const uint32_t i = sa[r];
    if (bad_index(i >= bl.npos, err, kErrPhi))
        return;
    const uint32_t j = r ? sa[r - 1] : kNone;
    phi[i] = j != kNone && bl.blk(j) == bl.blk(i) ? j : kNone;
}

// The same pairs for the staged scatter (scatter.hpp): index SA[r], value Phi.
struct PhiSrc {
    const uint32_t *sa;
    Blocks bl;
    __device__ __forceinline__ bool operator()(size_t r, uint32_t &idx, uint32_t &val) const
    {
        const uint32_t i = sa[r], jr = sa[r ? r - 1 : 0];  // (unconditional loads)
        const uint32_t j = r ? jr : kNone;
        idx = i;
        val = j != kNone && bl.blk(j) == bl.blk(i) ? j : kNone;
        return i < bl.npos;
    }
};

// PLCP[i] of position i by its first kShortBytes bytes: plv[i] = PLCP[i] + i for an irreducible
// i, 0 for a reducible one (the max-scan fills it in); returns true when i needs a longer compare.
__device__ __forceinline__ bool plcp_short_one(const uint8_t *__restrict__ T, const uint32_t *__restrict__ phi,
                                               const Blocks &bl, uint32_t i, uint32_t *__restrict__ plv)
{
    const uint32_t e = bl.end(i), b0 = bl.start(i);
    if (i >= e) {  // a batch's dead position: no suffix (the max-scan carries past it)
        plv[i] = 0;
        return false;
    }
    const uint32_t j = phi[i];
    if (j == kNone) {  // smallest suffix of its block: PLCP = 0
        plv[i] = i;
        return false;
    }
    const bool irr = i == b0 || j == b0 || T[i - 1] != T[j - 1];  // (j is in i's block)
    if (!irr) {
        plv[i] = 0;
        return false;
    }
    const uint32_t limit = e - (i > j ? i : j);
    uint32_t L = 0;
    bool done = false;
#pragma unroll
    for (int w = 0; w < (int)(kShortBytes / 8); w++) {
        if (!done && L < limit) {
            const uint64_t x = load_u64_any(T, (size_t)i + L) ^ load_u64_any(T, (size_t)j + L);
            if (x) {
                L += (uint32_t)__builtin_ctzll(x) >> 3;
                done = true;
            } else {
                L += 8;
            }
        }
    }
    if (L >= limit) {
        L = limit;
        done = true;
    }
    plv[i] = done ? L + i : 0u;
    return !done;
}

// Every position's short compare; the positions left for the long compares are gathered per
// workgroup in LDS and appended to the queue with one global atomic per workgroup (the grid is
// at most kShortGrid workgroups looping over the positions). A global counter bumped per wave
// served ~88 appends per microsecond: runs of 64 equal bytes at 256 MiB queue 4 M positions
// (one per run), which took ~45 ms that way.
constexpr uint32_t kShortGrid = 2048;
constexpr uint32_t kQBuf = 2048;  // LDS queue entries per workgroup before a flush
__global__ __launch_bounds__(kT) void k_plcp_short(const uint8_t *__restrict__ T, const uint32_t *__restrict__ phi,
                                                   Blocks bl, uint32_t *__restrict__ plv, uint32_t *__restrict__ queue,
                                                   uint32_t *__restrict__ qcount)
{
    __shared__ uint32_t lq[kQBuf];
    __shared__ uint32_t ln, lbase;
    const uint32_t tid = threadIdx.x;
    if (tid == 0)
        ln = 0;
    __syncthreads();
    auto flush = [&](uint32_t cnt) {  // (workgroup-uniform)
        if (tid == 0)
            lbase = atomicAdd(qcount, cnt);
        __syncthreads();
        for (uint32_t k = tid; k < cnt; k += kT)
            queue[lbase + k] = lq[k];
        __syncthreads();
        if (tid == 0)
            ln = 0;
        __syncthreads();
    };
    const size_t step = (size_t)gridDim.x * kT;
    for (size_t base = (size_t)blockIdx.x * kT; base < bl.npos; base += step) {  // (uniform bound)
        const size_t ii = base + tid;
        const bool push = ii < bl.npos && plcp_short_one(T, phi, bl, (uint32_t)ii, plv);
        const uint64_t m = wave_ballot(push);
        if (m) {
            const int leader = (int)__ffsll((unsigned long long)m) - 1;
            uint32_t at = 0;
            if ((int)lane_id() == leader)
                at = atomicAdd(&ln, (uint32_t)__popcll(m));
            at = shfl_u32(at, leader);
            if (push)
                lq[at + count_below(m)] = (uint32_t)ii;
        }
        __syncthreads();
        const uint32_t cur = ln;
        __syncthreads();
        if (cur + kT > kQBuf)  // the next round could overflow the buffer
            flush(cur);
    }
    const uint32_t cur = ln;
    __syncthreads();
    if (cur)
        flush(cur);
}

// One wave per 512-byte task: task t -> item t / nch, bytes [L + (t % nch) * 512, +512).
__global__ __launch_bounds__(256) void k_plcp_long(const uint8_t *__restrict__ T,
                                                   const uint32_t *__restrict__ phi, Blocks bl,
                                                   const uint32_t *__restrict__ items,
                                                   uint32_t nitems, uint32_t nch, uint32_t L,
                                                   uint32_t *__restrict__ found)
{
    size_t task = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned lane = threadIdx.x & 63;
    if (task >= (size_t)nitems * nch)
        return;
    uint32_t item = (uint32_t)(task / nch), ch = (uint32_t)(task % nch);
    uint32_t i = items[item], j = phi[i];
    uint32_t limit = bl.end(i) - (i > j ? i : j);
    uint64_t start = (uint64_t)L + (uint64_t)ch * kTaskBytes + (uint64_t)lane * 8;
    uint32_t mis = kNone;
    if (start < limit) {
        uint64_t x = load_u64_any(T, i + start) ^ load_u64_any(T, j + start);
        if (x) {
            uint64_t pos = start + ((uint32_t)__builtin_ctzll(x) >> 3);
            if (pos < limit)
                mis = (uint32_t)pos;
        }
    }
    mis = wave_min_u32(mis);
    if (lane == 0 && mis != kNone)
        atomicMin(&found[item], mis);
}

__global__ void k_plcp_resolve(const uint32_t *__restrict__ phi, Blocks bl,
                               const uint32_t *__restrict__ items, uint32_t nitems,
                               const uint32_t *__restrict__ found, uint64_t window_end,
                               uint32_t *__restrict__ plv, uint32_t *__restrict__ next_items,
                               uint32_t *__restrict__ next_count)
{
    size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    if (x >= nitems)
        return;
    uint32_t i = items[x], j = phi[i];
    uint32_t limit = bl.end(i) - (i > j ? i : j);
    uint32_t f = found[x];
    bool more = false;
    if (f != kNone)
        plv[i] = f + i;
    else if (window_end >= limit)
        plv[i] = limit + i;
    else
        more = true;
    const uint64_t m = wave_ballot(more);  // one atomic per wave
    if (m) {
        const int leader = (int)__ffsll((unsigned long long)m) - 1;
        uint32_t q = 0;
        if ((int)lane_id() == leader)
            q = atomicAdd(next_count, (uint32_t)__popcll(m));
        q = shfl_u32(q, leader);
        if (more)
            next_items[q + count_below(m)] = i;
    }
}

__global__ void k_lcp_final(const uint32_t *__restrict__ sa, const uint32_t *__restrict__ mx,
                            Blocks bl, uint32_t *__restrict__ lcp)
{
    size_t r = (size_t)blockIdx.x * kT + threadIdx.x;
    if (r >= bl.nsa())
        return;
    const uint32_t i = sa[r], j = r ? sa[r - 1] : i;  // (unconditional loads)
    // a block's first suffix has no predecessor: LCP 0 (the max-scan may carry a larger value)
    lcp[r] = r && bl.blk(j) == bl.blk(i) ? mx[i] - i : 0u;
}

}  // namespace

int stage_lcp(Workspace &ws, const Blocks &bl, uint32_t *lcp_out)
{
    const uint32_t n = bl.npos, nsa = bl.nsa();
    hipStream_t st = ws.stream;
    uint32_t *phi = ws.u0, *plv = ws.u1;
    uint32_t *qa = ws.valA, *qb = ws.valB, *found = ws.offA;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(ws.dscal) + 32;  // 2 counters

    ws.stats.lcp_long_bytes = 0;
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    if (scatter_stage_wanted((size_t)n * sizeof(uint32_t))) {  // (lsc and the radix counts are free here)
        if (scatter_staged(PhiSrc{ws.sa, bl}, nsa, n, phi, 1u, 0u, reinterpret_cast<uint2 *>(ws.lsc),
                           2 * ws.cap_s, ws.radix_counts, st) != 0)
            return -1;
    } else {
        hipLaunchKernelGGL(k_phi, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, ws.sa, bl, phi, derr);
        SALZ_LAUNCH_CHECK();
    }
    SALZ_HIP(fill_async(cnt, 0, 8, st));
    hipLaunchKernelGGL(k_plcp_short, dim3(grid_for(n, kT) < kShortGrid ? grid_for(n, kT) : kShortGrid), dim3(kT), 0,
                       st, ws.text, phi, bl, plv, qa, cnt);
    SALZ_LAUNCH_CHECK();
    if (read_scalars(ws, 0, 256, "lcp.q0") != 0)
        return -1;
    if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
        set_error("lcp: device index check failed (code 0x%x): suffix array corrupt", e);
        return -1;
    }
    uint32_t nitems = reinterpret_cast<uint32_t *>(ws.hscal)[32];

    uint64_t L = kShortBytes;
    while (nitems) {
        uint64_t W = L < kTaskBytes ? kTaskBytes : L;
        W = (W + kTaskBytes - 1) / kTaskBytes * kTaskBytes;
        uint32_t nch = (uint32_t)(W / kTaskBytes);
        SALZ_HIP(fill_async(found, 0xff, sizeof(uint32_t) * nitems, st));
        SALZ_HIP(fill_async(cnt + 1, 0, 4, st));
        size_t tasks = (size_t)nitems * nch;
        hipLaunchKernelGGL(k_plcp_long, dim3(grid_for(tasks * 64, 256)), dim3(256), 0, st,
                           ws.text, phi, bl, qa, nitems, nch, (uint32_t)L, found);
        SALZ_LAUNCH_CHECK();
        ws.stats.lcp_long_bytes += tasks * kTaskBytes;
        hipLaunchKernelGGL(k_plcp_resolve, dim3(grid_for(nitems, kT)), dim3(kT), 0, st, phi, bl,
                           qa, nitems, found, L + W, plv, qb, cnt + 1);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 256, "lcp.q") != 0)
            return -1;
        nitems = reinterpret_cast<uint32_t *>(ws.hscal)[33];
        uint32_t *t = qa;
        qa = qb;
        qb = t;
        L += W;
    }

    if (scan_max_u32(plv, plv, n, true, nullptr, ws, st) != 0)
        return -1;
    hipLaunchKernelGGL(k_lcp_final, dim3(grid_for(nsa, kT)), dim3(kT), 0, st, ws.sa, plv, bl,
                       lcp_out);
    SALZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace salz
