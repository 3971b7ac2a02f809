// parse.hip - optimal LZ parse (reference: optimize_factorization, lib/salz.c:610-662).
//
// The reference runs one backward min-plus pass: cost[p] = min(9 + cost[p+1],
// w(PSV) + cost[p+lenP], w(NSV) + cost[p+lenN]) in 32-bit signed arithmetic, strict '<',
// candidate order literal, PSV, NSV. Here the text is cut into chunks of kChunk positions,
// one lane per chunk, and the pass is iterated to a fixed point:
//
//   1. every chunk runs the backward pass over its own positions, reading the previous
//      iteration's exact costs for targets beyond its end; per position it records the
//      decision, the first position at or past the chunk end its path reaches (its exit)
//      and the bit sum along the way;
//   2. exact costs of the new decisions: exit targets E form a forest rooted at n; pointer
//      jumping over the compacted E gives their path sums, every other position adds its
//      in-chunk sum to its exit's cost;
//   3. repeat until no decision changes. At that point every decision is the argmin, with
//      the reference's tie order, over exact successor costs, so by backward induction from
//      n it is the reference's decision (DESIGN.md "Parse").
//
// The pointer-jumping snapshots of the final E forest are kept for emission's path marking.
#include "internal.hpp"

#include <cstdlib>
#include <vector>

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kChunk = 512;

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

// token bit + vnibble + offset byte + gr3 length (lib/salz.c:595-608, :632-634)
__device__ __forceinline__ uint32_t factor_bits(uint32_t off, uint32_t len)
{
    return 1u + 8u + 4u * vn_size((off - 1u) >> 8) + ((len - 3u) >> 3) + 4u;
}

__global__ __launch_bounds__(kT) void k_cost_seed(uint32_t *cost, uint32_t n)
{
    size_t q = (size_t)blockIdx.x * kT + threadIdx.x;
    if (q <= n)
        cost[q] = 9u * (n - (uint32_t)q);
}

__global__ __launch_bounds__(kT) void k_parse_chunk(
    const uint4 *__restrict__ cand, const uint32_t *__restrict__ cin, uint32_t *cloc,
    const uint8_t *__restrict__ chold, uint8_t *__restrict__ chnew, uint32_t *ex, uint32_t *sm,
    uint32_t n, uint32_t *__restrict__ changed)
{
    size_t g = (size_t)blockIdx.x * kT + threadIdx.x;
    size_t a64 = g * kChunk;
    if (a64 >= n)
        return;
    const uint32_t a = (uint32_t)a64;
    const uint32_t b = (n - a) < kChunk ? n : a + kChunk;
    uint32_t diff = 0;
    for (uint32_t p = b; p-- > a;) {
        uint32_t nx1 = p + 1;
        uint32_t best = 9u + (nx1 >= b ? cin[nx1] : cloc[nx1]);
        uint32_t len = 1, w = 9;
        uint8_t ch = 0;
        if (p != 0) {
            const uint4 c = cand[p];
            if (c.y >= 3u) {
                uint32_t wf = factor_bits(c.x, c.y), q = p + c.y;
                uint32_t alt = wf + (q >= b ? cin[q] : cloc[q]);
                if ((int32_t)alt < (int32_t)best) {
                    best = alt;
                    len = c.y;
                    w = wf;
                    ch = 1;
                }
            }
            if (c.w >= 3u) {
                uint32_t wf = factor_bits(c.z, c.w), q = p + c.w;
                uint32_t alt = wf + (q >= b ? cin[q] : cloc[q]);
                if ((int32_t)alt < (int32_t)best) {
                    best = alt;
                    len = c.w;
                    w = wf;
                    ch = 2;
                }
            }
        }
        uint32_t nx = p + len;
        if (nx >= b) {
            ex[p] = nx;
            sm[p] = w;
        } else {
            ex[p] = ex[nx];
            sm[p] = w + sm[nx];
        }
        cloc[p] = best;
        chnew[p] = ch;
        diff += ch != chold[p];
    }
    if (diff)
        atomicAdd(changed, diff);
}

__global__ void k_mark_exits(const uint32_t *__restrict__ ex, uint32_t n, uint32_t *eflag)
{
    size_t p = (size_t)blockIdx.x * kT + threadIdx.x;
    if (p < n)
        eflag[ex[p]] = 1u;
    if (p == 0)
        eflag[n] = 1u;
}

__global__ void k_compact_exits(const uint32_t *__restrict__ eflag,
                                const uint32_t *__restrict__ eidx, const uint32_t *__restrict__ ex,
                                const uint32_t *__restrict__ sm, uint32_t n,
                                uint32_t *__restrict__ elist, uint32_t *__restrict__ jt0,
                                uint32_t *__restrict__ js)
{
    size_t q = (size_t)blockIdx.x * kT + threadIdx.x;
    if (q > n || !eflag[q])
        return;
    uint32_t x = eidx[q];
    elist[x] = (uint32_t)q;
    if (q == n) {
        jt0[x] = x;
        js[x] = 0;
    } else {
        jt0[x] = eidx[ex[q]];
        js[x] = sm[q];
    }
}

__global__ void k_jump(const uint32_t *__restrict__ jt, const uint32_t *__restrict__ js,
                       uint32_t *__restrict__ jt2, uint32_t *__restrict__ js2, uint32_t ne)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= ne)
        return;
    uint32_t p = jt[x];
    js2[x] = js[x] + js[p];
    jt2[x] = jt[p];
}

__global__ void k_cost_exits(const uint32_t *__restrict__ elist, const uint32_t *__restrict__ js,
                             uint32_t ne, uint32_t *__restrict__ cost)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x < ne)
        cost[elist[x]] = js[x];
}

__global__ void k_cost_rest(const uint32_t *__restrict__ eflag, const uint32_t *__restrict__ ex,
                            const uint32_t *__restrict__ sm, uint32_t n, uint32_t *cost)
{
    size_t p = (size_t)blockIdx.x * kT + threadIdx.x;
    if (p >= n || eflag[p])
        return;
    cost[p] = sm[p] + cost[ex[p]];
}

static uint32_t host_vn_size(uint32_t v)
{
    static const uint32_t lim[10] = {8u, 72u, 584u, 4680u, 37448u, 299592u, 2396744u,
                                     19173960u, 153391688u, 1227133512u};
    uint32_t k = 1;
    for (int i = 0; i < 10; i++)
        k += v >= lim[i];
    return k;
}

// SALZ_DEBUG_CHECK: verify the exit forest and exact costs of one iteration on the host.
static void debug_check(Workspace &ws, uint32_t n, const uint8_t *dchoice, const uint32_t *dcost,
                        const uint32_t *dex, const uint32_t *dsm, const uint32_t *deflag,
                        const uint32_t *deidx, uint32_t ne, int it)
{
    hipStream_t st = ws.stream;
    (void)hipStreamSynchronize(st);
    std::vector<uint8_t> ch(n);
    std::vector<uint32_t> cost(n + 1), ex(n), sm(n), ef(n + 1), ei(n + 1);
    std::vector<uint4> cand(n);
    (void)hipMemcpy(ch.data(), dchoice, n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cost.data(), dcost, 4ull * (n + 1), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ex.data(), dex, 4ull * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(sm.data(), dsm, 4ull * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ef.data(), deflag, 4ull * (n + 1), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ei.data(), deidx, 4ull * (n + 1), hipMemcpyDeviceToHost);
    (void)hipMemcpy(cand.data(), ws.cand, 16ull * n, hipMemcpyDeviceToHost);
    auto tok = [&](uint32_t p, uint32_t &len, uint32_t &w) {
        len = 1;
        w = 9;
        if (p == 0 || ch[p] == 0)
            return;
        uint4 c = cand[p];
        uint32_t off = ch[p] == 1 ? c.x : c.z;
        len = ch[p] == 1 ? c.y : c.w;
        w = 1u + 8u + 4u * host_vn_size((off - 1u) >> 8) + ((len - 3u) >> 3) + 4u;
    };
    long bad_len = 0, bad_ex = 0, bad_flag = 0, bad_idx = 0, bad_cost = 0;
    std::vector<uint32_t> hc(n + 1);
    hc[n] = 0;
    for (uint32_t p = n; p-- > 0;) {
        uint32_t len, w;
        tok(p, len, w);
        if ((uint64_t)p + len > n) {
            if (!bad_len++)
                fprintf(stderr, "check it=%d: p=%u len=%u beyond n\n", it, p, len);
            hc[p] = 0;
            continue;
        }
        hc[p] = w + hc[p + len];
    }
    std::vector<uint32_t> hflag(n + 1, 0);
    for (uint32_t p = 0; p < n; p++) {
        uint32_t b = (p / kChunk) * kChunk + kChunk;
        if (b > n)
            b = n;
        uint32_t q = p, s = 0, len, w;
        while (q < b) {
            tok(q, len, w);
            s += w;
            q += len;
        }
        if (ex[p] != q || sm[p] != s)
            if (!bad_ex++)
                fprintf(stderr, "check it=%d: p=%u ex %u/%u sm %u/%u\n", it, p, ex[p], q, sm[p], s);
        if (q <= n)
            hflag[q] = 1;
    }
    hflag[n] = 1;
    uint32_t run = 0;
    for (uint32_t q = 0; q <= n; q++) {
        if (hflag[q] != ef[q] && !bad_flag++)
            fprintf(stderr, "check it=%d: eflag[%u] dev %u host %u\n", it, q, ef[q], hflag[q]);
        if (ei[q] != run && !bad_idx++)
            fprintf(stderr, "check it=%d: eidx[%u] dev %u host %u\n", it, q, ei[q], run);
        run += ef[q];
    }
    for (uint32_t p = 0; p <= n; p++)
        if (hc[p] != cost[p] && p > 0 && !bad_cost++)
            fprintf(stderr, "check it=%d: cost[%u] dev %u host %u\n", it, p, cost[p], hc[p]);
    fprintf(stderr, "check it=%d ne=%u host_ne=%u bad: len %ld ex %ld flag %ld idx %ld cost %ld\n", it,
            ne, run, bad_len, bad_ex, bad_flag, bad_idx, bad_cost);
}

}  // namespace

int stage_parse(Workspace &ws, uint32_t n)
{
    hipStream_t st = ws.stream;
    ParseState &ps = ws.parse;
    ps.chunk = kChunk;
    ps.nchunks = (n + kChunk - 1) / kChunk;
    uint32_t *cost[2] = {ws.u0, ws.u1};
    uint8_t *choice[2] = {reinterpret_cast<uint8_t *>(ws.valA), reinterpret_cast<uint8_t *>(ws.valB)};
    uint32_t *ex = ws.u2, *sm = ws.u3, *eflag = ws.offA, *eidx = ws.offB;
    uint32_t *elist = ws.rank;
    uint32_t *js[2] = {reinterpret_cast<uint32_t *>(ws.keyA),
                       reinterpret_cast<uint32_t *>(ws.keyA) + (ws.cap_n + 1)};
    uint32_t *snap = reinterpret_cast<uint32_t *>(ws.keyB);
    const size_t snap_cap = 2 * (ws.cap_n + 1);
    uint32_t *changed = reinterpret_cast<uint32_t *>(ws.dscal) + 48;
    uint32_t *etotal = reinterpret_cast<uint32_t *>(ws.dscal) + 49;

    hipLaunchKernelGGL(k_cost_seed, dim3(grid_for((size_t)n + 1, kT)), dim3(kT), 0, st, cost[0], n);
    SALZ_LAUNCH_CHECK();
    SALZ_HIP(hipMemsetAsync(choice[0], 0xff, n, st));

    ps.n_exit = 0;
    ps.levels = 0;
    int it = 0;
    for (;; it++) {
        const int cur = it & 1;
        uint32_t *cin = cost[cur], *cout = cost[cur ^ 1];
        uint8_t *chold = choice[cur], *chnew = choice[cur ^ 1];
        SALZ_HIP(hipMemsetAsync(changed, 0, 4, st));
        hipLaunchKernelGGL(k_parse_chunk, dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, ws.cand,
                           cin, cout, chold, chnew, ex, sm, n, changed);
        SALZ_LAUNCH_CHECK();
        if (read_scalars(ws, 0, 256, "parse.changed") != 0)
            return -1;
        const uint32_t nchanged = reinterpret_cast<uint32_t *>(ws.hscal)[48];
        if (getenv("SALZ_DEBUG_PARSE"))
            fprintf(stderr, "parse it=%d changed=%u\n", it, nchanged);
        if (nchanged == 0) {
            ps.choice = chnew;
            ps.cost = cin;
            break;
        }
        if (it > 4096) {
            set_error("parse fixed point did not converge");
            return -1;
        }
        // Exact costs for the new decisions.
        SALZ_HIP(hipMemsetAsync(eflag, 0, sizeof(uint32_t) * ((size_t)n + 1), st));
        hipLaunchKernelGGL(k_mark_exits, dim3(grid_for(n, kT)), dim3(kT), 0, st, ex, n, eflag);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(eflag, eidx, (size_t)n + 1, false, etotal, ws, st) != 0)
            return -1;
        if (read_scalars(ws, 0, 256, "parse.ne") != 0)
            return -1;
        const uint32_t ne = reinterpret_cast<uint32_t *>(ws.hscal)[49];
        if (getenv("SALZ_DEBUG_PARSE"))
            fprintf(stderr, "parse it=%d exits=%u\n", it, ne);
        const uint32_t K = (uint32_t)bit_width(ne > 1 ? ne - 1 : 0);
        if ((size_t)(K + 1) * ne > snap_cap) {
            set_error("parse: exit forest too large for snapshot area (|E|=%u)", ne);
            return -1;
        }
        hipLaunchKernelGGL(k_compact_exits, dim3(grid_for((size_t)n + 1, kT)), dim3(kT), 0, st,
                           eflag, eidx, ex, sm, n, elist, snap, js[0]);
        SALZ_LAUNCH_CHECK();
        int jc = 0;
        for (uint32_t k = 0; k < K; k++) {
            hipLaunchKernelGGL(k_jump, dim3(grid_for(ne, kT)), dim3(kT), 0, st, snap + (size_t)k * ne,
                               js[jc], snap + (size_t)(k + 1) * ne, js[jc ^ 1], ne);
            SALZ_LAUNCH_CHECK();
            jc ^= 1;
        }
        hipLaunchKernelGGL(k_cost_exits, dim3(grid_for(ne, kT)), dim3(kT), 0, st, elist, js[jc], ne,
                           cout);
        SALZ_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_cost_rest, dim3(grid_for(n, kT)), dim3(kT), 0, st, eflag, ex, sm, n,
                           cout);
        SALZ_LAUNCH_CHECK();
        static const bool check = getenv("SALZ_DEBUG_CHECK") != nullptr;
        if (check && (it == 1 || it == 5))
            debug_check(ws, n, chnew, cout, ex, sm, eflag, eidx, ne, it);
        ps.n_exit = ne;
        ps.levels = K;
        ps.elist = elist;
        ps.jt0 = snap;
    }
    ps.ex = ex;
    ps.sm = sm;
    ws.stats.parse_iters = it + 1;
    ws.stats.exit_nodes = ps.n_exit;
    return 0;
}

}  // namespace salz
