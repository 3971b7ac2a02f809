// ansv.hip - PSV/NSV candidates and their match lengths, in text order.
//
// Restates build_psvnsv_array + factorize (/root/reference/lib/salz.c:471-560) as an
// all-nearest-smaller-values query over the suffix array:
//   PSV(p) = SA[r'], r' = max{ r' < r : SA[r'] < p },  lenP = min LCP[r'+1 .. r]
//   NSV(p) = SA[r'], r' = min{ r' > r : SA[r'] < p },  lenN = min LCP[r+1 .. r']
// with r = rank(p). -1 (none) gives offset p + 1 and length 0, as the reference stores.
// The stack pass's PSV/NSV are exactly these nearest smaller values and its lengths are
// exact LCPs, so the range minimum reproduces them bit for bit.
//
// One heap-ordered min tree over np2 leaves holds (min SA, min LCP) per node. Each 256-thread
// workgroup builds the bottom 11 levels of its 2048-leaf block in LDS and writes its subtree
// out. Queries are answered first by a linear scan of the kNear neighbouring ranks (most
// nearest smaller values are close; lanes read consecutive LDS words), then the rest walk the
// block's tree as a compacted LDS queue (few, full waves instead of divergent ones); queries
// that leave the block climb the global tree from the block root (k_ansv_global).
// Output cand[p] = {p - PSV, lenP, p - NSV, lenN}, the reference's aux layout (:555-558).
#include "internal.hpp"

#include <cstdio>
#include <cstdlib>

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kB = 2048;  // leaves per workgroup block
constexpr uint32_t kInf = 0xffffffffu;
constexpr uint32_t kNear = 16;  // linear neighbour scan before the tree walk

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// cand is stored in the parse's chunk-interleaved layout (common.hpp, sidx).
__device__ __forceinline__ void put_psv(uint4 *cand, uint32_t klog, uint32_t p, uint32_t psv_pos,
                                        uint32_t len)
{
    uint2 v = psv_pos == kInf ? make_uint2(p + 1u, 0u) : make_uint2(p - psv_pos, len);
    reinterpret_cast<uint2 *>(cand)[2 * sidx(p, klog)] = v;
}

__device__ __forceinline__ void put_nsv(uint4 *cand, uint32_t klog, uint32_t p, uint32_t nsv_pos,
                                        uint32_t len)
{
    uint2 v = nsv_pos == kInf ? make_uint2(p + 1u, 0u) : make_uint2(p - nsv_pos, len);
    reinterpret_cast<uint2 *>(cand)[2 * sidx(p, klog) + 1] = v;
}

__global__ __launch_bounds__(kT) void k_ansv_local(
    const uint32_t *__restrict__ sa, const uint32_t *__restrict__ lcp, uint32_t n, uint32_t np2,
    uint32_t *__restrict__ tsa, uint32_t *__restrict__ tlcp, uint4 *__restrict__ cand,
    uint32_t *__restrict__ qp, uint32_t *__restrict__ qp_len, uint32_t *__restrict__ qn,
    uint32_t *__restrict__ qn_len, uint32_t *__restrict__ qcount, uint32_t klog,
    unsigned long long *prof)
{
    __shared__ uint32_t vsa[2 * kB];
    __shared__ uint32_t vlc[2 * kB];
    const uint32_t tid = threadIdx.x;
    const uint32_t b0 = blockIdx.x * kB;
    // SALZ_PROF_ANSV (diagnostics): per-phase cycle totals of thread 0
    const unsigned long long t0 = prof ? clock64() : 0ull;

    for (uint32_t l = tid; l < kB; l += kT) {
        uint32_t r = b0 + l;
        vsa[kB + l] = r < n ? sa[r] : kInf;
        vlc[kB + l] = r < n ? lcp[r] : kInf;
    }
    __syncthreads();
    for (uint32_t half = kB / 2; half >= 1; half >>= 1) {
        for (uint32_t k = half + tid; k < 2 * half; k += kT) {
            vsa[k] = umin(vsa[2 * k], vsa[2 * k + 1]);
            vlc[k] = umin(vlc[2 * k], vlc[2 * k + 1]);
        }
        __syncthreads();
    }
    // Publish this block's internal nodes into the global heap.
    const uint32_t root = np2 / kB + blockIdx.x;
    for (uint32_t k = 1 + tid; k < kB; k += kT) {
        uint32_t l = 31u - __builtin_clz(k);
        uint32_t g = (root << l) + (k - (1u << l));
        tsa[g] = vsa[k];
        tlcp[g] = vlc[k];
    }

    unsigned long long t1 = 0;
    if (prof) {
        __syncthreads();
        t1 = clock64();
    }
    // Phase 1: most nearest smaller values are a few ranks away. Scan up to kNear neighbours
    // on each side (lanes read consecutive LDS words: no bank conflicts); queue the rest.
    __shared__ uint16_t wq[2 * kB];
    __shared__ uint32_t wq_n;
    if (tid == 0)
        wq_n = 0;
    __syncthreads();
    for (uint32_t l = tid; l < kB; l += kT) {
        const uint32_t r = b0 + l;
        if (r >= n)
            break;
        const uint32_t v = vsa[kB + l];
        uint32_t lmP = vlc[kB + l], hitP = kInf;
        for (uint32_t d = 1; d <= kNear && d <= l; d++) {
            if (vsa[kB + l - d] < v) {
                hitP = l - d;
                break;
            }
            lmP = umin(lmP, vlc[kB + l - d]);
        }
        uint32_t lmN = kInf, hitN = kInf;
        for (uint32_t d = 1; d <= kNear && l + d < kB; d++) {
            lmN = umin(lmN, vlc[kB + l + d]);
            if (vsa[kB + l + d] < v) {
                hitN = l + d;
                break;
            }
        }
        if (hitP != kInf && hitN != kInf) {
            cand[sidx(v, klog)] = make_uint4(v - vsa[kB + hitP], lmP, v - vsa[kB + hitN], lmN);
        } else {
            if (hitP != kInf)
                put_psv(cand, klog, v, vsa[kB + hitP], lmP);
            else
                wq[atomicAdd(&wq_n, 1u)] = (uint16_t)(l << 1);
            if (hitN != kInf)
                put_nsv(cand, klog, v, vsa[kB + hitN], lmN);
            else
                wq[atomicAdd(&wq_n, 1u)] = (uint16_t)(l << 1 | 1u);
        }
    }
    __syncthreads();
    unsigned long long t2 = 0;
    if (prof)
        t2 = clock64();

    // Phase 2: the queued queries walk the block's min-tree; answers outside the block go to
    // the global queues (k_ansv_global continues from the block root).
    const uint32_t nw = wq_n;
    for (uint32_t w = tid; w < nw; w += kT) {
        const uint32_t e = wq[w], l = e >> 1, r = b0 + l;
        const uint32_t v = vsa[kB + l];
        if (!(e & 1u)) {
            // PSV: nearest smaller to the left; LCP minimum over (r', r].
            uint32_t lm = vlc[kB + l], node = kB + l, hit = kInf;
            while (node > 1) {
                if (node & 1u) {
                    uint32_t s = node - 1;
                    if (vsa[s] < v) {
                        while (s < kB) {
                            uint32_t rc = 2 * s + 1;
                            if (vsa[rc] < v) {
                                s = rc;
                            } else {
                                lm = umin(lm, vlc[rc]);
                                s = 2 * s;
                            }
                        }
                        hit = s - kB;
                        break;
                    }
                    lm = umin(lm, vlc[s]);
                }
                node >>= 1;
            }
            if (hit != kInf) {
                put_psv(cand, klog, v, vsa[kB + hit], lm);
            } else {
                uint32_t q = atomicAdd(&qcount[0], 1u);
                qp[q] = r;
                qp_len[q] = lm;
            }
        } else {
            // NSV: nearest smaller to the right; LCP minimum over (r, r'].
            uint32_t lm = kInf, node = kB + l, hit = kInf;
            while (node > 1) {
                if (!(node & 1u)) {
                    uint32_t s = node + 1;
                    if (vsa[s] < v) {
                        while (s < kB) {
                            uint32_t lc = 2 * s;
                            if (vsa[lc] < v) {
                                s = lc;
                            } else {
                                lm = umin(lm, vlc[lc]);
                                s = 2 * s + 1;
                            }
                        }
                        lm = umin(lm, vlc[s]);
                        hit = s - kB;
                        break;
                    }
                    lm = umin(lm, vlc[s]);
                }
                node >>= 1;
            }
            if (hit != kInf) {
                put_nsv(cand, klog, v, vsa[kB + hit], lm);
            } else {
                uint32_t q = atomicAdd(&qcount[1], 1u);
                qn[q] = r;
                qn_len[q] = lm;
            }
        }
    }
    if (prof) {
        __syncthreads();
        if (tid == 0) {
            const unsigned long long t3 = clock64();
            atomicAdd(&prof[0], t1 - t0);
            atomicAdd(&prof[1], t2 - t1);
            atomicAdd(&prof[2], t3 - t2);
            atomicAdd(&prof[3], (unsigned long long)nw);
        }
    }
}

__global__ void k_tree_level(uint32_t *__restrict__ tsa, uint32_t *__restrict__ tlcp,
                             uint32_t lo, uint32_t cnt)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= cnt)
        return;
    uint32_t k = lo + x;
    tsa[k] = umin(tsa[2 * k], tsa[2 * k + 1]);
    tlcp[k] = umin(tlcp[2 * k], tlcp[2 * k + 1]);
}

struct Tree {
    const uint32_t *tsa, *tlcp, *sa, *lcp;
    uint32_t n, np2;
    __device__ __forceinline__ uint32_t vmin(uint32_t k) const
    {
        if (k < np2)
            return tsa[k];
        uint32_t r = k - np2;
        return r < n ? sa[r] : kInf;
    }
    __device__ __forceinline__ uint32_t lmin(uint32_t k) const
    {
        if (k < np2)
            return tlcp[k];
        uint32_t r = k - np2;
        return r < n ? lcp[r] : kInf;
    }
};

// Queries that left their block: continue the climb from the block root.
__global__ void k_ansv_global(Tree t, const uint32_t *__restrict__ q,
                              const uint32_t *__restrict__ qlen, uint32_t nq, int nsv,
                              uint4 *__restrict__ cand, uint32_t klog)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= nq)
        return;
    const uint32_t r = q[x];
    uint32_t lm = qlen[x];
    const uint32_t v = t.sa[r];
    uint32_t node = t.np2 / kB + r / kB, hit = kInf;
    while (node > 1) {
        bool side = nsv ? !(node & 1u) : (node & 1u);
        if (side) {
            uint32_t s = nsv ? node + 1 : node - 1;
            if (t.vmin(s) < v) {
                while (s < t.np2) {
                    uint32_t near = nsv ? 2 * s : 2 * s + 1;  // child adjacent to the query
                    if (t.vmin(near) < v) {
                        s = near;
                    } else {
                        lm = umin(lm, t.lmin(near));
                        s = nsv ? 2 * s + 1 : 2 * s;
                    }
                }
                if (nsv)
                    lm = umin(lm, t.lmin(s));
                hit = s - t.np2;
                break;
            }
            lm = umin(lm, t.lmin(s));
        }
        node >>= 1;
    }
    uint32_t pos = hit == kInf ? kInf : t.sa[hit];
    if (nsv)
        put_nsv(cand, klog, v, pos, lm);
    else
        put_psv(cand, klog, v, pos, lm);
}

__global__ void k_cand_origin(uint4 *cand) { cand[0] = make_uint4(1u, 1u, 1u, 1u); }  // sidx(0) == 0

}  // namespace

int stage_candidates(Workspace &ws, uint32_t n, const uint32_t *lcp)
{
    hipStream_t st = ws.stream;
    uint32_t np2 = kB;
    while (np2 < n)
        np2 <<= 1;
    if ((size_t)np2 * sizeof(uint32_t) > (ws.cap_n + 1) * sizeof(uint64_t)) {
        set_error("ansv: tree does not fit workspace");
        return -1;
    }
    uint32_t *tsa = reinterpret_cast<uint32_t *>(ws.keyA);
    uint32_t *tlcp = reinterpret_cast<uint32_t *>(ws.keyB);
    uint32_t *qp = ws.valA, *qpl = ws.valB, *qn = ws.offA, *qnl = ws.offB;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(ws.dscal) + 40;

    SALZ_HIP(hipMemsetAsync(cnt, 0, 8, st));
    uint32_t nblocks = np2 / kB;
    uint32_t used_blocks = (n + kB - 1) / kB;
    // Blocks past the text only hold +inf leaves: fill their subtree roots directly.
    if (used_blocks < nblocks) {
        // Each unused block root and its descendants would be +inf; only nodes at or above
        // the block-root level are ever read for them, so set those roots to +inf.
        SALZ_HIP(hipMemsetAsync(tsa + nblocks + used_blocks, 0xff,
                                sizeof(uint32_t) * (nblocks - used_blocks), st));
        SALZ_HIP(hipMemsetAsync(tlcp + nblocks + used_blocks, 0xff,
                                sizeof(uint32_t) * (nblocks - used_blocks), st));
    }
    static const bool prof_on = getenv("SALZ_PROF_ANSV") != nullptr;
    unsigned long long *prof = prof_on ? reinterpret_cast<unsigned long long *>(ws.dscal) + 200 : nullptr;
    if (prof)
        SALZ_HIP(hipMemsetAsync(prof, 0, 32, st));
    hipLaunchKernelGGL(k_ansv_local, dim3(used_blocks), dim3(kT), 0, st, ws.sa, lcp, n, np2, tsa,
                       tlcp, ws.cand, qp, qpl, qn, qnl, cnt, ws.klog, prof);
    SALZ_LAUNCH_CHECK();
    if (prof) {
        if (read_scalars(ws, 1600, 32, "ansv.prof") != 0)
            return -1;
        const uint64_t *h = ws.hscal + 200;
        fprintf(stderr, "ansv_local: %u blocks, cycles/block build %.0f near %.0f tree %.0f; "
                "queued %.3f per leaf\n", used_blocks, (double)h[0] / used_blocks,
                (double)h[1] / used_blocks, (double)h[2] / used_blocks, (double)h[3] / n);
    }
    for (uint32_t lo = nblocks / 2; lo >= 1; lo >>= 1) {
        hipLaunchKernelGGL(k_tree_level, dim3(grid_for(lo, kT)), dim3(kT), 0, st, tsa, tlcp, lo,
                           lo);
        SALZ_LAUNCH_CHECK();
    }
    if (read_scalars(ws, 0, 256, "ansv.q") != 0)
        return -1;
    uint32_t nqp = reinterpret_cast<uint32_t *>(ws.hscal)[40];
    uint32_t nqn = reinterpret_cast<uint32_t *>(ws.hscal)[41];
    Tree t{tsa, tlcp, ws.sa, lcp, n, np2};
    if (nqp) {
        hipLaunchKernelGGL(k_ansv_global, dim3(grid_for(nqp, kT)), dim3(kT), 0, st, t, qp, qpl,
                           nqp, 0, ws.cand, ws.klog);
        SALZ_LAUNCH_CHECK();
    }
    if (nqn) {
        hipLaunchKernelGGL(k_ansv_global, dim3(grid_for(nqn, kT)), dim3(kT), 0, st, t, qn, qnl,
                           nqn, 1, ws.cand, ws.klog);
        SALZ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_cand_origin, dim3(1), dim3(1), 0, st, ws.cand);
    SALZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace salz
