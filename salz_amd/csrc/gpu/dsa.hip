// dsa.hip - one block's suffix array split over several GPUs.
//
// Replaces libsais() at /root/reference/lib/salz.c:463-469 when one block is spread over a
// node's GPUs. Every rank holds the whole block. The suffixes are bucketed by their first two
// bytes: the 65536 classes are cut into nranks contiguous ranges of about N / nranks suffixes,
// the same plan on every rank, so rank r's bucket is SA[offsets[r] .. offsets[r + 1]) and no
// group of equal prefixes ever spans two ranks. Each rank then runs the single-GPU prefix
// doubling (sa.hip) on its own suffixes, with global ranks (bucket offset + position). The one
// thing a rank cannot compute alone is rank[i + h] for a suffix i + h of another bucket, once
// per doubling round; those requests go to the owning rank and come back through the caller's
// all-to-all (RCCL over xGMI; gloo in the tests):
//   k_dist_req     per surviving suffix: (owner of i + h) << 32 | i + h, value = list slot
//   radix pass     on the owner bits: requests grouped by destination, in slot order
//   all-to-all     requests out, then k_dist_answer (rank[j] of the received j) and back
//   k_dist_place   next round's key of each slot from its answer
// Ranks whose bucket is sorted keep answering until an allreduce of the survivors is 0.
#include "internal.hpp"

#include <cstring>
#include <vector>

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kClasses = 65536;
constexpr uint32_t kClassPart = 16384;  // classes counted per pass (64 KB of LDS counters)

__device__ __forceinline__ uint32_t two_byte_class(const uint8_t *T, uint32_t i, uint32_t n)
{
    return ((uint32_t)T[i] << 8) | (i + 1 < n ? (uint32_t)T[i + 1] : 0u);
}

// Histogram of the two-byte classes of suffixes 0..n-1 in [lo, lo + kClassPart), LDS-privatised.
__global__ __launch_bounds__(kT) void k_class_hist(const uint8_t *__restrict__ T, uint32_t n, uint32_t lo,
                                                   uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[kClassPart];
    for (uint32_t k = threadIdx.x; k < kClassPart; k += kT)
        h[k] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * kT + threadIdx.x; i < n; i += (size_t)gridDim.x * kT) {
        const uint32_t c = two_byte_class(T, (uint32_t)i, n) - lo;
        if (c < kClassPart)
            atomicAdd(&h[c], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kClassPart; k += kT)
        if (h[k])
            atomicAdd(&hist[lo + k], h[k]);
}

// Own long suffixes (8 or more bytes left), flagged for compaction in text order.
__global__ void k_own_flags(const uint8_t *__restrict__ T, uint32_t n, uint32_t nlong,
                            const uint8_t *__restrict__ owner, int rank, uint32_t *__restrict__ flag)
{
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i < nlong)
        flag[i] = owner[two_byte_class(T, (uint32_t)i, n)] == (uint8_t)rank ? 1u : 0u;
}

__global__ void k_own_list(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ idx, uint32_t nlong,
                           uint32_t s0, uint32_t *__restrict__ list)
{
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i < nlong && flag[i])
        list[s0 + idx[i]] = (uint32_t)i;
}

// Requests for rank[i + h]: key = owner << 32 | j (j = i + h; j = n, the end of text, is
// answered by this rank itself: rank[n] = 0 everywhere), value = list slot.
__global__ void k_dist_req(const uint32_t *__restrict__ nval, uint32_t m, uint32_t h, uint32_t n,
                           const uint8_t *__restrict__ T, const uint8_t *__restrict__ owner, int rank,
                           uint64_t *__restrict__ key, uint32_t *__restrict__ val, uint32_t *err)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    uint32_t j = nval[c] + h;
    if (bad_index(j > n, err, kErrKeys))
        j = n;
    const uint32_t d = j < n ? owner[two_byte_class(T, j, n)] : (uint32_t)rank;
    key[c] = ((uint64_t)d << 32) | j;
    val[c] = (uint32_t)c;
}

// The packed request words, and where each destination's run starts in the list (sorted by
// destination): start[d] for d in (dest(c - 1), dest(c)] is c; past the last one, m.
__global__ void k_dist_pack(const uint64_t *__restrict__ key, uint32_t m, uint32_t nranks,
                            uint32_t *__restrict__ words, unsigned long long *__restrict__ start)
{
    const size_t c = (size_t)blockIdx.x * kT + threadIdx.x;
    if (c >= m)
        return;
    const uint64_t k = key[c];
    words[c] = (uint32_t)k;
    const uint32_t d = (uint32_t)(k >> 32);
    const int dp = c ? (int)(uint32_t)(key[c - 1] >> 32) : -1;
    for (int e = dp + 1; e <= (int)d; e++)
        start[e] = c;
    if (c + 1 == m)
        for (uint32_t e = d + 1; e <= nranks; e++)
            start[e] = m;
}

__global__ void k_dist_answer(const uint32_t *__restrict__ req, uint64_t total, uint32_t n,
                              const uint32_t *__restrict__ rank, uint32_t *__restrict__ ans, uint32_t *err)
{
    const size_t k = (size_t)blockIdx.x * kT + threadIdx.x;
    if (k >= total)
        return;
    const uint32_t j = req[k];
    if (bad_index(j > n, err, kErrKeys)) {
        ans[k] = 0;
        return;
    }
    ans[k] = rank[j];
}

__global__ void k_dist_place(const uint32_t *__restrict__ slot, const uint32_t *__restrict__ ans, uint32_t m,
                             const uint32_t *__restrict__ ngid, int kb, uint64_t *__restrict__ key)
{
    const size_t k = (size_t)blockIdx.x * kT + threadIdx.x;
    if (k >= m)
        return;
    const uint32_t c = slot[k];
    key[c] = ((uint64_t)ngid[c] << kb) | ans[k];
}

// Answers the other ranks' requests (xsend = rank[xrecv]) for one exchange pair.
int dist_answer_round(Workspace &ws, const DistSa &d, const uint64_t *send_counts)
{
    std::vector<uint64_t> recv(d.nranks, 0), back(d.nranks, 0);
    if (d.ops->alltoall(d.ops->user, send_counts, recv.data()) != 0) {
        set_error("split suffix sort: all-to-all of the rank requests failed");
        return -1;
    }
    uint64_t total = 0;
    for (uint64_t v : recv)
        total += v;
    if (total > d.xcap) {
        set_error("split suffix sort: %llu requests exceed the exchange buffer", (unsigned long long)total);
        return -1;
    }
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    if (total) {
        hipLaunchKernelGGL(k_dist_answer, dim3(grid_for(total, kT)), dim3(kT), 0, ws.stream, d.xrecv, total,
                           d.n, ws.rank, d.xsend, derr);
        SALZ_LAUNCH_CHECK();
    }
    SALZ_HIP(hipStreamSynchronize(ws.stream));
    if (d.ops->alltoall(d.ops->user, recv.data(), back.data()) != 0) {
        set_error("split suffix sort: all-to-all of the rank answers failed");
        return -1;
    }
    for (int r = 0; r < d.nranks; r++)
        if (back[r] != send_counts[r]) {
            set_error("split suffix sort: %llu answers from rank %d for %llu requests",
                      (unsigned long long)back[r], r, (unsigned long long)send_counts[r]);
            return -1;
        }
    return 0;
}

}  // namespace

int dist_keys(Workspace &ws, const DistSa &d, const uint32_t *nval, const uint32_t *ngid, uint32_t m, uint32_t h,
              int kb, uint64_t *key)
{
    hipStream_t st = ws.stream;
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    if (m > d.xcap) {
        set_error("split suffix sort: %u requests exceed the exchange buffer", m);
        return -1;
    }
    // scratch free between a round's commit and the next sort: pst, lsc and cand's first
    // 4 bytes per slot (the group table sits above them)
    uint64_t *rk = ws.pst, *rk_alt = ws.lsc;
    uint32_t *rv = reinterpret_cast<uint32_t *>(ws.cand);
    uint32_t *rv_alt = reinterpret_cast<uint32_t *>(ws.lsc + ws.cap_s);
    hipLaunchKernelGGL(k_dist_req, dim3(grid_for(m, kT)), dim3(kT), 0, st, nval, m, h, d.n, ws.text, d.owner,
                       d.rank, rk, rv, derr);
    SALZ_LAUNCH_CHECK();
    const int obits = bit_width((uint64_t)(d.nranks > 1 ? d.nranks - 1 : 1));
    if (radix_sort_pairs(&rk, &rv, rk_alt, rv_alt, m, 32, 32 + obits, ws, st) != 0)
        return -1;
    unsigned long long *start = reinterpret_cast<unsigned long long *>(ws.dscal) + 400;
    hipLaunchKernelGGL(k_dist_pack, dim3(grid_for(m, kT)), dim3(kT), 0, st, rk, m, (uint32_t)d.nranks, d.xsend,
                       start);
    SALZ_LAUNCH_CHECK();
    if (read_scalars(ws, 400 * 8, ((size_t)d.nranks + 1) * 8, "dsa.counts") != 0)
        return -1;
    std::vector<uint64_t> send(d.nranks);
    for (int r = 0; r < d.nranks; r++)
        send[r] = ws.hscal[400 + r + 1] - ws.hscal[400 + r];
    if (dist_answer_round(ws, d, send.data()) != 0)
        return -1;
    hipLaunchKernelGGL(k_dist_place, dim3(grid_for(m, kT)), dim3(kT), 0, st, rv, d.xrecv, m, ngid, kb, key);
    SALZ_LAUNCH_CHECK();
    return 0;
}

int dist_idle_rounds(Workspace &ws, const DistSa &d)
{
    const std::vector<uint64_t> none(d.nranks, 0);
    for (;;) {
        if (dist_answer_round(ws, d, none.data()) != 0)
            return -1;
        uint64_t g = 0;
        if (d.ops->allreduce_sum(d.ops->user, &g) != 0) {
            set_error("split suffix sort: allreduce failed");
            return -1;
        }
        if (g == 0)
            return 0;
    }
}

// This rank's bucket and its suffix array piece (see the file comment). ws.text holds the block.
int dist_suffix_array(Workspace &ws, uint32_t n, int nranks, int rank, const salz_dist_ops *ops, uint32_t *xsend,
                      uint32_t *xrecv, size_t xcap, uint64_t *offsets, uint32_t *m0_out)
{
    hipStream_t st = ws.stream;
    if (nranks < 1 || nranks > 255 || rank < 0 || rank >= nranks) {
        set_error("split suffix sort: rank %d of %d", rank, nranks);
        return -1;
    }
    if (!ws.dist_owner) {
        // owner byte per class, then the class histogram (its own room: a workspace sized for
        // a small block has fewer than kClasses words in any of its per-slot arrays)
        void *p = nullptr;
        SALZ_HIP(hipMalloc(&p, kClasses + kClasses * sizeof(uint32_t)));
        ws.dist_owner = static_cast<uint8_t *>(p);
    }
    // class histogram, read back; the plan is computed identically on every rank
    uint32_t *hist = reinterpret_cast<uint32_t *>(ws.dist_owner + kClasses);
    SALZ_HIP(hipMemsetAsync(hist, 0, kClasses * sizeof(uint32_t), st));
    const unsigned g = grid_for(n, kT * 64) < 1024u ? grid_for(n, kT * 64) : 1024u;
    for (uint32_t lo = 0; lo < kClasses; lo += kClassPart) {
        hipLaunchKernelGGL(k_class_hist, dim3(g), dim3(kT), 0, st, ws.text, n, lo, hist);
        SALZ_LAUNCH_CHECK();
    }
    std::vector<uint32_t> h(kClasses);
    if (read_device(ws, hist, kClasses * sizeof(uint32_t), h.data()) != 0)
        return -1;
    std::vector<uint8_t> owner(kClasses);
    uint64_t cum = 0;
    int r = 0;
    offsets[0] = 0;
    for (uint32_t c = 0; c < kClasses; c++) {
        // class c starts rank r + 1's bucket once r's share is reached
        while (r + 1 < nranks && cum >= (uint64_t)n * (r + 1) / nranks) {
            r++;
            offsets[r] = cum;
        }
        owner[c] = (uint8_t)r;
        cum += h[c];
    }
    while (r + 1 < nranks)
        offsets[++r] = cum;
    offsets[nranks] = cum;
    if (cum != n) {
        set_error("split suffix sort: class histogram counts %llu of %u suffixes", (unsigned long long)cum, n);
        return -1;
    }
    SALZ_HIP(hipMemcpyAsync(ws.dist_owner, owner.data(), kClasses, hipMemcpyHostToDevice, st));
    // own list (u3): suffixes with fewer than 8 bytes left first, shortest first, then text order
    const uint32_t nlong = n > 7 ? n - 7 : 0;
    uint8_t tail[32] = {0};
    const uint32_t t0 = (n > 16 ? n - 16 : 0) & ~3u;  // 4-byte aligned read
    if (read_device(ws, ws.text + t0, 32, tail) != 0)
        return -1;
    std::vector<uint32_t> shorts;
    for (uint32_t len = 1; len <= 7 && len <= n; len++) {
        const uint32_t i = n - len;
        const uint32_t c = ((uint32_t)tail[i - t0] << 8) | (i + 1 < n ? tail[i + 1 - t0] : 0u);
        if (owner[c] == (uint8_t)rank)
            shorts.push_back(i);
    }
    uint32_t *list = ws.u3;
    if (!shorts.empty())
        SALZ_HIP(hipMemcpyAsync(list, shorts.data(), shorts.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    const uint32_t m0 = (uint32_t)(offsets[rank + 1] - offsets[rank]);
    if (nlong) {
        uint32_t *flag = ws.offA, *idx = ws.offB;
        hipLaunchKernelGGL(k_own_flags, dim3(grid_for(nlong, kT)), dim3(kT), 0, st, ws.text, n, nlong, ws.dist_owner,
                           rank, flag);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(flag, idx, nlong, false, nullptr, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_own_list, dim3(grid_for(nlong, kT)), dim3(kT), 0, st, flag, idx, nlong,
                           (uint32_t)shorts.size(), list);
        SALZ_LAUNCH_CHECK();
    }
    // a round sends at most m0 requests and receives at most one per own suffix, plus j = n
    if ((size_t)m0 + 1 > xcap) {
        set_error("split suffix sort: exchange buffers of %zu words for a bucket of %u", xcap, m0);
        return -1;
    }
    const DistSa d{ops, rank, nranks, ws.dist_owner, list, m0, (uint32_t)offsets[rank], n, xsend, xrecv, xcap};
    if (m0 == 0) {  // an empty bucket still answers the other ranks until they are done
        SALZ_HIP(hipMemsetAsync(ws.rank + n, 0, sizeof(uint32_t), st));
        uint64_t g = 0;
        if (ops->allreduce_sum(ops->user, &g) != 0) {
            set_error("split suffix sort: allreduce failed");
            return -1;
        }
        if (g && dist_idle_rounds(ws, d) != 0)
            return -1;
    } else {
        const Blocks bl{0xffffffffu, 1u, n};
        if (stage_suffix_array(ws, bl, &d) != 0)
            return -1;
    }
    *m0_out = m0;
    return 0;
}

}  // namespace salz
