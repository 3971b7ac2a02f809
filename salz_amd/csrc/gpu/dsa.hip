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
// Round 1 of a text block (127 or fewer distinct bytes) is keyed by the text at i + h0, which every
// rank holds, so it needs no exchange (sa.hip's text round). With one rank, rank[i + h] is local
// and no collective runs at all (SALZ_SA=xchg forces the exchange there, for measurement).
//
// The collectives (DistXchg): the caller's callbacks (salz_dist_ops: torch.distributed from
// Python, gloo in the tests) or RCCL called from the library on its own stream
// (salz_gpu_dist_comm: no host callback per round; librccl is opened at run time, so the library
// neither links RCCL nor needs its headers to build, for callers that never split a block).
#include "internal.hpp"

#include <dlfcn.h>

#include <cstring>
#include <vector>

// The few RCCL declarations the split sort uses, restated from rccl/rccl.h (ROCm 7.2) so that the
// build needs no RCCL headers: the enums are int-sized in the C ABI.
typedef struct ncclComm *ncclComm_t;
#define NCCL_UNIQUE_ID_BYTES 128
typedef struct {
    char internal[NCCL_UNIQUE_ID_BYTES];
} ncclUniqueId;
typedef int ncclResult_t;
typedef int ncclDataType_t;
typedef int ncclRedOp_t;
constexpr ncclResult_t ncclSuccess = 0;
constexpr ncclDataType_t ncclUint32 = 3, ncclUint64 = 5;
constexpr ncclRedOp_t ncclSum = 0;

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kClasses = 65536;

__device__ __forceinline__ uint32_t two_byte_class(const uint8_t *T, uint32_t i, uint32_t n)
{
    return ((uint32_t)T[i] << 8) | (i + 1 < n ? (uint32_t)T[i + 1] : 0u);
}

// The bucket plan needs the two-byte class histogram only around the bucket boundaries: one pass
// counts the first bytes; then only the suffixes whose first byte holds a boundary (at most
// nranks - 1 byte values) count their second byte. Every other class of a byte has that byte's
// owner. (Round 4 counted all 65536 classes in four passes over the text: 1.1 ms per 100 MB.)
__global__ __launch_bounds__(kT) void k_byte_hist(const uint8_t *__restrict__ T, uint32_t n,
                                                  uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[4][256];  // one copy per wave
    for (uint32_t k = threadIdx.x; k < 4 * 256; k += kT)
        (&h[0][0])[k] = 0;
    __syncthreads();
    uint32_t *mine = h[threadIdx.x >> 6];
    for (size_t i = ((size_t)blockIdx.x * kT + threadIdx.x) * 16; i < n; i += (size_t)gridDim.x * kT * 16) {
        const uint4 x = *reinterpret_cast<const uint4 *>(T + i);  // (padded buffer)
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int b = 0; b < 16; b++)
            if (i + b < n)
                atomicAdd(&mine[(w[b >> 2] >> (8 * (b & 3))) & 255u], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < 256; k += kT) {
        const uint32_t v = h[0][k] + h[1][k] + h[2][k] + h[3][k];
        if (v)
            atomicAdd(&hist[k], v);
    }
}

// Second-byte counts of the suffixes whose first byte is one of the nsplit boundary bytes
// (slot[first byte] = its index, 0xff otherwise): hist2[slot * 256 + second byte].
constexpr uint32_t kMaxSplitBytes = 32;  // per pass (32 KB of LDS counters)
__global__ __launch_bounds__(kT) void k_pair_hist(const uint8_t *__restrict__ T, uint32_t n,
                                                  const uint8_t *__restrict__ slot, uint32_t nsplit,
                                                  uint32_t *__restrict__ hist2)
{
    __shared__ uint32_t h[kMaxSplitBytes * 256];
    __shared__ uint8_t sl[256];
    for (uint32_t k = threadIdx.x; k < nsplit * 256; k += kT)
        h[k] = 0;
    for (uint32_t k = threadIdx.x; k < 256; k += kT)
        sl[k] = slot[k];
    __syncthreads();
    for (size_t i = ((size_t)blockIdx.x * kT + threadIdx.x) * 16; i < n; i += (size_t)gridDim.x * kT * 16) {
        const uint4 x = *reinterpret_cast<const uint4 *>(T + i);  // (padded: byte i + 16 is readable)
        const uint32_t nx = T[i + 16];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const uint32_t c = (w[b >> 2] >> (8 * (b & 3))) & 255u;
            const uint32_t s = sl[c];
            if (s != 0xffu && i + b < n) {
                const uint32_t c2 = b < 15 ? (w[(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 255u : nx;
                atomicAdd(&h[s * 256u + (i + b + 1 < n ? c2 : 0u)], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nsplit * 256; k += kT)
        if (h[k])
            atomicAdd(&hist2[k], h[k]);
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
    if (d.x->alltoall(send_counts, recv.data()) != 0) {
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
    if (d.x->alltoall(recv.data(), back.data()) != 0) {
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

// ---- collectives -------------------------------------------------------------------------------
struct OpsXchg final : DistXchg {
    const salz_dist_ops *ops;
    explicit OpsXchg(const salz_dist_ops *o) : ops(o) {}
    int alltoall(const uint64_t *sc, uint64_t *rc) override { return ops->alltoall(ops->user, sc, rc); }
    int allreduce_sum(uint64_t *v) override { return ops->allreduce_sum(ops->user, v); }
};

// RCCL entry points, opened at run time (the copy already loaded in the process first: torch
// brings its own; then the ROCm one).
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*all_to_all)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl &rccl()
{
    static Rccl r = [] {
        Rccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h)
            h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            return x;
        auto sym = [&](auto &f, const char *name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            return f != nullptr;
        };
        x.ok = sym(x.get_unique_id, "ncclGetUniqueId") && sym(x.comm_init_rank, "ncclCommInitRank") &&
               sym(x.comm_destroy, "ncclCommDestroy") && sym(x.group_start, "ncclGroupStart") &&
               sym(x.group_end, "ncclGroupEnd") && sym(x.send, "ncclSend") && sym(x.recv, "ncclRecv") &&
               sym(x.all_reduce, "ncclAllReduce") && sym(x.all_to_all, "ncclAllToAll") &&
               sym(x.error_string, "ncclGetErrorString");
        return x;
    }();
    return r;
}

}  // namespace

// A communicator of the split suffix sort: RCCL over xGMI between the ranks' GPUs, plus 2 * nranks
// + 1 device words for the counts.
struct DistComm {
    ncclComm_t comm = nullptr;
    int device = 0, nranks = 0, rank = 0;
    uint64_t *dcnt = nullptr;
};

namespace {

#define SALZ_NCCL(expr)                                                                             \
    do {                                                                                            \
        const ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess) {                                                                    \
            set_error("%s:%d: %s -> %s", __FILE__, __LINE__, #expr, rccl().error_string(r_));        \
            return -1;                                                                              \
        }                                                                                           \
    } while (0)

// Where peer r's run starts in the send and receive buffers of one exchange: the runs lie in rank
// order, as in torch.distributed's all_to_all_single with split sizes (the gloo path, dist.py),
// which the grouped sends and receives below must reproduce (tests/test_dist.py checks both).
void xchg_offsets(int nr, const uint64_t *sc, const uint64_t *rc, uint64_t *so, uint64_t *ro)
{
    uint64_t s = 0, r = 0;
    for (int k = 0; k < nr; k++) {
        so[k] = s;
        ro[k] = r;
        s += sc[k];
        r += rc[k];
    }
}

struct RcclXchg final : DistXchg {
    DistComm *c;
    hipStream_t st;
    const uint32_t *xsend;
    uint32_t *xrecv;
    RcclXchg(DistComm *comm, hipStream_t s, const uint32_t *xs, uint32_t *xr) : c(comm), st(s), xsend(xs), xrecv(xr) {}
    // counts through one all-to-all of u64 words (read back: they size the data exchange), then the
    // data as grouped sends and receives on the library's stream
    int alltoall(const uint64_t *sc, uint64_t *rc) override
    {
        const Rccl &R = rccl();
        const int nr = c->nranks;
        SALZ_HIP(hipMemcpyAsync(c->dcnt, sc, (size_t)nr * 8, hipMemcpyHostToDevice, st));
        SALZ_NCCL(R.all_to_all(c->dcnt, c->dcnt + nr, 1, ncclUint64, c->comm, st));
        SALZ_HIP(hipMemcpyAsync(rc, c->dcnt + nr, (size_t)nr * 8, hipMemcpyDeviceToHost, st));
        SALZ_HIP(hipStreamSynchronize(st));
        std::vector<uint64_t> so(nr), ro(nr);
        xchg_offsets(nr, sc, rc, so.data(), ro.data());
        SALZ_NCCL(R.group_start());
        for (int r = 0; r < nr; r++) {
            if (sc[r])
                SALZ_NCCL(R.send(xsend + so[r], sc[r], ncclUint32, r, c->comm, st));
            if (rc[r])
                SALZ_NCCL(R.recv(xrecv + ro[r], rc[r], ncclUint32, r, c->comm, st));
        }
        SALZ_NCCL(R.group_end());
        return 0;
    }
    int allreduce_sum(uint64_t *v) override
    {
        const Rccl &R = rccl();
        uint64_t *d = c->dcnt + 2 * c->nranks;
        SALZ_HIP(hipMemcpyAsync(d, v, 8, hipMemcpyHostToDevice, st));
        SALZ_NCCL(R.all_reduce(d, d, 1, ncclUint64, ncclSum, c->comm, st));
        SALZ_HIP(hipMemcpyAsync(v, d, 8, hipMemcpyDeviceToHost, st));
        SALZ_HIP(hipStreamSynchronize(st));
        return 0;
    }
};

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

int dist_idle_rounds(Workspace &ws, const DistSa &d, int round)
{
    const std::vector<uint64_t> none(d.nranks, 0);
    for (;; round++) {
        // the keys of round + 1 (none to exchange when it is the text round), then its allreduce
        if (!(d.text1 && round == 0) && dist_answer_round(ws, d, none.data()) != 0)
            return -1;
        uint64_t g = 0;
        if (d.x->allreduce_sum(&g) != 0) {
            set_error("split suffix sort: allreduce failed");
            return -1;
        }
        if (g == 0)
            return 0;
    }
}

// This rank's bucket and its suffix array piece (see the file comment). ws.text holds the block.
int dist_suffix_array(Workspace &ws, uint32_t n, int nranks, int rank, DistXchg *x, uint32_t *xsend,
                      uint32_t *xrecv, size_t xcap, uint64_t *offsets, uint32_t *m0_out)
{
    hipStream_t st = ws.stream;
    if (nranks < 1 || nranks > 255 || rank < 0 || rank >= nranks) {
        set_error("split suffix sort: rank %d of %d", rank, nranks);
        return -1;
    }
    // A block the repetition probe sends to DC3 (long repeats everywhere: Fibonacci, periodic or
    // run-heavy blocks) is not split. Every suffix there survives ~log2(max LCP) doubling rounds
    // (26 on C5), each a full-width sort plus an exchange, and the split sorter has no DC3. Every
    // rank sees the same text and takes the same decision: all return 1 and the caller encodes the
    // block whole on one GPU (salz_gpu_encode_device, which takes DC3). Smaller blocks split as
    // usual (prefix doubling, like the single-GPU sorter below 2^20 suffixes).
    {
        const int rep = block_repetitive(ws, n);
        if (rep < 0)
            return -1;
        if (rep) {
            for (int r = 0; r <= nranks; r++)
                offsets[r] = 0;
            *m0_out = 0;
            return 1;
        }
    }
    if (!ws.dist_owner) {
        // owner byte per class, then the class histogram (its own room: a workspace sized for
        // a small block has fewer than kClasses words in any of its per-slot arrays)
        void *p = nullptr;
        SALZ_HIP(hipMalloc(&p, kClasses + kClasses * sizeof(uint32_t)));
        ws.dist_owner = static_cast<uint8_t *>(p);
    }
    // The plan, computed identically on every rank: classes in order, rank r + 1's bucket starts at
    // the first class whose preceding count reaches n (r + 1) / nranks. First-byte counts, then the
    // second-byte counts of the bytes a boundary falls strictly inside (the classes of any other
    // byte all go to one rank).
    uint32_t *hist = reinterpret_cast<uint32_t *>(ws.dist_owner + kClasses);  // 256 + 256 * splits
    SALZ_HIP(hipMemsetAsync(hist, 0, 256 * sizeof(uint32_t), st));
    const unsigned g = grid_for(n, kT * 64) < 1024u ? grid_for(n, kT * 64) : 1024u;
    hipLaunchKernelGGL(k_byte_hist, dim3(g), dim3(kT), 0, st, ws.text, n, hist);
    SALZ_LAUNCH_CHECK();
    std::vector<uint32_t> h1(256);
    if (read_device(ws, hist, 256 * sizeof(uint32_t), h1.data()) != 0)
        return -1;
    std::vector<uint8_t> slot(256, 0xff);
    std::vector<uint32_t> splits;
    {
        uint64_t before = 0;
        for (uint32_t b = 0; b < 256; b++) {
            const uint64_t after = before + h1[b];
            for (int r = 1; r < nranks; r++) {
                const uint64_t t = (uint64_t)n * r / nranks;
                if (before < t && t < after && slot[b] == 0xff) {
                    slot[b] = (uint8_t)splits.size();
                    splits.push_back(b);
                }
            }
            before = after;
        }
    }
    std::vector<uint32_t> h2(splits.size() * 256, 0);
    for (size_t s0 = 0; s0 < splits.size(); s0 += kMaxSplitBytes) {
        const uint32_t ns = (uint32_t)(splits.size() - s0 < kMaxSplitBytes ? splits.size() - s0 : kMaxSplitBytes);
        std::vector<uint8_t> sl(256, 0xff);
        for (uint32_t k = 0; k < ns; k++)
            sl[splits[s0 + k]] = (uint8_t)k;
        uint8_t *dslot = ws.dist_owner;  // (the owner table is written after the plan)
        uint32_t *hist2 = hist + 256;
        SALZ_HIP(hipMemcpyAsync(dslot, sl.data(), 256, hipMemcpyHostToDevice, st));
        SALZ_HIP(hipMemsetAsync(hist2, 0, (size_t)ns * 256 * sizeof(uint32_t), st));
        hipLaunchKernelGGL(k_pair_hist, dim3(g), dim3(kT), 0, st, ws.text, n, dslot, ns, hist2);
        SALZ_LAUNCH_CHECK();
        if (read_device(ws, hist2, (size_t)ns * 256 * sizeof(uint32_t), h2.data() + s0 * 256) != 0)
            return -1;
    }
    std::vector<uint8_t> owner(kClasses);
    uint64_t cum = 0;
    int r = 0;
    offsets[0] = 0;
    auto advance = [&]() {  // boundaries at the current class start
        while (r + 1 < nranks && cum >= (uint64_t)n * (r + 1) / nranks) {
            r++;
            offsets[r] = cum;
        }
    };
    for (uint32_t b = 0; b < 256; b++) {
        if (slot[b] == 0xff) {  // no boundary inside: the byte's classes go to one rank
            advance();
            memset(owner.data() + b * 256u, r, 256);
            cum += h1[b];
            continue;
        }
        for (uint32_t c2 = 0; c2 < 256; c2++) {
            advance();
            owner[b * 256u + c2] = (uint8_t)r;
            cum += h2[(size_t)slot[b] * 256 + c2];
        }
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
    // Round 1 keyed by the text: decided here from the block's alphabet, the same on every rank
    // (an empty bucket's rank too, whose idle rounds must skip that round's exchange with the rest)
    const int abits = block_alpha_bits(ws, n);
    if (abits < 0)
        return -1;
    const bool text1 = abits > 0;
    const bool local = nranks == 1 && !env_flag("SALZ_SA", "xchg");
    const DistSa d{x, rank, nranks, ws.dist_owner, list, m0, (uint32_t)offsets[rank], n, xsend, xrecv, xcap, text1,
                   local};
    if (m0 == 0) {  // an empty bucket still answers the other ranks until they are done
        SALZ_HIP(hipMemsetAsync(ws.rank + n, 0, sizeof(uint32_t), st));
        uint64_t g = 0;
        if (x->allreduce_sum(&g) != 0) {
            set_error("split suffix sort: allreduce failed");
            return -1;
        }
        if (g && dist_idle_rounds(ws, d, 0) != 0)
            return -1;
    } else {
        const Blocks bl{0xffffffffu, 1u, n};
        if (stage_suffix_array(ws, bl, &d) != 0)
            return -1;
    }
    *m0_out = m0;
    return 0;
}

// ---- C ABI --------------------------------------------------------------------------------------
int dist_suffix_array_ops(Workspace &ws, uint32_t n, int nranks, int rank, const salz_dist_ops *ops, uint32_t *xsend,
                          uint32_t *xrecv, size_t xcap, uint64_t *offsets, uint32_t *m0_out)
{
    OpsXchg x(ops);
    return dist_suffix_array(ws, n, nranks, rank, &x, xsend, xrecv, xcap, offsets, m0_out);
}

int dist_suffix_array_comm(Workspace &ws, uint32_t n, DistComm *c, uint32_t *xsend, uint32_t *xrecv, size_t xcap,
                           uint64_t *offsets, uint32_t *m0_out)
{
    if (c->device != ws.device) {
        set_error("split suffix sort: communicator of device %d, context of device %d", c->device, ws.device);
        return -1;
    }
    RcclXchg x(c, ws.stream, xsend, xrecv);
    return dist_suffix_array(ws, n, c->nranks, c->rank, &x, xsend, xrecv, xcap, offsets, m0_out);
}

}  // namespace salz

extern "C" {

int salz_gpu_dist_comm_id(uint8_t *id)
{
    using namespace salz;
    if (!id) {
        set_error("NULL argument");
        return -1;
    }
    if (!rccl().ok) {
        set_error("librccl.so.1 not found (or lacks an entry point): no in-library collectives");
        return -1;
    }
    ncclUniqueId u;
    SALZ_NCCL(rccl().get_unique_id(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

salz_gpu_dist_comm *salz_gpu_dist_comm_create(int device, int nranks, int rank, const uint8_t *id)
{
    using namespace salz;
    if (!id || nranks < 1 || nranks > 255 || rank < 0 || rank >= nranks) {
        set_error("invalid argument");
        return nullptr;
    }
    if (!rccl().ok) {
        set_error("librccl.so.1 not found (or lacks an entry point): no in-library collectives");
        return nullptr;
    }
    int prev = -1;  // the caller's device is restored on every return (as elsewhere in the C ABI)
    (void)hipGetDevice(&prev);
    struct Restore {
        int dev;
        ~Restore()
        {
            if (dev >= 0)
                (void)hipSetDevice(dev);
        }
    } restore{prev};
    if (hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice(%d) failed", device);
        return nullptr;
    }
    auto *c = new DistComm;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess || hipMalloc(reinterpret_cast<void **>(&c->dcnt), (2 * (size_t)nranks + 1) * 8) != hipSuccess) {
        set_error("RCCL communicator (rank %d of %d): %s", rank, nranks,
                  r != ncclSuccess ? rccl().error_string(r) : "hipMalloc failed");
        if (c->comm)
            rccl().comm_destroy(c->comm);
        delete c;
        return nullptr;
    }
    return reinterpret_cast<salz_gpu_dist_comm *>(c);
}

void salz_gpu_dist_comm_destroy(salz_gpu_dist_comm *comm)
{
    using namespace salz;
    auto *c = reinterpret_cast<DistComm *>(comm);
    if (!c)
        return;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    if (c->dcnt)
        (void)hipFree(c->dcnt);
    if (c->comm)
        rccl().comm_destroy(c->comm);
    delete c;
    if (prev >= 0)
        (void)hipSetDevice(prev);
}

// Test hook: the per-peer run offsets of one exchange (xchg_offsets).
int salz_debug_xchg_offsets(int nranks, const uint64_t *send_counts, const uint64_t *recv_counts, uint64_t *send_off,
                            uint64_t *recv_off)
{
    if (nranks < 1 || !send_counts || !recv_counts || !send_off || !recv_off)
        return -1;
    salz::xchg_offsets(nranks, send_counts, recv_counts, send_off, recv_off);
    return 0;
}

}  // extern "C"
