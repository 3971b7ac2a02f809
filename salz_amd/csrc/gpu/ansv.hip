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
//
// The answers come out in rank order but cand is indexed by text position, so writing them
// directly is a 16-byte random scatter over the whole 16n-byte array (1.6 GB at 100 MB, beyond
// the 256 MB Infinity Cache). Instead each workgroup appends its answers to per-text-range
// staging runs (ranges of 2^rlog positions, one global atomic per range and workgroup; the
// queries that leave the block keep their staging slot and k_ansv_global answers into it), and
// k_cand_scatter moves the staged answers range by range: its concurrent writes then all fall
// in one cache-resident window of the candidate array.
#include "internal.hpp"

#include <cstdio>
#include <cstdlib>

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kB = 2048;  // leaves per workgroup block
constexpr uint32_t kInf = 0xffffffffu;
constexpr uint32_t kNear = 16;  // linear neighbour scan before the tree walk
constexpr uint32_t kScan = 8;   // leaves under the deepest global tree node (scanned by the global walk)
constexpr uint32_t kWQ = 1408;  // LDS walk-queue entries per block
// Global-queue shards (blockIdx mod kShards), each with its own counter: about as many as
// workgroups are resident at once, so concurrent blocks append to different words. With 16
// shards, blocks whose queries nearly all leave them (a sorted run of equal bytes: every PSV is
// none) serialised on 16 counters (~88 appends per microsecond each): zeros at 256 MiB spent ~10
// ms of its 25 ms k_ansv_local there.
constexpr uint32_t kShards = 1024;
constexpr uint32_t kMaxRanges = 256;  // staging text ranges per block (rlog is raised to fit)
constexpr size_t kQMaxWord = 800;     // u32 index into Workspace::dscal: the largest shard per side
constexpr size_t kLinkWord = 2304;    // u32 index into Workspace::radix_counts: the block links
static_assert(kLinkWord >= 256 + 2 * 1024 && kLinkWord % 4 == 0, "past the range and queue counters, 16-byte aligned");
static_assert(kMaxRanges <= kT, "one thread per range");

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// One half of cand[p]: {p - pos, len}, or {local p + 1, 0} for none (pos == kInf). In a batch
// the suffix array is the blocks' arrays one after another, so a nearest smaller value found
// in another block's range means there is none in p's own (every value between lies outside
// p's range too): it is none as well.
__device__ __forceinline__ uint2 half(uint32_t p, uint32_t pos, uint32_t len, const Blocks &bl)
{
    return pos == kInf || bl.blk(pos) != bl.blk(p) ? make_uint2(p - bl.start(p) + 1u, 0u)
                                                   : make_uint2(p - pos, len);
}

// Packed staging (blocks of at most 2^27 positions, text ranges of at most 2^20): each half of a
// staged answer is one 64-bit word, offset (27 bits) | length (27) << 27 | ten bits of the
// suffix's position within its text range << 54 (PSV half: the low ten, NSV half: the high ten),
// so the scatter needs no separate position array (sp). A half still unanswered holds only its
// position bits; its answer comes later (block walk, or k_ansv_global straight into cand).
constexpr uint32_t kPk27 = (1u << 27) - 1u;
__device__ __forceinline__ uint2 pk_half(uint2 h, uint32_t p, uint32_t rlog, int side)
{
    const uint32_t lowp = p & ((1u << rlog) - 1u), part = side ? lowp >> 10 : lowp & 1023u;
    const uint64_t w = (uint64_t)h.x | ((uint64_t)h.y << 27) | ((uint64_t)part << 54);
    return make_uint2((uint32_t)w, (uint32_t)(w >> 32));
}

// First queue slot of shard s: the shards' regions hold as many entries as their blocks
// have leaves (a leaf misses at most once per side), so they tile [0, n) exactly. Shard t holds
// blocks t, t + kShards, ...: q + (t < rem) of them; the last block is short by short_by leaves.
__device__ __forceinline__ uint32_t shard_base(uint32_t s, uint32_t used_blocks, uint32_t n)
{
    const uint32_t q = used_blocks / kShards, rem = used_blocks % kShards;
    const uint32_t before = s * q + (s < rem ? s : rem);  // blocks of the shards below s
    const uint32_t short_by = used_blocks * kB - n;
    return before * kB - ((used_blocks - 1u) % kShards < s ? short_by : 0u);
}

// The largest shard per side (one workgroup): qmax[0] PSV, qmax[1] NSV.
__global__ __launch_bounds__(1024) void k_queue_max(const uint32_t *__restrict__ qcount, uint32_t *__restrict__ qmax)
{
    __shared__ uint32_t m[2];
    if (threadIdx.x < 2)
        m[threadIdx.x] = 0;
    __syncthreads();
    uint32_t a = 0, b = 0;
    for (uint32_t s = threadIdx.x; s < kShards; s += 1024) {
        a = qcount[2 * s] > a ? qcount[2 * s] : a;
        b = qcount[2 * s + 1] > b ? qcount[2 * s + 1] : b;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t x = shfl_xor_u32(a, o), y = shfl_xor_u32(b, o);
        a = x > a ? x : a;
        b = y > b ? y : b;
    }
    if (lane_id() == 0) {
        atomicMax(&m[0], a);
        atomicMax(&m[1], b);
    }
    __syncthreads();
    if (threadIdx.x < 2)
        qmax[threadIdx.x] = m[threadIdx.x];
}

// The min-tree's levels above the blocks with at most kTopNodes nodes, in one workgroup (a
// launch per level before: ~10 launches of a few microseconds each).
constexpr uint32_t kTopNodes = 1024;
__global__ __launch_bounds__(1024) void k_tree_top(uint32_t *__restrict__ tsa, uint32_t *__restrict__ tlcp,
                                                   uint32_t top)
{
    for (uint32_t lo = top; lo >= 1; lo >>= 1) {
        for (uint32_t x = threadIdx.x; x < lo; x += 1024) {
            const uint32_t k = lo + x;
            tsa[k] = umin(tsa[2 * k], tsa[2 * k + 1]);
            tlcp[k] = umin(tlcp[2 * k], tlcp[2 * k + 1]);
        }
        __syncthreads();  // (global writes of this level visible to the next in the workgroup)
    }
}

// One queued query of the block (e = leaf << 1 | nsv) walks the block's LDS min-tree; a
// query whose answer lies outside the block goes to the global queue (wave-aggregated).
__device__ __forceinline__ void block_walk(uint32_t e, uint32_t slot, const uint32_t *vsa,
                                           const uint32_t *vlc, uint32_t b0, uint2 *sh, uint32_t *qp, uint32_t *qp_len,
                                           uint32_t *qn, uint32_t *qn_len, uint32_t *qps, uint32_t *qns, uint32_t *qcount,
                                           uint32_t qbase, const Blocks &bl, int pk, uint32_t rlog)
{
    const uint32_t l = e >> 1, r = b0 + l;
    const uint32_t v = vsa[kB + l];
    const bool nsv = e & 1u;
    uint32_t lm, hit = kInf, node = kB + l;
    if (!nsv) {
        // PSV: nearest smaller to the left; LCP minimum over (r', r].
        lm = vlc[kB + l];
        while (node > 1) {
            if (node & 1u) {
                uint32_t s = node - 1;
                if (vsa[s] < v) {
                    while (s < kB) {
                        const uint32_t rc = 2 * s + 1;
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
            const uint2 hh = half(v, vsa[kB + hit], lm, bl);
            sh[2 * slot] = pk ? pk_half(hh, v, rlog, 0) : hh;
        }
    } else {
        // NSV: nearest smaller to the right; LCP minimum over (r, r'].
        lm = kInf;
        while (node > 1) {
            if (!(node & 1u)) {
                uint32_t s = node + 1;
                if (vsa[s] < v) {
                    while (s < kB) {
                        const uint32_t lc = 2 * s;
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
            const uint2 hh = half(v, vsa[kB + hit], lm, bl);
            sh[2 * slot + 1] = pk ? pk_half(hh, v, rlog, 1) : hh;
        }
    }
    // global queue: one atomic per wave and side on this block's shard counter
    const bool miss = hit == kInf;
#pragma unroll
    for (int side = 0; side < 2; side++) {
        const bool mine = miss && (int)nsv == side;
        const uint64_t mask = wave_ballot(mine);
        if (!mask)
            continue;
        const int leader = (int)__ffsll((unsigned long long)mask) - 1;
        uint32_t base = 0;
        if ((int)lane_id() == leader)
            base = qbase + atomicAdd(&qcount[2u * (blockIdx.x % kShards) + side],
                                     (uint32_t)__popcll(mask));
        base = shfl_u32(base, leader);
        if (mine) {
            const uint32_t q = base + count_below(mask);
            (side ? qn : qp)[q] = r;
            (side ? qn_len : qp_len)[q] = lm;
            (side ? qns : qps)[q] = slot;  // (k_ansv_global answers into the staging slot)
        }
    }
}

__global__ __launch_bounds__(kT) void k_ansv_local(
    const uint32_t *__restrict__ sa, const uint32_t *__restrict__ lcp, uint32_t n, Blocks bl, uint32_t np2,
    uint32_t *__restrict__ tsa, uint32_t *__restrict__ tlcp, uint4 *__restrict__ stage,
    uint32_t *__restrict__ sp, uint32_t *__restrict__ rfill,
    uint32_t rlog, uint32_t *__restrict__ qp, uint32_t *__restrict__ qp_len, uint32_t *__restrict__ qps,
    uint32_t *__restrict__ qns,
    uint32_t *__restrict__ qn, uint32_t *__restrict__ qn_len, uint32_t *__restrict__ qcount, int pk)
{
    __shared__ uint32_t vsa[2 * kB + kNear];  // heap: [1, kB) tree, [kB, 2kB) leaves, + pad
    __shared__ uint32_t vlc[2 * kB + kNear];
    __shared__ uint16_t loc[kB];             // leaf's index within its text range's run
    __shared__ uint32_t rbase[kMaxRanges];   // per text range: count, then the run's first slot
    uint2 *const sh = reinterpret_cast<uint2 *>(stage);  // halves: 2 slot (PSV), 2 slot + 1 (NSV)
    const uint32_t tid = threadIdx.x;
    if (tid < kMaxRanges)
        rbase[tid] = 0;
    const uint32_t b0 = blockIdx.x * kB;

    // Build the block's min-tree (heap: node k has children 2k, 2k + 1; leaves at kB + l) and
    // publish its internal nodes into the global heap. Thread t owns leaves 8t .. 8t + 7: the
    // three levels above them are formed in registers, the next six by butterflies within the
    // wave, the top two by one thread: two barriers instead of one per level.
    static_assert(kB == 8 * kT, "8 leaves per thread");
    const uint32_t root = np2 / kB + blockIdx.x;
    // Only the nodes over >= kScan leaves go to the global heap (k < 2 kB / kScan): the global
    // walks scan a node's kScan leaves from the suffix array and LCP arrays instead of descending
    // the last levels, so three quarters of the tree writes are saved.
    auto put = [&](uint32_t k, uint32_t a, uint32_t c) {
        vsa[k] = a;
        vlc[k] = c;
        if (k < 2 * kB / kScan) {
            const uint32_t lev = 31u - __builtin_clz(k);
            const uint32_t g = (root << lev) + (k - (1u << lev));
            tsa[g] = a;
            tlcp[g] = c;
        }
    };
    uint32_t a[8], c[8];
    {
        const uint32_t r0 = b0 + 8 * tid;
        if (r0 + 8 <= n) {
            const uint4 x0 = *reinterpret_cast<const uint4 *>(sa + r0);
            const uint4 x1 = *reinterpret_cast<const uint4 *>(sa + r0 + 4);
            const uint4 y0 = *reinterpret_cast<const uint4 *>(lcp + r0);
            const uint4 y1 = *reinterpret_cast<const uint4 *>(lcp + r0 + 4);
            a[0] = x0.x; a[1] = x0.y; a[2] = x0.z; a[3] = x0.w;
            a[4] = x1.x; a[5] = x1.y; a[6] = x1.z; a[7] = x1.w;
            c[0] = y0.x; c[1] = y0.y; c[2] = y0.z; c[3] = y0.w;
            c[4] = y1.x; c[5] = y1.y; c[6] = y1.z; c[7] = y1.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const bool in = r0 + j < n;
                a[j] = in ? sa[r0 + j] : kInf;
                c[j] = in ? lcp[r0 + j] : kInf;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
        vsa[kB + 8 * tid + j] = a[j];
        vlc[kB + 8 * tid + j] = c[j];
    }
    if (tid < kNear) {
        vsa[2 * kB + tid] = kInf;
        vlc[2 * kB + tid] = kInf;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {  // level of kB / 2 nodes
        a[j] = umin(a[2 * j], a[2 * j + 1]);
        c[j] = umin(c[2 * j], c[2 * j + 1]);
        put(kB / 2 + 4 * tid + j, a[j], c[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {  // kB / 4 nodes
        a[j] = umin(a[2 * j], a[2 * j + 1]);
        c[j] = umin(c[2 * j], c[2 * j + 1]);
        put(kB / 4 + 2 * tid + j, a[j], c[j]);
    }
    uint32_t x = umin(a[0], a[1]), y = umin(c[0], c[1]);  // kB / 8 = kT nodes
    put(kB / 8 + tid, x, y);
#pragma unroll
    for (uint32_t st = 1; st <= 6; st++) {  // kB / 16 .. kB / 512 nodes
        x = umin(x, shfl_xor_u32(x, 1 << (st - 1)));
        y = umin(y, shfl_xor_u32(y, 1 << (st - 1)));
        if ((tid & ((1u << st) - 1u)) == 0)
            put((kB >> (3 + st)) + (tid >> st), x, y);
    }
    __syncthreads();
    if (tid == 0) {  // nodes 2, 3 and the block root 1
        put(2, umin(vsa[4], vsa[5]), umin(vlc[4], vlc[5]));
        put(3, umin(vsa[6], vsa[7]), umin(vlc[6], vlc[7]));
        put(1, umin(vsa[2], vsa[3]), umin(vlc[2], vlc[3]));
    }
    // Staging slots: leaf l's answers go to slot rbase[p >> rlog] + loc[l] (one run per text
    // range in this workgroup; the run is reserved with one global atomic per range).
    for (uint32_t l = tid; l < kB && b0 + l < n; l += kT)
        loc[l] = (uint16_t)atomicAdd(&rbase[vsa[kB + l] >> rlog], 1u);
    __syncthreads();
    if (tid < kMaxRanges && rbase[tid])
        rbase[tid] = (tid << rlog) + atomicAdd(&rfill[tid], rbase[tid]);
    __syncthreads();

    // Phase 1: most nearest smaller values are a few ranks away. Scan up to kNear neighbours
    // on each side (lanes read consecutive LDS words: no bank conflicts); queue the rest.
    // The walk queue holds kWQ entries (12% of 2 kB queries miss on text); a full queue walks
    // in place. Kept small so 4 workgroups fit a CU's LDS.
    __shared__ uint16_t wq[kWQ];
    __shared__ uint32_t wq_n;
    const uint32_t qbase = shard_base(blockIdx.x % kShards, gridDim.x, n);
    auto slot_of = [&](uint32_t l) { return rbase[vsa[kB + l] >> rlog] + loc[l]; };
    // Both sides' misses of a wave's leaves take their queue slots with one LDS atomic per wave
    // (one per query before: a block whose PSVs all lie to its left, as in every descending run
    // of a periodic block's suffix array, queued 2048 queries through one LDS word).
    auto enqueue2 = [&](bool needP, bool needN, uint32_t l) {
        const uint64_t mP = wave_ballot(needP), mN = wave_ballot(needN);
        if (!(mP | mN))
            return;
        const int leader = (int)__ffsll((unsigned long long)(mP | mN)) - 1;
        uint32_t base = 0;
        if ((int)lane_id() == leader)
            base = atomicAdd(&wq_n, (uint32_t)(__popcll(mP) + __popcll(mN)));
        base = shfl_u32(base, leader);
        for (int side = 0; side < 2; side++) {
            if (!(side ? needN : needP))
                continue;
            const uint32_t q = base + (side ? (uint32_t)__popcll(mP) + count_below(mN) : count_below(mP));
            const uint32_t e = l << 1 | (uint32_t)side;
            if (q < kWQ)
                wq[q] = (uint16_t)e;
            else
                block_walk(e, slot_of(l), vsa, vlc, b0, sh, qp, qp_len, qn, qn_len, qps, qns, qcount, qbase, bl, pk,
                           rlog);
        }
    };
    if (tid == 0)
        wq_n = 0;
    __syncthreads();
    for (uint32_t l = tid; l < kB; l += kT) {
        const uint32_t r = b0 + l;
        if (r >= n)
            break;
        const uint32_t v = vsa[kB + l];
        // Fully unrolled: all 4 * kNear LDS reads are independent and issue back to back
        // (paired into ds_read2_b32 with constant offsets); the first hit is then selected
        // in registers. Reads left of the block's first leaf land in the tree levels and
        // right of its last leaf in the +inf pad; both are masked by the bounds tests.
        uint32_t sL[kNear], cL[kNear], sR[kNear], cR[kNear];
#pragma unroll
        for (uint32_t d = 1; d <= kNear; d++) {
            sL[d - 1] = vsa[kB + l - d];
            cL[d - 1] = vlc[kB + l - d];
            sR[d - 1] = vsa[kB + l + d];
            cR[d - 1] = vlc[kB + l + d];
        }
        // The first hit per side as the lowest bit of a kNear-bit mask of "smaller" tests (bounded
        // to the block), then the LCP minimum up to it: two compare-and-select sweeps per side
        // instead of one sequential chain of live / hit / minimum selects per neighbour.
        uint32_t mP = 0, mN = 0;
#pragma unroll
        for (uint32_t d = 0; d < kNear; d++) {
            mP |= (sL[d] < v ? 1u : 0u) << d;
            mN |= (sR[d] < v ? 1u : 0u) << d;
        }
        constexpr uint32_t kAll = kNear >= 32 ? 0xffffffffu : (1u << kNear) - 1u;
        mP &= l >= kNear ? kAll : (1u << l) - 1u;                          // d <= l
        mN &= kB - 1u - l >= kNear ? kAll : (1u << (kB - 1u - l)) - 1u;  // l + d < kB
        const uint32_t dP = mP ? (uint32_t)__builtin_ctz(mP) : kNear, dN = mN ? (uint32_t)__builtin_ctz(mN) : kNear;
        // PSV: LCP minimum over (r', r] = LCP[r] and the neighbours passed over; NSV: over
        // (r, r'] = the neighbours up to and including the hit
        uint32_t lmP = vlc[kB + l], lmN = kInf;
#pragma unroll
        for (uint32_t d = 0; d < kNear; d++) {
            lmP = d < dP ? umin(lmP, cL[d]) : lmP;
            lmN = d <= dN ? umin(lmN, cR[d]) : lmN;
        }
        const uint32_t hitP = mP ? l - dP - 1u : kInf, hitN = mN ? l + dN + 1u : kInf;
        const uint32_t pvP = mP ? vsa[kB + hitP] : 0u, pvN = mN ? vsa[kB + hitN] : 0u;
        const uint32_t slot = slot_of(l);
        if (pk) {  // both halves at once, an unanswered one with its position bits only
            const uint2 hp = pk_half(hitP != kInf ? half(v, pvP, lmP, bl) : make_uint2(0u, 0u), v, rlog, 0);
            const uint2 hn = pk_half(hitN != kInf ? half(v, pvN, lmN, bl) : make_uint2(0u, 0u), v, rlog, 1);
            stage[slot] = make_uint4(hp.x, hp.y, hn.x, hn.y);
        } else {
            sp[slot] = v;
            if (hitP != kInf && hitN != kInf) {
                const uint2 hp = half(v, pvP, lmP, bl), hn = half(v, pvN, lmN, bl);
                stage[slot] = make_uint4(hp.x, hp.y, hn.x, hn.y);
            } else {
                if (hitP != kInf)
                    sh[2 * slot] = half(v, pvP, lmP, bl);
                if (hitN != kInf)
                    sh[2 * slot + 1] = half(v, pvN, lmN, bl);
            }
        }
        enqueue2(hitP == kInf, hitN == kInf, l);
    }
    __syncthreads();

    // Phase 2: the queued queries walk the block's min-tree; answers outside the block go to
    // the global queues (k_ansv_global continues from the block root).
    const uint32_t nw = wq_n < kWQ ? wq_n : kWQ;
    for (uint32_t w = tid; w < nw; w += kT)
        block_walk(wq[w], slot_of(wq[w] >> 1), vsa, vlc, b0, sh, qp, qp_len, qn, qn_len, qps, qns,
                   qcount, qbase, bl, pk, rlog);
}

// Staged answers -> cand in the interleaved text-order layout. Slots are grouped by text
// range, so the workgroups in flight write into one cache-resident window of cand. It runs last:
// the halves that went to the global queues were filled in by k_ansv_global (round 6).
__global__ __launch_bounds__(kT) void k_cand_scatter(const uint32_t *__restrict__ sp,
                                                     const uint4 *__restrict__ stage, uint32_t npos,
                                                     uint4 *__restrict__ cand, uint32_t klog,
                                                     uint32_t rlog, uint32_t nranges,
                                                     const uint32_t *__restrict__ rfill,
                                                     uint32_t *__restrict__ err, int pk)
{
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs, so workgroup g runs on
    // XCD g mod 8; XCD x takes text ranges x, x + 8, ... in turn, and the lines of one cand
    // window are only ever written through one XCD's L2.
    const uint32_t g = blockIdx.x, tiles = 1u << (rlog - 8);
    const uint32_t k = g >> 3, r = (g & 7u) + 8u * (k >> (rlog - 8));
    if (r >= nranges)
        return;
    // One slot per thread: all three loads are issued under one EXEC mask (DESIGN.md,
    // "Concurrent encodes and the unaligned text load").
    // A range's run holds as many slots as the range has suffixes (all of its positions,
    // but for a batch's dead ones).
    const size_t x = (size_t)(k & (tiles - 1u)) * kT + threadIdx.x;
    if (x >= rfill[r])
        return;
    const size_t i = ((size_t)r << rlog) + x;
    const uint4 c = stage[i];
    if (pk) {  // (the position from the halves' bits, the halves back to {offset, length})
        const uint32_t p = (r << rlog) | (c.y >> 22) | ((c.w >> 22) << 10);
        if (bad_index(p >= npos, err, kErrAnsv))
            return;
        const uint64_t w0 = (uint64_t)c.y << 32 | c.x, w1 = (uint64_t)c.w << 32 | c.z;
        cand[sidx(p, klog)] = make_uint4((uint32_t)w0 & kPk27, (uint32_t)(w0 >> 27) & kPk27, (uint32_t)w1 & kPk27,
                                         (uint32_t)(w1 >> 27) & kPk27);
        return;
    }
    const uint32_t p = sp[i];
    if (bad_index(p >= npos, err, kErrAnsv))
        return;
    cand[sidx(p, klog)] = c;
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

// Climb from `node` (a node over >= kScan leaves, or a block root) towards the root: the first
// sibling on the query's side holding a smaller suffix is descended to its nearest node over
// kScan leaves, whose leaves are scanned. Returns the answer's rank (kInf: none); lm accumulates
// the LCP minimum (PSV: over the ranks passed to the left; NSV: up to and including the answer).
__device__ __forceinline__ uint32_t tree_walk(const Tree &t, uint32_t node, uint32_t v, uint32_t &lm, int nsv)
{
    const uint32_t low = t.np2 / kScan;  // nodes over kScan leaves: [low, 2 low)
    while (node > 1) {
        bool side = nsv ? !(node & 1u) : (node & 1u);
        if (side) {
            uint32_t s = nsv ? node + 1 : node - 1;
            if (t.vmin(s) < v) {
                while (s < low) {
                    uint32_t near = nsv ? 2 * s : 2 * s + 1;  // child adjacent to the query
                    if (t.vmin(near) < v) {
                        s = near;
                    } else {
                        lm = umin(lm, t.lmin(near));
                        s = nsv ? 2 * s + 1 : 2 * s;
                    }
                }
                // the node's kScan leaves, from the query's side: PSV takes the last leaf with a
                // smaller suffix (LCP minimum over the leaves after it), NSV the first (the
                // minimum up to and including it)
                const uint32_t r0 = (s - low) * kScan;
                uint32_t sv[kScan], lv[kScan];
#pragma unroll
                for (uint32_t k = 0; k < kScan; k++) {  // (leaves past n: +inf, like vmin / lmin)
                    const uint32_t rk = r0 + k, rc = rk < t.n ? rk : 0u;
                    const uint32_t a = t.sa[rc], c = t.lcp[rc];
                    sv[k] = rk < t.n ? a : kInf;
                    lv[k] = rk < t.n ? c : kInf;
                }
                uint32_t h = kInf, m = lm;
#pragma unroll
                for (uint32_t k = 0; k < kScan; k++) {
                    const uint32_t q = nsv ? k : kScan - 1u - k;
                    const bool live = h == kInf;
                    if (nsv)
                        m = live ? umin(m, lv[q]) : m;
                    h = live && sv[q] < v ? r0 + q : h;
                    if (!nsv)
                        m = h == kInf ? umin(m, lv[q]) : m;
                }
                lm = m;
                return h;
            }
            lm = umin(lm, t.lmin(s));
        }
        node >>= 1;
    }
    return kInf;
}

// Block links: per block B, the PSV of its left neighbour rank b0 - 1 and the NSV of its right
// neighbour b1 = b0 + kB with their LCP minima (x, y: PSV rank, minimum over (x, b0 - 1]; z, w: NSV
// rank, minimum over [b1, z]; kInf: none). A query that leaves its block with a suffix above the
// neighbour's but below the link's has the link as its answer: every rank between holds a larger
// suffix. In a periodic block's suffix array each phase is one descending run of positions across
// many blocks, whose PSVs all lie at the end of the run before: one walk per block instead of one
// per query.
__global__ void k_ansv_links(Tree t, uint32_t used_blocks, uint4 *__restrict__ link)
{
    const uint32_t B = blockIdx.x * kT + threadIdx.x;
    if (B >= used_blocks)
        return;
    const uint32_t low = t.np2 / kScan;
    uint4 out = make_uint4(kInf, kInf, kInf, kInf);
    if (B > 0 && (uint64_t)B * kB <= t.n) {
        const uint32_t r1 = B * kB - 1u, v1 = t.sa[r1], g0 = r1 & ~(kScan - 1u);
        uint32_t lm = t.lcp[r1], hit = kInf;
        for (uint32_t k = r1; k-- > g0;) {
            if (t.sa[k] < v1) {
                hit = k;
                break;
            }
            lm = umin(lm, t.lcp[k]);
        }
        if (hit == kInf)
            hit = tree_walk(t, low + r1 / kScan, v1, lm, 0);
        out.x = hit;
        out.y = lm;
    }
    if ((uint64_t)(B + 1) * kB < t.n) {
        const uint32_t r1 = (B + 1) * kB, v1 = t.sa[r1];
        const uint32_t gend = (r1 | (kScan - 1u)) + 1u < t.n ? (r1 | (kScan - 1u)) + 1u : t.n;
        uint32_t lm = t.lcp[r1], hit = kInf;
        for (uint32_t k = r1 + 1; k < gend; k++) {
            lm = umin(lm, t.lcp[k]);
            if (t.sa[k] < v1) {
                hit = k;
                break;
            }
        }
        if (hit == kInf)
            hit = tree_walk(t, low + r1 / kScan, v1, lm, 1);
        out.z = hit;
        out.w = lm;
    }
    link[B] = out;
}

// Queries that left their block: the block's neighbour or link when it answers (above), else the
// climb from the block root. blockIdx.y is the queue shard. The answer goes into the query's
// staging slot (qslot, from k_ansv_local), so k_cand_scatter moves it into cand with the block's
// own answers, window by window (a periodic block's PSVs almost all leave their blocks: written
// straight into cand in text order they were random 8-byte writes, period 3 at 256 MiB 10.7 ms).
__global__ void k_ansv_global(Tree t, const uint32_t *__restrict__ q,
                              const uint32_t *__restrict__ qlen, const uint32_t *__restrict__ qslot,
                              const uint32_t *__restrict__ qcount, uint32_t used_blocks, int nsv,
                              uint2 *__restrict__ sh, uint32_t rlog, int pk, Blocks bl,
                              const uint4 *__restrict__ link)
{
    const uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= qcount[2u * blockIdx.y + (uint32_t)nsv])
        return;
    const uint32_t e = shard_base(blockIdx.y, used_blocks, t.n) + x;
    const uint32_t r = q[e];
    uint32_t lm = qlen[e];
    const uint32_t v = t.sa[r], B = r / kB;
    uint32_t hit = kInf;
    bool done = false;  // (answered by the neighbour or the link, or none: the link has none)
    const uint4 lk = link ? link[B] : make_uint4(0u, 0u, 0u, 0u);
    if (!link) {
    } else if (!nsv) {
        if (B > 0) {
            const uint32_t r1 = B * kB - 1u;
            if (t.sa[r1] < v) {
                hit = r1;
                done = true;
            } else if (lk.x == kInf) {
                done = true;
            } else if (t.sa[lk.x] < v) {
                hit = lk.x;
                lm = umin(lm, lk.y);
                done = true;
            }
        }
    } else {
        const uint32_t r1 = (B + 1) * kB;
        if ((uint64_t)(B + 1) * kB < t.n) {
            if (t.sa[r1] < v) {
                hit = r1;
                lm = umin(lm, t.lcp[r1]);
                done = true;
            } else if (lk.z == kInf) {
                done = true;
            } else if (t.sa[lk.z] < v) {
                hit = lk.z;
                lm = umin(lm, lk.w);
                done = true;
            }
        }
    }
    if (!done)
        hit = tree_walk(t, t.np2 / kB + B, v, lm, nsv);
    const uint32_t pos = hit == kInf ? kInf : t.sa[hit];
    const uint2 hh = half(v, pos, lm, bl);
    sh[2 * qslot[e] + (uint32_t)nsv] = pk ? pk_half(hh, v, rlog, nsv) : hh;
}

// Every block's first position: no PSV / NSV, lengths 1 (lib/salz.c:547-548).
__global__ void k_cand_origin(uint4 *cand, Blocks bl, uint32_t klog)
{
    const uint32_t b = blockIdx.x * kT + threadIdx.x;
    if (b < bl.nb)
        cand[sidx(b * (bl.nb == 1 ? 0u : bl.bs), klog)] = make_uint4(1u, 1u, 1u, 1u);
}

}  // namespace

int stage_candidates(Workspace &ws, const Blocks &bl, const uint32_t *lcp)
{
    hipStream_t st = ws.stream;
    const uint32_t n = bl.nsa(), npos = bl.npos;  // suffix array entries, position space
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
    // range fills (rfill) in radix_counts[0, kMaxRanges), the shards' counters after them
    uint32_t *cnt = ws.radix_counts + kMaxRanges;
    uint32_t *qmax = reinterpret_cast<uint32_t *>(ws.dscal) + kQMaxWord;
    if (ws.radix_counts_elems < kMaxRanges + 2 * (size_t)kShards) {
        set_error("ansv: queue counters do not fit");
        return -1;
    }
    SALZ_HIP(fill_async(cnt, 0, 2 * kShards * sizeof(uint32_t), st));
    uint32_t nblocks = np2 / kB;
    uint32_t used_blocks = (n + kB - 1) / kB;
    // Blocks past the text only hold +inf leaves: fill their subtree roots directly.
    if (used_blocks < nblocks) {
        // Each unused block root and its descendants would be +inf; only nodes at or above
        // the block-root level are ever read for them, so set those roots to +inf.
        SALZ_HIP(fill_async(tsa + nblocks + used_blocks, 0xff,
                                sizeof(uint32_t) * (nblocks - used_blocks), st));
        SALZ_HIP(fill_async(tlcp + nblocks + used_blocks, 0xff,
                                sizeof(uint32_t) * (nblocks - used_blocks), st));
    }
    // Staging: text ranges of 2^rlog positions (cand windows of 16 << rlog bytes; 16 MB by
    // default: 2^19 and 2^21 measured slower on C2), at most kMaxRanges of them. Slots sp / stage
    // alias scratch that is free here. Past 2^27 positions (unpacked staging) 2^21: half the
    // range reservations, one global atomic per range and workgroup (C5 ANSV 11.83 -> 11.56 ms,
    // three of three on one box, profiles/r06u_ansv_ranges_ab.txt).
    uint32_t rlog = npos > (1u << 27) ? 21 : 20;
    while ((((uint64_t)npos - 1) >> rlog) + 1 > kMaxRanges)
        rlog++;
    uint32_t *rfill = ws.radix_counts;
    uint32_t *sp = ws.u0;
    uint4 *stage = reinterpret_cast<uint4 *>(ws.lsc);
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    if (ws.radix_counts_elems < kMaxRanges) {
        set_error("ansv: range counters do not fit");
        return -1;
    }
    SALZ_HIP(fill_async(rfill, 0, kMaxRanges * sizeof(uint32_t), st));
    // packed staging (no position array) where offsets, lengths and range bits fit 16 bytes
    // (round 5: C2 ANSV 3.72 -> 3.51 ms against the position array, which blocks past 2^27
    // positions keep). A second staging level (each run re-sorted into 2 MB windows before the
    // scatter) measured slower in round 5 (C2 ANSV 3.65 -> 4.04 ms) and was removed in round 6.
    const int pk = npos <= (1u << 27) && rlog <= 20 ? 1 : 0;
    // staging slots of the queued queries (u1, u2: free here)
    uint32_t *qps = ws.u1, *qns = ws.u2;
    hipLaunchKernelGGL(k_ansv_local, dim3(used_blocks), dim3(kT), 0, st, ws.sa, lcp, n, bl, np2, tsa,
                       tlcp, stage, sp, rfill, rlog, qp, qpl, qps, qns, qn, qnl, cnt, pk);
    SALZ_LAUNCH_CHECK();
    uint32_t lo = nblocks / 2;
    for (; lo > kTopNodes; lo >>= 1) {
        hipLaunchKernelGGL(k_tree_level, dim3(grid_for(lo, kT)), dim3(kT), 0, st, tsa, tlcp, lo,
                           lo);
        SALZ_LAUNCH_CHECK();
    }
    if (lo >= 1) {
        hipLaunchKernelGGL(k_tree_top, dim3(1), dim3(1024), 0, st, tsa, tlcp, lo);
        SALZ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_queue_max, dim3(1), dim3(1024), 0, st, cnt, qmax);
    SALZ_LAUNCH_CHECK();
    if (read_scalars(ws, 0, (kQMaxWord + 2) * sizeof(uint32_t), "ansv.q") != 0)
        return -1;
    if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
        set_error("ansv: device index check failed (code 0x%x): suffix array corrupt", e);
        return -1;
    }
    const uint32_t nqp = reinterpret_cast<uint32_t *>(ws.hscal)[kQMaxWord];  // largest shard per side
    const uint32_t nqn = reinterpret_cast<uint32_t *>(ws.hscal)[kQMaxWord + 1];
    Tree t{tsa, tlcp, ws.sa, lcp, n, np2};
    // block links in the radix counts past the range and queue counters
    // (a workspace whose counters cannot hold them walks every query: link = null)
    uint4 *link = ws.radix_counts_elems >= kLinkWord + 4 * (size_t)used_blocks
                      ? reinterpret_cast<uint4 *>(ws.radix_counts + kLinkWord)
                      : nullptr;
    if ((nqp || nqn) && link) {
        hipLaunchKernelGGL(k_ansv_links, dim3(grid_for(used_blocks, kT)), dim3(kT), 0, st, t, used_blocks, link);
        SALZ_LAUNCH_CHECK();
    }
    uint2 *sh = reinterpret_cast<uint2 *>(stage);
    if (nqp) {
        hipLaunchKernelGGL(k_ansv_global, dim3(grid_for(nqp, kT), kShards), dim3(kT), 0, st, t,
                           qp, qpl, qps, cnt, used_blocks, 0, sh, rlog, pk, bl, link);
        SALZ_LAUNCH_CHECK();
    }
    if (nqn) {
        hipLaunchKernelGGL(k_ansv_global, dim3(grid_for(nqn, kT), kShards), dim3(kT), 0, st, t,
                           qn, qnl, qns, cnt, used_blocks, 1, sh, rlog, pk, bl, link);
        SALZ_LAUNCH_CHECK();
    }
    // every answer staged: into cand, window by window
    const uint32_t nranges = (uint32_t)((((uint64_t)npos - 1) >> rlog) + 1);
    const uint32_t sgrid = 8u * ((nranges + 7u) / 8u) << (rlog - 8);
    hipLaunchKernelGGL(k_cand_scatter, dim3(sgrid), dim3(kT), 0, st, sp, stage, npos, ws.cand,
                       ws.klog, rlog, nranges, rfill, derr, pk);
    SALZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_cand_origin, dim3(grid_for(bl.nb, kT)), dim3(kT), 0, st, ws.cand, bl, ws.klog);
    SALZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace salz
