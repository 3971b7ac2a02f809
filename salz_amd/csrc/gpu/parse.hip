// parse.hip - optimal LZ parse (reference: optimize_factorization, lib/salz.c:610-662).
//
// The reference runs one backward min-plus pass: cost[p] = min(9 + cost[p+1],
// w(PSV) + cost[p+lenP], w(NSV) + cost[p+lenN]) in 32-bit signed arithmetic, strict '<',
// candidate order literal, PSV, NSV. Here the text is cut into chunks of K = 2^klog
// positions, one lane per chunk, and the pass is iterated to a fixed point:
//
//   1. every chunk runs the backward pass over its own positions, reading the previous
//      iteration's exact costs for targets beyond its end; per position it records the
//      decision, the chunk-local cost estimate and the first position at or past the chunk
//      end its path reaches (its exit). The estimate is (bits along the path to the exit)
//      + (previous cost at the exit), so the in-chunk bit sum is estimate - cin[exit];
//   2. exact costs of the new decisions: exit targets E form a forest rooted at n; pointer
//      jumping over the compacted E gives their path sums, every other position adds its
//      in-chunk sum to its exit's cost;
//   3. repeat until no decision changes. At that point every decision is the argmin, with
//      the reference's tie order, over exact successor costs, so by backward induction from
//      n it is the reference's decision (DESIGN.md "Parse").
//
// All per-position arrays (candidates, choices, costs, state) use the chunk-interleaved
// layout of common.hpp: the 64 lanes of a wave walk 64 neighbouring chunks in lockstep, so
// the streaming loads and stores of one step are one contiguous run per wave.
// The pointer-jumping snapshots of the final E forest are kept for emission's path marking.
#include "internal.hpp"

#include <cstdlib>
#include <vector>

namespace salz {
namespace {

constexpr int kT = 256;

// token bit + vnibble + offset byte + gr3 length (lib/salz.c:595-608, :632-634)
__device__ __forceinline__ uint32_t factor_bits(uint32_t off, uint32_t len)
{
    return 1u + 8u + 4u * vn_size((off - 1u) >> 8) + ((len - 3u) >> 3) + 4u;
}

// Candidates as the parse reads them: the full {p - PSV, lenP, p - NSV, lenN} (uint4), or packed
// per side as len | (vnibble size of the offset's high part) << 28 (uint2, half the bytes), for
// blocks under 2^28 positions. The first pass reads the full form and writes the packed one, which
// every later pass and skip test reads.
struct CandFull {
    using T = uint4;
    static __device__ __forceinline__ uint32_t lp(T c) { return c.y; }
    static __device__ __forceinline__ uint32_t ln(T c) { return c.w; }
    static __device__ __forceinline__ uint32_t bp(T c) { return factor_bits(c.x, c.y); }
    static __device__ __forceinline__ uint32_t bn(T c) { return factor_bits(c.z, c.w); }
};
struct CandPacked {
    using T = uint2;
    static __device__ __forceinline__ uint32_t lp(T c) { return c.x & kPackLen; }
    static __device__ __forceinline__ uint32_t ln(T c) { return c.y & kPackLen; }
    // factor_bits: 13 + 4 vn_size((off - 1) >> 8) + ((len - 3) >> 3)
    static __device__ __forceinline__ uint32_t bp(T c) { return 13u + 4u * (c.x >> 28) + (((c.x & kPackLen) - 3u) >> 3); }
    static __device__ __forceinline__ uint32_t bn(T c) { return 13u + 4u * (c.y >> 28) + (((c.y & kPackLen) - 3u) >> 3); }
};
__device__ __forceinline__ uint2 pack_cand(uint4 c) { return make_uint2(pack_side(c.x, c.y), pack_side(c.z, c.w)); }
__device__ __forceinline__ uint2 pack_cand(uint2 c) { return c; }  // (packed passes write none)

// Storage slots 0..S-1 -> cost seed 3 * (n - p); slots past n unused. Any seed gives the
// same fixed point (the final pass confirms every decision against exact costs); one near
// the typical optimum (~3 bits per byte) needs fewer passes on mixed data (tools/parse_sim.c).
__global__ __launch_bounds__(kT) void k_cost_seed(uint32_t *cost, Blocks bl, uint32_t klog,
                                                  size_t S)
{
    size_t s = (size_t)blockIdx.x * kT + threadIdx.x;
    if (s >= S)
        return;
    uint64_t p = spos(s, klog);
    if (p <= bl.npos) {  // 3 bits per byte to the block's end; its end / dead positions: 0
        const uint32_t e = bl.end((uint32_t)p);
        cost[s] = (uint32_t)p < e ? 3u * (e - (uint32_t)p) : 0u;
    }
}

// One lane per chunk, positions b-1 down to a. The states of the last kWin positions
// (p+1 .. p+kWin) stay in registers, so a factor of length <= kWin reads its target from
// there; a longer factor's target (p + len >= p + kWin + 1) was finished at least kWin + 1
// steps earlier, so its load can be issued early: kDepth = 4 steps ahead, from a candidate
// loaded kCDepth = 7 steps ahead. Every step issues the same memory operations at clamped,
// always-valid addresses, no loaded value is examined before the step that needs it, and the
// loop is unrolled by the rings' lengths (8 candidates, 4 far states), so the rings rotate by
// register renaming: the compiler's waits are s_waitcnt vmcnt(k) for the load in use. The
// previous form (conditional loads, selects on just-loaded values, rings shifted with moves
// of in-flight registers) drained every outstanding load each step: one HBM latency per step.
constexpr uint32_t kWin = 8;

// Raw target state of a long factor: one 8-byte load. Inside the chunk it is the target's
// state in pst; past it, the aligned pair of cin words holding cin[sidx(q)] (far_decode picks
// the half). A factor that is not long (or runs past the end) loads its own chunk's first
// state, pst[base]: the 64 lanes then read 512 contiguous bytes instead of 64 lines.
// Consecutive positions of one match share its end (p + len stays put while len shrinks by
// one), so a target equal to the one loaded for position p + 1 (lq) is not loaded again: the
// lane reads its chunk's first state instead and `same` tells the step to reuse p + 1's value.
__device__ __forceinline__ uint64_t far_load(const uint64_t *pst, const uint32_t *cin, size_t base,
                                             uint32_t a, uint32_t b, uint32_t klog, uint32_t p,
                                             uint32_t len, uint32_t n, uint32_t &lq, uint32_t &same,
                                             uint32_t &li)
{
    const bool far = len > kWin && p < n && len <= n - p;  // (inert steps past n: never far)
    same = far && p + len == lq ? 1u : 0u;
    lq = far ? p + len : 0xffffffffu;
    const uint32_t q = far && !same ? p + len : a;
    li = q >> klog;  // lazy costs: the chunk whose offset applies to a target past the chunk
    const uint64_t *addr = q < b ? pst + base + ((size_t)(q - a) << 6)
                                 : reinterpret_cast<const uint64_t *>(cin) + (sidx(q, klog) >> 1);
    return *addr;
}

// (cost << 32 | exit) of target q = p + len from its raw load; sidx(q) is odd iff its chunk
// q >> klog is (the lane bit of the interleaved layout). lv: the lazy offset of q's chunk (0
// outside the lazy passes).
__device__ __forceinline__ uint64_t far_decode(uint64_t raw, uint32_t q, uint32_t b, uint32_t klog, uint32_t lv)
{
    if (q < b)
        return raw;
    const uint32_t v = (((q >> klog) & 1u) ? (uint32_t)(raw >> 32) : (uint32_t)raw) + lv;
    return ((uint64_t)v << 32) | q;
}

// Lazy costs (the late passes, DESIGN.md "Parse"): the exact cost of position q is
// C[sidx(q)] + L[q >> klog]. A chunk whose decisions did not change and whose exits all moved by
// one delta only adds the delta to its L word instead of rewriting its K costs.
struct Lazy {
    const uint32_t *L;    // per chunk offset (null outside the lazy passes)
    uint32_t *summ;       // per chunk: its first kSumm distinct exits and an overflow flag
    uint8_t *chg;         // per chunk: a decision changed in this pass's walk
};
constexpr uint32_t kSumm = 8;
constexpr uint32_t kSummW = kSumm + 1;  // words per chunk

// wdirty (from the third pass on): one flag per wave of 64 chunks; a clean wave's chunks
// would repeat their decisions (k_parse_mark), so they only carry their choices over, and
// their states stay valid through dsum (the uniform cost shift added since their last pass).
// DEP / CDEP: far-target and candidate prefetch distances (8, 15 measured no faster in the late
// passes either); chunks of K <= 128 run 1 / 3 (the launch below).
template <class C, uint32_t DEP = 4, uint32_t CDEP = 7>
__global__ __launch_bounds__(kT) void k_parse_chunk(
    const typename C::T *__restrict__ cand, uint2 *__restrict__ pack_out, const uint32_t *__restrict__ cin,
    uint64_t *__restrict__ pst,
    const uint8_t *chold, uint8_t *chnew, uint32_t n, Blocks bl, uint32_t klog,
    uint32_t *__restrict__ changed, uint32_t *err, uint8_t *__restrict__ eflag,
    const uint8_t *__restrict__ wdirty, uint32_t *__restrict__ dsum, uint32_t *__restrict__ reach,
    uint32_t *__restrict__ rlo, Lazy lz, int first, uint8_t *__restrict__ ttouch, uint32_t tgen)
{
    constexpr uint32_t kDepth = DEP, kCDepth = CDEP;
    static_assert(kDepth <= kWin && kCDepth >= kDepth && ((kCDepth + 1) % kDepth) == 0, "ring depths");
    const uint32_t c = blockIdx.x * kT + threadIdx.x;  // chunk
    const uint64_t a64 = (uint64_t)c << klog;
    uint32_t diff = 0, errw = 0;
    uint32_t far_end = 0;  // farthest candidate target (first pass: k_parse_mark's range test)
    uint32_t reach_lo = 0;  // first position with a factor target at or past the chunk end
    if (c == 0)
        eflag[sidx(n, klog)] = 1u;  // the root of the exit forest
    if (a64 < n) {
        const uint32_t a = (uint32_t)a64;
        const uint32_t K = 1u << klog;
        // Live positions of the chunk: [a, b). A batch's chunks never straddle two blocks
        // (blocks are multiples of K); the 8 dead positions after a block's suffix text end
        // its last chunk and are inert like the steps past n: cost 0, exit n.
        const uint32_t e = bl.end(a), b0 = bl.start(a);
        const uint32_t b = (e - a) < K ? e : a + K;
        const size_t base = ((size_t)(c >> 6) << (klog + 6)) | (c & 63u);
        auto slot = [&](uint32_t j) { return base + ((size_t)j << 6); };
        if (wdirty && !wdirty[c >> 6]) {  // wave-uniform: a clean wave keeps its choices (in place)
            if (lz.chg)
                lz.chg[c] = 0;
            return;
        }
        if (dsum)
            dsum[c] = 0;  // this pass's states are computed from cin itself
        // Every lane walks K steps, a + K - 1 down to a: the text's last chunk starts past the
        // end (those steps are inert, below), so the loop count is wave-uniform (a scalar
        // counter, no EXEC change inside the loop) and the loop is unrolled by the rings'
        // length. Positions past n lie inside the layout's last tile; their slots are never read.
        // Rings, index k = position p - k for the current p.
        typename C::T cr[kCDepth + 1];
        uint8_t orr[kDepth];
        uint64_t fP[kDepth], fN[kDepth];
        uint32_t lP[kDepth], lN[kDepth];  // lazy offsets of the far targets' chunks
        uint64_t win[kWin];  // win[k] = state of p + 1 + k
        const uint32_t pK = a + K - 1;
        // ring bit k: the far target of position p - k equals p - k + 1's (value reused)
        uint32_t sameP = 0, sameN = 0, lqP = 0xffffffffu, lqN = 0xffffffffu;
        uint64_t prevP = 0, prevN = 0;  // decoded far targets of the previous step (p + 1)
#pragma unroll
        for (uint32_t k = 0; k <= kCDepth; k++)
            cr[k] = cand[slot(K - 1 - k)];
#pragma unroll
        for (uint32_t k = 0; k < kDepth; k++) {
            orr[k] = chold[slot(K - 1 - k)];
            uint32_t sp, sn, ip, in;
            fP[k] = far_load(pst, cin, base, a, b, klog, pK - k, C::lp(cr[k]), n, lqP, sp, ip);
            fN[k] = far_load(pst, cin, base, a, b, klog, pK - k, C::ln(cr[k]), n, lqN, sn, in);
            lP[k] = lz.L ? lz.L[ip] : 0u;
            lN[k] = lz.L ? lz.L[in] : 0u;
            sameP |= sp << k;
            sameN |= sn << k;
        }
#pragma unroll
        for (uint32_t k = 0; k < kWin; k++) {  // states a + K .. a + K + kWin - 1 (past n: unused)
            const uint32_t q = a + K + k, qq = q <= n ? q : n;
            const uint32_t v = cin[sidx(qq, klog)] + (lz.L ? lz.L[qq >> klog] : 0u);
            win[k] = q <= n ? (((uint64_t)v << 32) | q) : 0;
        }
        uint32_t last_ex = 0xffffffffu;
        uint32_t exs[kSumm], nex = 0, tex = 0xffffffffu;  // distinct exits (lz.summ)
#pragma unroll
        for (uint32_t k = 0; k < kSumm; k++)
            exs[k] = 0xffffffffu;
        far_end = b;
        reach_lo = b;
#pragma unroll CDEP + 1
        for (uint32_t j = K; j-- > 0;) {
            const uint32_t p = a + j;
            const bool live = p < b;
            const typename C::T c0 = cr[0];
            const uint32_t lenP = C::lp(c0), lenN = C::ln(c0);
            if (pack_out)  // (kernel-uniform) the first pass leaves the packed candidates
                pack_out[slot(j)] = pack_cand(cr[0]);
            if (reach) {
                const uint32_t tp = live && lenP >= 3u ? p + lenP : 0u, tn = live && lenN >= 3u ? p + lenN : 0u;
                far_end = tp > far_end ? tp : far_end;
                far_end = tn > far_end ? tn : far_end;
                reach_lo = tp >= b || tn >= b ? p : reach_lo;
            }
            uint32_t best = 9u + (uint32_t)(win[0] >> 32), ex = (uint32_t)win[0];
            uint8_t ch = 0;
            if (p != b0) {  // a block's first position is a literal (lib/salz.c:547-548)
                if (lenP >= 3u) {
                    errw |= live && lenP > e - p ? kErrParse : 0u;
                    uint64_t t;
                    if (lenP <= kWin) {
                        t = win[1];
#pragma unroll
                        for (uint32_t k = 2; k < kWin; k++)
                            t = lenP == k + 1 ? win[k] : t;
                    } else {
                        t = (sameP & 1u) ? prevP : far_decode(fP[0], p + lenP, b, klog, lP[0]);
                        prevP = t;
                    }
                    const uint32_t alt = C::bp(c0) + (uint32_t)(t >> 32);
                    if ((int32_t)alt < (int32_t)best) {
                        best = alt;
                        ex = (uint32_t)t;
                        ch = 1;
                    }
                }
                if (lenN >= 3u) {
                    errw |= live && lenN > e - p ? kErrParse : 0u;
                    uint64_t t;
                    if (lenN <= kWin) {
                        t = win[1];
#pragma unroll
                        for (uint32_t k = 2; k < kWin; k++)
                            t = lenN == k + 1 ? win[k] : t;
                    } else {
                        t = (sameN & 1u) ? prevN : far_decode(fN[0], p + lenN, b, klog, lN[0]);
                        prevN = t;
                    }
                    const uint32_t alt = C::bn(c0) + (uint32_t)(t >> 32);
                    if ((int32_t)alt < (int32_t)best) {
                        best = alt;
                        ex = (uint32_t)t;
                        ch = 2;
                    }
                }
            }
            // An inert step (past the end) leaves the state of a position no live one reads,
            // except n itself: (cost 0, exit n).
            if (!live)
                ex = n;
            const uint64_t stp = live ? ((uint64_t)best << 32) | ex : (uint64_t)n;
            pst[slot(j)] = stp;
            chnew[slot(j)] = ch;
            diff += live && (first || ch != orr[0]);  // (the first pass has no old choices)
            // Exit set E (every position's exit; consecutive positions mostly share one). The
            // store is issued every step, as a store under a narrower EXEC mask would leave
            // partial vmcnt waits depending on whether it ran (tests/test_codegen.py); a lane
            // whose exit did not change writes the root's flag (set anyway), so those lanes
            // share one line instead of each touching its own.
            const size_t sx = sidx(ex != last_ex ? ex : n, klog);
            eflag[sx] = 1u;
            if (ttouch)  // (skipping passes: the 64-chunk tiles whose exit flags this walk set)
                ttouch[sx >> (klog + 6)] = (uint8_t)tgen;
            last_ex = ex;
            if (lz.summ && live && ex != tex) {  // (consecutive positions mostly share their exit)
                tex = ex;
                bool seen = false;
#pragma unroll
                for (uint32_t k = 0; k < kSumm; k++)
                    seen |= exs[k] == ex;
                if (!seen) {
#pragma unroll
                    for (uint32_t k = 0; k < kSumm; k++)
                        exs[k] = k == nex ? ex : exs[k];
                    nex++;
                }
            }
            // shift the window and the rings one position down
#pragma unroll
            for (uint32_t k = kWin - 1; k > 0; k--)
                win[k] = win[k - 1];
            win[0] = stp;
#pragma unroll
            for (uint32_t k = 0; k < kCDepth; k++)
                cr[k] = cr[k + 1];
#pragma unroll
            for (uint32_t k = 0; k + 1 < kDepth; k++) {
                orr[k] = orr[k + 1];
                fP[k] = fP[k + 1];
                fN[k] = fN[k + 1];
                lP[k] = lP[k + 1];
                lN[k] = lN[k + 1];
            }
            // new loads (unconditional, clamped): position p - kDepth's old choice and far
            // targets (its candidate, cr[kDepth - 1], was loaded four steps ago), and position
            // p - 1 - kCDepth's candidate
            const uint32_t jd = j >= kDepth ? j - kDepth : 0u;
            const typename C::T cd = cr[kDepth - 1];
            orr[kDepth - 1] = chold[slot(jd)];
            uint32_t sp, sn, ip, in;
            fP[kDepth - 1] = far_load(pst, cin, base, a, b, klog, a + jd, C::lp(cd), n, lqP, sp, ip);
            fN[kDepth - 1] = far_load(pst, cin, base, a, b, klog, a + jd, C::ln(cd), n, lqN, sn, in);
            lP[kDepth - 1] = lz.L ? lz.L[ip] : 0u;
            lN[kDepth - 1] = lz.L ? lz.L[in] : 0u;
            sameP = (sameP >> 1) | (sp << (kDepth - 1));
            sameN = (sameN >> 1) | (sn << (kDepth - 1));
            cr[kCDepth] = cand[slot(j >= kCDepth + 1 ? j - kCDepth - 1 : 0u)];
        }
        if (lz.summ) {  // (unused entries repeat the first exit)
#pragma unroll
            for (uint32_t k = 0; k < kSumm; k++)
                lz.summ[kSummW * (size_t)c + k] = exs[k] != 0xffffffffu ? exs[k] : exs[0];
            lz.summ[kSummW * (size_t)c + kSumm] = nex > kSumm ? 1u : 0u;
        }
        if (lz.chg)
            lz.chg[c] = diff != 0 ? 1u : 0u;
    }
    if (reach && a64 < n) {
        reach[c] = far_end;
        rlo[c] = reach_lo;
    }
    if (errw)
        atomicOr(err, errw);  // a candidate past the end (reported once per lane)
    // one atomic per wave
    for (int m = 32; m >= 1; m >>= 1)
        diff += shfl_xor_u32(diff, m);
    if (lane_id() == 0 && diff)
        atomicAdd(changed, diff);
}

constexpr uint32_t kRowsBrk = 8;
// Breaks of the cost shift d[q] = cnew[q] - cold[q] (q >= 1 with d[q] != d[q - 1], or a cost at
// or above 2^30): flag[k] = 1 when chunk k holds one at some q in (kK, (k + 1)K] (flags cleared
// beforehand). A thread takes 8 rows of one chunk, the 64 lanes of a wave 64 neighbouring chunks,
// so every row is one contiguous run.
__global__ __launch_bounds__(kT) void k_shift_breaks(const uint32_t *__restrict__ cnew,
                                                     const uint32_t *__restrict__ cold, uint32_t n,
                                                     uint32_t klog, uint32_t nchunks, uint32_t *__restrict__ flag)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t lane = (uint32_t)(x & 63u), groups = (1u << klog) / kRowsBrk;
    const size_t rest = x >> 6;
    const uint32_t c = (uint32_t)((rest / groups) * 64 + lane), g = (uint32_t)(rest % groups);
    if (c >= nchunks)
        return;
    const uint32_t q0 = (c << klog) + g * kRowsBrk;  // compares q in (q0, q0 + 8]
    if (q0 >= n)
        return;
    uint32_t prev = cnew[sidx(q0, klog)] - cold[sidx(q0, klog)];
    bool brk = false;
#pragma unroll
    for (uint32_t r = 1; r <= kRowsBrk; r++) {
        const uint32_t q = q0 + r <= n ? q0 + r : n;  // (clamped: q = n repeats, no break)
        const size_t sq = sidx(q, klog);
        const uint32_t v = cnew[sq], d = v - cold[sq];
        brk |= d != prev || v >= (1u << 30);
        prev = d;
    }
    if (brk)
        flag[c] = 1u;
}

// Uniform-shift test, one chunk per lane, before every pass from the third on: every target
// at or past the chunk end b (the literal's b, and each candidate's p + len beyond it) must
// have moved by the same delta from cold (the costs the chunk's decisions are consistent
// with) to cnew (the exact costs of the current decisions); costs at or above 2^30 fail it
// (int32 compares could wrap). Then every option of every position moved by that delta, so the
// argmins repeat. A wave of 64 chunks that all pass is clean (wdirty = 0) and skips the pass;
// its chunks' states then lag cin by the delta, which dsum accumulates. ndirty counts the
// dirty waves; none left means the fixed point.
// A chunk whose targets [b, reach] hold no break of the shift (prefix counts pbrk over chunks)
// passes without looking at its candidates; only the others run the per-candidate test.
// Lazy passes: the shift of target q since the last test is dl[k] of its chunk k when that chunk
// was uniform (uni[k]), else D[sidx(q)].
struct LazyTest {
    const uint32_t *L;  // null: shifts from the cost arrays cnew - cold
    const uint8_t *uni;
    const uint32_t *dl, *D;
};

// (new cost, shift) of target q <= n; every load unconditional
__device__ __forceinline__ uint32_t shift_of(const LazyTest &lt, const uint32_t *cnew, const uint32_t *cold,
                                             uint32_t klog, uint32_t q, uint32_t &v)
{
    const size_t sq = sidx(q, klog);
    if (lt.L) {
        const uint32_t k = q >> klog;
        v = cnew[sq] + lt.L[k];
        const uint32_t dd = lt.D[sq], dk = lt.dl[k];
        return lt.uni[k] ? dk : dd;
    }
    v = cnew[sq];
    return v - cold[sq];
}

// Split test (a wave per chunk for the per-candidate part): k_parse_mark decides the chunks its
// range test passes and lists the others, k_mark_rows tests a listed chunk's candidates with a
// whole wave (K / 64 rows per lane, one memory latency), k_mark_final sets the wave flags. A wave
// whose one chunk needs the per-candidate test no longer walks K rows with 64 lanes.
struct MarkSplit {
    uint32_t *list, *count;  // chunks left to the per-candidate test
    uint8_t *cbad;           // per chunk: dirty
    uint32_t *d0s;           // per chunk: the shift at its end
};

// The range test of every chunk before a skipping pass: a chunk whose targets [b, reach] hold
// no break of the shift passes; the others (and no chunk whose end cost reaches 2^30) are listed
// for k_mark_rows, and k_mark_final sets the wave flags.
__global__ __launch_bounds__(kT) void k_parse_mark(const uint32_t *__restrict__ cnew,
                                                   const uint32_t *__restrict__ cold, uint32_t n, Blocks bl,
                                                   uint32_t klog, const uint32_t *__restrict__ reach,
                                                   const uint32_t *__restrict__ pbrk, LazyTest lt, MarkSplit ms)
{
    const uint32_t c = blockIdx.x * kT + threadIdx.x;
    const uint64_t a64 = (uint64_t)c << klog;
    if (a64 >= n)
        return;
    const uint32_t a = (uint32_t)a64, K = 1u << klog;
    // (a block's last chunk ends at its suffix text's end: a cost-0 end, never shifted)
    const uint32_t e = bl.end(a);
    const uint32_t b = (e - a) < K ? e : a + K;
    uint32_t nb;
    const uint32_t d0 = shift_of(lt, cnew, cold, klog, b, nb);
    const bool bad = nb >= (1u << 30);
    // breaks in (b, r] lie in chunks c + 1 .. (r - 1) >> klog (loads unconditional: an empty
    // range compares c + 1 twice)
    const uint32_t r = reach[c];
    const uint32_t hi = r > b ? ((r - 1) >> klog) + 1 : c + 1;
    const bool need = pbrk[hi] != pbrk[c + 1] && !bad;
    const uint64_t mk = wave_ballot(need);
    if (mk) {
        const int leader = (int)__ffsll((unsigned long long)mk) - 1;
        uint32_t at = 0;
        if ((int)lane_id() == leader)
            at = atomicAdd(ms.count, (uint32_t)__popcll(mk));
        at = shfl_u32(at, leader);
        if (need)
            ms.list[at + count_below(mk)] = c;
    }
    ms.cbad[c] = bad ? 1u : 0u;
    ms.d0s[c] = d0;
}

// Listed chunks' per-candidate tests (grid-stride over the list): a wave takes G = 512 / K chunks
// (one at K = 512, eight at K = 64), LP = 64 / G lanes each; lane l of a chunk takes rows
// rlo + l, rlo + l + LP, ... (at most 8), all loads issued before any is used.
template <class C>
__global__ __launch_bounds__(kT) void k_mark_rows(const typename C::T *__restrict__ cand,
                                                  const uint32_t *__restrict__ cnew,
                                                  const uint32_t *__restrict__ cold, uint32_t n, Blocks bl,
                                                  uint32_t klog, const uint32_t *__restrict__ rlo, LazyTest lt,
                                                  MarkSplit ms)
{
    const uint32_t lane = lane_id(), nwaves = gridDim.x * (kT / 64);
    const uint32_t K = 1u << klog, G = K >= 512u ? 1u : 512u / K, LP = 64u / G;
    const uint32_t sub = lane / LP, lic = lane % LP;
    const uint64_t gmask = (LP == 64u ? ~0ull : ((1ull << LP) - 1ull)) << (sub * LP);
    const uint32_t cnt = *ms.count;
    for (uint32_t w0 = ((blockIdx.x * kT + threadIdx.x) >> 6) * G; w0 < cnt; w0 += nwaves * G) {
        const uint32_t li = w0 + sub;
        const bool have = li < cnt;
        const uint32_t c = ms.list[have ? li : w0];
        const uint32_t a = c << klog;
        const uint32_t e = bl.end(a), b0 = bl.start(a);
        const uint32_t b = (e - a) < K ? e : a + K;
        const size_t base = ((size_t)(c >> 6) << (klog + 6)) | (c & 63u);
        const uint32_t d0 = ms.d0s[c];
        const uint32_t jl = rlo[c] - a, jn = b - a;
        typename C::T cd[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t j = jl + lic + u * LP;
            cd[u] = cand[base + ((size_t)(j < jn ? j : jl) << 6)];
        }
        bool bad = false;
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t j = jl + lic + u * LP, p = a + j;
            const bool on = have && j < jn && p != b0;
            const uint32_t lp = C::lp(cd[u]), ln = C::ln(cd[u]);
            const uint32_t qp = p + lp, qn = p + ln;
            const bool xp = on && lp >= 3u && qp >= b, xn = on && ln >= 3u && qn >= b;
            uint32_t vp, vn;
            const uint32_t dp = shift_of(lt, cnew, cold, klog, xp ? qp : b, vp);
            const uint32_t dn = shift_of(lt, cnew, cold, klog, xn ? qn : b, vn);
            bad |= dp != d0 || vp >= (1u << 30);
            bad |= dn != d0 || vn >= (1u << 30);
        }
        const uint64_t bm = wave_ballot(bad);
        if (lic == 0 && have && (bm & gmask))
            ms.cbad[c] = 1u;
    }
}

// Wave flags of the split test: a wave of chunks is clean when none of them is dirty.
__global__ __launch_bounds__(kT) void k_mark_final(uint32_t n, uint32_t klog, const uint8_t *__restrict__ cbad,
                                                   const uint32_t *__restrict__ d0s, uint8_t *__restrict__ wdirty,
                                                   uint32_t *__restrict__ dsum, uint32_t *__restrict__ ndirty)
{
    const uint32_t c = blockIdx.x * kT + threadIdx.x;
    const uint64_t a64 = (uint64_t)c << klog;
    if ((a64 & ~(((uint64_t)64 << klog) - 1)) >= n)
        return;  // whole wave past the end
    const bool in = a64 < n;
    const bool bad = in && cbad[in ? c : 0];
    const uint64_t m = wave_ballot(bad);
    if (lane_id() == 0) {
        wdirty[c >> 6] = m ? 1u : 0u;
        if (m)
            atomicAdd(ndirty, 1u);
    }
    if (!m && in)
        dsum[c] += d0s[c];
}

// Exit flags (bytes marked by the chunk pass, storage-slot order) -> ExitBits: the set as one
// bit per slot, 64 slots a word (one row of a 64-chunk tile), and per-word popcounts for the
// scan that numbers E. A thread packs 8 flag bytes, 8 lanes one word.
// (nd: the pass's dirty-wave count when its test ran; none dirty -> E unchanged, nothing to pack.
// ttouch: the tiles whose flags the pass's walk set (tagged with the pass's generation tgen); the
// flags of the others, which accumulate while waves skip passes, are as the last pack left them)
__global__ __launch_bounds__(kT) void k_exit_pack(const uint64_t *__restrict__ eflag8, size_t S8, ExitBits eb,
                                                  const uint32_t *__restrict__ nd,
                                                  const uint8_t *__restrict__ ttouch, uint32_t tgen, uint32_t klog)
{
    if (nd && *nd == 0u)
        return;
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;  // slots [8x, 8x + 8)
    if (ttouch && ttouch[(x < S8 ? 8 * x : 0) >> (klog + 6)] != (uint8_t)tgen)  // (tile-uniform: 8K slots per tile)
        return;
    uint64_t v = eflag8[x < S8 ? x : 0];  // (unconditional load, clamped)
    v |= v >> 4;
    v |= v >> 2;
    v |= v >> 1;
    v &= 0x0101010101010101ull;                                       // byte k's flag at bit 8k
    const uint64_t m8 = (v * 0x0102040810204080ull) >> 56;            // ... moved to bit k
    uint64_t w = m8 << (8u * (uint32_t)(x & 7u));
    w |= ((uint64_t)shfl_xor_u32((uint32_t)(w >> 32), 1) << 32) | shfl_xor_u32((uint32_t)w, 1);
    w |= ((uint64_t)shfl_xor_u32((uint32_t)(w >> 32), 2) << 32) | shfl_xor_u32((uint32_t)w, 2);
    w |= ((uint64_t)shfl_xor_u32((uint32_t)(w >> 32), 4) << 32) | shfl_xor_u32((uint32_t)w, 4);
    if ((x & 7u) == 0 && x < S8) {  // S8 is a multiple of 8 (slots come in 64-chunk tiles)
        eb.mask[x >> 3] = w;
        eb.wcnt[x >> 3] = (uint32_t)__popcll(w);
    }
}

// Compact E: node xi = index of exit position q in E; parent = exit of q, weight = in-chunk bit
// sum of q's path (estimate + dsum of q's chunk - cin[exit]). A thread takes 8 slots (one byte
// of an ExitBits word) and numbers their exits in slot order.
__global__ __launch_bounds__(kT) void k_compact_exits(ExitBits eb, const uint64_t *__restrict__ pst,
                                                      const uint32_t *__restrict__ cin, uint32_t n, uint32_t klog,
                                                      size_t S8, uint32_t *__restrict__ elist,
                                                      uint32_t *__restrict__ jt0, uint32_t *__restrict__ js,
                                                      const uint32_t *__restrict__ dsum,
                                                      const uint32_t *__restrict__ Lz, uint32_t *__restrict__ ce)
{
    // (lazy passes: a cost is cin + the chunk's offset Lz; ce = every node's cost before this pass)
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    if (x >= S8)
        return;
    const uint64_t word = eb.mask[x >> 3];
    const uint32_t sh = 8u * (uint32_t)(x & 7u);
    uint32_t bits = (uint32_t)(word >> sh) & 0xffu;
    uint32_t xi = eb.wpre[x >> 3] + (uint32_t)__popcll(word & ((1ull << sh) - 1ull));
    while (bits) {
        const size_t s = 8 * x + (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1u;
        const uint32_t q = (uint32_t)spos(s, klog);
        // every load unconditional (the root's reads use its own slot, results unused)
        const uint64_t v = pst[s];
        const uint32_t ev = q == n ? n : (uint32_t)v;
        const size_t se = sidx(ev, klog);
        const uint32_t parent = bits_index(eb.mask, eb.wpre, se);
        const uint32_t lq = Lz ? Lz[q >> klog] : 0u, le = Lz ? Lz[ev >> klog] : 0u;
        const uint32_t w = (uint32_t)(v >> 32) + dsum[(q < n ? q : 0u) >> klog] - (cin[se] + le);
        if (ce)
            ce[xi] = q == n ? 0u : cin[s] + lq;
        elist[xi] = q;
        jt0[xi] = q == n ? xi : parent;
        js[xi] = q == n ? 0u : w;
        xi++;
    }
}

// Node -> mask word of a sparse E: a thread per word writes its index at its nodes' numbers.
__global__ __launch_bounds__(kT) void k_node_words(ExitBits eb, size_t nw, uint32_t *__restrict__ nword)
{
    const size_t w = (size_t)blockIdx.x * kT + threadIdx.x;
    if (w >= nw)
        return;
    const uint32_t c = eb.wcnt[w], b = eb.wpre[w];
    for (uint32_t k = 0; k < c; k++)
        nword[b + k] = (uint32_t)w;
}

// The same, one thread per node of E (its word from k_node_words, its slot by selecting the set
// bit): |E| threads instead of one per 8 slots, where E is sparse.
__global__ __launch_bounds__(kT) void k_compact_nodes(ExitBits eb, const uint32_t *__restrict__ nword, uint32_t ne,
                                                      const uint64_t *__restrict__ pst,
                                                      const uint32_t *__restrict__ cin, uint32_t n, uint32_t klog,
                                                      uint32_t *__restrict__ elist, uint32_t *__restrict__ jt0,
                                                      uint32_t *__restrict__ js, const uint32_t *__restrict__ dsum,
                                                      const uint32_t *__restrict__ Lz, uint32_t *__restrict__ ce)
{
    const uint32_t xi = blockIdx.x * kT + threadIdx.x;
    if (xi >= ne)
        return;
    const uint32_t lo = nword[xi];
    uint64_t m = eb.mask[lo];
    uint32_t k = xi - eb.wpre[lo], p = 0;
#pragma unroll
    for (uint32_t w = 32; w >= 1; w >>= 1) {  // the k-th set bit of m
        const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
        const bool up = k >= c;
        k = up ? k - c : k;
        m = up ? m >> w : m;
        p += up ? w : 0u;
    }
    const size_t s = (size_t)lo * 64 + p;
    const uint32_t q = (uint32_t)spos(s, klog);
    const uint64_t v = pst[s];
    const uint32_t ev = q >= n ? n : (uint32_t)v;
    const size_t se = sidx(ev, klog);
    const uint32_t parent = bits_index(eb.mask, eb.wpre, se);
    const uint32_t qc = q < n ? q : 0u;
    const uint32_t lq = Lz ? Lz[qc >> klog] : 0u, le = Lz ? Lz[ev >> klog] : 0u;
    const uint32_t w = (uint32_t)(v >> 32) + dsum[qc >> klog] - (cin[se] + le);
    if (ce)
        ce[xi] = q == n ? 0u : cin[s] + lq;
    elist[xi] = q;
    jt0[xi] = q == n ? xi : parent;
    js[xi] = q == n ? 0u : w;
}

// Pointer jumping over E, two levels per launch (the snapshot of every level is kept for
// emission's path marking): from level k (jt, js) to k + 1 (jt1, written) and k + 2 (jt2, js2).
// A thread derives its node's level-(k + 1) successor itself, so no other thread's result of
// this launch is read.
// Three levels per launch (levels k + 1, k + 2, k + 3 from level k: eight dependent loads per
// thread through the L2-resident tables), for fewer launches where passes repeat.
__global__ void k_jump3(const uint32_t *__restrict__ jt, const uint32_t *__restrict__ js,
                        uint32_t *__restrict__ jt1, uint32_t *__restrict__ jt2, uint32_t *__restrict__ jt3,
                        uint32_t *__restrict__ js3, uint32_t ne)
{
    const uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= ne)
        return;
    uint32_t p[9];
    p[0] = x;
#pragma unroll
    for (int k = 1; k <= 8; k++)
        p[k] = jt[p[k - 1]];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        s += js[p[k]];
    jt1[x] = p[2];
    jt2[x] = p[4];
    jt3[x] = p[8];
    js3[x] = s;
}

__global__ void k_jump2(const uint32_t *__restrict__ jt, const uint32_t *__restrict__ js,
                        uint32_t *__restrict__ jt1, uint32_t *__restrict__ jt2,
                        uint32_t *__restrict__ js2, uint32_t ne, int two)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= ne)
        return;
    const uint32_t p = jt[x];
    const uint32_t pp = jt[p];
    const uint32_t s1 = js[x] + js[p];
    if (!two) {  // last odd level
        jt1[x] = pp;
        js2[x] = s1;
        return;
    }
    jt1[x] = pp;
    const uint32_t q = jt[pp];
    const uint32_t qq = jt[q];
    jt2[x] = qq;
    js2[x] = s1 + js[pp] + js[q];
}

// Exact cost of every position: an exit's is its path sum (js after the jumps, through its
// index in E), any other position adds its in-chunk bit sum to its exit's. A thread takes
// kRows consecutive positions of one chunk (the 64 lanes of a wave: 64 neighbouring chunks, so
// every row is one contiguous run); consecutive positions mostly share their exit, whose cost
// (cin and js through its index in E: dependent gathers) is then loaded once. (4 and 16 rows
// measured slower: C2 parse 3.52 -> 3.56 / 3.66 ms, mixed 8.26 -> 8.42 / 8.34 ms.)
constexpr uint32_t kRows = 8;
__global__ __launch_bounds__(kT) void k_cost_rest(ExitBits eb, const uint32_t *__restrict__ js,
                                                  const uint64_t *__restrict__ pst,
                                                  const uint32_t *__restrict__ cin, uint32_t n,
                                                  uint32_t klog, size_t S, uint32_t *cost,
                                                  const uint32_t *__restrict__ dsum)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t lane = (uint32_t)(x & 63u);
    const size_t rest = x >> 6;
    const uint32_t groups = (1u << klog) / kRows;
    const size_t t = rest / groups;
    const uint32_t g = (uint32_t)(rest % groups);
    if ((t << (klog + 6)) >= S)
        return;
    const uint32_t c = (uint32_t)(t * 64 + lane);  // chunk
    const size_t s0 = (t << (klog + 6)) | ((size_t)(g * kRows) << 6) | lane;
    if (spos(s0, klog) > n)
        return;  // (rows ascend: none of this thread's is a position)
    const uint32_t shift = (uint64_t)c << klog < n ? dsum[c] : 0u;
    // All rows at once, every load unconditional (rows past n repeat row 0, whose store then
    // repeats too): the state and mask word per row, then each row's exit index and costs. One
    // chain of three dependent latencies per thread instead of one per row.
    size_t sr[kRows];
    uint64_t v[kRows], mw[kRows];
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++) {
        const size_t s = s0 | ((size_t)r << 6);
        sr[r] = spos(s, klog) <= n ? s : s0;
        v[r] = pst[sr[r]];
        mw[r] = eb.mask[sr[r] >> 6];
    }
    uint32_t se[kRows];
    bool isx[kRows];
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++) {
        isx[r] = (mw[r] >> lane) & 1u;  // an exit node: its own path sum
        se[r] = isx[r] ? (uint32_t)sr[r] : (uint32_t)sidx((uint32_t)v[r], klog);
    }
    // The rows of a thread are consecutive positions of one chunk, whose paths mostly leave it
    // through the same exit: a row's cost comes from the node at its key slot se (its exit, or
    // itself when it is an exit node), and when every lane's rows have at most three distinct key
    // slots (a wave-uniform test) their index and cost loads are issued once per distinct slot
    // (12 scattered loads instead of 32: the kernel's time was the address processing of the
    // scattered loads).
    uint32_t kA = se[0], kB = kA, kC = kA;
#pragma unroll
    for (uint32_t r = 1; r < kRows; r++) {
        kB = kB == kA && se[r] != kA ? se[r] : kB;
        kC = kC == kA && se[r] != kA && se[r] != kB ? se[r] : kC;
    }
    bool few = true;
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++)
        few = few && (se[r] == kA || se[r] == kB || se[r] == kC);
    uint32_t out[kRows];
    if (wave_ballot(!few) == 0) {
        const uint32_t xA = bits_index(eb.mask, eb.wpre, kA), xB = bits_index(eb.mask, eb.wpre, kB);
        const uint32_t xC = bits_index(eb.mask, eb.wpre, kC);
        const uint32_t jA = js[xA], jB = js[xB], jC = js[xC], cA = cin[kA], cB = cin[kB], cC = cin[kC];
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++) {
            const bool a = se[r] == kA, b = se[r] == kB;
            const uint32_t jv = a ? jA : b ? jB : jC, cv = a ? cA : b ? cB : cC;
            out[r] = jv + (((uint32_t)(v[r] >> 32) + shift - cv) & (isx[r] ? 0u : 0xffffffffu));
        }
    } else {
        uint32_t xe[kRows];
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++) {
            const uint64_t m2 = eb.mask[se[r] >> 6];
            xe[r] = eb.wpre[se[r] >> 6] + (uint32_t)__popcll(m2 & ((1ull << (se[r] & 63u)) - 1ull));
        }
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++) {
            const uint32_t jv = js[xe[r]], cv = cin[se[r]];
            out[r] = jv + (((uint32_t)(v[r] >> 32) + shift - cv) & (isx[r] ? 0u : 0xffffffffu));
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++)
        cost[sr[r]] = sr[r] == s0 ? out[0] : out[r];
}

// Lazy passes, after the exact costs of the exit set: per chunk, whether its costs all moved by
// one delta (no decision changed in this pass's walk, at most kSumm (8) distinct exits, all
// moving by the same delta, every exit cost before and after under 2^30 - 2^20 so that no cost of
// the chunk reaches 2^30: a path inside one chunk adds far less than 2^20, and no compare wraps)
// -> Lnew = Lcur + delta; otherwise the chunk is rewritten (k_lazy_rewrite) with offset 0.
// (The bound was 2^29 on the new cost: a block whose stream passes 2^29 bits, mixed 256 MiB,
// rewrote the chunks of its first half in every pass.)
constexpr uint32_t kLazyMax = (1u << 30) - (1u << 20);
__global__ __launch_bounds__(kT) void k_lazy_chunks(uint32_t nchunks, const uint32_t *__restrict__ summ,
                                                    const uint8_t *__restrict__ chg, ExitBits eb,
                                                    const uint32_t *__restrict__ js, const uint32_t *__restrict__ ce,
                                                    const uint32_t *__restrict__ Lcur, uint32_t *__restrict__ Lnew,
                                                    uint32_t *__restrict__ dl, uint8_t *__restrict__ uni, uint32_t klog,
                                                    uint32_t n)
{
    const uint32_t c = blockIdx.x * kT + threadIdx.x;
    if (c >= nchunks)
        return;
    const uint32_t *sm = summ + kSummW * (size_t)c;
    bool u = !chg[c] && !sm[kSumm];
    uint32_t d0 = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSumm; k++) {
        const uint32_t e = sm[k] < n ? sm[k] : n;  // (every walked chunk has an exit)
        const uint32_t x = bits_index(eb.mask, eb.wpre, sidx(e, klog));
        const uint32_t v = js[x], d = v - ce[x];
        d0 = k == 0 ? d : d0;
        u &= d == d0 && v < kLazyMax && ce[x] < kLazyMax;
    }
    uni[c] = u ? 1u : 0u;
    dl[c] = d0;
    Lnew[c] = u ? Lcur[c] + d0 : 0u;
}

// The rewritten chunks of a lazy pass (k_cost_rest's shape and formula): C = the new exact cost
// (offset 0), D = new - old (the shift the next test reads).
__global__ __launch_bounds__(kT) void k_lazy_rewrite(ExitBits eb, const uint32_t *__restrict__ js,
                                                     const uint64_t *__restrict__ pst,
                                                     const uint32_t *__restrict__ ce, uint32_t n,
                                                     uint32_t klog, size_t S, uint32_t *__restrict__ C,
                                                     uint32_t *__restrict__ D, const uint32_t *__restrict__ Lcur,
                                                     const uint8_t *__restrict__ uni,
                                                     const uint32_t *__restrict__ dsum, uint32_t nchunks)
{
    const size_t x = (size_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t lane = (uint32_t)(x & 63u);
    const size_t rest = x >> 6;
    const uint32_t groups = (1u << klog) / kRows;
    const size_t t = rest / groups;
    const uint32_t g = (uint32_t)(rest % groups);
    if ((t << (klog + 6)) >= S)
        return;
    const uint32_t c = (uint32_t)(t * 64 + lane);  // chunk
    const uint32_t cc = c < nchunks ? c : 0u;  // (the chunk's words loaded together, unconditionally)
    const uint32_t shift = dsum[cc], lc = Lcur[cc];
    if (c >= nchunks || uni[cc])
        return;
    const size_t s0 = (t << (klog + 6)) | ((size_t)(g * kRows) << 6) | lane;
    if (spos(s0, klog) > n)
        return;
    // k_cost_rest's shape: every row's loads first (rows past n repeat row 0), an exit node's own
    // slot standing in for its exit, and one index / pre-pass cost load per distinct exit when the
    // wave's rows have few
    size_t sr[kRows];
    uint64_t v[kRows], mw[kRows];
    uint32_t old[kRows];
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++) {
        const size_t sq = s0 | ((size_t)r << 6);
        sr[r] = spos(sq, klog) <= n ? sq : s0;
        old[r] = C[sr[r]] + lc;
        v[r] = pst[sr[r]];
        mw[r] = eb.mask[sr[r] >> 6];
    }
    uint32_t se[kRows];
    bool isx[kRows];
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++) {
        isx[r] = (mw[r] >> lane) & 1u;
        se[r] = isx[r] ? (uint32_t)sr[r] : (uint32_t)sidx((uint32_t)v[r], klog);
    }
    uint32_t kA = se[0], kB = kA, kC = kA;  // (k_cost_rest's distinct key slots)
#pragma unroll
    for (uint32_t r = 1; r < kRows; r++) {
        kB = kB == kA && se[r] != kA ? se[r] : kB;
        kC = kC == kA && se[r] != kA && se[r] != kB ? se[r] : kC;
    }
    bool few = true;
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++)
        few = few && (se[r] == kA || se[r] == kB || se[r] == kC);
    uint32_t out[kRows];
    if (wave_ballot(!few) == 0) {
        const uint32_t xA = bits_index(eb.mask, eb.wpre, kA), xB = bits_index(eb.mask, eb.wpre, kB);
        const uint32_t xC = bits_index(eb.mask, eb.wpre, kC);
        const uint32_t jA = js[xA], jB = js[xB], jC = js[xC], cA = ce[xA], cB = ce[xB], cC = ce[xC];
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++) {
            const bool a = se[r] == kA, b = se[r] == kB;
            const uint32_t jv = a ? jA : b ? jB : jC, cv = a ? cA : b ? cB : cC;
            out[r] = jv + (((uint32_t)(v[r] >> 32) + shift - cv) & (isx[r] ? 0u : 0xffffffffu));
        }
    } else {
        uint32_t xe[kRows];
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++)
            xe[r] = bits_index(eb.mask, eb.wpre, se[r]);
#pragma unroll
        for (uint32_t r = 0; r < kRows; r++) {
            const uint32_t jv = js[xe[r]], cv = ce[xe[r]];
            out[r] = jv + (((uint32_t)(v[r] >> 32) + shift - cv) & (isx[r] ? 0u : 0xffffffffu));
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < kRows; r++) {
        D[sr[r]] = out[r] - old[r];
        C[sr[r]] = out[r];
    }
}

// Lazy breaks for the range test: brk[k] = 1 when the shift may change inside (kK, (k + 1)K]: chunk
// k or k + 1 rewritten, or their deltas differ (entries past the last chunk are uniform, delta 0).
__global__ __launch_bounds__(kT) void k_lazy_breaks(const uint8_t *__restrict__ uni, const uint32_t *__restrict__ dl,
                                                    uint32_t nchunks, uint32_t *__restrict__ brk)
{
    const uint32_t k = blockIdx.x * kT + threadIdx.x;
    if (k == 0)
        brk[nchunks] = 0u;  // (the scan's last entry)
    if (k >= nchunks)
        return;
    brk[k] = !uni[k] || !uni[k + 1] || dl[k] != dl[k + 1] ? 1u : 0u;
}

// Exact costs of a lazy parse (C + L) into out (the debug dump's cost array).
__global__ __launch_bounds__(kT) void k_lazy_materialize(const uint32_t *__restrict__ C, const uint32_t *__restrict__ L,
                                                         uint32_t n, uint32_t klog, size_t S, uint32_t *__restrict__ out)
{
    const size_t s = (size_t)blockIdx.x * kT + threadIdx.x;
    if (s >= S)
        return;
    const uint64_t p = spos(s, klog);
    out[s] = p <= n ? C[s] + L[p >> klog] : 0u;
}

}  // namespace

int parse_materialize_cost(Workspace &ws)
{
    ParseState &ps = ws.parse;
    if (!ps.lzC)
        return 0;
    const size_t tile = (size_t)kTileChunks << ws.klog;
    const uint32_t n = ps.lzn;
    const size_t S = ((size_t)n + 1 + tile - 1) / tile * tile;
    hipLaunchKernelGGL(k_lazy_materialize, dim3(grid_for(S, kT)), dim3(kT), 0, ws.stream, ps.lzC, ps.lzL, n, ws.klog, S,
                       ps.lzD);
    SALZ_LAUNCH_CHECK();
    ps.cost = ps.lzD;
    ps.lzC = nullptr;
    return 0;
}

// Chunk length from the block length N (bytes; n = N - 8 positions): the largest K <= 512
// that leaves MORE than 2^17 chunks (two waves per SIMD) for blocks up to 32 MiB, and more
// than 2^16 for larger blocks, whose longest chunks need fewer passes (64 MiB text blocks: 3
// passes instead of 4 at K = 512, C4 +7.7%), while 16 MiB mixed blocks measured slower with
// longer chunks. So: 1 MiB and 16 MiB blocks -> K = 64, 24 MB -> 128, 32 MiB -> 128,
// 32 MiB + 8 -> 256, 64 MiB / 100 MB / 256 MiB -> 512 (tests/test_abi.py pins these).
uint32_t parse_chunk_log(size_t N)
{
    const long k = env_num("SALZ_PARSE", "klog", 0);  // tests: force a chunk length
    if (k >= 6 && k <= (long)kMaxChunkLog)
        return (uint32_t)k;
    const uint64_t min_chunks = N > (1ull << 25) ? (1ull << 16) : (1ull << 17);
    uint32_t klog = kMaxChunkLog;
    while (klog > 6 && ((uint64_t)N >> klog) <= min_chunks)
        klog--;
    return klog;
}

int stage_parse(Workspace &ws, const Blocks &bl)
{
    const uint32_t n = bl.npos;
    hipStream_t st = ws.stream;
    ParseState &ps = ws.parse;
    const uint32_t klog = ws.klog;
    ps.chunk = 1u << klog;
    ps.nchunks = (n + ps.chunk - 1) / ps.chunk;
    const size_t tile = (size_t)kTileChunks << klog;
    const size_t S = ((size_t)n + 1 + tile - 1) / tile * tile;  // slots covering 0..n
    if (S > ws.cap_s) {
        set_error("parse: layout exceeds workspace (%zu > %zu)", S, ws.cap_s);
        return -1;
    }
    uint32_t *cost[2] = {ws.u0, ws.u1};
    uint8_t *choice[2] = {reinterpret_cast<uint8_t *>(ws.valA), reinterpret_cast<uint8_t *>(ws.valB)};
    uint8_t *eflag = reinterpret_cast<uint8_t *>(ws.offA);  // exit flags, one byte per slot
    // the same set as bits + word prefix counts (S / 4 bytes in offB; emission reads them)
    ExitBits eb{reinterpret_cast<uint64_t *>(ws.offB), nullptr, nullptr};
    eb.wcnt = reinterpret_cast<uint32_t *>(eb.mask + S / 64);
    eb.wpre = eb.wcnt + S / 64;
    ps.ebits = eb;
    uint32_t *elist = ws.rank;
    uint32_t *js[2] = {reinterpret_cast<uint32_t *>(ws.keyA),
                       reinterpret_cast<uint32_t *>(ws.keyA) + (ws.cap_n + 1)};
    uint32_t *snap = reinterpret_cast<uint32_t *>(ws.keyB);
    const size_t snap_cap = 2 * (ws.cap_n + 1);
    uint32_t *changed = reinterpret_cast<uint32_t *>(ws.dscal) + 48;
    uint32_t *etotal = reinterpret_cast<uint32_t *>(ws.dscal) + 49;
    uint32_t *ndirty = reinterpret_cast<uint32_t *>(ws.dscal) + 50;
    static const bool verbose = env_flag("SALZ_DEBUG", "parse");
    // Wave skipping from the third pass on (k_parse_mark); SALZ_PARSE=noskip runs every chunk
    // every pass (tests compare both).
    const bool skip_on = !env_flag("SALZ_PARSE", "noskip");
    // per chunk: uniform cost shift since its last pass; per wave: dirty flag (lsc is free here)
    uint32_t *dsum = reinterpret_cast<uint32_t *>(ws.lsc);
    uint8_t *wdirty = reinterpret_cast<uint8_t *>(dsum + ps.nchunks);
    SALZ_HIP(fill_async(dsum, 0, sizeof(uint32_t) * ps.nchunks, st));
    // Range test of k_parse_mark: each chunk's farthest target, and per test the shift breaks per
    // chunk and their prefix counts.
    uint32_t *reach = dsum + 2 * ((size_t)ps.nchunks + 64);
    uint32_t *brk = reach + ps.nchunks + 64, *pbrk = brk + ps.nchunks + 64;
    // Packed candidates from the second pass on (g64 is free during the parse)
    const bool pack = n < kPackLen;
    uint2 *cand8 = pack ? reinterpret_cast<uint2 *>(ws.g64) : nullptr;
    // Lazy costs from the first skipping pass on: per-chunk offsets (two generations), deltas,
    // uniform / changed flags, exit summaries, and the pre-pass cost of every exit node.
    const bool lazy_on = skip_on;
    const size_t nc64 = (size_t)ps.nchunks + 64;
    uint32_t *Lv[2] = {pbrk + nc64, pbrk + 2 * nc64};
    uint32_t *dl = pbrk + 3 * nc64;
    uint8_t *uni = reinterpret_cast<uint8_t *>(pbrk + 4 * nc64), *chg = uni + nc64;
    uint32_t *summ = pbrk + 5 * nc64;
    uint32_t *rlo = pbrk + (5 + kSummW) * nc64;  // per chunk: first row reaching past its end
    // split test: the chunks the range test does not pass get a wave each (k_mark_rows)
    uint32_t *ms_count = reinterpret_cast<uint32_t *>(ws.dscal) + 51;
    const MarkSplit ms{pbrk + (6 + kSummW) * nc64, ms_count,
                       reinterpret_cast<uint8_t *>(pbrk + (8 + kSummW) * nc64), pbrk + (7 + kSummW) * nc64};
    uint32_t *ce = pbrk + (9 + kSummW) * nc64;
    // per 64-chunk tile: exit flags set by this pass's walk (skipping passes)
    const size_t ntiles = S / tile;
    uint8_t *ttouch = reinterpret_cast<uint8_t *>(ce + ws.cap_n + 2);
    if ((size_t)(ce - reinterpret_cast<uint32_t *>(ws.lsc)) + ws.cap_n + 2 + ntiles / 4 + 1 >
        4 * (ws.cap_s > ws.cap_n + 2 ? ws.cap_s : ws.cap_n + 2)) {
        set_error("parse: lazy-cost scratch does not fit");
        return -1;
    }
    bool lazy = false;
    int lc = 0;
    uint32_t prev_listed = ps.nchunks;  // chunks the last split test listed (sizes k_mark_rows' grid)
    uint32_t *lzC = nullptr, *lzD = nullptr;
    ps.lzC = nullptr;

    hipLaunchKernelGGL(k_cost_seed, dim3(grid_for(S, kT)), dim3(kT), 0, st, cost[0], bl, klog, S);
    SALZ_LAUNCH_CHECK();
    // (no choice array init: the first pass writes every slot's choice and counts every live
    // position as changed)
    // counters changed (48), ndirty (50), listed chunks (51): zeroed here, then by the scalar reads
    // that consume them
    SALZ_HIP(fill_async(changed, 0, 16, st));

    ps.pst = ws.pst;
    ps.n_exit = 0;
    ps.levels = 0;
    int it = 0;
    uint32_t prev_changed = 0xffffffffu;
    for (;; it++) {
        const int cur = it & 1;
        uint32_t *cin = lazy ? lzC : cost[cur], *cout = lazy ? lzD : cost[cur ^ 1];
        // Choices are updated in place (chold == chnew, not restrict): a lane reads a position's
        // old choice kDepth steps before it writes the new one, and a clean wave keeps its choices
        // without a copy.
        (void)cur;
        uint8_t *chold = choice[0], *chnew = choice[0];
        // From the third pass on, waves of chunks whose decisions would repeat skip the pass,
        // and a pass with no dirty wave left walks no chunk (every wave clean) and ends the loop
        // at its host read: the previous decisions are the fixed point and cin their exact costs
        // (k_parse_mark, DESIGN.md "Parse"). The test
        // costs about a third of a pass. A large block's pass is latency-bound (its duration is
        // one lane's walk, however few waves run), so there it pays only as the stopping test:
        // before the third pass when the second changed few decisions (text stops there), later
        // once almost none change. Smaller blocks, encoded several at a time, where skipped waves
        // save throughput, run it before every pass from the third.
        const bool late = (uint64_t)prev_changed * 64 < n &&
                          (it == 2 || (uint64_t)prev_changed * 4096 < n);
        // (with lazy costs the test is cheap after its first pass: large blocks skip from the third
        // pass too)
        const bool skipping = it >= 2 && (n < (1u << 25) || late || lazy_on);
        // The first skipping pass enters the lazy costs (its test still reads the cost arrays).
        // (Entering at the second pass, so that the first test reads the shifts per chunk, was
        // slower on text: C2 parse 4.09 -> 4.23 ms, its second pass changes too many chunks.)
        const bool entering = lazy_on && skipping && !lazy;
        if (skipping) {
            LazyTest lt{lazy ? Lv[lc] : nullptr, uni, dl, lzD};
            if (lazy) {
                hipLaunchKernelGGL(k_lazy_breaks, dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, uni, dl, ps.nchunks,
                                   brk);
                SALZ_LAUNCH_CHECK();
                if (scan_sum_u32(brk, pbrk, (size_t)ps.nchunks + 1, false, nullptr, ws, st) != 0)
                    return -1;
            } else {
                SALZ_HIP(fill_async(brk, 0, sizeof(uint32_t) * ((size_t)ps.nchunks + 1), st));
                const size_t bthreads = (size_t)((ps.nchunks + 63) / 64) * 64 * (ps.chunk / kRowsBrk);
                hipLaunchKernelGGL(k_shift_breaks, dim3(grid_for(bthreads, kT)), dim3(kT), 0, st, cin, cout, n, klog,
                                   ps.nchunks, brk);
                SALZ_LAUNCH_CHECK();
                if (scan_sum_u32(brk, pbrk, (size_t)ps.nchunks + 1, false, nullptr, ws, st) != 0)
                    return -1;
            }
            hipLaunchKernelGGL(k_parse_mark, dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, cin, cout, n, bl, klog,
                               reach, pbrk, lt, ms);
            SALZ_LAUNCH_CHECK();
            {  // listed chunks: a wave each (2048 waves, grid-stride), then the wave flags
                // waves: the previous test's list length (lists shrink from pass to pass; any count is
                // served by the grid-stride loop), 64 to 16384; the first test lists up to every chunk
                const uint32_t per = klog >= 9 ? 1u : 512u >> klog;  // chunks per wave
                const uint32_t wv = (prev_listed + per - 1) / per;
                const uint32_t want = wv < 64 ? 64u : wv > 16384 ? 16384u : wv;
                const uint32_t rgrid = (want + kT / 64 - 1) / (kT / 64);
                if (pack)
                    hipLaunchKernelGGL(k_mark_rows<CandPacked>, dim3(rgrid), dim3(kT), 0, st, cand8, cin, cout, n, bl,
                                       klog, rlo, lt, ms);
                else
                    hipLaunchKernelGGL(k_mark_rows<CandFull>, dim3(rgrid), dim3(kT), 0, st, ws.cand, cin, cout, n, bl,
                                       klog, rlo, lt, ms);
                SALZ_LAUNCH_CHECK();
                hipLaunchKernelGGL(k_mark_final, dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, n, klog, ms.cbad, ms.d0s,
                                   wdirty, dsum, ndirty);
                SALZ_LAUNCH_CHECK();
            }
            // (no host read here: a pass with no dirty wave runs its chunk pass as a no-op, every
            // wave clean, and stops at the read below with nothing changed)
        }
        if (entering) {  // offsets 0 (entries past the last chunk: uniform, delta 0)
            SALZ_HIP(fill_async(Lv[0], 0, sizeof(uint32_t) * 4 * nc64, st));  // Lv[0], Lv[1], dl
            SALZ_HIP(fill_async(uni, 1, nc64, st));
        }
        // Exit flags accumulate once waves skip passes: a skipped chunk's exits stay marked
        // from the pass that chose them (stale exits only add nodes to the forest).
        if (!skipping)
            SALZ_HIP(fill_async(eflag, 0, S, st));
        uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
        uint8_t *wd = skipping && skip_on ? wdirty : nullptr;
        uint8_t *tt = wd ? ttouch : nullptr;  // (flags accumulate only while waves skip)
        // (tile flags carry the pass's generation 1..255: reset once every 255 passes, not per pass)
        const uint32_t tgen = (uint32_t)(it % 255) + 1u;
        if (ttouch && tgen == 1u)
            SALZ_HIP(fill_async(ttouch, 0, ntiles, st));
        uint32_t *rch = it == 0 ? reach : nullptr;
        const Lazy lzw{lazy ? Lv[lc] : nullptr, lazy_on ? summ : nullptr, lazy_on ? chg : nullptr};
        // Chunks of K <= 128 (non-text and mid-size blocks) prefetch far targets 1 step and
        // candidates 3 steps ahead instead of 4 and 7: mixed 100 MB parse 8.22 -> 7.9 ms, Silesia
        // blocks 3.1 -> 2.9 ms (profiles/r04zi_parse_near_prefetch_ab.txt); text at K = 512 is
        // 0.03 ms slower so
        // From the fourth pass on, where few waves walk and a pass is one lane's latency chain,
        // the 4 / 7 distances again (from the fourth pass: mixed 100 MB parse 7.88 -> 7.77 ms, 7.79
        // from the sixth, Silesia-sized blocks even to +1%: r05fl_parse_farlate_ab.txt)
        constexpr int far_late = 3;
        const bool near = klog <= 7 && it < far_late;
        if (pack && it > 0)
            hipLaunchKernelGGL((near ? k_parse_chunk<CandPacked, 1, 3> : k_parse_chunk<CandPacked, 4, 7>),
                               dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, cand8,
                               nullptr, cin, ws.pst, chold, chnew, n, bl, klog, changed, derr, eflag, wd, dsum, rch,
                               rlo, lzw, it == 0 ? 1 : 0, tt, tgen);
        else
            hipLaunchKernelGGL((near ? k_parse_chunk<CandFull, 1, 3> : k_parse_chunk<CandFull, 4, 7>),
                               dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, ws.cand,
                               it == 0 ? cand8 : nullptr, cin, ws.pst, chold, chnew, n, bl, klog, changed, derr,
                               eflag, wd, dsum, rch, rlo, lzw, it == 0 ? 1 : 0, tt, tgen);
        SALZ_LAUNCH_CHECK();
        // The exit set of the new decisions (E was marked by the chunk pass) as bits and word
        // counts, numbered by the scan, before the pass's one host read: that read then returns
        // the changed count, |E| (etotal), the dirty waves and the chunks the test listed
        // together. A pass that changed nothing leaves E as it was, so these are unchanged then.
        // Packing is skipped on "no dirty wave" only when the walk itself skipped the clean waves
        // (wd): under SALZ_PARSE=noskip every chunk is walked and E is packed every pass.
        hipLaunchKernelGGL(k_exit_pack, dim3(grid_for(S / 8, kT)), dim3(kT), 0, st,
                           reinterpret_cast<const uint64_t *>(eflag), S / 8, eb, wd ? ndirty : nullptr, tt, tgen, klog);
        SALZ_LAUNCH_CHECK();
        if (scan_sum_u32(eb.wcnt, eb.wpre, S / 64, false, etotal, ws, st) != 0)
            return -1;
        if (read_scalars(ws, 0, 256, "parse.pass", 48, 4) != 0)  // (changed, ndirty, listed reset)
            return -1;
        const uint32_t nchanged = reinterpret_cast<uint32_t *>(ws.hscal)[48];
        if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
            set_error("parse: device index check failed (code 0x%x): candidate length past the end", e);
            return -1;
        }
        if (skipping)
            prev_listed = reinterpret_cast<uint32_t *>(ws.hscal)[51];
        if (verbose) {
            if (skipping)
                fprintf(stderr, "parse it=%d dirty waves %u of %u\n", it, reinterpret_cast<uint32_t *>(ws.hscal)[50],
                        (ps.nchunks + 63) / 64);
            fprintf(stderr, "parse it=%d K=%u changed=%u\n", it, ps.chunk, nchanged);
        }
        if (nchanged == 0) {
            ps.choice = chnew;
            ps.cost = cin;
            break;
        }
        const bool lz_pass = lazy || entering;  // this pass updates the costs lazily
        prev_changed = nchanged;
        // After t passes the last t chunks hold exact decisions (the last one sees only exact
        // costs, then induction), so nchunks + 1 passes always suffice.
        if ((uint32_t)it > ps.nchunks + 1) {
            set_error("parse fixed point did not converge");
            return -1;
        }
        // Exact costs for the new decisions.
        const uint32_t ne = reinterpret_cast<uint32_t *>(ws.hscal)[49];
        const uint32_t K = (uint32_t)bit_width(ne > 1 ? ne - 1 : 0);
        // Every level's parents are kept for emission's path marking when they fit (the usual
        // case); a large E (short factors in short chunks) keeps level 0 only and jumps
        // through two ping-pong buffers, and emission recomputes the levels.
        const bool snaps = (size_t)(K + 1) * ne <= snap_cap;
        if (ne > ws.cap_n + 2) {
            set_error("parse: exit set larger than the text (|E|=%u)", ne);
            return -1;
        }
        if ((uint64_t)ne * 64 < S) {  // sparse E: a thread per node
            const size_t nw = S / 64;
            uint32_t *nword = ws.lcps;  // (the LCP array: read by the candidates stage only)
            hipLaunchKernelGGL(k_node_words, dim3(grid_for(nw, kT)), dim3(kT), 0, st, eb, nw, nword);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_compact_nodes, dim3(grid_for(ne, kT)), dim3(kT), 0, st, eb, nword, ne, ws.pst,
                               cin, n, klog, elist, snap, js[0], dsum, lz_pass ? Lv[lc] : nullptr,
                               lz_pass ? ce : nullptr);
        } else {
            hipLaunchKernelGGL(k_compact_exits, dim3(grid_for(S / 8, kT)), dim3(kT), 0, st, eb, ws.pst, cin, n, klog,
                               S / 8, elist, snap, js[0], dsum, lz_pass ? Lv[lc] : nullptr, lz_pass ? ce : nullptr);
        }
        SALZ_LAUNCH_CHECK();
        int jc = 0;
        if (snaps) {
            for (uint32_t k = 0; k < K;) {
                if (k + 3 <= K && (size_t)(k + 4) * ne <= snap_cap) {
                    hipLaunchKernelGGL(k_jump3, dim3(grid_for(ne, kT)), dim3(kT), 0, st, snap + (size_t)k * ne, js[jc],
                                       snap + (size_t)(k + 1) * ne, snap + (size_t)(k + 2) * ne,
                                       snap + (size_t)(k + 3) * ne, js[jc ^ 1], ne);
                    SALZ_LAUNCH_CHECK();
                    jc ^= 1;
                    k += 3;
                    continue;
                }
                const int two = k + 1 < K;
                hipLaunchKernelGGL(k_jump2, dim3(grid_for(ne, kT)), dim3(kT), 0, st,
                                   snap + (size_t)k * ne, js[jc], snap + (size_t)(k + 1) * ne,
                                   two ? snap + (size_t)(k + 2) * ne : nullptr, js[jc ^ 1], ne, two);
                SALZ_LAUNCH_CHECK();
                jc ^= 1;
                k += 2;
            }
        } else {
            uint32_t *pp[2] = {ws.u2, ws.u3};  // free during the parse
            const uint32_t *cur = snap;
            for (uint32_t k = 0; k < K; k++) {
                hipLaunchKernelGGL(k_jump2, dim3(grid_for(ne, kT)), dim3(kT), 0, st, cur, js[jc],
                                   pp[k & 1], nullptr, js[jc ^ 1], ne, 0);
                SALZ_LAUNCH_CHECK();
                cur = pp[k & 1];
                jc ^= 1;
            }
        }
        if (lz_pass) {
            if (entering) {  // C = the exact costs this pass read; the other array holds the shifts
                lazy = true;
                lzC = cin;
                lzD = cout;
            }
            hipLaunchKernelGGL(k_lazy_chunks, dim3(grid_for(ps.nchunks, kT)), dim3(kT), 0, st, ps.nchunks, summ, chg,
                               eb, js[jc], ce, Lv[lc], Lv[lc ^ 1], dl, uni, klog, n);
            SALZ_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_lazy_rewrite, dim3(grid_for(S / kRows, kT)), dim3(kT), 0, st, eb, js[jc], ws.pst, ce,
                               n, klog, S, lzC, lzD, Lv[lc], uni, dsum, ps.nchunks);
            SALZ_LAUNCH_CHECK();
            if (verbose) {  // chunks: uniform, changed by the walk, more than two exits
                std::vector<uint8_t> hu(ps.nchunks), hc(ps.nchunks);
                std::vector<uint32_t> hs(kSummW * (size_t)ps.nchunks);
                SALZ_HIP(hipMemcpyAsync(hu.data(), uni, ps.nchunks, hipMemcpyDeviceToHost, st));
                SALZ_HIP(hipMemcpyAsync(hc.data(), chg, ps.nchunks, hipMemcpyDeviceToHost, st));
                SALZ_HIP(hipMemcpyAsync(hs.data(), summ, 4 * hs.size(), hipMemcpyDeviceToHost, st));
                SALZ_HIP(hipStreamSynchronize(st));
                size_t nu = 0, nc = 0, no = 0;
                for (uint32_t c = 0; c < ps.nchunks; c++) {
                    nu += hu[c];
                    nc += hc[c];
                    no += hs[kSummW * (size_t)c + kSumm] != 0;
                }
                fprintf(stderr, "parse it=%d lazy: %zu uniform, %zu changed, %zu over %u exits of %u chunks, |E| %u\n", it,
                        nu, nc, no, kSumm, ps.nchunks, ne);
            }
            lc ^= 1;
        } else {
            hipLaunchKernelGGL(k_cost_rest, dim3(grid_for(S / kRows, kT)), dim3(kT), 0, st, eb, js[jc], ws.pst, cin,
                               n, klog, S, cout, dsum);
            SALZ_LAUNCH_CHECK();
        }
        ps.n_exit = ne;
        ps.levels = K;
        ps.snaps = snaps;
        ps.elist = elist;
        ps.jt0 = snap;
    }
    if (lazy) {  // the exact costs are C + L (parse_materialize_cost writes them out on demand)
        ps.cost = nullptr;
        ps.lzC = lzC;
        ps.lzL = Lv[lc];
        ps.lzD = lzD;
        ps.lzn = n;
    }
    ws.stats.parse_iters = it + 1;
    ws.stats.exit_nodes = ps.n_exit;
    return 0;
}

}  // namespace salz
