// emit.hip - bit-exact stream emission (reference: emit_encoding + finalize_encoding,
// /root/reference/lib/salz.c:664-775, bit writer :258-457).
//
// The reference interleaves 8-byte control words with raw bytes, reserving each word
// lazily at the byte cursor when its first bit is written. In closed form (SURVEY.md
// Appendix A.3): number the bits B and raw bytes Y in emission order; a raw byte emitted
// after B bits lands at 4 + 8*ceil(B/64) + Y, and control word k lands at 4 + 8k + Y_k where
// Y_k = raw bytes emitted before bit 64k. So:
//   1. mark the parse path from position 0 through the exit forest (pointer-jumping
//      snapshots from parse.hip) and find each chunk's entry position;
//   2. per chunk, count the path's bits and bytes (the trailing 8 literals of T[n,N) are a
//      virtual last chunk); exclusive scans give each chunk its (B, Y) origin;
//   3. per chunk, walk again: bytes go straight to their final offsets, bits are assembled
//      MSB-first into 64-bit words (whole words stored plainly, the <=2 words shared with a
//      neighbouring chunk merged with atomicOr), and Y_k is recorded for each word start;
//   4. place every word at 4 + 8k + Y_k, then the 4-byte header. A stream longer than N + 4
//      is replaced by the PLAIN form (header + raw copy), as in :755-767.
// A batch of blocks (common.hpp, Blocks) emits one stream per block: chunks never straddle two
// blocks, every block's path starts at its first position, the 8 dead positions after its
// suffix text are its 8 trailing literals, and (B, Y) restart at each block's first chunk.
// Block b's words take W[wbase_b ..] (each block word-aligned) and its Y_k are stored offset
// by the block's first global byte index, so one max-scan serves every block.
#include "internal.hpp"

#include <vector>

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kNone = 0xffffffffu;

// Closed form of encode_vnibble_le (lib/salz.c:352-445): k octal digits of
// v - S_{k-1} (S_j = sum_{i=1..j} 8^i), most significant first, terminator bit on the last.
__device__ __forceinline__ uint64_t vn_bits(uint32_t v, uint32_t k)
{
    uint64_t s = 0, p = 8;
    for (uint32_t j = 1; j < k; j++) {
        s += p;
        p *= 8;
    }
    uint64_t d = (uint64_t)v - s, r = 0;
    for (uint32_t j = 0; j < k; j++) {
        uint64_t dig = (d >> (3 * j)) & 7u;
        if (j == 0)
            dig |= 8u;
        r |= dig << (4 * j);
    }
    return r;
}

// exit of every block's first position (the start of its path)
__global__ void k_mark_start(ExitBits eb, const uint64_t *__restrict__ pst, uint32_t klog,
                             uint32_t *__restrict__ emark, Blocks bl)
{
    const uint32_t b = blockIdx.x * kT + threadIdx.x;
    if (b >= bl.nb)
        return;
    const uint32_t p0 = b * (bl.nb == 1 ? 0u : bl.bs);
    emark[bits_index(eb.mask, eb.wpre, sidx((uint32_t)pst[sidx(p0, klog)], klog))] = 1u;
}

// One block's path in one launch (instead of a launch per level): thread j marks the path nodes at
// distances [j L, (j + 1) L) from the start, reaching its first by binary lifting over the parse's
// stored levels (parents 2^k steps up at jt + k ne), then walking level 0. The root is its own
// parent, so lifting or walking past the path's end stays there.
__global__ void k_mark_path(ExitBits eb, const uint64_t *__restrict__ pst, uint32_t klog, const uint32_t *__restrict__ jt,
                            uint32_t ne, uint32_t levels, uint32_t L, uint32_t nthreads, uint32_t *emark)
{
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= nthreads)
        return;
    const uint64_t d = (uint64_t)j * L;
    if (d >> levels || d > (uint64_t)ne)
        return;  // (beyond every path)
    uint32_t x = bits_index(eb.mask, eb.wpre, sidx((uint32_t)pst[sidx(0u, klog)], klog));  // the start's exit
    for (uint32_t k = 0; k < levels; k++)
        if ((d >> k) & 1u)
            x = jt[(size_t)k * ne + x];
    for (uint32_t i = 0; i < L; i++) {
        emark[x] = 1u;
        const uint32_t nx = jt[x];
        if (nx == x)
            break;
        x = nx;
    }
}

__global__ void k_mark_step(const uint32_t *__restrict__ jt, uint32_t *emark, uint32_t ne)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x < ne && emark[x])
        emark[jt[x]] = 1u;
}

// next pointer-jumping level of the E forest's parents (emission without stored levels)
__global__ void k_jt_double(const uint32_t *__restrict__ jt, uint32_t *__restrict__ jt2, uint32_t ne)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x < ne)
        jt2[x] = jt[jt[x]];
}

__global__ void k_entries(const uint32_t *__restrict__ emark, const uint32_t *__restrict__ elist,
                          uint32_t ne, uint32_t n, uint32_t chunk, uint32_t *__restrict__ entry)
{
    uint32_t x = blockIdx.x * kT + threadIdx.x;
    if (x >= ne || !emark[x])
        return;
    uint32_t q = elist[x];
    // The smallest marked exit of a chunk is where the path enters it. A batch's path may also
    // mark the dead position after a block's suffix text inside the block's last chunk (a
    // factor ending exactly there exits to it): it is the entry only when nothing earlier is.
    if (q < n)
        atomicMin(&entry[q / chunk], q);
}

struct Token {
    uint32_t len, off;  // len 1 = literal
};

__device__ __forceinline__ Token token_at(const uint4 *cand, const uint8_t *choice, uint32_t p,
                                          uint32_t klog)
{
    // both loads issued together (one memory latency per token of the path walk, not two)
    const size_t s = sidx(p, klog);
    const uint8_t ch = choice[s];
    const uint4 c = cand[s];
    return ch == 0 ? Token{1u, 0u} : ch == 1 ? Token{c.y, c.x} : Token{c.w, c.z};
}

// Path walk range of chunk g: from its entry (a block's first chunk: the block's first
// position) to its end; a batch's non-last block walks its dead positions as literals, the
// last block's 8 trailing literals are the virtual chunk nch.
__device__ __forceinline__ uint32_t walk_start(const uint32_t *entry, uint32_t g, uint32_t chunk,
                                               const Blocks &bl)
{
    const uint32_t a = g * chunk;
    return a == bl.start(a) ? a : entry[g];
}

__device__ __forceinline__ uint32_t walk_end(uint32_t g, uint32_t chunk, const Blocks &bl)
{
    const uint32_t a = g * chunk;
    const uint32_t e = bl.blk(a) + 1u < bl.nb ? a + chunk : bl.npos;
    return (e - a) < chunk ? e : a + chunk;
}

// A chunk's token records (the path walk of k_emit_count, read back by k_emit_write): token k of
// chunk g at slot tok_slot(g, k), the chunk-interleaved layout of common.hpp (the 64 lanes of a
// wave store and load their k-th tokens as one contiguous run). A record is len << 32 | off for
// a factor and 1 << 32 | byte for a literal; a chunk's walk covers at most K positions, so at
// most K tokens.
__device__ __forceinline__ size_t tok_slot(uint32_t g, uint32_t k, uint32_t klog)
{
    return (((size_t)(g >> 6) << (klog + 6)) | (g & 63u)) + ((size_t)k << 6);
}

// Per chunk: the path's bits and raw bytes (scanned into the chunks' origins) and its tokens.
// The walk is a chain of dependent loads (the next position is this token's length past it);
// the writing pass then reads the records back in batches instead of walking again.
__global__ void k_emit_count(const uint4 *__restrict__ cand, const uint8_t *__restrict__ choice,
                             const uint8_t *__restrict__ T, const uint32_t *__restrict__ entry, Blocks bl,
                             uint32_t N_last, uint32_t chunk, uint32_t nch, uint64_t *__restrict__ cbits,
                             uint64_t *__restrict__ cbytes, uint32_t klog, uint64_t *__restrict__ tok,
                             uint32_t *__restrict__ ntok)
{
    uint32_t g = blockIdx.x * kT + threadIdx.x;
    if (g > nch)
        return;
    uint64_t bits = 0, bytes = 0;
    uint32_t k = 0;
    if (g == nch) {
        bits = N_last - bl.n_last();
        bytes = N_last - bl.n_last();
    } else {
        uint32_t p = walk_start(entry, g, chunk, bl);
        if (p != kNone) {
            const uint32_t b = walk_end(g, chunk, bl), e = bl.end(g * chunk);
            while (p < b) {
                // (the text byte is loaded with the token, unconditionally: the text is padded)
                const uint32_t lit = T[p];
                Token t = p < e ? token_at(cand, choice, p, klog) : Token{1u, 0u};
                uint64_t rec;
                if (t.len == 1) {
                    bits += 1;
                    bytes += 1;
                    rec = (1ull << 32) | lit;
                } else {
                    uint32_t gl = t.len - 3u;
                    bits += 1u + 4u * vn_size((t.off - 1u) >> 8) + (gl >> 3) + 4u;
                    bytes += 1;
                    rec = ((uint64_t)t.len << 32) | t.off;
                }
                tok[tok_slot(g, k, klog)] = rec;
                k++;
                p += t.len;
            }
        }
    }
    cbits[g] = bits;
    cbytes[g] = bytes;
    ntok[g] = k;
}

struct Sink {
    uint64_t *W;     // the block's words (W + wbase)
    uint32_t *Yk;    // the block's Y_k (Yk + wbase), stored + ys
    uint8_t *out;    // the block's stream
    uint64_t B, B0, B1, Y;  // block-local
    uint64_t cur, kc;
    uint32_t ys;     // the block's first global byte index
    bool have;

    __device__ __forceinline__ void flush()
    {
        if (have && cur) {
            bool own = kc * 64 >= B0 && kc * 64 + 64 <= B1;
            if (own)
                W[kc] = cur;
            else
                atomicOr(reinterpret_cast<unsigned long long *>(&W[kc]),
                         (unsigned long long)cur);
        }
        have = false;
        cur = 0;
    }
    __device__ __forceinline__ void enter(uint64_t k)
    {
        if (!have || k != kc) {
            flush();
            kc = k;
            have = true;
        }
    }
    __device__ __forceinline__ void put(uint64_t v, uint32_t cnt)  // cnt <= 64
    {
        while (cnt) {
            uint64_t k = B >> 6;
            uint32_t o = (uint32_t)(B & 63);
            uint32_t take = cnt < 64 - o ? cnt : 64 - o;
            uint64_t chunk = (v >> (cnt - take)) & (take == 64 ? ~0ull : ((1ull << take) - 1));
            enter(k);
            if (o == 0)
                Yk[k] = ys + (uint32_t)Y;
            cur |= chunk << (64 - o - take);
            B += take;
            cnt -= take;
        }
    }
    // A zero run: the words it covers whole are left as they are (W is zeroed beforehand; the
    // first one's Yk is written, the others' (0 here) are filled in by a max-scan, as no raw
    // byte is emitted inside the run),
    // so a factor of length L costs O(1) rather than O(L / 512) (Fibonacci: runs of 10^7 bits).
    __device__ __forceinline__ void zeros(uint64_t cnt)
    {
        if (!cnt)
            return;
        uint64_t k = B >> 6;
        uint32_t o = (uint32_t)(B & 63);
        const uint64_t take = cnt < (uint64_t)(64 - o) ? cnt : (uint64_t)(64 - o);
        enter(k);
        if (o == 0)
            Yk[k] = ys + (uint32_t)Y;
        B += take;
        cnt -= take;
        if (cnt >= 64) {  // whole words; B is at a word start here
            Yk[B >> 6] = ys + (uint32_t)Y;  // bytes may have been emitted inside the previous word
            B += cnt & ~(uint64_t)63;
            cnt &= 63;
        }
        if (cnt) {
            k = B >> 6;
            enter(k);
            Yk[k] = ys + (uint32_t)Y;
            B += cnt;
        }
    }
    __device__ __forceinline__ void byte(uint8_t c)
    {
        out[4 + 8 * ((B + 63) >> 6) + Y] = c;
        Y++;
    }
};

// Per block: first global bit / byte index, word base in W, stream length.
struct BlockOut {
    uint64_t bs, ys, wbase, len;
};

// Records are read in batches of kBatch, all lanes at once (clamped slots, a wave-uniform trip
// count), and the whole batch has arrived before any is used, so the stores of one batch (under
// the branches' masks) are never separated by a partial vmcnt wait from the next batch's loads
// ("Concurrent encodes and the unaligned text load"; tests/test_codegen.py).
constexpr uint32_t kBatch = 16;

__global__ void k_emit_write(const uint8_t *__restrict__ T, const uint64_t *__restrict__ tok,
                             const uint32_t *__restrict__ ntok, Blocks bl, uint32_t N_last, uint32_t chunk,
                             uint32_t nch, const uint64_t *__restrict__ bst, const uint64_t *__restrict__ yst,
                             uint64_t btotal, uint64_t *W, uint32_t *Yk, uint8_t *out, size_t stride,
                             const BlockOut *__restrict__ binfo, uint32_t klog)
{
    const uint32_t g = blockIdx.x * kT + threadIdx.x;
    // the wave's largest token count (every lane still active here)
    const uint32_t nt = g < nch ? ntok[g] : 0u;
    uint32_t ntmax = nt;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t o = shfl_xor_u32(ntmax, m);
        ntmax = o > ntmax ? o : ntmax;
    }
    if (g > nch)
        return;
    const uint32_t blk = g == nch ? bl.nb - 1u : bl.blk(g * chunk);
    const BlockOut bo = binfo[blk];
    Sink s;
    s.W = W + bo.wbase;
    s.Yk = Yk + bo.wbase;
    s.out = out + (size_t)blk * stride;
    s.ys = (uint32_t)bo.ys;
    s.B = s.B0 = bst[g] - bo.bs;
    s.B1 = (g == nch ? btotal : bst[g + 1]) - bo.bs;
    s.Y = yst[g] - bo.ys;
    s.cur = 0;
    s.kc = 0;
    s.have = false;
    if (g == nch) {
        if (s.B1 == s.B0)
            return;
        for (uint32_t i = bl.npos; i < bl.npos + (N_last - bl.n_last()); i++) {
            s.put(0, 1);
            s.byte(T[i]);
        }
        s.flush();
        return;
    }
    for (uint32_t k0 = 0; k0 < ntmax; k0 += kBatch) {
        uint64_t r[kBatch];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; q++) {
            const uint32_t k = k0 + q;
            r[q] = tok[tok_slot(g, k < nt ? k : 0u, klog)];
        }
        // every record of the batch is an operand: one full wait after the batch's loads
        static_assert(kBatch == 16, "operand list");
        asm volatile("" ::"v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]),
                     "v"(r[8]), "v"(r[9]), "v"(r[10]), "v"(r[11]), "v"(r[12]), "v"(r[13]), "v"(r[14]), "v"(r[15]));
        // (consumed in a loop: the unroller declines 16 bodies; the records stay in registers)
        for (uint32_t q = 0; q < kBatch; q++) {
            if (k0 + q >= nt)
                break;
            const uint32_t len = (uint32_t)(r[q] >> 32);
            if (len == 1) {
                s.put(0, 1);
                s.byte((uint8_t)r[q]);
            } else {
                uint32_t v = (uint32_t)r[q] - 1u;
                uint32_t kv = vn_size(v >> 8);
                s.put(1, 1);
                s.put(vn_bits(v >> 8, kv), 4 * kv);
                s.byte((uint8_t)(v & 0xffu));
                uint32_t gl = len - 3u;
                s.zeros(gl >> 3);
                s.put(8u | (gl & 7u), 4);  // unary terminator + 3 low bits
            }
        }
    }
    s.flush();
}

__global__ void k_place_words(const uint64_t *__restrict__ W, const uint32_t *__restrict__ Yk,
                              uint64_t nwords, uint8_t *__restrict__ out, size_t stride,
                              const BlockOut *__restrict__ binfo, uint32_t nb)
{
    size_t k = (size_t)blockIdx.x * kT + threadIdx.x;
    if (k >= nwords)
        return;
    uint32_t lo = 0, hi = nb;  // the block owning word k: last with wbase <= k
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (binfo[mid].wbase <= k)
            lo = mid;
        else
            hi = mid;
    }
    const BlockOut bo = binfo[lo];
    uint64_t w = W[k];
    uint8_t *d = out + (size_t)lo * stride + 4 + 8 * (k - bo.wbase) + (Yk[k] - (uint32_t)bo.ys);
#pragma unroll
    for (int i = 0; i < 8; i++)
        d[i] = (uint8_t)(w >> (8 * i));
}

// Per block: its bit / byte range from the chunk scans, words and stream length
// 4 + 8 ceil(B / 64) + Y. wcnt gets the word counts for the scan.
__global__ void k_block_info(Blocks bl, uint32_t chunk, uint32_t nch, const uint64_t *__restrict__ bst,
                             const uint64_t *__restrict__ yst, const uint64_t *__restrict__ tot,
                             BlockOut *__restrict__ binfo, uint64_t *__restrict__ wcnt)
{
    const uint32_t b = blockIdx.x * kT + threadIdx.x;
    if (b >= bl.nb)
        return;
    const uint32_t c0 = bl.nb == 1 ? 0u : b * (bl.bs / chunk);
    const bool last = b + 1u == bl.nb;
    const uint32_t c1 = last ? nch + 1u : (b + 1u) * (bl.bs / chunk);
    const uint64_t B0 = bst[c0], B1 = last ? tot[0] : bst[c1];
    const uint64_t Y0 = yst[c0], Y1 = last ? tot[1] : yst[c1];
    const uint64_t nw = (B1 - B0 + 63) / 64;
    binfo[b] = BlockOut{B0, Y0, 0, 4 + 8 * nw + (Y1 - Y0)};
    wcnt[b] = nw;
}

__global__ void k_block_wbase(BlockOut *__restrict__ binfo, const uint64_t *__restrict__ wpre, uint32_t nb)
{
    const uint32_t b = blockIdx.x * kT + threadIdx.x;
    if (b < nb)
        binfo[b].wbase = wpre[b];
}

// Headers (type << 24 | length & 0xffffff, lib/salz.c:760-772), one thread per block.
__global__ void k_finalize(Blocks bl, uint32_t N_last, const BlockOut *__restrict__ binfo,
                           uint8_t *__restrict__ out, size_t stride)
{
    const uint32_t b = blockIdx.x * kT + threadIdx.x;
    if (b >= bl.nb)
        return;
    const uint32_t N = b + 1u == bl.nb ? N_last : bl.bs;
    const uint64_t L = binfo[b].len;
    uint8_t *o = out + (size_t)b * stride;
    const bool plain = L > (uint64_t)N + 4;
    const uint32_t h = plain ? (N & 0xffffffu) : (1u << 24) | ((uint32_t)(L - 4) & 0xffffffu);
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
    o[3] = (uint8_t)(h >> 24);
}

// The PLAIN fallback (lib/salz.c:755-767): the raw block after the header, for blocks whose
// SALZ stream is longer than N + 4. grid (pieces of 4 KiB, blocks); 16 bytes per thread (an
// aligned 16-byte load of the text, byte stores after the 4-byte header).
__global__ __launch_bounds__(256) void k_plain_copy(const uint8_t *__restrict__ T, Blocks bl, uint32_t N_last,
                                                    const BlockOut *__restrict__ binfo,
                                                    uint8_t *__restrict__ out, size_t stride)
{
    const uint32_t b = blockIdx.y;
    const uint32_t N = b + 1u == bl.nb ? N_last : bl.bs;
    if (binfo[b].len <= (uint64_t)N + 4)
        return;
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i >= N)
        return;
    const uint8_t *src = T + (size_t)b * (bl.nb == 1 ? 0u : bl.bs);
    const uint4 v = *reinterpret_cast<const uint4 *>(src + i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t cnt = N - i < 16 ? (uint32_t)(N - i) : 16u;
    uint8_t *o = out + (size_t)b * stride + 4 + i;
    for (uint32_t k = 0; k < cnt; k++)
        o[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

}  // namespace

int stage_emit(Workspace &ws, const Blocks &bl, uint32_t N_last, uint8_t *dst, size_t stride,
               size_t cap, size_t *lens)
{
    hipStream_t st = ws.stream;
    ParseState &ps = ws.parse;
    const uint32_t n = bl.npos, nb = bl.nb;
    const uint32_t nch = ps.nchunks, ne = ps.n_exit;
    if (nb > 1 && bl.bs % ps.chunk != 0) {
        set_error("emit: batch block size %u is not a multiple of the parse chunk %u", bl.bs, ps.chunk);
        return -1;
    }
    if (nb > kMaxBatchBlocks) {
        set_error("emit: %u blocks exceed the batch limit %u", nb, kMaxBatchBlocks);
        return -1;
    }
    uint32_t *emark = ws.offA, *entry = ws.sa;
    uint64_t *cbits = ws.g64, *cbytes = ws.g64 + (nch + 2);
    uint64_t *W = ws.keyA;
    uint32_t *Yk = ws.u2;
    uint64_t *tot = ws.dscal + 64;  // [0] bits, [1] bytes, [2] words
    // per-block records after the chunk counts in g64 (free: n + 2 entries, counts use 2 nch + 4)
    BlockOut *binfo = reinterpret_cast<BlockOut *>(ws.g64 + 2 * ((size_t)nch + 2) + 2);
    uint64_t *wcnt = reinterpret_cast<uint64_t *>(binfo + nb);

    SALZ_HIP(fill_async(entry, 0xff, sizeof(uint32_t) * ((size_t)nch + 1), st));
    if (ne) {
        SALZ_HIP(fill_async(emark, 0, sizeof(uint32_t) * ne, st));
        // one block with its levels stored: the path in one launch (round 5: C2 emission 1.07 ->
        // 1.01 ms); batches, and a parse that kept level 0 only, a launch per level
        const bool one = nb == 1 && ps.snaps && ps.levels > 0;
        if (one) {
            // (a path takes at most one exit per chunk: nch + 1 nodes with the root)
            constexpr uint32_t kPathThreads = 32768;
            const uint64_t reach = (uint64_t)nch + 2;
            const uint32_t L = (uint32_t)((reach + kPathThreads - 1) / kPathThreads);
            hipLaunchKernelGGL(k_mark_path, dim3(grid_for(kPathThreads, kT)), dim3(kT), 0, st, ps.ebits, ps.pst,
                               ws.klog, ps.jt0, ne, ps.levels, L, kPathThreads, emark);
            SALZ_LAUNCH_CHECK();
        } else {
            hipLaunchKernelGGL(k_mark_start, dim3(grid_for(nb, kT)), dim3(kT), 0, st, ps.ebits, ps.pst, ws.klog,
                               emark, bl);
            SALZ_LAUNCH_CHECK();
            const uint32_t *lev = ps.jt0;  // parents 2^k steps up (level k)
            uint32_t *pp[2] = {ws.u2, ws.u3};  // recomputed levels when the parse kept only level 0
            for (uint32_t k = 0; k < ps.levels; k++) {
                if (k > 0) {
                    if (ps.snaps) {
                        lev = ps.jt0 + (size_t)k * ne;
                    } else {
                        hipLaunchKernelGGL(k_jt_double, dim3(grid_for(ne, kT)), dim3(kT), 0, st, lev,
                                           pp[k & 1], ne);
                        SALZ_LAUNCH_CHECK();
                        lev = pp[k & 1];
                    }
                }
                hipLaunchKernelGGL(k_mark_step, dim3(grid_for(ne, kT)), dim3(kT), 0, st, lev, emark, ne);
                SALZ_LAUNCH_CHECK();
            }
        }
        hipLaunchKernelGGL(k_entries, dim3(grid_for(ne, kT)), dim3(kT), 0, st, emark, ps.elist, ne,
                           n, ps.chunk, entry);
        SALZ_LAUNCH_CHECK();
    }
    // token records (keyB: the parse's jump snapshots, read only by the marking above) and their
    // counts per chunk (u3)
    uint64_t *tok = ws.keyB;
    uint32_t *ntok = ws.u3;
    hipLaunchKernelGGL(k_emit_count, dim3(grid_for((size_t)nch + 1, kT)), dim3(kT), 0, st,
                       ws.cand, ps.choice, ws.text, entry, bl, N_last, ps.chunk, nch, cbits, cbytes, ws.klog, tok,
                       ntok);
    SALZ_LAUNCH_CHECK();
    if (scan_sum_u64(cbits, cbits, (size_t)nch + 1, false, tot + 0, ws, st) != 0)
        return -1;
    if (scan_sum_u64(cbytes, cbytes, (size_t)nch + 1, false, tot + 1, ws, st) != 0)
        return -1;
    hipLaunchKernelGGL(k_block_info, dim3(grid_for(nb, kT)), dim3(kT), 0, st, bl, ps.chunk, nch,
                       cbits, cbytes, tot, binfo, wcnt);
    SALZ_LAUNCH_CHECK();
    if (scan_sum_u64(wcnt, wcnt, nb, false, tot + 2, ws, st) != 0)
        return -1;
    hipLaunchKernelGGL(k_block_wbase, dim3(grid_for(nb, kT)), dim3(kT), 0, st, binfo, wcnt, nb);
    SALZ_LAUNCH_CHECK();
    // one host round trip: the totals and every block's stream length
    std::vector<BlockOut> hb(nb);
    if (read_scalars(ws, 512, 24, "emit.tot") != 0 ||
        read_device(ws, binfo, sizeof(BlockOut) * nb, hb.data()) != 0)
        return -1;
    const uint64_t btotal = ws.hscal[64], ytotal = ws.hscal[65], nwords = ws.hscal[66];
    ws.stats.emit_bits = btotal;
    ws.stats.emit_bytes = ytotal;
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t N = b + 1 == nb ? N_last : bl.bs;
        const uint64_t L = hb[b].len, out = L > (uint64_t)N + 4 ? (uint64_t)N + 4 : L;
        if (L > cap || out > cap) {  // the reference's writer fails the same way (lib/salz.c:260, :274)
            set_error("encoded stream (%llu bytes) exceeds destination capacity (%zu)",
                      (unsigned long long)L, cap);
            return -1;
        }
        lens[b] = (size_t)out;
    }
    SALZ_HIP(fill_async(W, 0, sizeof(uint64_t) * (nwords + 1), st));
    SALZ_HIP(fill_async(Yk, 0, sizeof(uint32_t) * (nwords + 1), st));
    hipLaunchKernelGGL(k_emit_write, dim3(grid_for((size_t)nch + 1, kT)), dim3(kT), 0, st,
                       ws.text, tok, ntok, bl, N_last, ps.chunk, nch, cbits, cbytes, btotal, W, Yk, dst, stride,
                       binfo, ws.klog);
    SALZ_LAUNCH_CHECK();
    // Yk of the words inside zero runs (Sink::zeros): Yk is non-decreasing in k
    if (nwords && scan_max_u32(Yk, Yk, nwords, true, nullptr, ws, st) != 0)
        return -1;
    if (nwords) {
        hipLaunchKernelGGL(k_place_words, dim3(grid_for(nwords, kT)), dim3(kT), 0, st, W, Yk,
                           nwords, dst, stride, binfo, nb);
        SALZ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(nb, kT)), dim3(kT), 0, st, bl, N_last, binfo, dst, stride);
    SALZ_LAUNCH_CHECK();
    bool any_plain = false;
    for (uint32_t b = 0; b < nb; b++)
        any_plain |= lens[b] != hb[b].len;
    if (any_plain) {
        const uint32_t maxN = nb > 1 ? bl.bs : N_last;
        hipLaunchKernelGGL(k_plain_copy, dim3(grid_for(maxN, 4096), nb), dim3(256), 0, st, ws.text, bl,
                           N_last, binfo, dst, stride);
        SALZ_LAUNCH_CHECK();
    }
    return 0;
}

}  // namespace salz
