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
//   4. place every word at 4 + 8k + Y_k; the host writes the 4-byte header. A stream longer
//      than N + 4 is replaced by the PLAIN form (header + raw copy), as in :755-767.
#include "internal.hpp"

namespace salz {
namespace {

constexpr int kT = 256;
constexpr uint32_t kNone = 0xffffffffu;

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

__global__ void k_mark_start(const uint32_t *__restrict__ eidx, const uint64_t *__restrict__ pst,
                             uint32_t klog, uint32_t *__restrict__ emark)
{
    emark[eidx[sidx((uint32_t)pst[0], klog)]] = 1u;  // exit of position 0 (slot sidx(0) == 0)
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
    if (q < n)
        entry[q / chunk] = q;
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

__global__ void k_emit_count(const uint4 *__restrict__ cand, const uint8_t *__restrict__ choice,
                             const uint32_t *__restrict__ entry, uint32_t n, uint32_t N,
                             uint32_t chunk, uint32_t nch, uint64_t *__restrict__ cbits,
                             uint64_t *__restrict__ cbytes, uint32_t klog)
{
    uint32_t g = blockIdx.x * kT + threadIdx.x;
    if (g > nch)
        return;
    uint64_t bits = 0, bytes = 0;
    if (g == nch) {
        bits = N - n;
        bytes = N - n;
    } else {
        uint32_t p = g == 0 ? 0u : entry[g];
        if (p != kNone) {
            uint32_t b = (n - g * chunk) < chunk ? n : g * chunk + chunk;
            while (p < b) {
                Token t = token_at(cand, choice, p, klog);
                if (t.len == 1) {
                    bits += 1;
                    bytes += 1;
                } else {
                    uint32_t gl = t.len - 3u;
                    bits += 1u + 4u * vn_size((t.off - 1u) >> 8) + (gl >> 3) + 4u;
                    bytes += 1;
                }
                p += t.len;
            }
        }
    }
    cbits[g] = bits;
    cbytes[g] = bytes;
}

struct Sink {
    uint64_t *W;
    uint32_t *Yk;
    uint8_t *out;
    uint64_t B, B0, B1, Y;
    uint64_t cur, kc;
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
                Yk[k] = (uint32_t)Y;
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
            Yk[k] = (uint32_t)Y;
        B += take;
        cnt -= take;
        if (cnt >= 64) {  // whole words; B is at a word start here
            Yk[B >> 6] = (uint32_t)Y;  // bytes may have been emitted inside the previous word
            B += cnt & ~(uint64_t)63;
            cnt &= 63;
        }
        if (cnt) {
            k = B >> 6;
            enter(k);
            Yk[k] = (uint32_t)Y;
            B += cnt;
        }
    }
    __device__ __forceinline__ void byte(uint8_t c)
    {
        out[4 + 8 * ((B + 63) >> 6) + Y] = c;
        Y++;
    }
};

__global__ void k_emit_write(const uint8_t *__restrict__ T, const uint4 *__restrict__ cand,
                             const uint8_t *__restrict__ choice, const uint32_t *__restrict__ entry,
                             uint32_t n, uint32_t N, uint32_t chunk, uint32_t nch,
                             const uint64_t *__restrict__ bst, const uint64_t *__restrict__ yst,
                             uint64_t btotal, uint64_t *W, uint32_t *Yk, uint8_t *out,
                             uint32_t klog)
{
    uint32_t g = blockIdx.x * kT + threadIdx.x;
    if (g > nch)
        return;
    Sink s;
    s.W = W;
    s.Yk = Yk;
    s.out = out;
    s.B = s.B0 = bst[g];
    s.B1 = g == nch ? btotal : bst[g + 1];
    s.Y = yst[g];
    s.cur = 0;
    s.kc = 0;
    s.have = false;
    if (s.B1 == s.B0)
        return;
    if (g == nch) {
        for (uint32_t i = n; i < N; i++) {
            s.put(0, 1);
            s.byte(T[i]);
        }
    } else {
        uint32_t p = g == 0 ? 0u : entry[g];
        uint32_t b = (n - g * chunk) < chunk ? n : g * chunk + chunk;
        while (p < b) {
            Token t = token_at(cand, choice, p, klog);
            if (t.len == 1) {
                s.put(0, 1);
                s.byte(T[p]);
            } else {
                uint32_t v = t.off - 1u;
                uint32_t k = vn_size(v >> 8);
                s.put(1, 1);
                s.put(vn_bits(v >> 8, k), 4 * k);
                s.byte((uint8_t)(v & 0xffu));
                uint32_t gl = t.len - 3u;
                s.zeros(gl >> 3);
                s.put(8u | (gl & 7u), 4);  // unary terminator + 3 low bits
            }
            p += t.len;
        }
    }
    s.flush();
}

__global__ void k_place_words(const uint64_t *__restrict__ W, const uint32_t *__restrict__ Yk,
                              uint64_t nwords, uint8_t *__restrict__ out)
{
    size_t k = (size_t)blockIdx.x * kT + threadIdx.x;
    if (k >= nwords)
        return;
    uint64_t w = W[k];
    uint8_t *d = out + 4 + 8 * k + Yk[k];
#pragma unroll
    for (int i = 0; i < 8; i++)
        d[i] = (uint8_t)(w >> (8 * i));
}

}  // namespace

int stage_emit(Workspace &ws, uint32_t n, uint32_t N, uint8_t *dst, size_t cap, size_t *out_len)
{
    hipStream_t st = ws.stream;
    ParseState &ps = ws.parse;
    const uint32_t nch = ps.nchunks, ne = ps.n_exit;
    uint32_t *emark = ws.offA, *eidx = ws.offB, *entry = ws.sa;
    uint64_t *cbits = ws.g64, *cbytes = ws.g64 + (nch + 2);
    uint64_t *W = ws.keyA;
    uint32_t *Yk = ws.u2;
    uint64_t *tot = ws.dscal + 64;  // [0] bits, [1] bytes

    SALZ_HIP(hipMemsetAsync(entry, 0xff, sizeof(uint32_t) * ((size_t)nch + 1), st));
    if (ne) {
        SALZ_HIP(hipMemsetAsync(emark, 0, sizeof(uint32_t) * ne, st));
        hipLaunchKernelGGL(k_mark_start, dim3(1), dim3(1), 0, st, eidx, ps.pst, ws.klog, emark);
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
        hipLaunchKernelGGL(k_entries, dim3(grid_for(ne, kT)), dim3(kT), 0, st, emark, ps.elist, ne,
                           n, ps.chunk, entry);
        SALZ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_emit_count, dim3(grid_for((size_t)nch + 1, kT)), dim3(kT), 0, st,
                       ws.cand, ps.choice, entry, n, N, ps.chunk, nch, cbits, cbytes, ws.klog);
    SALZ_LAUNCH_CHECK();
    if (scan_sum_u64(cbits, cbits, (size_t)nch + 1, false, tot + 0, ws, st) != 0)
        return -1;
    if (scan_sum_u64(cbytes, cbytes, (size_t)nch + 1, false, tot + 1, ws, st) != 0)
        return -1;
    if (read_scalars(ws, 512, 16, "emit.tot") != 0)
        return -1;
    const uint64_t btotal = ws.hscal[64], ytotal = ws.hscal[65];
    const uint64_t nwords = (btotal + 63) / 64;
    const uint64_t L = 4 + 8 * nwords + ytotal;
    ws.stats.emit_bits = btotal;
    ws.stats.emit_bytes = ytotal;

    uint32_t *hdr = reinterpret_cast<uint32_t *>(ws.hscal + 100);
    if (L > cap) {
        set_error("encoded stream (%llu bytes) exceeds destination capacity (%zu)",
                  (unsigned long long)L, cap);
        return -1;  // the reference's writer fails the same way (lib/salz.c:260, :274)
    }
    if (L > (uint64_t)N + 4) {  // PLAIN fallback (lib/salz.c:755-767)
        if ((size_t)N + 4 > cap) {
            set_error("PLAIN stream exceeds destination capacity");
            return -1;
        }
        *hdr = (0u << 24) | (N & 0xffffffu);
        SALZ_HIP(hipMemcpyAsync(dst + 4, ws.text, N, hipMemcpyDeviceToDevice, st));
        *out_len = (size_t)N + 4;
    } else {
        *hdr = (1u << 24) | ((uint32_t)(L - 4) & 0xffffffu);
        SALZ_HIP(hipMemsetAsync(W, 0, sizeof(uint64_t) * (nwords + 1), st));
        SALZ_HIP(hipMemsetAsync(Yk, 0, sizeof(uint32_t) * (nwords + 1), st));
        hipLaunchKernelGGL(k_emit_write, dim3(grid_for((size_t)nch + 1, kT)), dim3(kT), 0, st,
                           ws.text, ws.cand, ps.choice, entry, n, N, ps.chunk, nch, cbits, cbytes,
                           btotal, W, Yk, dst, ws.klog);
        SALZ_LAUNCH_CHECK();
        // Yk of the words inside zero runs (Sink::zeros): Yk is non-decreasing in k
        if (scan_max_u32(Yk, Yk, nwords, true, nullptr, ws, st) != 0)
            return -1;
        hipLaunchKernelGGL(k_place_words, dim3(grid_for(nwords, kT)), dim3(kT), 0, st, W, Yk,
                           nwords, dst);
        SALZ_LAUNCH_CHECK();
        *out_len = L;
    }
    SALZ_HIP(hipMemcpyAsync(dst, hdr, 4, hipMemcpyHostToDevice, st));
    return 0;
}

}  // namespace salz
