/*
 * salz_oracle.c - CPU restatement of the reference SA-LZ codec.
 *
 * TEST INFRASTRUCTURE ONLY (see salz_oracle.h): the parity checker and the CPU
 * baseline ("kind": "port") for bench.py. The shipped product never links this file.
 *
 * Every stage cites the reference lines it restates (/root/reference/lib/salz.c).
 * The suffix array is built by our own SA-IS (Nong, Zhang & Chan 2009) in place of the
 * absent libsais submodule (.gitmodules:1-3, called at lib/salz.c:465).
 */
#include "salz_oracle.h"

#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------
 * SA-IS. Text symbols are u8 (top level) or int32 (recursion); an implicit sentinel
 * smaller than every symbol terminates the text, which gives exactly the ordering
 * libsais produces: a suffix sorts before every longer suffix it is a prefix of.
 * ---------------------------------------------------------------------------------- */

typedef struct {
    const uint8_t *t8;
    const int32_t *t32;
} sym_t;

static inline int32_t sym_at(sym_t s, int32_t i)
{
    return s.t8 ? (int32_t)s.t8[i] : s.t32[i];
}

static void bucket_bounds(sym_t s, int32_t n, int32_t k, int32_t *bkt, bool ends)
{
    memset(bkt, 0, sizeof(*bkt) * (size_t)k);
    for (int32_t i = 0; i < n; i++)
        bkt[sym_at(s, i)]++;
    int32_t run = 0;
    for (int32_t c = 0; c < k; c++) {
        run += bkt[c];
        bkt[c] = ends ? run : run - bkt[c];
    }
}

/* stype[i] != 0 iff suffix i is S-type; an LMS position is S-type with L-type left. */
static inline bool is_lms(const uint8_t *stype, int32_t i)
{
    return i > 0 && stype[i] && !stype[i - 1];
}

static void induce(sym_t s, const uint8_t *stype, int32_t *SA, int32_t n, int32_t k,
                   int32_t *bkt)
{
    /* L-type pass, left to right. The virtual sentinel induces suffix n-1 first. */
    bucket_bounds(s, n, k, bkt, false);
    SA[bkt[sym_at(s, n - 1)]++] = n - 1;
    for (int32_t r = 0; r < n; r++) {
        int32_t j = SA[r] - 1;
        if (SA[r] > 0 && !stype[j])
            SA[bkt[sym_at(s, j)]++] = j;
    }
    /* S-type pass, right to left. */
    bucket_bounds(s, n, k, bkt, true);
    for (int32_t r = n - 1; r >= 0; r--) {
        int32_t j = SA[r] - 1;
        if (SA[r] > 0 && stype[j])
            SA[--bkt[sym_at(s, j)]] = j;
    }
}

static int sais_rec(sym_t s, int32_t *SA, int32_t n, int32_t k)
{
    if (n == 1) {
        SA[0] = 0;
        return 0;
    }

    uint8_t *stype = malloc((size_t)n);
    int32_t *bkt = malloc(sizeof(int32_t) * (size_t)k);
    if (!stype || !bkt) {
        free(stype);
        free(bkt);
        return -1;
    }

    stype[n - 1] = 0; /* last suffix is larger than the sentinel: L-type */
    for (int32_t i = n - 2; i >= 0; i--) {
        int32_t a = sym_at(s, i), b = sym_at(s, i + 1);
        stype[i] = (a < b || (a == b && stype[i + 1])) ? 1 : 0;
    }

    /* Stage 1: bucket LMS positions at bucket ends, induce, sorting LMS substrings. */
    for (int32_t r = 0; r < n; r++)
        SA[r] = -1;
    bucket_bounds(s, n, k, bkt, true);
    for (int32_t i = 1; i < n; i++)
        if (is_lms(stype, i))
            SA[--bkt[sym_at(s, i)]] = i;
    induce(s, stype, SA, n, k, bkt);

    /* Compact the sorted LMS positions to SA[0, m). */
    int32_t m = 0;
    for (int32_t r = 0; r < n; r++)
        if (is_lms(stype, SA[r]))
            SA[m++] = SA[r];

    /* Name LMS substrings; names stored at SA[m + pos/2] (LMS positions are >= 2 apart). */
    for (int32_t r = m; r < n; r++)
        SA[r] = -1;
    int32_t names = 0, prev = -1;
    for (int32_t r = 0; r < m; r++) {
        int32_t pos = SA[r];
        bool differ = prev < 0;
        for (int32_t d = 0; !differ; d++) {
            if (pos + d == n || prev + d == n ||
                sym_at(s, pos + d) != sym_at(s, prev + d) ||
                stype[pos + d] != stype[prev + d]) {
                differ = true;
                break;
            }
            if (d > 0 && (is_lms(stype, pos + d) || is_lms(stype, prev + d)))
                break; /* both substrings end here and are equal */
        }
        if (differ) {
            names++;
            prev = pos;
        }
        SA[m + (pos >> 1)] = names - 1;
    }

    /* Reduced string in text order at SA[n - m, n). */
    for (int32_t r = n - 1, w = n - 1; r >= m; r--)
        if (SA[r] >= 0)
            SA[w--] = SA[r];
    int32_t *s1 = SA + n - m;

    if (names < m) {
        sym_t rs = { NULL, s1 };
        if (sais_rec(rs, SA, m, names) != 0) {
            free(stype);
            free(bkt);
            return -1;
        }
    } else {
        for (int32_t i = 0; i < m; i++)
            SA[s1[i]] = i;
    }

    /* Stage 3: map reduced ranks back to LMS positions, seed bucket ends, induce. */
    for (int32_t i = 1, w = 0; i < n; i++)
        if (is_lms(stype, i))
            s1[w++] = i;
    for (int32_t r = 0; r < m; r++)
        SA[r] = s1[SA[r]];
    for (int32_t r = m; r < n; r++)
        SA[r] = -1;
    bucket_bounds(s, n, k, bkt, true);
    for (int32_t r = m - 1; r >= 0; r--) {
        int32_t pos = SA[r];
        SA[r] = -1;
        SA[--bkt[sym_at(s, pos)]] = pos;
    }
    induce(s, stype, SA, n, k, bkt);

    free(stype);
    free(bkt);
    return 0;
}

int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n)
{
    if (n < 0 || (n > 0 && (!T || !SA)))
        return -1;
    if (n == 0)
        return 0;
    sym_t s = { T, NULL };
    return sais_rec(s, SA, n, 256);
}

/* ------------------------------------------------------------------------------------
 * Variable-nibble code (lib/salz.c:352-445, :565-588).
 * ---------------------------------------------------------------------------------- */

/* Thresholds at which one more nibble is needed (lib/salz.c:567-587). */
static const uint32_t vn_limit[10] = {
    8u, 72u, 584u, 4680u, 37448u, 299592u, 2396744u, 19173960u, 153391688u, 1227133512u,
};

size_t oracle_vnibble_size(uint32_t val)
{
    size_t k = 1;
    while (k <= 10 && val >= vn_limit[k - 1])
        k++;
    return k;
}

/*
 * Byte-packing restatement of encode_vnibble_le (lib/salz.c:352-445): byte j carries a
 * low nibble taken from (val - base_j) >> 6j and a high nibble ((val - base_j) >> (6j+3)) - 1,
 * where base_j = 0, 72, 4680, 299592, 19173960, 1227133512; byte 0's low nibble carries the
 * terminator bit 0x8. Only the low 4k bits are meaningful (callers mask them).
 */
size_t oracle_encode_vnibble_le(uint32_t val, uint64_t *res)
{
    static const uint32_t base[6] = { 0u, 72u, 4680u, 299592u, 19173960u, 1227133512u };
    size_t k = oracle_vnibble_size(val);
    uint8_t p[8] = { 0 };

    for (size_t j = 0; 2 * j < k; j++) {
        uint32_t v = val - base[j];
        uint32_t lo = j == 0 ? ((v & 7u) | 8u) : ((v >> (6 * j)) & 7u);
        uint32_t hi = 0;
        if (2 * j + 1 < k)
            hi = ((v >> (6 * j + 3)) - 1u) & 7u;
        p[j] = (uint8_t)((hi << 4) | lo);
    }
    memcpy(res, p, sizeof(*res));
    return k;
}

/* ------------------------------------------------------------------------------------
 * Encoder (lib/salz.c:175-823).
 * ---------------------------------------------------------------------------------- */

/* Sequential bit writer with lazily reserved 8-byte control words (lib/salz.c:258-330).
 * A word slot is reserved at the current byte cursor when its first bit is written. */
typedef struct {
    uint8_t *dst;
    size_t cap;
    size_t pos;      /* byte cursor; starts after the 4-byte header */
    uint64_t word;   /* bits of the current control word, LSB-aligned */
    unsigned room;   /* free bits left in the current word */
    size_t word_pos; /* reserved slot of the current word */
    bool fail;
} bitw_t;

static void bw_store_word(bitw_t *w)
{
    memcpy(w->dst + w->word_pos, &w->word, 8);
}

/* flush_bits (lib/salz.c:268-283): store the current word, reserve the next one. */
static void bw_next_word(bitw_t *w)
{
    bw_store_word(w);
    if (w->pos + 8 > w->cap) {
        w->fail = true;
        return;
    }
    w->word = 0;
    w->room = 64;
    w->word_pos = w->pos;
    w->pos += 8;
}

/* Append `count` (<= 64) bits, MSB first (write_bit/bits/zeros, lib/salz.c:285-330). */
static void bw_put(bitw_t *w, uint64_t bits, unsigned count)
{
    while (count && !w->fail) {
        if (w->room == 0) {
            bw_next_word(w);
            if (w->fail)
                return;
        }
        unsigned take = count < w->room ? count : w->room;
        uint64_t chunk = (bits >> (count - take)) & ((take == 64) ? ~0ull : ((1ull << take) - 1));
        w->word = (take == 64) ? chunk : ((w->word << take) | chunk);
        w->room -= take;
        count -= take;
    }
}

static void bw_zeros(bitw_t *w, uint32_t count)
{
    while (count) {
        unsigned c = count > 32 ? 32 : count;
        bw_put(w, 0, c);
        count -= c;
    }
}

static void bw_byte(bitw_t *w, uint8_t b)
{
    if (w->pos >= w->cap) {
        w->fail = true;
        return;
    }
    w->dst[w->pos++] = b;
}

/* build_psvnsv_array (lib/salz.c:471-490): a single left-to-right stack pass over the SA
 * with -1 sentinels on both ends; each popped suffix gets the element beneath it as PSV
 * and the element that popped it as NSV. */
static void psv_nsv_pass(const int32_t *sa, int32_t n, int32_t *psv, int32_t *nsv)
{
    int32_t *stack = malloc(sizeof(int32_t) * ((size_t)n + 2));
    int32_t top = 0;
    stack[0] = -1;
    for (int32_t r = 0; r <= n; r++) {
        int32_t cur = r < n ? sa[r] : -1;
        while (stack[top] > cur) {
            int32_t p = stack[top];
            psv[p] = stack[top - 1];
            nsv[p] = cur;
            top--;
        }
        stack[++top] = cur;
    }
    free(stack);
}

/* lcp_cmp (lib/salz.c:492-514): extend a known common prefix of suffixes a < b of T[0,n). */
static int32_t lcp_extend(const uint8_t *T, int32_t n, int32_t a, int32_t b, int32_t len)
{
    while (b + len + 8 <= n) {
        uint64_t x, y;
        memcpy(&x, T + a + len, 8);
        memcpy(&y, T + b + len, 8);
        if (x != y)
            return len + (__builtin_ctzll(x ^ y) >> 3);
        len += 8;
    }
    while (b + len < n && T[a + len] == T[b + len])
        len++;
    return len;
}

/* factorize / factorize_pos (lib/salz.c:516-560): candidate lengths with the KKP lower
 * bound max(prev - 1, 0) carried from the previous position. */
static void candidate_lengths(const uint8_t *T, int32_t n, const int32_t *psv,
                              const int32_t *nsv, int32_t *lp, int32_t *ln)
{
    int32_t prev_p = 0, prev_n = 0;
    lp[0] = 1; /* position 0 is forced literal (lib/salz.c:547-548) */
    ln[0] = 1;
    for (int32_t pos = 1; pos < n; pos++) {
        int32_t a = 0, b = 0;
        if (psv[pos] != -1)
            a = lcp_extend(T, n, psv[pos], pos, prev_p > 0 ? prev_p - 1 : 0);
        if (nsv[pos] != -1)
            b = lcp_extend(T, n, nsv[pos], pos, prev_n > 0 ? prev_n - 1 : 0);
        lp[pos] = a;
        ln[pos] = b;
        prev_p = a;
        prev_n = b;
    }
}

/* Bit cost of a factor (lib/salz.c:595-608), plus the token bit. */
static uint32_t factor_bits(uint32_t off, uint32_t len)
{
    return 1u + 8u + 4u * (uint32_t)oracle_vnibble_size((off - 1u) >> 8) + ((len - 3u) >> 3) + 4u;
}

/* optimize_factorization (lib/salz.c:610-662): backward shortest path in 32-bit signed
 * arithmetic; ties keep the earlier candidate (literal, then PSV, then NSV). */
static void optimal_parse(int32_t n, const int32_t *psv, const int32_t *nsv,
                          const int32_t *lp, const int32_t *ln, int32_t *dlen, int32_t *doff,
                          int32_t *cost)
{
    cost[n] = 0;
    dlen[0] = 1;
    doff[0] = 0;
    for (int32_t p = n - 1; p >= 1; p--) {
        int32_t best_len = 1, best_off = 0;
        int32_t best = (int32_t)(9u + (uint32_t)cost[p + 1]);
        const int32_t lens[2] = { lp[p], ln[p] };
        const int32_t offs[2] = { p - psv[p], p - nsv[p] };
        for (int c = 0; c < 2; c++) {
            if (lens[c] < 3)
                continue;
            int32_t alt = (int32_t)(factor_bits((uint32_t)offs[c], (uint32_t)lens[c]) +
                                    (uint32_t)cost[p + lens[c]]);
            if (alt < best) {
                best = alt;
                best_len = lens[c];
                best_off = offs[c];
            }
        }
        dlen[p] = best_len;
        doff[p] = best_off;
        cost[p] = best;
    }
}

/* Token emission and stream finalisation (lib/salz.c:664-775). */
static int emit_stream(const uint8_t *src, size_t N, int32_t n, const int32_t *dlen,
                       const int32_t *doff, uint8_t *dst, size_t cap, size_t *out_len)
{
    if (cap < 4)
        return -1;
    bitw_t w = { dst, cap, 4, 0, 0, 0, false };

    size_t p = 0;
    while (p < (size_t)n && !w.fail) {
        uint32_t len = (uint32_t)dlen[p];
        if (len == 1) {
            bw_put(&w, 0, 1);
            if (!w.fail)
                bw_byte(&w, src[p]);
            p += 1;
        } else {
            uint32_t v = (uint32_t)doff[p] - 1u;
            uint64_t nib;
            size_t k = oracle_encode_vnibble_le(v >> 8, &nib);
            bw_put(&w, 1, 1);
            bw_put(&w, nib & ((1ull << (4 * k)) - 1), (unsigned)(4 * k));
            if (!w.fail)
                bw_byte(&w, (uint8_t)(v & 0xffu));
            uint32_t g = len - 3u;
            bw_zeros(&w, g >> 3);
            bw_put(&w, 1, 1);
            bw_put(&w, g & 7u, 3);
            p += len;
        }
    }
    /* The 8 reserved trailing bytes as literals (lib/salz.c:743-749). */
    for (size_t i = (size_t)n; i < N && !w.fail; i++) {
        bw_put(&w, 0, 1);
        if (!w.fail)
            bw_byte(&w, src[i]);
    }
    if (w.fail)
        return -1;

    /* Left-align and store the last word (lib/salz.c:752-753). */
    w.word = (w.room >= 64) ? 0 : (w.word << w.room);
    bw_store_word(&w);

    uint32_t hdr;
    if (w.pos > N + 4) { /* PLAIN fallback (lib/salz.c:755-767) */
        if (N + 4 > cap)
            return -1;
        hdr = (0u << 24) | ((uint32_t)N & 0xffffffu);
        memcpy(dst + 4, src, N);
        w.pos = N + 4;
    } else {
        hdr = (1u << 24) | ((uint32_t)(w.pos - 4) & 0xffffffu);
    }
    memcpy(dst, &hdr, 4);
    *out_len = w.pos;
    return 0;
}

/* Run stages a3..a7 (lib/salz.c:463-662). Output arrays the caller passes as NULL are
 * allocated here; *own records which ones, so the caller can free them. */
enum { S_SA, S_PSV, S_NSV, S_LP, S_LN, S_DLEN, S_DOFF, S_COST, S_COUNT };

static int run_stages(const uint8_t *src, size_t N, int32_t *arr[S_COUNT], bool own[S_COUNT])
{
    for (int i = 0; i < S_COUNT; i++)
        own[i] = false;
    if (N <= 8 || N - 8 > 0x7ffffff0u)
        return -1; /* reference: lib/salz.c:197 wraps for N < 8 and crashes for N == 8 */
    int32_t n = (int32_t)(N - 8);
    size_t sz = sizeof(int32_t) * ((size_t)n + 1);
    for (int i = 0; i < S_COUNT; i++) {
        if (!arr[i]) {
            arr[i] = malloc(sz);
            own[i] = true;
            if (!arr[i])
                return -1;
        }
    }
    if (oracle_suffix_array(src, arr[S_SA], n) != 0)
        return -1;
    psv_nsv_pass(arr[S_SA], n, arr[S_PSV], arr[S_NSV]);
    candidate_lengths(src, n, arr[S_PSV], arr[S_NSV], arr[S_LP], arr[S_LN]);
    optimal_parse(n, arr[S_PSV], arr[S_NSV], arr[S_LP], arr[S_LN], arr[S_DLEN], arr[S_DOFF],
                  arr[S_COST]);
    return 0;
}

static void free_owned(int32_t *arr[S_COUNT], const bool own[S_COUNT])
{
    for (int i = 0; i < S_COUNT; i++)
        if (own[i])
            free(arr[i]);
}

int oracle_stages(const uint8_t *src, size_t src_len, int32_t *sa, int32_t *psv,
                  int32_t *nsv, int32_t *lp, int32_t *ln, int32_t *dlen, int32_t *doff,
                  int32_t *cost)
{
    if (!src)
        return -1;
    int32_t *arr[S_COUNT] = { sa, psv, nsv, lp, ln, dlen, doff, cost };
    bool own[S_COUNT];
    int rc = run_stages(src, src_len, arr, own);
    free_owned(arr, own);
    return rc;
}

int oracle_encode(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len)
{
    if (!src || !dst || !dst_len)
        return -1;
    int32_t *arr[S_COUNT] = { NULL };
    bool own[S_COUNT];
    int rc = run_stages(src, src_len, arr, own);
    size_t out = 0;
    if (rc == 0)
        rc = emit_stream(src, src_len, (int32_t)(src_len - 8), arr[S_DLEN], arr[S_DOFF], dst,
                         *dst_len, &out);
    free_owned(arr, own);
    if (rc == 0)
        *dst_len = out; /* set only on success (lib/salz.c:818) */
    return rc;
}

/* ------------------------------------------------------------------------------------
 * Decoder (lib/salz.c:829-1228).
 * ---------------------------------------------------------------------------------- */

typedef struct {
    const uint8_t *s;
    size_t len, pos;
    uint64_t word;  /* unread bits, MSB-aligned */
    unsigned avail; /* unread bits in word */
} bitr_t;

static bool br_refill(bitr_t *r)
{
    if (r->pos + 8 > r->len)
        return false;
    memcpy(&r->word, r->s + r->pos, 8);
    r->pos += 8;
    r->avail = 64;
    return true;
}

static bool br_bits(bitr_t *r, unsigned count, uint32_t *out)
{
    uint32_t v = 0;
    while (count) {
        if (r->avail == 0 && !br_refill(r))
            return false;
        unsigned take = count < r->avail ? count : r->avail;
        v = (v << take) | (uint32_t)(r->word >> (64 - take));
        r->word = take == 64 ? 0 : r->word << take;
        r->avail -= take;
        count -= take;
    }
    *out = v;
    return true;
}

/* read_unary (lib/salz.c:958-979): count zeros up to and including a terminating 1. */
static bool br_unary(bitr_t *r, uint32_t *out)
{
    uint32_t z = 0;
    if (r->avail == 0 && !br_refill(r))
        return false;
    while (r->word == 0) {
        z += r->avail;
        if (!br_refill(r))
            return false;
    }
    unsigned lead = (unsigned)__builtin_clzll(r->word);
    r->word = (lead + 1 == 64) ? 0 : r->word << (lead + 1);
    r->avail -= lead + 1;
    *out = z + lead;
    return true;
}

int oracle_decode(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len)
{
    if (!src || !dst || !dst_len)
        return -1;
    if (src_len < 4)
        return -1;
    uint32_t hdr;
    memcpy(&hdr, src, 4);
    uint32_t type = hdr >> 24, len = hdr & 0xffffffu;
    if (type >= 2 || len > src_len - 4)
        return -1;
    size_t cap = *dst_len, o = 0;

    if (type == 0) { /* PLAIN (lib/salz.c:1082-1091) */
        if (len > cap)
            return -1;
        memcpy(dst, src + 4, len);
        *dst_len = len;
        return 0;
    }

    bitr_t r = { src + 4, len, 0, 0, 0 };
    while (r.pos < r.len) {
        uint32_t tok;
        if (!br_bits(&r, 1, &tok))
            return -1;
        if (tok == 0) { /* literal (lib/salz.c:161-169) */
            if (r.pos >= r.len || o >= cap)
                return -1;
            dst[o++] = r.s[r.pos++];
            continue;
        }
        /* offset: vnibble high part, then a raw low byte (lib/salz.c:1008-1114) */
        uint32_t v = 0, nib;
        for (int i = 0; i < 11; i++) {
            if (!br_bits(&r, 4, &nib))
                return -1;
            v = (i == 0) ? (nib & 7u) : (((v + 1u) << 3) | (nib & 7u));
            if (nib & 8u)
                break;
        }
        if (r.pos >= r.len)
            return -1;
        uint32_t off = ((v << 8) | r.s[r.pos++]) + 1u;
        uint32_t q, lo;
        if (!br_unary(&r, &q) || !br_bits(&r, 3, &lo))
            return -1;
        uint32_t flen = ((q << 3) | lo) + 3u;
        if (o + flen > cap || off > o)
            return -1;
        for (uint32_t i = 0; i < flen; i++, o++) /* overlapping copy (lib/salz.c:1126-1168) */
            dst[o] = dst[o - off];
    }
    *dst_len = o;
    return 0;
}
