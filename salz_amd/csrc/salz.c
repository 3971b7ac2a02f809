/*
 * salz.c - host C side of libsalz.so: the reference API entry points.
 *
 *   salz_encode_safe   argument handling of lib/salz.c:777-823; the block itself is encoded
 *                      on the GPU through the C ABI in gpu/pipeline.hip
 *                      (salz_gpu_encode_default). No GPU -> -1 with a message, never a CPU
 *                      fallback.
 *   salz_decode_safe   host decoder (lib/salz.c:825-1228), word-at-a-time bit reader
 *   salz_decode_frame  the same with the frame-length rule for > 16 MiB streams (§8 b4)
 *   salz_decode_blocks container decode, blocks spread over host threads
 *   encode_vnibble_le, vnibble_size   exported helpers (lib/salz.c:352, :565)
 */
#include "../../include/salz.h"
#include "../../include/salz_gpu.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

int salz_gpu_encode_default(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len);

int salz_encode_safe(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len)
{
    if (src == NULL || dst == NULL || dst_len == NULL)
        return -1; /* lib/salz.c:783-786 */
    if (*dst_len < 4)
        return -1; /* lib/salz.c:219-222 */
    int rc = salz_gpu_encode_default(src, src_len, dst, dst_len);
    if (rc != 0 && getenv("SALZ_QUIET") == NULL && src_len > 8)
        fprintf(stderr, "salz_encode_safe: %s\n", salz_gpu_last_error());
    return rc;
}

/* ---- variable-nibble code (lib/salz.c:352-445, :565-588) -------------------------------- */

size_t vnibble_size(uint32_t val)
{
    /* k nibbles cover [S_{k-1}, S_k) with S_j = 8 + 64 + ... + 8^j */
    uint64_t limit = 8, step = 8;
    size_t k = 1;
    while (k < 11 && (uint64_t)val >= limit) {
        step *= 8;
        limit += step;
        k++;
    }
    return k;
}

size_t encode_vnibble_le(uint32_t val, uint64_t *res)
{
    /* k octal digits of val - S_{k-1}, most significant in the highest nibble, terminator
     * bit 0x8 on the lowest nibble. Like the reference, only the ceil(k / 2) bytes that hold
     * the k nibbles are stored (the last one's high nibble zero when k is odd); the bytes of
     * *res beyond them are left as the caller had them. */
    size_t k = vnibble_size(val);
    uint64_t s = 0, p = 8;
    for (size_t j = 1; j < k; j++) {
        s += p;
        p *= 8;
    }
    uint64_t d = (uint64_t)val - s, r = 0;
    for (size_t j = 0; j < k; j++)
        r |= (((d >> (3 * j)) & 7u) | (j == 0 ? 8u : 0u)) << (4 * j);
    memcpy(res, &r, (k + 1) / 2); /* little-endian: nibble j in byte j / 2 */
    return k;
}

/* ---- decoder ------------------------------------------------------------------------------ */

typedef struct {
    const uint8_t *in;
    size_t len, pos;
    uint64_t bits; /* unread control bits, MSB-aligned */
    unsigned avail;
} rd_t;

static inline bool rd_word(rd_t *r)
{
    if (r->pos + 8 > r->len)
        return false;
    memcpy(&r->bits, r->in + r->pos, 8);
    r->pos += 8;
    r->avail = 64;
    return true;
}

/* read `count` (<= 32) bits MSB-first (read_bit / read_bits, lib/salz.c:919-956) */
static inline bool rd_bits(rd_t *r, unsigned count, uint32_t *out)
{
    if (r->avail == 0 && !rd_word(r))
        return false;
    if (count <= r->avail) {
        *out = (uint32_t)(r->bits >> (64 - count));
        r->bits = count == 64 ? 0 : r->bits << count;
        r->avail -= count;
        return true;
    }
    unsigned first = r->avail;
    uint32_t hi = first ? (uint32_t)(r->bits >> (64 - first)) : 0;
    count -= first;
    if (!rd_word(r))
        return false;
    *out = (hi << count) | (uint32_t)(r->bits >> (64 - count));
    r->bits <<= count;
    r->avail -= count;
    return true;
}

/* unary: zeros up to and including a terminating 1 (lib/salz.c:958-979) */
static inline bool rd_unary(rd_t *r, uint32_t *out)
{
    uint32_t z = 0;
    if (r->avail == 0 && !rd_word(r))
        return false;
    while (r->bits == 0) {
        z += r->avail;
        if (!rd_word(r))
            return false;
    }
    unsigned lead = (unsigned)__builtin_clzll(r->bits);
    r->bits = lead == 63 ? 0 : r->bits << (lead + 1);
    r->avail -= lead + 1;
    *out = z + lead;
    return true;
}

static int decode_stream(const uint8_t *body, size_t body_len, int type, uint8_t *dst,
                         size_t *dst_len)
{
    size_t cap = *dst_len, o = 0;
    if (type == 0) { /* PLAIN, lib/salz.c:1082-1091 */
        if (body_len > cap)
            return -1;
        memcpy(dst, body, body_len);
        *dst_len = body_len;
        return 0;
    }
    rd_t r = { body, body_len, 0, 0, 0 };
    while (r.pos < r.len) {
        uint32_t tok;
        if (!rd_bits(&r, 1, &tok))
            return -1;
        if (tok == 0) {
            if (r.pos >= r.len || o >= cap)
                return -1;
            dst[o++] = r.in[r.pos++];
            continue;
        }
        uint32_t v = 0, nib = 0;
        for (int i = 0; i < 11; i++) { /* read_vnibble, lib/salz.c:1008-1076 */
            if (!rd_bits(&r, 4, &nib))
                return -1;
            v = i == 0 ? (nib & 7u) : (((v + 1u) << 3) | (nib & 7u));
            if (nib & 8u)
                break;
        }
        if (r.pos >= r.len)
            return -1;
        uint32_t off = ((v << 8) | r.in[r.pos++]) + 1u;
        uint32_t q, low;
        if (!rd_unary(&r, &q) || !rd_bits(&r, 3, &low))
            return -1;
        size_t flen = (size_t)((q << 3) | low) + 3u;
        if (o + flen > cap || off > o)
            return -1;
        uint8_t *d = dst + o;
        const uint8_t *s = d - off;
        if (off >= 8) {
            size_t i = 0;
            for (; i + 8 <= flen; i += 8)
                memcpy(d + i, s + i, 8);
            for (; i < flen; i++)
                d[i] = s[i];
        } else {
            for (size_t i = 0; i < flen; i++) /* overlapping copy, lib/salz.c:1126-1168 */
                d[i] = s[i];
        }
        o += flen;
    }
    *dst_len = o;
    return 0;
}

static int parse_header(const uint8_t *src, size_t src_len, size_t frame_len, int *type,
                        size_t *body_len)
{
    if (src_len < 4)
        return -1;
    uint32_t hdr;
    memcpy(&hdr, src, 4);
    *type = (int)(hdr >> 24);
    size_t len = hdr & 0xffffffu;
    if (*type >= 2)
        return -1;
    if (frame_len >= 4 && ((frame_len - 4) & 0xffffffu) == len)
        len = frame_len - 4; /* frame-length rule for > 16 MiB streams */
    if (len > src_len - 4)
        return -1;
    *body_len = len;
    return 0;
}

int salz_decode_safe(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len)
{
    if (src == NULL || dst == NULL || dst_len == NULL)
        return -1;
    int type;
    size_t body;
    if (parse_header(src, src_len, 0, &type, &body) != 0)
        return -1;
    return decode_stream(src + 4, body, type, dst, dst_len);
}

int salz_decode_frame(const uint8_t *src, size_t frame_len, uint8_t *dst, size_t *dst_len)
{
    if (src == NULL || dst == NULL || dst_len == NULL)
        return -1;
    int type;
    size_t body;
    if (parse_header(src, frame_len, frame_len, &type, &body) != 0)
        return -1;
    return decode_stream(src + 4, body, type, dst, dst_len);
}

/* ---- container decode over host threads ---------------------------------------------------- */

typedef struct {
    const uint8_t *frame;
    size_t frame_len;
    size_t out_off;
    size_t out_cap;
    size_t out_len;
} block_job;

typedef struct {
    block_job *jobs;
    size_t njobs;
    uint8_t *dst;
    size_t block_size;
    atomic_size_t next;
    atomic_int failed;
} decode_pool;

static void *decode_worker(void *arg)
{
    decode_pool *p = arg;
    for (;;) {
        size_t j = atomic_fetch_add(&p->next, 1);
        if (j >= p->njobs || atomic_load(&p->failed))
            break;
        block_job *b = &p->jobs[j];
        size_t cap = b->out_cap;
        if (salz_decode_frame(b->frame, b->frame_len, p->dst + b->out_off, &cap) != 0) {
            atomic_store(&p->failed, 1);
            break;
        }
        b->out_len = cap;
    }
    return NULL;
}

int salz_decode_blocks(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len,
                       int threads)
{
    if (!src || !dst || !dst_len || src_len < 8)
        return -1;
    uint32_t magic, bs;
    memcpy(&magic, src, 4);
    memcpy(&bs, src + 4, 4);
    if (magic != 0x53414C5Au || bs == 0) /* programs/salzcli.c:199-207 */
        return -1;
    size_t cap = 16, n = 0, pos = 8;
    block_job *jobs = malloc(cap * sizeof(*jobs));
    if (!jobs)
        return -1;
    while (pos + 4 <= src_len) {
        uint32_t L;
        memcpy(&L, src + pos, 4);
        pos += 4;
        if (L > (size_t)salz_encoded_len_max(bs) || pos + L > src_len) {
            free(jobs);
            return -1;
        }
        if (n == cap) {
            cap *= 2;
            block_job *nj = realloc(jobs, cap * sizeof(*jobs));
            if (!nj) {
                free(jobs);
                return -1;
            }
            jobs = nj;
        }
        jobs[n].frame = src + pos;
        jobs[n].frame_len = L;
        jobs[n].out_off = n * (size_t)bs;
        jobs[n].out_len = 0;
        n++;
        pos += L;
    }
    if (pos != src_len) {
        free(jobs);
        return -1;
    }
    /* every block but the last decodes to exactly bs bytes; the last gets what is left */
    for (size_t j = 0; j < n; j++) {
        if (jobs[j].out_off > *dst_len) {
            free(jobs);
            return -1;
        }
        size_t room = *dst_len - jobs[j].out_off;
        jobs[j].out_cap = room < bs ? room : bs;
    }
    decode_pool pool;
    pool.jobs = jobs;
    pool.njobs = n;
    pool.dst = dst;
    pool.block_size = bs;
    atomic_init(&pool.next, 0);
    atomic_init(&pool.failed, 0);
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    int nt = threads > 0 ? threads : (int)(ncpu > 0 ? ncpu : 1);
    if (nt > 64)
        nt = 64;
    if ((size_t)nt > n)
        nt = n ? (int)n : 1;
    pthread_t th[64];
    int started = 0;
    for (int t = 0; t < nt; t++)
        if (pthread_create(&th[t], NULL, decode_worker, &pool) == 0)
            started++;
    if (started == 0)
        decode_worker(&pool);
    for (int t = 0; t < started; t++)
        pthread_join(th[t], NULL);
    int rc = atomic_load(&pool.failed) ? -1 : 0;
    size_t total = 0;
    for (size_t j = 0; rc == 0 && j < n; j++) {
        if (j + 1 < n && jobs[j].out_len != bs)
            rc = -1; /* only the last block may be short */
        total += jobs[j].out_len;
    }
    free(jobs);
    if (rc == 0)
        *dst_len = total;
    return rc;
}

/* ---- streaming container decode ---------------------------------------------------------- */

typedef struct {
    uint8_t *frame;
    size_t frame_len;
    uint8_t *plain;
    size_t plain_cap, plain_len;
    int rc;
} stream_job;

static void *stream_decode_worker(void *arg)
{
    stream_job *j = arg;
    size_t cap = j->plain_cap;
    j->rc = salz_decode_frame(j->frame, j->frame_len, j->plain, &cap);
    j->plain_len = cap;
    return NULL;
}

static int read_full(salz_read_fn rd, void *user, uint8_t *buf, size_t len, size_t *got)
{
    *got = 0;
    while (*got < len) {
        long long n = rd(user, buf + *got, len - *got);
        if (n < 0)
            return -1;
        if (n == 0)
            break;
        *got += (size_t)n;
    }
    return 0;
}

int salz_decode_stream(salz_read_fn rd, void *rd_user, salz_write_fn wr, void *wr_user, int threads,
                       uint64_t *in_total, uint64_t *out_total)
{
    if (!rd || !wr)
        return -1;
    uint8_t hdr[8];
    size_t got;
    if (read_full(rd, rd_user, hdr, 8, &got) != 0 || got != 8)
        return -1;
    uint32_t magic, bs;
    memcpy(&magic, hdr, 4);
    memcpy(&bs, hdr + 4, 4);
    if (magic != 0x53414C5Au || bs == 0) /* programs/salzcli.c:199-207 */
        return -1;
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    /* default: one thread per core, at most 8 (8 x ~2 blocks of buffers bound the memory) */
    int nt = threads > 0 ? threads : (int)(ncpu > 0 ? (ncpu < 8 ? ncpu : 8) : 1);
    if (nt > 32)
        nt = 32;
    const size_t fcap = (size_t)salz_encoded_len_max(bs);
    stream_job *jobs = calloc((size_t)nt, sizeof(*jobs));
    int rc = jobs ? 0 : -1;
    for (int t = 0; rc == 0 && t < nt; t++) {
        jobs[t].frame = malloc(fcap);
        jobs[t].plain = malloc((size_t)bs + 8);
        jobs[t].plain_cap = bs;
        if (!jobs[t].frame || !jobs[t].plain)
            rc = -1;
    }
    uint64_t nin = 8, nout = 0;
    int eof = 0;
    while (rc == 0 && !eof) {
        int k = 0;
        for (; k < nt; k++) { /* up to nt frames: u32 length + stream (programs/salzcli.c:223-264) */
            uint8_t lb[4];
            if (read_full(rd, rd_user, lb, 4, &got) != 0) {
                rc = -1;
                break;
            }
            if (got == 0) {
                eof = 1;
                break;
            }
            uint32_t L;
            memcpy(&L, lb, 4);
            if (got != 4 || L > fcap || read_full(rd, rd_user, jobs[k].frame, L, &got) != 0 || got != L) {
                rc = -1;
                break;
            }
            jobs[k].frame_len = L;
            nin += 4 + (uint64_t)L;
        }
        if (rc != 0 || k == 0)
            break;
        pthread_t th[32];
        int started[32] = {0};
        for (int t = 0; t < k; t++)
            started[t] = pthread_create(&th[t], NULL, stream_decode_worker, &jobs[t]) == 0;
        for (int t = 0; t < k; t++) {
            if (started[t])
                pthread_join(th[t], NULL);
            else
                stream_decode_worker(&jobs[t]);
        }
        for (int t = 0; t < k && rc == 0; t++) {
            if (jobs[t].rc != 0 || wr(wr_user, jobs[t].plain, jobs[t].plain_len) != 0)
                rc = -1;
            nout += jobs[t].plain_len;
        }
    }
    for (int t = 0; jobs && t < nt; t++) {
        free(jobs[t].frame);
        free(jobs[t].plain);
    }
    free(jobs);
    if (rc == 0) {
        if (in_total)
            *in_total = nin;
        if (out_total)
            *out_total = nout;
    }
    return rc;
}
