/*
 * datagen.c - deterministic synthetic inputs for parity tests and bench.py.
 *
 * Generators:
 *   fib   : Fibonacci word s0="a", s1="ab", s_{k+1} = s_k s_{k-1}; first N bytes (C5).
 *   smx   : splitmix64 stream, byte = z & 0xff (alphabet 256) or 'a' + z % A.
 *   text  : wiki-dump-like text surrogate standing in for enwik8/enwik9 (absent from
 *           the container and the GPU box): XML page scaffolding, Zipf-distributed
 *           pseudo-words, wiki markup, and occasional near-verbatim repeats of earlier
 *           passages. Stable for a given (N, seed) on every platform.
 *   mixed : Silesia-like blend of text, binary records, runs and splitmix noise (C3).
 *
 * Workload generation only: used by tests and bench.py, never by the codec itself.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t smx_next(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void datagen_fib(uint8_t *out, size_t n)
{
    if (n == 0)
        return;
    /* Grow in place: s_{k+1} = s_k s_{k-1}, so out holds s_k and we append s_{k-1}. */
    out[0] = 'a';
    if (n == 1)
        return;
    out[1] = 'b';
    size_t len = 2, prev = 1; /* out[0,len) = s_k, its prefix of length prev = s_{k-1} */
    while (len < n) {
        size_t add = prev;
        if (len + add > n)
            add = n - len;
        memcpy(out + len, out, add);
        prev = len;
        len += add;
    }
}

void datagen_smx(uint8_t *out, size_t n, uint64_t seed, uint32_t alphabet)
{
    uint64_t s = seed;
    for (size_t i = 0; i < n; i++) {
        uint64_t z = smx_next(&s);
        out[i] = alphabet >= 256 ? (uint8_t)(z & 0xff) : (uint8_t)('a' + z % alphabet);
    }
}

/* ---------------------------------------------------------------------------------- */

typedef struct {
    uint8_t *out;
    size_t n, pos;
    uint64_t rng;
} tw_t;

static inline uint64_t tw_rand(tw_t *w) { return smx_next(&w->rng); }
static inline uint32_t tw_below(tw_t *w, uint32_t k) { return (uint32_t)(tw_rand(w) % k); }

static void tw_put(tw_t *w, const char *s, size_t len)
{
    if (w->pos >= w->n)
        return;
    if (len > w->n - w->pos)
        len = w->n - w->pos;
    memcpy(w->out + w->pos, s, len);
    w->pos += len;
}

static void tw_str(tw_t *w, const char *s) { tw_put(w, s, strlen(s)); }

static void tw_num(tw_t *w, uint64_t v, int width)
{
    char buf[24];
    int i = 23;
    buf[i] = 0;
    do {
        buf[--i] = (char)('0' + v % 10);
        v /= 10;
        width--;
    } while (v || width > 0);
    tw_str(w, buf + i);
}

#define VOCAB 40000
#define WORD_MAX 14

typedef struct {
    char words[VOCAB][WORD_MAX + 1];
    uint8_t wlen[VOCAB];
    uint32_t cdf[VOCAB]; /* Zipf(1.0) cumulative weights scaled to 2^32 - 1 */
} vocab_t;

static void vocab_build(vocab_t *v, uint64_t seed)
{
    static const char *onset[] = { "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n",
        "p", "r", "s", "t", "v", "w", "st", "th", "ch", "sh", "pr", "tr", "gr", "br",
        "cl", "fl", "pl", "", "", "" };
    static const char *nucleus[] = { "a", "e", "i", "o", "u", "ea", "io", "ou", "ai", "e",
        "a", "o", "i", "y" };
    static const char *coda[] = { "", "", "", "n", "r", "s", "t", "l", "nd", "st", "ng",
        "rt", "m", "ck", "ss", "ll" };
    uint64_t s = seed ^ 0xC0FFEEull;
    double total = 0.0;
    static double wts[VOCAB];
    for (int i = 0; i < VOCAB; i++) {
        char buf[64] = { 0 };
        int syl = 1 + (int)(i < 60 ? 0 : (i < 2000 ? smx_next(&s) % 2 : smx_next(&s) % 3 + (i > 15000)));
        for (int k = 0; k < syl; k++) {
            strcat(buf, onset[smx_next(&s) % (sizeof(onset) / sizeof(*onset))]);
            strcat(buf, nucleus[smx_next(&s) % (sizeof(nucleus) / sizeof(*nucleus))]);
            strcat(buf, coda[smx_next(&s) % (sizeof(coda) / sizeof(*coda))]);
        }
        size_t L = strlen(buf);
        if (L > WORD_MAX)
            L = WORD_MAX;
        memcpy(v->words[i], buf, L);
        v->words[i][L] = 0;
        v->wlen[i] = (uint8_t)L;
        wts[i] = 1.0 / (double)(i + 2);
        total += wts[i];
    }
    double run = 0.0;
    for (int i = 0; i < VOCAB; i++) {
        run += wts[i];
        double c = run / total * 4294967295.0;
        v->cdf[i] = c >= 4294967295.0 ? 0xffffffffu : (uint32_t)c;
    }
    v->cdf[VOCAB - 1] = 0xffffffffu;
}

static int vocab_pick(const vocab_t *v, tw_t *w)
{
    uint32_t u = (uint32_t)(tw_rand(w) >> 32);
    int lo = 0, hi = VOCAB - 1;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (v->cdf[mid] >= u)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

static void tw_word(tw_t *w, const vocab_t *v, int cap)
{
    int i = vocab_pick(v, w);
    char buf[WORD_MAX + 1];
    memcpy(buf, v->words[i], v->wlen[i] + 1u);
    if (cap && buf[0] >= 'a' && buf[0] <= 'z')
        buf[0] = (char)(buf[0] - 32);
    tw_put(w, buf, v->wlen[i]);
}

static void tw_sentence(tw_t *w, const vocab_t *v)
{
    int words = 4 + (int)tw_below(w, 18);
    for (int k = 0; k < words; k++) {
        if (k)
            tw_str(w, " ");
        uint32_t r = tw_below(w, 100);
        if (r < 6) {
            tw_str(w, "[[");
            tw_word(w, v, 1);
            if (tw_below(w, 3) == 0) {
                tw_str(w, " ");
                tw_word(w, v, 1);
            }
            tw_str(w, "]]");
        } else if (r < 8) {
            tw_num(w, tw_below(w, 3000), 0);
        } else if (r < 9) {
            tw_str(w, "'''");
            tw_word(w, v, 1);
            tw_str(w, "'''");
        } else {
            tw_word(w, v, k == 0 || r < 12);
        }
        if (k + 1 < words && tw_below(w, 12) == 0)
            tw_str(w, ",");
    }
    tw_str(w, tw_below(w, 10) == 0 ? "; " : ". ");
}

static void tw_page(tw_t *w, const vocab_t *v, uint64_t *page_id)
{
    tw_str(w, "  <page>\n    <title>");
    tw_word(w, v, 1);
    if (tw_below(w, 2)) {
        tw_str(w, " ");
        tw_word(w, v, 1);
    }
    tw_str(w, "</title>\n    <id>");
    tw_num(w, (*page_id)++, 0);
    tw_str(w, "</id>\n    <revision>\n      <id>");
    tw_num(w, 15898000 + tw_below(w, 900000), 0);
    tw_str(w, "</id>\n      <timestamp>200");
    tw_num(w, 2 + tw_below(w, 5), 0);
    tw_str(w, "-");
    tw_num(w, 1 + tw_below(w, 12), 2);
    tw_str(w, "-");
    tw_num(w, 1 + tw_below(w, 28), 2);
    tw_str(w, "T");
    tw_num(w, tw_below(w, 24), 2);
    tw_str(w, ":");
    tw_num(w, tw_below(w, 60), 2);
    tw_str(w, ":");
    tw_num(w, tw_below(w, 60), 2);
    tw_str(w, "Z</timestamp>\n      <contributor>\n        <username>");
    tw_word(w, v, 1);
    tw_str(w, "</username>\n        <id>");
    tw_num(w, tw_below(w, 500000), 0);
    tw_str(w, "</id>\n      </contributor>\n      <text xml:space=\"preserve\">");
    if (tw_below(w, 4) == 0) {
        tw_str(w, "{{");
        tw_word(w, v, 1);
        tw_str(w, " box\n| name = ");
        tw_word(w, v, 1);
        tw_str(w, "\n| image = ");
        tw_word(w, v, 0);
        tw_str(w, ".jpg\n}}\n");
    }
    int paras = 1 + (int)tw_below(w, 7);
    for (int p = 0; p < paras && w->pos < w->n; p++) {
        if (p && tw_below(w, 3) == 0) {
            tw_str(w, "\n== ");
            tw_word(w, v, 1);
            tw_str(w, " ==\n");
        }
        if (p && w->pos > 4096 && tw_below(w, 40) == 0) {
            /* near-verbatim repeat of an earlier passage (quoted / duplicated text) */
            size_t len = 200 + tw_below(w, 2800);
            size_t back = 1024 + (size_t)(tw_rand(w) % (w->pos - 1024 < 8000000 ? w->pos - 1024 : 8000000));
            size_t from = w->pos - back;
            if (from + len > w->pos)
                len = w->pos - from;
            for (size_t i = 0; i < len && w->pos < w->n; i++) {
                uint8_t c = w->out[from + i];
                if (tw_below(w, 400) == 0)
                    c = (uint8_t)('a' + tw_below(w, 26));
                w->out[w->pos++] = c;
            }
            tw_str(w, "\n");
            continue;
        }
        int sents = 1 + (int)tw_below(w, 8);
        if (tw_below(w, 5) == 0) {
            for (int s = 0; s < sents; s++) {
                tw_str(w, "* ");
                tw_sentence(w, v);
                tw_str(w, "\n");
            }
        } else {
            for (int s = 0; s < sents; s++)
                tw_sentence(w, v);
            tw_str(w, "\n\n");
        }
    }
    tw_str(w, "</text>\n    </revision>\n  </page>\n");
}

static void text_fill(uint8_t *out, size_t n, uint64_t seed, size_t start_pos)
{
    vocab_t *v = malloc(sizeof(*v));
    if (!v)
        return;
    vocab_build(v, seed);
    tw_t w = { out, n, start_pos, seed * 0x9E3779B97F4A7C15ull + 1 };
    uint64_t page_id = 10;
    if (start_pos == 0)
        tw_str(&w, "<mediawiki xmlns=\"http://www.mediawiki.org/xml/export-0.3/\" version=\"0.3\">\n");
    while (w.pos < w.n)
        tw_page(&w, v, &page_id);
    free(v);
}

void datagen_text(uint8_t *out, size_t n, uint64_t seed)
{
    text_fill(out, n, seed, 0);
}

/* Silesia-like mix: alternating segments of text, structured binary records,
 * low-entropy runs and splitmix noise. */
void datagen_mixed(uint8_t *out, size_t n, uint64_t seed)
{
    uint64_t s = seed ^ 0x5EED5EEDull;
    size_t pos = 0;
    while (pos < n) {
        size_t seg = 65536 + (size_t)(smx_next(&s) % (1u << 20));
        if (seg > n - pos)
            seg = n - pos;
        uint32_t kind = (uint32_t)(smx_next(&s) % 8);
        if (kind < 3) { /* text */
            uint8_t *tmp = malloc(seg);
            if (!tmp)
                return;
            datagen_text(tmp, seg, smx_next(&s));
            memcpy(out + pos, tmp, seg);
            free(tmp);
        } else if (kind < 5) { /* binary records: little-endian ints with slow drift */
            uint32_t base = (uint32_t)smx_next(&s);
            for (size_t i = 0; i + 4 <= seg; i += 4) {
                uint32_t val = base + (uint32_t)(smx_next(&s) % 64);
                if (smx_next(&s) % 16 == 0)
                    base += (uint32_t)(smx_next(&s) % 4096);
                memcpy(out + pos + i, &val, 4);
            }
            for (size_t i = seg & ~(size_t)3; i < seg; i++)
                out[pos + i] = 0;
        } else if (kind < 6) { /* runs of zeros and small symbols */
            for (size_t i = 0; i < seg;) {
                size_t run = 1 + (size_t)(smx_next(&s) % 300);
                uint8_t c = (smx_next(&s) % 3 == 0) ? (uint8_t)(smx_next(&s) % 8) : 0;
                for (size_t k = 0; k < run && i < seg; k++, i++)
                    out[pos + i] = c;
            }
        } else if (kind < 7) { /* random bytes */
            for (size_t i = 0; i < seg; i++)
                out[pos + i] = (uint8_t)smx_next(&s);
        } else { /* repeated table rows */
            uint8_t row[97];
            for (size_t i = 0; i < sizeof(row); i++)
                row[i] = (uint8_t)smx_next(&s);
            for (size_t i = 0; i < seg; i++) {
                uint8_t c = row[i % sizeof(row)];
                if (i % sizeof(row) == 0)
                    row[smx_next(&s) % sizeof(row)] ^= (uint8_t)smx_next(&s);
                out[pos + i] = c;
            }
        }
        pos += seg;
    }
}
