/*
 * parse_sim.c - CPU simulation of the GPU parse fixed point (design tool, not shipped).
 * Given candidate arrays (offP, lenP, offN, lenN per position), runs the chunked fixed-point
 * iteration for a chunk size and reports iterations and exit-node counts; checks the result
 * against the sequential DP.
 *   int parse_sim(const int32_t *psv, const int32_t *lp, const int32_t *nsv, const int32_t *ln,
 *                 int32_t n, int32_t chunk, int32_t seed_mode, int32_t *iters_out,
 *                 int64_t *exits_out)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

static uint32_t vn(uint32_t v)
{
    static const uint32_t lim[10] = {8u, 72u, 584u, 4680u, 37448u, 299592u, 2396744u,
                                     19173960u, 153391688u, 1227133512u};
    uint32_t k = 1;
    for (int i = 0; i < 10; i++)
        k += v >= lim[i];
    return k;
}

static uint32_t fbits(uint32_t off, uint32_t len)
{
    return 1u + 8u + 4u * vn((off - 1u) >> 8) + ((len - 3u) >> 3) + 4u;
}

int parse_sim(const int32_t *psv, const int32_t *lp, const int32_t *nsv, const int32_t *ln,
              int32_t n, int32_t chunk, int32_t seed_mode, int32_t *iters_out, int64_t *exits_out)
{
    uint32_t *cin = malloc(4ull * (n + 1)), *cout = malloc(4ull * (n + 1));
    uint32_t *ex = malloc(4ull * n), *sm = malloc(4ull * n), *ref = malloc(4ull * (n + 1));
    uint8_t *chold = malloc(n), *chnew = malloc(n), *flag = calloc(n + 1, 1);
    uint8_t *refch = malloc(n);
    /* sequential reference DP */
    ref[n] = 0;
    for (int32_t p = n - 1; p >= 0; p--) {
        uint32_t best = 9u + ref[p + 1];
        uint8_t ch = 0;
        if (p) {
            if (lp[p] >= 3) {
                uint32_t a = fbits(p - psv[p], lp[p]) + ref[p + lp[p]];
                if ((int32_t)a < (int32_t)best) { best = a; ch = 1; }
            }
            if (ln[p] >= 3) {
                uint32_t a = fbits(p - nsv[p], ln[p]) + ref[p + ln[p]];
                if ((int32_t)a < (int32_t)best) { best = a; ch = 2; }
            }
        }
        ref[p] = best;
        refch[p] = ch;
    }
    if (seed_mode >= 3) {
        /* local bits-per-byte estimate, suffix-summed (x16 fixed point) */
        uint64_t acc = 0;
        cin[n] = 0;
        for (int32_t q = n - 1; q >= 0; q--) {
            uint32_t b = 9u * 16u;
            if (q) {
                if (lp[q] >= 3) { uint32_t c = 16u * fbits(q - psv[q], lp[q]) / (uint32_t)lp[q]; if (c < b) b = c; }
                if (ln[q] >= 3) { uint32_t c = 16u * fbits(q - nsv[q], ln[q]) / (uint32_t)ln[q]; if (c < b) b = c; }
            }
            if (seed_mode == 4 && b < 16u) b = 16u;
            acc += b;
            cin[q] = (uint32_t)(acc / 16u);
        }
    } else
    for (int32_t q = 0; q <= n; q++)
        cin[q] = seed_mode == 0 ? 9u * (uint32_t)(n - q) : (seed_mode == 1 ? 0u : 3u * (uint32_t)(n - q));
    memset(chold, 0xff, n);
    /* PARSE_SIM_OVL=V, PARSE_SIM_OVL_IT=t: the first t passes walk V positions past each chunk's
       end first (their states used only by that chunk, targets past them read cin) */
    const int32_t ovl = getenv("PARSE_SIM_OVL") ? atoi(getenv("PARSE_SIM_OVL")) : 0;
    const int ovl_it = getenv("PARSE_SIM_OVL_IT") ? atoi(getenv("PARSE_SIM_OVL_IT")) : 1;
    uint32_t *oc = malloc(4ull * (ovl + 1)), *oe = malloc(4ull * (ovl + 1)), *os = malloc(4ull * (ovl + 1));
    int it;
    int64_t exits = 0;
    /* PARSE_SIM_SEG=S: Gauss-Seidel over S segments of chunks, right to left: a segment's chunks
       read the exact costs the pass already made for later segments, and the segment's own exact
       costs are formed before the next segment walks (one cost array, cin) */
    const int32_t segs = getenv("PARSE_SIM_SEG") ? atoi(getenv("PARSE_SIM_SEG")) : 0;
    if (segs > 0) {
        const int32_t nch = (n + chunk - 1) / chunk, per = (nch + segs - 1) / segs;
        for (it = 0; it < 100000; it++) {
            long changed = 0;
            const int inter = getenv("PARSE_SIM_INTERLEAVE") != NULL;
            for (int32_t sg = segs - 1; sg >= 0; sg--) {
                const int32_t s0 = inter ? sg * chunk : sg * per * chunk;
                const int32_t s1 = inter ? n : ((sg + 1) * per * chunk < n ? (sg + 1) * per * chunk : n);
                if (s0 >= s1)
                    continue;
                for (int32_t a = s0; a < s1; a += inter ? segs * chunk : chunk) {
                    int32_t b = a + chunk < n ? a + chunk : n;
                    for (int32_t p = b - 1; p >= a; p--) {
                        uint32_t nx1 = p + 1;
                        uint32_t best = 9u + (nx1 >= (uint32_t)b ? cin[nx1] : cout[nx1]);
                        uint32_t len = 1, w = 9;
                        uint8_t ch = 0;
                        if (p) {
                            if (lp[p] >= 3) {
                                uint32_t q = p + lp[p], wf = fbits(p - psv[p], lp[p]);
                                uint32_t alt = wf + (q >= (uint32_t)b ? cin[q] : cout[q]);
                                if ((int32_t)alt < (int32_t)best) { best = alt; len = lp[p]; w = wf; ch = 1; }
                            }
                            if (ln[p] >= 3) {
                                uint32_t q = p + ln[p], wf = fbits(p - nsv[p], ln[p]);
                                uint32_t alt = wf + (q >= (uint32_t)b ? cin[q] : cout[q]);
                                if ((int32_t)alt < (int32_t)best) { best = alt; len = ln[p]; w = wf; ch = 2; }
                            }
                        }
                        uint32_t nx = p + len;
                        if (nx >= (uint32_t)b) { ex[p] = nx; sm[p] = w; }
                        else { ex[p] = ex[nx]; sm[p] = w + sm[nx]; }
                        cout[p] = best;
                        changed += ch != chold[p];
                        chold[p] = ch;
                    }
                }
                if (inter) { /* exact costs of the current decisions everywhere */
                    cin[n] = 0;
                    for (int32_t q = n - 1; q >= 0; q--)
                        cin[q] = sm[q] + cin[ex[q]];
                } else {
                    for (int32_t q = s1 - 1; q >= s0; q--) /* the segment's exact costs */
                        cin[q] = sm[q] + cin[ex[q]];
                }
            }
            if (getenv("PARSE_SIM_VERBOSE"))
                fprintf(stderr, "seg it %d changed %ld\n", it, changed);
            if (!changed)
                break;
        }
        int ok = 1;
        for (int32_t p = 1; p < n; p++)
            if (chold[p] != refch[p]) { ok = 0; break; }
        *iters_out = it + 1;
        *exits_out = 0;
        free(oc); free(oe); free(os); free(cin); free(cout); free(ex); free(sm); free(ref); free(chold); free(chnew); free(flag); free(refch);
        return ok;
    }
    for (it = 0; it < 100000; it++) {
        long changed = 0;
        const int32_t V = it < ovl_it ? ovl : 0;
        for (int32_t a = 0; a < n; a += chunk) {
            int32_t b = a + chunk < n ? a + chunk : n;
            const int32_t bv = b + V < n ? b + V : n;
            /* target q >= b: overlap state (cost, exit, sum) or cin */
#define TC(q) ((q) < (uint32_t)bv ? oc[(q) - b] : cin[q])
            for (int32_t p = bv - 1; p >= b; p--) {
                uint32_t best = 9u + TC((uint32_t)p + 1), len = 1, w = 9;
                if (lp[p] >= 3) {
                    uint32_t q = p + lp[p], wf = fbits(p - psv[p], lp[p]), alt = wf + TC(q);
                    if ((int32_t)alt < (int32_t)best) { best = alt; len = lp[p]; w = wf; }
                }
                if (ln[p] >= 3) {
                    uint32_t q = p + ln[p], wf = fbits(p - nsv[p], ln[p]), alt = wf + TC(q);
                    if ((int32_t)alt < (int32_t)best) { best = alt; len = ln[p]; w = wf; }
                }
                uint32_t nx = p + len;
                oc[p - b] = best;
                if (nx >= (uint32_t)bv) { oe[p - b] = nx; os[p - b] = w; }
                else { oe[p - b] = oe[nx - b]; os[p - b] = w + os[nx - b]; }
            }
            for (int32_t p = b - 1; p >= a; p--) {
                uint32_t nx1 = p + 1;
                uint32_t best = 9u + (nx1 >= (uint32_t)b ? TC(nx1) : cout[nx1]);
                uint32_t len = 1, w = 9;
                uint8_t ch = 0;
                if (p) {
                    if (lp[p] >= 3) {
                        uint32_t q = p + lp[p], wf = fbits(p - psv[p], lp[p]);
                        uint32_t alt = wf + (q >= (uint32_t)b ? TC(q) : cout[q]);
                        if ((int32_t)alt < (int32_t)best) { best = alt; len = lp[p]; w = wf; ch = 1; }
                    }
                    if (ln[p] >= 3) {
                        uint32_t q = p + ln[p], wf = fbits(p - nsv[p], ln[p]);
                        uint32_t alt = wf + (q >= (uint32_t)b ? TC(q) : cout[q]);
                        if ((int32_t)alt < (int32_t)best) { best = alt; len = ln[p]; w = wf; ch = 2; }
                    }
                }
                uint32_t nx = p + len;
                if (nx >= (uint32_t)bv) { ex[p] = nx; sm[p] = w; }
                else if (nx >= (uint32_t)b) { ex[p] = oe[nx - b]; sm[p] = w + os[nx - b]; }
                else { ex[p] = ex[nx]; sm[p] = w + sm[nx]; }
                cout[p] = best;
                changed += ch != chold[p];
                chnew[p] = ch;
            }
        }
        uint8_t *t = chold; chold = chnew; chnew = t;
        if (getenv("PARSE_SIM_VERBOSE")) {
            /* changed positions: how many, and the span of chunks they fall in */
            fprintf(stderr, "it %d changed %ld\n", it, changed);
        }
        if (!changed && it > ovl_it - 1 + (ovl ? 1 : 0))
            break;
        /* exact costs of the new decisions */
        memset(flag, 0, n + 1);
        for (int32_t p = 0; p < n; p++)
            flag[ex[p]] = 1;
        flag[n] = 1;
        exits = 0;
        for (int32_t q = 0; q <= n; q++)
            exits += flag[q];
        cout[n] = 0;
        for (int32_t q = n - 1; q >= 0; q--) /* backward: targets are exact already */
            cout[q] = sm[q] + cout[ex[q]];
        uint32_t *tc = cin; cin = cout; cout = tc;
        if (getenv("PARSE_SIM_VERBOSE")) {
            /* chunks whose out-of-chunk targets did not all shift by one delta (cin = new
               exact costs, cout = the costs the pass just used) */
            long bad = 0, nch = 0;
            for (int32_t a = 0; a < n; a += chunk, nch++) {
                int32_t b = a + chunk < n ? a + chunk : n;
                int have = 0, fail = 0;
                uint32_t d0 = 0;
                for (int32_t p = a; p < b && !fail; p++) {
                    uint32_t qs[3] = {(uint32_t)p + 1, p && lp[p] >= 3 ? (uint32_t)(p + lp[p]) : 0,
                                      p && ln[p] >= 3 ? (uint32_t)(p + ln[p]) : 0};
                    for (int k = 0; k < 3; k++) {
                        uint32_t q = qs[k];
                        if (q < (uint32_t)b)
                            continue;
                        uint32_t d = cin[q] - cout[q];
                        if (!have) { d0 = d; have = 1; }
                        else if (d != d0) { fail = 1; break; }
                    }
                }
                bad += fail;
            }
            fprintf(stderr, "   after it %d: %ld of %ld chunks see non-uniform target shifts\n", it, bad, nch);
        }
    }
    int ok = 1;
    for (int32_t p = 1; p < n; p++)
        if (chold[p] != refch[p]) { ok = 0; break; }
    *iters_out = it + 1;
    *exits_out = exits;
    free(oc); free(oe); free(os); free(cin); free(cout); free(ex); free(sm); free(ref); free(chold); free(chnew); free(flag); free(refch);
    return ok;
}
