/*
 * runs_share.c - how much of each prefix-doubling round (salz_amd/csrc/gpu/sa.hip) on the mixed
 * surrogate starts inside runs of equal bytes, or inside rows repeated with period 97. Test
 * infrastructure / measurement aid for DESIGN.md §9 (round 6): the CPU oracle's suffix array
 * (oracle/liboracle.so) gives each suffix's larger LCP with an SA neighbour, which decides the
 * round in which the doubling sort finishes it.
 *
 *   gcc -O2 -o /tmp/runs_share tests/sim/runs_share.c -Loracle -loracle -Ltools -ldatagen \
 *       -Wl,-rpath,$PWD/oracle:$PWD/tools
 *   /tmp/runs_share 16777216
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);
void datagen_mixed(uint8_t *out, size_t n, uint64_t seed);

int main(int argc, char **argv)
{
    const size_t N = argc > 1 ? (size_t)atol(argv[1]) : 16777216;
    uint8_t *T = calloc(N + 64, 1);
    datagen_mixed(T, N, 1);
    const int32_t n = (int32_t)(N - 8);
    int32_t *SA = malloc(4 * (size_t)n), *R = malloc(4 * (size_t)n), *L = malloc(4 * ((size_t)n + 1));
    int32_t *M = malloc(4 * (size_t)n), *run = malloc(4 * (size_t)n);
    if (!T || !SA || !R || !L || !M || !run || oracle_suffix_array(T, SA, n) != 0)
        return 1;
    for (int32_t r = 0; r < n; r++)
        R[SA[r]] = r;
    int32_t h = 0;  // Kasai
    L[0] = 0;
    L[n] = 0;
    for (int32_t i = 0; i < n; i++) {
        if (R[i] > 0) {
            const int32_t j = SA[R[i] - 1];
            while (i + h < n && j + h < n && T[i + h] == T[j + h])
                h++;
            L[R[i]] = h;
            if (h > 0)
                h--;
        } else {
            h = 0;
        }
    }
    for (int32_t r = 0; r < n; r++) {
        const int32_t a = L[r], b = r + 1 < n ? L[r + 1] : 0;
        M[SA[r]] = a > b ? a : b;
    }
    run[n - 1] = 1;  // equal bytes from i on
    for (int32_t i = n - 2; i >= 0; i--)
        run[i] = T[i] == T[i + 1] ? run[i + 1] + 1 : 1;
    for (int t = 1; t < 14; t++) {
        const long d = 8L << (t - 1);  // raw 8-byte round-0 keys: depth 8 after round 0
        long tot = 0, inrun = 0, per = 0;
        for (int32_t i = 0; i < n; i++) {
            if (M[i] < d)
                continue;
            tot++;
            if (run[i] >= 16)
                inrun++;
            else if (i + 97 + 64 < n && !memcmp(T + i, T + i + 97, 64))
                per++;
        }
        if (!tot)
            break;
        printf("round %d (depth %ld): list %ld, in runs >= 16: %ld (%.0f%%), period-97 rows: %ld (%.0f%%)\n", t, d,
               tot, inrun, 100.0 * inrun / tot, per, 100.0 * per / tot);
    }
    return 0;
}
