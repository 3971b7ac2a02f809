/*
 * rank_reads.c - which rank writes of the prefix-doubling suffix sort (salz_amd/csrc/gpu/sa.hip)
 * does a later round read? Test infrastructure / measurement aid for DESIGN.md §9 (round 6): it
 * uses the CPU oracle's suffix array (oracle/liboracle.so) only to get each suffix's largest LCP
 * with a neighbour, which decides the round in which the doubling sort finishes it.
 *
 *   gcc -O2 -o /tmp/rank_reads tests/sim/rank_reads.c -Loracle -loracle -Ltools -ldatagen \
 *       -Wl,-rpath,$PWD/oracle:$PWD/tools
 *   /tmp/rank_reads 100000000 0      # text surrogate (h0 = 9); 1: mixed data (h0 = 8)
 *
 * Model (sa.hip): suffix i is finished after the round whose depth d exceeds M[i], the larger LCP
 * with its two SA neighbours. Round t >= 2 sorts its list {i : M[i] >= d_{t-1}} by rank[i + d_{t-1}]
 * (round 1, the text round, reads the text), so position j's rank is read in round t iff
 * M[j - d_{t-1}] >= d_{t-1}. Printed per round: the list, its singletons (whose ranks are final),
 * its survivors and how many of those the next round reads; then, per round, how many of the
 * singletons' final ranks any later round reads at all.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);
void datagen_text(uint8_t *out, size_t n, uint64_t seed);
void datagen_mixed(uint8_t *out, size_t n, uint64_t seed);

int main(int argc, char **argv)
{
    const size_t N = argc > 1 ? (size_t)atol(argv[1]) : 20000000;
    const int kind = argc > 2 ? atoi(argv[2]) : 0;
    uint8_t *T = calloc(N + 64, 1);
    if (kind == 0)
        datagen_text(T, N, 1);
    else
        datagen_mixed(T, N, 1);
    const int32_t n = (int32_t)(N - 8);
    int32_t *SA = malloc(4 * (size_t)n), *R = malloc(4 * (size_t)n), *L = malloc(4 * ((size_t)n + 1));
    int32_t *M = malloc(4 * (size_t)n);
    uint8_t *rd = calloc((size_t)n, 1);
    if (!T || !SA || !R || !L || !M || !rd || oracle_suffix_array(T, SA, n) != 0)
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
    const long h0 = kind == 0 ? 9 : 8;  // round 0's depth (9 symbols of 7 bits, or 8 raw bytes)
    for (int t = 1; t < 14; t++) {
        const long dp = h0 << (t - 1), d = h0 << t;
        long list = 0, sing = 0, surv = 0, next = 0;
        for (int32_t i = 0; i < n; i++) {
            if (M[i] < dp)
                continue;
            list++;
            if (M[i] < d) {
                sing++;
            } else {
                surv++;
                next += i >= d && M[i - d] >= d;
            }
        }
        if (!list)
            break;
        printf("round %d depth %ld->%ld: list %ld, singletons %ld, survivors %ld, of which read next round %ld\n", t,
               dp, d, list, sing, surv, next);
    }
    long reads = 0;
    for (int tp = 2; tp < 16; tp++) {
        const long d = h0 << (tp - 1);
        for (int32_t i = 0; i + d < n; i++)
            if (M[i] >= d) {
                rd[i + d] = 1;
                reads++;
            }
    }
    long r0 = 0, r0r = 0;
    for (int32_t j = 0; j < n; j++)
        if (M[j] < h0) {
            r0++;
            r0r += rd[j];
        }
    printf("rank reads in rounds >= 2: %ld; round 0 finishes %ld, of whose ranks %ld are ever read\n", reads, r0, r0r);
    for (int t = 1; t < 14; t++) {
        const long dp = h0 << (t - 1), d = h0 << t;
        long s = 0, sr = 0;
        for (int32_t j = 0; j < n; j++)
            if (M[j] >= dp && M[j] < d) {
                s++;
                sr += rd[j];
            }
        if (s)
            printf("round %d: singletons %ld, ranks ever read %ld\n", t, s, sr);
    }
    return 0;
}
