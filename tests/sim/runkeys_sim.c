/*
 * runkeys_sim.c - prefix doubling (salz_amd/csrc/gpu/sa.hip) with "run keys": in a rank round of
 * depth h, a suffix inside a run of one byte c with a >= h bytes of the run left is keyed by
 * (c < the byte after the run, +-a, rank of the suffix after the run) instead of rank[i + h], so
 * the suffixes of runs are ordered by their run remainders in one round instead of peeling off
 * h .. 2h per round. Test infrastructure / measurement aid for DESIGN.md: the CPU oracle's suffix
 * array (oracle/liboracle.so) gives each suffix's largest LCP with an SA neighbour (M).
 *
 *   gcc -O2 -o /tmp/runkeys_sim tests/sim/runkeys_sim.c -Loracle -loracle -Ltools -ldatagen \
 *       -Wl,-rpath,$PWD/oracle:$PWD/tools
 *   /tmp/runkeys_sim 16777216 1     # mixed surrogate (round-0 depth 8); 0: text (depth 9)
 *
 * Model: after round 0 (depth h0) suffix i is unfinished iff M[i] >= h0. A round of depth h -> 2h
 * finishes i iff M[i] < 2h, or, with run keys and a(i) >= h, iff M[i] < a(i) + h (its group after
 * the round is the suffixes sharing its first a(i) + h bytes).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);
void datagen_text(uint8_t *out, size_t n, uint64_t seed);
void datagen_mixed(uint8_t *out, size_t n, uint64_t seed);

int main(int argc, char **argv)
{
    const size_t N = argc > 1 ? (size_t)atol(argv[1]) : 16777216;
    const int kind = argc > 2 ? atoi(argv[2]) : 1;
    uint8_t *T = calloc(N + 64, 1);
    if (kind == 0)
        datagen_text(T, N, 1);
    else
        datagen_mixed(T, N, 1);
    const int32_t n = (int32_t)(N - 8);
    int32_t *SA = malloc(4 * (size_t)n), *R = malloc(4 * (size_t)n), *L = malloc(4 * ((size_t)n + 1));
    int32_t *M = malloc(4 * (size_t)n), *A = malloc(4 * (size_t)n);
    uint8_t *done = calloc((size_t)n, 1);
    if (!T || !SA || !R || !L || !M || !A || !done || oracle_suffix_array(T, SA, n) != 0)
        return 1;
    for (int32_t r = 0; r < n; r++)
        R[SA[r]] = r;
    int32_t h = 0;
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
    A[n - 1] = 1;  // bytes of the run left at i (within the suffix text)
    for (int32_t i = n - 2; i >= 0; i--)
        A[i] = T[i] == T[i + 1] ? A[i + 1] + 1 : 1;
    const long h0 = kind == 0 ? 9 : 8;
    for (int mode = 0; mode < 2; mode++) {
        long total = 0, runkeyed = 0;
        for (int32_t i = 0; i < n; i++)
            done[i] = M[i] < h0;
        printf("%s:", mode ? "run keys" : "doubling");
        for (int t = 1; t < 40; t++) {
            const long d = h0 << (t - 1);
            long list = 0;
            for (int32_t i = 0; i < n; i++) {
                if (done[i])
                    continue;
                list++;
                const long reach = mode && A[i] >= d ? A[i] + d : 2 * d;
                runkeyed += mode && A[i] >= d;
                if (M[i] < reach)
                    done[i] = 1;
            }
            if (!list)
                break;
            total += list;
            printf(" %ld", list);
        }
        printf("  | rounds' lists %ld (%.2f n), run-keyed entries %ld\n", total, (double)total / n, runkeyed);
    }
    return 0;
}
