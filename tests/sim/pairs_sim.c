/*
 * pairs_sim.c - prefix doubling (salz_amd/csrc/gpu/sa.hip) on a text repeated once at distance
 * d = N / 2 ("halves"), with and without resolving two-member groups {i, i + d} directly (their
 * order and LCP from the first mismatch on diagonal d). Test infrastructure / measurement aid for
 * it uses the CPU oracle's suffix array (oracle/liboracle.so) for each suffix's LCPs
 * with its SA neighbours.
 *
 *   gcc -O2 -o /tmp/pairs_sim tests/sim/pairs_sim.c -Loracle -loracle -Ltools -ldatagen \
 *       -Wl,-rpath,$PWD/oracle:$PWD/tools
 *   /tmp/pairs_sim 33554432        # halves of N bytes, and the plain text of N bytes
 *
 * Model: suffix i leaves the list after the round whose depth exceeds M[i], the larger LCP with
 * its SA neighbours; with pair resolution, a suffix whose twin (i +- d) is an SA neighbour leaves
 * once the depth exceeds the pair's outer LCPs instead. Depths 9, 18, 36, ... (h0 << t).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);
void datagen_text(uint8_t *out, size_t n, uint64_t seed);

static void rounds(const char *name, const int32_t *M, int32_t n)
{
    long total = 0;
    printf("%s:", name);
    for (int t = 0; t < 40; t++) {
        const long dp = t ? 9l << (t - 1) : -1, list_min = dp;
        long list = 0;
        for (int32_t i = 0; i < n; i++)
            list += M[i] >= list_min;
        if (!list)
            break;
        total += list;
        printf(" %ld", list);
    }
    printf("  | total %ld (%.2f n)\n", total, (double)total / n);
}

static void run(uint8_t *T, int32_t n, int32_t d, const char *name)
{
    int32_t *SA = malloc(4 * (size_t)n), *R = malloc(4 * (size_t)n), *L = malloc(4 * ((size_t)n + 2));
    int32_t *M = malloc(4 * (size_t)n), *P = malloc(4 * (size_t)n);
    if (!SA || !R || !L || !M || !P || oracle_suffix_array(T, SA, n) != 0)
        exit(1);
    for (int32_t r = 0; r < n; r++)
        R[SA[r]] = r;
    int32_t h = 0;  // Kasai: L[r] = LCP(SA[r - 1], SA[r])
    L[0] = 0;
    L[n] = 0;
    L[n + 1] = 0;
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
    long adj = 0;
    for (int32_t r = 0; r < n; r++) {
        const int32_t a = L[r], b = L[r + 1];
        M[SA[r]] = a > b ? a : b;
        P[SA[r]] = M[SA[r]];
    }
    if (d > 0)
        for (int32_t r = 0; r + 1 < n; r++) {  // SA neighbours at distance d: a pair
            const int32_t x = SA[r], y = SA[r + 1];
            if (x - y != d && y - x != d)
                continue;
            adj++;
            const int32_t outer = L[r] > L[r + 2] ? L[r] : L[r + 2];
            if (outer < P[x])
                P[x] = outer;
            if (outer < P[y])
                P[y] = outer;
        }
    rounds(name, M, n);
    if (d > 0) {
        printf("  adjacent twins: %ld pairs (%.1f%% of suffixes)\n", adj, 200.0 * adj / n);
        rounds("  with pairs", P, n);
    }
    free(SA); free(R); free(L); free(M); free(P);
}

int main(int argc, char **argv)
{
    const size_t N = argc > 1 ? (size_t)atol(argv[1]) : 33554432;
    uint8_t *T = calloc(N + 64, 1);
    if (!T)
        return 1;
    datagen_text(T, N, 1);
    run(T, (int32_t)(N - 8), 0, "text");
    datagen_text(T, N / 2, 11);
    memcpy(T + N / 2, T, N - N / 2);
    run(T, (int32_t)(N - 8), (int32_t)(N / 2), "halves");
    return 0;
}
