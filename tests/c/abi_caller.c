/*
 * abi_caller.c - a plain C caller of the drop-in library, built against include/salz.h alone
 * (no salz_gpu.h, no HIP headers) with the reference's warning flags (CMakeLists.txt:14).
 * It exercises the API exactly as an embedding program of the reference would
 * (salz_encoded_len_max -> salz_encode_safe -> salz_decode_safe):
 *
 *   abi_caller <in> <out>   encode file <in> as one block into <out>; if the stream fits the
 *                           24-bit header (lib/salz.c:760-772) decode it back and compare
 *   abi_caller --errors     the reference's error conventions (lib/salz.c:777-823)
 *
 * Prints one line "ok <in bytes> <out bytes> <encode ns>" and exits 0, or exits 1.
 * The common.h surface (min, roundup, unused, get_time_ns) comes through salz.h, as it does
 * for programs/salzcli.c.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "salz.h"

static int fail(const char *what)
{
    fprintf(stderr, "abi_caller: %s\n", what);
    return 1;
}

static int check_errors(void)
{
    uint8_t src[64], dst[256];
    size_t len;
    memset(src, 'a', sizeof(src));
    /* NULL buffers (lib/salz.c:783-786) */
    len = sizeof(dst);
    if (salz_encode_safe(NULL, sizeof(src), dst, &len) != -1 ||
        salz_encode_safe(src, sizeof(src), NULL, &len) != -1 ||
        salz_encode_safe(src, sizeof(src), dst, NULL) != -1)
        return fail("NULL argument accepted");
    /* blocks of <= 8 bytes: the reference fails (or crashes at 8, lib/salz.c:197, :622) */
    for (size_t n = 0; n <= 8; n++) {
        len = sizeof(dst);
        if (salz_encode_safe(src, n, dst, &len) != -1 || len != sizeof(dst))
            return fail("short block accepted");
    }
    /* success, then a capacity one byte short: -1 and *dst_len untouched (lib/salz.c:818) */
    len = sizeof(dst);
    if (salz_encode_safe(src, sizeof(src), dst, &len) != 0)
        return fail("64-byte block failed");
    const size_t need = len;
    len = need - 1;
    if (salz_encode_safe(src, sizeof(src), dst, &len) != -1 || len != need - 1)
        return fail("short destination accepted");
    uint8_t back[64];
    size_t blen = sizeof(back);
    if (salz_decode_safe(dst, need, back, &blen) != 0 || blen != sizeof(src) ||
        memcmp(back, src, sizeof(src)) != 0)
        return fail("round trip of the 64-byte block");
    blen = sizeof(src) - 1;
    if (salz_decode_safe(dst, need, back, &blen) != -1)
        return fail("decode into a short buffer accepted");
    printf("ok errors %zu\n", need);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc == 2 && strcmp(argv[1], "--errors") == 0)
        return check_errors();
    if (argc != 3)
        return fail("usage: abi_caller <in> <out> | --errors");
    FILE *f = fopen(argv[1], "rb");
    if (!f)
        return fail("cannot open input");
    fseek(f, 0, SEEK_END);
    const long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *src = malloc(sz > 0 ? (size_t)sz : 1);
    if (!src || fread(src, 1, (size_t)sz, f) != (size_t)sz)
        return fail("cannot read input");
    fclose(f);

    const size_t n = (size_t)sz;
    size_t cap = (size_t)salz_encoded_len_max(n);
    uint8_t *dst = malloc(roundup(cap, 64));
    if (!dst)
        return fail("out of memory");
    size_t len = cap;
    uint64_t t0 = 0, t1 = 0;
    get_time_ns(&t0);
    if (salz_encode_safe(src, n, dst, &len) != 0)
        return fail("salz_encode_safe failed");
    get_time_ns(&t1);
    f = fopen(argv[2], "wb");
    if (!f || fwrite(dst, 1, len, f) != len || fclose(f) != 0)
        return fail("cannot write output");

    /* the reference decoder only accepts streams whose length fits the 24-bit field */
    if (len - 4 <= 0xffffffu) {
        uint8_t *back = malloc(n + 8);
        size_t blen = n + 8;
        if (!back || salz_decode_safe(dst, len, back, &blen) != 0 || blen != n ||
            memcmp(back, src, n) != 0)
            return fail("round trip failed");
        free(back);
    }
    printf("ok %zu %zu %llu\n", n, len, (unsigned long long)(t1 - t0));
    unused(min(0, 1));
    free(src);
    free(dst);
    return 0;
}
