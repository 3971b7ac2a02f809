/*
 * salzcli.c - gzip-like command line harness over libsalz.so.
 *
 * Mirrors /root/reference/programs/salzcli.c: levels -0..-9 select a block size of
 * 1 << (15 + level) (:109, default level 5 = 1 MiB), -d decompresses, -f overwrites, -k keeps
 * the input, -q quiets; the ".salz" container is byte-identical ("ZLAS", u32 block size, then
 * u32 length + stream per block, :115-169). Blocks are encoded across GPUs by
 * salz_encode_blocks (--gpus N, default all) and decoded across host threads.
 */
#include "../../include/salz.h"
#include "../../include/salz_gpu.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

static int level = 5, decompress_mode = 0, force = 0, keep = 0, verbosity = 1, gpus = 0;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

static uint8_t *read_all(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    struct stat st;
    if (fstat(fileno(f), &st) != 0) {
        fclose(f);
        return NULL;
    }
    size_t n = (size_t)st.st_size;
    uint8_t *buf = malloc(n ? n : 1);
    if (buf && n && fread(buf, 1, n, f) != n) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    *len = n;
    return buf;
}

static int write_all(const char *path, const uint8_t *buf, size_t len)
{
    if (!force && access(path, F_OK) == 0) {
        fprintf(stderr, "salz: %s already exists (use -f)\n", path);
        return -1;
    }
    FILE *f = fopen(path, "wb");
    if (!f)
        return -1;
    int ok = fwrite(buf, 1, len, f) == len;
    ok &= fclose(f) == 0;
    if (!ok)
        unlink(path);
    return ok ? 0 : -1;
}

static int process(const char *path)
{
    size_t in_len = 0;
    uint8_t *in = read_all(path, &in_len);
    if (!in) {
        fprintf(stderr, "salz: cannot read %s\n", path);
        return -1;
    }
    double t0 = now_s();
    char out_path[4096];
    uint8_t *out = NULL;
    size_t out_len = 0;
    int rc;
    if (!decompress_mode) {
        size_t bs = (size_t)1 << (15 + level);
        out_len = salz_blocks_len_max(in_len, bs);
        out = malloc(out_len);
        rc = out ? salz_encode_blocks(in, in_len, bs, out, &out_len, gpus) : -1;
        snprintf(out_path, sizeof(out_path), "%s.salz", path);
    } else {
        size_t L = strlen(path);
        if (L < 6 || strcmp(path + L - 5, ".salz") != 0) {
            fprintf(stderr, "salz: %s: unknown suffix\n", path);
            free(in);
            return -1;
        }
        snprintf(out_path, sizeof(out_path), "%.*s", (int)(L - 5), path);
        /* the container does not record the plain size: bound it by blocks x block size */
        uint32_t bs = 0;
        if (in_len >= 8)
            memcpy(&bs, in + 4, 4);
        size_t blocks = 0, pos = 8;
        while (pos + 4 <= in_len) {
            uint32_t fl;
            memcpy(&fl, in + pos, 4);
            pos += 4 + fl;
            blocks++;
        }
        out_len = blocks * (size_t)bs;
        out = malloc(out_len ? out_len : 1);
        rc = out ? salz_decode_blocks(in, in_len, out, &out_len, 0) : -1;
    }
    if (rc == 0)
        rc = write_all(out_path, out, out_len);
    double dt = now_s() - t0;
    if (rc == 0 && verbosity > 0)
        printf("%s %zu bytes to %zu bytes (%.3f) in %.3f seconds\n",
               decompress_mode ? "decompressed" : "compressed", in_len, out_len,
               out_len ? (double)in_len / (double)out_len : 0.0, dt);
    if (rc != 0)
        fprintf(stderr, "salz: %s: %s\n", path, decompress_mode ? "decode failed" : salz_gpu_last_error());
    if (rc == 0 && !keep)
        unlink(path);
    free(in);
    free(out);
    return rc;
}

int main(int argc, char **argv)
{
    int files = 0, failed = 0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (a[0] == '-' && a[1] >= '0' && a[1] <= '9' && a[2] == 0)
            level = a[1] - '0';
        else if (!strcmp(a, "-d"))
            decompress_mode = 1;
        else if (!strcmp(a, "-f"))
            force = 1;
        else if (!strcmp(a, "-k"))
            keep = 1;
        else if (!strcmp(a, "-q"))
            verbosity--;
        else if (!strcmp(a, "--gpus") && i + 1 < argc)
            gpus = atoi(argv[++i]);
        else if (a[0] == '-') {
            fprintf(stderr, "usage: salz [-0..-9] [-d] [-f] [-k] [-q] [--gpus N] file...\n");
            return 1;
        } else {
            files++;
            failed |= process(a) != 0;
        }
    }
    if (!files) {
        fprintf(stderr, "usage: salz [-0..-9] [-d] [-f] [-k] [-q] [--gpus N] file...\n");
        return 1;
    }
    return failed;
}
