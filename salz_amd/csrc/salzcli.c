/*
 * salzcli.c - gzip-like command line harness over libsalz.so.
 *
 * Mirrors /root/reference/programs/salzcli.c: levels -0..-9 select a block size of
 * 1 << (15 + level) (:109, default level 5 = 1 MiB), -d decompresses, -f overwrites, -k keeps
 * the input, -q quiets; the ".salz" container is byte-identical ("ZLAS", u32 block size, then
 * u32 length + stream per block, :115-169). Files stream through the library with bounded
 * host memory: blocks are encoded across GPUs by salz_encode_stream (--gpus N, default all),
 * with reads, transfers, encodes and writes overlapped, and decoded across host threads by
 * salz_decode_stream.
 */
#include "../../include/salz.h"
#include "../../include/salz_gpu.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static int level = 5, decompress_mode = 0, force = 0, keep = 0, verbosity = 1, gpus = 0;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

static long long file_read(void *user, uint8_t *buf, size_t cap)
{
    FILE *f = user;
    size_t n = fread(buf, 1, cap, f);
    if (n == 0 && ferror(f))
        return -1;
    return (long long)n;
}

static int file_write(void *user, const uint8_t *buf, size_t len)
{
    return fwrite(buf, 1, len, (FILE *)user) == len ? 0 : -1;
}

/* Streams the file through the library: read -> H2D -> encode -> D2H -> write, block by
 * block with bounded host memory (salz_encode_stream / salz_decode_stream), like the
 * reference's fread / salz_encode_safe / fwrite loop (programs/salzcli.c:143-179). */
static int process(const char *path)
{
    char out_path[4096];
    if (!decompress_mode) {
        snprintf(out_path, sizeof(out_path), "%s.salz", path);
    } else {
        size_t L = strlen(path);
        if (L < 6 || strcmp(path + L - 5, ".salz") != 0) {
            fprintf(stderr, "salz: %s: unknown suffix\n", path);
            return -1;
        }
        snprintf(out_path, sizeof(out_path), "%.*s", (int)(L - 5), path);
    }
    FILE *in = fopen(path, "rb");
    if (!in) {
        fprintf(stderr, "salz: cannot read %s\n", path);
        return -1;
    }
    if (!force && access(out_path, F_OK) == 0) {
        fprintf(stderr, "salz: %s already exists (use -f)\n", out_path);
        fclose(in);
        return -1;
    }
    FILE *out = fopen(out_path, "wb");
    if (!out) {
        fprintf(stderr, "salz: cannot write %s\n", out_path);
        fclose(in);
        return -1;
    }
    double t0 = now_s();
    uint64_t nin = 0, nout = 0;
    int rc;
    if (!decompress_mode)
        rc = salz_encode_stream(file_read, in, file_write, out, (size_t)1 << (15 + level), gpus, &nin, &nout);
    else
        rc = salz_decode_stream(file_read, in, file_write, out, 0, &nin, &nout);
    fclose(in);
    if (fclose(out) != 0)
        rc = -1;
    double dt = now_s() - t0;
    if (rc != 0) {
        unlink(out_path); /* programs/salzcli.c:350-353 */
        fprintf(stderr, "salz: %s: %s\n", path, decompress_mode ? "decode failed" : salz_gpu_last_error());
        return rc;
    }
    if (verbosity > 0)
        printf("%s %llu bytes to %llu bytes (%.3f) in %.3f seconds\n",
               decompress_mode ? "decompressed" : "compressed", (unsigned long long)nin,
               (unsigned long long)nout, nout ? (double)nin / (double)nout : 0.0, dt);
    if (!keep)
        unlink(path);
    return 0;
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
