/*
 * salz_gpu.h - MI355X extensions of the SA-LZ C ABI (libsalz.so).
 *
 * Additive to the reference API (salz.h): explicit device contexts, device-resident
 * encode for callers that already hold blocks in HBM, batched multi-block / multi-GPU
 * encode for the CLI's block loop (programs/salzcli.c:143-179), a frame-aware decoder for
 * streams longer than the 24-bit header can describe, per-stage
 * statistics, and a stage-dump hook used by the parity tests.
 *
 * Plain C types only; `stream` arguments are hipStream_t passed as void*.
 */
#ifndef SALZ_GPU_H
#define SALZ_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct salz_gpu_ctx salz_gpu_ctx;

/* Number of visible HIP devices; 0 when no GPU is usable. */
int salz_gpu_device_count(void);

/* log2 of the parse chunk length chosen for a block of block_len bytes (host-only helper;
 * no device call; SALZ_PARSE_KLOG overrides it for tests). */
uint32_t salz_gpu_parse_chunk_log(size_t block_len);

/* Message of the last failure on this thread ("" if none). */
const char *salz_gpu_last_error(void);

/* Device memory helpers (so callers need no second HIP runtime in their process). */
void *salz_gpu_malloc(int device, size_t bytes);
void salz_gpu_free(int device, void *ptr);
int salz_gpu_memcpy_h2d(int device, void *dst, const void *src, size_t bytes);
int salz_gpu_memcpy_d2h(int device, void *dst, const void *src, size_t bytes);
int salz_gpu_synchronize(int device);

/* Context on `device` with device workspace for blocks of up to max_block bytes
 * (about 90 bytes of HBM per block byte). NULL on failure. */
salz_gpu_ctx *salz_gpu_ctx_create(int device, size_t max_block);
void salz_gpu_ctx_destroy(salz_gpu_ctx *ctx);

/*
 * Encode one block already resident in device memory. d_src holds src_len bytes, d_dst has
 * dst_cap bytes; *dst_len receives the stream length (bit-identical to salz_encode_safe).
 * `stream` (hipStream_t or NULL for the context's own) orders the call; the function
 * returns after the stream has drained. Returns 0 / -1 like salz_encode_safe.
 */
int salz_gpu_encode_device(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t src_len,
                           uint8_t *d_dst, size_t dst_cap, size_t *dst_len, void *stream);

/* salz_encode_safe on an explicit context (host buffers). */
int salz_gpu_encode_host(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, uint8_t *dst,
                         size_t *dst_len);

/* Intermediate arrays of one encode (n = src_len - 8 entries; cost has n + 1).
 * Any member may be NULL. Layout and meaning: oracle/salz_oracle.h (oracle_stages). */
typedef struct {
    int32_t *sa, *psv, *nsv, *lp, *ln, *dlen, *doff, *cost;
} salz_gpu_dump;

int salz_gpu_encode_dump(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, uint8_t *dst,
                         size_t *dst_len, const salz_gpu_dump *dump);

/*
 * A batch: src_len bytes as consecutive blocks of block_size bytes (the last may be shorter),
 * all encoded in ONE pass of the pipeline (the suffix array of every block, candidates, parse
 * and emission run over the whole batch, each block independent and bit-identical to
 * salz_encode_safe on that block). dst receives the packed frames: per block a u32 LE stream
 * length then the stream, in block order (the body of the CLI container). *dst_len: [in]
 * capacity, [out] bytes. Needs block_size % 512 == 0 when there is more than one block, at
 * most 4096 blocks, and every block longer than 8 bytes. Returns 0 / -1.
 */
int salz_gpu_encode_batch(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, size_t block_size,
                          uint8_t *dst, size_t *dst_len);

/* salz_gpu_encode_batch for a batch already in device memory: the packed frames go to device
 * buffer d_dst (dst_cap bytes); `stream` as for salz_gpu_encode_device. Returns 0 / -1. */
int salz_gpu_encode_batch_device(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t src_len,
                                 size_t block_size, uint8_t *d_dst, size_t dst_cap, size_t *dst_len,
                                 void *stream);

/* ---- one block's suffix array split over several GPUs -------------------
 * Every rank holds the whole block in its HBM. The suffixes are bucketed by their first two
 * bytes (contiguous ranges of the 65536 classes, about N / nranks suffixes each, the same plan on
 * every rank), and each rank prefix-doubles its own bucket with the single-GPU kernels. The only
 * exchange is rank[i + h] for suffixes i + h of other buckets, once per doubling round: requests
 * and answers go through the caller's all-to-all over fixed device buffers (RCCL over xGMI, or
 * gloo with host staging in the tests); an allreduce tells when every bucket is sorted. The
 * pieces are SA[offsets[r] .. offsets[r + 1]) of the block's suffix array, with their LCPs. */
typedef struct salz_dist_ops {
    void *user;
    /* All-to-all of u32 words from xsend to xrecv (the buffers given below): send_counts[d]
     * words for rank d, packed in rank order; fill recv_counts[s] (packed in rank order in
     * xrecv). The library has finished writing xsend when it calls; the data must be in xrecv
     * when this returns. Return 0 on success. */
    int (*alltoall)(void *user, const uint64_t *send_counts, uint64_t *recv_counts);
    /* Sum of *value over the ranks, into *value. Return 0 on success. */
    int (*allreduce_sum)(void *user, uint64_t *value);
} salz_dist_ops;

/* This rank's piece of the suffix array of the block d_text[0, N) (device memory, N - 8
 * suffixes as salz_encode_safe sorts them). xsend / xrecv: device buffers of xcap u32 words
 * (N words always suffice). d_sa_piece / d_lcp_piece: device buffers of N words; they receive
 * this rank's SA range and the LCP of each entry with its predecessor (entry 0 of a piece is
 * left for the caller to fix, see salz_gpu_encode_from_sa). offsets: nranks + 1 values.
 * *lcp_ok = 0 when the LCPs were not kept (very long repeats: the PLCP stage recomputes them).
 * Collective: every rank calls it with the same block. Returns 0 / -1, or 1 on every rank when
 * the block is not split: blocks of 2^20 suffixes or more that the repetition probe sends to DC3
 * (long repeats everywhere), which the split sorter does not run; encode those whole on one GPU
 * (salz_gpu_encode_device). */
int salz_gpu_dist_suffix_array(salz_gpu_ctx *ctx, const uint8_t *d_text, size_t N, int nranks, int rank,
                               const salz_dist_ops *ops, uint32_t *d_xsend, uint32_t *d_xrecv,
                               size_t xcap, uint32_t *d_sa_piece, uint32_t *d_lcp_piece,
                               uint64_t *offsets, int *lcp_ok);

/* The same with the collectives inside the library: RCCL over xGMI on the context's own stream
 * (no host callback per round; librccl.so.1 is opened at run time). One communicator per rank:
 * salz_gpu_dist_comm_id on one rank gives the 128-byte id that every rank passes, with its rank,
 * to salz_gpu_dist_comm_create (collective: it returns once every rank has joined). The
 * communicator's device must be the context's. */
typedef struct salz_gpu_dist_comm salz_gpu_dist_comm;
int salz_gpu_dist_comm_id(uint8_t *id128);
salz_gpu_dist_comm *salz_gpu_dist_comm_create(int device, int nranks, int rank, const uint8_t *id128);
void salz_gpu_dist_comm_destroy(salz_gpu_dist_comm *comm);
int salz_gpu_dist_suffix_array_comm(salz_gpu_ctx *ctx, const uint8_t *d_text, size_t N, salz_gpu_dist_comm *comm,
                                    uint32_t *d_xsend, uint32_t *d_xrecv, size_t xcap, uint32_t *d_sa_piece,
                                    uint32_t *d_lcp_piece, uint64_t *offsets, int *lcp_ok);

/* Encode one block from its suffix array (device memory, N - 8 entries, e.g. gathered from the
 * pieces above) and, when d_lcp is not NULL, its LCP array: the LCPs at the nfix positions in
 * lcp_fix (a piece's first entry) are recomputed from the text. The stream goes to device buffer
 * d_dst (capacity dst_cap); *dst_len its length. Returns 0 / -1. */
int salz_gpu_encode_from_sa(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t N, const uint32_t *d_sa,
                            const uint32_t *d_lcp, const uint64_t *lcp_fix, size_t nfix, uint8_t *d_dst,
                            size_t dst_cap, size_t *dst_len);

typedef struct {
    double ms_upload, ms_sa, ms_lcp, ms_ansv, ms_parse, ms_emit, ms_total;
    int32_t sa_rounds, parse_iters;
    uint64_t sa_sorted_elems, lcp_long_bytes, emit_bits, emit_bytes;
    uint32_t exit_nodes;
    uint32_t radix_scatter_launches;
    double ms_radix_scatter;
    uint64_t radix_scatter_elems;
    int32_t sa_dc3_levels; /* > 0: the suffix array came from the DC3 sorter (repetitive block) */
    uint64_t radix_scatter_bytes; /* algorithmic bytes of the timed scatter launches (24 per element,
                                     + 1 where the next pass's digit byte is written) */
} salz_gpu_stats;

/*
 * The context pool behind salz_encode_safe (the reference keeps no state between calls,
 * lib/salz.c:175-256; here workspaces are cached for the next call). slots_per_device: contexts
 * per device (1..8; default SALZ_SAFE_SLOTS or 4); cache_bytes: device memory idle cached
 * workspaces may hold per device before the largest are released after a call (default
 * SALZ_SAFE_CACHE_BYTES or 32 GiB); any_device: 1 lets a caller borrow contexts of other
 * devices when its own are busy, 0 keeps every call on the caller's current device (default).
 * A value <= 0 (< 0 for any_device) leaves that setting unchanged.
 */
void salz_gpu_pool_config(int slots_per_device, size_t cache_bytes, int any_device);
/* Device memory held by the pool's workspaces on `device`. */
size_t salz_gpu_pool_bytes(int device);
/* Device workspaces allocated by this process so far (every context, every device): a pool whose
   workspaces are reused across calls keeps this flat. */
size_t salz_gpu_workspace_allocs(void);

/* Per-stage HIP-event timing of subsequent calls (small overhead when on). */
void salz_gpu_set_timing(salz_gpu_ctx *ctx, int on);
int salz_gpu_get_stats(const salz_gpu_ctx *ctx, salz_gpu_stats *out);

/*
 * Encode src as consecutive blocks of block_size bytes (the last may be shorter), spreading
 * blocks over `n_devices` GPUs (<= 0: all visible) with one host thread per device pulling
 * block indices from a shared counter. Output is the reference CLI container
 * (programs/salzcli.c:102-185): "ZLAS" magic, u32 block size, then per block u32 length +
 * stream, in block order. *dst_len: [in] capacity, [out] bytes written.
 * Returns 0 / -1.
 */
int salz_encode_blocks(const uint8_t *src, size_t src_len, size_t block_size, uint8_t *dst,
                       size_t *dst_len, int n_devices);

/*
 * Streaming form of salz_encode_blocks for inputs of any size (the CLI pipeline,
 * programs/salzcli.c:102-185): blocks are pulled through `rd` (fread-like: returns bytes read,
 * 0 at end of input, < 0 on error), encoded on the GPUs with reads, transfers, encodes and
 * writes overlapped, and the container is pushed through `wr` (0 on success) in block order.
 * Host memory is bounded by a ring of (encoder slots + 2) pinned block buffers. As in the
 * reference loop, the trailing short (possibly empty) block is always encoded, so inputs whose
 * size mod block_size is in [0, 8] fail. *in_total / *out_total (may be NULL) receive the
 * byte counts. Returns 0 / -1.
 */
typedef long long (*salz_read_fn)(void *user, uint8_t *buf, size_t cap);
typedef int (*salz_write_fn)(void *user, const uint8_t *buf, size_t len);
int salz_encode_stream(salz_read_fn rd, void *rd_user, salz_write_fn wr, void *wr_user,
                       size_t block_size, int n_devices, uint64_t *in_total, uint64_t *out_total);

/* Upper bound of salz_encode_blocks output for (src_len, block_size). */
size_t salz_blocks_len_max(size_t src_len, size_t block_size);

/*
 * Decode one stream whose true length is frame_len (the container's u32 length field).
 * Identical to salz_decode_safe except that when the 24-bit header length equals
 * (frame_len - 4) mod 2^24 the frame length is used, so streams longer than 16 MiB - 1
 * (whose header field the reference truncates, lib/salz.c:770) decode. Returns 0 / -1.
 */
int salz_decode_frame(const uint8_t *src, size_t frame_len, uint8_t *dst, size_t *dst_len);

/* Decode a salz_encode_blocks / salzcli container with `threads` host threads
 * (<= 0: one per core). *dst_len: [in] capacity, [out] bytes. Returns 0 / -1. */
int salz_decode_blocks(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len,
                       int threads);

/* Streaming container decode (host threads): frames are pulled through `rd`, decoded `threads`
 * at a time (<= 0: one per core, at most 8; at most 32) and the plain bytes pushed through `wr` in order.
 * Host memory: threads x (block + encoded_len_max(block)). Returns 0 / -1. */
int salz_decode_stream(salz_read_fn rd, void *rd_user, salz_write_fn wr, void *wr_user, int threads,
                       uint64_t *in_total, uint64_t *out_total);

#ifdef __cplusplus
}
#endif

#endif /* SALZ_GPU_H */
