/*
 * salz.h - drop-in public API of the MI355X SA-LZ codec.
 *
 * Same declarations, argument meaning and error behaviour as the reference header
 * /root/reference/lib/salz.h (akiutoslahti/salz), so existing callers recompile unchanged:
 *   salz_encoded_len_max  <- lib/salz.h:25-28 (header-only inline, identical formula)
 *   salz_encode_safe      <- lib/salz.h:42-43, lib/salz.c:777-823
 *   salz_decode_safe      <- lib/salz.h:57-58, lib/salz.c:1194-1228
 *   encode_vnibble_le     <- lib/salz.c:352   (exported, undeclared in the reference header)
 *   vnibble_size          <- lib/salz.c:565   (exported, undeclared in the reference header)
 *
 * Encoding runs on an MI355X (gfx950) through libsalz.so; output bytes are identical to
 * the reference encoder's. With no usable GPU, salz_encode_safe fails (-1) and reports why
 * on stderr and in salz_gpu_last_error() (salz_gpu.h); there is no silent CPU fallback.
 * Decoding is host C.
 *
 * Like the reference (lib/salz.h:16), this header includes common.h, so includers get its
 * min/divup/roundup/unlikely/unused/get_time_ns. Code that cannot take a function-like `min`
 * macro (C++ translation units of the library itself) defines SALZ_NO_COMMON_H first.
 */
#ifndef SALZ_H
#define SALZ_H

#include <stddef.h>
#include <stdint.h>

#ifndef SALZ_NO_COMMON_H
#include "common.h"
#endif

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Worst case length of an encoded segment: header + plain bytes + one control word per
 * 64 bytes (lib/salz.h:25-28).
 */
static inline int salz_encoded_len_max(size_t plain_len)
{
    return (int)(4 + plain_len + ((plain_len + 63) / 64 * 64) / 8);
}

/*
 * Encode plain segment with SALZ.
 *   src, src_len   plain segment (src_len > 8; the reference fails for shorter blocks)
 *   dst            preallocated output
 *   dst_len        [in] capacity of dst, [out] encoded length (set only on success)
 * Returns 0 on success, -1 otherwise (NULL buffers, capacity, device failure).
 */
int salz_encode_safe(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len);

/*
 * Decode SALZ encoded segment.
 *   src, src_len   encoded segment
 *   dst            preallocated output
 *   dst_len        [in] capacity of dst, [out] decoded length (set only on success)
 * Returns 0 on success, -1 otherwise.
 */
int salz_decode_safe(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len);

/* Variable-nibble helpers exported by the reference library (lib/salz.c:352, :565). */
size_t encode_vnibble_le(uint32_t val, uint64_t *res);
size_t vnibble_size(uint32_t val);

#ifdef __cplusplus
}
#endif

#endif /* SALZ_H */
