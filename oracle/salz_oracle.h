/*
 * salz_oracle.h - CPU restatement of the reference SA-LZ codec (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X build. It is a clean-room, sequential C
 * restatement of /root/reference/lib/salz.c (akiutoslahti/salz @ v1), with its own
 * SA-IS standing in for the un-vendored libsais dependency (the suffix array of a text
 * is unique, so any correct SACA yields identical output bytes).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline. The product (salz_amd/libsalz.so)
 * never links or calls it.
 *
 * Pinning: the restatement reproduces the golden hashes of SURVEY.md Appendix C, which
 * were produced by the unmodified reference lib/salz.c in the survey container
 * (tests/golden/appendix_c.json, tests/test_oracle.py).
 */
#ifndef SALZ_ORACLE_H
#define SALZ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Suffix array of T[0,n) (no sentinel; a suffix sorts before every longer suffix it
 * prefixes). Replaces libsais() at lib/salz.c:465. Returns 0 on success. */
int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);

/* Whole-block encoder, lib/salz.c:777-823. Same contract as salz_encode_safe. */
int oracle_encode(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len);

/* Whole-block decoder, lib/salz.c:1194-1228. Same contract as salz_decode_safe. */
int oracle_decode(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len);

/*
 * Stage dump for per-stage GPU parity (n = src_len - 8 entries each, cost has n + 1):
 *   sa[r]          suffix array (lib/salz.c:463-469)
 *   psv[p], nsv[p] nearest rank before/after with smaller position, -1 if none (:471-490)
 *   lp[p], ln[p]   factor lengths against psv / nsv (:492-560)
 *   dlen[p]        chosen length (1 = literal) (:610-662); dlen[0] = 1
 *   doff[p]        chosen offset (0 for literals)
 *   cost[p]        optimal suffix cost in bits, cost[n] = 0
 * Any pointer may be NULL. Returns 0, or -1 for src_len <= 8 / allocation failure.
 */
int oracle_stages(const uint8_t *src, size_t src_len, int32_t *sa, int32_t *psv,
                  int32_t *nsv, int32_t *lp, int32_t *ln, int32_t *dlen, int32_t *doff,
                  int32_t *cost);

/* Literal restatement of the reference's exported vnibble helpers (lib/salz.c:352-445,
 * :565-588), used to cross-check the closed-form encoder in the product. */
size_t oracle_encode_vnibble_le(uint32_t val, uint64_t *res);
size_t oracle_vnibble_size(uint32_t val);

#ifdef __cplusplus
}
#endif

#endif /* SALZ_ORACLE_H */
