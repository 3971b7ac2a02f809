/*
 * common.h - helper macros and the monotonic timer that the reference header pulls into
 * every includer of salz.h (/root/reference/include/common.h:19-38, included from
 * lib/salz.h:16). Callers such as programs/salzcli.c use min() (:491), get_time_ns()
 * (:331, :344) and roundup() through it, so the drop-in ships the same surface:
 *
 *   min(a, b)        smaller of two values (macro, arguments evaluated twice)
 *   divup(a, b)      ceiling division
 *   roundup(a, b)    a rounded up to a multiple of b
 *   unlikely(x)      branch hint
 *   unused(x)        silence an unused-variable warning
 *   get_time_ns(&t)  CLOCK_MONOTONIC in nanoseconds; 0 or errno
 */
#ifndef SALZ_COMMON_H
#define SALZ_COMMON_H

#include <errno.h>
#include <stdint.h>
#include <time.h>

#ifndef min
#define min(a, b) (((a) < (b)) ? (a) : (b))
#endif
#define divup(a, b) (((a) + (b) - 1) / (b))
#define roundup(a, b) (divup((a), (b)) * (b))

#define unlikely(x) __builtin_expect((x), 0)

#define unused(x) ((void)(x))

#define NS_IN_SEC (1000 * 1000 * 1000)

static inline int get_time_ns(uint64_t *res)
{
    struct timespec now;

    if (clock_gettime(CLOCK_MONOTONIC, &now) != 0)
        return errno;
    *res = (uint64_t)now.tv_sec * NS_IN_SEC + (uint64_t)now.tv_nsec;
    return 0;
}

#endif /* SALZ_COMMON_H */
