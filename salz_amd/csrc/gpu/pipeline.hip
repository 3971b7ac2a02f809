// pipeline.hip - device contexts, stage orchestration and the extern "C" ABI of libsalz.so.
//
// salz_encode_safe (/root/reference/lib/salz.c:777-823) becomes:
//   H2D (or D2D) of the block into a padded HBM copy
//   -> stage_suffix_array (sa.hip)     replaces libsais, :463-469
//   -> stage_lcp          (lcp.hip)    exact LCP array (feeds the candidate lengths)
//   -> stage_candidates   (ansv.hip)   :471-560
//   -> stage_parse        (parse.hip)  :610-662
//   -> stage_emit         (emit.hip)   :664-775
//   -> D2H of the encoded stream.
// One Workspace per context, reused across calls; a mutex per context keeps the reference
// API's reentrancy (concurrent callers serialise per device).
#include "internal.hpp"
#define SALZ_NO_COMMON_H  // std headers below use min(); the C API does not need common.h here
#include "../../../include/salz.h"
#include "../../../include/salz_gpu.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace salz {

static thread_local char g_err[512];

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// value of `name` in the comma-separated list $var: "" for a bare name, nullptr if absent
static const char *env_find(const char *var, const char *name)
{
    const char *v = getenv(var);
    const size_t nl = strlen(name);
    for (const char *p = v; p && *p;) {
        const char *end = strchr(p, ',');
        const size_t len = end ? (size_t)(end - p) : strlen(p);
        if (len >= nl && !strncmp(p, name, nl) && (len == nl || p[nl] == '='))
            return len == nl ? "" : p + nl + 1;
        p = end ? end + 1 : nullptr;
    }
    return nullptr;
}

bool env_flag(const char *var, const char *name) { return env_find(var, name) != nullptr; }

long env_num(const char *var, const char *name, long dflt)
{
    const char *v = env_find(var, name);
    return !v ? dflt : *v ? strtol(v, nullptr, 0) : 1;
}

// SALZ_CHECK=guard (diagnostics): every workspace buffer gets a guard zone filled with a
// pattern; guard_check() reports the first buffer whose zone was written.
constexpr size_t kGuardBytes = 1 << 20;
struct Guard {
    const char *name;
    uint8_t *zone;
};
static thread_local std::vector<Guard> *g_guards = nullptr;
static bool guard_on() { static const bool on = env_flag("SALZ_CHECK", "guard"); return on; }

template <typename T> static int dalloc_named(T **p, size_t count, const char *name, size_t *held)
{
    void *q = nullptr;
    const size_t bytes = count * sizeof(T) + 256;
    *held += bytes;
    hipError_t e = hipMalloc(&q, bytes + (guard_on() ? kGuardBytes : 0));
    if (e != hipSuccess) {
        set_error("hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
        return -1;
    }
    if (guard_on()) {
        uint8_t *zone = static_cast<uint8_t *>(q) + bytes;
        (void)hipMemset(zone, 0xA5, kGuardBytes);
        if (!g_guards)
            g_guards = new std::vector<Guard>();
        g_guards->push_back({name, zone});
    }
    *p = static_cast<T *>(q);
    return 0;
}
#define dalloc(p, count) dalloc_named(p, count, #p, &held)

int guard_check(Workspace &ws, const char *stage)
{
    if (!guard_on() || !g_guards)
        return 0;
    (void)hipStreamSynchronize(ws.stream);
    std::vector<uint8_t> h(kGuardBytes);
    for (const Guard &g : *g_guards) {
        (void)hipMemcpy(h.data(), g.zone, kGuardBytes, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < kGuardBytes; i++)
            if (h[i] != 0xA5) {
                fprintf(stderr, "GUARD: %s overrun after %s at +%zu\n", g.name, stage, i);
                set_error("guard zone of %s written after %s", g.name, stage);
                return -1;
            }
    }
    return 0;
}

void workspace_free(Workspace &ws)
{
    if (ws.device >= 0)
        (void)hipSetDevice(ws.device);
    void *ptrs[] = {ws.text, ws.rank,     ws.sa,   ws.keyA, ws.keyB, ws.valA, ws.valB,
                    ws.u0,   ws.u1,       ws.u2,   ws.u3,   ws.g64,  ws.offA, ws.offB, ws.lcps,
                    ws.cand, ws.pst, ws.lsc, ws.lrec, ws.lg2g, ws.dc3, ws.dist_owner, ws.out, ws.radix_counts,  ws.scan_tmp,      ws.dscal};
    for (void *p : ptrs)
        if (p)
            (void)hipFree(p);
    if (ws.hscal)
        (void)hipHostFree(ws.hscal);
    for (hipEvent_t &e : ws.ev)
        if (e)
            (void)hipEventDestroy(e);
    for (hipEvent_t e : ws.rx_pool)
        (void)hipEventDestroy(e);
    if (ws.own_stream && ws.stream)
        (void)hipStreamDestroy(ws.stream);
    for (int b = 0; b < 2; b++) {
        if (ws.hstage[b])
            (void)hipHostFree(ws.hstage[b]);
        if (ws.hstage_ev[b])
            (void)hipEventDestroy(ws.hstage_ev[b]);
    }
    ws = Workspace{};
}

// Free every buffer but keep the device: the next encode reallocates (every path that takes a
// cached context grows its workspace on demand).
void workspace_release(Workspace &ws)
{
    const int dev = ws.device;
    workspace_free(ws);
    ws.device = dev;
}

// Whether a host buffer is pinned (registered or hipHostMalloc'ed) or device memory, so a
// copy can skip the staging.
static bool dma_ready(const void *p)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

static int stage_ready(Workspace &ws)
{
    for (int b = 0; b < 2; b++) {
        if (!ws.hstage[b]) {
            void *h = nullptr;
            SALZ_HIP(hipHostMalloc(&h, kStageChunk, hipHostMallocDefault));
            ws.hstage[b] = static_cast<uint8_t *>(h);
        }
        if (!ws.hstage_ev[b])
            SALZ_HIP(hipEventCreateWithFlags(&ws.hstage_ev[b], hipEventDisableTiming));
    }
    return 0;
}

constexpr size_t kRuntimeCopy = 16u << 20;

int copy_h2d(Workspace &ws, uint8_t *dst, const uint8_t *src, size_t bytes)
{
    if (bytes == 0)
        return 0;
    // Pageable copies of 16 MiB and more go through the runtime (ROCm 7.2: C2 from host buffers
    // 2950 -> 3190 MB/s, Silesia-sized blocks 2578 -> 2691, four salz_encode_safe threads on
    // 16 MiB blocks 3394 -> 3509; profiles/r04q_h2d_ab.txt); smaller ones (the batches of the
    // container encoders, several in flight) through the context's pinned chunks, which the
    // 512 KiB-block level sweep ran faster (1760 vs 1313 MB/s).
    if (bytes <= (64u << 10) || bytes >= kRuntimeCopy || dma_ready(src)) {
        SALZ_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ws.stream));
        return 0;
    }
    if (stage_ready(ws) != 0)
        return -1;
    for (size_t o = 0, k = 0; o < bytes; o += kStageChunk, k++) {
        const size_t len = bytes - o < kStageChunk ? bytes - o : kStageChunk;
        const int b = (int)(k & 1);
        // the DMA that last read this chunk, in this call or an earlier one (an event that was
        // never recorded, or has completed, returns at once)
        SALZ_HIP(hipEventSynchronize(ws.hstage_ev[b]));
        memcpy(ws.hstage[b], src + o, len);
        SALZ_HIP(hipMemcpyAsync(dst + o, ws.hstage[b], len, hipMemcpyHostToDevice, ws.stream));
        SALZ_HIP(hipEventRecord(ws.hstage_ev[b], ws.stream));
    }
    return 0;
}

int copy_d2h(Workspace &ws, uint8_t *dst, const uint8_t *src, size_t bytes)
{
    if (bytes == 0)
        return 0;
    if (bytes <= (64u << 10) || bytes >= kRuntimeCopy || dma_ready(dst)) {
        SALZ_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ws.stream));
        SALZ_HIP(hipStreamSynchronize(ws.stream));
        return 0;
    }
    if (stage_ready(ws) != 0)
        return -1;
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    auto len_of = [&](size_t k) { return bytes - k * kStageChunk < kStageChunk ? bytes - k * kStageChunk : kStageChunk; };
    auto issue = [&](size_t k) -> int {
        SALZ_HIP(hipMemcpyAsync(ws.hstage[k & 1], src + k * kStageChunk, len_of(k), hipMemcpyDeviceToHost,
                                ws.stream));
        SALZ_HIP(hipEventRecord(ws.hstage_ev[k & 1], ws.stream));
        return 0;
    };
    for (size_t k = 0; k < nch && k < 2; k++)
        if (issue(k) != 0)
            return -1;
    for (size_t k = 0; k < nch; k++) {
        SALZ_HIP(hipEventSynchronize(ws.hstage_ev[k & 1]));
        memcpy(dst + k * kStageChunk, ws.hstage[k & 1], len_of(k));
        if (k + 2 < nch && issue(k + 2) != 0)
            return -1;
    }
    return 0;
}

// Room for one stream (or a batch's streams at batch_stride apart) with margin: a SALZ stream
// is at most 12 + 9N/8 bytes before the PLAIN fallback replaces it.
static size_t batch_stride(size_t bs) { return ((size_t)salz_encoded_len_max(bs) + bs / 4 + 64 + 63) & ~(size_t)63; }
static size_t out_bound(size_t N) { return (size_t)salz_encoded_len_max(N) + N / 4 + 4096 + 128 * (size_t)kMaxBatchBlocks; }

static std::atomic<size_t> g_ws_allocs{0};

int workspace_alloc(Workspace &ws, int device, size_t max_block)
{
    g_ws_allocs.fetch_add(1);
    workspace_free(ws);
    SALZ_HIP(hipSetDevice(device));
    ws.device = device;
    size_t N = max_block < 8192 ? 8192 : max_block;
    ws.cap_N = N;
    ws.cap_n = N - 8;
    ws.np2 = 2048;
    while (ws.np2 < ws.cap_n)
        ws.np2 <<= 1;
    // Every per-position array has room for the interleaved layout of positions 0..cap_n.
    ws.cap_s = (ws.cap_n + 1 + kLayoutPad - 1) / kLayoutPad * kLayoutPad;
    const size_t n1 = ws.cap_s > ws.cap_n + 2 ? ws.cap_s : ws.cap_n + 2;
    const size_t ntiles = (ws.cap_n + kRadixTile - 1) / kRadixTile;
    // (at least 4096 words: ANSV keeps its range fills and 2 x 1024 queue counters there)
    ws.radix_counts_elems = (size_t)kMaxDigits * ntiles + kMaxDigits < 4096 ? 4096 : (size_t)kMaxDigits * ntiles + kMaxDigits;
    ws.out_cap = out_bound(N);
    size_t scan_elems = scan_temp_elems(ws.radix_counts_elems > n1 ? ws.radix_counts_elems : n1);
    ws.scan_tmp_bytes = scan_elems * sizeof(uint64_t);
    size_t held = 0;
    if (dalloc(&ws.text, N + 256) || dalloc(&ws.rank, n1) || dalloc(&ws.sa, n1) ||
        dalloc(&ws.keyA, n1) || dalloc(&ws.keyB, n1) || dalloc(&ws.valA, n1) ||
        dalloc(&ws.valB, n1) || dalloc(&ws.u0, n1) || dalloc(&ws.u1, n1) || dalloc(&ws.u2, n1) ||
        dalloc(&ws.u3, n1) || dalloc(&ws.lcps, n1) || dalloc(&ws.g64, n1) || dalloc(&ws.offA, n1) ||
        dalloc(&ws.offB, n1) || dalloc(&ws.cand, ws.cap_s) || dalloc(&ws.pst, ws.cap_s) ||
        dalloc(&ws.lsc, 2 * n1) || dalloc(&ws.lrec, n1 / 1024 + 2) || dalloc(&ws.lg2g, n1 / 1024 + 2) || dalloc(&ws.out, ws.out_cap) ||
        dalloc(&ws.radix_counts, ws.radix_counts_elems) ||
        dalloc(reinterpret_cast<uint8_t **>(&ws.scan_tmp), ws.scan_tmp_bytes) ||
        dalloc(&ws.dscal, 1024)) {
        std::string keep = g_err;
        workspace_free(ws);
        set_error("%s", keep.c_str());
        return -1;
    }
    ws.bytes = held;
    if (env_flag("SALZ_CHECK", "poison")) {
        // tests/diagnostics (SALZ_CHECK=poison=N): fill the workspace with a pattern so reads of
        // never-written memory misbehave deterministically instead of depending on what VRAM held
        const int v = (int)env_num("SALZ_CHECK", "poison", 0) & 0xff;
        void *ptrs[] = {ws.rank, ws.sa, ws.keyA, ws.keyB, ws.valA, ws.valB, ws.u0, ws.u1, ws.u2,
                        ws.u3, ws.g64, ws.offA, ws.offB, ws.cand, ws.pst, ws.lsc};
        size_t sizes[] = {4 * n1, 4 * n1, 8 * n1, 8 * n1, 4 * n1, 4 * n1, 4 * n1, 4 * n1, 4 * n1,
                          4 * n1, 8 * n1, 4 * n1, 4 * n1, 16 * ws.cap_s, 8 * ws.cap_s, 16 * n1};
        for (size_t k = 0; k < sizeof(ptrs) / sizeof(ptrs[0]); k++)
            SALZ_HIP(hipMemset(ptrs[k], v, sizes[k]));
        SALZ_HIP(hipMemset(ws.lrec, v, 8 * (n1 / 1024 + 2)));
        SALZ_HIP(hipMemset(ws.lg2g, v, 4 * (n1 / 1024 + 2)));
        SALZ_HIP(hipMemset(ws.text, v, N + 256));
    }
    // Host mirror of the device scalars, mapped into the device: a one-wave kernel on the
    // workspace's stream stores the words there (read_scalars), so no runtime copy path
    // (and none of its staging buffers) is shared between concurrently encoding contexts.
    void *h = nullptr;
    SALZ_HIP(hipHostMalloc(&h, kHostScal, hipHostMallocMapped | hipHostMallocCoherent));
    ws.hscal = static_cast<uint64_t *>(h);
    void *hd = nullptr;
    SALZ_HIP(hipHostGetDevicePointer(&hd, h, 0));
    ws.hscal_dev = static_cast<uint64_t *>(hd);
    SALZ_HIP(hipStreamCreateWithFlags(&ws.stream, hipStreamNonBlocking));
    ws.own_stream = true;
    for (hipEvent_t &e : ws.ev)
        SALZ_HIP(hipEventCreate(&e));
    return 0;  // rx_pool (radix-scatter timing events) is created on the first timed call
}

// (reset: after the copy, counters [zlo, zlo + nz) of d are zeroed for their next use, which saves
// a fill launch per counter)
__global__ void k_read_scalars(const uint32_t *__restrict__ d, uint32_t *h, uint32_t words, uint32_t *z = nullptr,
                               uint32_t nz = 0)
{
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
        __hip_atomic_store(&h[i], d[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (nz) {
        __syncthreads();
        if (threadIdx.x < nz)
            z[threadIdx.x] = 0u;
    }
}

// Arbitrary device memory through the upper half of the mapped buffer, in pieces.
int read_device(Workspace &ws, const void *src, size_t bytes, void *dst)
{
    constexpr size_t kHalf = kHostScal / 2;
    uint32_t *h = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(ws.hscal_dev) + kHalf);
    for (size_t o = 0; o < bytes; o += kHalf) {
        const size_t len = bytes - o < kHalf ? bytes - o : kHalf;
        hipLaunchKernelGGL(k_read_scalars, dim3(1), dim3(256), 0, ws.stream,
                           reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(src) + o), h,
                           (uint32_t)((len + 3) / 4));
        SALZ_LAUNCH_CHECK();
        SALZ_HIP(hipStreamSynchronize(ws.stream));
        memcpy(static_cast<uint8_t *>(dst) + o, reinterpret_cast<uint8_t *>(ws.hscal) + kHalf, len);
    }
    return 0;
}

int read_scalars(Workspace &ws, size_t off, size_t bytes, const char *tag, uint32_t zlo, uint32_t nz)
{
    (void)tag;
    const uint32_t *d = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(ws.dscal) + off);
    uint32_t *h = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(ws.hscal_dev) + off);
    hipLaunchKernelGGL(k_read_scalars, dim3(1), dim3(64), 0, ws.stream, d, h,
                       (uint32_t)((bytes + 3) / 4), reinterpret_cast<uint32_t *>(ws.dscal) + zlo, nz);
    SALZ_LAUNCH_CHECK();
    SALZ_HIP(hipStreamSynchronize(ws.stream));
    return 0;
}

enum : int { EV_START, EV_UP, EV_SA, EV_LCP, EV_ANSV, EV_PARSE, EV_EMIT };

// SALZ_CHECK_STAGES=1 (diagnostics): bound checks of the LCP array and the candidates.
__global__ void k_check_lcp(const uint32_t *sa, const uint32_t *lcp, const uint8_t *T, uint32_t n,
                            uint32_t *err)
{
    size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r == 0 || r >= n)
        return;
    const uint32_t a = sa[r - 1], b = sa[r], l = lcp[r];
    const uint32_t mx = a > b ? a : b;
    bool bad = l > n - mx;
    if (!bad && a + l < n && b + l < n && T[a + l] >= T[b + l])
        bad = true;  // adjacent suffixes must differ right after the LCP, in order
    if (!bad && l > 0 && T[a + l - 1] != T[b + l - 1])
        bad = true;
    if (bad)
        atomicOr(err, 0x200u);
}

// adjacent suffixes in order on their first 16 bytes (end of text sorts first)
__global__ void k_check_sa(const uint32_t *sa, const uint8_t *T, uint32_t n, uint32_t *err)
{
    size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r == 0 || r >= n)
        return;
    const uint32_t a = sa[r - 1], b = sa[r];
    for (uint32_t k = 0; k < 16; k++) {
        const bool ea = a + k >= n, eb = b + k >= n;
        if (ea || eb) {
            if (!ea)  // b ended first: b < a, out of order
                atomicOr(err, 0x800u);
            return;
        }
        if (T[a + k] != T[b + k]) {
            if (T[a + k] > T[b + k])
                atomicOr(err, 0x800u);
            return;
        }
    }
}

__global__ void k_check_cand(const uint4 *cand, uint32_t n, uint32_t klog, uint32_t *err)
{
    size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n)
        return;
    const uint4 c = cand[sidx((uint32_t)p, klog)];
    if (c.y > n - p || c.w > n - p || c.x == 0 || c.z == 0 || c.x > p + 1 || c.z > p + 1)
        atomicOr(err, 0x400u);
}

static int check_stage(Workspace &ws, uint32_t n, int which, const uint32_t *lcp = nullptr)
{
    static const bool on = env_flag("SALZ_CHECK", "stages");
    if (!on)
        return 0;
    uint32_t *derr = reinterpret_cast<uint32_t *>(ws.dscal) + kErrWord;
    if (which == 2)
        hipLaunchKernelGGL(k_check_sa, dim3(grid_for(n, 256)), dim3(256), 0, ws.stream, ws.sa,
                           ws.text, n, derr);
    else if (which == 0)
        hipLaunchKernelGGL(k_check_lcp, dim3(grid_for(n, 256)), dim3(256), 0, ws.stream, ws.sa,
                           lcp, ws.text, n, derr);
    else
        hipLaunchKernelGGL(k_check_cand, dim3(grid_for(n, 256)), dim3(256), 0, ws.stream, ws.cand,
                           n, ws.klog, derr);
    if (read_scalars(ws, 0, 256, "check") != 0)
        return -1;
    if (const uint32_t e = reinterpret_cast<uint32_t *>(ws.hscal)[kErrWord]) {
        set_error("stage check after %s failed (code 0x%x)",
                  which == 2 ? "sa" : which == 0 ? "lcp" : "ansv", e);
        return -1;
    }
    return 0;
}

static int mark(Workspace &ws, int which)
{
    if (ws.timing)
        SALZ_HIP(hipEventRecord(ws.ev[which], ws.stream));
    return 0;
}

static float elapsed(Workspace &ws, int a, int b)
{
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ws.ev[a], ws.ev[b]);
    return ms;
}

struct HostDump {
    const salz_gpu_dump *d;
};

static int dump_after_sa(Workspace &ws, uint32_t n, const salz_gpu_dump *d)
{
    if (d && d->sa) {
        SALZ_HIP(hipMemcpyAsync(d->sa, ws.sa, sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                                ws.stream));
        SALZ_HIP(hipStreamSynchronize(ws.stream));
    }
    return 0;
}

static int dump_after_parse(Workspace &ws, uint32_t n, const salz_gpu_dump *d)
{
    if (!d || !(d->psv || d->nsv || d->lp || d->ln || d->dlen || d->doff || d->cost))
        return 0;
    // the parse arrays are chunk-interleaved (common.hpp): copy the slots, index by sidx
    const size_t tile = (size_t)kTileChunks << ws.klog;
    const size_t S = ((size_t)n + 1 + tile - 1) / tile * tile;
    std::vector<uint4> cand(S);
    std::vector<uint8_t> choice(S);
    std::vector<uint32_t> cost(S);
    SALZ_HIP(hipMemcpyAsync(cand.data(), ws.cand, sizeof(uint4) * S, hipMemcpyDeviceToHost,
                            ws.stream));
    SALZ_HIP(hipMemcpyAsync(choice.data(), ws.parse.choice, S, hipMemcpyDeviceToHost, ws.stream));
    if (parse_materialize_cost(ws) != 0)
        return -1;
    SALZ_HIP(hipMemcpyAsync(cost.data(), ws.parse.cost, sizeof(uint32_t) * S,
                            hipMemcpyDeviceToHost, ws.stream));
    SALZ_HIP(hipStreamSynchronize(ws.stream));
    for (uint32_t p = 0; p < n; p++) {
        const size_t s = sidx(p, ws.klog);
        const uint4 c = cand[s];
        if (d->psv) d->psv[p] = (int32_t)(p - c.x);
        if (d->lp) d->lp[p] = (int32_t)c.y;
        if (d->nsv) d->nsv[p] = (int32_t)(p - c.z);
        if (d->ln) d->ln[p] = (int32_t)c.w;
        int32_t len = 1, off = 0;
        if (choice[s] == 1) {
            len = (int32_t)c.y;
            off = (int32_t)c.x;
        } else if (choice[s] == 2) {
            len = (int32_t)c.w;
            off = (int32_t)c.z;
        }
        if (d->dlen) d->dlen[p] = len;
        if (d->doff) d->doff[p] = off;
    }
    if (d->cost)
        for (size_t q = 0; q <= n; q++)
            d->cost[q] = (int32_t)cost[sidx((uint32_t)q, ws.klog)];
    return 0;
}

// LCP of SA[r - 1] and SA[r] for the listed ranks r (a split suffix array's piece starts):
// one wave per entry, 8 bytes per lane and step.
__global__ void k_lcp_fix(const uint32_t *__restrict__ sa, const uint8_t *__restrict__ T, uint32_t n,
                          const uint64_t *__restrict__ fix, uint32_t nfix, uint32_t *__restrict__ lcp)
{
    const uint32_t e = blockIdx.x;
    if (e >= nfix)
        return;
    const uint64_t r = fix[e];
    if (r >= n)
        return;
    if (r == 0) {
        if (threadIdx.x == 0)
            lcp[0] = 0;
        return;
    }
    const uint32_t a = sa[r - 1], b = sa[r];
    const uint32_t lim = n - (a > b ? a : b);
    uint32_t res = lim;
    for (uint32_t base = 0; base < lim; base += 64 * 8) {
        const uint32_t off = base + threadIdx.x * 8;
        const uint64_t x = load_u64_any(T, (size_t)a + off) ^ load_u64_any(T, (size_t)b + off);
        uint32_t mm = 0xffffffffu;
        if (off < lim && x)
            mm = off + ((uint32_t)__builtin_ctzll(x) >> 3);
        mm = wave_min_u32(mm);
        if (mm != 0xffffffffu) {
            res = mm < lim ? mm : lim;
            break;
        }
    }
    if (threadIdx.x == 0)
        lcp[r] = res;
}

// A suffix array (and LCP array) computed elsewhere, e.g. gathered from the pieces of a split
// suffix sort (dsa.hip): encode_core then starts at the candidates.
struct ExtSa {
    const uint32_t *sa, *lcp;
    const uint64_t *fix;  // host: LCP entries to recompute
    size_t nfix;
};

// Encode a batch: P bytes of src (host or device memory) as consecutive blocks of bs bytes
// (bs >= P: one block), every block's stream into device memory at dst + b * stride (at most
// cap bytes each), lens[b] = its length. A batch of several blocks needs bs to be a multiple
// of 512 (parse chunks never straddle two blocks) and every block longer than 8 bytes.
static int encode_core(Workspace &ws, const uint8_t *src, bool src_dev, size_t P, size_t bs,
                       uint8_t *dst, size_t stride, size_t cap, size_t *lens, const salz_gpu_dump *dump,
                       const ExtSa *ext = nullptr)
{
    const size_t nbz = bs >= P ? 1 : (P + bs - 1) / bs;
    const size_t N_last = nbz == 1 ? P : P - (nbz - 1) * bs;
    if (N_last <= 8) {
        set_error("block of %zu bytes: the reference codec needs more than 8 bytes", N_last);
        return -1;  // lib/salz.c:197 wraps (N < 8) or crashes (N == 8)
    }
    if (P > ws.cap_N || P - 8 >= 0x7fffffffu) {
        set_error("input of %zu bytes exceeds context capacity %zu", P, ws.cap_N);
        return -1;
    }
    if (nbz > 1 && bs % 512 != 0) {
        set_error("batch block size %zu is not a multiple of 512", bs);
        return -1;
    }
    if (nbz > kMaxBatchBlocks) {
        set_error("%zu blocks exceed the batch limit %u", nbz, kMaxBatchBlocks);
        return -1;
    }
    const Blocks bl{nbz == 1 ? 0xffffffffu : (uint32_t)bs, (uint32_t)nbz, (uint32_t)(P - 8)};
    SALZ_HIP(hipSetDevice(ws.device));
    hipStream_t st = ws.stream;
    const uint32_t n = bl.npos;
    ws.stats = StageStats{};
    ws.rx_used = 0;
    if (ws.timing && ws.rx_pool.empty()) {
        ws.rx_pool.resize(2048);
        for (hipEvent_t &e : ws.rx_pool)
            SALZ_HIP(hipEventCreate(&e));
    }

    if (mark(ws, EV_START)) return -1;
    if (src_dev)
        SALZ_HIP(hipMemcpyAsync(ws.text, src, P, hipMemcpyDeviceToDevice, st));
    else if (copy_h2d(ws, ws.text, src, P) != 0)
        return -1;
    SALZ_HIP(fill_async(ws.text + P, 0, 128, st));
    // (a batch's chunk length follows its block size: the per-block trade-off of pass count
    // against pass length, parse.hip)
    ws.klog = parse_chunk_log(nbz == 1 ? P : bs);
    if (nbz > 1 && bs % ((size_t)1 << ws.klog) != 0) {
        set_error("batch block size %zu is not a multiple of the parse chunk", bs);
        return -1;
    }
    if (mark(ws, EV_UP)) return -1;
    ws.sigma = 0;
    ws.stats.sa_dc3_levels = 0;  // (a suffix array handed in says nothing about repeats)
    if (ext) {
        SALZ_HIP(hipMemcpyAsync(ws.sa, ext->sa, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        ws.lcps_ok = ext->lcp != nullptr;
        if (ws.lcps_ok) {
            SALZ_HIP(hipMemcpyAsync(ws.lcps, ext->lcp, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            if (ext->nfix) {
                uint64_t *dfix = reinterpret_cast<uint64_t *>(ws.lsc);  // free before the candidates
                SALZ_HIP(hipMemcpyAsync(dfix, ext->fix, ext->nfix * sizeof(uint64_t), hipMemcpyHostToDevice, st));
                hipLaunchKernelGGL(k_lcp_fix, dim3((unsigned)ext->nfix), dim3(64), 0, st, ws.sa, ws.text, n, dfix,
                                   (uint32_t)ext->nfix, ws.lcps);
                SALZ_LAUNCH_CHECK();
            }
        }
    } else if (stage_suffix_array(ws, bl)) {
        return -1;
    }
    // A large single block (> 32 MiB) of more than 127 distinct bytes (binary or mixed data, no
    // text alphabet) parses with 128-position chunks: its pass count barely depends on the chunk
    // length, and the late passes walk a quarter as far (mixed 100 MB: 43.2 -> 42.0 ms); text
    // keeps K = 512, whose passes are fewer (3 instead of 6 at K = 128 on 100 MB).
    // Single blocks of 8–16 MiB take K = 128 instead of the size rule's 64 whatever the data:
    // mixed 16 MiB blocks, 4 slots: C3 2650 -> 2725 MB/s; text 16 MiB blocks in the same layout
    // 3224 / 3191 -> 3570 / 3567 MB/s (profiles/r03zzz_c3text_klog_ab.txt), though one block alone
    // parses 0.4 ms slower than at K = 64: fewer chunks and exits cost less GPU time in total
    // while other slots keep the GPU busy.
    // A block the suffix sort sent to DC3 over an alphabet of at most 4 bytes (Fibonacci, zeros,
    // short periods: long factors everywhere, so its pass count barely depends on K) parses at
    // K = 128 as well: Fibonacci 256 MiB parse 9.9 -> 7.9 ms (profiles/r04zd_klog_probe.txt; random
    // small alphabets, which stay on prefix doubling, need twice the passes at K = 128). Other DC3
    // blocks keep the size rule, wider alphabets included: their factors mix long and short, and K
    // = 512 takes fewer passes (256 MiB, K = 128 -> 512: runs of 64 equal bytes 16 -> 13 passes,
    // parse 26.5 -> 22.7 ms; a text repeated at distance n / 2, 6 -> 3 passes, 11.6 -> 8.1 ms; a
    // period of 1000 or a 0..255 sawtooth 4.4 -> 5.0 ms; profiles/r06g_klog_probe.txt).
    const bool repetitive = ws.stats.sa_dc3_levels > 0;
    const bool k128 = repetitive ? ws.sigma <= 4 : ws.sigma > 127;
    if (nbz == 1 && !env_flag("SALZ_PARSE", "klog") && ((k128 && ws.klog > 7) || (ws.klog < 7 && n > (8u << 20))))
        ws.klog = 7;
    if (guard_check(ws, "sa") || (nbz == 1 && check_stage(ws, n, 2))) return -1;
    if (mark(ws, EV_SA)) return -1;
    if (dump_after_sa(ws, bl.nsa(), dump)) return -1;
    // The suffix sorter usually leaves the LCP array behind (sa.hip, "LCP"); otherwise the
    // Phi / PLCP stage computes it.
    uint32_t *lcp = ws.lcps_ok ? ws.lcps : ws.u3;
    if ((!ws.lcps_ok && stage_lcp(ws, bl, lcp)) || guard_check(ws, "lcp") ||
        (nbz == 1 && check_stage(ws, n, 0, lcp)))
        return -1;
    if (mark(ws, EV_LCP)) return -1;
    if (stage_candidates(ws, bl, lcp) || guard_check(ws, "ansv") || (nbz == 1 && check_stage(ws, n, 1)))
        return -1;
    if (mark(ws, EV_ANSV)) return -1;
    if (stage_parse(ws, bl) || guard_check(ws, "parse")) return -1;
    if (mark(ws, EV_PARSE)) return -1;
    if (dump_after_parse(ws, n, dump)) return -1;
    if (stage_emit(ws, bl, (uint32_t)N_last, dst, stride, cap, lens) || guard_check(ws, "emit")) return -1;
    if (mark(ws, EV_EMIT)) return -1;
    SALZ_HIP(hipStreamSynchronize(st));
    if (ws.timing) {
        ws.stats.ms_upload = elapsed(ws, EV_START, EV_UP);
        ws.stats.ms_sa = elapsed(ws, EV_UP, EV_SA);
        ws.stats.ms_lcp = elapsed(ws, EV_SA, EV_LCP);
        ws.stats.ms_ansv = elapsed(ws, EV_LCP, EV_ANSV);
        ws.stats.ms_parse = elapsed(ws, EV_ANSV, EV_PARSE);
        ws.stats.ms_emit = elapsed(ws, EV_PARSE, EV_EMIT);
        ws.stats.ms_total = elapsed(ws, EV_START, EV_EMIT);
        float rx = 0.f;
        for (size_t i = 0; i + 1 < ws.rx_used; i += 2) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ws.rx_pool[i], ws.rx_pool[i + 1]);
            rx += ms;
        }
        ws.stats.ms_radix_scatter = rx;
    }
    return 0;
}

// Frames of a batch, packed: u32 length + stream per block, in block order (the CLI container's
// body, programs/salzcli.c:163-169). One workgroup per block; foff = exclusive scan of 4 + len.
__global__ void k_frame_len(const size_t *__restrict__ lens, uint64_t *__restrict__ flen, uint32_t nb)
{
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b < nb)
        flen[b] = 4 + (uint64_t)lens[b];
}

// grid (pieces of 4 KiB, blocks): a thread moves 16 bytes, one aligned 16-byte load from the
// block's region (regions are 64-byte aligned) and 16 byte stores (frames are unaligned).
__global__ __launch_bounds__(256) void k_pack_frames(const uint8_t *__restrict__ regions, size_t stride,
                                                     const size_t *__restrict__ lens,
                                                     const uint64_t *__restrict__ foff,
                                                     uint8_t *__restrict__ out)
{
    const uint32_t b = blockIdx.y;
    const uint32_t L = (uint32_t)lens[b];
    uint8_t *o = out + foff[b];
    if (blockIdx.x == 0 && threadIdx.x < 4)
        o[threadIdx.x] = (uint8_t)(L >> (8 * threadIdx.x));
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i >= L)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(regions + (size_t)b * stride + i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t cnt = L - i < 16 ? (uint32_t)(L - i) : 16u;
    for (uint32_t k = 0; k < cnt; k++)
        o[4 + i + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// A batch: every block encoded in one pipeline pass and its frames packed (u32 length +
// stream per block) into device memory `packed` (capacity packed_cap); *total = bytes.
// Grow the workspace (reallocating every buffer) until a batch of P bytes in blocks of bs fits.
static int ensure_batch_room(Workspace &ws, size_t P, size_t bs)
{
    const size_t nb = bs >= P ? 1 : (P + bs - 1) / bs;
    const size_t need = nb * batch_stride(bs < P ? bs : P);  // every block's stream slot
    if (P <= ws.cap_N && need <= ws.out_cap)
        return 0;
    // The output buffer follows the block capacity (out_bound): a batch whose last block is short
    // needs more stream slots than out_bound(P) covers, so grow until it does.
    size_t N = P > ws.cap_N ? P : ws.cap_N;
    while (out_bound(N) < need)
        N += bs < P ? bs : P;
    return workspace_alloc(ws, ws.device, N);
}

static int encode_batch_packed(Workspace &ws, const uint8_t *src, bool src_dev, size_t P, size_t bs,
                               uint8_t *packed, size_t packed_cap, size_t *total,
                               const salz_gpu_dump *dump)
{
    const size_t nb = bs >= P ? 1 : (P + bs - 1) / bs;
    const size_t stride = batch_stride(bs < P ? bs : P);
    if (P > ws.cap_N || nb * stride > ws.out_cap) {  // callers grow the workspace beforehand
        set_error("batch of %zu bytes exceeds the context's workspace", P);
        return -1;
    }
    // Every block gets the reference CLI's output capacity, salz_encoded_len_max(block size)
    // (programs/salzcli.c:130, :156), so a block the reference fails on (an incompressible
    // block whose SALZ stream runs a few bytes past that bound before the PLAIN fallback)
    // fails here too.
    const size_t cap = (size_t)salz_encoded_len_max(bs);
    std::vector<size_t> lens(nb);
    if (encode_core(ws, src, src_dev, P, bs, ws.out, stride, cap < stride ? cap : stride, lens.data(), dump) != 0)
        return -1;
    size_t sum = 0;
    for (size_t L : lens)
        sum += 4 + L;
    if (sum > packed_cap) {
        set_error("batch frames (%zu bytes) exceed the destination capacity (%zu)", sum, packed_cap);
        return -1;
    }
    // lens to the device (plain host -> device copy), frame offsets by a device scan
    size_t *dlens = reinterpret_cast<size_t *>(ws.lrec);  // free after the suffix sort
    uint64_t *foff = reinterpret_cast<uint64_t *>(ws.lrec) + nb;
    if (2 * nb + 2 > ws.cap_n / 1024 + 2) {
        set_error("batch of %zu blocks: no room for the frame table", nb);
        return -1;
    }
    SALZ_HIP(hipMemcpyAsync(dlens, lens.data(), sizeof(size_t) * nb, hipMemcpyHostToDevice, ws.stream));
    hipLaunchKernelGGL(k_frame_len, dim3(grid_for(nb, 256)), dim3(256), 0, ws.stream, dlens, foff, (uint32_t)nb);
    SALZ_LAUNCH_CHECK();
    if (scan_sum_u64(foff, foff, nb, false, nullptr, ws, ws.stream) != 0)
        return -1;
    size_t maxL = 0;
    for (size_t L : lens)
        maxL = L > maxL ? L : maxL;
    hipLaunchKernelGGL(k_pack_frames, dim3(grid_for(maxL, 4096), (unsigned)nb), dim3(256), 0, ws.stream,
                       ws.out, stride, dlens, foff, packed);
    SALZ_LAUNCH_CHECK();
    *total = sum;
    return 0;
}

// The same from host memory to host memory dst (capacity *dst_len; set to the bytes written).
static int encode_batch_locked(Workspace &ws, const uint8_t *src, size_t P, size_t bs, uint8_t *dst,
                               size_t *dst_len, const salz_gpu_dump *dump = nullptr)
{
    if (ensure_batch_room(ws, P, bs) != 0)
        return -1;
    uint8_t *packed = reinterpret_cast<uint8_t *>(ws.keyB);  // free after emission (8 bytes per position)
    size_t total = 0;
    if (encode_batch_packed(ws, src, false, P, bs, packed, 8 * ws.cap_s, &total, dump) != 0)
        return -1;
    if (total > *dst_len) {
        set_error("batch frames (%zu bytes) exceed the destination capacity (%zu)", total, *dst_len);
        return -1;
    }
    if (copy_d2h(ws, dst, packed, total) != 0)
        return -1;
    *dst_len = total;
    return 0;
}

// One block (the reference's unit): the stream to device buffer dst (capacity cap).
static int encode_one(Workspace &ws, const uint8_t *src, bool src_dev, size_t N, uint8_t *dst,
                      size_t cap, size_t *out_len, const salz_gpu_dump *dump)
{
    return encode_core(ws, src, src_dev, N, N, dst, 0, cap, out_len, dump);
}

}  // namespace salz

using namespace salz;

struct salz_gpu_ctx {
    Workspace ws;
    std::mutex mu;
    std::atomic<size_t> held{0};  // ws.bytes as of its last pooled call (read without mu)
};

extern "C" {

const char *salz_gpu_last_error(void) { return g_err; }

uint32_t salz_gpu_parse_chunk_log(size_t block_len) { return parse_chunk_log(block_len); }

// Test hook (host only): the round-0 list order of a batch (common.hpp init_suffix), so the
// CPU tests can check it enumerates every live suffix once, shortest-first per block.
int salz_debug_init_order(size_t src_len, size_t block_size, uint32_t *out)
{
    if (!out || src_len <= 8)
        return -1;
    const size_t nb = block_size >= src_len ? 1 : (src_len + block_size - 1) / block_size;
    const Blocks bl{nb == 1 ? 0xffffffffu : (uint32_t)block_size, (uint32_t)nb, (uint32_t)(src_len - 8)};
    for (uint32_t c = 0; c < bl.nsa(); c++)
        out[c] = init_suffix(c, bl);
    return (int)bl.nsa();
}

int salz_gpu_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

void *salz_gpu_malloc(int device, size_t bytes)
{
    void *p = nullptr;
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        set_error("hipMalloc(%zu) on device %d failed", bytes, device);
        return nullptr;
    }
    return p;
}

void salz_gpu_free(int device, void *ptr)
{
    if (ptr && hipSetDevice(device) == hipSuccess)
        (void)hipFree(ptr);
}

int salz_gpu_memcpy_h2d(int device, void *dst, const void *src, size_t bytes)
{
    SALZ_HIP(hipSetDevice(device));
    SALZ_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return 0;
}

int salz_gpu_memcpy_d2h(int device, void *dst, const void *src, size_t bytes)
{
    SALZ_HIP(hipSetDevice(device));
    SALZ_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}

int salz_gpu_synchronize(int device)
{
    SALZ_HIP(hipSetDevice(device));
    SALZ_HIP(hipDeviceSynchronize());
    return 0;
}

salz_gpu_ctx *salz_gpu_ctx_create(int device, size_t max_block)
{
    salz_gpu_ctx *c = new (std::nothrow) salz_gpu_ctx();
    if (!c) {
        set_error("out of host memory");
        return nullptr;
    }
    if (workspace_alloc(c->ws, device, max_block) != 0) {
        delete c;
        return nullptr;
    }
    c->held.store(c->ws.bytes);
    return c;
}

void salz_gpu_ctx_destroy(salz_gpu_ctx *ctx)
{
    if (!ctx)
        return;
    workspace_free(ctx->ws);
    delete ctx;
}

void salz_gpu_set_timing(salz_gpu_ctx *ctx, int on)
{
    if (ctx)
        ctx->ws.timing = on != 0;
}

int salz_gpu_get_stats(const salz_gpu_ctx *ctx, salz_gpu_stats *o)
{
    if (!ctx || !o)
        return -1;
    const StageStats &s = ctx->ws.stats;
    o->ms_upload = s.ms_upload;
    o->ms_sa = s.ms_sa;
    o->ms_lcp = s.ms_lcp;
    o->ms_ansv = s.ms_ansv;
    o->ms_parse = s.ms_parse;
    o->ms_emit = s.ms_emit;
    o->ms_total = s.ms_total;
    o->sa_rounds = s.sa_rounds;
    o->parse_iters = s.parse_iters;
    o->sa_sorted_elems = s.sa_sorted_elems;
    o->lcp_long_bytes = s.lcp_long_bytes;
    o->emit_bits = s.emit_bits;
    o->emit_bytes = s.emit_bytes;
    o->exit_nodes = s.exit_nodes;
    o->radix_scatter_launches = s.radix_scatter_launches;
    o->ms_radix_scatter = s.ms_radix_scatter;
    o->radix_scatter_elems = s.radix_scatter_elems;
    o->sa_dc3_levels = s.sa_dc3_levels;
    o->radix_scatter_bytes = s.radix_scatter_bytes;
    return 0;
}

int salz_gpu_encode_device(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t src_len,
                           uint8_t *d_dst, size_t dst_cap, size_t *dst_len, void *stream)
{
    if (!ctx || !d_src || !d_dst || !dst_len) {
        set_error("NULL argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    Workspace &ws = ctx->ws;
    hipStream_t saved = ws.stream;
    if (stream)
        ws.stream = static_cast<hipStream_t>(stream);
    size_t len = 0;
    int rc = encode_one(ws, d_src, true, src_len, d_dst, dst_cap, &len, nullptr);
    ws.stream = saved;
    if (rc == 0)
        *dst_len = len;
    return rc;
}

static int encode_host_locked(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, uint8_t *dst,
                              size_t *dst_len, const salz_gpu_dump *dump)
{
    Workspace &ws = ctx->ws;
    if (src_len > ws.cap_N) {
        int dev = ws.device;
        if (workspace_alloc(ws, dev, src_len) != 0)
            return -1;
    }
    size_t cap = *dst_len < ws.out_cap ? *dst_len : ws.out_cap;
    size_t len = 0;
    if (encode_one(ws, src, false, src_len, ws.out, cap, &len, dump) != 0)
        return -1;
    if (copy_d2h(ws, dst, ws.out, len) != 0) {
        set_error("D2H copy of the encoded stream failed");
        return -1;
    }
    *dst_len = len;  // set only on success (lib/salz.c:818)
    return 0;
}

}  // extern "C"

// The split suffix sort's piece of this rank (dsa.hip), through either kind of collectives.
template <typename Sort>
static int dist_piece(salz_gpu_ctx *ctx, const uint8_t *d_text, size_t N, uint32_t *d_sa_piece,
                      uint32_t *d_lcp_piece, int *lcp_ok, Sort sort)
{
    if (N <= 8 || N - 8 >= 0x7fffffffu) {
        set_error("block of %zu bytes: the reference codec needs more than 8 bytes", N);
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    Workspace &ws = ctx->ws;
    if (N > ws.cap_N && workspace_alloc(ws, ws.device, N) != 0)
        return -1;
    SALZ_HIP(hipSetDevice(ws.device));
    hipStream_t st = ws.stream;
    ws.stats = StageStats{};
    SALZ_HIP(hipMemcpyAsync(ws.text, d_text, N, hipMemcpyDeviceToDevice, st));
    SALZ_HIP(fill_async(ws.text + N, 0, 128, st));
    const uint32_t n = (uint32_t)(N - 8);
    uint32_t m0 = 0;
    const int rc = sort(ws, n, &m0);
    if (rc < 0)
        return -1;
    if (rc == 1) {  // not split (a repetitive block): the caller encodes it whole
        *lcp_ok = 0;
        return 1;
    }
    if (m0) {
        SALZ_HIP(hipMemcpyAsync(d_sa_piece, ws.sa, (size_t)m0 * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        if (ws.lcps_ok)
            SALZ_HIP(hipMemcpyAsync(d_lcp_piece, ws.lcps, (size_t)m0 * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                    st));
    }
    SALZ_HIP(hipStreamSynchronize(st));
    *lcp_ok = m0 == 0 || ws.lcps_ok ? 1 : 0;
    return 0;
}

extern "C" {

int salz_gpu_dist_suffix_array(salz_gpu_ctx *ctx, const uint8_t *d_text, size_t N, int nranks, int rank,
                               const salz_dist_ops *ops, uint32_t *d_xsend, uint32_t *d_xrecv,
                               size_t xcap, uint32_t *d_sa_piece, uint32_t *d_lcp_piece,
                               uint64_t *offsets, int *lcp_ok)
{
    if (!ctx || !d_text || !ops || !ops->alltoall || !ops->allreduce_sum || !d_xsend || !d_xrecv ||
        !d_sa_piece || !d_lcp_piece || !offsets || !lcp_ok) {
        set_error("NULL argument");
        return -1;
    }
    return dist_piece(ctx, d_text, N, d_sa_piece, d_lcp_piece, lcp_ok, [&](Workspace &ws, uint32_t n, uint32_t *m0) {
        return dist_suffix_array_ops(ws, n, nranks, rank, ops, d_xsend, d_xrecv, xcap, offsets, m0);
    });
}

int salz_gpu_dist_suffix_array_comm(salz_gpu_ctx *ctx, const uint8_t *d_text, size_t N, salz_gpu_dist_comm *comm,
                                    uint32_t *d_xsend, uint32_t *d_xrecv, size_t xcap, uint32_t *d_sa_piece,
                                    uint32_t *d_lcp_piece, uint64_t *offsets, int *lcp_ok)
{
    if (!ctx || !d_text || !comm || !d_xsend || !d_xrecv || !d_sa_piece || !d_lcp_piece || !offsets || !lcp_ok) {
        set_error("NULL argument");
        return -1;
    }
    return dist_piece(ctx, d_text, N, d_sa_piece, d_lcp_piece, lcp_ok, [&](Workspace &ws, uint32_t n, uint32_t *m0) {
        return dist_suffix_array_comm(ws, n, reinterpret_cast<DistComm *>(comm), d_xsend, d_xrecv, xcap, offsets, m0);
    });
}

int salz_gpu_encode_from_sa(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t N, const uint32_t *d_sa,
                            const uint32_t *d_lcp, const uint64_t *lcp_fix, size_t nfix, uint8_t *d_dst,
                            size_t dst_cap, size_t *dst_len)
{
    if (!ctx || !d_src || !d_sa || !d_dst || !dst_len || (nfix && !lcp_fix)) {
        set_error("NULL argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    Workspace &ws = ctx->ws;
    if (N > ws.cap_N && workspace_alloc(ws, ws.device, N) != 0)
        return -1;
    const ExtSa ext{d_sa, d_lcp, lcp_fix, nfix};
    size_t len = 0;
    if (encode_core(ws, d_src, true, N, N, d_dst, 0, dst_cap, &len, nullptr, &ext) != 0)
        return -1;
    *dst_len = len;
    return 0;
}

int salz_gpu_encode_host(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, uint8_t *dst,
                         size_t *dst_len)
{
    if (!ctx || !src || !dst || !dst_len) {
        set_error("NULL argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_host_locked(ctx, src, src_len, dst, dst_len, nullptr);
}

int salz_gpu_encode_dump(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, uint8_t *dst,
                         size_t *dst_len, const salz_gpu_dump *dump)
{
    if (!ctx || !src || !dst || !dst_len) {
        set_error("NULL argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_host_locked(ctx, src, src_len, dst, dst_len, dump);
}

int salz_gpu_encode_batch(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len, size_t block_size,
                          uint8_t *dst, size_t *dst_len)
{
    if (!ctx || !src || !dst || !dst_len || block_size == 0) {
        set_error("invalid argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_batch_locked(ctx->ws, src, src_len, block_size, dst, dst_len);
}

int salz_gpu_encode_batch_device(salz_gpu_ctx *ctx, const uint8_t *d_src, size_t src_len,
                                 size_t block_size, uint8_t *d_dst, size_t dst_cap, size_t *dst_len,
                                 void *stream)
{
    if (!ctx || !d_src || !d_dst || !dst_len || block_size == 0) {
        set_error("invalid argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    Workspace &ws = ctx->ws;
    if (ensure_batch_room(ws, src_len, block_size) != 0)  // (before the stream swap: it recreates ws)
        return -1;
    hipStream_t saved = ws.stream;
    if (stream)
        ws.stream = static_cast<hipStream_t>(stream);
    size_t total = 0;
    int rc = encode_batch_packed(ws, d_src, true, src_len, block_size, d_dst, dst_cap, &total, nullptr);
    if (rc == 0 && hipStreamSynchronize(ws.stream) != hipSuccess) {
        set_error("stream synchronize failed");
        rc = -1;
    }
    ws.stream = saved;
    if (rc == 0)
        *dst_len = total;
    return rc;
}

// Test hook: read workspace scratch left by the last encode (0: ws.sa = emission's chunk
// entries, 1: ws.g64 = emission's chunk bit / byte starts), `count` u32 / u64 words from `off`.
int salz_debug_ws_read(salz_gpu_ctx *ctx, int which, size_t off, size_t count, void *out)
{
    if (!ctx || !out)
        return -1;
    std::lock_guard<std::mutex> lk(ctx->mu);
    Workspace &ws = ctx->ws;
    if (which == 0)
        return read_device(ws, ws.sa + off, count * 4, out);
    return read_device(ws, ws.g64 + off, count * 8, out);
}

// Test hook: salz_gpu_encode_batch with the stage arrays of the whole batch (suffix array of
// nsa entries in global text positions; the per-position arrays over the position space).
int salz_debug_encode_batch_dump(salz_gpu_ctx *ctx, const uint8_t *src, size_t src_len,
                                 size_t block_size, uint8_t *dst, size_t *dst_len,
                                 const salz_gpu_dump *dump)
{
    if (!ctx || !src || !dst || !dst_len || block_size == 0) {
        set_error("invalid argument");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_batch_locked(ctx->ws, src, src_len, block_size, dst, dst_len, dump);
}

// ---- default contexts behind salz_encode_safe ----------------------------------------------

// Cached contexts: slot 0 of each device serves salz_encode_safe; salz_encode_blocks uses
// slots 0..k-1 so that k blocks are in flight per device (their own streams and workspaces).
// A slot being filled holds kCreating while its context is created outside g_default_mu (a
// workspace is several hipMallocs of up to tens of GB: no other caller waits behind them).
constexpr int kMaxSlots = 8;
static std::mutex g_default_mu;
static std::condition_variable g_pool_cv;
static std::vector<salz_gpu_ctx *> g_default;  // [device * kMaxSlots + slot]
static salz_gpu_ctx g_creating_tag;
static salz_gpu_ctx *const kCreating = &g_creating_tag;

static bool pool_init_locked()
{
    if (g_default.empty()) {
        const int n = salz_gpu_device_count();
        g_default.assign(n > 0 ? (size_t)n * kMaxSlots : 0, nullptr);
    }
    return !g_default.empty();
}

// Create the context of a slot that holds kCreating (the caller reserved it), outside the pool
// lock, and publish it (locked by the caller when `lock`) or clear the reservation on failure.
static salz_gpu_ctx *pool_fill_slot(size_t idx, int device, size_t need, bool lock)
{
    salz_gpu_ctx *c = salz_gpu_ctx_create(device, need);
    if (c && lock)
        c->mu.lock();  // not yet visible to anyone else
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        g_default[idx] = c;
    }
    g_pool_cv.notify_all();
    return c;
}

static salz_gpu_ctx *default_ctx(int device, size_t need, int slot = 0)
{
    std::unique_lock<std::mutex> lk(g_default_mu);
    if (!pool_init_locked() || device < 0 || (size_t)device * kMaxSlots >= g_default.size() || slot < 0 ||
        slot >= kMaxSlots) {
        set_error("no usable HIP device (gfx950) for salz_encode_safe");
        return nullptr;
    }
    const size_t idx = (size_t)device * kMaxSlots + slot;
    g_pool_cv.wait(lk, [&] { return g_default[idx] != kCreating; });
    if (salz_gpu_ctx *c = g_default[idx])
        return c;
    g_default[idx] = kCreating;
    lk.unlock();
    return pool_fill_slot(idx, device, need, false);
}

// salz_encode_safe's context pool. The reference encoder keeps no state between calls
// (lib/salz.c:175-256, :777-823), so T threads calling it encode T blocks at once. Here a call
// takes an idle cached context on the caller's current device, or creates one there, up to
// SALZ_SAFE_SLOTS (default 4) per device; when every one is busy it waits for one. Contexts on
// other devices are borrowed only after salz_gpu_pool_config(any_device = 1). Contexts are
// shared with salz_encode_blocks / salz_encode_stream (same slots, same mutexes).
// The reference frees its scratch after every call (lib/salz.c:175-256); the pool keeps
// workspaces for the next call but caps what idle contexts hold per device (SALZ_SAFE_CACHE_BYTES
// or salz_gpu_pool_config, default 32 GiB): after a call, idle workspaces are released, the
// largest first, until the device's pool is under the cap (a released context reallocates
// on its next call).
static std::atomic<int> g_pool_slots{0};
static std::atomic<size_t> g_pool_cap{0};
static std::atomic<int> g_pool_any_dev{0};

static int safe_slots_per_device()
{
    int v = g_pool_slots.load();
    if (v == 0) {
        const char *e = getenv("SALZ_SAFE_SLOTS");
        const int k = e ? atoi(e) : 4;
        v = k < 1 ? 1 : k > kMaxSlots ? kMaxSlots : k;
        g_pool_slots.store(v);
    }
    return v;
}

static size_t pool_cap_bytes()
{
    size_t v = g_pool_cap.load();
    if (v == 0) {
        const char *e = getenv("SALZ_SAFE_CACHE_BYTES");
        v = e ? (size_t)strtoull(e, nullptr, 0) : (size_t)32 << 30;
        g_pool_cap.store(v ? v : 1);
    }
    return v;
}

// An idle context, locked (ctx->mu held on return), or nullptr when all are busy and no new
// one may be created. Creates at most one context per call; *create_failed reports a failed
// creation (device memory exhausted) and *have_any whether any context exists to wait for.
static salz_gpu_ctx *pool_try_acquire(int cur, size_t need, bool *create_failed, bool *have_any)
{
    *create_failed = false;
    *have_any = false;
    const int ndev = salz_gpu_device_count();
    if (ndev <= 0)
        return nullptr;
    const int per = safe_slots_per_device();
    const int ndev_use = g_pool_any_dev.load() ? ndev : 1;
    std::vector<salz_gpu_ctx *> snap;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        if (!pool_init_locked())
            return nullptr;
        snap = g_default;
    }
    for (int k = 0; k < ndev_use; k++) {  // existing idle contexts, current device first
        const int d = (cur + k) % ndev;
        for (int s = 0; s < kMaxSlots; s++) {
            salz_gpu_ctx *c = snap[(size_t)d * kMaxSlots + s];
            *have_any = *have_any || c != nullptr;
            if (c && c != kCreating && c->mu.try_lock())
                return c;
        }
    }
    // all busy: a new context on the device with the fewest (the caller's own on a tie)
    size_t idx = 0;
    int best = -1;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        int best_n = per;
        for (int k = 0; k < ndev_use; k++) {
            const int d = (cur + k) % ndev;
            int cnt = 0;
            for (int s = 0; s < per; s++)
                cnt += g_default[(size_t)d * kMaxSlots + s] != nullptr;
            if (cnt < best_n) {
                best = d;
                best_n = cnt;
            }
        }
        if (best < 0)
            return nullptr;
        for (int s = 0; s < per; s++)
            if (!g_default[(size_t)best * kMaxSlots + s]) {
                idx = (size_t)best * kMaxSlots + s;
                g_default[idx] = kCreating;
                break;
            }
    }
    salz_gpu_ctx *c = pool_fill_slot(idx, best, need, true);
    *create_failed = c == nullptr;
    return c;
}

// After a call on `dev`: while the device's IDLE workspaces (`mine`, whose caller still holds it
// and is about to let it go, and every other context not busy right now) hold more than the cap,
// release the largest. Busy contexts neither count nor get released: their callers trim after
// their own calls. (Counting them let two concurrent 256 MiB callers, ~30 GB each against the
// 32 GiB default, free their own workspace after every call and reallocate it on the next.)
// The usual case, every workspace of the device together under the cap, takes no lock at all;
// otherwise each context is locked only while its bytes are read or while it is released, so
// another thread's pool_try_acquire never finds the whole pool locked by a trim.
static void pool_trim(int dev, salz_gpu_ctx *mine)
{
    const size_t cap = pool_cap_bytes();
    std::vector<salz_gpu_ctx *> snap;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        if ((size_t)(dev + 1) * kMaxSlots > g_default.size())
            return;
        snap.assign(g_default.begin() + (size_t)dev * kMaxSlots, g_default.begin() + (size_t)(dev + 1) * kMaxSlots);
    }
    size_t all = 0;  // busy ones included: an upper bound of the idle total
    for (salz_gpu_ctx *c : snap)
        if (c && c != kCreating)
            all += c->held.load();
    if (all <= cap)
        return;
    for (int round = 0; round < 2 * kMaxSlots; round++) {  // (each round releases one workspace)
        size_t total = 0, big = 0;
        salz_gpu_ctx *victim = nullptr;
        for (salz_gpu_ctx *c : snap) {
            if (!c || c == kCreating || (c != mine && !c->mu.try_lock()))
                continue;  // busy: not counted
            const size_t b = c->held.load();
            total += b;
            if (b > big) {
                big = b;
                victim = c;
            }
            if (c != mine)
                c->mu.unlock();
        }
        if (total <= cap || !victim)
            break;
        if (victim != mine && !victim->mu.try_lock())
            continue;  // taken meanwhile: the next round counts without it
        workspace_release(victim->ws);
        victim->held.store(0);
        if (victim != mine)
            victim->mu.unlock();
    }
}

// Restores the calling thread's current HIP device (the pool may create or run a context on
// another device, and every encode sets the device of its workspace).
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard()
    {
        if (dev >= 0)
            (void)hipSetDevice(dev);
    }
};

// Called by salz_encode_safe (salz.c) after argument checks.
int salz_gpu_encode_default(const uint8_t *src, size_t src_len, uint8_t *dst, size_t *dst_len)
{
    DeviceGuard guard;
    const int cur = guard.dev < 0 ? 0 : guard.dev;
    if (salz_gpu_device_count() <= 0 || cur >= salz_gpu_device_count()) {
        set_error("no usable HIP device (gfx950) for salz_encode_safe");
        return -1;
    }
    salz_gpu_ctx *c = nullptr;
    for (;;) {
        bool create_failed, have_any;
        c = pool_try_acquire(cur, src_len < 9 ? 9 : src_len, &create_failed, &have_any);
        if (c)
            break;
        if (create_failed && !have_any)
            return -1;  // not even one context fits the device: report the allocation error
        std::unique_lock<std::mutex> lk(g_default_mu);
        g_pool_cv.wait_for(lk, std::chrono::milliseconds(2));
    }
    int rc = encode_host_locked(c, src, src_len, dst, dst_len, nullptr);
    c->held.store(c->ws.bytes);
    pool_trim(c->ws.device >= 0 ? c->ws.device : cur, c);
    c->mu.unlock();
    g_pool_cv.notify_one();
    return rc;
}

void salz_gpu_pool_config(int slots_per_device, size_t cache_bytes, int any_device)
{
    if (slots_per_device > 0)
        g_pool_slots.store(slots_per_device > kMaxSlots ? kMaxSlots : slots_per_device);
    if (cache_bytes > 0)
        g_pool_cap.store(cache_bytes);
    if (any_device >= 0)
        g_pool_any_dev.store(any_device ? 1 : 0);
}

size_t salz_gpu_workspace_allocs(void) { return g_ws_allocs.load(); }

size_t salz_gpu_pool_bytes(int device)
{
    std::lock_guard<std::mutex> lk(g_default_mu);
    size_t total = 0;
    if (device < 0 || (size_t)(device + 1) * kMaxSlots > g_default.size())
        return 0;
    for (int s = 0; s < kMaxSlots; s++) {
        salz_gpu_ctx *c = g_default[(size_t)device * kMaxSlots + s];
        if (c && c != kCreating)
            total += c->held.load();
    }
    return total;
}

// ---- multi-block / multi-GPU container encode ---------------------------------------------

size_t salz_blocks_len_max(size_t src_len, size_t block_size)
{
    if (block_size == 0)
        return 0;
    size_t blocks = src_len / block_size + 1;
    return 8 + blocks * 4 + (size_t)salz_encoded_len_max(block_size) * blocks;
}

}  // extern "C"

namespace {

// Batching plan of the container encoders: blocks whose size is a multiple of 512 are encoded
// kBatchBytes at a time (one pipeline pass per batch, salz_gpu_encode_batch), with 2 batches in
// flight per device; other block sizes go one block per pass with the slot counts below.
struct BatchPlan {
    size_t bpb;   // blocks per batch
    int per_dev;  // encoder contexts (slots) per device
};

BatchPlan batch_plan(size_t block_size)
{
    // Blocks of up to 4 MiB share passes: 8 MiB batches, 4 in flight per device (1 MiB blocks
    // 864 -> 2292 MB/s, 32 KiB blocks 122 -> 1746; profiles/r02h_*, r02i_*). From 8 MiB a
    // block fills the GPU on its own and four concurrent single-block passes beat batches
    // (16 MiB mixed blocks: 2045 vs 1625 with 64 MiB batches).
    const char *e = getenv("SALZ_BATCH_BYTES");  // tuning / tests
    const long long v = e ? atoll(e) : 0;
    const size_t kBatchBytes = v > 0 ? (size_t)v : (size_t)8 << 20;
    const char *se = getenv("SALZ_SLOTS");  // tuning: encoder contexts per device
    const int slots = se ? atoi(se) : 0;
    if (block_size % 512 == 0 && (block_size <= (4u << 20) || v > 0)) {
        size_t bpb = kBatchBytes / block_size;
        bpb = bpb < 1 ? 1 : bpb > kMaxBatchBlocks ? kMaxBatchBlocks : bpb;
        return {bpb, slots > 0 ? slots : 4};
    }
    return {1, slots > 0 ? slots : block_size >= (256u << 20) ? 2 : block_size >= (1u << 20) ? 4 : kMaxSlots};
}

size_t frames_cap(size_t bpb, size_t block_size)
{
    return bpb * ((size_t)salz_encoded_len_max(block_size) + 4);
}

}  // namespace

extern "C" {

int salz_encode_blocks(const uint8_t *src, size_t src_len, size_t block_size, uint8_t *dst,
                       size_t *dst_len, int n_devices)
{
    if (!src || !dst || !dst_len || block_size == 0 || block_size > 0xffffffffu) {
        set_error("invalid argument");
        return -1;
    }
    int avail = salz_gpu_device_count();
    if (avail <= 0) {
        set_error("no usable HIP device");
        return -1;
    }
    int ndev = (n_devices <= 0 || n_devices > avail) ? avail : n_devices;
    // Block count follows the reference CLI loop (programs/salzcli.c:143-179): it always
    // encodes the trailing fread() chunk, even an empty one when src_len is a multiple.
    const size_t nblocks = src_len / block_size + 1;
    if (src_len % block_size == 0) {  // the trailing block is empty: lib/salz.c:197 fails it
        set_error("block %zu: a block of 0 bytes (the input is a multiple of the block size)", nblocks - 1);
        return -1;
    }
    const BatchPlan plan = batch_plan(block_size);
    const size_t nbatches = (nblocks + plan.bpb - 1) / plan.bpb;
    int per_dev = plan.per_dev;
    const size_t per_dev_batches = (nbatches + ndev - 1) / ndev;
    if ((size_t)per_dev > per_dev_batches)
        per_dev = (int)per_dev_batches;
    std::vector<std::vector<uint8_t>> frames(nbatches);
    std::vector<int> rcs(nbatches, -1);
    std::atomic<size_t> next{0};
    std::vector<std::string> werr((size_t)ndev * per_dev);
    auto worker = [&](int dev, int slot) {
        // cached contexts (workspace reused across calls), one per batch in flight
        const size_t span = plan.bpb * block_size;
        size_t need = span < src_len ? span : src_len;
        salz_gpu_ctx *c = default_ctx(dev, need < 9 ? 9 : need, slot);
        std::string &err = werr[(size_t)dev * per_dev + slot];
        if (!c) {
            err = g_err;
            return;
        }
        for (;;) {
            size_t t = next.fetch_add(1);
            if (t >= nbatches)
                break;
            const size_t b0 = t * plan.bpb, b1 = b0 + plan.bpb < nblocks ? b0 + plan.bpb : nblocks;
            const size_t off = b0 * block_size;
            const size_t len = (b1 == nblocks ? src_len : b1 * block_size) - off;
            size_t out = frames_cap(b1 - b0, block_size);
            frames[t].resize(out);
            {
                std::lock_guard<std::mutex> lk(c->mu);
                rcs[t] = encode_batch_locked(c->ws, src + off, len, block_size, frames[t].data(), &out);
                c->held.store(c->ws.bytes);
            }
            if (rcs[t] != 0) {
                err = g_err;
                next.store(nbatches);
                break;
            }
            frames[t].resize(out);
        }
    };
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; d++)
        for (int k = 0; k < per_dev; k++)
            th.emplace_back(worker, d, k);
    for (auto &t : th)
        t.join();
    for (int d = 0; d < ndev; d++)  // the pool's per-device cache cap holds here too
        pool_trim(d, nullptr);
    size_t need = 8;
    for (size_t t = 0; t < nbatches; t++) {
        if (rcs[t] != 0) {
            std::string e;
            for (auto &s_ : werr)
                if (!s_.empty())
                    e = s_;
            set_error("batch %zu (blocks %zu..) failed: %s", t, t * plan.bpb, e.c_str());
            return -1;
        }
        need += frames[t].size();
    }
    if (need > *dst_len) {
        set_error("container exceeds destination capacity");
        return -1;
    }
    const uint32_t magic = 0x53414C5Au, bs = (uint32_t)block_size;
    size_t o = 0;
    memcpy(dst + o, &magic, 4);
    memcpy(dst + o + 4, &bs, 4);
    o += 8;
    for (size_t t = 0; t < nbatches; t++) {
        memcpy(dst + o, frames[t].data(), frames[t].size());
        o += frames[t].size();
    }
    *dst_len = o;
    return 0;
}

// ---- streaming container encode (the CLI pipeline, programs/salzcli.c:102-185) ------------
//
// One reader thread, the encoder slots, and the caller's thread as the in-order writer. A ring
// of R pinned buffers (R = slots + 2), each holding one batch of blocks (batch_plan) and its
// packed frames, bounds host memory whatever the input size; reads, H2D/encode/D2H of several
// batches and writes overlap. The block loop is the reference's: blocks are read until a short
// read, and that last (possibly empty) block is encoded too, so inputs with size mod block in
// [0, 8] fail exactly as the reference CLI does.

namespace {
struct RingSlot {
    uint8_t *in = nullptr, *out = nullptr;
    size_t in_len = 0, out_len = 0;
    size_t batch = 0;    // batch index held
    bool last = false;
    int state = 0;       // 0 free, 1 read (queued for encode), 2 encoded, 3 failed
};
}  // namespace

int salz_encode_stream(salz_read_fn rd, void *rd_user, salz_write_fn wr, void *wr_user,
                       size_t block_size, int n_devices, uint64_t *in_total, uint64_t *out_total)
{
    if (!rd || !wr || block_size == 0 || block_size > 0xffffffffu) {
        set_error("invalid argument");
        return -1;
    }
    const int avail = salz_gpu_device_count();
    if (avail <= 0) {
        set_error("no usable HIP device");
        return -1;
    }
    const int ndev = (n_devices <= 0 || n_devices > avail) ? avail : n_devices;
    const BatchPlan plan = batch_plan(block_size);
    const int per_dev = plan.per_dev;
    const int W = ndev * per_dev;
    const size_t R = (size_t)W + 2;
    const size_t span = plan.bpb * block_size;   // input bytes per batch
    const size_t cap = frames_cap(plan.bpb, block_size);
    std::vector<RingSlot> ring(R);
    auto free_ring = [&]() {
        for (RingSlot &r : ring) {
            if (r.in) (void)hipHostFree(r.in);
            if (r.out) (void)hipHostFree(r.out);
        }
    };
    // ring buffers are pinned lazily, when the reader first fills a slot: a small input touches
    // one slot, a large one all R
    std::mutex mu;
    std::condition_variable cv;
    std::deque<size_t> todo;       // ring indices waiting for an encoder, in batch order
    bool stop = false, reader_done = false;
    std::string err;
    uint64_t nin = 0, nout = 0;

    auto fail = [&](const std::string &e) {  // with mu held
        if (err.empty())
            err = e;
        stop = true;
        cv.notify_all();
    };
    auto reader = [&]() {
        size_t t = 0;
        for (;;) {
            size_t k;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || ring[t % R].state == 0; });
                if (stop)
                    break;
                k = t % R;
            }
            RingSlot &r = ring[k];
            if (!r.in && (hipHostMalloc(reinterpret_cast<void **>(&r.in), span) != hipSuccess ||
                          hipHostMalloc(reinterpret_cast<void **>(&r.out), cap) != hipSuccess)) {
                std::lock_guard<std::mutex> lk(mu);
                fail("pinned host buffers for the batch ring (" + std::to_string(span + cap) + " bytes)");
                break;
            }
            size_t got = 0;
            bool eof = false, bad = false;
            while (got < span) {  // fill the batch like fread (short only at EOF)
                const long long n = rd(rd_user, r.in + got, span - got);
                if (n < 0) { bad = true; break; }
                if (n == 0) { eof = true; break; }
                got += (size_t)n;
            }
            std::lock_guard<std::mutex> lk(mu);
            if (bad) {
                fail("read error on the input stream");
                break;
            }
            r.in_len = got;
            r.batch = t;
            r.last = eof;  // a full batch at EOF is followed by the (empty) trailing block
            r.state = 1;
            nin += got;
            todo.push_back(k);
            cv.notify_all();
            t++;
            if (r.last)
                break;
        }
        std::lock_guard<std::mutex> lk(mu);
        reader_done = true;
        cv.notify_all();
    };
    auto worker = [&](int dev, int slot) {
        salz_gpu_ctx *c = nullptr;  // created at the first batch this worker takes
        for (;;) {
            size_t k;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !todo.empty() || reader_done; });
                if (stop || (todo.empty() && reader_done))
                    break;
                k = todo.front();
                todo.pop_front();
            }
            RingSlot &r = ring[k];
            if (!c) {
                // workspace sized to this batch (a small input gets a small one; it grows on
                // demand if a later batch is larger)
                c = default_ctx(dev, r.in_len < 9 ? 9 : r.in_len, slot);
                if (!c) {
                    std::lock_guard<std::mutex> lk(mu);
                    r.state = 3;
                    fail(g_err);
                    break;
                }
            }
            size_t out = cap;
            int rc;
            if (r.last && r.in_len % block_size == 0) {
                // the trailing fread() chunk is empty: the reference fails it (lib/salz.c:197)
                set_error("a block of 0 bytes (the input is a multiple of the block size)");
                rc = -1;
            } else {
                std::lock_guard<std::mutex> lk(c->mu);
                rc = encode_batch_locked(c->ws, r.in, r.in_len, block_size, r.out, &out);
                c->held.store(c->ws.bytes);
            }
            std::lock_guard<std::mutex> lk(mu);
            if (rc != 0) {
                r.state = 3;
                fail(std::string("batch ") + std::to_string(r.batch) + ": " + g_err);
                break;
            }
            r.out_len = out;
            r.state = 2;
            cv.notify_all();
        }
    };

    const uint32_t hdr[2] = {0x53414C5Au, (uint32_t)block_size};
    if (wr(wr_user, reinterpret_cast<const uint8_t *>(hdr), 8) != 0) {
        free_ring();
        set_error("write error on the output stream");
        return -1;
    }
    nout = 8;
    std::thread rth(reader);
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; d++)
        for (int k = 0; k < per_dev; k++)
            th.emplace_back(worker, d, k);
    // in-order writer
    for (size_t t = 0;; t++) {
        RingSlot &r = ring[t % R];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || (r.state == 2 && r.batch == t); });
            if (stop)
                break;
        }
        const bool last = r.last;
        if (wr(wr_user, r.out, r.out_len) != 0) {
            std::lock_guard<std::mutex> lk(mu);
            fail("write error on the output stream");
            break;
        }
        std::lock_guard<std::mutex> lk(mu);
        nout += r.out_len;
        r.state = 0;
        cv.notify_all();
        if (last) {
            stop = true;  // done: release the reader (it has already finished) and the workers
            cv.notify_all();
            break;
        }
    }
    rth.join();
    for (auto &t : th)
        t.join();
    for (int d = 0; d < ndev; d++)  // the pool's per-device cache cap holds here too
        pool_trim(d, nullptr);
    free_ring();
    if (!err.empty()) {
        set_error("%s", err.c_str());
        return -1;
    }
    if (in_total)
        *in_total = nin;
    if (out_total)
        *out_total = nout;
    return 0;
}

}  // extern "C"
