// internal.hpp - device workspace and stage entry points of the MI355X SA-LZ pipeline.
//
// One Workspace per (device, max block size). Every array is sized for the largest block
// the context accepts and reused across calls; stages that run later alias the scratch
// of stages that ran earlier (see DESIGN.md "Data layout in HBM").
#pragma once

#include "common.hpp"
#include "../../../include/salz_gpu.h"

#include <cstdlib>
#include <vector>

namespace salz {

// Per-call statistics, filled when Workspace::timing is set (bench.py / tests).
struct StageStats {
    float ms_upload, ms_sa, ms_lcp, ms_ansv, ms_parse, ms_emit, ms_total;
    int sa_rounds;
    int parse_iters;
    uint64_t sa_sorted_elems;  // sum over rounds of active suffixes sorted
    int sa_dc3_levels;         // DC3 levels (0: prefix doubling built the suffix array)
    uint32_t exit_nodes;
    uint64_t lcp_long_bytes;
    float ms_radix_scatter;   // summed over every radix scatter launch (HIP events)
    uint32_t radix_scatter_launches;
    uint64_t radix_scatter_elems;
    uint64_t radix_scatter_bytes;
    uint64_t emit_bits, emit_bytes;
};

// Parse/emit scratch carving (parse.hip owns the layout, emit.hip reads it). Per-position
// arrays are in the chunk-interleaved layout (common.hpp, sidx with Workspace::klog).
// The parse's exit set E as bits in storage-slot order: one word per 64 slots, its popcount, and
// the exclusive scan of those (a slot's index in E = wpre + the set bits below it in its word).
struct ExitBits {
    uint64_t *mask;
    uint32_t *wcnt;
    uint32_t *wpre;
};

struct ParseState {
    ExitBits ebits;         // exit set of the last pass (read by emission's path marking)
    uint32_t chunk;         // positions per parse lane (1 << klog)
    uint32_t nchunks;
    uint8_t *choice;        // final decisions: 0 literal, 1 PSV, 2 NSV
    uint32_t *cost;         // exact suffix costs, cost[n] = 0
    uint64_t *pst;          // per position: chunk-local cost estimate << 32 | chunk exit
    uint32_t n_exit;        // |E|
    uint32_t *elist;        // E nodes (positions), ascending; last is n
    uint32_t *jt0;          // parent (compact) per E node, snapshot level 0
    uint32_t levels;        // pointer-jumping levels
    bool snaps;             // all levels stored at jt0 + k*n_exit (else emission recomputes
                            // them from level 0 in two ping-pong buffers)
    // lazy costs at the end of the parse (cost is then null until parse_materialize_cost):
    // cost = lzC + lzL[chunk], written into lzD
    uint32_t *lzC = nullptr, *lzL = nullptr, *lzD = nullptr;
    uint32_t lzn = 0;
};

struct Workspace {
    int device = -1;
    size_t cap_N = 0;  // largest block (bytes) this workspace accepts
    size_t cap_n = 0;  // cap_N - 8
    size_t np2 = 0;    // power of two >= cap_n (ANSV tree leaves)
    size_t cap_s = 0;  // storage slots of the interleaved per-position arrays (>= cap_n + 1)
    uint32_t klog = 9; // parse chunk = 1 << klog positions for the current block
    uint32_t sigma = 0; // distinct bytes of the current block, when the suffix sorter counted them

    uint8_t *text = nullptr;  // padded copy of the block
    uint32_t *rank = nullptr, *sa = nullptr;
    uint64_t *keyA = nullptr, *keyB = nullptr;  // n+1 each
    uint32_t *valA = nullptr, *valB = nullptr;
    uint32_t *u0 = nullptr, *u1 = nullptr, *u2 = nullptr, *u3 = nullptr;  // n+2 each
    uint32_t *lcps = nullptr;  // LCP array in SA order, filled by the suffix sorter (n+2)
    bool lcps_ok = false;      // lcps is complete for the current block
    uint64_t *g64 = nullptr;                                             // n+2
    uint32_t *offA = nullptr, *offB = nullptr;                           // n+2 each
    uint4 *cand = nullptr;                                               // cap_s, interleaved
    uint64_t *pst = nullptr;                                             // cap_s, interleaved
    uint64_t *lsc = nullptr;   // 2 n1: suffix sorter's large-group scan; ANSV staging (uint4)
    uint64_t *lrec = nullptr;  // per large group: (start in extracted array << 32) | start
    uint32_t *lg2g = nullptr;  // per large group: its group id
    uint8_t *dc3 = nullptr;    // DC3 suffix sorter's level arena (dc3.hip), allocated on first use
    uint8_t *dist_owner = nullptr;  // split suffix sort: owning rank per two-byte class (dsa.hip)
    size_t dc3_bytes = 0;
    size_t bytes = 0;  // device memory held by this workspace (the salz_encode_safe pool's cap)
    uint8_t *out = nullptr;                                              // encoded_len_max
    size_t out_cap = 0;
    uint32_t *radix_counts = nullptr;
    size_t radix_counts_elems = 0;
    void *scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    uint64_t *dscal = nullptr;  // device scalars
    uint64_t *hscal = nullptr;      // pinned host mirror (mapped), kHostScal bytes
    uint64_t *hscal_dev = nullptr;  // its device-side address
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool timing = false;
    StageStats stats{};
    ParseState parse{};
    hipEvent_t ev[16] = {};
    // begin/end event pairs around every radix scatter launch, resolved after the call
    std::vector<hipEvent_t> rx_pool;
    size_t rx_used = 0;
    // Pinned staging of pageable host buffers (copy_h2d / copy_d2h), two chunks ping-ponged,
    // allocated on first use: each context copies through its own, so concurrent encodes
    // from host memory do not queue on the runtime's shared staging path.
    uint8_t *hstage[2] = {nullptr, nullptr};
    hipEvent_t hstage_ev[2] = {};
};

constexpr size_t kStageChunk = 4 << 20;  // bytes per pinned staging chunk
// Host <-> device copies on ws.stream: pinned (or device) host memory goes straight to the DMA
// engine; pageable memory through the context's pinned chunks (the CPU copy of one chunk
// overlaps the DMA of the other). copy_h2d returns once the source may be reused, before the
// last DMA finishes; copy_d2h returns with the data in dst.
int copy_h2d(Workspace &ws, uint8_t *dst, const uint8_t *src, size_t bytes);
int copy_d2h(Workspace &ws, uint8_t *dst, const uint8_t *src, size_t bytes);

constexpr size_t kHostScal = 64 << 10;  // mapped host buffer: scalars below, read_device above

// Test and diagnostic switches: SALZ_DEBUG, SALZ_CHECK, SALZ_SA and SALZ_PARSE
// each hold comma-separated names, bare ("noskip") or with a value ("klog=7").
bool env_flag(const char *var, const char *name);               // `name` listed in $var
long env_num(const char *var, const char *name, long dflt);     // its value (bare name: 1)

int workspace_alloc(Workspace &ws, int device, size_t max_block);
void workspace_release(Workspace &ws);  // free the buffers, keep the device

// Copy device scalars dscal[off, off + bytes) to hscal (same offset) and wait for them.
// (zlo, nz: device words dscal[zlo, zlo + nz) zeroed after they are read)
int read_scalars(Workspace &ws, size_t off, size_t bytes, const char *tag, uint32_t zlo = 0, uint32_t nz = 0);
// Copy `bytes` of device memory to host memory `dst` through the same mapped buffer.
int read_device(Workspace &ws, const void *src, size_t bytes, void *dst);
void workspace_free(Workspace &ws);

// scans (scan.hip)
size_t scan_temp_elems(size_t n);
// hipMemsetAsync's semantics in one kernel launch (scan.hip)
hipError_t fill_async(void *ptr, int value, size_t bytes, hipStream_t st);
int scan_sum_u32(const uint32_t *in, uint32_t *out, size_t n, bool inclusive,
                 uint32_t *total_out, Workspace &ws, hipStream_t st);
int scan_max_u32(const uint32_t *in, uint32_t *out, size_t n, bool inclusive,
                 uint32_t *total_out, Workspace &ws, hipStream_t st);
// u8 flags -> u32 prefix sums
int scan_sum_u8(const uint8_t *in, uint32_t *out, size_t n, bool inclusive, uint32_t *total_out,
                Workspace &ws, hipStream_t st);
int scan_sum_u64(const uint64_t *in, uint64_t *out, size_t n, bool inclusive,
                 uint64_t *total_out, Workspace &ws, hipStream_t st);

// radix sort of (u64 key, u32 value) pairs on key bits [bit_lo, bit_hi) (radix.hip).
// On return *keys / *vals point at whichever buffer holds the sorted result.
constexpr int kRadixTile = 4096;
constexpr int kMaxDigits = 512;  // 9-bit radix digits (radix.hip)
// With `text` set, the first pass builds the round-0 suffix keys from the text itself (m =
// every live suffix of `blocks`; *keys / *vals are not read); a batch of several blocks then
// gets extra passes on the block of each value, so the result is ordered by (block, key).
// With `digits` (m bytes of scratch) every scatter pass also writes the next pass's digit of
// each key at its output position, and the next histogram reads those bytes instead of the keys
// (digits_ready: the caller wrote the first pass's digits as well).
int radix_sort_pairs(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt,
                     uint32_t m, int bit_lo, int bit_hi, Workspace &ws, hipStream_t st,
                     const uint8_t *text = nullptr, const Blocks *blocks = nullptr,
                     const Alpha *alpha = nullptr, uint8_t *digits = nullptr, bool digits_ready = false,
                     bool prefer9 = false);

// Stable radix sort of (key, value) pairs whose values are indices into the extraction ranges of
// GL large groups (lrec[g] >> 32 = start of group g's range, ascending; tmap[t] = the group of
// index 256 t, groups longer than 256): by the group of each value, so a list sorted by key
// becomes sorted by (group, key) (sa.hip's text round).
int radix_sort_by_group(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt, uint32_t m,
                        const uint64_t *lrec, const uint32_t *tmap, uint32_t GL, Workspace &ws, hipStream_t st);
// A list of whole radix tiles cut into segments sorted each on its own (sa.hip's large groups of a
// rank round): segment s owns tiles [pt0[s], pt0[s] + ptn[s]), its entries first; tile t belongs
// to segment tseg[t] and holds tcnt[t] entries; segtot: scratch of kMaxDigits words per segment.
struct SegTiles {
    const uint32_t *tseg, *tcnt, *pt0, *ptn;
    uint32_t *segtot;
    uint32_t ntiles, mvalid;  // (mvalid: entries in all, for the pass statistics)
};
constexpr uint32_t kSegScanMaxTiles = 512 * 24;  // one LDS row per digit (radix.hip k_radix_segscan)
// Stable sort of every segment on key bits [0, bits) (digits: 2 bytes per list slot of scratch).
int radix_sort_segmented(uint64_t **keys, uint32_t **vals, uint64_t *keys_alt, uint32_t *vals_alt,
                         const SegTiles &sg, int bits, Workspace &ws, hipStream_t st, uint8_t *digits);

// Blocks per batch (one pipeline pass over several blocks, common.hpp Blocks).
constexpr uint32_t kMaxBatchBlocks = 4096;

// stages; every one takes the batch geometry (one block: Blocks{0xffffffff, 1, n})
// One block's suffix array split over ranks (dsa.hip): this rank sorts the suffixes whose first
// two bytes fall in its bucket (list, m0 of them, global SA positions gbase ..); rank[i + h] of
// other buckets comes through the exchange (the caller's salz_dist_ops callbacks, or RCCL inside
// the library: salz_gpu_dist_comm).
struct DistXchg {
    virtual ~DistXchg() = default;
    // all-to-all of u32 words xsend -> xrecv, packed in rank order; recv_counts filled
    virtual int alltoall(const uint64_t *send_counts, uint64_t *recv_counts) = 0;
    virtual int allreduce_sum(uint64_t *value) = 0;
};
struct DistSa {
    DistXchg *x;
    int rank, nranks;
    const uint8_t *owner;  // device: owning rank per two-byte class (65536)
    const uint32_t *list;  // device: own suffixes in round-0 order
    uint32_t m0, gbase;
    uint32_t n;               // the block's suffixes
    uint32_t *xsend, *xrecv;  // device exchange buffers (u32 words), xcap each
    size_t xcap;
    bool text1;   // round 1 keyed by the text (no exchange before it); the same on every rank
    bool local;   // one rank: rank[i + h] is read here, no collectives at all
};
int dist_suffix_array(Workspace &ws, uint32_t n, int nranks, int rank, DistXchg *x, uint32_t *xsend,
                      uint32_t *xrecv, size_t xcap, uint64_t *offsets, uint32_t *m0_out);
int dist_keys(Workspace &ws, const DistSa &d, const uint32_t *nval, const uint32_t *ngid, uint32_t m, uint32_t h,
              int kb, uint64_t *key);
struct DistComm;  // RCCL communicator of the split suffix sort (dsa.hip, salz_gpu_dist_comm)
int dist_suffix_array_ops(Workspace &ws, uint32_t n, int nranks, int rank, const salz_dist_ops *ops, uint32_t *xsend,
                          uint32_t *xrecv, size_t xcap, uint64_t *offsets, uint32_t *m0_out);
int dist_suffix_array_comm(Workspace &ws, uint32_t n, DistComm *c, uint32_t *xsend, uint32_t *xrecv, size_t xcap,
                           uint64_t *offsets, uint32_t *m0_out);
// An idle rank (its bucket sorted after round `round`; an empty bucket: round 0, after the first
// allreduce) keeps answering the others' requests, one exchange and one allreduce per round,
// until every bucket is sorted.
int dist_idle_rounds(Workspace &ws, const DistSa &d, int round);
// The round-0 alphabet's symbol width (0: raw bytes), as stage_suffix_array computes it (sa.hip).
int block_alpha_bits(Workspace &ws, uint32_t n);
// 1 when the repetition probe (sa.hip) finds this single block of n suffixes repetitive (blocks
// of at least 2^20 suffixes: DC3, or doubling with twin pairs), 0 otherwise, -1 on failure.
int block_repetitive(Workspace &ws, uint32_t n);
int stage_suffix_array(Workspace &ws, const Blocks &bl, const DistSa *dist = nullptr);  // sa.hip -> ws.sa
// dc3.hip -> ws.sa for one block (repetitive inputs); symbols = codes.code[byte] (1..sigma) or
// byte + 1 when raw
int stage_suffix_array_dc3(Workspace &ws, const Blocks &bl, const Alpha &codes, int raw);
// dc3.hip: the DC3 arena grown to at least `bytes` (the twin-pair table of sa.hip borrows it)
uint8_t *dc3_arena_reserve(Workspace &ws, size_t bytes);
int stage_lcp(Workspace &ws, const Blocks &bl, uint32_t *lcp_out); // lcp.hip  -> lcp[r]
int stage_candidates(Workspace &ws, const Blocks &bl, const uint32_t *lcp);  // ansv.hip -> ws.cand
int stage_parse(Workspace &ws, const Blocks &bl);                  // parse.hip
int parse_materialize_cost(Workspace &ws);                         // parse.hip: lazy costs -> parse.cost
uint32_t parse_chunk_log(size_t N);                                // parse.hip: klog for N bytes
// emit.hip: block b's stream at dst + b * stride (at most cap bytes); lens[b] its length
int stage_emit(Workspace &ws, const Blocks &bl, uint32_t N_last, uint8_t *dst, size_t stride,
               size_t cap, size_t *lens);


}  // namespace salz
