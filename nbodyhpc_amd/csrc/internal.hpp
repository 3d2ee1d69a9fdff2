// Internal declarations of libnbkd.so (MI355X / gfx950).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nbkd.h"

namespace nbkd {

// Grow-only scratch for queries.  A tree holds up to NBKD_MAX_WS of them
// (Tree::ws + Tree::ws_extra): each call locks one for its whole duration, so
// calls from several host threads on one const tree run concurrently, as the
// reference's `const` query does (kdtree/src/cpp/pybind.cpp:90).
enum WsSlot {
    WS_Q = 0, WS_KEYS, WS_KEYS2, WS_ORDER, WS_TMP, WS_HIST, WS_SUMS, WS_OUTD, WS_OUTI,
    WS_COUNT, WS_OFF, WS_IDX, WS_STATS, WS_LIST, WS_LT, WS_TG, WS_CAND, WS_CCOUNT,
    WS_LIST2, WS_RSORT, WS_KTHD, WS_KTHI, WS_KB, WS_ANCH, WS_PAIR,
    // host-buffer pipeline (query.hip host_pipeline): two slots of queries and
    // of up to two result arrays
    WS_HQ0, WS_HQ1, WS_HO00, WS_HO01, WS_HO10, WS_HO11, WS_NSLOTS
};
constexpr int NBKD_MAX_WS = 4;
struct Workspace {
    std::mutex mu;
    void *p[WS_NSLOTS] = {};
    size_t cap[WS_NSLOTS] = {};
    int dev = -1; // device of the slots (set when one is allocated)
    // the last call's stream and an event recorded at its end: a call on
    // another stream first waits for it on the device (enter), since its
    // kernels may still read or write the slots when the host call returned
    hipStream_t last = nullptr;
    hipEvent_t done = nullptr;
    bool used = false;
    // the host-buffer pipeline's copy stream (non-blocking) and its events:
    // [0..1] queries in, [2..3] batch computed, [4..5] results out, per slot
    hipStream_t copy = nullptr;
    hipEvent_t pev[6] = {};
    hipError_t pipe_init(); // creates copy / pev once
    // the pipeline's two pinned host staging slots (hipHostMalloc, grow-only,
    // kept across calls: pinning is paid once per workspace, not per call)
    void *hpin[2] = {};
    size_t hpin_cap[2] = {};
    // nullptr when pinning fails or the process-wide cap (8 GiB) is reached:
    // the pipeline then streams through pageable memory
    void *host_pinned(int slot, size_t bytes);
    void free_pinned();
    // returns nullptr on failure (hip error recorded via set_error)
    void *get(int slot, size_t bytes, hipStream_t s);
    void release();
    void trim(); // with mu held: wait for the last call, free every slot
    // every workspace is listed (api.cpp) so that an out-of-memory retry can
    // trim the idle ones of its device
    Workspace();
    ~Workspace();
    Workspace(const Workspace &) = delete;
    Workspace &operator=(const Workspace &) = delete;
    hipError_t enter(hipStream_t s); // with mu held, before the first enqueue
    void leave(hipStream_t s);       // with mu held, after the last enqueue
};

// scratch this thread holds locked (a workspace, the build scratch): the
// out-of-memory retry leaves it alone (its try_lock would be the owner's)
void hold_mark(const void *p);
void hold_unmark(const void *p);
bool held_here(const void *p);

// one call's use of a workspace: lock, order after the previous call, record the end
struct WsCall {
    std::unique_lock<std::mutex> lk;
    Workspace &w;
    hipStream_t s;
    hipError_t err;
    WsCall(Workspace &w_, hipStream_t s_) : lk(w_.mu), w(w_), s(s_) {
        hold_mark(&w);
        err = w.enter(s);
    }
    // a workspace already locked by acquire_ws
    WsCall(Workspace &w_, hipStream_t s_, std::adopt_lock_t)
        : lk(w_.mu, std::adopt_lock), w(w_), s(s_) {
        hold_mark(&w);
        err = w.enter(s);
    }
    ~WsCall() {
        w.leave(s);
        hold_unmark(&w);
    }
};

constexpr int NBKD_PAD_LEAVES = 8;
constexpr int NBKD_GROUP = 8;   // points per sub-leaf group (leaf counts are multiples of 8)
constexpr int NBKD_GBLOCK = 128; // points ordered together into groups (<= 64 lanes x 2)

// Device-resident tree.  Points are SoA in tree order (the reference layout,
// kdtree/src/cpp/include/kdtree/position_array.hpp:166-271): x, y, z, original
// index; leaves are contiguous ranges.  Nodes are the reference's 16-B records.
// Split axis per depth, 2 bits each for depths 0..31 (deeper: depth % 3).
// The reference splits on depth % 3 (kdtree_impl.hpp:98-146); a tree built
// with nbkd_build_ext follows its points' extent instead (axes_for_extent).
constexpr uint64_t axes_ref() {
    uint64_t a = 0;
    for (int d = 0; d < 32; ++d) a |= (uint64_t)(d % 3) << (2 * d);
    return a;
}
constexpr uint64_t AXES_REF = axes_ref();
__host__ __device__ inline int axis_at(uint64_t axes, int depth) {
    return depth < 32 ? (int)((axes >> (2 * depth)) & 3u) : depth % 3;
}
// each depth splits the axis with the largest remaining extent (halved per
// split; ties to the lower axis): e = (1, 1, 1) gives depth % 3
uint64_t axes_for_extent(const float e[3]);

struct Tree {
    int device = 0;
    uint64_t n = 0;  // caller's point count
    uint64_t n8 = 0; // padded to a multiple of 8
    uint64_t nnodes = 0;
    int periodic = 0;
    float box = 0.0f;
    int leaf = 16; // effective leaf size max(leaf_size, 16)
    int depth = 0; // max node depth (root = 0)
    uint64_t axes = AXES_REF; // split axis per depth (axis_at)
    float *x = nullptr, *y = nullptr, *z = nullptr;
    uint32_t *idx = nullptr;
    // the same points packed (x, y, z, idx bits) per tree position: the packet
    // kernels stage a leaf with one 16-B-per-lane direct-to-LDS load and carry
    // the original id with each candidate (build.hip pack4_kernel; nbkd_set_ids
    // remaps both idx and .w)
    float4 *p4 = nullptr;
    nbkd_node *nodes = nullptr;
    // descent helpers: split value per node and the shape table
    // (count -> subtree node count, sorted by count) of this (n8, leaf)
    float *splits = nullptr;
    uint32_t *shape_c = nullptr, *shape_n = nullptr;
    int shape_len = 0;
    // per node id, leaves only: tight box lo.xyz, hi.xyz, left, right (8 words)
    uint32_t *leafinfo = nullptr;
    // 8-point groups: the points of each leaf are ordered (per run of 128) by
    // median splits on the widest axis into groups of NBKD_GROUP consecutive
    // positions; ginfo[6 g .. 6 g + 6) = the tight box of group g (positions
    // 8g .. 8g+7, real points only) as lo.x, hi.x, lo.y, hi.y, lo.z, hi.z
    float *ginfo = nullptr;
    // leaves of 65..128 points (leafsize > 64 only): per node id, the tight
    // boxes of the leaf's two halves (first cut at m = floor(count/2/8)*8), 12
    // floats: lo.xyz, hi.xyz per half (leafinfo's word order)
    float *hinfo = nullptr;
    // internal nodes' split values in the 4-level blocked heap order below
    // (hblk_blocks(depth) lines of 16 floats), or nullptr
    float *hsplit = nullptr;
    // per node id: its cell box (the root box cut by the splits on its path:
    // [0, L]^3 periodic, [-FLT_MAX, FLT_MAX]^3 otherwise) as lo.x, hi.x, lo.y,
    // hi.y, lo.z, hi.z, 0, 0 (32 B): the packet walk's stack holds node ids
    // only and reads a popped node's box here
    float *nbox = nullptr;
    float bbox_lo[3] = {0.0f, 0.0f, 0.0f}, bbox_hi[3] = {0.0f, 0.0f, 0.0f}; // of the real points
    // self queries (query.hip self_order): the device array the tree was built
    // from (nullptr for a host input), and the build's permutation (tree
    // position -> input row) once nbkd_set_ids has replaced idx's ids;
    // nullptr: idx is that permutation
    const float *src = nullptr;
    uint32_t *sidx = nullptr;
    // leaves holding padding points (FLT_MAX, n <= position id < n8): node ids
    int npad_leaves = 0;
    uint32_t pad_leaves[NBKD_PAD_LEAVES] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                            0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // nbkd_set_kth_out: self queries with device outputs also write each
    // row's last column to kth_side[row] (rows < kth_side_cap)
    mutable float *kth_side = nullptr;
    mutable uint64_t kth_side_cap = 0;
    mutable Workspace ws;
    // further workspaces for concurrent calls (created on demand, at most
    // NBKD_MAX_WS - 1), guarded by ws_mu
    mutable std::mutex ws_mu;
    mutable std::vector<std::unique_ptr<Workspace>> ws_extra;
};

// a workspace of t, locked: the first free one, else a new one (up to
// NBKD_MAX_WS), else wait for the tree's first workspace (api.cpp)
Workspace &acquire_ws(const Tree &t);
// every workspace of t locked and drained on stream s (nbkd_set_ids)
struct AllWs {
    const Tree &t;
    std::unique_lock<std::mutex> pool;
    std::vector<std::unique_lock<std::mutex>> locks;
    AllWs(const Tree &t_, hipStream_t s);
    ~AllWs();
};

// plain-value view passed to kernels
struct DevTree {
    const float *__restrict__ x;
    const float *__restrict__ y;
    const float *__restrict__ z;
    const uint32_t *__restrict__ idx;
    const float4 *__restrict__ p4;
    const nbkd_node *__restrict__ nodes;
    uint32_t n8;
    uint32_t nnodes;
    float box;
    const float *__restrict__ nbox;
};

inline DevTree view(const Tree &t) {
    return DevTree{t.x, t.y, t.z, t.idx, t.p4, t.nodes, (uint32_t)t.n8, (uint32_t)t.nnodes, t.box,
                   t.nbox};
}

// Tuning.  The production library reads no environment variable: every
// algorithm choice is its measured default, and the caller can change the
// few exposed knobs only through nbkd_set_tuning.  A build with
// -DNBKD_EXPERIMENTS (`python -m nbodyhpc_amd.build --experiments`, a separate
// library under lib/exp/) compiles in the A/B variants and lets the NBKD_*
// environment variables override the knobs.
#ifdef NBKD_EXPERIMENTS
inline const char *knob(const char *env) { return getenv(env); }
#else
inline const char *knob(const char *) { return nullptr; }
#endif
enum TuneId {
    TUNE_KNN_SEED = 0,
    TUNE_CAND_BYTES,
    TUNE_HOST_BATCH,
    TUNE_HOST_THREADS,
    TUNE_SELF_ORDER,
    TUNE_PINNED_BYTES,
    TUNE_N
};
// host memcpy split over the library's copy threads (api.cpp): the host-buffer
// pipeline's pinned staging <-> the caller's arrays; small copies stay on the
// calling thread
void host_copy(void *dst, const void *src, size_t bytes);
// the calling thread's interrupt check (nbkd_set_interrupt): true = abandon
// the call (host-buffer calls check it between batches)
bool interrupted();
double tuning(int id); // api.cpp (nbkd_set_tuning)

// error plumbing (api.cpp)
void set_error(const std::string &msg);
nbkd_status hip_fail(hipError_t e, const char *what);

#define NBKD_HIP(call)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) return ::nbkd::hip_fail(e_, #call);                          \
    } while (0)

// event timing (api.cpp)
// HIP events around a phase on stream s when nbkd_timing_enable is on (and
// `on`); name must be a string literal (kept until the events are read)
struct TimedScope {
    TimedScope(const char *name, hipStream_t s, bool on = true);
    ~TimedScope();
    const char *name_;
    hipStream_t s_;
    hipEvent_t a_ = nullptr;
    int dev_ = 0;
};
bool timing_enabled();
bool stats_enabled();
constexpr int NBKD_NSTATS = 17; // see capi.STATS_NAMES (collect kernel) + exact-kernel and retried queries
// the calling thread's counters of its last query call: zeroed when a call
// starts, summed over the call's batches (a host-buffer call runs several)
void stats_reset();
void stats_add(const uint64_t *v);

// hipMalloc that, when the device is out of memory, first returns what the
// device holds idle -- the cached tree blocks (api.cpp, tree_malloc), the build
// scratch and every workspace no call holds -- and retries once; the query
// workspace, the build scratch and DevBuf allocate through it
hipError_t malloc_or_release(void **p, size_t bytes);
void release_idle_build_scratch(int dev); // build.hip

// RAII device allocation (plain hipMalloc; freed after the stream drained).
// The stream-ordered pool (hipMallocAsync) is deliberately not used: mixing it
// with hipMalloc'd tree storage and pageable copies produced corrupted inputs.
struct DevBuf {
    void *p = nullptr;
    hipStream_t s = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() {
        if (p) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(p);
        }
    }
    hipError_t alloc(size_t bytes, hipStream_t stream) {
        s = stream;
        return malloc_or_release(&p, bytes ? bytes : 16);
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
};

// Device block cache for a tree's own arrays (api.cpp): a freed tree's blocks
// are kept per (device, size) and handed to the next allocation of that size,
// as framework caching allocators do; hipMalloc of the four n * 4-byte point
// arrays dominated a rebuild's host time.  tree_free follows a device
// synchronisation in free_tree (hipFree's own semantics).
hipError_t tree_malloc(void **p, size_t bytes);
void tree_free(void *p);


// build.hip
nbkd_status build_tree(Tree &t, const float *xyz, uint64_t n, int32_t leaf_size, bool input_dev,
                       hipStream_t s);

// The queries one collect / select pass handles (order[0 .. m)): a count known
// on the host (count == nullptr: m), or, for the retry rounds, a count the
// previous round left in device memory: m = min(*count - base, cap), 0 when
// *count <= base, and 0 unless the density mode matches (mode 1: only when the
// failures are dense, *count * 512 >= total, walked as packets of 64; mode 2:
// only when they are sparse, one query per wave).  A device-counted pass is
// launched on a fixed grid that strides over its packets, so the host never
// reads the count: the kNN call returns without waiting on the device.
struct QSpan {
    uint32_t m;            // the count, or the cap of a device-counted pass
    const uint32_t *count; // device count, or nullptr
    uint32_t base;         // this pass's first entry of the device-counted list
    uint32_t total;        // queries of the call (density test)
    int mode;              // 0: always; 1: only dense; 2: only sparse
    // a device-counted pass that is usually empty (round 1's later batches):
    // its select runs on a capped grid that strides over the wave-blocks
    // (cheap when empty) instead of one wave per 64 queries of the cap
    bool capped = false;
    // tg is indexed by the position in this pass's order (self queries: the
    // seed per tree position), not by query id
    bool tg_pos = false;
    // first pass, periodic trees: the collect appends the queries outside
    // [0, L]^3 to out_list (count at out_count) for the exact kernel
    uint32_t *out_list = nullptr;
    uint32_t *out_count = nullptr;
};
__host__ __device__ inline QSpan static_span(uint32_t m) { return QSpan{m, nullptr, 0u, 0u, 0}; }
__device__ __forceinline__ uint32_t span_m(const QSpan &s) {
    if (!s.count) return s.m;
    const uint32_t c = __builtin_amdgcn_readfirstlane(*s.count);
    if (s.mode != 0 && (((uint64_t)c * 512u >= (uint64_t)s.total) != (s.mode == 1))) return 0u;
    return c > s.base ? min(c - s.base, s.m) : 0u;
}

// (oi == nullptr: od receives only the k-th distance of each query, m floats)
// knn_collect.hip: candidate column capacity for k, and one collect + select
// pass over m queries (order[0..m) = query ids; tg = seed bounds, scaled by
// seed_mul; qpp = queries per packet, 64 or 1; failures are listed as query
// ids, or as sorted positions pos_base + i when pos_base != ~0u; retry names
// the timers)
uint32_t collect_capacity(int k);
// seed-failure retry: adaptive per-query seeds written by the first select
// pass (on by default) instead of a fixed 4x seed
bool retry_adaptive();
// fail_bits != nullptr: failures are marked at bit pos_base + gq (first pass)
// instead of appended to fail_list
nbkd_status launch_knn_collect(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                               int k, const float *tg, float seed_mul, uint32_t qpp, uint2 *cand,
                               uint32_t capg, uint32_t *ccount, float *od, uint32_t *oi,
                               uint32_t *fail_list, uint32_t *fail_count, uint32_t *fail_bits,
                               uint32_t pos_base, bool retry, bool fix_seed, bool sq, float *kb,
                               unsigned long long *stats, hipStream_t s,
                               float *kth_side = nullptr, uint32_t *pair_scratch = nullptr);

// the same pass as its two halves
nbkd_status launch_collect_pass(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                                int k, const float *tg, float seed_mul, uint32_t qpp, uint2 *cand,
                                uint32_t capg, uint32_t *ccount, bool retry, float *kb,
                                unsigned long long *stats, hipStream_t s);
nbkd_status launch_select_pass(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                               int k, const float *tg, uint32_t qpp, const uint2 *cand,
                               uint32_t capg, const uint32_t *ccount, float *od, uint32_t *oi,
                               uint32_t *fail_list, uint32_t *fail_count, uint32_t *fail_bits,
                               uint32_t pos_base, bool retry, bool fix_seed, bool sq, float *kb,
                               hipStream_t s, float *kth_side = nullptr,
                               uint32_t *pair_scratch = nullptr);
// pair_scratch (64 < k <= 128, first pass): m + 16 words; the wave select then
// runs two queries per wave where it can (knn_select_wave_pair_kernel)

// ball.hip: radius count (out_idx == nullptr) or CSR fill over m kd-ordered
// queries (periodic queries outside [0, L]^3 are skipped: query.hip answers them)
// (stats != nullptr, count mode: the instrumented instance adds its work
// counters and phase clocks there, capi.BALL_STATS_NAMES)
void launch_ball_packet(const Tree &t, const float *q, const uint32_t *order, uint32_t m, float r2,
                        uint32_t *out_count, const uint64_t *row_offsets, uint32_t *out_idx,
                        unsigned long long *stats, hipStream_t s);
// the listed periodic queries outside [0, L]^3, every point tested (fill: nout
// zeroed scratch words when out_idx is set)
// count mode with the list's length in device memory (no host read)
void launch_ball_outside_dev(const Tree &t, const float *q, const uint32_t *list,
                             const uint32_t *nout, float r2, uint32_t *out_count, hipStream_t s);
void launch_ball_outside(const Tree &t, const float *q, const uint32_t *list, uint32_t nout,
                         float r2, uint32_t *out_count, uint32_t *fill,
                         const uint64_t *row_offsets, uint32_t *out_idx, hipStream_t s);

// per-row sort of a CSR batch (row offsets `off`, nrows + 1 entries, device):
// rows of up to csr_sort_row_cap() ids in place; longer rows are appended to
// long_rows (count in *nlong, zeroed by the caller) for the caller to sort
void launch_csr_sort_rows(const uint64_t *off, uint32_t *ids, uint32_t nrows, uint32_t *long_rows,
                          uint32_t *nlong, hipStream_t s);
uint32_t csr_sort_row_cap();

// query.hip
nbkd_status query_knn(const Tree &t, const float *q, uint64_t m, int k, float *out_d,
                      uint32_t *out_i, uint32_t flags, hipStream_t s);
// distance to the k-th neighbour only (out_d: m floats)
nbkd_status query_kth(const Tree &t, const float *q, uint64_t m, int k, float *out_d,
                      uint32_t flags, hipStream_t s);
nbkd_status query_ball_count(const Tree &t, const float *q, uint64_t m, float r,
                             uint32_t *out_count, uint32_t flags, hipStream_t s);
nbkd_status query_ball_csr(const Tree &t, const float *q, uint64_t m, float r, uint64_t *offsets,
                           uint32_t *out_idx, uint64_t capacity, uint32_t flags, hipStream_t s);

// query.hip: LSD radix sort of (key, value) pairs by the low nbits of the keys,
// ping-ponging (k0, v0) <-> (k1, v1); *vout = the buffer holding the sorted values
nbkd_status sort_pairs(Workspace &ws, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1,
                       uint32_t n, int nbits, hipStream_t s, uint32_t **vout);

// deposit.hip: spheres onto a voxel grid (render_points_volume / render_points)
nbkd_status deposit(const float *xyz, const float *weight, const float *radius, uint64_t n, int gx,
                    int gy, int nz, float ppu, const float *period, int S, int mode, int x0, int wx,
                    float *out, uint32_t flags, hipStream_t s);

// order-preserving float -> uint32 key (IEEE-754 total order of non-NaN values)
__host__ __device__ inline uint32_t fkey(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float fkey_inv(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __builtin_bit_cast(float, u);
}

// 4-level blocked heap: the splits of a heap of `depth` levels, cut into
// 15-split subtrees of 4 levels, one 64-B line each (slot 15 unused), so the
// bucketing descent reads one line per 4 levels.  The real root sits at level
// o = hblk_offset(depth) of the first line, so the last level of splits ends a
// line.  Lines are stored level by level: one at block level 0, 16 >> o at
// level 1, then x16 per level; a line's 16 children are consecutive.
__host__ __device__ inline int hblk_offset(int depth) { return (4 - depth % 4) % 4; }
__host__ __device__ inline uint64_t hblk_level_lines(int j, int o) {
    return j == 0 ? 1ull : (1ull << (4 * j - o));
}
__host__ __device__ inline uint64_t hblk_blocks(int depth) {
    const int o = hblk_offset(depth);
    uint64_t b = 0;
    for (int j = 0; 4 * j < depth + o; ++j) b += hblk_level_lines(j, o);
    return b;
}
// float slot of heap index h (level l, position p within its level)
__host__ __device__ inline uint64_t hblk_slot(uint64_t h, int o) {
    const int l = 63 - __builtin_clzll(h + 1);
    const uint64_t p = h + 1 - (1ull << l);
    const int v = l + o, j = v >> 2, ll = v & 3;
    uint64_t base = 0;
    for (int jj = 0; jj < j; ++jj) base += hblk_level_lines(jj, o);
    const uint64_t loc = (1ull << ll) - 1 + (p & ((1ull << ll) - 1));
    return (base + (p >> ll)) * 16 + loc;
}

} // namespace nbkd

struct nbkd_tree {
    nbkd::Tree t;
};
