// Device helpers shared by the packet kernels (knn_collect.hip, ball.hip):
// direct-to-LDS loads, wave-local sync, the scalar-cache
// view of the node table, LDS-staged row stores and the fallback listing.
#pragma once

#include "metric.hpp"

namespace nbkd {
namespace dev {

typedef __attribute__((address_space(1))) const void *gas_ptr;
typedef __attribute__((address_space(3))) void *las_ptr;

// lanes < n copy src[lane] into dst[lane] (LDS) without passing through VGPRs
__device__ __forceinline__ void glds_f32(const float *src, float *dst, int lane, uint32_t n) {
    if ((uint32_t)lane < n)
        __builtin_amdgcn_global_load_lds((gas_ptr)(src + lane), (las_ptr)dst, 4, 0, 0);
}

// lanes < n copy the 16-B src[lane] into dst[lane] (LDS), one instruction for 64 points
__device__ __forceinline__ void glds_f4(const float4 *src, float4 *dst, int lane, uint32_t n) {
    if ((uint32_t)lane < n)
        __builtin_amdgcn_global_load_lds((gas_ptr)(src + lane), (las_ptr)dst, 16, 0, 0);
}

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt untouched): the direct-to-LDS loads have landed
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

constexpr int pow2_floor(int v) { return v >= 64 ? 64 : v >= 32 ? 32 : v >= 16 ? 16 : v >= 8 ? 8 : 4; }
constexpr int pow2_ceil(int v) { return v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : v <= 32 ? 32 : 64; }

// node records through the scalar cache: a constant-address-space view of the
// (read-only, wave-uniformly indexed) node table lowers to s_load_dwordx4
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) nbkd_node *cnode_ptr;
#else
typedef const nbkd_node *cnode_ptr;
#endif

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Staged registers j = 0..CC-1 of the 64 lanes (word (j, row) at j*64 + (row ^ j))
// are output columns c = c0 + j of row `row` (query rowq[row]; 0xFFFFFFFF = no
// query); columns outside [0, k) are skipped.  Consecutive lanes store
// consecutive columns of a row: whole rows per store instruction.
// remap != nullptr: the staged words are tree positions, stored as remap[pos]
// (0xFFFFFFFF = no neighbour, stored as is).
template <int CC>
__device__ __forceinline__ void store_rows(const uint32_t *stage, const uint32_t *rowq,
                                           uint32_t *__restrict__ dst, int k, int c0, int lane,
                                           const uint32_t *__restrict__ remap = nullptr) {
    const int jlo = c0 < 0 ? -c0 : 0;           // first staged register in [0, k)
    const int nc = min(CC, k - c0) - jlo;       // staged registers in [0, k)
    if (nc <= 0) return;
    if (nc == CC) {
        // every staged register is an output column (jlo == 0): the row and
        // column of element e = it*64 + lane are shifts of a constant, and the
        // unrolled iterations keep their LDS reads in flight together (the
        // generic loop below divides by a runtime nc and waits on each read)
        constexpr int RPI = 64 / CC; // rows per store instruction
        const int j = lane % CC, r0 = lane / CC;
#pragma unroll 8
        for (int it = 0; it < CC; ++it) {
            const int row = it * RPI + r0;
            const uint32_t qr = rowq[row];
            uint32_t v = stage[j * 64 + (row ^ j)];
            if (qr != 0xFFFFFFFFu) {
                if (remap && v != 0xFFFFFFFFu) v = remap[v];
                // rows are written once: non-temporal stores (with the
                // select's non-temporal column loads, select 14.95 -> 14.83 ms
                // per 1e8 queries, same rows, profiles/r05i_ab.txt)
                __builtin_nontemporal_store(v, &dst[(size_t)qr * k + c0 + j]);
            }
        }
        return;
    }
    for (int e = lane; e < 64 * nc; e += 64) {
        const int row = e / nc, j = jlo + (e - row * nc);
        const uint32_t qr = rowq[row];
        if (qr != 0xFFFFFFFFu) {
            uint32_t v = stage[j * 64 + (row ^ j)];
            if (remap && v != 0xFFFFFFFFu) v = remap[v];
            dst[(size_t)qr * k + c0 + j] = v;
        }
    }
}

// a seeded lane whose k-th slot still holds the sentinel id found fewer than k
// points inside its seed radius: list it for the exact kernel.  Periodic
// queries outside [0, L]^3 are already listed (outside_box_kernel), so each
// query is listed at most once.
template <bool PER>
__device__ __forceinline__ void knn_fail_check(bool valid, bool seeded, uint32_t kth_id, float qx,
                                               float qy, float qz, float L, uint32_t qo,
                                               uint32_t *fail_list, uint32_t *fail_count) {
    const bool listed =
        PER && !(qx >= 0.0f && qx <= L && qy >= 0.0f && qy <= L && qz >= 0.0f && qz <= L);
    if (valid && seeded && !listed && kth_id == 0xFFFFFFFFu)
        fail_list[atomicAdd(fail_count, 1u)] = qo;
}


// ------------------------------------------------------------------ packet walk
// The wave's depth-first walk (knn_collect.hip, ball.hip).  The macros expect in
// scope: lane, qx/qy/qz, the bound kth, L, cnodes, the walk state node / nd (its
// record while `have`) / have / wm / bx[6] / tm[3], the wave stack sp / sk_node,
// the cell boxes cboxes, the metric switch M and STATS / st (node visits in
// st[0]).
// v = lanes in `mask` ? val : old, as one v_cndmask (a select of a uniform
// value into one lane otherwise compiles to exec-masked branches)
__device__ __forceinline__ float lane_set(float old, float val, uint64_t mask) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(old), "v"(val), "s"(mask));
    return r;
}
__device__ __forceinline__ uint32_t lane_set(uint32_t old, uint32_t val, uint64_t mask) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(old), "v"(val), "s"(mask));
    return r;
}

// The wave stack holds node ids only: a pushed far child's id in lane sp of
// sk_node.  A popped node's box is read back from the tree's per-node cell
// boxes (Tree::nbox: the root box cut by the splits on the node's path, the
// values bx held when it was pushed), one s_load_dwordx8 beside the node
// record.  Round 2 kept the box in six more stack VGPRs (six selects per push,
// six readlanes per pop): collect 50.03 -> 48.80 ms, radius count 126.1 ->
// 121.8 ms at 1e8, same output SHA (profiles/r03_ab7_node_stack.txt); the
// collect kernel needs 58 VGPRs instead of 64.
struct NodeBox {
    float b[8];
};
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) NodeBox *cbox_ptr;
#else
typedef const NodeBox *cbox_ptr;
#endif

// Tried and dropped (r04s): 64-B node blocks (a node's record and its
// children's) so a descent waits on one scalar load per two levels: collect
// 46.7 -> 50.1 ms, radius count 112.3 -> 124.5 ms at 1e8
// (profiles/r04s_ab_seg_wide.txt).  The node loads mostly hit the scalar
// cache; four times the bytes per record and 12 more live SGPRs (spilled
// kernel arguments) cost more than the shorter chains save.
//
// one internal node with split axis D (compile-time): test both children for
// every lane; a single wanted child is entered, and only when both are wanted
// the lanes vote which one is near (entered) and which far (pushed, its seven
// selects under a uniform branch).  The walk branches on the node's axis, so
// no per-lane selects pick the axis.  Against the form that voted and ran the
// push's selects at every node: collect 51.96 -> 49.4 ms at 1e8 with
// knn_collect's clamped stores (profiles/r03_ab1_collect_variants.txt,
// r03_ab3_lazy_vote.txt), radius count 129.0 -> 126.1 ms (r03_ab2_push_ball.txt).
#define NBKD_GSTEP(D)                                                                              \
    {                                                                                              \
        const float split = nd.split;                                                              \
        const float qd = (D) == 0 ? qx : ((D) == 1 ? qy : qz);                                     \
        float tl, tr;                                                                              \
        if constexpr (M) {                                                                         \
            tl = box_lb_axis<M>(qd, bx[2 * (D)], split, L);                                        \
            tr = box_lb_axis<M>(qd, split, bx[2 * (D) + 1], L);                                    \
        } else {                                                                                   \
            /* plain: the child on q's side keeps the slab's bound tm[D] (the   */                 \
            /* same bits box_lb_axis gives), the other one is (q - split)^2    */                 \
            const float dd_ = qd - split;                                                          \
            const float m2_ = dd_ * dd_;                                                           \
            tl = dd_ > 0.0f ? m2_ : tm[D];                                                         \
            tr = dd_ > 0.0f ? tm[D] : m2_;                                                         \
        }                                                                                          \
        const float dl = (((D) == 0 ? tl : tm[0]) + ((D) == 1 ? tl : tm[1])) + ((D) == 2 ? tl : tm[2]); \
        const float dr = (((D) == 0 ? tr : tm[0]) + ((D) == 1 ? tr : tm[1])) + ((D) == 2 ? tr : tm[2]); \
        const uint64_t wl = __ballot(dl <= kth), wr = __ballot(dr <= kth);                         \
        bool go_right = wr != 0;                                                                   \
        if (wl != 0 && wr != 0) {                                                                  \
            const uint32_t right_votes = (uint32_t)__popcll(wm & __ballot(qd > split));            \
            const bool right_first = 2 * right_votes > (uint32_t)__popcll(wm);                     \
            const uint64_t pmask = 1ull << sp;                                                     \
            sk_node = lane_set(sk_node, right_first ? nd.left : nd.right, pmask);                  \
            ++sp;                                                                                  \
            go_right = right_first;                                                                \
        } else if (wl == 0 && wr == 0) {                                                           \
            continue;                                                                              \
        }                                                                                          \
        node = go_right ? nd.right : nd.left;                                                      \
        nd = cnodes[node];                                                                         \
        tm[D] = go_right ? tr : tl;                                                                \
        if (go_right)                                                                              \
            bx[2 * (D)] = unif(split);                                                             \
        else                                                                                       \
            bx[2 * (D) + 1] = unif(split);                                                         \
        wm = go_right ? wr : wl;                                                                   \
        have = true;                                                                               \
    }

// advance the packet walk to the next leaf some lane wants (FOUND = false: done)
#define NBKD_GWALK(FOUND, LPOS, LEND)                                                              \
    FOUND = false;                                                                                 \
    for (;;) {                                                                                     \
        if (!have) {                                                                               \
            if (sp == 0) break;                                                                    \
            --sp;                                                                                  \
            node = (uint32_t)__builtin_amdgcn_readlane((int)sk_node, sp);                          \
            {                                                                                      \
                const NodeBox nb_ = cboxes[node];                                                  \
                _Pragma("unroll") for (int a = 0; a < 6; ++a) bx[a] = nb_.b[a];                    \
            }                                                                                      \
            tm[0] = box_lb_axis<M>(qx, bx[0], bx[1], L);                                           \
            tm[1] = box_lb_axis<M>(qy, bx[2], bx[3], L);                                           \
            tm[2] = box_lb_axis<M>(qz, bx[4], bx[5], L);                                           \
            wm = __ballot((tm[0] + tm[1]) + tm[2] <= kth);                                         \
            if (wm == 0) continue;                                                                 \
            nd = cnodes[node];                                                                     \
        }                                                                                          \
        have = false;                                                                              \
        if constexpr (STATS) ++st[0];                                                              \
        if (nd.dimension < 0) {                                                                    \
            LPOS = nd.left;                                                                        \
            LEND = nd.right;                                                                       \
            FOUND = true;                                                                          \
            break;                                                                                 \
        }                                                                                          \
        if (nd.dimension == 0)                                                                     \
            NBKD_GSTEP(0)                                                                          \
        else if (nd.dimension == 1)                                                                \
            NBKD_GSTEP(1)                                                                          \
        else                                                                                       \
            NBKD_GSTEP(2)                                                                          \
    }

} // namespace dev
} // namespace nbkd
