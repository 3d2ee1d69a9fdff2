// Radius queries (NEW, SURVEY.md §8(a) a14 / §8(f) rank 1: the reference has
// no radius search): count, or list, the points with d2 <= r2 around each
// query, d2 in the reference's f32 point metric (kdtree.hpp:20-121, the a10
// formula: ((dx^2 + dy^2) + dz^2), periodic per-axis minimum image).
//
// The kNN collect kernel's packet walk with a fixed bound r2: one wave64
// walks the tree for a packet of kd-ordered queries, near child first by
// majority vote; at a leaf the queries whose ball reaches the leaf's tight box
// take part.  A query whose ball CONTAINS the tight box (an upper bound of the
// f32 d2 over the box <= r2) counts the leaf's points without evaluating them;
// the others evaluate the points staged in LDS.  The count
// (ball_count2_kernel) runs packets of 128 queries, two per lane, the partial
// ones mostly by transposed steps (lanes = points, one step = one query); the
// CSR fill (ball_fill_kernel) packets of 64, one query per lane.
//
// Tried and dropped: the kNN collect's 8-point groups here (whole groups
// counted, partial (lane, group) pairs compacted 8 lanes per pair): the same
// counts, but 161 ms against 139 ms at leafsize 64 (198 vs 163 at 32, r02n).
// The per-lane group box tests (lower and upper bound, 8 per chunk) and the
// compacted pairs cost more than the ~45 % of evaluations they save against
// the transposed count below.
//
// Periodic queries outside [0, L]^3 are excluded here (their minimum-image
// pruning is not a bound) and answered by ball_brute_kernel below.
#include <algorithm>

#include "internal.hpp"
#include "metric.hpp"
#include "packet.hpp"

namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64;
constexpr int CHUNK = 64; // one staged chunk per leaf up to leafsize 64

struct PadLeaves {
    uint32_t id[NBKD_PAD_LEAVES];
};

struct alignas(16) BallLds {
    float4 p4[CHUNK]; // the staged points: x, y, z, original id bits (Tree::p4)
};

// upper bound of the f32 d2 of point_d2_fast over every point of the box: per
// axis |fl(x - q)| is monotone in x, so it is at most the larger end value; the
// periodic minimum image only lowers it
template <bool PER>
__device__ __forceinline__ float box_ub2(float qx, float qy, float qz, const float b[6]) {
    const float ux = fmaxf(fabsf(b[0] - qx), fabsf(b[1] - qx));
    const float uy = fmaxf(fabsf(b[2] - qy), fabsf(b[3] - qy));
    const float uz = fmaxf(fabsf(b[4] - qz), fabsf(b[5] - qz));
    return (ux * ux + uy * uy) + uz * uz;
}

// The CSR fill (nbkd_query_ball_csr's second pass): 64-query packets, the
// packet walk, and at each leaf the lanes whose ball contains the tight box
// write all its ids, the partial ones loop over the staged points.  (Until
// round 5 this kernel counted too, with the transposed steps that
// ball_count2_kernel below now runs over 128-query packets.)  M: the metric's
// formulas, plain for a packet whose balls all clear the box faces.
template <bool PER, bool M>
__device__ __forceinline__ void ball_fill_walk(const DevTree &t, const uint32_t *__restrict__ linfo,
                                               const PadLeaves &pad, uint32_t *__restrict__ out_idx,
                                               BallLds &W, const int lane, const float qx,
                                               const float qy, const float qz, const float thr,
                                               const uint64_t wpos) {
    const float L = t.box;
    uint32_t sk_node = 0;
    int sp = 0;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;
    const cbox_ptr cboxes = (cbox_ptr)t.nbox;
    uint32_t node = 0;
    float bx[6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        bx[2 * a] = PER ? 0.0f : -FLT_MAX;
        bx[2 * a + 1] = PER ? L : FLT_MAX;
    }
    float tm[3] = {box_lb_axis<M>(qx, bx[0], bx[1], L), box_lb_axis<M>(qy, bx[2], bx[3], L),
                   box_lb_axis<M>(qz, bx[4], bx[5], L)};
    uint64_t wm = __ballot((tm[0] + tm[1]) + tm[2] <= thr);
    bool have = wm != 0;
    nbkd_node nd = cnodes[0]; // record of `node` while `have`
    // the shared packet walk (packet.hpp: per-axis steps, node-id stack)
    constexpr bool STATS = false;
    const float kth = thr;
    uint32_t st[1] = {0};
    (void)st;
    uint32_t cnt = 0;
    for (;;) {
        bool found;
        uint32_t lpos = 0, lend = 0;
        NBKD_GWALK(found, lpos, lend);
        if (!found) break;
        // the leaf's tight box (leafinfo lo.xyz, hi.xyz): one s_load_dwordx8
        const NodeBox lb_ = ((cbox_ptr)linfo)[node];
        const float tb[6] = {lb_.b[0], lb_.b[3], lb_.b[1], lb_.b[4], lb_.b[2], lb_.b[5]};
        const bool need = box_lb2<M>(qx, qy, qz, tb, L) <= thr;
        if (!__any(need)) continue;
        // a leaf holding padding points (FLT_MAX, never inside) is always evaluated
        bool padded = false;
#pragma unroll
        for (int j = 0; j < NBKD_PAD_LEAVES; ++j) padded |= pad.id[j] == node;
        const bool full = need && !padded && box_ub2<PER>(qx, qy, qz, tb) <= thr;
        const bool part = need && !full;
        for (uint32_t c0 = lpos; c0 < lend; c0 += CHUNK) {
            const uint32_t cn = min((uint32_t)CHUNK, lend - c0);
            wave_sync();
            glds_f4(t.p4 + c0, W.p4, lane, cn);
            wait_vm0();
            wave_sync();
            if (full) {
#pragma unroll 1
                for (uint32_t u = 0; u < cn; ++u)
                    out_idx[wpos + cnt + u] = __float_as_uint(W.p4[u].w);
                cnt += cn;
            }
            if (part) {
#pragma unroll 2
                for (uint32_t u = 0; u < cn; ++u) {
                    const float4 a = W.p4[u];
                    if (point_d2_fast<M>(qx, qy, qz, a.x, a.y, a.z, L) <= thr) {
                        out_idx[wpos + cnt] = __float_as_uint(a.w);
                        ++cnt;
                    }
                }
            }
        }
    }
}

template <bool PER>
__global__ void __launch_bounds__(TB, 8)
ball_fill_kernel(DevTree t, const uint32_t *__restrict__ linfo, const float *__restrict__ q,
                 const uint32_t *__restrict__ order, uint32_t m, float r2, PadLeaves pad,
                 const uint64_t *__restrict__ row_offsets, uint32_t *__restrict__ out_idx) {
    __shared__ BallLds Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    BallLds &W = Wl[wave];
    const uint32_t gq = (xcd_block(blockIdx.x, gridDim.x) * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;
    const bool inside =
        !PER || (qx >= 0.0f && qx <= L && qy >= 0.0f && qy <= L && qz >= 0.0f && qz <= L);
    const bool active = valid && inside;
    const float thr = active ? r2 : -INFINITY;
    const uint64_t wpos = active ? row_offsets[qo] : 0;
    // every active lane's ball clears the box faces by a margin r' > r: the
    // plain formulas then give the periodic ones' bits for every point within
    // r and fail the test for every point beyond (knn_collect.hip
    // collect_packet), so the packet walks and tests with them
    bool plain = false;
    if constexpr (PER) {
        const float r1 = sqrtf(fmaxf(r2, 0.0f)) * 1.01f + L * 1e-6f;
        const bool wf = !active || (r1 <= 0.25f * L && qx >= r1 && L - qx >= r1 && qy >= r1 &&
                                    L - qy >= r1 && qz >= r1 && L - qz >= r1);
        plain = __all(wf);
    }
    if (plain)
        ball_fill_walk<PER, false>(t, linfo, pad, out_idx, W, lane, qx, qy, qz, thr, wpos);
    else
        ball_fill_walk<PER, PER>(t, linfo, pad, out_idx, W, lane, qx, qy, qz, thr, wpos);
}

// STATS (ball_count2_kernel's instrumented instance): bst = node visits,
// points evaluated, leaves needed, transposed steps, points staged, full
// (query, leaf) pairs, partial (query, leaf) pairs, per-lane-loop chunks,
// then the s_memtime phase clocks walk / leaf test / staging wait /
// transposed steps / per-lane loop
constexpr int BALL_NST = 13;

// ------------------------------------------------------ 128-query packets (count)
// Two queries per lane: A = sorted position 128 p + lane, B = A + 64.  One walk
// and one leaf test serve 128 spatially adjacent queries, so their walk cost
// (31.7 % of the 64-query kernel's wave clocks at 1e8, r = 0.01, with 309 node
// visits and 104 leaves per packet; the leaf test 22.9 %; profiles/r05c_probes.txt)
// spreads over twice the queries, while the per-(query, leaf) work -- the
// transposed steps and the per-lane loop -- stays what it was.  The packet's
// balls cover a region only ~1.3x the volume of a 64-query packet's, so far
// fewer than twice the nodes and leaves are visited.
// NBKD_BALL_PAIRS (round 6; 0 = round 5's loop, A/B): a leaf's partial
// queries of both sets are compacted into pair-interleaved records, so the
// transposed loop runs over a uniform counter, two queries a step whose
// coordinates load as packed pairs, and writes counts into lane (rank) of two
// registers that one ds_bpermute per set maps back
#ifndef NBKD_BALL_PAIRS
#define NBKD_BALL_PAIRS 1
#endif

struct alignas(16) BallLds2 {
    float4 p4[CHUNK]; // the staged points
#if NBKD_BALL_PAIRS
    // the partial queries by rank r: record r / 2 = {x[2], y[2], z[2], -, -}
    float pq[64 * 8];
#else
    float4 qs[128];   // the packet's query coordinates (A at lane, B at 64 + lane)
#endif
};

// one internal node with split axis D for both query sets (NBKD_GSTEP's logic)
#define NBKD_GSTEP2(D)                                                                             \
    {                                                                                              \
        const float split = nd.split;                                                              \
        const float qa = (D) == 0 ? ax : ((D) == 1 ? ay : az);                                     \
        const float qb = (D) == 0 ? bx_ : ((D) == 1 ? by : bz);                                    \
        float tlA, trA, tlB, trB;                                                                  \
        if constexpr (M) {                                                                         \
            tlA = box_lb_axis<M>(qa, bx[2 * (D)], split, L);                                       \
            trA = box_lb_axis<M>(qa, split, bx[2 * (D) + 1], L);                                   \
            tlB = box_lb_axis<M>(qb, bx[2 * (D)], split, L);                                       \
            trB = box_lb_axis<M>(qb, split, bx[2 * (D) + 1], L);                                   \
        } else {                                                                                   \
            const float da_ = qa - split, ma_ = da_ * da_;                                         \
            const float db_ = qb - split, mb_ = db_ * db_;                                         \
            tlA = da_ > 0.0f ? ma_ : tmA[D];                                                       \
            trA = da_ > 0.0f ? tmA[D] : ma_;                                                       \
            tlB = db_ > 0.0f ? mb_ : tmB[D];                                                       \
            trB = db_ > 0.0f ? tmB[D] : mb_;                                                       \
        }                                                                                          \
        const float dlA = (((D) == 0 ? tlA : tmA[0]) + ((D) == 1 ? tlA : tmA[1])) + ((D) == 2 ? tlA : tmA[2]); \
        const float drA = (((D) == 0 ? trA : tmA[0]) + ((D) == 1 ? trA : tmA[1])) + ((D) == 2 ? trA : tmA[2]); \
        const float dlB = (((D) == 0 ? tlB : tmB[0]) + ((D) == 1 ? tlB : tmB[1])) + ((D) == 2 ? tlB : tmB[2]); \
        const float drB = (((D) == 0 ? trB : tmB[0]) + ((D) == 1 ? trB : tmB[1])) + ((D) == 2 ? trB : tmB[2]); \
        const uint64_t wlA = __ballot(dlA <= thrA), wrA = __ballot(drA <= thrA);                  \
        const uint64_t wlB = __ballot(dlB <= thrB), wrB = __ballot(drB <= thrB);                  \
        const bool wl = (wlA | wlB) != 0, wr = (wrA | wrB) != 0;                                   \
        bool go_right = wr;                                                                        \
        if (wl && wr) {                                                                            \
            const uint32_t votes = (uint32_t)__popcll(wmA & __ballot(qa > split)) +               \
                                   (uint32_t)__popcll(wmB & __ballot(qb > split));                \
            const bool right_first = 2 * votes > (uint32_t)(__popcll(wmA) + __popcll(wmB));        \
            const uint64_t pmask = 1ull << sp;                                                     \
            sk_node = lane_set(sk_node, right_first ? nd.left : nd.right, pmask);                  \
            ++sp;                                                                                  \
            go_right = right_first;                                                                \
        } else if (!wl && !wr) {                                                                   \
            continue;                                                                              \
        }                                                                                          \
        node = go_right ? nd.right : nd.left;                                                      \
        nd = cnodes[node];                                                                         \
        tmA[D] = go_right ? trA : tlA;                                                             \
        tmB[D] = go_right ? trB : tlB;                                                             \
        if (go_right)                                                                              \
            bx[2 * (D)] = unif(split);                                                             \
        else                                                                                       \
            bx[2 * (D) + 1] = unif(split);                                                         \
        wmA = go_right ? wrA : wlA;                                                                \
        wmB = go_right ? wrB : wlB;                                                                \
        have = true;                                                                               \
    }

// advance the walk to the next leaf a query of either set wants
#define NBKD_GWALK2(FOUND, LPOS, LEND)                                                             \
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
            tmA[0] = box_lb_axis<M>(ax, bx[0], bx[1], L);                                          \
            tmA[1] = box_lb_axis<M>(ay, bx[2], bx[3], L);                                          \
            tmA[2] = box_lb_axis<M>(az, bx[4], bx[5], L);                                          \
            tmB[0] = box_lb_axis<M>(bx_, bx[0], bx[1], L);                                         \
            tmB[1] = box_lb_axis<M>(by, bx[2], bx[3], L);                                          \
            tmB[2] = box_lb_axis<M>(bz, bx[4], bx[5], L);                                          \
            wmA = __ballot((tmA[0] + tmA[1]) + tmA[2] <= thrA);                                    \
            wmB = __ballot((tmB[0] + tmB[1]) + tmB[2] <= thrB);                                    \
            if ((wmA | wmB) == 0) continue;                                                        \
            nd = cnodes[node];                                                                     \
        }                                                                                          \
        have = false;                                                                              \
        if constexpr (STATS) ++bst[0];                                                             \
        if (nd.dimension < 0) {                                                                    \
            LPOS = nd.left;                                                                        \
            LEND = nd.right;                                                                       \
            FOUND = true;                                                                          \
            break;                                                                                 \
        }                                                                                          \
        if (nd.dimension == 0)                                                                     \
            NBKD_GSTEP2(0)                                                                         \
        else if (nd.dimension == 1)                                                                \
            NBKD_GSTEP2(1)                                                                         \
        else                                                                                       \
            NBKD_GSTEP2(2)                                                                         \
    }

// transposed count of the partial queries in rem (query j of the set at
// W.qs[base + j]) against the staged points (lanes past the chunk hold FLT_MAX,
// so their d2 is inf and no mask is needed): two queries a step, each one's
// count written into lane j of the returned register (v_writelane, lane select
// in M0, written early)
template <bool M>
__device__ __forceinline__ uint32_t ball_tcount(uint64_t rem, const float4 *qs, float ux, float uy,
                                                float uz, float r2, float L) {
    uint32_t tc = 0;
    while (rem) {
        const int j = __builtin_ctzll(rem);
        rem &= ~(1ull << j);
        asm volatile("s_mov_b32 m0, %0" : : "s"(j) : "m0");
        const float4 sq = qs[j]; // LDS broadcast
        if (rem) {
            const int j2 = __builtin_ctzll(rem);
            rem &= ~(1ull << j2);
            const float4 sq2 = qs[j2];
            const float d = point_d2_fast<M>(sq.x, sq.y, sq.z, ux, uy, uz, L);
            const float d2 = point_d2_fast<M>(sq2.x, sq2.y, sq2.z, ux, uy, uz, L);
            const uint32_t c = (uint32_t)__popcll(__ballot(d <= r2));
            const uint32_t c2 = (uint32_t)__popcll(__ballot(d2 <= r2));
            asm volatile("v_writelane_b32 %0, %1, m0\n\ts_mov_b32 m0, %2\n\ts_nop 1\n\t"
                         "v_writelane_b32 %0, %3, m0"
                         : "+v"(tc) : "s"(c), "s"(j2), "s"(c2) : "m0");
        } else {
            const float d = point_d2_fast<M>(sq.x, sq.y, sq.z, ux, uy, uz, L);
            const uint32_t c = (uint32_t)__popcll(__ballot(d <= r2));
            asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(tc) : "s"(c));
        }
    }
    return tc;
}

#if NBKD_BALL_PAIRS
// two v_writelane_b32 (lane selects in M0: one SGPR operand per VALU
// instruction), values and lanes written by SALU
__device__ __forceinline__ uint32_t write_lanes2(uint32_t old, int v0, int l0, int v1, int l1) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 1\n\tv_writelane_b32 %0, %1, m0\n\t"
                 "s_mov_b32 m0, %4\n\ts_nop 1\n\tv_writelane_b32 %0, %3, m0"
                 : "+v"(old) : "s"(v0), "s"(l0), "s"(v1), "s"(l1) : "m0");
    return old;
}

// the partial queries of ranks [i0, i1) (pair-interleaved records in pq,
// compacted by rank; i0 even, i1 - i0 <= 64) against the staged points (lanes
// past the chunk hold FLT_MAX): two queries a step; the count of rank r lands
// in lane r - i0 of the result
template <bool M>
__device__ __forceinline__ uint32_t ball_tcount_pairs(uint32_t i0, uint32_t i1, const float *pq,
                                                      float ux, float uy, float uz, float r2,
                                                      float L) {
    uint32_t tc = 0;
#pragma unroll 1
    for (uint32_t i = i0; i < i1; i += 2) {
        const float4 xy = *reinterpret_cast<const float4 *>(pq + 4 * i); // x0 x1 y0 y1
        const float2 zz = *reinterpret_cast<const float2 *>(pq + 4 * i + 4);
        const float d0 = point_d2_fast<M>(xy.x, xy.z, zz.x, ux, uy, uz, L);
        const float d1 = point_d2_fast<M>(xy.y, xy.w, zz.y, ux, uy, uz, L);
        const int c0 = __popcll(__ballot(d0 <= r2));
        const int c1 = __popcll(__ballot(d1 <= r2));
        // (uniform; readfirstlane keeps the compiler from a VGPR copy of i)
        const int iu = __builtin_amdgcn_readfirstlane((int)(i - i0));
        tc = write_lanes2(tc, c0, iu, c1, iu + 1);
    }
    return tc;
}
#endif

template <bool PER, bool M, bool STATS>
__device__ __forceinline__ void ball_walk2(const DevTree &t, const uint32_t *__restrict__ linfo,
                                           float r2, const PadLeaves &pad, uint32_t tnum,
                                           bool plain_ok, BallLds2 &W, const int lane,
                                           const float ax, const float ay, const float az,
                                           const float bx_, const float by, const float bz,
                                           const float thrA, const float thrB, uint32_t &cntA,
                                           uint32_t &cntB, uint32_t (&bst)[BALL_NST]) {
    const float L = t.box;
    uint32_t sk_node = 0;
    int sp = 0;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;
    const cbox_ptr cboxes = (cbox_ptr)t.nbox;
    uint32_t node = 0;
    float bx[6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        bx[2 * a] = PER ? 0.0f : -FLT_MAX;
        bx[2 * a + 1] = PER ? L : FLT_MAX;
    }
    float tmA[3] = {box_lb_axis<M>(ax, bx[0], bx[1], L), box_lb_axis<M>(ay, bx[2], bx[3], L),
                    box_lb_axis<M>(az, bx[4], bx[5], L)};
    float tmB[3] = {box_lb_axis<M>(bx_, bx[0], bx[1], L), box_lb_axis<M>(by, bx[2], bx[3], L),
                    box_lb_axis<M>(bz, bx[4], bx[5], L)};
    uint64_t wmA = __ballot((tmA[0] + tmA[1]) + tmA[2] <= thrA);
    uint64_t wmB = __ballot((tmB[0] + tmB[1]) + tmB[2] <= thrB);
    bool have = (wmA | wmB) != 0;
    nbkd_node nd = cnodes[0];
    uint64_t tclk = STATS ? clock64() : 0;
#define NBKD_BPH(I)                                                                                \
    do {                                                                                           \
        if constexpr (STATS) {                                                                     \
            const uint64_t t_ = clock64();                                                         \
            bst[8 + (I)] += (uint32_t)(t_ - tclk);                                                 \
            tclk = t_;                                                                             \
        }                                                                                          \
    } while (0)
    for (;;) {
        bool found;
        uint32_t lpos = 0, lend = 0;
        NBKD_GWALK2(found, lpos, lend);
        NBKD_BPH(0);
        if (!found) break;
        const NodeBox lb_ = ((cbox_ptr)linfo)[node];
        const float tb[6] = {lb_.b[0], lb_.b[3], lb_.b[1], lb_.b[4], lb_.b[2], lb_.b[5]};
        const bool needA = box_lb2<M>(ax, ay, az, tb, L) <= thrA;
        const bool needB = box_lb2<M>(bx_, by, bz, tb, L) <= thrB;
        if (!__any(needA || needB)) continue;
        bool padded = false;
#pragma unroll
        for (int j = 0; j < NBKD_PAD_LEAVES; ++j) padded |= pad.id[j] == node;
        const bool fullA = needA && !padded && box_ub2<PER>(ax, ay, az, tb) <= thrA;
        const bool fullB = needB && !padded && box_ub2<PER>(bx_, by, bz, tb) <= thrB;
        const bool partA = needA && !fullA, partB = needB && !fullB;
        if (fullA) cntA += lend - lpos;
        if (fullB) cntB += lend - lpos;
        const uint64_t pmA = __ballot(partA), pmB = __ballot(partB);
        if constexpr (STATS) {
            ++bst[2];
            bst[5] += (uint32_t)(__popcll(__ballot(fullA)) + __popcll(__ballot(fullB)));
            bst[6] += (uint32_t)(__popcll(pmA) + __popcll(pmB));
        }
        NBKD_BPH(1);
        if ((pmA | pmB) == 0) continue;
        const uint32_t nA = (uint32_t)__popcll(pmA);
        const uint32_t np = nA + (uint32_t)__popcll(pmB);
        // the plain d2 where no partial query wraps around (wrap_free)
        const bool plain_leaf =
            !M || (plain_ok && __all((!partA || wrap_free(ax, ay, az, tb, L)) &&
                                     (!partB || wrap_free(bx_, by, bz, tb, L))));
#if NBKD_BALL_PAIRS
        bool pq_written = false;
#endif
        for (uint32_t c0 = lpos; c0 < lend; c0 += CHUNK) {
            const uint32_t cn = min((uint32_t)CHUNK, lend - c0);
            wave_sync();
            glds_f4(t.p4 + c0, W.p4, lane, cn);
            wait_vm0();
            wave_sync();
            if constexpr (STATS) bst[4] += cn;
            NBKD_BPH(2);
            if (np * 8u <= cn * tnum) {
                const bool pv = (uint32_t)lane < cn;
                const float4 pl = W.p4[lane];
                const float ux = pv ? pl.x : FLT_MAX, uy = pv ? pl.y : FLT_MAX,
                            uz = pv ? pl.z : FLT_MAX;
#if NBKD_BALL_PAIRS
                // each partial query's rank: set A first, then set B
                if (!pq_written) { // once per leaf: the partial queries by rank
                    pq_written = true;
                    if (partA) {
                        const uint32_t r = mbcnt64(pmA);
                        float *r_ = W.pq + 8 * (r >> 1) + (r & 1);
                        r_[0] = ax;
                        r_[2] = ay;
                        r_[4] = az;
                    }
                    if (partB) {
                        const uint32_t r = nA + mbcnt64(pmB);
                        float *r_ = W.pq + 8 * (r >> 1) + (r & 1);
                        r_[0] = bx_;
                        r_[2] = by;
                        r_[4] = bz;
                    }
                    wave_sync();
                }
                // ranks 0..63 (all of A's), then 64..127; each batch's counts
                // go back to their queries by one ds_bpermute per set
                for (uint32_t i0 = 0; i0 < np; i0 += 64) {
                    const uint32_t i1 = min(np, i0 + 64u);
                    const uint32_t tc = plain_leaf
                                            ? ball_tcount_pairs<false>(i0, i1, W.pq, ux, uy, uz, r2, L)
                                            : ball_tcount_pairs<M>(i0, i1, W.pq, ux, uy, uz, r2, L);
                    const uint32_t rA = mbcnt64(pmA) - i0, rB = nA + mbcnt64(pmB) - i0;
                    const uint32_t cA = (uint32_t)__shfl((int)tc, (int)(rA & 63u), 64);
                    const uint32_t cB = (uint32_t)__shfl((int)tc, (int)(rB & 63u), 64);
                    if (partA && rA < 64u) cntA += cA;
                    if (partB && rB < 64u) cntB += cB;
                }
#else
                if (plain_leaf) {
                    cntA += ball_tcount<false>(pmA, W.qs, ux, uy, uz, r2, L);
                    cntB += ball_tcount<false>(pmB, W.qs + 64, ux, uy, uz, r2, L);
                } else {
                    cntA += ball_tcount<M>(pmA, W.qs, ux, uy, uz, r2, L);
                    cntB += ball_tcount<M>(pmB, W.qs + 64, ux, uy, uz, r2, L);
                }
#endif
                if constexpr (STATS) {
                    bst[3] += np;
                    bst[1] += np * cn;
                }
                NBKD_BPH(3);
            } else {
                // many partial queries: each lane loops over the staged points
                // for its two queries (one LDS read per point for both; one
                // loop per set read every point twice and, latency-bound, ran
                // the count 78.4 -> 88.2 ms per 1e8, profiles/r05f_ball_ab.txt;
                // unrolled by 2 it spilled 16 B and ran 77.2 -> 78.0 ms, r05g)
#pragma unroll 1
                for (uint32_t u = 0; u < cn; ++u) {
                    const float4 a = W.p4[u];
                    cntA += (partA && point_d2_fast<M>(ax, ay, az, a.x, a.y, a.z, L) <= thrA) ? 1u : 0u;
                    cntB += (partB && point_d2_fast<M>(bx_, by, bz, a.x, a.y, a.z, L) <= thrB) ? 1u : 0u;
                }
                if constexpr (STATS) {
                    ++bst[7];
                    bst[1] += np * cn;
                }
                NBKD_BPH(4);
            }
        }
    }
#undef NBKD_BPH
}

template <bool PER, bool STATS>
__global__ void __launch_bounds__(TB, STATS ? 4 : 8) // (the instrumented instance would spill)
ball_count2_kernel(DevTree t, const uint32_t *__restrict__ linfo, const float *__restrict__ q,
                   const uint32_t *__restrict__ order, uint32_t m, float r2, PadLeaves pad,
                   uint32_t *__restrict__ out_count, uint32_t tnum, bool plain_ok,
                   unsigned long long *__restrict__ stats) {
    __shared__ BallLds2 Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    BallLds2 &W = Wl[wave];
    const uint32_t ga = (xcd_block(blockIdx.x, gridDim.x) * WPB + wave) * 128u + lane;
    const uint32_t gb = ga + 64u;
    const bool va = ga < m, vb = gb < m;
    uint32_t oa = va ? order[ga] : 0u, ob = vb ? order[gb] : 0u;
    const float ax = va ? q[3 * (size_t)oa] : 0.0f, ay = va ? q[3 * (size_t)oa + 1] : 0.0f,
                az = va ? q[3 * (size_t)oa + 2] : 0.0f;
    const float bx_ = vb ? q[3 * (size_t)ob] : 0.0f, by = vb ? q[3 * (size_t)ob + 1] : 0.0f,
                bz = vb ? q[3 * (size_t)ob + 2] : 0.0f;
    const float L = t.box;
    const bool ina = !PER || (ax >= 0.0f && ax <= L && ay >= 0.0f && ay <= L && az >= 0.0f && az <= L);
    const bool inb = !PER || (bx_ >= 0.0f && bx_ <= L && by >= 0.0f && by <= L && bz >= 0.0f && bz <= L);
    const bool acta = va && ina, actb = vb && inb;
    const float thrA = acta ? r2 : -INFINITY, thrB = actb ? r2 : -INFINITY;
#if !NBKD_BALL_PAIRS
    W.qs[lane] = make_float4(ax, ay, az, 0.0f);
    W.qs[64 + lane] = make_float4(bx_, by, bz, 0.0f);
#endif
    bool plain = false;
    if constexpr (PER) {
        const float r1 = sqrtf(fmaxf(r2, 0.0f)) * 1.01f + L * 1e-6f;
        const bool wa = !acta || (r1 <= 0.25f * L && ax >= r1 && L - ax >= r1 && ay >= r1 &&
                                  L - ay >= r1 && az >= r1 && L - az >= r1);
        const bool wb = !actb || (r1 <= 0.25f * L && bx_ >= r1 && L - bx_ >= r1 && by >= r1 &&
                                  L - by >= r1 && bz >= r1 && L - bz >= r1);
        plain = plain_ok && __all(wa && wb);
    }
    uint32_t cntA = 0, cntB = 0;
    uint32_t bst[BALL_NST] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (plain)
        ball_walk2<PER, false, STATS>(t, linfo, r2, pad, tnum, plain_ok, W, lane, ax, ay, az, bx_,
                                      by, bz, thrA, thrB, cntA, cntB, bst);
    else
        ball_walk2<PER, PER, STATS>(t, linfo, r2, pad, tnum, plain_ok, W, lane, ax, ay, az, bx_,
                                    by, bz, thrA, thrB, cntA, cntB, bst);
    // the ids again (not kept live through the walk: registers)
    oa = acta ? order[ga] : 0u;
    ob = actb ? order[gb] : 0u;
    if (acta) out_count[oa] = cntA;
    if (actb) out_count[ob] = cntB;
    if constexpr (STATS) {
        constexpr int slot[BALL_NST] = {0, 1, 2, 3, 4, 6, 7, 8, 10, 11, 12, 13, 14};
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < BALL_NST; ++i)
                atomicAdd(&stats[slot[i]], (unsigned long long)bst[i]);
            atomicAdd(&stats[5], 1ull);
        }
    }
}

// Periodic queries outside [0, L]^3 (unvalidated input, as in the reference's
// kNN): no box bound is valid for the reference's per-axis metric there, so
// every point is tested.  Grid: x = point tiles, y = listed query.  Counts
// accumulate with atomics into out_count (zeroed first); a fill appends at
// row_offsets[q] + atomicAdd(fill[j]) (rows are sets).
constexpr int BR_ITEMS = 8;
__global__ void __launch_bounds__(TB)
ball_brute_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ list,
                  float r2, uint32_t *__restrict__ out_count, uint32_t *__restrict__ fill,
                  const uint64_t *__restrict__ row_offsets, uint32_t *__restrict__ out_idx) {
    const uint32_t j = blockIdx.y, qo = list[j];
    const float qx = q[3 * (size_t)qo], qy = q[3 * (size_t)qo + 1], qz = q[3 * (size_t)qo + 2];
    const float L = t.box;
    uint32_t c = 0;
    const uint32_t base = blockIdx.x * (uint32_t)(TB * BR_ITEMS) + threadIdx.x;
#pragma unroll
    for (int u = 0; u < BR_ITEMS; ++u) {
        const uint32_t p = base + u * TB;
        if (p < t.n8 && point_d2<true>(qx, qy, qz, t.x[p], t.y[p], t.z[p], L) <= r2) {
            if (out_idx) out_idx[row_offsets[qo] + atomicAdd(&fill[j], 1u)] = t.idx[p];
            ++c;
        }
    }
    if (out_count) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(&out_count[qo], c);
    }
}

__global__ void ball_zero_kernel(const uint32_t *__restrict__ list, uint32_t nout,
                                 uint32_t *__restrict__ out_count, uint32_t *__restrict__ fill) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nout) return;
    if (out_count) out_count[list[j]] = 0;
    if (fill) fill[j] = 0;
}

// the same for a list whose length is in device memory (count mode): fixed
// grids that stride over (query, point tile) pairs, so the host never reads it
__global__ void __launch_bounds__(TB)
ball_zero_dev_kernel(const uint32_t *__restrict__ list, const uint32_t *__restrict__ nout,
                     uint32_t *__restrict__ out_count) {
    const uint32_t c = *nout;
    for (uint32_t j = blockIdx.x * TB + threadIdx.x; j < c; j += gridDim.x * TB)
        out_count[list[j]] = 0;
}

__global__ void __launch_bounds__(TB)
ball_brute_dev_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ list,
                      const uint32_t *__restrict__ nout, uint32_t ntiles, float r2,
                      uint32_t *__restrict__ out_count) {
    const uint64_t total = (uint64_t)__builtin_amdgcn_readfirstlane(*nout) * ntiles;
    const float L = t.box;
    for (uint64_t w = blockIdx.x; w < total; w += gridDim.x) {
        const uint32_t j = (uint32_t)(w / ntiles), tile = (uint32_t)(w - (uint64_t)j * ntiles);
        const uint32_t qo = list[j];
        const float qx = q[3 * (size_t)qo], qy = q[3 * (size_t)qo + 1], qz = q[3 * (size_t)qo + 2];
        uint32_t c = 0;
        const uint32_t base = tile * (uint32_t)(TB * BR_ITEMS) + threadIdx.x;
#pragma unroll
        for (int u = 0; u < BR_ITEMS; ++u) {
            const uint32_t p = base + u * TB;
            if (p < t.n8 && point_d2<true>(qx, qy, qz, t.x[p], t.y[p], t.z[p], L) <= r2) ++c;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(&out_count[qo], c);
    }
}

// Per-row sort of a CSR batch (nbkd_query_ball_csr with NBKD_SORTED; VERDICT
// r05 #4: the rows were sorted by a Python loop on the host).  One wave per
// row: a row of up to RS_CAP ids is loaded into the wave's LDS, padded to a
// power of two >= 64 with 0xFFFFFFFF, bitonic-sorted there (each stage's
// compare-exchanges spread over the 64 lanes) and written back.  Longer rows
// are listed for query.hip, which sorts them one by one with the radix sort.
constexpr uint32_t RS_CAP = 2048;

__global__ void __launch_bounds__(TB)
csr_sort_rows_kernel(const uint64_t *__restrict__ off, uint32_t *__restrict__ ids, uint32_t nrows,
                     uint32_t *__restrict__ long_rows, uint32_t *__restrict__ nlong) {
    __shared__ uint32_t buf_all[WPB][RS_CAP];
    const int lane = threadIdx.x & 63, w = wave_id();
    uint32_t *const buf = buf_all[w];
    for (uint32_t row = blockIdx.x * WPB + w; row < nrows; row += gridDim.x * WPB) {
        const uint64_t a = off[row];
        const uint64_t len = off[row + 1] - a;
        if (len <= 1) continue;
        if (len > RS_CAP) {
            if (lane == 0) long_rows[atomicAdd(nlong, 1u)] = row;
            continue;
        }
        const uint32_t L = (uint32_t)len;
        uint32_t N = 64;
        while (N < L) N <<= 1;
        uint32_t *const src = ids + a;
        for (uint32_t i = lane; i < N; i += 64) buf[i] = i < L ? src[i] : 0xFFFFFFFFu;
        wave_sync();
        for (uint32_t size = 2; size <= N; size <<= 1)
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t i = lane; i < N / 2; i += 64) {
                    const uint32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                    const bool asc = (lo & size) == 0;
                    const uint32_t x = buf[lo], y = buf[hi];
                    if (asc ? x > y : x < y) {
                        buf[lo] = y;
                        buf[hi] = x;
                    }
                }
                wave_sync();
            }
        for (uint32_t i = lane; i < L; i += 64) src[i] = buf[i];
        wave_sync(); // the row's reads are done before the next row's loads
    }
}

} // namespace

void launch_ball_outside_dev(const Tree &t, const float *q, const uint32_t *list,
                             const uint32_t *nout, float r2, uint32_t *out_count, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)((t.n8 + TB * BR_ITEMS - 1) / (TB * BR_ITEMS));
    ball_zero_dev_kernel<<<64, TB, 0, s>>>(list, nout, out_count);
    ball_brute_dev_kernel<<<2048, TB, 0, s>>>(view(t), q, list, nout, ntiles, r2, out_count);
}

void launch_ball_outside(const Tree &t, const float *q, const uint32_t *list, uint32_t nout,
                         float r2, uint32_t *out_count, uint32_t *fill,
                         const uint64_t *row_offsets, uint32_t *out_idx, hipStream_t s) {
    if (nout == 0) return;
    ball_zero_kernel<<<(nout + TB - 1) / TB, TB, 0, s>>>(list, nout, out_count, fill);
    const dim3 grid((unsigned)((t.n8 + TB * BR_ITEMS - 1) / (TB * BR_ITEMS)), nout);
    ball_brute_kernel<<<grid, TB, 0, s>>>(view(t), q, list, r2, out_count, fill, row_offsets,
                                          out_idx);
}

void launch_ball_packet(const Tree &t, const float *q, const uint32_t *order, uint32_t m, float r2,
                        uint32_t *out_count, const uint64_t *row_offsets, uint32_t *out_idx,
                        unsigned long long *stats, hipStream_t s) {
    // transposed-count threshold: a chunk runs the transposed steps while
    // #partial queries x 8 <= #points x tnum (128-query packets: 12 measured
    // best of 8, 12, 16, 24, 32, profiles/r05g_ball_ab.txt); 0 = never
    static const uint32_t tnum = [] {
        const char *e = knob("NBKD_BALL_T");
        return e ? (uint32_t)atoi(e) : 12u;
    }();
    // NBKD_BALL_PLAIN=0 (experiments build): the periodic d2 at every leaf (A/B)
    static const bool plain_ok = [] {
        const char *e = knob("NBKD_BALL_PLAIN");
        return !(e && atoi(e) == 0);
    }();
    PadLeaves pad;
    for (int j = 0; j < NBKD_PAD_LEAVES; ++j)
        pad.id[j] = t.npad_leaves <= NBKD_PAD_LEAVES ? t.pad_leaves[j] : 0xFFFFFFFFu;
    if (out_idx) { // CSR fill: 64-query packets
        const unsigned blocks = (unsigned)((m + TB - 1) / TB);
        if (t.periodic)
            ball_fill_kernel<true><<<blocks, TB, 0, s>>>(view(t), t.leafinfo, q, order, m, r2, pad,
                                                         row_offsets, out_idx);
        else
            ball_fill_kernel<false><<<blocks, TB, 0, s>>>(view(t), t.leafinfo, q, order, m, r2,
                                                          pad, row_offsets, out_idx);
        return;
    }
    // count: 128-query packets
    const unsigned blocks2 = (unsigned)((m + 128 * WPB - 1) / (128 * WPB));
#define NBKD_BALL2(PER, STATS)                                                                     \
    ball_count2_kernel<PER, STATS><<<blocks2, TB, 0, s>>>(view(t), t.leafinfo, q, order, m, r2,   \
                                                          pad, out_count, tnum, plain_ok, stats)
    if (t.periodic) {
        if (stats) NBKD_BALL2(true, true); else NBKD_BALL2(true, false);
    } else {
        if (stats) NBKD_BALL2(false, true); else NBKD_BALL2(false, false);
    }
#undef NBKD_BALL2
}

void launch_csr_sort_rows(const uint64_t *off, uint32_t *ids, uint32_t nrows, uint32_t *long_rows,
                          uint32_t *nlong, hipStream_t s) {
    if (nrows == 0) return;
    const unsigned blocks = (unsigned)std::min<uint64_t>(((uint64_t)nrows + WPB - 1) / WPB, 8192u);
    csr_sort_rows_kernel<<<blocks, TB, 0, s>>>(off, ids, nrows, long_rows, nlong);
}

uint32_t csr_sort_row_cap() { return RS_CAP; }

} // namespace nbkd
