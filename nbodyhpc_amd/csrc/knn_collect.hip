// Collect / select kNN for gfx950: the production path for k <= 64.
//
// Reference semantics (what the rows must equal): KDTreeQuery::compute
// (kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:226-268), the leaf scan of
// kdtree_asm_systemv.asm:148-188 (insert iff d2 < current k-th) and the
// finalisation of KDTree::find_closest (kdtree/src/cpp/kdtree.cpp:133-159: sort
// by d2, sqrtf, pad with (sqrtf(FLT_MAX), 0xFFFFFFFF)).  Every exact k-nearest
// search returns the same rows (up to the order inside exact-distance ties and
// the member of a tie group kept at the k boundary, which the parity contract
// leaves free), so this path splits the reference's single traversal into two
// kernels that each map to the hardware:
//
//   collect  one wave64 = one packet of 64 kd-ordered queries (query.hip's
//            bucket sort).  The wave walks the tree once, near child first by
//            majority vote of the lanes that want the node; a leaf is scanned
//            only by the lanes whose query ball reaches its TIGHT bounding box
//            (leafinfo), its points staged in LDS by direct global->LDS loads.
//            Each query's ball is its seed radius (leaf_key3_kernel), which is
//            expected to hold k + 3.5 sqrt(k) + 3.5 points; every point inside it
//            is appended to the query's candidate column in HBM.  No top-k is
//            kept, so the kernel needs few VGPRs and ~3 KB of LDS per wave and
//            runs 8 waves per SIMD.
//   select   one lane per query merges its column 16 candidates at a time into
//            a sorted register top-k (bitonic networks) and writes the rows
//            through LDS as whole-row stores.
//
// A query whose ball holds fewer than k points (seed too small) or more than
// the column capacity is listed for the reference-exact kernel (query.hip).
#include <algorithm>

#include "internal.hpp"
#include "metric.hpp"
#include "packet.hpp"

namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64;

// Round-6 scan / column variants (A/B: scripts/build_flags.sh <name> "-DX=0"):
//   NBKD_COL_ROWMAJOR  a query's candidate column contiguous (slot s of query
//                      row r at r * capg + s) in every pass; before, the first
//                      pass's columns were blocked (16-slot blocks of 64 rows),
//                      whose store address took 5 VALU per hit instead of 2
//   NBKD_PAIR_PAD      the pair list padded to whole scan steps with pairs of a
//                      never-hitting slot (bound -inf): no per-step range test
//   NBKD_PAIR_ATOMIC   one returning LDS atomic per (pair, owner) instead of
//                      one per hit (VERDICT r05 #1a): collect 40.89 -> 38.07 ms
//                      per 1e8 queries, same rows (profiles/r06b_scan_ab.txt;
//                      the two variants above alone: 40.54)
#ifndef NBKD_COL_ROWMAJOR
#define NBKD_COL_ROWMAJOR 1
#endif
#ifndef NBKD_PAIR_PAD
#define NBKD_PAIR_PAD 1
#endif
#ifndef NBKD_PAIR_ATOMIC
#define NBKD_PAIR_ATOMIC 1
#endif
//   NBKD_SEL_FIRST     lane-per-query select, k == KC: the first 16-candidate
//                      block, sorted, IS the top-k state (the rest FLT_MAX),
//                      so it is copied in without the take and the 32-wide
//                      merge (80 compare-exchanges per query fewer), in its
//                      own instance (one instance for both: 54 VGPRs spilled,
//                      select 14.1 -> 24.0 ms; split: 14.59 -> 13.47 ms per
//                      1e8 queries, profiles/r06s_select_first_ab.txt)
#ifndef NBKD_SEL_FIRST
#define NBKD_SEL_FIRST 1
#endif
//   NBKD_WAVE_KEY64    wave selects (k > 64): a lane-exchange stage compares
//                      (d2, id) as one 64-bit key (one compare, no equal-key
//                      case) instead of two float compares: k = 100 select
//                      74.50 -> 69.07 ms per 1e8 queries, same distances, ties
//                      now by id (profiles/r06u_wave_key64_ab.txt)
#ifndef NBKD_WAVE_KEY64
#define NBKD_WAVE_KEY64 1
#endif
#ifndef NBKD_WAVE_PAIR
#define NBKD_WAVE_PAIR 4 // 64 < k <= 128: queries per wave in the first pass's wave select (0: one)
#endif
// a short first-pass column (n < k points in the seed ball): the retry's seed
// volume grows to hold NBKD_RETRY_GROW mu points at the density n measured,
// at least NBKD_RETRY_MINV x and at most 8 x
#ifndef NBKD_LOOP_AHEAD
#define NBKD_LOOP_AHEAD 1 // the re-walk rounds' (LOOP) collect with the first pass's look-ahead
#endif
#ifndef NBKD_RETRY_GROW
#define NBKD_RETRY_GROW 1.0f
#endif
#ifndef NBKD_RETRY_MINV
#define NBKD_RETRY_MINV 2.0f
#endif
#ifndef NBKD_PAIR_PREFETCH
#define NBKD_PAIR_PREFETCH 0 // (with NBKD_PAIR_PAD) the next step's pair entry read one step early
#endif

constexpr int NB = 16; // distance buckets of the bound histogram

// Bound tightening without a top-k: the seed ball [0, S) is cut into NB
// buckets of width S/NB in d2; a candidate is counted in bucket j only if
// d2 < fl((j+1) * fl(S/NB)).  Once the buckets 0..j hold >= k candidates, k
// points lie strictly inside that edge, so the k-th distance does too and it
// becomes the lane's new bound (candidates already appended beyond it are
// harmless: select keeps the k smallest).  The bucket is floor(d2 * c) with
// c = fl(fl(NB/S) * (1 + 2^-20)): the 2^-20 margin exceeds the few roundings
// (2^-24 each) between d2 * c and the edge, so the property holds without a
// check (a candidate near an edge may land one bucket high: a looser bound).
// Non-finite or tiny seeds: c = 0 and edge scale +inf (no tightening).
__device__ __forceinline__ uint32_t d2_bucket(float d, float c) {
    return min((uint32_t)(d * c), (uint32_t)(NB - 1));
}


// ---------------------------------------------------------------- group variant
// The same packet walk over a tree whose leaves are cut into 8-point groups
// with their own tight boxes (build.hip group_kernel).  At a leaf the lanes
// whose ball reaches the leaf's tight box (~12 of 64 at 1e8) are compacted;
// their (lane, group) box tests run 8 lanes per needing lane over the staged
// chunk (up to 64 points, 8 groups), and the groups reached form a pair list:
// a query evaluates only the points of groups its ball reaches (about half of
// the leaf-level count at leafsize 32, a third at 64:
// tests/tools/knn_group_estimate.py), each pair's 8 (pair, point) evaluations
// on 8 consecutive lanes.
//
// Tried and dropped: scanning groups that >= 20..44 lanes need with every
// lane (dense) instead (r02i: all-compacted was fastest); the per-lane test
// of every group before the compaction (r02s: 8 tests per lane where only
// ~12 lanes need the leaf).
//
// Tried and dropped: testing each chunk's tight box (scalar loads of leafinfo /
// hinfo) before staging it, so chunks no lane reaches skip the staging and its
// wait: collect 54.0 -> 54.2 ms (r02as; few staged chunks are unreached).
//
// Packets whose seed balls all clear the box faces walk with the plain
// (non-periodic) formulas (collect_packet): round 4, one kernel holding both
// instances of grp_packet at 56 VGPRs without spills, collect 46.95 -> 44.01
// ms per 1e8 queries, same rows (profiles/r04t_ab_packet_plain.txt).  In
// round 2 the same kernel spilled VGPRs at the 8-wave budget, and two launches
// left the wrap packets (~4 %) as a latency-bound tail (+10.9 ms), or, on a
// side stream beside the main launch, still cost +5 ms (r02f/r02g).  Round 3
// tried the plain formulas per chunk instead (the needing lanes within L/2
// of the chunk's tight box): slower (r03_ab1), and again on top of the packet
// switch in round 4 (44.01 -> 44.21 ms, r04t).
//
constexpr int GCHUNK = 64; // points staged per step (a multiple of NBKD_GROUP)
constexpr int GMAX = GCHUNK / NBKD_GROUP;

// pair entries: slot | owner lane << PR_OWNER | group << PR_G (16 bits); with
// NBKD_PAIR_PAD slot 64 is the padding pairs' query (bound -inf, never a hit)
constexpr uint32_t PR_OWNER = NBKD_PAIR_PAD ? 7 : 6, PR_G = NBKD_PAIR_PAD ? 13 : 12;
constexpr uint32_t PR_SLOT = (1u << PR_OWNER) - 1u;
constexpr uint32_t PAIR_DUMMY = 64u;

struct CollectLdsG {
    float4 sq[64 + NBKD_PAIR_PAD]; // per lane: query xyz + bound (+ the padding pairs' query)
    float scl[64]; // per lane: bucket factor (d2_bucket)
    uint32_t cnt[64];
    uint32_t hist[NB / 4][65];  // padded rows: one lane's 4 words sit in 4 banks
    float4 p4[GCHUNK];           // the staged points: x, y, z, original id bits
    float gb[6 * GMAX];          // the chunk's group boxes (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z)
    float tb[8];                 // the leaf's tight box (leafinfo words 0..5)
    uint16_t pairs[64 * GMAX];   // (slot, lane, group) pairs: slot | lane << PR_OWNER | group << PR_G
    uint8_t slot[64];            // lanes needing the leaf, compacted
};

// a chunk of CN points at LPOS, its group boxes and its tight box TBOX (6
// words: lo.xyz, hi.xyz)
#define NBKD_COLLECT_STAGE_G(LPOS, CN, TBOX)                                                       \
    do {                                                                                           \
        glds_f4(t.p4 + (LPOS), W.p4, lane, (CN));                                                  \
        glds_f32(ginfo + 6 * (size_t)((LPOS) / NBKD_GROUP), W.gb, lane, 6 * ((CN) / NBKD_GROUP));  \
        glds_f32((TBOX), W.tb, lane, 6);                                                           \
    } while (0)

// st: node visits, leaves scanned, points staged, leaves reached, sparse
// iterations, pair evaluations, then 6 phase clocks, then lanes needing a
// staged chunk summed over chunks (STATS only)
template <bool PER, bool M, bool STATS, bool AHEAD>
__device__ __forceinline__ void grp_packet(const DevTree &t, const float *__restrict__ ginfo,
                                           const uint32_t *__restrict__ linfo,
                                           const float *__restrict__ hinfo,
                                           CollectLdsG &W, const int lane, const float qx,
                                           const float qy, const float qz, float &kth,
                                           const float s_over_nb, const float nb_over_s,
                                           uint2 *__restrict__ col, const uint32_t qpp,
                                           const uint32_t capg, const int kq, uint32_t &cnt,
                                           uint32_t (&st)[13]) {
    const float L = t.box;
    uint32_t last_cnt = 0;
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
    uint64_t wm = __ballot((tm[0] + tm[1]) + tm[2] <= kth);
    bool have = wm != 0;
    nbkd_node nd = cnodes[0]; // record of `node` while `have`
    uint64_t tclk = STATS ? clock64() : 0;
#define NBKD_PH(I)                                                                                 \
    do {                                                                                           \
        if constexpr (STATS) {                                                                     \
            const uint64_t t_ = clock64();                                                         \
            st[6 + (I)] += (uint32_t)(t_ - tclk);                                                              \
            tclk = t_;                                                                             \
        }                                                                                          \
    } while (0)
    uint32_t pa = 0, ea = 0;
    // AHEAD: while a leaf's staging loads are in flight the walk goes on to the
    // next leaf (its node loads are scalar, lgkmcnt, so the staging's vmcnt wait
    // does not wait for them); the walk ahead prunes with the bounds from before
    // this leaf's scan, which are looser, so it may reach a leaf the tightened
    // bounds would skip: no lane then needs it (the per-leaf test below uses the
    // current bounds), never a wrong result
    bool ha_next = false;
    uint32_t pa_next = 0, ea_next = 0, node_next = 0;
    if constexpr (AHEAD) {
        NBKD_GWALK(ha_next, pa_next, ea_next);
        node_next = node;
    }
    for (;;) {
        bool ha;
        uint32_t lnode;
        if constexpr (AHEAD) {
            ha = ha_next;
            pa = pa_next;
            ea = ea_next;
            lnode = node_next;
        } else {
            NBKD_GWALK(ha, pa, ea);
            lnode = node;
        }
        if (!ha) break;
        if constexpr (STATS) ++st[3]; // leaves reached (staged), needed by some lane or not
        // chunks: a leaf of 65..128 points is staged as its two halves, each
        // with its own tight box (hinfo); other leaves in runs of 64 points
        // under the leaf's tight box (leafinfo)
        const uint32_t lend = ea;
        const uint32_t lc = lend - pa;
        const bool halves = hinfo != nullptr && lc > (uint32_t)GCHUNK && lc <= 2u * GCHUNK;
        const uint32_t hm = (lc / 2) / 8 * 8;
        const float *const lbox = halves ? hinfo + 12 * (size_t)lnode
                                         : reinterpret_cast<const float *>(linfo) + 8 * (size_t)lnode;
        uint32_t c0 = pa;
        uint32_t cn = halves ? hm : min((uint32_t)GCHUNK, lc);
        NBKD_COLLECT_STAGE_G(pa, cn, lbox);
        NBKD_PH(0);
        if constexpr (AHEAD) {
            NBKD_GWALK(ha_next, pa_next, ea_next);
            node_next = node;
            NBKD_PH(0);
        }
        // Tried and dropped (r04aa): pulling the next leaf's lines (points,
        // group boxes, tight box) toward L2 here with one 4-B direct-to-LDS
        // load per line, waiting vmcnt(1) for this leaf's staging only:
        // collect 43.68 -> 46.97 ms per 1e8 (profiles/r04aa_ab_prefetch_anchor.txt)
        wait_vm0();
        wave_sync();
        NBKD_PH(1);
        bool any_leaf = false;
        for (;;) {
            const uint32_t ng = cn / NBKD_GROUP;
            // the lanes whose ball reaches the leaf's tight box (leafinfo);
            // ~12 of 64 on average at 1e8, so the group tests run compacted
            const float tb[6] = {W.tb[0], W.tb[3], W.tb[1], W.tb[4], W.tb[2], W.tb[5]};
            const bool need = box_lb2<M>(qx, qy, qz, tb, L) <= kth;
            const uint64_t nm = __ballot(need);
            if (nm != 0) {
                any_leaf = true;
                const uint32_t nneed = (uint32_t)__popcll(nm);
                if constexpr (STATS) {
                    st[2] += cn;
                    st[12] += nneed;
                }
                W.cnt[lane] = cnt;
                // the needing lanes' queries by compacted slot: 8 consecutive
                // slots per 64 lanes below read 8 distinct, adjacent LDS words
                // (indexed by lane, owners 16 apart hit the same banks)
                if (need) {
                    const uint32_t r = mbcnt64(nm);
                    W.slot[r] = (uint8_t)lane;
                    W.sq[r] = make_float4(qx, qy, qz, kth);
                    W.scl[r] = nb_over_s;
                }
                wave_sync();
                // (needing lane, group) box tests, 8 lanes per needing lane (one
                // per group); the groups reached become the pair list, entries
                // slot | owner lane << 6 | group << 12
                uint32_t np = 0;
                const uint32_t ntest = nneed * GMAX;
#pragma unroll 1
                for (uint32_t t0 = 0; t0 < ntest; t0 += 64) {
                    const uint32_t ti = t0 + lane;
                    const uint32_t g = ti % GMAX;
                    const uint32_t sl = ti / GMAX;
                    uint32_t owner = 0;
                    bool hit = false;
                    if (ti < ntest && g < ng) {
                        owner = W.slot[sl];
                        const float4 qq = W.sq[sl];
                        const float gbx[6] = {W.gb[6 * g], W.gb[6 * g + 1], W.gb[6 * g + 2],
                                              W.gb[6 * g + 3], W.gb[6 * g + 4], W.gb[6 * g + 5]};
                        hit = box_lb2<M>(qq.x, qq.y, qq.z, gbx, L) <= qq.w;
                    }
                    const uint64_t hm = __ballot(hit);
                    if (hit)
                        W.pairs[np + mbcnt64(hm)] = (uint16_t)(sl | (owner << PR_OWNER) | (g << PR_G));
                    np += (uint32_t)__popcll(hm);
                }
                if constexpr (STATS) st[5] += np * NBKD_GROUP; // (pair, point) evaluations
#if NBKD_PAIR_PAD
                // whole scan steps: the last one's missing pairs never hit
                const uint32_t npp = (np + 7u) & ~7u;
                if ((uint32_t)lane < npp - np) W.pairs[np + lane] = (uint16_t)PAIR_DUMMY;
                np = npp;
#endif
                NBKD_PH(2);
                wave_sync();
                // Tried and dropped (r04s): the hit's column slot as the owner's
                // count plus the hits below it in its run of lanes (the pair list
                // is slot-major), with no returning LDS atomic and all of a step's
                // LDS reads issued together: collect 46.7 -> 55.1 ms per 1e8
                // queries (profiles/r04s_ab_seg_wide.txt); the 64-bit lane-mask
                // arithmetic costs more issue than the atomics' waits.
                // each pair's 8 points spread over 8 consecutive lanes
                const uint32_t ntrip = np * NBKD_GROUP;
#if NBKD_PAIR_PAD && NBKD_PAIR_PREFETCH
                // the next step's pair entry is read while this step computes
                uint32_t pr_next = ntrip ? W.pairs[(uint32_t)lane >> 3] : 0u;
#endif
#pragma unroll 1
                for (uint32_t t0 = 0; t0 < ntrip; t0 += 64) {
                    if constexpr (STATS) ++st[4];
#if NBKD_PAIR_PAD
                    // every lane of every step holds a pair (padding pairs never hit)
                    {
#if NBKD_PAIR_PREFETCH
                        const uint32_t pr = pr_next;
                        if (t0 + 64 < ntrip) pr_next = W.pairs[((t0 + 64) >> 3) + ((uint32_t)lane >> 3)];
#else
                        const uint32_t pr = W.pairs[(t0 >> 3) + ((uint32_t)lane >> 3)];
#endif
                        const uint32_t pi = (pr >> PR_G) * NBKD_GROUP + ((uint32_t)lane & 7u);
#else
                    const uint32_t ti = t0 + lane;
                    if (ti < ntrip) {
                        const uint32_t pr = W.pairs[ti / NBKD_GROUP];
                        const uint32_t pi = (pr >> PR_G) * NBKD_GROUP + (ti % NBKD_GROUP);
#endif
                        const uint32_t qs = pr & PR_SLOT, owner = (pr >> PR_OWNER) & 63u;
                        const float4 qq = W.sq[qs];
                        const float4 pp = W.p4[pi];
                        const float d = point_d2_fast<M>(qq.x, qq.y, qq.z, pp.x, pp.y, pp.z, L);
#if NBKD_PAIR_ATOMIC
                        // the hits of a pair (8 consecutive lanes, one owner):
                        // ranked by mbcnt inside the 8-lane group, one returning
                        // atomic by the group's last lane, its base broadcast by
                        // two DPP moves (quad broadcast of lane 3, half-row mirror)
                        const bool hit = d < qq.w;
                        const uint64_t hm = __ballot(hit);
                        const uint32_t gbits = (uint32_t)(hm >> ((uint32_t)lane & ~7u)) & 0xFFu;
                        const uint32_t rank = __popc(gbits & ((1u << ((uint32_t)lane & 7u)) - 1u));
                        uint32_t base = 0;
                        if (((uint32_t)lane & 7u) == 7u && gbits != 0u)
                            base = atomicAdd(&W.cnt[owner], (uint32_t)__popc(gbits));
                        // quad_perm [3,3,3,3]: lanes 0-3 of the group read lane 3, 4-7 lane 7;
                        // row_half_mirror into banks 0 and 2 only: lanes 0-3 read 7-4
                        base = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)base, 0xFF, 0xF, 0xF, false);
                        base = (uint32_t)__builtin_amdgcn_update_dpp((int)base, (int)base, 0x141, 0xF, 0x5,
                                                                     false);
                        if (hit) {
                            const uint32_t j = d2_bucket(d, W.scl[qs]);
                            atomicAdd(&W.hist[j >> 2][owner], 1u << (8 * (j & 3)));
                            const uint32_t sl = base + rank;
#else
                        if (d < qq.w) {
                            const uint32_t j = d2_bucket(d, W.scl[qs]);
                            atomicAdd(&W.hist[j >> 2][owner], 1u << (8 * (j & 3)));
                            const uint32_t sl = atomicAdd(&W.cnt[owner], 1u);
#endif
                            // a row past capg is a failure whose column is never read (both
                            // selects): its extra hits overwrite its last slot (no branch)
                            const uint32_t sw = min(sl, capg - 1u);
                            // the candidate carries the point's original id (p4.w):
                            // the selects write it without a gather
                            // a 32-bit byte offset from the packet's (SGPR) column base:
                            // one saddr store, no 64-bit address arithmetic per hit
#if NBKD_COL_ROWMAJOR
                            const uint32_t off = (__umul24(owner, capg) + sw) << 3;
#else
                            const uint32_t off = (((__umul24(sw >> 4, qpp) + owner) << 4) | (sw & 15u)) << 3;
#endif
                            *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(col) + off) =
                                make_uint2(__float_as_uint(d), __float_as_uint(pp.w));
                        }
                    }
                }
                wave_sync();
                cnt = W.cnt[lane];
                NBKD_PH(4);
            }
            c0 += cn;
            if (c0 >= lend) {
                if constexpr (STATS) st[1] += any_leaf ? 1 : 0;
                // tighten: smallest bucket edge with >= k candidates below it
                // (after every leaf that added candidates; re-tightening only
                // after 3 or 6 more was slower, 63.66 -> 64.00 / 63.98 ms per
                // 1e8 step: the staler bound costs the select more than the
                // skipped passes save, profiles/r04ag_ab_tighten_delta.txt)
                const bool upd = cnt >= (uint32_t)kq && cnt != last_cnt;
                if (__any(upd)) {
                    wave_sync();
                    if (upd) {
                        last_cnt = cnt;
                        const uint32_t p0 = W.hist[0][lane] * 0x01010101u;
                        const uint32_t p1 = W.hist[1][lane] * 0x01010101u;
                        const uint32_t p2 = W.hist[2][lane] * 0x01010101u;
                        const uint32_t p3 = W.hist[3][lane] * 0x01010101u;
                        const uint32_t c0w = p0 >> 24, c1w = c0w + (p1 >> 24), c2w = c1w + (p2 >> 24);
                        const uint32_t kk = (uint32_t)kq;
                        const uint32_t w = c0w >= kk ? 0u : c1w >= kk ? 1u : c2w >= kk ? 2u : 3u;
                        const uint32_t base = w == 0 ? 0u : w == 1 ? c0w : w == 2 ? c1w : c2w;
                        const uint32_t pw = w == 0 ? p0 : w == 1 ? p1 : w == 2 ? p2 : p3;
                        const uint32_t need_k = kk - base;
                        const uint32_t nb = (((pw & 0xFFu) < need_k) ? 1u : 0u) +
                                            ((((pw >> 8) & 0xFFu) < need_k) ? 1u : 0u) +
                                            ((((pw >> 16) & 0xFFu) < need_k) ? 1u : 0u) +
                                            (((pw >> 24) < need_k) ? 1u : 0u);
                        const uint32_t jstar = 4 * w + nb;
                        if (jstar < (uint32_t)(NB - 1))
                            kth = fminf(kth, (float)(jstar + 1) * s_over_nb);
                    }
                }
                NBKD_PH(5);
                break;
            }
            cn = halves ? lc - hm : min((uint32_t)GCHUNK, lend - c0);
            wave_sync();
            NBKD_COLLECT_STAGE_G(c0, cn, halves ? lbox + 6 : lbox);
            wait_vm0();
            wave_sync();
        }
        wave_sync();
    }
    NBKD_PH(0);
#undef NBKD_PH
}

// one packet of the collect pass
template <bool PER, bool STATS, bool AHEAD>
__device__ __forceinline__ void collect_packet(
    const DevTree &t, const float *__restrict__ ginfo, const uint32_t *__restrict__ linfo,
    const float *__restrict__ hinfo, const float *__restrict__ q, const uint32_t *__restrict__ order,
    uint32_t m, int kq, const float *__restrict__ tg, bool tg_pos, float seed_mul, uint32_t qpp,
    uint2 *__restrict__ cand, uint32_t capg, uint32_t *__restrict__ ccount,
    unsigned long long *__restrict__ stats, float *__restrict__ kbound, CollectLdsG &W, int lane,
    uint32_t pk, uint32_t *__restrict__ out_list, uint32_t *__restrict__ out_count) {
    const uint32_t gq = pk * qpp + lane;
    const bool valid = (uint32_t)lane < qpp && gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    // the first pass lists the periodic queries outside [0, L]^3 for the
    // exact kernel (QSpan::out_list; until round 6 a separate outside_box_kernel
    // pass re-read every query); the packet still walks them, and their
    // select skips them as failures (mark_failure)
    if constexpr (PER) {
        if (out_list && valid &&
            !(qx >= 0.0f && qx <= t.box && qy >= 0.0f && qy <= t.box && qz >= 0.0f && qz <= t.box))
            out_list[atomicAdd(out_count, 1u)] = qo;
    }
    const float seed = valid ? fminf(tg[tg_pos ? gq : qo] * seed_mul, FLT_MAX) : -INFINITY;
    const bool fin = seed < FLT_MAX && seed >= 1e-30f;
    const float s_over_nb = fin ? seed * (1.0f / NB) : (seed > 0.0f ? INFINITY : 0.0f);
    const float nb_over_s = fin ? (float)NB / seed * 1.00000095367431640625f : 0.0f;
#pragma unroll
    for (int w = 0; w < NB / 4; ++w) W.hist[w][lane] = 0u;
#if NBKD_PAIR_PAD
    if (lane == 0) W.sq[PAIR_DUMMY] = make_float4(0.0f, 0.0f, 0.0f, -INFINITY);
#endif
    uint2 *const col = cand + (size_t)pk * qpp * capg;
    uint32_t cnt = 0;
    // per-packet work counters and phase clocks (STATS only): 32 bits each, so
    // the instrumented instance keeps them in SGPRs without spilling
    uint32_t st[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float kth = seed;
    // Every lane's seed ball clears the box faces (a margin r' > sqrt(seed) on
    // every axis): a point within the ball is then within L/2 of the query on
    // every axis, where the plain per-axis distance has the periodic minimum's
    // bits (metric.hpp point_d2_fast), and a point beyond it fails both tests.
    // So the packet walks with the plain formulas: the same candidates, the
    // same d2 bits, box bounds that are valid for every point that can be a
    // candidate.  The bound only shrinks, so the test at the start holds for
    // the whole walk.
    bool plain = false;
    if constexpr (PER) {
        const float r1 = sqrtf(fmaxf(seed, 0.0f)) * 1.01f + t.box * 1e-6f;
        const bool wf = !valid || (fin && r1 <= 0.25f * t.box && qx >= r1 && t.box - qx >= r1 &&
                                   qy >= r1 && t.box - qy >= r1 && qz >= r1 && t.box - qz >= r1);
        plain = __all(wf);
    }
    if (plain)
        grp_packet<PER, false, STATS, AHEAD>(t, ginfo, linfo, hinfo, W, lane, qx, qy, qz, kth,
                                             s_over_nb, nb_over_s, col, qpp, capg, kq, cnt, st);
    else
        grp_packet<PER, PER, STATS, AHEAD>(t, ginfo, linfo, hinfo, W, lane, qx, qy, qz, kth,
                                           s_over_nb, nb_over_s, col, qpp, capg, kq, cnt, st);
    if (valid) ccount[gq] = cnt;
    // the final bound: at least k candidates lie strictly below it (bound
    // histogram), so none at or above it is among the k smallest
    if (valid && kbound) kbound[gq] = kth;
    if (STATS && lane == 0) {
        atomicAdd(&stats[0], (unsigned long long)st[0]);
        atomicAdd(&stats[1], (unsigned long long)st[5]);
        atomicAdd(&stats[2], (unsigned long long)st[3]);
        atomicAdd(&stats[3], (unsigned long long)st[4]);
        atomicAdd(&stats[4], (unsigned long long)st[2]);
        atomicAdd(&stats[5], 1ull);
        atomicAdd(&stats[7], (unsigned long long)st[1]);
#pragma unroll
        for (int i = 0; i < 6; ++i) atomicAdd(&stats[10 + i], (unsigned long long)st[6 + i]);
        atomicAdd(&stats[16], (unsigned long long)st[12]);
    }
    if (STATS) {
        uint32_t c = valid ? cnt : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) atomicAdd(&stats[6], (unsigned long long)c);
    }
}

// A static pass launches one wave per packet; a device-counted pass (the
// retry rounds: LOOP) a fixed grid that strides over its packets.  Only the
// LOOP instance carries the loop (in the first pass it cost a 12-28 B spill).
template <bool PER, int OCC, bool STATS, bool LOOP, bool AHEAD>
__global__ void __launch_bounds__(TB, OCC)
knn_collect_grp_kernel(DevTree t, const float *__restrict__ ginfo,
                       const uint32_t *__restrict__ linfo, const float *__restrict__ hinfo,
                       const float *__restrict__ q,
                       const uint32_t *__restrict__ order, QSpan span, int kq,
                       const float *__restrict__ tg, float seed_mul, uint32_t qpp,
                       uint2 *__restrict__ cand, uint32_t capg,
                       uint32_t *__restrict__ ccount, unsigned long long *__restrict__ stats,
                       bool xcd, float *__restrict__ kbound) {
    __shared__ CollectLdsG Wl[WPB];
    const int lane = threadIdx.x & 63, wave = wave_id();
    CollectLdsG &W = Wl[wave];
    const uint32_t m = span_m(span);
    const uint32_t npk = (m + qpp - 1) / qpp;
    const uint32_t bid = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    if constexpr (LOOP) {
        for (uint32_t pk = bid * WPB + wave; pk < npk; pk += gridDim.x * WPB) {
            wave_sync(); // the previous packet's LDS reads are done
            collect_packet<PER, STATS, AHEAD>(t, ginfo, linfo, hinfo, q, order, m, kq, tg, span.tg_pos,
                                              seed_mul, qpp, cand, capg, ccount, stats, kbound,
                                              W, lane, pk, span.out_list, span.out_count);
        }
    } else {
        const uint32_t pk = bid * WPB + wave;
        if (pk < npk)
            collect_packet<PER, STATS, AHEAD>(t, ginfo, linfo, hinfo, q, order, m, kq, tg, span.tg_pos,
                                              seed_mul, qpp, cand, capg, ccount, stats, kbound,
                                              W, lane, pk, span.out_list, span.out_count);
    }
}

// a query whose seed ball held fewer than k points (or more than the column):
// marked in the failure bitmap at its sorted position (first pass: the next
// round reads the bitmap in kd order), else appended by query id to the next
// round's list.  Periodic queries outside [0, L]^3 are listed for the exact
// kernel already (outside_box_kernel).
template <bool PER>
__device__ __forceinline__ void mark_failure(float qx, float qy, float qz, float L, uint32_t id,
                                             uint32_t *fail_list, uint32_t *fail_count,
                                             uint32_t *fail_bits) {
    if (PER && !(qx >= 0.0f && qx <= L && qy >= 0.0f && qy <= L && qz >= 0.0f && qz <= L)) return;
    if (fail_bits)
        atomicOr(&fail_bits[id >> 5], 1u << (id & 31u));
    else
        fail_list[atomicAdd(fail_count, 1u)] = id;
}

// One 8-KB candidate block (64 rows x 8 pieces of 16 B, row-contiguous) into
// LDS by direct loads, no VGPR staging: LDS piece x = i*64 + lane takes the
// block's row r = x/8, piece (x%8) ^ (r%8), so row r's piece j sits at
// r*8 + (j ^ (r & 7)) and the per-row reads are bank-conflict free.
// row_stride4: uint4s between two rows' lines (8: blocked columns; capg / 2:
// row-major columns, NBKD_COL_ROWMAJOR)
__device__ __forceinline__ void issue_block(const uint4 *b4, uint4 *lds4, int lane, uint64_t rows,
                                            uint32_t row_stride4) {
    // rows: bit r set = row r holds candidates in this block; the other rows'
    // 128-B lines are not read (their LDS slots keep stale data, masked by count)
    const uint32_t r0 = (uint32_t)lane >> 3, jj = (uint32_t)lane & 7u;
    const uint4 *src = b4 + r0 * row_stride4 + (jj ^ r0);
    // bits r0, r0+8, .., r0+56 of rows -> bits 0..7 of m
    const uint32_t m = (uint32_t)((((rows >> r0) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (m & (1u << i))
            // non-temporal (aux 2 = nt): each column line is read once
            __builtin_amdgcn_global_load_lds((gas_ptr)(src + (size_t)(8 * i) * row_stride4),
                                             (las_ptr)(lds4 + 64 * i), 16, 0, 2);
}

// One lane per query: the k smallest of its candidate column, sorted, as rows.
template <int KC> constexpr int select_stage_words() {
    return (KC < 32 ? KC : 32) < 32 ? 32 * 64 : (KC < 32 ? KC : 32) * 64; // >= 8 KB: one block
}

// the 64 queries of wave-block wb (m: the pass's query count)
template <int KC, bool PER, bool WHOLE, bool EX = false>
__device__ __forceinline__ void
select_block(const DevTree &t, const float *__restrict__ q, const uint32_t *__restrict__ order,
             uint32_t m, uint32_t wb, int k, const uint2 *__restrict__ cand, uint32_t capg,
             const uint32_t *__restrict__ ccount, float *__restrict__ out_d,
             uint32_t *__restrict__ out_i, uint32_t *__restrict__ fail_list,
             uint32_t *__restrict__ fail_count, uint32_t pos_base, uint64_t all_rows,
             float *__restrict__ tg_fix, bool tg_pos, float mu, bool sq,
             uint32_t *__restrict__ fail_bits, uint32_t *stage, uint32_t *rowq, const int lane,
             float *__restrict__ kth_side) {
    constexpr int NS = 16;                  // candidates merged per pass
    constexpr int CC = KC < 32 ? KC : 32;   // top-k registers staged per output pass
    // lane = one query gq; its candidates: packet gq / qpp, row gq % qpp
    const uint32_t gq = wb * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const uint32_t n = valid ? ccount[gq] : 0u;
    const bool ok = valid && n >= (uint32_t)k && n <= capg;
    if (valid && !ok) {
        const float qx = q[3 * (size_t)qo], qy = q[3 * (size_t)qo + 1], qz = q[3 * (size_t)qo + 2];
        // outside-box periodic queries are listed already (outside_box_kernel);
        // pos_base != ~0: list the sorted position (pos_base + gq), not the id
        mark_failure<PER>(qx, qy, qz, t.box, pos_base == 0xFFFFFFFFu ? qo : pos_base + gq,
                          fail_list, fail_count, fail_bits);
        // the retry's seed (tg_fix: first pass only); n counted every point
        // inside the seed ball, so it measured the local density.  n < k:
        // grow the volume to hold ~mu at that density (2x..8x; 1.5 mu until
        // round 6: log-normal 1e8 re-walks 9.48 -> 9.09 ms,
        // profiles/r06l_retry_ab.txt).  An
        // overflowing column (n > capg): the retry's column is 8 capg, so keep
        // the seed while n fits half of it, else shrink it to that.
        if (tg_fix) {
            float fv;
            if (n < (uint32_t)k)
                fv = fminf(8.0f, fmaxf(NBKD_RETRY_MINV, NBKD_RETRY_GROW * mu / fmaxf((float)n, 0.5f)));
            else
                fv = fminf(1.0f, 4.0f * (float)capg / (float)n);
            const uint32_t ti = tg_pos ? gq : qo;
            tg_fix[ti] = fminf(tg_fix[ti] * cbrtf(fv * fv), FLT_MAX);
        }
    }
    const uint32_t nn = ok ? n : 0u;
    uint32_t maxn = nn;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxn = max(maxn, (uint32_t)__shfl_xor((int)maxn, o, 64));

    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : FLT_MAX;
        ti[j] = 0xFFFFFFFFu;
    }
    // qpp == 64: the wave's 64 lanes are one packet's 64 rows (blocked, read
    // through LDS); qpp == 1: each lane's row is contiguous at gq * capg
    constexpr bool whole = WHOLE; // == (qpp == 64)
    const uint4 *blk = reinterpret_cast<const uint4 *>(
        cand + (whole ? (size_t)(gq >> 6) * 64u * capg : (size_t)gq * capg));
    uint4 *const lds4 = reinterpret_cast<uint4 *>(stage);
    // all_rows: read every row's line (A/B of the per-row masking)
    // a block's rows: 128 B apart (blocked) or one column apart (row-major)
    const uint32_t rs4 = NBKD_COL_ROWMAJOR ? capg / 2u : 8u, bs4 = NBKD_COL_ROWMAJOR ? 8u : 512u;
    if (whole && maxn > 0) issue_block(blk, lds4, lane, __ballot(nn > 0u) | all_rows, rs4);
    // block s0/16 into (bd, bi); the whole-packet path also issues block s0/16 + 1
    auto read_block = [&](uint32_t s0, float (&bd)[NS], uint32_t (&bi)[NS]) {
        // block s0/16: 8 KB contiguous -> LDS (row r, 16-B piece j at r*8 + (j ^ (r&7)))
        if constexpr (!whole) { // scattered packets: each lane reads its own row directly
#pragma unroll
            for (int j = 0; j < NS; j += 2) {
                const uint32_t s = s0 + j;
                const bool h0 = s < nn, h1 = s + 1 < nn;
                const uint4 e = h0 ? blk[s >> 1] : make_uint4(0u, 0u, 0u, 0u);
                bd[j] = h0 ? __uint_as_float(e.x) : INFINITY;
                bi[j] = h0 ? e.y : 0xFFFFFFFFu;
                bd[j + 1] = h1 ? __uint_as_float(e.z) : INFINITY;
                bi[j + 1] = h1 ? e.w : 0xFFFFFFFFu;
            }
        } else {
            // block s0/16, loaded into LDS one pass ahead (issue_block)
            wait_vm0();
            wave_sync();
#pragma unroll
            for (int j = 0; j < NS; j += 2) {
                const uint4 e = lds4[lane * 8 + ((uint32_t)(j >> 1) ^ ((uint32_t)lane & 7u))];
                const uint32_t s = s0 + j;
                const bool h0 = s < nn, h1 = s + 1 < nn;
                bd[j] = h0 ? __uint_as_float(e.x) : INFINITY;
                bi[j] = h0 ? e.y : 0xFFFFFFFFu;
                bd[j + 1] = h1 ? __uint_as_float(e.z) : INFINITY;
                bi[j + 1] = h1 ? e.w : 0xFFFFFFFFu;
            }
            // the reads have retired before the next block's DMA overwrites the buffer
            __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0)
            wave_sync();
            if (s0 + NS < maxn)
                issue_block(blk + (size_t)((s0 + NS) >> 4) * bs4, lds4, lane,
                            __ballot(nn > s0 + NS) | all_rows, rs4);
        }
    };
    uint32_t s_first = 0;
    if constexpr (EX && KC > NS) {
        // EX: k == KC (no -inf placeholders): td is all FLT_MAX, so the take
        // and the merge of the first block would leave [block ascending,
        // FLT_MAX ...]; it is copied in instead (empty slots, INFINITY, stay
        // FLT_MAX; maxn == 0 reads nothing: every slot is empty)
        {
            float bd[NS];
            uint32_t bi[NS];
            read_block(0u, bd, bi);
            bitonic_sort<NS>(bd, bi);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                td[s] = fminf(bd[s], FLT_MAX);
                ti[s] = bi[s];
            }
            s_first = NS;
        }
    }
    for (uint32_t s0 = s_first; s0 < maxn; s0 += NS) {
        float bd[NS];
        uint32_t bi[NS];
        read_block(s0, bd, bi);
        // a block with nothing below any lane's current k-th changes nothing
        bool useful = false;
#pragma unroll
        for (int j = 0; j < NS; ++j) useful |= bd[j] < td[KC - 1];
        if (!__any(useful)) continue;
        bitonic_sort<NS>(bd, bi);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int pos = KC - NS + s, o = NS - 1 - s;
            const bool take = bd[o] < td[pos];
            td[pos] = take ? bd[o] : td[pos];
            ti[pos] = take ? bi[o] : ti[pos];
        }
        bitonic_merge<KC>(td, ti);
    }

    if (out_i == nullptr) { // k-th distance only (nbkd_query_kth): column k-1
        if (valid) out_d[qo] = sq ? td[KC - 1] : sqrtf(td[KC - 1]);
        return;
    }
    // the row's last column beside it (nbkd_set_kth_out); a failed row is
    // written again by its re-walk
    if (kth_side && ok) kth_side[qo] = sq ? td[KC - 1] : sqrtf(td[KC - 1]);
    rowq[lane] = valid ? qo : 0xFFFFFFFFu;
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j)
            stage[j * 64 + (lane ^ j)] = __float_as_uint(sq ? td[j0 + j] : sqrtf(td[j0 + j]));
        wave_sync();
        store_rows<CC>(stage, rowq, reinterpret_cast<uint32_t *>(out_d), k, j0 - (KC - k), lane);
    }
    // ti holds original ids (the collect kernel stores them with the candidates)
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j) stage[j * 64 + (lane ^ j)] = ti[j0 + j];
        wave_sync();
        store_rows<CC>(stage, rowq, out_i, k, j0 - (KC - k), lane);
    }
}

// A static pass launches one wave per 64 queries; a device-counted pass (the
// retry rounds: LOOP) a grid of at most resident_blocks() blocks that strides
// over its wave-blocks, so a pass whose count is zero (round 1 is launched in
// batches enough for every query failing) costs one short launch,
// not its cap's worth of workgroups.  Only the LOOP instance carries the loop,
// at half the occupancy: at the static instance's 128 VGPRs (k <= 32) the
// loop spilled ~300 B per lane; the static instance keeps 4 waves per SIMD.
template <int KC, bool PER, bool WHOLE, bool LOOP>
__global__ void __launch_bounds__(TB, (KC <= 32 ? 4 : 2) / (LOOP ? 2 : 1))
knn_select_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  QSpan span, int k, uint32_t qpp, const uint2 *__restrict__ cand, uint32_t capg,
                  const uint32_t *__restrict__ ccount, float *__restrict__ out_d,
                  uint32_t *__restrict__ out_i, uint32_t *__restrict__ fail_list,
                  uint32_t *__restrict__ fail_count, uint32_t pos_base, uint64_t all_rows,
                  float *__restrict__ tg_fix, float mu, bool sq, uint32_t *__restrict__ fail_bits,
                  float *__restrict__ kth_side) {
    constexpr int SW = select_stage_words<KC>();
    __shared__ uint32_t stage_all[WPB][SW];
    __shared__ uint32_t rowq_all[WPB][64];
    const int lane = threadIdx.x & 63, wave = wave_id();
    uint32_t *stage = stage_all[wave], *rowq = rowq_all[wave];
    const uint32_t m = span_m(span);
    if constexpr (LOOP) {
        for (uint32_t wb = blockIdx.x * WPB + wave; wb * 64u < m; wb += gridDim.x * WPB) {
            wave_sync(); // the previous wave-block's LDS reads are done
            select_block<KC, PER, WHOLE>(t, q, order, m, wb, k, cand, capg, ccount, out_d, out_i,
                                         fail_list, fail_count, pos_base, all_rows, tg_fix,
                                         span.tg_pos, mu, sq, fail_bits, stage, rowq, lane,
                                         kth_side);
        }
    } else {
        const uint32_t wb = blockIdx.x * WPB + wave;
        if (wb * 64u >= m) return;
        if (NBKD_SEL_FIRST && k == KC) // a separate instance: no join of the two td states
            select_block<KC, PER, WHOLE, true>(t, q, order, m, wb, k, cand, capg, ccount, out_d,
                                               out_i, fail_list, fail_count, pos_base, all_rows,
                                               tg_fix, span.tg_pos, mu, sq, fail_bits, stage,
                                               rowq, lane, kth_side);
        else
            select_block<KC, PER, WHOLE>(t, q, order, m, wb, k, cand, capg, ccount, out_d, out_i,
                                         fail_list, fail_count, pos_base, all_rows, tg_fix,
                                         span.tg_pos, mu, sq, fail_bits, stage, rowq, lane,
                                         kth_side);
    }
}

// ---------------------------------------------------------------- k > 64: one wave per query
// The top-K (K = pow2 >= k, 128..1024) of ONE query spread over the wave's 64
// lanes: R = K/64 registers per lane, element e = r*64 + lane.  The query's
// column is read in chunks of K slots (16 consecutive slots are one 128-B
// line), each chunk bitonic-sorted across the wave (exchanges between
// registers for strides >= 64, DPP / permlane lane exchanges below) and merged
// into the top-K: with the chunk sorted descending, min(top[e], chunk[e])
// holds the K smallest of both as a bitonic sequence, which log2(K)
// half-cleaner stages sort.  A chunk with nothing
// below the current k-th is skipped.  The rows leave as 64-wide contiguous
// stores.  Same result rows as the lane-per-query select (the k smallest d2
// of the column, ascending; ties in any order): find_closest,
// kdtree/src/cpp/kdtree.cpp:133-159; tournament_tree.hpp:42-105 (any k).
// the lanes l with (l & b) == 0, as an exec-style mask (compile time)
constexpr uint64_t lanes_bit_clear(int b) {
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l)
        if ((l & b) == 0) m |= 1ull << l;
    return m;
}

// the value of lane (lane ^ S), as VALU data movement where gfx950 has it:
// DPP quad permutes (S = 1, 2); two DPP row shifts whose bank masks pick the
// lanes each serves (S = 4, 8: the lower half of every 2S-lane group reads
// lane + S, the upper half lane - S); v_permlane32_swap (S = 32: lanes 0-31 of
// one copy trade places with lanes 32-63 of the other); S = 16 by ds_swizzle
// (xor within 32-lane groups).  ds_bpermute (__shfl_xor) ran the k = 100
// select through the LDS crossbar: 196 ms at 1e8 (r03d).
template <int S> __device__ __forceinline__ int lane_xor(int x) {
    if constexpr (S == 1) {
        return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, true); // quad_perm [1,0,3,2]
    } else if constexpr (S == 2) {
        return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, true); // quad_perm [2,3,0,1]
    } else if constexpr (S == 4) {
        // banks (4-lane groups of a 16-lane row) 0, 2 read lane + 4; 1, 3 lane - 4
        const int t = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0x5, false); // row_shl:4
        return __builtin_amdgcn_update_dpp(t, x, 0x114, 0xF, 0xA, false);        // row_shr:4
    } else if constexpr (S == 8) {
        const int t = __builtin_amdgcn_update_dpp(x, x, 0x108, 0xF, 0x3, false); // row_shl:8
        return __builtin_amdgcn_update_dpp(t, x, 0x118, 0xF, 0xC, false);        // row_shr:8
    } else if constexpr (S == 16) {
        return __builtin_amdgcn_ds_swizzle(x, 0x401F); // bit mode: and 0x1F, xor 0x10
    } else {
        static_assert(S == 32, "lane_xor: stride");
        const auto pr = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (int)lane_set((uint32_t)pr[1], (uint32_t)pr[0], ~lanes_bit_clear(32));
    }
}

// compare-exchange of element pairs (e, e ^ STRIDE), ascending where
// ((e & SIZE) == 0) != DESC.  A lane keeps its partner's value iff
// (lower == ascending) ? partner < own : partner > own; that choice is a
// compile-time lane mask M, so take = (M & lt) | (~M & gt) is scalar work on
// the two compare masks (equal keys: neither partner takes the other's)
template <int R, int SIZE, int STRIDE, bool DESC>
__device__ __forceinline__ void wave_cx(float (&d)[R], uint32_t (&p)[R], int lane) {
    if constexpr (STRIDE >= 64) {
        constexpr int rs = STRIDE / 64;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r & rs) continue;
            const int r2 = r | rs;
            // e & SIZE for SIZE >= 128 depends on the register only
            const bool asc = ((((r * 64) & SIZE) == 0)) != DESC;
            const bool sw = asc ? (d[r2] < d[r]) : (d[r2] > d[r]);
            const float a = d[r], b = d[r2];
            const uint32_t pa = p[r], pb = p[r2];
            d[r] = sw ? b : a;
            d[r2] = sw ? a : b;
            p[r] = sw ? pb : pa;
            p[r2] = sw ? pa : pb;
        }
    } else {
        constexpr uint64_t lower = lanes_bit_clear(STRIDE);
        float od[R];
        uint32_t op[R];
        // every exchange of the stage first: the DPP reads of a register then
        // sit several instructions after its last write (fewer hazard nops)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            od[r] = __int_as_float(lane_xor<STRIDE>(__float_as_int(d[r])));
            op[r] = (uint32_t)lane_xor<STRIDE>((int)p[r]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            constexpr uint64_t ones = ~0ull;
            const uint64_t asc_m = SIZE >= 64 ? ((((r * 64) & SIZE) == 0) ? ones : 0ull)
                                              : lanes_bit_clear(SIZE);
            const uint64_t M = ~(lower ^ (DESC ? ~asc_m : asc_m)); // lower == ascending
#if NBKD_WAVE_KEY64
            // (d2 bits, id) as one unsigned 64-bit key: d2 >= 0, so the bits
            // order as the values, and the ids of one column are distinct, so
            // partners differ unless both are padding (equal: either way)
            const uint64_t ko = ((uint64_t)__float_as_uint(od[r]) << 32) | op[r];
            const uint64_t kw = ((uint64_t)__float_as_uint(d[r]) << 32) | p[r];
            const uint64_t take = ~(M ^ __ballot(ko < kw));
#else
            const uint64_t lt = __ballot(od[r] < d[r]), gt = __ballot(od[r] > d[r]);
            const uint64_t take = (M & lt) | (~M & gt);
#endif
            d[r] = lane_set(d[r], od[r], take);
            p[r] = lane_set(p[r], op[r], take);
        }
    }
    (void)lane;
}

template <int R, int SIZE, int STRIDE, bool DESC>
__device__ __forceinline__ void wave_merge_stages(float (&d)[R], uint32_t (&p)[R], int lane) {
    wave_cx<R, SIZE, STRIDE, DESC>(d, p, lane);
    if constexpr (STRIDE > 1) wave_merge_stages<R, SIZE, STRIDE / 2, DESC>(d, p, lane);
}

template <int R, int SIZE, bool DESC>
__device__ __forceinline__ void wave_sort_stages(float (&d)[R], uint32_t (&p)[R], int lane) {
    wave_merge_stages<R, SIZE, SIZE / 2, DESC>(d, p, lane);
    if constexpr (SIZE < 64 * R) wave_sort_stages<R, SIZE * 2, DESC>(d, p, lane);
}

// the bitonic sort stages of sizes SIZE..MAXSIZE only: with MAXSIZE < 64 R the
// register blocks of MAXSIZE elements are sorted independently, alternately
// ascending and descending
template <int R, int SIZE, int MAXSIZE, bool DESC>
__device__ __forceinline__ void wave_sort_upto(float (&d)[R], uint32_t (&p)[R], int lane) {
    wave_merge_stages<R, SIZE, SIZE / 2, DESC>(d, p, lane);
    if constexpr (SIZE < MAXSIZE) wave_sort_upto<R, SIZE * 2, MAXSIZE, DESC>(d, p, lane);
}

// 64 < k <= 128, a first pass (round 6): TWO queries per wave, sorted in one
// network of four registers (positions p and p + 1 of the pass: registers 0-1
// hold the first, ascending; 2-3 the second, descending), so every stage has
// two independent exchange chains.  The one-query wave select issues each
// stage's DPP exchange, ballot compare, scalar mask logic and select as one
// dependent chain; its counters at k = 100 (profiles/r06f_pmc_select_wave.txt)
// show more issue-stall than issuing cycles.  Only the common case runs here:
// both columns complete (k <= n <= capg, n <= 256) and at most 128 candidates
// below the collect kernel's final bound; any other position of the pair is
// appended to `leftover` for the one-query kernel (pos_list), which also
// marks the failures.
template <bool PER, int NQ>
__global__ void __launch_bounds__(TB)
knn_select_wave_pair_kernel(const uint32_t *__restrict__ order, QSpan span, int k,
                            const uint2 *__restrict__ cand, uint32_t capg,
                            const uint32_t *__restrict__ ccount, float *__restrict__ out_d,
                            uint32_t *__restrict__ out_i, bool sq,
                            const float *__restrict__ kbound, uint32_t *__restrict__ leftover,
                            uint32_t *__restrict__ nleft) {
    constexpr int K = 128, NS = 2 * K; // sorted per query; slots read per query
    constexpr int RR = 2 * NQ;         // registers: query j in 2j, 2j + 1
    __shared__ uint2 cl_all[WPB][NQ][K];
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    const uint32_t m = span_m(span);
    const uint32_t ngroups = (m + NQ - 1) / NQ;
    for (uint32_t gi = blockIdx.x * WPB + w; gi < ngroups; gi += gridDim.x * WPB) {
        float td[RR];
        uint32_t tp[RR];
        bool fast[NQ];
        uint32_t qo[NQ];
        bool any = false;
#pragma unroll
        for (int s2 = 0; s2 < NQ; ++s2) {
            const uint32_t g = NQ * gi + s2;
            const bool valid = g < m;
            const uint32_t n = valid ? ccount[g] : 0u;
            const bool ok = valid && n >= (uint32_t)k && n <= capg && n <= (uint32_t)NS;
            qo[s2] = valid ? order[g] : 0u;
            const float bnd = (valid && kbound) ? kbound[g] : INFINITY;
            const uint2 *col = cand + (size_t)g * capg;
            uint2 e[NS / 64];
#pragma unroll
            for (int j = 0; j < NS / 64; ++j) {
                const uint32_t sl = (uint32_t)(j * 64 + lane);
                e[j] = (ok && sl < n) ? col[sl] : make_uint2(0x7F800000u, 0xFFFFFFFFu);
            }
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < NS / 64; ++j) {
                const bool v = __uint_as_float(e[j].x) < bnd;
                const uint64_t bal = __ballot(v);
                const uint32_t at = c + mbcnt64(bal);
                if (v && at < (uint32_t)K) cl_all[w][s2][at] = e[j];
                c += (uint32_t)__popcll(bal);
            }
            fast[s2] = ok && c <= (uint32_t)K;
            any |= fast[s2];
            if (valid && !fast[s2] && lane == 0) leftover[atomicAdd(nleft, 1u)] = g;
            // the entries past the compacted ones read as +inf
            if ((uint32_t)lane >= c) cl_all[w][s2][lane] = make_uint2(0x7F800000u, 0xFFFFFFFFu);
            if ((uint32_t)(lane + 64) >= c)
                cl_all[w][s2][lane + 64] = make_uint2(0x7F800000u, 0xFFFFFFFFu);
        }
        if (!any) continue;
        wave_sync();
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint2 v = cl_all[w][r >> 1][(r & 1) * 64 + lane];
            td[r] = __uint_as_float(v.x);
            tp[r] = v.y;
        }
        // one network for all NQ queries: blocks of 128 alternately ascending
        // and descending
        wave_sort_upto<RR, 2, K, false>(td, tp, lane);
        wave_sync(); // the LDS reads are done before the next group's writes
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const int s2 = r >> 1, rr = (r & 1) * 64 + lane;
            const int e = (s2 & 1) == 0 ? rr : 127 - rr; // odd blocks descending
            if (!fast[s2] || e >= k) continue;
            const float dv = sq ? td[r] : sqrtf(td[r]);
            if (out_i == nullptr) { // k-th distance only
                if (e == k - 1) out_d[qo[s2]] = dv;
                continue;
            }
            out_d[(size_t)qo[s2] * k + e] = dv;
            out_i[(size_t)qo[s2] * k + e] = tp[r];
        }
    }
}

template <int R, bool PER, bool WHOLE>
__global__ void __launch_bounds__(TB)
knn_select_wave_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                       QSpan span, int k, const uint2 *__restrict__ cand, uint32_t capg,
                       const uint32_t *__restrict__ ccount, float *__restrict__ out_d,
                       uint32_t *__restrict__ out_i, uint32_t *__restrict__ fail_list,
                       uint32_t *__restrict__ fail_count, uint32_t pos_base,
                       float *__restrict__ tg_fix, float mu, bool sq,
                       const float *__restrict__ kbound, uint32_t *__restrict__ fail_bits,
                       const uint32_t *__restrict__ pos_list) {
    constexpr int K = 64 * R;
    // per wave: the query's candidates below its final bound, compacted
    __shared__ uint2 cl_all[WPB][2 * K];
    const int lane = threadIdx.x & 63;
    uint2 *const cl = cl_all[wave_id()];
    const uint32_t m = span_m(span);
    // pos_list (the pair kernel's leftovers): entry i of this pass is the
    // pass position pos_list[i]; else entry i is position i
    auto pos = [&](uint32_t i) { return pos_list ? pos_list[i] : i; };
    const uint32_t nwaves = gridDim.x * WPB;
    // software pipeline, two deep: the next query's bound and first 2K slots
    // are loaded before this query is sorted, and the count of the query after
    // it one iteration earlier, so that only the slots below its count are
    // read (until round 6 every slot up to 2K was read, clamped to the
    // column's last one: at k = 100 ~1.7 KB per query for ~1 KB of candidates)
    auto slot_ptr = [&](uint32_t g, uint32_t sl) {
        const uint32_t c = min(sl, capg - 1u);
        return (WHOLE && !NBKD_COL_ROWMAJOR)
                   ? cand + (size_t)(g >> 6) * 64u * capg + ((c >> 4) * 64u + (g & 63u)) * 16u + (c & 15u)
                   : cand + (size_t)g * capg + c;
    };
    uint32_t gq = blockIdx.x * WPB + wave_id();
    uint32_t n_nx = gq < m ? ccount[pos(gq)] : 0u, qo_nx = 0;
    uint32_t n_nn = gq + nwaves < m ? ccount[pos(gq + nwaves)] : 0u; // one query further
    float b_nx = INFINITY;
    uint2 e_nx[2 * R];
    auto prefetch = [&](uint32_t gi, uint32_t ng) {
        if (gi >= m) return;
        const uint32_t g = pos(gi);
        qo_nx = order[g];
        b_nx = kbound ? kbound[g] : INFINITY;
        // a failed column (fewer than k, or past capg) is never sorted
        const uint32_t lim = (ng >= (uint32_t)k && ng <= capg) ? ng : 0u;
#pragma unroll
        for (int j = 0; j < 2 * R; ++j) {
            const uint32_t sl = (uint32_t)(j * 64 + lane);
            e_nx[j] = sl < lim ? *slot_ptr(g, sl) : make_uint2(0x7F800000u, 0xFFFFFFFFu);
        }
    };
    prefetch(gq, n_nx);
    uint32_t pend_q = 0xFFFFFFFFu; // the query whose ids are still to be stored
    uint32_t pend_i[R];
    for (; gq < m; gq += nwaves) {
        const uint32_t qo = qo_nx;
        const uint32_t n = n_nx;
        const float bnd = b_nx;
        uint2 e[2 * R];
#pragma unroll
        for (int j = 0; j < 2 * R; ++j) e[j] = e_nx[j];
        n_nx = n_nn;
        prefetch(gq + nwaves, n_nx);
        n_nn = gq + 2 * nwaves < m ? ccount[pos(gq + 2 * nwaves)] : 0u;
        const uint32_t gp = pos(gq); // this query's position in the pass
        if (!(n >= (uint32_t)k && n <= capg)) {
            if (lane == 0) {
                const float qx = q[3 * (size_t)qo], qy = q[3 * (size_t)qo + 1],
                            qz = q[3 * (size_t)qo + 2];
                mark_failure<PER>(qx, qy, qz, t.box, pos_base == 0xFFFFFFFFu ? qo : pos_base + gp,
                                  fail_list, fail_count, fail_bits);
                if (tg_fix) { // the retry's seed, as knn_select_kernel
                    float fv;
                    if (n < (uint32_t)k)
                        fv = fminf(8.0f, fmaxf(NBKD_RETRY_MINV, NBKD_RETRY_GROW * mu / fmaxf((float)n, 0.5f)));
                    else
                        fv = fminf(1.0f, 4.0f * (float)capg / (float)n);
                    const uint32_t ti = span.tg_pos ? gp : qo;
                    tg_fix[ti] = fminf(tg_fix[ti] * cbrtf(fv * fv), FLT_MAX);
                }
            }
            continue;
        }
        constexpr bool BLOCKED = WHOLE && !NBKD_COL_ROWMAJOR;
        const uint2 *col = BLOCKED ? cand + (size_t)(gp >> 6) * 64u * capg : cand + (size_t)gp * capg;
        const uint32_t row = gp & 63u;
        // at least k candidates lie strictly below the collect kernel's final
        // bound (bnd), so the k smallest are all below it
        float td[R], cd[R];
        uint32_t tp[R], cp[R];
        const int kr = (k - 1) >> 6, kl = (k - 1) & 63; // element k-1: register kr, lane kl
        if (n <= (uint32_t)(2 * K)) {
            // one pass: all 2K slots loaded at once, the candidates below the
            // bound compacted into LDS (typically k + a bucket's worth), then
            // one sort of K (or a sort + merge when more than K survive)
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 2 * R; ++j) {
                const bool v = (uint32_t)(j * 64 + lane) < n && __uint_as_float(e[j].x) < bnd;
                const uint64_t bal = __ballot(v);
                if (v) cl[c + mbcnt64(bal)] = e[j];
                c += (uint32_t)__popcll(bal);
            }
            wave_sync();
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t x = (uint32_t)(r * 64 + lane);
                const uint2 v = x < c ? cl[x] : make_uint2(0x7F800000u, 0xFFFFFFFFu);
                td[r] = __uint_as_float(v.x);
                tp[r] = v.y;
            }
            wave_sort_stages<R, 2, false>(td, tp, lane);
            if (c > (uint32_t)K) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t x = (uint32_t)(K + r * 64 + lane);
                    const uint2 v = x < c ? cl[x] : make_uint2(0x7F800000u, 0xFFFFFFFFu);
                    cd[r] = __uint_as_float(v.x);
                    cp[r] = v.y;
                }
                wave_sort_stages<R, 2, true>(cd, cp, lane);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool take = cd[r] < td[r];
                    td[r] = take ? cd[r] : td[r];
                    tp[r] = take ? cp[r] : tp[r];
                }
                wave_merge_stages<R, 2 * K, K / 2, false>(td, tp, lane);
            }
            wave_sync(); // the LDS reads are done before the next query's writes
        } else {
            // long columns (retry rounds): chunks of K from global memory
            for (uint32_t c0 = 0; c0 < n; c0 += K) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t sl = c0 + (uint32_t)(r * 64 + lane);
                    const uint2 e = sl < n ? (BLOCKED ? col[((sl >> 4) * 64u + row) * 16u + (sl & 15u)]
                                                      : col[sl])
                                           : make_uint2(0x7F800000u, 0xFFFFFFFFu);
                    const float d = __uint_as_float(e.x);
                    cd[r] = d < bnd ? d : INFINITY;
                    cp[r] = d < bnd ? e.y : 0xFFFFFFFFu;
                }
                if (c0 > 0) {
                    // nothing below the current k-th: the chunk changes nothing
                    float kth = 0.0f;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        if (r == kr) kth = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(td[r]), kl));
                    bool useful = false;
#pragma unroll
                    for (int r = 0; r < R; ++r) useful |= cd[r] < kth;
                    if (!__any(useful)) continue;
                }
                if (c0 == 0) {
                    wave_sort_stages<R, 2, false>(cd, cp, lane);
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        td[r] = cd[r];
                        tp[r] = cp[r];
                    }
                } else {
                    // the chunk sorted DESCENDING: min(top[e], chunk[e]) holds the K
                    // smallest of both as a bitonic sequence
                    wave_sort_stages<R, 2, true>(cd, cp, lane);
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const bool take = cd[r] < td[r];
                        td[r] = take ? cd[r] : td[r];
                        tp[r] = take ? cp[r] : tp[r];
                    }
                    wave_merge_stages<R, 2 * K, K / 2, false>(td, tp, lane);
                }
            }
        }
        if (out_i == nullptr) { // k-th distance only
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (r == kr && lane == kl) out_d[qo] = sq ? td[r] : sqrtf(td[r]);
            continue;
        }
        const size_t base = (size_t)qo * (size_t)k;
        // the original ids are gathered now and stored one query later, so the
        // gathers' latency overlaps the next query's sort
        uint32_t gi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = r * 64 + lane;
            gi[r] = e < k ? tp[r] : 0xFFFFFFFFu; // ids, or the no-neighbour sentinel
            if (e < k) out_d[base + e] = sq ? td[r] : sqrtf(td[r]);
        }
        if (pend_q != 0xFFFFFFFFu) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (r * 64 + lane < k) out_i[(size_t)pend_q * (size_t)k + r * 64 + lane] = pend_i[r];
        }
        pend_q = qo;
#pragma unroll
        for (int r = 0; r < R; ++r) pend_i[r] = gi[r];
    }
    if (pend_q != 0xFFFFFFFFu) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r * 64 + lane < k) out_i[(size_t)pend_q * (size_t)k + r * 64 + lane] = pend_i[r];
    }
}


// walk ahead to the next leaf while a leaf's staging is in flight (grp_packet
// AHEAD, on by default since round 4: collect 49.80 -> 48.28 ms per 1e8
// queries, profiles/r04c_ab_collect_ahead.txt; every distance row identical
// at 1e8, only the order inside exact ties changes, profiles/r04e_ahead_rows.json);
// NBKD_COLLECT_AHEAD=0 in an experiments build restores the walk after the scan
bool collect_ahead() {
    const char *e = knob("NBKD_COLLECT_AHEAD"); // read per launch: A/B within one process
    return !(e && atoi(e) == 0);
}

// a device-counted pass's fixed grid: 8 blocks of 4 waves per CU
unsigned resident_blocks() {
    static const unsigned b = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        (void)hipGetLastError();
        return 8u * (unsigned)std::max(cus, 1);
    }();
    return b;
}

template <bool PER>
void launch_collect(const Tree &t, const float *q, const uint32_t *order, QSpan span, int k,
                    const float *tg, float seed_mul, uint32_t qpp, uint2 *cand, uint32_t capg,
                    uint32_t *ccount, unsigned long long *stats, bool retry, float *kbound,
                    hipStream_t s) {
    const char *const name = retry ? "knn_retry" : "knn_collect";
    const uint32_t m = span.m;
    const unsigned blocks =
        span.count ? std::min<unsigned>(resident_blocks(),
                                        (unsigned)((((uint64_t)m + qpp - 1) / qpp + WPB - 1) / WPB))
                   : (unsigned)((((uint64_t)m + qpp - 1) / qpp + WPB - 1) / WPB);
    // the bound histogram's 8-bit bucket counts are exact while the cumulative
    // count below the k-th's bucket is < 256, i.e. for k <= 255 (a wrapped or
    // carried byte can only make a larger cumulative count); above, no tightening
    if (k > 255) k = 0x7FFFFFFF;
    {
        // NBKD_XCD_MAP=0: hardware block order (A/B of the XCD-contiguous packet ranges)
        static const bool xcd = [] {
            const char *e = knob("NBKD_XCD_MAP");
            return !(e && atoi(e) == 0);
        }();
        // the re-walk rounds are timed as one phase by the caller (query.hip)
        TimedScope ts(name, s, !retry);
#define NBKD_GRP(STATS, LOOP, AHEAD, STP, XCD)                                                     \
    knn_collect_grp_kernel<PER, 8, STATS, LOOP, AHEAD><<<blocks, TB, 0, s>>>(                      \
        view(t), t.ginfo, t.leafinfo, t.hinfo, q, order, span, k, tg, seed_mul, qpp, cand, capg,   \
        ccount, STP, XCD, kbound)
        if (span.count)
            NBKD_GRP(false, true, NBKD_LOOP_AHEAD != 0, nullptr, false);
        else if (collect_ahead()) {
            if (stats)
                NBKD_GRP(true, false, true, stats, xcd);
            else
                NBKD_GRP(false, false, true, nullptr, xcd);
        } else if (stats)
            NBKD_GRP(true, false, false, stats, xcd);
        else
            NBKD_GRP(false, false, false, nullptr, xcd);
#undef NBKD_GRP
        return;
    }
}

template <int R>
void launch_select_wave(const Tree &t, const float *q, const uint32_t *order, QSpan span, int k,
                        uint32_t qpp, const uint2 *cand, uint32_t capg, const uint32_t *ccount,
                        float *od, uint32_t *oi, uint32_t *fail_list, uint32_t *fail_count,
                        uint32_t *fail_bits, uint32_t pos_base, float *tg_fix, float mu, bool sq,
                        const float *kbound, hipStream_t s, uint32_t *pair_scratch) {
    const uint32_t *pos_list = nullptr;
    if constexpr (R == 2 && NBKD_COL_ROWMAJOR && NBKD_WAVE_PAIR > 0) {
        if (pair_scratch && !span.count && kbound) {
            // two queries per wave for the common case; the rest (failures, long
            // columns, more than 128 below the bound) by the one-query kernel
            uint32_t *nleft = pair_scratch + ((size_t)span.m + 15) / 16 * 16;
            if (hipMemsetAsync(nleft, 0, 4, s) != hipSuccess) goto one_query; // every query below
            {
            constexpr int NQ = NBKD_WAVE_PAIR;
            const unsigned pblocks = (unsigned)std::min<uint64_t>(
                (((uint64_t)span.m + NQ - 1) / NQ + WPB - 1) / WPB, 32768u);
            if (t.periodic)
                knn_select_wave_pair_kernel<true, NQ><<<pblocks, TB, 0, s>>>(
                    order, span, k, cand, capg, ccount, od, oi, sq, kbound, pair_scratch, nleft);
            else
                knn_select_wave_pair_kernel<false, NQ><<<pblocks, TB, 0, s>>>(
                    order, span, k, cand, capg, ccount, od, oi, sq, kbound, pair_scratch, nleft);
            QSpan lsp = span;
            lsp.count = nleft;
            lsp.base = 0;
            lsp.mode = 0;
            lsp.capped = true;
            span = lsp;
            pos_list = pair_scratch;
            }
        }
    }
one_query:
    const unsigned blocks = (unsigned)std::min<uint64_t>(((uint64_t)span.m + WPB - 1) / WPB,
                                                         span.count ? resident_blocks() : 32768u);
#define NBKD_SELW(PER, WH)                                                                         \
    knn_select_wave_kernel<R, PER, WH><<<blocks, TB, 0, s>>>(view(t), q, order, span, k, cand,     \
                                                            capg, ccount, od, oi, fail_list,       \
                                                            fail_count, pos_base, tg_fix, mu, sq,  \
                                                            kbound, fail_bits, pos_list)
    if (t.periodic) {
        if (qpp == 64) NBKD_SELW(true, true); else NBKD_SELW(true, false);
    } else {
        if (qpp == 64) NBKD_SELW(false, true); else NBKD_SELW(false, false);
    }
#undef NBKD_SELW
}

template <int KC>
void launch_select(const Tree &t, const float *q, const uint32_t *order, QSpan span, int k,
                   uint32_t qpp, const uint2 *cand, uint32_t capg, const uint32_t *ccount,
                   float *od, uint32_t *oi, uint32_t *fail_list, uint32_t *fail_count,
                   uint32_t *fail_bits, uint32_t pos_base, float *tg_fix, float mu, bool sq,
                   hipStream_t s, float *kth_side) {
    // a capped pass (round 1's later batches, usually empty): at most
    // resident_blocks() blocks striding over its wave-blocks (LOOP); any other
    // pass one wave per 64 queries of its count or cap, at 4 waves per SIMD
    // (the LOOP instance runs at 2: the dense log-normal retry's select took
    // 8.7 -> 10.4 ms per 1e8 with every round-1 batch capped, r05i suite)
    const bool loop = span.count && span.capped;
    const unsigned blocks =
        loop ? (unsigned)std::min<uint64_t>((span.m + TB - 1) / TB, resident_blocks())
             : (span.m + TB - 1) / TB;
    static const uint64_t all_rows = [] { // NBKD_SELECT_ROWMASK=0: read whole blocks
        const char *e = knob("NBKD_SELECT_ROWMASK");
        return (e && atoi(e) == 0) ? ~0ull : 0ull;
    }();
#define NBKD_SELECT(PER, WH, LP)                                                                   \
    knn_select_kernel<KC, PER, WH, LP><<<blocks, TB, 0, s>>>(view(t), q, order, span, k, qpp,     \
                                                            cand, capg, ccount, od, oi, fail_list, \
                                                            fail_count, pos_base, all_rows,        \
                                                            tg_fix, mu, sq, fail_bits, kth_side)
    if (loop) {
        if (t.periodic) {
            if (qpp == 64) NBKD_SELECT(true, true, true); else NBKD_SELECT(true, false, true);
        } else {
            if (qpp == 64) NBKD_SELECT(false, true, true); else NBKD_SELECT(false, false, true);
        }
    } else {
        if (t.periodic) {
            if (qpp == 64) NBKD_SELECT(true, true, false); else NBKD_SELECT(true, false, false);
        } else {
            if (qpp == 64) NBKD_SELECT(false, true, false); else NBKD_SELECT(false, false, false);
        }
    }
#undef NBKD_SELECT
}

} // namespace

bool retry_adaptive() {
    static const bool on = [] { // NBKD_RETRY_ADAPT=0: every retry seed is 4x (A/B)
        const char *e = knob("NBKD_RETRY_ADAPT");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

uint32_t collect_capacity(int k) {
    // seed balls hold mu = k + 4 sqrt(k) + 4 points on average; the column
    // takes mu + 5 sqrt(mu), rounded up to a multiple of 16
    const double mu = k + 4.0 * std::sqrt((double)k) + 4.0;
    double c = mu + 5.0 * std::sqrt(mu);
    if (const char *e = knob("NBKD_KNN_CAP")) c *= std::max(0.25, atof(e)); // experiments only
    return (uint32_t)((c + 15.0) / 16.0) * 16u;
}

nbkd_status launch_knn_collect(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                               int k, const float *tg, float seed_mul, uint32_t qpp, uint2 *cand,
                               uint32_t capg, uint32_t *ccount, float *od, uint32_t *oi,
                               uint32_t *fail_list, uint32_t *fail_count, uint32_t *fail_bits,
                               uint32_t pos_base, bool retry, bool fix_seed, bool sq, float *kb,
                               unsigned long long *stats, hipStream_t s, float *kth_side,
                               uint32_t *pair_scratch) {
    nbkd_status rc = launch_collect_pass(t, q, order, span, k, tg, seed_mul, qpp, cand, capg,
                                         ccount, retry, kb, stats, s);
    if (rc) return rc;
    return launch_select_pass(t, q, order, span, k, tg, qpp, cand, capg, ccount, od, oi,
                              fail_list, fail_count, fail_bits, pos_base, retry, fix_seed, sq, kb,
                              s, kth_side, pair_scratch);
}

nbkd_status launch_collect_pass(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                                int k, const float *tg, float seed_mul, uint32_t qpp, uint2 *cand,
                                uint32_t capg, uint32_t *ccount, bool retry, float *kb,
                                unsigned long long *stats, hipStream_t s) {
    if (span.m == 0) return NBKD_OK;
    // k > 64: the collect kernel hands each query's final bound to the wave select
    float *kbound = k > 64 ? kb : nullptr;
    if (t.periodic)
        launch_collect<true>(t, q, order, span, k, tg, seed_mul, qpp, cand, capg, ccount, stats,
                             retry, kbound, s);
    else
        launch_collect<false>(t, q, order, span, k, tg, seed_mul, qpp, cand, capg, ccount, stats,
                              retry, kbound, s);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

nbkd_status launch_select_pass(const Tree &t, const float *q, const uint32_t *order, QSpan span,
                               int k, const float *tg, uint32_t qpp, const uint2 *cand,
                               uint32_t capg, const uint32_t *ccount, float *od, uint32_t *oi,
                               uint32_t *fail_list, uint32_t *fail_count, uint32_t *fail_bits,
                               uint32_t pos_base, bool retry, bool fix_seed, bool sq, float *kb,
                               hipStream_t s, float *kth_side, uint32_t *pair_scratch) {
    if (span.m == 0) return NBKD_OK;
    float *kbound = k > 64 ? kb : nullptr;
    {
        TimedScope ts("knn_select", s, !retry);
        // a retry round follows: failures rewrite their seed for it
        float *tg_fix = fix_seed ? const_cast<float *>(tg) : nullptr;
        const float mu = (float)k + 4.0f * sqrtf((float)k) + 4.0f;
        if (k <= 16)
            launch_select<16>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi, fail_list,
                              fail_count, fail_bits, pos_base, tg_fix, mu, sq, s, kth_side);
        else if (k <= 32)
            launch_select<32>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi, fail_list,
                              fail_count, fail_bits, pos_base, tg_fix, mu, sq, s, kth_side);
        else if (k <= 64)
            launch_select<64>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi, fail_list,
                              fail_count, fail_bits, pos_base, tg_fix, mu, sq, s, kth_side);
        else if (k <= 128)
            launch_select_wave<2>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi,
                                  fail_list, fail_count, fail_bits, pos_base, tg_fix, mu, sq, kbound, s,
                                  pair_scratch);
        else if (k <= 256)
            launch_select_wave<4>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi,
                                  fail_list, fail_count, fail_bits, pos_base, tg_fix, mu, sq, kbound, s,
                                   nullptr);
        else if (k <= 512)
            launch_select_wave<8>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi,
                                  fail_list, fail_count, fail_bits, pos_base, tg_fix, mu, sq, kbound, s,
                                   nullptr);
        else
            launch_select_wave<16>(t, q, order, span, k, qpp, cand, capg, ccount, od, oi,
                                   fail_list, fail_count, fail_bits, pos_base, tg_fix, mu, sq, kbound, s,
                                   nullptr);
        NBKD_HIP(hipGetLastError());
    }
    return NBKD_OK;
}

} // namespace nbkd
