// Packet kNN kernel (gfx950).  Reference semantics: KDTreeQuery::compute
// (kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:226-268) + the leaf scan of
// kdtree_asm_systemv.asm:148-188; see query.hip for the driver.
//
// One wave64 = one packet of 64 kd-ordered queries (one per lane).  The wave
// walks the tree once, depth-first and near-child-first by majority vote of
// the lanes that want the node (stack of node id + box in VGPRs, one entry per
// lane, popped with v_readlane); a node is entered iff some lane's box
// distance <= that lane's current k-th, and `need` = the mask of those lanes.
// Each leaf chunk (<= CHUNK points) is staged once into LDS with coalesced SoA
// loads, then processed in rounds of R = 8 points:
//   * dense round  (> 32 lanes need the leaf): every lane evaluates the 8
//     points for its own query; coordinates come as LDS broadcasts
//     (ds_read_b128 of 4 points per axis);
//   * sparse round (<= 32 lanes need it): the (needing query, point) pairs are
//     compacted onto the 64 lanes, slot = pair & (C2-1), point = pair >> log2 C2
//     with C2 = next pow2 >= #needing lanes; a lane reads its query (xyz + k-th)
//     and point from LDS and appends a hit to the owner's candidate column with
//     an LDS atomic (faster on gfx950 than a ballot/bpermute formulation).
// Candidates (d2 < k-th) go to per-lane LDS columns of CAP = 16 slots; after a
// round, if any lane holds more than CAP - R, the wave merges: bitonic sort of
// the column + bitonic merge into the sorted register top-K_CAP (K_CAP - k
// -inf sentinels keep the k-th at index K_CAP-1).  The merge network exists at
// exactly one site in the code (an inlined-per-point network thrashes the
// instruction cache).
#include "internal.hpp"
#include "metric.hpp"
#include "packet.hpp"

#include <cstdlib>

// A/B only: the production library (no NBKD_EXPERIMENTS) always has a seed
// bound and runs the collect / select path (knn_collect.hip).
#ifdef NBKD_EXPERIMENTS
namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64;

// CAP: candidate slots per lane; R: points per round; CHUNK: staged leaf points
template <int CAP, int CHUNK> struct WaveLds {
    union {
        struct {
            float bd[CAP][64];
            uint32_t bi[CAP][64];
        };
        uint32_t stage[2 * CAP * 64]; // output staging after the traversal
    };
    float4 qt[64]; // query xyz + current k-th
    uint32_t cnt[64];
    uint8_t owners[64];
    float px[CHUNK], py[CHUNK], pz[CHUNK];
};

// LDS of one wave of the streaming kernel: CAPS candidate slots per lane (the
// merge network sorts pow2_ceil(CAPS)), and two CHUNK-point SoA buffers filled
// by direct global->LDS loads (no VGPR staging)
template <int CAPS, int CHUNK> struct StreamLds {
    union {
        struct {
            float bd[CAPS][64];
            uint32_t bi[CAPS][64];
        };
        uint32_t stage[2 * CAPS * 64]; // output staging after the traversal
    };
    float4 qt[64]; // query xyz + current k-th
    uint32_t cnt[64];
    uint8_t owners[64];
    float pb[2][3][CHUNK]; // [buffer][axis][point]
};

// MODE bit 1: distances-only networks (timing experiment, wrong indices);
// bit 2: between merges prune with the tightened bound max(td[KC-1-cnt], max
// buffered d) instead of the stale td[KC-1]; bit 3: load the node record before
// the box test so its latency overlaps the test
template <int KC, bool PER, int CAP, int R, int CHUNK, int OCC, int MODE>
__global__ void __launch_bounds__(TB, OCC)
knn4_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  uint32_t m, int k, const float *__restrict__ tg, float *__restrict__ out_d,
                  uint32_t *__restrict__ out_i, uint32_t *__restrict__ fail_list,
                  uint32_t *__restrict__ fail_count, unsigned long long *__restrict__ stats) {
    static_assert(CHUNK % R == 0 && CAP > R && CAP <= KC, "tuning");
    __shared__ WaveLds<CAP, CHUNK> Wl[WPB];
    constexpr bool HOIST = (MODE & 8) != 0;
    constexpr bool IDX = (MODE & 2) == 0;
    // bit 4 (timing experiment): prune with the final k-th distance read from
    // out_d (a previous run's result), no merges, no output
    constexpr bool FIXEDR = (MODE & 16) != 0;
    // bit 5 (timing experiment, with bit 4): skip the leaf scans (traversal only)
    constexpr bool NOLEAF = (MODE & 32) != 0;
    // bit 6: per-lane direct output stores instead of the LDS-staged rows
    constexpr bool DIRECT = (MODE & 64) != 0;
    // bit 7: work counters (nbkd_stats_*); a separate instance so the production
    // kernel carries no counter registers
    constexpr bool STATS = (MODE & 128) != 0;
    // bit 8 (timing experiment): stage leaf chunks but skip their evaluation
    constexpr bool STAGEONLY = (MODE & 256) != 0;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds<CAP, CHUNK> &W = Wl[wave];
    const uint32_t gq = (blockIdx.x * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;

    // seed bound (leaf_key2_kernel's guess_r2): the k real slots of the top-k
    // start at (seed, none) instead of (FLT_MAX, none), so candidates and nodes
    // are pruned against min(seed, k-th) from the start with no extra register;
    // every accepted candidate is < seed, so a lane still holding a sentinel at
    // the end found fewer than k points inside the seed and is re-run by the
    // exact kernel (fail_list)
    const float seed = valid ? ((tg != nullptr) ? tg[qo] : FLT_MAX) : -INFINITY;
    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : seed;
        ti[j] = 0xFFFFFFFFu;
    }
    float kth = seed;
    if constexpr (FIXEDR) {
        if (valid) {
            const float r = out_d[(size_t)qo * k + (k - 1)];
            kth = r * r * 1.000001f;
        }
    }
    uint32_t cnt = 0;
    W.qt[lane] = make_float4(qx, qy, qz, kth);

    uint64_t n_nodes = 0, n_dense = 0, n_sparse = 0, n_merge = 0, n_evals = 0, n_cand = 0, n_fill = 0;
    WaveStack stk;
    stk.node = 0;
    stk.b0 = stk.b1 = stk.b2 = stk.b3 = stk.b4 = stk.b5 = 0.0f;
    int sp = 0;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;
    uint32_t node = 0;
    float b0 = PER ? 0.0f : -FLT_MAX, b1 = PER ? L : FLT_MAX;
    float b2 = b0, b3 = b1, b4 = b0, b5 = b1;
    bool have = true;
    uint32_t leaf_pos = 0, leaf_end = 0, chunk_base = 0, chunk_end = 0;
    uint64_t need = 0;

    for (;;) {
        bool done = false;
        if (leaf_pos >= leaf_end) {
            bool found = false;
            for (;;) {
                if (!have) {
                    if (sp == 0) break;
                    --sp;
                    node = __builtin_amdgcn_readlane(stk.node, sp);
                    b0 = rdlane(stk.b0, sp);
                    b1 = rdlane(stk.b1, sp);
                    b2 = rdlane(stk.b2, sp);
                    b3 = rdlane(stk.b3, sp);
                    b4 = rdlane(stk.b4, sp);
                    b5 = rdlane(stk.b5, sp);
                }
                have = false;
                nbkd_node nd;
                if constexpr (HOIST) nd = cnodes[node];
                const float box[6] = {b0, b1, b2, b3, b4, b5};
                const float bdist = box_d2<PER>(qx, qy, qz, box, L);
                const bool want = bdist <= kth;
                const uint64_t wm = __ballot(want);
                if (wm == 0) continue;
                if constexpr (STATS) ++n_nodes;
                if constexpr (!HOIST) nd = cnodes[node];
                const int dim = nd.dimension;
                if (dim < 0) {
                    leaf_pos = nd.left;
                    leaf_end = nd.right;
                    chunk_end = leaf_pos;
                    need = wm;
                    found = true;
                    break;
                }
                const float split = nd.split;
                const float qd = dim == 0 ? qx : (dim == 1 ? qy : qz);
                const uint32_t right_votes = (uint32_t)__popcll(__ballot(want && qd > split));
                const bool right_first = 2 * right_votes > (uint32_t)__popcll(wm);
                // left child: hi[dim] = split; right child: lo[dim] = split
                const int far_slot = right_first ? 2 * dim + 1 : 2 * dim;
                const int near_slot = right_first ? 2 * dim : 2 * dim + 1;
                float fb[6] = {b0, b1, b2, b3, b4, b5};
#pragma unroll
                for (int a = 0; a < 6; ++a) fb[a] = a == far_slot ? split : fb[a];
                const uint32_t far_node = right_first ? nd.left : nd.right;
                NBKD_PUSH(sp, far_node, fb);
                node = right_first ? nd.right : nd.left;
                b0 = near_slot == 0 ? split : b0;
                b1 = near_slot == 1 ? split : b1;
                b2 = near_slot == 2 ? split : b2;
                b3 = near_slot == 3 ? split : b3;
                b4 = near_slot == 4 ? split : b4;
                b5 = near_slot == 5 ? split : b5;
                have = true;
            }
            if (!found) done = true;
        }
        if (NOLEAF && !done) {
            if constexpr (STATS) n_evals += (uint64_t)(leaf_end - leaf_pos) * (uint32_t)__popcll(need);
            leaf_pos = leaf_end;
        } else if (!done) {
            if (leaf_pos >= chunk_end) { // stage the next <= 64 points of the leaf
                const uint32_t cn = min((uint32_t)CHUNK, leaf_end - leaf_pos);
                if ((uint32_t)lane < cn) {
                    W.px[lane] = t.x[leaf_pos + lane];
                    W.py[lane] = t.y[leaf_pos + lane];
                    W.pz[lane] = t.z[leaf_pos + lane];
                }
                chunk_base = leaf_pos;
                chunk_end = leaf_pos + cn;
                wave_sync();
            }
            const uint32_t off = leaf_pos - chunk_base; // multiple of 8: leaves are
            const uint32_t nneed = (uint32_t)__popcll(need); // multiples of 8 points
            if (STAGEONLY) {
                leaf_pos = chunk_end - R;
            } else if (nneed > 32) {
                if constexpr (STATS) {
                    ++n_dense;
                    n_evals += (uint64_t)R * 64;
                }
                float px[R], py[R], pz[R];
#pragma unroll
                for (int u = 0; u < R; u += 4) {
                    const float4 xv = *reinterpret_cast<const float4 *>(&W.px[off + u]);
                    const float4 yv = *reinterpret_cast<const float4 *>(&W.py[off + u]);
                    const float4 zv = *reinterpret_cast<const float4 *>(&W.pz[off + u]);
                    px[u] = xv.x; px[u + 1] = xv.y; px[u + 2] = xv.z; px[u + 3] = xv.w;
                    py[u] = yv.x; py[u + 1] = yv.y; py[u + 2] = yv.z; py[u + 3] = yv.w;
                    pz[u] = zv.x; pz[u + 1] = zv.y; pz[u + 2] = zv.z; pz[u + 3] = zv.w;
                }
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    const float d = point_d2<PER>(qx, qy, qz, px[u], py[u], pz[u], L);
                    if (d < kth) {
                        W.bd[cnt][lane] = d;
                        W.bi[cnt][lane] = leaf_pos + u;
                        ++cnt;
                    }
                }
            } else {
                W.cnt[lane] = cnt;
                if ((need >> lane) & 1ull) W.owners[mbcnt64(need)] = lane;
                wave_sync();
                // C2 = next power of two >= nneed
                uint32_t c2 = 1;
                while (c2 < nneed) c2 <<= 1;
                const uint32_t lgc = (uint32_t)__builtin_ctz(c2);
                if constexpr (STATS) n_evals += (uint64_t)R * nneed;
                const uint32_t pairs = (uint32_t)R << lgc;
                for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                    if constexpr (STATS) ++n_sparse;
                    const uint32_t pi = p0 + lane;
                    const uint32_t slot = pi & (c2 - 1u), pr = pi >> lgc;
                    if (slot < nneed && pi < pairs) {
                        const uint32_t owner = W.owners[slot];
                        const float4 qq = W.qt[owner];
                        const float d = point_d2<PER>(qq.x, qq.y, qq.z, W.px[off + pr],
                                                      W.py[off + pr], W.pz[off + pr], L);
                        if (d < qq.w) {
                            const uint32_t sl = atomicAdd(&W.cnt[owner], 1u);
                            W.bd[sl][owner] = d;
                            W.bi[sl][owner] = leaf_pos + pr;
                        }
                    }
                }
                wave_sync();
                cnt = W.cnt[lane];
            }
            leaf_pos += R;
        }
        const bool merge = __any(cnt > (uint32_t)(CAP - R)) || (done && __any(cnt > 0));
        if (FIXEDR && merge) {
            if constexpr (STATS) {
                ++n_merge;
                uint32_t c = cnt;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                n_cand += c;
            }
            cnt = 0;
        } else if (merge) {
            if constexpr (STATS) {
                ++n_merge;
                n_cand += (uint64_t)__builtin_amdgcn_readfirstlane(0u);
                uint32_t c = cnt;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                n_cand += c;
                n_fill += __any(kth == FLT_MAX) ? 1u : 0u;
            }
            float bd[CAP];
            uint32_t bi[CAP];
#pragma unroll
            for (int s = 0; s < CAP; ++s) {
                const float dv = W.bd[s][lane];
                const uint32_t iv = W.bi[s][lane];
                const bool have = (uint32_t)s < cnt;
                bd[s] = have ? dv : INFINITY;
                bi[s] = have ? iv : 0xFFFFFFFFu;
            }
            bitonic_sort<CAP, IDX>(bd, bi);
#pragma unroll
            for (int s = 0; s < CAP; ++s) {
                const int pos = KC - CAP + s, o = CAP - 1 - s;
                const bool take = bd[o] < td[pos];
                td[pos] = take ? bd[o] : td[pos];
                ti[pos] = take ? bi[o] : ti[pos];
            }
            bitonic_merge<KC, IDX>(td, ti);
            if (valid) kth = td[KC - 1];
            cnt = 0;
            W.qt[lane].w = kth;
        }
        if (done) break;
    }

    if constexpr (DIRECT && !FIXEDR) {
        knn_fail_check<PER>(valid, tg != nullptr, ti[KC - 1], qx, qy, qz, L, qo, fail_list,
                            fail_count);
        if (valid) {
            const size_t row = (size_t)qo * (size_t)k;
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                if (j >= KC - k) {
                    out_d[row + (j - (KC - k))] = sqrtf(td[j]);
                    const uint32_t p = ti[j];
                    out_i[row + (j - (KC - k))] = p == 0xFFFFFFFFu ? p : t.idx[p];
                }
            }
        }
    } else if constexpr (!FIXEDR) {
        knn_fail_check<PER>(valid, tg != nullptr, ti[KC - 1], qx, qy, qz, L, qo, fail_list,
                            fail_count);
        // Output rows (k floats / ids per query) are staged through the wave's
        // candidate columns (2*CAP*64 words) so that each store instruction
        // writes whole contiguous rows instead of 64 scattered dwords.
        // Column-major with an XOR swizzle: word (c, row) at c*64 + (row ^ c),
        // conflict-free for both the per-lane column writes and the row reads.
        W.cnt[lane] = valid ? qo : 0xFFFFFFFFu;
        // register j of the top-KC is output column j - (KC - k)
        constexpr int CC = 2 * CAP < KC ? 2 * CAP : KC; // registers staged per pass
#pragma unroll
        for (int j0 = 0; j0 < KC; j0 += CC) {
            wave_sync();
#pragma unroll
            for (int j = 0; j < CC; ++j) W.stage[j * 64 + (lane ^ j)] = __float_as_uint(sqrtf(td[j0 + j]));
            wave_sync();
            store_rows<CC>(W.stage, W.cnt, reinterpret_cast<uint32_t *>(out_d), k, j0 - (KC - k), lane);
        }
#pragma unroll
        for (int j0 = 0; j0 < KC; j0 += CC) {
            wave_sync();
#pragma unroll
            for (int j = 0; j < CC; ++j) W.stage[j * 64 + (lane ^ j)] = ti[j0 + j];
            wave_sync();
            store_rows<CC>(W.stage, W.cnt, out_i, k, j0 - (KC - k), lane, t.idx);
        }
    }
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (STATS && lane == 0) {
        atomicAdd(&stats[0], (unsigned long long)n_nodes * nvalid);
        atomicAdd(&stats[1], (unsigned long long)n_evals);
        atomicAdd(&stats[2], (unsigned long long)n_dense);
        atomicAdd(&stats[3], (unsigned long long)n_sparse);
        atomicAdd(&stats[4], (unsigned long long)n_merge);
        atomicAdd(&stats[5], 1ull);
        atomicAdd(&stats[6], (unsigned long long)n_cand);
        atomicAdd(&stats[7], (unsigned long long)n_fill);
    }
}

struct KnnArgs {
    const float *tg;
    float *od;
    uint32_t *oi;
    uint32_t *fail_list, *fail_count;
    unsigned long long *stats;
};

// ------------------------------------------------------------------ streaming packet kNN
// Same packet semantics as knn4_kernel, restructured so that no memory latency
// sits on the critical path of the leaf scans:
//   phase A  the wave walks the tree (near-first by majority vote, pruning
//            against the current k-th of each lane) and lists up to 64 wanted
//            leaves (node ids, one per lane of a VGPR) without touching points;
//   phase B  it streams the listed leaves chunk by chunk: the points of chunk
//            c+1 (and the leafinfo record of leaf l+2) are loaded while chunk c
//            is evaluated; each leaf is re-tested against the lanes' current
//            k-th with its TIGHT bounding box (leafinfo), which also prunes
//            better than the split-plane box.
// Phase A resumes from its stack after phase B, with the tightened bounds.
template <int KC, bool PER, int CAPS, int R, int CHUNK, int OCC, bool STATS>
__global__ void __launch_bounds__(TB, OCC)
knn5_kernel(DevTree t, const uint32_t *__restrict__ linfo, const float *__restrict__ q,
            const uint32_t *__restrict__ order, uint32_t m, int k, const float *__restrict__ tg,
            float *__restrict__ out_d, uint32_t *__restrict__ out_i,
            uint32_t *__restrict__ fail_list, uint32_t *__restrict__ fail_count,
            unsigned long long *__restrict__ stats) {
    constexpr int NS = pow2_ceil(CAPS); // merge network size
    static_assert(CHUNK % R == 0 && CHUNK <= 64 && CAPS > R && NS <= KC, "tuning");
    __shared__ StreamLds<CAPS, CHUNK> Wl[WPB];

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    StreamLds<CAPS, CHUNK> &W = Wl[wave];
    const uint32_t gq = (blockIdx.x * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;

    // seed bound: see knn4_kernel
    const float seed = valid ? ((tg != nullptr) ? tg[qo] : FLT_MAX) : -INFINITY;
    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : seed;
        ti[j] = 0xFFFFFFFFu;
    }
    float kth = seed;
    uint32_t cnt = 0;
    W.qt[lane] = make_float4(qx, qy, qz, kth);

    uint64_t n_nodes = 0, n_dense = 0, n_sparse = 0, n_merge = 0, n_evals = 0, n_cand = 0, n_leaf = 0;
    WaveStack stk;
    stk.node = 0;
    stk.b0 = stk.b1 = stk.b2 = stk.b3 = stk.b4 = stk.b5 = 0.0f;
    int sp = 0;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;
    uint32_t node = 0;
    float b0 = PER ? 0.0f : -FLT_MAX, b1 = PER ? L : FLT_MAX;
    float b2 = b0, b3 = b1, b4 = b0, b5 = b1;
    bool have = true, tree_done = false;

    for (;;) {
        // ---------------------------------------------------------- phase A
        uint32_t lst = 0, nl = 0;
        while (nl < 64u) {
            if (!have) {
                if (sp == 0) {
                    tree_done = true;
                    break;
                }
                --sp;
                node = __builtin_amdgcn_readlane(stk.node, sp);
                b0 = rdlane(stk.b0, sp);
                b1 = rdlane(stk.b1, sp);
                b2 = rdlane(stk.b2, sp);
                b3 = rdlane(stk.b3, sp);
                b4 = rdlane(stk.b4, sp);
                b5 = rdlane(stk.b5, sp);
            }
            have = false;
            const nbkd_node nd = cnodes[node];
            const float box[6] = {b0, b1, b2, b3, b4, b5};
            const float bdist = box_d2<PER>(qx, qy, qz, box, L);
            const bool want = bdist <= kth;
            const uint64_t wm = __ballot(want);
            if (wm == 0) continue;
            if constexpr (STATS) ++n_nodes;
            const int dim = nd.dimension;
            if (dim < 0) {
                lst = lane == (int)nl ? node : lst;
                ++nl;
                continue;
            }
            const float split = nd.split;
            const float qd = dim == 0 ? qx : (dim == 1 ? qy : qz);
            const uint32_t right_votes = (uint32_t)__popcll(__ballot(want && qd > split));
            const bool right_first = 2 * right_votes > (uint32_t)__popcll(wm);
            // left child: hi[dim] = split; right child: lo[dim] = split
            const int far_slot = right_first ? 2 * dim + 1 : 2 * dim;
            const int near_slot = right_first ? 2 * dim : 2 * dim + 1;
            float fb[6] = {b0, b1, b2, b3, b4, b5};
#pragma unroll
            for (int a = 0; a < 6; ++a) fb[a] = a == far_slot ? split : fb[a];
            const uint32_t far_node = right_first ? nd.left : nd.right;
            NBKD_PUSH(sp, far_node, fb);
            node = right_first ? nd.right : nd.left;
            b0 = near_slot == 0 ? split : b0;
            b1 = near_slot == 1 ? split : b1;
            b2 = near_slot == 2 ? split : b2;
            b3 = near_slot == 3 ? split : b3;
            b4 = near_slot == 4 ? split : b4;
            b5 = near_slot == 5 ? split : b5;
            have = true;
        }

        // ---------------------------------------------------------- phase B
        // info: lanes 8h..8h+7 hold the 8 leafinfo words of listed leaf j with
        // j & 1 == h (two leaves resident: the current one and the next)
        uint32_t info = 0;
        if (nl > 0) {
            const uint32_t h = (uint32_t)lane >> 3;
            const uint32_t n0 = __builtin_amdgcn_readlane(lst, 0);
            const uint32_t n1 = __builtin_amdgcn_readlane(lst, nl > 1 ? 1 : 0);
            if (lane < 16 && h < nl) info = linfo[8 * (size_t)(h ? n1 : n0) + (lane & 7)];
        }
        // cursor of the chunk being evaluated (leaf li, points [cpos, cpos+cn))
        uint32_t li = 0, lend = 0, cpos = 0, cn = 0, off = 0, buf = 0;
        uint64_t need = 0;
        bool active = nl > 0;
        if (active) {
            cpos = __builtin_amdgcn_readlane(info, 6);
            lend = __builtin_amdgcn_readlane(info, 7);
            cn = min((uint32_t)CHUNK, lend - cpos);
            glds_f32(t.x + cpos, W.pb[0][0], lane, cn);
            glds_f32(t.y + cpos, W.pb[0][1], lane, cn);
            glds_f32(t.z + cpos, W.pb[0][2], lane, cn);
        }
        for (;;) {
            const bool ended = !active;
            if (active) {
                const float *px_ = W.pb[buf][0], *py_ = W.pb[buf][1], *pz_ = W.pb[buf][2];
                if (off == 0) {
                    // the chunk's direct-to-LDS loads (and the info loads) have landed
                    wait_vm0();
                    wave_sync();
                    if (cpos == __builtin_amdgcn_readlane(info, 8 * (li & 1) + 6)) {
                        // first chunk of leaf li: test its tight box, then reuse
                        // its info slot for leaf li + 2
                        const int hb = 8 * (int)(li & 1);
                        const float bx[6] = {rdlane(__uint_as_float(info), hb + 0),
                                             rdlane(__uint_as_float(info), hb + 3),
                                             rdlane(__uint_as_float(info), hb + 1),
                                             rdlane(__uint_as_float(info), hb + 4),
                                             rdlane(__uint_as_float(info), hb + 2),
                                             rdlane(__uint_as_float(info), hb + 5)};
                        need = __ballot(box_d2<PER>(qx, qy, qz, bx, L) <= kth);
                        if constexpr (STATS) n_leaf += need != 0;
                        if (li + 2 < nl) {
                            const uint32_t n2 = __builtin_amdgcn_readlane(lst, (int)li + 2);
                            if ((lane >> 3) == (int)(li & 1)) info = linfo[8 * (size_t)n2 + (lane & 7)];
                        }
                    }
                    // next chunk: rest of this leaf, or the first chunk of leaf li + 1
                    uint32_t npos = cpos + cn;
                    if (npos >= lend && li + 1 < nl) npos = __builtin_amdgcn_readlane(info, 8 * ((li + 1) & 1) + 6);
                    const uint32_t nend = (cpos + cn >= lend && li + 1 < nl)
                                               ? __builtin_amdgcn_readlane(info, 8 * ((li + 1) & 1) + 7)
                                               : lend;
                    if (cpos + cn < lend || li + 1 < nl) {
                        const uint32_t ncn = min((uint32_t)CHUNK, nend - npos);
                        glds_f32(t.x + npos, W.pb[buf ^ 1][0], lane, ncn);
                        glds_f32(t.y + npos, W.pb[buf ^ 1][1], lane, ncn);
                        glds_f32(t.z + npos, W.pb[buf ^ 1][2], lane, ncn);
                    }
                }
                const uint32_t nneed = (uint32_t)__popcll(need);
                if (nneed > 32) {
                    if constexpr (STATS) {
                        ++n_dense;
                        n_evals += (uint64_t)R * 64;
                    }
                    float px[R], py[R], pz[R];
#pragma unroll
                    for (int u = 0; u < R; u += 4) {
                        const float4 xv = *reinterpret_cast<const float4 *>(&px_[off + u]);
                        const float4 yv = *reinterpret_cast<const float4 *>(&py_[off + u]);
                        const float4 zv = *reinterpret_cast<const float4 *>(&pz_[off + u]);
                        px[u] = xv.x; px[u + 1] = xv.y; px[u + 2] = xv.z; px[u + 3] = xv.w;
                        py[u] = yv.x; py[u + 1] = yv.y; py[u + 2] = yv.z; py[u + 3] = yv.w;
                        pz[u] = zv.x; pz[u + 1] = zv.y; pz[u + 2] = zv.z; pz[u + 3] = zv.w;
                    }
#pragma unroll
                    for (int u = 0; u < R; ++u) {
                        const float d = point_d2<PER>(qx, qy, qz, px[u], py[u], pz[u], L);
                        if (d < kth) {
                            W.bd[cnt][lane] = d;
                            W.bi[cnt][lane] = cpos + off + u;
                            ++cnt;
                        }
                    }
                } else if (nneed > 0) {
                    W.cnt[lane] = cnt;
                    if ((need >> lane) & 1ull) W.owners[mbcnt64(need)] = lane;
                    wave_sync();
                    uint32_t c2 = 1;
                    while (c2 < nneed) c2 <<= 1;
                    const uint32_t lgc = (uint32_t)__builtin_ctz(c2);
                    if constexpr (STATS) n_evals += (uint64_t)R * nneed;
                    const uint32_t pairs = (uint32_t)R << lgc;
                    for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                        if constexpr (STATS) ++n_sparse;
                        const uint32_t pi = p0 + lane;
                        const uint32_t slot = pi & (c2 - 1u), pr = off + (pi >> lgc);
                        if (slot < nneed && pi < pairs) {
                            const uint32_t owner = W.owners[slot];
                            const float4 qq = W.qt[owner];
                            const float d = point_d2<PER>(qq.x, qq.y, qq.z, px_[pr], py_[pr],
                                                          pz_[pr], L);
                            if (d < qq.w) {
                                const uint32_t sl = atomicAdd(&W.cnt[owner], 1u);
                                W.bd[sl][owner] = d;
                                W.bi[sl][owner] = cpos + pr;
                            }
                        }
                    }
                    wave_sync();
                    cnt = W.cnt[lane];
                }
                // advance the cursor by one round
                off += R;
                if (off >= cn) {
                    off = 0;
                    buf ^= 1u;
                    cpos += cn;
                    if (cpos >= lend) {
                        ++li;
                        if (li < nl) {
                            cpos = __builtin_amdgcn_readlane(info, 8 * (li & 1) + 6);
                            lend = __builtin_amdgcn_readlane(info, 8 * (li & 1) + 7);
                        } else {
                            active = false;
                        }
                    }
                    if (active) cn = min((uint32_t)CHUNK, lend - cpos);
                }
            }
            const bool fin = ended && tree_done;
            const bool merge = __any(cnt > (uint32_t)(CAPS - R)) || (fin && __any(cnt > 0));
            if (merge) {
                if constexpr (STATS) {
                    ++n_merge;
                    uint32_t c = cnt;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                    n_cand += c;
                }
                float bd[NS];
                uint32_t bi[NS];
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    if (s < CAPS) {
                        const float dv = W.bd[s][lane];
                        const uint32_t iv = W.bi[s][lane];
                        const bool hv = (uint32_t)s < cnt;
                        bd[s] = hv ? dv : INFINITY;
                        bi[s] = hv ? iv : 0xFFFFFFFFu;
                    } else {
                        bd[s] = INFINITY;
                        bi[s] = 0xFFFFFFFFu;
                    }
                }
                bitonic_sort<NS>(bd, bi);
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int pos = KC - NS + s, o = NS - 1 - s;
                    const bool take = bd[o] < td[pos];
                    td[pos] = take ? bd[o] : td[pos];
                    ti[pos] = take ? bi[o] : ti[pos];
                }
                bitonic_merge<KC>(td, ti);
                if (valid) kth = td[KC - 1];
                cnt = 0;
                W.qt[lane].w = kth;
            }
            if (ended) break;
        }
        if (tree_done) break;
    }

    knn_fail_check<PER>(valid, tg != nullptr, ti[KC - 1], qx, qy, qz, L, qo, fail_list, fail_count);
    W.cnt[lane] = valid ? qo : 0xFFFFFFFFu;
    constexpr int CC = pow2_floor(2 * CAPS < KC ? 2 * CAPS : KC); // registers staged per pass
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j) W.stage[j * 64 + (lane ^ j)] = __float_as_uint(sqrtf(td[j0 + j]));
        wave_sync();
        store_rows<CC>(W.stage, W.cnt, reinterpret_cast<uint32_t *>(out_d), k, j0 - (KC - k), lane);
    }
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j) W.stage[j * 64 + (lane ^ j)] = ti[j0 + j];
        wave_sync();
        store_rows<CC>(W.stage, W.cnt, out_i, k, j0 - (KC - k), lane, t.idx);
    }
    if (STATS && lane == 0) {
        const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
        atomicAdd(&stats[0], (unsigned long long)n_nodes * nvalid);
        atomicAdd(&stats[1], (unsigned long long)n_evals);
        atomicAdd(&stats[2], (unsigned long long)n_dense);
        atomicAdd(&stats[3], (unsigned long long)n_sparse);
        atomicAdd(&stats[4], (unsigned long long)n_merge);
        atomicAdd(&stats[5], 1ull);
        atomicAdd(&stats[6], (unsigned long long)n_cand);
        atomicAdd(&stats[7], (unsigned long long)n_leaf);
    }
}

template <int KC, int CAPS, int R, int CHUNK, int OCC>
void launch5(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
             const struct KnnArgs &a, hipStream_t s);

template <int KC, int CAP, int R, int CHUNK, int OCC, int MODE = 0>
void launch4(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
             const KnnArgs &a, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        if (a.stats)
            knn4_kernel<KC, true, CAP, R, CHUNK, OCC, MODE | 128><<<blocks, TB, 0, s>>>(
                view(t), q, order, m, k, a.tg, a.od, a.oi, a.fail_list, a.fail_count, a.stats);
        else
            knn4_kernel<KC, true, CAP, R, CHUNK, OCC, MODE><<<blocks, TB, 0, s>>>(
                view(t), q, order, m, k, a.tg, a.od, a.oi, a.fail_list, a.fail_count, nullptr);
    else if (a.stats)
        knn4_kernel<KC, false, CAP, R, CHUNK, OCC, MODE | 128><<<blocks, TB, 0, s>>>(
            view(t), q, order, m, k, a.tg, a.od, a.oi, a.fail_list, a.fail_count, a.stats);
    else
        knn4_kernel<KC, false, CAP, R, CHUNK, OCC, MODE><<<blocks, TB, 0, s>>>(
            view(t), q, order, m, k, a.tg, a.od, a.oi, a.fail_list, a.fail_count, nullptr);
}

template <int KC, int CAPS, int R, int CHUNK, int OCC>
void launch5(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
             const KnnArgs &a, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
#define NBKD_K5(PER, ST)                                                                           \
    knn5_kernel<KC, PER, CAPS, R, CHUNK, OCC, ST><<<blocks, TB, 0, s>>>(                            \
        view(t), t.leafinfo, q, order, m, k, a.tg, a.od, a.oi, a.fail_list, a.fail_count,        \
        ST ? a.stats : nullptr)
    if (t.periodic) {
        if (a.stats) NBKD_K5(true, true); else NBKD_K5(true, false);
    } else {
        if (a.stats) NBKD_K5(false, true); else NBKD_K5(false, false);
    }
#undef NBKD_K5
}

int variant() {
    const char *e = knob("NBKD_KNN_VARIANT"); // read per call: tuning sweeps flip it
    return e ? atoi(e) : 0;
}

} // namespace

void launch_knn_packet(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
                       const float *tg, float *od, uint32_t *oi, uint32_t *fail_list,
                       uint32_t *fail_count, unsigned long long *stats, hipStream_t s) {
    const int v = variant();
    const KnnArgs a{tg, od, oi, fail_list, fail_count, stats};
    if (k <= 16) {
        launch4<16, 16, 8, 32, 4, 8>(t, q, order, m, k, a, s);
    } else if (k <= 32) {
        switch (v) { // tuning experiments (NBKD_KNN_VARIANT); see DESIGN.md
        case 1: launch4<32, 16, 8, 32, 3, 8>(t, q, order, m, k, a, s); break;  // 3 waves/SIMD, no spill
        case 3: launch4<32, 16, 8, 32, 4, 10>(t, q, order, m, k, a, s); break; // d-only (timing)
        case 4: launch4<32, 16, 8, 32, 4, 24>(t, q, order, m, k, a, s); break; // fixed r (timing)
        case 5: launch4<32, 16, 8, 32, 4, 56>(t, q, order, m, k, a, s); break; // fixed r, no leaves
        case 6: launch4<32, 16, 8, 32, 4, 72>(t, q, order, m, k, a, s); break; // direct stores
        case 7: launch4<32, 16, 8, 32, 4, 280>(t, q, order, m, k, a, s); break; // fixed r, stage only
        case 8: launch5<32, 15, 8, 32, 4>(t, q, order, m, k, a, s); break;        // streaming
        case 9: launch5<32, 16, 8, 32, 3>(t, q, order, m, k, a, s); break;        // streaming, 3 waves
        default: launch4<32, 16, 8, 32, 4, 8>(t, q, order, m, k, a, s); break;
        }
    } else {
        launch4<64, 16, 8, 32, 2, 8>(t, q, order, m, k, a, s);
    }
}

} // namespace nbkd
#endif // NBKD_EXPERIMENTS
