// Packet kNN kernel, v2 (gfx950).  See query.hip for the reference semantics.
//
// One wave64 = one packet of 64 kd-ordered queries (one per lane).  The wave
// walks the tree once (stack of node id + box in VGPRs, one entry per lane);
// a node is entered iff some lane's box distance <= that lane's k-th distance,
// and `need` = the mask of those lanes.  Each leaf chunk (<= 64 points) is
// staged once into LDS with coalesced SoA loads, then processed in rounds of
// R = 8 points:
//   * dense round  (> 32 lanes need the leaf): every lane evaluates the 8
//     points for its own query; coordinates come as LDS broadcasts
//     (ds_read_b128 of 4 points per axis);
//   * sparse round (<= 32 lanes need it): the (needing query, point) pairs are
//     compacted onto the 64 lanes, slot = pair & (C2-1), point = pair >> log2 C2
//     with C2 = next pow2 >= #needing lanes; a lane reads its query (xyz + k-th)
//     and point from LDS and appends a hit to the owner's candidate column with
//     an LDS atomic.  Saves the wasted lane-work of the packet union.
// Candidates (d2 < k-th) go to per-lane LDS columns of CAP = 16 slots; after a
// round, if any lane holds more than CAP - R, the wave merges: bitonic sort of
// the column + bitonic merge into the sorted register top-K_CAP (K_CAP - k
// -inf sentinels keep the k-th at index K_CAP-1).  The merge network exists at
// exactly one site in the code (a 1100-instruction network inlined per point
// thrashed the instruction cache in v1).
#include "internal.hpp"
#include "metric.hpp"

#include <cstdlib>

namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64;

// CAP: candidate slots per lane; R: points per round; CHUNK: staged leaf points
template <int CAP, int CHUNK> struct WaveLds {
    float bd[CAP][64];
    uint32_t bi[CAP][64];
    float4 qt[64]; // query xyz + current k-th
    uint32_t cnt[64];
    uint32_t owners[64];
    float px[CHUNK], py[CHUNK], pz[CHUNK];
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int KC, bool PER, int CAP, int R, int CHUNK, int OCC>
__global__ void __launch_bounds__(TB, OCC)
knn_packet_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  uint32_t m, int k, float *__restrict__ out_d, uint32_t *__restrict__ out_i,
                  unsigned long long *__restrict__ stats) {
    static_assert(CHUNK % R == 0 && CAP > R && CAP <= KC, "tuning");
    __shared__ WaveLds<CAP, CHUNK> Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds<CAP, CHUNK> &W = Wl[wave];
    const uint32_t gq = (blockIdx.x * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;

    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : FLT_MAX;
        ti[j] = 0xFFFFFFFFu;
    }
    float kth = valid ? FLT_MAX : -INFINITY;
    uint32_t cnt = 0;
    W.qt[lane] = make_float4(qx, qy, qz, kth);

    uint64_t n_nodes = 0, n_dense = 0, n_sparse = 0, n_merge = 0, n_evals = 0;
    WaveStack stk;
    stk.node = 0;
    stk.b0 = stk.b1 = stk.b2 = stk.b3 = stk.b4 = stk.b5 = 0.0f;
    int sp = 0;
    {
        float box[6];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            box[2 * a] = PER ? 0.0f : -FLT_MAX;
            box[2 * a + 1] = PER ? L : FLT_MAX;
        }
        NBKD_PUSH(sp, 0u, box);
    }
    uint32_t leaf_pos = 0, leaf_end = 0, chunk_base = 0, chunk_end = 0;
    uint64_t need = 0;

    for (;;) {
        bool done = false;
        if (leaf_pos >= leaf_end) {
            bool found = false;
            while (sp > 0) {
                --sp;
                const uint32_t node = __builtin_amdgcn_readlane(stk.node, sp);
                float box[6] = {rdlane(stk.b0, sp), rdlane(stk.b1, sp), rdlane(stk.b2, sp),
                                rdlane(stk.b3, sp), rdlane(stk.b4, sp), rdlane(stk.b5, sp)};
                const float bdist = box_d2<PER>(qx, qy, qz, box, L);
                const bool want = bdist <= kth;
                const uint64_t wm = __ballot(want);
                if (wm == 0) continue;
                ++n_nodes;
                const nbkd_node nd = t.nodes[node];
                const int dim = (int)uni((uint32_t)nd.dimension);
                if (dim < 0) {
                    leaf_pos = uni(nd.left);
                    leaf_end = uni(nd.right);
                    chunk_end = leaf_pos;
                    need = wm;
                    found = true;
                    break;
                }
                const float split = unif(nd.split);
                const uint32_t lchild = uni(nd.left), rchild = uni(nd.right);
                const float qd = dim == 0 ? qx : (dim == 1 ? qy : qz);
                const uint32_t right_votes = (uint32_t)__popcll(__ballot(want && qd > split));
                const bool right_first = 2 * right_votes > (uint32_t)__popcll(wm);
                float lbox[6], rbox[6];
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    lbox[a] = box[a];
                    rbox[a] = box[a];
                }
                if (dim == 0) {
                    lbox[1] = split;
                    rbox[0] = split;
                } else if (dim == 1) {
                    lbox[3] = split;
                    rbox[2] = split;
                } else {
                    lbox[5] = split;
                    rbox[4] = split;
                }
                if (right_first) {
                    NBKD_PUSH(sp, lchild, lbox);
                    NBKD_PUSH(sp, rchild, rbox);
                } else {
                    NBKD_PUSH(sp, rchild, rbox);
                    NBKD_PUSH(sp, lchild, lbox);
                }
            }
            if (!found) done = true;
        }
        if (!done) {
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
            if (nneed > 32) {
                ++n_dense;
                n_evals += (uint64_t)R * 64;
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
                n_evals += (uint64_t)R * nneed;
                const uint32_t pairs = (uint32_t)R << lgc;
                for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                    ++n_sparse;
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
        if (merge) {
            ++n_merge;
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
            bitonic_sort<CAP>(bd, bi);
#pragma unroll
            for (int s = 0; s < CAP; ++s) {
                const int pos = KC - CAP + s, o = CAP - 1 - s;
                const bool take = bd[o] < td[pos];
                td[pos] = take ? bd[o] : td[pos];
                ti[pos] = take ? bi[o] : ti[pos];
            }
            bitonic_merge<KC>(td, ti);
            if (valid) kth = td[KC - 1];
            cnt = 0;
            W.qt[lane].w = kth;
        }
        if (done) break;
    }

    if (valid) {
        const int skip = KC - k;
        const size_t row = (size_t)qo * (size_t)k;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= skip) {
                out_d[row + (j - skip)] = sqrtf(td[j]);
                const uint32_t p = ti[j];
                out_i[row + (j - skip)] = p == 0xFFFFFFFFu ? p : t.idx[p];
            }
        }
    }
    if (stats && lane == 0) {
        const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
        atomicAdd(&stats[0], (unsigned long long)n_nodes * nvalid);
        atomicAdd(&stats[1], (unsigned long long)n_evals);
        atomicAdd(&stats[2], (unsigned long long)n_dense);
        atomicAdd(&stats[3], (unsigned long long)n_sparse);
        atomicAdd(&stats[4], (unsigned long long)n_merge);
        atomicAdd(&stats[5], 1ull);
    }
}

// ---------------------------------------------------------------- v3
// Differences to v2: the wave descends into the near child directly (its box
// stays wave-uniform) and pushes only the far child; node records come through
// the scalar cache (constant address space -> s_load_dwordx4); candidates of a
// round are folded into the top-k before the next round (k-th always exact):
// with >= 4 pending in some lane, a merge of the 8-slot column (sort 8 + take +
// bitonic merge K_CAP), otherwise one sorted-insertion step per pending
// candidate (5 VALU per element).  8 LDS slots per lane, 16 merge temporaries.
template <int N>
__device__ __forceinline__ void insert_sorted(float (&d)[N], uint32_t (&id)[N], float v,
                                              uint32_t vi) {
    // new[j] = v < d[j-1] ? d[j-1] : (v < d[j] ? v : d[j]); ties keep the older entry first
    bool c_hi = v < d[N - 1];
#pragma unroll
    for (int j = N - 1; j > 0; --j) {
        const bool c_lo = v < d[j - 1];
        const float nd = c_lo ? d[j - 1] : (c_hi ? v : d[j]);
        const uint32_t ni = c_lo ? id[j - 1] : (c_hi ? vi : id[j]);
        d[j] = nd;
        id[j] = ni;
        c_hi = c_lo;
        if ((j & 3) == 0) __builtin_amdgcn_sched_barrier(0);
    }
    d[0] = c_hi ? v : d[0];
    id[0] = c_hi ? vi : id[0];
}

// node records through the scalar cache: a constant-address-space view of the
// (read-only, wave-uniformly indexed) node table lowers to s_load_dwordx4
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) nbkd_node *cnode_ptr;
#else
typedef const nbkd_node *cnode_ptr;
#endif

template <int CHUNK> struct WaveLds3 {
    float bd[8][64];
    uint32_t bi[8][64];
    float4 qt[64];
    uint32_t cnt[64];
    uint32_t owners[64];
    float px[CHUNK], py[CHUNK], pz[CHUNK];
};

template <int KC, bool PER, int CHUNK, int OCC>
__global__ void __launch_bounds__(TB, OCC)
knn3_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order, uint32_t m,
            int k, float *__restrict__ out_d, uint32_t *__restrict__ out_i,
            unsigned long long *__restrict__ stats) {
    constexpr int R = 8;
    static_assert(CHUNK % R == 0, "tuning");
    __shared__ WaveLds3<CHUNK> Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds3<CHUNK> &W = Wl[wave];
    const uint32_t gq = (blockIdx.x * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;

    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : FLT_MAX;
        ti[j] = 0xFFFFFFFFu;
    }
    float kth = valid ? FLT_MAX : -INFINITY;
    W.qt[lane] = make_float4(qx, qy, qz, kth);

    uint64_t n_nodes = 0, n_dense = 0, n_sparse = 0, n_merge = 0, n_evals = 0, n_ins = 0;
    WaveStack stk;
    stk.node = 0;
    stk.b0 = stk.b1 = stk.b2 = stk.b3 = stk.b4 = stk.b5 = 0.0f;
    int sp = 0;
    // current node and its (wave-uniform) box
    uint32_t node = 0;
    float b0 = PER ? 0.0f : -FLT_MAX, b1 = PER ? L : FLT_MAX;
    float b2 = b0, b3 = b1, b4 = b0, b5 = b1;
    bool have = true;
    uint32_t leaf_pos = 0, leaf_end = 0, chunk_base = 0, chunk_end = 0;
    uint64_t need = 0;

    for (;;) {
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
                const float box[6] = {b0, b1, b2, b3, b4, b5};
                const float bdist = box_d2<PER>(qx, qy, qz, box, L);
                const bool want = bdist <= kth;
                const uint64_t wm = __ballot(want);
                if (wm == 0) continue;
                ++n_nodes;
                const nbkd_node nd = cnodes[node];
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
                // far child: its box = current box with one bound replaced by split
                float fb[6] = {b0, b1, b2, b3, b4, b5};
                // left child: hi[dim] = split; right child: lo[dim] = split
                const int far_slot = right_first ? 2 * dim + 1 : 2 * dim;
                const int near_slot = right_first ? 2 * dim : 2 * dim + 1;
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
            if (!found) break;
        }
        // ---- one round of R points of the current leaf
        if (leaf_pos >= chunk_end) {
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
        const uint32_t off = leaf_pos - chunk_base;
        const uint32_t nneed = (uint32_t)__popcll(need);
        uint32_t cnt = 0;
        if (nneed > 32) {
            ++n_dense;
            n_evals += (uint64_t)R * 64;
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
            W.cnt[lane] = 0;
            if ((need >> lane) & 1ull) W.owners[mbcnt64(need)] = lane;
            wave_sync();
            uint32_t c2 = 1;
            while (c2 < nneed) c2 <<= 1;
            const uint32_t lgc = (uint32_t)__builtin_ctz(c2);
            n_evals += (uint64_t)R * nneed;
            const uint32_t pairs = (uint32_t)R << lgc;
            for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                ++n_sparse;
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
        // ---- fold this round's candidates into the top-k
        if (__any(cnt >= 4)) {
            ++n_merge;
            float bd[R];
            uint32_t bi[R];
#pragma unroll
            for (int s2 = 0; s2 < R; ++s2) {
                const float dv = W.bd[s2][lane];
                const uint32_t iv = W.bi[s2][lane];
                const bool hv = (uint32_t)s2 < cnt;
                bd[s2] = hv ? dv : INFINITY;
                bi[s2] = hv ? iv : 0xFFFFFFFFu;
            }
            bitonic_sort<R>(bd, bi);
#pragma unroll
            for (int s2 = 0; s2 < R; ++s2) {
                const int pos = KC - R + s2, o = R - 1 - s2;
                const bool take = bd[o] < td[pos];
                td[pos] = take ? bd[o] : td[pos];
                ti[pos] = take ? bi[o] : ti[pos];
            }
            bitonic_merge<KC>(td, ti);
        } else {
            for (uint32_t j = 0; __any(cnt > j); ++j) {
                ++n_ins;
                const bool hv = j < cnt;
                const float dv = hv ? W.bd[j][lane] : INFINITY;
                const uint32_t iv = hv ? W.bi[j][lane] : 0xFFFFFFFFu;
                insert_sorted<KC>(td, ti, dv, iv);
            }
        }
        if (valid) kth = td[KC - 1];
        W.qt[lane].w = kth;
    }

    if (valid) {
        const int skip = KC - k;
        const size_t row = (size_t)qo * (size_t)k;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= skip) {
                out_d[row + (j - skip)] = sqrtf(td[j]);
                const uint32_t p = ti[j];
                out_i[row + (j - skip)] = p == 0xFFFFFFFFu ? p : t.idx[p];
            }
        }
    }
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (stats && lane == 0) {
        atomicAdd(&stats[0], (unsigned long long)n_nodes * nvalid);
        atomicAdd(&stats[1], (unsigned long long)n_evals);
        atomicAdd(&stats[2], (unsigned long long)n_dense);
        atomicAdd(&stats[3], (unsigned long long)n_sparse);
        atomicAdd(&stats[4], (unsigned long long)(n_merge + n_ins * 1000000ull));
        atomicAdd(&stats[5], 1ull);
    }
}

template <int KC, int CHUNK, int OCC>
void launch3(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k, float *od,
             uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        knn3_kernel<KC, true, CHUNK, OCC><<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi,
                                                                 stats);
    else
        knn3_kernel<KC, false, CHUNK, OCC><<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi,
                                                                  stats);
}

// ---------------------------------------------------------------- v4
// v2's merge scheme with v3's traversal (near-child descent, far-only push,
// scalar-cache node records).
template <int KC, bool PER, int CAP, int R, int CHUNK, int OCC>
__global__ void __launch_bounds__(TB, OCC)
knn4_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  uint32_t m, int k, float *__restrict__ out_d, uint32_t *__restrict__ out_i,
                  unsigned long long *__restrict__ stats) {
    static_assert(CHUNK % R == 0 && CAP > R && CAP <= KC, "tuning");
    __shared__ WaveLds<CAP, CHUNK> Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds<CAP, CHUNK> &W = Wl[wave];
    const uint32_t gq = (blockIdx.x * WPB + wave) * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;

    float td[KC];
    uint32_t ti[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        td[j] = (j < KC - k) ? -INFINITY : FLT_MAX;
        ti[j] = 0xFFFFFFFFu;
    }
    float kth = valid ? FLT_MAX : -INFINITY;
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
                const float box[6] = {b0, b1, b2, b3, b4, b5};
                const float bdist = box_d2<PER>(qx, qy, qz, box, L);
                const bool want = bdist <= kth;
                const uint64_t wm = __ballot(want);
                if (wm == 0) continue;
                ++n_nodes;
                const nbkd_node nd = cnodes[node];
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
        if (!done) {
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
            if (nneed > 32) {
                ++n_dense;
                n_evals += (uint64_t)R * 64;
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
                n_evals += (uint64_t)R * nneed;
                const uint32_t pairs = (uint32_t)R << lgc;
                for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                    ++n_sparse;
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
        if (merge) {
            ++n_merge;
            if (stats) {
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
            bitonic_sort<CAP>(bd, bi);
#pragma unroll
            for (int s = 0; s < CAP; ++s) {
                const int pos = KC - CAP + s, o = CAP - 1 - s;
                const bool take = bd[o] < td[pos];
                td[pos] = take ? bd[o] : td[pos];
                ti[pos] = take ? bi[o] : ti[pos];
            }
            bitonic_merge<KC>(td, ti);
            if (valid) kth = td[KC - 1];
            cnt = 0;
            W.qt[lane].w = kth;
        }
        if (done) break;
    }

    if (valid) {
        const int skip = KC - k;
        const size_t row = (size_t)qo * (size_t)k;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= skip) {
                out_d[row + (j - skip)] = sqrtf(td[j]);
                const uint32_t p = ti[j];
                out_i[row + (j - skip)] = p == 0xFFFFFFFFu ? p : t.idx[p];
            }
        }
    }
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (stats && lane == 0) {
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

template <int KC, int CAP, int R, int CHUNK, int OCC>
void launch4(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k, float *od,
             uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        knn4_kernel<KC, true, CAP, R, CHUNK, OCC>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
    else
        knn4_kernel<KC, false, CAP, R, CHUNK, OCC>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
}

template <int KC, int CAP, int R, int CHUNK, int OCC>
void launch(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k, float *od,
            uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        knn_packet_kernel<KC, true, CAP, R, CHUNK, OCC>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
    else
        knn_packet_kernel<KC, false, CAP, R, CHUNK, OCC>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
}

int variant() {
    static int v = [] {
        const char *e = getenv("NBKD_KNN_VARIANT");
        return e ? atoi(e) : 0;
    }();
    return v;
}

} // namespace

void launch_knn_packet(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
                       float *od, uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const int v = variant();
    if (k <= 16) {
        launch4<16, 16, 8, 32, 5>(t, q, order, m, k, od, oi, stats, s);
    } else if (k <= 32) {
        switch (v) { // tuning experiments (NBKD_KNN_VARIANT)
        case 1: launch<32, 16, 8, 32, 4>(t, q, order, m, k, od, oi, stats, s); break;   // v2
        case 2: launch3<32, 32, 1>(t, q, order, m, k, od, oi, stats, s); break;         // v3
        case 3: launch4<32, 16, 8, 32, 1>(t, q, order, m, k, od, oi, stats, s); break;
        case 4: launch4<32, 16, 8, 64, 4>(t, q, order, m, k, od, oi, stats, s); break;
        default: launch4<32, 16, 8, 32, 4>(t, q, order, m, k, od, oi, stats, s); break;
        }
    } else {
        launch4<64, 16, 8, 32, 2>(t, q, order, m, k, od, oi, stats, s);
    }
}

} // namespace nbkd
