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
    uint32_t bmax[64];
    uint8_t owners[64];
    float px[CHUNK], py[CHUNK], pz[CHUNK];
};

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

// MODE bit 1: distances-only networks (timing experiment, wrong indices);
// bit 2: between merges prune with the tightened bound max(td[KC-1-cnt], max
// buffered d) instead of the stale td[KC-1]; bit 3: load the node record before
// the box test so its latency overlaps the test
template <int KC, bool PER, int CAP, int R, int CHUNK, int OCC, int MODE>
__global__ void __launch_bounds__(TB, OCC)
knn4_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  uint32_t m, int k, float *__restrict__ out_d, uint32_t *__restrict__ out_i,
                  unsigned long long *__restrict__ stats) {
    static_assert(CHUNK % R == 0 && CAP > R && CAP <= KC, "tuning");
    __shared__ WaveLds<CAP, CHUNK> Wl[WPB];
    constexpr bool TIGHT = (MODE & 4) != 0, HOIST = (MODE & 8) != 0;
    constexpr bool IDX = (MODE & 2) == 0;
    // bit 4 (timing experiment): prune with the final k-th distance read from
    // out_d (a previous run's result), no merges, no output
    constexpr bool FIXEDR = (MODE & 16) != 0;

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
    if constexpr (FIXEDR) {
        if (valid) {
            const float r = out_d[(size_t)qo * k + (k - 1)];
            kth = r * r * 1.000001f;
        }
    }
    uint32_t cnt = 0;
    float bmax = 0.0f; // largest buffered distance (TIGHT)
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
                ++n_nodes;
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
                        if constexpr (TIGHT) bmax = fmaxf(bmax, d);
                    }
                }
            } else {
                W.cnt[lane] = cnt;
                if constexpr (TIGHT) W.bmax[lane] = __float_as_uint(bmax);
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
                            if constexpr (TIGHT) atomicMax(&W.bmax[owner], __float_as_uint(d));
                        }
                    }
                }
                wave_sync();
                cnt = W.cnt[lane];
                if constexpr (TIGHT) bmax = __uint_as_float(W.bmax[lane]);
            }
            leaf_pos += R;
        }
        const bool merge = __any(cnt > (uint32_t)(CAP - R)) || (done && __any(cnt > 0));
        if (FIXEDR && merge) {
            ++n_merge;
            if (stats) {
                uint32_t c = cnt;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                n_cand += c;
            }
            cnt = 0;
        } else if (merge) {
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
            bmax = 0.0f;
            W.qt[lane].w = kth;
        } else if (TIGHT && !done) {
            // the KC-cnt smallest kept entries plus the cnt buffered ones are KC
            // values <= max(td[KC-1-cnt], bmax): an upper bound of the current k-th
            float tk = td[KC - 1];
#pragma unroll
            for (int c = 1; c <= CAP - R; ++c) tk = cnt == (uint32_t)c ? td[KC - 1 - c] : tk;
            if (valid) kth = fmaxf(tk, bmax);
            W.qt[lane].w = kth;
        }
        if (done) break;
    }

    if (valid && !FIXEDR) {
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

template <int KC, int CAP, int R, int CHUNK, int OCC, int MODE = 0>
void launch4(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k, float *od,
             uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        knn4_kernel<KC, true, CAP, R, CHUNK, OCC, MODE>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
    else
        knn4_kernel<KC, false, CAP, R, CHUNK, OCC, MODE>
            <<<blocks, TB, 0, s>>>(view(t), q, order, m, k, od, oi, stats);
}

int variant() {
    const char *e = getenv("NBKD_KNN_VARIANT"); // read per call: tuning sweeps flip it
    return e ? atoi(e) : 0;
}

} // namespace

void launch_knn_packet(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
                       float *od, uint32_t *oi, unsigned long long *stats, hipStream_t s) {
    const int v = variant();
    if (k <= 16) {
        launch4<16, 16, 8, 32, 4, 8>(t, q, order, m, k, od, oi, stats, s);
    } else if (k <= 32) {
        switch (v) { // tuning experiments (NBKD_KNN_VARIANT); see DESIGN.md
        case 1: launch4<32, 16, 8, 32, 4, 0>(t, q, order, m, k, od, oi, stats, s); break;  // no hoist
        case 2: launch4<32, 16, 8, 32, 4, 12>(t, q, order, m, k, od, oi, stats, s); break; // tight bound
        case 3: launch4<32, 16, 8, 32, 4, 10>(t, q, order, m, k, od, oi, stats, s); break; // d-only (timing)
        case 4: launch4<32, 16, 8, 32, 4, 24>(t, q, order, m, k, od, oi, stats, s); break; // fixed r (timing)
        default: launch4<32, 16, 8, 32, 4, 8>(t, q, order, m, k, od, oi, stats, s); break;
        }
    } else {
        launch4<64, 16, 8, 32, 2, 8>(t, q, order, m, k, od, oi, stats, s);
    }
}

} // namespace nbkd
