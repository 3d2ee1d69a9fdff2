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
//            Each query's ball is its seed radius (leaf_key2_kernel), which is
//            expected to hold k + 4 sqrt(k) + 4 points; every point inside it
//            is appended to the query's candidate column in HBM.  No top-k is
//            kept, so the kernel needs few VGPRs and ~2 KB of LDS per wave and
//            runs 8 waves per SIMD.
//   select   one lane per query merges its column 16 candidates at a time into
//            a sorted register top-k (bitonic networks) and writes the rows
//            through LDS as whole-row stores.
//
// A query whose ball holds fewer than k points (seed too small) or more than
// the column capacity is listed for the reference-exact kernel (query.hip).
#include "internal.hpp"
#include "metric.hpp"
#include "packet.hpp"

namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64;
constexpr int CHUNK = 32; // leaf points staged per step (leaves hold <= 32 at leafsize 32)

struct CollectLds {
    float4 qt[64]; // query xyz + seed bound
    uint32_t cnt[64];
    uint8_t owners[64];
    float pb[3][CHUNK];
};

// Candidate columns are slot-major per packet: entry (slot s, lane l) of packet
// pk at cand[(pk * capg + s) * 64 + l] = {d2 bits, tree position}.
template <bool PER, int DENSE_MIN, bool STATS>
__global__ void __launch_bounds__(TB, 8)
knn_collect_kernel(DevTree t, const uint32_t *__restrict__ linfo, const float *__restrict__ q,
                   const uint32_t *__restrict__ order, uint32_t m, const float *__restrict__ tg,
                   uint2 *__restrict__ cand, uint32_t capg, uint32_t *__restrict__ ccount,
                   unsigned long long *__restrict__ stats) {
    __shared__ CollectLds Wl[WPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    CollectLds &W = Wl[wave];
    const uint32_t pk = blockIdx.x * WPB + wave;
    const uint32_t gq = pk * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const float qx = valid ? q[3 * (size_t)qo] : 0.0f;
    const float qy = valid ? q[3 * (size_t)qo + 1] : 0.0f;
    const float qz = valid ? q[3 * (size_t)qo + 2] : 0.0f;
    const float L = t.box;
    const float kth = valid ? tg[qo] : -INFINITY;
    W.qt[lane] = make_float4(qx, qy, qz, kth);
    uint2 *const col = cand + (size_t)pk * capg * 64u;
    uint32_t cnt = 0;

    uint64_t n_nodes = 0, n_leaves = 0, n_scanned = 0, n_dense = 0, n_sparse = 0, n_evals = 0;
    WaveStack stk;
    stk.node = 0;
    stk.b0 = stk.b1 = stk.b2 = stk.b3 = stk.b4 = stk.b5 = 0.0f;
    int sp = 0;
    const cnode_ptr cnodes = (cnode_ptr)t.nodes;
    uint32_t node = 0;
    float b0 = PER ? 0.0f : -FLT_MAX, b1 = PER ? L : FLT_MAX;
    float b2 = b0, b3 = b1, b4 = b0, b5 = b1;
    bool have = true;

    for (;;) {
        // ---------------------------------------------------- next wanted leaf
        bool found = false;
        uint32_t lpos = 0, lend = 0;
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
            const nbkd_node nd = cnodes[node];
            const float box[6] = {b0, b1, b2, b3, b4, b5};
            const bool want = box_d2<PER>(qx, qy, qz, box, L) <= kth;
            const uint64_t wm = __ballot(want);
            if (wm == 0) continue;
            if constexpr (STATS) ++n_nodes;
            const int dim = nd.dimension;
            if (dim < 0) {
                lpos = nd.left;
                lend = nd.right;
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
        if (!found) break;

        // ------------------------------------- scan the leaf, chunk by chunk
        // first chunk's points and the leaf's tight box load together
        uint32_t cn = min((uint32_t)CHUNK, lend - lpos);
        glds_f32(t.x + lpos, W.pb[0], lane, cn);
        glds_f32(t.y + lpos, W.pb[1], lane, cn);
        glds_f32(t.z + lpos, W.pb[2], lane, cn);
        const uint32_t iw = lane < 6 ? linfo[8 * (size_t)node + lane] : 0u;
        wait_vm0();
        wave_sync();
        const float tb[6] = {rdlane(__uint_as_float(iw), 0), rdlane(__uint_as_float(iw), 3),
                             rdlane(__uint_as_float(iw), 1), rdlane(__uint_as_float(iw), 4),
                             rdlane(__uint_as_float(iw), 2), rdlane(__uint_as_float(iw), 5)};
        const uint64_t need = __ballot(box_d2<PER>(qx, qy, qz, tb, L) <= kth);
        if (need == 0) continue;
        const uint32_t nneed = (uint32_t)__popcll(need);
        if constexpr (STATS) ++n_leaves;
        for (uint32_t c0 = lpos;;) {
            if constexpr (STATS) n_scanned += cn;
            if (nneed >= (uint32_t)DENSE_MIN) {
                // every lane scans the chunk for its own query
                if constexpr (STATS) {
                    n_dense += cn;
                    n_evals += (uint64_t)cn * 64;
                }
                for (uint32_t u0 = 0; u0 < cn; u0 += 8) {
                    float px[8], py[8], pz[8];
#pragma unroll
                    for (int u = 0; u < 8; u += 4) {
                        const float4 xv = *reinterpret_cast<const float4 *>(&W.pb[0][u0 + u]);
                        const float4 yv = *reinterpret_cast<const float4 *>(&W.pb[1][u0 + u]);
                        const float4 zv = *reinterpret_cast<const float4 *>(&W.pb[2][u0 + u]);
                        px[u] = xv.x; px[u + 1] = xv.y; px[u + 2] = xv.z; px[u + 3] = xv.w;
                        py[u] = yv.x; py[u + 1] = yv.y; py[u + 2] = yv.z; py[u + 3] = yv.w;
                        pz[u] = zv.x; pz[u + 1] = zv.y; pz[u + 2] = zv.z; pz[u + 3] = zv.w;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const float d = point_d2<PER>(qx, qy, qz, px[u], py[u], pz[u], L);
                        if (d < kth) {
                            if (cnt < capg)
                                col[(size_t)cnt * 64 + lane] = make_uint2(__float_as_uint(d), c0 + u0 + u);
                            ++cnt;
                        }
                    }
                }
            } else {
                // (needing query, point) pairs compacted onto the 64 lanes:
                // slot = pair & (c2-1), point = pair >> log2(c2), c2 = pow2 >= nneed
                W.cnt[lane] = cnt;
                if ((need >> lane) & 1ull) W.owners[mbcnt64(need)] = (uint8_t)lane;
                wave_sync();
                uint32_t c2 = 1;
                while (c2 < nneed) c2 <<= 1;
                const uint32_t lgc = (uint32_t)__builtin_ctz(c2);
                const uint32_t pairs = cn << lgc;
                if constexpr (STATS) n_evals += (uint64_t)cn * nneed;
                for (uint32_t p0 = 0; p0 < pairs; p0 += 64) {
                    if constexpr (STATS) ++n_sparse;
                    const uint32_t pi = p0 + lane;
                    const uint32_t slot = pi & (c2 - 1u), pr = pi >> lgc;
                    if (slot < nneed && pi < pairs) {
                        const uint32_t owner = W.owners[slot];
                        const float4 qq = W.qt[owner];
                        const float d = point_d2<PER>(qq.x, qq.y, qq.z, W.pb[0][pr], W.pb[1][pr],
                                                      W.pb[2][pr], L);
                        if (d < qq.w) {
                            const uint32_t sl = atomicAdd(&W.cnt[owner], 1u);
                            if (sl < capg)
                                col[(size_t)sl * 64 + owner] = make_uint2(__float_as_uint(d), c0 + pr);
                        }
                    }
                }
                wave_sync();
                cnt = W.cnt[lane];
            }
            c0 += cn;
            if (c0 >= lend) break;
            cn = min((uint32_t)CHUNK, lend - c0);
            wave_sync();
            glds_f32(t.x + c0, W.pb[0], lane, cn);
            glds_f32(t.y + c0, W.pb[1], lane, cn);
            glds_f32(t.z + c0, W.pb[2], lane, cn);
            wait_vm0();
            wave_sync();
        }
    }
    if (valid) ccount[gq] = cnt;
    if (STATS && lane == 0) {
        const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
        atomicAdd(&stats[0], (unsigned long long)n_nodes * nvalid);
        atomicAdd(&stats[1], (unsigned long long)n_evals);
        atomicAdd(&stats[2], (unsigned long long)n_dense);
        atomicAdd(&stats[3], (unsigned long long)n_sparse);
        atomicAdd(&stats[4], (unsigned long long)n_scanned);
        atomicAdd(&stats[5], 1ull);
        atomicAdd(&stats[7], (unsigned long long)n_leaves);
    }
    if (STATS) {
        uint32_t c = valid ? cnt : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) atomicAdd(&stats[6], (unsigned long long)c);
    }
}

// One lane per query: the k smallest of its candidate column, sorted, as rows.
template <int KC, bool PER>
__global__ void __launch_bounds__(TB)
knn_select_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ order,
                  uint32_t m, int k, const uint2 *__restrict__ cand, uint32_t capg,
                  const uint32_t *__restrict__ ccount, float *__restrict__ out_d,
                  uint32_t *__restrict__ out_i, uint32_t *__restrict__ fail_list,
                  uint32_t *__restrict__ fail_count) {
    constexpr int NS = 16;                  // candidates merged per pass
    constexpr int CC = KC < 32 ? KC : 32;   // top-k registers staged per output pass
    __shared__ uint32_t stage_all[WPB][CC * 64];
    __shared__ uint32_t rowq_all[WPB][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *stage = stage_all[wave], *rowq = rowq_all[wave];
    const uint32_t pk = blockIdx.x * WPB + wave;
    const uint32_t gq = pk * 64u + lane;
    const bool valid = gq < m;
    const uint32_t qo = valid ? order[gq] : 0u;
    const uint32_t n = valid ? ccount[gq] : 0u;
    const bool ok = valid && n >= (uint32_t)k && n <= capg;
    if (valid && !ok) {
        const float qx = q[3 * (size_t)qo], qy = q[3 * (size_t)qo + 1], qz = q[3 * (size_t)qo + 2];
        // outside-box periodic queries are listed already (outside_box_kernel)
        knn_fail_check<PER>(true, true, 0xFFFFFFFFu, qx, qy, qz, t.box, qo, fail_list, fail_count);
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
    const uint2 *colp = cand + (size_t)pk * capg * 64u + lane;
    for (uint32_t s0 = 0; s0 < maxn; s0 += NS) {
        float bd[NS];
        uint32_t bi[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const uint32_t s = s0 + j;
            uint2 e = make_uint2(0x7F800000u, 0xFFFFFFFFu); // (+inf, none)
            if (s < nn) e = colp[(size_t)s * 64];
            bd[j] = __uint_as_float(e.x);
            bi[j] = e.y;
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
    }

    rowq[lane] = valid ? qo : 0xFFFFFFFFu;
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j) stage[j * 64 + (lane ^ j)] = __float_as_uint(sqrtf(td[j0 + j]));
        wave_sync();
        store_rows<CC>(stage, rowq, reinterpret_cast<uint32_t *>(out_d), k, j0 - (KC - k), lane);
    }
#pragma unroll
    for (int j0 = 0; j0 < KC; j0 += CC) {
        wave_sync();
#pragma unroll
        for (int j = 0; j < CC; ++j) stage[j * 64 + (lane ^ j)] = ti[j0 + j];
        wave_sync();
        store_rows<CC>(stage, rowq, out_i, k, j0 - (KC - k), lane, t.idx);
    }
}

int dense_min() {
    const char *e = getenv("NBKD_DENSE_MIN"); // tuning experiments only
    return e ? atoi(e) : 17;
}

template <bool PER>
void launch_collect(const Tree &t, const float *q, const uint32_t *order, uint32_t m,
                    const float *tg, uint2 *cand, uint32_t capg, uint32_t *ccount,
                    unsigned long long *stats, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    const int dm = dense_min();
#define NBKD_COLLECT(DM)                                                                           \
    do {                                                                                           \
        if (stats)                                                                                 \
            knn_collect_kernel<PER, DM, true><<<blocks, TB, 0, s>>>(                               \
                view(t), t.leafinfo, q, order, m, tg, cand, capg, ccount, stats);                  \
        else                                                                                       \
            knn_collect_kernel<PER, DM, false><<<blocks, TB, 0, s>>>(                              \
                view(t), t.leafinfo, q, order, m, tg, cand, capg, ccount, nullptr);                \
    } while (0)
    if (dm <= 9) NBKD_COLLECT(9);
    else if (dm <= 17) NBKD_COLLECT(17);
    else if (dm <= 25) NBKD_COLLECT(25);
    else NBKD_COLLECT(33);
#undef NBKD_COLLECT
}

template <int KC>
void launch_select(const Tree &t, const float *q, const uint32_t *order, uint32_t m, int k,
                   const uint2 *cand, uint32_t capg, const uint32_t *ccount, float *od,
                   uint32_t *oi, uint32_t *fail_list, uint32_t *fail_count, hipStream_t s) {
    const unsigned blocks = (m + TB - 1) / TB;
    if (t.periodic)
        knn_select_kernel<KC, true><<<blocks, TB, 0, s>>>(view(t), q, order, m, k, cand, capg,
                                                          ccount, od, oi, fail_list, fail_count);
    else
        knn_select_kernel<KC, false><<<blocks, TB, 0, s>>>(view(t), q, order, m, k, cand, capg,
                                                           ccount, od, oi, fail_list, fail_count);
}

} // namespace

uint32_t collect_capacity(int k) {
    // seed balls hold mu = k + 4 sqrt(k) + 4 points on average; the column
    // takes mu + 5 sqrt(mu), rounded up to a multiple of 16
    const double mu = k + 4.0 * std::sqrt((double)k) + 4.0;
    const double c = mu + 5.0 * std::sqrt(mu);
    return (uint32_t)((c + 15.0) / 16.0) * 16u;
}

nbkd_status launch_knn_collect(const Tree &t, const float *q, const uint32_t *order, uint32_t m,
                               int k, const float *tg, uint2 *cand, uint32_t capg,
                               uint32_t *ccount, float *od, uint32_t *oi, uint32_t *fail_list,
                               uint32_t *fail_count, unsigned long long *stats, hipStream_t s) {
    if (m == 0) return NBKD_OK;
    {
        TimedScope ts("knn_collect", s);
        if (t.periodic)
            launch_collect<true>(t, q, order, m, tg, cand, capg, ccount, stats, s);
        else
            launch_collect<false>(t, q, order, m, tg, cand, capg, ccount, stats, s);
        NBKD_HIP(hipGetLastError());
    }
    {
        TimedScope ts("knn_select", s);
        if (k <= 16)
            launch_select<16>(t, q, order, m, k, cand, capg, ccount, od, oi, fail_list, fail_count, s);
        else if (k <= 32)
            launch_select<32>(t, q, order, m, k, cand, capg, ccount, od, oi, fail_list, fail_count, s);
        else
            launch_select<64>(t, q, order, m, k, cand, capg, ccount, od, oi, fail_list, fail_count, s);
        NBKD_HIP(hipGetLastError());
    }
    return NBKD_OK;
}

} // namespace nbkd
