// Batched kNN / radius queries for gfx950.
//
// Reference semantics (what the results must equal):
//   traversal       KDTreeQuery::compute   kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:226-268
//   point metric    L2 / L2Periodic        kdtree/src/cpp/include/kdtree/kdtree.hpp:23-31, 72-84
//   box metric      box_distance           kdtree/src/cpp/include/kdtree/kdtree.hpp:35-45, 89-107
//   insertion       d2 < current k-th      kdtree/src/cpp/kdtree_asm_systemv.asm:148-188
//   finalisation    sort by d2, sqrtf      kdtree/src/cpp/kdtree.cpp:149-156
//
// MI355X mapping ("packet traversal"):
//   1. every query is bucketed by the leaf it falls in (one thread per query
//      descends the tree), and the (leaf, query) pairs are radix-sorted, so
//      consecutive queries are spatially adjacent in the kd order;
//   2. one wave64 owns a PACKET of 64 consecutive queries, one per lane, and
//      walks the tree ONCE for all of them: the stack (node id + 6-float box)
//      lives in the wave's VGPRs, one entry per lane (v_writelane / v_readlane);
//      a node is entered iff any lane's box distance <= its own k-th distance;
//   3. a leaf's points are wave-uniform: their SoA coordinates come through the
//      scalar cache (s_load), and every lane computes its own d2 against them;
//   4. each lane keeps its top-k as a sorted register array (K_CAP = 8..64,
//      with K_CAP-k -inf sentinels so the k-th is always element K_CAP-1) and
//      appends candidates (d2 < k-th) to a per-lane LDS buffer of 16 slots; when
//      any lane's buffer is full the wave merges: bitonic sort of the buffer +
//      bitonic merge into the top-k.  No per-candidate divergence.
//   d2 is evaluated exactly as the reference ((dx^2 + dy^2) + dz^2, periodic
//   per-axis min of the three images; min of squares == square of the min |.|),
//   compiled with -ffp-contract=off, so distances are bit-identical.
#include <algorithm>
#include <cstdlib>

#include "internal.hpp"
#include "metric.hpp"

namespace nbkd {
namespace {
using namespace dev;

constexpr int TB = 256;
constexpr int WPB = TB / 64; // waves per block

// ------------------------------------------------------------------ query bucketing
__global__ void __launch_bounds__(TB)
leaf_key_kernel(DevTree t, const float *__restrict__ q, uint32_t m, uint32_t *__restrict__ keys,
                uint32_t *__restrict__ vals) {
    uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= m) return;
    float p[3] = {q[3 * (size_t)i], q[3 * (size_t)i + 1], q[3 * (size_t)i + 2]};
    uint32_t node = 0;
    nbkd_node nd = t.nodes[0];
    while (nd.dimension >= 0) {
        float v = p[nd.dimension];
        node = v > nd.split ? nd.right : nd.left; // near child, kdtree_impl.hpp:239
        nd = t.nodes[node];
    }
    keys[i] = nd.left >> 3;
    vals[i] = i;
}

// Same descent without touching the 16-B node records: the shape is a pure
// function of (n8, leaf) — left child = id + 1, right child = id + 1 +
// |subtree(m)|, m = (count/2)/8*8, axis = depth % 3 — so only the 4-B split
// values are read (a 33 MB array at 1e8 points, Infinity-Cache resident).
constexpr int SHAPE_MAX = 256;

// Guessed squared search radius of a query from the point density of the
// subtree it falls in (count points in the box lo..hi): the radius of a sphere
// expected to hold `mu_c` * 4/3*pi points, mu = k + a sqrt(k) + a, a = 3 (Poisson
// tail ~8e-4 below k at k = 32; seed_params).  Only a pruning seed: the kNN kernel starts with this
// bound instead of +inf and sends every query that finds fewer than k points
// inside it to the reference-exact kernel, so a bad guess costs time, never
// correctness.
// Degenerate subtrees (points on a plane or a line: a zero extent) use the
// density of their dimension: pi r^2 = mu A / count, 2 r = mu len / count.
__device__ __forceinline__ float guess_r2(uint32_t count, const float lo[3], const float hi[3],
                                          float mu_c) {
    const float e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
    if (count == 0 || !(e0 >= 0.0f) || !(e1 >= 0.0f) || !(e2 >= 0.0f)) return FLT_MAX;
    const int dd = (e0 > 0.0f) + (e1 > 0.0f) + (e2 > 0.0f);
    float r2;
    if (dd == 3) {
        const float r3 = mu_c * ((e0 * e1) * e2) / (float)count;
        r2 = cbrtf(r3 * r3);
    } else if (dd == 2) { // mu_c * 4/3 = mu / pi
        const float a = (e0 > 0.0f ? e0 : 1.0f) * (e1 > 0.0f ? e1 : 1.0f) * (e2 > 0.0f ? e2 : 1.0f);
        r2 = mu_c * (4.0f / 3.0f) * a / (float)count;
    } else if (dd == 1) { // mu_c * 2 pi / 3 = mu / 2
        const float r = mu_c * (2.0f * 3.14159265f / 3.0f) * (e0 + e1 + e2) / (float)count;
        r2 = r * r;
    } else {
        return FLT_MAX; // all points identical: no scale
    }
    return (r2 > 0.0f && r2 < FLT_MAX) ? r2 : FLT_MAX;
}

// Bucketing descent over the blocked heap of splits (internal.hpp hblk_*,
// build.hip heap_splits_kernel): same turns, same leaf key and seed as
// leaf_key2_kernel, one 64-B line (4 levels) per load instead of one dependent
// load per level.  The kernel keeps the texture addresser ~80 % busy with
// these divergent 16-B gathers (profiles/r04w_pmc_sq_tcc.txt), but fewer of
// them cost more in latency than they save: reading a line's last quarter
// only after the first three levels' turns (3 gathers a line) 3.15 -> 3.59 ms,
// block levels 0 and 1 from LDS 3.86 ms, both 3.73 ms at 1e8
// (profiles/r04x_ab_leaf_key.txt).
__global__ void __launch_bounds__(TB)
leaf_key3_kernel(const float4 *__restrict__ hb, int o, uint32_t n8, uint32_t leaf,
                 const float *__restrict__ q, uint32_t m, uint32_t *__restrict__ keys,
                 uint32_t *__restrict__ vals, float *__restrict__ tg, float mu_c, uint32_t anchor,
                 float3 box_lo, float3 box_hi, uint64_t axes, float child_th, float child_s) {
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < m; i += gridDim.x * TB) {
        const float p[3] = {q[3 * (size_t)i], q[3 * (size_t)i + 1], q[3 * (size_t)i + 2]};
        uint32_t left = 0, count = n8;
        int depth = 0;
        float lo[3] = {box_lo.x, box_lo.y, box_lo.z}, hi[3] = {box_hi.x, box_hi.y, box_hi.z};
        float r2 = FLT_MAX;
        bool have_r2 = tg == nullptr;
        bool half = false; // the anchor's half the query falls in is next (anchor_chunk_kernel's rule)
        // line b of block level j (level start `base`, `nb` lines); first level l0
        uint32_t b = 0, base = 0, nb = 1;
        int l0 = o;
        while (count > leaf) {
            const float4 a0 = hb[4 * (size_t)b], a1 = hb[4 * (size_t)b + 1];
            const float4 a2 = hb[4 * (size_t)b + 2], a3 = hb[4 * (size_t)b + 3];
            uint32_t pos = 0; // position within the line's current level
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                if (l < l0) continue;
                if (count <= leaf) break;
                if (!have_r2 && count <= anchor) {
                    r2 = guess_r2(count, lo, hi, mu_c);
                    have_r2 = true;
                    half = child_th > 0.0f && count >= 64u && r2 < FLT_MAX;
                }
                float s;
                if (l == 0)
                    s = a0.x;
                else if (l == 1)
                    s = pos ? a0.z : a0.y;
                else if (l == 2)
                    s = (pos & 2) ? ((pos & 1) ? a1.z : a1.y) : ((pos & 1) ? a1.x : a0.w);
                else
                    s = (pos & 4) ? ((pos & 2) ? ((pos & 1) ? a3.z : a3.y)
                                               : ((pos & 1) ? a3.x : a2.w))
                                  : ((pos & 2) ? ((pos & 1) ? a2.z : a2.y)
                                               : ((pos & 1) ? a2.x : a1.w));
                const uint32_t mm = (count / 2) / 8 * 8;
                const int dim = axis_at(axes, depth++);
                const bool right = p[dim] > s; // near child, kdtree_impl.hpp:239
                if (right) {
                    lo[dim] = s;
                    left += mm;
                    count -= mm;
                } else {
                    hi[dim] = s;
                    count = mm;
                }
                pos = 2 * pos + (right ? 1u : 0u);
                if (half) {
                    const float rc = guess_r2(count, lo, hi, mu_c);
                    if (rc < FLT_MAX && rc > child_th * r2) r2 = fmaxf(r2, child_s * rc);
                    half = false;
                }
            }
            if (count <= leaf) break;
            // pos = child index 0..15 of the next line
            const uint32_t nbase = base + nb;
            b = nbase + (b - base) * 16u + pos;
            nb = base == 0 ? (16u >> o) : nb * 16u;
            base = nbase;
            l0 = 0;
        }
        if (!have_r2) r2 = guess_r2(count, lo, hi, mu_c);
        keys[i] = left >> 3;
        vals[i] = i;
        if (tg) tg[i] = r2;
    }
}

// Self queries (self_order below): the seed of the point at tree position p
// comes from its anchor, the first subtree of <= anchor points that holds
// position p -- the subtree leaf_key3_kernel's descent by the point's
// coordinates reaches (a point tied with a split value may sit on the split's
// other side; its seed is then only a different guess).  An anchor holds >= 64
// points (its parent held more than anchor >= 128, and a split's smaller
// child gets floor(count / 16) * 8), so the 64 positions of chunk c
// (64c .. 64c + 63) meet at most two anchors: the one holding 64c and the one
// holding 64(c + 1).  anchor_chunk_kernel finds, per chunk, the anchor holding
// its first position -- its first position and seed -- and self_seed_kernel
// gives position p the seed of chunk p / 64's anchor, or of the next chunk's
// if p lies at or past that anchor's start.
//
// The descent turns by the counts alone (right iff p >= left + m), so it
// loads nothing on the way: it records where in the blocked heap (internal.hpp
// hblk_*) the last split bounding each axis from below and from above sits,
// and the six split values load together at the end.
struct SeedPath {
    uint32_t left, count, b, base, nb, lp;
    int l, depth;
    // heap index + 1 of the last split bounding axis d from below / above
    // (0: none, the box face); named, not an indexed private array
    uint32_t lo0, lo1, lo2, hi0, hi1, hi2;
};

__device__ __forceinline__ void seed_turn(SeedPath &w, bool right, int o, uint64_t axes) {
    const uint32_t mm = (w.count / 2) / 8 * 8;
    const uint32_t at = 16u * w.b + (1u << w.l) + w.lp; // heap index + 1
    const int dim = axis_at(axes, w.depth++);
    if (right) {
        w.lo0 = dim == 0 ? at : w.lo0;
        w.lo1 = dim == 1 ? at : w.lo1;
        w.lo2 = dim == 2 ? at : w.lo2;
        w.left += mm;
        w.count -= mm;
    } else {
        w.hi0 = dim == 0 ? at : w.hi0;
        w.hi1 = dim == 1 ? at : w.hi1;
        w.hi2 = dim == 2 ? at : w.hi2;
        w.count = mm;
    }
    w.lp = 2 * w.lp + (right ? 1u : 0u);
    if (++w.l == 4) { // next line: child lp of this one
        const uint32_t nbase = w.base + w.nb;
        w.b = nbase + (w.b - w.base) * 16u + w.lp;
        w.nb = w.base == 0 ? (16u >> o) : w.nb * 16u;
        w.base = nbase;
        w.l = 0;
        w.lp = 0;
    }
}

// anch[c] = (first position, boundary, seed bits below it, seed bits at or
// past it) of the anchor holding position 64c.  The boundary splits the
// anchor into its two halves (its children; child_th != 0 and the anchor not
// a leaf): a half sparser than the anchor as a whole -- its seed above
// child_th times the anchor's -- gives its positions max(anchor seed,
// child_s x its own).  On log-normal 1e8 (k = 32) 6.3 % of the self queries
// found fewer than k points in the anchor's seed ball; with child_th = 1.1
// the re-walks drop 7.07 M -> 4.32 M and the step 62.98 -> 61.39 ms, while
// uniform data (whose halves' volumes differ by ~12 %) moves by noise
// (82 k -> 64 k re-walks, 52.49 -> 52.32 ms).  1.0 re-walks 4.03 M
// log-normal but costs uniform +0.4 ms; each half its own seed (-1) 6.09 M,
// and at x1.1 3.89 M but +0.9 ms uniform (profiles/r06l_retry_ab.txt).
// (tried and dropped: the anchor's tight span from its 8-point group boxes
// where the cell reaches through empty space -- the same seed failures on
// slab trees and log-normal data, +0.13 ms per 1e8; profiles/r05s_ab.txt)
__global__ void __launch_bounds__(TB)
anchor_chunk_kernel(const float *__restrict__ hf, int o, uint32_t n8, uint32_t stop,
                    uint32_t nchunks, uint4 *__restrict__ anch, float mu_c, float3 box_lo,
                    float3 box_hi, uint64_t axes, uint32_t leaf, float child_th, float child_s) {
    const uint32_t c = blockIdx.x * TB + threadIdx.x;
    if (c >= nchunks) return;
    const uint32_t p = c * 64u;
    SeedPath w{0u, n8, 0u, 0u, 1u, 0u, o, 0, 0u, 0u, 0u, 0u, 0u, 0u};
    while (w.count > stop) seed_turn(w, p >= w.left + (w.count / 2) / 8 * 8, o, axes);
    float lo[3] = {w.lo0 ? hf[w.lo0 - 1] : box_lo.x, w.lo1 ? hf[w.lo1 - 1] : box_lo.y,
                   w.lo2 ? hf[w.lo2 - 1] : box_lo.z};
    float hi[3] = {w.hi0 ? hf[w.hi0 - 1] : box_hi.x, w.hi1 ? hf[w.hi1 - 1] : box_hi.y,
                   w.hi2 ? hf[w.hi2 - 1] : box_hi.z};
    const float ra = guess_r2(w.count, lo, hi, mu_c);
    uint32_t bnd = w.left + w.count;
    float r0 = ra, r1 = ra;
    if (child_th != 0.0f && w.count > leaf && w.count >= 64u && ra < FLT_MAX) {
        // the anchor's own split: heap index + 1 as seed_turn computes it
        const uint32_t at = 16u * w.b + (1u << w.l) + w.lp;
        const float sv = hf[at - 1];
        const int dim = axis_at(axes, w.depth);
        const uint32_t mm = (w.count / 2) / 8 * 8;
        bnd = w.left + mm;
        const float keep_hi = hi[dim], keep_lo = lo[dim];
        hi[dim] = sv;
        const float rl = guess_r2(mm, lo, hi, mu_c);
        hi[dim] = keep_hi;
        lo[dim] = sv;
        const float rr = guess_r2(w.count - mm, lo, hi, mu_c);
        lo[dim] = keep_lo;
        if (child_th < 0.0f) { // experiments: each half its own seed
            r0 = rl < FLT_MAX ? rl * child_s : ra;
            r1 = rr < FLT_MAX ? rr * child_s : ra;
        } else {
            if (rl < FLT_MAX && rl > child_th * ra) r0 = fmaxf(ra, rl * child_s);
            if (rr < FLT_MAX && rr > child_th * ra) r1 = fmaxf(ra, rr * child_s);
        }
    }
    anch[c] = make_uint4(w.left, bnd, __float_as_uint(r0), __float_as_uint(r1));
}

// tgp[i] = the seed of position pos[i] (pos nullptr: i); with pos, also
// order[i] = perm[pos[i]]; tgp nullptr: the order alone
__global__ void __launch_bounds__(TB)
self_seed_kernel(const uint4 *__restrict__ anch, uint32_t nchunks,
                 const uint32_t *__restrict__ pos, const uint32_t *__restrict__ perm, uint32_t m,
                 uint32_t *__restrict__ order, float *__restrict__ tgp) {
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < m; i += gridDim.x * TB) {
        const uint32_t p = pos ? pos[i] : i;
        if (pos) order[i] = perm[p];
        if (!tgp) continue;
        const uint32_t c = p >> 6;
        uint4 a = anch[c];
        if (c + 1 < nchunks) {
            const uint4 b = anch[c + 1];
            if (p >= b.x) a = b;
        }
        tgp[i] = __uint_as_float(p < a.y ? a.z : a.w);
    }
}

// the same for the identity order (pos nullptr): four positions per thread,
// one 16-B store, one pass over the grid (the grid-stride form above spent
// 0.24 ms per 1e8 positions, latency-bound)
__global__ void __launch_bounds__(TB)
self_seed4_kernel(const uint4 *__restrict__ anch, uint32_t nchunks, uint32_t m,
                  float *__restrict__ tgp) {
    const uint32_t p0 = (blockIdx.x * TB + threadIdx.x) * 4u;
    if (p0 >= m) return;
    const uint32_t c = p0 >> 6; // the four positions share a chunk (64 = 16 x 4)
    const uint4 a = anch[c];
    const uint4 b = c + 1 < nchunks ? anch[c + 1] : a;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t p = p0 + j;
        const uint4 e = p >= b.x ? b : a;
        v[j] = __uint_as_float(p < e.y ? e.z : e.w);
    }
    if (p0 + 4 <= m) { // tgp is a 256-B aligned workspace buffer
        *reinterpret_cast<float4 *>(tgp + p0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        for (int j = 0; j < 4; ++j)
            if (p0 + j < m) tgp[p0 + j] = v[j];
    }
}

// bits[p / 32] bit p % 32 = perm[p] < m: the tree positions of the first m
// input rows (self queries over a prefix of the build input, e.g. a slab's
// owned particles ahead of its halo)
__global__ void __launch_bounds__(TB)
self_bits_kernel(const uint32_t *__restrict__ perm, uint64_t n8, uint32_t m,
                 uint32_t *__restrict__ bits) {
    const uint64_t p = (uint64_t)blockIdx.x * TB + threadIdx.x;
    const bool in = p < n8 && perm[p] < m;
    const uint64_t bal = __ballot(in);
    const int lane = threadIdx.x & 63;
    const uint64_t w = p / 32;
    if ((lane & 31) == 0 && p < n8) bits[w] = (uint32_t)(lane ? bal >> 32 : bal);
}

__global__ void __launch_bounds__(TB)
leaf_key2_kernel(const float *__restrict__ splits, const uint32_t *__restrict__ shape_c,
                 const uint32_t *__restrict__ shape_n, int shape_len, uint32_t n8, uint32_t leaf,
                 const float *__restrict__ q, uint32_t m, uint32_t *__restrict__ keys,
                 uint32_t *__restrict__ vals, float *__restrict__ tg, float mu_c, uint32_t anchor,
                 float3 box_lo, float3 box_hi, uint64_t axes) {
    __shared__ uint32_t sc[SHAPE_MAX], sn[SHAPE_MAX];
    for (int i = threadIdx.x; i < shape_len; i += TB) {
        sc[i] = shape_c[i];
        sn[i] = shape_n[i];
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < m; i += gridDim.x * TB) {
        const float p[3] = {q[3 * (size_t)i], q[3 * (size_t)i + 1], q[3 * (size_t)i + 2]};
        uint32_t node = 0, left = 0, count = n8;
        int depth = 0;
        float lo[3] = {box_lo.x, box_lo.y, box_lo.z}, hi[3] = {box_hi.x, box_hi.y, box_hi.z};
        float r2 = FLT_MAX;
        bool have_r2 = tg == nullptr;
        while (count > leaf) {
            if (!have_r2 && count <= anchor) {
                r2 = guess_r2(count, lo, hi, mu_c);
                have_r2 = true;
            }
            const uint32_t mm = (count / 2) / 8 * 8;
            const float s = splits[node];
            const int dim = axis_at(axes, depth++);
            if (p[dim] > s) { // near child, kdtree_impl.hpp:239
                lo[dim] = s;
                uint32_t sub = 1;
                if (mm > leaf) {
                    int bl = 0, bh = shape_len - 1;
                    while (bl < bh) {
                        const int mid = (bl + bh) >> 1;
                        if (sc[mid] < mm)
                            bl = mid + 1;
                        else
                            bh = mid;
                    }
                    sub = sn[bl];
                }
                node += 1 + sub;
                left += mm;
                count -= mm;
            } else {
                hi[dim] = s;
                node += 1;
                count = mm;
            }
        }
        if (!have_r2) r2 = guess_r2(count, lo, hi, mu_c);
        keys[i] = left >> 3;
        vals[i] = i;
        if (tg) tg[i] = r2;
    }
}

// ------------------------------------------------------------------ LSD radix sort (keys + values)
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = TB * RS_ITEMS; // 2048

__global__ void __launch_bounds__(TB)
rs_hist_kernel(const uint32_t *__restrict__ keys, uint32_t n, int shift, uint32_t ntiles,
               uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * RS_TILE;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        uint32_t e = base + r * TB + threadIdx.x;
        if (e < n) atomicAdd(&h[(keys[e] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ void __launch_bounds__(TB)
rs_scatter_kernel(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin, uint32_t n,
                  int shift, uint32_t ntiles, const uint32_t *__restrict__ hist_scanned,
                  uint32_t *__restrict__ kout, uint32_t *__restrict__ vout) {
    __shared__ uint16_t cnt[RS_ITEMS][WPB][256];
    __shared__ uint32_t gofs[256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int j = threadIdx.x; j < RS_ITEMS * WPB * 256; j += TB) (&cnt[0][0][0])[j] = 0;
    gofs[threadIdx.x] = hist_scanned[(size_t)threadIdx.x * ntiles + blockIdx.x];
    __syncthreads();
    const uint32_t base = blockIdx.x * RS_TILE;
    uint32_t kk[RS_ITEMS], vv[RS_ITEMS], rk[RS_ITEMS];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        uint32_t e = base + r * TB + threadIdx.x;
        bool valid = e < n;
        kk[r] = valid ? kin[e] : 0u;
        vv[r] = valid ? vin[e] : 0u;
        uint32_t d = (kk[r] >> shift) & 255u;
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t bb = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? bb : ~bb;
        }
        uint32_t below = mbcnt64(same);
        rk[r] = below;
        if (valid && below == 0) cnt[r][wave][d] = (uint16_t)__popcll(same);
    }
    __syncthreads();
    { // per digit: exclusive prefix over (round, wave) in element order
        uint32_t acc = 0;
        const int d = threadIdx.x;
        for (int r = 0; r < RS_ITEMS; ++r)
            for (int w = 0; w < WPB; ++w) {
                uint32_t v = cnt[r][w][d];
                cnt[r][w][d] = (uint16_t)acc;
                acc += v;
            }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        uint32_t e = base + r * TB + threadIdx.x;
        if (e < n) {
            uint32_t d = (kk[r] >> shift) & 255u;
            uint32_t dst = gofs[d] + cnt[r][wave][d] + rk[r];
            kout[dst] = kk[r];
            vout[dst] = vv[r];
        }
    }
    (void)lane;
}

// exclusive scan of a uint32 array, 3 kernels
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = TB * SC_ITEMS;

__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t *sh, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = blockDim.x / 64;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        uint32_t s = sh[w];
        if (w < wave) base += s;
        tot += s;
    }
    if (total) *total = tot;
    __syncthreads();
    return base + x - v;
}

__global__ void __launch_bounds__(TB)
scan_up_kernel(const uint32_t *__restrict__ a, uint64_t n, uint32_t *__restrict__ sums) {
    __shared__ uint32_t sh[WPB];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j)
        if (base + j < n) s += a[base + j];
    uint32_t tot;
    block_scan_excl(s, sh, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) scan_mid_kernel(uint32_t *__restrict__ sums, uint32_t nb) {
    __shared__ uint32_t sh[16];
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += sums[b];
    uint32_t ex = block_scan_excl(s, sh, nullptr);
    for (uint32_t b = b0; b < b1; ++b) {
        uint32_t v = sums[b];
        sums[b] = ex;
        ex += v;
    }
}

__global__ void __launch_bounds__(TB)
scan_down_kernel(uint32_t *__restrict__ a, uint64_t n, const uint32_t *__restrict__ sums) {
    __shared__ uint32_t sh[WPB];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
    uint32_t v[SC_ITEMS], s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        v[j] = base + j < n ? a[base + j] : 0u;
        s += v[j];
    }
    uint32_t ex = block_scan_excl(s, sh, nullptr) + sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        if (base + j < n) a[base + j] = ex;
        ex += v[j];
    }
}

nbkd_status device_excl_scan(Workspace &ws, uint32_t *a, uint64_t n, hipStream_t s) {
    if (n == 0) return NBKD_OK;
    uint64_t nb = (n + SC_TILE - 1) / SC_TILE;
    uint32_t *sums = (uint32_t *)ws.get(WS_SUMS, nb * 4, s);
    if (!sums) return NBKD_ENOMEM;
    scan_up_kernel<<<(unsigned)nb, TB, 0, s>>>(a, n, sums);
    scan_mid_kernel<<<1, 1024, 0, s>>>(sums, (uint32_t)nb);
    scan_down_kernel<<<(unsigned)nb, TB, 0, s>>>(a, n, sums);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

// ------------------------------------------------------------------ one-sweep LSD radix sort
// One histogram read of the keys for all passes, then per 8-bit pass ONE kernel:
// each 4096-item tile ranks its items (stable), publishes its digit counts,
// finds its global digit offsets by decoupled look-back over the tiles before
// it (tiles are numbered in start order by an atomic ticket, so every tile it
// waits on is running), stages the tile digit-sorted in LDS and writes it out
// in digit runs.  Per pass: 8 B read + 8 B written per item.
constexpr int OS_ITEMS = 16;
constexpr int OS_TILE = TB * OS_ITEMS; // 4096
constexpr uint32_t OS_AGG = 1u << 30, OS_PRE = 2u << 30, OS_VAL = OS_AGG - 1;
constexpr int OS_MAXP = 4;

__global__ void __launch_bounds__(TB)
os_hist_kernel(const uint32_t *__restrict__ keys, uint32_t n, int passes,
               uint32_t *__restrict__ ghist) {
    __shared__ uint32_t h[OS_MAXP][256];
    for (int j = threadIdx.x; j < OS_MAXP * 256; j += TB) (&h[0][0])[j] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < n; i += gridDim.x * TB) {
        const uint32_t k = keys[i];
        for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int p = 0; p < passes; ++p) {
        const uint32_t v = h[p][threadIdx.x];
        if (v) atomicAdd(&ghist[p * 256 + threadIdx.x], v);
    }
}

// exclusive scan of each pass's 256 counts, in place (one block)
__global__ void __launch_bounds__(TB) os_scan_kernel(uint32_t *__restrict__ ghist, int passes) {
    __shared__ uint32_t sh[WPB];
    for (int p = 0; p < passes; ++p) {
        const uint32_t v = ghist[p * 256 + threadIdx.x];
        ghist[p * 256 + threadIdx.x] = block_scan_excl(v, sh, nullptr);
    }
}

__global__ void __launch_bounds__(TB)
os_pass_kernel(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin, uint32_t n,
               int shift, const uint32_t *__restrict__ gexcl, uint32_t *__restrict__ status,
               uint32_t *__restrict__ ticket, uint32_t *__restrict__ kout,
               uint32_t *__restrict__ vout) {
    __shared__ uint32_t wh[WPB][256]; // per wave digit counts, then wave-exclusive offsets
    __shared__ uint32_t ls[256];      // tile-local digit start
    __shared__ uint32_t gofs[256];    // global position of local index 0 of digit d
    __shared__ uint32_t sk[OS_TILE], sv[OS_TILE];
    __shared__ uint32_t sh[WPB];
    __shared__ uint32_t tile_sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) tile_sh = atomicAdd(ticket, 1u);
    for (int j = tid; j < WPB * 256; j += TB) (&wh[0][0])[j] = 0;
    __syncthreads();
    const uint32_t tile = tile_sh;
    const uint32_t t0 = tile * (uint32_t)OS_TILE;
    const uint32_t base = t0 + (uint32_t)wave * (OS_ITEMS * 64);
    uint32_t kk[OS_ITEMS], vv[OS_ITEMS], rk[OS_ITEMS];
#pragma unroll
    for (int r = 0; r < OS_ITEMS; ++r) {
        const uint32_t e = base + r * 64 + lane;
        kk[r] = e < n ? kin[e] : 0xFFFFFFFFu;
        vv[r] = e < n ? vin[e] : 0u;
    }
    // stable rank: items of wave w in element order, round by round
#pragma unroll
    for (int r = 0; r < OS_ITEMS; ++r) {
        const uint32_t e = base + r * 64 + lane;
        const uint32_t d = (kk[r] >> shift) & 255u;
        uint64_t same = __ballot(e < n);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t below = mbcnt64(same);
        const uint32_t old = wh[wave][d];
        rk[r] = old + below;
        if (e < n && below == 0) wh[wave][d] = old + (uint32_t)__popcll(same);
    }
    __syncthreads();
    {
        const int d = tid;
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < WPB; ++w) {
            const uint32_t x = wh[w][d];
            wh[w][d] = c;
            c += x;
        }
        uint32_t *st = status + (size_t)tile * 256 + d;
        __hip_atomic_store(st, (tile == 0 ? OS_PRE : OS_AGG) | c, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lsd = block_scan_excl(c, sh, nullptr);
        ls[d] = lsd;
        uint32_t acc = 0;
        if (tile > 0) {
            uint32_t tt = tile - 1;
            for (;;) {
                const uint32_t v = __hip_atomic_load(status + (size_t)tt * 256 + d, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if ((v >> 30) == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                acc += v & OS_VAL;
                if (v & OS_PRE) break;
                --tt;
            }
            __hip_atomic_store(st, OS_PRE | (acc + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        gofs[d] = gexcl[d] + acc - lsd;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < OS_ITEMS; ++r) {
        const uint32_t e = base + r * 64 + lane;
        if (e < n) {
            const uint32_t d = (kk[r] >> shift) & 255u;
            const uint32_t pos = ls[d] + wh[wave][d] + rk[r];
            sk[pos] = kk[r];
            sv[pos] = vv[r];
        }
    }
    __syncthreads();
    const uint32_t cnt = min((uint32_t)OS_TILE, n - t0);
#pragma unroll
    for (int r = 0; r < OS_ITEMS; ++r) {
        const uint32_t i = r * TB + tid;
        if (i < cnt) {
            const uint32_t k = sk[i];
            const uint32_t dst = gofs[(k >> shift) & 255u] + i;
            kout[dst] = k;
            vout[dst] = sv[i];
        }
    }
}

nbkd_status onesweep_sort(Workspace &ws, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1,
                          uint32_t n, int passes, hipStream_t s) {
    const uint32_t ntiles = (n + OS_TILE - 1) / OS_TILE;
    // [passes][256] histogram | [passes] tickets (padded to 64 words) | [passes][ntiles][256] status
    const size_t words = (size_t)passes * 256 + 64 + (size_t)passes * ntiles * 256;
    uint32_t *w = (uint32_t *)ws.get(WS_HIST, words * 4, s);
    if (!w) return NBKD_ENOMEM;
    NBKD_HIP(hipMemsetAsync(w, 0, words * 4, s));
    uint32_t *ghist = w, *tickets = w + passes * 256, *status = tickets + 64;
    const unsigned hb = (unsigned)std::min<uint32_t>((n + TB - 1) / TB, 2048);
    os_hist_kernel<<<hb, TB, 0, s>>>(k0, n, passes, ghist);
    os_scan_kernel<<<1, TB, 0, s>>>(ghist, passes);
    for (int p = 0; p < passes; ++p) {
        uint32_t *ki = (p & 1) ? k1 : k0, *vi = (p & 1) ? v1 : v0;
        uint32_t *ko = (p & 1) ? k0 : k1, *vo = (p & 1) ? v0 : v1;
        os_pass_kernel<<<ntiles, TB, 0, s>>>(ki, vi, n, 8 * p, ghist + p * 256, status +
                                             (size_t)p * ntiles * 256, tickets + p, ko, vo);
    }
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

// sorts (keys, vals) by the low `nbits` of keys, ceil(nbits/8) LSD passes
// ping-ponging between (k0, v0) and (k1, v1); *vout = the sorted values
nbkd_status radix_sort(Workspace &ws, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1,
                       uint32_t n, int nbits, hipStream_t s, uint32_t **vout) {
    *vout = v0;
    if (n <= 1) return NBKD_OK;
    {
        static const bool old_sort = knob("NBKD_OLD_SORT") != nullptr; // A/B only
        const int passes = (nbits + 7) / 8;
        if (!old_sort && n < OS_VAL && passes <= OS_MAXP) {
            *vout = (passes & 1) ? v1 : v0;
            return onesweep_sort(ws, k0, v0, k1, v1, n, passes, s);
        }
    }
    const uint32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    uint32_t *hist = (uint32_t *)ws.get(WS_HIST, (size_t)256 * ntiles * 4, s);
    if (!hist) return NBKD_ENOMEM;
    const int passes = (nbits + 7) / 8;
    *vout = (passes & 1) ? v1 : v0;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        uint32_t *ki = (p & 1) ? k1 : k0, *vi = (p & 1) ? v1 : v0;
        uint32_t *ko = (p & 1) ? k0 : k1, *vo = (p & 1) ? v0 : v1;
        rs_hist_kernel<<<ntiles, TB, 0, s>>>(ki, n, shift, ntiles, hist);
        nbkd_status st = device_excl_scan(ws, hist, (uint64_t)256 * ntiles, s);
        if (st) return st;
        rs_scatter_kernel<<<ntiles, TB, 0, s>>>(ki, vi, n, shift, ntiles, hist, ko, vo);
        NBKD_HIP(hipGetLastError());
    }
    return NBKD_OK;
}

// ------------------------------------------------------------------ reference-exact traversal
// One lane per query, replaying KDTreeQuery::compute (kdtree_impl.hpp:226-268)
// step for step: near child first (left unless q[dim] > split), near visited iff
// box_d2 < k-th, far skipped iff k-th < box_d2 (checked after the near subtree),
// leaf points inserted iff d2 < k-th into the reference's loser tree
// (tournament_tree.hpp:18-105), then sorted by d2 and sqrt'd.  Used where the
// packet traversal's result could differ from the reference's:
//   * periodic queries outside [0, L]^3: the reference does not validate
//     queries (pybind.cpp:90-98) and its periodic box distance is then not a
//     lower bound, so its pruning can drop true neighbours; this replays it;
//   * k > 64 (beyond the register top-k of the packet kernel).
struct LtEntry {
    float d;
    uint32_t id;
    uint32_t slot;
    uint32_t win; // scratch for the initial winners
};

__device__ __forceinline__ void lt_init(LtEntry *lt, uint32_t n) {
    for (uint32_t i = 0; i < 2 * n; ++i) {
        lt[i].d = FLT_MAX;
        lt[i].id = 0xFFFFFFFFu;
    }
    for (uint32_t i = 0; i < n; ++i) lt[i + n].win = i;
    for (uint32_t i = n - 1; i > 0; --i) {
        uint32_t a = lt[2 * i].win, b = lt[2 * i + 1].win;
        lt[i].win = a > b ? a : b;
        lt[i].slot = (a < b ? a : b) + n;
    }
    for (uint32_t i = n; i < 2 * n; ++i) lt[i].slot = i;
    lt[0].slot = 2 * n - 1;
}

__device__ __forceinline__ void lt_replace_top(LtEntry *lt, float d, uint32_t id) {
    const uint32_t s = lt[0].slot;
    float wd = d;
    uint32_t wid = id, wslot = s;
    lt[s].d = d;
    lt[s].id = id;
    lt[s].slot = s;
    uint32_t i = s;
    while (i > 1) {
        i >>= 1;
        const float od = lt[i].d;
        if (wd < od) {
            const uint32_t oid = lt[i].id, oslot = lt[i].slot;
            lt[i].d = wd;
            lt[i].id = wid;
            lt[i].slot = wslot;
            wd = od;
            wid = oid;
            wslot = oslot;
        }
    }
    lt[0].d = wd;
    lt[0].id = wid;
    lt[0].slot = wslot;
}

template <bool PER>
__global__ void __launch_bounds__(TB)
knn_exact_kernel(DevTree t, const float *__restrict__ q, const uint32_t *__restrict__ list,
                 const uint32_t *__restrict__ list_count, uint32_t m_all, int k,
                 LtEntry *__restrict__ scratch, float *__restrict__ out_d,
                 uint32_t *__restrict__ out_i, bool sq) {
    const uint32_t tid = blockIdx.x * TB + threadIdx.x;
    const uint32_t nthreads = gridDim.x * TB;
    const uint32_t count = list_count ? *list_count : m_all;
    const float L = t.box;
    LtEntry *lt = scratch + (size_t)tid * 2 * (size_t)k;
    for (uint32_t w = tid; w < count; w += nthreads) {
        const uint32_t qi = list ? list[w] : w;
        const float qv[3] = {q[3 * (size_t)qi], q[3 * (size_t)qi + 1], q[3 * (size_t)qi + 2]};
        lt_init(lt, (uint32_t)k);
        uint32_t stk_node[64];
        float stk_box[64][6];
        int sp = 0;
        float box[6];
        for (int a = 0; a < 3; ++a) {
            box[2 * a] = PER ? 0.0f : -FLT_MAX;
            box[2 * a + 1] = PER ? L : FLT_MAX;
        }
        uint32_t node = 0;
        for (;;) {
            const nbkd_node nd = t.nodes[node];
            bool descend = false;
            if (nd.dimension < 0) {
                float top = lt[0].d;
                for (uint32_t j = nd.left; j < nd.right; ++j) {
                    const float d = point_d2<PER>(qv[0], qv[1], qv[2], t.x[j], t.y[j], t.z[j], L);
                    if (d < top) {
                        lt_replace_top(lt, d, j);
                        top = lt[0].d;
                    }
                }
            } else {
                const int dim = nd.dimension;
                const bool right_near = qv[dim] > nd.split;
                float nb[6], fb[6];
                for (int a = 0; a < 6; ++a) {
                    nb[a] = box[a];
                    fb[a] = box[a];
                }
                nb[right_near ? 2 * dim : 2 * dim + 1] = nd.split;
                fb[right_near ? 2 * dim + 1 : 2 * dim] = nd.split;
                stk_node[sp] = right_near ? nd.left : nd.right;
                for (int a = 0; a < 6; ++a) stk_box[sp][a] = fb[a];
                ++sp;
                if (box_d2<PER>(qv[0], qv[1], qv[2], nb, L) < lt[0].d) {
                    node = right_near ? nd.right : nd.left;
                    for (int a = 0; a < 6; ++a) box[a] = nb[a];
                    descend = true;
                }
            }
            if (descend) continue;
            // pop deferred far children: skip iff kth < box_d2
            bool found = false;
            while (sp > 0) {
                --sp;
                const float bd = box_d2<PER>(qv[0], qv[1], qv[2], stk_box[sp], L);
                if (lt[0].d < bd) continue;
                node = stk_node[sp];
                for (int a = 0; a < 6; ++a) box[a] = stk_box[sp][a];
                found = true;
                break;
            }
            if (!found) break;
        }
        // copy_values + sort by d2 (stable) + sqrt, kdtree.cpp:149-156
        LtEntry *res = lt + k;
        for (int i = 1; i < k; ++i) {
            const LtEntry v = res[i];
            int j = i;
            while (j > 0 && v.d < res[j - 1].d) {
                res[j] = res[j - 1];
                --j;
            }
            res[j] = v;
        }
        if (!out_i) { // k-th distance only
            out_d[qi] = sq ? res[k - 1].d : sqrtf(res[k - 1].d);
            continue;
        }
        const size_t row = (size_t)qi * (size_t)k;
        for (int j = 0; j < k; ++j) {
            out_d[row + j] = sq ? res[j].d : sqrtf(res[j].d);
            const uint32_t p = res[j].id;
            out_i[row + j] = p == 0xFFFFFFFFu ? p : t.idx[p];
        }
    }
}

// periodic queries outside [0, L]^3 -> list (order irrelevant: rows are independent)
__global__ void __launch_bounds__(TB)
outside_box_kernel(const float *__restrict__ q, uint32_t m, float L, uint32_t *__restrict__ list,
                   uint32_t *__restrict__ count) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= m) return;
    const float x = q[3 * (size_t)i], y = q[3 * (size_t)i + 1], z = q[3 * (size_t)i + 2];
    const bool inside = x >= 0.0f && x <= L && y >= 0.0f && y <= L && z >= 0.0f && z <= L;
    if (!inside) list[atomicAdd(count, 1u)] = i;
}

// The failure bitmap over sorted positions -> query ids in kd order + count:
// per-word popcounts, an exclusive scan of them, then each word's set bits in
// order.  Every grid is sized by the call's query count, so nothing here needs
// the failure count on the host.
__global__ void __launch_bounds__(TB)
bits_popc_kernel(const uint32_t *__restrict__ bits, uint64_t nwords, uint32_t *__restrict__ pc) {
    const uint64_t w = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (w < nwords) pc[w] = (uint32_t)__popc(bits[w]);
}

// out = ord[j] for every set bit j in order (ord == nullptr: j itself); with
// tgp, also tgi[ord[j]] = tgp[j] (self queries: a failure's seed, kept per
// position in the first pass, by query id for the retry rounds)
__global__ void __launch_bounds__(TB)
bits_emit_kernel(const uint32_t *__restrict__ bits, const uint32_t *__restrict__ pc_excl,
                 uint64_t nwords, const uint32_t *__restrict__ ord, uint32_t *__restrict__ out,
                 uint32_t *__restrict__ count, const float *__restrict__ tgp,
                 float *__restrict__ tgi) {
    const uint64_t w = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (w >= nwords) return;
    uint32_t b = bits[w], o = pc_excl[w];
    if (w == nwords - 1) *count = o + (uint32_t)__popc(b);
    while (b) {
        const uint32_t j = (uint32_t)__builtin_ctz(b);
        b &= b - 1u;
        const uint32_t pj = (uint32_t)(w * 32 + j);
        const uint32_t id = ord ? ord[pj] : pj;
        out[o++] = id;
        if (tgp) tgi[id] = tgp[pj];
    }
}

// the set bits' indices in order, one thread per bit (consecutive threads
// write consecutive entries): a dense bitmap, as the self order's
// prefix selection (most bits set), where bits_emit_kernel's per-word loop
// would write 32 scattered runs per wave
__global__ void __launch_bounds__(TB)
bits_emit_dense_kernel(const uint32_t *__restrict__ bits, const uint32_t *__restrict__ pc_excl,
                       uint64_t nbits, uint32_t *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= nbits) return;
    const uint32_t w = bits[j >> 5], b = (uint32_t)j & 31u;
    if ((w >> b) & 1u) out[pc_excl[j >> 5] + (uint32_t)__popc(w & ((1u << b) - 1u))] = (uint32_t)j;
}

// kth[id] = rows[id * k + k - 1] for the ids of a device-counted list (list
// nullptr: every row below m): the rows no lane select wrote (the exact
// kernel's, every row at k > 64) into the nbkd_set_kth_out array
__global__ void __launch_bounds__(TB)
kth_patch_kernel(const float *__restrict__ rows, int k, const uint32_t *__restrict__ list,
                 const uint32_t *__restrict__ count, uint32_t m, float *__restrict__ kth) {
    const uint32_t n = list ? min(*count, m) : m;
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < n; i += gridDim.x * TB) {
        const uint32_t id = list ? list[i] : i;
        kth[id] = rows[(size_t)id * k + k - 1];
    }
}

// the entries of a device-counted list past what the rounds handled: appended
// to the next list (order irrelevant there: one query per wave, or the exact
// kernel)
__global__ void __launch_bounds__(TB)
spill_kernel(const uint32_t *__restrict__ from, const uint32_t *__restrict__ from_count,
             uint32_t handled, uint32_t *__restrict__ to, uint32_t *__restrict__ to_count) {
    const uint32_t c = *from_count;
    for (uint32_t i = handled + blockIdx.x * TB + threadIdx.x; i < c; i += gridDim.x * TB)
        to[atomicAdd(to_count, 1u)] = from[i];
}

nbkd_status compact_failures(Workspace &ws, const uint32_t *bits, uint32_t mm, const uint32_t *ord,
                             uint32_t *out, uint32_t *count, hipStream_t s,
                             const float *tgp = nullptr, float *tgi = nullptr) {
    const uint64_t nwords = ((uint64_t)mm + 31) / 32;
    uint32_t *pc = (uint32_t *)ws.get(WS_KEYS2, nwords * 4u + 16u, s);
    if (!pc) return NBKD_ENOMEM;
    const unsigned blocks = (unsigned)((nwords + TB - 1) / TB);
    bits_popc_kernel<<<blocks, TB, 0, s>>>(bits, nwords, pc);
    nbkd_status rc = device_excl_scan(ws, pc, nwords, s);
    if (rc) return rc;
    bits_emit_kernel<<<blocks, TB, 0, s>>>(bits, pc, nwords, ord, out, count, tgp, tgi);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

int key_bits(const Tree &t) {
    uint64_t maxkey = t.n8 >> 3;
    int b = 1;
    while (b < 32 && (1ull << b) <= maxkey) ++b;
    return b;
}

// bucket + sort queries by leaf: order[] = query ids in kd order
// order[] (workspace slot WS_ORDER) = query ids sorted by leaf
// Seed radius (guess_r2) parameters: mu = k + a sqrt(k) + b expected points in
// the seed sphere, density from the first subtree of <= anchor points on the
// query's descent.  NBKD_KNN_SEED=0 disables the seed (every bound starts +inf).
// the collect / select path serves k <= 1024 (knn_select_kernel for k <= 64,
// knn_select_wave_kernel above); larger k replays the reference per lane
constexpr int KNN_PACKET_KMAX = 1024;
// internal flag (never a caller's): this knn_locked call is an nbkd_query_knn
// whose CALLER asked for device rows, so it may write the nbkd_set_kth_out
// array (host_pipeline adds NBKD_OUTPUT_DEVICE to its batch calls,
// and kth_locked's k > 1024 rows go to scratch; neither may touch it)
constexpr uint32_t KNN_SIDE_OK = 0x80000000u;

#ifndef NBKD_KNN_CHILD_TH
#define NBKD_KNN_CHILD_TH 1.1f
#endif
#ifndef NBKD_KNN_CHILD_S
#define NBKD_KNN_CHILD_S 1.0f
#endif
struct SeedParams {
    bool on;
    float mu_c;
    uint32_t anchor;
    float child_th, child_s; // self seeds: a sparse anchor half's own seed (anchor_chunk_kernel)
};
SeedParams seed_params(const Tree &t, int k) {
    // a = 3.0 (round 5, with the self order, profiles/r05ab_seed_margin_ab.txt,
    // r05ac): 1e8 uniform 57.13 -> 56.92 ms (20.6 k -> 82 k re-walks, 49.9 ->
    // 47.9 candidates per query), log-normal 69.23 -> 69.11; 2.5 and below are
    // faster on uniform (56.46 at 2.25) but slower on log-normal (+0.43 ms at
    // 2.5, +1.6 at 2.0).  Until round 4 a = 3.5: 1.400e9 q/s at 1e8 uniform
    // (20.5 k retries) vs 1.376e9 at 4 (4.9 k), 1.393e9 at 3, 1.372e9 at 2.5,
    // 1.361e9 at 5; log-normal 82.3 ms at both 3.5 and 4 (r02bg, r02bi).  The
    // column capacity keeps a = 4.  nbkd_set_tuning("knn_seed_margin")
    // (default 3.0); NBKD_KNN_SEED in an experiments build (0 there: no seed,
    // the register top-k packet kernel)
    const char *e = knob("NBKD_KNN_SEED");
    const float a = e ? (float)atof(e) : (float)tuning(TUNE_KNN_SEED);
    SeedParams p;
    p.on = a > 0.0f;
    const float mu = (float)k + a * sqrtf((float)k) + a;
    p.mu_c = mu / (4.0f / 3.0f * 3.14159265f);
    // the density comes from the first subtree of <= anchor points on the
    // descent: 128 points, or the leaf when leaves are larger (at leafsize 64
    // the former 4-leaf anchor, 256 points, smoothed clustered densities too
    // much: log-normal 1e8 retried 5.7 M queries)
    const char *ea = knob("NBKD_KNN_ANCHOR"); // tuning only: anchor in points
    p.anchor = std::max<uint32_t>((uint32_t)t.leaf, ea ? (uint32_t)std::max(1, atoi(ea)) : 128u);
    const char *ec = knob("NBKD_KNN_CHILD"); // tuning only: 0 = the anchor's seed everywhere
    p.child_th = ec ? (float)atof(ec) : NBKD_KNN_CHILD_TH;
    const char *es = knob("NBKD_KNN_CHILD_S");
    p.child_s = es ? (float)atof(es) : NBKD_KNN_CHILD_S;
    return p;
}

// The box the seeds' density estimates cut with the splits: the real points'
// bounding box, periodic trees too (the density estimate only; the traversal
// starts from the box or unbounded).  A slab tree's points fill a strip of
// the periodic box; cells at the strip's faces reaching through the empty
// rest diluted their density, and their seeds overflowed the columns: with
// the extent-scheduled slab axes (nbkd_build_ext), 558 k of 12.5 M queries
// of an N = 8 slab were re-walked instead of 7 k (profiles/r05t_slab_ab.txt).
// For a filled box it is the box up to its outermost points.
float3 seed_lo(const Tree &t) { return make_float3(t.bbox_lo[0], t.bbox_lo[1], t.bbox_lo[2]); }
float3 seed_hi(const Tree &t) { return make_float3(t.bbox_hi[0], t.bbox_hi[1], t.bbox_hi[2]); }

nbkd_status sort_queries(const Tree &t, Workspace &ws, const float *dq, uint32_t m, uint32_t *&order,
                         hipStream_t s, float *tg = nullptr, const SeedParams *sp = nullptr) {
    order = (uint32_t *)ws.get(WS_ORDER, (size_t)m * 4, s);
    uint32_t *tmp = (uint32_t *)ws.get(WS_TMP, (size_t)m * 4, s);
    uint32_t *keys = (uint32_t *)ws.get(WS_KEYS, (size_t)m * 4, s);
    uint32_t *keys2 = (uint32_t *)ws.get(WS_KEYS2, (size_t)m * 4, s);
    if (!order || !tmp || !keys || !keys2) return NBKD_ENOMEM;
    {
        TimedScope ts("leaf_key", s);
        static const bool no_heap = knob("NBKD_NO_HEAP_SPLITS") != nullptr; // A/B only
        if (t.hsplit && !no_heap) {
            const unsigned blocks = (unsigned)std::min<uint64_t>((m + TB - 1) / TB, 8192);
            const float3 lo = seed_lo(t), hi = seed_hi(t);
            leaf_key3_kernel<<<blocks, TB, 0, s>>>((const float4 *)t.hsplit, hblk_offset(t.depth),
                                                   (uint32_t)t.n8, (uint32_t)t.leaf, dq, m,
                                                   keys, order, tg, sp ? sp->mu_c : 0.0f,
                                                   sp ? sp->anchor : 0u, lo, hi, t.axes,
                                                   sp ? sp->child_th : 0.0f, sp ? sp->child_s : 1.0f);
        } else if (t.shape_len <= SHAPE_MAX) {
            const unsigned blocks = (unsigned)std::min<uint64_t>((m + TB - 1) / TB, 8192);
            const float3 lo = seed_lo(t), hi = seed_hi(t);
            leaf_key2_kernel<<<blocks, TB, 0, s>>>(
                t.splits, t.shape_c, t.shape_n, t.shape_len, (uint32_t)t.n8, (uint32_t)t.leaf, dq,
                m, keys, order, tg, sp ? sp->mu_c : 0.0f, sp ? sp->anchor : 0u, lo, hi, t.axes);
        } else {
            if (tg) NBKD_HIP(hipMemsetD32Async((hipDeviceptr_t)tg, 0x7F7FFFFF, m, s)); // FLT_MAX: no seed
            leaf_key_kernel<<<(m + TB - 1) / TB, TB, 0, s>>>(view(t), dq, m, keys, order);
        }
        NBKD_HIP(hipGetLastError());
    }
    TimedScope ts("sort", s);
    return radix_sort(ws, keys, order, keys2, tmp, m, key_bits(t), s, &order);
}

// Self queries: the call's queries are the first m rows of the device array
// the tree was built from (the same pointer), as in the kNN of every particle
// that the bench and the density estimates run.  Tree order is then kd order
// already: the queries need neither the bucketing descent nor the sort, and
// each seed comes from the query's tree position (self_seed_kernel), indexed
// by its position in the order (QSpan::tg_pos).  Nothing checks that the
// array still holds the points the tree was built from, and nothing needs to:
// the order and the seeds only steer the work (a seed too small or too large
// is a seed failure and re-walked), every distance is computed from the
// queries as given.  nbkd_set_tuning("self_order", 0) turns it off.
bool self_query(const Tree &t, const float *q, uint64_t m, uint32_t flags) {
    return (flags & NBKD_INPUT_DEVICE) && q != nullptr && q == t.src && m > 0 && m <= t.n &&
           t.n8 < (1ull << 32) && t.hsplit != nullptr && tuning(TUNE_SELF_ORDER) != 0.0;
}

// tgp / sp nullptr: the order alone (radius queries)
nbkd_status self_order(const Tree &t, Workspace &ws, uint32_t m, uint32_t *&order, hipStream_t s,
                       float *tgp = nullptr, const SeedParams *sp = nullptr) {
    TimedScope ts("self_order", s);
    const uint32_t *perm = t.sidx ? t.sidx : t.idx;
    // the padding rows (FLT_MAX) sort after every real point on every axis,
    // so they hold the positions n..n8-1 unless a real coordinate is FLT_MAX
    const bool pads_last = t.n8 == t.n || t.periodic ||
                           (t.bbox_hi[0] < FLT_MAX && t.bbox_hi[1] < FLT_MAX && t.bbox_hi[2] < FLT_MAX);
    const uint32_t *pos = nullptr;
    if (m == t.n && pads_last) {
        order = const_cast<uint32_t *>(perm); // read only
    } else {
        // the tree positions of input rows 0..m-1, in tree order
        const uint64_t nwords = (t.n8 + 31) / 32;
        uint32_t *bits = (uint32_t *)ws.get(WS_KEYS2, nwords * 4u + 64u, s);
        uint32_t *plist = (uint32_t *)ws.get(WS_TMP, (size_t)m * 4 + 16, s);
        order = (uint32_t *)ws.get(WS_ORDER, (size_t)m * 4, s);
        if (!bits || !plist || !order) return NBKD_ENOMEM;
        uint32_t *pc = (uint32_t *)ws.get(WS_RSORT, nwords * 4u + 16u, s);
        if (!pc) return NBKD_ENOMEM;
        const unsigned pblocks = (unsigned)((t.n8 + TB - 1) / TB);
        self_bits_kernel<<<pblocks, TB, 0, s>>>(perm, t.n8, m, bits);
        bits_popc_kernel<<<(unsigned)((nwords + TB - 1) / TB), TB, 0, s>>>(bits, nwords, pc);
        const nbkd_status rc = device_excl_scan(ws, pc, nwords, s);
        if (rc) return rc;
        bits_emit_dense_kernel<<<pblocks, TB, 0, s>>>(bits, pc, t.n8, plist);
        NBKD_HIP(hipGetLastError());
        pos = plist;
    }
    if (!pos && !tgp) return NBKD_OK;
    const uint32_t nchunks = (uint32_t)((t.n8 + 63) / 64);
    uint4 *anch = nullptr;
    if (tgp) {
        anch = (uint4 *)ws.get(WS_ANCH, (size_t)nchunks * 16, s);
        if (!anch) return NBKD_ENOMEM;
        const float3 lo = seed_lo(t), hi = seed_hi(t);
        // an anchor below 64 points would break the two-anchors-per-chunk rule
        const uint32_t stop = std::max<uint32_t>({sp->anchor, (uint32_t)t.leaf, 128u});
        anchor_chunk_kernel<<<(nchunks + TB - 1) / TB, TB, 0, s>>>(
            t.hsplit, hblk_offset(t.depth), (uint32_t)t.n8, stop, nchunks, anch, sp->mu_c, lo, hi,
            t.axes, (uint32_t)t.leaf, sp->child_th, sp->child_s);
        NBKD_HIP(hipGetLastError());
    }
    if (!pos) {
        const uint64_t th = ((uint64_t)m + 3) / 4;
        self_seed4_kernel<<<(unsigned)((th + TB - 1) / TB), TB, 0, s>>>(anch, nchunks, m, tgp);
    } else {
        const unsigned blocks = (unsigned)std::min<uint64_t>(((uint64_t)m + TB - 1) / TB, 65536);
        self_seed_kernel<<<blocks, TB, 0, s>>>(anch, nchunks, pos, perm, m, order, tgp);
    }
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

nbkd_status stage_queries(Workspace &ws, const float *q, uint64_t m, uint32_t flags,
                          const float *&dq, hipStream_t s) {
    if (flags & NBKD_INPUT_DEVICE) {
        dq = q;
        return NBKD_OK;
    }
    float *buf = (float *)ws.get(WS_Q, m * 3 * sizeof(float), s);
    if (!buf) return NBKD_ENOMEM;
    NBKD_HIP(hipMemcpyAsync(buf, q, m * 3 * sizeof(float), hipMemcpyHostToDevice, s));
    NBKD_HIP(hipStreamSynchronize(s));
    dq = buf;
    return NBKD_OK;
}

} // namespace

// Candidate-column budget per collect/select batch: NBKD_CAND_BYTES, else the
// smaller of 96 GiB and a third of the free device memory.  Fewer, larger
// batches shorten the per-launch tails: 9 batches of 11 M queries (8 GiB) ->
// 3 at 1e8 is 53.9 -> 51.5 ms of collect (r02at); 3 (24 GiB, the cap until
// round 4) -> 1 (80 GiB) is 65.05 -> 63.95 ms per step
// (profiles/r04z_ab_budget_anchor.txt).  A 1e8 query on an otherwise empty
// MI355X (288 GB) now takes one batch of 77 GB of columns.
uint64_t cand_budget(bool *is_auto) {
    if (is_auto) *is_auto = false;
    const char *eb = knob("NBKD_CAND_BYTES");
    if (eb) return strtoull(eb, nullptr, 10);
    const double tb = tuning(TUNE_CAND_BYTES); // nbkd_set_tuning("candidate_bytes"), 0 = auto
    if (tb > 0.0) return (uint64_t)tb;
    if (is_auto) *is_auto = true;
    size_t free_b = 0, total_b = 0;
    uint64_t b = 96ull << 30;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
        // a third of the free memory, never more than what is free (the
        // callers' minimum is one 64-query packet's column)
        b = std::min<uint64_t>(b, free_b / 3);
    else
        (void)hipGetLastError();
    return b;
}

// LSD radix sort of (key, value) pairs for other translation units (deposit.hip)
nbkd_status sort_pairs(Workspace &ws, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1,
                       uint32_t n, int nbits, hipStream_t s, uint32_t **vout) {
    return radix_sort(ws, k0, v0, k1, v1, n, nbits, s, vout);
}

namespace {

bool collect_disabled() {
    static const bool off = [] {
        const char *e = knob("NBKD_KNN_COLLECT");
        return e && atoi(e) == 0;
    }();
    return off;
}

// out_i == nullptr: k-th distance only (out_d: m floats); the caller
// (query_kth) uses it only where the collect/select path runs
nbkd_status knn_locked(const Tree &t, Workspace &ws, const float *q, uint64_t m, int k, float *out_d,
                       uint32_t *out_i, uint32_t flags, hipStream_t s) {
    const uint32_t mm = (uint32_t)m;
    const bool kth_only = out_i == nullptr;
    const bool sq = (flags & NBKD_SQUARED) != 0;
    const size_t row_words = kth_only ? 1 : (size_t)k;
    const float *dq = nullptr;
    nbkd_status rc = stage_queries(ws, q, m, flags, dq, s);
    if (rc) return rc;
    // the collect / select path needs the sub-leaf groups (every non-empty
    // tree has them); k > 1024 and the empty tree take the exact kernel
    const bool packet = k <= KNN_PACKET_KMAX && t.ginfo != nullptr;
    const SeedParams sp = seed_params(t, k);
    float *tg = nullptr;
    if (packet && sp.on) {
        tg = (float *)ws.get(WS_TG, (size_t)mm * 4, s);
        if (!tg) return NBKD_ENOMEM;
    }
    uint32_t *ord = nullptr;
    // self queries: tree order, seeds per position (tgp) for the first pass
    const bool self = packet && tg && self_query(t, q, m, flags);
    float *tgp = nullptr;
    if (self) {
        tgp = (float *)ws.get(WS_KEYS, (size_t)mm * 4, s);
        if (!tgp) return NBKD_ENOMEM;
        rc = self_order(t, ws, mm, ord, s, tgp, &sp);
    } else {
        rc = sort_queries(t, ws, dq, mm, ord, s, tg, &sp);
    }
    if (rc) return rc;
    // nbkd_set_kth_out: a query of the tree's own rows (the first m of the
    // device array it was built from) with device rows also leaves each row's
    // last column in t.kth_side (the slab layer's exactness test reads it).
    // On every path: the self order or the sorted one
    // (self_order = 0), the lane selects write it (select_block indexes it by
    // query id), the exact kernel's rows and every row at k > 64 (including
    // k > 1024, no packet path) are copied by kth_patch_kernel below
    const bool own_rows = (flags & NBKD_INPUT_DEVICE) && q != nullptr && q == t.src && m > 0 &&
                          m <= t.n;
    float *const ks = own_rows && !kth_only && (flags & KNN_SIDE_OK) && t.kth_side &&
                              m <= t.kth_side_cap ? t.kth_side : nullptr;
    float *dd = out_d;
    uint32_t *di = out_i;
    if (!(flags & NBKD_OUTPUT_DEVICE)) {
        dd = (float *)ws.get(WS_OUTD, m * row_words * 4, s);
        di = kth_only ? nullptr : (uint32_t *)ws.get(WS_OUTI, m * (size_t)k * 4, s);
        if (!dd || (!di && !kth_only)) return NBKD_ENOMEM;
    }
    unsigned long long *stats = nullptr;
    if (stats_enabled()) {
        stats = (unsigned long long *)ws.get(WS_STATS, NBKD_NSTATS * 8, s);
        if (!stats) return NBKD_ENOMEM;
        NBKD_HIP(hipMemsetAsync(stats, 0, NBKD_NSTATS * 8, s));
    }
    // queries the packet kernel cannot answer exactly go through the
    // reference-exact lane-per-query kernel: periodic queries outside [0, L]^3
    // and queries whose seed radius held fewer than k points
    uint32_t *list = nullptr, *count = nullptr;
    if (packet && (t.periodic || tg)) {
        list = (uint32_t *)ws.get(WS_LIST, (size_t)mm * 4 + 16, s);
        if (!list) return NBKD_ENOMEM;
        count = list + mm;
        NBKD_HIP(hipMemsetAsync(count, 0, 4, s));
        // the collect / select path lists them in its first pass (QSpan::out_list)
        if (t.periodic && !(tg && !collect_disabled())) {
            TimedScope ts("knn_outside_box", s);
            outside_box_kernel<<<(mm + TB - 1) / TB, TB, 0, s>>>(dq, mm, t.box, list, count);
            NBKD_HIP(hipGetLastError());
        }
    }
    if (!packet) { // all queries through the reference-exact lane-per-query kernel
        TimedScope ts("knn_exact", s);
        uint32_t threads = (uint32_t)std::min<uint64_t>(
            std::max<uint64_t>((512ull << 20) / (32ull * (uint64_t)k), TB), 65536ull);
        threads = (uint32_t)std::min<uint64_t>(threads, ((uint64_t)mm + TB - 1) / TB * TB);
        threads = std::max<uint32_t>(threads / TB * TB, TB);
        LtEntry *lt = (LtEntry *)ws.get(WS_LT, (size_t)threads * 2 * k * sizeof(LtEntry), s);
        if (!lt) return NBKD_ENOMEM;
        if (t.periodic)
            knn_exact_kernel<true><<<threads / TB, TB, 0, s>>>(view(t), dq, ord, nullptr, mm, k,
                                                                lt, dd, di, sq);
        else
            knn_exact_kernel<false><<<threads / TB, TB, 0, s>>>(view(t), dq, ord, nullptr, mm, k,
                                                                 lt, dd, di, sq);
        NBKD_HIP(hipGetLastError());
    } else {
        if (tg && !collect_disabled()) {
            // collect + select in batches sized to the candidate-column budget
            const uint32_t capg = collect_capacity(k);
            // automatic budget: the columns this workspace already holds count
            // too (free memory no longer includes them), so a second call of
            // the same size splits the same way as the first (one batch at
            // 1e8); an explicit candidate_bytes is taken as given
            bool auto_budget = false;
            uint64_t budget = cand_budget(&auto_budget);
            if (auto_budget) budget = std::max<uint64_t>(budget, ws.cap[WS_CAND]);
            uint64_t batch = budget / ((uint64_t)capg * 8u) / 64u * 64u;
            batch = std::max<uint64_t>(batch, 64);
            batch = std::min<uint64_t>(batch, ((uint64_t)mm + 63) / 64 * 64);
            // the re-walk rounds' columns: 8 capg (packets of 64 or one query
            // per wave), then 64 capg (one query per wave)
            const uint32_t capr = capg * 8u, capr2 = capg * 64u;
            // A round-1 batch holds at most rb queries: the larger of ~10 % of
            // the queries and what the first pass's columns hold at 8 capg per
            // query (memory the call has anyway), within the columns' budget.
            // Round 1 runs up to RB1_MAX such batches, so it takes every
            // failure of any first pass with rb >= m / RB1_MAX (ADVICE r04:
            // round 4 took ~10 % and sent the rest to round 2 and the exact
            // kernel); the batches past the failure count exit at once on the
            // device.  Round 2: rb2 per batch, up to ~1 %.  The columns are
            // sized for THAT, not for every query failing at 64 capg: at
            // m = 1e5, k = 32 sizing them for m held ~5.7 GB of scratch where
            // the first pass needs ~90 MB.  What a round cannot take spills to
            // the next round, the last to the exact kernel.
            const uint64_t mm64 = ((uint64_t)mm + 63) / 64 * 64;
            const uint64_t rb = std::min<uint64_t>(
                std::max<uint64_t>(budget / ((uint64_t)capr * 8u) / 64u * 64u, 64),
                std::max<uint64_t>({64, ((uint64_t)mm / 10 + 63) / 64 * 64,
                                    batch * capg / capr / 64u * 64u}));
            const uint64_t rb2 = std::min<uint64_t>(
                std::max<uint64_t>(budget / ((uint64_t)capr2 * 8u), 64),
                std::max<uint64_t>(64, (uint64_t)mm / 100 + 1));
            // a round's pass covers at most min(cap, mm) queries, in packets of 64
            const uint64_t cap1 = std::min<uint64_t>(rb, mm64), cap2 = std::min<uint64_t>(rb2, mm);
            const uint64_t cand_bytes =
                std::max<uint64_t>({batch * capg * 8u, cap1 * capr * 8u, cap2 * capr2 * 8u});
            const uint64_t cc_words = std::max<uint64_t>(batch, cap1);
            uint2 *cand = (uint2 *)ws.get(WS_CAND, cand_bytes, s);
            uint32_t *ccount = (uint32_t *)ws.get(WS_CCOUNT, cc_words * 4u, s);
            // k > 64: per-query final bounds, collect -> wave select (any batch
            // of any round holds at most max(batch, mm) queries)
            float *kb = nullptr;
            if (k > 64) {
                kb = (float *)ws.get(WS_KB, std::max<uint64_t>(batch, (uint64_t)mm) * 4u, s);
                if (!kb) return NBKD_ENOMEM;
            }
            // 64 < k <= 128: the first pass's wave select takes two queries
            // per wave where it can; the leftover positions list here
            uint32_t *pair_scratch = nullptr;
            if (k > 64 && k <= 128) {
                pair_scratch = (uint32_t *)ws.get(WS_PAIR, (batch + 32) * 4u, s);
                if (!pair_scratch) return NBKD_ENOMEM;
            }
            // Seed failures (fewer than k points in the seed ball, or more than
            // the column holds) are re-walked without the host reading how many
            // there are: the first pass marks them in a bitmap over the sorted
            // positions; an ordered compaction turns it into query ids in kd
            // order plus a count in device memory; the rounds below run on
            // fixed grids that read that count (QSpan), and what a round does
            // not resolve goes to the next one, the last to the exact kernel.
            const uint64_t nwords = ((uint64_t)mm + 31) / 32;
            uint32_t *bits = (uint32_t *)ws.get(WS_RSORT, nwords * 4u + 64u, s);
            uint32_t *rq = (uint32_t *)ws.get(WS_LIST2, (size_t)mm * 8 + 256, s);
            if (!cand || !ccount || !bits || !rq) return NBKD_ENOMEM;
            uint32_t *rq_count = rq + (size_t)mm;      // round-1 queries (compaction)
            uint32_t *r2 = rq_count + 16;               // round-2 list (ids)
            uint32_t *r2_count = r2 + (size_t)mm;
            NBKD_HIP(hipMemsetAsync(bits, 0, nwords * 4u, s));
            NBKD_HIP(hipMemsetAsync(rq_count, 0, 4, s));
            NBKD_HIP(hipMemsetAsync(r2_count, 0, 4, s));
            const bool adaptive = retry_adaptive();
            {
                TimedScope ts("knn", s);
                for (uint64_t b0 = 0; b0 < mm; b0 += batch) {
                    const uint32_t nb = (uint32_t)std::min<uint64_t>(batch, mm - b0);
                    QSpan sp1 = static_span(nb);
                    sp1.tg_pos = self; // seeds (and the first pass's rewritten ones) per position
                    if (t.periodic) {
                        sp1.out_list = list;
                        sp1.out_count = count;
                    }
                    rc = launch_knn_collect(t, dq, ord + b0, sp1, k, self ? tgp + b0 : tg, 1.0f, 64u,
                                            cand, capg, ccount, dd, di, nullptr, nullptr, bits,
                                            (uint32_t)b0, false, adaptive, sq, kb, stats, s, ks,
                                            pair_scratch);
                    if (rc) return rc;
                }
            }
            {
                TimedScope ts2("knn_retry_order", s);
                // self queries: the failures' seeds move to tg by query id
                rc = compact_failures(ws, bits, mm, ord, rq, rq_count, s, self ? tgp : nullptr,
                                      self ? tg : nullptr);
                if (rc) return rc;
            }
            if (stats) NBKD_HIP(hipMemcpyAsync(stats + 9, rq_count, 4, hipMemcpyDeviceToDevice, s));
            // round 1: the failures in kd order, as packets of 64 where they
            // are dense (>= 1/512 of the queries, as on clustered inputs: a
            // coherent walk) and one query per wave where they are sparse
            // (uniform 1e8, r02bi: 82 k failures 1.1 ms one per wave vs 1.9 ms
            // as packets); up to RB1_MAX batches of rb, enough for every
            // failure when rb >= m / RB1_MAX (the later batches exit at once
            // on the device); what remains goes straight to round 2
            constexpr uint64_t RB1_MAX = 10;
            const uint32_t nb1 =
                (uint32_t)std::min<uint64_t>(RB1_MAX, std::max<uint64_t>(1, (mm64 + rb - 1) / rb));
            // the re-walk rounds as one timed phase (one pair of events, not
            // one per launch of their ~40 mostly empty launches)
            TimedScope ts3("knn_retry", s);
            for (uint32_t bi = 0; bi < nb1; ++bi) {
                for (int mode = 1; mode <= 2; ++mode) {
                    const QSpan sp{(uint32_t)cap1, rq_count, (uint32_t)(bi * rb), mm, mode, bi > 0};
                    rc = launch_knn_collect(t, dq, rq + bi * rb, sp, k, tg, adaptive ? 1.0f : 4.0f,
                                            mode == 1 ? 64u : 1u, cand, capr, ccount, dd, di,
                                            adaptive ? r2 : list, adaptive ? r2_count : count,
                                            nullptr, 0xFFFFFFFFu, true, adaptive, sq, kb, nullptr, s,
                                            ks);
                    if (rc) return rc;
                }
            }
            spill_kernel<<<64, TB, 0, s>>>(rq, rq_count, (uint32_t)std::min<uint64_t>(nb1 * rb, mm64),
                                           adaptive ? r2 : list, adaptive ? r2_count : count);
            NBKD_HIP(hipGetLastError());
            if (adaptive) {
                // round 2, one query per wave: the seed each failure rewrote
                // (2x..8x volume when short, the same seed when the 8x column
                // overflowed) and a 64x column; what still fails joins the
                // exact kernel's list
                const uint32_t nb2 = (uint32_t)std::min<uint64_t>(
                    4, std::max<uint64_t>(1, ((uint64_t)mm / 100 + rb2 - 1) / rb2));
                for (uint32_t bi = 0; bi < nb2; ++bi) {
                    const QSpan sp{(uint32_t)cap2, r2_count, (uint32_t)(bi * rb2), mm, 0};
                    rc = launch_knn_collect(t, dq, r2 + bi * rb2, sp, k, tg, 1.0f, 1u, cand, capr2,
                                            ccount, dd, di, list, count, nullptr, 0xFFFFFFFFu, true,
                                            false, sq, kb, nullptr, s, ks);
                    if (rc) return rc;
                }
                spill_kernel<<<64, TB, 0, s>>>(r2, r2_count, (uint32_t)std::min<uint64_t>(nb2 * rb2, mm),
                                               list, count);
                NBKD_HIP(hipGetLastError());
            }
        } else {
            // a seed margin <= 0 exists only in experiments builds (NBKD_KNN_SEED);
            // the round-1 no-seed packet kernel it selected is retired
            set_error("internal: the kNN query has no seed bound (knn_seed_margin <= 0)");
            return NBKD_EINVAL;
        }
        if (list) {
            TimedScope ts("knn_fallback", s);
            const uint32_t threads = 16384;
            LtEntry *lt = (LtEntry *)ws.get(WS_LT, (size_t)threads * 2 * k * sizeof(LtEntry), s);
            if (!lt) return NBKD_ENOMEM;
            if (t.periodic)
                knn_exact_kernel<true><<<threads / TB, TB, 0, s>>>(view(t), dq, list, count, mm, k,
                                                                   lt, dd, di, sq);
            else
                knn_exact_kernel<false><<<threads / TB, TB, 0, s>>>(view(t), dq, list, count, mm,
                                                                    k, lt, dd, di, sq);
            NBKD_HIP(hipGetLastError());
            if (stats) NBKD_HIP(hipMemcpyAsync(stats + 8, count, 4, hipMemcpyDeviceToDevice, s));
        }
    }
    if (ks) { // rows the lane selects did not write: the exact kernel's, or all at k > 64
        const bool all = !packet || k > 64;
        if (all || list) {
            kth_patch_kernel<<<all ? std::max(1u, std::min(65536u, (mm + TB - 1) / TB)) : 64, TB, 0,
                               s>>>(dd, k, all ? nullptr : list, all ? nullptr : count, mm, ks);
            NBKD_HIP(hipGetLastError());
        }
    }
    if (stats) {
        uint64_t h[NBKD_NSTATS];
        NBKD_HIP(hipMemcpyAsync(h, stats, NBKD_NSTATS * 8, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
        stats_add(h);
    }
    if (!(flags & NBKD_OUTPUT_DEVICE)) {
        NBKD_HIP(hipMemcpyAsync(out_d, dd, m * row_words * 4, hipMemcpyDeviceToHost, s));
        if (!kth_only)
            NBKD_HIP(hipMemcpyAsync(out_i, di, m * (size_t)k * 4, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
    }
    return NBKD_OK;
}

nbkd_status knn_args(int k, uint64_t m) {
    if (k <= 0) {
        set_error("k must be positive integer");
        return NBKD_EINVAL;
    }
    if (m >= (1ull << 32)) {
        set_error("more than 2^32 - 1 queries per call are not supported");
        return NBKD_EINVAL;
    }
    return NBKD_OK;
}

// out[i] = rows[i * k + k - 1]
__global__ void __launch_bounds__(TB)
kth_column_kernel(const float *__restrict__ rows, uint32_t m, int k, float *__restrict__ out) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i < m) out[i] = rows[(size_t)i * k + (k - 1)];
}

} // namespace

// Host-buffer calls of any size (a 1e9-query host call needed
// ~256 GB of device row scratch).  The m queries run in batches of hb through
// two device slots and two pinned host staging slots (Workspace::host_pinned,
// kept across calls): the host copies batch i's queries from the caller's
// array into pinned slot i % 2 (host_copy: a few threads), the copy stream
// `cp` moves them to the device, batch i computes on `s`, `cp` DMAs its results
// into the same pinned slot, and while batch i computes and moves, the host
// copies batch i-1's results from pinned memory into the caller's arrays.
// Each hop waits on events only.  Until round 4 the copies went straight
// between pageable memory and the device (the runtime stages those through
// its own small pinned buffers) with a stream synchronisation per batch:
// 8.8e7 queries/s host to host at 1e8, k = 32 (profiles/r04ar_suite.json).
// Device scratch is bounded by hb whatever m is: hb counts the caller's bytes
// per query plus the per-query device scratch a batch call allocates that no
// budget bounds (scratch_per_q).  Inputs or outputs already on the device are
// used in place.  The thread's interrupt check (nbkd_set_interrupt) runs
// between batches.
uint64_t host_batch(size_t bytes_per_query, uint64_t m) {
    const double tb = tuning(TUNE_HOST_BATCH);
    uint64_t hb = tb > 0.0 ? (uint64_t)tb
                           : (1ull << 30) / std::max<size_t>(bytes_per_query, 1);
    hb = std::max<uint64_t>(hb / 64 * 64, 64);
    return std::min<uint64_t>(hb, m);
}

template <typename Run>
nbkd_status host_pipeline(Workspace &ws, const float *q, uint64_t m, uint32_t flags, int nout,
                          const size_t *obytes, void *const *outs, size_t scratch_per_q, Run run,
                          hipStream_t s) {
    const bool in_dev = (flags & NBKD_INPUT_DEVICE) != 0, out_dev = (flags & NBKD_OUTPUT_DEVICE) != 0;
    size_t per_q = in_dev ? 0 : 12;
    for (int j = 0; j < nout; ++j) per_q += out_dev ? 0 : obytes[j];
    const uint64_t hb = host_batch(per_q + scratch_per_q, m);
    NBKD_HIP(ws.pipe_init());
    hipStream_t cp = ws.copy;
    hipEvent_t *ev_in = ws.pev, *ev_comp = ws.pev + 2, *ev_out = ws.pev + 4;
    // the previous call of this workspace may still use the device slots
    if (ws.used && ws.done) NBKD_HIP(hipStreamWaitEvent(cp, ws.done, 0));
    const int nslots = m > hb ? 2 : 1;
    float *qslot[2] = {nullptr, nullptr};
    void *oslot[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    char *hp[2] = {nullptr, nullptr};
    bool pageable = false;
    // pinned slot layout: [queries hb x 12 B][output 0][output 1]
    size_t ooff[2] = {in_dev ? 0 : hb * 12, 0};
    if (nout > 1) ooff[1] = ooff[0] + (out_dev ? 0 : hb * obytes[0]);
    for (int b = 0; b < nslots; ++b) {
        if (!in_dev) {
            qslot[b] = (float *)ws.get(WS_HQ0 + b, hb * 12, s);
            if (!qslot[b]) return NBKD_ENOMEM;
        }
        if (!out_dev)
            for (int j = 0; j < nout; ++j) {
                oslot[b][j] = ws.get(WS_HO00 + 2 * b + j, hb * obytes[j], s);
                if (!oslot[b][j]) return NBKD_ENOMEM;
            }
        if (per_q && !pageable) {
            hp[b] = (char *)ws.host_pinned(b, hb * per_q);
            // pinning failed or the process cap is reached:
            // stream between the caller's pageable arrays and the device
            if (!hp[b]) pageable = true;
        }
    }
    nbkd_status rc = NBKD_OK;
    bool in_rec[2] = {false, false}, comp_rec[2] = {false, false}, out_rec[2] = {false, false};
    const uint64_t nbat = (m + hb - 1) / hb;
    auto fail = [&](hipError_t e, const char *what) {
        rc = hip_fail(e, what);
        return rc;
    };
#define NBKD_PIPE(call)                                                                            \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            fail(e_, #call);                                                                       \
            goto drain;                                                                            \
        }                                                                                          \
    } while (0)
    for (uint64_t i = 0; i <= nbat; ++i) {
        if (i < nbat) {
            const int b = (int)(i & 1) % nslots;
            const uint64_t b0 = i * hb, nb = std::min<uint64_t>(hb, m - b0);
            if (i > 0 && interrupted()) {
                set_error("interrupted");
                rc = NBKD_EINTR;
                break;
            }
            const float *dq = q + 3 * b0;
            if (!in_dev) {
                // pinned slot b's previous queries (batch i-2) have left for the device
                if (in_rec[b]) NBKD_PIPE(hipEventSynchronize(ev_in[b]));
                if (!pageable) host_copy(hp[b], q + 3 * b0, nb * 12);
                // device slot b is free once batch i-2 finished reading it
                if (comp_rec[b]) NBKD_PIPE(hipStreamWaitEvent(cp, ev_comp[b], 0));
                NBKD_PIPE(hipMemcpyAsync(qslot[b], pageable ? (const void *)(q + 3 * b0) : hp[b],
                                         nb * 12, hipMemcpyHostToDevice, cp));
                NBKD_PIPE(hipEventRecord(ev_in[b], cp));
                in_rec[b] = true;
                NBKD_PIPE(hipStreamWaitEvent(s, ev_in[b], 0));
                dq = qslot[b];
            }
            void *o[2] = {nullptr, nullptr};
            for (int j = 0; j < nout; ++j)
                o[j] = out_dev ? (void *)((char *)outs[j] + b0 * obytes[j]) : oslot[b][j];
            // device output slot b is free once batch i-2's results left it
            if (!out_dev && out_rec[b]) NBKD_PIPE(hipStreamWaitEvent(s, ev_out[b], 0));
            rc = run(dq, nb, o, s);
            if (rc) break;
            NBKD_PIPE(hipEventRecord(ev_comp[b], s));
            comp_rec[b] = true;
            if (!out_dev) {
                NBKD_PIPE(hipStreamWaitEvent(cp, ev_comp[b], 0));
                for (int j = 0; j < nout; ++j)
                    NBKD_PIPE(hipMemcpyAsync(pageable ? (char *)outs[j] + b0 * obytes[j]
                                                      : hp[b] + ooff[j],
                                             oslot[b][j], nb * obytes[j], hipMemcpyDeviceToHost, cp));
                NBKD_PIPE(hipEventRecord(ev_out[b], cp));
                out_rec[b] = true;
            }
        }
        if (i >= 1 && !out_dev) {
            // batch i-1's results: pinned -> the caller's arrays, while batch i
            // computes and moves
            const int pb = (int)((i - 1) & 1) % nslots;
            const uint64_t p0 = (i - 1) * hb, pn = std::min<uint64_t>(hb, m - p0);
            NBKD_PIPE(hipEventSynchronize(ev_out[pb]));
            if (!pageable)
                for (int j = 0; j < nout; ++j)
                    host_copy((char *)outs[j] + p0 * obytes[j], hp[pb] + ooff[j], pn * obytes[j]);
        }
    }
#undef NBKD_PIPE
drain:
    if (rc) {
        // nothing of this call may still touch the slots or the caller's memory
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(cp);
        return rc;
    }
    // the pinned query slots are free for the next call once their DMA is done
    if (!in_dev) NBKD_HIP(hipStreamSynchronize(cp));
    return NBKD_OK;
}

// device scratch per query of one batch call that no budget bounds: the
// order / seed / list / failure buffers (~40 B), plus the full rows the k-th
// distance takes where the collect / select path does not run (k > 1024, the
// empty tree): kth_locked.  The candidate columns are budgeted
// (cand_budget) and not counted here.
static size_t knn_scratch_per_query(const Tree &t, int k, bool kth) {
    size_t b = 40;
    if (kth && !(k <= KNN_PACKET_KMAX && t.ginfo && seed_params(t, k).on && !collect_disabled()))
        b += (size_t)k * 8;
    return b;
}

nbkd_status query_knn(const Tree &t, const float *q, uint64_t m, int k, float *out_d,
                      uint32_t *out_i, uint32_t flags, hipStream_t s) {
    nbkd_status rc = knn_args(k, m);
    if (rc || m == 0) return rc;
    if (stats_enabled()) stats_reset(); // this call's counters, summed over its batches
    Workspace &ws = acquire_ws(t);
    WsCall call(ws, s, std::adopt_lock);
    NBKD_HIP(call.err);
    const uint32_t dev_io = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE;
    flags &= ~KNN_SIDE_OK;
    if ((flags & dev_io) == dev_io)
        return knn_locked(t, ws, q, m, k, out_d, out_i, flags | KNN_SIDE_OK, s);
    const size_t ob[2] = {(size_t)k * 4, (size_t)k * 4};
    void *const outs[2] = {out_d, out_i};
    return host_pipeline(ws, q, m, flags, 2, ob, outs, knn_scratch_per_query(t, k, false),
                         [&](const float *dq, uint64_t nb, void *const *o, hipStream_t st) {
                             return knn_locked(t, ws, dq, nb, k, (float *)o[0], (uint32_t *)o[1],
                                               flags | dev_io, st);
                         }, s);
}

// device in, device out: the k-th distances of m queries
static nbkd_status kth_locked(const Tree &t, Workspace &ws, const float *dq, uint64_t m, int k,
                              float *out_d, uint32_t flags, hipStream_t s) {
    // the collect/select path writes the k-th distance alone; elsewhere the
    // rows go to scratch and column k-1 is copied out
    if (k <= KNN_PACKET_KMAX && t.ginfo && seed_params(t, k).on && !collect_disabled())
        return knn_locked(t, ws, dq, m, k, out_d, nullptr, flags, s);
    float *rd = (float *)ws.get(WS_KTHD, m * (size_t)k * 4, s);
    uint32_t *ri = (uint32_t *)ws.get(WS_KTHI, m * (size_t)k * 4, s);
    if (!rd || !ri) return NBKD_ENOMEM;
    nbkd_status rc = knn_locked(t, ws, dq, m, k, rd, ri, flags, s);
    if (rc) return rc;
    kth_column_kernel<<<(unsigned)((m + TB - 1) / TB), TB, 0, s>>>(rd, (uint32_t)m, k, out_d);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

nbkd_status query_kth(const Tree &t, const float *q, uint64_t m, int k, float *out_d,
                      uint32_t flags, hipStream_t s) {
    nbkd_status rc = knn_args(k, m);
    if (rc || m == 0) return rc;
    if (stats_enabled()) stats_reset(); // this call's counters, summed over its batches
    Workspace &ws = acquire_ws(t);
    WsCall call(ws, s, std::adopt_lock);
    NBKD_HIP(call.err);
    const uint32_t dev_io = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE;
    if ((flags & dev_io) == dev_io) return kth_locked(t, ws, q, m, k, out_d, flags, s);
    const size_t ob[1] = {4};
    void *const outs[1] = {out_d};
    return host_pipeline(ws, q, m, flags, 1, ob, outs, knn_scratch_per_query(t, k, true),
                         [&](const float *dq, uint64_t nb, void *const *o, hipStream_t st) {
                             return kth_locked(t, ws, dq, nb, k, (float *)o[0], flags | dev_io, st);
                         }, s);
}

// the radius count of m device queries (count into out_count: device memory
// when NBKD_OUTPUT_DEVICE, else staged)
static nbkd_status ball_common(const Tree &t, Workspace &ws, const float *q, uint64_t m, float r,
                               uint32_t *out_count, uint32_t flags, hipStream_t s) {
    if (m >= (1ull << 32)) {
        set_error("more than 2^32 - 1 queries per call are not supported");
        return NBKD_EINVAL;
    }
    if (m == 0) return NBKD_OK;
    const uint32_t mm = (uint32_t)m;
    const float *dq = nullptr;
    nbkd_status rc = stage_queries(ws, q, m, flags, dq, s);
    if (rc) return rc;
    uint32_t *ord = nullptr;
    rc = self_query(t, q, m, flags) ? self_order(t, ws, mm, ord, s)
                                    : sort_queries(t, ws, dq, mm, ord, s);
    if (rc) return rc;
    const float r2 = r * r;
    // periodic queries outside [0, L]^3: listed (their count stays in device
    // memory), every point tested for them
    uint32_t *list = nullptr;
    if (t.periodic) {
        list = (uint32_t *)ws.get(WS_LIST, (size_t)mm * 8 + 16, s);
        if (!list) return NBKD_ENOMEM;
        NBKD_HIP(hipMemsetAsync(list + mm, 0, 4, s));
        outside_box_kernel<<<(mm + TB - 1) / TB, TB, 0, s>>>(dq, mm, t.box, list, list + mm);
    }
    unsigned long long *stats = nullptr;
    if (stats_enabled()) {
        stats = (unsigned long long *)ws.get(WS_STATS, NBKD_NSTATS * 8, s);
        if (!stats) return NBKD_ENOMEM;
        NBKD_HIP(hipMemsetAsync(stats, 0, NBKD_NSTATS * 8, s));
    }
    uint32_t *cnt = out_count;
    const bool dev_out = flags & NBKD_OUTPUT_DEVICE;
    if (!dev_out) {
        cnt = (uint32_t *)ws.get(WS_COUNT, m * 4, s);
        if (!cnt) return NBKD_ENOMEM;
    }
    {
        TimedScope ts("ball_count", s);
        launch_ball_packet(t, dq, ord, mm, r2, cnt, nullptr, nullptr, stats, s);
        if (list) launch_ball_outside_dev(t, dq, list, list + mm, r2, cnt, s);
        NBKD_HIP(hipGetLastError());
    }
    if (stats) {
        uint64_t h[NBKD_NSTATS];
        NBKD_HIP(hipMemcpyAsync(h, stats, NBKD_NSTATS * 8, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
        stats_add(h);
    }
    if (!dev_out) {
        NBKD_HIP(hipMemcpyAsync(out_count, cnt, m * 4, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
    }
    return NBKD_OK;
}

nbkd_status query_ball_count(const Tree &t, const float *q, uint64_t m, float r,
                             uint32_t *out_count, uint32_t flags, hipStream_t s) {
    if (m >= (1ull << 32)) {
        set_error("more than 2^32 - 1 queries per call are not supported");
        return NBKD_EINVAL;
    }
    if (m == 0) return NBKD_OK;
    if (stats_enabled()) stats_reset();
    Workspace &ws = acquire_ws(t);
    WsCall call(ws, s, std::adopt_lock);
    NBKD_HIP(call.err);
    const uint32_t dev_io = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE;
    if ((flags & dev_io) == dev_io)
        return ball_common(t, ws, q, m, r, out_count, flags, s);
    const size_t ob[1] = {4};
    void *const outs[1] = {out_count};
    return host_pipeline(ws, q, m, flags, 1, ob, outs, 40,
                         [&](const float *dq, uint64_t nb, void *const *o, hipStream_t st) {
                             return ball_common(t, ws, dq, nb, r, (uint32_t *)o[0], flags | dev_io,
                                                st);
                         }, s);
}

namespace {

// The CSR fill of one batch: nb device queries, their rows at the device
// offsets doff (nb + 1, relative to the batch), ids into di
nbkd_status ball_fill_batch(const Tree &t, Workspace &ws, const float *dq, uint32_t nb, float r,
                            const uint64_t *doff, uint32_t *di, hipStream_t s) {
    uint32_t *ord = nullptr;
    nbkd_status rc = self_query(t, dq, nb, NBKD_INPUT_DEVICE) ? self_order(t, ws, nb, ord, s)
                                                               : sort_queries(t, ws, dq, nb, ord, s);
    if (rc) return rc;
    const float r2 = r * r;
    uint32_t *list = nullptr, nout = 0;
    if (t.periodic) { // periodic queries outside [0, L]^3: every point tested for them
        list = (uint32_t *)ws.get(WS_LIST, (size_t)nb * 8 + 16, s);
        if (!list) return NBKD_ENOMEM;
        NBKD_HIP(hipMemsetAsync(list + nb, 0, 4, s));
        outside_box_kernel<<<(nb + TB - 1) / TB, TB, 0, s>>>(dq, nb, t.box, list, list + nb);
        NBKD_HIP(hipMemcpyAsync(&nout, list + nb, 4, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
    }
    TimedScope ts("ball_fill", s);
    launch_ball_packet(t, dq, ord, nb, r2, nullptr, doff, di, nullptr, s);
    launch_ball_outside(t, dq, list, nout, r2, nullptr, list ? list + nb + 4 : nullptr, doff, di,
                        s);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

// NBKD_SORTED: every row of a batch ascending, on the device.  Rows of up to
// csr_sort_row_cap() ids are sorted in LDS by one wave each (ball.hip); the
// longer ones, listed by that kernel, one by one by the LSD radix sort
// (values = keys)
nbkd_status sort_csr_batch(Workspace &ws, const uint64_t *doff, uint32_t *di, uint32_t nb,
                           const uint64_t *hrel, hipStream_t s) {
    uint32_t *lr = (uint32_t *)ws.get(WS_LIST2, (size_t)nb * 4 + 64, s);
    if (!lr) return NBKD_ENOMEM;
    uint32_t *nl = lr + nb;
    NBKD_HIP(hipMemsetAsync(nl, 0, 4, s));
    {
        TimedScope ts("csr_sort", s);
        launch_csr_sort_rows(doff, di, nb, lr, nl, s);
        NBKD_HIP(hipGetLastError());
    }
    uint32_t nlong = 0;
    NBKD_HIP(hipMemcpyAsync(&nlong, nl, 4, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    if (nlong == 0) return NBKD_OK;
    std::vector<uint32_t> rows(nlong);
    NBKD_HIP(hipMemcpyAsync(rows.data(), lr, (size_t)nlong * 4, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    for (uint32_t row : rows) {
        const uint64_t a = hrel[row], len = hrel[row + 1] - a;
        if (len >= (1ull << 32)) {
            set_error("query_ball_csr: a row of 2^32 or more neighbours cannot be sorted");
            return NBKD_EINVAL;
        }
        const size_t bytes = (size_t)len * 4;
        uint32_t *k0 = (uint32_t *)ws.get(WS_KTHD, bytes, s);
        uint32_t *v0 = (uint32_t *)ws.get(WS_KTHI, bytes, s);
        uint32_t *k1 = (uint32_t *)ws.get(WS_RSORT, bytes, s);
        uint32_t *v1 = (uint32_t *)ws.get(WS_CCOUNT, bytes, s);
        if (!k0 || !v0 || !k1 || !v1) return NBKD_ENOMEM;
        NBKD_HIP(hipMemcpyAsync(k0, di + a, bytes, hipMemcpyDeviceToDevice, s));
        NBKD_HIP(hipMemcpyAsync(v0, di + a, bytes, hipMemcpyDeviceToDevice, s));
        uint32_t *vout = nullptr;
        nbkd_status rc = radix_sort(ws, k0, v0, k1, v1, (uint32_t)len, 32, s, &vout);
        if (rc) return rc;
        NBKD_HIP(hipMemcpyAsync(di + a, vout, bytes, hipMemcpyDeviceToDevice, s));
    }
    return NBKD_OK;
}

// ids per fill batch (device scratch ~4 B each, twice for the two slots, plus
// the pinned staging of the same size)
constexpr uint64_t CSR_BATCH_IDS = 1ull << 26;

} // namespace

// Round 6: counts through the host-buffer pipeline (any m),
// then the fill in batches bounded by CSR_BATCH_IDS ids and host_batch
// queries, each batch sorted per row on the device (NBKD_SORTED) and copied
// out through two pinned slots while the next batch is filled.  Until round 5
// the call held every query, count and id in device scratch at once.
nbkd_status query_ball_csr(const Tree &t, const float *q, uint64_t m, float r, uint64_t *offsets,
                           uint32_t *out_idx, uint64_t capacity, uint32_t flags, hipStream_t s) {
    if (m >= (1ull << 32)) {
        set_error("more than 2^32 - 1 queries per call are not supported");
        return NBKD_EINVAL;
    }
    if (m == 0) {
        if (offsets) offsets[0] = 0;
        return NBKD_OK;
    }
    Workspace &ws = acquire_ws(t);
    WsCall call(ws, s, std::adopt_lock);
    NBKD_HIP(call.err);
    const uint32_t dev_io = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE;
    const bool out_dev = (flags & NBKD_OUTPUT_DEVICE) != 0;
    const uint32_t cflags = flags & (NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE);
    nbkd_status rc;
    {
        // 1. every query's count, streamed into host memory
        std::vector<uint32_t> hc(m);
        const size_t ob[1] = {4};
        void *const outs[1] = {hc.data()};
        rc = host_pipeline(ws, q, m, cflags & ~NBKD_OUTPUT_DEVICE, 1, ob, outs, 40,
                           [&](const float *dq, uint64_t nb, void *const *o, hipStream_t st) {
                               return ball_common(t, ws, dq, nb, r, (uint32_t *)o[0],
                                                  cflags | dev_io, st);
                           }, s);
        if (rc) return rc;
        offsets[0] = 0;
        for (uint64_t i = 0; i < m; ++i) offsets[i + 1] = offsets[i] + hc[i];
    }
    if (!out_idx) return NBKD_OK;
    if (capacity < offsets[m]) {
        set_error("query_ball_csr: capacity smaller than the number of neighbours");
        return NBKD_EINVAL;
    }
    if (offsets[m] == 0) return NBKD_OK;
    // 2. the fill, batch by batch
    const uint64_t qcap = host_batch(12 + 8 + 40, m);
    NBKD_HIP(ws.pipe_init());
    hipStream_t cp = ws.copy;
    hipEvent_t *ev_comp = ws.pev + 2, *ev_out = ws.pev + 4;
    if (ws.used && ws.done) NBKD_HIP(hipStreamWaitEvent(cp, ws.done, 0));
    bool out_rec[2] = {false, false};
    uint64_t prev_b0 = 0, prev_nnz = 0;
    int prev_slot = -1;
    char *hp[2] = {nullptr, nullptr};
    bool pageable = out_dev;
    std::vector<uint64_t> rel;
    auto drain_prev = [&]() -> nbkd_status { // batch i-1's ids: pinned -> the caller's array
        if (prev_slot < 0 || out_dev) return NBKD_OK;
        NBKD_HIP(hipEventSynchronize(ev_out[prev_slot]));
        if (hp[prev_slot]) host_copy(out_idx + offsets[prev_b0], hp[prev_slot], prev_nnz * 4);
        prev_slot = -1;
        return NBKD_OK;
    };
    int it = 0;
    for (uint64_t b0 = 0, b1; b0 < m; b0 = b1, ++it) {
        if (b0 > 0 && interrupted()) {
            set_error("interrupted");
            rc = NBKD_EINTR;
            break;
        }
        // the longest run of queries from b0 holding at most CSR_BATCH_IDS ids
        // (at least one query) and qcap queries
        const uint64_t lim = std::min<uint64_t>(m, b0 + qcap);
        b1 = (uint64_t)(std::upper_bound(offsets + b0 + 1, offsets + lim + 1,
                                         offsets[b0] + CSR_BATCH_IDS) - offsets) - 1;
        b1 = std::max<uint64_t>(b1, b0 + 1);
        const uint32_t nb = (uint32_t)(b1 - b0);
        const uint64_t nnz = offsets[b1] - offsets[b0];
        const int b = it & 1;
        const float *dq = nullptr;
        rc = stage_queries(ws, q + 3 * b0, nb, cflags, dq, s);
        if (rc) break;
        rel.resize(nb + 1);
        for (uint32_t i = 0; i <= nb; ++i) rel[i] = offsets[b0 + i] - offsets[b0];
        uint64_t *doff = (uint64_t *)ws.get(WS_OFF, (size_t)(nb + 1) * 8, s);
        if (!doff) {
            rc = NBKD_ENOMEM;
            break;
        }
        NBKD_HIP(hipMemcpyAsync(doff, rel.data(), (size_t)(nb + 1) * 8, hipMemcpyHostToDevice, s));
        uint32_t *di = out_idx + offsets[b0];
        if (!out_dev) {
            // device slot b is free once batch i-2's ids left it
            if (out_rec[b]) NBKD_HIP(hipStreamWaitEvent(s, ev_out[b], 0));
            di = (uint32_t *)ws.get(b == 0 ? WS_IDX : WS_HO11, std::max<uint64_t>(nnz, 1) * 4, s);
            if (!di) {
                rc = NBKD_ENOMEM;
                break;
            }
        }
        if (nnz) {
            rc = ball_fill_batch(t, ws, dq, nb, r, doff, di, s);
            if (rc) break;
            if (flags & NBKD_SORTED) {
                rc = sort_csr_batch(ws, doff, di, nb, rel.data(), s);
                if (rc) break;
            }
        }
        // the host copy of batch i-1 (its D2H overlapped this batch's fill)
        rc = drain_prev();
        if (rc) break;
        if (!out_dev && nnz) {
            NBKD_HIP(hipEventRecord(ev_comp[b], s));
            NBKD_HIP(hipStreamWaitEvent(cp, ev_comp[b], 0));
            // pinned slot b (kept by the workspace); refused pinning, or a
            // batch of one row longer than the slot: straight to the caller
            hp[b] = nullptr;
            if (!pageable && nnz <= CSR_BATCH_IDS) {
                hp[b] = (char *)ws.host_pinned(b, CSR_BATCH_IDS * 4);
                if (!hp[b]) pageable = true;
            }
            if (hp[b]) {
                NBKD_HIP(hipMemcpyAsync(hp[b], di, nnz * 4, hipMemcpyDeviceToHost, cp));
                NBKD_HIP(hipEventRecord(ev_out[b], cp));
                out_rec[b] = true;
                prev_slot = b;
                prev_b0 = b0;
                prev_nnz = nnz;
            } else {
                NBKD_HIP(hipMemcpyAsync(out_idx + offsets[b0], di, nnz * 4, hipMemcpyDeviceToHost, cp));
                NBKD_HIP(hipEventRecord(ev_out[b], cp));
                out_rec[b] = true;
                NBKD_HIP(hipEventSynchronize(ev_out[b]));
            }
        }
    }
    if (rc) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(cp);
        return rc;
    }
    rc = drain_prev();
    if (rc) return rc;
    NBKD_HIP(hipStreamSynchronize(s));
    NBKD_HIP(hipStreamSynchronize(cp));
    return NBKD_OK;
}

} // namespace nbkd
