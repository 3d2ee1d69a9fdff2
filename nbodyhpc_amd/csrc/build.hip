// GPU tree builder for gfx950.
//
// Produces the reference's node table (KDTreeBuilder::build_node,
// kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:98-146) on the device:
//   * leaf iff count <= max(leaf_size, 16)     (kdtree_impl.hpp:101-104)
//   * m = (count / 2) / 8 * 8; split = m-th order statistic of the
//     segment's coordinate on axis depth % 3    (kdtree_impl.hpp:107-116)
//     (Tree::axes; a tree built with nbkd_build_ext splits the axis of
//     largest remaining extent instead: slab trees, not the reference's)
//   * preorder ids, left child = id + 1, right = id + 1 + |left subtree|
// The tree SHAPE is a pure function of (n8, leaf); only the split VALUES and
// the point permutation depend on the data.  The shape (ids, segment ranges)
// is enumerated on the host down to segments of SMALL points (~2 n / SMALL
// records), the order statistics are found on the GPU:
//
//   large levels (segment > SMALL points), one launch sequence per depth:
//     4 x { hist (tiles of 4096 keys -> per-segment 256-bin histograms, LDS
//           then global atomics) ; select (one block per segment picks the
//           digit holding rank m) }            -> exact m-th key = split
//     count (per tile #<, #== pivot) ; scan (per segment over tiles) ;
//     scatter (stable three-way partition, ballot/mbcnt ranks, SoA
//           ping-pong A <-> B)
//   small segments (<= SMALL points): one workgroup loads the segment into
//     LDS (SoA, 2 x 32 KB) and finishes the whole subtree there, level by
//     level, one wave per sub-segment (wave radix select + ballot partition),
//     writing nodes and the final tree-ordered points to buffer A.
//
// Memory: SoA float x,y,z + uint32 original index = 16 B/point, two copies.
#include <algorithm>
#include <map>

#include "internal.hpp"

namespace nbkd {
namespace {

constexpr int TB = 256;              // threads per block
constexpr int TILE = 4096;           // keys per tile in large-level passes
constexpr int PER_T = TILE / TB;     // 16 keys per thread
constexpr int SMALL = 2048;          // segments <= SMALL points finish in LDS
constexpr int MAX_SUB = SMALL / 8;   // max sub-segments per level inside a block

struct LSeg {
    uint32_t node, left, count, m;
    uint32_t lchild, rchild, tile_begin, tile_end;
};
struct Tile {
    uint32_t seg, begin, count, pad;
};
struct SelState {
    uint32_t prefix, rank, below, eq;
};
struct SSeg {
    uint32_t node, left, count, depth; // source buffer: B at odd depths
};
struct SubSeg {
    uint32_t node, off, count, depth; // split axis axis_at(axes, depth)
};

struct Soa {
    float *x, *y, *z;
    uint32_t *i;
};

__device__ __forceinline__ float pick(int dim, float x, float y, float z) {
    return dim == 0 ? x : (dim == 1 ? y : z);
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ prepare
// pybind.cpp:14-56: AoS -> SoA, periodic range check, FLT_MAX padding, iota.
__global__ void __launch_bounds__(TB)
prepare_kernel(const float *__restrict__ aos, uint64_t n, uint64_t n8, int periodic, float L,
               Soa out, uint32_t *bad) {
    uint32_t flag = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)TB + threadIdx.x; i < n8;
         i += (uint64_t)gridDim.x * TB) {
        float px = FLT_MAX, py = FLT_MAX, pz = FLT_MAX;
        if (i < n) {
            px = aos[3 * i];
            py = aos[3 * i + 1];
            pz = aos[3 * i + 2];
            if (periodic && !(px >= 0.0f && px <= L && py >= 0.0f && py <= L && pz >= 0.0f &&
                              pz <= L))
                flag = 1;
        }
        out.x[i] = px;
        out.y[i] = py;
        out.z[i] = pz;
        out.i[i] = (uint32_t)i;
    }
    if (__any(flag) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

// ------------------------------------------------------------------ large levels
// One block per run of `per` consecutive tiles of the level (a segment's
// tiles are consecutive): the tile records and segment state are scalar
// loads, the LDS histogram is flushed to the segment's global one only when
// the run moves to another segment.  One tile per block made the top levels
// (1-8 segments, 24 k tiles adding into the same 256 words) atomic-bound:
// hist<1> 468 us at depth 0 vs 140 at depth 12 (r02bk trace).
template <int PASS>
__global__ void __launch_bounds__(TB)
hist_kernel(const Tile *__restrict__ tiles, const LSeg *__restrict__ segs,
            const SelState *__restrict__ st, const float *__restrict__ key_src,
            uint32_t *__restrict__ hist, uint32_t ntile, uint32_t per) {
    __shared__ uint32_t h[256];
    const uint32_t t0 = blockIdx.x * per, t1 = min(t0 + per, ntile);
    h[threadIdx.x] = 0;
    uint32_t cur = t0 < t1 ? tiles[t0].seg : 0u;
    __syncthreads();
    constexpr int shift = 24 - 8 * PASS;
    for (uint32_t t = t0; t < t1; ++t) {
        const Tile tl = tiles[t];
        if (tl.seg != cur) {
            __syncthreads();
            const uint32_t c = h[threadIdx.x];
            if (c) atomicAdd(&hist[(size_t)cur * 256 + threadIdx.x], c);
            h[threadIdx.x] = 0;
            cur = tl.seg;
            __syncthreads();
        }
        const LSeg sg = segs[tl.seg];
        const uint32_t prefix = PASS > 0 ? st[tl.seg].prefix : 0u;
        // 16-B loads (segments start at multiples of 8 points and hold
        // multiples of 8, so a float4 never straddles a tile's end); the key
        // order inside a tile does not matter to a histogram
        const float4 *src4 = reinterpret_cast<const float4 *>(key_src + sg.left + tl.begin);
        float4 v[PER_T / 4];
#pragma unroll
        for (int r = 0; r < PER_T / 4; ++r) {
            const uint32_t e4 = r * TB + threadIdx.x;
            v[r] = 4 * e4 < tl.count ? src4[e4] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
#pragma unroll
        for (int r = 0; r < PER_T; ++r) {
            const uint32_t e = 4 * ((r / 4) * TB + threadIdx.x) + (r % 4);
            const float4 q = v[r / 4];
            const float f = r % 4 == 0 ? q.x : r % 4 == 1 ? q.y : r % 4 == 2 ? q.z : q.w;
            const uint32_t k = e < tl.count ? fkey(f) : 0u;
            const bool in = e < tl.count && ((uint64_t)k >> (shift + 8)) == prefix;
            const uint32_t dg = (k >> shift) & 255u;
            if constexpr (PASS > 0) {
                if (in) atomicAdd(&h[dg], 1u);
                continue;
            }
            // pass 0 (sign + 7 exponent bits: a segment's keys share one to
            // three digits, and same-address LDS atomics serialise): the
            // wave's first two digits take one atomic each, other keys one per
            // lane.  1e8, 16 levels: 3.2 ms with per-lane atomics, 2.4 with the
            // first digit aggregated, 2.0 with two (r02bk, r02br, r02bs).
            const uint64_t im = __ballot(in);
            if (im == 0) continue;
            const int l0 = __builtin_ctzll(im);
            const uint32_t d0 = __builtin_amdgcn_readlane(dg, l0);
            const uint64_t m0 = __ballot(in && dg == d0);
            const uint64_t r0 = im & ~m0;
            const int lane = threadIdx.x & 63;
            if (lane == l0) atomicAdd(&h[d0], (uint32_t)__popcll(m0));
            if (r0 == 0) continue;
            const int l1 = __builtin_ctzll(r0);
            const uint32_t d1 = __builtin_amdgcn_readlane(dg, l1);
            const uint64_t m1 = __ballot(in && dg == d1);
            if (lane == l1) atomicAdd(&h[d1], (uint32_t)__popcll(m1));
            if (((r0 & ~m1) >> lane) & 1u) atomicAdd(&h[dg], 1u);
        }
    }
    __syncthreads();
    const uint32_t c = h[threadIdx.x];
    if (c && t0 < t1) atomicAdd(&hist[(size_t)cur * 256 + threadIdx.x], c);
}

// block-wide exclusive scan of one value per thread (TB threads)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *sh, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int w = 0; w < TB / 64; ++w) {
        uint32_t s = sh[w];
        if (w < wave) base += s;
        tot += s;
    }
    if (total) *total = tot;
    __syncthreads();
    return base + x - v;
}

template <int PASS>
__global__ void __launch_bounds__(TB)
select_kernel(const LSeg *__restrict__ segs, SelState *__restrict__ st,
              const uint32_t *__restrict__ hist, nbkd_node *__restrict__ nodes, int dim) {
    __shared__ uint32_t sh[TB / 64];
    const uint32_t seg = blockIdx.x;
    const uint32_t c = hist[(size_t)seg * 256 + threadIdx.x];
    // read the state before the scan's barriers: the selecting thread rewrites it
    const SelState s0 = PASS == 0 ? SelState{0u, segs[seg].m, 0u, 0u} : st[seg];
    const uint32_t ex = block_excl_scan(c, sh, nullptr);
    if (s0.rank >= ex && s0.rank < ex + c) {
        SelState s;
        s.prefix = (s0.prefix << 8) | threadIdx.x;
        s.rank = s0.rank - ex;
        s.below = s0.below + ex;
        s.eq = c;
        st[seg] = s;
        if (PASS == 3) {
            const LSeg sg = segs[seg];
            nodes[sg.node] = nbkd_node{dim, fkey_inv(s.prefix), sg.lchild, sg.rchild};
        }
    }
}

// per tile #< and #== pivot, over runs of `per` tiles as hist_kernel
__global__ void __launch_bounds__(TB)
count_kernel(const Tile *__restrict__ tiles, const LSeg *__restrict__ segs,
             const SelState *__restrict__ st, const float *__restrict__ key_src,
             uint2 *__restrict__ tile_cnt, uint32_t ntile, uint32_t per) {
    __shared__ uint32_t sh[TB / 64];
    const uint32_t t0 = blockIdx.x * per, t1 = min(t0 + per, ntile);
    for (uint32_t t = t0; t < t1; ++t) {
        const Tile tl = tiles[t];
        const LSeg sg = segs[tl.seg];
        const uint32_t piv = st[tl.seg].prefix;
        const float4 *src4 = reinterpret_cast<const float4 *>(key_src + sg.left + tl.begin);
        uint32_t lt = 0, eq = 0;
#pragma unroll
        for (int r = 0; r < PER_T / 4; ++r) {
            const uint32_t e4 = r * TB + threadIdx.x;
            if (4 * e4 < tl.count) {
                const float4 q = src4[e4];
                const uint32_t k[4] = {fkey(q.x), fkey(q.y), fkey(q.z), fkey(q.w)};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    lt += k[u] < piv;
                    eq += k[u] == piv;
                }
            }
        }
        uint32_t tlt, teq;
        block_excl_scan(lt, sh, &tlt);
        block_excl_scan(eq, sh, &teq);
        if (threadIdx.x == 0) tile_cnt[t] = make_uint2(tlt, teq);
    }
}

// one block per segment: exclusive prefix of (lt, eq) over its tiles
__global__ void __launch_bounds__(TB)
scan_kernel(const LSeg *__restrict__ segs, const uint2 *__restrict__ tile_cnt,
            uint2 *__restrict__ tile_off, uint32_t tile_base) {
    __shared__ uint32_t sh[TB / 64];
    const LSeg sg = segs[blockIdx.x];
    const uint32_t b = sg.tile_begin - tile_base, e = sg.tile_end - tile_base;
    const uint32_t nt = e - b;
    const uint32_t per = (nt + TB - 1) / TB;
    const uint32_t t0 = b + threadIdx.x * per;
    const uint32_t t1 = min(t0 + per, e);
    uint32_t lt = 0, eq = 0;
    for (uint32_t t = t0; t < t1; ++t) {
        uint2 c = tile_cnt[t];
        lt += c.x;
        eq += c.y;
    }
    uint32_t blt = block_excl_scan(lt, sh, nullptr);
    uint32_t beq = block_excl_scan(eq, sh, nullptr);
    for (uint32_t t = t0; t < t1; ++t) {
        tile_off[t] = make_uint2(blt, beq);
        uint2 c = tile_cnt[t];
        blt += c.x;
        beq += c.y;
    }
}

// stable three-way partition of one tile into dst
__global__ void __launch_bounds__(TB)
scatter_kernel(const Tile *__restrict__ tiles, const LSeg *__restrict__ segs,
               const SelState *__restrict__ st, const uint2 *__restrict__ tile_off, int dim,
               Soa src, Soa dst) {
    __shared__ uint32_t cnt[PER_T][TB / 64][3];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const Tile tl = tiles[blockIdx.x];
    const LSeg sg = segs[tl.seg];
    const SelState s = st[tl.seg];
    const uint32_t piv = s.prefix;
    const uint2 off = tile_off[blockIdx.x];
    const uint32_t base = sg.left + tl.begin;

    float vx[PER_T], vy[PER_T], vz[PER_T];
    uint32_t vi[PER_T];
    uint32_t cls[PER_T];
#pragma unroll
    for (int r = 0; r < PER_T; ++r) {
        uint32_t e = r * TB + threadIdx.x;
        bool valid = e < tl.count;
        uint32_t c = 3;
        if (valid) {
            vx[r] = src.x[base + e];
            vy[r] = src.y[base + e];
            vz[r] = src.z[base + e];
            vi[r] = src.i[base + e];
            uint32_t k = fkey(pick(dim, vx[r], vy[r], vz[r]));
            c = k < piv ? 0u : (k == piv ? 1u : 2u);
        }
        cls[r] = c;
        uint64_t b0 = __ballot(c == 0), b1 = __ballot(c == 1), b2 = __ballot(c == 2);
        if (lane == 0) {
            cnt[r][wave][0] = __popcll(b0);
            cnt[r][wave][1] = __popcll(b1);
            cnt[r][wave][2] = __popcll(b2);
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint32_t acc = 0;
        for (int r = 0; r < PER_T; ++r)
            for (int w = 0; w < TB / 64; ++w) {
                uint32_t v = cnt[r][w][threadIdx.x];
                cnt[r][w][threadIdx.x] = acc;
                acc += v;
            }
    }
    __syncthreads();
    const uint32_t need = sg.m - s.below; // equal keys that go left
    const uint32_t gt_prev = tl.begin - off.x - off.y;
#pragma unroll
    for (int r = 0; r < PER_T; ++r) {
        uint32_t c = cls[r];
        uint64_t b0 = __ballot(c == 0), b1 = __ballot(c == 1), b2 = __ballot(c == 2);
        if (c < 3) {
            uint64_t mine = c == 0 ? b0 : (c == 1 ? b1 : b2);
            uint32_t rk = cnt[r][wave][c] + mbcnt64(mine);
            uint32_t d;
            if (c == 0) {
                d = sg.left + off.x + rk;
            } else if (c == 1) {
                uint32_t er = off.y + rk;
                d = er < need ? sg.left + s.below + er : sg.left + sg.m + (er - need);
            } else {
                d = sg.left + sg.m + (s.eq - need) + gt_prev + rk;
            }
            dst.x[d] = vx[r];
            dst.y[d] = vy[r];
            dst.z[d] = vz[r];
            dst.i[d] = vi[r];
        }
    }
}

// ------------------------------------------------------------------ cell boxes
// Per node: the root box cut by the splits on its path (what the packet walk
// carries in bx when it reaches the node).  One thread per node descends from
// the root; in preorder the left subtree of c is [c + 1, right(c)).
__global__ void __launch_bounds__(TB)
cellbox_kernel(const nbkd_node *__restrict__ nodes, uint64_t nnodes, float lo0, float hi0,
               float *__restrict__ nbox) {
    for (uint64_t i = blockIdx.x * (uint64_t)TB + threadIdx.x; i < nnodes;
         i += (uint64_t)gridDim.x * TB) {
        float b[6] = {lo0, hi0, lo0, hi0, lo0, hi0};
        uint32_t c = 0;
        while (c != (uint32_t)i) {
            const nbkd_node nd = nodes[c];
            if (nd.dimension < 0) break; // not reached for a valid id
            if ((uint32_t)i < nd.right) {
                b[2 * nd.dimension + 1] = nd.split;
                c = c + 1;
            } else {
                b[2 * nd.dimension] = nd.split;
                c = nd.right;
            }
        }
        float4 *o = reinterpret_cast<float4 *>(nbox + 8 * i);
        o[0] = make_float4(b[0], b[1], b[2], b[3]);
        o[1] = make_float4(b[4], b[5], 0.0f, 0.0f);
    }
}

// ------------------------------------------------------------------ small segments
__device__ __forceinline__ uint32_t subtree_nodes(uint32_t count, uint32_t leaf,
                                                  const uint32_t *__restrict__ tab_c,
                                                  const uint32_t *__restrict__ tab_n, int tab_len) {
    if (count <= leaf) return 1u;
    int lo = 0, hi = tab_len - 1;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (tab_c[mid] < count)
            lo = mid + 1;
        else
            hi = mid;
    }
    return tab_n[lo];
}

struct SmallLds {
    float x[2][SMALL];
    float y[2][SMALL];
    float z[2][SMALL];
    uint32_t i[2][SMALL];
    uint32_t hist[TB / 64][256];
    SubSeg list[2][MAX_SUB];
    uint32_t nlist[2];
    uint32_t tsel[2][4];       // team split: per team, the pass's digit / before / eq count
    uint32_t tcnt[TB / 64][4]; // team split: per wave, its chunk's < / == / > counts
};

// A level with one or two sub-segments (the first two levels of a block):
// each is split by a team of TS = 4 or 2 waves instead of one wave while the
// others idle.  Team-wide radix select (shared LDS histogram, the team's first
// wave picks the digit) and a stable partition in which wave wt of the team
// takes the contiguous chunk wt of the sub-segment after an exclusive count
// over the team's earlier chunks.  Every wave reaches the same barriers (a
// team whose sub-segment is a leaf only copies it out), and the result equals
// the one-wave path's: the same order statistic, the same stable order.
template <int TS>
__device__ void team_level(SmallLds &L, const SSeg &sg, uint32_t leaf, Soa out,
                           nbkd_node *__restrict__ nodes, const uint32_t *__restrict__ tab_c,
                           const uint32_t *__restrict__ tab_n, int tab_len, int cur, int lc,
                           uint64_t axes) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t s = (uint32_t)wave / TS, wt = (uint32_t)wave % TS;
    const SubSeg ss = L.list[lc][s];
    const uint32_t sdim = (uint32_t)axis_at(axes, (int)ss.depth);
    const bool work = ss.count > leaf;
    const uint32_t tl = wt * 64 + lane; // thread within the team
    if (!work) {
        if (tl == 0)
            nodes[ss.node] = nbkd_node{-1, 0.0f, sg.left + ss.off, sg.left + ss.off + ss.count};
        for (uint32_t e = tl; e < ss.count; e += 64 * TS) {
            const uint32_t g = sg.left + ss.off + e;
            out.x[g] = L.x[cur][ss.off + e];
            out.y[g] = L.y[cur][ss.off + e];
            out.z[g] = L.z[cur][ss.off + e];
            out.i[g] = L.i[cur][ss.off + e];
        }
    }
    const float *kx = sdim == 0 ? L.x[cur] : (sdim == 1 ? L.y[cur] : L.z[cur]);
    const uint32_t m = (ss.count / 2) / 8 * 8;
    uint32_t rank = m, prefix = 0, below = 0, eqc = 0;
    uint32_t *h = L.hist[s * TS];
#pragma unroll 1
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        for (uint32_t b = tl; b < 256; b += 64 * TS) h[b] = 0;
        __syncthreads();
        if (work) {
            if (pass == 0) {
                // first two digits of the wave aggregated, as small_kernel's pass 0
                for (uint32_t e0 = wt * 64; e0 < ss.count; e0 += 64 * TS) {
                    const uint32_t e = e0 + lane;
                    const bool in = e < ss.count;
                    const uint32_t dg = in ? fkey(kx[ss.off + e]) >> 24 : 0u;
                    const uint64_t im = __ballot(in);
                    const int l0 = __builtin_ctzll(im);
                    const uint32_t d0 = __builtin_amdgcn_readlane(dg, l0);
                    const uint64_t m0 = __ballot(in && dg == d0);
                    const uint64_t r0 = im & ~m0;
                    if (lane == l0) atomicAdd(&h[d0], (uint32_t)__popcll(m0));
                    if (r0 == 0) continue;
                    const int l1 = __builtin_ctzll(r0);
                    const uint32_t d1 = __builtin_amdgcn_readlane(dg, l1);
                    const uint64_t m1 = __ballot(in && dg == d1);
                    if (lane == l1) atomicAdd(&h[d1], (uint32_t)__popcll(m1));
                    if (((r0 & ~m1) >> lane) & 1u) atomicAdd(&h[dg], 1u);
                }
            } else {
                for (uint32_t e = tl; e < ss.count; e += 64 * TS) {
                    const uint32_t k = fkey(kx[ss.off + e]);
                    if (((uint64_t)k >> (shift + 8)) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
                }
            }
        }
        __syncthreads();
        if (work && wt == 0) {
            const uint32_t c0 = h[lane * 4], c1 = h[lane * 4 + 1], c2 = h[lane * 4 + 2],
                           c3 = h[lane * 4 + 3];
            const uint32_t sum = c0 + c1 + c2 + c3;
            uint32_t x = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            const uint32_t ex = x - sum;
            const bool hit = rank >= ex && rank < x;
            const int sel = __ffsll((unsigned long long)__ballot(hit)) - 1;
            const uint32_t r = rank - ex;
            uint32_t j = 0, acc = 0, cc = c0;
            if (r >= c0) {
                acc = c0;
                j = 1;
                cc = c1;
                if (r >= c0 + c1) {
                    acc = c0 + c1;
                    j = 2;
                    cc = c2;
                    if (r >= c0 + c1 + c2) {
                        acc = c0 + c1 + c2;
                        j = 3;
                        cc = c3;
                    }
                }
            }
            const uint32_t digit = 4u * (uint32_t)sel + __shfl(j, sel, 64);
            const uint32_t before = __shfl(ex + acc, sel, 64);
            const uint32_t ecnt = __shfl(cc, sel, 64);
            if (lane == 0) {
                L.tsel[s][0] = digit;
                L.tsel[s][1] = before;
                L.tsel[s][2] = ecnt;
            }
        }
        __syncthreads();
        if (work) {
            const uint32_t digit = L.tsel[s][0], before = L.tsel[s][1];
            eqc = L.tsel[s][2];
            prefix = (prefix << 8) | digit;
            below += before;
            rank -= before;
        }
    }
    const uint32_t piv = prefix, need = m - below;
    // the team's chunks: wave wt takes [wt * cw, (wt + 1) * cw), cw a multiple of 64
    const uint32_t cw = (ss.count + 64 * TS - 1) / (64 * TS) * 64;
    const uint32_t c_lo = min(wt * cw, ss.count), c_hi = min(c_lo + cw, ss.count);
    uint32_t clt = 0, ceq = 0;
    if (work) {
        for (uint32_t e0 = c_lo; e0 < c_hi; e0 += 64) {
            const uint32_t e = e0 + lane;
            const bool valid = e < c_hi;
            const uint32_t k = valid ? fkey(kx[ss.off + e]) : 0u;
            clt += (uint32_t)__popcll(__ballot(valid && k < piv));
            ceq += (uint32_t)__popcll(__ballot(valid && k == piv));
        }
        if (lane == 0) {
            L.tcnt[wave][0] = clt;
            L.tcnt[wave][1] = ceq;
        }
    }
    __syncthreads();
    if (work) {
        uint32_t nlt = 0, neq = 0, ngt = 0;
        for (uint32_t w = 0; w < wt; ++w) {
            const uint32_t a = L.tcnt[s * TS + w][0], b = L.tcnt[s * TS + w][1];
            const uint32_t n = min(cw, ss.count - min(w * cw, ss.count));
            nlt += a;
            neq += b;
            ngt += n - a - b;
        }
        for (uint32_t e0 = c_lo; e0 < c_hi; e0 += 64) {
            const uint32_t e = e0 + lane;
            const bool valid = e < c_hi;
            uint32_t c = 3;
            float px = 0, py = 0, pz = 0;
            uint32_t pi = 0;
            if (valid) {
                px = L.x[cur][ss.off + e];
                py = L.y[cur][ss.off + e];
                pz = L.z[cur][ss.off + e];
                pi = L.i[cur][ss.off + e];
                const uint32_t k = fkey(pick(sdim, px, py, pz));
                c = k < piv ? 0u : (k == piv ? 1u : 2u);
            }
            const uint64_t b0 = __ballot(c == 0), b1 = __ballot(c == 1), b2 = __ballot(c == 2);
            if (valid) {
                uint32_t d;
                if (c == 0) {
                    d = nlt + mbcnt64(b0);
                } else if (c == 1) {
                    const uint32_t er = neq + mbcnt64(b1);
                    d = er < need ? below + er : m + (er - need);
                } else {
                    d = m + (eqc - need) + ngt + mbcnt64(b2);
                }
                L.x[cur ^ 1][ss.off + d] = px;
                L.y[cur ^ 1][ss.off + d] = py;
                L.z[cur ^ 1][ss.off + d] = pz;
                L.i[cur ^ 1][ss.off + d] = pi;
            }
            nlt += __popcll(b0);
            neq += __popcll(b1);
            ngt += __popcll(b2);
        }
        if (tl == 0) {
            const uint32_t rid = ss.node + 1 + subtree_nodes(m, leaf, tab_c, tab_n, tab_len);
            nodes[ss.node] = nbkd_node{(int32_t)sdim, fkey_inv(piv), ss.node + 1, rid};
            const uint32_t slot = atomicAdd(&L.nlist[lc ^ 1], 2u);
            L.list[lc ^ 1][slot] = SubSeg{ss.node + 1, ss.off, m, ss.depth + 1};
            L.list[lc ^ 1][slot + 1] = SubSeg{rid, ss.off + m, ss.count - m, ss.depth + 1};
        }
    }
}

__global__ void __launch_bounds__(TB)
small_kernel(const SSeg *__restrict__ list, uint32_t leaf, Soa bufA, Soa bufB,
             nbkd_node *__restrict__ nodes, const uint32_t *__restrict__ tab_c,
             const uint32_t *__restrict__ tab_n, int tab_len, int team, uint64_t axes) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    SmallLds &L = *reinterpret_cast<SmallLds *>(smem_raw);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const SSeg sg = list[blockIdx.x];
    const Soa src = (sg.depth & 1u) ? bufB : bufA;
    const Soa out = bufA;

    if (sg.count > SMALL) { // a leaf larger than SMALL (leaf_size > SMALL): move it to A
        if (threadIdx.x == 0) nodes[sg.node] = nbkd_node{-1, 0.0f, sg.left, sg.left + sg.count};
        if (src.x != out.x)
            for (uint32_t e = threadIdx.x; e < sg.count; e += TB) {
                out.x[sg.left + e] = src.x[sg.left + e];
                out.y[sg.left + e] = src.y[sg.left + e];
                out.z[sg.left + e] = src.z[sg.left + e];
                out.i[sg.left + e] = src.i[sg.left + e];
            }
        return;
    }
    for (uint32_t e = threadIdx.x; e < sg.count; e += TB) {
        L.x[0][e] = src.x[sg.left + e];
        L.y[0][e] = src.y[sg.left + e];
        L.z[0][e] = src.z[sg.left + e];
        L.i[0][e] = src.i[sg.left + e];
    }
    if (threadIdx.x == 0) {
        L.list[0][0] = SubSeg{sg.node, 0u, sg.count, sg.depth};
        L.nlist[0] = 1;
        L.nlist[1] = 0;
    }
    __syncthreads();
    int cur = 0, lc = 0;
    while (L.nlist[lc] > 0) {
        const uint32_t nsub = L.nlist[lc];
        if (nsub <= 2 && team) {
            if (nsub == 1)
                team_level<4>(L, sg, leaf, out, nodes, tab_c, tab_n, tab_len, cur, lc, axes);
            else
                team_level<2>(L, sg, leaf, out, nodes, tab_c, tab_n, tab_len, cur, lc, axes);
        } else
        for (uint32_t s = wave; s < nsub; s += TB / 64) {
            const SubSeg ss = L.list[lc][s];
            const uint32_t sdim = (uint32_t)axis_at(axes, (int)ss.depth);
            if (ss.count <= leaf) {
                if (lane == 0)
                    nodes[ss.node] =
                        nbkd_node{-1, 0.0f, sg.left + ss.off, sg.left + ss.off + ss.count};
                for (uint32_t e = lane; e < ss.count; e += 64) {
                    uint32_t g = sg.left + ss.off + e;
                    out.x[g] = L.x[cur][ss.off + e];
                    out.y[g] = L.y[cur][ss.off + e];
                    out.z[g] = L.z[cur][ss.off + e];
                    out.i[g] = L.i[cur][ss.off + e];
                }
                continue;
            }
            const float *kx = sdim == 0 ? L.x[cur] : (sdim == 1 ? L.y[cur] : L.z[cur]);
            const uint32_t m = (ss.count / 2) / 8 * 8;
            // wave radix select of rank m, 4 x 8-bit digits
            uint32_t rank = m, prefix = 0, below = 0, eqc = 0;
            uint32_t *h = L.hist[wave];
#pragma unroll 1
            for (int pass = 0; pass < 4; ++pass) {
                const int shift = 24 - 8 * pass;
                for (int j = 0; j < 4; ++j) h[lane * 4 + j] = 0;
                wave_sync();
                // 64-bit shift: a 32-bit shift by 32 (pass 0) is poison in LLVM IR
                if (pass == 0) {
                    // the sign + top exponent bits: a sub-segment's keys share
                    // one to three digits; same-address LDS atomics serialise,
                    // so the wave's first two digits take one atomic each (as
                    // hist_kernel<0>)
                    for (uint32_t e0 = 0; e0 < ss.count; e0 += 64) {
                        const uint32_t e = e0 + lane;
                        const bool in = e < ss.count;
                        const uint32_t dg = in ? fkey(kx[ss.off + e]) >> 24 : 0u;
                        const uint64_t im = __ballot(in);
                        const int l0 = __builtin_ctzll(im);
                        const uint32_t d0 = __builtin_amdgcn_readlane(dg, l0);
                        const uint64_t m0 = __ballot(in && dg == d0);
                        const uint64_t r0 = im & ~m0;
                        if (lane == l0) atomicAdd(&h[d0], (uint32_t)__popcll(m0));
                        if (r0 == 0) continue;
                        const int l1 = __builtin_ctzll(r0);
                        const uint32_t d1 = __builtin_amdgcn_readlane(dg, l1);
                        const uint64_t m1 = __ballot(in && dg == d1);
                        if (lane == l1) atomicAdd(&h[d1], (uint32_t)__popcll(m1));
                        if (((r0 & ~m1) >> lane) & 1u) atomicAdd(&h[dg], 1u);
                    }
                } else {
                    for (uint32_t e = lane; e < ss.count; e += 64) {
                        uint32_t k = fkey(kx[ss.off + e]);
                        if (((uint64_t)k >> (shift + 8)) == prefix)
                            atomicAdd(&h[(k >> shift) & 255u], 1u);
                    }
                }
                wave_sync();
                uint32_t c0 = h[lane * 4], c1 = h[lane * 4 + 1], c2 = h[lane * 4 + 2],
                         c3 = h[lane * 4 + 3];
                uint32_t sum = c0 + c1 + c2 + c3, x = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    uint32_t y = __shfl_up(x, o, 64);
                    if (lane >= o) x += y;
                }
                uint32_t ex = x - sum;
                bool hit = rank >= ex && rank < x;
                uint64_t bal = __ballot(hit);
                int sel = __ffsll((unsigned long long)bal) - 1;
                uint32_t r = rank - ex, j = 0, acc = 0, cc = c0;
                if (r >= c0) {
                    acc = c0;
                    j = 1;
                    cc = c1;
                    if (r >= c0 + c1) {
                        acc = c0 + c1;
                        j = 2;
                        cc = c2;
                        if (r >= c0 + c1 + c2) {
                            acc = c0 + c1 + c2;
                            j = 3;
                            cc = c3;
                        }
                    }
                }
                uint32_t digit = 4u * (uint32_t)sel + __shfl(j, sel, 64);
                uint32_t before = __shfl(ex + acc, sel, 64);
                eqc = __shfl(cc, sel, 64);
#ifdef NBKD_DEBUG
                if (blockIdx.x == 0 && lane == 0 && ss.node < 2)
                    printf("node %u cnt %u m %u pass %d sel %d digit %u before %u eqc %u tot %u rank %u\n",
                           ss.node, ss.count, m, pass, sel, digit, before, eqc, __shfl(x, 63, 64), rank);
#endif
                prefix = (prefix << 8) | digit;
                below += before;
                rank -= before;
                wave_sync();
            }
            const uint32_t piv = prefix, need = m - below;
            // stable three-way partition into the other buffer
            uint32_t nlt = 0, neq = 0, ngt = 0;
            for (uint32_t e0 = 0; e0 < ss.count; e0 += 64) {
                uint32_t e = e0 + lane;
                bool valid = e < ss.count;
                uint32_t c = 3;
                float px = 0, py = 0, pz = 0;
                uint32_t pi = 0;
                if (valid) {
                    px = L.x[cur][ss.off + e];
                    py = L.y[cur][ss.off + e];
                    pz = L.z[cur][ss.off + e];
                    pi = L.i[cur][ss.off + e];
                    uint32_t k = fkey(pick(sdim, px, py, pz));
                    c = k < piv ? 0u : (k == piv ? 1u : 2u);
                }
                uint64_t b0 = __ballot(c == 0), b1 = __ballot(c == 1), b2 = __ballot(c == 2);
                if (valid) {
                    uint32_t d;
                    if (c == 0) {
                        d = nlt + mbcnt64(b0);
                    } else if (c == 1) {
                        uint32_t er = neq + mbcnt64(b1);
                        d = er < need ? below + er : m + (er - need);
                    } else {
                        d = m + (eqc - need) + ngt + mbcnt64(b2);
                    }
                    L.x[cur ^ 1][ss.off + d] = px;
                    L.y[cur ^ 1][ss.off + d] = py;
                    L.z[cur ^ 1][ss.off + d] = pz;
                    L.i[cur ^ 1][ss.off + d] = pi;
                }
                nlt += __popcll(b0);
                neq += __popcll(b1);
                ngt += __popcll(b2);
            }
            const uint32_t rid = ss.node + 1 + subtree_nodes(m, leaf, tab_c, tab_n, tab_len);
            if (lane == 0) {
                nodes[ss.node] = nbkd_node{(int32_t)sdim, fkey_inv(piv), ss.node + 1, rid};
                uint32_t slot = atomicAdd(&L.nlist[lc ^ 1], 2u);
                L.list[lc ^ 1][slot] = SubSeg{ss.node + 1, ss.off, m, ss.depth + 1};
                L.list[lc ^ 1][slot + 1] = SubSeg{rid, ss.off + m, ss.count - m, ss.depth + 1};
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) L.nlist[lc] = 0;
        cur ^= 1;
        lc ^= 1;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(TB)
extract_splits_kernel(const nbkd_node *__restrict__ nodes, uint64_t nn, float *__restrict__ splits) {
    for (uint64_t i = blockIdx.x * (uint64_t)TB + threadIdx.x; i < nn; i += (uint64_t)gridDim.x * TB)
        splits[i] = nodes[i].split;
}

// Per-leaf record for the streaming kNN kernel (8 words per node id, leaves
// only): the tight bounding box of the leaf's real points (padding rows,
// idx >= n, excluded) and its point range.  A tight box is a valid (and
// better) pruning bound than the split-plane box: every point of the leaf
// lies inside it.
__global__ void __launch_bounds__(TB)
leafinfo_kernel(const nbkd_node *__restrict__ nodes, uint64_t nn, const float *__restrict__ x,
                const float *__restrict__ y, const float *__restrict__ z,
                const uint32_t *__restrict__ idx, uint64_t n, uint32_t *__restrict__ info,
                uint32_t *__restrict__ bbox) {
    // bbox[0..6): data bounding box keys; bbox[6]: number of leaves holding
    // padding, bbox[7..7+NBKD_PAD_LEAVES): their node ids
    float blo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint64_t i = blockIdx.x * (uint64_t)TB + threadIdx.x; i < nn; i += (uint64_t)gridDim.x * TB) {
        const nbkd_node nd = nodes[i];
        if (nd.dimension >= 0) continue;
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        bool pad = false;
        for (uint32_t j = nd.left; j < nd.right; ++j) {
            if (idx[j] >= n) {
                pad = true;
                continue;
            }
            const float p[3] = {x[j], y[j], z[j]};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(lo[a], p[a]);
                hi[a] = fmaxf(hi[a], p[a]);
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            blo[a] = fminf(blo[a], lo[a]);
            bhi[a] = fmaxf(bhi[a], hi[a]);
        }
        if (pad && bbox) {
            const uint32_t slot = atomicAdd(&bbox[6], 1u);
            if (slot < (uint32_t)NBKD_PAD_LEAVES) bbox[7 + slot] = (uint32_t)i;
        }
        uint32_t *o = info + 8 * i;
        const float4 w0 = make_float4(lo[0], lo[1], lo[2], hi[0]);
        const float4 w1 = make_float4(hi[1], hi[2], __uint_as_float(nd.left), __uint_as_float(nd.right));
        reinterpret_cast<float4 *>(o)[0] = w0;
        reinterpret_cast<float4 *>(o)[1] = w1;
    }
    // data bounding box (order-preserving keys; the seed radius of non-periodic
    // queries needs finite subtree volumes): reduced over the wave first, so one
    // lane per wave issues the atomics
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            blo[a] = fminf(blo[a], __shfl_xor(blo[a], o, 64));
            bhi[a] = fmaxf(bhi[a], __shfl_xor(bhi[a], o, 64));
        }
    }
    if (bbox && (threadIdx.x & 63) == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (blo[a] <= bhi[a]) {
                atomicMin(&bbox[a], fkey(blo[a]));
                atomicMax(&bbox[3 + a], fkey(bhi[a]));
            }
        }
    }
}

// Sub-leaf groups (internal.hpp Tree::ginfo).  One wave per leaf, up to
// GPL points per lane, per run of NBKD_GBLOCK positions: the run is cut
// recursively like the tree itself (m = floor(count / 2 / 8) * 8, so every
// piece is a multiple of 8) but on the widest axis of the piece's real points,
// each piece ordered by (coordinate, position), until pieces hold NBKD_GROUP
// points; then each group's tight box is written.  Only the order inside a
// leaf changes: leaf membership, the node table and every query result stay
// the same (the kNN parity contract compares leaves and tie groups as sets),
// and padding rows (FLT_MAX) sort last and are left out of the boxes.
// GPL points per lane: NBKD_GBLOCK / 64 = 2, or 1 when no leaf exceeds 64
// points (leafsize <= 64: half the registers, no idle second point per lane)

//
// The same pass writes leafinfo (8 words per leaf: its tight box, the union of
// its group boxes, and its point range), lists the leaves holding padding and
// reduces the data bounding box (bbox as in leafinfo_kernel, which it replaces
// whenever there are points: one lane per leaf there read 64 scattered points).
template <int GPL>
__global__ void __launch_bounds__(TB)
group_kernel(const nbkd_node *__restrict__ nodes, uint64_t nn, float *__restrict__ x,
             float *__restrict__ y, float *__restrict__ z, uint32_t *__restrict__ idx, uint64_t n,
             float *__restrict__ ginfo, float *__restrict__ hinfo, uint32_t *__restrict__ info,
             uint32_t *__restrict__ bbox) {
    constexpr int WPB = TB / 64;
    __shared__ __attribute__((aligned(16))) float sp[WPB][3][NBKD_GBLOCK];
    __shared__ __attribute__((aligned(16))) uint32_t sr[WPB][NBKD_GBLOCK];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float (*const P)[NBKD_GBLOCK] = sp[wave];
    uint32_t *const R = sr[wave];
    const uint64_t nw = (uint64_t)gridDim.x * WPB;
    float dlo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, dhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint64_t i = (uint64_t)blockIdx.x * WPB + wave; i < nn; i += nw) {
        const nbkd_node nd = nodes[i];
        if (nd.dimension >= 0) continue;
        // this lane's running union of its group boxes, and padding seen
        float llo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        bool pad = false;
        for (uint32_t b0 = nd.left; b0 < nd.right; b0 += NBKD_GBLOCK) {
            const uint32_t c = min((uint32_t)NBKD_GBLOCK, nd.right - b0);
            // point h of this lane: run position lane + 64 h
            float p[GPL][3];
            uint32_t id[GPL], real[GPL], pos[GPL], s[GPL], l[GPL], pc[GPL];
#pragma unroll
            for (int h = 0; h < GPL; ++h) {
                const uint32_t j = (uint32_t)(lane + 64 * h);
                const bool on = j < c;
                p[h][0] = on ? x[b0 + j] : FLT_MAX;
                p[h][1] = on ? y[b0 + j] : FLT_MAX;
                p[h][2] = on ? z[b0 + j] : FLT_MAX;
                id[h] = on ? idx[b0 + j] : 0xFFFFFFFFu;
                real[h] = (on && id[h] < n) ? 1u : 0u;
                pad |= on && id[h] >= n;
                pos[h] = j;
                pc[h] = 0;
                s[h] = 0;
                l[h] = on ? c : 0u;
            }
            // the boxes of the first two cuts' pieces (the whole run, then its
            // two halves) are wave reductions over the lanes' real points of
            // each piece instead of every lane scanning its piece
            float rlo[2][3], rhi[2][3];
            auto piece_boxes = [&](int np) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (q >= np) break;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        float lo = FLT_MAX, hi = -FLT_MAX;
#pragma unroll
                        for (int h = 0; h < GPL; ++h) {
                            const bool in = real[h] && pc[h] == (uint32_t)q;
                            lo = in ? fminf(lo, p[h][a]) : lo;
                            hi = in ? fmaxf(hi, p[h][a]) : hi;
                        }
#pragma unroll
                        for (int o = 32; o > 0; o >>= 1) {
                            lo = fminf(lo, __shfl_xor(lo, o, 64));
                            hi = fmaxf(hi, __shfl_xor(hi, o, 64));
                        }
                        rlo[q][a] = lo;
                        rhi[q][a] = hi;
                    }
                }
            };
            int cut = 0;
            for (;;) {
                bool more = false;
#pragma unroll
                for (int h = 0; h < GPL; ++h) more |= l[h] > (uint32_t)NBKD_GROUP;
                if (!__any(more)) break;
#pragma unroll
                for (int h = 0; h < GPL; ++h) {
                    P[0][pos[h]] = p[h][0];
                    P[1][pos[h]] = p[h][1];
                    P[2][pos[h]] = p[h][2];
                    R[pos[h]] = real[h];
                }
                wave_sync();
                if (cut < 2) piece_boxes(cut + 1);
                uint32_t npos[GPL];
#pragma unroll
                for (int h = 0; h < GPL; ++h) {
                    npos[h] = pos[h];
                    if (l[h] <= (uint32_t)NBKD_GROUP) continue;
                    // pieces hold multiples of 8 points: both scans unrolled by 8,
                    // branch-free, so the LDS reads of an 8-run issue together
                    const uint32_t q = pc[h] & 1u;
                    float lo[3] = {q ? rlo[1][0] : rlo[0][0], q ? rlo[1][1] : rlo[0][1],
                                   q ? rlo[1][2] : rlo[0][2]};
                    float hi[3] = {q ? rhi[1][0] : rhi[0][0], q ? rhi[1][1] : rhi[0][1],
                                   q ? rhi[1][2] : rhi[0][2]};
                    if (cut >= 2) {
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            lo[a] = FLT_MAX;
                            hi[a] = -FLT_MAX;
                        }
                        for (uint32_t j0 = s[h]; j0 < s[h] + l[h]; j0 += 8) {
                            const uint4 r0 = *reinterpret_cast<const uint4 *>(&R[j0]);
                            const uint4 r1 = *reinterpret_cast<const uint4 *>(&R[j0 + 4]);
                            const uint32_t rv[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
                            for (int a = 0; a < 3; ++a) {
                                const float4 v0 = *reinterpret_cast<const float4 *>(&P[a][j0]);
                                const float4 v1 = *reinterpret_cast<const float4 *>(&P[a][j0 + 4]);
                                const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                                for (uint32_t u = 0; u < 8; ++u) {
                                    lo[a] = rv[u] ? fminf(lo[a], vv[u]) : lo[a];
                                    hi[a] = rv[u] ? fmaxf(hi[a], vv[u]) : hi[a];
                                }
                            }
                        }
                    }
                    const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
                    const int ax = (ey > ex && ey >= ez) ? 1 : (ez > ex && ez > ey ? 2 : 0);
                    const float key = p[h][ax];
                    uint32_t rank = 0;
                    // pieces start at multiples of 8: two 16-B LDS reads per 8 keys
                    for (uint32_t j0 = s[h]; j0 < s[h] + l[h]; j0 += 8) {
                        const float4 k0 = *reinterpret_cast<const float4 *>(&P[ax][j0]);
                        const float4 k1 = *reinterpret_cast<const float4 *>(&P[ax][j0 + 4]);
                        const float kv[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
                        for (uint32_t u = 0; u < 8; ++u) {
                            const uint32_t j = j0 + u;
                            rank += (kv[u] < key || (kv[u] == key && j < pos[h])) ? 1u : 0u;
                        }
                    }
                    const uint32_t m = (l[h] / 2) / 8 * 8;
                    npos[h] = s[h] + rank;
                    pc[h] = 2 * pc[h] + (rank < m ? 0u : 1u);
                    if (rank < m) {
                        l[h] = m;
                    } else {
                        s[h] += m;
                        l[h] -= m;
                    }
                }
                wave_sync();
#pragma unroll
                for (int h = 0; h < GPL; ++h) pos[h] = npos[h];
                ++cut;
            }
#pragma unroll
            for (int h = 0; h < GPL; ++h) {
                if ((uint32_t)(lane + 64 * h) < c) {
                    x[b0 + pos[h]] = p[h][0];
                    y[b0 + pos[h]] = p[h][1];
                    z[b0 + pos[h]] = p[h][2];
                    idx[b0 + pos[h]] = id[h];
                }
                P[0][pos[h]] = p[h][0];
                P[1][pos[h]] = p[h][1];
                P[2][pos[h]] = p[h][2];
                R[pos[h]] = real[h];
            }
            wave_sync();
            if ((uint32_t)lane < c / NBKD_GROUP) {
                float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                for (int j = lane * NBKD_GROUP; j < (lane + 1) * NBKD_GROUP; ++j) {
                    if (!R[j]) continue;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = fminf(lo[a], P[a][j]);
                        hi[a] = fmaxf(hi[a], P[a][j]);
                    }
                }
                float *o = ginfo + 6 * ((size_t)(b0 / NBKD_GROUP) + lane);
                o[0] = lo[0];
                o[1] = hi[0];
                o[2] = lo[1];
                o[3] = hi[1];
                o[4] = lo[2];
                o[5] = hi[2];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    llo[a] = fminf(llo[a], lo[a]);
                    lhi[a] = fmaxf(lhi[a], hi[a]);
                }
            }
            // a leaf of 65..128 points: the tight boxes of its two halves (the
            // first cut above, at m), the kNN collect kernel's staging chunks
            const uint32_t cnt_leaf = nd.right - nd.left;
            if (hinfo && b0 == nd.left && cnt_leaf > 64 && cnt_leaf <= NBKD_GBLOCK && lane < 2) {
                const uint32_t m = (c / 2) / 8 * 8;
                const uint32_t j0 = lane == 0 ? 0u : m, j1 = lane == 0 ? m : c;
                float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                for (uint32_t j = j0; j < j1; ++j) {
                    if (!R[j]) continue;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = fminf(lo[a], P[a][j]);
                        hi[a] = fmaxf(hi[a], P[a][j]);
                    }
                }
                float *o = hinfo + 12 * (size_t)i + 6 * lane; // leafinfo's word order
                o[0] = lo[0];
                o[1] = lo[1];
                o[2] = lo[2];
                o[3] = hi[0];
                o[4] = hi[1];
                o[5] = hi[2];
            }
            wave_sync();
        }
        // leafinfo of leaf i: the union of the lanes' group-box unions
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                llo[a] = fminf(llo[a], __shfl_xor(llo[a], o, 64));
                lhi[a] = fmaxf(lhi[a], __shfl_xor(lhi[a], o, 64));
            }
        }
        const bool any_pad = __any(pad);
        if (lane == 0) {
            float4 *o = reinterpret_cast<float4 *>(info + 8 * i);
            o[0] = make_float4(llo[0], llo[1], llo[2], lhi[0]);
            o[1] = make_float4(lhi[1], lhi[2], __uint_as_float(nd.left), __uint_as_float(nd.right));
            if (any_pad) {
                const uint32_t slot = atomicAdd(&bbox[6], 1u);
                if (slot < (uint32_t)NBKD_PAD_LEAVES) bbox[7 + slot] = (uint32_t)i;
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            dlo[a] = fminf(dlo[a], llo[a]);
            dhi[a] = fmaxf(dhi[a], lhi[a]);
        }
    }
    // data bounding box (wave-uniform already): reduced over the block, then one
    // lane per block issues the atomics (all blocks hit the same six words)
    __shared__ float sbox[WPB][6];
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            sbox[wave][a] = dlo[a];
            sbox[wave][3 + a] = dhi[a];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float lo = sbox[0][a], hi = sbox[0][3 + a];
            for (int w = 1; w < WPB; ++w) {
                lo = fminf(lo, sbox[w][a]);
                hi = fmaxf(hi, sbox[w][3 + a]);
            }
            if (lo <= hi) {
                atomicMin(&bbox[a], fkey(lo));
                atomicMax(&bbox[3 + a], fkey(hi));
            }
        }
    }
}

// Split values in heap (BFS) order for the query bucketing descent: the node
// reached by turns t_1..t_d (0 left, 1 right) has heap index h, children 2h+1 /
// 2h+2, so the descent needs neither child ids nor the shape table, and the top
// levels sit together in a few KB (cache resident).  One thread per leaf walks
// from the root and writes every ancestor whose first point is the leaf's first
// point (each internal node exactly once); preorder ids come from the shape
// table as in leaf_key2_kernel.  Stored in the 4-level blocked layout
// (internal.hpp hblk_slot): one 64-B line per 4-level subtree.
__global__ void __launch_bounds__(TB)
heap_splits_kernel(const nbkd_node *__restrict__ nodes, uint64_t nn, const float *__restrict__ splits,
                   const uint32_t *__restrict__ shape_c, const uint32_t *__restrict__ shape_n,
                   int shape_len, uint32_t n8, uint32_t leaf, int o, float *__restrict__ heap) {
    for (uint64_t i = blockIdx.x * (uint64_t)TB + threadIdx.x; i < nn; i += (uint64_t)gridDim.x * TB) {
        const nbkd_node nd = nodes[i];
        if (nd.dimension >= 0) continue;
        const uint32_t target = nd.left;
        uint32_t node = 0, left = 0, count = n8;
        uint64_t h = 0;
        while (count > leaf) {
            if (left == target) heap[hblk_slot(h, o)] = splits[node];
            const uint32_t mm = (count / 2) / 8 * 8;
            if (target >= left + mm) {
                uint32_t sub = 1;
                if (mm > leaf) {
                    int bl = 0, bh = shape_len - 1;
                    while (bl < bh) {
                        const int mid = (bl + bh) >> 1;
                        if (shape_c[mid] < mm)
                            bl = mid + 1;
                        else
                            bh = mid;
                    }
                    sub = shape_n[bl];
                }
                node += 1 + sub;
                left += mm;
                count -= mm;
                h = 2 * h + 2;
            } else {
                node += 1;
                count = mm;
                h = 2 * h + 1;
            }
        }
    }
}

// ------------------------------------------------------------------ host side
struct Skeleton {
    std::map<uint64_t, uint32_t> memo; // count -> subtree node count
    std::map<uint64_t, int> dmemo;     // count -> subtree depth
    uint32_t leaf;
    int max_depth = 0;
    std::vector<std::vector<LSeg>> levels;
    std::vector<SSeg> small;

    uint32_t nodes(uint64_t c) {
        if (c <= leaf) return 1;
        auto it = memo.find(c);
        if (it != memo.end()) return it->second;
        uint64_t m = (c / 2) / 8 * 8;
        uint64_t r = 1 + (uint64_t)nodes(m) + nodes(c - m);
        memo[c] = (uint32_t)r;
        return (uint32_t)r;
    }
    int depth_of(uint64_t c) {
        if (c <= leaf) return 0;
        auto it = dmemo.find(c);
        if (it != dmemo.end()) return it->second;
        uint64_t m = (c / 2) / 8 * 8;
        int d = 1 + std::max(depth_of(m), depth_of(c - m));
        dmemo[c] = d;
        return d;
    }
    void rec(uint32_t node, uint32_t left, uint32_t count, int depth) {
        if (count <= SMALL || count <= leaf) {
            small.push_back(SSeg{node, left, count, (uint32_t)depth});
            return;
        }
        uint32_t m = (count / 2) / 8 * 8;
        uint32_t l = node + 1, r = node + 1 + nodes(m);
        if ((int)levels.size() <= depth) levels.resize(depth + 1);
        levels[depth].push_back(LSeg{node, left, count, m, l, r, 0, 0});
        rec(l, left, m, depth + 1);
        rec(r, left + m, count - m, depth + 1);
    }
};

} // namespace

namespace {

// Build scratch (the B ping-pong copy of the points, the level tables, the
// input staging copy): one device buffer per device, kept between builds and
// grown on demand, carved into 256-B aligned pieces.  A build holds its
// device's lock until it has synchronised its stream, so builds on one device
// never share the buffer while kernels use it.  Per build this saves ~15
// hipMalloc/hipFree pairs, four of them n * 4 bytes (r02ce).
struct LevelInfo {
    uint32_t seg0, nseg, tile0, ntile;
};
// The tree's shape (segments, tiles, small subtrees, the count -> node-count
// table) is a pure function of (n8, leaf): rebuilding a tree of the same size
// (a simulation's every step) reuses the host tables and their device copies.
// Enumerating them took ~3.4 ms of host time before the first kernel at 1e8.
struct ShapeTables {
    bool valid = false, uploaded = false;
    uint64_t n8 = 0;
    uint32_t leaf = 0;
    std::vector<LSeg> segs;
    std::vector<Tile> tiles;
    std::vector<LevelInfo> info;
    std::vector<SSeg> small;
    std::vector<uint32_t> tab_c, tab_n;
    size_t max_seg = 0, max_tile = 0;
};
struct BuildScratch {
    std::mutex mu;
    void *p = nullptr;
    size_t bytes = 0;
    ShapeTables shape;
};
BuildScratch &build_scratch(int dev) {
    static BuildScratch pool[64];
    return pool[dev & 63];
}

} // namespace

void release_idle_build_scratch(int dev) {
    BuildScratch &b = build_scratch(dev);
    if (held_here(&b) || !b.mu.try_lock()) return;
    // unlocked scratch has no kernel in flight (the lock outlives the stream)
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    b.shape.uploaded = false;
    b.mu.unlock();
}

namespace {

struct Carve {
    size_t off = 0;
    size_t take(size_t b) {
        const size_t o = off;
        off += (std::max<size_t>(b, 16) + 255) / 256 * 256;
        return o;
    }
};

} // namespace

// the points packed per tree position, after group_kernel's final order
__global__ void __launch_bounds__(256)
pack4_kernel(const float *__restrict__ x, const float *__restrict__ y, const float *__restrict__ z,
             const uint32_t *__restrict__ idx, uint64_t n8, float4 *__restrict__ p4) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * 256)
        p4[i] = make_float4(x[i], y[i], z[i], __uint_as_float(idx[i]));
}

nbkd_status build_tree(Tree &t, const float *xyz, uint64_t n, int32_t leaf_size, bool input_dev,
                       hipStream_t s) {
    const uint64_t n8 = (n + 7) / 8 * 8;
    if (n8 > (uint64_t)UINT32_MAX) {
        set_error("More than uint32_t points are not supported.");
        return NBKD_ETOOMANY;
    }
    // leaf_size_ = max(leaf_size, 2 * block_size): size_t comparison, so a
    // negative int becomes huge (kdtree_impl.hpp:88-92)
    uint64_t leaf64 = leaf_size < 0 ? (uint64_t)(int64_t)leaf_size : (uint64_t)leaf_size;
    leaf64 = std::max<uint64_t>(leaf64, 16);
    const uint32_t leaf = (uint32_t)std::min<uint64_t>(leaf64, UINT32_MAX);

    Skeleton sk;
    sk.leaf = leaf;
    t.n = n;
    t.n8 = n8;
    t.leaf = (int)std::min<uint64_t>(leaf, INT32_MAX);
    t.nnodes = sk.nodes(n8);
    t.depth = sk.depth_of(n8);

    const size_t pbytes = (size_t)std::max<uint64_t>(n8, 1) * 4;
    NBKD_HIP(tree_malloc((void **)&t.x, pbytes));
    NBKD_HIP(tree_malloc((void **)&t.y, pbytes));
    NBKD_HIP(tree_malloc((void **)&t.z, pbytes));
    NBKD_HIP(tree_malloc((void **)&t.idx, pbytes));
    NBKD_HIP(tree_malloc((void **)&t.nodes, t.nnodes * sizeof(nbkd_node)));
    Soa A{t.x, t.y, t.z, t.idx};

    int dev = 0;
    NBKD_HIP(hipGetDevice(&dev));
    BuildScratch &scr = build_scratch(dev);
    // held until the stream has drained, on every return path
    struct ScratchLock {
        BuildScratch &b;
        hipStream_t s;
        ScratchLock(BuildScratch &b_, hipStream_t s_) : b(b_), s(s_) {
            b.mu.lock();
            hold_mark(&b);
        }
        ~ScratchLock() {
            (void)hipStreamSynchronize(s);
            hold_unmark(&b);
            b.mu.unlock();
        }
    } scr_lock(scr, s);
    ShapeTables &sh = scr.shape;
    if (!(sh.valid && sh.n8 == n8 && sh.leaf == leaf)) {
        // enumerate the shape down to SMALL-point segments
        sh.valid = sh.uploaded = false;
        sk.rec(0, 0, (uint32_t)n8, 0);
        sh.tab_c.clear();
        sh.tab_n.clear();
        for (auto &kv : sk.memo) {
            sh.tab_c.push_back((uint32_t)kv.first);
            sh.tab_n.push_back(kv.second);
        }
        if (sh.tab_c.empty()) {
            sh.tab_c.push_back(0);
            sh.tab_n.push_back(1);
        }
        // flatten large levels and their tiles
        sh.segs.clear();
        sh.tiles.clear();
        sh.info.clear();
        sh.max_seg = sh.max_tile = 0;
        for (auto &lv : sk.levels) {
            LevelInfo li{(uint32_t)sh.segs.size(), (uint32_t)lv.size(), (uint32_t)sh.tiles.size(), 0};
            for (uint32_t si = 0; si < lv.size(); ++si) {
                LSeg g = lv[si];
                g.tile_begin = (uint32_t)sh.tiles.size();
                for (uint32_t b = 0; b < g.count; b += TILE)
                    sh.tiles.push_back(Tile{si, b, std::min<uint32_t>(TILE, g.count - b), 0});
                g.tile_end = (uint32_t)sh.tiles.size();
                sh.segs.push_back(g);
            }
            li.ntile = (uint32_t)sh.tiles.size() - li.tile0;
            sh.max_seg = std::max<size_t>(sh.max_seg, li.nseg);
            sh.max_tile = std::max<size_t>(sh.max_tile, li.ntile);
            sh.info.push_back(li);
        }
        sh.small = std::move(sk.small);
        sh.n8 = n8;
        sh.leaf = leaf;
        sh.valid = true;
    }
    const std::vector<LSeg> &segs = sh.segs;
    const std::vector<Tile> &tiles = sh.tiles;
    const std::vector<LevelInfo> &info = sh.info;
    const std::vector<SSeg> &small = sh.small;
    const std::vector<uint32_t> &tab_c = sh.tab_c, &tab_n = sh.tab_n;
    const size_t max_seg = sh.max_seg, max_tile = sh.max_tile;

    // scratch: carve every temporary from the device's cached buffer (the
    // read-only shape tables first, so their place does not depend on the input)
    constexpr int NW = 7 + NBKD_PAD_LEAVES; // data box, padding leaves (group_kernel)
    Carve cv;
    const size_t o_segs = cv.take(segs.size() * sizeof(LSeg));
    const size_t o_tiles = cv.take(tiles.size() * sizeof(Tile));
    const size_t o_small = cv.take(small.size() * sizeof(SSeg));
    const size_t o_tabc = cv.take(tab_c.size() * 4);
    const size_t o_tabn = cv.take(tab_n.size() * 4);
    const size_t o_bx = cv.take(pbytes), o_by = cv.take(pbytes), o_bz = cv.take(pbytes),
                 o_bi = cv.take(pbytes);
    const size_t o_bad = cv.take(sizeof(uint32_t) * (NW + 1));
    const size_t o_st = cv.take(max_seg * sizeof(SelState));
    const size_t o_hist = cv.take(max_seg * 256 * sizeof(uint32_t));
    const size_t o_cnt = cv.take(max_tile * sizeof(uint2));
    const size_t o_off = cv.take(max_tile * sizeof(uint2));
    const size_t o_in = cv.take(!input_dev && n > 0 ? n * 3 * sizeof(float) : 0);
    if (scr.bytes < cv.off) {
        sh.uploaded = false;
        if (scr.p) NBKD_HIP(hipFree(scr.p));
        scr.p = nullptr;
        scr.bytes = 0;
        NBKD_HIP(malloc_or_release(&scr.p, cv.off));
        scr.bytes = cv.off;
    }
    char *const base = static_cast<char *>(scr.p);
    auto at = [&](size_t o) { return static_cast<void *>(base + o); };
    Soa B{(float *)at(o_bx), (float *)at(o_by), (float *)at(o_bz), (uint32_t *)at(o_bi)};
    uint32_t *const d_bad = (uint32_t *)at(o_bad); // [0]: box check, [1..]: group_kernel words
    const LSeg *const d_segs = (const LSeg *)at(o_segs);
    const Tile *const d_tiles = (const Tile *)at(o_tiles);
    SelState *const d_st = (SelState *)at(o_st);
    uint32_t *const d_hist = (uint32_t *)at(o_hist);
    uint2 *const d_cnt = (uint2 *)at(o_cnt), *const d_off = (uint2 *)at(o_off);
    const SSeg *const d_small = (const SSeg *)at(o_small);
    const uint32_t *const d_tabc = (const uint32_t *)at(o_tabc);
    const uint32_t *const d_tabn = (const uint32_t *)at(o_tabn);

    const float *aos = xyz;
    if (!input_dev && n > 0) {
        NBKD_HIP(hipMemcpyAsync(at(o_in), xyz, n * 3 * sizeof(float), hipMemcpyHostToDevice, s));
        aos = (const float *)at(o_in);
    }
    NBKD_HIP(hipMemsetAsync(d_bad, 0, sizeof(uint32_t), s));
    {
        TimedScope ts("prepare", s);
        uint64_t blocks = std::min<uint64_t>((n8 + TB - 1) / TB, 8192);
        if (blocks == 0) blocks = 1;
        prepare_kernel<<<(unsigned)blocks, TB, 0, s>>>(aos, n, n8, t.periodic, t.box, A, d_bad);
        NBKD_HIP(hipGetLastError());
    }
    // the shape tables (pageable copies, stream-ordered after prepare), once
    // per shape and scratch buffer
    if (!sh.uploaded) {
        if (!segs.empty()) {
            NBKD_HIP(hipMemcpyAsync(at(o_segs), segs.data(), segs.size() * sizeof(LSeg),
                                    hipMemcpyHostToDevice, s));
            NBKD_HIP(hipMemcpyAsync(at(o_tiles), tiles.data(), tiles.size() * sizeof(Tile),
                                    hipMemcpyHostToDevice, s));
        }
        NBKD_HIP(hipMemcpyAsync(at(o_small), small.data(), small.size() * sizeof(SSeg),
                                hipMemcpyHostToDevice, s));
        NBKD_HIP(hipMemcpyAsync(at(o_tabc), tab_c.data(), tab_c.size() * 4, hipMemcpyHostToDevice,
                                s));
        NBKD_HIP(hipMemcpyAsync(at(o_tabn), tab_n.data(), tab_n.size() * 4, hipMemcpyHostToDevice,
                                s));
        sh.uploaded = true;
    }
    // periodic box check: read back with the build's last words (the kernels
    // below run on any input; a bad box discards the tree)
    {
        TimedScope ts("build_levels", s);
        uint32_t run_blocks = 2048;
        {
            int dev = 0, cus = 256;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
                run_blocks = 8u * (uint32_t)std::max(cus, 1);
            (void)hipGetLastError();
            const char *e = knob("NBKD_RUN_BLOCKS"); // A/B only
            if (e) run_blocks = (uint32_t)std::max(1, atoi(e));
        }
        for (size_t d = 0; d < info.size(); ++d) {
            const LevelInfo &li = info[d];
            if (li.nseg == 0) continue;
            const int dim = axis_at(t.axes, (int)d);
            const Soa src = (d & 1) ? B : A;
            const Soa dst = (d & 1) ? A : B;
            const float *key = dim == 0 ? src.x : (dim == 1 ? src.y : src.z);
            const LSeg *lsegs = d_segs + li.seg0;
            const Tile *ltiles = d_tiles + li.tile0;
            SelState *st = d_st;
            uint32_t *hist = d_hist;
            // runs of `per` tiles, ~8 blocks per CU
            const uint32_t per = std::max<uint32_t>(1u, (li.ntile + run_blocks - 1) / run_blocks);
            const uint32_t nrun = (li.ntile + per - 1) / per;
#define NBKD_PASS(P)                                                                               \
    NBKD_HIP(hipMemsetAsync(hist, 0, (size_t)li.nseg * 256 * 4, s));                              \
    hist_kernel<P><<<nrun, TB, 0, s>>>(ltiles, lsegs, st, key, hist, li.ntile, per);              \
    select_kernel<P><<<li.nseg, TB, 0, s>>>(lsegs, st, hist, t.nodes, dim);
            NBKD_PASS(0)
            NBKD_PASS(1)
            NBKD_PASS(2)
            NBKD_PASS(3)
#undef NBKD_PASS
            count_kernel<<<nrun, TB, 0, s>>>(ltiles, lsegs, st, key, d_cnt, li.ntile,
                                             per);
            scan_kernel<<<li.nseg, TB, 0, s>>>(lsegs, d_cnt, d_off,
                                               li.tile0);
            scatter_kernel<<<li.ntile, TB, 0, s>>>(ltiles, lsegs, st, d_off, dim,
                                                   src, dst);
            NBKD_HIP(hipGetLastError());
        }
    }
    {
        TimedScope ts("build_small", s);
        static const int small_team = [] { // NBKD_SMALL_TEAM=0: one wave per sub-segment (A/B)
            const char *e = knob("NBKD_SMALL_TEAM");
            return (e && atoi(e) == 0) ? 0 : 1;
        }();
        if (!small.empty()) {
            NBKD_HIP(hipFuncSetAttribute((const void *)small_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)sizeof(SmallLds)));
            small_kernel<<<(unsigned)small.size(), TB, sizeof(SmallLds), s>>>(
                d_small, leaf, A, B, t.nodes, d_tabc,
                d_tabn, (int)tab_c.size(), small_team, t.axes);
            NBKD_HIP(hipGetLastError());
        }
    }
    // descent helpers for query bucketing: split per node + the shape table
    NBKD_HIP(tree_malloc((void **)&t.splits, std::max<uint64_t>(t.nnodes, 1) * 4));
    NBKD_HIP(tree_malloc((void **)&t.shape_c, tab_c.size() * 4));
    NBKD_HIP(tree_malloc((void **)&t.shape_n, tab_n.size() * 4));
    t.shape_len = (int)tab_c.size();
    NBKD_HIP(hipMemcpyAsync(t.shape_c, tab_c.data(), tab_c.size() * 4, hipMemcpyHostToDevice, s));
    NBKD_HIP(hipMemcpyAsync(t.shape_n, tab_n.data(), tab_n.size() * 4, hipMemcpyHostToDevice, s));
    {
        uint64_t blocks = std::min<uint64_t>((t.nnodes + TB - 1) / TB, 4096);
        extract_splits_kernel<<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(
            t.nodes, t.nnodes, t.splits);
        NBKD_HIP(hipGetLastError());
    }
    {
        NBKD_HIP(tree_malloc((void **)&t.nbox, std::max<uint64_t>(t.nnodes, 1) * 32));
        uint64_t blocks = std::min<uint64_t>((t.nnodes + TB - 1) / TB, 16384);
        const float lo0 = t.periodic ? 0.0f : -FLT_MAX, hi0 = t.periodic ? t.box : FLT_MAX;
        cellbox_kernel<<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(t.nodes, t.nnodes,
                                                                              lo0, hi0, t.nbox);
        NBKD_HIP(hipGetLastError());
    }
    if (t.depth <= 30) {
        NBKD_HIP(tree_malloc((void **)&t.hsplit, std::max<uint64_t>(hblk_blocks(t.depth), 1) * 64));
        uint64_t blocks = std::min<uint64_t>((t.nnodes + TB - 1) / TB, 16384);
        heap_splits_kernel<<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(
            t.nodes, t.nnodes, t.splits, t.shape_c, t.shape_n, t.shape_len, (uint32_t)t.n8,
            (uint32_t)t.leaf, hblk_offset(t.depth), t.hsplit);
        NBKD_HIP(hipGetLastError());
    }
    {
        // groups (ginfo, hinfo) and leafinfo + padding leaves + data box in one pass
        // (leafinfo_kernel only for a tree without points)
        TimedScope ts("build_groups", s);
        NBKD_HIP(tree_malloc((void **)&t.leafinfo, std::max<uint64_t>(t.nnodes, 1) * 32));
        uint32_t *const d_bbox = d_bad + 1;
        static const uint32_t init[NW] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u, 0u};
        NBKD_HIP(hipMemcpyAsync(d_bbox, init, sizeof(init), hipMemcpyHostToDevice, s));
        if (n8 > 0) {
            NBKD_HIP(tree_malloc((void **)&t.ginfo, (n8 / NBKD_GROUP) * 6 * sizeof(float)));
            if (t.leaf > 64) NBKD_HIP(tree_malloc((void **)&t.hinfo, t.nnodes * 12 * sizeof(float)));
            int dev = 0, cus = 256;
            NBKD_HIP(hipGetDevice(&dev));
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            const char *eg = knob("NBKD_GROUP_BLOCKS_PER_CU"); // A/B only
            const uint64_t per_cu = eg ? (uint64_t)std::max(1, atoi(eg)) : 128u;
            const uint64_t blocks = std::min<uint64_t>((t.nnodes + 3) / 4, (uint64_t)cus * per_cu);
            // leaves hold <= max(leaf, 16) points
            if (std::max<uint64_t>(t.leaf, 16) <= 64)
                group_kernel<1><<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(
                    t.nodes, t.nnodes, t.x, t.y, t.z, t.idx, t.n, t.ginfo, t.hinfo,
                    reinterpret_cast<uint32_t *>(t.leafinfo), d_bbox);
            else
                group_kernel<NBKD_GBLOCK / 64><<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(
                    t.nodes, t.nnodes, t.x, t.y, t.z, t.idx, t.n, t.ginfo, t.hinfo,
                    reinterpret_cast<uint32_t *>(t.leafinfo), d_bbox);
            NBKD_HIP(hipGetLastError());
            NBKD_HIP(tree_malloc((void **)&t.p4, n8 * sizeof(float4)));
            pack4_kernel<<<(unsigned)std::min<uint64_t>((n8 + 255) / 256, (uint64_t)cus * 16), 256,
                           0, s>>>(t.x, t.y, t.z, t.idx, n8, t.p4);
        } else {
            uint64_t blocks = std::min<uint64_t>((t.nnodes + TB - 1) / TB, 16384);
            leafinfo_kernel<<<(unsigned)std::max<uint64_t>(blocks, 1), TB, 0, s>>>(
                t.nodes, t.nnodes, t.x, t.y, t.z, t.idx, t.n, t.leafinfo, d_bbox);
        }
        NBKD_HIP(hipGetLastError());
        uint32_t hw[NW + 1]; // box-check flag, then the data box and padding leaves
        NBKD_HIP(hipMemcpyAsync(hw, d_bad, sizeof(hw), hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
        if (t.periodic && hw[0]) {
            set_error("When using periodic boundary conditions, all points must be within the "
                      "box (0 <= x <= box_size).");
            return NBKD_EBOX;
        }
        const uint32_t *const hb = hw + 1;
        // padding sits in the last leaf; should ties ever spread it, up to
        // NBKD_PAD_LEAVES leaves are listed, beyond that the shortcut is off
        t.npad_leaves = (int)hb[6];
        for (int j = 0; j < NBKD_PAD_LEAVES; ++j)
            t.pad_leaves[j] = j < (int)hb[6] ? hb[7 + j] : 0xFFFFFFFFu;
        for (int a = 0; a < 3; ++a) {
            t.bbox_lo[a] = hb[a] == 0xFFFFFFFFu ? 0.0f : fkey_inv(hb[a]);
            t.bbox_hi[a] = hb[3 + a] == 0u ? 0.0f : fkey_inv(hb[3 + a]);
        }
    }
    NBKD_HIP(hipStreamSynchronize(s));
    return NBKD_OK;
}

} // namespace nbkd
