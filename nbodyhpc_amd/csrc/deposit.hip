// Mass deposit of spheres onto a voxel grid: the MI355X replacement of the
// reference's Vulkan point-volume rasteriser (rasterization/, the consumer of
// per-point smoothing lengths).  Semantics follow
// oracle/deposit_oracle.c, which restates the reference's vertex + fragment
// shaders (rasterization/shaders/triangle.vert:27-69, triangle.frag:14-44),
// periodic image augmentation (rasterization/src/cpp/vertex_utilities.cpp:15-42)
// and slice planes (rasterization/src/cpp/point_renderer.cpp:877-880).
//
// Layout: particles as given (row-major xyz, weight, radius); grid float32
// [nz][gy][gx] (index px + gx * (py + gy * s)), i.e. the reference's
// column-major (gx, gy, nz) result (pybind.cpp:141-145).  A caller may hold
// only the columns [x0, x0 + wx) (index px - x0 + wx * (py + gy * s)): the
// x-slab of one rank (nbodyhpc_amd/slab.py deposit_slab).
//
// Global float atomics execute at the memory side on MI355X (every request
// leaves L2, ~1.3 TB/s chip-wide; MI355X_MICROARCH.md "Global float atomics"),
// and a kNN-sized ball touches ~2,500 voxels, so the grid is accumulated in
// LDS instead, one 32 x 32 x 8 voxel tile per workgroup:
//   1. pair lists: every periodic image of every ball of at least half a voxel
//      radius is listed under each tile its sprite box overlaps (count, scan,
//      fill; a lane enumerates the tiles of a small box, the whole wave those
//      of a large one);
//   2. tiles: a workgroup takes a tile from a counter, its 4 waves take the
//      tile's balls from an LDS counter and sweep each ball's sprite rectangle
//      (cut to the tile) 64 voxels at a time, slice by slice.  A voxel whose
//      farthest sub-sample is inside the ball takes the full weight, one whose
//      nearest sub-sample is outside takes nothing (per-axis min / max
//      offsets: exact, because float subtraction, squaring and addition are
//      monotone), and straddling voxels go to a per-wave LDS ring; whenever 64
//      are queued each lane counts one voxel's S^3 sub-samples with the
//      fragment shader's own arithmetic.  Contributions are LDS float atomics;
//      the finished tile is written once with plain coalesced stores (zeros
//      included, so the grid needs no clearing);
//   3. sub-voxel balls (the vertex stage's snap, triangle.vert:45-57): one
//      lane each, one global atomic per image, after the tiles are written.
// Measured on the 256^3-ball / 1024^3-grid case (scripts/bench_deposit.py):
// one wave per ball with global atomics took 1775 ms in input order and 574 ms
// in Morton order (r02_deposit profiles); see DESIGN.md for this version.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "internal.hpp"
#include "packet.hpp"

namespace nbkd {
namespace {

constexpr int DB = 512; // threads per block (8 waves; two blocks per CU share the LDS)
constexpr int TX = 32, TY = 32, TZ = 8;
constexpr int TVOX = TX * TY * TZ;
constexpr int QCAP = 128; // straddling voxels queued per wave

struct DepositArgs {
    const float *xyz, *w, *r;
    uint64_t n;
    int gx, gy, nz;
    int x0, wx; // the columns [x0, x0 + wx) held in `grid` (a slab of a gx-wide grid)
    int ntx, nty, ntz;
    float ppu;
    float period[3];
    int S; // runtime S (template S == 0)
    int mode;
    bool accumulate;
    const float *planes; // nz x (depth, lower, upper)
    const float *tbl;    // overlap after c additions of 1 / S^3
    float *grid;
    uint32_t *tile_count; // per tile: pairs (count pass), then fill cursor
    const uint64_t *tile_off;
    uint64_t *pairs; // particle | image << 32
    uint32_t *work;  // tile counter
};

struct StraddleRing {
    float dx[QCAP], dy[QCAP], dz[QCAP], r2[QCAP], dens[QCAP];
    uint32_t li[QCAP];
};

__device__ __forceinline__ void lds_add(float *p, float v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// periodic images along one axis (vertex_utilities.cpp:21-40): the value itself,
// minus P when p + r > P, plus P when p - r < 0
__device__ __forceinline__ int images(float p, float r, float P, float sh[3]) {
    int n = 1;
    sh[0] = p;
    if (P > 0.0f) {
        if (p + r > P) sh[n++] = p - P;
        if (p - r < 0.0f) sh[n++] = p + P;
    }
    return n;
}

// sprite pixel range per axis: centres px + 0.5 in [xw - h, xw + h), cut to [0, g)
__device__ __forceinline__ void sprite_range(float xw, float h, int g, int &lo, int &hi) {
    const float a = ceilf(xw - h - 0.5f), b = ceilf(xw + h - 0.5f) - 1.0f;
    lo = (int)fminf(fmaxf(a, 0.0f), (float)g); // clamped before the casts
    hi = (int)fmaxf(fminf(b, (float)(g - 1)), -1.0f);
}

// slices a ball can reach: |zoff| <= r + 1/ppu passes the clip test (with margin)
__device__ __forceinline__ void slice_range(const DepositArgs &a, float z, float r, int &lo,
                                            int &hi) {
    if (a.mode == 1) {
        lo = hi = 0;
        return;
    }
    const float zl = floorf((z - r) * a.ppu) - 2.0f, zh = ceilf((z + r) * a.ppu) + 2.0f;
    lo = (int)fminf(fmaxf(zl, 0.0f), (float)a.nz);
    hi = (int)fmaxf(fminf(zh, (float)(a.nz - 1)), -1.0f);
}

// tile box of one ball image (sprites of every slice fit the widest one, taken
// with a voxel of margin); false when it misses the grid
__device__ __forceinline__ bool tile_box(const DepositArgs &a, float x, float y, float z, float r,
                                         int &tx0, int &tx1, int &ty0, int &ty1, int &tz0,
                                         int &tz1) {
    const float h = ceilf(r * a.ppu) + 2.0f;
    int px0, px1, py0, py1, s0, s1;
    sprite_range(x * a.ppu, h, a.gx, px0, px1);
    sprite_range(y * a.ppu, h, a.gy, py0, py1);
    px0 = max(px0, a.x0);
    px1 = min(px1, a.x0 + a.wx - 1);
    slice_range(a, z, r, s0, s1);
    if (px1 < px0 || py1 < py0 || s1 < s0) return false;
    tx0 = (px0 - a.x0) / TX;
    tx1 = (px1 - a.x0) / TX;
    ty0 = py0 / TY;
    ty1 = py1 / TY;
    tz0 = s0 / TZ;
    tz1 = s1 / TZ;
    return true;
}

// sub-sample offset (i + 0.5) / S (triangle.frag:25-33); with S a template
// constant and i unrolled this folds to the same correctly rounded constant
template <int S> __device__ __forceinline__ float off(int i, int Srt) {
    return ((float)i + 0.5f) / (float)(S ? S : Srt);
}

// min / max over the sub-sample offsets of |d - off_i|
template <int S>
__device__ __forceinline__ void axis_range(float d, int Srt, float &mn, float &mx) {
    const int n = S ? S : Srt;
    mx = fmaxf(fabsf(d - off<S>(0, Srt)), fabsf(d - off<S>(n - 1, Srt)));
    mn = fabsf(d - off<S>(0, Srt));
    if constexpr (S > 0) {
#pragma unroll
        for (int i = 1; i < S; ++i) mn = fminf(mn, fabsf(d - off<S>(i, Srt)));
    } else {
        for (int i = 1; i < n; ++i) mn = fminf(mn, fabsf(d - off<S>(i, Srt)));
    }
}

// number of the S^3 sub-samples inside the ball, d = (sx^2 + sy^2) + sz^2 < r2
template <int S>
__device__ __forceinline__ int subsample_count(float dx, float dy, float dz, float r2, int Srt) {
    int c = 0;
    if constexpr (S > 0) {
        float x2[S], y2[S], z2[S];
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const float sx = dx - off<S>(i, Srt), sy = dy - off<S>(i, Srt),
                        sz = dz - off<S>(i, Srt);
            x2[i] = sx * sx;
            y2[i] = sy * sy;
            z2[i] = sz * sz;
        }
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const float t = x2[i] + y2[j];
#pragma unroll
                for (int k = 0; k < S; ++k) c += (t + z2[k] < r2) ? 1 : 0;
            }
    } else {
        for (int i = 0; i < Srt; ++i) {
            const float sx = dx - off<S>(i, Srt);
            for (int j = 0; j < Srt; ++j) {
                const float sy = dy - off<S>(j, Srt);
                const float t = sx * sx + sy * sy;
                for (int k = 0; k < Srt; ++k) {
                    const float sz = dz - off<S>(k, Srt);
                    c += (t + sz * sz < r2) ? 1 : 0;
                }
            }
        }
    }
    return c;
}

// lanes < cnt count and deposit ring entries head + lane
template <int S>
__device__ __forceinline__ void drain(const DepositArgs &a, StraddleRing &Q, float *acc,
                                      const float *tbl, uint32_t head, uint32_t cnt, int lane) {
    if ((uint32_t)lane < cnt) {
        const uint32_t e = (head + lane) % QCAP;
        const int c = subsample_count<S>(Q.dx[e], Q.dy[e], Q.dz[e], Q.r2[e], a.S);
        if (c) lds_add(acc + Q.li[e], Q.dens[e] * tbl[c]);
    }
}

// one ball image (radius >= half a voxel) cut to the tile [X0, X0+TX) x
// [Y0, Y0+TY) x [Z0, Z0+TZ), deposited by the whole wave into acc.  Lane k
// first takes slice s_lo + k (clip test, sprite rectangle, z terms); the wave
// then sweeps the union of those rectangles 64 (x, y) columns at a time, each
// lane computing its column's x / y terms once and walking the slices.
template <int S>
__device__ void tile_image(const DepositArgs &a, StraddleRing &Q, float *acc, const float *tbl,
                           const float *depth, uint32_t &head, uint32_t &tail, int lane, float x,
                           float y, float z, float w, float r, float full, int X0, int Y0,
                           int Z0) {
    const float ppu = a.ppu;
    const float o = r * ppu;
    const float r2 = o * o;
    const float vol = 4.0f / 3.0f * 3.14159265358979f * o * o * o;
    const float dens = w / vol;
    const float vfull = dens * full;
    const float xw = x * ppu, yw = y * ppu;
    int s_lo, s_hi;
    slice_range(a, z, r, s_lo, s_hi);
    s_lo = max(s_lo, Z0);
    s_hi = min(s_hi, min(Z0 + TZ, a.nz) - 1);
    const int ns = s_hi - s_lo + 1;
    if (ns <= 0) return;
    const int gxe = min(X0 + TX, a.x0 + a.wx), gye = min(Y0 + TY, a.gy);
    // this lane's slice (lanes >= ns hold a copy of the last one, never used)
    const int ks = s_lo + min(lane, ns - 1);
    const float zoff = z - depth[ks - Z0];
    const float pr = sqrtf(fmaxf(0.0f, r * r - zoff * zoff));
    const float psize = 2.0f * ceilf(pr * ppu) + 2.0f;
    int sx0, sx1, sy0, sy1;
    sprite_range(xw, 0.5f * psize, gxe, sx0, sx1);
    sprite_range(yw, 0.5f * psize, gye, sy0, sy1);
    sx0 = max(sx0, X0);
    sy0 = max(sy0, Y0);
    const bool pass = lane < ns && !(ppu * (r - fabsf(zoff)) + 1.0f < 0.0f) && sx1 >= sx0 &&
                      sy1 >= sy0; // gl_ClipDistance, sprite inside the tile
    const uint64_t pm = __ballot(pass);
    if (!pm) return;
    const float dz = zoff * ppu + 0.5f;
    float zmn, zmx;
    axis_range<S>(dz, a.S, zmn, zmx);
    const float zmn2 = zmn * zmn, zmx2 = zmx * zmx;
    // union rectangle of the passing slices (lanes < TZ)
    int ux0 = pass ? sx0 : 0x7FFFFFFF, uy0 = pass ? sy0 : 0x7FFFFFFF;
    int ux1 = pass ? sx1 : -1, uy1 = pass ? sy1 : -1;
#pragma unroll
    for (int m = 1; m < TZ; m <<= 1) {
        ux0 = min(ux0, __shfl_xor(ux0, m, 64));
        uy0 = min(uy0, __shfl_xor(uy0, m, 64));
        ux1 = max(ux1, __shfl_xor(ux1, m, 64));
        uy1 = max(uy1, __shfl_xor(uy1, m, 64));
    }
    ux0 = __builtin_amdgcn_readfirstlane(ux0);
    uy0 = __builtin_amdgcn_readfirstlane(uy0);
    ux1 = __builtin_amdgcn_readfirstlane(ux1);
    uy1 = __builtin_amdgcn_readfirstlane(uy1);
    const int rw = ux1 - ux0 + 1;
    const int ncol = rw * (uy1 - uy0 + 1); // <= TX * TY
    const float rcp = 1.0f / (float)rw;
    for (int c0 = 0; c0 < ncol; c0 += 64) {
        const int c = c0 + lane;
        const bool act = c < ncol;
        // row of column c: (c + 0.5) / rw is at least 0.5 / rw from an integer
        const int ry = (int)(((float)c + 0.5f) * rcp);
        const int px = ux0 + (c - ry * rw), py = uy0 + ry;
        const float dx = xw - (float)px, dy = yw - (float)py;
        float xmn, xmx, ymn, ymx;
        axis_range<S>(dx, a.S, xmn, xmx);
        axis_range<S>(dy, a.S, ymn, ymx);
        const float xy_mx = xmx * xmx + ymx * ymx, xy_mn = xmn * xmn + ymn * ymn;
        const int li0 = (px - X0) + TX * (py - Y0);
        uint64_t sl = pm;
        while (sl) {
            const int k = __builtin_ctzll(sl);
            sl &= sl - 1;
            const int kx0 = __builtin_amdgcn_readlane(sx0, k), kx1 = __builtin_amdgcn_readlane(sx1, k);
            const int ky0 = __builtin_amdgcn_readlane(sy0, k), ky1 = __builtin_amdgcn_readlane(sy1, k);
            const float kmx2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zmx2), k));
            const float kmn2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zmn2), k));
            const bool in = act && px >= kx0 && px <= kx1 && py >= ky0 && py <= ky1;
            const bool inside = xy_mx + kmx2 < r2;
            const bool reach = xy_mn + kmn2 < r2;
            const int li = li0 + TX * TY * (s_lo + k - Z0);
            if (in && inside) lds_add(acc + li, vfull);
            const bool str = in && reach && !inside;
            const uint64_t m = __ballot(str);
            if (!m) continue;
            if (str) {
                const uint32_t e =
                    (tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))) %
                    QCAP;
                Q.dx[e] = dx;
                Q.dy[e] = dy;
                Q.dz[e] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), k));
                Q.r2[e] = r2;
                Q.dens[e] = dens;
                Q.li[e] = (uint32_t)li;
            }
            tail += (uint32_t)__popcll(m);
            if (tail - head >= 64) {
                dev::wave_sync();
                drain<S>(a, Q, acc, tbl, head, 64, lane);
                head += 64;
                dev::wave_sync();
            }
        }
    }
}

// the image `im` (ia * 9 + ib * 3 + ic over the per-axis image lists) of ball p
__device__ __forceinline__ void image_of(const DepositArgs &a, uint32_t p, uint32_t im, float &x,
                                         float &y, float &z, float &w, float &r) {
    r = a.r[p];
    w = a.w[p];
    float sx[3], sy[3], sz[3];
    images(a.xyz[3 * (uint64_t)p], r, a.period[0], sx);
    images(a.xyz[3 * (uint64_t)p + 1], r, a.period[1], sy);
    images(a.xyz[3 * (uint64_t)p + 2], r, a.period[2], sz);
    const uint32_t ia = im / 9, ib = (im / 3) % 3, ic = im % 3;
    x = ia == 0 ? sx[0] : ia == 1 ? sx[1] : sx[2];
    y = ib == 0 ? sy[0] : ib == 1 ? sy[1] : sy[2];
    z = ic == 0 ? sz[0] : ic == 1 ? sz[1] : sz[2];
}

// pair lists.  COUNT: tile_count[t] += 1 per (ball image, tile); FILL: place
// the pair at tile_off[t] + (--tile_count[t])
template <bool FILL>
__device__ __forceinline__ void emit(const DepositArgs &a, uint32_t t, uint64_t pair) {
    if constexpr (FILL) {
        const uint32_t pos = atomicSub(a.tile_count + t, 1u) - 1u;
        a.pairs[a.tile_off[t] + pos] = pair;
    } else {
        atomicAdd(a.tile_count + t, 1u);
    }
}

template <bool FILL> __global__ void __launch_bounds__(DB) deposit_pairs_kernel(DepositArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * DB + threadIdx.x;
    const bool valid = i < a.n;
    const uint32_t p = (uint32_t)i;
    float r = 0.0f, x = 0.0f, y = 0.0f, z = 0.0f;
    if (valid) {
        r = a.r[p];
        x = a.xyz[3 * i];
        y = a.xyz[3 * i + 1];
        z = a.xyz[3 * i + 2];
    }
    // sub-voxel balls: deposit_tiny_kernel.  A non-finite radius or centre
    // contributes nothing: the shader's w / (4/3 pi R^3) is 0 for R = inf (the
    // kth_distance padding when k > n), and NaN vertices are not rasterised
    const bool finite = isfinite(r) && isfinite(x) && isfinite(y) && isfinite(z);
    const bool ball = valid && finite && !(r * a.ppu < 0.5f);
    float sx[3], sy[3], sz[3];
    int nx = 0, ny = 0, nzi = 0;
    if (ball) {
        nx = images(x, r, a.period[0], sx);
        ny = images(y, r, a.period[1], sy);
        nzi = images(z, r, a.period[2], sz);
    }
    uint32_t big = 0; // images with more than 64 tiles: enumerated by the whole wave
    for (int ia = 0; ia < nx; ++ia)
        for (int ib = 0; ib < ny; ++ib)
            for (int ic = 0; ic < nzi; ++ic) {
                int tx0, tx1, ty0, ty1, tz0, tz1;
                if (!tile_box(a, sx[ia], sy[ib], sz[ic], r, tx0, tx1, ty0, ty1, tz0, tz1))
                    continue;
                const uint32_t im = ia * 9 + ib * 3 + ic;
                const int nt = (tx1 - tx0 + 1) * (ty1 - ty0 + 1) * (tz1 - tz0 + 1);
                if (nt > 64) {
                    big |= 1u << im;
                    continue;
                }
                const uint64_t pair = (uint64_t)p | ((uint64_t)im << 32);
                for (int tz = tz0; tz <= tz1; ++tz)
                    for (int ty = ty0; ty <= ty1; ++ty)
                        for (int tx = tx0; tx <= tx1; ++tx)
                            emit<FILL>(a, (uint32_t)(tx + a.ntx * (ty + a.nty * tz)), pair);
            }
    const int lane = threadIdx.x & 63;
    uint64_t todo = __ballot(big != 0);
    while (todo) {
        const int l = __builtin_ctzll(todo);
        const uint32_t bl = (uint32_t)__shfl((int)big, l);
        const uint32_t im = (uint32_t)__builtin_ctz(bl);
        if (lane == l) big &= big - 1;
        if (!__shfl((int)(big != 0), l)) todo &= todo - 1;
        const uint32_t bp = (uint32_t)__shfl((int)p, l);
        float bx, by, bz, bw, br;
        image_of(a, bp, im, bx, by, bz, bw, br);
        int tx0, tx1, ty0, ty1, tz0, tz1;
        tile_box(a, bx, by, bz, br, tx0, tx1, ty0, ty1, tz0, tz1);
        const int wx = tx1 - tx0 + 1, wy = ty1 - ty0 + 1;
        const int nt = wx * wy * (tz1 - tz0 + 1);
        const uint64_t pair = (uint64_t)bp | ((uint64_t)im << 32);
        for (int j = lane; j < nt; j += 64) {
            const int tz = tz0 + j / (wx * wy), rem = j % (wx * wy);
            const int ty = ty0 + rem / wx, tx = tx0 + rem % wx;
            emit<FILL>(a, (uint32_t)(tx + a.ntx * (ty + a.nty * tz)), pair);
        }
    }
}

template <int S> __global__ void __launch_bounds__(DB) deposit_tile_kernel(DepositArgs a) {
    __shared__ float acc[TVOX];
    __shared__ StraddleRing rings[DB / 64];
    __shared__ uint32_t sh_tile, sh_next;
    __shared__ float sh_depth[TZ];                   // the tile's slice depths
    __shared__ float sh_tbl[S ? S * S * S + 1 : 1]; // overlap table (template S)
    const int lane = threadIdx.x & 63;
    StraddleRing &Q = rings[threadIdx.x >> 6];
    const int S3 = S ? S * S * S : a.S * a.S * a.S;
    const float full = a.tbl[S3];
    if constexpr (S > 0)
        for (int i = threadIdx.x; i <= S3; i += DB) sh_tbl[i] = a.tbl[i];
    const float *tbl = S ? sh_tbl : a.tbl;
    const uint32_t ntiles = (uint32_t)(a.ntx * a.nty * a.ntz);
    for (;;) {
        if (threadIdx.x == 0) {
            sh_tile = atomicAdd(a.work, 1u);
            sh_next = 0;
        }
        for (int v = threadIdx.x; v < TVOX; v += DB) acc[v] = 0.0f;
        __syncthreads();
        const uint32_t t = sh_tile;
        if (t >= ntiles) break;
        const int tx = (int)(t % a.ntx), ty = (int)((t / a.ntx) % a.nty), tz = (int)(t / (a.ntx * a.nty));
        const int X0 = a.x0 + tx * TX, Y0 = ty * TY, Z0 = tz * TZ;
        if (threadIdx.x < TZ) sh_depth[threadIdx.x] = a.planes[3 * min(Z0 + (int)threadIdx.x, a.nz - 1)];
        __syncthreads();
        const uint64_t beg = a.tile_off[t], cnt = a.tile_off[t + 1] - beg;
        uint32_t head = 0, tail = 0;
        // the next ball's record and coordinates are loaded while this one is swept
        auto take = [&]() {
            uint32_t j = 0;
            if (lane == 0) j = atomicAdd(&sh_next, 1u);
            return __builtin_amdgcn_readfirstlane(__shfl(j, 0));
        };
        uint32_t j = take();
        float x = 0.0f, y = 0.0f, z = 0.0f, w = 0.0f, r = 0.0f;
        if (j < cnt) {
            const uint64_t pair = a.pairs[beg + j];
            image_of(a, (uint32_t)pair, (uint32_t)(pair >> 32), x, y, z, w, r);
        }
        while (j < cnt) {
            const uint32_t jn = take();
            float nx = 0.0f, ny = 0.0f, nz = 0.0f, nw = 0.0f, nr = 0.0f;
            if (jn < cnt) {
                const uint64_t pair = a.pairs[beg + jn];
                image_of(a, (uint32_t)pair, (uint32_t)(pair >> 32), nx, ny, nz, nw, nr);
            }
            tile_image<S>(a, Q, acc, tbl, sh_depth, head, tail, lane, x, y, z, w, r, full, X0, Y0,
                          Z0);
            j = jn;
            x = nx;
            y = ny;
            z = nz;
            w = nw;
            r = nr;
        }
        dev::wave_sync();
        drain<S>(a, Q, acc, tbl, head, tail - head, lane);
        __syncthreads();
        // the finished tile: one plain store per voxel (rows of 32 floats)
        for (int v = threadIdx.x; v < TVOX; v += DB) {
            const int lx = v % TX, ly = (v / TX) % TY, lz = v / (TX * TY);
            const int px = X0 + lx, py = Y0 + ly, s = Z0 + lz;
            if (px < a.x0 + a.wx && py < a.gy && s < a.nz) {
                const uint64_t gi =
                    (uint64_t)(px - a.x0) + (uint64_t)a.wx * ((uint64_t)py + (uint64_t)a.gy * s);
                a.grid[gi] = a.accumulate ? a.grid[gi] + acc[v] : acc[v];
            }
        }
        __syncthreads();
    }
}

// sub-voxel balls: one lane each, one voxel per image (global atomics, after the tiles)
__global__ void __launch_bounds__(DB) deposit_tiny_kernel(DepositArgs a) {
    const uint64_t p = (uint64_t)blockIdx.x * DB + threadIdx.x;
    if (p >= a.n) return;
    const float r = a.r[p], ppu = a.ppu;
    if (!(r * ppu < 0.5f)) return;
    const float x = a.xyz[3 * p], y = a.xyz[3 * p + 1], z = a.xyz[3 * p + 2], w = a.w[p];
    if (!isfinite(x) || !isfinite(y) || !isfinite(z)) return; // as deposit_pairs_kernel
    float sx[3], sy[3], sz[3];
    const int nx = images(x, r, a.period[0], sx), ny = images(y, r, a.period[1], sy),
              nzi = images(z, r, a.period[2], sz);
    for (int ic = 0; ic < nzi; ++ic) {
        const float zz = sz[ic];
        // the slice with lower < z <= upper (only those pass the snap test)
        int s = 0;
        if (a.mode == 0) {
            int c = (int)fminf(fmaxf(floorf(zz * ppu), -2.0f), (float)a.nz) - 1;
            int t3 = 0;
            for (; t3 < 3; ++t3, ++c)
                if (c >= 0 && c < a.nz && zz > a.planes[3 * c + 1] && zz <= a.planes[3 * c + 2])
                    break;
            if (t3 == 3) continue;
            s = c;
        }
        const float depth = a.planes[3 * s], lower = a.planes[3 * s + 1],
                    upper = a.planes[3 * s + 2];
        if (ppu * (r - fabsf(zz - depth)) + 1.0f < 0.0f) continue;
        if (zz <= lower || zz > upper) continue;
        for (int ia = 0; ia < nx; ++ia)
            for (int ib = 0; ib < ny; ++ib) {
                int px0, px1, py0, py1;
                sprite_range(sx[ia] * ppu, 0.5f, a.gx, px0, px1);
                sprite_range(sy[ib] * ppu, 0.5f, a.gy, py0, py1);
                if (px1 < px0 || py1 < py0 || px0 < a.x0 || px0 >= a.x0 + a.wx) continue;
                unsafeAtomicAdd(a.grid + (uint64_t)(px0 - a.x0) +
                                    (uint64_t)a.wx * ((uint64_t)py0 + (uint64_t)a.gy * s),
                                w);
            }
    }
}

// exclusive scan of n uint32 counts into uint64 offsets (out[n] = total):
// 1024-element blocks, then the block sums by one block, then the carry-in
constexpr int SB = 1024;
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t v, uint64_t *wsum) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint64_t s = threadIdx.x < SB / 64 ? wsum[threadIdx.x] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t u = __shfl_up(s, o, 64);
            if ((int)threadIdx.x >= o) s += u;
        }
        if (threadIdx.x < SB / 64) wsum[threadIdx.x] = s;
    }
    __syncthreads();
    const uint64_t r = v + (wv ? wsum[wv - 1] : 0);
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(SB) scan_blocks_kernel(const uint32_t *in, uint64_t n,
                                                         uint64_t *out, uint64_t *bsum) {
    __shared__ uint64_t wsum[SB / 64];
    const uint64_t i = (uint64_t)blockIdx.x * SB + threadIdx.x;
    const uint64_t v = i < n ? in[i] : 0;
    const uint64_t inc = block_incl_scan(v, wsum);
    if (i <= n) out[i] = inc - v;
    if (threadIdx.x == SB - 1) bsum[blockIdx.x] = inc;
}

__global__ void __launch_bounds__(SB) scan_sums_kernel(uint64_t *bsum, uint32_t nb) {
    __shared__ uint64_t wsum[SB / 64];
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += SB) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t v = b < nb ? bsum[b] : 0;
        const uint64_t inc = block_incl_scan(v, wsum);
        if (b < nb) bsum[b] = carry + inc - v;
        carry += wsum[SB / 64 - 1]; // the chunk's total
        __syncthreads();
    }
}

__global__ void __launch_bounds__(SB) scan_add_kernel(uint64_t *out, uint64_t n,
                                                      const uint64_t *bsum) {
    const uint64_t i = (uint64_t)blockIdx.x * SB + threadIdx.x;
    if (i <= n) out[i] += bsum[blockIdx.x];
}

// one workspace per device for the deposit's scratch, locked for the whole
// call (WsCall: a call on another stream first waits for the previous call's
// kernels, which may still use the scratch after a device-output call returned)
Workspace &deposit_ws(int dev) {
    static std::mutex mu;
    static std::map<int, Workspace *> ws;
    std::lock_guard<std::mutex> lk(mu);
    Workspace *&w = ws[dev];
    if (!w) w = new Workspace();
    return *w;
}

template <int S> void launch_tiles(const DepositArgs &a, uint64_t blocks, hipStream_t s) {
    deposit_tile_kernel<S><<<(unsigned)blocks, DB, 0, s>>>(a);
}

} // namespace

nbkd_status deposit(const float *xyz, const float *weight, const float *radius, uint64_t n, int gx,
                    int gy, int nz, float ppu, const float *period, int S, int mode, int x0, int wx,
                    float *out, uint32_t flags, hipStream_t s) {
    const uint64_t cells = (uint64_t)wx * (uint64_t)gy * (uint64_t)nz;
    const bool in_dev = flags & NBKD_INPUT_DEVICE, out_dev = flags & NBKD_OUTPUT_DEVICE;
    const bool accumulate = flags & NBKD_ACCUMULATE;
    if (n >= (1ull << 32)) {
        set_error("nbkd_deposit: at most 2^32 - 1 particles per call");
        return NBKD_EINVAL;
    }
    const int ntx = (wx + TX - 1) / TX, nty = (gy + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    const uint64_t ntiles = (uint64_t)ntx * nty * ntz;
    if (ntiles >= (1ull << 31)) {
        set_error("nbkd_deposit: grid too large");
        return NBKD_EINVAL;
    }
    int dev = 0, cus = 256;
    NBKD_HIP(hipGetDevice(&dev));
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    Workspace &ws = deposit_ws(dev);
    WsCall call(ws, s);
    NBKD_HIP(call.err);
    const float *dx = xyz, *dw = weight, *dr = radius;
    if (!in_dev && n) {
        float *b = (float *)ws.get(WS_Q, n * 20, s);
        if (!b) return NBKD_ENOMEM;
        NBKD_HIP(hipMemcpyAsync(b, xyz, n * 12, hipMemcpyHostToDevice, s));
        NBKD_HIP(hipMemcpyAsync(b + 3 * n, weight, n * 4, hipMemcpyHostToDevice, s));
        NBKD_HIP(hipMemcpyAsync(b + 4 * n, radius, n * 4, hipMemcpyHostToDevice, s));
        dx = b;
        dw = b + 3 * n;
        dr = b + 4 * n;
    }
    float *dg = out;
    if (!out_dev) {
        dg = (float *)ws.get(WS_OUTD, cells * 4, s);
        if (!dg) return NBKD_ENOMEM;
        if (accumulate) NBKD_HIP(hipMemcpyAsync(dg, out, cells * 4, hipMemcpyHostToDevice, s));
    }
    // small tables: overlap after c float additions of 1 / S^3 (triangle.frag:16,39),
    // slice planes (point_renderer.cpp:878-880; 2-D: depth 0, bounds +-0.5), counter
    const int S3 = S * S * S;
    std::vector<float> host((size_t)S3 + 1 + 3 * (size_t)nz + 1);
    {
        const float inc = 1.0f / (float)S3;
        float acc = 0.0f;
        host[0] = 0.0f;
        for (int c = 1; c <= S3; ++c) host[c] = (acc += inc);
        float *pl = host.data() + S3 + 1;
        for (int i = 0; i < nz; ++i) {
            if (mode == 1) {
                pl[3 * i] = 0.0f;
                pl[3 * i + 1] = -0.5f;
                pl[3 * i + 2] = 0.5f;
            } else {
                pl[3 * i] = (float)(((double)i + 0.5) / (double)ppu);
                pl[3 * i + 1] = (float)((double)i / (double)ppu);
                pl[3 * i + 2] = (float)((double)(i + 1) / (double)ppu);
            }
        }
        host.back() = 0.0f; // tile counter
    }
    float *dtab = (float *)ws.get(WS_TMP, host.size() * 4, s);
    uint32_t *tcount = (uint32_t *)ws.get(WS_COUNT, ntiles * 4, s);
    uint64_t *toff = (uint64_t *)ws.get(WS_OFF, (ntiles + 1) * 8, s);
    const uint32_t nsb = (uint32_t)((ntiles + 1 + SB - 1) / SB);
    uint64_t *bsum = (uint64_t *)ws.get(WS_SUMS, (size_t)nsb * 8, s);
    if (!dtab || !tcount || !toff || !bsum) return NBKD_ENOMEM;
    NBKD_HIP(hipMemcpyAsync(dtab, host.data(), host.size() * 4, hipMemcpyHostToDevice, s));
    NBKD_HIP(hipMemsetAsync(tcount, 0, ntiles * 4, s));
    DepositArgs a;
    a.xyz = dx;
    a.w = dw;
    a.r = dr;
    a.n = n;
    a.gx = gx;
    a.x0 = x0;
    a.wx = wx;
    a.gy = gy;
    a.nz = nz;
    a.ntx = ntx;
    a.nty = nty;
    a.ntz = ntz;
    a.ppu = ppu;
    for (int d = 0; d < 3; ++d) a.period[d] = period ? period[d] : -1.0f;
    a.S = S;
    a.mode = mode;
    a.accumulate = accumulate;
    a.tbl = dtab;
    a.planes = dtab + S3 + 1;
    a.grid = dg;
    a.tile_count = tcount;
    a.tile_off = toff;
    a.pairs = nullptr;
    a.work = (uint32_t *)(dtab + host.size() - 1);
    const unsigned nb = (unsigned)std::max<uint64_t>((n + DB - 1) / DB, 1);
    {
        TimedScope ts("deposit_pairs", s);
        if (n) deposit_pairs_kernel<false><<<nb, DB, 0, s>>>(a);
        scan_blocks_kernel<<<nsb, SB, 0, s>>>(tcount, ntiles, toff, bsum);
        scan_sums_kernel<<<1, SB, 0, s>>>(bsum, nsb);
        scan_add_kernel<<<nsb, SB, 0, s>>>(toff, ntiles, bsum);
        NBKD_HIP(hipGetLastError());
    }
    uint64_t npairs = 0;
    NBKD_HIP(hipMemcpyAsync(&npairs, toff + ntiles, 8, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    a.pairs = (uint64_t *)ws.get(WS_CAND, std::max<uint64_t>(npairs, 1) * 8, s);
    if (!a.pairs) return NBKD_ENOMEM;
    {
        TimedScope ts("deposit_fill", s);
        if (npairs) deposit_pairs_kernel<true><<<nb, DB, 0, s>>>(a);
        NBKD_HIP(hipGetLastError());
    }
    {
        // persistent blocks over the tiles: 56 KB of LDS each, 2 per CU
        const uint64_t blocks = std::min<uint64_t>(ntiles, (uint64_t)cus * 2);
        TimedScope ts("deposit", s);
        switch (S) {
        case 1: launch_tiles<1>(a, blocks, s); break;
        case 2: launch_tiles<2>(a, blocks, s); break;
        case 3: launch_tiles<3>(a, blocks, s); break;
        case 4: launch_tiles<4>(a, blocks, s); break;
        case 5: launch_tiles<5>(a, blocks, s); break;
        default: launch_tiles<0>(a, blocks, s); break;
        }
        NBKD_HIP(hipGetLastError());
    }
    if (n) {
        TimedScope ts("deposit_tiny", s);
        deposit_tiny_kernel<<<nb, DB, 0, s>>>(a);
        NBKD_HIP(hipGetLastError());
    }
    if (!out_dev) {
        NBKD_HIP(hipMemcpyAsync(out, dg, cells * 4, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
    }
    return NBKD_OK;
}

} // namespace nbkd
