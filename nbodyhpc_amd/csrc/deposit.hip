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
// column-major (gx, gy, nz) result (pybind.cpp:141-145), accumulated with
// float atomics in L2.
//
// Work split: one wave takes 64 consecutive particles (a dynamic counter hands
// out the groups).  Sub-pixel particles (radius < half a voxel) land in one
// voxel per image and are deposited by their own lane.  Every other particle
// is processed by the whole wave: for each slice its sprite rectangle is swept
// 64 voxels at a time; a voxel whose farthest sub-sample lies inside the ball
// takes the full weight, one whose nearest sub-sample lies outside takes
// nothing, and the straddling voxels are compacted into LDS and counted with
// the wave's lanes over the S^3 sub-samples (one voxel per pass at S = 4), so
// that the per-sub-sample test is exactly the fragment shader's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "internal.hpp"
#include "packet.hpp"

namespace nbkd {
namespace {

constexpr int DB = 256; // threads per block (4 waves)

struct DepositArgs {
    const float *xyz, *w, *r;
    uint64_t n;
    int gx, gy, nz;
    float ppu;
    float period[3];
    int S, S3;
    int mode; // 0: volume; 1: one plane at z = 0 (render_points)
    const float *tbl;
    float *grid;
    uint32_t *work;
};

struct WaveLds {
    float dx[64], dy[64];
    uint64_t idx[64];
};

__device__ __forceinline__ void grid_add(float *g, uint64_t i, float v) {
    unsafeAtomicAdd(g + i, v);
}

// slice plane depth and bounds (point_renderer.cpp:878-880; 2-D: :632-644)
__device__ __forceinline__ void plane(int mode, int64_t s, float ppu, float &depth, float &lower,
                                      float &upper) {
    if (mode == 1) {
        depth = 0.0f;
        lower = -0.5f;
        upper = 0.5f;
        return;
    }
    depth = (float)(((double)s + 0.5) / (double)ppu);
    lower = (float)((double)s / (double)ppu);
    upper = (float)((double)(s + 1) / (double)ppu);
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

// min / max over the S sub-sample offsets of |d - (i + 0.5) / S|, as the
// fragment shader rounds them: subtraction is monotone in the offset, so the
// max sits at an end and the min next to floor(d * S)
__device__ __forceinline__ void axis_range(float d, int S, float fS, float &mn, float &mx) {
    mx = fmaxf(fabsf(d - 0.5f / fS), fabsf(d - ((float)(S - 1) + 0.5f) / fS));
    const float t = floorf(d * fS);
    const int c = (int)fminf(fmaxf(t, 0.0f), (float)(S - 1));
    mn = fabsf(d - ((float)c + 0.5f) / fS);
    if (c > 0) mn = fminf(mn, fabsf(d - ((float)(c - 1) + 0.5f) / fS));
    if (c < S - 1) mn = fminf(mn, fabsf(d - ((float)(c + 1) + 0.5f) / fS));
}

// sprite pixel range per axis: centres px + 0.5 in [xw - h, xw + h), cut to [0, g)
__device__ __forceinline__ void sprite_range(float xw, float h, int g, int &lo, int &hi) {
    const float a = ceilf(xw - h - 0.5f), b = ceilf(xw + h - 0.5f) - 1.0f;
    lo = (int)fminf(fmaxf(a, 0.0f), (float)g); // clamped before the casts
    hi = (int)fmaxf(fminf(b, (float)(g - 1)), -1.0f);
}

// one particle image deposited by the whole wave (x..r wave-uniform)
__device__ void wave_image(const DepositArgs &a, WaveLds &L, int lane, float x, float y, float z,
                           float w, float r, float lxo, float lyo, float lzo, int slot, int sub,
                           int V) {
    const float ppu = a.ppu;
    const float o = r * ppu;
    const float r2 = o * o;
    const float vol = 4.0f / 3.0f * 3.14159265358979f * o * o * o;
    const float xw = x * ppu, yw = y * ppu;
    const float fS = (float)a.S;
    const float full = a.tbl[a.S3];
    int64_t s_lo = 0, s_hi = 0;
    if (a.mode == 0) {
        const float zl = floorf((z - r) * ppu) - 2.0f, zh = ceilf((z + r) * ppu) + 2.0f;
        s_lo = (int64_t)fminf(fmaxf(zl, 0.0f), (float)a.nz);
        s_hi = (int64_t)fmaxf(fminf(zh, (float)(a.nz - 1)), -1.0f);
    }
    for (int64_t s = s_lo; s <= s_hi; ++s) {
        float depth, lower, upper;
        plane(a.mode, s, ppu, depth, lower, upper);
        const float zoff = z - depth;
        if (ppu * (r - fabsf(zoff)) + 1.0f < 0.0f) continue; // gl_ClipDistance
        float dens, psize;
        if (o < 0.5f) {
            if (z <= lower || z > upper) continue;
            dens = w;
            psize = 1.0f;
        } else {
            const float pr = sqrtf(fmaxf(0.0f, r * r - zoff * zoff));
            psize = 2.0f * ceilf(pr * ppu) + 2.0f;
            dens = w / vol;
        }
        int px0, px1, py0, py1;
        sprite_range(xw, 0.5f * psize, a.gx, px0, px1);
        sprite_range(yw, 0.5f * psize, a.gy, py0, py1);
        if (px1 < px0 || py1 < py0) continue;
        const int rw = px1 - px0 + 1;
        const int nvox = rw * (py1 - py0 + 1);
        const float dz = zoff * ppu + 0.5f;
        float zmn, zmx;
        axis_range(dz, a.S, fS, zmn, zmx);
        const uint64_t sbase = (uint64_t)a.gy * (uint64_t)s;
        for (int c0 = 0; c0 < nvox; c0 += 64) {
            const int c = c0 + lane;
            const bool act = c < nvox;
            const int ry = c / rw;
            const int px = px0 + (c - ry * rw), py = py0 + ry;
            const uint64_t gi = (uint64_t)px + (uint64_t)a.gx * ((uint64_t)py + sbase);
            if (r2 < 0.25f) {
                if (act) grid_add(a.grid, gi, dens);
                continue;
            }
            const float dx = xw - (float)px, dy = yw - (float)py;
            float xmn, xmx, ymn, ymx;
            axis_range(dx, a.S, fS, xmn, xmx);
            axis_range(dy, a.S, fS, ymn, ymx);
            const float dmax = xmx * xmx + ymx * ymx + zmx * zmx;
            const float dmin = xmn * xmn + ymn * ymn + zmn * zmn;
            if (act && dmax < r2) grid_add(a.grid, gi, dens * full);
            const bool str = act && !(dmax < r2) && dmin < r2;
            const uint64_t m = __ballot(str);
            if (!m) continue;
            const int nstr = __popcll(m);
            if (str) {
                const int p = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                L.dx[p] = dx;
                L.dy[p] = dy;
                L.idx[p] = gi;
            }
            dev::wave_sync();
            if (a.S3 <= 64) {
                // V voxels per pass, S^3 lanes each
                const uint64_t seg = a.S3 == 64 ? ~0ull : ((1ull << a.S3) - 1ull);
                for (int e0 = 0; e0 < nstr; e0 += V) {
                    const int e = e0 + slot;
                    const bool ok = slot < V && e < nstr;
                    bool in = false;
                    if (ok) {
                        const float sx = L.dx[e] - lxo, sy = L.dy[e] - lyo, sz = dz - lzo;
                        in = sx * sx + sy * sy + sz * sz < r2;
                    }
                    const uint64_t b = __ballot(in);
                    if (ok && sub == 0) {
                        const int cnt = __popcll((b >> (slot * a.S3)) & seg);
                        if (cnt) grid_add(a.grid, L.idx[e], dens * a.tbl[cnt]);
                    }
                }
            } else {
                for (int e = 0; e < nstr; ++e) {
                    const float ex = L.dx[e], ey = L.dy[e];
                    int cnt = 0;
                    for (int t0 = 0; t0 < a.S3; t0 += 64) {
                        const int t = t0 + lane;
                        bool in = false;
                        if (t < a.S3) {
                            const int i = t / (a.S * a.S), j = (t / a.S) % a.S, k = t % a.S;
                            const float sx = ex - ((float)i + 0.5f) / fS;
                            const float sy = ey - ((float)j + 0.5f) / fS;
                            const float sz = dz - ((float)k + 0.5f) / fS;
                            in = sx * sx + sy * sy + sz * sz < r2;
                        }
                        cnt += __popcll(__ballot(in));
                    }
                    if (lane == 0 && cnt) grid_add(a.grid, L.idx[e], dens * a.tbl[cnt]);
                }
            }
            dev::wave_sync();
        }
    }
}

// a sub-pixel particle image: one voxel (the vertex stage's snap, triangle.vert:45-57)
__device__ __forceinline__ void lane_image(const DepositArgs &a, float x, float y, float z, float w,
                                           float r) {
    const float ppu = a.ppu;
    int64_t s = 0;
    if (a.mode == 0) {
        s = (int64_t)fminf(fmaxf(floorf(z * ppu), -2.0f), (float)a.nz) - 1;
        float d, lo, up;
        int t = 0;
        for (; t < 3; ++t, ++s) {
            if (s < 0 || s >= a.nz) continue;
            plane(0, s, ppu, d, lo, up);
            if (z > lo && z <= up) break;
        }
        if (t == 3) return;
    }
    float depth, lower, upper;
    plane(a.mode, s, ppu, depth, lower, upper);
    if (ppu * (r - fabsf(z - depth)) + 1.0f < 0.0f) return;
    if (z <= lower || z > upper) return;
    int px0, px1, py0, py1;
    sprite_range(x * ppu, 0.5f, a.gx, px0, px1);
    sprite_range(y * ppu, 0.5f, a.gy, py0, py1);
    if (px1 < px0 || py1 < py0) return;
    grid_add(a.grid, (uint64_t)px0 + (uint64_t)a.gx * ((uint64_t)py0 + (uint64_t)a.gy * s), w);
}

__global__ void __launch_bounds__(DB) deposit_kernel(DepositArgs a) {
    __shared__ WaveLds lds[DB / 64];
    const int lane = threadIdx.x & 63;
    WaveLds &L = lds[threadIdx.x >> 6];
    // this lane's sub-sample for the S^3 <= 64 path: voxel slot `slot`, sample `sub`
    const int S = a.S, S3 = a.S3;
    const int V = S3 <= 64 ? 64 / S3 : 1;
    const int slot = S3 <= 64 ? lane / S3 : 0, sub = S3 <= 64 ? lane % S3 : 0;
    const float fS = (float)S;
    const float lxo = ((float)(sub / (S * S)) + 0.5f) / fS;
    const float lyo = ((float)((sub / S) % S) + 0.5f) / fS;
    const float lzo = ((float)(sub % S) + 0.5f) / fS;
    for (;;) {
        uint32_t g = 0;
        if (lane == 0) g = atomicAdd(a.work, 1u);
        g = __builtin_amdgcn_readfirstlane(__shfl(g, 0));
        const uint64_t base = (uint64_t)g * 64u;
        if (base >= a.n) break;
        const uint64_t i = base + lane;
        const bool valid = i < a.n;
        float x = 0.0f, y = 0.0f, z = 0.0f, w = 0.0f, r = 0.0f;
        if (valid) {
            x = a.xyz[3 * i];
            y = a.xyz[3 * i + 1];
            z = a.xyz[3 * i + 2];
            w = a.w[i];
            r = a.r[i];
        }
        const bool tiny = valid && r * a.ppu < 0.5f;
        if (tiny) {
            float sx[3], sy[3], sz[3];
            const int nx = images(x, r, a.period[0], sx), ny = images(y, r, a.period[1], sy),
                      nzi = images(z, r, a.period[2], sz);
            for (int ia = 0; ia < nx; ++ia)
                for (int ib = 0; ib < ny; ++ib)
                    for (int ic = 0; ic < nzi; ++ic) lane_image(a, sx[ia], sy[ib], sz[ic], w, r);
        }
        uint64_t big = __ballot(valid && !tiny);
        while (big) {
            const int l = __builtin_ctzll(big);
            big &= big - 1;
            const float bx = __shfl(x, l), by = __shfl(y, l), bz = __shfl(z, l);
            const float bw = __shfl(w, l), br = __shfl(r, l);
            float sx[3], sy[3], sz[3];
            const int nx = images(bx, br, a.period[0], sx), ny = images(by, br, a.period[1], sy),
                      nzi = images(bz, br, a.period[2], sz);
            for (int ia = 0; ia < nx; ++ia)
                for (int ib = 0; ib < ny; ++ib)
                    for (int ic = 0; ic < nzi; ++ic)
                        wave_image(a, L, lane, sx[ia], sy[ib], sz[ic], bw, br, lxo, lyo, lzo, slot,
                                   sub, V);
        }
    }
}

} // namespace

nbkd_status deposit(const float *xyz, const float *weight, const float *radius, uint64_t n, int gx,
                    int gy, int nz, float ppu, const float *period, int S, int mode, float *out,
                    uint32_t flags, hipStream_t s) {
    const uint64_t cells = (uint64_t)gx * (uint64_t)gy * (uint64_t)nz;
    const bool in_dev = flags & NBKD_INPUT_DEVICE, out_dev = flags & NBKD_OUTPUT_DEVICE;
    const bool accumulate = flags & NBKD_ACCUMULATE;
    if ((n + 63) / 64 >= (1ull << 32)) {
        set_error("nbkd_deposit: too many particles per call");
        return NBKD_EINVAL;
    }
    DevBuf bx, bw, br, bg, bt, bc;
    const float *dx = xyz, *dw = weight, *dr = radius;
    if (!in_dev && n) {
        NBKD_HIP(bx.alloc(n * 12, s));
        NBKD_HIP(bw.alloc(n * 4, s));
        NBKD_HIP(br.alloc(n * 4, s));
        NBKD_HIP(hipMemcpyAsync(bx.p, xyz, n * 12, hipMemcpyHostToDevice, s));
        NBKD_HIP(hipMemcpyAsync(bw.p, weight, n * 4, hipMemcpyHostToDevice, s));
        NBKD_HIP(hipMemcpyAsync(br.p, radius, n * 4, hipMemcpyHostToDevice, s));
        dx = bx.as<float>();
        dw = bw.as<float>();
        dr = br.as<float>();
    }
    float *dg = out;
    if (!out_dev) {
        NBKD_HIP(bg.alloc(cells * 4, s));
        dg = bg.as<float>();
        if (accumulate) NBKD_HIP(hipMemcpyAsync(dg, out, cells * 4, hipMemcpyHostToDevice, s));
    }
    if (!accumulate) NBKD_HIP(hipMemsetAsync(dg, 0, cells * 4, s));
    // overlap after c float additions of 1 / S^3 (triangle.frag:16,39)
    const int S3 = S * S * S;
    std::vector<float> tbl(S3 + 1);
    {
        const float inc = 1.0f / (float)S3;
        float acc = 0.0f;
        tbl[0] = 0.0f;
        for (int c = 1; c <= S3; ++c) tbl[c] = (acc += inc);
    }
    NBKD_HIP(bt.alloc(tbl.size() * 4, s));
    NBKD_HIP(hipMemcpyAsync(bt.p, tbl.data(), tbl.size() * 4, hipMemcpyHostToDevice, s));
    NBKD_HIP(bc.alloc(4, s));
    NBKD_HIP(hipMemsetAsync(bc.p, 0, 4, s));
    if (n) {
        DepositArgs a;
        a.xyz = dx;
        a.w = dw;
        a.r = dr;
        a.n = n;
        a.gx = gx;
        a.gy = gy;
        a.nz = nz;
        a.ppu = ppu;
        for (int d = 0; d < 3; ++d) a.period[d] = period ? period[d] : -1.0f;
        a.S = S;
        a.S3 = S3;
        a.mode = mode;
        a.tbl = bt.as<float>();
        a.grid = dg;
        a.work = bc.as<uint32_t>();
        int dev = 0, cus = 256;
        NBKD_HIP(hipGetDevice(&dev));
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint64_t groups = (n + 63) / 64;
        const uint64_t blocks = std::min<uint64_t>((groups + 3) / 4, (uint64_t)cus * 8);
        TimedScope ts("deposit", s);
        deposit_kernel<<<(unsigned)blocks, DB, 0, s>>>(a);
        NBKD_HIP(hipGetLastError());
    }
    if (!out_dev) {
        NBKD_HIP(hipMemcpyAsync(out, dg, cells * 4, hipMemcpyDeviceToHost, s));
        NBKD_HIP(hipStreamSynchronize(s));
    }
    return NBKD_OK;
}

} // namespace nbkd
