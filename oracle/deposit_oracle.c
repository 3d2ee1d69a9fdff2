/*
 * ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into libnbkd.so.
 *
 * CPU restatement of the reference's point-volume rasteriser
 * (rasterization/, the consumer of per-point smoothing lengths named in
 * SURVEY.md 8(f) rank 3), one particle image and one slice at a time:
 *
 *   assemble_vertices                 rasterization/src/cpp/pybind.cpp:25-71
 *   augment_vertices_periodic         rasterization/src/cpp/vertex_utilities.cpp:15-42
 *   per-slice plane depth / bounds    rasterization/src/cpp/point_renderer.cpp:877-880
 *   2-D slice (depth 0, bounds +-0.5) rasterization/src/cpp/point_renderer.cpp:632-644
 *   vertex stage (clip, point size,   rasterization/shaders/triangle.vert:27-69
 *     density = w / volume, snap of sub-pixel points)
 *   fragment stage (S^3 sub-samples)  rasterization/shaders/triangle.frag:14-44
 *   additive blending                 rasterization/src/cpp/point_renderer.cpp:306-313
 *   output layout [x, y, slice]       rasterization/src/cpp/pybind.cpp:101-105,141-145
 *
 * Fixed-function behaviour the shaders leave to the rasteriser is restated as:
 *   - window coordinates of a point are (x * ppu, y * ppu) (the vertex stage's
 *     NDC transform and the viewport transform composed);
 *   - a point sprite of size P covers the pixels whose centres c satisfy
 *     xw - P/2 <= c < xw + P/2 (per axis), cut to the viewport; points are not
 *     clipped against the view volume (only by gl_ClipDistance), so periodic
 *     images off the edge still reach the pixels inside it.
 * No Vulkan implementation runs in this container, so this restatement is
 * "parity unpinned" against the reference's GPU output.
 *
 * Arithmetic is float32 with no contraction (-ffp-contract=off) so that
 * every sub-sample decision equals the HIP kernel's; the grid accumulates in
 * double (the GPU's float atomics sum in no fixed order, so grids are
 * compared with a tolerance, tests/test_gpu_deposit.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define ORC_API __attribute__((visibility("default")))

/* float -> integer with the value first clamped to [lo, hi] */
static int64_t clampi(float v, float lo, float hi) {
    return (int64_t)fminf(fmaxf(v, lo), hi);
}

/* (float)((double)s / ppu) etc., point_renderer.cpp:878-880 */
static void plane(int mode, int64_t s, float ppu, float *depth, float *lower, float *upper) {
    if (mode == 1) { /* render_points: one plane at z = 0 with bounds +-0.5 */
        *depth = 0.0f;
        *lower = -0.5f;
        *upper = 0.5f;
        return;
    }
    *depth = (float)(((double)s + 0.5) / (double)ppu);
    *lower = (float)((double)s / (double)ppu);
    *upper = (float)((double)(s + 1) / (double)ppu);
}

/* number of the S^3 fragment sub-samples inside the ball (triangle.frag:23-42) */
static int subsample_count(float dx, float dy, float dz, float r2, int S) {
    int c = 0;
    for (int i = 0; i < S; ++i) {
        const float xo = ((float)i + 0.5f) / (float)S;
        for (int j = 0; j < S; ++j) {
            const float yo = ((float)j + 0.5f) / (float)S;
            for (int k = 0; k < S; ++k) {
                const float zo = ((float)k + 0.5f) / (float)S;
                const float sx = dx - xo, sy = dy - yo, sz = dz - zo;
                const float d = sx * sx + sy * sy + sz * sz;
                if (d < r2) ++c;
            }
        }
    }
    return c;
}

/* overlap after c additions of 1/S^3 in float (triangle.frag:16,39) */
ORC_API void orc_deposit_overlap_table(int S, float *tbl) {
    const float inc = 1.0f / (float)(S * S * S);
    float acc = 0.0f;
    tbl[0] = 0.0f;
    for (int c = 1; c <= S * S * S; ++c) {
        acc += inc;
        tbl[c] = acc;
    }
}

static void deposit_image(float x, float y, float z, float w, float r, int gx, int gy, int nz,
                          float ppu, int S, int mode, const float *tbl, double *grid) {
    const float o = r * ppu;  /* out_radius */
    const float r2 = o * o;   /* outRadiusSquared */
    const float vol = 4.0f / 3.0f * 3.14159265358979f * o * o * o;
    const float xw = x * ppu, yw = y * ppu;
    int64_t s_lo = 0, s_hi = 0;
    if (mode == 0) {
        s_lo = clampi(floorf((z - r) * ppu) - 2.0f, 0.0f, (float)nz);
        s_hi = clampi(ceilf((z + r) * ppu) + 2.0f, -1.0f, (float)(nz - 1));
    }
    for (int64_t s = s_lo; s <= s_hi; ++s) {
        float depth, lower, upper;
        plane(mode, s, ppu, &depth, &lower, &upper);
        const float zoff = z - depth;
        const float clip = ppu * (r - fabsf(zoff)) + 1.0f;
        if (clip < 0.0f) continue;
        float dens;
        float psize;
        if (o < 0.5f) { /* sub-pixel: snapped into one slice, weight as is */
            if (z <= lower || z > upper) continue;
            dens = w;
            psize = 1.0f;
        } else {
            const float pr = sqrtf(fmaxf(0.0f, r * r - zoff * zoff));
            psize = 2.0f * ceilf(pr * ppu) + 2.0f;
            dens = w / vol;
        }
        const float h = 0.5f * psize;
        /* pixel centres px + 0.5 in [xw - h, xw + h) */
        const int64_t px0 = clampi(ceilf(xw - h - 0.5f), 0.0f, (float)gx);
        const int64_t px1 = clampi(ceilf(xw + h - 0.5f) - 1.0f, -1.0f, (float)(gx - 1));
        const int64_t py0 = clampi(ceilf(yw - h - 0.5f), 0.0f, (float)gy);
        const int64_t py1 = clampi(ceilf(yw + h - 0.5f) - 1.0f, -1.0f, (float)(gy - 1));
        const float dz = zoff * ppu + 0.5f;
        for (int64_t py = py0; py <= py1; ++py)
            for (int64_t px = px0; px <= px1; ++px) {
                float v;
                if (r2 < 0.25f) {
                    v = dens;
                } else {
                    const int c = subsample_count(xw - (float)px, yw - (float)py, dz, r2, S);
                    if (c == 0) continue;
                    v = dens * tbl[c];
                }
                grid[(size_t)px + (size_t)gx * ((size_t)py + (size_t)gy * (size_t)s)] += v;
            }
    }
}

/* per-axis image lists of one ball, augment_vertices_periodic
 * (rasterization/src/cpp/vertex_utilities.cpp:13-42): for each axis in turn
 * every vertex made so far gains a copy shifted by -P if x + r > P and one by
 * +P if x - r < 0, i.e. the cartesian product of these per-axis lists */
static void images(const float *p3, float r, const float *period, float sh[3][3], int ns[3]) {
    for (int d = 0; d < 3; ++d) {
        const float p = p3[d];
        ns[d] = 1;
        sh[d][0] = p;
        if (period[d] > 0.0f) {
            if (p + r > period[d]) sh[d][ns[d]++] = p - period[d];
            if (p - r < 0.0f) sh[d][ns[d]++] = p + period[d];
        }
    }
}

/* the periodic images of each ball (test hook): out[27 * i + j] (x, y, z) for
 * j < counts[i] */
ORC_API void orc_deposit_images(const float *xyz, const float *radius, int64_t n,
                                const float *period, float *out, int32_t *counts) {
    for (int64_t i = 0; i < n; ++i) {
        float sh[3][3];
        int ns[3];
        images(xyz + 3 * i, radius[i], period, sh, ns);
        int j = 0;
        for (int a = 0; a < ns[0]; ++a)
            for (int b = 0; b < ns[1]; ++b)
                for (int c = 0; c < ns[2]; ++c, ++j) {
                    float *o = out + 3 * (27 * i + j);
                    o[0] = sh[0][a];
                    o[1] = sh[1][b];
                    o[2] = sh[2][c];
                }
        counts[i] = j;
    }
}

/*
 * Deposit n particles (xyz row-major (n, 3), weight[n], radius[n]) into
 * grid[gx * gy * nz] (zeroed by the caller; index px + gx * (py + gy * s)).
 * period[d] > 0 makes axis d periodic with that length (images as
 * augment_vertices_periodic: shift -P if x + r > P, +P if x - r < 0, for every
 * image made so far).  mode 0: render_points_volume; 1: render_points (nz = 1).
 */
ORC_API int orc_deposit(const float *xyz, const float *weight, const float *radius, int64_t n,
                        int gx, int gy, int nz, float ppu, const float *period, int S, int mode,
                        double *grid) {
    if (S < 1 || S > 16 || gx < 1 || gy < 1 || nz < 1) return 1;
    float *tbl = (float *)malloc(sizeof(float) * (size_t)(S * S * S + 1));
    if (!tbl) return 1;
    orc_deposit_overlap_table(S, tbl);
    for (int64_t i = 0; i < n; ++i) {
        const float r = radius[i], w = weight[i];
        /* w / (4/3 pi R^3) is 0 for R = inf (and a NaN vertex is not
         * rasterised): such a ball contributes nothing */
        if (!isfinite(r) || !isfinite(xyz[3 * i]) || !isfinite(xyz[3 * i + 1]) ||
            !isfinite(xyz[3 * i + 2]))
            continue;
        float sh[3][3];
        int ns[3];
        images(xyz + 3 * i, r, period, sh, ns);
        for (int a = 0; a < ns[0]; ++a)
            for (int b = 0; b < ns[1]; ++b)
                for (int c = 0; c < ns[2]; ++c)
                    deposit_image(sh[0][a], sh[1][b], sh[2][c], w, r, gx, gy, nz, ppu, S, mode,
                                  tbl, grid);
    }
    free(tbl);
    return 0;
}
