// Device helpers shared by the query kernels (gfx950).  Metric formulas follow
// the reference bit for bit: kdtree/src/cpp/include/kdtree/kdtree.hpp:23-31,
// 35-45, 72-84, 89-107; compile with -ffp-contract=off.
#pragma once

#include "internal.hpp"

namespace nbkd {
namespace dev {

__device__ __forceinline__ uint32_t mbcnt64(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// the wave's index in its block, as a wave-uniform (SGPR) value: the compiler
// does not know threadIdx.x >> 6 is uniform, and everything derived from it
// (packet ids, column and LDS bases) would otherwise live in VGPRs
__device__ __forceinline__ int wave_id() { return (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Workgroups are dealt round-robin over the 8 XCDs (observed, not promised:
// MI355X_MICROARCH.md "Workgroup dispatch, XCD placement").  This bijection of
// [0, nb) gives each XCD a contiguous range of logical blocks instead, so
// neighbouring packets (which stage the same leaves) share one XCD's L2.  Speed
// only: every placement computes the same result.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u, j = b >> 3;
    return x * q + (x < r ? x : r) + j;
}
__device__ __forceinline__ float unif(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, v)));
}

// ------------------------------------------------------------------ metrics
template <bool PER>
__device__ __forceinline__ float point_d2(float qx, float qy, float qz, float px, float py, float pz,
                                          float L) {
    float dx = px - qx, dy = py - qy, dz = pz - qz;
    if constexpr (PER) {
        // min(d^2, (d-L)^2, (d+L)^2) == (min(|d|, |d-L|, |d+L|))^2 exactly
        dx = fminf(fminf(fabsf(dx), fabsf(dx - L)), fabsf(dx + L));
        dy = fminf(fminf(fabsf(dy), fabsf(dy - L)), fabsf(dy + L));
        dz = fminf(fminf(fabsf(dz), fabsf(dz - L)), fabsf(dz + L));
    }
    float a = dx * dx, b = dy * dy, c = dz * dz;
    return (a + b) + c;
}

template <bool PER>
__device__ __forceinline__ float box_axis(float p, float lo, float hi, float L) {
    if constexpr (PER) {
        // kdtree.hpp:93-103
        float below = fminf(lo - p, (p + L) - hi);
        float above = fminf(p - hi, (lo + L) - p);
        float m = p < lo ? below : (p > hi ? above : 0.0f);
        return m * m;
    } else {
        // kdtree.hpp:39-41
        float dl = fmaxf(lo - p, 0.0f), dr = fmaxf(p - hi, 0.0f);
        float a = dl * dl, b = dr * dr;
        return a + b;
    }
}

template <bool PER>
__device__ __forceinline__ float box_d2(float qx, float qy, float qz, const float b[6], float L) {
    float r = box_axis<PER>(qx, b[0], b[1], L);
    r += box_axis<PER>(qy, b[2], b[3], L);
    r += box_axis<PER>(qz, b[4], b[5], L);
    return r;
}

// Same d2 bits as point_d2 with fewer instructions, for |x - q| <= L per axis
// (both points in [0, L]): fl(d - L) = -fl(L - d) exactly, and of the three
// images only |d| and L - |d| can be the smallest, so min(|d|, L - |d|) is the
// reference's per-axis minimum before squaring (and min commutes with the
// monotone square).  Callers use it only for queries inside the periodic box;
// queries outside it are answered by the reference-exact kernel.
template <bool PER>
__device__ __forceinline__ float point_d2_fast(float qx, float qy, float qz, float px, float py,
                                               float pz, float L) {
    float dx = px - qx, dy = py - qy, dz = pz - qz;
    if constexpr (PER) {
        dx = fminf(fabsf(dx), L - fabsf(dx));
        dy = fminf(fabsf(dy), L - fabsf(dy));
        dz = fminf(fabsf(dz), L - fabsf(dz));
    }
    float a = dx * dx, b = dy * dy, c = dz * dz;
    return (a + b) + c;
}

// Lower bound of the squared distance from q to any point of the box, for the
// packet kernels' pruning (not the reference's box_distance, whose exact bits
// only the reference-exact kernel needs).  Per axis, a = lo - q, b = q - hi:
// non-periodic max(a, b, 0); periodic the shorter way round,
// med3(max(a, b), L + min(a, b), 0) (L + min(a, b) >= 0 for q, lo, hi in
// [0, L]).  Each term is monotone in the same roundings point_d2_fast uses
// (fl(L + (q - hi)) = fl(L - (hi - q))), so it never exceeds the d2 of a point
// inside the box.
template <bool PER>
__device__ __forceinline__ float box_lb_axis(float p, float lo, float hi, float L) {
    const float a = lo - p, b = p - hi;
    float m;
    if constexpr (PER)
        m = __builtin_amdgcn_fmed3f(fmaxf(a, b), L + fminf(a, b), 0.0f);
    else
        m = fmaxf(fmaxf(a, b), 0.0f);
    return m * m;
}

template <bool PER>
__device__ __forceinline__ float box_lb2(float qx, float qy, float qz, const float b[6], float L) {
    float r = box_lb_axis<PER>(qx, b[0], b[1], L);
    r += box_lb_axis<PER>(qy, b[2], b[3], L);
    r += box_lb_axis<PER>(qz, b[4], b[5], L);
    return r;
}

// Every point p of the box lies within L/2 of q on every axis: then the
// periodic per-axis minimum min(d^2, (L - |d|)^2) (the reference's
// min(d^2, (d-L)^2, (d+L)^2), kdtree.hpp:72-84) is d^2 itself with the same
// bits, since |fl(p - q)| <= max(|fl(lo - q)|, |fl(hi - q)|) <= L/2 <= fl(L - |d|)
// (monotone rounding; L/2 is exact).  So the plain formula may replace it.
__device__ __forceinline__ bool wrap_free(float qx, float qy, float qz, const float b[6], float L) {
    const float h = 0.5f * L;
    return fmaxf(fabsf(b[0] - qx), fabsf(b[1] - qx)) <= h &&
           fmaxf(fabsf(b[2] - qy), fabsf(b[3] - qy)) <= h &&
           fmaxf(fabsf(b[4] - qz), fabsf(b[5] - qz)) <= h;
}

// ------------------------------------------------------------------ register sorting networks
template <int N, bool IDX = true>
__device__ __forceinline__ void ce(float (&d)[N], uint32_t (&i)[N], int a, int b) {
    // ascending: d[a] <= d[b]
    float da = d[a], db = d[b];
    if constexpr (!IDX) { // distances only (timing experiments)
        d[a] = fminf(da, db);
        d[b] = fmaxf(da, db);
        return;
    }
    bool sw = db < da;
    d[a] = sw ? db : da;
    d[b] = sw ? da : db;
    uint32_t ia = i[a], ib = i[b];
    i[a] = sw ? ib : ia;
    i[b] = sw ? ia : ib;
}

template <int N, bool IDX = true>
__device__ __forceinline__ void bitonic_sort(float (&d)[N], uint32_t (&i)[N]) {
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
            for (int a = 0; a < N; ++a) {
                int b = a ^ stride;
                if (b > a) {
                    if ((a & size) == 0)
                        ce<N, IDX>(d, i, a, b);
                    else
                        ce<N, IDX>(d, i, b, a);
                    if ((a & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// sched_barrier between groups of compare-exchanges: without it the scheduler
// hoists a whole stage's compares and the live masks/temporaries push the
// kernel past the VGPR budget of the occupancy it needs
template <int N, bool IDX = true>
__device__ __forceinline__ void bitonic_merge(float (&d)[N], uint32_t (&i)[N]) {
#pragma unroll
    for (int stride = N >> 1; stride > 0; stride >>= 1) {
#pragma unroll
        for (int a = 0; a < N; ++a) {
            int b = a ^ stride;
            if (b > a) {
                ce<N, IDX>(d, i, a, b);
                if ((a & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ------------------------------------------------------------------ packet traversal
struct WaveStack {
    uint32_t node;
    float b0, b1, b2, b3, b4, b5;
};

// push: the lane whose id equals the stack pointer takes the entry
#define NBKD_PUSH(SP, NODE, BX)                                                                    \
    do {                                                                                           \
        const bool me_ = lane == (SP);                                                             \
        stk.node = me_ ? (NODE) : stk.node;                                                        \
        stk.b0 = me_ ? (BX)[0] : stk.b0;                                                           \
        stk.b1 = me_ ? (BX)[1] : stk.b1;                                                           \
        stk.b2 = me_ ? (BX)[2] : stk.b2;                                                           \
        stk.b3 = me_ ? (BX)[3] : stk.b3;                                                           \
        stk.b4 = me_ ? (BX)[4] : stk.b4;                                                           \
        stk.b5 = me_ ? (BX)[5] : stk.b5;                                                           \
        ++(SP);                                                                                    \
    } while (0)

__device__ __forceinline__ float rdlane(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(uint32_t, v), l));
}


} // namespace dev
} // namespace nbkd
