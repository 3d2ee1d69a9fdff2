// Device helpers shared by the packet kNN kernels (knn_packet.hip,
// knn_collect.hip): direct-to-LDS loads, wave-local sync, the scalar-cache
// view of the node table, LDS-staged row stores and the fallback listing.
#pragma once

#include "metric.hpp"

namespace nbkd {
namespace dev {

typedef __attribute__((address_space(1))) const void *gas_ptr;
typedef __attribute__((address_space(3))) void *las_ptr;

// lanes < n copy src[lane] into dst[lane] (LDS) without passing through VGPRs
__device__ __forceinline__ void glds_f32(const float *src, float *dst, int lane, uint32_t n) {
    if ((uint32_t)lane < n)
        __builtin_amdgcn_global_load_lds((gas_ptr)(src + lane), (las_ptr)dst, 4, 0, 0);
}

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt untouched): the direct-to-LDS loads have landed
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

constexpr int pow2_floor(int v) { return v >= 64 ? 64 : v >= 32 ? 32 : v >= 16 ? 16 : v >= 8 ? 8 : 4; }
constexpr int pow2_ceil(int v) { return v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : v <= 32 ? 32 : 64; }

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

// Staged registers j = 0..CC-1 of the 64 lanes (word (j, row) at j*64 + (row ^ j))
// are output columns c = c0 + j of row `row` (query rowq[row]; 0xFFFFFFFF = no
// query); columns outside [0, k) are skipped.  Consecutive lanes store
// consecutive columns of a row: whole rows per store instruction.
// remap != nullptr: the staged words are tree positions, stored as remap[pos]
// (0xFFFFFFFF = no neighbour, stored as is).
template <int CC>
__device__ __forceinline__ void store_rows(const uint32_t *stage, const uint32_t *rowq,
                                           uint32_t *__restrict__ dst, int k, int c0, int lane,
                                           const uint32_t *__restrict__ remap = nullptr) {
    const int jlo = c0 < 0 ? -c0 : 0;           // first staged register in [0, k)
    const int nc = min(CC, k - c0) - jlo;       // staged registers in [0, k)
    if (nc <= 0) return;
    if (nc == CC) {
        // every staged register is an output column (jlo == 0): the row and
        // column of element e = it*64 + lane are shifts of a constant, and the
        // unrolled iterations keep their LDS reads in flight together (the
        // generic loop below divides by a runtime nc and waits on each read)
        constexpr int RPI = 64 / CC; // rows per store instruction
        const int j = lane % CC, r0 = lane / CC;
#pragma unroll 8
        for (int it = 0; it < CC; ++it) {
            const int row = it * RPI + r0;
            const uint32_t qr = rowq[row];
            uint32_t v = stage[j * 64 + (row ^ j)];
            if (qr != 0xFFFFFFFFu) {
                if (remap && v != 0xFFFFFFFFu) v = remap[v];
                dst[(size_t)qr * k + c0 + j] = v;
            }
        }
        return;
    }
    for (int e = lane; e < 64 * nc; e += 64) {
        const int row = e / nc, j = jlo + (e - row * nc);
        const uint32_t qr = rowq[row];
        if (qr != 0xFFFFFFFFu) {
            uint32_t v = stage[j * 64 + (row ^ j)];
            if (remap && v != 0xFFFFFFFFu) v = remap[v];
            dst[(size_t)qr * k + c0 + j] = v;
        }
    }
}

// a seeded lane whose k-th slot still holds the sentinel id found fewer than k
// points inside its seed radius: list it for the exact kernel.  Periodic
// queries outside [0, L]^3 are already listed (outside_box_kernel), so each
// query is listed at most once.
template <bool PER>
__device__ __forceinline__ void knn_fail_check(bool valid, bool seeded, uint32_t kth_id, float qx,
                                               float qy, float qz, float L, uint32_t qo,
                                               uint32_t *fail_list, uint32_t *fail_count) {
    const bool listed =
        PER && !(qx >= 0.0f && qx <= L && qy >= 0.0f && qy <= L && qz >= 0.0f && qz <= L);
    if (valid && seeded && !listed && kth_id == 0xFFFFFFFFu)
        fail_list[atomicAdd(fail_count, 1u)] = qo;
}


} // namespace dev
} // namespace nbkd
