// WRITE_SIZE / FETCH_SIZE calibration for the store and load shapes of this
// code: each kernel moves a KNOWN number of bytes in one
// access shape, so counter / known is the counter's scale for that shape.
//
//   store16_line   16 B per lane, contiguous (the guide's exact case)
//   store4_line    4 B per lane, contiguous: knn_select's whole-row stores
//                  (store_rows: 32 lanes x 4 B = one 128-B row per half wave)
//   store8_line    8 B per lane, contiguous (uint2)
//   col8_append    the collect kernel's candidate columns: per wave 64 rows of
//                  16 x 8-B slots (one 128-B line per row), filled one slot per
//                  step by every lane (8-B stores 128 B apart), with streamed
//                  loads between steps (leaf staging) that evict lines early
//   sparse8        one 8-B store per 128-B line (lines never completed)
//   sparse4        one 4-B store per 128-B line
//   scatter4       4-B stores at a random permutation (ball count scatter)
//   load16_line    16 B per lane, contiguous loads (the guide's x2 case)
//   load4_line     4 B per lane, contiguous loads
//   lds4_line      global_load_lds 4 B per lane (the collect kernel's staging)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/calib/pmc_calib scripts/calib/pmc_calib.hip
// Run:   scripts/calib/pmc_calib > known.json, under rocprofv3 --pmc WRITE_SIZE
//        (and, separately, FETCH_SIZE); scripts/calib/summarize.py joins them.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr size_t BIG = size_t(1) << 30; // 1 GiB buffers: 4x the 256-MiB Infinity Cache

__global__ void store16_line(uint4 *o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void store8_line(uint2 *o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = make_uint2((uint32_t)i, 7u);
}
__global__ void store4_line(uint32_t *o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = (uint32_t)i;
}
// one 8-B (or 4-B) store per 128-B line
__global__ void sparse8(uint2 *o, size_t lines) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
        o[i * 16] = make_uint2((uint32_t)i, 5u);
}
__global__ void sparse4(uint32_t *o, size_t lines) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
        o[i * 32] = (uint32_t)i;
}
__global__ void scatter4(uint32_t *o, const uint32_t *perm, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[perm[i]] = (uint32_t)i;
}
// candidate columns: wave w owns SLOTS/16 blocks of 64 rows x 128 B; at step s
// every lane writes slot s of its row; between steps the wave streams LOADB
// bytes of `src` (counted separately as fetch, never stored)
template <int SLOTS, int LOADB>
__global__ void col8_append(uint2 *col, const uint4 *src, size_t src_n, uint32_t *sink) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    uint2 *c = col + wave * (size_t)SLOTS * 64;
    uint32_t acc = 0;
    size_t sp = (wave * 977) % (src_n / 64) * 64;
    for (int s = 0; s < SLOTS; ++s) {
        c[((s >> 4) * 64 + lane) * 16 + (s & 15)] = make_uint2((uint32_t)s, (uint32_t)wave);
#pragma unroll
        for (int b = 0; b < LOADB / 1024; ++b) { // 1 KB per wave per iteration
            const uint4 v = src[(sp + lane) % src_n];
            acc += v.x;
            sp += 64;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc; // keeps the loads (never true)
}
__global__ void load16_line(const uint4 *a, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void load4_line(const uint32_t *a, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += a[i];
    if (acc == 0x12345678u) sink[0] = acc;
}
typedef __attribute__((address_space(1))) void *gas_ptr;
typedef __attribute__((address_space(3))) void *las_ptr;
__global__ void lds4_line(const uint32_t *a, size_t n, uint32_t *sink) {
    __shared__ uint32_t buf[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (size_t base = (blockIdx.x * (size_t)blockDim.x + (size_t)w * 64); base < n;
         base += (size_t)gridDim.x * blockDim.x) {
        __builtin_amdgcn_global_load_lds((gas_ptr)(a + base + lane), (las_ptr)buf[w], 4, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70); // vmcnt(0)
        acc += buf[w][lane ^ 1];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    void *a, *b, *sinkp;
    CK(hipMalloc(&a, BIG));
    CK(hipMalloc(&b, BIG));
    CK(hipMalloc(&sinkp, 256));
    CK(hipMemset(b, 1, BIG));
    CK(hipMemset(a, 0, BIG));
    uint32_t *sink = (uint32_t *)sinkp;
    const int grid = 256 * 8 * 4, tb = 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\n");
    bool first = true;
    auto report = [&](const char *name, double wbytes, double rbytes, float ms) {
        printf("%s \"%s\": {\"write_bytes\": %.0f, \"read_bytes\": %.0f, \"ms\": %.4f}\n",
               first ? "" : ",", name, wbytes, rbytes, ms);
        first = false;
    };
#define RUN(NAME, WB, RB, LAUNCH)                                                                  \
    do {                                                                                           \
        LAUNCH;                                                                                    \
        CK(hipDeviceSynchronize());                                                                \
        CK(hipEventRecord(e0));                                                                    \
        LAUNCH;                                                                                    \
        CK(hipEventRecord(e1));                                                                    \
        CK(hipEventSynchronize(e1));                                                               \
        float ms_;                                                                                 \
        CK(hipEventElapsedTime(&ms_, e0, e1));                                                     \
        report(NAME, WB, RB, ms_);                                                                 \
    } while (0)
    // every kernel is launched twice (warm, timed): the counters are per dispatch
    RUN("store16_line", (double)BIG, 0.0, (store16_line<<<grid, tb>>>((uint4 *)a, BIG / 16)));
    RUN("store8_line", (double)BIG, 0.0, (store8_line<<<grid, tb>>>((uint2 *)a, BIG / 8)));
    RUN("store4_line", (double)BIG, 0.0, (store4_line<<<grid, tb>>>((uint32_t *)a, BIG / 4)));
    RUN("sparse8", (double)(BIG / 128) * 8, 0.0, (sparse8<<<grid, tb>>>((uint2 *)a, BIG / 128)));
    RUN("sparse4", (double)(BIG / 128) * 4, 0.0, (sparse4<<<grid, tb>>>((uint32_t *)a, BIG / 128)));
    {
        const size_t n = size_t(64) << 20; // 64 Mi counts (256 MB) at a random permutation
        std::vector<uint32_t> perm(n);
        for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
        uint64_t s = 88172645463325252ull;
        for (size_t i = n - 1; i > 0; --i) {
            s ^= s << 13;
            s ^= s >> 7;
            s ^= s << 17;
            std::swap(perm[i], perm[s % (i + 1)]);
        }
        CK(hipMemcpy(b, perm.data(), n * 4, hipMemcpyHostToDevice));
        RUN("scatter4", (double)n * 4, (double)n * 4, (scatter4<<<grid, tb>>>((uint32_t *)a, (const uint32_t *)b, n)));
        CK(hipMemset(b, 1, BIG));
    }
    {
        // 48 slots per row (3 blocks) per wave; waves sized so the columns fill 512 MiB
        constexpr int SL = 48;
        const size_t waves = (size_t(512) << 20) / (SL * 64 * 8);
        const int g = (int)(waves * 64 / tb);
        RUN("col8_append_noload", (double)waves * 64 * SL * 8, 0.0,
            (col8_append<SL, 0><<<g, tb>>>((uint2 *)a, (const uint4 *)b, BIG / 16, sink)));
        RUN("col8_append_4k", (double)waves * 64 * SL * 8, (double)waves * SL * 4096,
            (col8_append<SL, 4096><<<g, tb>>>((uint2 *)a, (const uint4 *)b, BIG / 16, sink)));
    }
    RUN("load16_line", 0.0, (double)BIG, (load16_line<<<grid, tb>>>((const uint4 *)b, BIG / 16, sink)));
    RUN("load4_line", 0.0, (double)BIG, (load4_line<<<grid, tb>>>((const uint32_t *)b, BIG / 4, sink)));
    RUN("lds4_line", 0.0, (double)BIG, (lds4_line<<<grid, tb>>>((const uint32_t *)b, BIG / 4, sink)));
    printf("}\n");
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sinkp));
    return 0;
}
