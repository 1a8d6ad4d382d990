// Throughput of the CT butterfly sequence alone (glasm::ct_bfly_x4, the NTT kernels' inner op)
// at a chosen occupancy, with no memory traffic: 32 elements per thread in VGPRs run the five
// register stages of a tail phase over and over.  It separates the butterfly's own issue rate
// from the kernels' load / LDS / barrier overheads.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I era-boojum_amd/csrc -o tools/bfly_bench tools/bfly_bench.hip
// Prints one JSON line per occupancy: butterflies/s and the fraction of the issue-slot model
// (slots per butterfly from the static census of this kernel's loop body).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "gl_asm.hpp"

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                   \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

constexpr int ITERS = 64;

__device__ __forceinline__ constexpr int pair_lo(int q, int hk) { return (q / hk) * 2 * hk + (q % hk); }

__device__ __forceinline__ void bfly4(uint64_t* x, int i0, int i1, int i2, int i3, int h, const uint64_t* w) {
    uint64_t A[4], C[4];
    glasm::ct_bfly_x4((uint32_t)x[i0], (uint32_t)(x[i0] >> 32), (uint32_t)x[i0 + h], (uint32_t)(x[i0 + h] >> 32),
                      (uint32_t)w[0], (uint32_t)(w[0] >> 32), A[0], C[0], (uint32_t)x[i1], (uint32_t)(x[i1] >> 32),
                      (uint32_t)x[i1 + h], (uint32_t)(x[i1 + h] >> 32), (uint32_t)w[1], (uint32_t)(w[1] >> 32), A[1],
                      C[1], (uint32_t)x[i2], (uint32_t)(x[i2] >> 32), (uint32_t)x[i2 + h],
                      (uint32_t)(x[i2 + h] >> 32), (uint32_t)w[2], (uint32_t)(w[2] >> 32), A[2], C[2],
                      (uint32_t)x[i3], (uint32_t)(x[i3] >> 32), (uint32_t)x[i3 + h], (uint32_t)(x[i3 + h] >> 32),
                      (uint32_t)w[3], (uint32_t)(w[3] >> 32), A[3], C[3]);
    x[i0] = A[0]; x[i0 + h] = C[0];
    x[i1] = A[1]; x[i1 + h] = C[1];
    x[i2] = A[2]; x[i2 + h] = C[2];
    x[i3] = A[3]; x[i3 + h] = C[3];
}

template <int HK>
__device__ __forceinline__ void stage(uint64_t* x, const uint64_t* w) {
#pragma unroll
    for (int b = 0; b < 4; b++)
        bfly4(x, pair_lo(4 * b, HK), pair_lo(4 * b + 1, HK), pair_lo(4 * b + 2, HK), pair_lo(4 * b + 3, HK), HK,
              w + 4 * b);
}

__global__ __launch_bounds__(256, 2) void bfly_kernel(uint64_t* out, uint64_t seed) {
    extern __shared__ uint64_t occupancy_limiter[];
    uint64_t x[32], w[16];
#pragma unroll
    for (int k = 0; k < 32; k++) x[k] = (seed + threadIdx.x) * (2 * k + 1);
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = (seed ^ 0x9e3779b97f4a7c15ull) * (k + 3) % 0xffffffff00000001ull;
    for (int i = 0; i < ITERS; i++) {
        stage<16>(x, w);
        stage<8>(x, w);
        stage<4>(x, w);
        stage<2>(x, w);
        stage<1>(x, w);
    }
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) acc ^= x[k];
    if (threadIdx.x == 0) occupancy_limiter[0] = acc;
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CHECK(hipFuncSetAttribute((const void*)bfly_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    // dynamic LDS per block sets the blocks per CU (160 KB LDS): 1 block = 1 wave per SIMD
    const int lds_for[] = {0, 150 * 1024, 70 * 1024, 50 * 1024, 38 * 1024};
    for (int waves = 1; waves <= 4; waves++) {
        const int blocks = cus * waves * 8;
        uint64_t* out;
        CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
        hipLaunchKernelGGL(bfly_kernel, dim3(blocks), dim3(256), lds_for[waves], 0, out, 7ull);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; r++)
            hipLaunchKernelGGL(bfly_kernel, dim3(blocks), dim3(256), lds_for[waves], 0, out, 7ull);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        const double bflies = (double)blocks * 256 * ITERS * 5 * 16;
        printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"butterflies_per_s\": %.4e}\n", waves, ms, bflies / (ms * 1e-3));
        CHECK(hipFree(out));
    }
    return 0;
}
