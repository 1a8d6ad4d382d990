// HBM rates of the streams the G = 2D sender fold moves (lde3_inv_fold_kernel, C3 at G = 8:
// per rank 1 GiB read, 4 GiB written as 8 targets x 512 MiB), without its arithmetic:
//   write : 4 GiB of 16-byte stores, grid-stride;
//   copy1x4 : read 1 GiB, write it 4 times (to 4 regions), 8-byte lanes as the kernel does;
//   fold8 : read 1 GiB in 64 KiB tiles (one block per tile), write 8 targets x (tile / 2) each,
//           buffer stores with a per-target base, the kernel's exact address pattern.
// usage: write_rate_probe [reps]
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/write_rate_probe tools/write_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void write_kernel(uint4* dst, size_t n16) {
    const uint4 v = make_uint4(threadIdx.x, blockIdx.x, 1, 2);
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = v;
}

__global__ __launch_bounds__(256) void copy1x4_kernel(const uint64_t* src, uint64_t* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint64_t v = src[i];
#pragma unroll
        for (int r = 0; r < 4; r++) dst[r * n + i] = v + r;
    }
}

// one block per 8192-word tile, 256 threads x 32 words; 8 targets x 4096 words per tile
__global__ __launch_bounds__(256, 2) void fold8_kernel(const uint64_t* src, uint64_t* dst, size_t target_stride) {
    const uint32_t t = threadIdx.x;
    const size_t tile = blockIdx.x;
    uint64_t x[32];
#pragma unroll
    for (int k = 0; k < 32; k++) x[k] = src[tile * 8192 + t + 256 * k];
    for (uint32_t P = 0; P < 8; P++) {
        uint64_t* d = dst + P * target_stride + tile * 4096;
#pragma unroll
        for (int k = 0; k < 16; k++) d[t + 256 * k] = x[2 * k] + x[2 * k + 1] * (P + 1);
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const size_t n = (size_t)1 << 27;  // 1 GiB of words
    uint64_t *src, *dst;
    CHECK(hipMalloc(&src, n * 8));
    CHECK(hipMalloc(&dst, 4 * n * 8));
    CHECK(hipMemset(src, 1, n * 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int which = 0; which < 3; which++) {
        const char* name = which == 0 ? "write" : which == 1 ? "copy1x4" : "fold8";
        const double bytes = which == 0 ? 4.0 * n * 8 : 5.0 * n * 8;
        auto launch = [&]() {
            if (which == 0) hipLaunchKernelGGL(write_kernel, dim3(256 * 32), dim3(256), 0, 0, (uint4*)dst, n * 4 * 8 / 16);
            else if (which == 1) hipLaunchKernelGGL(copy1x4_kernel, dim3(256 * 32), dim3(256), 0, 0, src, dst, n);
            else hipLaunchKernelGGL(fold8_kernel, dim3((unsigned)(n / 8192)), dim3(256), 0, 0, src, dst, n / 2);
            return hipGetLastError();
        };
        CHECK(launch());
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < reps; r++) {
            CHECK(hipEventRecord(a));
            CHECK(launch());
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        printf("write_rate %s bytes=%.3e best_ms=%.4f TB/s=%.3f\n", name, bytes, best, bytes / best / 1e9);
        fflush(stdout);
    }
    return 0;
}
