// Leaf-kernel microbenchmark for A/B-ing permutation variants (test tooling, not product):
// the C3 leaf shape (256 columns) over 2^22 leaves, one leaf per lane exactly as
// csrc/merkle.hip's leaf_hash_kernel<false, true>.  The permutation comes from whichever
// poseidon2.hpp the include path names, so several builds of this file time several
// variants on one box; the printed checksum of the digests must agree between them.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I<variant csrc dir> -o <bin> tools/leaf_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "poseidon2.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint64_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        p[i] = z >= 0xFFFFFFFF00000001ULL ? z - 0xFFFFFFFF00000001ULL : z;
    }
}

__global__ __launch_bounds__(256) void leaf(const uint64_t* __restrict__ src, size_t col_stride, uint32_t n_cols,
                                            size_t n_leaves, uint64_t* out) {
    const size_t L = blockIdx.x * (size_t)256 + threadIdx.x;
    if (L >= n_leaves) return;
    const uint64_t* p = src + L;
    p2::State s;
#pragma unroll
    for (int i = 0; i < 12; i++) s.lo[i] = s.hi[i] = 0;
    const uint32_t full = n_cols >> 3;
    uint64_t nxt[8];
#pragma unroll
    for (int i = 0; i < 8; i++) nxt[i] = p[(size_t)i * col_stride];
    for (uint32_t g = 0; g + 1 < full; g++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            s.lo[i] = (uint32_t)nxt[i];
            s.hi[i] = (uint32_t)(nxt[i] >> 32);
        }
        const uint64_t* q = p + (size_t)(g + 1) * 8 * col_stride;
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = q[(size_t)i * col_stride];
        p2::permute<p2::OUT_CAP>(s);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        s.lo[i] = (uint32_t)nxt[i];
        s.hi[i] = (uint32_t)(nxt[i] >> 32);
    }
    p2::permute<p2::OUT_DIGEST>(s);
#pragma unroll
    for (int i = 0; i < 4; i++) out[4 * L + i] = ((uint64_t)s.hi[i] << 32) | s.lo[i];
}

int main(int argc, char** argv) {
    const uint32_t log_leaves = argc > 1 ? atoi(argv[1]) : 22, cols = 256;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t n = (size_t)1 << log_leaves;
    uint64_t *src, *out;
    CHECK(hipMalloc(&src, n * cols * 8));
    CHECK(hipMalloc(&out, n * 32));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, n * cols);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const dim3 g((unsigned)(n / 256));
    hipLaunchKernelGGL(leaf, g, dim3(256), 0, 0, src, n, cols, n, out);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(leaf, g, dim3(256), 0, 0, src, n, cols, n, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        sum += ms;
    }
    uint64_t* h = (uint64_t*)malloc(n * 32);
    CHECK(hipMemcpy(h, out, n * 32, hipMemcpyDeviceToHost));
    uint64_t x = 0;
    for (size_t i = 0; i < 4 * n; i++) x = x * 0x100000001B3ULL ^ (h[i] % 0xFFFFFFFF00000001ULL);
    printf("leaf_bench %s leaves=2^%u cols=%u best_ms=%.3f mean_ms=%.3f checksum=%016llx\n", argc > 3 ? argv[3] : "-",
           log_leaves, cols, best, sum / reps, (unsigned long long)x);
    return 0;
}
