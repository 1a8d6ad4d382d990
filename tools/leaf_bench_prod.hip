// The product's own leaf kernel (csrc/merkle.hip, bj::launch_leaves) in the harness of
// tools/leaf_bench.hip: same shape, data and timing, so a same-box comparison separates the
// kernel's code from the commit's environment (buffers from the torch allocator, LDE data).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/leaf_bench_prod tools/leaf_bench_prod.hip
#include "../era-boojum_amd/csrc/merkle.hip"
#include <cstdio>

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
    CHECK(bj::launch_leaves(src, n, cols, n, out, 0));
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(a));
        CHECK(bj::launch_leaves(src, n, cols, n, out, 0));
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
    printf("leaf_bench_prod %s leaves=2^%u cols=%u best_ms=%.3f mean_ms=%.3f checksum=%016llx\n", argc > 3 ? argv[3] : "-",
           log_leaves, cols, best, sum / reps, (unsigned long long)x);
    return 0;
}
