// Leaf grids of k x 65536 leaves (k waves per SIMD on 256 CUs x 4 SIMDs), the product's leaf
// kernel (csrc/merkle.hip) over 128 columns (16 permutations per leaf): does a grid's time step
// with ceil(k / 3) (three leaf waves per SIMD, each wave's chain latency-bound, so a partly
// filled last round costs a whole one) or grow with k?  The per-rank leaf grids of the collective
// commit hold 32 (C3 at G = 8) or 64 (G = 4) waves per SIMD.
// usage: leaf_tail_probe [cols] [reps]; one line per (k, kernel form)
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/leaf_tail_probe tools/leaf_tail_probe.hip
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
    const uint32_t cols = argc > 1 ? atoi(argv[1]) : 128;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t unit = 65536, kmax = 36, nmax = kmax * unit;
    uint64_t *src, *state, *out;
    CHECK(hipMalloc(&src, nmax * cols * 8));
    CHECK(hipMalloc(&state, nmax * 32));
    CHECK(hipMalloc(&out, nmax * 32));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, nmax * cols);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, state, nmax * 4);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int form = 0; form < 2; form++) {
        for (size_t k = 28; k <= kmax; k++) {
            const size_t n = k * unit;
            // form 0: a chunk grid in the middle of the column pipeline (state in, state out);
            // form 1: the one-GPU commit's single grid (no state in, digests out)
            auto launch = [&]() {
                return form == 0 ? bj::launch_leaves_partial(src, nmax, cols, n, state, out, false, 0)
                                 : bj::launch_leaves_partial(src, nmax, cols, n, nullptr, out, true, 0);
            };
            CHECK(launch());
            CHECK(hipDeviceSynchronize());
            float best = 1e30f, sum = 0;
            for (int r = 0; r < reps; r++) {
                CHECK(hipEventRecord(a));
                CHECK(launch());
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
                sum += ms;
            }
            printf("leaf_tail form=%s cols=%u k=%zu leaves=%zu best_ms=%.4f mean_ms=%.4f best_us_per_k=%.2f\n",
                   form == 0 ? "partial" : "single", cols, k, n, best, sum / reps, 1e3 * best / k);
            fflush(stdout);
        }
    }
    return 0;
}
