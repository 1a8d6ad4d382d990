// Leaf grids of k x 65536 leaves (k waves per SIMD on 256 CUs x 4 SIMDs), the product's leaf
// kernel (csrc/merkle.hip) over 128 columns (16 permutations per leaf): does a grid's time step
// with ceil(k / 3) (three leaf waves per SIMD, each wave's chain latency-bound, so a partly
// filled last round costs a whole one) or grow with k?  The per-rank leaf grids of the collective
// commit hold 32 (C3 at G = 8) or 64 (G = 4) waves per SIMD.
// With a third argument "stride": k = 32 (2^21 leaves, C3 at G = 8) read with column strides
// 2^21 (the collective's LDE buffer), 2^21 + 64 / 512 / 4096 words, 2^22 and 2^24 words.
// With "after": the k = 32 grid timed alone and right behind an HBM-bound copy of 4 x 2 GiB
// (~4 ms, as the collective's leaf grids follow the LDE's final pass): a clock that drops while
// HBM streams and climbs back only after some time would show here.
// usage: leaf_tail_probe [cols] [reps] [stride|after]; one line per (k, form), stride or order
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/leaf_tail_probe tools/leaf_tail_probe.hip
#include "../era-boojum_amd/csrc/merkle.hip"
#include <cstdio>
#include <cstring>

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
    const bool by_stride = argc > 3 && !strcmp(argv[3], "stride");
    const bool after = argc > 3 && !strcmp(argv[3], "after");
    const size_t unit = 65536, kmax = 36, nmax = kmax * unit;
    uint64_t *src, *state, *out;
    if (after) {
        const size_t n = (size_t)1 << 21, cw = (size_t)1 << 28;  // 2 GiB copies
        uint64_t *a0, *a1;
        CHECK(hipMalloc(&src, n * cols * 8));
        CHECK(hipMalloc(&state, n * 32));
        CHECK(hipMalloc(&out, n * 32));
        CHECK(hipMalloc(&a0, cw * 8));
        CHECK(hipMalloc(&a1, cw * 8));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, n * cols);
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, state, n * 4);
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a0, cw);
        hipEvent_t a, b, c0;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        CHECK(hipEventCreate(&c0));
        for (int pass = 0; pass < 3; pass++)
            for (int behind = 0; behind < 2; behind++) {
                float best = 1e30f, sum = 0, copy_ms = 0;
                for (int r = 0; r < reps; r++) {
                    CHECK(hipDeviceSynchronize());
                    if (behind) {
                        CHECK(hipEventRecord(c0));
                        for (int k = 0; k < 4; k++)
                            CHECK(hipMemcpyAsync(k & 1 ? a0 : a1, k & 1 ? a1 : a0, cw * 8, hipMemcpyDeviceToDevice, 0));
                    }
                    CHECK(hipEventRecord(a));
                    CHECK(bj::launch_leaves_partial(src, n, cols, n, state, out, false, 0));
                    CHECK(hipEventRecord(b));
                    CHECK(hipEventSynchronize(b));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, a, b));
                    if (behind) {
                        float cm;
                        CHECK(hipEventElapsedTime(&cm, c0, a));
                        copy_ms += cm;
                    }
                    best = ms < best ? ms : best;
                    sum += ms;
                }
                printf("leaf_after pass=%d behind_copy=%d cols=%u leaves=%zu best_ms=%.4f mean_ms=%.4f copy_ms=%.3f\n",
                       pass, behind, cols, n, best, sum / reps, copy_ms / reps);
                fflush(stdout);
            }
        return 0;
    }
    if (by_stride) {
        const size_t n = (size_t)1 << 21, strides[] = {n, n + 64, n + 512, n + 4096, 2 * n, 8 * n};
        CHECK(hipMalloc(&src, 8 * n * cols * 8));
        CHECK(hipMalloc(&state, n * 32));
        CHECK(hipMalloc(&out, n * 32));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, 8 * n * cols);
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, state, n * 4);
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int pass = 0; pass < 2; pass++)
            for (size_t cs : strides) {
                CHECK(bj::launch_leaves_partial(src, cs, cols, n, state, out, false, 0));
                CHECK(hipDeviceSynchronize());
                float best = 1e30f;
                for (int r = 0; r < reps; r++) {
                    CHECK(hipEventRecord(a));
                    CHECK(bj::launch_leaves_partial(src, cs, cols, n, state, out, false, 0));
                    CHECK(hipEventRecord(b));
                    CHECK(hipEventSynchronize(b));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, a, b));
                    best = ms < best ? ms : best;
                }
                printf("leaf_stride pass=%d cols=%u leaves=%zu col_stride=%zu best_ms=%.4f\n", pass, cols, n, cs, best);
                fflush(stdout);
            }
        return 0;
    }
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
