// Microbenchmark: issue cost of the 32-bit integer VALU forms the Goldilocks arithmetic
// uses on gfx950 (v_mad_u64_u32, v_mul_lo_u32, v_mul_hi_u32, v_add_co_u32/v_addc_co_u32,
// v_lshlrev_b64) and of a full Goldilocks multiply, plus the Poseidon2 permutation rate.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench_valu tools/microbench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../era-boojum_amd/csrc/gl.hpp"
#include "../era-boojum_amd/csrc/poseidon2.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t acc0 = a, acc1 = b, acc2 = a ^ b, acc3 = a + b;
    for (int i = 0; i < ITERS; i++) {
        acc0 = (uint64_t)(uint32_t)acc0 * b + acc1;
        acc1 = (uint64_t)(uint32_t)acc1 * a + acc2;
        acc2 = (uint64_t)(uint32_t)acc2 * b + acc3;
        acc3 = (uint64_t)(uint32_t)acc3 * a + acc0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 ^ acc1 ^ acc2 ^ acc3;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint32_t x0 = a, x1 = b, x2 = a ^ b, x3 = a + b;
    for (int i = 0; i < ITERS; i++) {
        x0 = x0 * b; x1 = x1 * a; x2 = x2 * b; x3 = x3 * a;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
}

__global__ void k_add64(uint64_t* out, uint32_t seed) {
    uint64_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t x0 = a, x1 = b, x2 = a ^ b, x3 = a + b;
    for (int i = 0; i < ITERS; i++) {
        x0 += x1; x1 += x2; x2 += x3; x3 += x0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
}

__global__ void k_glmul(uint64_t* out, uint32_t seed) {
    uint64_t a = (uint64_t)threadIdx.x * 0x9E3779B97F4A7C15ULL ^ seed, b = blockIdx.x + 0x12345678ULL * seed;
    uint64_t x0 = a, x1 = b, x2 = a ^ b, x3 = a + b;
    for (int i = 0; i < ITERS / 4; i++) {
        x0 = gl::mul(x0, b); x1 = gl::mul(x1, a); x2 = gl::mul(x2, b); x3 = gl::mul(x3, a);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
}

__global__ __launch_bounds__(256) void k_perm(uint64_t* out, uint32_t seed, int reps) {
    uint64_t s[12];
    for (int i = 0; i < 12; i++) s[i] = (uint64_t)(threadIdx.x + i) * 0x9E3779B97F4A7C15ULL ^ seed ^ blockIdx.x;
    for (int r = 0; r < reps; r++) p2::permute(s);
    uint64_t x = 0;
    for (int i = 0; i < 12; i++) x ^= s[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <typename F>
float time_kernel(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < 5; i++) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8, threads = 256;
    uint64_t* out;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 8));
    const double lanes = (double)blocks * threads;
    const double wave_instr_peak = 256.0 * 4 * 2.4e9 / 2;  // wave64 VALU instr/s at full rate
    struct { const char* name; void (*k)(uint64_t*, uint32_t); double ops_per_iter; } tests[] = {
        {"v_mad_u64_u32 (dependent x4)", k_mad64, 4},
        {"v_mul_lo_u32 (x4)", k_mullo, 4},
        {"u64 add (x4)", k_add64, 4},
    };
    for (auto& t : tests) {
        float ms = time_kernel([&] { hipLaunchKernelGGL(t.k, dim3(blocks), dim3(threads), 0, 0, out, 7u); });
        double per_s = lanes * ITERS * t.ops_per_iter / (ms * 1e-3);
        printf("%-32s %8.3f ms  %.3e lane-ops/s  = %.3f of full-rate wave-instr peak\n", t.name, ms, per_s,
               per_s / 64 / wave_instr_peak);
    }
    {
        float ms = time_kernel([&] { hipLaunchKernelGGL(k_glmul, dim3(blocks), dim3(threads), 0, 0, out, 7u); });
        double per_s = lanes * ITERS / (ms * 1e-3);
        printf("%-32s %8.3f ms  %.3e gl-mul/s  (%.1f full-rate instr-slots per mul)\n", "goldilocks mul", ms, per_s,
               64 * wave_instr_peak / per_s);
    }
    for (int reps : {8}) {
        float ms = time_kernel([&] { hipLaunchKernelGGL(k_perm, dim3(blocks), dim3(threads), 0, 0, out, 7u, reps); });
        double per_s = lanes * reps / (ms * 1e-3);
        printf("%-32s %8.3f ms  %.3e perm/s  (%.0f full-rate instr-slots per perm)\n", "poseidon2 permutation", ms,
               per_s, 64 * wave_instr_peak / per_s);
    }
    CHECK(hipFree(out));
    return 0;
}
