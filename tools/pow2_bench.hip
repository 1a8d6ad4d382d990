// Register DFTs with power-of-two twiddles (csrc/ntt_pow2.hpp, tools/gen_ntt_pow2.py):
// 1. correctness of dft{2,4,8,16,32}_{fwd,inv} against the CT network with general twiddles
//    (host, gl.hpp), on random and edge inputs (0, 1, p - 1, p .. 2^64 - 1);
// 2. throughput of one 5-stage register phase two ways, no memory traffic, 2 waves per SIMD:
//    five CT stages of general butterflies (ct_bfly_x4, the kernels' current phase) against a
//    prescale by 32 general factors (mul_x4) + dft32_fwd.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I era-boojum_amd/csrc -o tools/pow2_bench tools/pow2_bench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "ntt_pow2.hpp"

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                   \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

template <int LOGN, bool INV>
__device__ __forceinline__ void dft(uint64_t* x) {
    if constexpr (LOGN == 1) { if constexpr (INV) bj::p2dft::dft2_inv<0>(x); else bj::p2dft::dft2_fwd<0>(x); }
    if constexpr (LOGN == 2) { if constexpr (INV) bj::p2dft::dft4_inv<0>(x); else bj::p2dft::dft4_fwd<0>(x); }
    if constexpr (LOGN == 3) { if constexpr (INV) bj::p2dft::dft8_inv<0>(x); else bj::p2dft::dft8_fwd<0>(x); }
    if constexpr (LOGN == 4) { if constexpr (INV) bj::p2dft::dft16_inv<0>(x); else bj::p2dft::dft16_fwd<0>(x); }
    if constexpr (LOGN == 5) { if constexpr (INV) bj::p2dft::dft32_inv<0>(x); else bj::p2dft::dft32_fwd<0>(x); }
}

template <int LOGN, bool INV>
__global__ void check_kernel(const uint64_t* in, uint64_t* out, int count) {
    constexpr int N = 1 << LOGN;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t x[N];
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = in[(size_t)i * N + k];
    dft<LOGN, INV>(x);
#pragma unroll
    for (int k = 0; k < N; k++) out[(size_t)i * N + k] = gl::canon(x[k]);
}

// host reference: the natural -> bit-reversed CT network, twiddle w_{2^(u+1)}^bitrev_u(g)
static void ref_dft(uint64_t* x, int logn, bool inv) {
    const int n = 1 << logn;
    for (int u = 0; u < logn; u++) {
        const int h = n >> (u + 1);
        uint64_t w = gl::domain_generator(u + 1);
        if (inv) w = gl::inv(w);
        for (int g = 0; g < (1 << u); g++) {
            const uint64_t t = gl::pow(w, gl::bitrev32(g, u));
            for (int j = 0; j < h; j++) {
                const int a = g * 2 * h + j, c = a + h;
                const uint64_t m = gl::mul(x[c], t);
                const uint64_t s = gl::add(gl::canon(x[a]), m), d = gl::sub(gl::canon(x[a]), m);
                x[a] = s;
                x[c] = d;
            }
        }
    }
    for (int k = 0; k < n; k++) x[k] = gl::canon(x[k]);
}

template <int LOGN, bool INV>
int check_one(int count, uint64_t* din, uint64_t* dout, int& bad) {
    const int n = 1 << LOGN;
    std::vector<uint64_t> h((size_t)count * n), r((size_t)count * n);
    uint64_t s = 0x9e3779b97f4a7c15ull ^ (LOGN * 131 + INV);
    const uint64_t edge[] = {0, 1, gl::P - 1, gl::P, gl::P + 1, ~0ull, ~0ull - 1, 0xFFFFFFFFull, 1ull << 32};
    for (size_t i = 0; i < h.size(); i++) {
        s += 0x9e3779b97f4a7c15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        z ^= z >> 31;
        h[i] = (i / n) % 4 == 0 ? edge[(z >> 7) % 9] : z;  // every 4th vector from edge values only
    }
    CHECK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((check_kernel<LOGN, INV>), dim3((count + 255) / 256), dim3(256), 0, 0, din, dout, count);
    CHECK(hipMemcpy(r.data(), dout, r.size() * 8, hipMemcpyDeviceToHost));
    int wrong = 0;
    for (int v = 0; v < count; v++) {
        ref_dft(&h[(size_t)v * n], LOGN, INV);
        for (int k = 0; k < n; k++) wrong += h[(size_t)v * n + k] != r[(size_t)v * n + k];
    }
    printf("{\"check\": \"dft%d_%s\", \"vectors\": %d, \"wrong\": %d}\n", n, INV ? "inv" : "fwd", count, wrong);
    bad += wrong;
    return 0;
}

constexpr int ITERS = 64;

__device__ __forceinline__ constexpr int pair_lo(int q, int hk) { return (q / hk) * 2 * hk + (q % hk); }

template <int HK>
__device__ __forceinline__ void gstage(uint64_t* x, const uint64_t* w) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
        uint64_t A[4], C[4];
        const int i0 = pair_lo(4 * b, HK), i1 = pair_lo(4 * b + 1, HK), i2 = pair_lo(4 * b + 2, HK),
                  i3 = pair_lo(4 * b + 3, HK);
        glasm::ct_bfly_x4((uint32_t)x[i0], (uint32_t)(x[i0] >> 32), (uint32_t)x[i0 + HK], (uint32_t)(x[i0 + HK] >> 32),
                          (uint32_t)w[4 * b], (uint32_t)(w[4 * b] >> 32), A[0], C[0], (uint32_t)x[i1],
                          (uint32_t)(x[i1] >> 32), (uint32_t)x[i1 + HK], (uint32_t)(x[i1 + HK] >> 32),
                          (uint32_t)w[4 * b + 1], (uint32_t)(w[4 * b + 1] >> 32), A[1], C[1], (uint32_t)x[i2],
                          (uint32_t)(x[i2] >> 32), (uint32_t)x[i2 + HK], (uint32_t)(x[i2 + HK] >> 32),
                          (uint32_t)w[4 * b + 2], (uint32_t)(w[4 * b + 2] >> 32), A[2], C[2], (uint32_t)x[i3],
                          (uint32_t)(x[i3] >> 32), (uint32_t)x[i3 + HK], (uint32_t)(x[i3 + HK] >> 32),
                          (uint32_t)w[4 * b + 3], (uint32_t)(w[4 * b + 3] >> 32), A[3], C[3]);
        x[i0] = A[0]; x[i0 + HK] = C[0];
        x[i1] = A[1]; x[i1 + HK] = C[1];
        x[i2] = A[2]; x[i2 + HK] = C[2];
        x[i3] = A[3]; x[i3 + HK] = C[3];
    }
}

__device__ __forceinline__ void mul4(uint64_t* x, const uint64_t* f) {
    uint32_t z0[4], z1[4];
    glasm::mul_x4((uint32_t)x[0], (uint32_t)(x[0] >> 32), (uint32_t)f[0], (uint32_t)(f[0] >> 32), z0[0], z1[0],
                  (uint32_t)x[1], (uint32_t)(x[1] >> 32), (uint32_t)f[1], (uint32_t)(f[1] >> 32), z0[1], z1[1],
                  (uint32_t)x[2], (uint32_t)(x[2] >> 32), (uint32_t)f[2], (uint32_t)(f[2] >> 32), z0[2], z1[2],
                  (uint32_t)x[3], (uint32_t)(x[3] >> 32), (uint32_t)f[3], (uint32_t)(f[3] >> 32), z0[3], z1[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = ((uint64_t)z1[i] << 32) | z0[i];
}

template <bool POW2>
__global__ __launch_bounds__(256, 2) void bench_kernel(uint64_t* out, const uint64_t* __restrict__ tw) {
    extern __shared__ uint64_t occupancy_limiter[];
    uint64_t x[32];
#pragma unroll
    for (int k = 0; k < 32; k++) x[k] = (threadIdx.x + 7) * (2 * k + 1);
    for (int i = 0; i < ITERS; i++) {
        const uint64_t* t = tw + (i & 7) * 80;  // wave-uniform: scalar loads, as in the kernels
        if constexpr (POW2) {
#pragma unroll
            for (int k = 0; k < 32; k += 4) mul4(x + k, t + k);
            bj::p2dft::dft32_fwd<0>(x);
        } else {
            gstage<16>(x, t);
            gstage<8>(x, t + 16);
            gstage<4>(x, t + 32);
            gstage<2>(x, t + 48);
            gstage<1>(x, t + 64);
        }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) acc ^= x[k];
    if (threadIdx.x == 0) occupancy_limiter[0] = acc;
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    uint64_t *din, *dout;
    const int count = 4096;
    CHECK(hipMalloc(&din, (size_t)count * 32 * 8));
    CHECK(hipMalloc(&dout, (size_t)count * 32 * 8));
    int bad = 0;
    if (check_one<1, false>(count, din, dout, bad) || check_one<1, true>(count, din, dout, bad) ||
        check_one<2, false>(count, din, dout, bad) || check_one<2, true>(count, din, dout, bad) ||
        check_one<3, false>(count, din, dout, bad) || check_one<3, true>(count, din, dout, bad) ||
        check_one<4, false>(count, din, dout, bad) || check_one<4, true>(count, din, dout, bad) ||
        check_one<5, false>(count, din, dout, bad) || check_one<5, true>(count, din, dout, bad))
        return 1;
    if (bad) {
        printf("{\"error\": \"%d wrong outputs\"}\n", bad);
        return 2;
    }
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint64_t> tw(8 * 80);
    for (size_t i = 0; i < tw.size(); i++) tw[i] = gl::pow(7, i + 3);
    uint64_t* dtw;
    CHECK(hipMalloc(&dtw, tw.size() * 8));
    CHECK(hipMemcpy(dtw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipFuncSetAttribute((const void*)bench_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute((const void*)bench_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int blocks = cus * 2 * 8;
    uint64_t* out;
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; rep++) {
        for (int pow2 = 0; pow2 < 2; pow2++) {
            auto launch = [&]() {
                if (pow2) hipLaunchKernelGGL(bench_kernel<true>, dim3(blocks), dim3(256), 70 * 1024, 0, out, dtw);
                else hipLaunchKernelGGL(bench_kernel<false>, dim3(blocks), dim3(256), 70 * 1024, 0, out, dtw);
            };
            launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a));
            for (int r = 0; r < 5; r++) launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            ms /= 5;
            const double phases = (double)blocks * 256 * ITERS;  // 32-element 5-stage phases
            printf("{\"variant\": \"%s\", \"ms\": %.3f, \"ns_per_phase_per_lane\": %.4f}\n",
                   pow2 ? "prescale+dft32_pow2" : "5 general CT stages", ms, ms * 1e6 / phases);
        }
    }
    return 0;
}
