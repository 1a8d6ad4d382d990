// Does sustained compute slow the SDMA device-to-host copies that follow it, and does a kernel
// copy (CUs storing straight to pinned host memory) avoid that?  Not product code.
// build: hipcc -O2 --offload-arch=gfx950 -I include -o tools/d2h_after_compute_probe tools/d2h_after_compute_probe.cpp
//        -L era-boojum_amd/boojum_amd -lboojum_mi355x
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include "boojum_mi355x.h"

__global__ void copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double sdma(void* slot, const char* d, hipStream_t st) {
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 16; i++) hipMemcpyAsync(slot, d + ((size_t)i << 26), 64 << 20, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    return 1.0 * (1 << 30) / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 1e9;
}

static double kcopy(void* slot, const char* d, hipStream_t st, int blocks) {
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 16; i++)
        copy_kernel<<<blocks, 256, 0, st>>>((uint4*)slot, (const uint4*)(d + ((size_t)i << 26)), (64 << 20) / 16);
    hipStreamSynchronize(st);
    return 1.0 * (1 << 30) / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 1e9;
}

int main() {
    const uint32_t log_n = 20, c = 128, log_d = 1, cap = 16;
    const size_t n = 1 << log_n, nl = n << log_d;
    uint64_t *tr, *scratch, *lde, *lv, *nd;
    hipMalloc(&tr, 8 * n * c);
    hipMalloc(&scratch, 8 * n * c);
    hipMalloc(&lde, 8 * nl * c);
    hipMalloc(&lv, 32 * nl);
    hipMalloc(&nd, 32 * nl);
    bj_fill_synthetic_d(tr, c, n, log_n, 42, 0, nullptr);
    char* d;
    hipMalloc(&d, 1 << 30);
    hipMemset(d, 1, 1 << 30);
    void* slot;
    hipHostMalloc(&slot, 64 << 20, 0);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    printf("{\"idle\": true, \"sdma_GBs\": %.1f, \"kernel_copy_GBs_64blk\": %.1f, \"kernel_copy_GBs_512blk\": %.1f}\n",
           sdma(slot, d, st), kcopy(slot, d, st, 64), kcopy(slot, d, st, 512));
    for (int i = 0; i < 5; i++) bj_lde_commit_d(tr, c, n, log_n, log_d, cap, scratch, lde, lv, nd, nullptr, nullptr);
    printf("{\"after_compute\": true, \"sdma_GBs\": %.1f, \"kernel_copy_GBs_64blk\": %.1f, \"kernel_copy_GBs_512blk\": %.1f}\n",
           sdma(slot, d, st), kcopy(slot, d, st, 64), kcopy(slot, d, st, 512));
    for (int i = 0; i < 5; i++) bj_lde_commit_d(tr, c, n, log_n, log_d, cap, scratch, lde, lv, nd, nullptr, nullptr);
    printf("{\"after_compute_kernel_first\": true, \"kernel_copy_GBs_512blk\": %.1f, \"sdma_GBs\": %.1f}\n",
           kcopy(slot, d, st, 512), sdma(slot, d, st));
    return 0;
}
