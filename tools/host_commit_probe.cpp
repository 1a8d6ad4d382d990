// bj_lde_commit_h timed from C++ (no Python), C2 geometry, with per-call wall time.
// build: hipcc -O2 --offload-arch=gfx950 -I include -o tools/host_commit_probe tools/host_commit_probe.cpp
//        -L era-boojum_amd/boojum_amd -lboojum_mi355x -Wl,-rpath,$PWD/era-boojum_amd/boojum_amd
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include "boojum_mi355x.h"

int main(int argc, char** argv) {
    const uint32_t log_n = 20, c = 128, log_d = 1, cap = 16;
    const size_t n = 1 << log_n, nl = n << log_d;
    uint64_t* tr = (uint64_t*)malloc(8 * n * c);
    for (size_t i = 0; i < n * c; i++) tr[i] = i * 0x9E3779B97F4A7C15ull >> 1;
    uint64_t* lde = (uint64_t*)malloc(8 * nl * c);
    uint64_t* lv = (uint64_t*)malloc(32 * nl);
    uint64_t* nd = (uint64_t*)malloc(32 * nl);
    uint64_t capo[64];
    memset(lde, 0, 8 * nl * c);
    const bool reg = argc > 1 && argv[1][0] == 'r';
    if (reg) {
        hipHostRegister(tr, 8 * n * c, 0);
        hipHostRegister(lde, 8 * nl * c, 0);
    }
    if (argc > 2) {
        void* d0;
        void* s0;
        hipMalloc(&d0, 1 << 30);
        hipMemset(d0, 1, 1 << 30);
        hipHostMalloc(&s0, 64 << 20, 0);
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 16; i++) hipMemcpy(s0, (char*)d0 + ((size_t)i << 26), 64 << 20, hipMemcpyDeviceToHost);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"before_commit_slot_d2h_GBs\": %.1f}\n", 1.0 * (1 << 30) / dt / 1e9);
    }
    for (int rep = 0; rep < 4; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        int rc = bj_lde_commit_h(tr, c, log_n, log_d, cap, lde, lv, nd, capo);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"rep\": %d, \"rc\": %d, \"registered\": %d, \"ms\": %.1f}\n", rep, rc, reg, dt * 1e3);
    }
    // raw D2H of the same volume from a fresh device buffer into the same host buffer
    void* d;
    hipMalloc(&d, 8 * nl * c);
    for (int rep = 0; rep < 2; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        hipMemcpy(lde, d, 8 * nl * c, hipMemcpyDeviceToHost);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"raw_d2h_GBs\": %.1f}\n", 8.0 * nl * c / dt / 1e9);
    }
    // 64 MiB pieces from a written device buffer into one pinned 64 MiB slot, as pinned_probe
    void* slot;
    hipHostMalloc(&slot, 64 << 20, 0);
    hipMemset(d, 1, 8 * nl * c);
    for (int pre = 0; pre < 4; pre++) {
        if (pre == 2) {
            hipDeviceSynchronize();
            std::this_thread::sleep_for(std::chrono::seconds(2));
        }
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 32; i++) hipMemcpy(slot, (char*)d + ((size_t)i << 26), 64 << 20, hipMemcpyDeviceToHost);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"slot_d2h_GBs\": %.1f}\n", 2.0 * (1 << 30) / dt / 1e9);
    }
    return 0;
}
