// D2H / H2D rate into pinned host memory by allocation flavour (sizing bj_lde_commit_h's staging
// slots).  Not product code.  build: hipcc -O2 --offload-arch=gfx950 -o tools/pinned_probe tools/pinned_probe.cpp
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double rate(void* host, void* dev, size_t bytes, size_t piece, hipMemcpyKind kind, hipStream_t st) {
    double best = 1e9;
    for (int rep = 0; rep < 4; rep++) {
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (size_t off = 0; off < bytes; off += piece) {
            if (kind == hipMemcpyDeviceToHost)
                hipMemcpyAsync((char*)host + off % (256 << 20), (char*)dev + off, piece, kind, st);
            else
                hipMemcpyAsync((char*)dev + off, (char*)host + off % (256 << 20), piece, kind, st);
        }
        hipStreamSynchronize(st);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt < best) best = dt;
    }
    return bytes / best / 1e9;
}

int main() {
    const size_t total = (size_t)1 << 30, slot = (size_t)256 << 20, piece = (size_t)64 << 20;
    void* dev = nullptr;
    hipMalloc(&dev, total);
    hipMemset(dev, 1, total);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    struct { const char* name; unsigned flags; } kinds[] = {
        {"hipHostMallocDefault", hipHostMallocDefault},
        {"hipHostMallocNumaUser", hipHostMallocNumaUser},
        {"hipHostMallocCoherent", hipHostMallocCoherent},
        {"hipHostMallocNonCoherent", hipHostMallocNonCoherent},
        {"hipHostMallocPortable", hipHostMallocPortable},
    };
    for (auto& k : kinds) {
        void* h = nullptr;
        if (hipHostMalloc(&h, slot, k.flags) != hipSuccess) {
            printf("%s: alloc failed\n", k.name);
            continue;
        }
        memset(h, 0, slot);
        printf("{\"alloc\": \"%s\", \"d2h_GBs\": %.1f, \"h2d_GBs\": %.1f}\n", k.name,
               rate(h, dev, total, piece, hipMemcpyDeviceToHost, st), rate(h, dev, total, piece, hipMemcpyHostToDevice, st));
        hipHostFree(h);
    }
    {
        // the device source from the stream-ordered pool (as bj_lde_commit_h's workspace)
        void* pdev = nullptr;
        hipMallocAsync(&pdev, total, st);
        hipMemsetAsync(pdev, 1, total, st);
        hipStreamSynchronize(st);
        void* hm = nullptr;
        hipHostMalloc(&hm, slot, hipHostMallocDefault);
        memset(hm, 0, slot);
        printf("{\"alloc\": \"pool source, hipHostMallocDefault\", \"d2h_GBs\": %.1f, \"h2d_GBs\": %.1f}\n",
               rate(hm, pdev, total, piece, hipMemcpyDeviceToHost, st), rate(hm, pdev, total, piece, hipMemcpyHostToDevice, st));
        hipHostFree(hm);
        hipFreeAsync(pdev, st);
        hipStreamSynchronize(st);
    }
    {
        // per-stream rates: copy engines are assigned per stream
        void* hm = nullptr;
        hipHostMalloc(&hm, slot, hipHostMallocDefault);
        memset(hm, 0, slot);
        for (int i = 0; i < 6; i++) {
            hipStream_t si;
            hipStreamCreateWithFlags(&si, hipStreamNonBlocking);
            printf("{\"stream\": %d, \"d2h_GBs\": %.1f, \"h2d_GBs\": %.1f}\n", i,
                   rate(hm, dev, total, piece, hipMemcpyDeviceToHost, si), rate(hm, dev, total, piece, hipMemcpyHostToDevice, si));
        }
        hipHostFree(hm);
    }
    void* h = aligned_alloc(4096, slot);
    memset(h, 0, slot);
    hipHostRegister(h, slot, hipHostRegisterDefault);
    printf("{\"alloc\": \"aligned_alloc+hipHostRegister\", \"d2h_GBs\": %.1f, \"h2d_GBs\": %.1f}\n",
           rate(h, dev, total, piece, hipMemcpyDeviceToHost, st), rate(h, dev, total, piece, hipMemcpyHostToDevice, st));
    hipHostUnregister(h);
    free(h);
    return 0;
}
