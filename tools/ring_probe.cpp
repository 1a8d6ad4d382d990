// The copy-out ring of bj_lde_commit_h in isolation: D2H DMA into RING pinned slots, host
// threads copying each landed slot into a pageable buffer.  Not product code.
// build: hipcc -O2 --offload-arch=gfx950 -o tools/ring_probe tools/ring_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static void par_copy(char* d, const char* s, size_t n, int th) {
    std::vector<std::thread> ts;
    size_t per = (n + th - 1) / th;
    for (int i = 0; i < th; i++) {
        size_t o = i * per;
        if (o >= n) break;
        ts.emplace_back([=] { memcpy(d + o, s + o, std::min(per, n - o)); });
    }
    for (auto& t : ts) t.join();
}

int main() {
    const size_t total = (size_t)2 << 30, slot = (size_t)64 << 20;
    const int RING = 3;
    char* dev;
    hipMalloc((void**)&dev, total);
    hipMemset(dev, 1, total);
    char* dst = (char*)malloc(total);
    memset(dst, 0, total);
    char* slots[RING];
    hipEvent_t ev[RING];
    for (int i = 0; i < RING; i++) {
        hipHostMalloc((void**)&slots[i], slot, hipHostMallocDefault);
        memset(slots[i], 0, slot);
        hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    }
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int mode = 0; mode < 7; mode++) {
        // mode 0: DMA only; 1: + host copy 1 thread; 2: 4 threads; 3: 8 threads;
        // 4: 4 threads, issued from a second host thread; 5: 4 threads, source rewritten by a
        // memset before each pass; 6: 4 threads, a second stream's event waited before each pass
        const int th = mode == 0 ? 0 : mode == 1 ? 1 : mode == 3 ? 8 : 4;
        double best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            if (mode == 5) hipMemsetAsync(dev, rep, total, st);
            if (mode == 6) {
                hipStream_t s2;
                hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
                hipEvent_t e2;
                hipEventCreateWithFlags(&e2, hipEventDisableTiming);
                hipMemsetAsync(dev, rep, 1 << 20, s2);
                hipEventRecord(e2, s2);
                hipStreamWaitEvent(st, e2, 0);
            }
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            auto body = [&] {
            size_t pieces = total / slot, issued = 0, done = 0;
            while (done < pieces) {
                while (issued < pieces && issued - done < (size_t)RING) {
                    int k = issued % RING;
                    hipMemcpyAsync(slots[k], dev + issued * slot, slot, hipMemcpyDeviceToHost, st);
                    hipEventRecord(ev[k], st);
                    issued++;
                }
                int k = done % RING;
                hipEventSynchronize(ev[k]);
                if (th) par_copy(dst + done * slot, slots[k], slot, th);
                done++;
            }
            };
            if (mode == 4) {
                std::thread t([&] { hipSetDevice(0); body(); });
                t.join();
            } else {
                body();
            }
            double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt < best) best = dt;
        }
        printf("{\"mode\": %d, \"host_copy_threads\": %d, \"GBs\": %.1f}\n", mode, th, total / best / 1e9);
    }
    return 0;
}
