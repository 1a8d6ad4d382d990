// Probe: can one process drive two RCCL ranks on the same device (ncclCommInitAll with a
// repeated device)?  Decides whether the native sharded commit can be tested multi-rank on a
// one-GPU box through RCCL itself.
// build: hipcc -O2 -o tools/rccl_probe tools/rccl_probe.cpp -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <vector>

int main() {
    int devs[2] = {0, 0};
    ncclComm_t comms[2];
    ncclResult_t r = ncclCommInitAll(comms, 2, devs);
    printf("ncclCommInitAll({0,0}) -> %d (%s)\n", (int)r, ncclGetErrorString(r));
    if (r != ncclSuccess) return 0;
    const size_t n = 1 << 20;
    uint64_t *send[2], *recv[2];
    hipStream_t st[2];
    for (int i = 0; i < 2; i++) {
        hipMalloc(&send[i], n * 8);
        hipMalloc(&recv[i], 2 * n * 8);
        std::vector<uint64_t> h(n, 1000 + i);
        hipMemcpy(send[i], h.data(), n * 8, hipMemcpyHostToDevice);
        hipStreamCreate(&st[i]);
    }
    ncclGroupStart();
    for (int i = 0; i < 2; i++) ncclAllGather(send[i], recv[i], n, ncclUint64, comms[i], st[i]);
    r = ncclGroupEnd();
    printf("allgather group -> %d\n", (int)r);
    for (int i = 0; i < 2; i++) hipStreamSynchronize(st[i]);
    std::vector<uint64_t> h(2 * n);
    hipMemcpy(h.data(), recv[1], 2 * n * 8, hipMemcpyDeviceToHost);
    printf("rank1 recv[0]=%llu recv[n]=%llu\n", (unsigned long long)h[0], (unsigned long long)h[n]);
    for (int i = 0; i < 2; i++) ncclCommDestroy(comms[i]);
    return 0;
}
