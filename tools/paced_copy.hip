// An RCCL-shaped disturbance for tools/shard_compute_probe.py (test infrastructure, not product):
// `channels` workgroups stay resident for the whole exchange, as RCCL's collective kernels do (one
// or two workgroups per channel, polling between chunks), and move the bytes a rank receives at
// a paced rate, the rate its xGMI ingress allows, instead of in one HBM-speed burst.  Each
// workgroup copies 256 KiB chunks (16-byte lanes, coalesced) and then sleeps until the wall
// clock (s_memrealtime, read only) reaches its next deadline.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC -o tools/libpaced_copy.so tools/paced_copy.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint32_t CHUNK = 256u << 10;  // bytes per workgroup step

__global__ __launch_bounds__(256) void paced_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         size_t ring16, size_t total16, uint64_t ticks_per_chunk) {
    // workgroup w copies global chunks w, w + G, ... of the stream (ring-buffer addresses, so a
    // small buffer stands for many GiB of traffic); the k-th chunk of this workgroup is due at
    // t0 + (k + 1) * ticks_per_chunk
    const uint32_t G = gridDim.x, w = blockIdx.x;
    constexpr uint32_t per = CHUNK / 16;
    __shared__ uint64_t t0;
    if (threadIdx.x == 0) t0 = wall_clock64();
    __syncthreads();
    uint64_t k = 0;
    for (size_t c = w; c * per < total16; c += G, k++) {
        const size_t base = (c * per) & (ring16 - 1);  // ring16: a power of two, a multiple of per
        // 8 loads in flight per lane before their stores (32 KiB per workgroup), so a workgroup
        // moves ~10 GB/s or more and the pacing, not the copy loop, sets the rate
        for (uint32_t i0 = 0; i0 < per; i0 += 8 * 256) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = src[base + i0 + u * 256 + threadIdx.x];
#pragma unroll
            for (int u = 0; u < 8; u++) dst[base + i0 + u * 256 + threadIdx.x] = v[u];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t due = t0 + (k + 1) * ticks_per_chunk;
            while (wall_clock64() < due) __builtin_amdgcn_s_sleep(8);
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

// Move `total_bytes` through `ring_bytes`-sized device buffers (a power of two >= 256 KiB) with `channels` resident
// workgroups of 256 threads at `gbps` GB/s in all (0: unpaced), on `stream`.  Returns a hipError_t.
int paced_copy(const void* src, void* dst, size_t ring_bytes, size_t total_bytes, int channels, double gbps,
               void* stream) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 1;
    // one workgroup's chunk interval: channels workgroups share the rate
    const double sec_per_chunk = gbps > 0 ? (double)CHUNK * channels / (gbps * 1e9) : 0.0;
    const uint64_t ticks = (uint64_t)(sec_per_chunk * khz * 1e3);
    hipLaunchKernelGGL(paced_copy_kernel, dim3(channels), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), ring_bytes / 16,
                       total_bytes / 16, ticks);
    return (int)hipGetLastError();
}

int wall_clock_khz(void) {
    int dev = 0, khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    return khz;
}

}  // extern "C"
