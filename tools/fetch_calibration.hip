// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access shapes of this library's kernels,
// on buffers of known size (MI355X_MICROARCH.md, HBM: FETCH_SIZE reports half the bytes of a
// wide streaming read; other widths are uncalibrated -- calibrate in your own access pattern).
// Each kernel touches every byte of a 2 GiB buffer exactly once; rocprofv3 --pmc FETCH_SIZE (one
// pass) and --pmc WRITE_SIZE (another) then give the counter per known byte:
//   col8    one 8-byte element per lane per load, 64 lanes = 512 contiguous bytes, columns at a
//           stride (the leaf kernel's column loads: leaf_hash_kernel, merkle.hip);
//   run128  8 bytes per lane in runs of 16 lanes = 128 bytes, runs at a large stride (the NTT
//           head's strided rows, ntt_ct.hip);
//   vec16   16 bytes per lane, contiguous (the guide's reference shape);
//   store8  8-byte stores per lane, contiguous (the NTT / LDE output shape).
// Usage: fetch_calibration   (prints the byte count of each kernel; the counters come from rocprofv3)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = (size_t)2 << 30;
constexpr size_t WORDS = BYTES / 8;

__global__ __launch_bounds__(256) void col8(const uint64_t* __restrict__ src, size_t rows, uint32_t cols,
                                            uint64_t* __restrict__ sink) {
    const size_t r = blockIdx.x * (size_t)256 + threadIdx.x;
    uint64_t acc = 0;
    for (uint32_t c = 0; c < cols; c++) acc ^= src[(size_t)c * rows + r];
    if (acc == 0x0123456789abcdefull) sink[r & 1023] = acc;  // keeps the loads, ~never stores
}

// 16 lanes read 128 contiguous bytes; consecutive lane groups read runs 1 MiB apart
__global__ __launch_bounds__(256) void run128(const uint64_t* __restrict__ src, uint64_t* __restrict__ sink) {
    const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
    const size_t lane = t & 15, grp = t >> 4;
    const size_t n_rows = WORDS >> 17;                        // rows of 2^17 words (1 MiB)
    const size_t row = grp % n_rows, col = grp / n_rows;      // group -> (row, 16-word run)
    uint64_t acc = src[(row << 17) + col * 16 + lane];
    if (acc == 0x0123456789abcdefull) sink[t & 1023] = acc;
}

__global__ __launch_bounds__(256) void vec16(const ulonglong2* __restrict__ src, uint64_t* __restrict__ sink,
                                             size_t n16) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const ulonglong2 v = src[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x0123456789abcdefull) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void store8(uint64_t* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = i;
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

int main() {
    uint64_t *buf = nullptr, *sink = nullptr;
    CK(hipMalloc(&buf, BYTES));
    CK(hipMalloc(&sink, 8192));
    CK(hipMemset(buf, 1, BYTES));
    CK(hipDeviceSynchronize());
    // col8: 16 columns of 2^24 rows
    const uint32_t cols = 16;
    const size_t rows = WORDS / cols;
    hipLaunchKernelGGL(col8, dim3((unsigned)(rows / 256)), dim3(256), 0, 0, buf, rows, cols, sink);
    CK(hipGetLastError());
    // run128: WORDS / 16 runs, one 16-lane group each
    hipLaunchKernelGGL(run128, dim3((unsigned)(WORDS / 256)), dim3(256), 0, 0, buf, sink);
    CK(hipGetLastError());
    hipLaunchKernelGGL(vec16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const ulonglong2*>(buf), sink,
                       BYTES / 16);
    CK(hipGetLastError());
    hipLaunchKernelGGL(store8, dim3(8192), dim3(256), 0, 0, buf, WORDS);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"col8\", \"run128\", \"vec16\", \"store8\"]}\n", BYTES);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
