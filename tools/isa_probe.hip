// Semantics probe for gfx950 instructions whose documented operand ranges the assembler does
// not enforce: v_lshl_add_u64 with shift amounts 0..7 (D = (S0 << S1) + S2).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/isa_probe tools/isa_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define SH(N) asm volatile("v_lshl_add_u64 %0, %1, " #N ", %2" : "=v"(r[N]) : "v"(a), "v"(b));

__global__ void probe(uint64_t* out, uint64_t a, uint64_t b) {
    uint64_t r[8];
    SH(0) SH(1) SH(2) SH(3) SH(4) SH(5) SH(6) SH(7)
    if (threadIdx.x == 0)
        for (int i = 0; i < 8; i++) out[i] = r[i];
}

int main() {
    uint64_t* d;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    const uint64_t a = 0x0123456789abcdefull, b = 0x1111111111111111ull;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, a, b);
    uint64_t h[8];
    if (hipMemcpy(h, d, 64, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int bad = 0;
    for (int i = 0; i < 8; i++) {
        const uint64_t want = (a << i) + b;
        printf("v_lshl_add_u64 shift %d: %s (got %016llx want %016llx)\n", i, h[i] == want ? "ok" : "DIFFERS",
               (unsigned long long)h[i], (unsigned long long)want);
        bad += h[i] != want;
    }
    return bad ? 2 : 0;
}
