// Batched Goldilocks arithmetic through the device field layer (gl_asm.hpp): a utility
// entry point so the inline-asm primitives get direct parity tests against the
// reference's field semantics (field/goldilocks/mod.rs:186-325).  Outputs canonical.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "bj_internal.hpp"

namespace bj {

__global__ __launch_bounds__(256) void gl_op_kernel(int op, const uint64_t* __restrict__ a,
                                                    const uint64_t* __restrict__ b, uint64_t* __restrict__ out,
                                                    size_t n) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t x = a[i], y = b[i];
    uint32_t z0, z1;
    const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
    switch (op) {
        case 0: glasm::mul_x1(x0, x1, y0, y1, z0, z1); break;
        case 1: glasm::add_x1(x0, x1, y0, y1, z0, z1); break;
        case 2: glasm::sub_x1(x0, x1, y0, y1, z0, z1); break;
        case 3: {  // limb reduction: L = a (< 2^63), H = b (< 2^63 with hi word < 2^31)
            uint64_t z;
            glasm::reduce_x1(x, y0, y1, z);
            z0 = (uint32_t)z;
            z1 = (uint32_t)(z >> 32);
            break;
        }
        default: z0 = x0; z1 = x1; break;  // 4: canonicalise a
    }
    uint32_t c0, c1;
    glasm::canon_x1(z0, z1, c0, c1);
    out[i] = ((uint64_t)c1 << 32) | c0;
}

hipError_t launch_gl_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gl_op_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, op, a, b, out, n);
    return hipGetLastError();
}

}  // namespace bj
