// Census-only kernels (tools/valu_census.py; never launched): one Poseidon2 permutation per lane
// in each output form of csrc/poseidon2.hpp, so the static census can price the leaf kernel's
// absorptions (all but the last: capacity words only; the last: the digest) and the full
// permutation of bj_poseidon2_permute_d separately.
#include <hip/hip_runtime.h>
#include "../era-boojum_amd/csrc/poseidon2.hpp"

template <int OUT>
__device__ __forceinline__ void census_body(uint64_t* st) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    p2::State s;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const uint64_t v = st[12 * i + k];
        s.lo[k] = (uint32_t)v;
        s.hi[k] = (uint32_t)(v >> 32);
    }
    p2::permute<OUT>(s);
    const int b = OUT == p2::OUT_ALL ? 0 : OUT == p2::OUT_CAP ? 8 : 0, e = OUT == p2::OUT_ALL ? 12 : b + 4;
#pragma unroll
    for (int k = b; k < e; k++) st[12 * i + k] = ((uint64_t)s.hi[k] << 32) | s.lo[k];
}

__global__ void census_perm_all(uint64_t* st) { census_body<p2::OUT_ALL>(st); }
__global__ void census_perm_cap(uint64_t* st) { census_body<p2::OUT_CAP>(st); }
__global__ void census_perm_digest(uint64_t* st) { census_body<p2::OUT_DIGEST>(st); }
