// Keccak256 tree hashing kernels (gfx950): the TreeHasher impl for sha3::Keccak256
// (cs/oracle/mod.rs:247-313).  Keccak256 = Keccak[c = 512]: rate 136 bytes = 17 lanes, the
// original pad10*1 with domain byte 0x01, 32-byte digest (the first 4 lanes).
//
// Leaf (hash_into_leaf, :271-283): the canonical little-endian bytes of the leaf's elements,
// so element k is XORed into lane k mod 17 and every 17th element permutes; the final block
// gets 0x01 in the lane after the last element and 0x80 in the top byte of lane 16 (both in
// lane 16 when 16 elements remain; a padding-only block when none remain).  Node (:302-313):
// l || r = 8 lanes, padding in lanes 8 and 16, one permutation.  Digests are 4 little-endian
// u64 words, the same (N, 4) layout as the other tree hashers.
//
// One leaf per lane as in merkle.hip / blake2s.hip; the 25-lane state lives in 50 VGPRs.
// Keccak-f[1600] on 32-bit halves: 64-bit rotates are v_alignbit pairs (swaps for 32), the
// 5-way column parities and chi's a ^ (~b & c) are 3-input logic (v_bitop3_b32, full rate on
// gfx950).
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

constexpr int KC_THREADS = 256;
constexpr int KC_RATE = 17;  // lanes per 136-byte block

// rho offsets of lane x + 5 y
constexpr int KC_RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

__device__ __constant__ uint32_t KC_RC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
    0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
    0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__device__ __constant__ uint32_t KC_RC_HI[24] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u,
    0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u,
    0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

// 3-input logic (v_bitop3_b32): truth table over (a, b, c) = (0xF0, 0xCC, 0xAA)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t chi(uint32_t a, uint32_t b, uint32_t c) {  // a ^ (~b & c)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xD2);
}

// (hi:lo) rotated left by R (compile-time): v_alignbit pairs, a swap for R >= 32
template <int R>
__device__ __forceinline__ void rotl(uint32_t lo, uint32_t hi, uint32_t& olo, uint32_t& ohi) {
    if constexpr (R == 0) {
        olo = lo;
        ohi = hi;
    } else if constexpr (R == 32) {
        olo = hi;
        ohi = lo;
    } else if constexpr (R < 32) {
        ohi = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
        olo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    } else {
        rotl<R - 32>(hi, lo, olo, ohi);
    }
}

// rho + pi for lane x + 5 y (compile-time): B[y + 5 ((2x + 3y) mod 5)] = rotl(A[x + 5y], rho)
template <int I>
__device__ __forceinline__ void rho_pi(const uint32_t* Al, const uint32_t* Ah, uint32_t* Bl, uint32_t* Bh) {
    if constexpr (I < 25) {
        constexpr int x = I % 5, y = I / 5;
        constexpr int J = y + 5 * ((2 * x + 3 * y) % 5);
        rotl<KC_RHO[I]>(Al[I], Ah[I], Bl[J], Bh[J]);
        rho_pi<I + 1>(Al, Ah, Bl, Bh);
    }
}

// Keccak-f[1600] (FIPS 202 section 3.2) on 32-bit lane halves; lane x + 5 y
__device__ __forceinline__ void keccak_f(uint32_t* Al, uint32_t* Ah) {
#pragma unroll 1
    for (int round = 0; round < 24; round++) {
        uint32_t Cl[5], Ch[5], Rl[5], Rh[5], Bl[25], Bh[25];
#pragma unroll
        for (int x = 0; x < 5; x++) {
            Cl[x] = xor3(xor3(Al[x], Al[x + 5], Al[x + 10]), Al[x + 15], Al[x + 20]);
            Ch[x] = xor3(xor3(Ah[x], Ah[x + 5], Ah[x + 10]), Ah[x + 15], Ah[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; x++) rotl<1>(Cl[x], Ch[x], Rl[x], Rh[x]);
        // theta: A ^= C[x-1] ^ rotl(C[x+1], 1)
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++) {
                Al[x + 5 * y] = xor3(Al[x + 5 * y], Cl[(x + 4) % 5], Rl[(x + 1) % 5]);
                Ah[x + 5 * y] = xor3(Ah[x + 5 * y], Ch[(x + 4) % 5], Rh[(x + 1) % 5]);
            }
        rho_pi<0>(Al, Ah, Bl, Bh);
#pragma unroll
        for (int y = 0; y < 5; y++)
#pragma unroll
            for (int x = 0; x < 5; x++) {
                Al[x + 5 * y] = chi(Bl[x + 5 * y], Bl[(x + 1) % 5 + 5 * y], Bl[(x + 2) % 5 + 5 * y]);
                Ah[x + 5 * y] = chi(Bh[x + 5 * y], Bh[(x + 1) % 5 + 5 * y], Bh[(x + 2) % 5 + 5 * y]);
            }
        Al[0] ^= KC_RC_LO[round];
        Ah[0] ^= KC_RC_HI[round];
    }
}

// the 64-bit lane view over the split state
struct KState {
    uint32_t lo[25], hi[25];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < 25; i++) lo[i] = hi[i] = 0;
    }
    __device__ __forceinline__ void absorb(int i, uint64_t v) {
        lo[i] ^= (uint32_t)v;
        hi[i] ^= (uint32_t)(v >> 32);
    }
    __device__ __forceinline__ void permute() { keccak_f(lo, hi); }
    __device__ __forceinline__ void store4(uint64_t* o) const {
#pragma unroll
        for (int i = 0; i < 4; i++) o[i] = ((uint64_t)hi[i] << 32) | lo[i];
    }
};

__device__ __forceinline__ void pad_final(KState& S, uint32_t filled) {
    // filled < 17 lanes of the last block hold message bytes
#pragma unroll
    for (int i = 0; i < KC_RATE; i++)
        if ((uint32_t)i == filled) S.lo[i] ^= 0x01u;
    S.hi[16] ^= 0x80000000u;
}

// Leaf L = the elements src[c][L], c < n_cols.
__global__ __launch_bounds__(KC_THREADS) void kc_leaf_kernel(const uint64_t* __restrict__ src, size_t col_stride,
                                                             uint32_t n_cols, size_t n_leaves,
                                                             uint64_t* __restrict__ out) {
    const size_t L = blockIdx.x * (size_t)KC_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint64_t* p = src + L;
    KState S;
    S.clear();
    const uint32_t full = n_cols / KC_RATE;
    for (uint32_t g = 0; g < full; g++) {
        const uint64_t* q = p + (size_t)g * KC_RATE * col_stride;
#pragma unroll
        for (int i = 0; i < KC_RATE; i++) S.absorb(i, gl::canon(q[(size_t)i * col_stride]));
        S.permute();
    }
    const uint32_t rem = n_cols - full * KC_RATE;
    const uint64_t* q = p + (size_t)full * KC_RATE * col_stride;
#pragma unroll
    for (int i = 0; i < KC_RATE - 1; i++)
        if ((uint32_t)i < rem) S.absorb(i, gl::canon(q[(size_t)i * col_stride]));
    pad_final(S, rem);
    S.permute();
    S.store4(out + 4 * L);
}

// construct_by_chunking leaves (merkle_tree.rs:176-386): leaf L absorbs, for each source
// column c in order, the E = 2^log_e consecutive elements src[c][L*E .. (L+1)*E).
__global__ __launch_bounds__(KC_THREADS) void kc_leaf_chunk_kernel(const uint64_t* __restrict__ src,
                                                                   size_t col_stride, uint32_t n_cols,
                                                                   uint32_t log_e, size_t n_leaves,
                                                                   uint64_t* __restrict__ out) {
    const size_t L = blockIdx.x * (size_t)KC_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint32_t E = 1u << log_e;
    const uint64_t* p = src + (L << log_e);
    KState S;
    S.clear();
    const uint32_t total = n_cols << log_e;
    uint32_t k = 0;
    for (; k + KC_RATE <= total; k += KC_RATE) {
#pragma unroll
        for (int i = 0; i < KC_RATE; i++) {
            const uint32_t e = k + i;
            S.absorb(i, gl::canon(p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))]));
        }
        S.permute();
    }
    const uint32_t rem = total - k;
#pragma unroll
    for (int i = 0; i < KC_RATE - 1; i++) {
        const uint32_t e = k + i;
        if ((uint32_t)i < rem) S.absorb(i, gl::canon(p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))]));
    }
    pad_final(S, rem);
    S.permute();
    S.store4(out + 4 * L);
}

__device__ __forceinline__ void node_hash(const uint64_t* l, const uint64_t* r, uint64_t* o) {
    KState S;
    S.clear();
#pragma unroll
    for (int i = 0; i < 4; i++) {
        S.absorb(i, l[i]);
        S.absorb(4 + i, r[i]);
    }
    S.lo[8] = 0x01u;
    S.hi[16] = 0x80000000u;
    S.permute();
    S.store4(o);
}

__global__ __launch_bounds__(256) void kc_node_level_kernel(const uint64_t* __restrict__ prev,
                                                            uint64_t* __restrict__ next, size_t m) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i >= m) return;
    uint64_t lr[8];
#pragma unroll
    for (int k = 0; k < 8; k++) lr[k] = prev[8 * i + k];
    node_hash(lr, lr + 4, next + 4 * i);
}

// Remaining levels from `len` digests (len <= 4096) down to cap_size, one workgroup.
__global__ __launch_bounds__(256) void kc_node_tail_kernel(const uint64_t* __restrict__ prev, uint64_t* next,
                                                           uint32_t len, uint32_t cap_size) {
    __shared__ uint64_t buf[2][2048 * 4];
    int cur = 0;
    uint64_t* outp = next;
    uint32_t m = len / 2;
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        uint64_t lr[8];
        for (int k = 0; k < 8; k++) lr[k] = prev[8 * (size_t)i + k];
        uint64_t o[4];
        node_hash(lr, lr + 4, o);
        for (int k = 0; k < 4; k++) {
            buf[cur][4 * i + k] = o[k];
            outp[4 * (size_t)i + k] = o[k];
        }
    }
    outp += 4 * (size_t)m;
    __syncthreads();
    while (m > cap_size) {
        const uint32_t m2 = m / 2;
        for (uint32_t i = threadIdx.x; i < m2; i += 256) {
            uint64_t o[4];
            node_hash(&buf[cur][8 * i], &buf[cur][8 * i + 4], o);
            for (int k = 0; k < 4; k++) {
                buf[cur ^ 1][4 * i + k] = o[k];
                outp[4 * (size_t)i + k] = o[k];
            }
        }
        outp += 4 * (size_t)m2;
        cur ^= 1;
        m = m2;
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_kc_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves, uint64_t* out,
                            hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    hipLaunchKernelGGL(kc_leaf_kernel, dim3((unsigned)((n_leaves + KC_THREADS - 1) / KC_THREADS)), dim3(KC_THREADS),
                       0, st, src, col_stride, n_cols, n_leaves, out);
    return hipGetLastError();
}

hipError_t launch_kc_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                    size_t n_leaves, uint64_t* out, hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    hipLaunchKernelGGL(kc_leaf_chunk_kernel, dim3((unsigned)((n_leaves + KC_THREADS - 1) / KC_THREADS)),
                       dim3(KC_THREADS), 0, st, src, col_stride, n_cols, log_e, n_leaves, out);
    return hipGetLastError();
}

hipError_t launch_kc_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                           hipStream_t st) {
    const uint64_t* prev = leaves;
    uint64_t* out = nodes;
    size_t len = n_leaves;
    while (len > cap_size && len > 4096) {
        const size_t m = len / 2;
        hipLaunchKernelGGL(kc_node_level_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, prev, out, m);
        prev = out;
        out += 4 * m;
        len = m;
    }
    if (len > cap_size)
        hipLaunchKernelGGL(kc_node_tail_kernel, dim3(1), dim3(256), 0, st, prev, out, (uint32_t)len, cap_size);
    return hipGetLastError();
}

}  // namespace bj
