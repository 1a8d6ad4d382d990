// Poseidon2 over Goldilocks, width 12 / rate 8 / capacity 4, for gfx950 device code.
//
// Same permutation as the reference's State::poseidon2_permutation
// (implementations/poseidon2/state_generic_impl.rs:221-236):
//   external MDS; 4 full rounds (RC[r][i], x^7, external MDS); 22 partial rounds
//   (state[0] += RC[r][0], x^7 on state[0], internal M_I); 4 full rounds.
// External MDS = block-circulant(2*M4, M4, M4) (implementations/suggested_mds.rs:19-97),
// M_I = diag(2^sh) + 1 1^T with sh = [4,14,11,8,0,5,2,9,13,6,3,12]
// (state_generic_impl.rs:71-84, 166-202).  Round constants: poseidon2_rc.inc (data
// extracted by tools/gen_poseidon2_constants.py from poseidon_goldilocks_params.rs).
//
// The state lives in 24 VGPRs (one permutation per lane).  Linear layers are evaluated
// lazily: 64-bit limbs plus a 32-bit overflow word, reduced once per output, which
// yields the same field elements as the reference's per-add reduction (all results are
// compared in canonical form).
#pragma once
#include "gl.hpp"

namespace p2 {

__device__ __constant__ static const uint64_t RC[30][12] = {
#include "poseidon2_rc.inc"
};

// Wide (lazy) value: lo + hi * 2^64, hi small.
struct W {
    uint64_t lo;
    uint32_t hi;
};

__device__ __forceinline__ W w_of(uint64_t x) { return W{x, 0u}; }

__device__ __forceinline__ W w_add(W a, W b) {
    uint64_t lo = a.lo + b.lo;
    uint32_t hi = a.hi + b.hi + (lo < a.lo ? 1u : 0u);
    return W{lo, hi};
}

__device__ __forceinline__ W w_shl(W a, int k) {  // a * 2^k, k small (1..2)
    uint64_t lo = a.lo << k;
    uint32_t hi = (a.hi << k) | (uint32_t)(a.lo >> (64 - k));
    return W{lo, hi};
}

// lo + hi * 2^64 mod p, hi < 2^32: 2^64 = EPS (mod p).
__device__ __forceinline__ uint64_t w_reduce(W a) {
    uint64_t t1 = ((uint64_t)a.hi << 32) - a.hi;  // hi * EPS < 2^64
    uint64_t t2 = a.lo + t1;
    return t2 + (t2 < a.lo ? gl::EPS : 0);
}

// M4 block (suggested_mds.rs block_mul) on wide values.
__device__ __forceinline__ void m4(W& x0, W& x1, W& x2, W& x3) {
    W t0 = w_add(x0, x1);
    W t1 = w_add(x2, x3);
    W t2 = w_add(w_shl(x1, 1), t1);
    W t3 = w_add(w_shl(x3, 1), t0);
    W t4 = w_add(w_shl(t1, 2), t3);
    W t5 = w_add(w_shl(t0, 2), t2);
    W t6 = w_add(t3, t5);
    W t7 = w_add(t2, t4);
    x0 = t6; x1 = t5; x2 = t7; x3 = t4;
}

// External MDS: coefficients are <= 64 in row sum, so the wide sums stay < 2^71.
__device__ __forceinline__ void mds_ext(uint64_t s[12]) {
    W x[12];
#pragma unroll
    for (int i = 0; i < 12; i++) x[i] = w_of(s[i]);
    m4(x[0], x[1], x[2], x[3]);
    m4(x[4], x[5], x[6], x[7]);
    m4(x[8], x[9], x[10], x[11]);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        W a = x[i], b = x[i + 4], c = x[i + 8];
        W sum = w_add(w_add(a, b), c);
        s[i] = w_reduce(w_add(sum, a));
        s[i + 4] = w_reduce(w_add(sum, b));
        s[i + 8] = w_reduce(w_add(sum, c));
    }
}

__device__ __forceinline__ uint64_t sbox(uint64_t x) {  // x^7, state_generic_impl.rs:141-147
    uint64_t x2 = gl::mul(x, x);
    uint64_t x3 = gl::mul(x2, x);
    uint64_t x4 = gl::mul(x2, x2);
    return gl::mul(x4, x3);
}

__device__ __forceinline__ void mds_int(uint64_t s[12]) {
    constexpr int SH[12] = {4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12};
    W sum = w_of(s[0]);
#pragma unroll
    for (int i = 1; i < 12; i++) sum = w_add(sum, w_of(s[i]));
    // s_i * 2^sh_i + sum: (lo, hi) with hi < 2^14 + 12, reduced once.
#pragma unroll
    for (int i = 0; i < 12; i++) {
        W v;
        if (SH[i] == 0) {
            v = w_of(s[i]);
        } else {
            v.lo = s[i] << SH[i];
            v.hi = (uint32_t)(s[i] >> (64 - SH[i]));
        }
        s[i] = w_reduce(w_add(v, sum));
    }
}

__device__ __forceinline__ void permute(uint64_t s[12]) {
    mds_ext(s);
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int i = 0; i < 12; i++) s[i] = sbox(gl::add(s[i], RC[r][i]));
        mds_ext(s);
    }
#pragma unroll
    for (int r = 4; r < 26; r++) {
        s[0] = sbox(gl::add(s[0], RC[r][0]));
        mds_int(s);
    }
#pragma unroll
    for (int r = 26; r < 30; r++) {
#pragma unroll
        for (int i = 0; i < 12; i++) s[i] = sbox(gl::add(s[i], RC[r][i]));
        mds_ext(s);
    }
}

}  // namespace p2
