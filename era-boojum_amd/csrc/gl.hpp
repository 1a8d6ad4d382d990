// Goldilocks field (p = 2^64 - 2^32 + 1) arithmetic for gfx950 device code and host.
//
// Semantics follow the reference's GoldilocksField (field/goldilocks/mod.rs:82-255):
// values are u64 representatives in [0, 2^64), not necessarily canonical; every value
// that leaves a kernel is canonicalised (to_reduced_u64, mod.rs:146-153), which is the
// representation the reference serialises and compares (mod.rs:96-105, 257-261).
//
// The device forms are written for the 32-bit VALU: a 64x64 product is four
// v_mad_u64_u32, and the reduction uses 2^64 = 2^32 - 1 and 2^96 = -1 (mod p).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GL_FN __host__ __device__ __forceinline__
#else
#define GL_FN static inline
#endif

namespace gl {

constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
constexpr uint64_t EPS = 0xFFFFFFFFULL;  // 2^32 - 1
constexpr uint64_t GENERATOR = 7;        // MULTIPLICATIVE_GROUP_GENERATOR, mod.rs:107
constexpr uint64_t ROOT_2_32 = 0x185629dcda58878cULL;  // RADIX_2_SUBGROUP_GENERATOR, mod.rs:108

GL_FN uint64_t canon(uint64_t x) { return x >= P ? x - P : x; }

// a + b mod p for any a, b < 2^64 (add_assign_impl, mod.rs:213-231).
GL_FN uint64_t add(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    uint64_t t = s + (s < a ? EPS : 0);
    return t + (t < s ? EPS : 0);
}

// a - b mod p for any a, b < 2^64 (sub_assign, mod.rs:307-325).
GL_FN uint64_t sub(uint64_t a, uint64_t b) {
    uint64_t d = a - b;
    uint64_t t = d - (a < b ? EPS : 0);
    return t - (t > d ? EPS : 0);
}

// 128-bit value (hi:lo) mod p (from_u128_with_reduction, mod.rs:186-199).
GL_FN uint64_t reduce128(uint64_t lo, uint64_t hi) {
    uint64_t hi_hi = hi >> 32;
    uint64_t hi_lo = hi & EPS;
    uint64_t t0 = lo - hi_hi;
    t0 -= (lo < hi_hi) ? EPS : 0;
    uint64_t t1 = (hi_lo << 32) - hi_lo;  // hi_lo * EPS
    uint64_t t2 = t0 + t1;
    return t2 + (t2 < t0 ? EPS : 0);
}

GL_FN void mul_wide(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
    uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    uint64_t p00 = (uint64_t)a0 * b0;
    uint64_t p01 = (uint64_t)a0 * b1;
    uint64_t p10 = (uint64_t)a1 * b0;
    uint64_t p11 = (uint64_t)a1 * b1;
    uint64_t mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;  // < 3 * 2^32
    lo = (p00 & EPS) | (mid << 32);
    hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}

// a * b mod p (mul_assign_impl, mod.rs:243-247).
GL_FN uint64_t mul(uint64_t a, uint64_t b) {
    uint64_t lo, hi;
    mul_wide(a, b, lo, hi);
    return reduce128(lo, hi);
}

// a * 2^k mod p for 0 <= k < 32: the product fits in 96 bits (hi < 2^32), so the
// 2^96 term vanishes.  Used for the Poseidon2 internal diagonal (2^sh,
// state_generic_impl.rs:71-84) -- the same value as a general multiply.
GL_FN uint64_t mul_pow2_small(uint64_t a, int k) {
    if (k == 0) return a;
    uint64_t lo = a << k;
    uint64_t hi = a >> (64 - k);  // < 2^k <= 2^31
    uint64_t t1 = (hi << 32) - hi;  // hi * EPS
    uint64_t t2 = lo + t1;
    return t2 + (t2 < lo ? EPS : 0);
}

GL_FN uint64_t pow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = mul(r, b);
        b = mul(b, b);
        e >>= 1;
    }
    return r;
}

GL_FN uint64_t inv(uint64_t a) { return pow(a, P - 2); }

// omega_{2^log_n} (domain_generator_for_size, cs/implementations/utils.rs:13-28).
GL_FN uint64_t domain_generator(uint32_t log_n) {
    uint64_t w = ROOT_2_32;
    for (uint32_t i = log_n; i < 32; i++) w = mul(w, w);
    return canon(w);
}

GL_FN uint32_t bitrev32(uint32_t x, uint32_t bits) {
    if (bits == 0) return 0;
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x) >> (32 - bits);
#else
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
#endif
}

}  // namespace gl
