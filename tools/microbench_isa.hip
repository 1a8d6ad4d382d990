// Throughput microbenchmark of gfx950 integer VALU instructions (independent chains),
// to price the Goldilocks multiply/add building blocks.  Reports cycles per wave64
// instruction per SIMD (2.0 = full rate on the SIMD-32 units).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench_isa tools/microbench_isa.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

// K64: 8 independent 64-bit accumulators %0..%7, inputs %8 (v32), %9 (s32).
#define K64(NAME, I0, I1, I2, I3, I4, I5, I6, I7)                                                      \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed) {                       \
        uint64_t x0 = threadIdx.x + seed, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 9,            \
                 x5 = x0 * 11, x6 = x0 * 13, x7 = x0 * 15;                                            \
        uint32_t b32 = blockIdx.x | 1u;                                                                \
        uint32_t s32 = __builtin_amdgcn_readfirstlane(seed * 3 + 1);                                  \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(I0 I1 I2 I3 I4 I5 I6 I7 I0 I1 I2 I3 I4 I5 I6 I7                               \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6),        \
                           "+v"(x7)                                                                    \
                         : "v"(b32), "s"(s32)                                                         \
                         : "vcc", "s40", "s41", "s42", "s43");                                                      \
        }                                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;            \
    }
// K32: 8 independent pairs of 32-bit accumulators: lo %0..%7, hi %8..%15, inputs %16 (v), %17 (s)
#define K32(NAME, I0, I1, I2, I3, I4, I5, I6, I7)                                                      \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed) {                       \
        uint32_t a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,            \
                 a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;                                            \
        uint32_t h0 = a0 ^ 1, h1 = a1 ^ 1, h2 = a2 ^ 1, h3 = a3 ^ 1, h4 = a4 ^ 1, h5 = a5 ^ 1,            \
                 h6 = a6 ^ 1, h7 = a7 ^ 1;                                                             \
        uint32_t b32 = blockIdx.x | 1u;                                                                \
        uint32_t s32 = __builtin_amdgcn_readfirstlane(seed * 3 + 1);                                  \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(I0 I1 I2 I3 I4 I5 I6 I7 I0 I1 I2 I3 I4 I5 I6 I7                               \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),        \
                           "+v"(a7), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4), "+v"(h5),        \
                           "+v"(h6), "+v"(h7)                                                          \
                         : "v"(b32), "s"(s32)                                                         \
                         : "vcc", "s40", "s41", "s42", "s43");                                                      \
        }                                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] =                                                   \
            (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) << 32 | (h0 ^ h1 ^ h2 ^ h3 ^ h4 ^ h5 ^ h6 ^ h7); \
    }
#define E8(M) M(0, 8), M(1, 9), M(2, 10), M(3, 11), M(4, 12), M(5, 13), M(6, 14), M(7, 15)
#define S(x) #x
#define K64X(...) K64(__VA_ARGS__)
#define K32X(...) K32(__VA_ARGS__)

#define MAD(i, j) "v_mad_u64_u32 %" S(i) ", s[40:41], %8, %9, %" S(i) "\n"
K64X(k_mad_u64_u32, E8(MAD))
#define LSHLADD(i, j) "v_lshl_add_u64 %" S(i) ", %" S(i) ", 0, %" S(i) "\n"
K64X(k_lshl_add_u64, E8(LSHLADD))
#define LSHR64(i, j) "v_lshrrev_b64 %" S(i) ", 3, %" S(i) "\n"
K64X(k_lshrrev_b64, E8(LSHR64))
#define CMP64(i, j) "v_cmp_lt_u64 vcc, %" S(i) ", %0\n"
K64X(k_cmp_u64, E8(CMP64))
#define FMA64(i, j) "v_fma_f64 %" S(i) ", %" S(i) ", %" S(i) ", %" S(i) "\n"
K64X(k_fma_f64, E8(FMA64))
#define PKFMA(i, j) "v_pk_fma_f32 %" S(i) ", %" S(i) ", %" S(i) ", %" S(i) "\n"
K64X(k_pk_fma_f32, E8(PKFMA))

#define MULLO(i, j) "v_mul_lo_u32 %" S(i) ", %" S(i) ", %16\n"
K32X(k_mul_lo_u32, E8(MULLO))
#define MULHI(i, j) "v_mul_hi_u32 %" S(i) ", %" S(i) ", %16\n"
K32X(k_mul_hi_u32, E8(MULHI))
#define MUL24(i, j) "v_mul_u32_u24 %" S(i) ", %" S(i) ", %16\n"
K32X(k_mul_u32_u24, E8(MUL24))
#define MULHI24(i, j) "v_mul_hi_u32_u24 %" S(j) ", %" S(i) ", %16\n"
K32X(k_mul_hi_u32_u24, E8(MULHI24))
#define MADU24(i, j) "v_mad_u32_u24 %" S(i) ", %" S(i) ", %16, %" S(j) "\n"
K32X(k_mad_u32_u24, E8(MADU24))
#define ADD32(i, j) "v_add_u32 %" S(i) ", %" S(i) ", %16\n"
K32X(k_add_u32, E8(ADD32))
#define ADD3(i, j) "v_add3_u32 %" S(i) ", %" S(i) ", %16, %" S(j) "\n"
K32X(k_add3_u32, E8(ADD3))
#define ADDC(i, j) "v_add_co_u32 %" S(i) ", vcc, %" S(i) ", %16\nv_addc_co_u32 %" S(j) ", vcc, %" S(j) ", 0, vcc\n"
K32X(k_add_co_pair, E8(ADDC))
#define SUBC(i, j) "v_sub_co_u32 %" S(i) ", vcc, %" S(i) ", %16\nv_subb_co_u32 %" S(j) ", vcc, %" S(j) ", 0, vcc\n"
K32X(k_sub_co_pair, E8(SUBC))
#define CND(i, j) "v_cndmask_b32 %" S(i) ", %" S(i) ", %16, vcc\n"
K32X(k_cndmask, E8(CND))
#define ALIGN(i, j) "v_alignbit_b32 %" S(i) ", %" S(j) ", %" S(i) ", 7\n"
K32X(k_alignbit, E8(ALIGN))
#define CMP32(i, j) "v_cmp_lt_u32 vcc, %" S(i) ", %16\n"
K32X(k_cmp_u32, E8(CMP32))
#define ADDCSG(i, j) "v_add_co_u32 %" S(i) ", s[40:41], %" S(i) ", %16\nv_addc_co_u32 %" S(j) ", s[40:41], %" S(j) ", 0, s[40:41]\n"
K32X(k_add_co_pair_sgpr, E8(ADDCSG))

#define CNDE64(i, j) "v_cmp_lt_u32 s[40:41], %" S(i) ", %16\nv_cndmask_b32_e64 %" S(j) ", 0, 1, s[40:41]\n"
K32X(k_cmp_cnd_e64, E8(CNDE64))
#define CNDE64B(i, j) "v_cndmask_b32_e64 %" S(j) ", 0, 1, s[40:41]\n"
K32X(k_cnd_e64_only, E8(CNDE64B))
#define ADDCZ(i, j) "v_addc_co_u32_e64 %" S(j) ", s[42:43], 0, 0, s[40:41]\n"
K32X(k_addc_zero, E8(ADDCZ))
#define MOV(i, j) "v_mov_b32 %" S(i) ", %" S(j) "\n"
K32X(k_mov, E8(MOV))
#define AND(i, j) "v_and_b32 %" S(i) ", %" S(j) ", %16\n"
K32X(k_and, E8(AND))
#define CNDVCC(i, j) "v_cndmask_b32_e32 %" S(i) ", %" S(j) ", %" S(i) ", vcc\n"
K32X(k_cnd_vcc_vv, E8(CNDVCC))
#define XOR(i, j) "v_xor_b32 %" S(i) ", %" S(j) ", %" S(i) "\n"
K32X(k_xor, E8(XOR))

// 32-bit ALU candidates for BLAKE2s (rotate / xor / add forms)
#define PERM(i, j) "v_perm_b32 %" S(i) ", %" S(i) ", %" S(i) ", %17\n"
K32X(k_perm, E8(PERM))
#define ALIGNBYTE(i, j) "v_alignbyte_b32 %" S(i) ", %" S(j) ", %" S(i) ", 2\n"
K32X(k_alignbyte, E8(ALIGNBYTE))
#define LSHLOR(i, j) "v_lshl_or_b32 %" S(i) ", %" S(i) ", 7, %" S(j) "\n"
K32X(k_lshl_or, E8(LSHLOR))
#define XAD(i, j) "v_xad_u32 %" S(i) ", %" S(i) ", %16, %" S(j) "\n"
K32X(k_xad, E8(XAD))
#define BITOP3(i, j) "v_bitop3_b32 %" S(i) ", %" S(i) ", %16, %" S(j) " bitop3:0x96\n"
K32X(k_bitop3, E8(BITOP3))
#define OR3(i, j) "v_or3_b32 %" S(i) ", %" S(i) ", %16, %" S(j) "\n"
K32X(k_or3, E8(OR3))
#define LSHLADD32(i, j) "v_lshl_add_u32 %" S(i) ", %" S(i) ", 3, %" S(j) "\n"
K32X(k_lshl_add_u32, E8(LSHLADD32))
#define PKADD16(i, j) "v_pk_add_u16 %" S(i) ", %" S(i) ", %16\n"
K32X(k_pk_add_u16, E8(PKADD16))
#define LSHR32(i, j) "v_lshrrev_b32 %" S(i) ", 7, %" S(i) "\n"
K32X(k_lshr32, E8(LSHR32))

int main() {
    const int blocks = 256 * 8, threads = 256;
    uint64_t* out;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct T { const char* name; void (*k)(uint64_t*, uint32_t); int instr_per_body; };
    T tests[] = {
        {"v_add_u32", k_add_u32, 16},           {"v_add3_u32", k_add3_u32, 16},
        {"v_add_co+v_addc_co (per instr)", k_add_co_pair, 32},
        {"v_sub_co+v_subb_co (per instr)", k_sub_co_pair, 32},
        {"v_lshl_add_u64", k_lshl_add_u64, 16}, {"v_lshrrev_b64", k_lshrrev_b64, 16},
        {"v_alignbit_b32", k_alignbit, 16},     {"v_cndmask_b32", k_cndmask, 16},
        {"v_cmp_lt_u64", k_cmp_u64, 16},       {"v_cmp_lt_u32", k_cmp_u32, 16},
        {"v_add_co+v_addc_co sgpr carry (per instr)", k_add_co_pair_sgpr, 32},
        {"v_mad_u64_u32", k_mad_u64_u32, 16},   {"v_mul_lo_u32", k_mul_lo_u32, 16},
        {"v_mul_hi_u32", k_mul_hi_u32, 16},     {"v_mul_u32_u24", k_mul_u32_u24, 16},
        {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 16}, {"v_mad_u32_u24", k_mad_u32_u24, 16},
        {"v_cmp_lt_u32+v_cndmask_e64 s-pair (per instr)", k_cmp_cnd_e64, 32},
        {"v_cndmask_e64 0,1,s-pair", k_cnd_e64_only, 16},
        {"v_addc_co_u32_e64 v,0,0,carry", k_addc_zero, 16},
        {"v_mov_b32", k_mov, 16}, {"v_and_b32", k_and, 16}, {"v_xor_b32", k_xor, 16},
        {"v_cndmask_b32_e32 v,v,vcc", k_cnd_vcc_vv, 16},
        {"v_fma_f64", k_fma_f64, 16},           {"v_pk_fma_f32", k_pk_fma_f32, 16},
        {"v_perm_b32", k_perm, 16},             {"v_alignbyte_b32", k_alignbyte, 16},
        {"v_lshl_or_b32", k_lshl_or, 16},       {"v_xad_u32", k_xad, 16},
        {"v_bitop3_b32", k_bitop3, 16},         {"v_or3_b32", k_or3, 16},
        {"v_lshl_add_u32", k_lshl_add_u32, 16}, {"v_pk_add_u16", k_pk_add_u16, 16},
        {"v_lshrrev_b32", k_lshr32, 16},
    };
    // clock: assume 2.4 GHz nominal; also report absolute ns
    for (auto& t : tests) {
        hipLaunchKernelGGL(t.k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(t.k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        double waves = (double)blocks * threads / 64;
        double wave_instr = waves * ITERS * t.instr_per_body;
        double per_simd = wave_instr / 1024.0;           // 256 CUs x 4 SIMDs
        double cycles = ms * 1e-3 * 2.4e9;
        printf("%-36s %8.3f ms   %.2f cycles / wave-instr / SIMD (@2.4GHz)\n", t.name, ms, cycles / per_simd);
    }
    CHECK(hipFree(out));
    return 0;
}
