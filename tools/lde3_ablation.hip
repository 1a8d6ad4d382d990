// Where the three-pass LDE's time goes at C3 (2^22 x 256, D = 4): the final pass
// (lde3_final_kernel<9, F2MODE> for both phase-2 factor modes) next to copies of its first
// version (F1 and F2 loaded from the tables directly) with one part removed, and the middle pass with and
// without the monomial store and with 0 / 1 / 4 cosets.  Ablated variants compute garbage: only
// the time matters.  DESIGN.md section 4.4.
//   final 0  copy of the production sequence
//         1  no F1 loads (phase-1 factors from registers)
//         2  no F2 loads (phase-2 factors from registers)
//         3  neither
//         4  no global data load (x from the thread id)
//         5  no store
//         6  phase-2 factors made as A[M][rl] * U[p][rl] (16 per-M loads, 32 loads from a
//            512-entry table, 32 extra products) instead of 32 loads of F2
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/lde3_ablation tools/lde3_ablation.hip
#include "../era-boojum_amd/csrc/ntt_ct.hip"
#include "../era-boojum_amd/csrc/ntt_lde3.hip"
#include <cstdio>

#define CHECK(x)                                                                                 \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

namespace bj {
namespace {

template <int ABL>
__global__ __launch_bounds__(NT, 2) void final_ablation(uint64_t* lde, size_t col_stride, size_t coset_stride,
                                                        uint32_t n_cols, uint32_t n_cosets,
                                                        const uint64_t* __restrict__ tabs, size_t tab_stride) {
    constexpr int R = 9;
    constexpr int LW = 13 - R;
    constexpr uint32_t W = 1u << LW;
    constexpr bool F1L = ABL != 1 && ABL != 3, F2L = ABL != 2 && ABL != 3 && ABL != 6, LOAD = ABL != 4,
                   STORE = ABL != 5;
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t t = threadIdx.x;
    const uint32_t c = blockIdx.x % n_cols;
    const uint32_t rest = blockIdx.x / n_cols;
    const uint32_t i = rest % n_cosets;
    const uint32_t T = rest / n_cosets;
    uint64_t* d = lde + (size_t)c * col_stride + (size_t)i * coset_stride + (size_t)T * TILE;
    const uint64_t* tab = tabs + (size_t)i * tab_stride;
    const uint32_t o = t & (W - 1), qh = t >> LW;
    const uint32_t M = T * W + o;
    uint64_t x[PT], y[PT], f[PT];
    const uint32_t vi = qh * 32 * W + o;
    if constexpr (LOAD) {
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = d[vi + k * W];
    } else {
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = (uint64_t)(t + 1) * (2 * k + 1) + T;
    }
    if constexpr (F1L) {
        const uint64_t* f1 = tab + L3_F1 + M;
#pragma unroll
        for (int k = 0; k < PT; k++) f[k] = f1[(size_t)k << 13];
    } else {
#pragma unroll
        for (int k = 0; k < PT; k++) f[k] = 0x123456789ull * (k + 1) + M;
    }
    prescale32_brev(y, x, f);
    dft_p2<5, false, 0>(y);
    const uint32_t b1 = fin_p1<R>(t, 0);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[b1 + (fin_p1<R>(0, k) - fin_p1<R>(0, 0))] = y[k];
    constexpr int RL = R - 5;
    const uint32_t pl = t >> LW;
    if constexpr (F2L) {
        const uint64_t* f2 = tab + L3_F2 + M;
#pragma unroll
        for (int k = 0; k < PT; k++) {
            const uint32_t h = k >> RL, rl = k & ((1u << RL) - 1);
            f[k] = f2[((size_t)(rl * 32 + (h << RL)) << 13) + ((size_t)pl << 13)];
        }
    } else if constexpr (ABL == 6) {
        // A[M][rl] from the F1 region (stand-in, 16 per M), U[p][rl] from the HB region (512 used)
        uint64_t a[16];
        const uint64_t* A = tab + L3_F1 + (size_t)M * 16;
#pragma unroll
        for (int rl = 0; rl < 16; rl++) a[rl] = A[rl];
        const uint64_t* U = tab + L3_HB;
#pragma unroll
        for (int k = 0; k < PT; k++) {
            const uint32_t h = k >> RL, rl = k & ((1u << RL) - 1);
            f[k] = U[((pl + (h << RL)) << 4) + rl];
        }
        uint64_t a2[PT];
#pragma unroll
        for (int k = 0; k < PT; k++) a2[k] = a[k & 15];
        prescale32(f, a2);  // the 32 extra products
    } else {
#pragma unroll
        for (int k = 0; k < PT; k++) f[k] = 0x987654321ull * (k + 3) + M;
    }
    __syncthreads();
    const uint32_t b2 = fin_p2<R>(t, 0);
#pragma unroll
    for (int k = 0; k < PT; k++) y[k] = lds[b2 + (fin_p2<R>(0, k) - fin_p2<R>(0, 0))];
    prescale32(y, f);
    dft_p2_groups<RL, false>(y);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[b2 + (fin_p2<R>(0, k) - fin_p2<R>(0, 0))] = y[k];
    __syncthreads();
    const uint32_t b3 = fin_p3<R>(t, 0);
#pragma unroll
    for (int k = 0; k < PT; k++) y[k] = lds[b3 + (fin_p3<R>(0, k) - fin_p3<R>(0, 0))];
#pragma unroll
    for (int k = 0; k < PT; k += 4) canon4(y + k);
    if constexpr (STORE) {
#pragma unroll
        for (int k = 0; k < PT; k++) d[t + NT * k] = y[k];
    } else {
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < PT; k++) acc ^= y[k];
        if (acc == 0x5555555555555555ull) d[t] = acc;
    }
}

}  // namespace
}  // namespace bj

template <typename F>
static float time_ms(F launch, int reps = 3) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; r++) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / reps;
}

int main() {
    using namespace bj;
    const uint32_t log_n = 22, cols = 256, cosets = 4, R = 9;
    const size_t n = (size_t)1 << log_n;
    uint64_t *scratch = nullptr, *lde = nullptr, *tabs = nullptr, *inv = nullptr;
    CHECK(hipMalloc(&scratch, n * cols * 8));
    CHECK(hipMalloc(&lde, n * cols * cosets * 8));
    const size_t L = lde3_table_len(log_n);
    CHECK(hipMalloc(&tabs, L * cosets * 8));
    CHECK(hipMalloc(&inv, ct_table_len(log_n) * 8));
    CHECK(hipMemset(scratch, 1, n * cols * 8));
    CHECK(hipMemset(lde, 3, n * cols * cosets * 8));
    for (uint32_t c = 0; c < cosets; c++) CHECK(launch_lde3_table(tabs + c * L, log_n, 7 + c, 0));
    CHECK(launch_ct_table(inv, log_n, true, 1, 5, 0));
    CHECK(hipDeviceSynchronize());
    const dim3 gf((cols * cosets) << R), gm(cols << R);
    using KF = void (*)(uint64_t*, size_t, size_t, uint32_t, uint32_t, const uint64_t*, size_t);
    const KF kf[] = {final_ablation<0>, final_ablation<1>, final_ablation<2>, final_ablation<3>,
                     final_ablation<4>, final_ablation<5>, final_ablation<6>};
    const char* names[] = {"copy of production", "no F1 loads", "no F2 loads", "no F1/F2 loads", "no data load",
                           "no store", "F2 as A*U (16 + 32 small-table loads, 32 extra products)"};
    float ms = time_ms([&] {
        hipLaunchKernelGGL((lde3_final_kernel<9, 1>), gf, dim3(NT), 0, 0, lde, n * cosets, n, (size_t)0, 31u, cols,
                           cosets, (const uint64_t*)tabs, L);
    });
    printf("{\"kernel\": \"final\", \"variant\": \"production (F1 in LDS, phase 2 = A U from LDS)\", \"ms\": %.3f}\n", ms);
    ms = time_ms([&] {
        hipLaunchKernelGGL((lde3_final_kernel<9, 0>), gf, dim3(NT), 0, 0, lde, n * cosets, n, (size_t)0, 31u, cols,
                           cosets, (const uint64_t*)tabs, L);
    });
    printf("{\"kernel\": \"final\", \"variant\": \"F1 in LDS, tabulated F2 prefetched\", \"ms\": %.3f}\n", ms);
    for (int v = 0; v < 7; v++) {
        ms = time_ms([&] {
            hipLaunchKernelGGL(kf[v], gf, dim3(NT), 0, 0, lde, n * cosets, n, cols, cosets, (const uint64_t*)tabs, L);
        });
        CHECK(hipGetLastError());
        printf("{\"kernel\": \"final\", \"variant\": %d, \"name\": \"%s\", \"ms\": %.3f}\n", v, names[v], ms);
    }
    for (uint32_t nc : {0u, 1u, 4u}) {
        ms = time_ms([&] {
            hipLaunchKernelGGL((lde3_mid_kernel<9, true, true>), gm, dim3(NT), 0, 0, (const uint64_t*)scratch, n,
                               scratch, n, lde, n * cosets, n, (size_t)0, 31u, cols, nc, (const uint64_t*)inv,
                               (const uint64_t*)tabs, L);
        });
        printf("{\"kernel\": \"mid\", \"variant\": \"inverse + mono + %u cosets\", \"ms\": %.3f}\n", nc, ms);
        ms = time_ms([&] {
            hipLaunchKernelGGL((lde3_mid_kernel<9, true, false>), gm, dim3(NT), 0, 0, (const uint64_t*)scratch, n,
                               scratch, n, lde, n * cosets, n, (size_t)0, 31u, cols, nc, (const uint64_t*)inv,
                               (const uint64_t*)tabs, L);
        });
        printf("{\"kernel\": \"mid\", \"variant\": \"inverse + %u cosets (no mono)\", \"ms\": %.3f}\n", nc, ms);
    }
    ms = time_ms([&] {
        hipLaunchKernelGGL((lde3_mid_kernel<9, false, false>), gm, dim3(NT), 0, 0, (const uint64_t*)scratch, n,
                           scratch, n, lde, n * cosets, n, (size_t)0, 31u, cols, cosets, (const uint64_t*)inv,
                           (const uint64_t*)tabs, L);
    });
    printf("{\"kernel\": \"mid\", \"variant\": \"monomial source, 4 cosets\", \"ms\": %.3f}\n", ms);
    CHECK(hipFree(scratch));
    CHECK(hipFree(lde));
    CHECK(hipFree(tabs));
    CHECK(hipFree(inv));
    return 0;
}
