// Where the forward CT head's time goes (csrc/ntt_ct.hip, ct_head_kernel<9, 1, false>: the first 9
// stages of C3's four coset transforms, gathering the bit-reversed monomials), next to copies
// with one part removed at a time.  Results are garbage for the ablated variants: only the
// time matters.  DESIGN.md section 4.2.  This is the general-twiddle head of round 2's first
// half; C3 now runs the power-of-two form (ct_head_kernel<9, 1, false, false, true>, section 4.3).
//   0 full                 the production kernel's sequence
//   1 no global load       x from registers (thread id), no gather, no staging exchange
//   2 no store             results feed one predicated store (never taken)
//   3 no LDS               gather staging and the A'->B' exchange removed (loads kept)
//   4 no twiddle loads     twiddles from registers
//   5 butterflies only     1 + 2 + 3 + 4
//   6 the general head as it now stands in ntt_ct.hip (variant 0 is the sequence this tool copied)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I era-boojum_amd/csrc -o tools/ntt_head_ablation tools/ntt_head_ablation.hip
#include "../era-boojum_amd/csrc/ntt_ct.hip"
#include <cstdio>

namespace bj {
namespace {

template <int ABL>
__global__ __launch_bounds__(NT, 2) void head_ablation(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                       const uint64_t* src, size_t src_stride, uint32_t log_n,
                                                       const uint64_t* __restrict__ tab, size_t tab_stride,
                                                       uint32_t n_cosets, uint32_t log_tiles) {
    constexpr int R = 9;
    constexpr bool LOAD = ABL != 1 && ABL != 5, STORE = ABL != 2 && ABL != 5, LDSX = ABL != 3 && ABL != 5 && ABL != 1,
                   TWL = ABL != 4 && ABL != 5;
    constexpr int LOGW = 13 - R;
    constexpr uint32_t W = 1u << LOGW;
    constexpr uint32_t T = 1u << (R - 5);
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t tid = threadIdx.x;
    const size_t n = (size_t)1 << log_n;
    const size_t S = n >> R;
    uint32_t coset, unit;
    head_unit(blockIdx.x, n_cosets, true, coset, unit);
    const uint32_t col = unit >> log_tiles;
    const size_t o0 = (size_t)(unit & ((1u << log_tiles) - 1)) * W;
    const uint64_t* sc = src + (size_t)col * src_stride;
    const uint64_t* ct = tab + (size_t)coset * tab_stride;
    const uint32_t w = tid & (W - 1);
    const uint32_t s = tid >> LOGW;
    const size_t o = o0 + w;
    uint64_t x[PT];
    if constexpr (LOAD) {
        const uint32_t wg = tid / T, sg = tid % T;
        const size_t run = (size_t)gl::bitrev32((uint32_t)(o0 + wg), log_n - R) << R;
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = sc[run + sg + T * k];
        if constexpr (LDSX) {
#pragma unroll
            for (int k = 0; k < PT; k++) lds[swz_gather(gl::bitrev32(sg + T * k, R) * W + wg)] = x[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = lds[swz_gather((s + T * k) * W + w)];
        }
    } else {
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = (uint64_t)(tid + 1) * (2 * k + 1) + o0;
    }
    auto twA = [&](uint64_t* wv, auto vtag) {
        constexpr int V = decltype(vtag)::value;
        if constexpr (TWL) tw_ct_headA<V>(wv, ct, 1u);
        else {
#pragma unroll
            for (int q = 0; q < 16; q++) wv[q] = 0x123456789ull * (q + V + 1) + coset;
        }
    };
    {
        uint64_t wa[16], wb[16];
        twA(wa, std::integral_constant<int, 0>{});
        twA(wb, std::integral_constant<int, 1>{});
        ct_stage<16>(x, wa);
        twA(wa, std::integral_constant<int, 2>{});
        ct_stage<8>(x, wb);
        twA(wb, std::integral_constant<int, 3>{});
        ct_stage<4>(x, wa);
        twA(wa, std::integral_constant<int, 4>{});
        ct_stage<2>(x, wb);
        ct_stage<1>(x, wa);
    }
    if constexpr (LDSX) {
        __syncthreads();
        const uint32_t pa = tid + (tid >> 5);
        const uint32_t pd = 33 * W * s + w + (w >> 5);
#pragma unroll
        for (int k = 0; k < PT; k++) lds[pa + 264 * k] = x[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[pd + k * W + ((k * W) >> 5)];
    }
    if constexpr (TWL) {
        head_b_stage<R, 5>(x, ct, s, 1u);
    } else {
        uint64_t wv[16];
#pragma unroll
        for (int q = 0; q < 16; q++) wv[q] = 0x987654321ull * (q + 1) + s;
        ct_stage<8>(x, wv);
        ct_stage<4>(x, wv);
        ct_stage<2>(x, wv);
        ct_stage<1>(x, wv);
    }
    uint64_t* dc = dst + (size_t)col * dst_col_stride + (size_t)coset * coset_stride;
    if constexpr (STORE) {
#pragma unroll
        for (int k = 0; k < PT; k++) dc[(size_t)(32 * s + k) * S + o] = x[k];
    } else {
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < PT; k++) acc ^= x[k];
        if (acc == 0x0123456789abcdefull) dc[o] = acc;
    }
}

}  // namespace
}  // namespace bj

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                   \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

int main() {
    const uint32_t log_n = 22, cols = 256, cosets = 4;
    const size_t n = (size_t)1 << log_n;
    uint64_t *src = nullptr, *dst = nullptr, *tab = nullptr;
    CHECK(hipMalloc(&src, n * cols * 8));
    CHECK(hipMalloc(&dst, n * cols * cosets * 8));
    const size_t L = bj::ct_table_len(log_n);  // the CT table + the power-of-two prescale tables
    CHECK(hipMalloc(&tab, L * cosets * 8));
    CHECK(hipMemset(src, 1, n * cols * 8));
    for (uint32_t c = 0; c < cosets; c++) CHECK(bj::launch_ct_table(tab + c * L, log_n, false, 7 + c, 1, 0));
    CHECK(hipDeviceSynchronize());
    const uint32_t log_tiles = log_n - 13;
    const dim3 g(cols * (1u << log_tiles) * cosets);
    using K = void (*)(uint64_t*, size_t, size_t, const uint64_t*, size_t, uint32_t, const uint64_t*, size_t, uint32_t,
                       uint32_t);
    const K ks[] = {bj::head_ablation<0>, bj::head_ablation<1>, bj::head_ablation<2>,
                    bj::head_ablation<3>, bj::head_ablation<4>, bj::head_ablation<5>};
    const char* names[] = {"full", "no global load", "no store", "no LDS", "no twiddle loads", "butterflies only"};
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int v = 0; v < 7; v++) {
        if (v == 6) {  // the production kernel (csrc/ntt_ct.hip as built into this tool)
            const int xcd = 1;
            hipLaunchKernelGGL((bj::ct_head_kernel<9, 1, false>), g, dim3(bj::NT), 0, 0, dst, n * cosets, n,
                               (const uint64_t*)src, n, log_n, (const uint64_t*)tab, L, (uint64_t)0, cosets,
                               log_tiles, xcd, 0u, (size_t)0);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a));
            for (int r = 0; r < 3; r++)
                hipLaunchKernelGGL((bj::ct_head_kernel<9, 1, false>), g, dim3(bj::NT), 0, 0, dst, n * cosets, n,
                                   (const uint64_t*)src, n, log_n, (const uint64_t*)tab, L, (uint64_t)0, cosets,
                                   log_tiles, xcd, 0u, (size_t)0);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            printf("{\"variant\": 6, \"name\": \"production kernel\", \"ms\": %.3f}\n", ms / 3);
            continue;
        }
        hipLaunchKernelGGL(ks[v], g, dim3(bj::NT), 0, 0, dst, n * cosets, n, src, n, log_n, tab, L, cosets, log_tiles);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 3; r++)
            hipLaunchKernelGGL(ks[v], g, dim3(bj::NT), 0, 0, dst, n * cosets, n, src, n, log_n, tab, L, cosets,
                               log_tiles);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"variant\": %d, \"name\": \"%s\", \"ms\": %.3f}\n", v, names[v], ms / 3);
    }
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    CHECK(hipFree(tab));
    return 0;
}
