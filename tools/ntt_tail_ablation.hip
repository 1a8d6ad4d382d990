// Where the CT tail's time goes: the production tail (csrc/ntt_ct.hip, ct_tail_kernel) next to
// copies with one part removed at a time, timed at C3's forward shape (256 columns x 2^22
// rows x 4 cosets; the tail's 13 stages on 8192-element tiles).  Results are garbage for the
// ablated variants: only the time matters.  DESIGN.md section 4.1.
//   0 full                 the production kernel's sequence
//   1 no global load       x from registers (thread id), no HBM read
//   2 no store             results feed one predicated store (never taken)
//   3 no LDS exchanges     the three exchanges and their barriers removed
//   4 no twiddle loads     twiddles from registers
//   5 butterflies only     1 + 2 + 3 + 4
//   6 nontemporal stores   the full kernel with streaming stores
//   7 ... and loads        streaming loads and stores
//   8 uniform-base loads/stores ((d + 256 k)[t] instead of d[t + 256 k])
//   9 the full kernel again (box drift between the first and the last timing)
//  10 no final C -> A exchange: each thread stores its 32 contiguous elements as 16-byte writes
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I era-boojum_amd/csrc -o tools/ntt_tail_ablation tools/ntt_tail_ablation.hip
#include "../era-boojum_amd/csrc/ntt_ct.hip"
#include <cstdio>

namespace bj {
namespace {

template <int ABL>
__device__ __forceinline__ void tail_unit_body(uint64_t* lds, uint64_t* d, const uint64_t* __restrict__ ct, size_t q,
                                               uint32_t u0) {
    constexpr bool LOAD = ABL != 1 && ABL != 5, STORE = ABL != 2 && ABL != 5, EXCH = ABL != 3 && ABL != 5,
                   TWL = ABL != 4 && ABL != 5, NTS = ABL == 6 || ABL == 7, NTL = ABL == 7, SADDR = ABL == 8,
                   CSTORE = ABL == 10;
    const uint32_t t = threadIdx.x;
    uint64_t x[PT], wa[16], wb[16];
    if constexpr (LOAD) {
#pragma unroll
        for (int k = 0; k < PT; k++)
            x[k] = NTL ? __builtin_nontemporal_load(d + t + NT * k) : (SADDR ? (d + NT * k)[t] : d[t + NT * k]);
    } else {
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = (uint64_t)(t + 1) * (2 * k + 1) + q;
    }
    auto twA = [&](uint64_t* w, auto vtag) {
        constexpr int V = decltype(vtag)::value;
        if constexpr (TWL) tw_ct_tailA<V>(w, ct, u0, q);
        else {
#pragma unroll
            for (int p = 0; p < 16; p++) w[p] = 0x123456789ull * (p + V + 1) + q;
        }
    };
    auto twB = [&](uint64_t* w, auto vtag, uint32_t thi) {
        constexpr int V = decltype(vtag)::value;
        if constexpr (TWL) tw_ct_tailB<V>(w, ct, u0, q, thi);
        else {
#pragma unroll
            for (int p = 0; p < 16; p++) w[p] = 0x987654321ull * (p + V + 1) + thi;
        }
    };
    auto twC = [&](uint64_t* w, auto vtag) {
        constexpr int V = decltype(vtag)::value;
        if constexpr (TWL) tw_ct_tailC<V>(w, ct, u0, q, t);
        else {
#pragma unroll
            for (int p = 0; p < 16; p++) w[p] = 0x55555555ull * (p + V + 1) + t;
        }
    };
    using I0 = std::integral_constant<int, 0>;
    twA(wa, I0{});
    twA(wb, std::integral_constant<int, 1>{});
    ct_stage<16>(x, wa);
    twA(wa, std::integral_constant<int, 2>{});
    ct_stage<8>(x, wb);
    twA(wb, std::integral_constant<int, 3>{});
    ct_stage<4>(x, wa);
    twA(wa, std::integral_constant<int, 4>{});
    ct_stage<2>(x, wb);
    const uint32_t tlo = t & 7, thi = t >> 3;
    const uint32_t ba = tail_base_a(t), bb = tail_base_b(thi, tlo), bc = tail_base_c(t);
    twB(wb, std::integral_constant<int, 5>{}, thi);
    ct_stage<1>(x, wa);
    if constexpr (EXCH) {
#pragma unroll
        for (int k = 0; k < PT; k++) lds[ba + tail_off_a(k)] = x[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[bb + tail_off_b(k)];
    }
    twB(wa, std::integral_constant<int, 6>{}, thi);
    ct_stage<16>(x, wb);
    twB(wb, std::integral_constant<int, 7>{}, thi);
    ct_stage<8>(x, wa);
    twB(wa, std::integral_constant<int, 8>{}, thi);
    ct_stage<4>(x, wb);
    twB(wb, std::integral_constant<int, 9>{}, thi);
    ct_stage<2>(x, wa);
    twC(wa, std::integral_constant<int, 10>{});
    ct_stage<1>(x, wb);
    if constexpr (EXCH) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) lds[bb + tail_off_b(k)] = x[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[bc + k];
    }
    twC(wb, std::integral_constant<int, 11>{});
    ct_stage<4>(x, wa);
    twC(wa, std::integral_constant<int, 12>{});
    ct_stage<2>(x, wb);
    ct_stage<1>(x, wa);
    if constexpr (CSTORE) {
        // no final exchange: layout C (element 32 t + k) stored as it stands, 16 bytes per lane
        uint64_t* dt = d + 32 * t;
#pragma unroll
        for (int k = 0; k < PT; k += 2) {
            ulonglong2 v;
            v.x = canon_u64(x[k]);
            v.y = canon_u64(x[k + 1]);
            *reinterpret_cast<ulonglong2*>(dt + k) = v;
        }
        return;
    }
    if constexpr (EXCH) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) lds[bc + k] = x[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[ba + tail_off_a(k)];
    }
    if constexpr (STORE) {
#pragma unroll
        for (int k = 0; k < PT; k++) {
            if constexpr (NTS) __builtin_nontemporal_store(canon_u64(x[k]), d + t + NT * k);
            else if constexpr (SADDR) (d + NT * k)[t] = canon_u64(x[k]);
            else d[t + NT * k] = canon_u64(x[k]);
        }
    } else {
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < PT; k++) acc ^= x[k];
        if (acc == 0x0123456789abcdefull) d[t] = acc;
    }
}

template <int ABL>
__global__ __launch_bounds__(NT, 2) void tail_ablation(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                       uint32_t log_n, const uint64_t* __restrict__ tab,
                                                       size_t tab_stride) {
    __shared__ uint64_t lds[PAD_LDS];
    const size_t q = blockIdx.y;
    tail_unit_body<ABL>(lds, dst + (size_t)blockIdx.x * dst_col_stride + (size_t)blockIdx.z * coset_stride + q * TILE,
                        tab + (size_t)blockIdx.z * tab_stride, q, log_n - 13);
}

// persistent: gridDim.x blocks walk the units (column fastest); the previous unit's stores
// drain while the next unit loads and computes
__global__ __launch_bounds__(NT, 2) void tail_persistent(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                         uint32_t log_n, const uint64_t* __restrict__ tab,
                                                         size_t tab_stride, uint32_t cols, uint32_t tiles,
                                                         uint32_t units) {
    __shared__ uint64_t lds[PAD_LDS];
    for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint32_t col = u % cols, rest = u / cols, q = rest % tiles, coset = rest / tiles;
        tail_unit_body<0>(lds, dst + (size_t)col * dst_col_stride + (size_t)coset * coset_stride + (size_t)q * TILE,
                          tab + (size_t)coset * tab_stride, q, log_n - 13);
        __syncthreads();
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
    uint64_t *buf = nullptr, *tab = nullptr;
    CHECK(hipMalloc(&buf, n * cols * cosets * 8));
    CHECK(hipMalloc(&tab, n * cosets * 8));
    CHECK(hipMemset(buf, 1, n * cols * cosets * 8));
    for (uint32_t c = 0; c < cosets; c++) CHECK(bj::launch_ct_table(tab + c * n, log_n, false, 7 + c, 1, 0));
    CHECK(hipDeviceSynchronize());
    const dim3 g(cols, (unsigned)(n / bj::TILE), cosets);
    using K = void (*)(uint64_t*, size_t, size_t, uint32_t, const uint64_t*, size_t);
    const K ks[] = {bj::tail_ablation<0>, bj::tail_ablation<1>, bj::tail_ablation<2>,
                    bj::tail_ablation<3>, bj::tail_ablation<4>, bj::tail_ablation<5>,
                    bj::tail_ablation<6>, bj::tail_ablation<7>, bj::tail_ablation<8>, bj::tail_ablation<0>,
                    bj::tail_ablation<10>, bj::tail_ablation<0>};
    const char* names[] = {"full", "no global load", "no store", "no LDS exchanges", "no twiddle loads",
                           "butterflies only", "nontemporal stores", "nontemporal loads and stores",
                           "uniform-base addressing", "full (again)", "no final exchange: 16-byte stores from layout C",
                           "full (third)"};
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int mult = 2; mult <= 2; mult *= 2) {
        const uint32_t units = g.x * g.y * g.z, blocks = cus * mult;
        hipLaunchKernelGGL(bj::tail_persistent, dim3(blocks), dim3(bj::NT), 0, 0, buf, n * cosets, n, log_n, tab, n,
                           g.x, g.y, units);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 3; r++)
            hipLaunchKernelGGL(bj::tail_persistent, dim3(blocks), dim3(bj::NT), 0, 0, buf, n * cosets, n, log_n, tab,
                               n, g.x, g.y, units);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"variant\": \"persistent %d blocks/CU\", \"ms\": %.3f}\n", mult, ms / 3);
    }
    for (int v = 0; v < 12; v++) {
        hipLaunchKernelGGL(ks[v], g, dim3(bj::NT), 0, 0, buf, n * cosets, n, log_n, tab, n);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 3; r++) hipLaunchKernelGGL(ks[v], g, dim3(bj::NT), 0, 0, buf, n * cosets, n, log_n, tab, n);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"variant\": %d, \"name\": \"%s\", \"ms\": %.3f}\n", v, names[v], ms / 3);
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(tab));
    return 0;
}
