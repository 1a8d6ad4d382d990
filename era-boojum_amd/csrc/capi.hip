// C ABI of the MI355X witness-commitment path (include/boojum_mi355x.h).
// Host-side orchestration only: argument checks (the reference's asserts), the per-device
// twiddle / coset-power cache, and the kernel launch sequences for each entry point.
#include <hip/hip_runtime.h>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>
#include <cstring>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <thread>
#include <condition_variable>

#include "../../include/boojum_mi355x.h"
#include "gl.hpp"
#include "bj_internal.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(BJ_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                       \
    do {                                          \
        hipError_t _e = (expr);                   \
        if (_e != hipSuccess) return hip_fail(_e, what); \
    } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------ device cache
// Twiddle, power and LDE factor tables per device and size.  Entries are computed
// synchronously on a private stream when first inserted, so any caller stream can use them
// afterwards without ordering concerns; they stay until bj_release_tables (~180 MiB for a
// 2^22-row LDE at degree 4).
struct Cache {
    std::mutex mu;
    std::map<std::tuple<int, uint32_t, int>, uint64_t*> tw;
    std::map<std::tuple<int, uint32_t, int>, uint64_t*> pyr;
    std::map<std::tuple<int, uint32_t, uint64_t, uint64_t>, std::pair<uint64_t*, uint64_t*>> pw;
    std::map<std::tuple<int, uint32_t, uint32_t, int>, uint64_t*> lde_pw;
    std::map<std::tuple<int, uint32_t, int, uint64_t>, uint64_t*> ct;
    std::map<std::tuple<int, uint32_t, uint32_t>, uint64_t*> ct_lde;
    std::map<std::tuple<int, uint32_t, uint64_t>, uint64_t*> lde3;
    std::map<std::tuple<int, uint32_t, uint32_t>, uint64_t*> lde3_lde;
};
Cache& cache() {
    static Cache* c = new Cache();
    return *c;
}

// A table of `words` u64 on the current device, filled by fill(p, stream) on a private stream and
// synchronised; nothing is kept on any failure.
template <class Fill>
int make_table(size_t words, const char* what, Fill fill, uint64_t** out) {
    uint64_t* p = nullptr;
    HIP_TRY(hipMalloc(&p, words * sizeof(uint64_t)), what);
    hipStream_t st;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) {
        e = fill(p, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    if (e != hipSuccess) {
        (void)hipFree(p);
        return hip_fail(e, what);
    }
    *out = p;
    return BJ_OK;
}

// Look `key` up in `m` under the cache lock, else make and insert the table.
template <class Map, class Key, class Fill>
int cached_table(Map& m, const Key& key, size_t words, const char* what, Fill fill, const uint64_t** out) {
    std::lock_guard<std::mutex> lk(cache().mu);
    auto it = m.find(key);
    if (it != m.end()) {
        *out = it->second;
        return BJ_OK;
    }
    uint64_t* p;
    if (int r = make_table(words, what, fill, &p)) return r;
    m[key] = p;
    *out = p;
    return BJ_OK;
}

int current_device(int* dev) {
    HIP_TRY(hipGetDevice(dev), "hipGetDevice");
    return BJ_OK;
}

int get_twiddles(uint32_t log_n, bool inverse, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const size_t half = log_n ? ((size_t)1 << (log_n - 1)) : 1;
    return cached_table(cache().tw, std::make_tuple(dev, log_n, inverse ? 1 : 0), half, "twiddles",
                        [&](uint64_t* p, hipStream_t st) { return bj::launch_twiddles(p, log_n, inverse, st); }, out);
}

int get_powers(uint32_t log_n, uint64_t e_, uint64_t scale, const uint64_t** lo, const uint64_t** hi) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const uint64_t e = gl::canon(e_);
    Cache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto key = std::make_tuple(dev, log_n, e, gl::canon(scale));
    auto it = c.pw.find(key);
    if (it == c.pw.end()) {
        uint64_t* p;
        if (int r = make_table(4096 + bj::pw_hi_len(log_n), "power tables", [&](uint64_t* q, hipStream_t st) {
                return bj::launch_power_tables(q, q + 4096, log_n, e, scale, st);
            }, &p))
            return r;
        it = c.pw.emplace(key, std::make_pair(p, p + 4096)).first;
    }
    *lo = it->second.first;
    *hi = it->second.second;
    return BJ_OK;
}

// DIF twiddle pyramid (ntt_dif.hip): n entries, TW[m/2 + j] = w_m^j.
int get_pyramid(uint32_t log_n, bool inverse, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const size_t n = (size_t)1 << log_n;
    return cached_table(cache().pyr, std::make_tuple(dev, log_n, inverse ? 1 : 0), n < 2 ? 2 : n, "pyramid",
                        [&](uint64_t* p, hipStream_t st) { return bj::launch_twiddle_pyramid(p, log_n, inverse, st); },
                        out);
}

uint64_t lde_coset(uint32_t log_n, uint32_t log_d, uint32_t i);

// Power tables for all D cosets of an LDE: coset i at out + i * pw_stride, each
// [lo 4096 | hi n/4096] for scale * s_i^j (scale = n^-1 when the source is the raw iNTT).
int get_lde_powers(uint32_t log_n, uint32_t log_d, bool with_ninv, const uint64_t** out, size_t* stride) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const size_t pstride = 4096 + bj::pw_hi_len(log_n);
    *stride = pstride;
    const uint32_t D = 1u << log_d;
    const uint64_t scale = with_ninv ? gl::canon(gl::inv((uint64_t)1 << log_n)) : 1;
    return cached_table(cache().lde_pw, std::make_tuple(dev, log_n, log_d, with_ninv ? 1 : 0), D * pstride,
                        "lde powers", [&](uint64_t* p, hipStream_t st) {
                            hipError_t e = hipSuccess;
                            for (uint32_t i = 0; i < D && e == hipSuccess; i++)
                                e = bj::launch_power_tables(p + i * pstride, p + i * pstride + 4096, log_n,
                                                            lde_coset(log_n, log_d, i), scale, st);
                            return e;
                        }, out);
}

// Coset-folded CT twiddle table (ntt_ct.hip) for shift s, n entries. The inverse table
// (s = 1) carries n^-1 in its stage-0 entry.
int get_ct(uint32_t log_n, bool inverse, uint64_t shift_, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const uint64_t shift = gl::canon(shift_);
    const uint64_t scale1 = inverse ? gl::canon(gl::inv((uint64_t)1 << log_n)) : 1;
    return cached_table(cache().ct, std::make_tuple(dev, log_n, inverse ? 1 : 0, shift), bj::ct_table_len(log_n),
                        "ct table", [&](uint64_t* p, hipStream_t st) {
                            return bj::launch_ct_table(p, log_n, inverse, shift, scale1, st);
                        }, out);
}

// The D coset tables of an LDE, table i (shift 7 * w_{nD}^bitrev(i)) at out + i * ct_table_len.
int get_ct_lde(uint32_t log_n, uint32_t log_d, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const size_t n = bj::ct_table_len(log_n);
    const uint32_t D = 1u << log_d;
    return cached_table(cache().ct_lde, std::make_tuple(dev, log_n, log_d), D * n, "ct lde tables",
                        [&](uint64_t* p, hipStream_t st) {
                            hipError_t e = hipSuccess;
                            for (uint32_t i = 0; i < D && e == hipSuccess; i++)
                                e = bj::launch_ct_table(p + i * n, log_n, false, lde_coset(log_n, log_d, i), 1, st);
                            return e;
                        }, out);
}

// Three-pass LDE tables (ntt_lde3.hip) of one shift, and of the D coset shifts of an LDE (table i
// at out + i * lde3_table_len).
int get_lde3(uint32_t log_n, uint64_t shift_, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const uint64_t shift = gl::canon(shift_);
    return cached_table(cache().lde3, std::make_tuple(dev, log_n, shift), bj::lde3_table_len(log_n), "lde3 table",
                        [&](uint64_t* p, hipStream_t st) { return bj::launch_lde3_table(p, log_n, shift, st); }, out);
}

int get_lde3_lde(uint32_t log_n, uint32_t log_d, const uint64_t** out) {
    int dev = 0;
    if (int r = current_device(&dev)) return r;
    const size_t L = bj::lde3_table_len(log_n);
    const uint32_t D = 1u << log_d;
    return cached_table(cache().lde3_lde, std::make_tuple(dev, log_n, log_d), D * L, "lde3 lde tables",
                        [&](uint64_t* p, hipStream_t st) {
                            hipError_t e = hipSuccess;
                            for (uint32_t i = 0; i < D && e == hipSuccess; i++)
                                e = bj::launch_lde3_table(p + i * L, log_n, lde_coset(log_n, log_d, i), st);
                            return e;
                        }, out);
}

// The three-pass LDE (ntt_lde3.hip) is the default for 2^18..2^23; BJ_LDE_PASSES=2 (an experiment
// knob, bj_internal.hpp) selects the two-pass CT path (head + tail per transform) instead, for
// same-binary A/B measurements.
bool use_lde3(uint32_t log_n) { return bj::knobs().lde_passes != 2 && bj::lde3_supported(log_n); }

inline bool is_pow2(size_t x) { return x && !(x & (x - 1)); }

int log2_exact(size_t len, uint32_t* out) {
    if (!is_pow2(len)) return fail(BJ_EINVAL, "length must be a power of two");
    uint32_t l = 0;
    while (((size_t)1 << l) < len) l++;
    *out = l;
    return BJ_OK;
}

int check_log_n(uint32_t log_n) {
    if (log_n > 32) return fail(BJ_EINVAL, "log_n exceeds the 2-adicity (32) of the field");
    return BJ_OK;
}

// LDE coset shifts 7 * w_{nD}^{bitrev_{log D}(i)} (utils.rs:334-347, 370-373).
uint64_t lde_coset(uint32_t log_n, uint32_t log_d, uint32_t i) {
    uint64_t g = gl::domain_generator(log_n + log_d);
    return gl::canon(gl::mul(gl::pow(g, gl::bitrev32(i, log_d)), gl::GENERATOR));
}

// The *_h entry points run on a stream of their own per calling thread and device (created
// once; stream creation costs milliseconds on ROCm), with stream-ordered device buffers and
// explicit copies + synchronisation.  Nothing of theirs touches the legacy null stream, which
// every host thread shares.
int seam_stream(hipStream_t* out) {
    thread_local std::map<int, hipStream_t> tl;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto it = tl.find(dev);
    if (it == tl.end()) {
        hipStream_t st;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
        it = tl.emplace(dev, st).first;
    }
    *out = it->second;
    return BJ_OK;
}

// Stream-ordered device buffer RAII for the *_h entry points.
struct DBuf {
    uint64_t* p = nullptr;
    hipStream_t st = nullptr;
    explicit DBuf(hipStream_t s) : st(s) {}
    hipError_t alloc(size_t bytes) { return bj::pool_alloc((void**)&p, bytes, st); }
    ~DBuf() { if (p) (void)hipFreeAsync(p, st); }
};

}  // namespace

namespace {
// Inverse transform of the trace into monomials c_j stored at bitrev_n(j) (the exchange
// format of bj_lde_coeffs_d), canonical.
int inverse_to_bitrev(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                      uint32_t log_n, hipStream_t st) {
    if (bj::ct_ntt_supported(log_n)) {
        const uint64_t* tab;
        if (int r = get_ct(log_n, true, 1, &tab)) return r;
        HIP_TRY(bj::launch_ct(dst, dst_stride, 0, 1, src, src_stride, false, n_cols, log_n, tab, 0,
                              gl::canon(gl::inv((uint64_t)1 << log_n)), true, st),
                "ifft");
        return BJ_OK;
    }
    const uint64_t* ipyr;
    if (int r = get_pyramid(log_n, true, &ipyr)) return r;
    HIP_TRY(bj::launch_dif(dst, dst_stride, src, src_stride, n_cols, log_n, ipyr, false, st), "ifft");
    if (log_n)
        HIP_TRY(bj::launch_scale(dst, dst_stride, n_cols, (size_t)1 << log_n, gl::canon(gl::inv((uint64_t)1 << log_n)),
                                 st),
                "scale");
    else
        HIP_TRY(bj::launch_scale(dst, dst_stride, n_cols, 1, 1, st), "canon");
    return BJ_OK;
}

// Forward coset transforms of bit-reversed monomials (or natural ones, src_bitrev false) for
// the n_cosets cosets [first, first + n_cosets) of a 2^log_lde LDE.
int lde_forward(uint64_t* lde, size_t col_stride, size_t coset_stride, uint32_t first, uint32_t n_cosets,
                const uint64_t* src, size_t src_stride, bool src_bitrev, uint32_t n_cols, uint32_t log_n,
                uint32_t log_lde, hipStream_t st) {
    const size_t n = (size_t)1 << log_n;
    if (src_bitrev && use_lde3(log_n)) {
        // forward stages 0..12 of every coset from each bit-reversed block, then the last log n - 13
        const uint64_t* tabs;
        if (int r = get_lde3_lde(log_n, log_lde, &tabs)) return r;
        const size_t L = bj::lde3_table_len(log_n);
        HIP_TRY(bj::launch_lde3(lde, col_stride, coset_stride, n_cosets, src, src_stride, nullptr, 0, n_cols, log_n,
                                nullptr, tabs + (size_t)first * L, L, st),
                "coset fft");
        return BJ_OK;
    }
    if (bj::ct_ntt_supported(log_n)) {
        const uint64_t* tabs;
        if (int r = get_ct_lde(log_n, log_lde, &tabs)) return r;
        const size_t L = bj::ct_table_len(log_n);
        HIP_TRY(bj::launch_ct(lde, col_stride, coset_stride, n_cosets, src, src_stride, src_bitrev, n_cols, log_n,
                              tabs + (size_t)first * L, L, 0, true, st),
                "coset fft");
        return BJ_OK;
    }
    const uint64_t *pyr, *pw;
    size_t pws;
    if (int r = get_pyramid(log_n, false, &pyr)) return r;
    if (int r = get_lde_powers(log_n, log_lde, false, &pw, &pws)) return r;
    if (coset_stride != n) return fail(BJ_EINVAL, "internal: coset stride");
    HIP_TRY(bj::launch_lde_forward(lde, col_stride, n_cosets, src, src_stride, src_bitrev, n_cols, log_n, pyr,
                                   pw + (size_t)first * pws, pws, st),
            "coset fft");
    return BJ_OK;
}
}  // namespace

namespace {
// s' = 7 * w_{nD}^{bitrev_{log G}(P)}: the shift of shard P's sub-coset (G > D)
uint64_t shard_shift(uint32_t log_n, uint32_t log_lde, uint32_t log_shards, uint32_t shard) {
    const uint64_t g = gl::domain_generator(log_n + log_lde);
    return gl::canon(gl::mul(gl::pow(g, gl::bitrev32(shard, log_shards)), gl::GENERATOR));
}

int check_shards(uint32_t log_n, uint32_t log_lde, uint32_t log_shards) {
    if (int r = check_log_n(log_n + log_lde)) return r;
    if (log_lde == 0) return fail(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    if (log_shards > log_n + log_lde) return fail(BJ_EINVAL, "more shards than leaves");
    return BJ_OK;
}

// the m-point coset-s' transform of folded (bit-reversed) columns into shard P's leaf range
int shard_from_folded(const uint64_t* folded, size_t folded_stride, uint32_t n_cols, uint32_t log_m, uint64_t sp,
                      uint64_t* lde, hipStream_t st) {
    const size_t m = (size_t)1 << log_m;
    if (use_lde3(log_m)) {
        const uint64_t* tab;
        if (int r = get_lde3(log_m, sp, &tab)) return r;
        HIP_TRY(bj::launch_lde3(lde, m, 0, 1, folded, folded_stride, nullptr, 0, n_cols, log_m, nullptr, tab, 0, st),
                "coset fft");
        return BJ_OK;
    }
    if (bj::ct_ntt_supported(log_m)) {
        const uint64_t* tab;
        if (int r = get_ct(log_m, false, sp, &tab)) return r;
        HIP_TRY(bj::launch_ct(lde, m, 0, 1, folded, folded_stride, true, n_cols, log_m, tab, 0, 0, true, st),
                "coset fft");
        return BJ_OK;
    }
    const uint64_t *pyr, *lo, *hi;
    if (int r = get_pyramid(log_m, false, &pyr)) return r;
    if (int r = get_powers(log_m, sp, 1, &lo, &hi)) return r;
    HIP_TRY(bj::launch_lde_forward(lde, m, 1, folded, folded_stride, true, n_cols, log_m, pyr, lo,
                                   4096 + bj::pw_hi_len(log_m), st),
            "coset fft");
    return BJ_OK;
}
}  // namespace

namespace bj {
int set_error(int code, const char* msg) { return fail(code, msg); }

bool lde_fused_supported(uint32_t log_n) { return use_lde3(log_n); }

int lde_fused_blocks(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                     uint32_t log_k, uint64_t* scratch, uint64_t* lde, size_t col_stride, size_t block_stride,
                     hipStream_t st) {
    if (!use_lde3(log_n)) return fail(BJ_EINVAL, "internal: fused LDE outside 2^18..2^23");
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    const uint64_t *inv, *tabs;
    if (int r = get_ct(log_n, true, 1, &inv)) return r;
    if (int r = get_lde3_lde(log_n, log_lde, &tabs)) return r;
    HIP_TRY(bj::launch_ct_inverse_head(scratch, n, trace, trace_stride, n_cols, log_n, inv, st), "ifft");
    HIP_TRY(bj::launch_lde3(lde, col_stride, n, 1u << log_lde, scratch, n, nullptr, 0, n_cols, log_n, inv, tabs,
                            bj::lde3_table_len(log_n), st, log_k, block_stride),
            "lde");
    return BJ_OK;
}

int lde_own_shard(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                  uint32_t log_shards, uint32_t shard, uint64_t* mono, size_t mono_stride, uint64_t* lde,
                  size_t col_stride, uint32_t passes, hipStream_t st) {
    if (!use_lde3(log_n) || log_shards > log_lde) return fail(BJ_EINVAL, "internal: own-shard LDE needs 2^18..2^23, G <= D");
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    const uint32_t per = 1u << (log_lde - log_shards);
    const uint64_t *inv, *tabs;
    if (int r = get_ct(log_n, true, 1, &inv)) return r;
    if (int r = get_lde3_lde(log_n, log_lde, &tabs)) return r;
    const size_t L = bj::lde3_table_len(log_n);
    if (passes & bj::LDE3_MID)
        HIP_TRY(bj::launch_ct_inverse_head(mono, mono_stride, trace, trace_stride, n_cols, log_n, inv, st), "ifft");
    // the middle pass reads each block's 8192 words before writing its monomials back to the
    // same words, so the head's output and the monomials share `mono`
    HIP_TRY(bj::launch_lde3(lde, col_stride, n, per, mono, mono_stride, mono, mono_stride, n_cols, log_n, inv,
                            tabs + (size_t)shard * per * L, L, st, 31, 0, passes),
            "lde");
    return BJ_OK;
}

bool inverse_fold_supported(uint32_t log_n, uint32_t log_f, uint32_t targets) {
    return use_lde3(log_n) && lde3_inv_fold_supported(log_n, log_f, targets);
}

int inverse_fold_all(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_f,
                     uint32_t targets, const uint64_t* s_pow_m, uint64_t* scratch, size_t scratch_stride,
                     uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, hipStream_t st) {
    if (!inverse_fold_supported(log_n, log_f, targets)) return fail(BJ_EINVAL, "internal: unsupported inverse fold");
    if (n_cols == 0) return BJ_OK;
    const uint64_t* inv;
    if (int r = get_ct(log_n, true, 1, &inv)) return r;
    HIP_TRY(launch_ct_inverse_head(scratch, scratch_stride, trace, trace_stride, n_cols, log_n, inv, st), "ifft");
    HIP_TRY(launch_lde3_inv_fold(dst, dst_col_stride, dst_shard_stride, scratch, scratch_stride, n_cols, log_n, log_f,
                            targets, s_pow_m, inv, st),
            "ifft fold");
    return BJ_OK;
}

uint64_t shard_shift(uint32_t log_n, uint32_t log_lde, uint32_t log_shards, uint32_t shard) {
    return ::shard_shift(log_n, log_lde, log_shards, shard);
}

// The library's own stream-ordered pool per device.  The process's default pool is left
// alone (its release threshold belongs to the host application); ours keeps freed memory
// mapped between calls, so a repeated commit does not re-map its workspace after every
// synchronisation (~20 ms for C2's 5 GB).
static std::mutex g_pool_mu;
static std::map<int, hipMemPool_t>* g_pools = new std::map<int, hipMemPool_t>();

hipError_t pool_trim_all() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto& kv : *g_pools) {
        hipError_t e = hipMemPoolTrimTo(kv.second, 0);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t pool_alloc(void** p, size_t bytes, hipStream_t st) {
    std::mutex& mu = g_pool_mu;
    std::map<int, hipMemPool_t>* pools = g_pools;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    hipMemPool_t pool = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = pools->find(dev);
        if (it == pools->end()) {
            hipMemPoolProps props;
            std::memset(&props, 0, sizeof(props));
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            e = hipMemPoolCreate(&pool, &props);
            if (e != hipSuccess) return e;
            uint64_t keep = UINT64_MAX;
            e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
            if (e != hipSuccess) return e;
            it = pools->emplace(dev, pool).first;
        }
        pool = it->second;
    }
    return hipMallocFromPoolAsync(p, bytes ? bytes : 8, pool, st);
}
}  // namespace bj

extern "C" {

const char* bj_last_error(void) { return g_err.c_str(); }
uint32_t bj_abi_version(void) { return (2u << 16) | 6u; }

int bj_experiment_knob(const char* name, uint64_t* value) {
    if (!name || !value) return fail(BJ_EINVAL, "bj_experiment_knob: null argument");
    const bj::Knobs& k = bj::knobs();
    if (!strcmp(name, "BJ_EXPERIMENTS")) *value = k.enabled;
    else if (!strcmp(name, "BJ_LEAVES_DEFER")) *value = k.leaves_defer;
    else if (!strcmp(name, "BJ_LEAVES_GROUP")) *value = k.leaves_group;
    else if (!strcmp(name, "BJ_INV_FOLD_UNPAIRED")) *value = k.inv_fold_unpaired;
    else if (!strcmp(name, "BJ_LDE_PASSES")) *value = k.lde_passes;
    else if (!strcmp(name, "BJ_NODE_Q4_MAX")) *value = k.node_q4_max;
    else if (!strcmp(name, "BJ_NODE_FUSED")) *value = k.node_fused;
    else if (!strcmp(name, "BJ_LDE_OWN_FUSED")) *value = k.lde_own_fused;
    else return fail(BJ_EINVAL, std::string("bj_experiment_knob: unknown knob ") + name);
    return BJ_OK;
}

int bj_release_workspace(void) {
    HIP_TRY(bj::pool_trim_all(), "hipMemPoolTrimTo");
    return BJ_OK;
}

int bj_release_tables(void) {
    Cache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur), "hipGetDevice");
    // every table, grouped by the device it lives on (the first key element); each device is
    // synchronised before its tables go, so work already queued on it has finished reading them
    std::map<int, std::vector<uint64_t*>> per_dev;
    auto take = [&](auto& m, auto ptr_of) {
        for (auto& kv : m) per_dev[std::get<0>(kv.first)].push_back(ptr_of(kv.second));
        m.clear();
    };
    auto self = [](uint64_t* p) { return p; };
    take(c.tw, self);
    take(c.pyr, self);
    take(c.pw, [](const std::pair<uint64_t*, uint64_t*>& v) { return v.first; });
    take(c.lde_pw, self);
    take(c.ct, self);
    take(c.ct_lde, self);
    take(c.lde3, self);
    take(c.lde3_lde, self);
    hipError_t first = hipSuccess;
    for (auto& dv : per_dev) {
        hipError_t e = hipSetDevice(dv.first);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        for (uint64_t* p : dv.second) {
            const hipError_t f = hipFree(p);
            if (e == hipSuccess) e = f;
        }
        if (first == hipSuccess) first = e;
    }
    const hipError_t e = hipSetDevice(cur);
    if (first == hipSuccess) first = e;
    if (first != hipSuccess) return hip_fail(first, "bj_release_tables");
    return BJ_OK;
}

int bj_prepare(uint32_t log_n) {
    if (int r = check_log_n(log_n)) return r;
    const uint64_t* t;
    if (int r = get_pyramid(log_n, false, &t)) return r;
    if (int r = get_pyramid(log_n, true, &t)) return r;
    if (bj::ct_ntt_supported(log_n))
        if (int r = get_ct(log_n, true, 1, &t)) return r;
    return BJ_OK;
}

int bj_precompute_twiddles_d(uint32_t log_n, int inverse, uint64_t* out_d, void* stream) {
    if (int r = check_log_n(log_n)) return r;
    if (log_n == 0) return fail(BJ_EINVAL, "twiddles need n >= 2");
    HIP_TRY(bj::launch_twiddles(out_d, log_n, inverse != 0, S(stream)), "twiddles");
    return BJ_OK;
}

int bj_precompute_twiddles_h(uint32_t log_n, int inverse, uint64_t* out_h) {
    if (int r = check_log_n(log_n)) return r;
    if (log_n == 0) return fail(BJ_EINVAL, "twiddles need n >= 2");
    const uint64_t* t;
    if (int r = get_twiddles(log_n, inverse != 0, &t)) return r;
    hipStream_t st;
    if (int r = seam_stream(&st)) return r;
    HIP_TRY(hipMemcpyAsync(out_h, t, ((size_t)1 << (log_n - 1)) * 8, hipMemcpyDeviceToHost, st), "memcpy");
    HIP_TRY(hipStreamSynchronize(st), "sync");
    return BJ_OK;
}

int bj_precompute_twiddles_natural_d(uint32_t log_n, int inverse, uint64_t* out_d, void* stream) {
    if (int r = check_log_n(log_n)) return r;
    if (log_n == 0) return fail(BJ_EINVAL, "twiddles need n >= 2");
    HIP_TRY(bj::launch_twiddles_natural(out_d, log_n, inverse != 0, S(stream)), "twiddles");
    return BJ_OK;
}

int bj_bitreverse_enumeration_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n, void* stream) {
    if (int r = check_log_n(log_n)) return r;
    HIP_TRY(bj::launch_bitrev_inplace(cols, col_stride, n_cols, log_n, S(stream)), "bitreverse");
    return BJ_OK;
}

int bj_distribute_powers_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n, uint64_t element,
                           void* stream) {
    if (int r = check_log_n(log_n)) return r;
    const uint64_t *lo, *hi;
    if (int r = get_powers(log_n, element, 1, &lo, &hi)) return r;
    HIP_TRY(bj::launch_distribute(cols, col_stride, n_cols, log_n, lo, hi, S(stream)), "distribute");
    return BJ_OK;
}

// Sizes 2^13..2^23 run the coset-folded CT network of ntt_ct.hip, the shift folded
// into its twiddle table; smaller ones a DIF network (ntt_dif.hip) over its own cached twiddle
// pyramid. A twiddle pointer in the reference's format is accepted for signature parity and
// not read.
int bj_fft_natural_to_bitreversed_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n,
                                    uint64_t coset, const uint64_t* twiddles_d, void* stream) {
    (void)twiddles_d;
    if (int r = check_log_n(log_n)) return r;
    if (n_cols == 0) return BJ_OK;
    if (bj::ct_ntt_supported(log_n)) {
        const uint64_t* tab;
        if (int r = get_ct(log_n, false, coset, &tab)) return r;
        HIP_TRY(bj::launch_ct(cols, col_stride, 0, 1, cols, col_stride, false, n_cols, log_n, tab, 0, 0, true,
                              S(stream)),
                "fft");
        return BJ_OK;
    }
    if (gl::canon(coset) != 1)
        if (int r = bj_distribute_powers_d(cols, n_cols, col_stride, log_n, coset, stream)) return r;
    const uint64_t* pyr;
    if (int r = get_pyramid(log_n, false, &pyr)) return r;
    HIP_TRY(bj::launch_dif(cols, col_stride, cols, col_stride, n_cols, log_n, pyr, true, S(stream)), "fft");
    return BJ_OK;
}


int bj_ifft_natural_to_natural_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n,
                                 uint64_t coset, const uint64_t* inv_twiddles_d, void* stream) {
    (void)inv_twiddles_d;
    if (int r = check_log_n(log_n)) return r;
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    // monomials in bit-reversed order into a temporary, then the bit reversal back in place
    uint64_t* tmp = nullptr;
    HIP_TRY(bj::pool_alloc((void**)&tmp, n * n_cols * 8, S(stream)), "pool_alloc");
    int r = inverse_to_bitrev(tmp, n, cols, col_stride, n_cols, log_n, S(stream));
    hipError_t e = r == BJ_OK ? bj::launch_bitrev_scale(cols, col_stride, tmp, n, n_cols, log_n, 1, S(stream))
                              : hipSuccess;
    hipError_t e2 = hipFreeAsync(tmp, S(stream));
    if (r) return r;
    if (e != hipSuccess) return hip_fail(e, "ifft bitreverse");
    if (e2 != hipSuccess) return hip_fail(e2, "hipFreeAsync");
    if (gl::canon(coset) != 1) {
        const uint64_t *lo, *hi;
        if (int r2 = get_powers(log_n, gl::inv(gl::canon(coset)), 1, &lo, &hi)) return r2;
        HIP_TRY(bj::launch_distribute(cols, col_stride, n_cols, log_n, lo, hi, S(stream)), "distribute");
    }
    return BJ_OK;
}

int bj_monomials_to_lde_d(const uint64_t* monomials, uint32_t n_cols, size_t mono_stride, uint32_t log_n,
                          uint32_t log_lde, uint64_t* lde, void* stream) {
    if (int r = check_log_n(log_n + log_lde)) return r;
    if (log_lde == 0) return fail(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    const uint32_t D = 1u << log_lde;
    return lde_forward(lde, (size_t)D * n, n, 0, D, monomials, mono_stride, false, n_cols, log_n, log_lde, S(stream));
}

int bj_lde_ex_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                uint64_t* scratch, uint64_t* lde, uint32_t flags, void* stream) {
    if (flags & ~BJ_LDE_KEEP_MONOMIALS) return fail(BJ_EINVAL, "unknown bj_lde_ex_d flags");
    if (int r = check_log_n(log_n + log_lde)) return r;
    if (log_lde == 0) return fail(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    const uint32_t D = 1u << log_lde;
    if (use_lde3(log_n)) {
        // three passes (ntt_lde3.hip): the inverse head into scratch; the inverse tail fused with
        // forward stages 0..12 of all D cosets (with BJ_LDE_KEEP_MONOMIALS the canonical
        // monomials are written back to scratch, c_j at bitrev_n(j)); the last log n - 13 forward
        // stages in place on the LDE
        const uint64_t *inv, *tabs;
        if (int r = get_ct(log_n, true, 1, &inv)) return r;
        if (int r = get_lde3_lde(log_n, log_lde, &tabs)) return r;
        uint64_t* mono = (flags & BJ_LDE_KEEP_MONOMIALS) ? scratch : nullptr;
        const size_t L = bj::lde3_table_len(log_n);
        hipStream_t st = S(stream);
        HIP_TRY(bj::launch_ct_inverse_head(scratch, n, trace, trace_stride, n_cols, log_n, inv, st), "ifft");
        HIP_TRY(bj::launch_lde3(lde, (size_t)D * n, n, D, scratch, n, mono, n, n_cols, log_n, inv, tabs, L, st),
                "lde");
        return BJ_OK;
    }
    // iFFT (utils.rs:295-304): scratch = monomials in bit-reversed order; the forward pass
    // gathers them back in natural order, all D cosets (utils.rs:363-379).  These paths leave
    // the monomials in scratch with or without the flag.
    if (int r = inverse_to_bitrev(scratch, n, trace, trace_stride, n_cols, log_n, S(stream))) return r;
    return lde_forward(lde, (size_t)D * n, n, 0, D, scratch, n, true, n_cols, log_n, log_lde, S(stream));
}

int bj_lde_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
             uint64_t* scratch, uint64_t* lde, void* stream) {
    return bj_lde_ex_d(trace, n_cols, trace_stride, log_n, log_lde, scratch, lde, BJ_LDE_KEEP_MONOMIALS, stream);
}

int bj_lde_coeffs_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint64_t* coeffs,
                    size_t coeffs_stride, void* stream) {
    if (int r = check_log_n(log_n)) return r;
    if (n_cols == 0) return BJ_OK;
    return inverse_to_bitrev(coeffs, coeffs_stride, trace, trace_stride, n_cols, log_n, S(stream));
}

int bj_lde_shard_d(const uint64_t* coeffs, uint32_t n_cols, size_t coeffs_stride, uint32_t log_n, uint32_t log_lde,
                   uint32_t log_shards, uint32_t shard, uint64_t* work, uint64_t* lde, void* stream) {
    if (int r = check_shards(log_n, log_lde, log_shards)) return r;
    if (shard >= (1u << log_shards)) return fail(BJ_EINVAL, "shard index out of range");
    if (n_cols == 0) return BJ_OK;
    const size_t n = (size_t)1 << log_n;
    if (log_shards <= log_lde) {
        // whole cosets [P * D/G, (P+1) * D/G)
        const uint32_t per = 1u << (log_lde - log_shards);
        return lde_forward(lde, (size_t)per * n, n, shard * per, per, coeffs, coeffs_stride, true, n_cols, log_n,
                           log_lde, S(stream));
    }
    const uint32_t log_f = log_shards - log_lde;
    if ((1u << log_f) > bj::kMaxFold) return fail(BJ_EINVAL, "G / D exceeds 64");
    if (!work) return fail(BJ_EINVAL, "work buffer required when shards exceed the lde degree");
    const uint32_t log_m = log_n - log_f;
    const size_t m = (size_t)1 << log_m;
    // h_t = sum_a c_{t+am} (s'^m)^a (shard.hip), then the m-point coset-s' transform of h
    const uint64_t sp = shard_shift(log_n, log_lde, log_shards, shard);
    HIP_TRY(bj::launch_fold(work, m, coeffs, coeffs_stride, n_cols, log_m, log_f, gl::pow(sp, m), S(stream)), "fold");
    return shard_from_folded(work, m, n_cols, log_m, sp, lde, S(stream));
}

int bj_lde_fold_shards_d(const uint64_t* coeffs, uint32_t n_cols, size_t coeffs_stride, uint32_t log_n,
                         uint32_t log_lde, uint32_t log_shards, uint64_t* out, size_t out_shard_stride,
                         void* stream) {
    if (int r = check_shards(log_n, log_lde, log_shards)) return r;
    if (log_shards <= log_lde) return fail(BJ_EINVAL, "folding needs more shards than the lde degree");
    const uint32_t log_f = log_shards - log_lde;
    if ((1u << log_f) > bj::kMaxFold) return fail(BJ_EINVAL, "G / D exceeds 64");
    const uint32_t log_m = log_n - log_f;
    const size_t m = (size_t)1 << log_m;
    const uint32_t G = 1u << log_shards;
    if (out_shard_stride < (size_t)n_cols * m) return fail(BJ_EINVAL, "out_shard_stride < n_cols * m");
    if (n_cols == 0) return BJ_OK;
    std::vector<uint64_t> spm(G);
    for (uint32_t P = 0; P < G; P++) spm[P] = gl::pow(shard_shift(log_n, log_lde, log_shards, P), m);
    HIP_TRY(bj::launch_fold_all(out, m, out_shard_stride, coeffs, coeffs_stride, n_cols, log_m, log_f, G, spm.data(),
                                S(stream)),
            "fold");
    return BJ_OK;
}

int bj_lde_shard_folded_d(const uint64_t* folded, uint32_t n_cols, size_t folded_stride, uint32_t log_n,
                          uint32_t log_lde, uint32_t log_shards, uint32_t shard, uint64_t* lde, void* stream) {
    if (int r = check_shards(log_n, log_lde, log_shards)) return r;
    if (shard >= (1u << log_shards)) return fail(BJ_EINVAL, "shard index out of range");
    if (log_shards <= log_lde) return fail(BJ_EINVAL, "folded input needs more shards than the lde degree");
    const uint32_t log_f = log_shards - log_lde;
    if ((1u << log_f) > bj::kMaxFold) return fail(BJ_EINVAL, "G / D exceeds 64");
    if (n_cols == 0) return BJ_OK;
    const uint32_t log_m = log_n - log_f;
    return shard_from_folded(folded, folded_stride, n_cols, log_m, shard_shift(log_n, log_lde, log_shards, shard),
                             lde, S(stream));
}

int bj_fri_fold_d(const uint64_t* c0, const uint64_t* c1, size_t n_src, const uint64_t* roots,
                  uint64_t coset_inverse, uint64_t ch0, uint64_t ch1, uint64_t* dst_c0, uint64_t* dst_c1,
                  void* stream) {
    if (n_src < 2 || (n_src & 1)) return fail(BJ_EINVAL, "a fold needs an even source length >= 2");
    HIP_TRY(bj::launch_fri_fold(c0, c1, n_src / 2, roots, coset_inverse, ch0, ch1, dst_c0, dst_c1, S(stream)),
            "fri fold");
    return BJ_OK;
}

int bj_fill_synthetic_d(uint64_t* dst, uint32_t n_cols, size_t col_stride, uint32_t log_n, uint64_t seed,
                        uint64_t first_col, void* stream) {
    if (int r = check_log_n(log_n)) return r;
    HIP_TRY(bj::launch_synthetic(dst, col_stride, n_cols, log_n, seed, first_col, S(stream)), "synthetic");
    return BJ_OK;
}

int bj_gl_op_d(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, void* stream) {
    if (op < 0 || op > 4) return fail(BJ_EINVAL, "op must be 0 mul, 1 add, 2 sub, 3 reduce, 4 canon");
    HIP_TRY(bj::launch_gl_op(op, a, b, out, n, S(stream)), "gl_op");
    return BJ_OK;
}

int bj_poseidon2_permute_d(uint64_t* states, size_t count, void* stream) {
    HIP_TRY(bj::launch_permute(states, count, S(stream)), "permute");
    return BJ_OK;
}

int bj_merkle_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves, uint64_t* leaves,
                       void* stream) {
    HIP_TRY(bj::launch_leaves(src, col_stride, n_cols, n_leaves, leaves, S(stream)), "leaves");
    return BJ_OK;
}

int bj_merkle_leaves_partial_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                               const uint64_t* cap_in, uint64_t* out, int final_, void* stream) {
    if (!final_ && (n_cols & 7))
        return fail(BJ_EINVAL, "a non-final column range must be a multiple of the sponge rate (8)");
    if (final_ && cap_in && n_cols == 0)
        return fail(BJ_EINVAL, "the final column range of a continued sponge must be non-empty");
    HIP_TRY(bj::launch_leaves_partial(src, col_stride, n_cols, n_leaves, cap_in, out, final_ != 0, S(stream)),
            "leaves");
    return BJ_OK;
}

int bj_merkle_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                               uint32_t elems_per_leaf, uint64_t* out, void* stream) {
    if (!is_pow2(elems_per_leaf)) return fail(BJ_EINVAL, "elements_to_take_per_leaf must be a power of two");
    uint32_t log_e = 0;
    while ((1u << log_e) < elems_per_leaf) log_e++;
    if ((uint64_t)n_cols << log_e > 0xFFFFFFFFull) return fail(BJ_EINVAL, "leaf too long");
    HIP_TRY(bj::launch_leaves_chunked(src, col_stride, n_cols, log_e, n_leaves, out, S(stream)), "leaves");
    return BJ_OK;
}

int bj_merkle_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes, void* stream) {
    if (!is_pow2(n_leaves) || !is_pow2(cap_size) || n_leaves <= cap_size)
        return fail(BJ_EINVAL, "need power-of-two n_leaves > cap_size (merkle_tree.rs:83-96)");
    HIP_TRY(bj::launch_nodes(leaves, n_leaves, cap_size, nodes, S(stream)), "nodes");
    return BJ_OK;
}

// ------------------------------------------------------------ Blake2s256 trees

int bj_blake2s_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves, uint64_t* leaves,
                        void* stream) {
    HIP_TRY(bj::launch_b2s_leaves(src, col_stride, n_cols, n_leaves, 0, nullptr, leaves, true, S(stream)), "leaves");
    return BJ_OK;
}

int bj_blake2s_leaves_partial_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                uint64_t cols_before, const uint64_t* state_in, uint64_t* out, int final_,
                                void* stream) {
    if (cols_before & 7) return fail(BJ_EINVAL, "cols_before must be a multiple of the block (8 elements)");
    if ((cols_before != 0) != (state_in != nullptr))
        return fail(BJ_EINVAL, "state_in is required exactly when cols_before > 0");
    if (!final_ && (n_cols & 7))
        return fail(BJ_EINVAL, "a non-final column range must be a multiple of the block (8 elements)");
    if (final_ && cols_before && n_cols == 0)
        return fail(BJ_EINVAL, "the final column range of a continued message must be non-empty");
    HIP_TRY(bj::launch_b2s_leaves(src, col_stride, n_cols, n_leaves, cols_before, state_in, out, final_ != 0,
                                  S(stream)),
            "leaves");
    return BJ_OK;
}

int bj_blake2s_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                uint32_t elems_per_leaf, uint64_t* out, void* stream) {
    if (!is_pow2(elems_per_leaf)) return fail(BJ_EINVAL, "elements_to_take_per_leaf must be a power of two");
    uint32_t log_e = 0;
    while ((1u << log_e) < elems_per_leaf) log_e++;
    if ((uint64_t)n_cols << log_e > 0xFFFFFFFFull) return fail(BJ_EINVAL, "leaf too long");
    HIP_TRY(bj::launch_b2s_leaves_chunked(src, col_stride, n_cols, log_e, n_leaves, out, S(stream)), "leaves");
    return BJ_OK;
}

int bj_blake2s_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes, void* stream) {
    if (!is_pow2(n_leaves) || !is_pow2(cap_size) || n_leaves <= cap_size)
        return fail(BJ_EINVAL, "need power-of-two n_leaves > cap_size (merkle_tree.rs:83-96)");
    HIP_TRY(bj::launch_b2s_nodes(leaves, n_leaves, cap_size, nodes, S(stream)), "nodes");
    return BJ_OK;
}

// ------------------------------------------------------------ Keccak256 trees

int bj_keccak256_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves, uint64_t* leaves,
                          void* stream) {
    HIP_TRY(bj::launch_kc_leaves(src, col_stride, n_cols, n_leaves, leaves, S(stream)), "leaves");
    return BJ_OK;
}

int bj_keccak256_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                  uint32_t elems_per_leaf, uint64_t* out, void* stream) {
    if (!is_pow2(elems_per_leaf)) return fail(BJ_EINVAL, "elements_to_take_per_leaf must be a power of two");
    uint32_t log_e = 0;
    while ((1u << log_e) < elems_per_leaf) log_e++;
    if ((uint64_t)n_cols << log_e > 0xFFFFFFFFull) return fail(BJ_EINVAL, "leaf too long");
    HIP_TRY(bj::launch_kc_leaves_chunked(src, col_stride, n_cols, log_e, n_leaves, out, S(stream)), "leaves");
    return BJ_OK;
}

int bj_keccak256_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                         void* stream) {
    if (!is_pow2(n_leaves) || !is_pow2(cap_size) || n_leaves <= cap_size)
        return fail(BJ_EINVAL, "need power-of-two n_leaves > cap_size (merkle_tree.rs:83-96)");
    HIP_TRY(bj::launch_kc_nodes(leaves, n_leaves, cap_size, nodes, S(stream)), "nodes");
    return BJ_OK;
}

namespace {
int commit_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
             uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* scratch, uint64_t* lde, uint64_t* leaves,
             uint64_t* nodes, bool keep_mono, void* stream) {
    if (log_commit_cosets > log_lde)
        return fail(BJ_EINVAL, "committed cosets exceed the lde degree (prover.rs:313, lde.rs:298-308)");
    if (int r = check_log_n(log_n + log_lde)) return r;
    if (log_lde == 0) return fail(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    // the tree covers the first k = 2^log_commit_cosets cosets of every column
    // (subset_for_degree, lde.rs:298-308): leaf L < k * n of column c is lde[c * D * n + L]
    const size_t nd = (size_t)1 << (log_n + log_lde);
    const size_t nl = (size_t)1 << (log_n + log_commit_cosets);
    if (!is_pow2(cap_size) || nl <= cap_size)
        return fail(BJ_EINVAL, "need power-of-two cap_size < n * k (merkle_tree.rs:83-96)");
    if (int r = bj_lde_ex_d(trace, n_cols, trace_stride, log_n, log_lde, scratch, lde,
                            keep_mono ? BJ_LDE_KEEP_MONOMIALS : 0, stream))
        return r;
    if (int r = bj_merkle_leaves_d(lde, n_cols, nd, nl, leaves, stream)) return r;
    if (int r = bj_merkle_nodes_d(leaves, nl, cap_size, nodes, stream)) return r;
    return BJ_OK;
}
}  // namespace

namespace {
int copy_cap(const uint64_t* nodes, size_t nl, uint32_t cap_size, uint64_t* cap_h, void* stream) {
    if (!cap_h) return BJ_OK;
    HIP_TRY(hipMemcpyAsync(cap_h, nodes + 4 * (nl - 2 * (size_t)cap_size), (size_t)cap_size * 32,
                           hipMemcpyDeviceToHost, S(stream)),
            "memcpy cap");
    HIP_TRY(hipStreamSynchronize(S(stream)), "sync");
    return BJ_OK;
}
}  // namespace

int bj_lde_commit_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                    uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* scratch, uint64_t* lde, uint64_t* leaves,
                    uint64_t* nodes, uint64_t* cap_h, void* stream) {
    return bj_lde_commit_ex_d(trace, n_cols, trace_stride, log_n, log_lde, log_commit_cosets, cap_size, scratch, lde,
                              leaves, nodes, cap_h, BJ_LDE_KEEP_MONOMIALS, stream);
}

int bj_lde_commit_ex_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                       uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* scratch, uint64_t* lde,
                       uint64_t* leaves, uint64_t* nodes, uint64_t* cap_h, uint32_t flags, void* stream) {
    if (flags & ~BJ_LDE_KEEP_MONOMIALS) return fail(BJ_EINVAL, "unknown bj_lde_commit_ex_d flags");
    if (int r = commit_d(trace, n_cols, trace_stride, log_n, log_lde, log_commit_cosets, cap_size, scratch, lde,
                         leaves, nodes, (flags & BJ_LDE_KEEP_MONOMIALS) != 0, stream))
        return r;
    return copy_cap(nodes, (size_t)1 << (log_n + log_commit_cosets), cap_size, cap_h, stream);
}

// --------------------------------------------------------- host-pointer seam

#define SEAM_BEGIN            \
    hipStream_t st;           \
    if (int r_ = seam_stream(&st)) return r_
#define H2D(dst, src, bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st), "memcpy")
#define D2H(dst, src, bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st), "memcpy")
#define SEAM_END HIP_TRY(hipStreamSynchronize(st), "sync")

int bj_distribute_powers_h(uint64_t* col, size_t len, uint64_t element) {
    uint32_t log_n;
    if (int r = log2_exact(len, &log_n)) return r;
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(len * 8), "hipMallocAsync");
    H2D(d.p, col, len * 8);
    if (int r = bj_distribute_powers_d(d.p, 1, len, log_n, element, st)) return r;
    D2H(col, d.p, len * 8);
    SEAM_END;
    return BJ_OK;
}

int bj_fft_natural_to_bitreversed_h(uint64_t* col, size_t len, uint64_t coset) {
    uint32_t log_n;
    if (int r = log2_exact(len, &log_n)) return r;
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(len * 8), "hipMallocAsync");
    H2D(d.p, col, len * 8);
    if (int r = bj_fft_natural_to_bitreversed_d(d.p, 1, len, log_n, coset, nullptr, st)) return r;
    D2H(col, d.p, len * 8);
    SEAM_END;
    return BJ_OK;
}

int bj_ifft_natural_to_natural_h(uint64_t* col, size_t len, uint64_t coset) {
    uint32_t log_n;
    if (int r = log2_exact(len, &log_n)) return r;
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(len * 8), "hipMallocAsync");
    H2D(d.p, col, len * 8);
    if (int r = bj_ifft_natural_to_natural_d(d.p, 1, len, log_n, coset, nullptr, st)) return r;
    D2H(col, d.p, len * 8);
    SEAM_END;
    return BJ_OK;
}

int bj_poseidon2_permute_h(uint64_t* state12) {
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(96), "hipMallocAsync");
    H2D(d.p, state12, 96);
    if (int r = bj_poseidon2_permute_d(d.p, 1, st)) return r;
    D2H(state12, d.p, 96);
    SEAM_END;
    return BJ_OK;
}

int bj_hash_into_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4) {
    SEAM_BEGIN;
    DBuf d(st), o(st);
    HIP_TRY(d.alloc(n_elems * 8), "hipMallocAsync");
    HIP_TRY(o.alloc(32), "hipMallocAsync");
    if (n_elems) H2D(d.p, elems, n_elems * 8);
    if (int r = bj_merkle_leaves_d(d.p, (uint32_t)n_elems, 1, 1, o.p, st)) return r;
    D2H(out4, o.p, 32);
    SEAM_END;
    return BJ_OK;
}

int bj_hash_into_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4) {
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(96), "hipMallocAsync");
    H2D(d.p, left4, 32);
    H2D(d.p + 4, right4, 32);
    if (int r = bj_merkle_nodes_d(d.p, 2, 1, d.p + 8, st)) return r;
    D2H(out4, d.p + 8, 32);
    SEAM_END;
    return BJ_OK;
}

int bj_blake2s_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4) {
    if (n_elems > 0xFFFFFFFFull) return fail(BJ_EINVAL, "leaf too long");
    SEAM_BEGIN;
    DBuf d(st), o(st);
    HIP_TRY(d.alloc(n_elems * 8), "hipMallocAsync");
    HIP_TRY(o.alloc(32), "hipMallocAsync");
    if (n_elems) H2D(d.p, elems, n_elems * 8);
    HIP_TRY(bj::launch_b2s_words(d.p, (uint32_t)n_elems, o.p, st), "blake2s");
    D2H(out4, o.p, 32);
    SEAM_END;
    return BJ_OK;
}

int bj_blake2s_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4) {
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(96), "hipMallocAsync");
    H2D(d.p, left4, 32);
    H2D(d.p + 4, right4, 32);
    if (int r = bj_blake2s_nodes_d(d.p, 2, 1, d.p + 8, st)) return r;
    D2H(out4, d.p + 8, 32);
    SEAM_END;
    return BJ_OK;
}

int bj_keccak256_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4) {
    if (n_elems > 0xFFFFFFFFull) return fail(BJ_EINVAL, "leaf too long");
    SEAM_BEGIN;
    DBuf d(st), o(st);
    HIP_TRY(d.alloc(n_elems * 8), "hipMallocAsync");
    HIP_TRY(o.alloc(32), "hipMallocAsync");
    if (n_elems) H2D(d.p, elems, n_elems * 8);
    // the elements as n_elems one-row columns of one leaf
    HIP_TRY(bj::launch_kc_leaves(d.p, 1, (uint32_t)n_elems, 1, o.p, st), "keccak256");
    D2H(out4, o.p, 32);
    SEAM_END;
    return BJ_OK;
}

int bj_keccak256_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4) {
    SEAM_BEGIN;
    DBuf d(st);
    HIP_TRY(d.alloc(96), "hipMallocAsync");
    H2D(d.p, left4, 32);
    H2D(d.p + 4, right4, 32);
    if (int r = bj_keccak256_nodes_d(d.p, 2, 1, d.p + 8, st)) return r;
    D2H(out4, d.p + 8, 32);
    SEAM_END;
    return BJ_OK;
}

// bj_lde_commit_h: host_commit.hip

}  // extern "C"
